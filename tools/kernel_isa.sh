#!/bin/bash
# Disassemble one kernel of a built transform unit (diagnostic):
#   tools/kernel_isa.sh <unit .o> <kernel-name substring> <out.dis>
# then: python tools/isa_bytes.py <out.dis> <substring>; the code object's
# notes (VGPRs, SGPR spills, LDS) go to <out.dis>.notes
set -e
O=$1; K=$2; OUT=$3
T=$(mktemp -d)
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section=.hip_fatbin=$T/fb.bin "$O"
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$T/fb.bin \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/t.co
/opt/rocm/lib/llvm/bin/llvm-objdump -d --mcpu=gfx950 $T/t.co > "$OUT"
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $T/t.co > "$OUT.notes"
rm -rf $T
