"""Code bytes of the loops of one kernel in an llvm-objdump -d listing (diagnostic).

usage: python tools/isa_bytes.py file.dis kernel-substring
(objdump of the gfx950 code object: clang-offload-bundler --unbundle, then
llvm-objdump -d --mcpu=gfx950).  The fused kernel is bound by instruction
fetch (SQC_ICACHE_BUSY_CYCLES ~97 % of the kernel's cycles), so the bytes a
wave streams per frame are the quantity to minimise.  Prints, per loop, its
instruction count, bytes, and bytes by opcode class and by encoding size.
"""
import collections
import re
import sys


def main():
    text = open(sys.argv[1]).read().split('\n')
    start = end = None
    for i, l in enumerate(text):
        m = re.match(r'^[0-9a-f]+ <(\S+)>:', l)
        if m:
            if start is not None and end is None:
                end = i
            if sys.argv[2] in m.group(1) and start is None:
                start = i
    end = end or len(text)
    ins = []
    for l in text[start:end]:
        m = re.search(r'//\s*([0-9A-Fa-f]+):((?:\s+[0-9A-Fa-f]{8}\b)+)', l)
        if m:
            ins.append((int(m.group(1), 16), len(m.group(2).split()) * 4,
                        l.split('//')[0].strip()))
    addr_idx = {a: i for i, (a, _, _) in enumerate(ins)}
    loops = []
    for i, (a, n, t) in enumerate(ins):
        m = re.match(r's_(?:cbranch_\w+|branch)\s+(\d+)', t)
        if m:  # objdump prints the signed dword offset from the next instruction
            tgt = a + n + 4 * int(m.group(1)) if int(m.group(1)) < 32768 else \
                a + n + 4 * (int(m.group(1)) - 65536)
            if tgt < a and tgt in addr_idx:
                loops.append((addr_idx[tgt], i))
    total = sum(n for _, n, _ in ins)
    print(f'kernel: {len(ins)} instructions, {total} bytes')
    for lo, hi in sorted(loops, key=lambda x: x[0] - x[1])[:12]:
        seg = ins[lo:hi + 1]
        by_cls, by_size = collections.Counter(), collections.Counter()
        for _, n, t in seg:
            op = t.split()[0]
            cls = ('ds' if op.startswith('ds_') else 'vmem' if op.startswith(('buffer_', 'global_'))
                   else 'salu' if op.startswith('s_') else 'v_pk' if op.startswith('v_pk')
                   else 'valu')
            by_cls[cls] += n
            by_size[(cls, n)] += 1
        print(f'loop {lo}-{hi}: {len(seg)} instructions, {sum(n for _, n, _ in seg)} bytes;'
              f' bytes by class {dict(by_cls)}')
        print('   (class, bytes): count', dict(sorted(by_size.items())))


if __name__ == '__main__':
    main()
