// Which CU runs each workgroup (diagnostic for tools/cumask_probe.py):
// out[block] = xcc_id << 16 | se_id << 8 | sh_id << 4 | cu_id (gfx950 HW_ID).
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void k_where(uint32_t* out, int spin) {
  uint32_t hw, xcc;
  __asm__ volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  __asm__ volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  const uint32_t cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
  // keep the block resident a while so later blocks spread over free CUs
  for (int i = 0; i < spin; ++i) __builtin_amdgcn_s_sleep(10);
  if (threadIdx.x == 0) out[blockIdx.x] = ((xcc & 15) << 16) | (se << 8) | (sh << 4) | cu;
}

extern "C" int cu_probe(uint32_t* out, int blocks, int spin, void* stream) {
  hipLaunchKernelGGL(k_where, dim3(blocks), dim3(64), 0, (hipStream_t)stream, out, spin);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
