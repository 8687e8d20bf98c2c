// VGPR bank-conflict probe (diagnostic): cycles per v_fma_f32 / v_add_f32 when
// the source operands sit in the same or in different VGPR banks (reg % 4).
#include <hip/hip_runtime.h>
#include <stdint.h>

#define REP8(x) x x x x x x x x
#define REP64(x) REP8(REP8(x))

template <int K>
__global__ void k_bank(uint64_t* out, int iters) {
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if constexpr (K == 0)  // fma, sources in 3 different banks, rotating destinations
      __asm__ volatile(REP64("v_fma_f32 v20, v1, v2, v3\n v_fma_f32 v21, v5, v6, v7\n v_fma_f32 v22, v9, v10, v11\n v_fma_f32 v23, v13, v14, v15\n")
                       ::: "v20", "v21", "v22", "v23");
    else if constexpr (K == 1)  // fma, all 3 sources in one bank
      __asm__ volatile(REP64("v_fma_f32 v20, v1, v5, v9\n v_fma_f32 v21, v2, v6, v10\n v_fma_f32 v22, v3, v7, v11\n v_fma_f32 v23, v4, v8, v12\n")
                       ::: "v20", "v21", "v22", "v23");
    else if constexpr (K == 2)  // add, two different banks
      __asm__ volatile(REP64("v_add_f32 v20, v1, v2\n v_add_f32 v21, v5, v6\n v_add_f32 v22, v9, v10\n v_add_f32 v23, v13, v14\n")
                       ::: "v20", "v21", "v22", "v23");
    else if constexpr (K == 3)  // add, same bank
      __asm__ volatile(REP64("v_add_f32 v20, v1, v5\n v_add_f32 v21, v2, v6\n v_add_f32 v22, v3, v7\n v_add_f32 v23, v4, v8\n")
                       ::: "v20", "v21", "v22", "v23");
    else if constexpr (K == 4)  // fmac (dst is a source), sources in different banks
      __asm__ volatile(REP64("v_fmac_f32 v20, v1, v2\n v_fmac_f32 v21, v5, v6\n v_fmac_f32 v22, v9, v10\n v_fmac_f32 v23, v13, v14\n")
                       ::: "v20", "v21", "v22", "v23");
    else if constexpr (K == 5)  // fmac, all in bank 0
      __asm__ volatile(REP64("v_fmac_f32 v20, v4, v8\n v_fmac_f32 v24, v12, v16\n v_fmac_f32 v28, v32, v36\n v_fmac_f32 v40, v44, v48\n")
                       ::: "v20", "v24", "v28", "v40");
    else if constexpr (K == 6)  // fmamk with literal, sources in different banks
      __asm__ volatile(REP64("v_fmamk_f32 v20, v1, 0x3e4bafaf, v2\n v_fmamk_f32 v21, v5, 0x3e4bafaf, v6\n v_fmamk_f32 v22, v9, 0x3e4bafaf, v10\n v_fmamk_f32 v23, v13, 0x3e4bafaf, v14\n")
                       ::: "v20", "v21", "v22", "v23");
    else if constexpr (K == 7)  // dependent chains (4 chains) of fma
      __asm__ volatile(REP64("v_fma_f32 v20, v20, v2, v3\n v_fma_f32 v21, v21, v6, v7\n v_fma_f32 v22, v22, v10, v11\n v_fma_f32 v23, v23, v14, v15\n")
                       ::: "v20", "v21", "v22", "v23");
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

extern "C" int bank_probe(int kind, uint64_t* out, int blocks, int threads, int iters, void* s) {
  switch (kind) {
#define K_(k) case k: hipLaunchKernelGGL(k_bank<k>, dim3(blocks), dim3(threads), 0, (hipStream_t)s, out, iters); break;
    K_(0) K_(1) K_(2) K_(3) K_(4) K_(5) K_(6) K_(7)
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
