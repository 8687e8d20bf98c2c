// Instruction-fetch probe (diagnostic): cycles per v_add_f32 (VOP2, 4 B) and
// per v_fma_f32 (VOP3, 8 B) for a loop body of 256 vs 4096 straight-line
// instructions (1-32 KB of code), waves per SIMD set by the block size.
#include <hip/hip_runtime.h>
#include <stdint.h>

#define R4(x) x x x x
#define R16(x) R4(R4(x))
#define R256(x) R16(R16(x))
#define ADD4 "v_add_f32 v20, v1, v2\n v_add_f32 v21, v5, v6\n v_add_f32 v22, v9, v10\n v_add_f32 v23, v13, v14\n"
#define FMA4 "v_fma_f32 v20, v1, v2, v3\n v_fma_f32 v21, v5, v6, v7\n v_fma_f32 v22, v9, v10, v11\n v_fma_f32 v23, v13, v14, v15\n"

template <int K>
__global__ void k_fetch(uint64_t* out, int iters) {
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if constexpr (K == 0) __asm__ volatile(R16(ADD4) ::: "v20", "v21", "v22", "v23");        // 64 instr, 256 B
    if constexpr (K == 1) __asm__ volatile(R256(ADD4) ::: "v20", "v21", "v22", "v23");       // 1024 instr, 4 KB
    if constexpr (K == 2) __asm__ volatile(R4(R256(ADD4)) ::: "v20", "v21", "v22", "v23");   // 4096 instr, 16 KB
    if constexpr (K == 3) __asm__ volatile(R16(FMA4) ::: "v20", "v21", "v22", "v23");        // 64 instr, 512 B
    if constexpr (K == 4) __asm__ volatile(R256(FMA4) ::: "v20", "v21", "v22", "v23");       // 1024, 8 KB
    if constexpr (K == 5) __asm__ volatile(R4(R256(FMA4)) ::: "v20", "v21", "v22", "v23");   // 4096, 32 KB
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

extern "C" int fetch_probe(int kind, uint64_t* out, int blocks, int threads, int iters, void* s) {
  switch (kind) {
#define K_(k) case k: hipLaunchKernelGGL(k_fetch<k>, dim3(blocks), dim3(threads), 0, (hipStream_t)s, out, iters); break;
    K_(0) K_(1) K_(2) K_(3) K_(4) K_(5)
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
