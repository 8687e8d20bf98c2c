// valu_probe.hip — VALU issue-rate probe for gfx950 (diagnostic, not product).
// Each wave runs ITER iterations of 16 independent fp32 chains, as scalar
// v_fma_f32 / v_add_f32 or packed v_pk_fma_f32 / v_pk_add_f32 (inline asm, so
// the compiler cannot re-pack), launched with W waves per SIMD.  Reports the
// fp32 lane-operations per cycle per SIMD and cycles per instruction per wave
// from s_memtime.  Build: hipcc --offload-arch=gfx950 -O3 tools/valu_probe.hip
// -o tools/valu_probe ; run on the GPU box.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int KIND>  // 0 v_fma_f32, 1 v_pk_fma_f32, 2 v_add_f32, 3 v_pk_add_f32,
                    // 4 v_mul_f32, 5 v_pk_mul_f32, 6 v_fmac_f32 with a literal, 7 v_fma_f32 SGPR operand
__global__ __launch_bounds__(1024) void k_probe(float* out, int iters, unsigned long long* cyc) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 a[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) a[u] = f2{threadIdx.x * 1e-3f + u, u * 0.5f};
  const f2 b = {0.999f, 0.998f}, c = {1e-4f, 2e-4f};
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if constexpr (KIND == 0) {
        float x = a[u].x, y = a[u].y;
        __asm__ volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(b.x), "v"(c.x));
        __asm__ volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(y) : "v"(b.y), "v"(c.y));
        a[u] = f2{x, y};
      } else if constexpr (KIND == 1) {
        __asm__ volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(a[u]) : "v"(b), "v"(c));
      } else if constexpr (KIND == 2) {
        float x = a[u].x, y = a[u].y;
        __asm__ volatile("v_add_f32 %0, %0, %1" : "+v"(x) : "v"(c.x));
        __asm__ volatile("v_add_f32 %0, %0, %1" : "+v"(y) : "v"(c.y));
        a[u] = f2{x, y};
      } else if constexpr (KIND == 3) {
        __asm__ volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a[u]) : "v"(c));
      } else if constexpr (KIND == 4) {
        float x = a[u].x, y = a[u].y;
        __asm__ volatile("v_mul_f32 %0, %0, %1" : "+v"(x) : "v"(b.x));
        __asm__ volatile("v_mul_f32 %0, %0, %1" : "+v"(y) : "v"(b.y));
        a[u] = f2{x, y};
      } else if constexpr (KIND == 5) {
        __asm__ volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(a[u]) : "v"(b));
      } else if constexpr (KIND == 6) {
        float x = a[u].x, y = a[u].y;
        __asm__ volatile("v_fmac_f32 %0, 0x3f7fbe77, %1" : "+v"(x) : "v"(c.x));
        __asm__ volatile("v_fmac_f32 %0, 0x3f7fbe77, %1" : "+v"(y) : "v"(c.y));
        a[u] = f2{x, y};
      } else {
        float x = a[u].x, y = a[u].y;
        __asm__ volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x) : "s"(b.x), "v"(c.x));
        __asm__ volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(y) : "s"(b.y), "v"(c.y));
        a[u] = f2{x, y};
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < 8; ++u) s += a[u].x + a[u].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) atomicAdd(cyc, t1 - t0);
}

template <int KIND>
void run(const char* name, int ncu, float* out, unsigned long long* cyc) {
  const int iters = 4096;
  const int instr_per_iter = (KIND == 1 || KIND == 3 || KIND == 5) ? 8 : 16;
  for (int w = 1; w <= 4; ++w) {
    double cpw = 0;
    for (int pass = 0; pass < 2; ++pass) {
      (void)hipMemset(cyc, 0, 8);
      hipLaunchKernelGGL((k_probe<KIND>), dim3(ncu), dim3(256 * w), 0, 0, out, iters, cyc);
      (void)hipDeviceSynchronize();
      unsigned long long h = 0;
      (void)hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
      cpw = (double)h / ((double)ncu * 4 * w);
    }
    const double instr = (double)iters * instr_per_iter;
    const double lane_ops = (double)iters * 16;  // fp32 ops per lane
    printf("%-14s waves/SIMD %d: %5.2f cyc/instr/wave  %.3f instr/cyc/SIMD  %.3f fp32-op/cyc/SIMD-lane\n",
           name, w, cpw / instr, instr * w / cpw, lane_ops * w / cpw);
  }
}

int main() {
  hipDeviceProp_t pr;
  (void)hipGetDeviceProperties(&pr, 0);
  const int ncu = pr.multiProcessorCount;
  float* out;
  unsigned long long* cyc;
  (void)hipMalloc(&out, 1024 * ncu * sizeof(float));
  (void)hipMalloc(&cyc, 8);
  run<0>("v_fma_f32", ncu, out, cyc);
  run<1>("v_pk_fma_f32", ncu, out, cyc);
  run<2>("v_add_f32", ncu, out, cyc);
  run<3>("v_pk_add_f32", ncu, out, cyc);
  run<4>("v_mul_f32", ncu, out, cyc);
  run<5>("v_pk_mul_f32", ncu, out, cyc);
  run<6>("v_fmac_f32 lit", ncu, out, cyc);
  run<7>("v_fma_f32 sgpr", ncu, out, cyc);
  return 0;
}
