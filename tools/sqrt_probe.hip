// Exhaustive check (diagnostic): is gfx950's v_sqrt_f32 correctly rounded for
// every float a in [lo, +inf)?  The reference is the neighbour-residual
// correction the fused levels use (lv_sqrt_fast, tm_transform.hip) and, as a
// second opinion, the double-precision sqrt rounded to float (innocuous double
// rounding: 53 >= 2 * 24 + 2).  Also checks the rsq-based one-step sequence.
// build: hipcc --offload-arch=gfx950 -O3 tools/sqrt_probe.hip -o tools/sqrt_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ float fix_nb(float a, float s) {
  const float sd = __int_as_float(__float_as_int(s) - 1);
  const float su = __int_as_float(__float_as_int(s) + 1);
  const float vd = __builtin_fmaf(-sd, s, a), vu = __builtin_fmaf(-su, s, a);
  float m = vd <= 0.f ? sd : s;
  m = vu > 0.f ? su : m;
  return m;
}

__global__ void probe(uint32_t lo, uint32_t hi, unsigned long long* cnt, uint32_t* first) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t b = lo + blockIdx.x * blockDim.x + threadIdx.x; b < hi && b >= lo; b += stride) {
    const float a = __uint_as_float(b);
    const float hw = __builtin_amdgcn_sqrtf(a);
    const float nb = fix_nb(a, hw);
    const float dd = (float)__builtin_sqrt((double)a);
    const float m_hw = hw * hw, m_nb = nb * nb;
    // one-step sequence from rsq: s = a y, e = a - s s, m = s + e (y / 2)
    const float y = __builtin_amdgcn_rsqf(a);
    const float s0 = a * y;
    const float e = __builtin_fmaf(-s0, s0, a);
    const float rq = __builtin_fmaf(e, 0.5f * y, s0);
    if (hw != nb) atomicAdd(cnt + 0, 1ull);
    if (nb != dd) atomicAdd(cnt + 1, 1ull);
    if (m_hw != m_nb) atomicAdd(cnt + 2, 1ull);
    if (rq != nb) atomicAdd(cnt + 3, 1ull);
    if (hw != nb) atomicMin(first, b);
  }
}

int main() {
  unsigned long long* cnt;
  uint32_t* first;
  hipMalloc(&cnt, 4 * sizeof(unsigned long long));
  hipMalloc(&first, 4);
  hipMemset(cnt, 0, 4 * sizeof(unsigned long long));
  hipMemset(first, 0xff, 4);
  const uint32_t lo = 0x0f800000u, hi = 0x7f800000u;  // [2^-96, inf)
  probe<<<4096, 256>>>(lo, hi, cnt, first);
  unsigned long long h[4];
  uint32_t f;
  hipMemcpy(h, cnt, sizeof h, hipMemcpyDeviceToHost);
  hipMemcpy(&f, first, 4, hipMemcpyDeviceToHost);
  printf("inputs %u  hw!=nb %llu  nb!=f64 %llu  hw^2!=nb^2 %llu  rsq-step!=nb %llu  first hw mismatch 0x%08x\n",
         hi - lo, h[0], h[1], h[2], h[3], f);
  return hipDeviceSynchronize() != hipSuccess;
}
