// HBM copy-bandwidth variants (diagnostic for bench.py's roofline.achievable_peak):
// hipcc --offload-arch=gfx950 -O3 tools/copy_probe.hip -o /tmp/copy_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef float f4v __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void k_copy(const f4v* __restrict__ x, f4v* __restrict__ y, long n4) {
  const long stride = (long)gridDim.x * blockDim.x;
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n4; i += U * stride) {
    f4v t[U];
#pragma unroll
    for (int u = 0; u < U; ++u) t[u] = NT ? __builtin_nontemporal_load(x + i + u * stride) : x[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT) __builtin_nontemporal_store(t[u], y + i + u * stride);
      else y[i + u * stride] = t[u];
    }
  }
  for (; i < n4; i += stride) y[i] = x[i];
}
// contiguous chunk per block: block b copies [b*per, (b+1)*per)
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_copy_chunk(const f4v* __restrict__ x, f4v* __restrict__ y, long n4, long per) {
  const long a = (long)blockIdx.x * per, e = a + per < n4 ? a + per : n4;
  for (long i = a + threadIdx.x; i < e; i += 256 * U) {
    f4v t[U];
#pragma unroll
    for (int u = 0; u < U; ++u) if (i + 256 * u < e) t[u] = NT ? __builtin_nontemporal_load(x + i + 256 * u) : x[i + 256 * u];
#pragma unroll
    for (int u = 0; u < U; ++u) if (i + 256 * u < e) { if (NT) __builtin_nontemporal_store(t[u], y + i + 256 * u); else y[i + 256 * u] = t[u]; }
  }
}

int main() {
  const long n4 = 1270080000L / 16;  // C2's input bytes
  f4v *x, *y;
  hipMalloc(&x, n4 * 16);
  hipMalloc(&y, n4 * 16);
  hipMemset(x, 1, n4 * 16);
  hipMemset(y, 0, n4 * 16);
  int ncu = 256;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto timeit = [&](const char* name, auto launch) {
    for (int w = 0; w < 3; ++w) launch();
    hipEventRecord(e0);
    for (int r = 0; r < 10; ++r) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    printf("%-40s %8.1f GB/s\n", name, 2.0 * n4 * 16 * 10 / (ms * 1e-3) / 1e9);
  };
  for (int bpc : {2, 4, 8, 16}) {
    const int g = ncu * bpc;
    char nm[64];
    snprintf(nm, 64, "stride U4 nt  blocks/cu %d", bpc);
    timeit(nm, [&] { hipLaunchKernelGGL((k_copy<4, true>), dim3(g), dim3(256), 0, 0, x, y, n4); });
    snprintf(nm, 64, "stride U4 ld  blocks/cu %d", bpc);
    timeit(nm, [&] { hipLaunchKernelGGL((k_copy<4, false>), dim3(g), dim3(256), 0, 0, x, y, n4); });
    snprintf(nm, 64, "stride U8 nt  blocks/cu %d", bpc);
    timeit(nm, [&] { hipLaunchKernelGGL((k_copy<8, true>), dim3(g), dim3(256), 0, 0, x, y, n4); });
    snprintf(nm, 64, "stride U1 ld  blocks/cu %d", bpc);
    timeit(nm, [&] { hipLaunchKernelGGL((k_copy<1, false>), dim3(g), dim3(256), 0, 0, x, y, n4); });
  }
  for (long per : {4096L, 16384L, 65536L}) {
    const long g = (n4 + per - 1) / per;
    char nm[64];
    snprintf(nm, 64, "chunk %ld U4 nt", per);
    timeit(nm, [&] { hipLaunchKernelGGL((k_copy_chunk<4, true>), dim3(g), dim3(256), 0, 0, x, y, n4, per); });
    snprintf(nm, 64, "chunk %ld U4 ld", per);
    timeit(nm, [&] { hipLaunchKernelGGL((k_copy_chunk<4, false>), dim3(g), dim3(256), 0, 0, x, y, n4, per); });
  }
  hipLaunchKernelGGL((k_copy<1, false>), dim3(n4 / 256), dim3(256), 0, 0, x, y, n4);
  timeit("one float4 per thread (n4/256 blocks)", [&] { hipLaunchKernelGGL((k_copy<1, false>), dim3(n4 / 256), dim3(256), 0, 0, x, y, n4); });
  return 0;
}
