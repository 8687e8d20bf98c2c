// tm_lds_fft.h — forward complex FFT of N = 2^k points held in LDS (natural
// order in and out), Stockham autosort: one radix-2 stage when log2 N is odd,
// then radix-4 stages; THREADS threads of the workgroup cooperate, barriers
// between stages.  Twiddles tw[t] = exp(-2 pi i t / N) (float2, any memory).
// lds_dft<M, BLUE>: DFT of any length n in LDS — M = n (power of two) or
// Bluestein's chirp-z over M = 2^k >= 2n - 1 (tables from tm_host_dsp.h).
// Used by the analysis spectra (tm_analysis.hip) and the any-size STFT path
// of the transform unit (tm_transform.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace tlds {

__device__ __forceinline__ float2 cmul(float2 a, float2 w) {
  return make_float2(a.x * w.x - a.y * w.y, a.x * w.y + a.y * w.x);
}
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }

template <int N, int kT = 256>
__device__ __forceinline__ void lds_fft(float2* __restrict__ buf, const float2* __restrict__ tw) {
  constexpr int n = N;
  constexpr int logn = __builtin_ctz(N);
  constexpr int kMaxU2 = (N / 2 + kT - 1) / kT;  // radix-2 butterflies per thread
  constexpr int kMaxU4 = (N / 4 + kT - 1) / kT > 0 ? (N / 4 + kT - 1) / kT : 1;  // radix-4 per thread
  const int t = threadIdx.x;
  int Ns = 1;
  if constexpr (logn & 1) {  // radix-2 stage at Ns = 1: out[2j + q] = a +- b
    const int h = n >> 1;
    float2 o0[kMaxU2], o1[kMaxU2];
#pragma unroll
    for (int u = 0; u < kMaxU2; ++u) {
      const int j = t + u * kT;
      if (j < h) {
        const float2 a = buf[j], b = buf[j + h];
        o0[u] = cadd(a, b);
        o1[u] = csub(a, b);
      }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kMaxU2; ++u) {
      const int j = t + u * kT;
      if (j < h) {
        buf[2 * j] = o0[u];
        buf[2 * j + 1] = o1[u];
      }
    }
    __syncthreads();
    Ns = 2;
  }
  const int q4 = n >> 2;
  for (; Ns < n; Ns <<= 2) {
    const int ts = n / (4 * Ns);  // twiddle index stride
    float2 v[kMaxU4][4];
#pragma unroll
    for (int u = 0; u < kMaxU4; ++u) {
      const int j = t + u * kT;
      if (j < q4) {
        const int k = j & (Ns - 1);
        float2 a0 = buf[j], a1 = buf[j + q4], a2 = buf[j + 2 * q4], a3 = buf[j + 3 * q4];
        if (Ns > 1) {
          a1 = cmul(a1, tw[k * ts]);
          a2 = cmul(a2, tw[2 * k * ts]);
          a3 = cmul(a3, tw[3 * k * ts]);
        }
        const float2 s0 = cadd(a0, a2), s1 = csub(a0, a2);
        const float2 s2 = cadd(a1, a3), s3 = csub(a1, a3);
        v[u][0] = cadd(s0, s2);
        v[u][2] = csub(s0, s2);
        v[u][1] = make_float2(s1.x + s3.y, s1.y - s3.x);  // s1 - i s3
        v[u][3] = make_float2(s1.x - s3.y, s1.y + s3.x);  // s1 + i s3
      }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kMaxU4; ++u) {
      const int j = t + u * kT;
      if (j < q4) {
        const int k = j & (Ns - 1);
        const int d = (j - k) * 4 + k;
        buf[d] = v[u][0];
        buf[d + Ns] = v[u][1];
        buf[d + 2 * Ns] = v[u][2];
        buf[d + 3 * Ns] = v[u][3];
      }
    }
    __syncthreads();
  }
}

__device__ __forceinline__ float2 conjf2(float2 a) { return make_float2(a.x, -a.y); }
__device__ __forceinline__ float2 cmul_conj(float2 a, float2 b) {  // a * conj(b)
  return make_float2(a.x * b.x + a.y * b.y, a.y * b.x - a.x * b.y);
}

// Forward DFT of buf[0, n) in LDS, in place; callers synchronise before.
// BLUE: X[k] = conj(b_k) * IFFT_M(FFT_M(z * conj(b)) * H)[k] with
// b_n = exp(i pi n^2 / n) and H = FFT_M(h) / M (h = b on [0, n), mirrored at
// the top of [0, M)); the inverse FFT is conj(FFT(conj(.))).  buf holds M.
template <int M, bool BLUE, int kT = 256>
__device__ __forceinline__ void lds_dft(float2* buf, int n, const float2* __restrict__ tw,
                                        const float2* __restrict__ bb,
                                        const float2* __restrict__ bh) {
  if constexpr (!BLUE) {
    lds_fft<M, kT>(buf, tw);
  } else {
    for (int i = threadIdx.x; i < M; i += kT)
      buf[i] = i < n ? cmul_conj(buf[i], bb[i]) : make_float2(0.f, 0.f);
    __syncthreads();
    lds_fft<M, kT>(buf, tw);
    for (int k = threadIdx.x; k < M; k += kT) buf[k] = conjf2(cmul(buf[k], bh[k]));
    __syncthreads();
    lds_fft<M, kT>(buf, tw);
    for (int k = threadIdx.x; k < n; k += kT) buf[k] = conjf2(cmul(buf[k], bb[k]));
    __syncthreads();
  }
}

}  // namespace tlds
