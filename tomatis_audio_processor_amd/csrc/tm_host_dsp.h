// tm_host_dsp.h — host-side tables shared by the processor plan (tm_kernels.hip)
// and the analysis spectra (tm_analysis.hip): Bluestein chirp tables for a DFT
// of any length, and numpy's pairwise-sum tree over a frame as leaves + a
// postfix program (the device sums leaves, one thread replays the program).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <complex>
#include <vector>

namespace thost {

// in-place radix-2 FFT in double precision (table construction only)
inline void fft_host(std::vector<std::complex<double>>& a) {
  const size_t n = a.size();
  for (size_t i = 1, j = 0; i < n; ++i) {
    size_t bit = n >> 1;
    for (; j & bit; bit >>= 1) j ^= bit;
    j ^= bit;
    if (i < j) std::swap(a[i], a[j]);
  }
  for (size_t len = 2; len <= n; len <<= 1) {
    for (size_t i = 0; i < n; i += len)
      for (size_t k = 0; k < len / 2; ++k) {
        const std::complex<double> w = std::polar(1.0, -2.0 * M_PI * (double)k / (double)len);
        const std::complex<double> u = a[i + k], v = a[i + k + len / 2] * w;
        a[i + k] = u + v;
        a[i + k + len / 2] = u - v;
      }
  }
}

// smallest power of two M >= 2n - 1 (Bluestein's convolution length)
inline int bluestein_m(int n) {
  int M = 1;
  while (M < 2 * n - 1) M <<= 1;
  return M;
}

// chirp b_n = exp(i pi n^2 / N) (n^2 mod 2N exact in integers) and the
// convolution kernel's spectrum H = FFT_M(h) / M, h = b on [0, N) mirrored at
// the top of [0, M); both built in double, stored as float2
inline void bluestein_tables(int N, int M, std::vector<float2>& bf, std::vector<float2>& hf) {
  std::vector<std::complex<double>> bd(N), h(M, 0.0);
  bf.assign(N, make_float2(0.f, 0.f));
  hf.assign(M, make_float2(0.f, 0.f));
  for (int n = 0; n < N; ++n) {
    const int64_t q = ((int64_t)n * n) % (2 * (int64_t)N);
    bd[n] = std::polar(1.0, M_PI * (double)q / (double)N);
    bf[n] = make_float2((float)bd[n].real(), (float)bd[n].imag());
  }
  for (int n = 0; n < N; ++n) h[n] = bd[n];
  for (int n = 1; n < N; ++n) h[M - n] = bd[n];
  fft_host(h);
  for (int k = 0; k < M; ++k)
    hf[k] = make_float2((float)(h[k].real() / M), (float)(h[k].imag() / M));
}

// numpy pairwise_sum's tree over n elements at offset off (loops_utils.h.src:
// blocks of <= 128, split at n/2 rounded down to a multiple of 8): leaves in
// order, and the postfix combination program (>= 0: push that leaf, -1: add)
inline void pw_build(int off, int n, std::vector<int2>& lv, std::vector<int16_t>& prog) {
  if (n <= 128) {
    prog.push_back((int16_t)lv.size());
    lv.push_back(make_int2(off, n));
    return;
  }
  int n2 = n / 2;
  n2 -= n2 % 8;
  pw_build(off, n2, lv, prog);
  pw_build(off + n2, n - n2, lv, prog);
  prog.push_back(-1);
}

// the whole frame of N: numpy's reduction hands the pairwise sum at most
// NPY_BUFSIZE = 8192 elements per inner-loop call and adds the calls' results
// in order
inline void pw_program(int N, std::vector<int2>& lv, std::vector<int16_t>& prog) {
  lv.clear();
  prog.clear();
  for (int c0 = 0; c0 < N; c0 += 8192) {
    pw_build(c0, std::min(8192, N - c0), lv, prog);
    if (c0 > 0) prog.push_back(-1);
  }
}

}  // namespace thost
