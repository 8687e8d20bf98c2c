// tm_common.h — device-side helpers for the gfx950 STFT-gate-OLA kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

namespace tdsp {

// ---------------------------------------------------------------------------
// compile-time loops and trig (twiddles are folded into the instruction stream)
// ---------------------------------------------------------------------------
template <int I, int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    sfor<I + 1, N>(f);
  }
}

constexpr double kPi = 3.14159265358979323846264338327950288;

constexpr double ct_sin_poly(double x) {  // |x| <= pi/4
  double x2 = x * x, term = x, sum = x;
  for (int n = 1; n < 14; ++n) {
    term *= -x2 / ((2.0 * n) * (2.0 * n + 1.0));
    sum += term;
  }
  return sum;
}
constexpr double ct_cos_poly(double x) {  // |x| <= pi/4
  double x2 = x * x, term = 1.0, sum = 1.0;
  for (int n = 1; n < 14; ++n) {
    term *= -x2 / ((2.0 * n - 1.0) * (2.0 * n));
    sum += term;
  }
  return sum;
}
// cos / sin of 2*pi*m/M with exact octant reduction on the integer m.
constexpr double ct_cos2pi(long m, long M) {
  m %= M;
  if (m < 0) m += M;
  // angle = 2*pi*m/M ; octant o = floor(8m/M), remainder
  long m8 = 8 * m;
  long o = m8 / M;
  double r = (double)(m8 - o * M) / (double)M * (kPi / 4.0);  // in [0, pi/4)
  switch (o) {
    case 0: return ct_cos_poly(r);
    case 1: return ct_sin_poly(kPi / 4.0 - r);
    case 2: return -ct_sin_poly(r);
    case 3: return -ct_cos_poly(kPi / 4.0 - r);
    case 4: return -ct_cos_poly(r);
    case 5: return -ct_sin_poly(kPi / 4.0 - r);
    case 6: return ct_sin_poly(r);
    default: return ct_cos_poly(kPi / 4.0 - r);
  }
}
constexpr double ct_sin2pi(long m, long M) { return ct_cos2pi(m - M / 4, M); }  // M % 4 == 0

// ---------------------------------------------------------------------------
// complex float in registers
// ---------------------------------------------------------------------------
struct cf {
  float x, y;
};
#ifdef TM_PACKED  // complex add/sub as one v_pk_add_f32 (gfx950 packed fp32)
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ cf operator+(cf a, cf b) {
  const f2v r = f2v{a.x, a.y} + f2v{b.x, b.y};
  return {r.x, r.y};
}
__device__ __forceinline__ cf operator-(cf a, cf b) {
  const f2v r = f2v{a.x, a.y} - f2v{b.x, b.y};
  return {r.x, r.y};
}
#else
__device__ __forceinline__ cf operator+(cf a, cf b) { return {a.x + b.x, a.y + b.y}; }
__device__ __forceinline__ cf operator-(cf a, cf b) { return {a.x - b.x, a.y - b.y}; }
#endif
__device__ __forceinline__ cf cmul(cf a, cf w) {  // a * w
  return {__builtin_fmaf(a.x, w.x, -(a.y * w.y)), __builtin_fmaf(a.x, w.y, a.y * w.x)};
}
__device__ __forceinline__ cf cmulc(cf a, cf w) {  // a * conj(w)
  return {__builtin_fmaf(a.x, w.x, a.y * w.y), __builtin_fmaf(a.y, w.x, -(a.x * w.y))};
}
__device__ __forceinline__ cf cscale(cf a, float s) { return {a.x * s, a.y * s}; }

// multiply by W_M^m = exp(-+2*pi*i*m/M) (forward: minus, INV: plus), m,M compile-time
template <int M, int m, bool INV>
__device__ __forceinline__ cf twid(cf v) {
  constexpr int mm = ((m % M) + M) % M;
  if constexpr (mm == 0) {
    return v;
  } else if constexpr (2 * mm == M) {
    return {-v.x, -v.y};
  } else if constexpr (4 * mm == M) {  // fwd: -i ; inv: +i
    if constexpr (INV) return {-v.y, v.x};
    else return {v.y, -v.x};
  } else if constexpr (4 * mm == 3 * M) {  // fwd: +i ; inv: -i
    if constexpr (INV) return {v.y, -v.x};
    else return {-v.y, v.x};
  } else if constexpr (8 * mm == M || 8 * mm == 3 * M || 8 * mm == 5 * M || 8 * mm == 7 * M) {
    constexpr float h = 0.70710678118654752440f;
    constexpr double c = ct_cos2pi(mm, M);
    constexpr double s = INV ? ct_sin2pi(mm, M) : -ct_sin2pi(mm, M);
    // (x + iy)(c + is) with |c| = |s| = h
    constexpr float sc = (c > 0) ? 1.f : -1.f, ss = (s > 0) ? 1.f : -1.f;
    const float a = sc * v.x - ss * v.y;  // c*x - s*y over h
    const float b = ss * v.x + sc * v.y;  // s*x + c*y over h
    return {a * h, b * h};
  } else {
    constexpr float c = (float)ct_cos2pi(mm, M);
    constexpr float s = INV ? (float)ct_sin2pi(mm, M) : (float)-ct_sin2pi(mm, M);
    return {__builtin_fmaf(v.x, c, -(v.y * s)), __builtin_fmaf(v.x, s, v.y * c)};
  }
}

// ---------------------------------------------------------------------------
// In-register radix-2 DIF DFT; output in natural order.  v[OFF + STR*i].
// ---------------------------------------------------------------------------
template <int M, bool INV, int OFF, int STR, int NT>
__device__ __forceinline__ void dif_bitrev(cf (&v)[NT]) {
  if constexpr (M > 1) {
    sfor<0, M / 2>([&](auto ii) {
      constexpr int I = decltype(ii)::value;
      const cf a = v[OFF + I * STR], b = v[OFF + (I + M / 2) * STR];
      v[OFF + I * STR] = a + b;
      v[OFF + (I + M / 2) * STR] = twid<M, I, INV>(a - b);
    });
    dif_bitrev<M / 2, INV, OFF, STR, NT>(v);
    dif_bitrev<M / 2, INV, OFF + (M / 2) * STR, STR, NT>(v);
  }
}

constexpr int ct_bitrev(int k, int M) {
  int r = 0;
  for (int b = 1; b < M; b <<= 1) {
    r = (r << 1) | (k & 1);
    k >>= 1;
  }
  return r;
}

// DFT of size M over registers v[OFF + STR*i], i < M (natural order in/out).
template <int M, bool INV, int OFF, int STR, int NT>
__device__ __forceinline__ void dft(cf (&v)[NT]) {
  dif_bitrev<M, INV, OFF, STR, NT>(v);
  cf t[M];
  sfor<0, M>([&](auto kk) {
    constexpr int K = decltype(kk)::value;
    t[K] = v[OFF + ct_bitrev(K, M) * STR];
  });
  sfor<0, M>([&](auto kk) {
    constexpr int K = decltype(kk)::value;
    v[OFF + K * STR] = t[K];
  });
}

// ---------------------------------------------------------------------------
// misc
// ---------------------------------------------------------------------------
// an opaque copy of a lane value: values derived from it inside a rarely taken
// branch are computed there, instead of being hoisted out of the frame loop by
// LICM and kept live in VGPRs for the whole kernel (the edge-frame addresses
// alone cost 64 VGPRs, i.e. a wave of occupancy)
__device__ __forceinline__ int opaque(int v) {
  int r;
  __asm__ volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(v));
  return r;
}

__device__ __forceinline__ float wave_max(float v) {
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  return v;
}

}  // namespace tdsp
