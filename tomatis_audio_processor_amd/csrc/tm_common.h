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
__device__ __forceinline__ cf operator+(cf a, cf b) { return {a.x + b.x, a.y + b.y}; }
__device__ __forceinline__ cf operator-(cf a, cf b) { return {a.x - b.x, a.y - b.y}; }
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
// Scaled DIF network (pending scales).  Every register carries a compile-time
// positive scale sigma (true value = sigma * register).  A twiddle c + i s
// becomes two FMAs in tangent form (sigma *= max(|c|, |s|)), so W8 and every
// other compile-time twiddle lose their multiplies; a butterfly of registers
// with different scales folds their ratio (<= 1) into one FMA per component,
// the same count as the plain add.  The output scales are absorbed by the
// runtime tables the outputs meet next (twiddle tables, gain rows, synthesis
// window), built on the host from the same constexpr plans.
// ---------------------------------------------------------------------------
struct SOp {
  int kind;   // 0 butterfly (a, b) -> (a + b, a - b); 1 general twiddle on a;
              // 2 negate a; 3 multiply a by -i (sg = -1) or +i (sg = +1)
  int a, b;
  int big;    // butterfly: 0 -> a' = a + r b, b' = a - r b; 1 -> a' = r a + b, b' = r a - b
  double r;   // butterfly ratio; twiddle: t (form 0) or ct (form 1)
  int form;   // twiddle: 0 tangent (sigma *= |c|), 1 cotangent (sigma *= |s|)
  int sg;     // twiddle: sign of c (form 0) / of s (form 1); kind 3: -1 => -i
};
constexpr int kMaxSM = 64;
struct SigIn {
  double s[kMaxSM];
};
template <int M>
struct SPlan {
  SOp op[M * 8];
  int n;
  double sig[M];  // scales of the natural-order outputs
};
constexpr double ct_abs(double x) { return x < 0 ? -x : x; }
constexpr SigIn sig_ones() {
  SigIn o{};
  for (int i = 0; i < kMaxSM; ++i) o.s[i] = 1.0;
  return o;
}
template <int M>
constexpr SPlan<M> make_splan(bool inv, SigIn in) {
  SPlan<M> P{};
  double sg[M] = {};
  for (int k = 0; k < M; ++k) sg[k] = in.s[k];
  P.n = 0;
  int st_off[64] = {}, st_m[64] = {};
  int sp = 0;
  st_off[sp] = 0;
  st_m[sp] = M;
  ++sp;
  while (sp > 0) {
    --sp;
    const int off = st_off[sp], m = st_m[sp];
    if (m < 2) continue;
    for (int I = 0; I < m / 2; ++I) {
      const int a = off + I, b = off + I + m / 2;
      SOp o{};
      o.kind = 0;
      o.a = a;
      o.b = b;
      if (sg[a] >= sg[b]) {
        o.big = 0;
        o.r = sg[b] / sg[a];
        sg[b] = sg[a];
      } else {
        o.big = 1;
        o.r = sg[a] / sg[b];
        sg[a] = sg[b];
      }
      P.op[P.n++] = o;
      const int mm = I % m;
      if (mm == 0) continue;
      SOp t{};
      t.a = b;
      if (2 * mm == m) {
        t.kind = 2;
      } else if (4 * mm == m) {
        t.kind = 3;
        t.sg = inv ? 1 : -1;
      } else if (4 * mm == 3 * m) {
        t.kind = 3;
        t.sg = inv ? -1 : 1;
      } else {
        const double c = ct_cos2pi(mm, m);
        const double s = inv ? ct_sin2pi(mm, m) : -ct_sin2pi(mm, m);
        t.kind = 1;
        if (ct_abs(c) >= ct_abs(s)) {
          t.form = 0;
          t.r = s / ct_abs(c);
          t.sg = c > 0 ? 1 : -1;
          sg[b] *= ct_abs(c);
        } else {
          t.form = 1;
          t.r = c / ct_abs(s);
          t.sg = s > 0 ? 1 : -1;
          sg[b] *= ct_abs(s);
        }
      }
      P.op[P.n++] = t;
    }
    st_off[sp] = off + m / 2;  // right half after the left one
    st_m[sp] = m / 2;
    ++sp;
    st_off[sp] = off;
    st_m[sp] = m / 2;
    ++sp;
  }
  for (int K = 0; K < M; ++K) P.sig[K] = sg[ct_bitrev(K, M)];
  return P;
}
template <int M>
constexpr SigIn sig_recip(const SPlan<M>& p) {
  SigIn o = sig_ones();
  for (int k = 0; k < M; ++k) o.s[k] = 1.0 / p.sig[k];
  return o;
}
// forward / inverse plans from unit input scales (their output scales agree:
// they depend on |c|, |s| only), and the inverse over inputs scaled by
// 1 / (forward output scales) -- the inverse first step's input after the
// scaled step-2 twiddle table
template <int M>
inline constexpr SPlan<M> kSPlanF = make_splan<M>(false, sig_ones());
template <int M>
inline constexpr SPlan<M> kSPlanI = make_splan<M>(true, sig_ones());
template <int M>
inline constexpr SPlan<M> kSPlanI1 = make_splan<M>(true, sig_recip<M>(kSPlanF<M>));

template <int M, int W>
__host__ __device__ constexpr const SPlan<M>& splan() {
  if constexpr (W == 0) return kSPlanF<M>;
  else if constexpr (W == 1) return kSPlanI<M>;
  else return kSPlanI1<M>;
}

// forward output scale of DFT_M output k at a runtime index (table set-up only)
template <int M>
__device__ __forceinline__ float sig_at(int k) {
  float r = 1.f;
  sfor<0, M>([&](auto kk) {
    constexpr int K = decltype(kk)::value;
    if (k == K) r = (float)splan<M, 0>().sig[K];
  });
  return r;
}

// DFT of size M over registers v[OFF + i] (natural order in/out) through plan W
// (0 forward, 1 inverse, 2 inverse with scaled inputs); outputs carry
// splan<M, W>().sig.
template <int M, int W, int OFF, int NT>
__device__ __forceinline__ void sdft(cf (&v)[NT]) {
  constexpr const SPlan<M>& PL = splan<M, W>();
  sfor<0, PL.n>([&](auto ii) {
    constexpr SOp o = PL.op[decltype(ii)::value];
    if constexpr (o.kind == 0) {
      const cf A = v[OFF + o.a], B = v[OFF + o.b];
      if constexpr (o.r == 1.0) {
        v[OFF + o.a] = A + B;
        v[OFF + o.b] = A - B;
      } else if constexpr (o.big == 0) {
        constexpr float r = (float)o.r;
        v[OFF + o.a] = {__builtin_fmaf(B.x, r, A.x), __builtin_fmaf(B.y, r, A.y)};
        v[OFF + o.b] = {__builtin_fmaf(B.x, -r, A.x), __builtin_fmaf(B.y, -r, A.y)};
      } else {
        constexpr float r = (float)o.r;
        v[OFF + o.a] = {__builtin_fmaf(A.x, r, B.x), __builtin_fmaf(A.y, r, B.y)};
        v[OFF + o.b] = {__builtin_fmaf(A.x, r, -B.x), __builtin_fmaf(A.y, r, -B.y)};
      }
    } else if constexpr (o.kind == 2) {
      const cf x = v[OFF + o.a];
      v[OFF + o.a] = {-x.x, -x.y};
    } else if constexpr (o.kind == 3) {
      const cf x = v[OFF + o.a];
      if constexpr (o.sg < 0) v[OFF + o.a] = {x.y, -x.x};   // * -i
      else v[OFF + o.a] = {-x.y, x.x};                      // * +i
    } else {
      const cf x = v[OFF + o.a];
      constexpr float t = (float)o.r;
      const float sx = o.sg > 0 ? x.x : -x.x, sy = o.sg > 0 ? x.y : -x.y;
      if constexpr (o.form == 0) {   // |c| [(sc x - t y) + i (sc y + t x)]
        if constexpr (t == 1.0f) v[OFF + o.a] = {sx - x.y, sy + x.x};
        else if constexpr (t == -1.0f) v[OFF + o.a] = {sx + x.y, sy - x.x};
        else v[OFF + o.a] = {__builtin_fmaf(-t, x.y, sx), __builtin_fmaf(t, x.x, sy)};
      } else {                       // |s| [(ct x - ss y) + i (ct y + ss x)]
        v[OFF + o.a] = {__builtin_fmaf(t, x.x, -sy), __builtin_fmaf(t, x.y, sx)};
      }
    }
  });
  cf tt[M];
  sfor<0, M>([&](auto kk) {
    constexpr int K = decltype(kk)::value;
    tt[K] = v[OFF + ct_bitrev(K, M)];
  });
  sfor<0, M>([&](auto kk) {
    constexpr int K = decltype(kk)::value;
    v[OFF + K] = tt[K];
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

__device__ __forceinline__ float opaque_f(float v) {
  float r;
  __asm__ volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(v));
  return r;
}

__device__ __forceinline__ float wave_max(float v) {
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  return v;
}

}  // namespace tdsp
