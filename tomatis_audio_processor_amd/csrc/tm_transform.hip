// tm_transform.hip — the fused framing -> window -> FFT -> gain -> IFFT ->
// window -> OLA -> normalise (-> limiter) kernels for gfx950, and their
// launchers.  Own translation unit (LLVM's default scheduler: max-ilp,
// max-memory-clause and the iterative strategies measured within 1 %).
// Reference: src/process_tomatis.py:394-406,419-426,451-453 (see tm_kernels.hip).
//
// Build switches (none set in the product build): TM_DEV_ONE_KERNEL,
// TM_DEV_ONLY_2048_512, TM_DEV_WG (one instantiation, 15 s development builds)
// and TM_PROFILE (per-phase cycles of the interior loop).  The alternatives
// measured and rejected in rounds 1-2 (register-resident tables, packed fp32,
// cache policies, flush placement, timing-only variants) are in git history
// and their numbers in DESIGN.md §6.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

#include "tm_common.h"
#include "tm_fft.h"
#include "tm_lds_fft.h"
#include "tm_shared.h"
#include "tm_gate.h"

using namespace tdsp;
using namespace tshared;
using namespace tgate;

#ifndef TM_DEV_WG
#define TM_DEV_WG 256
#endif

namespace {
#ifdef TM_PROFILE  // diagnostic builds: per-phase wave cycles of the interior loop
#define TPROF(i, dep)                                              \
  {                                                                \
    __asm__ volatile("" ::"v"(dep));                               \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();    \
    tacc[i] += t_ - tlast;                                         \
    tlast = t_;                                                    \
  }
#else
#define TPROF(i, dep)
#endif
// gain entry t of the per-lane layout ([rows][N], entry e = lq(i, L) of a row)
// from rows [rows][n_bins]: the bin the forward FFT leaves in register i of lane
// L (mirrored: the gain is real and even), x 1/N (exact) x that register's
// output scale (FX: the single-exchange FFT's layout, fftx_bin)
template <int P, int NR, bool FX>
__device__ __forceinline__ float gain_perm_at(const float* __restrict__ g, int n_bins, int t) {
  constexpr int N = NR * P;
  const int row = t / N, e = t - row * N;
  const int q = e >> 2, L = q % P, i = (q / P) * 4 + (e & 3);
  int b = !FX ? fft_bin<P, NR>(L, i) : (P == 64 ? fftx_bin(L, i) : fftx128_bin(L, i));
  b = (b <= N / 2) ? b : N - b;
  return (g[(int64_t)row * n_bins + b] * (1.0f / (float)N)) * (FX ? sig_at<32>(i) : sig_at<8>(i & 7));
}

// ===========================================================================
// Fused STFT -> gain -> ISTFT -> OLA -> normalise (register OLA, hop % P == 0)
// ===========================================================================

__device__ __forceinline__ float norm_den(float w, int mode) {
  return mode == TOMATIS_NORM_MAX ? fmaxf(w, 1e-8f) : (w + kEps32);
}

// wsum at position rel = p - first_start, frames in ascending order (bit-exact
// with the reference's w_buf)
__device__ float wsum_rel(int64_t rel, int64_t n_frames, int hop, int N, const float* win2) {
  int64_t jhi = floordiv(rel, hop);
  if (jhi > n_frames - 1) jhi = n_frames - 1;
  int64_t jlo = floordiv(rel - N, hop) + 1;
  if (jlo < 0) jlo = 0;
  float w = 0.f;
  for (int64_t j = jlo; j <= jhi; ++j) w = w + win2[rel - j * hop];
  return w;
}

__device__ __forceinline__ int chunk_of(int64_t p, const TomatisStream& S) {
  if (S.n_chunks <= 1 || p < S.chunk_first) return 0;
  const int64_t c = 1 + (p - S.chunk_first) / S.chunk_len;
  return (int)min<int64_t>(c, S.n_chunks - 1);
}

template <int P>
__device__ __forceinline__ void flush_peak(float& pk, int cid, const TomatisStream& S,
                                           uint32_t* peaks, int L, uint32_t* done) {
  const float m = wave_max(pk);  // P > 64: each wave flushes its partial max
  if ((L & 63) == 0) {
    if (m > 0.f) atomicMax(peaks + S.chunk_base + cid, __float_as_uint(m));
    if (done) {  // fused limiter: the max lands before the flush is counted
      __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_fetch_add(done + S.chunk_base + cid, 1u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  pk = 0.f;
}

// fused limiter tail of one wave: wait until every flush of chunk gc has been
// counted (all contributors are dispatched no later than this wave's
// neighbours), then scale this wave's own samples of the chunk.
// prev: the previous pipelined batch's chunk gc (final: no wait; its peaks and
// output from A.peaks_prev / A.yprev)
template <int CH>
__device__ void limit_own(const MainArgs& A, const TomatisStream& S, int gc, int64_t lo,
                          int64_t hi, int lane, bool prev = false) {
  if (!prev) {
    const uint32_t need = A.chunk_need[gc];
    uint32_t got = 0;
    for (int spin = 0; spin < A.lim_spin; ++spin) {
      got = __hip_atomic_load(A.chunk_done + gc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      got = __builtin_amdgcn_readfirstlane(got);
      if (got >= need) break;
      __builtin_amdgcn_s_sleep(32);
    }
    if (got < need) {  // never expected; leaves the chunk unscaled and reports it (the
      // host re-runs the launch unfused, engine.py _finish)
      if (lane == 0) atomicOr(A.err, TOMATIS_ERR_LIMITER_WAIT);
      return;
    }
  }
  const float peak = __uint_as_float(__builtin_amdgcn_readfirstlane(
      __hip_atomic_load((prev ? A.peaks_prev : A.peaks) + gc, __ATOMIC_RELAXED,
                        __HIP_MEMORY_SCOPE_AGENT)));
  if (!(peak > A.limit)) return;
  const float sc = A.limit / peak;
  const int64_t* const rng = prev ? A.chunk_rng_prev : A.chunk_rng;
  const int64_t a = max(lo, rng[2 * gc]), b = min(hi, rng[2 * gc + 1]);
  if (b <= a) return;
  float* base = (prev ? A.yprev : A.y) + S.out_off + a * CH;
  int64_t n = (b - a) * CH;
  // scalar head up to 16-byte alignment, float4 body (16 in flight per lane), tail
  const int head = (int)min<int64_t>(n, (4 - (int)((reinterpret_cast<uintptr_t>(base) >> 2) & 3)) & 3);
  if (lane < head) base[lane] = base[lane] * sc;
  base += head;
  n -= head;
  typedef float f4v __attribute__((ext_vector_type(4)));
  f4v* b4 = reinterpret_cast<f4v*>(base);
  const int64_t n4 = n >> 2;
  constexpr int U = 16;
  for (int64_t i = lane; i < n4; i += 64 * U) {
    f4v t[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + 64 * u < n4) t[u] = __builtin_nontemporal_load(b4 + i + 64 * u);
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + 64 * u < n4) __builtin_nontemporal_store(t[u] * sc, b4 + i + 64 * u);
  }
  const int64_t t0 = n4 << 2;
  if (t0 + lane < n) base[t0 + lane] = base[t0 + lane] * sc;
}

// Pipelined batches: the limiter over partner run pr's output (the previous
// batch's plan, A.runs_prev / A.st_prev) except its blocks [p_lead, p_done),
// which the frame loop scaled; output-relative ranges split over the nw waves
// of the sequence (this is wave w)
template <int CH>
__device__ void partner_tail(const MainArgs& A, int pr, int HOP, int N, int p_lead, int p_done,
                             int nw, int w, int lane) {
  const Run RP = A.runs_prev[pr];
  const TomatisStream SP = A.st_prev[RP.s];
  const int64_t s_kaP = SP.first_start + RP.ka * HOP;
  const int64_t s_lastP = SP.first_start + (RP.kb - 1) * HOP;
  const int64_t endP = SP.out_begin + SP.out_len;
  auto tail = [&](int64_t lo, int64_t hi) {  // output-relative [lo, hi)
    if (lo >= hi) return;
    const int64_t span = hi - lo, per = (span + nw - 1) / nw;
    const int64_t wlo = lo + per * w, whi = min(hi, wlo + per);
    const int c0 = chunk_of(lo + SP.out_begin, SP), c1 = chunk_of(hi - 1 + SP.out_begin, SP);
    for (int c = c0; c <= c1; ++c) {
      if (((A.edge_mask & 1) && c == 0) || ((A.edge_mask & 2) && c == SP.n_chunks - 1)) continue;
      limit_own<CH>(A, SP, SP.chunk_base + c, wlo, whi, lane, true);
    }
  };
  const int64_t hi = min(s_lastP + ((RP.last & 1) ? (int64_t)N : (int64_t)HOP), endP) - SP.out_begin;
  if (p_lead > 0)  // the leading partial blocks
    tail(max(s_kaP, SP.out_begin) - SP.out_begin, min(s_kaP + (int64_t)p_lead * HOP - SP.out_begin, hi));
  tail(max(s_kaP + (int64_t)max(p_done, p_lead) * HOP, SP.out_begin) - SP.out_begin, hi);
}

template <int CH>
__device__ __forceinline__ cf load_cf(const float* xs, int64_t p) {
  if constexpr (CH == 2) {
    const float2 t = *reinterpret_cast<const float2*>(xs + 2 * p);
    return {t.x, t.y};
  } else {
    return {xs[p], 0.f};
  }
}
template <int CH>
__device__ __forceinline__ void store_cf(float* ys, int64_t o, cf v) {
  if constexpr (CH == 2) *reinterpret_cast<float2*>(ys + 2 * o) = make_float2(v.x, v.y);
  else ys[o] = v.x;
}
template <int CH>
__device__ __forceinline__ float cmag(cf v) {
  if constexpr (CH == 2) return fmaxf(fabsf(v.x), fabsf(v.y));
  else return fabsf(v.x);
}

// ---- buffer-resource memory ops: one 32-bit lane offset + SGPR/immediate offsets
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int f32x4 __attribute__((ext_vector_type(4)));  // raw b128 payload
__device__ __forceinline__ __amdgpu_buffer_rsrc_t mk_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
// AUX: cache policy (gfx950: bit 1 = nt, streaming / evict-first)
template <int CH, int AUX = 0>
__device__ __forceinline__ cf bload(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  if constexpr (CH == 2) {
    const u32x2 t = __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, AUX);
    return {__uint_as_float(t.x), __uint_as_float(t.y)};
  } else {
    return {__uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, AUX)), 0.f};
  }
}
template <int CH, int AUX = 0>
__device__ __forceinline__ void bstore(cf v, __amdgpu_buffer_rsrc_t r, int voff, int soff) {
  if constexpr (CH == 2) {
    const u32x2 t = {__float_as_uint(v.x), __float_as_uint(v.y)};
    __builtin_amdgcn_raw_buffer_store_b64(t, r, voff, soff, AUX);
  } else {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v.x), r, voff, soff, AUX);
  }
}
__device__ __forceinline__ float bloadf(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}

// ---------------------------------------------------------------------------
// In-kernel levels (n_fft 2048, hop 256 / 512; src/process_tomatis.py:43-52,
// 369-371).  numpy's frame r is a perfect binary tree over the frame's 16
// leaves of 128 samples (pairwise_sum), and each leaf is 8 sequential chains
// (samples c, c+8, ..., c+120) combined as ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7));
// a hop block is LB = hop/128 whole leaves shared by every frame covering it,
// so each frame adds the leaves of its newest block only.  The block (lane L,
// register j = sample L + 64 j) goes through LDS into chain order (conflict-free
// layout: chain stride 20, leaf stride 160 floats), each chain is summed in
// order by one lane, the 8 chains reduce by DPP, and the frame's 16 leaf sums
// sit in lanes 0..15 of one VGPR (the "window").  Every operation is a plain
// IEEE float32 op in numpy's order (no contraction: bit-identical to k_leaves).
// ---------------------------------------------------------------------------
constexpr int kLvCS = 20, kLvLS = 160;

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, true));
}
constexpr int kDppXor1 = 0xB1, kDppXor2 = 0x4E, kDppHalfMirror = 0x141, kDppRowMirror = 0x140;
template <int N> constexpr int kDppRowShl = 0x100 + N;
template <int N> constexpr int kDppRowShr = 0x110 + N;

// a value the compiler may not look through (no instruction: the empty asm
// only ends FMA contraction and value tracking at this point)
__device__ __forceinline__ float lv_opq(float v) {
  __asm__ volatile("" : "+v"(v));
  return v;
}
// a = mean over channels of x^2 for one sample (CH = 2: L + iR), as numpy's
// frame**2 then mean(axis=1).  This unit compiles with -ffp-contract=fast,
// which lets the backend fuse any multiply-add whatever the source pragmas: the
// squares pass through lv_opq so L^2 + R^2 stays two roundings.
template <int CH>
__device__ __forceinline__ float lv_a(cf v) {
  if constexpr (CH == 2) {
    const float ll = lv_opq(v.x * v.x), rr = lv_opq(v.y * v.y);
    return (ll + rr) * 0.5f;
  } else {
    return v.x * v.x;
  }
}
// sqrtf(a) correctly rounded for a >= 2^-96, 0, +inf or NaN: v_sqrt_f32
// (<= 1 ulp) and one step to the neighbour whose residual says so -- the
// expansion hipcc emits for sqrtf without its small-input scaling and its
// zero / inf fix-up, which these inputs do not need (0: the residuals are NaN /
// -0 and keep 0; +inf: NaN residuals keep +inf)
__device__ __forceinline__ float lv_sqrt_fast(float a) {
  const float s = __builtin_amdgcn_sqrtf(a);
  const float sd = __int_as_float(__float_as_int(s) - 1);
  const float su = __int_as_float(__float_as_int(s) + 1);
  const float vd = __builtin_fmaf(-sd, s, a), vu = __builtin_fmaf(-su, s, a);
  float m = vd <= 0.f ? sd : s;
  m = vu > 0.f ? su : m;
  return m;
}
// any a >= 0 (or NaN): below 2^-96 through a x 2^64 (sqrt scales by exactly
// 2^32, no rounding moves: every m here is normal)
__device__ __forceinline__ float lv_sqrt_any(float a) {
  const bool sc = a < 0x1p-96f;
  const float m = lv_sqrt_fast(sc ? a * 0x1p64f : a);
  return sc ? m * 0x1p-32f : m;
}
// bits(a) - 1 for the tiny test: 0 < a < 2^-96 <=> bits(a) - 1 < bits(2^-96) - 1
// (a >= +0 or NaN here: a sum of squares).  (A v_rsq_f32 form, s = a y,
// m = s + (a - s^2) y / 2, is correctly rounded on every float in [2^-96, inf)
// -- checked exhaustively on gfx950, tools/sqrt_probe.hip -- and two VALU
// cheaper per sample, but it pushed the frame loop into scratch spills and
// measured slower; not used.)
constexpr uint32_t kLvTiny = 0x0f800000u - 1u;

// leaf sums of the hop block in the last SH registers of v; returns them in
// lanes 8 l (l < LB).  scr: this sequence's LDS scratch (>= LB * kLvLS floats).
// A wave whose block holds no 0 < a < 2^-96 (anything but near-silent
// non-zero samples below 2^-47) takes the short sqrt; otherwise the same
// neighbour-residual form with the small-input scaling.
template <int CH, int SH, int NRV>
__device__ __forceinline__ float lv_leaves(const cf (&v)[NRV], float* scr, int L) {
  constexpr int LB = SH / 2;
  float a[SH];
  uint32_t umin = 0xffffffffu;
#pragma unroll
  for (int j = 0; j < SH; ++j) {
    a[j] = lv_a<CH>(v[NRV - SH + j]);
    umin = min(umin, __float_as_uint(a[j]) - 1u);
  }
  auto slot = [&](int j) -> float& {
    return scr[(j >> 1) * kLvLS + (L & 7) * kLvCS + (L >> 3) + 8 * (j & 1)];
  };
  if (__builtin_amdgcn_ballot_w64(umin < kLvTiny) == 0) {
#pragma unroll
    for (int j = 0; j < SH; ++j) {
      const float m = lv_sqrt_fast(a[j]);
      slot(j) = m * m;
    }
  } else {
#pragma unroll
    for (int j = 0; j < SH; ++j) {
      const float m = lv_sqrt_any(a[j]);
      slot(j) = m * m;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int leaf = min(L >> 3, LB - 1);
  const float4* p = reinterpret_cast<const float4*>(scr + leaf * kLvLS + (L & 7) * kLvCS);
  const float4 q0 = p[0], q1 = p[1], q2 = p[2], q3 = p[3];
  float a0 = q0.x;
  a0 = a0 + q0.y; a0 = a0 + q0.z; a0 = a0 + q0.w;
  a0 = a0 + q1.x; a0 = a0 + q1.y; a0 = a0 + q1.z; a0 = a0 + q1.w;
  a0 = a0 + q2.x; a0 = a0 + q2.y; a0 = a0 + q2.z; a0 = a0 + q2.w;
  a0 = a0 + q3.x; a0 = a0 + q3.y; a0 = a0 + q3.z; a0 = a0 + q3.w;
  a0 = a0 + dpp<kDppXor1>(a0);        // lanes c, c^1: r0 + r1 ...
  a0 = a0 + dpp<kDppXor2>(a0);        // (r0 + r1) + (r2 + r3) in lanes 0..3
  a0 = a0 + dpp<kDppHalfMirror>(a0);  // lane 0: + ((r4 + r5) + (r6 + r7)) from lane 7
  // the scratch is reused by the next block / the FFT exchanges: reads done
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return a0;
}

// window of the next frame: drop the oldest block's LB leaves, append the new
// block's (lanes 16 - LB + l <- lane 8 l); FWD false: the previous frame
// (backward scan), prepend at lanes 0..LB-1 and drop the newest
template <int SH, bool FWD>
__device__ __forceinline__ float lv_window(float lw, float nl) {
  constexpr int LB = SH / 2;
  lw = FWD ? dpp<kDppRowShl<LB>>(lw) : dpp<kDppRowShr<LB>>(lw);
#pragma unroll
  for (int l = 0; l < LB; ++l) {
    const int v = __builtin_amdgcn_readlane(__float_as_int(nl), 8 * l);
    __asm__("v_writelane_b32 %0, %1, %2" : "+v"(lw) : "s"(v), "n"(FWD ? 16 - LB + l : l));
  }
  return lw;
}

// frame r from the window: perfect tree over lanes 0..15, mean, + EPS, sqrt
// (k_frame_r's order); wave-uniform
__device__ __forceinline__ float lv_frame_r(float lw) {
  float t = lw + dpp<kDppRowShl<1>>(lw);
  t = t + dpp<kDppRowShl<2>>(t);
  t = t + dpp<kDppRowShl<4>>(t);
  t = t + dpp<kDppRowShl<8>>(t);
  const float tot = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(t)));
  const float mean = tot * (1.0f / 2048.0f);  // exact (numpy divides by n = 2^11)
  return lv_sqrt_fast(lv_opq(mean) + kEps32);  // mean + EPS >= 1e-12 (or NaN / inf)
}

// ---- n_fft 4096: a 32-leaf window ----
// lanes 0..31 hold the frame's leaves in order; FWD: drop the oldest LB, append
// the new block's (lanes 32 - LB + l <- lane 8 l of nl); !FWD (backward
// scan): prepend at lanes 0..LB-1, drop the newest.  The shift crosses the
// 16-lane DPP rows: ds_bpermute.
template <int LB, bool FWD>
__device__ __forceinline__ float lv_window32(float lw, float nl, int lane) {
  const int src = FWD ? min(lane + LB, 63) : max(lane - LB, 0);
  float w = __int_as_float(__builtin_amdgcn_ds_bpermute(src * 4, __float_as_int(lw)));
#pragma unroll
  for (int l = 0; l < LB; ++l) {
    const int v = __builtin_amdgcn_readlane(__float_as_int(nl), 8 * l);
    __asm__("v_writelane_b32 %0, %1, %2" : "+v"(w) : "s"(v), "n"(FWD ? 32 - LB + l : l));
  }
  return w;
}
// frame r from a 32-leaf window: numpy's pairwise tree (two 16-leaf trees as
// lv_frame_r's, then their sum), mean over 4096, + EPS, sqrt; wave-uniform
__device__ __forceinline__ float lv_frame_r32(float lw) {
  float t = lw + dpp<kDppRowShl<1>>(lw);
  t = t + dpp<kDppRowShl<2>>(t);
  t = t + dpp<kDppRowShl<4>>(t);
  t = t + dpp<kDppRowShl<8>>(t);
  const float t0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(t), 0));
  const float t1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(t), 16));
  const float mean = (t0 + t1) * (1.0f / 4096.0f);  // exact (n = 2^12)
  return lv_sqrt_fast(lv_opq(mean) + kEps32);
}
// window / frame r of a W-leaf window (W = n_fft / 128: 16 or 32); LB leaves per block
template <int W, int LB, bool FWD>
__device__ __forceinline__ float lv_win(float lw, float nl, int lane) {
  if constexpr (W == 16) return lv_window<2 * LB, FWD>(lw, nl);
  else return lv_window32<LB, FWD>(lw, nl, lane);
}
template <int W>
__device__ __forceinline__ float lv_r(float lw) {
  if constexpr (W == 16) return lv_frame_r(lw);
  else return lv_frame_r32(lw);
}

// ---- n_fft 4096 in the transform (P = 128: two waves per frame; lane
// l = L & 63 of wave w holds sample 64 w + l of every 128-sample leaf) ----
// per sequence: [leaf q][chain c][position i] (16 positions, chains padded)
constexpr int kL2CS = 20, kL2LS = 8 * kL2CS;
// m^2 of the hop block in the last SH registers of v (leaf q = register
// NRV - SH + q) to scr: chain (64 w + l) & 7, position (64 w + l) >> 3.  The
// same per-sample arithmetic as lv_leaves (the short sqrt unless the wave holds
// a 0 < a < 2^-96); the partner wave writes the other 8 positions of each chain
template <int CH, int SH, int NRV>
__device__ __forceinline__ void lv_put128(const cf (&v)[NRV], float* scr, int l, int w) {
  float a[SH];
  uint32_t umin = 0xffffffffu;
#pragma unroll
  for (int j = 0; j < SH; ++j) {
    a[j] = lv_a<CH>(v[NRV - SH + j]);
    umin = min(umin, __float_as_uint(a[j]) - 1u);
  }
  const int e = 64 * w + l;
  float* const p = scr + (e & 7) * kL2CS + (e >> 3);
  if (__builtin_amdgcn_ballot_w64(umin < kLvTiny) == 0) {
#pragma unroll
    for (int j = 0; j < SH; ++j) {
      const float m = lv_sqrt_fast(a[j]);
      p[j * kL2LS] = m * m;
    }
  } else {
#pragma unroll
    for (int j = 0; j < SH; ++j) {
      const float m = lv_sqrt_any(a[j]);
      p[j * kL2LS] = m * m;
    }
  }
}
// leaf sums of the SH leaves in scr (both waves' lv_put128 ordered before this
// by a pair barrier): lane 8 q holds leaf q -- each lane sums one chain's 16
// positions in order, then the 8 chains as numpy combines its accumulators
// ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)) (lv_leaves' tree)
template <int SH>
__device__ __forceinline__ float lv_chains128(const float* scr, int l) {
  const int q = min(l >> 3, SH - 1);
  const float4* p = reinterpret_cast<const float4*>(scr + q * kL2LS + (l & 7) * kL2CS);
  const float4 q0 = p[0], q1 = p[1], q2 = p[2], q3 = p[3];
  float a0 = q0.x;
  a0 = a0 + q0.y; a0 = a0 + q0.z; a0 = a0 + q0.w;
  a0 = a0 + q1.x; a0 = a0 + q1.y; a0 = a0 + q1.z; a0 = a0 + q1.w;
  a0 = a0 + q2.x; a0 = a0 + q2.y; a0 = a0 + q2.z; a0 = a0 + q2.w;
  a0 = a0 + q3.x; a0 = a0 + q3.y; a0 = a0 + q3.z; a0 = a0 + q3.w;
  a0 = a0 + dpp<kDppXor1>(a0);
  a0 = a0 + dpp<kDppXor2>(a0);
  a0 = a0 + dpp<kDppHalfMirror>(a0);
  return a0;
}

// read-only (for the kernel's lifetime) data through the scalar cache: a
// constant-address-space view makes uniform loads s_load (lgkmcnt-counted)
typedef __attribute__((address_space(4))) const uint32_t cu32;

// Chained gate carries (k_gate_carry marked run r kGateChained): the transfer
// tables of the chained runs from the nearest earlier resolved run r0 up to r,
// applied in run order to carry[r0] (-1, unresolved, stays -1).  A stream's
// first run never chains (its look-back reaches frame 0), so r0 is in r's own
// stream.  Wave-uniform; every value was written by the previous launch.
__device__ int gate_chain_carry(const MainArgs& A, int r) {
  int r0 = r - 1, c = -1;
  while (r0 >= 0 && (c = __builtin_amdgcn_readfirstlane(A.gcarry[r0])) == kGateChained) --r0;
  if (r0 < 0) c = -1;
  const int nst = A.gate_D + 2;
  for (int q = r0 + 1; q <= r && c >= 0; ++q)
    c = __builtin_amdgcn_readfirstlane((int)A.gtf[(int64_t)q * nst + c]);
  return c;
}

// Fused framing -> window -> FFT -> gain -> IFFT -> window -> OLA -> normalise.
// One sequence of P lanes (P/64 waves) processes frames [ka - (rmax-1), kb) of
// one stream and emits the hop block of every frame >= ka.  Lane L register i
// holds stream position s_k + L + P*i; the OLA accumulator for the next frame
// is this frame's registers shifted by SH = hop/P.
// GM: where the gain rows live (per-lane layout).  0: global (L2) only;
// 1: all (<= 2) rows in LDS; 2: the two pure rows A.lds_row[0..1] in LDS, the
// cross-fade lattice rows from global (row is wave-uniform, so is the branch).
// PR: a pipelined batch (MainArgs::yprev): each run also applies the limiter
// to its own slot of the previous batch's output inside its frame loop (its
// "partner": the same run of the previous batch) -- by LDS-DMA in the n_fft
// 2048 interior loop, through VGPRs in the generic loop (n_fft 4096).
// GT: in-kernel levels + gate (MainArgs::gated): each frame's r and state come
// from the frame the kernel has loaded (no separate level pass, no row ids).
template <int P, int NR, int SH, int CH, int GM, bool PF, bool NT, int WG, bool PR = false,
          bool GT = false>
__global__ __launch_bounds__(WG, WG / 256 > 2 ? WG / 256 : 2) void k_stft_ola(MainArgs A) {
#ifdef TM_PROFILE
  const unsigned long long t_k0 = __builtin_amdgcn_s_memtime();
  const unsigned long long rt_k0 = __builtin_amdgcn_s_memrealtime();
#endif
  using G = FftGeo<P, NR>;
  constexpr int N = G::N;
  constexpr int NSEQ = WG / P;
  constexpr int HOP = SH * P;
  constexpr int NC = NR - SH;  // carried accumulator registers
  constexpr int SHQ = (SH + 3) & ~3;  // winv registers padded to a quad
  // single-exchange FFTs (tm_fft.h fftx_*): one wave per frame at n_fft 2048,
  // two at 4096 (fftx128_*: one cross-wave trade per direction)
  constexpr bool FX = kFftX && P == 64 && NR == 32;
  constexpr bool FX2 = kFftX && P == 128 && NR == 32;
  // per sequence: FX one wave's exchange rows; FX2 two waves' rows + the pair
  // counter (cf units)
  constexpr int SEQ_CF = FX ? kXBuf / 2 : (FX2 ? kXBuf + 2 : G::SEQ_LDS);
  constexpr int CTR_CF = FX2 ? kXBuf : G::BUF;  // pair-barrier counter slot
  constexpr bool LT = P == 64 && !FX;  // per-lane step-3 twiddle table
  __shared__ __attribute__((aligned(16))) cf s_twN[NR * P];
  __shared__ __attribute__((aligned(16))) cf s_twP[LT ? 8 * P : P];
  __shared__ __attribute__((aligned(16))) float s_win[N];      // lane-quad layout
  __shared__ __attribute__((aligned(16))) float s_winS[N];     // synthesis, scaled
  __shared__ __attribute__((aligned(16))) float s_winv[SHQ * P];  // lane-quad layout
  __shared__ __attribute__((aligned(16))) cf s_buf[NSEQ][SEQ_CF];
  __shared__ __attribute__((aligned(16))) float s_gain[GM ? 2 * N : 4];
  // PR: one hop block per sequence for the partner rescale (LDS-DMA target;
  // n_fft 4096 has no LDS left and takes the blocks through VGPRs)
  __shared__ __attribute__((aligned(16))) char s_pbuf[PR && P == 64 ? NSEQ * SH * P * CH * 4 : 16];
  // GT at n_fft 4096: per sequence the m^2 of a hop block's leaves (lv_put128)
  __shared__ __attribute__((aligned(16))) float s_lv[GT && P == 128 ? NSEQ * SH * kL2LS : 4];
  for (int i = threadIdx.x; i < NR * P; i += WG) s_twN[i] = A.twN[i];
  if constexpr (LT) {  // [m/2][l][m&1] = W_P^{(l%8)*m}
    for (int i = threadIdx.x; i < 8 * P; i += WG) {
      const int m = 2 * (i / (2 * P)) + (i & 1), l = (i / 2) % P;
      s_twP[i] = cscale(A.twP[((l & 7) * m) & (P - 1)], sig_at<8>(m));
    }
  } else if constexpr (FX2) {  // W_128^{l} (1 - 2 w): wave 1's butterflies are mirrored
    for (int i = threadIdx.x; i < P; i += WG) {
      const cf t = A.twP[i & 63];
      s_twP[i] = (i < 64) ? t : cf{-t.x, -t.y};
    }
  } else {
    for (int i = threadIdx.x; i < P; i += WG) s_twP[i] = A.twP[i];
  }
  for (int e = threadIdx.x; e < N; e += WG) {  // e = lq(i, l)
    const int q = e >> 2, l = q % P, i = (q / P) * 4 + (e & 3);
    s_win[e] = A.win[l + P * i];
    s_winS[e] = A.winS[l + P * i];
  }
  for (int e = threadIdx.x; e < SHQ * P; e += WG) {
    const int q = e >> 2, l = q % P, i = (q / P) * 4 + (e & 3);
    s_winv[e] = (i < SH) ? A.winv[l + P * i] : 0.f;
  }
  if constexpr (GM == 1) {
    const int nr = A.n_rows_lds;
    if (A.graw) {
      for (int i = threadIdx.x; i < nr * N; i += WG) s_gain[i] = gain_perm_at<P, NR, FX>(A.graw, A.g_nb, i);
    } else {
      for (int i = threadIdx.x; i < nr * N; i += WG) s_gain[i] = A.gains[i];
    }
  } else if constexpr (GM == 2) {
    for (int i = threadIdx.x; i < 2 * N; i += WG)
      s_gain[i] = A.gains[(int64_t)A.lds_row[i >= N] * N + (i >= N ? i - N : i)];
  }
  if constexpr (P > 64) {  // pair-barrier counters (tm_fft.h)
    if (threadIdx.x < NSEQ) reinterpret_cast<uint32_t*>(s_buf[threadIdx.x] + CTR_CF)[0] = 0u;
  }
  __syncthreads();
  const float4* const w4 = reinterpret_cast<const float4*>(s_win);
  const float4* const ws4 = reinterpret_cast<const float4*>(s_winS);
#ifdef TM_PROFILE
  const unsigned long long t_k1 = __builtin_amdgcn_s_memtime();
#endif

  const int seq = threadIdx.x / P, L = threadIdx.x % P;
  // wave-uniform run id (readfirstlane: run and stream descriptors load as scalars)
  const int run_loc = __builtin_amdgcn_readfirstlane(blockIdx.x * NSEQ + seq);
  const int run_id = A.run_base + run_loc;
  Run R{0, 0, 0, 0};
  const bool valid = run_loc < A.n_runs;
  if (valid) R = A.runs[run_id];
  if constexpr (P <= 64) {
    if (!valid) return;
  }
  const TomatisStream S = A.st[R.s];
  const int64_t kfirst = max<int64_t>(0, R.ka - (A.rmax - 1));
  const int nit = valid ? (int)(R.kb - kfirst) : 0;
  cf* buf = s_buf[seq];
  const float* xs = A.x + S.in_off;
  float* ys = A.y + S.out_off;
  const int64_t out_end = S.out_begin + S.out_len;
  const float oscale = S.out_scale;
  const float iscale = S.in_scale;

  // ---- in-kernel gate: carry-in state from k_gate_carry ----
  static_assert(!GT || (P == 64 && NR == 32 && (SH == 4 || SH == 8)) ||
                    (P == 128 && NR == 32 && SH == 8),
                "in-kernel levels: n_fft 2048 with hop 256 / 512, n_fft 4096 with hop 1024");
  constexpr int NBLK = NR / SH;  // hop blocks per frame
  // n_fft 4096 (two waves per frame): the leaves of a hop block go through
  // s_lv, the cross-fade alpha (A.gate_xf >= 0) is stepped in-kernel
  constexpr bool GX = GT && P == 128;
  static_assert(!GX || FX2, "n_fft 4096 in-kernel levels: the single-trade FFT's pair counter");
  float lw = 0.f;                // lanes 0..15 (0..31 at 4096): the current frame's leaf sums
  int gid = 0;                   // gate state id (tm_gate.h)
  double alpha = 0.0;            // GX: cross-fade alpha after the previous frame
  if constexpr (GT) {
    gid = __builtin_amdgcn_readfirstlane(A.gcarry[run_id]);
    if (gid == kGateChained) gid = gate_chain_carry(A, run_id);
    if (gid < 0) {  // look-back did not resolve: the host re-runs the two-pass path
      if (L == 0) atomicOr(A.err, TOMATIS_ERR_GATE_CARRY);
      gid = 0;
    }
    if constexpr (GX) {
      if (A.gate_xf >= 0) alpha = A.gacarry[run_id];
    }
  }
  float* const lscr = reinterpret_cast<float*>(buf);  // leaf scratch (free at the frame top)
  // the run's first frame: the leaves of its first NBLK - 1 blocks into the
  // window's last lanes, so the first gate_frame (which appends the newest
  // block) completes that frame's window (the same leaf code, the same samples)
  auto start_window = [&](const cf (&fr)[NR]) -> float {
    float w = 0.f;
    sfor<0, NBLK - 1>([&](auto bb) {
      constexpr int B = decltype(bb)::value;
      w = lv_window<SH, true>(
          w, lv_leaves<CH, SH, SH * (B + 1)>(*reinterpret_cast<const cf(*)[SH * (B + 1)]>(&fr[0]), lscr, L));
    });
    return w;
  };
  // predicate thresholds in SGPRs; the exception lists (numpy log10's
  // non-monotone steps, rarely non-empty) are read from the stream table only
  // when present, so the frame loop does not hold 10 more SGPRs
  const uint32_t g_on = S.on_bits, g_off = S.off_bits;
  const bool g_exc = (S.n_on_exc | S.n_off_exc) != 0;
  // frame k from its r: predicate, state (and alpha); r, state (alpha) of
  // emitted frames stored by lane 0; the gain row
  auto gate_r = [&](float r, int64_t k, bool emit) -> uint32_t {
    // r is wave-uniform: its bits through readfirstlane keep the predicate and
    // the automaton in SGPRs / SALU
    const uint32_t b = __builtin_amdgcn_readfirstlane(__float_as_uint(r));
    uint32_t pr;
    if (g_exc) {
      pr = __builtin_amdgcn_readfirstlane(gate_pred(__uint_as_float(b), A.st[opaque(R.s)]));
    } else {
      pr = ((b & 0x7fffffffu) > 0x7f800000u) ? 0u : ((b >= g_on ? 1u : 0u) | (b <= g_off ? 2u : 0u));
    }
    gid = gate_step(gid, pr, A.gate_D);
    const bool c2 = gid == A.gate_D + 1;
    uint32_t row = c2 ? 1u : 0u;
    if constexpr (GX) {
      // process_tomatis_xfade.py:262-278: alpha toward the state's target, the
      // gain row from alpha (pure rows 0 / 1, lattice rows 2 + m)
      const int xf = A.gate_xf;
      if (xf >= 0) {
        const double tgt = c2 ? 1.0 : 0.0;
        alpha = xf > 0 ? alpha_step(alpha, tgt, A.gate_astep) : tgt;
        row = xfade_row(alpha, xf);
      }
    }
    if (emit && L == 0) {
      const int64_t fo = S.frame_base + k;
      A.r_out[fo] = r;
      A.st_out[fo] = (uint8_t)(c2 ? 2 : 1);
      if constexpr (GX) {
        if (A.gate_xf >= 0) A.a_out[fo] = alpha;
      }
    }
    return row;
  };
  // frame k: leaves of its newest block (the last SH registers of fr), r, gate
  auto gate_frame = [&](const cf (&fr)[NR], int64_t k, bool emit) -> uint32_t {
    lw = lv_window<SH, true>(lw, lv_leaves<CH, SH, NR>(fr, lscr, L));
    return gate_r(lv_frame_r(lw), k, emit);
  };
  // n_fft 4096: lv_put128 of the frame's newest block went to s_lv and a pair
  // barrier ordered both waves' writes before this (both waves read every leaf
  // and step the same gate); the partner overwrites s_lv only after this
  // frame's FFT trades, i.e. after these reads
  const int Lw = L & 63, Wv = __builtin_amdgcn_readfirstlane(L >> 6);
  float* const lv2 = s_lv + (GX ? seq * SH * kL2LS : 0);
  auto gate_frame128 = [&](int64_t k, bool emit) -> uint32_t {
    lw = lv_window32<SH, true>(lw, lv_chains128<SH>(lv2, Lw), Lw);
    return gate_r(lv_frame_r32(lw), k, emit);
  };
  // n_fft 4096, the run's first frame: the leaves of its first NBLK - 1 blocks
  // (two pair barriers per block: written by both waves, read by both)
  uint32_t* const pctr = reinterpret_cast<uint32_t*>(reinterpret_cast<float*>(buf) + 2 * kXBuf);
  auto start_window128 = [&](const cf (&fr)[NR]) {
    lw = 0.f;
    sfor<0, NBLK - 1>([&](auto bb) {
      constexpr int B = decltype(bb)::value;
      lv_put128<CH, SH, SH * (B + 1)>(*reinterpret_cast<const cf(*)[SH * (B + 1)]>(&fr[0]), lv2, Lw, Wv);
      pair_barrier(pctr, A.err);
      lw = lv_window32<SH, true>(lw, lv_chains128<SH>(lv2, Lw), Lw);
      pair_barrier(pctr, A.err);
    });
  };

  if (valid && R.ka == 0 && S.first_start > S.out_begin) {  // adaptive: zeros before frame 0
    for (int64_t p = S.out_begin + L; p < min(S.first_start, out_end); p += P)
      store_cf<CH>(ys, p - S.out_begin, cf{0.f, 0.f});
  }

  // chunk tracking by frame index (host guarantees hop-aligned chunk boundaries)
  const int64_t s_ka = S.first_start + R.ka * HOP;
  int cid = chunk_of(s_ka, S);
  const int cid_first = cid;
  // flush counters only for the in-launch limiter (a pipelined batch limits later)
  uint32_t* const done = (A.limit > 0.f && !A.defer_self) ? A.chunk_done : nullptr;
  int64_t next_chunk_k = INT64_MAX;
  if (S.n_chunks > 1 && cid < S.n_chunks - 1)
    next_chunk_k = (S.chunk_first + (int64_t)cid * S.chunk_len - S.first_start) / HOP;
  const int64_t chunk_k_step = S.n_chunks > 1 ? S.chunk_len / HOP : 0;
  float pk = 0.f;

  cf acc[NC];
#pragma unroll
  for (int i = 0; i < NC; ++i) acc[i] = {0.f, 0.f};

#ifdef TM_PROFILE
  unsigned long long tacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tlast = __builtin_amdgcn_s_memtime();
#endif
  // window -> FFT -> gain row -> IFFT -> window, OLA into the accumulator
  // row_of(): the frame's gain row, asked for after the forward FFT
  auto transform = [&](cf (&v)[NR], auto row_of) {
      // ---- analysis window (x * in_scale first, two roundings as the reference) ----
      if (iscale != 1.0f) {
  #pragma unroll
        for (int n2 = 0; n2 < NR; ++n2) v[n2] = cscale(v[n2], iscale);
      }
  #pragma unroll
      for (int n4 = 0; n4 < NR / 4; ++n4) {
        const float4 w = w4[n4 * P + L];
        v[4 * n4] = cscale(v[4 * n4], w.x);
        v[4 * n4 + 1] = cscale(v[4 * n4 + 1], w.y);
        v[4 * n4 + 2] = cscale(v[4 * n4 + 2], w.z);
        v[4 * n4 + 3] = cscale(v[4 * n4 + 3], w.w);
      }
      TPROF(1, v[NR - 1].x);
      if constexpr (FX) fftx_fwd(v, L, s_twN, s_twP[L & 31], reinterpret_cast<float*>(buf));
      else if constexpr (FX2)
        fftx128_fwd(v, L, s_twN, s_twP[L], s_twP[2 * (L & 31)], reinterpret_cast<float*>(buf), A.err);
      else fft_fwd<P, NR, LT>(v, L, s_twN, s_twP, buf, A.err);
      TPROF(2, v[NR - 1].x);
      if constexpr (GT && P == 64) __builtin_amdgcn_s_setprio(0);  // (raised for the gate)
      // ---- gain row (real, even, 1/N folded in), per-lane layout ----
      const uint32_t row = row_of();
      bool g_lds = GM == 1;
      if constexpr (GM == 2) g_lds = row == A.lds_row[0] || row == A.lds_row[1];
      if (g_lds) {
        const float4* g4 =
            reinterpret_cast<const float4*>(s_gain + ((GM == 1 ? row : row == A.lds_row[1]) ? N : 0));
  #pragma unroll
        for (int n4 = 0; n4 < NR / 4; ++n4) {
          const float4 g = g4[n4 * P + L];
          v[4 * n4] = cscale(v[4 * n4], g.x);
          v[4 * n4 + 1] = cscale(v[4 * n4 + 1], g.y);
          v[4 * n4 + 2] = cscale(v[4 * n4 + 2], g.z);
          v[4 * n4 + 3] = cscale(v[4 * n4 + 3], g.w);
        }
      } else if constexpr (GM != 1) {
        const __amdgpu_buffer_rsrc_t rg = mk_rsrc(A.gains + (int64_t)row * N, N * 4);
  #pragma unroll
        for (int n4 = 0; n4 < NR / 4; ++n4) {
          const f32x4 g = __builtin_amdgcn_raw_buffer_load_b128(rg, L * 16, n4 * P * 16, 0);
          v[4 * n4] = cscale(v[4 * n4], __uint_as_float(g.x));
          v[4 * n4 + 1] = cscale(v[4 * n4 + 1], __uint_as_float(g.y));
          v[4 * n4 + 2] = cscale(v[4 * n4 + 2], __uint_as_float(g.z));
          v[4 * n4 + 3] = cscale(v[4 * n4 + 3], __uint_as_float(g.w));
        }
      }
      TPROF(3, v[NR - 1].x);
      if constexpr (FX) fftx_inv(v, L, s_twN, s_twP[L & 31], reinterpret_cast<float*>(buf));
      else if constexpr (FX2)
        fftx128_inv(v, L, s_twN, s_twP[L], s_twP[2 * (L & 31)], reinterpret_cast<float*>(buf), A.err);
      else fft_inv<P, NR, LT>(v, L, s_twN, s_twP, buf, A.err);
      TPROF(4, v[NR - 1].x);
      // ---- synthesis window (x the inverse FFT's output scales) + register OLA ----
  #pragma unroll
      for (int n4 = 0; n4 < NR / 4; ++n4) {
        const float4 w = ws4[n4 * P + L];
        const float ww[4] = {w.x, w.y, w.z, w.w};
  #pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int i = 4 * n4 + u;
          if (i < NC)
            v[i] = {__builtin_fmaf(v[i].x, ww[u], acc[i].x), __builtin_fmaf(v[i].y, ww[u], acc[i].y)};
          else
            v[i] = cscale(v[i], ww[u]);
        }
      }
  };
  // the first SH registers of an emitted frame: normalise (interior 1/sum w^2),
  // output scale, store at byte offset so of ry, chunk peak
  auto emit_full = [&](const cf (&v)[NR], __amdgpu_buffer_rsrc_t ry, int so) {
    float wv[SHQ];
#pragma unroll
    for (int q = 0; q < SHQ / 4; ++q) {
      const float4 t = reinterpret_cast<const float4*>(s_winv)[q * P + L];
      wv[4 * q] = t.x;
      wv[4 * q + 1] = t.y;
      wv[4 * q + 2] = t.z;
      wv[4 * q + 3] = t.w;
    }
#pragma unroll
    for (int i = 0; i < SH; ++i) {
      const cf o = cscale(cscale(v[i], wv[i]), oscale);
      if constexpr (NT) bstore<CH, 2>(o, ry, L * CH * 4, so + P * i * CH * 4);
      else bstore<CH>(o, ry, L * CH * 4, so + P * i * CH * 4);
      pk = fmaxf(pk, cmag<CH>(o));
    }
  };

  bool fast_run = false;
  if constexpr (P == 64) fast_run = valid && (R.last & kRunInterior);
  int p_done = 0;  // PR: partner blocks [p_lead, p_done) handled in the frame loop
  int p_lead = 0;   // (leading partial output blocks of a stream's first run: tail)
  // PR: k_r2_plan's list of this run's partner blocks (previous batch's output)
  typedef float f4v __attribute__((ext_vector_type(4)));
  constexpr int HOPB = HOP * CH * 4;
  cu32* plist = nullptr;
  int np = 0;
  float* yP = ys;
  if constexpr (PR) {
    if (valid) {
      // partner: this run's slot in the previous batch's output
      const int pr = run_id;
      plist = (cu32*)(A.pieces) + (int64_t)run_loc * 2 * (A.max_pieces + 1);
      np = (int)plist[0];
      if (np > 0) {  // (k_r2_plan lists pieces only for partners pr < n_runs_prev)
        const Run RP = A.runs_prev[pr];
        const TomatisStream SP = A.st_prev[RP.s];
        const int64_t off = SP.out_off + CH * (SP.first_start + RP.ka * HOP - SP.out_begin);
        const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)off);
        const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)off >> 32));
        yP = (A.yprev ? A.yprev : A.y) + (int64_t)(((uint64_t)hi << 32) | lo);
      }
    }
  }
  constexpr bool PL = PR && P == 64;  // the partner's blocks by LDS-DMA (fast loop)
  // list entry of frame it (entry np past the list: empty resource)
  auto pent = [&](int it) { return min(it, np); };
  if (fast_run) {
    // Interior run (host-marked): every frame of [kfirst, kb) reads a full frame
    // and every emitted hop block is a full interior block (no stream edges, no
    // stream tail).  One buffer resource per run for input and for output; the
    // hot loop carries only the frame counter, the chunk walk and the OLA.
    const int nwarm = (int)(R.ka - kfirst);
    const int64_t s0 = S.first_start + kfirst * HOP;
    const __amdgpu_buffer_rsrc_t rx =
        mk_rsrc(xs + CH * s0, (uint32_t)(((int64_t)(nit - 1) * HOP + N) * CH * 4));
    const __amdgpu_buffer_rsrc_t ry =
        mk_rsrc(ys + CH * (s_ka - S.out_begin), (uint32_t)((int64_t)(nit - nwarm) * HOP * CH * 4));
    // gain-row ids through the scalar cache: the aligned 32-bit word holding the
    // frame's u16 id, loaded one frame ahead (s_load: lgkmcnt, so waiting for it
    // never waits for this wave's vector stores as an in-order vmcnt wait would)
    cu32* const rw32 = (cu32*)(A.rows);
    const int64_t fb = S.frame_base + kfirst;
    auto row_word = [&](int it) -> uint32_t { return rw32[(fb + it) >> 1]; };
    auto row_of = [&](uint32_t w, int it) -> uint32_t {
      return ((fb + it) & 1) ? (w >> 16) : (w & 0xffffu);
    };
    // Input pipeline.  Registers 0..NO-1 of frame it+1 are registers SH.. of
    // frame it (L2-resident): they are loaded at the end of frame it, after its
    // transforms and before its stores.  The frame's new hop (registers NO..NR-1,
    // from HBM) is loaded a whole frame earlier.  Every iteration issues the same
    // vector-memory ops in the same order (clamped frame indices; warm-up frames
    // store to a null buffer, which drops the stores), so the vmcnt wait for a
    // frame's input never waits for the previous frame's stores or for the next
    // new hop; and the load destinations are not live during the transforms.
    constexpr int NO = NR - SH;
    auto ld_old = [&](int it, cf (&dst)[NR]) {
      const int so = it * (HOP * CH * 4);
#pragma unroll
      for (int n2 = 0; n2 < NO; ++n2) {  // the frame's first hop is read for the last time (nt)
        if (NT && n2 < SH) dst[n2] = bload<CH, 2>(rx, L * CH * 4, so + P * n2 * CH * 4);
        else dst[n2] = bload<CH>(rx, L * CH * 4, so + P * n2 * CH * 4);
      }
    };
    auto ld_new = [&](int it, cf (&dst)[SH]) {
      const int so = it * (HOP * CH * 4) + P * NO * CH * 4;
#pragma unroll
      for (int j = 0; j < SH; ++j) dst[j] = bload<CH>(rx, L * CH * 4, so + P * j * CH * 4);
    };
    const __amdgpu_buffer_rsrc_t rnull = mk_rsrc(ys, 0u);
    float wv[SHQ];
#pragma unroll
    for (int q = 0; q < SHQ / 4; ++q) {
      const float4 t4 = reinterpret_cast<const float4*>(s_winv)[q * P + L];
      wv[4 * q] = t4.x;
      wv[4 * q + 1] = t4.y;
      wv[4 * q + 2] = t4.z;
      wv[4 * q + 3] = t4.w;
    }
    auto store_out = [&](const cf (&o)[SH], __amdgpu_buffer_rsrc_t r, int so) {
#pragma unroll
      for (int i = 0; i < SH; ++i) {
        if constexpr (NT) bstore<CH, 2>(o[i], r, L * CH * 4, so + P * i * CH * 4);
        else bstore<CH>(o[i], r, L * CH * 4, so + P * i * CH * 4);
      }
    };
    cf v[NR], nh[SH], o[SH];
    // ---- pipelined: rescale the partner's (previous batch) blocks in this loop ----
    // k_r2_plan listed, for this run, the partner's hop blocks to scale (chunks
    // whose final peak exceeds the limit) with their scale, at most
    // one per frame: frame it loads piece it into this sequence's LDS slot by
    // LDS-DMA at its top and scales and stores it at its end (no VGPRs in
    // flight across the transform, which is at its register limit).
    constexpr int BQ = PL ? HOPB / 1024 : 1;  // b128 per lane per block
    static_assert(!PL || HOPB % 1024 == 0, "a hop block is whole b128 per lane");
    // (wave-uniform values made explicit: a VGPR resource or LDS address here
    // becomes a waterfall loop)
    char* const pslot = s_pbuf + (PL ? __builtin_amdgcn_readfirstlane(seq * HOPB) : 0);
    uint32_t rw_nx = GT ? 0u : row_word(0);  // (GT: no row ids)
    {  // frame 0, null stores (the loop's issue pattern), new hop of frame 1
      ld_old(0, v);
      cf t[SH];
      ld_new(0, t);
#pragma unroll
      for (int j = 0; j < SH; ++j) v[NO + j] = t[j];
#pragma unroll
      for (int i = 0; i < SH; ++i) o[i] = cf{0.f, 0.f};
      store_out(o, rnull, 0);
      ld_new(min(1, nit - 1), nh);
    }
    if constexpr (GT) lw = start_window(v);
    for (int it = 0; it < nit; ++it) {
      const bool emit = it >= nwarm;
      uint32_t row;
      if constexpr (GT) {
        // the in-kernel gate is a latency chain (leaf sums through LDS, DPP
        // trees, sqrt, readfirstlane, the SALU automaton): the wave runs it and
        // its forward FFT at raised priority, so the SIMD's other wave fills
        // the gaps instead of holding the issue slots (C2 -3 %, C4 -6 %,
        // quiet C2 -6 %: DESIGN.md §6, profiles/r06/prio/); back to 0 after
        // the forward FFT (transform)
        __builtin_amdgcn_s_setprio(2);
        row = gate_frame(v, kfirst + it, emit);
      } else {
        row = row_of(rw_nx, it);
        rw_nx = row_word(min(it + 1, nit - 1));
      }
      if constexpr (PL) {
        // piece it of the partner -> LDS slot (branch-free: past the list the
        // resource is empty, the load returns zeros and the store drops)
        const int blk = (int)plist[2 + 2 * pent(it)];
        const __amdgpu_buffer_rsrc_t rpl =
            mk_rsrc(yP + (int64_t)blk * (HOP * CH), it < np ? (uint32_t)HOPB : 0u);
#pragma unroll
        for (int u = 0; u < BQ; ++u)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(
              rpl, (__attribute__((address_space(3))) void*)(pslot + u * 1024), 16, L * 16,
              u * 1024, 0, 2);
      }
      TPROF(0, v[0].x);
      transform(v, [&] { return row; });
      TPROF(5, v[NR - 1].x);
      // a frame that starts a new chunk flushes the previous chunk's peak first
      // (pk holds frames < k only)
      if (emit && kfirst + it == next_chunk_k) {
        flush_peak<P>(pk, cid, S, A.peaks, L, done);
        ++cid;
        next_chunk_k = (cid < S.n_chunks - 1) ? next_chunk_k + chunk_k_step : INT64_MAX;
      }
      // outputs of this frame's first hop: interior 1/sum w^2 (per lane, loaded
      // once before the loop), output scale, peak
      float pf = 0.f;
#pragma unroll
      for (int i = 0; i < SH; ++i) {
        o[i] = cscale(cscale(v[i], wv[i]), oscale);
        pf = fmaxf(pf, cmag<CH>(o[i]));
      }
      if (emit) pk = fmaxf(pk, pf);
#pragma unroll
      for (int i = 0; i < NC; ++i) acc[i] = v[i + SH];
      // next frame's input (clamped), then this frame's stores, then the new hop
      // of the frame after next
      ld_old(min(it + 1, nit - 1), v);
      // the arrived new hop moves into the frame here, through opaque copies: a
      // plain assignment lets the loop-carried copy land after the next
      // prefetch's issue, where it waits for that HBM load
#pragma unroll
      for (int j = 0; j < SH; ++j) v[NO + j] = cf{opaque_f(nh[j].x), opaque_f(nh[j].y)};
      store_out(o, emit ? ry : rnull, emit ? (it - nwarm) * (HOP * CH * 4) : 0);
      ld_new(min(it + 2, nit - 1), nh);
      if constexpr (PL) {
        // piece it: scale, store (its LDS-DMA is counted by vmcnt only)
        // behind this frame's critical loads: only ld_old / store_out / ld_new
        // (NO + 2 SH instructions) were issued after the LDS-DMA, so this count
        // waits for the DMA (counted by vmcnt only) and nothing issued later
        constexpr int kAfter = NO + 2 * SH;
        static_assert(kAfter < 63, "vmcnt range");
        __asm__ volatile("s_waitcnt vmcnt(%0)" ::"n"(kAfter) : "memory");
        const int blk = (int)plist[2 + 2 * pent(it)];
        const float sc = __uint_as_float(plist[3 + 2 * pent(it)]);
        const __amdgpu_buffer_rsrc_t rps =
            mk_rsrc(yP + (int64_t)blk * (HOP * CH), it < np ? (uint32_t)HOPB : 0u);
#pragma unroll
        for (int u = 0; u < BQ; ++u) {
          const f4v t = *reinterpret_cast<const f4v*>(pslot + u * 1024 + L * 16) * sc;
          const f32x4 b = {__float_as_uint(t.x), __float_as_uint(t.y), __float_as_uint(t.z),
                           __float_as_uint(t.w)};
          __builtin_amdgcn_raw_buffer_store_b128(b, rps, L * 16, u * 1024, 2);
          // a 16-byte store reads its data VGPRs after issue: one wait state
          // before any VALU write of them (hipcc scheduled the next piece's
          // product into the same registers directly behind the store, and the
          // store wrote the new value for the last lanes; tools/store_hazard.py)
          __builtin_amdgcn_sched_barrier(0);
          __asm__ volatile("s_nop 0");
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      TPROF(6, acc[0].x);
    }
    if constexpr (PL) p_done = (int)(plist[1] & 0xffffffu);  // first block the loop left
#ifdef TM_PROFILE
    if (L == 0) {
      for (int i = 0; i < 7; ++i) atomicAdd(A.prof + i, tacc[i]);
      atomicAdd(A.prof + 15, (unsigned long long)nit);
    }
#endif
  } else {
    // frame loads are software-pipelined one frame ahead (the next frame's HBM/L2
    // latency hides behind this frame's transforms)
    auto load_frame = [&](int64_t kk, cf (&dst)[NR]) {
      const bool lv = valid && (kk < R.kb);
      const int64_t sk = S.first_start + kk * HOP;
      if (lv && sk >= 0 && sk + N <= S.n) {
        const __amdgpu_buffer_rsrc_t rx = mk_rsrc(xs + CH * sk, N * CH * 4);
  #pragma unroll
        for (int n2 = 0; n2 < NR; ++n2) {
          // the frame's first hop is read for the last time: stream it (nt)
          if (NT && n2 < SH) dst[n2] = bload<CH, 2>(rx, L * CH * 4, P * n2 * CH * 4);
          else dst[n2] = bload<CH>(rx, L * CH * 4, P * n2 * CH * 4);
        }
      } else {
        const int Lo = opaque(L);
  #pragma unroll
        for (int n2 = 0; n2 < NR; ++n2) {
          const int64_t p = sk + Lo + P * n2;
          dst[n2] = (lv && p >= 0 && p < S.n) ? load_cf<CH>(xs, p) : cf{0.f, 0.f};
        }
      }
    };
    // gain-row id of a frame: an unconditional load at a clamped index, issued one
    // frame ahead at the top of the previous frame, i.e. before that frame's
    // output stores, so the in-order vmcnt wait for it does not wait for them.
    const int64_t kmax = valid ? R.kb - 1 : 0;
    auto load_row = [&](int64_t kk) -> uint32_t {
      return A.rows[S.frame_base + min(kk, kmax)];
    };
    cf nx[NR];
    uint32_t row_nx = GT ? 0u : load_row(kfirst);  // (GT: no row ids)
    if constexpr (PF) load_frame(kfirst, nx);
    // PR (n_fft 4096: no LDS left for the LDS-DMA slots): piece it of the
    // partner through VGPRs, loaded right after frame it's input, scaled and
    // stored after its transform -- before the frame's own stores, so the wait
    // for it waits for nothing issued later; past the list the resource is
    // empty (zero loads, dropped stores).  Streaming (nt) accesses: the pieces
    // must not evict the frames' overlap from L2
    constexpr bool PV = PR && P > 64;
    constexpr int PQ = PV ? HOPB / (16 * P) : 1;  // b128 per lane per block
    static_assert(!PV || HOPB % (16 * P) == 0, "a hop block is whole b128 per lane");

    if constexpr (GX) {
      // the run's first frame's leaves, before the loop (its pair barriers --
      // volatile asm with a memory clobber -- inside the loop body constrain
      // the scheduling of every iteration)
      if (nit > 0) {
        cf v0[NR];
        load_frame(kfirst, v0);
        start_window128(v0);
      }
    }
    for (int it = 0; it < nit; ++it) {
      const int64_t k = kfirst + it;
      const bool live = valid && (k < R.kb);
      const int64_t s_k = S.first_start + k * HOP;
      uint32_t row = 0;
      if constexpr (!GT) {
        row = __builtin_amdgcn_readfirstlane(live ? row_nx : 0u);
        row_nx = load_row(k + 1);
      }
      cf v[NR];
      if constexpr (PF) {
  #pragma unroll
        for (int n2 = 0; n2 < NR; ++n2) v[n2] = nx[n2];
        if (it + 1 < nit) load_frame(k + 1, nx);
      } else {
        load_frame(k, v);
      }
      // (the piece's loads after the frame's: the in-order wait for the frame's
      // input does not wait for them)
      f32x4 pbk[PQ];
      __amdgpu_buffer_rsrc_t rpp;
      float psc = 1.f;
      if constexpr (PV) {
        const int blk = (int)plist[2 + 2 * pent(it)];
        psc = __uint_as_float(plist[3 + 2 * pent(it)]);
        rpp = mk_rsrc(yP + (int64_t)blk * (HOP * CH), it < np ? (uint32_t)HOPB : 0u);
  #pragma unroll
        for (int u = 0; u < PQ; ++u)
          pbk[u] = __builtin_amdgcn_raw_buffer_load_b128(rpp, L * 16, u * 16 * P, 2);  // (nt)
      }
      if constexpr (GX) {
        // n_fft 4096: the new block's m^2 into s_lv, a pair barrier, then its
        // leaves, r, gate and alpha: the gain row is known before the forward
        // FFT, so its L2 loads issue early (asked for after the FFT, the row
        // exposed their latency every frame)
        lv_put128<CH, SH, NR>(v, lv2, Lw, Wv);
        pair_barrier(pctr, A.err);
        row = gate_frame128(k, live && k >= R.ka);
        transform(v, [&] { return row; });
      } else {
        if constexpr (GT) {
          if (it == 0) lw = start_window(v);
          __builtin_amdgcn_s_setprio(2);  // (as the interior loop: until after the forward FFT)
          row = gate_frame(v, k, live && k >= R.ka);
        }
        transform(v, [&] { return row; });
      }
      if constexpr (PV) {
  #pragma unroll
        for (int u = 0; u < PQ; ++u) {
          const f4v t = f4v{__uint_as_float(pbk[u].x), __uint_as_float(pbk[u].y),
                            __uint_as_float(pbk[u].z), __uint_as_float(pbk[u].w)} * psc;
          const f32x4 b = {__float_as_uint(t.x), __float_as_uint(t.y), __float_as_uint(t.z),
                           __float_as_uint(t.w)};
          __builtin_amdgcn_raw_buffer_store_b128(b, rpp, L * 16, u * 16 * P, 2);  // (nt)
          // one wait state before any VALU write of the store's data VGPRs
          // (tools/store_hazard.py)
          __builtin_amdgcn_sched_barrier(0);
          __asm__ volatile("s_nop 0");
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      if (live && k >= R.ka) {
        if (k == next_chunk_k) {
          flush_peak<P>(pk, cid, S, A.peaks, L, done);
          ++cid;
          next_chunk_k = (cid < S.n_chunks - 1) ? next_chunk_k + chunk_k_step : INT64_MAX;
        }
        const bool full = (s_k >= S.out_begin) && (s_k + HOP <= out_end);
        const bool edge = (k < A.rmax - 1);
        if (full && !edge) {
          emit_full(v, mk_rsrc(ys + CH * (s_k - S.out_begin), HOP * CH * 4), 0);
        } else {
          const int Lo = opaque(L);
  #pragma unroll
          for (int i = 0; i < SH; ++i) {
            const int64_t p = s_k + Lo + P * i;
            if (p >= S.out_begin && p < out_end) {
              const float d = norm_den(wsum_rel(p - S.first_start, S.n_frames, HOP, N, A.win2),
                                       A.norm_mode);
              const cf o = cscale(cf{v[i].x / d, v[i].y / d}, oscale);
              store_cf<CH>(ys, p - S.out_begin, o);
              pk = fmaxf(pk, cmag<CH>(o));
            }
          }
        }
        if ((R.last & 1) && k == R.kb - 1) {  // stream tail after the last frame
          const int Lo = opaque(L);
  #pragma unroll
          for (int i = SH; i < NR; ++i) {
            const int64_t p = s_k + Lo + P * i;
            if (p >= S.out_begin && p < out_end) {
              const float d = norm_den(wsum_rel(p - S.first_start, S.n_frames, HOP, N, A.win2),
                                       A.norm_mode);
              const cf o = cscale(cf{v[i].x / d, v[i].y / d}, oscale);
              store_cf<CH>(ys, p - S.out_begin, o);
              pk = fmaxf(pk, cmag<CH>(o));
            }
          }
        }
      }
  #pragma unroll
      for (int i = 0; i < NC; ++i) acc[i] = v[i + SH];
    }
    if constexpr (PV) {
      p_done = valid ? (int)(plist[1] & 0xffffffu) : 0;
      p_lead = valid ? (int)(plist[1] >> 24) : 0;
    }
  }
  if (valid) flush_peak<P>(pk, cid, S, A.peaks, L, done);
  if (valid && done) {
    // this wave's own output range (stores of frames [ka, kb) and the stream tail)
    const int64_t s_last = S.first_start + (R.kb - 1) * HOP;
    const int64_t lo = max(s_ka, S.out_begin) - S.out_begin;
    const int64_t hi = min(s_last + ((R.last & 1) ? (int64_t)N : (int64_t)HOP), out_end) - S.out_begin;
    // P > 64: both waves of the sequence cover the same range; split it by wave
    const int nw = P / 64, w = L >> 6;
    const int64_t span = hi - lo, per = (span + nw - 1) / nw;
    const int64_t wlo = lo + per * w, whi = min(hi, wlo + per);
    for (int c = cid_first; c <= cid; ++c) {
      // edge chunks (shared with a neighbouring time shard) are scaled after
      // the peak exchange instead (tomatis_apply_limiter_edges)
      if (((A.edge_mask & 1) && c == 0) || ((A.edge_mask & 2) && c == S.n_chunks - 1)) continue;
      limit_own<CH>(A, S, S.chunk_base + c, wlo, whi, L & 63);
    }
  }
  if constexpr (PR) {  // the partner's output not scaled in the frame loop (final, no waits)
    const int pr = valid ? run_id : -1;
    if (pr >= 0 && pr < A.n_runs_prev && A.limit > 0.f)
      partner_tail<CH>(A, pr, HOP, N, p_lead, p_done, P / 64, L >> 6, L & 63);
  }
#ifdef TM_PROFILE
  if (valid && (R.last & kRunInterior) && L == 0) {
    const unsigned long long t_k2 = __builtin_amdgcn_s_memtime();
    const unsigned long long rt_k2 = __builtin_amdgcn_s_memrealtime();
    atomicAdd(A.prof + 7, t_k1 - t_k0);    // prologue (tables -> LDS)
    atomicAdd(A.prof + 8, t_k2 - t_k0);    // wave lifetime
    atomicAdd(A.prof + 9, rt_k2 - rt_k0);  // lifetime in 100 MHz ticks
    atomicAdd(A.prof + 10, 1ull);          // waves
  }
#endif
}

// Pipelined batches: for each run, the hop blocks of the same run of the
// previous batch that its frame loop scales (one per frame): blocks of chunks
// whose final peak exceeds the limit, in order, up to the run's frame count
// (the rest go to its tail).  Scale = limit / peak in float32, as the limiter
// (src/process_tomatis.py:351-355).  any_run: the transform scales pieces in
// its generic loop too (n_fft 4096), so any run takes them, up to the partner's
// first block that is not a full output block; otherwise (n_fft 2048: the
// interior loop only) both runs must be interior.
__global__ __launch_bounds__(64) void k_r2_plan(MainArgs A, uint32_t* __restrict__ out,
                                                int n_zero, int any_run) {
  // one wave per run; lanes take the partner's blocks 64 at a time
  const int t = blockIdx.x, lane = threadIdx.x;
  for (int i = t * 64 + lane; i < n_zero; i += gridDim.x * 64) A.peaks[i] = 0u;
  if (t >= A.n_runs) return;
  uint32_t* o = out + (int64_t)t * 2 * (A.max_pieces + 1);
  const int run = A.run_base + t;
  const int pr = run;  // the same run of the previous batch (its plan's runs)
  int n = 0, stop = 0, lead = 0;
  if (pr >= 0 && pr < A.n_runs_prev &&
      (any_run || ((A.runs_prev[pr].last & kRunInterior) && (A.runs[run].last & kRunInterior)))) {
    const Run R = A.runs[run], RP = A.runs_prev[pr];
    const TomatisStream SP = A.st_prev[RP.s];
    const int hop = A.hop;
    const int nit = (int)(R.kb - max<int64_t>(0, R.ka - (A.rmax - 1)));
    const int cap = min(nit, A.max_pieces);
    const int nb = (int)(RP.kb - RP.ka);
    const int64_t s0 = SP.first_start + RP.ka * hop;
    // leading blocks that start before the output (a stream's first run):
    // skipped here, scaled by the tail
    lead = (int)min<int64_t>(min(nb, 255), max<int64_t>(0, (SP.out_begin - s0 + hop - 1) / hop));
    stop = nb;
    for (int j0 = 0; j0 < nb && j0 < stop; j0 += 64) {
      const int j = j0 + lane;
      bool want = false, halt = false;
      float sc = 1.f;
      if (j < nb) {
        const int64_t sj = s0 + (int64_t)j * hop;
        const int c = chunk_of(sj, SP);
        const int g = SP.chunk_base + c;
        halt = ((A.edge_mask & 1) && c == 0) || ((A.edge_mask & 2) && c == SP.n_chunks - 1) ||
               (j >= lead && (sj < SP.out_begin || sj + hop > SP.out_begin + SP.out_len));
        if (!halt && j >= lead) {
          const float peak = __uint_as_float(A.peaks_prev[g]);
          want = peak > A.limit;
          sc = A.limit / peak;
        }
      }
      // the walk ends at the first block of an edge chunk (time shards) or the
      // first partial output block
      const uint64_t hb = __ballot(halt);
      const int first_halt = hb ? j0 + __builtin_ctzll(hb) : INT_MAX;
      want = want && j < first_halt;
      const uint64_t wb = __ballot(want);
      const int before = __builtin_popcountll(wb & ((1ull << lane) - 1ull));
      if (want && n + before < cap) {
        o[2 + 2 * (n + before)] = (uint32_t)j;
        o[3 + 2 * (n + before)] = __float_as_uint(sc);
      }
      const int cnt = __builtin_popcountll(wb);
      if (n + cnt > cap) {
        // the frame loop is full: the tail takes the rest from the first block left
        const int k = cap - n;  // wanted blocks of this batch that fit
        uint64_t m = wb;
        for (int i = 0; i < k; ++i) m &= m - 1;
        stop = min(stop, j0 + __builtin_ctzll(m));
        n = cap;
        break;
      }
      n += cnt;
      if (first_halt != INT_MAX) stop = min(stop, first_halt);
    }
  }
  if (lane == 0) {  // (stop < 2^24: runs are at most 2^20 frames; lead < 256)
    o[0] = (uint32_t)n;
    o[1] = (uint32_t)stop | ((uint32_t)lead << 24);
  }
}

// Pipelined batches whose previous batch's plan has more runs than this one:
// partner runs [n_runs, n_runs_prev) get the limiter here (one wave each, no
// piece list: the whole run, as a transform's tail does)
template <int CH>
__global__ __launch_bounds__(64) void k_prev_runs(MainArgs A, int N) {
  const int pr = A.n_runs + blockIdx.x;
  if (pr >= A.n_runs_prev || !(A.limit > 0.f)) return;
  partner_tail<CH>(A, pr, A.hop, N, 0, 0, 1, 0, threadIdx.x);
}

// In-kernel gate, part 1 (tomatis_stft_ola_gated): per run, the gate state
// before its first frame kf = max(0, ka - rmax + 1), from which the fused
// kernel continues frame by frame (its leaf window it builds from its own
// first frame's registers).  The gate
// automaton forgets its past at an anchor frame: a frame that is not "on" and
// "off" leaves C1 idle whatever came before, and D + 1 consecutive frames "on"
// and not "off" leave C2 (every pending count matures, C2 stays).  One wave
// per run walks back from kf - 1 computing frame levels exactly as the fused
// kernel (the same leaf / window / tree code, blocks read from HBM, zeros
// outside the stream) until the nearest anchor, frame 0 (the automaton starts
// C1 idle, src/process_tomatis.py:288-289) or kGateLookback frames (then the
// run is left unresolved, carry = -1, and the host falls back to the two-pass
// path); the state then runs forward over the recorded predicates to kf.
// Blocks are prefetched 4 ahead.  n_fft = 64 NR (2048: NR 32, a 16-leaf
// window; 4096: NR 64, 32 leaves), hop = 64 SH.
// Chained runs: a look-back that reaches kc, the first frame of the previous
// run of the same stream, without an anchor needs no more frames -- the state
// before kf is the state before kc (that run's own carry-in) stepped over the
// predicates of frames [kc, kf), which the walk has recorded.  The run then
// stores the automaton's transfer function over those frames (one lane per
// start state: tf[run][s], s < nst = D + 2) and carry = kGateChained; the
// transform's prologue composes them (gate_chain_carry).  Only a run whose
// look-back exceeds kGateLookbackMax frames (or nst > kGateChainStates) stays
// unresolved (carry -1: the host's two-pass fallback).
// Cross-fade (A.gate_xf >= 0, process_tomatis_xfade.py:251-274): the run also
// needs alpha before kf.  J = xf + 2 consecutive frames of one state pin alpha
// to that state's target whatever it was (k_alpha_sync), and frames before 0
// count as C1 with alpha 0.  So at an anchor the walk replays the states
// forward and looks for such a run of equal states among the frames whose
// state it knows; alpha then steps (float64, the reference's operations) from
// there to kf - 1 (acarry).  Without one the walk goes on to an earlier
// anchor (the replay is tried at anchors whose distance has doubled since the
// last try), up to kXfLookback frames; no chaining.
constexpr int kXfLookback = 1024;
template <int CH, int SH, int NR, bool XA>
__global__ __launch_bounds__(64) void k_gate_carry(MainArgs A, int32_t* __restrict__ carry,
                                                   uint16_t* __restrict__ tf,
                                                   double* __restrict__ acarry) {
#ifndef TM_GC_PFD
#define TM_GC_PFD 4
#endif
  constexpr int P = 64, HOP = SH * P, NB = NR / SH, LB = SH / 2, PFD = TM_GC_PFD, W = NR / 2;
  constexpr float kInvN = 1.0f / (64 * NR);
  __shared__ __attribute__((aligned(16))) float scr[LB * kLvLS];
  __shared__ uint8_t prs[kGateLookbackMax];
  const int run = blockIdx.x;
  if (run >= A.n_runs) return;
  const int L = threadIdx.x;
  const Run R = A.runs[run];
  const TomatisStream S = A.st[R.s];
  const int D = A.gate_D;
  const int xf = A.gate_xf;  // XA: cross-fade alpha (xf >= 0)
  constexpr bool xa = XA;
  const int J = xf + 2;
  const double astep = A.gate_astep;
  const int64_t kf = max<int64_t>(0, R.ka - (A.rmax - 1));
  // chain point: the first frame of the previous run of this stream (runs are
  // in stream / frame order); 0 for a stream's first run (the stream start
  // anchors it).  Without a tf table the walk keeps the kGateLookback limit.
  int64_t kc = 0;
  if (run > 0 && A.runs[run - 1].s == R.s) kc = max<int64_t>(0, A.runs[run - 1].ka - (A.rmax - 1));
  const bool can_chain = !xa && tf != nullptr && kc > 0 && kf - kc <= kGateLookbackMax;
  const int cap = xa ? kXfLookback : (can_chain ? kGateLookbackMax : kGateLookback);
  const __amdgpu_buffer_rsrc_t rx =
      mk_rsrc(A.x + S.in_off, (uint32_t)min<int64_t>(S.n * CH * 4, 0x7fffffffll));
  auto load_block = [&](int64_t b, cf (&dst)[SH]) {  // block b of the frame grid
    const int64_t p0 = S.first_start + b * HOP + L;
#pragma unroll
    for (int j = 0; j < SH; ++j)  // negative / past-the-end positions: out of range -> 0
      dst[j] = bload<CH>(rx, (int)(uint32_t)((p0 + 64 * j) * (CH * 4)), 0);
  };
  // block energy (sum of the channel-mean squares) for the fast walk
  auto block_energy = [&](const cf (&b)[SH]) -> float {
    float e = 0.f;
#pragma unroll
    for (int q = 0; q < SH; ++q) e += CH == 2 ? (b[q].x * b[q].x + b[q].y * b[q].y) * 0.5f : b[q].x * b[q].x;
    // wave sum, any order (DPP within 16-lane rows, then the 4 row sums)
    e += dpp<kDppXor1>(e);
    e += dpp<kDppXor2>(e);
    e += dpp<kDppHalfMirror>(e);
    e += dpp<kDppRowMirror>(e);
    const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(e), 0));
    const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(e), 16));
    const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(e), 32));
    const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(e), 48));
    return (r0 + r1) + (r2 + r3);
  };
  // cross-fade: from anchor ak (the state after frame ak is aid; ak = -1:
  // before frame 0, alpha 0 there) over the recorded predicates of frames
  // (ak, kf): the state id and alpha before kf; false when no run of J equal
  // known states pins alpha
  double a_res = 0.0;
  int id_res = 0;
  auto replay_xf = [&](int64_t ak, int aid) -> bool {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    int id = aid, st = (aid == D + 1) ? 2 : 1, rl = 1;
    bool pin = ak < 0 || xf == 0;
    double a = ak < 0 ? 0.0 : (st == 2 ? 1.0 : 0.0);
    for (int64_t k = ak + 1; k < kf; ++k) {
      id = gate_step(id, prs[kf - 1 - k], D);
      const int s2 = (id == D + 1) ? 2 : 1;
      rl = (s2 == st) ? rl + 1 : 1;
      st = s2;
      const double tgt = st == 2 ? 1.0 : 0.0;
      if (pin) {
        a = xf > 0 ? alpha_step(a, tgt, astep) : tgt;
      } else if (rl >= J) {
        pin = true;
        a = tgt;
      }
    }
    id_res = id;
    a_res = a;
    return pin;
  };
  // frame kf - 1 = blocks kf - 1 .. kf + NB - 2: their energies for the fast
  // walk (the exact leaf window only if the exact walk runs: the transform
  // builds its own from its first frame's registers)
  float lw = 0.f;
  float eb[NB];  // fast walk: energies of the current frame's blocks, eb[0] the earliest
  {
    cf b[NB][SH];
#pragma unroll
    for (int i = 0; i < NB; ++i) load_block(kf - 1 + i, b[i]);  // all loads in flight at once
#pragma unroll
    for (int i = 0; i < NB; ++i) eb[i] = block_energy(b[i]);
  }
  int id = 0;
  double alpha = 0.0;
  if (kf > 0) {
    int64_t j = kf - 1;          // the window holds frame j
    int64_t a_k = -2;            // anchor: the state after frame a_k is a_id (-2: none)
    int a_id = 0, on_run = 0, n = 0;
    int next_try = 0;            // cross-fade: replay at an anchor once n >= next_try
    // an anchor at frame ak (state aid after it) ends the walk: always for the
    // standard gate; for the cross-fade only if the replay pins alpha
    auto take = [&](int64_t ak, int aid) -> bool {
      if constexpr (!xa) {
        a_k = ak;
        a_id = aid;
        return true;
      }
      if (ak >= 0 && n < next_try) return false;
      if (replay_xf(ak, aid)) {
        a_k = -4;  // resolved with alpha (id_res, a_res)
        return true;
      }
      next_try = 2 * n;
      return false;
    };
    cf bq[PFD][SH];              // blocks j - 1 - u, prefetched
    sfor<0, PFD>([&](auto uu) { load_block(j - 1 - decltype(uu)::value, bq[decltype(uu)::value]); });
    // Fast walk: the predicate of each frame from an approximate r (block
    // energies summed in any order: within ~1e-5 relative of numpy's pairwise
    // r) decided only when r is more than 0.1 % away from both thresholds.  A
    // frame closer to a threshold (or a NaN, or a stream with exception lists)
    // ends it, and the exact walk below recomputes the look-back from kf - 1.
    bool exact = (S.n_on_exc | S.n_off_exc) != 0;
    if (!exact) {
      const float t_on = __uint_as_float(S.on_bits), t_off = __uint_as_float(S.off_bits);
      constexpr float kM = 1e-3f;
      bool go = true;
      while (go) {
        sfor<0, PFD>([&](auto uu) {
          constexpr int u = decltype(uu)::value;
          if (go) {
            float es = 0.f;
#pragma unroll
            for (int i = 0; i < NB; ++i) es += eb[i];
            const float ra = sqrtf(es * kInvN + kEps32);
            const bool on_s = ra >= t_on * (1.f + kM), non_s = ra < t_on * (1.f - kM);
            const bool off_s = ra <= t_off * (1.f - kM), noff_s = ra > t_off * (1.f + kM);
            if (!(on_s || non_s) || !(off_s || noff_s)) {
              exact = true;  // too close to call
              go = false;
            } else {
              const uint8_t pr = (uint8_t)((on_s ? 1 : 0) | (off_s ? 2 : 0));
              if (L == 0) prs[n] = pr;
              ++n;
              on_run = (on_s && !off_s) ? on_run + 1 : 0;
              if (!on_s && off_s && take(j, 0)) {
                go = false;
              } else if (on_run == D + 1 && take(j + D, D + 1)) {
                go = false;
              } else if (j == 0) {
                go = !take(-1, 0);  // (always resolves)
              } else if (can_chain && j == kc) {
                a_k = -3;  // chained: frames [kc, kf) recorded
                go = false;
              } else if (n >= cap) {
                exact = true;  // let the exact walk decide (and flag) this run
                go = false;
              } else {
#pragma unroll
                for (int i = NB - 1; i > 0; --i) eb[i] = eb[i - 1];
                eb[0] = block_energy(bq[u]);
                load_block(j - 1 - PFD, bq[u]);
                --j;
              }
            }
          }
        });
      }
    }
    if (exact) {  // restart from frame kf - 1 on the exact levels (numpy's r)
      j = kf - 1;
      a_k = -2;
      a_id = 0;
      on_run = 0;
      n = 0;
      next_try = 0;
      {
        cf b[NB][SH];
#pragma unroll
        for (int i = 0; i < NB; ++i) load_block(kf - 1 + i, b[i]);
#pragma unroll
        for (int i = 0; i < NB; ++i) lw = lv_win<W, LB, true>(lw, lv_leaves<CH, SH, SH>(b[i], scr, L), L);
      }
      sfor<0, PFD>([&](auto uu) { load_block(j - 1 - decltype(uu)::value, bq[decltype(uu)::value]); });
    }
    bool more = exact;
    while (more) {
      sfor<0, PFD>([&](auto uu) {
        constexpr int u = decltype(uu)::value;
        if (more) {
          const uint8_t pr = gate_pred(lv_r<W>(lw), S);
          if (L == 0) prs[n] = pr;
          ++n;
          on_run = ((pr & 1) && !(pr & 2)) ? on_run + 1 : 0;
          if (!(pr & 1) && (pr & 2) && take(j, 0)) {
            more = false;  // sync: C1 idle after j
          } else if (on_run == D + 1 && take(j + D, D + 1)) {
            more = false;  // D + 1 frames on: C2 after j + D
          } else if (j == 0) {
            more = !take(-1, 0);  // stream start: C1 idle before frame 0
          } else if (can_chain && j == kc) {
            a_k = -3;  // chained: frames [kc, kf) recorded
            more = false;
          } else if (n >= cap) {
            more = false;  // unresolved
          } else {
            lw = lv_win<W, LB, false>(lw, lv_leaves<CH, SH, SH>(bq[u], scr, L), L);
            load_block(j - 1 - PFD, bq[u]);
            --j;
          }
        }
      });
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (a_k == -4) {
      id = id_res;
      alpha = a_res;
    } else if (a_k == -2) {
      id = -1;
    } else if (a_k == -3) {
      // transfer function over frames [kc, kf): lane s replays from state s
      const int nst = D + 2;
      for (int s0 = 0; s0 < nst; s0 += 64) {
        int t = s0 + L;
        for (int64_t k = kc; k < kf; ++k) t = gate_step(t, prs[kf - 1 - k], D);
        if (s0 + L < nst) tf[(int64_t)run * nst + s0 + L] = (uint16_t)t;
      }
      id = kGateChained;
    } else {
      id = a_id;
      for (int64_t k = a_k + 1; k < kf; ++k) id = gate_step(id, prs[kf - 1 - k], D);
    }
  }
  if (L == 0) {
    carry[run] = id;
    if constexpr (xa) acarry[run] = alpha;
  }
}

// Generic hop: same transform, windowed frame outputs to scratch, then a gather.
template <int P, int NR>
__global__ __launch_bounds__(256, 2) void k_stft_frames(MainArgs A) {
  using G = FftGeo<P, NR>;
  constexpr int N = G::N;
  constexpr int NSEQ = 256 / P;
  __shared__ __attribute__((aligned(16))) cf s_twN[NR * P];
  __shared__ cf s_twP[P];
  __shared__ float s_win[N];
  __shared__ float s_winS[N];
  __shared__ cf s_buf[NSEQ][G::SEQ_LDS];
  for (int i = threadIdx.x; i < NR * P; i += 256) s_twN[i] = A.twN[i];
  for (int i = threadIdx.x; i < P; i += 256) s_twP[i] = A.twP[i];
  for (int i = threadIdx.x; i < N; i += 256) {
    s_win[i] = A.win[i];
    s_winS[i] = A.winS[i];
  }
  if constexpr (P > 64) {  // pair-barrier counters (tm_fft.h)
    if (threadIdx.x < NSEQ) reinterpret_cast<uint32_t*>(s_buf[threadIdx.x] + G::BUF)[0] = 0u;
  }
  __syncthreads();
  const int seq = threadIdx.x / P, L = threadIdx.x % P;
  const int run_id = blockIdx.x * NSEQ + seq;
  Run R{0, 0, 0, 0};
  const bool valid = run_id < A.n_runs;
  if (valid) R = A.runs[run_id];
  if constexpr (P <= 64) {
    if (!valid) return;
  }
  const TomatisStream S = A.st[R.s];
  const int nit = valid ? (int)(R.kb - R.ka) : 0;
  cf* buf = s_buf[seq];
  const float* xs = A.x + S.in_off;
  const int hop = A.hop;
  for (int it = 0; it < nit; ++it) {
    const int64_t k = R.ka + it;
    const bool live = valid && (k < R.kb);
    const int64_t s_k = S.first_start + k * hop;
    cf v[NR];
#pragma unroll
    for (int n2 = 0; n2 < NR; ++n2) {
      const int64_t p = s_k + L + P * n2;
      cf z = {0.f, 0.f};
      if (live && p >= 0 && p < S.n) {
        if (A.ch == 2) z = load_cf<2>(xs, p);
        else z = load_cf<1>(xs, p);
      }
      const float w = s_win[L + P * n2];
      v[n2] = {(z.x * S.in_scale) * w, (z.y * S.in_scale) * w};
    }
    fft_fwd<P, NR>(v, L, s_twN, s_twP, buf, A.err);
    const uint16_t row = live ? A.rows[S.frame_base + k] : 0;
    const float* g = A.gains + (int64_t)row * N;
#pragma unroll
    for (int i = 0; i < NR; ++i) v[i] = cscale(v[i], g[lq<P>(i, L)]);
    fft_inv<P, NR>(v, L, s_twN, s_twP, buf, A.err);
    if (live) {
      cf* dst = A.scratch + (S.frame_base + k) * (int64_t)N;
#pragma unroll
      for (int n2 = 0; n2 < NR; ++n2) dst[L + P * n2] = cscale(v[n2], s_winS[L + P * n2]);
    }
  }
}

// gain rows [rows][n_bins] -> [rows][N] in the per-lane bin layout of fft_fwd,
// mirrored (real even gain) and scaled by 1/N (exact: power of two)
// (FX: the single-exchange FFT's layout, fftx_bin)
template <int P, int NR, bool FX = false>
__global__ void k_gain_perm(const float* __restrict__ g, int n_rows, int n_bins,
                            float* __restrict__ out) {
  constexpr int N = NR * P;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_rows * N) return;
  out[t] = gain_perm_at<P, NR, FX>(g, n_bins, t);
}

// generic-hop OLA gather: one thread per output position (frame order preserved)
__global__ __launch_bounds__(256) void k_ola_gather(MainArgs A, int n_streams,
                                                    const int64_t* __restrict__ pos_base,
                                                    int64_t total, int N) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  // stream lookup (binary search over position prefix)
  int lo = 0, hi = n_streams - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) / 2;
    if (pos_base[mid] <= t) lo = mid;
    else hi = mid - 1;
  }
  const TomatisStream S = A.st[lo];
  const int64_t p = S.out_begin + (t - pos_base[lo]);
  const int hop = A.hop;
  const int64_t rel = p - S.first_start;
  int64_t jhi = floordiv(rel, hop);
  if (jhi > S.n_frames - 1) jhi = S.n_frames - 1;
  int64_t jlo = floordiv(rel - N, hop) + 1;
  if (jlo < 0) jlo = 0;
  float w = 0.f;
  cf acc = {0.f, 0.f};
  for (int64_t j = jlo; j <= jhi; ++j) {
    const int off = (int)(rel - j * hop);
    acc = acc + A.scratch[(S.frame_base + j) * (int64_t)N + off];
    w = w + A.win2[off];
  }
  const float d = norm_den(w, A.norm_mode);
  cf o = {acc.x / d, acc.y / d};
  o = cscale(o, S.out_scale);
  float* ys = A.y + S.out_off;
  const int64_t oi = (p - S.out_begin) * A.ch;
  if (A.ch == 2) *reinterpret_cast<float2*>(ys + oi) = make_float2(o.x, o.y);
  else ys[oi] = o.x;
  const float mag = (A.ch == 2) ? fmaxf(fabsf(o.x), fabsf(o.y)) : fabsf(o.x);
  if (mag > 0.f) atomicMax(A.peaks + S.chunk_base + chunk_of(p, S), __float_as_uint(mag));
}


// ---------------------------------------------------------------------------
// Any-size path: any n_fft in [2, 65536], any hop, 1..128 channels (the
// register kernels above cover n_fft 2048 / 4096 with <= 2 channels).
// Reference: the same per-frame filter, src/process_tomatis.py:394-406 (and the
// adaptive :298-327 / layer2 :155-198 copies), whose np.fft.rfft / irfft take
// any length.  Work item = (frame, channel pair c0, c1): frame of
// (x*in_scale)*win packed as c0 + i c1, forward DFT, real even gain row (1/N
// folded in), inverse as conj(DFT(conj(.))), synthesis window, to scratch; the
// OLA is a per-position gather below.  The DFT is a Stockham FFT of length
// M = n_fft when n_fft is a power of two, otherwise Bluestein's chirp-z form
// over M = 2^k >= 2 n_fft - 1:
//   X[k] = conj(b_k) * IFFT_M(FFT_M(z * conj(b)) * FFT_M(h))[k],
//   b_n = exp(i pi n^2 / N), h = b on [0, N) and mirrored at the top of [0, M).
// M <= 16384 runs in LDS (one workgroup per item); larger M in per-block HBM
// ping-pong buffers (radix-2 Stockham, workgroup barriers between stages).
// ---------------------------------------------------------------------------
__device__ __forceinline__ int stream_of_frame(const TomatisStream* st, int n, int64_t fg) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {  // last stream whose frame_base <= fg (empty streams share a base)
    const int mid = (lo + hi + 1) / 2;
    if (st[mid].frame_base <= fg) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

using tlds::conjf2;
using tlds::cmul_conj;

// forward DFT of buf[0, N) in LDS, in place (callers synchronise before)
template <int M, bool BLUE>
__device__ __forceinline__ void lds_dft(float2* buf, const LdsArgs& A) {
  tlds::lds_dft<M, BLUE>(buf, A.n_fft, A.tw, A.blue_b, A.blue_h);
}

// radix-2 Stockham over HBM buffers a -> b -> a ...; returns the buffer holding
// FFT_m(a) (the workgroup's own buffers; barriers order the stages)
__device__ float2* glb_fft(float2* a, float2* b, int m, const float2* __restrict__ tw) {
  const int h = m >> 1;
  for (int Ns = 1; Ns < m; Ns <<= 1) {
    const int ts = m / (2 * Ns);
    for (int j = threadIdx.x; j < h; j += blockDim.x) {
      const int k = j & (Ns - 1);
      const float2 v0 = a[j];
      float2 v1 = a[j + h];
      if (Ns > 1) v1 = tlds::cmul(v1, tw[k * ts]);
      const int d = (j - k) * 2 + k;
      b[d] = tlds::cadd(v0, v1);
      b[d + Ns] = tlds::csub(v0, v1);
    }
    __syncthreads();
    float2* t = a;
    a = b;
    b = t;
  }
  return a;
}

// forward DFT of w0[0, N) (w0, w1: the workgroup's two M-element buffers);
// returns the buffer holding the result
__device__ float2* glb_dft(float2* w0, float2* w1, const LdsArgs& A) {
  const int N = A.n_fft, M = A.M;
  if (!A.blue) return glb_fft(w0, w1, M, A.tw);
  for (int n = threadIdx.x; n < M; n += blockDim.x)
    w0[n] = n < N ? cmul_conj(w0[n], A.blue_b[n]) : make_float2(0.f, 0.f);
  __syncthreads();
  float2* r = glb_fft(w0, w1, M, A.tw);
  for (int k = threadIdx.x; k < M; k += blockDim.x) r[k] = conjf2(tlds::cmul(r[k], A.blue_h[k]));
  __syncthreads();
  float2* o = (r == w0) ? w1 : w0;
  r = glb_fft(r, o, M, A.tw);
  for (int k = threadIdx.x; k < N; k += blockDim.x) r[k] = conjf2(tlds::cmul(r[k], A.blue_b[k]));
  __syncthreads();
  return r;
}

struct FrameItem {
  TomatisStream S;
  int64_t fg, s_k;
  int c0, c1;
  bool has1;
};
__device__ __forceinline__ FrameItem frame_item(const LdsArgs& A, int64_t fg, int pair) {
  FrameItem it;
  it.S = A.st[stream_of_frame(A.st, A.n_streams, fg)];
  it.fg = fg;
  it.s_k = it.S.first_start + (fg - it.S.frame_base) * A.hop;
  it.c0 = 2 * pair;
  it.c1 = it.c0 + 1;
  it.has1 = it.c1 < A.ch;
  return it;
}
__device__ __forceinline__ void load_frame(const LdsArgs& A, const FrameItem& it, float2* buf) {
  const int ch = A.ch, N = A.n_fft;
  const float* xs = A.x + it.S.in_off;
  const float isc = it.S.in_scale;
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    const int64_t p = it.s_k + i;
    const bool in = p >= 0 && p < it.S.n;
    float a = in ? xs[p * ch + it.c0] : 0.f;
    float b = (in && it.has1) ? xs[p * ch + it.c1] : 0.f;
    const float w = A.win[i];
    a = (a * isc) * w;  // x * in_scale first, then the window: two roundings as the reference
    b = (b * isc) * w;
    buf[i] = make_float2(a, b);
  }
}
// spectrum -> conj(X * g / N) for the inverse pass
__device__ __forceinline__ void apply_gain(const LdsArgs& A, const FrameItem& it, float2* buf) {
  const int N = A.n_fft;
  const uint16_t row = A.rows[it.fg];
  const float* g = A.gains + (int64_t)row * A.n_bins;
  const float inv_n = 1.0f / (float)N;
  for (int b = threadIdx.x; b < N; b += blockDim.x) {
    const float gk = g[b <= N / 2 ? b : N - b] * inv_n;
    const float2 v = buf[b];
    buf[b] = make_float2(v.x * gk, -(v.y * gk));
  }
}
__device__ __forceinline__ void store_frame(const LdsArgs& A, const FrameItem& it, const float2* buf) {
  const int ch = A.ch, N = A.n_fft;
  float* out = A.scratch + it.fg * (int64_t)N * ch;
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    const float2 v = buf[i];
    const float w = A.win[i];
    out[(int64_t)i * ch + it.c0] = v.x * w;
    if (it.has1) out[(int64_t)i * ch + it.c1] = -v.y * w;
  }
}

template <int M, bool BLUE>
__global__ __launch_bounds__(256) void k_stft_lds(LdsArgs A) {
  __shared__ float2 buf[M];
  const FrameItem it = frame_item(A, blockIdx.x, blockIdx.y);
  load_frame(A, it, buf);
  __syncthreads();
  lds_dft<M, BLUE>(buf, A);
  apply_gain(A, it, buf);
  __syncthreads();
  lds_dft<M, BLUE>(buf, A);
  store_frame(A, it, buf);
}

// M > kLdsMaxM: blocks walk the (frame, pair) items; each owns two M-element
// HBM buffers
__global__ __launch_bounds__(1024) void k_stft_glb(LdsArgs A) {
  const int npair = (A.ch + 1) / 2;
  const int64_t items = A.total_frames * npair;
  float2* w0 = A.work + (int64_t)blockIdx.x * 2 * A.M;
  float2* w1 = w0 + A.M;
  for (int64_t t = blockIdx.x; t < items; t += gridDim.x) {
    const FrameItem it = frame_item(A, t / npair, (int)(t % npair));
    load_frame(A, it, w0);
    __syncthreads();
    float2* r = glb_dft(w0, w1, A);
    apply_gain(A, it, r);
    __syncthreads();
    r = glb_dft(r, r == w0 ? w1 : w0, A);
    store_frame(A, it, r);
    __syncthreads();
  }
}

// OLA gather of the any-size path: one thread per output position and group of
// up to 8 channels (grid.y); frames summed in ascending order (the reference's
// accumulation order), sum w^2 likewise, normalise, output scale, chunk peak.
__global__ __launch_bounds__(256) void k_ola_gather_lds(LdsArgs A) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= A.total_out) return;
  int lo = 0, hi = A.n_streams - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) / 2;
    if (A.pos_base[mid] <= t) lo = mid;
    else hi = mid - 1;
  }
  const TomatisStream S = A.st[lo];
  const int64_t p = S.out_begin + (t - A.pos_base[lo]);
  const int hop = A.hop, N = A.n_fft, ch = A.ch;
  const int cg = 8 * blockIdx.y, nc = min(8, ch - cg);
  const int64_t rel = p - S.first_start;
  int64_t jhi = floordiv(rel, hop);
  if (jhi > S.n_frames - 1) jhi = S.n_frames - 1;
  int64_t jlo = floordiv(rel - N, hop) + 1;
  if (jlo < 0) jlo = 0;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float w = 0.f;
  for (int64_t j = jlo; j <= jhi; ++j) {
    const int off = (int)(rel - j * hop);
    const float* src = A.scratch + ((S.frame_base + j) * (int64_t)N + off) * ch + cg;
#pragma unroll
    for (int c = 0; c < 8; ++c)
      if (c < nc) acc[c] = acc[c] + src[c];
    w = w + A.win2[off];
  }
  const float d = norm_den(w, A.norm_mode);
  float* ys = A.y + S.out_off + (p - S.out_begin) * ch + cg;
  float mag = 0.f;
#pragma unroll
  for (int c = 0; c < 8; ++c)
    if (c < nc) {
      const float o = (acc[c] / d) * S.out_scale;
      ys[c] = o;
      mag = fmaxf(mag, fabsf(o));
    }
  if (mag > 0.f) atomicMax(A.peaks + S.chunk_base + chunk_of(p, S), __float_as_uint(mag));
}

template <int P, int NR, int SH, bool PF, bool NT, int WG>
void launch_main_pf(const MainArgs& A, int ch, hipStream_t s) {
  // n_fft 4096 keeps its gain rows in L2: two LDS windows (analysis, scaled
  // synthesis) + 4 sequences' exchange rows leave no room for 32 KB of gains
  // (per-frame gain reads measured off the critical path, C3)
  constexpr bool kNoLdsGains = P == 128 && NR == 32;
  const int gm = kNoLdsGains ? 0 : (A.n_rows_lds > 0 ? (A.lds_mixed ? 2 : 1) : 0);
  const dim3 g((A.n_runs + WG / P - 1) / (WG / P)), b(WG);
  if constexpr (P == 64 && (SH == 4 || SH == 8)) {
    if (A.gated) {  // in-kernel levels + gate (two-row tables: gm == 1, host-checked)
      if (A.yprev) {
        if constexpr (WG == 512 && SH <= 8) {
          if (ch == 2)
            hipLaunchKernelGGL((k_stft_ola<P, NR, SH, 2, 1, PF, NT, WG, true, true>), g, b, 0, s, A);
          else
            hipLaunchKernelGGL((k_stft_ola<P, NR, SH, 1, 1, PF, NT, WG, true, true>), g, b, 0, s, A);
        }
      } else if (ch == 2) {
        hipLaunchKernelGGL((k_stft_ola<P, NR, SH, 2, 1, PF, NT, WG, false, true>), g, b, 0, s, A);
      } else {
        hipLaunchKernelGGL((k_stft_ola<P, NR, SH, 1, 1, PF, NT, WG, false, true>), g, b, 0, s, A);
      }
      return;
    }
  }
  if constexpr (P == 64 && WG == 512 && SH <= 8) {  // (LDS slots: the host limits PR to hop <= 512)
    if (A.yprev) {  // pipelined batch (LDS gain rows: gm 1, or gm 2 at hop 512)
      if constexpr (SH == 8) {
        // pipelined adaptive batches (cross-fade lattice: the pure rows in LDS)
        if (gm == 2) {
          if (ch == 2) hipLaunchKernelGGL((k_stft_ola<P, NR, SH, 2, 2, PF, NT, WG, true>), g, b, 0, s, A);
          else hipLaunchKernelGGL((k_stft_ola<P, NR, SH, 1, 2, PF, NT, WG, true>), g, b, 0, s, A);
          return;
        }
      }
      if (ch == 2) hipLaunchKernelGGL((k_stft_ola<P, NR, SH, 2, 1, PF, NT, WG, true>), g, b, 0, s, A);
      else hipLaunchKernelGGL((k_stft_ola<P, NR, SH, 1, 1, PF, NT, WG, true>), g, b, 0, s, A);
      return;
    }
  }
  if constexpr (P == 128 && NR == 32 && WG == 512 && SH == 8) {
    if (A.gated) {  // in-kernel levels + gate (+ cross-fade alpha), n_fft 4096, hop 1024
      if (A.yprev) {
        if (ch == 2) hipLaunchKernelGGL((k_stft_ola<P, NR, SH, 2, 0, PF, NT, WG, true, true>), g, b, 0, s, A);
        else hipLaunchKernelGGL((k_stft_ola<P, NR, SH, 1, 0, PF, NT, WG, true, true>), g, b, 0, s, A);
      } else if (ch == 2) {
        hipLaunchKernelGGL((k_stft_ola<P, NR, SH, 2, 0, PF, NT, WG, false, true>), g, b, 0, s, A);
      } else {
        hipLaunchKernelGGL((k_stft_ola<P, NR, SH, 1, 0, PF, NT, WG, false, true>), g, b, 0, s, A);
      }
      return;
    }
  }
  if constexpr (P == 128 && NR == 32 && WG == 512 && SH <= 8) {
    if (A.yprev) {  // pipelined batch, n_fft 4096 (gain rows in L2; partner blocks in VGPRs)
      if (ch == 2) hipLaunchKernelGGL((k_stft_ola<P, NR, SH, 2, 0, PF, NT, WG, true>), g, b, 0, s, A);
      else hipLaunchKernelGGL((k_stft_ola<P, NR, SH, 1, 0, PF, NT, WG, true>), g, b, 0, s, A);
      return;
    }
  }
#ifdef TM_DEV_ONE_KERNEL  // dev/asm studies: one instantiation (stereo, LDS gains)
  (void)gm;
  (void)ch;
  hipLaunchKernelGGL((k_stft_ola<P, NR, SH, 2, 1, PF, NT, WG>), g, b, 0, s, A);
#else
  if constexpr (kNoLdsGains) {
    if (ch == 2) hipLaunchKernelGGL((k_stft_ola<P, NR, SH, 2, 0, PF, NT, WG>), g, b, 0, s, A);
    else hipLaunchKernelGGL((k_stft_ola<P, NR, SH, 1, 0, PF, NT, WG>), g, b, 0, s, A);
  } else if (ch == 2) {
    if (gm == 1) hipLaunchKernelGGL((k_stft_ola<P, NR, SH, 2, 1, PF, NT, WG>), g, b, 0, s, A);
    else if (gm == 2) hipLaunchKernelGGL((k_stft_ola<P, NR, SH, 2, 2, PF, NT, WG>), g, b, 0, s, A);
    else hipLaunchKernelGGL((k_stft_ola<P, NR, SH, 2, 0, PF, NT, WG>), g, b, 0, s, A);
  } else {
    if (gm == 1) hipLaunchKernelGGL((k_stft_ola<P, NR, SH, 1, 1, PF, NT, WG>), g, b, 0, s, A);
    else if (gm == 2) hipLaunchKernelGGL((k_stft_ola<P, NR, SH, 1, 2, PF, NT, WG>), g, b, 0, s, A);
    else hipLaunchKernelGGL((k_stft_ola<P, NR, SH, 1, 0, PF, NT, WG>), g, b, 0, s, A);
  }
#endif
}
template <int P, int NR, int SH>
void launch_main(const MainArgs& A, int ch, int wg, hipStream_t s) {
  // frame prefetch pays for NR = 16 (2 waves/SIMD kept); NR = 32 is register-bound.
  // Streaming (nt) hints on last-use input and on output keep the frame overlap
  // resident in L2 (FETCH_SIZE 4.5 -> 1.8 GB per C2 launch at P = 64).
  // Workgroup size: the LDS tables (twiddles, window, gain rows) are per block,
  // so wider blocks share them among more sequences and lift the LDS-bound
  // occupancy (see transform_wg).
  // P = 64: the interior loop pipelines its own input; PF only affects the
  // generic edge loop, where it stays off (register-bound).
  constexpr bool PF = NR == 16;
#ifdef TM_DEV_ONE_KERNEL
  (void)wg;
  return launch_main_pf<P, NR, SH, false, true, TM_DEV_WG>(A, ch, s);
#endif
  if constexpr (P == 64) {
    // single-exchange FFT: 8.5 KB of exchange rows per sequence, so the tables
    // are shared by 8 sequences (one 512-thread block per CU).  Otherwise a
    // pipelined batch takes 512-thread blocks (the per-sequence LDS slots of
    // the partner rescale fit once per CU)
    if constexpr (kFftX) {
      (void)wg;
      return launch_main_pf<P, NR, SH, false, true, 512>(A, ch, s);
    } else {
      if (wg == 512 || A.yprev) return launch_main_pf<P, NR, SH, false, true, 512>(A, ch, s);
      return launch_main_pf<P, NR, SH, false, true, 256>(A, ch, s);
    }
  }
  if constexpr (P == 128 && NR == 32) {
    if (wg == 512) return launch_main_pf<P, NR, SH, PF, true, 512>(A, ch, s);
  }
  if constexpr (P == 128 && NR == 16) {  // 114 VGPRs: 3 waves/SIMD at 768 threads
    if (wg == 768) return launch_main_pf<P, NR, SH, PF, true, 768>(A, ch, s);
    if (wg == 512) return launch_main_pf<P, NR, SH, PF, true, 512>(A, ch, s);
  }
  if constexpr (P != 64) launch_main_pf<P, NR, SH, PF, true, 256>(A, ch, s);
}

}  // namespace

namespace tshared {

int transform_wg(int P, int NR) {
#ifdef TM_DEV_ONE_KERNEL
  (void)P, (void)NR;
  return TM_DEV_WG;
#endif
  // P = 64 (n_fft 2048): the interior loop needs ~250 VGPRs (2 waves/SIMD), so
  // two 4-sequence blocks per CU (TOMATIS_WG=512: one 8-sequence block, the
  // same occupancy with one copy of the tables; measured equal).
  // P = 128, NR = 32 (n_fft 4096): 4 two-wave sequences (~120 KB, 2 waves/SIMD).
  const int dflt = P == 64 ? (kFftX ? 512 : 256) : (NR == 32 ? 512 : 256);
  const int w = dev_opt(TOMATIS_DEV_WG, dflt);
  if (P == 64 && kFftX) return 512;  // the single-exchange FFT's LDS (see launch_main)
  if (P == 64 && (w == 256 || w == 512)) return w;
  if (P == 128 && NR == 32 && (w == 256 || w == 512)) return w;
  if (P == 128 && NR == 16 && (w == 256 || w == 512 || w == 768)) return w;
  return dflt;
}

int transform_slots_per_cu(int P, int NR) {
  // resident sequences per CU: 256-thread blocks run two per CU, wider ones one
  const int wg = transform_wg(P, NR);
  return (wg == 256 ? 2 : 1) * (wg / P);
}

void launch_transform(const MainArgs& A, int P, int NR, int SH, int ch, int wg, hipStream_t s) {
#ifdef TM_DEV_ONLY_2048_512  // development builds: the headline configuration only
  if (P == 64 && SH == 8) launch_main<64, 32, 8>(A, ch, wg, s);
#else
  if (P == 64) {
    if (SH == 4) launch_main<64, 32, 4>(A, ch, wg, s);
    else if (SH == 8) launch_main<64, 32, 8>(A, ch, wg, s);
    else launch_main<64, 32, 16>(A, ch, wg, s);
  } else if (NR == 16) {
    if (SH == 2) launch_main<128, 16, 2>(A, ch, wg, s);
    else if (SH == 4) launch_main<128, 16, 4>(A, ch, wg, s);
    else launch_main<128, 16, 8>(A, ch, wg, s);
  } else {
    if (SH == 4) launch_main<128, 32, 4>(A, ch, wg, s);
    else if (SH == 8) launch_main<128, 32, 8>(A, ch, wg, s);
    else launch_main<128, 32, 16>(A, ch, wg, s);
  }
#endif
}

void launch_frames(const MainArgs& A, int P, int NR, int blocks, hipStream_t s) {
#ifdef TM_DEV_ONE_KERNEL
  (void)A, (void)P, (void)NR, (void)blocks, (void)s;
#else
  if (P == 64) hipLaunchKernelGGL((k_stft_frames<64, 32>), dim3(blocks), dim3(256), 0, s, A);
  else if (NR == 16) hipLaunchKernelGGL((k_stft_frames<128, 16>), dim3(blocks), dim3(256), 0, s, A);
  else hipLaunchKernelGGL((k_stft_frames<128, 32>), dim3(blocks), dim3(256), 0, s, A);
#endif
}

void launch_gain_perm(int P, int NR, bool fx, const float* gains, int n_rows, int n_bins,
                      float* out, hipStream_t s) {
  const int N = P * NR;
  const int nb = (n_rows * N + 255) / 256;
  if (P == 64 && fx)
    hipLaunchKernelGGL((k_gain_perm<64, 32, true>), dim3(nb), dim3(256), 0, s, gains, n_rows, n_bins, out);
  else if (P == 128 && NR == 32 && fx)
    hipLaunchKernelGGL((k_gain_perm<128, 32, true>), dim3(nb), dim3(256), 0, s, gains, n_rows, n_bins, out);
  else if (P == 64)
    hipLaunchKernelGGL((k_gain_perm<64, 32>), dim3(nb), dim3(256), 0, s, gains, n_rows, n_bins, out);
  else if (NR == 16)
    hipLaunchKernelGGL((k_gain_perm<128, 16>), dim3(nb), dim3(256), 0, s, gains, n_rows, n_bins, out);
  else
    hipLaunchKernelGGL((k_gain_perm<128, 32>), dim3(nb), dim3(256), 0, s, gains, n_rows, n_bins, out);
}

void launch_lds_frames(const LdsArgs& A, hipStream_t s) {
  if (A.M > kLdsMaxM) {
    hipLaunchKernelGGL(k_stft_glb, dim3((unsigned)A.work_blocks), dim3(1024), 0, s, A);
    return;
  }
  const dim3 g((unsigned)A.total_frames, (unsigned)((A.ch + 1) / 2));
#define LDS_M(MM)                                                                      \
  if (A.M == MM) {                                                                     \
    if (A.blue) hipLaunchKernelGGL((k_stft_lds<MM, true>), g, dim3(256), 0, s, A);     \
    else hipLaunchKernelGGL((k_stft_lds<MM, false>), g, dim3(256), 0, s, A);           \
  }
#ifndef TM_DEV_ONE_KERNEL
  LDS_M(2) LDS_M(4) LDS_M(8) LDS_M(16) LDS_M(32) LDS_M(64) LDS_M(128) LDS_M(256) LDS_M(512)
  LDS_M(1024) LDS_M(2048) LDS_M(4096) LDS_M(8192) LDS_M(16384)
#endif
#undef LDS_M
}

void launch_r2_plan(const MainArgs& A, uint32_t* pieces, int n_zero, int P, hipStream_t s) {
  if (A.n_runs <= 0) {
    if (n_zero > 0) (void)hipMemsetAsync(A.peaks, 0, (size_t)n_zero * 4, s);
    return;
  }
  hipLaunchKernelGGL(k_r2_plan, dim3(A.n_runs), dim3(64), 0, s, A, pieces, n_zero, P > 64 ? 1 : 0);
}

void launch_prev_runs(const MainArgs& A, int N, hipStream_t s) {
  const int n = A.n_runs_prev - A.n_runs;
  if (n <= 0 || !A.yprev) return;
  if (A.ch == 2) hipLaunchKernelGGL(k_prev_runs<2>, dim3(n), dim3(64), 0, s, A, N);
  else hipLaunchKernelGGL(k_prev_runs<1>, dim3(n), dim3(64), 0, s, A, N);
}

void launch_gate_carry(const MainArgs& A, int P, int SH, int ch, int32_t* gcarry,
                       uint16_t* gtf, double* gacarry, hipStream_t s) {
  if (A.n_runs <= 0) return;
  const dim3 g(A.n_runs), b(64);
  // (the look-back reads blocks in the P = 64 layout: hop = 64 x its SH)
#define TM_GC(C, S, R, X) hipLaunchKernelGGL((k_gate_carry<C, S, R, X>), g, b, 0, s, A, gcarry, gtf, gacarry)
  if (P == 64 && SH == 8) {
    if (ch == 2) TM_GC(2, 8, 32, false);
    else TM_GC(1, 8, 32, false);
  } else if (P == 64 && SH == 4) {
    if (ch == 2) TM_GC(2, 4, 32, false);
    else TM_GC(1, 4, 32, false);
  } else if (P == 128 && SH == 8) {  // n_fft 4096, hop 1024 (cross-fade: alpha too)
    if (A.gate_xf >= 0) {
      if (ch == 2) TM_GC(2, 16, 64, true);
      else TM_GC(1, 16, 64, true);
    } else if (ch == 2) {
      TM_GC(2, 16, 64, false);
    } else {
      TM_GC(1, 16, 64, false);
    }
  }
#undef TM_GC
}

void launch_lds_gather(const LdsArgs& A, hipStream_t s) {
  const int64_t ng = (A.total_out + 255) / 256;
  hipLaunchKernelGGL(k_ola_gather_lds, dim3((unsigned)ng, (unsigned)((A.ch + 7) / 8)), dim3(256),
                     0, s, A);
}

void launch_ola_gather(const MainArgs& A, int n_streams, const int64_t* pos_base, int64_t total,
                       int N, hipStream_t s) {
  const int64_t ng = (total + 255) / 256;
  hipLaunchKernelGGL(k_ola_gather, dim3((unsigned)ng), dim3(256), 0, s, A, n_streams, pos_base,
                     total, N);
}

}  // namespace tshared
