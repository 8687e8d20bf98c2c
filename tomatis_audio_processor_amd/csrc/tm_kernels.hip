// tm_kernels.hip — gfx950 kernels + C ABI of the STFT-gate-OLA engine.
//
// Reference semantics (xyjk0511/tomatis-audio-processor, file:line):
//   levels        src/process_tomatis.py:43-52,369-371  (power-mono RMS, numpy pairwise mean)
//   gate (std)    src/process_tomatis.py:373-385         (hysteresis + up-delay)
//   alpha (xfade) src/process_tomatis_xfade.py:251-274
//   gate (minhold) + bisection  src/process_tomatis_adaptive.py:87-154
//   alpha (adaptive)            src/process_tomatis_adaptive.py:253-265
//   STFT/OLA      src/process_tomatis.py:394-406 ; normalise :422,452 ; limiter :331-357
//   adaptive OLA  src/process_tomatis_adaptive.py:298-345
//   layer-2(b)    src/layer2_apply_eq.py:143-214 ; src/layer2b_apply_residual_eq.py:120-160
// Design: DESIGN.md.  Compiled with -ffp-contract=off: every FMA below is explicit.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <complex>
#include <cstdio>
#include <cstring>
#include <new>
#include <vector>

#include "tm_common.h"
#include "tm_host_dsp.h"
#include "tm_fft.h"
#include "tm_shared.h"
#include "tm_gate.h"
#include "../../include/tomatis_hip.h"

using namespace tdsp;
using namespace tshared;
using namespace tgate;

namespace {

constexpr int kSeg = 1024;           // gate segment length (frames)
// xfade alpha segment length (frames): each segment's alpha recurrence is one
// lane's latency chain (k_alpha_sync / k_alpha_prefix), so short segments, many
// waves (C5x: 3.5 k segments of 128 frames instead of 440 of 1024)
constexpr int kASeg = 128;
constexpr int kLevelLds = 12288;     // floats of LDS for the levels span
constexpr int kMaxGateStates = 65535;  // uint16 state ids (transfer tables)

struct LvlBlock {     // levels work item
  int32_t s;
  int32_t nf;
  int64_t k0;
};
struct GateSeg {      // gate segment
  int32_t s;
  int32_t nf;
  int64_t k0;         // first frame (stream-local)
};


// ===========================================================================
// Levels: r = sqrt(mean(m*m) + EPS), m = sqrt(mean_c(x_c^2)), numpy pairwise
// ===========================================================================
template <typename T>
__device__ __forceinline__ T sq_ch(const float* xs, int c, T scale) {
  const T v = (T)xs[c] * scale;
  return v * v;
}

// frame**2 -> mean over channels -> sqrt -> square.  numpy reduces the channel
// axis with its pairwise sum: sequential from 0 below 8 channels, otherwise 8
// accumulators, the fixed tree and a sequential remainder (plan: ch <= 128).
template <typename T>
__device__ __forceinline__ T msq_of(const float* xs, int ch, T scale) {
  T acc;
  if (ch < 8) {
    acc = (T)0;
    for (int c = 0; c < ch; ++c) acc = acc + sq_ch<T>(xs, c, scale);
  } else {
    T r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = sq_ch<T>(xs, j, scale);
    int i = 8;
    for (; i < ch - (ch % 8); i += 8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] = r[j] + sq_ch<T>(xs, i + j, scale);
    }
    acc = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < ch; ++i) acc = acc + sq_ch<T>(xs, i, scale);
  }
  const T mean = (ch == 1) ? acc : ((ch == 2) ? acc * (T)0.5 : acc / (T)ch);
  T m;
  if constexpr (sizeof(T) == 4) m = sqrtf(mean);
  else m = sqrt(mean);
  return m * m;
}

// padded LDS index (one 4-element pad per 128 elements -> conflict-free b128 leaf reads)
template <bool PAD>
__device__ __forceinline__ int lidx(int i) {
  if constexpr (PAD) return i + 4 * (i >> 7);
  else return i;
}

// numpy pairwise block for n == 128 (8 accumulators, then a fixed tree)
template <typename T, bool PAD>
__device__ __forceinline__ T leaf128(const T* lds, int start) {
  T r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = lds[lidx<PAD>(start + j)];
#pragma unroll
  for (int i = 8; i < 128; i += 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = r[j] + lds[lidx<PAD>(start + i + j)];
  }
  return ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
}

template <typename T, bool PAD>
__global__ __launch_bounds__(256) void k_levels(const float* __restrict__ x,
                                                const TomatisStream* __restrict__ st,
                                                const LvlBlock* __restrict__ blocks, int n_fft,
                                                int hop, int ch, T* __restrict__ r_out) {
  __shared__ T lds[kLevelLds * sizeof(float) / sizeof(T) + 256];
  __shared__ T leaves[1024];
  const LvlBlock blk = blocks[blockIdx.x];
  const TomatisStream S = st[blk.s];
  const int64_t span0 = S.first_start + blk.k0 * hop;
  const int span = (blk.nf - 1) * hop + n_fft;
  const T scale = (T)S.in_scale;
  const float* xs = x + S.in_off;
  if (span0 >= 0 && span0 + span <= S.n && ch == 2) {
    // interior: 8 independent 8-byte loads in flight per thread, then compute
    const float2* src = reinterpret_cast<const float2*>(xs) + span0;
    constexpr int U = 8;
    for (int base = threadIdx.x; base < span; base += 256 * U) {
      float2 t[U];
#pragma unroll
      for (int j = 0; j < U; ++j) {
        const int i = base + 256 * j;
        t[j] = (i < span) ? src[i] : make_float2(0.f, 0.f);
      }
#pragma unroll
      for (int j = 0; j < U; ++j) {
        const int i = base + 256 * j;
        const float pair[2] = {t[j].x, t[j].y};
        if (i < span) lds[lidx<PAD>(i)] = msq_of<T>(pair, 2, scale);
      }
    }
  } else {
    for (int i = threadIdx.x; i < span; i += blockDim.x) {
      const int64_t p = span0 + i;
      T v = (T)0;
      if (p >= 0 && p < S.n) v = msq_of<T>(xs + p * ch, ch, scale);
      lds[lidx<PAD>(i)] = v;
    }
  }
  __syncthreads();
  const int nleaf = n_fft >> 7;  // n_fft power of two >= 256
  const int total = blk.nf * nleaf;
  for (int t = threadIdx.x; t < total; t += blockDim.x) {
    const int f = t / nleaf, l = t - f * nleaf;
    leaves[t] = leaf128<T, PAD>(lds, f * hop + 128 * l);
  }
  __syncthreads();
  if (threadIdx.x < blk.nf) {
    T* lv = leaves + threadIdx.x * nleaf;
    for (int w = nleaf; w > 1; w >>= 1)
      for (int i = 0; i < w / 2; ++i) lv[i] = lv[2 * i] + lv[2 * i + 1];
    const T sum = lv[0];
    const T mean = sum / (T)n_fft;
    const T r = sqrt(mean + (T)(sizeof(T) == 4 ? (double)kEps32 : kEps64));
    r_out[S.frame_base + blk.k0 + threadIdx.x] = r;
  }
}

// ---------------------------------------------------------------------------
// Levels for any n_fft (not a power of two in [256, 8192], or a frame larger
// than the block LDS): numpy's pairwise_sum(a, n) splits at n2 = n/2 - (n/2)%8
// until n <= 128, so its tree over a frame is fixed by n alone.  The host
// records the leaves (offset, length) and the combination order as a postfix
// program (leaf index >= 0 pushes that leaf's sum, -1 adds the top two).  One
// block per frame: threads sum leaves straight from HBM (numpy's block rule:
// sequential below 8, else 8 accumulators + tree + sequential remainder), one
// thread runs the program.
// ---------------------------------------------------------------------------
constexpr int kPwMaxLeaves = 2048;

template <typename T>
__device__ T pw_leaf(const float* xs, int64_t n, int ch, int64_t p0, int len, T scale) {
  auto m2 = [&](int i) -> T {
    const int64_t p = p0 + i;
    return (p >= 0 && p < n) ? msq_of<T>(xs + p * ch, ch, scale) : (T)0;
  };
  if (len < 8) {
    T acc = (T)0;
    for (int i = 0; i < len; ++i) acc = acc + m2(i);
    return acc;
  }
  T r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = m2(j);
  int i = 8;
  for (; i < len - (len % 8); i += 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = r[j] + m2(i + j);
  }
  T res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < len; ++i) res = res + m2(i);
  return res;
}

template <typename T>
__global__ __launch_bounds__(256) void k_levels_any(const float* __restrict__ x,
                                                    const TomatisStream* __restrict__ st,
                                                    int n_streams, int n_fft, int hop, int ch,
                                                    const int2* __restrict__ leaf, int n_leaf,
                                                    const int16_t* __restrict__ prog, int n_prog,
                                                    int64_t total_frames, T* __restrict__ r_out) {
  __shared__ T ls[kPwMaxLeaves];
  for (int64_t f = blockIdx.x; f < total_frames; f += gridDim.x) {
    int lo = 0, hi = n_streams - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (st[mid].frame_base <= f) lo = mid;
      else hi = mid - 1;
    }
    const TomatisStream S = st[lo];
    const int64_t s_k = S.first_start + (f - S.frame_base) * hop;
    const float* xs = x + S.in_off;
    const T scale = (T)S.in_scale;
    for (int l = threadIdx.x; l < n_leaf; l += blockDim.x) {
      const int2 lf = leaf[l];
      ls[l] = pw_leaf<T>(xs, S.n, ch, s_k + lf.x, lf.y, scale);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      T stk[40];
      int sp = 0;
      for (int i = 0; i < n_prog; ++i) {
        const int op = prog[i];
        if (op >= 0) {
          stk[sp++] = ls[op];
        } else {
          const T b = stk[--sp];
          stk[sp - 1] = stk[sp - 1] + b;
        }
      }
      const T mean = stk[0] / (T)n_fft;
      r_out[f] = sqrt(mean + (T)(sizeof(T) == 4 ? (double)kEps32 : kEps64));
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Streaming levels (hop % 128 == 0): numpy's pairwise mean over a power-of-two
// frame is a perfect binary tree over 128-sample leaves aligned to the frame
// start, so every 128-sample block (aligned to first_start) has ONE leaf sum
// shared by all frames covering it.  k_leaves: one wave per group of 8 blocks
// (1024 samples) of one stream (blockIdx.y); the group is read with 16-byte
// lane-contiguous loads (1 KB per load instruction), every sample's m^2 goes
// to LDS in chain order, then lane (block b, chain c) sums m^2 of samples c,
// c+8, .., c+120 in order (numpy's 8 accumulators) and the 8 chains combine as
// ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) via xor-shuffles (IEEE add commutes).
// (The first form, each lane loading its own chain's 8-byte samples, ran at
// 3.0 TB/s on C5x: 0.61 ms for 1.84 GB.)
// k_frame_r: per frame, perfect-tree sum of n_fft/128 leaves, mean, sqrt.
// ---------------------------------------------------------------------------
constexpr int kLfC = 24;          // LDS stride of a chain (16 values + pad: conflict-free writes)
constexpr int kLfB = 8 * kLfC + 4;  // LDS stride of a block
template <typename T, int CH>
__global__ __launch_bounds__(256) void k_leaves(const float* __restrict__ x,
                                                const TomatisStream* __restrict__ st,
                                                int n_streams,
                                                const int64_t* __restrict__ grp_base,
                                                const int64_t* __restrict__ leaf_base,
                                                int64_t n_groups, T* __restrict__ leaves) {
  __shared__ T sm[4][8 * kLfB];
  const int lane = threadIdx.x & 63;
  T* const w = sm[threadIdx.x >> 6];
  const int lo = blockIdx.y;  // stream
  const int64_t gl = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);  // 8-block group of the stream
  if (lo >= n_streams || gl >= grp_base[lo + 1] - grp_base[lo]) return;
  (void)n_groups;
  const TomatisStream S = st[lo];
  const int64_t nblk = leaf_base[lo + 1] - leaf_base[lo];
  const int64_t p0 = S.first_start + gl * 1024;  // first sample of the group
  const T scale = (T)S.in_scale;
  const float* xs = x + S.in_off;
  // sample i of the group -> block i >> 7, chain i & 7, position (i >> 3) & 15
  auto slot = [&](int i) -> T& { return w[(i >> 7) * kLfB + (i & 7) * kLfC + ((i >> 3) & 15)]; };
  const bool full = p0 >= 0 && p0 + 1024 <= S.n && ((uintptr_t)(xs + p0 * CH) & 15) == 0;
  if (full) {
    const float4* x4 = reinterpret_cast<const float4*>(xs + p0 * CH);
    constexpr int NL = 1024 * CH / 4 / 64;  // float4 per lane: 8 (stereo) / 4 (mono)
    float4 t[NL];
#pragma unroll
    for (int u = 0; u < NL; ++u) t[u] = x4[u * 64 + lane];  // all loads in flight
#pragma unroll
    for (int u = 0; u < NL; ++u) {
      const int f = u * 64 + lane;  // float4 index within the group
      if constexpr (CH == 2) {
        const float a0[2] = {t[u].x, t[u].y}, a1[2] = {t[u].z, t[u].w};
        slot(2 * f) = msq_of<T>(a0, 2, scale);
        slot(2 * f + 1) = msq_of<T>(a1, 2, scale);
      } else {
        const float a[4] = {t[u].x, t[u].y, t[u].z, t[u].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) slot(4 * f + e) = msq_of<T>(a + e, 1, scale);
      }
    }
  } else {  // a stream edge (zeros outside the stream) or an unaligned stream: per sample
#pragma unroll 4
    for (int i = lane; i < 1024; i += 64) {
      const int64_t p = p0 + i;
      slot(i) = (p >= 0 && p < S.n) ? msq_of<T>(xs + p * CH, CH, scale) : (T)0;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int b = lane >> 3, c = lane & 7;
  const T* ch = w + b * kLfB + c * kLfC;
  T acc = ch[0];
#pragma unroll
  for (int q = 1; q < 16; ++q) acc = acc + ch[q];
  // pairwise tree over the 8 chains of a block
  acc = acc + __shfl_xor(acc, 1, 64);
  acc = acc + __shfl_xor(acc, 2, 64);
  acc = acc + __shfl_xor(acc, 4, 64);
  const int64_t blk = gl * 8 + b;
  if (c == 0 && blk < nblk) leaves[leaf_base[lo] + blk] = acc;
}

template <typename T>
__global__ __launch_bounds__(256) void k_frame_r(const TomatisStream* __restrict__ st,
                                                 int n_streams, const int64_t* __restrict__ leaf_base,
                                                 const T* __restrict__ leaves, int n_fft, int hop,
                                                 int64_t total_frames, T* __restrict__ r_out) {
  const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= total_frames) return;
  int lo = 0, hi = n_streams - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (st[mid].frame_base <= f) lo = mid;
    else hi = mid - 1;
  }
  const int64_t k = f - st[lo].frame_base;
  const T* lv = leaves + leaf_base[lo] + k * (hop >> 7);
  const int nleaf = n_fft >> 7;  // 16 or 32
  T t[32];
  for (int i = 0; i < nleaf; ++i) t[i] = lv[i];
  for (int w = nleaf; w > 1; w >>= 1)
    for (int i = 0; i < w / 2; ++i) t[i] = t[2 * i] + t[2 * i + 1];
  const T mean = t[0] / (T)n_fft;
  r_out[f] = sqrt(mean + (T)(sizeof(T) == 4 ? (double)kEps32 : kEps64));
}

// ===========================================================================
// Standard gate (process_tomatis.py:373-385) as a transfer-function scan.
// state id: 0 = C1 idle, 1..D = C1 pending for (id-1) frames, D+1 = C2.
// ===========================================================================
__global__ __launch_bounds__(256) void k_gate_tf(const float* __restrict__ r,
                                                 const TomatisStream* __restrict__ st,
                                                 const GateSeg* __restrict__ segs, int nseg,
                                                 int D, uint16_t* __restrict__ tf) {
  __shared__ uint8_t pr[4][kSeg];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int sg = blockIdx.x * 4 + wv;
  if (sg >= nseg) return;
  const GateSeg G = segs[sg];
  const TomatisStream S = st[G.s];
  for (int i = lane; i < G.nf; i += 64) pr[wv][i] = gate_pred(r[S.frame_base + G.k0 + i], S);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int ns = D + 2;
  for (int s0 = 0; s0 < ns; s0 += 64) {
    int id = s0 + lane;
    if (id < ns) {
      for (int i = 0; i < G.nf; ++i) id = gate_step(id, pr[wv][i], D);
      tf[(int64_t)sg * ns + s0 + lane] = (uint16_t)id;
    }
  }
}

// sequential composition over a stream's segments (one thread per stream)
__global__ void k_gate_chain(const TomatisStream* __restrict__ st, int n_streams,
                             const int32_t* __restrict__ seg_first,
                             const int32_t* __restrict__ seg_count, int ns,
                             const uint16_t* __restrict__ tf, uint16_t* __restrict__ seg_start,
                             int init_id) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_streams) return;
  int id = init_id;
  const int a = seg_first[s], n = seg_count[s];
  for (int i = 0; i < n; ++i) {
    seg_start[a + i] = (uint16_t)id;
    id = tf[(int64_t)(a + i) * ns + id];
  }
}

// one wave per segment: lanes evaluate 64 predicates at a time, the automaton
// advances on the (wave-uniform) scalar path, lane i keeps the state of frame i
__global__ __launch_bounds__(256) void k_gate_resolve(const float* __restrict__ r,
                                                      const TomatisStream* __restrict__ st,
                                                      const GateSeg* __restrict__ segs, int nseg,
                                                      int D, const uint16_t* __restrict__ seg_start,
                                                      uint8_t* __restrict__ states,
                                                      uint16_t* __restrict__ rows) {
  const int lane = threadIdx.x & 63;
  const int sg = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (sg >= nseg) return;
  const GateSeg G = segs[sg];
  const TomatisStream S = st[G.s];
  int id = seg_start[sg];
  const int64_t f0 = S.frame_base + G.k0;
  for (int base = 0; base < G.nf; base += 64) {
    const int i = base + lane;
    const int pr = (i < G.nf) ? (int)gate_pred(r[f0 + i], S) : 0;
    const int cnt = min(64, G.nf - base);
    int mine = 0;
    for (int t = 0; t < cnt; ++t) {
      const int pt = __builtin_amdgcn_readlane(pr, t);
      id = gate_step(id, (uint8_t)pt, D);
      mine = (lane == t) ? id : mine;
    }
    if (i < G.nf) {
      const uint8_t stt = (mine == D + 1) ? 2 : 1;
      states[f0 + i] = stt;
      if (rows) rows[f0 + i] = (uint16_t)(stt - 1);
    }
  }
}

// ---------------------------------------------------------------------------
// Run-scan gate: the same automaton in closed form when no r can be both "on"
// and "off" (host-checked from the bit thresholds + exception lists).
//   A(k) = last frame <= k that is not "on"   (the pending run restarts there)
//   entry at k  <=>  on(k) and k - A(k) >= D + 1   (pending matured: s_k >= pending)
//   E(k) = last entry <= k,  F(k) = last "off" frame <= k
//   state(k) = C2  <=>  E(k) > F(k)
// Segment summaries compose associatively, so a segment is reduced and scanned
// in parallel (wave shuffles + LDS), segments are scanned per stream, and every
// frame resolves from its segment's carry-in.  Frame indices are stream-local.
// ---------------------------------------------------------------------------
constexpr int kNI = INT_MIN / 4;  // "none"
struct GSum {
  int all_on;  // every frame on
  int not_on;  // last not-on frame
  int l_end;   // last frame of the leading on-run (kNI if the first frame is not on)
  int e_int;   // last entry after the first not-on frame
  int off;     // last off frame
};
struct GCarry {
  int a, e, f;
};
__device__ __forceinline__ GSum gs_identity() { return GSum{1, kNI, kNI, kNI, kNI}; }
__device__ __forceinline__ GSum gs_frame(int k, uint8_t pr) {
  if (pr & 1) return GSum{1, kNI, k, kNI, kNI};
  return GSum{0, k, kNI, kNI, (pr & 2) ? k : kNI};
}
__device__ __forceinline__ GSum gs_cat(const GSum& X, const GSum& Y, int D) {
  GSum Z;
  Z.all_on = X.all_on & Y.all_on;
  Z.not_on = max(X.not_on, Y.not_on);
  Z.off = max(X.off, Y.off);
  if (X.all_on) {
    Z.l_end = (Y.l_end != kNI) ? Y.l_end : X.l_end;
    Z.e_int = Y.e_int;
  } else {
    Z.l_end = X.l_end;
    const int lead = (Y.l_end != kNI && Y.l_end >= X.not_on + D + 1) ? Y.l_end : kNI;
    Z.e_int = max(max(X.e_int, Y.e_int), lead);
  }
  return Z;
}
__device__ __forceinline__ GCarry gs_apply(const GCarry& c, const GSum& S, int D) {
  GCarry o;
  o.a = S.all_on ? c.a : S.not_on;
  const int lead = (S.l_end != kNI && S.l_end >= c.a + D + 1) ? S.l_end : kNI;
  o.e = max(max(c.e, S.e_int), lead);
  o.f = max(c.f, S.off);
  return o;
}
__device__ __forceinline__ GSum gs_shfl_up(const GSum& x, int d) {
  return GSum{__shfl_up(x.all_on, d, 64), __shfl_up(x.not_on, d, 64), __shfl_up(x.l_end, d, 64),
              __shfl_up(x.e_int, d, 64), __shfl_up(x.off, d, 64)};
}
// inclusive scan over the 256 threads of a block (thread order); returns the
// thread's EXCLUSIVE prefix and sets tot to the block total
__device__ GSum gs_block_scan(GSum v, int D, GSum& tot) {
  __shared__ GSum s_w[4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  GSum inc = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const GSum y = gs_shfl_up(inc, d);
    if (lane >= d) inc = gs_cat(y, inc, D);
  }
  if (lane == 63) s_w[wv] = inc;
  __syncthreads();
  GSum wpre = gs_identity();
  for (int w = 0; w < wv; ++w) wpre = gs_cat(wpre, s_w[w], D);
  tot = gs_identity();
  for (int w = 0; w < 4; ++w) tot = gs_cat(tot, s_w[w], D);
  GSum ex = gs_shfl_up(inc, 1);
  if (lane == 0) ex = gs_identity();
  __syncthreads();
  return gs_cat(wpre, ex, D);
}

// pass 1: one block per gate segment (<= 1024 frames, 4 per thread) -> summary
__global__ __launch_bounds__(256) void k_gate_sum(const float* __restrict__ r,
                                                  const TomatisStream* __restrict__ st,
                                                  const GateSeg* __restrict__ segs, int D,
                                                  GSum* __restrict__ sums) {
  const GateSeg G = segs[blockIdx.x];
  const TomatisStream S = st[G.s];
  GSum v = gs_identity();
  const int i0 = 4 * threadIdx.x;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int i = i0 + j;
    if (i < G.nf) v = gs_cat(v, gs_frame((int)G.k0 + i, gate_pred(r[S.frame_base + G.k0 + i], S)), D);
  }
  GSum tot;
  (void)gs_block_scan(v, D, tot);
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

// pass 2: one block per stream, scan of segment summaries -> carry-in per segment
__global__ __launch_bounds__(256) void k_gate_carry(const int32_t* __restrict__ seg_first,
                                                    const int32_t* __restrict__ seg_count, int D,
                                                    const GSum* __restrict__ sums,
                                                    GCarry* __restrict__ carry,
                                                    const GCarry* __restrict__ carry_in) {
  const int a = seg_first[blockIdx.x], n = seg_count[blockIdx.x];
  // initial C1 idle: run "restarts" just before frame 0; a time shard starts
  // from the carry its predecessors' summaries compose to (timeshard.py)
  GCarry c = carry_in ? carry_in[blockIdx.x] : GCarry{-1, kNI, kNI};
  for (int t0 = 0; t0 < n; t0 += 256) {
    const int i = t0 + threadIdx.x;
    const GSum v = (i < n) ? sums[a + i] : gs_identity();
    GSum tot;
    const GSum ex = gs_block_scan(v, D, tot);
    if (i < n) carry[a + i] = gs_apply(c, ex, D);
    c = gs_apply(c, tot, D);
  }
}

// pass 3: one block per segment: frame states from the carry-in
__global__ __launch_bounds__(256) void k_gate_states(const float* __restrict__ r,
                                                     const TomatisStream* __restrict__ st,
                                                     const GateSeg* __restrict__ segs, int D,
                                                     const GCarry* __restrict__ carry,
                                                     uint8_t* __restrict__ states,
                                                     uint16_t* __restrict__ rows) {
  const GateSeg G = segs[blockIdx.x];
  const TomatisStream S = st[G.s];
  const int i0 = 4 * threadIdx.x;
  uint8_t pr[4];
  GSum v = gs_identity();
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int i = i0 + j;
    pr[j] = (i < G.nf) ? gate_pred(r[S.frame_base + G.k0 + i], S) : 0;
    if (i < G.nf) v = gs_cat(v, gs_frame((int)G.k0 + i, pr[j]), D);
  }
  GSum tot;
  const GSum ex = gs_block_scan(v, D, tot);
  GCarry c = gs_apply(carry[blockIdx.x], ex, D);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int i = i0 + j;
    if (i < G.nf) {
      c = gs_apply(c, gs_frame((int)G.k0 + i, pr[j]), D);
      const uint8_t stt = (c.e > c.f) ? 2 : 1;
      states[S.frame_base + G.k0 + i] = stt;
      if (rows) rows[S.frame_base + G.k0 + i] = (uint16_t)(stt - 1);
    }
  }
}

// time shards (timeshard.py): the summary of this shard's first n_seg segments
// (stream 0) re-indexed by +shift frames; and the carry-in composed from the
// summaries of ranks 0..rank-1, re-indexed by -shift.  One thread each: a few
// hundred segments / ranks.
__device__ __forceinline__ int gs_sh(int v, int off) { return v == kNI ? kNI : v + off; }
__global__ void k_ts_fold(const GSum* __restrict__ sums, int n_seg, int D, int shift,
                          int32_t* __restrict__ out) {
  if (threadIdx.x != 0) return;
  GSum S = gs_identity();
  for (int i = 0; i < n_seg; ++i) S = gs_cat(S, sums[i], D);
  out[0] = S.all_on;
  out[1] = gs_sh(S.not_on, shift);
  out[2] = gs_sh(S.l_end, shift);
  out[3] = gs_sh(S.e_int, shift);
  out[4] = gs_sh(S.off, shift);
}
__global__ void k_ts_carry(const int32_t* __restrict__ all, int rank, int D, int shift,
                           GCarry* __restrict__ carry) {
  if (threadIdx.x != 0) return;
  GCarry c{-1, kNI, kNI};
  for (int q = 0; q < rank; ++q) {
    const int32_t* v = all + 5 * q;
    c = gs_apply(c, GSum{v[0], v[1], v[2], v[3], v[4]}, D);
  }
  carry[0] = GCarry{c.a + shift, gs_sh(c.e, shift), gs_sh(c.f, shift)};
}

// ===========================================================================
// alpha scans (sequential per stream; f64 exactly as the reference)
// ===========================================================================
// alpha_step, xfade_row: tm_gate.h

// xfade (process_tomatis_xfade.py:251-274): alpha starts at 0.0.
// xfade alpha (process_tomatis_xfade.py:251-274) in three passes over the gate
// segments.  alpha moves by +-step toward the frame's target (0 in C1, 1 in C2)
// and snaps to it once within step, so after J = xf + 2 consecutive frames of
// one state it equals that target exactly, whatever it was before (frames
// before 0 count as C1: alpha starts at 0.0).  From a segment's first such
// "sync" frame on, alpha depends only on the states; only the prefix before it
// needs the previous segment's final alpha.  Every value is produced by the
// same float64 operations in the same order as the sequential reference loop.

// pass 1: one wave per segment: sync frame, alpha from it to the segment end.
// The segment's states are staged in LDS by all lanes; the recurrence runs in
// lane 0 from LDS (four frames per read); alpha and rows go back out through
// LDS as coalesced stores (one thread per segment walking global memory frame
// by frame took 0.35 ms on C5x: 440 segments = 7 waves on the chip)
__global__ __launch_bounds__(64) void k_alpha_sync(const TomatisStream* __restrict__ st,
                                                   const GateSeg* __restrict__ segs, int nseg,
                                                   const uint8_t* __restrict__ states, int xf,
                                                   uint16_t* __restrict__ rows,
                                                   double* __restrict__ alpha,
                                                   int32_t* __restrict__ seg_q,
                                                   double* __restrict__ seg_final) {
  __shared__ __attribute__((aligned(16))) uint8_t s_st[kASeg];
  __shared__ double s_a[kASeg];
  __shared__ int s_q;
  const int i = blockIdx.x;
  if (i >= nseg) return;
  const int L = threadIdx.x;
  const GateSeg G = segs[i];
  const TomatisStream S = st[G.s];
  const uint8_t* stt = states + S.frame_base;
  const int J = xf + 2;
  const double step = xf > 0 ? 1.0 / xf : 1.0;
  for (int j = L; j < G.nf; j += 64) s_st[j] = stt[G.k0 + j];
  // run of equal states ending just before k0 (frames < 0 are C1 forever):
  // lanes test 64 earlier frames at a time
  uint8_t prev = 1;
  int run = J;
  if (G.k0 > 0) {
    prev = stt[G.k0 - 1];
    run = 1;
    bool open = true;  // the run has not met a different state yet
    for (int64_t base = G.k0 - 2; open && run < J && base >= 0; base -= 64) {
      const int64_t k = base - L;
      const bool diff = (k >= 0) && stt[k] != prev;
      const uint64_t m = __ballot(diff);
      const int avail = (int)min<int64_t>(64, base + 1);  // frames base .. base - avail + 1
      const int same = m ? __builtin_ctzll(m) : avail;
      run = min(run + same, J);
      if (m || same < 64) open = false;
      if (!m && base - 64 < 0 && same == avail && run < J && prev == 1) run = J;  // C1 pre-history
    }
    if (open && run < J && prev == 1 && G.k0 - 1 - (run - 1) <= 0) run = J;
  }
  __syncthreads();
  if (L == 0) {
    // 16 states per LDS read (the loops are latency chains in one lane)
    const uint4* s4 = reinterpret_cast<const uint4*>(s_st);
    auto st_of = [](const uint4& w, int u) -> uint8_t {
      const uint32_t d = u < 4 ? w.x : (u < 8 ? w.y : (u < 12 ? w.z : w.w));
      return (uint8_t)(d >> (8 * (u & 3)));
    };
    int q = G.nf;
    for (int b = 0; b * 16 < G.nf && q == G.nf; ++b) {
      const uint4 w = s4[b];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int j = b * 16 + u;
        if (j < G.nf && q == G.nf) {
          const uint8_t t = st_of(w, u);
          run = (t == prev) ? min(run + 1, J) : 1;
          prev = t;
          if (xf == 0 || run >= J) q = j;
        }
      }
    }
    s_q = q;
    seg_q[i] = q;
    if (q < G.nf) {
      double a = s_st[q] == 1 ? 0.0 : 1.0;
      s_a[q] = a;
      for (int b = (q + 1) >> 4; b * 16 < G.nf; ++b) {
        const uint4 w = s4[b];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int j = b * 16 + u;
          if (j > q && j < G.nf) {
            const double tgt = st_of(w, u) == 1 ? 0.0 : 1.0;
            a = (xf > 0) ? alpha_step(a, tgt, step) : tgt;
            s_a[j] = a;
          }
        }
      }
      seg_final[i] = a;
    }
  }
  __syncthreads();
  const int q = s_q;
  for (int j = q + L; j < G.nf; j += 64) {
    const int64_t f = S.frame_base + G.k0 + j;
    const double a = s_a[j];
    if (alpha) alpha[f] = a;
    rows[f] = xfade_row(a, xf);
  }
}

// pass 2: one wave per stream: carry-in alpha of every segment.  Lanes take 64
// segments at a time; a segment with a sync frame hands its final alpha on
// directly, one without is walked from its carry-in in segment order (lane by
// lane, wave-uniform)
__global__ __launch_bounds__(64) void k_alpha_chain(const TomatisStream* __restrict__ st,
                                                    int n_streams,
                                                    const GateSeg* __restrict__ segs,
                                                    const int32_t* __restrict__ seg_first,
                                                    const int32_t* __restrict__ seg_count,
                                                    const uint8_t* __restrict__ states, int xf,
                                                    const int32_t* __restrict__ seg_q,
                                                    const double* __restrict__ seg_final,
                                                    double* __restrict__ carry_in) {
  const int s = blockIdx.x;
  if (s >= n_streams) return;
  const int lane = threadIdx.x;
  const TomatisStream S = st[s];
  const double step = xf > 0 ? 1.0 / xf : 1.0;
  double c = 0.0;  // alpha before the chunk's first segment (wave-uniform)
  const int first = seg_first[s], end = seg_first[s] + seg_count[s];
  for (int base = first; base < end; base += 64) {
    const int i = base + lane;
    const bool valid = i < end;
    const GateSeg G = valid ? segs[i] : GateSeg{0, 1, 0};
    const bool synced = valid && seg_q[i] < G.nf;
    double after = synced ? seg_final[i] : 0.0;  // alpha after segment i
    uint64_t um = __ballot(valid && !synced);
    while (um) {  // unsynced segments in order: walk each from its carry-in
      const int u = __builtin_ctzll(um);
      um &= um - 1;
      const double prev = __shfl(after, u > 0 ? u - 1 : 0);
      double a = u > 0 ? prev : c;
      const GateSeg Gu = segs[base + u];
      for (int j = 0; j < Gu.nf; ++j) {
        const double tgt = states[S.frame_base + Gu.k0 + j] == 1 ? 0.0 : 1.0;
        a = (xf > 0) ? alpha_step(a, tgt, step) : tgt;
      }
      if (lane == u) after = a;
    }
    const double up = __shfl_up(after, 1);
    if (valid) carry_in[i] = lane == 0 ? c : up;
    const int last = min(63, end - 1 - base);
    c = __shfl(after, last);
  }
}

// pass 3: one wave per segment: the frames before its sync frame (all of them
// when the segment has none), from the carry-in; staged through LDS as pass 1
__global__ __launch_bounds__(64) void k_alpha_prefix(const TomatisStream* __restrict__ st,
                                                     const GateSeg* __restrict__ segs, int nseg,
                                                     const uint8_t* __restrict__ states, int xf,
                                                     const int32_t* __restrict__ seg_q,
                                                     const double* __restrict__ carry_in,
                                                     uint16_t* __restrict__ rows,
                                                     double* __restrict__ alpha) {
  __shared__ __attribute__((aligned(16))) uint8_t s_st[kASeg];
  __shared__ double s_a[kASeg];
  const int i = blockIdx.x;
  if (i >= nseg) return;
  const int q = seg_q[i];
  if (q == 0) return;
  const int L = threadIdx.x;
  const GateSeg G = segs[i];
  const TomatisStream S = st[G.s];
  const double step = xf > 0 ? 1.0 / xf : 1.0;
  for (int j = L; j < q; j += 64) s_st[j] = states[S.frame_base + G.k0 + j];
  __syncthreads();
  if (L == 0) {
    const uint4* s4 = reinterpret_cast<const uint4*>(s_st);
    double a = carry_in[i];
    for (int b = 0; b * 16 < q; ++b) {
      const uint4 w = s4[b];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int j = b * 16 + u;
        if (j < q) {
          const uint32_t d = u < 4 ? w.x : (u < 8 ? w.y : (u < 12 ? w.z : w.w));
          const double tgt = (uint8_t)(d >> (8 * (u & 3))) == 1 ? 0.0 : 1.0;
          a = (xf > 0) ? alpha_step(a, tgt, step) : tgt;
          s_a[j] = a;
        }
      }
    }
  }
  __syncthreads();
  for (int j = L; j < q; j += 64) {
    const int64_t f = S.frame_base + G.k0 + j;
    const double a = s_a[j];
    if (alpha) alpha[f] = a;
    rows[f] = xfade_row(a, xf);
  }
}

// sequential reference of the three passes (kept for TOMATIS_ALPHA_SEQ=1)
__global__ void k_alpha_xfade(const TomatisStream* __restrict__ st, int n_streams,
                              const uint8_t* __restrict__ states, int xf,
                              uint16_t* __restrict__ rows, double* __restrict__ alpha) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_streams) return;
  const TomatisStream S = st[s];
  const double step = xf > 0 ? 1.0 / xf : 1.0;
  double a = 0.0;
  for (int64_t k = 0; k < S.n_frames; ++k) {
    const int64_t f = S.frame_base + k;
    const double tgt = states[f] == 1 ? 0.0 : 1.0;
    a = (xf > 0) ? alpha_step(a, tgt, step) : tgt;
    if (alpha) alpha[f] = a;
    uint16_t row;
    if (xf > 0 && a > 0.0 && a < 1.0) row = (uint16_t)(2 + (int)rint(a * xf));
    else row = (a < 0.5) ? 0 : 1;
    rows[f] = row;
  }
}

// ===========================================================================
// Adaptive: min-hold gate, bisection, final states, alpha (one block per stream)
// state id = (C - 1) * (mh + 1) + min(since, mh)
// ===========================================================================
constexpr int kMhAlphaChunks = 2048;  // alpha chunks per stream (LDS carries)
constexpr int kMhLdsTf = 8192;        // (segment, start state) transfer entries held in LDS
constexpr int kMhLdsSym = 4096;       // symbol words held in LDS (65536 frames)

// Segment length (frames, a multiple of 16 = one symbol word): at least 256,
// few enough segments that the (segment, start) transfer table fits in LDS and
// the final pass's segment starts fit its 4096-entry table.  Host and device.
__host__ __device__ inline int64_t mh_seg_len(int64_t F, int ns) {
  int64_t seg = 256;
  const int64_t a = (F * ns + kMhLdsTf - 1) / kMhLdsTf, b = (F + 4095) / 4096;
  seg = a > seg ? a : seg;
  seg = b > seg ? b : seg;
  return (seg + 15) & ~(int64_t)15;
}

// Per bisection threshold the levels reduce to 2-bit symbols per frame
// (bit 0: level >= t_on, bit 1: level <= t_off; NaN sets neither), 16 frames
// per u32 word; the min-hold walk then only needs the symbols.
__device__ void mh_symbols(const double* __restrict__ lv, int64_t F, double ton, double toff,
                           uint32_t* __restrict__ sym) {
  const int64_t nw = (F + 15) >> 4;
  for (int64_t w = threadIdx.x; w < nw; w += blockDim.x) {
    const int64_t k0 = w << 4;
    const int n = (int)min<int64_t>(16, F - k0);
    uint32_t b = 0;
    for (int j = 0; j < n; ++j) {
      const double l = lv[k0 + j];
      b |= (l >= ton ? 1u : 0u) << (2 * j);
      b |= (l <= toff ? 1u : 0u) << (2 * j + 1);
    }
    sym[w] = b;
  }
}

// state (c2, since): since = min(since + 1, mh); once saturated a C1 frame with
// symbol bit 0 switches to (C2, 0), a C2 frame with bit 1 to (C1, 0)
// (src/process_tomatis_adaptive.py:87-120, simulate_gate with min_hold).
// State id = c2 * (mh + 1) + since.
struct MhState {
  int c2, since;
};
__device__ __forceinline__ void mh_word(MhState& st, uint32_t w, int n, int mh, int& c) {
  for (int j = 0; j < n; ++j) {
    st.since = min(st.since + 1, mh);
    const int sw = (st.since == mh) & (int)((w >> (2 * j + st.c2)) & 1u);
    st.c2 ^= sw;
    st.since = sw ? 0 : st.since;
    c += st.c2;
  }
}

// transfer table of every (segment, start state): end state and C2 frames
__device__ void mh_simulate(const uint32_t* sym, int64_t F, int64_t seg, int mh,
                            uint16_t* tf, int32_t* cnt) {
  const int ns = 2 * (mh + 1);
  const int nseg = (int)((F + seg - 1) / seg);
  const int nwork = nseg * ns;
  for (int w = threadIdx.x; w < nwork; w += blockDim.x) {
    const int sg = w / ns, s0 = w - sg * ns;
    const int64_t k0 = (int64_t)sg * seg;
    const int64_t k1 = min<int64_t>(k0 + seg, F);
    MhState st{s0 > mh ? 1 : 0, s0 > mh ? s0 - (mh + 1) : s0};
    int c = 0;
    for (int64_t k = k0; k < k1; k += 16)
      mh_word(st, sym[k >> 4], (int)min<int64_t>(16, k1 - k), mh, c);
    tf[w] = (uint16_t)(st.c2 * (mh + 1) + st.since);
    cnt[w] = c;
  }
}

// ---------------------------------------------------------------------------
// adaptive: per-stream order statistics of the valid levels
// (src/process_tomatis_adaptive.py:123-131: valid = levels > -70;
//  np.percentile(valid, 5), np.percentile(valid, 95), np.median(valid); with no
//  valid level the threshold is np.median(levels)).  Exact selection by an
//  8-bit radix walk over order-preserving u64 keys of the f64 levels, for up
//  to six ranks at once (the two neighbours of each percentile position and
//  the one or two middle ranks); the numpy 'linear' interpolation and median
//  rule are then evaluated in the same IEEE operations as numpy (no
//  contraction), so t_lo_hi_med is bit-identical to the host statistics.
// ---------------------------------------------------------------------------
constexpr double kValidLevel = -70.0;
constexpr int kSelRanks = 6;

// h[d] += 1 for every lane with pred, the wave's equal digits merged into one
// LDS atomic each (up to 4 distinct digits; the rest add per lane)
__device__ __forceinline__ void wave_hist_add(uint32_t* h, uint32_t d, bool pred, int lane) {
  uint64_t todo = __ballot(pred);
  for (int it = 0; it < 4 && todo; ++it) {
    const int leader = __ffsll((long long)todo) - 1;
    const uint32_t ld = (uint32_t)__shfl((int)d, leader, 64);
    const uint64_t same = __ballot(pred && d == ld) & todo;
    if (lane == leader) atomicAdd(&h[ld], (uint32_t)__popcll(same));
    todo &= ~same;
    if ((same >> lane) & 1ull) pred = false;
  }
  if (pred) atomicAdd(&h[d], 1u);
}

__device__ __forceinline__ uint64_t f64_key(double v) {
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ double key_f64(uint64_t k) {
  const uint64_t u = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
  return __longlong_as_double((long long)u);
}

__global__ __launch_bounds__(1024) void k_level_stats(const double* __restrict__ levels,
                                                      const TomatisStream* __restrict__ st,
                                                      double* __restrict__ tlh) {
#pragma clang fp contract(off)
  const int s = blockIdx.x;
  const int64_t F = st[s].n_frames;
  const double* lv = levels + st[s].frame_base;
  __shared__ uint32_t hist[kSelRanks][256];
  __shared__ uint64_t pre[kSelRanks];
  __shared__ int64_t want[kSelRanks];
  __shared__ unsigned long long sh_cnt;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid == 0) sh_cnt = 0;
  __syncthreads();
  unsigned long long c = 0;
  for (int64_t i = tid; i < F; i += blockDim.x) c += (lv[i] > kValidLevel) ? 1 : 0;
  for (int o = 32; o; o >>= 1) c += __shfl_xor(c, o);
  if (lane == 0) atomicAdd(&sh_cnt, c);
  __syncthreads();
  const int64_t nv = (int64_t)sh_cnt;
  const bool all = (nv == 0);   // no valid level: median over every level
  const int64_t n = all ? F : nv;
  if (n == 0) {
    if (tid == 0) {
      // no frame at all: find_optimal_threshold's np.median(levels) of an
      // empty array is NaN (process_tomatis_adaptive.py:124-127)
      tlh[3 * s + 0] = __longlong_as_double(0x7ff8000000000000ll);
      tlh[3 * s + 1] = __longlong_as_double(0x7ff8000000000000ll);
      tlh[3 * s + 2] = __longlong_as_double(0x7ff8000000000000ll);
    }
    return;
  }
  // ranks (numpy 2.x _quantile 'linear': virtual index (n-1)*q)
  const double q[2] = {5.0 / 100.0, 95.0 / 100.0};
  int64_t pi[2], ni[2];
  double gam[2];
  for (int j = 0; j < 2; ++j) {
    const double vi = (double)(n - 1) * q[j];
    const double prev = floor(vi);
    const bool above = vi >= (double)(n - 1);
    pi[j] = above ? n - 1 : (int64_t)prev;
    ni[j] = above ? n - 1 : (int64_t)prev + 1;
    gam[j] = above ? 0.0 : vi - prev;
  }
  const int64_t h = n / 2;
  if (tid == 0) {
    want[0] = pi[0]; want[1] = ni[0]; want[2] = pi[1]; want[3] = ni[1];
    want[4] = (n % 2 == 0) ? h - 1 : h;
    want[5] = h;
    for (int r = 0; r < kSelRanks; ++r) pre[r] = 0;
  }
  __syncthreads();
  for (int pass = 0; pass < 8; ++pass) {
    const int shift = 56 - 8 * pass;
    const uint64_t hmask = pass ? (~0ull << (shift + 8)) : 0ull;
    for (int i = tid; i < kSelRanks * 256; i += blockDim.x) (&hist[0][0])[i] = 0;
    __syncthreads();
    // ranks whose prefixes agree share one histogram (cls: the first such
    // rank); levels cluster, so the adds are aggregated per wave and digit
    uint64_t pr[kSelRanks];
    int cls[kSelRanks];
#pragma unroll
    for (int r = 0; r < kSelRanks; ++r) {
      pr[r] = pre[r];
      cls[r] = r;
      for (int r2 = r - 1; r2 >= 0; --r2)
        if (pr[r2] == pr[r]) cls[r] = r2;
    }
    for (int64_t i0 = 0; i0 < F; i0 += blockDim.x) {  // wave-uniform trip count
      const int64_t i = i0 + tid;
      const double v = i < F ? lv[i] : 0.0;
      const bool ok = i < F && (all || v > kValidLevel);
      const uint64_t k = f64_key(v);
      const uint32_t d = (uint32_t)(k >> shift) & 255u;
#pragma unroll
      for (int r = 0; r < kSelRanks; ++r)
        if (cls[r] == r) wave_hist_add(hist[r], d, ok && (k & hmask) == pr[r], lane);
    }
    __syncthreads();
    if (wv < kSelRanks) {   // wave r resolves rank r's digit
      const int r = wv;
      int cr = 0;
#pragma unroll
      for (int j = 0; j < kSelRanks; ++j)
        if (j == r) cr = cls[j];
      const uint32_t b0 = hist[cr][4 * lane], b1 = hist[cr][4 * lane + 1],
                     b2 = hist[cr][4 * lane + 2], b3 = hist[cr][4 * lane + 3];
      const uint32_t tot = b0 + b1 + b2 + b3;
      uint32_t incl = tot;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(incl, o);
        if (lane >= o) incl += t;
      }
      const int64_t k = want[r];   // rank within the remaining prefix class
      const int64_t ex = (int64_t)(incl - tot);
      if (k >= ex && k < (int64_t)incl) {
        int64_t acc = ex;
        int dsel = 4 * lane;
        const uint32_t bb[4] = {b0, b1, b2, b3};
        for (int j = 0; j < 4; ++j) {
          if (k < acc + (int64_t)bb[j]) { dsel = 4 * lane + j; break; }
          acc += bb[j];
        }
        want[r] = k - acc;
        pre[r] = pre[r] | ((uint64_t)dsel << shift);
      }
    }
    __syncthreads();
  }
  if (tid == 0) {
    double val[kSelRanks];
    for (int r = 0; r < kSelRanks; ++r) val[r] = key_f64(pre[r]);
    double med;
    if (n % 2) med = val[5] + 0.0;
    else med = ((0.0 + val[4]) + val[5]) / 2.0;
    if (all) {
      tlh[3 * s + 0] = __longlong_as_double(0x7ff8000000000000ll);
      tlh[3 * s + 1] = __longlong_as_double(0x7ff8000000000000ll);
      tlh[3 * s + 2] = med;
      return;
    }
    for (int j = 0; j < 2; ++j) {
      const double a = val[2 * j], b = val[2 * j + 1];
      const double d = b - a;
      double lerp = a + d * gam[j];
      if (gam[j] >= 0.5) lerp = b - d * (1.0 - gam[j]);
      tlh[3 * s + j] = lerp;
    }
    tlh[3 * s + 2] = med;
  }
}

// ---------------------------------------------------------------------------
// Speculative bisection (process_tomatis_adaptive.py:133-154, find_optimal_
// threshold): the reference's 30-step bisection is sequential, one threshold
// per step, and k_minhold runs it on one CU per stream.  k_mh_probe instead
// evaluates the next THREE steps at once: the 7 midpoints of the depth-3 tree
// of possible (t_low, t_high) paths, each over a few workgroups, computed by the same
// (lo + hi) / 2 operations the sequential loop would apply along each path.
// The last workgroup of a stream to finish (agent-scope arrival counter)
// walks the taken path with the reference's best-diff, early-exit (diff <
// 0.01) and branch rules, so the result is the sequential bisection's, bit
// for bit, in 10 launches of 7 x parts x n_streams workgroups instead of 30
// steps on n_streams CUs.  An 11th launch builds best_T's transfer tables the
// same way; k_minhold then finishes states / alpha from them.
// Streams whose tables spill to the HBM workspace keep the sequential kernel.
// ---------------------------------------------------------------------------
struct MhBisect {
  double lo, hi, best_T, best_diff;
  int32_t it, done, arrive, pad;
};
constexpr int kMhProbes = 7;

__global__ void k_mh_init(const TomatisStream* __restrict__ st, int n_streams,
                          const double* __restrict__ tlh, MhBisect* __restrict__ bs) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_streams) return;
  const double lo = tlh[3 * s + 0], hi = tlh[3 * s + 1];
  MhBisect B;
  B.lo = lo;
  B.hi = hi;
  B.best_T = tlh[3 * s + 2];
  B.best_diff = 1.0;
  B.it = 0;
  B.done = (st[s].n_frames > 0 && !(lo != lo)) ? 0 : 1;
  B.arrive = 0;
  B.pad = 0;
  bs[s] = B;
}

// One probe (or the final threshold) per (stream, slot) is split over `parts`
// workgroups, each simulating a contiguous range of segments from every start
// state into the slot's global tables; the last of them (agent-scope arrival
// counter) stages the tables in LDS and runs the segment chain.  Slots 0-6:
// the tree midpoints (then, per stream, the last probe walks the taken path);
// slot 7: best_T, whose tables k_minhold consumes.
constexpr int kMhSlots = kMhProbes + 1;

__global__ __launch_bounds__(1024) void k_mh_probe(const double* __restrict__ levels,
                                                   const TomatisStream* __restrict__ st,
                                                   double target, double hyst, int mh,
                                                   MhBisect* __restrict__ bs,
                                                   int32_t* __restrict__ counts,
                                                   uint16_t* __restrict__ gtf,
                                                   int32_t* __restrict__ gcnt,
                                                   const int64_t* __restrict__ goff,
                                                   int32_t* __restrict__ arrive, int final_T) {
  const int s = blockIdx.x, j = final_T ? kMhProbes : blockIdx.y;
  const int part = blockIdx.z, parts = gridDim.z;
  const MhBisect B = bs[s];  // written by the previous launch
  if (B.done && !final_T) return;  // uniform over the stream's workgroups
  const TomatisStream S = st[s];
  const int64_t F = S.n_frames;
  if (F == 0) return;
  const double* lv = levels + S.frame_base;
  const int ns = 2 * (mh + 1);
  const int64_t seg = mh_seg_len(F, ns);
  const int nseg = (int)((F + seg - 1) / seg);
  __shared__ uint16_t tf_l[kMhLdsTf];
  __shared__ int32_t cnt_l[kMhLdsTf];
  __shared__ uint32_t sym[kMhLdsSym];
  __shared__ int last;
  double t_mid;
  if (final_T) {
    t_mid = B.best_T;
  } else {
    // node j (BFS order; child 2n+1: c2 < target, so t_high = mid; 2n+2: t_low = mid)
    const int depth = j == 0 ? 0 : (j < 3 ? 1 : 2);
    int path[2] = {0, 0};
    for (int n = j, d = depth; d > 0; --d) {
      path[d - 1] = n;
      n = (n - 1) / 2;
    }
    double lo = B.lo, hi = B.hi;
    for (int d = 0; d < depth; ++d) {
      const double mid = (lo + hi) / 2;
      if (path[d] & 1) hi = mid;
      else lo = mid;
    }
    t_mid = (lo + hi) / 2;
  }
  const double ton = t_mid + hyst / 2, toff = t_mid - hyst / 2;
  // this workgroup's segments [g0, g1): symbols of their frames, then every
  // (segment, start state) walked into the slot's tables
  const int g0 = (int)((int64_t)nseg * part / parts), g1 = (int)((int64_t)nseg * (part + 1) / parts);
  uint16_t* tf = gtf + goff[s] + (int64_t)j * nseg * ns;
  int32_t* cn = gcnt + goff[s] + (int64_t)j * nseg * ns;
  if (g0 < g1) {
    const int64_t k0 = (int64_t)g0 * seg, k1 = min<int64_t>((int64_t)g1 * seg, F);
    mh_symbols(lv + k0, k1 - k0, ton, toff, sym);  // seg % 16 == 0: word-aligned
    __syncthreads();
    const int nwork = (g1 - g0) * ns;
    for (int w = threadIdx.x; w < nwork; w += blockDim.x) {
      const int sg = w / ns, s0 = w - sg * ns;
      const int64_t a = (int64_t)sg * seg, b = min<int64_t>(a + seg, k1 - k0);
      MhState q{s0 > mh ? 1 : 0, s0 > mh ? s0 - (mh + 1) : s0};
      int c = 0;
      for (int64_t k = a; k < b; k += 16) mh_word(q, sym[k >> 4], (int)min<int64_t>(16, b - k), mh, c);
      const int64_t e = (int64_t)(g0 + sg) * ns + s0;
      tf[e] = (uint16_t)(q.c2 * (mh + 1) + q.since);
      cn[e] = c;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();  // this workgroup's tables before its arrival
    const int old = __hip_atomic_fetch_add(arrive + (int64_t)s * kMhSlots + j, 1, __ATOMIC_ACQ_REL,
                                           __HIP_MEMORY_SCOPE_AGENT);
    last = old == parts - 1;
  }
  __syncthreads();
  if (!last || final_T) {
    if (last && threadIdx.x == 0) arrive[(int64_t)s * kMhSlots + j] = 0;
    return;  // the final tables are read by k_minhold (next launch)
  }
  // the other workgroups' tables.  Ordering: every producer's tables are
  // released by its __threadfence() before its arrival; the acquire side is
  // thread 0's agent-scope ACQ_REL fetch_add above (it MUST stay acq_rel: a
  // relaxed arrival would let these loads see stale tables, and the
  // speculative and serial bisections would then differ only intermittently),
  // extended to the other threads by the __syncthreads() after it; the loads
  // are agent scope (served by L2, never a stale L1 line).  No extra
  // cache-wide acquire fence: it would invalidate this CU's L1 under the
  // concurrent probes for nothing.
  for (int e = threadIdx.x; e < nseg * ns; e += blockDim.x) {
    tf_l[e] = __hip_atomic_load(tf + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    cnt_l[e] = __hip_atomic_load(cn + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    arrive[(int64_t)s * kMhSlots + j] = 0;
    int id = mh, c = 0;  // start state: C1, since = mh
    for (int g = 0; g < nseg; ++g) {
      c += cnt_l[g * ns + id];
      id = tf_l[g * ns + id];
    }
    __hip_atomic_store(counts + (int64_t)s * kMhProbes + j, c, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    const int old = __hip_atomic_fetch_add(&bs[s].arrive, 1, __ATOMIC_ACQ_REL,
                                           __HIP_MEMORY_SCOPE_AGENT);
    if (old == kMhProbes - 1) {  // last of the stream's probes: walk the taken path
      MhBisect R = B;
      int node = 0;
      for (int d = 0; d < 3; ++d) {
        const double mid = (R.lo + R.hi) / 2;
        const int cnv = __hip_atomic_load(counts + (int64_t)s * kMhProbes + node,
                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const double c2 = (double)cnv / (double)F;
        const double diff = fabs(c2 - target);
        if (diff < R.best_diff) {
          R.best_diff = diff;
          R.best_T = mid;
        }
        ++R.it;
        if (diff < 0.01) {
          R.done = 1;
          break;
        }
        if (c2 < target) {
          R.hi = mid;
          node = 2 * node + 1;
        } else {
          R.lo = mid;
          node = 2 * node + 2;
        }
      }
      if (R.it >= 30) R.done = 1;
      R.arrive = 0;
      bs[s] = R;  // read by the next launch
    }
  }
}

__global__ __launch_bounds__(1024) void k_minhold(const double* __restrict__ levels,
                                                  const TomatisStream* __restrict__ st,
                                                  const double* __restrict__ tlh,
                                                  double target, double hyst, int mh, int xf,
                                                  int alpha_adaptive, uint16_t* __restrict__ ws_tf,
                                                  int32_t* __restrict__ ws_cnt,
                                                  const int64_t* __restrict__ ws_off,
                                                  uint32_t* __restrict__ ws_sym,
                                                  const int64_t* __restrict__ ws_soff,
                                                  double* __restrict__ t_out,
                                                  uint8_t* __restrict__ states,
                                                  uint16_t* __restrict__ rows,
                                                  double* __restrict__ alpha,
                                                  const MhBisect* __restrict__ bisected,
                                                  const uint16_t* __restrict__ gtf,
                                                  const int32_t* __restrict__ gcnt,
                                                  const int64_t* __restrict__ goff) {
  const int s = blockIdx.x;
  const TomatisStream S = st[s];
  const int64_t F = S.n_frames;
  const double* lv = levels + S.frame_base;
  const int ns = 2 * (mh + 1);
  const int64_t seg = mh_seg_len(F, ns);
  const int nseg = (int)((F + seg - 1) / seg);
  const int init_id = mh;  // C1, since = mh
  __shared__ uint16_t tf_l[kMhLdsTf];
  __shared__ int32_t cnt_l[kMhLdsTf];
  __shared__ uint32_t sym_l[kMhLdsSym];
  const bool tf_lds = (int64_t)nseg * ns <= kMhLdsTf;
  uint16_t* tf = tf_lds ? tf_l : ws_tf + ws_off[s];
  int32_t* cnt = tf_lds ? cnt_l : ws_cnt + ws_off[s];
  const int64_t nw = (F + 15) >> 4;
  uint32_t* sym = nw <= kMhLdsSym ? sym_l : ws_sym + ws_soff[s];
  __shared__ double sh_T;
  __shared__ int sh_count;
  double t_low = tlh[3 * s + 0], t_high = tlh[3 * s + 1];
  double best_T = tlh[3 * s + 2], best_diff = 1.0;
  const bool have_valid = !(t_low != t_low);
  if (bisected) {
    best_T = bisected[s].best_T;  // k_mh_probe rounds did the bisection
  } else if (F > 0 && have_valid) {
    for (int it = 0; it < 30; ++it) {
      const double t_mid = (t_low + t_high) / 2;
      const double ton = t_mid + hyst / 2, toff = t_mid - hyst / 2;
      mh_symbols(lv, F, ton, toff, sym);
      __syncthreads();
      mh_simulate(sym, F, seg, mh, tf, cnt);
      __syncthreads();
      if (threadIdx.x == 0) {
        int id = init_id, c = 0;
        for (int g = 0; g < nseg; ++g) {
          c += cnt[(int64_t)g * ns + id];
          id = tf[(int64_t)g * ns + id];
        }
        sh_count = c;
      }
      __syncthreads();
      const double c2 = (double)sh_count / (double)F;
      const double diff = fabs(c2 - target);
      if (diff < best_diff) {
        best_diff = diff;
        best_T = t_mid;
      }
      if (diff < 0.01) break;
      if (c2 < target) t_high = t_mid;
      else t_low = t_mid;
    }
  }
  if (threadIdx.x == 0) {
    sh_T = best_T;
    if (t_out) t_out[s] = best_T;
  }
  __syncthreads();
  const double T = sh_T;
  const double ton = T + hyst / 2, toff = T - hyst / 2;
  // final states: segment transfer tables, sequential segment starts, then
  // every segment re-walked from its start writing states
  mh_symbols(lv, F, ton, toff, sym);
  if (bisected) {  // tables of best_T from k_mh_probe's final slot: stage in LDS
    const int64_t o = goff[s] + (int64_t)kMhProbes * nseg * ns;
    for (int e = threadIdx.x; e < nseg * ns; e += blockDim.x) {
      tf[e] = gtf[o + e];
      cnt[e] = gcnt[o + e];
    }
    __syncthreads();
  } else {
    __syncthreads();
    mh_simulate(sym, F, seg, mh, tf, cnt);
    __syncthreads();
  }
  __shared__ uint16_t seg_start[4096];
  if (threadIdx.x == 0) {
    int id = init_id;
    for (int g = 0; g < nseg; ++g) {
      seg_start[g] = (uint16_t)id;
      id = tf[(int64_t)g * ns + id];
    }
  }
  __syncthreads();
  // the states also go to LDS (the transfer counts are no longer needed) so the
  // alpha passes below read them without HBM round trips
  uint8_t* st_l = (F <= (int64_t)sizeof(cnt_l)) ? reinterpret_cast<uint8_t*>(cnt_l) : nullptr;
  for (int g = threadIdx.x; g < nseg; g += blockDim.x) {
    const int id0 = seg_start[g];
    MhState stt{id0 > mh ? 1 : 0, id0 > mh ? id0 - (mh + 1) : id0};
    const int64_t k0 = (int64_t)g * seg;
    const int64_t k1 = min<int64_t>(k0 + seg, F);
    for (int64_t k = k0; k < k1; k += 16) {
      const uint32_t w = sym[k >> 4];
      const int n = (int)min<int64_t>(16, k1 - k);
      for (int j = 0; j < n; ++j) {
        int c = 0;
        mh_word(stt, w >> (2 * j), 1, mh, c);
        const uint8_t v = stt.c2 ? 2 : 1;
        states[S.frame_base + k + j] = v;
        if (st_l) st_l[k + j] = v;
      }
    }
  }
  __syncthreads();
  // alpha (process_tomatis_adaptive.py:253-265): a_0 = target(s_0), then
  // a_k = step(a_{k-1}, target(s_k)).  Segment-parallel and exact, as the xfade
  // alpha: after J = xf + 2 equal states alpha equals the target exactly (and
  // a_0 is exact), so every chunk computes from its first such "sync" frame on;
  // one thread chains the chunk carries; the prefixes follow from the carries.
  if (F > 0) {
    const double step = xf > 0 ? 1.0 / xf : 1.0;
    const int xfe = xf > 0 ? xf : 1;
    const int J = xf + 2;
    const uint8_t* stt = st_l ? st_l : states + S.frame_base;
    const int64_t CHK = max<int64_t>(256, (F + kMhAlphaChunks - 1) / kMhAlphaChunks);
    const int nch = (int)((F + CHK - 1) / CHK);
    __shared__ int32_t a_q[kMhAlphaChunks];
    __shared__ double a_fin[kMhAlphaChunks], a_carry[kMhAlphaChunks];
    auto put = [&](int64_t k, double a) {
      const int64_t f = S.frame_base + k;
      if (alpha) alpha[f] = a;
      if (rows) rows[f] = (uint16_t)(2 + (int)rint(a * xfe));
    };
    for (int c = threadIdx.x; c < nch; c += blockDim.x) {
      const int64_t k0 = c * CHK;
      const int nf = (int)min<int64_t>(CHK, F - k0);
      int q = 0;
      if (k0 > 0) {
        uint8_t prev = stt[k0 - 1];
        int run = 1;
        int64_t k = k0 - 2;
        for (; k >= 0 && run < J && stt[k] == prev; --k) ++run;
        if (k < 0) run = J;  // equal back to frame 0, whose alpha is exact
        q = nf;
        for (int j = 0; j < nf; ++j) {
          const uint8_t t = stt[k0 + j];
          run = (t == prev) ? min(run + 1, J) : 1;
          prev = t;
          if (xf == 0 || run >= J) {
            q = j;
            break;
          }
        }
      }
      a_q[c] = q;
      if (q < nf) {
        double a = stt[k0 + q] == 2 ? 1.0 : 0.0;
        put(k0 + q, a);
        for (int j = q + 1; j < nf; ++j) {
          a = alpha_step(a, stt[k0 + j] == 2 ? 1.0 : 0.0, step);
          put(k0 + j, a);
        }
        a_fin[c] = a;
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      double cur = 0.0;
      for (int c = 0; c < nch; ++c) {
        a_carry[c] = cur;
        const int64_t k0 = c * CHK;
        const int nf = (int)min<int64_t>(CHK, F - k0);
        if (a_q[c] < nf) {
          cur = a_fin[c];
        } else {
          for (int j = 0; j < nf; ++j) cur = alpha_step(cur, stt[k0 + j] == 2 ? 1.0 : 0.0, step);
        }
      }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < nch; c += blockDim.x) {
      const int64_t k0 = c * CHK;
      double a = a_carry[c];
      for (int j = 0; j < a_q[c]; ++j) {
        a = alpha_step(a, stt[k0 + j] == 2 ? 1.0 : 0.0, step);
        put(k0 + j, a);
      }
    }
  }
  (void)alpha_adaptive;
}

// ===========================================================================
// limiter fix-up, absmax, scale, synth
// ===========================================================================
struct ChunkDesc {
  int32_t s, c;
  int64_t p0, p1;  // output-relative sample range [p0, p1)
};

// sel 0: every chunk; 1: all but the edge chunks of edge_mask; 2: only those
__global__ __launch_bounds__(256) void k_limiter(float* __restrict__ y,
                                                 const TomatisStream* __restrict__ st,
                                                 const ChunkDesc* __restrict__ chunks,
                                                 const uint32_t* __restrict__ peaks, float limit,
                                                 int ch, int sel, int edge_mask) {
  const ChunkDesc C = chunks[blockIdx.y];
  const TomatisStream S = st[C.s];
  if (sel) {
    const bool edge = ((edge_mask & 1) && C.c == 0) || ((edge_mask & 2) && C.c == S.n_chunks - 1);
    if (edge != (sel == 2)) return;
  }
  const float peak = __uint_as_float(peaks[S.chunk_base + C.c]);
  if (!(peak > limit)) return;
  const float sc = limit / peak;
  const int64_t n = (C.p1 - C.p0) * ch;
  float* base = y + S.out_off + C.p0 * ch;
  // 16-byte accesses: scalar head to alignment, float4 body, scalar tail
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t head = std::min<int64_t>(n, (int64_t)((16 - ((uintptr_t)base & 15)) & 15) >> 2);
  const int64_t nb = (n - head) >> 2;
  if (tid < head) base[tid] = base[tid] * sc;
  float4* __restrict__ b4 = reinterpret_cast<float4*>(base + head);
  for (int64_t i = tid; i < nb; i += stride) {
    float4 v = b4[i];
    v.x = v.x * sc;
    v.y = v.y * sc;
    v.z = v.z * sc;
    v.w = v.w * sc;
    b4[i] = v;
  }
  const int64_t t0 = head + 4 * nb;
  if (tid < n - t0) base[t0 + tid] = base[t0 + tid] * sc;
}

__device__ __forceinline__ void absmax_body(const float* __restrict__ x, int64_t n,
                                            uint32_t* __restrict__ out, int64_t tid,
                                            int64_t stride) {
  // scalar head up to 16-byte alignment, float4 body (4 independent loads in
  // flight per thread per iteration), scalar tail
  const int64_t head = std::min<int64_t>(n, (int64_t)((16 - ((uintptr_t)x & 15)) & 15) >> 2);
  const int64_t nb = (n - head) >> 2;
  const float4* __restrict__ x4 = reinterpret_cast<const float4*>(x + head);
  float m0 = 0.f, m1 = 0.f, m2 = 0.f, m3 = 0.f;
  if (tid < head) m0 = fabsf(x[tid]);
  int64_t i = tid;
  for (; i + 3 * stride < nb; i += 4 * stride) {
    const float4 a = x4[i], b = x4[i + stride], c = x4[i + 2 * stride], d = x4[i + 3 * stride];
    m0 = fmaxf(m0, fmaxf(fmaxf(fabsf(a.x), fabsf(a.y)), fmaxf(fabsf(a.z), fabsf(a.w))));
    m1 = fmaxf(m1, fmaxf(fmaxf(fabsf(b.x), fabsf(b.y)), fmaxf(fabsf(b.z), fabsf(b.w))));
    m2 = fmaxf(m2, fmaxf(fmaxf(fabsf(c.x), fabsf(c.y)), fmaxf(fabsf(c.z), fabsf(c.w))));
    m3 = fmaxf(m3, fmaxf(fmaxf(fabsf(d.x), fabsf(d.y)), fmaxf(fabsf(d.z), fabsf(d.w))));
  }
  for (; i < nb; i += stride) {
    const float4 a = x4[i];
    m0 = fmaxf(m0, fmaxf(fmaxf(fabsf(a.x), fabsf(a.y)), fmaxf(fabsf(a.z), fabsf(a.w))));
  }
  const int64_t t0 = head + nb * 4;
  if (t0 + tid < n) m1 = fmaxf(m1, fabsf(x[t0 + tid]));
  float m = fmaxf(fmaxf(m0, m1), fmaxf(m2, m3));
  m = wave_max(m);
  // one atomic per block: same-address atomics serialise in L2 (one per wave
  // cost ~80 us for a 5-min stream)
  __shared__ float wm[4];
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    m = fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]));
    if (m > 0.f) atomicMax(out, __float_as_uint(m));
  }
}
__global__ __launch_bounds__(256) void k_absmax(const float* __restrict__ x, int64_t n,
                                                uint32_t* __restrict__ out) {
  absmax_body(x, n, out, (int64_t)blockIdx.x * blockDim.x + threadIdx.x,
              (int64_t)gridDim.x * blockDim.x);
}
// every stream of a plan in one launch: blockIdx.y = stream
__global__ __launch_bounds__(256) void k_absmax_streams(const float* __restrict__ x,
                                                        const TomatisStream* __restrict__ st,
                                                        int ch, uint32_t* __restrict__ out) {
  const TomatisStream S = st[blockIdx.y];
  absmax_body(x + S.in_off, S.n * ch, out + blockIdx.y,
              (int64_t)blockIdx.x * blockDim.x + threadIdx.x, (int64_t)gridDim.x * blockDim.x);
}

__global__ __launch_bounds__(256) void k_scale_copy(const float* __restrict__ x,
                                                    float* __restrict__ y, int64_t n, float s) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    y[i] = x[i] * s;
}

// HBM bandwidth probe (bench.py's roofline.achievable_peak):
// y = x, one 16-byte load and store per thread, one 256-thread block per 4 KB
// (tools/copy_probe.hip: 6.2 TB/s on MI355X, the fastest of the grid-stride,
// unrolled, streaming-hint and per-block-chunk forms measured)
__global__ __launch_bounds__(256) void k_copy_probe(const float4* __restrict__ x,
                                                    float4* __restrict__ y, int64_t n4) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n4) y[i] = x[i];
}

// PCM <-> float at the file boundary, libsndfile's
// normalisation as audio_io implements it: int -> float divides by 2^(bps-1)
// (correctly rounded: double division, then float); float -> int multiplies by
// 2^(bps-1) - 1 in double, rounds half to even and clips to the bps range.
__global__ __launch_bounds__(256) void k_pcm_to_float(const int32_t* __restrict__ pcm, int64_t n,
                                                      double inv, float* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (float)((double)pcm[i] * inv);
}

__global__ __launch_bounds__(256) void k_float_to_pcm(const float* __restrict__ x, int64_t n,
                                                      double scale, double lo, double hi,
                                                      int32_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    double v = rint((double)x[i] * scale);
    v = v < lo ? lo : (v > hi ? hi : v);
    out[i] = (int32_t)v;
  }
}

__device__ __forceinline__ uint32_t lowbias32(uint32_t v) {
  v ^= v >> 16;
  v *= 0x7FEB352Du;
  v ^= v >> 15;
  v *= 0x846CA68Bu;
  v ^= v >> 16;
  return v;
}

__global__ __launch_bounds__(256) void k_synth(float* __restrict__ x, int64_t n, int ch, int sr,
                                               uint32_t seed, int64_t start) {
  const uint32_t base = (uint32_t)((uint64_t)seed * 4u + 0x1234567u);
  uint32_t key[4];
  for (int j = 0; j < 4; ++j) key[j] = lowbias32(base + (uint32_t)j * 0x9E3779B9u);
  const int64_t period = 3LL * sr, half = period / 2;
  const int64_t ramp = max(1, sr / 100);
  const float LOUD = 0.1f, QUIET = 0.001f;
  const float d = QUIET - LOUD;
  const int64_t total = n * ch;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t smp = start + e / ch;
    const uint64_t eg = (uint64_t)(smp * ch + (e % ch));
    const uint32_t lo = (uint32_t)eg, hi = (uint32_t)(eg >> 32);
    float u[4];
    for (int j = 0; j < 4; ++j) {
      const uint32_t v = lowbias32(lo ^ lowbias32(hi + key[j]));
      u[j] = (float)(v >> 8) * (1.0f / 16777216.0f);
    }
    const float g = (((u[0] + u[1]) + (u[2] + u[3])) - 2.0f) * 1.7320508f;
    const int64_t ph = smp % period;
    float amp = ph < half ? QUIET : LOUD;
    if (ph < ramp) amp = LOUD + d * ((float)ph / (float)ramp);
    else if (ph >= half && ph < half + ramp) amp = QUIET + (-d) * ((float)(ph - half) / (float)ramp);
    float v = g * amp;
    v = fminf(fmaxf(v, -1.0f), 1.0f);
    x[e] = v;
  }
}

}  // namespace


// ===========================================================================
// Host side: plan + C ABI
// ===========================================================================
struct tomatis_plan_s {
  TomatisPlanDesc d{};
  int32_t n_streams = 0;
  int64_t total_frames = 0;
  int32_t total_chunks = 0;
  int P = 0, NR = 32, SH = 0, rmax = 1;
  bool generic = false;
  bool fx = false;  // fused kernel runs the single-exchange FFT (tm_fft.h fftx_*)
  bool lds = false;        // any-size path (k_stft_lds + k_ola_gather_lds)
  float2* twL = nullptr;   // lds path: exp(-2 pi i t / N)
  std::vector<TomatisStream> hs;
  int lvl_nf = 0;
  // device
  TomatisStream* st = nullptr;
  Run* runs = nullptr;
  int n_runs = 0;
  std::vector<Run> hruns;  // host copy of the runs
  LvlBlock* lblocks = nullptr;
  int n_lblocks = 0;
  GateSeg* segs = nullptr;
  int n_segs = 0;
  int32_t* seg_first = nullptr;
  int32_t* seg_count = nullptr;
  GateSeg* asegs = nullptr;        // xfade alpha segments (kASeg frames)
  int n_asegs = 0;
  int32_t* aseg_first = nullptr;
  int32_t* aseg_count = nullptr;
  uint16_t* tf = nullptr;
  uint16_t* seg_start = nullptr;
  float* win = nullptr;
  float* winS = nullptr;  // synthesis window x the register FFT's inverse output scales
  float* win2 = nullptr;
  float* winv = nullptr;
  cf* twN = nullptr;
  cf* twP = nullptr;
  cf* scratch = nullptr;
  int64_t* pos_base = nullptr;
  int64_t total_out = 0;
  ChunkDesc* chunks = nullptr;
  int n_chunkdesc = 0;
  int64_t max_chunk = 0;
  uint16_t* mh_tf = nullptr;
  int32_t* mh_cnt = nullptr;
  int64_t* mh_off = nullptr;
  uint32_t* mh_sym = nullptr;
  int64_t* mh_soff = nullptr;
  MhBisect* mh_bs = nullptr;  // speculative bisection state per stream
  int mh_serial = 0;          // TOMATIS_OPT_MINHOLD_SERIAL
  int32_t* mh_pc = nullptr;   // probe counts [stream][kMhProbes]
  uint16_t* mh_gtf = nullptr; // probe tables [stream][kMhSlots][nseg * ns]
  int32_t* mh_gcnt = nullptr;
  int64_t* mh_goff = nullptr;
  int32_t* mh_arr = nullptr;  // probe arrival counters [stream][kMhSlots]
  int mh_parts = 1;           // workgroups per probe
  float* gperm = nullptr;
  int gperm_rows = 0;
  // fused limiter
  uint32_t* chunk_need = nullptr;
  uint32_t* chunk_done = nullptr;
  int64_t* chunk_rng = nullptr;
  uint32_t* err = nullptr;
  int fuse_span = 0;  // max runs contributing to one chunk
  int64_t run_slots = 0;  // resident sequences of the fused kernel
  int edge_mask = 0;      // set for one tomatis_stft_ola_limited_edges call
  int fuse_enabled = 1;   // TOMATIS_OPT_FUSE_LIMITER
  int lim_spin = 1 << 18; // TOMATIS_OPT_LIMITER_SPIN: fused-limiter wait bound (polls)
  // pipelined batches (tomatis_stft_ola_gated_pipelined): per run the previous
  // batch's blocks to rescale in the frame loop (k_r2_plan output)
  uint32_t* xs_pieces = nullptr;
  int xs_max_pieces = 0;
  // in-kernel levels + gate (tomatis_stft_ola_gated): per-run carry-in
  int32_t* gate_carry = nullptr;
  int gate_cap = 0;
  uint16_t* gate_tf = nullptr;     // chained runs' transfer tables [gate_cap][D + 2]
  double* gate_acarry = nullptr;   // cross-fade: alpha before each run's first frame
  double* gate_aout = nullptr;     // cross-fade: the caller's per-frame alpha (set_gate_alpha)
  // the look-back the carries in gate_carry belong to (input, run layout)
  const float* gl_x = nullptr;
  int gl_gen = -1;
  int runs_gen = 0;                // bumped whenever build_runs re-lays the runs
  // run-scan gate (exclusive on/off predicates)
  bool gate_excl = false;
  void* gsum = nullptr;
  void* gcarry = nullptr;
  void* gcarry_in = nullptr;  // time shards: carry-in per stream
  int32_t* aq = nullptr;      // xfade alpha passes: sync frame per gate segment
  double* afin = nullptr;     //   alpha at the segment end (when synced)
  double* acin = nullptr;     //   carry-in alpha per segment
  // streaming levels (hop % 128 == 0): per-stream 8-block groups and leaves
  bool leaf_path = false;
  int64_t n_groups = 0;
  int64_t max_groups = 0;          // most groups of one stream (k_leaves grid x)
  int64_t* grp_base = nullptr;
  int64_t* leaf_base = nullptr;
  void* leaves = nullptr;
  // levels for any n_fft (k_levels_any): numpy pairwise leaves + postfix program
  bool lvl_any = false;
  int2* pw_leaf = nullptr;
  int16_t* pw_prog = nullptr;
  int n_pw_leaf = 0, n_pw_prog = 0;
  // any-size transform: FFT length M (= n_fft, or Bluestein's power of two)
  int lds_M = 0;
  bool blue = false;
  float2* blue_b = nullptr;   // chirp exp(i pi n^2 / N), n < N
  float2* blue_h = nullptr;   // FFT_M of the chirp filter / M
  float2* glb_work = nullptr; // M > kLdsMaxM: per-block ping-pong buffers in HBM
  int glb_blocks = 0;
};

namespace {

int hipfail(hipError_t e) { return e == hipSuccess ? TOMATIS_OK : TOMATIS_E_HIP; }

template <typename T>
int dalloc_copy(T** dst, const std::vector<T>& v) {
  *dst = nullptr;
  if (v.empty()) return TOMATIS_OK;
  if (hipMalloc(reinterpret_cast<void**>(dst), v.size() * sizeof(T)) != hipSuccess) {
    *dst = nullptr;
    return TOMATIS_E_NOMEM;
  }
  return hipfail(hipMemcpy(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
}

void dfree(void* p) {
  if (p) (void)hipFree(p);
}


int launch_check() { return hipfail(hipGetLastError()); }


}  // namespace

namespace tshared {
// development overrides (tomatis_set_dev_option); -1 = the default
constexpr int kDevKeys = 16;
static int g_dev[kDevKeys] = {-1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1};
int dev_opt(int key, int dflt) {
  const int v = (key > 0 && key < kDevKeys) ? g_dev[key] : -1;
  return v < 0 ? dflt : v;
}
}  // namespace tshared

extern "C" {

int tomatis_abi_version(void) { return TOMATIS_ABI_VERSION; }

const char* tomatis_status_string(int s) {
  switch (s) {
    case TOMATIS_OK: return "ok";
    case TOMATIS_E_ARG: return "invalid argument";
    case TOMATIS_E_UNSUPPORTED: return "configuration not supported by the gfx950 kernels";
    case TOMATIS_E_HIP: return "HIP runtime error";
    case TOMATIS_E_NOMEM: return "device allocation failed";
    default: return "unknown status";
  }
}

int tomatis_plan_destroy(tomatis_plan_t p) {
  if (!p) return TOMATIS_OK;
  void* ptrs[] = {p->st, p->runs, p->lblocks, p->segs, p->seg_first, p->seg_count, p->tf,
                  p->asegs, p->aseg_first, p->aseg_count,
                  p->seg_start, p->win, p->winS, p->win2, p->winv, p->twN, p->twP, p->scratch,
                  p->pos_base, p->chunks, p->mh_tf, p->mh_cnt, p->mh_off, p->mh_sym, p->mh_soff, p->mh_bs, p->mh_pc, p->mh_gtf, p->mh_gcnt, p->mh_goff, p->mh_arr, p->gperm,
                  p->grp_base, p->leaf_base, p->leaves, p->gsum, p->gcarry, p->gcarry_in,
                  p->aq, p->afin, p->acin,
                  p->chunk_need, p->chunk_done, p->chunk_rng, p->err, p->twL,
                  p->xs_pieces, p->gate_carry,
                  p->gate_tf, p->gate_acarry,
                  p->pw_leaf, p->pw_prog, p->blue_b, p->blue_h, p->glb_work};
  for (void* q : ptrs) dfree(q);
  delete p;
  return TOMATIS_OK;
}

int64_t tomatis_plan_total_frames(tomatis_plan_t p) { return p ? p->total_frames : -1; }
int32_t tomatis_plan_total_chunks(tomatis_plan_t p) { return p ? p->total_chunks : -1; }

// no float32 bit pattern can satisfy both gate predicates (run-scan gate valid)
static bool gate_exclusive(const TomatisStream& S) {
  auto in = [](uint32_t b, const uint32_t* e, int n) {
    for (int i = 0; i < n; ++i)
      if (e[i] == b) return true;
    return false;
  };
  auto on = [&](uint32_t b) { return (b >= S.on_bits) != in(b, S.on_exc, S.n_on_exc); };
  auto off = [&](uint32_t b) { return (b <= S.off_bits) != in(b, S.off_exc, S.n_off_exc); };
  if (S.n_on_exc < 0 || S.n_on_exc > 4 || S.n_off_exc < 0 || S.n_off_exc > 4) return false;
  if (S.on_bits <= S.off_bits) return false;
  for (int i = 0; i < S.n_on_exc; ++i)
    if (on(S.on_exc[i]) && off(S.on_exc[i])) return false;
  for (int i = 0; i < S.n_off_exc; ++i)
    if (on(S.off_exc[i]) && off(S.off_exc[i])) return false;
  return true;
}

// Runs of the fused kernel (plan creation), then the fused-limiter accounting
// that depends on them.
static int build_runs(tomatis_plan_s* p) {
  const TomatisPlanDesc& d = p->d;
  const int N = d.n_fft, hop = d.hop, P = p->P;
  const int ns = p->n_streams;
  int rc;
  const int64_t tf_total = std::max<int64_t>(1, p->total_frames);
  // Runs.  Per stream, the emitted frames [e_lo, e_hi) whose run can take the
  // fused kernel's interior loop (full frame loads back to the warm-up frames,
  // full interior output blocks, not the stream's last frame) are cut into
  // equal runs; the few edge frames before/after form one generic run each.
  // One run per resident sequence slot of the fused kernel (a single wave of
  // blocks, every wave busy to the end), at least 48 frames per interior run
  // so the rmax-1 warm-up frames per run stay a few percent.
  const int rmax_ = (N + hop - 1) / hop;
  const bool fast_ok = !p->generic && P == 64 && dev_opt(TOMATIS_DEV_FAST_LOOP, 1) != 0;
  std::vector<int64_t> e_lo(ns, 0), e_hi(ns, 0);
  int64_t fast_total = 0, n_edge = 0;
  for (int s = 0; s < ns; ++s) {
    const TomatisStream& S = p->hs[s];
    const int64_t F = S.n_frames;
    int64_t lo = F, hi = F;
    if (fast_ok && F > 0) {
      auto sk = [&](int64_t k) { return S.first_start + k * hop; };
      auto ceil_div = [](int64_t a_, int64_t b_) { return a_ >= 0 ? (a_ + b_ - 1) / b_ : -((-a_) / b_); };
      lo = rmax_ - 1;                                                   // not an edge frame
      lo = std::max(lo, ceil_div(S.out_begin - S.first_start, hop));     // s_k >= out_begin
      lo = std::max(lo, ceil_div(-S.first_start, hop) + rmax_ - 1);      // warm-up frames load fully
      // s_k + hop <= out_end, s_k + N <= n, k <= F - 2
      hi = F - 1;
      const int64_t out_end = S.out_begin + S.out_len;
      auto fdiv = [](int64_t a_, int64_t b_) { return a_ >= 0 ? a_ / b_ : -((-a_ + b_ - 1) / b_); };
      hi = std::min(hi, fdiv(out_end - hop - S.first_start, hop) + 1);
      hi = std::min(hi, fdiv(S.n - N - S.first_start, hop) + 1);
      lo = std::max<int64_t>(0, lo);
      if (hi - lo < 48) lo = hi = F;  // too short: all generic
      else {
        (void)sk;
        n_edge += (lo > 0) + (hi < F);
      }
    }
    e_lo[s] = lo;
    e_hi[s] = hi;
    fast_total += hi - lo;
  }
  // resident sequence slots of the fused kernel
  int64_t slots;
  {
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) == hipSuccess)
      (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    slots = (int64_t)std::max(1, ncu) * (p->generic ? 8 : transform_slots_per_cu(P, p->NR));
    const int dslots = dev_opt(TOMATIS_DEV_SLOTS, 0);  // tests: long runs on small inputs
    if (dslots > 0) slots = dslots;
  }
  p->run_slots = slots;
  // Runs the in-kernel gate may take (tomatis_stft_ola_gated: standard mode at
  // n_fft 2048) are at most kGateLookbackMax frames, so every run's look-back
  // can chain to its predecessor's carry (k_gate_carry): a batch larger than
  // slots x kGateLookbackMax frames gets more rounds of runs instead of longer
  // runs, and a stream hovering inside the hysteresis band never sends the
  // pass back to the two-pass chain (src/process_tomatis.py:373-385 has no
  // horizon either)
  const bool gate_runs = d.alpha_mode == 0 && N == 2048 && P == 64 && !p->generic && !p->lds;
  // rounds: the runs fill the slots this many times over, in stream/position
  // order, so (in-order dispatch) early streams and chunks complete while later
  // runs still compute, and their limiter rescale overlaps that compute
  // (adaptive: every stream is one limiter chunk, measured 1.4 ms faster on C3
  // with 2 rounds; standard 10 s chunks gain nothing and pay warm-up frames)
  int rounds = std::max(1, dev_opt(TOMATIS_DEV_RUN_ROUNDS, (d.alpha_mode == 2 && ns > 1) ? 2 : 1));
  int T = dev_opt(TOMATIS_DEV_RUN_FRAMES, 0);
  if (T <= 0) {
    // generic streams and the edge runs take slots first
    int64_t gen_frames = 0;
    for (int s = 0; s < ns; ++s)
      if (e_lo[s] == e_hi[s]) gen_frames += p->hs[s].n_frames;
    const int64_t work = fast_total + gen_frames;
    if (gate_runs) {  // enough rounds that runs stay within the chained look-back
      const int64_t per_round = std::max<int64_t>(1, slots - n_edge) * (int64_t)(kGateLookbackMax - 64);
      rounds = (int)std::max<int64_t>(rounds, (work + per_round - 1) / per_round);
    }
    const int64_t avail = std::max<int64_t>(1, rounds * slots - n_edge);
    T = (int)std::max<int64_t>(rounds > 1 ? 32 : 48, (work + avail - 1) / avail);
    auto count = [&](int64_t t) {
      int64_t c = n_edge;
      for (int s = 0; s < ns; ++s) {
        const int64_t len = (e_lo[s] == e_hi[s]) ? p->hs[s].n_frames : e_hi[s] - e_lo[s];
        c += (len + t - 1) / t;
      }
      return c;
    };
    while (count(T) > rounds * slots && T < tf_total) T += std::max(1, T / 64);
  }
  T = std::min(T, 1 << 20);  // interior buffer resources stay far below 4 GB
  if (gate_runs) T = std::min(T, kGateLookbackMax);
  std::vector<Run> runs;
  auto add_runs = [&](int s, int64_t a0, int64_t a1, int32_t flags) {
    // equal cuts of [a0, a1) into ceil(len / T) runs
    const int64_t len = a1 - a0;
    if (len <= 0) return;
    const int64_t nr = (len + T - 1) / T;
    for (int64_t j = 0; j < nr; ++j) {
      Run r;
      r.s = s;
      r.ka = a0 + len * j / nr;
      r.kb = a0 + len * (j + 1) / nr;
      r.last = flags | ((r.kb == p->hs[s].n_frames) ? 1 : 0);
      runs.push_back(r);
    }
  };
  for (int s = 0; s < ns; ++s) {
    const int64_t F = p->hs[s].n_frames;
    if (e_lo[s] == e_hi[s]) {
      add_runs(s, 0, F, 0);
      continue;
    }
    if (e_lo[s] > 0) add_runs(s, 0, e_lo[s], 0);
    add_runs(s, e_lo[s], e_hi[s], kRunInterior);
    if (e_hi[s] < F) add_runs(s, e_hi[s], F, 0);
  }
  p->n_runs = (int)runs.size();
  dfree(p->runs);
  p->runs = nullptr;
  if ((rc = dalloc_copy(&p->runs, runs))) return rc;
  p->hruns = runs;
  ++p->runs_gen;  // carries of an earlier look-back no longer match these runs
  return TOMATIS_OK;
}

// Fused-limiter accounting over the plan's runs: flushes expected per chunk
// (host mirror of the kernel's frame-indexed chunk walk) and the largest run
// span of a chunk.
static int limiter_accounting(tomatis_plan_s* p) {
  if (p->generic || p->total_chunks <= 0) return TOMATIS_OK;
  const int HOP = p->d.hop, wpr = p->P / 64;
  const std::vector<Run>& runs = p->hruns;
  int rc;
  std::vector<uint32_t> need(p->total_chunks, 0);
  std::vector<int32_t> first_run(p->total_chunks, -1), last_run(p->total_chunks, -1);
  for (int ri = 0; ri < (int)runs.size(); ++ri) {
    const Run& R = runs[ri];
    const TomatisStream& S = p->hs[R.s];
    const int64_t s_ka = S.first_start + R.ka * HOP;
    int cid = 0;
    if (S.n_chunks > 1 && s_ka >= S.chunk_first)
      cid = (int)std::min<int64_t>(1 + (s_ka - S.chunk_first) / S.chunk_len, S.n_chunks - 1);
    int64_t next_k = INT64_MAX;
    if (S.n_chunks > 1 && cid < S.n_chunks - 1)
      next_k = (S.chunk_first + (int64_t)cid * S.chunk_len - S.first_start) / HOP;
    const int64_t step = S.n_chunks > 1 ? S.chunk_len / HOP : 0;
    auto mark = [&](int c) {
      const int g = S.chunk_base + c;
      need[g] += wpr;
      if (first_run[g] < 0) first_run[g] = ri;
      last_run[g] = ri;
    };
    while (next_k < R.kb) {
      if (next_k >= R.ka) {
        mark(cid);
        ++cid;
        next_k = (cid < S.n_chunks - 1) ? next_k + step : INT64_MAX;
      } else {
        break;  // cannot happen: next chunk starts after the run's first frame
      }
    }
    mark(cid);
  }
  int span = 0;
  for (int g = 0; g < p->total_chunks; ++g)
    if (first_run[g] >= 0) span = std::max(span, last_run[g] - first_run[g] + 1);
  p->fuse_span = span;
  dfree(p->chunk_need);
  p->chunk_need = nullptr;
  if ((rc = dalloc_copy(&p->chunk_need, need))) return rc;
  dfree(p->xs_pieces);  // re-sized for these runs on the next pipelined batch
  p->xs_pieces = nullptr;
  p->xs_max_pieces = 0;
  return TOMATIS_OK;
}

// in-place iterative radix-2 FFT in double (plan set-up: Bluestein filter)
static int plan_build(tomatis_plan_s* p, const float* window) {
  const TomatisPlanDesc& d = p->d;
  const int N = d.n_fft, hop = d.hop, P = p->P;
  int rc;
  const int ns = p->n_streams;
  // --- stream table ---
  if ((rc = dalloc_copy(&p->st, p->hs))) return rc;
  if ((rc = build_runs(p))) return rc;
  // --- levels: any n_fft (numpy pairwise program) ---
  // k_levels holds a block's span in LDS (f64: half as many samples); frames
  // that do not fit, and every n_fft that is not a power of two >= 256, take
  // k_levels_any
  {
    const bool pow2 = (N & (N - 1)) == 0;
    const int cap32 = ((kLevelLds + 256) * 128) / 132 - 8;
    const int cap64 = ((kLevelLds / 2 + 256) * 128) / 132 - 8;
    p->lvl_any = !pow2 || N < 256 || N > cap32;
    if (p->lvl_any || N > cap64) {
      std::vector<int2> lv;
      std::vector<int16_t> prog;
      thost::pw_program(N, lv, prog);
      if ((int)lv.size() > kPwMaxLeaves) return TOMATIS_E_UNSUPPORTED;
      p->n_pw_leaf = (int)lv.size();
      p->n_pw_prog = (int)prog.size();
      if ((rc = dalloc_copy(&p->pw_leaf, lv))) return rc;
      if ((rc = dalloc_copy(&p->pw_prog, prog))) return rc;
    }
  }
  // --- levels blocks ---
  if (!p->lvl_any) {
    const int arr_f32 = kLevelLds + 256;  // matches k_levels<float> LDS
    const int cap = (arr_f32 * 128) / 132 - 8;
    p->lvl_nf = std::max(1, (cap - N) / hop + 1);
    const int nleaf = N >> 7;
    p->lvl_nf = std::min(p->lvl_nf, 1024 / nleaf);
    std::vector<LvlBlock> lb;
    for (int s = 0; s < ns; ++s) {
      const int64_t F = p->hs[s].n_frames;
      for (int64_t a = 0; a < F; a += p->lvl_nf) {
        LvlBlock b;
        b.s = s;
        b.k0 = a;
        b.nf = (int)std::min<int64_t>(p->lvl_nf, F - a);
        lb.push_back(b);
      }
    }
    p->n_lblocks = (int)lb.size();
    if ((rc = dalloc_copy(&p->lblocks, lb))) return rc;
  }
  // --- streaming levels: leaves of 128 samples aligned to first_start ---
  p->leaf_path = (hop % 128 == 0) && N >= 256 && N <= 4096 && (N & (N - 1)) == 0 &&
                 (d.ch == 1 || d.ch == 2) && dev_opt(TOMATIS_DEV_LEVELS_LEGACY, 0) == 0;
  if (p->leaf_path) {
    std::vector<int64_t> gb(ns + 1, 0), lbase(ns + 1, 0);
    for (int s = 0; s < ns; ++s) {
      const int64_t F = p->hs[s].n_frames;
      const int64_t nblk = F > 0 ? ((F - 1) * hop + N) / 128 : 0;
      lbase[s + 1] = lbase[s] + nblk;
      gb[s + 1] = gb[s] + (nblk + 7) / 8;
      p->max_groups = std::max<int64_t>(p->max_groups, (nblk + 7) / 8);
    }
    p->n_groups = gb[ns];
    if ((rc = dalloc_copy(&p->grp_base, gb))) return rc;
    if ((rc = dalloc_copy(&p->leaf_base, lbase))) return rc;
    if (hipMalloc(&p->leaves, (size_t)std::max<int64_t>(1, lbase[ns]) * sizeof(double)))
      return TOMATIS_E_NOMEM;
  }
  // --- gate segments ---
  {
    std::vector<GateSeg> sg;
    std::vector<int32_t> first(ns), count(ns);
    auto segment = [&](int len) {
      sg.clear();
      for (int s = 0; s < ns; ++s) {
        const int64_t F = p->hs[s].n_frames;
        first[s] = (int32_t)sg.size();
        for (int64_t a = 0; a < F; a += len) {
          GateSeg g;
          g.s = s;
          g.k0 = a;
          g.nf = (int)std::min<int64_t>(len, F - a);
          sg.push_back(g);
        }
        count[s] = (int32_t)sg.size() - first[s];
      }
    };
    if (d.alpha_mode == 1) {
      segment(kASeg);
      p->n_asegs = (int)sg.size();
      if ((rc = dalloc_copy(&p->asegs, sg))) return rc;
      if ((rc = dalloc_copy(&p->aseg_first, first))) return rc;
      if ((rc = dalloc_copy(&p->aseg_count, count))) return rc;
    }
    segment(kSeg);
    p->n_segs = (int)sg.size();
    if ((rc = dalloc_copy(&p->segs, sg))) return rc;
    p->gate_excl = dev_opt(TOMATIS_DEV_GATE_TF, 0) == 0;
    for (int s = 0; s < ns; ++s) p->gate_excl = p->gate_excl && gate_exclusive(p->hs[s]);
    if (p->n_segs > 0) {
      if (hipMalloc(&p->gsum, (size_t)p->n_segs * 5 * sizeof(int))) return TOMATIS_E_NOMEM;
      if (hipMalloc(&p->gcarry, (size_t)p->n_segs * 3 * sizeof(int))) return TOMATIS_E_NOMEM;
    }
    if ((rc = dalloc_copy(&p->seg_first, first))) return rc;
    if ((rc = dalloc_copy(&p->seg_count, count))) return rc;
    const int nstate = d.up_delay_frames + 2;
    if (p->n_segs > 0) {
      if (hipMalloc(reinterpret_cast<void**>(&p->tf), (size_t)p->n_segs * nstate * sizeof(uint16_t)))
        return TOMATIS_E_NOMEM;
      if (hipMalloc(reinterpret_cast<void**>(&p->seg_start), (size_t)p->n_segs * sizeof(uint16_t)))
        return TOMATIS_E_NOMEM;
    }
  }
  // --- tables ---
  {
    std::vector<float> w(window, window + N), w2(N);
    for (int i = 0; i < N; ++i) w2[i] = w[i] * w[i];
    std::vector<float> winv(hop);
    for (int m = 0; m < hop; ++m) {
      // frames covering an interior position with hop-offset m, ascending frame order
      const int Rm = (N - m + hop - 1) / hop;
      float acc = 0.f;
      for (int j = Rm - 1; j >= 0; --j) acc = acc + w2[m + j * hop];
      const float den = (d.norm_mode == TOMATIS_NORM_MAX) ? std::max(acc, 1e-8f) : (acc + 1e-12f);
      winv[m] = 1.0f / den;
    }
    p->rmax = (N + hop - 1) / hop;
    if (!p->lds) {  // register kernels only (NR = 16 or 32)
      const int NRr = p->NR;
      // scaled-DIF output scales of the register FFT (tm_common.h): the step-2
      // table absorbs the forward NR-point DFT's, the synthesis window the
      // inverse's (whose inputs carry 1 / the forward's)
      const double* sigF = NRr == 32 ? splan<32, 0>().sig : splan<16, 0>().sig;
      const double* sigI = NRr == 32 ? splan<32, 2>().sig : splan<16, 2>().sig;
      // n_fft 4096 single-exchange FFT (tm_fft.h fftx128_*): wave 1 (lanes >= 64)
      // holds k2 rotated by 16 in register r: its step-2 row r twiddles
      // k2 = (r + 16) mod 32, and both its windows carry (-1)^n2
      const bool fx = p->fx, rot = fx && P == 128;
      std::vector<cf> twN((size_t)NRr * P), twP(P);
      for (int r = 0; r < NRr; ++r)
        for (int n1 = 0; n1 < P; ++n1) {
          const int k2 = (rot && n1 >= 64) ? (r + 16) % 32 : r;
          const double ang = -2.0 * M_PI * (double)((int64_t)n1 * k2 % N) / (double)N;
          twN[((size_t)(r >> 1) * P + n1) * 2 + (r & 1)] = {(float)(cos(ang) * sigF[r]),
                                                           (float)(sin(ang) * sigF[r])};
        }
      std::vector<float> winS(N);
      // single-exchange FFTs (fftx_inv / fftx128_inv): lane m's first-DFT output scale too
      for (int t = 0; t < N; ++t) {
        const double sgn = (rot && (t % P) >= 64 && ((t / P) & 1)) ? -1.0 : 1.0;
        winS[t] = (float)(sgn * (double)w[t] * sigI[t / P] *
                          (fx ? splan<32, 1>().sig[(t % P) & 31] : 1.0));
        if (rot && sgn < 0) w[t] = -w[t];  // analysis window (w2 / winv are built above)
      }
      for (int m = 0; m < P; ++m) {
        const double ang = -2.0 * M_PI * (double)m / (double)P;
        twP[m] = {(float)cos(ang), (float)sin(ang)};
      }
      if ((rc = dalloc_copy(&p->winS, winS))) return rc;
      if ((rc = dalloc_copy(&p->twN, twN))) return rc;
      if ((rc = dalloc_copy(&p->twP, twP))) return rc;
    }
    if ((rc = dalloc_copy(&p->win, w))) return rc;
    if ((rc = dalloc_copy(&p->win2, w2))) return rc;
    if ((rc = dalloc_copy(&p->winv, winv))) return rc;
    if (p->lds) {
      const int M = p->lds_M;
      std::vector<float2> tl(M);
      for (int t = 0; t < M; ++t) {
        const double ang = -2.0 * M_PI * (double)t / (double)M;
        tl[t] = make_float2((float)cos(ang), (float)sin(ang));
      }
      if ((rc = dalloc_copy(&p->twL, tl))) return rc;
      if (p->blue) {
        std::vector<float2> bf, hf;
        thost::bluestein_tables(N, M, bf, hf);
        if ((rc = dalloc_copy(&p->blue_b, bf))) return rc;
        if ((rc = dalloc_copy(&p->blue_h, hf))) return rc;
      }
      if (M > kLdsMaxM && p->total_frames > 0) {
        const int64_t items = p->total_frames * ((d.ch + 1) / 2);
        // one 1024-thread block per CU keeps the chip busy; each owns two
        // M-element buffers (2 MiB at M = 131072)
        int dev = 0, ncu = 256;
        if (hipGetDevice(&dev) == hipSuccess)
          (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
        p->glb_blocks = (int)std::min<int64_t>(items, std::max(1, ncu));
        if (hipMalloc(reinterpret_cast<void**>(&p->glb_work),
                      (size_t)p->glb_blocks * 2 * M * sizeof(float2)))
          return TOMATIS_E_NOMEM;
      }
    }
  }
  // --- limiter chunk descriptors, output prefix ---
  {
    std::vector<ChunkDesc> cd;
    std::vector<int64_t> pb(ns);
    int64_t tot = 0, mx = 0;
    for (int s = 0; s < ns; ++s) {
      const TomatisStream& S = p->hs[s];
      pb[s] = tot;
      tot += S.out_len;
      const int64_t ob = S.out_begin, oe = S.out_begin + S.out_len;
      for (int c = 0; c < S.n_chunks; ++c) {
        int64_t b0 = (c == 0) ? INT64_MIN / 4 : S.chunk_first + (int64_t)(c - 1) * S.chunk_len;
        int64_t b1 = (c == S.n_chunks - 1) ? INT64_MAX / 4 : S.chunk_first + (int64_t)c * S.chunk_len;
        b0 = std::max(b0, ob);
        b1 = std::min(b1, oe);
        if (b1 <= b0) continue;
        ChunkDesc C;
        C.s = s;
        C.c = c;
        C.p0 = b0 - ob;
        C.p1 = b1 - ob;
        mx = std::max(mx, b1 - b0);
        cd.push_back(C);
      }
    }
    p->n_chunkdesc = (int)cd.size();
    p->max_chunk = mx;
    p->total_out = tot;
    if ((rc = dalloc_copy(&p->chunks, cd))) return rc;
    if ((rc = dalloc_copy(&p->pos_base, pb))) return rc;
    // fused limiter: chunk output ranges (the per-run accounting: build_runs)
    if (!p->generic && p->total_chunks > 0) {
      std::vector<int64_t> rng(2 * (size_t)p->total_chunks, 0);
      for (const ChunkDesc& C : cd) {
        rng[2 * (p->hs[C.s].chunk_base + C.c)] = C.p0;
        rng[2 * (p->hs[C.s].chunk_base + C.c) + 1] = C.p1;
      }
      if ((rc = dalloc_copy(&p->chunk_rng, rng))) return rc;
      if (hipMalloc(reinterpret_cast<void**>(&p->chunk_done), (size_t)p->total_chunks * 4))
        return TOMATIS_E_NOMEM;
    }
    if ((rc = limiter_accounting(p))) return rc;
    if (hipMalloc(reinterpret_cast<void**>(&p->err), 4)) return TOMATIS_E_NOMEM;
    if (hipMemset(p->err, 0, 4)) return TOMATIS_E_HIP;
  }
  // --- generic-hop scratch ---
  if (p->generic && p->total_frames > 0) {
    // register generic path: cf per position (L, R); any-size path: ch floats
    const size_t per = p->lds ? (size_t)std::max(2, (int)d.ch) * sizeof(float) : sizeof(cf);
    if (hipMalloc(reinterpret_cast<void**>(&p->scratch), (size_t)p->total_frames * N * per))
      return TOMATIS_E_NOMEM;
  }
  // --- min-hold workspace (used when a stream's tables exceed the kernel's LDS) ---
  if (d.min_hold_frames >= 0) {
    const int nsm = 2 * (d.min_hold_frames + 1);
    std::vector<int64_t> off(ns + 1, 0), soff(ns + 1, 0);
    for (int s = 0; s < ns; ++s) {
      const int64_t F = p->hs[s].n_frames;
      const int64_t nseg = (F + mh_seg_len(F, nsm) - 1) / mh_seg_len(F, nsm);
      off[s + 1] = off[s] + (nseg * nsm > kMhLdsTf ? nseg * nsm : 0);
      soff[s + 1] = soff[s] + (((F + 15) >> 4) > kMhLdsSym ? (F + 15) >> 4 : 0);
    }
    if ((rc = dalloc_copy(&p->mh_off, off))) return rc;
    if ((rc = dalloc_copy(&p->mh_soff, soff))) return rc;
    if (off[ns] > 0) {
      if (hipMalloc(reinterpret_cast<void**>(&p->mh_tf), off[ns] * sizeof(uint16_t))) return TOMATIS_E_NOMEM;
      if (hipMalloc(reinterpret_cast<void**>(&p->mh_cnt), off[ns] * sizeof(int32_t))) return TOMATIS_E_NOMEM;
    }
    if (soff[ns] > 0 &&
        hipMalloc(reinterpret_cast<void**>(&p->mh_sym), soff[ns] * sizeof(uint32_t)))
      return TOMATIS_E_NOMEM;
    if (ns > 0 && off[ns] == 0 && soff[ns] == 0) {  // speculative path: tables fit
      if (hipMalloc(reinterpret_cast<void**>(&p->mh_bs), ns * sizeof(MhBisect))) return TOMATIS_E_NOMEM;
      if (hipMalloc(reinterpret_cast<void**>(&p->mh_pc), ns * kMhProbes * sizeof(int32_t)))
        return TOMATIS_E_NOMEM;
      std::vector<int64_t> goff(ns + 1, 0);
      int max_nseg = 1;
      for (int s = 0; s < ns; ++s) {
        const int64_t F = p->hs[s].n_frames;
        const int64_t nseg = F > 0 ? (F + mh_seg_len(F, nsm) - 1) / mh_seg_len(F, nsm) : 0;
        goff[s + 1] = goff[s] + kMhSlots * nseg * nsm;
        max_nseg = std::max(max_nseg, (int)nseg);
      }
      // workgroups per probe: a few segments each (one pass of the block's
      // threads over their (segment, start) pairs), at most 8
      p->mh_parts = std::max(1, std::min(8, (max_nseg * nsm + 767) / 768));
      if (const int e = tshared::dev_opt(TOMATIS_DEV_MH_PARTS, 0)) p->mh_parts = std::max(1, std::min(32, e));
      if ((rc = dalloc_copy(&p->mh_goff, goff))) return rc;
      if (goff[ns] > 0) {
        if (hipMalloc(reinterpret_cast<void**>(&p->mh_gtf), goff[ns] * sizeof(uint16_t))) return TOMATIS_E_NOMEM;
        if (hipMalloc(reinterpret_cast<void**>(&p->mh_gcnt), goff[ns] * sizeof(int32_t))) return TOMATIS_E_NOMEM;
      }
      if (hipMalloc(reinterpret_cast<void**>(&p->mh_arr), ns * kMhSlots * sizeof(int32_t))) return TOMATIS_E_NOMEM;
      if (hipMemset(p->mh_arr, 0, ns * kMhSlots * sizeof(int32_t))) return TOMATIS_E_HIP;
    }
  }
  return TOMATIS_OK;
}

int tomatis_plan_create(tomatis_plan_t* out, const TomatisPlanDesc* desc, const float* window,
                        TomatisStream* streams, int32_t n_streams) {
  if (!out || !desc || !window || (!streams && n_streams > 0) || n_streams < 0) return TOMATIS_E_ARG;
  *out = nullptr;
  const TomatisPlanDesc d = *desc;
  if (d.n_fft < 2 || d.n_fft > kMaxNfft) return TOMATIS_E_UNSUPPORTED;
  if (d.ch < 1 || d.ch > kMaxCh) return TOMATIS_E_UNSUPPORTED;
  if (d.hop < 1 || d.hop > d.n_fft) return TOMATIS_E_ARG;
  if (d.up_delay_frames < 0 || d.up_delay_frames + 2 > kMaxGateStates) return TOMATIS_E_UNSUPPORTED;
  if (d.min_hold_frames < 0 || 2 * (d.min_hold_frames + 1) > 65535) return TOMATIS_E_UNSUPPORTED;
  if (d.norm_mode != TOMATIS_NORM_EPS && d.norm_mode != TOMATIS_NORM_MAX) return TOMATIS_E_ARG;
  auto* p = new (std::nothrow) tomatis_plan_s();
  if (!p) return TOMATIS_E_NOMEM;
  p->d = d;
  p->n_streams = n_streams;
  const int N = d.n_fft, hop = d.hop;
  // (lanes P, registers NR) per transform: 2048 = 128 x 16, 4096 = 128 x 32
  // n_fft 2048: one wave per frame (P = 64, 32 registers, wave-local exchanges)
  // unless TOMATIS_P64=0; otherwise two waves per frame (P = 128)
  // register kernels: n_fft 2048 / 4096 with <= 2 channels (L + iR); every
  // other n_fft or more channels: the any-size path (Stockham FFT of length M,
  // Bluestein when n_fft is not a power of two)
  p->lds = !(N == 2048 || N == 4096) || d.ch > 2 || dev_opt(TOMATIS_DEV_FORCE_LDS, 0) != 0;
  if (p->lds) {
    p->blue = (N & (N - 1)) != 0;
    int M = 1;
    while (M < (p->blue ? 2 * N - 1 : N)) M <<= 1;
    p->lds_M = M;
  }
  p->P = p->lds ? 64 : ((N == 2048 && dev_opt(TOMATIS_DEV_P64, 1)) ? 64 : 128);
  p->NR = N / p->P;
  p->SH = (!p->lds && hop % p->P == 0) ? hop / p->P : 0;
  p->generic = p->lds || (p->NR == 16 ? !(p->SH == 2 || p->SH == 4 || p->SH == 8)
                                      : !(p->SH == 4 || p->SH == 8 || p->SH == 16));
  for (int i = 0; i < n_streams && !p->generic; ++i) {
    const TomatisStream& s = streams[i];
    if (s.n_chunks > 1 && (((s.chunk_first - s.first_start) % hop) != 0 || (s.chunk_len % hop) != 0))
      p->generic = true;  // chunk boundaries not on emit blocks: per-sample gather path
  }
  // n_fft 2048 fused kernels: the single-exchange FFT (its bin layout and scales)
  p->fx = kFftX && !p->generic && (p->P == 64 || p->P == 128) && p->NR == 32;
  int64_t fb = 0;
  int32_t cb = 0;
  for (int i = 0; i < n_streams; ++i) {
    TomatisStream& s = streams[i];
    bool bad = s.n < 0 || s.n_frames < 0 || s.out_len < 0 || s.n_chunks < 1 ||
               (s.n_chunks > 1 && s.chunk_len <= 0);
    if (!bad && s.n_frames > 0 && s.out_begin + s.out_len > s.first_start + (s.n_frames - 1) * hop + N)
      bad = true;  // output beyond the last frame end is never produced
    if (!bad && s.n_frames == 0 && s.out_len > 0) bad = true;
    if (bad) {
      delete p;
      return TOMATIS_E_ARG;
    }
    s.frame_base = fb;
    s.chunk_base = cb;
    fb += s.n_frames;
    cb += s.n_chunks;
  }
  p->total_frames = fb;
  p->total_chunks = cb;
  p->hs.assign(streams, streams + n_streams);
  const int rc = plan_build(p, window);
  if (rc != TOMATIS_OK) {
    tomatis_plan_destroy(p);
    return rc;
  }
  *out = p;
  return TOMATIS_OK;
}

int tomatis_plan_update_streams(tomatis_plan_t p, const TomatisStream* streams, void* hs) {
  if (!p || !streams) return TOMATIS_E_ARG;
  for (int i = 0; i < p->n_streams; ++i) {  // geometry is fixed at plan creation
    const TomatisStream &a = streams[i], &b = p->hs[i];
    if (a.in_off != b.in_off || a.out_off != b.out_off || a.n != b.n ||
        a.first_start != b.first_start || a.n_frames != b.n_frames ||
        a.out_begin != b.out_begin || a.out_len != b.out_len || a.chunk_first != b.chunk_first ||
        a.chunk_len != b.chunk_len || a.n_chunks != b.n_chunks)
      return TOMATIS_E_ARG;
  }
  bool excl = dev_opt(TOMATIS_DEV_GATE_TF, 0) == 0;
  for (int i = 0; i < p->n_streams; ++i) {
    TomatisStream s = streams[i];
    s.frame_base = p->hs[i].frame_base;
    s.chunk_base = p->hs[i].chunk_base;
    p->hs[i] = s;
    excl = excl && gate_exclusive(s);
  }
  p->gate_excl = excl;
  if (p->n_streams == 0) return TOMATIS_OK;
  return hipfail(hipMemcpyAsync(p->st, p->hs.data(), p->hs.size() * sizeof(TomatisStream),
                                hipMemcpyHostToDevice, (hipStream_t)hs));
}

int tomatis_levels(tomatis_plan_t p, const float* x, void* r_out, int32_t prec, void* hs) {
  if (!p || !x || !r_out) return TOMATIS_E_ARG;
  if (p->total_frames == 0) return TOMATIS_OK;
  hipStream_t s = (hipStream_t)hs;
  const bool any = p->lvl_any || (prec == TOMATIS_F64 && p->n_pw_prog > 0);
  if (any && (prec == TOMATIS_F32 || prec == TOMATIS_F64)) {
    const unsigned g = (unsigned)std::min<int64_t>(p->total_frames, 1 << 16);
    if (g == 0) return TOMATIS_OK;
    if (prec == TOMATIS_F32)
      hipLaunchKernelGGL(k_levels_any<float>, dim3(g), dim3(256), 0, s, x, p->st, p->n_streams,
                         p->d.n_fft, p->d.hop, p->d.ch, p->pw_leaf, p->n_pw_leaf, p->pw_prog,
                         p->n_pw_prog, p->total_frames, (float*)r_out);
    else
      hipLaunchKernelGGL(k_levels_any<double>, dim3(g), dim3(256), 0, s, x, p->st, p->n_streams,
                         p->d.n_fft, p->d.hop, p->d.ch, p->pw_leaf, p->n_pw_leaf, p->pw_prog,
                         p->n_pw_prog, p->total_frames, (double*)r_out);
    return launch_check();
  }
  if (p->leaf_path && (prec == TOMATIS_F32 || prec == TOMATIS_F64)) {
    const dim3 gblk((unsigned)((p->max_groups + 3) / 4), (unsigned)p->n_streams);
    const unsigned fblk = (unsigned)((p->total_frames + 255) / 256);
    const int ch = p->d.ch, N = p->d.n_fft, hop = p->d.hop, ns = p->n_streams;
    if (prec == TOMATIS_F32) {
      float* lv = (float*)p->leaves;
      if (ch == 2)
        hipLaunchKernelGGL((k_leaves<float, 2>), dim3(gblk), dim3(256), 0, s, x, p->st, ns,
                           p->grp_base, p->leaf_base, p->n_groups, lv);
      else
        hipLaunchKernelGGL((k_leaves<float, 1>), dim3(gblk), dim3(256), 0, s, x, p->st, ns,
                           p->grp_base, p->leaf_base, p->n_groups, lv);
      hipLaunchKernelGGL(k_frame_r<float>, dim3(fblk), dim3(256), 0, s, p->st, ns, p->leaf_base,
                         lv, N, hop, p->total_frames, (float*)r_out);
    } else {
      double* lv = (double*)p->leaves;
      if (ch == 2)
        hipLaunchKernelGGL((k_leaves<double, 2>), dim3(gblk), dim3(256), 0, s, x, p->st, ns,
                           p->grp_base, p->leaf_base, p->n_groups, lv);
      else
        hipLaunchKernelGGL((k_leaves<double, 1>), dim3(gblk), dim3(256), 0, s, x, p->st, ns,
                           p->grp_base, p->leaf_base, p->n_groups, lv);
      hipLaunchKernelGGL(k_frame_r<double>, dim3(fblk), dim3(256), 0, s, p->st, ns, p->leaf_base,
                         lv, N, hop, p->total_frames, (double*)r_out);
    }
    return launch_check();
  }
  if (prec == TOMATIS_F32) {
    hipLaunchKernelGGL((k_levels<float, true>), dim3(p->n_lblocks), dim3(256), 0, s, x, p->st,
                       p->lblocks, p->d.n_fft, p->d.hop, p->d.ch, (float*)r_out);
  } else if (prec == TOMATIS_F64) {
    // f64 blocks hold half the frames: launch twice the blocks over half-size items
    const int N = p->d.n_fft, hop = p->d.hop;
    const int cap = ((kLevelLds / 2 + 256) * 128) / 132 - 8;
    const int nf64 = std::max(1, (cap - N) / hop + 1);
    if (nf64 < p->lvl_nf) {
      // build a finer block list on the fly (small host work, cached per call)
      std::vector<LvlBlock> lb;
      for (int st = 0; st < p->n_streams; ++st) {
        const int64_t F = p->hs[st].n_frames;
        for (int64_t a = 0; a < F; a += nf64) {
          LvlBlock b;
          b.s = st;
          b.k0 = a;
          b.nf = (int)std::min<int64_t>(nf64, F - a);
          lb.push_back(b);
        }
      }
      LvlBlock* dlb = nullptr;
      int rc = dalloc_copy(&dlb, lb);
      if (rc) return rc;
      hipLaunchKernelGGL((k_levels<double, true>), dim3((unsigned)lb.size()), dim3(256), 0, s, x,
                         p->st, dlb, N, hop, p->d.ch, (double*)r_out);
      rc = launch_check();
      (void)hipStreamSynchronize(s);
      dfree(dlb);
      return rc;
    }
    hipLaunchKernelGGL((k_levels<double, true>), dim3(p->n_lblocks), dim3(256), 0, s, x, p->st,
                       p->lblocks, p->d.n_fft, p->d.hop, p->d.ch, (double*)r_out);
  } else {
    return TOMATIS_E_ARG;
  }
  return launch_check();
}

int tomatis_gate_std(tomatis_plan_t p, const float* r, uint8_t* states, uint16_t* rows,
                     double* alpha_out, void* hs) {
  if (!p || !r || !states || !rows) return TOMATIS_E_ARG;
  if (p->n_segs == 0) return TOMATIS_OK;
  hipStream_t s = (hipStream_t)hs;
  const int D = p->d.up_delay_frames;
  const bool xf = p->d.alpha_mode == 1;
  if (p->gate_excl) {
    hipLaunchKernelGGL(k_gate_sum, dim3(p->n_segs), dim3(256), 0, s, r, p->st, p->segs, D,
                       (GSum*)p->gsum);
    hipLaunchKernelGGL(k_gate_carry, dim3(p->n_streams), dim3(256), 0, s, p->seg_first,
                       p->seg_count, D, (const GSum*)p->gsum, (GCarry*)p->gcarry,
                       (const GCarry*)nullptr);
    hipLaunchKernelGGL(k_gate_states, dim3(p->n_segs), dim3(256), 0, s, r, p->st, p->segs, D,
                       (const GCarry*)p->gcarry, states, xf ? nullptr : rows);
  } else {
    hipLaunchKernelGGL(k_gate_tf, dim3((p->n_segs + 3) / 4), dim3(256), 0, s, r, p->st, p->segs,
                       p->n_segs, D, p->tf);
    hipLaunchKernelGGL(k_gate_chain, dim3((p->n_streams + 63) / 64), dim3(64), 0, s, p->st,
                       p->n_streams, p->seg_first, p->seg_count, D + 2, p->tf, p->seg_start, 0);
    hipLaunchKernelGGL(k_gate_resolve, dim3((p->n_segs + 3) / 4), dim3(256), 0, s, r, p->st,
                       p->segs, p->n_segs, D, p->seg_start, states, xf ? nullptr : rows);
  }
  if (xf) {
    const int nxf = p->d.xfade_frames;
    if (dev_opt(TOMATIS_DEV_ALPHA_SEQ, 0) != 0) {
      hipLaunchKernelGGL(k_alpha_xfade, dim3((p->n_streams + 63) / 64), dim3(64), 0, s, p->st,
                         p->n_streams, states, nxf, rows, alpha_out);
      return launch_check();
    }
    if (p->n_asegs == 0) return launch_check();
    if (!p->aq) {
      const size_t na = (size_t)p->n_asegs;
      if (hipMalloc(reinterpret_cast<void**>(&p->aq), na * sizeof(int32_t)) ||
          hipMalloc(reinterpret_cast<void**>(&p->afin), na * sizeof(double)) ||
          hipMalloc(reinterpret_cast<void**>(&p->acin), na * sizeof(double)))
        return TOMATIS_E_NOMEM;
    }
    const unsigned gs = (unsigned)p->n_asegs;  // one wave per alpha segment
    hipLaunchKernelGGL(k_alpha_sync, dim3(gs), dim3(64), 0, s, p->st, p->asegs, p->n_asegs, states,
                       nxf, rows, alpha_out, p->aq, p->afin);
    hipLaunchKernelGGL(k_alpha_chain, dim3(p->n_streams), dim3(64), 0, s, p->st,
                       p->n_streams, p->asegs, p->aseg_first, p->aseg_count, states, nxf, p->aq,
                       p->afin, p->acin);
    hipLaunchKernelGGL(k_alpha_prefix, dim3(gs), dim3(64), 0, s, p->st, p->asegs, p->n_asegs,
                       states, nxf, p->aq, p->acin, rows, alpha_out);
  }
  return launch_check();
}

int32_t tomatis_plan_gate_segments(tomatis_plan_t p) { return p ? p->n_segs : -1; }

int tomatis_gate_segment_sums(tomatis_plan_t p, const float* r, int32_t* sums_host, void* hs) {
  if (!p || !r || !sums_host) return TOMATIS_E_ARG;
  if (!p->gate_excl) return TOMATIS_E_UNSUPPORTED;
  if (p->n_segs == 0) return TOMATIS_OK;
  hipStream_t s = (hipStream_t)hs;
  hipLaunchKernelGGL(k_gate_sum, dim3(p->n_segs), dim3(256), 0, s, r, p->st, p->segs,
                     p->d.up_delay_frames, (GSum*)p->gsum);
  int rc = launch_check();
  if (rc) return rc;
  static_assert(sizeof(GSum) == 5 * sizeof(int32_t), "GSum layout");
  if (hipMemcpyAsync(sums_host, p->gsum, (size_t)p->n_segs * sizeof(GSum), hipMemcpyDeviceToHost, s))
    return TOMATIS_E_HIP;
  return hipfail(hipStreamSynchronize(s));
}

int tomatis_gate_std_carry(tomatis_plan_t p, const float* r, const int32_t* carry_host,
                           uint8_t* states, uint16_t* rows, void* hs) {
  if (!p || !r || !carry_host || !states || !rows) return TOMATIS_E_ARG;
  if (!p->gate_excl || p->d.alpha_mode != 0) return TOMATIS_E_UNSUPPORTED;
  if (p->n_segs == 0) return TOMATIS_OK;
  hipStream_t s = (hipStream_t)hs;
  static_assert(sizeof(GCarry) == 3 * sizeof(int32_t), "GCarry layout");
  if (!p->gcarry_in && hipMalloc(&p->gcarry_in, (size_t)std::max(1, p->n_streams) * sizeof(GCarry)))
    return TOMATIS_E_NOMEM;
  if (hipMemcpyAsync(p->gcarry_in, carry_host, (size_t)p->n_streams * sizeof(GCarry),
                     hipMemcpyHostToDevice, s))
    return TOMATIS_E_HIP;
  const int D = p->d.up_delay_frames;
  hipLaunchKernelGGL(k_gate_sum, dim3(p->n_segs), dim3(256), 0, s, r, p->st, p->segs, D,
                     (GSum*)p->gsum);
  hipLaunchKernelGGL(k_gate_carry, dim3(p->n_streams), dim3(256), 0, s, p->seg_first,
                     p->seg_count, D, (const GSum*)p->gsum, (GCarry*)p->gcarry,
                     (const GCarry*)p->gcarry_in);
  hipLaunchKernelGGL(k_gate_states, dim3(p->n_segs), dim3(256), 0, s, r, p->st, p->segs, D,
                     (const GCarry*)p->gcarry, states, rows);
  int rc = launch_check();
  if (rc) return rc;
  return hipfail(hipStreamSynchronize(s));  // carry_host may be reused by the caller
}

int tomatis_ts_summary(tomatis_plan_t p, const float* r, int32_t n_seg, int32_t shift,
                       int32_t* sum_out, void* hs) {
  if (!p || !r || !sum_out || n_seg < 0) return TOMATIS_E_ARG;
  if (!p->gate_excl || p->n_streams != 1) return TOMATIS_E_UNSUPPORTED;
  hipStream_t s = (hipStream_t)hs;
  const int D = p->d.up_delay_frames;
  if (p->n_segs > 0)
    hipLaunchKernelGGL(k_gate_sum, dim3(p->n_segs), dim3(256), 0, s, r, p->st, p->segs, D,
                       (GSum*)p->gsum);
  hipLaunchKernelGGL(k_ts_fold, dim3(1), dim3(64), 0, s, (const GSum*)p->gsum,
                     std::min<int>(n_seg, p->n_segs), D, shift, sum_out);
  return launch_check();
}

int tomatis_ts_gate(tomatis_plan_t p, const float* r, const int32_t* sums_all, int32_t rank,
                    int32_t shift, uint8_t* states, uint16_t* rows, void* hs) {
  if (!p || !r || !sums_all || rank < 0 || !states || !rows) return TOMATIS_E_ARG;
  if (!p->gate_excl || p->d.alpha_mode != 0 || p->n_streams != 1) return TOMATIS_E_UNSUPPORTED;
  if (p->n_segs == 0) return TOMATIS_OK;
  hipStream_t s = (hipStream_t)hs;
  if (!p->gcarry_in && hipMalloc(&p->gcarry_in, sizeof(GCarry))) return TOMATIS_E_NOMEM;
  const int D = p->d.up_delay_frames;
  hipLaunchKernelGGL(k_ts_carry, dim3(1), dim3(64), 0, s, sums_all, rank, D, shift,
                     (GCarry*)p->gcarry_in);
  hipLaunchKernelGGL(k_gate_sum, dim3(p->n_segs), dim3(256), 0, s, r, p->st, p->segs, D,
                     (GSum*)p->gsum);
  hipLaunchKernelGGL(k_gate_carry, dim3(p->n_streams), dim3(256), 0, s, p->seg_first,
                     p->seg_count, D, (const GSum*)p->gsum, (GCarry*)p->gcarry,
                     (const GCarry*)p->gcarry_in);
  hipLaunchKernelGGL(k_gate_states, dim3(p->n_segs), dim3(256), 0, s, r, p->st, p->segs, D,
                     (const GCarry*)p->gcarry, states, rows);
  return launch_check();
}

int tomatis_level_stats(tomatis_plan_t p, const double* levels, double* tlh, void* hs) {
  if (!p || !levels || !tlh) return TOMATIS_E_ARG;
  if (p->n_streams == 0) return TOMATIS_OK;
  hipLaunchKernelGGL(k_level_stats, dim3(p->n_streams), dim3(1024), 0, (hipStream_t)hs, levels,
                     p->st, tlh);
  return launch_check();
}

int tomatis_minhold_bisect(tomatis_plan_t p, const double* levels, const double* tlh,
                           double target_c2, double hyst_db, double* t_out, uint8_t* states,
                           uint16_t* rows, double* alpha_out, void* hs) {
  if (!p || !levels || !tlh || !states) return TOMATIS_E_ARG;
  if (p->n_streams == 0) return TOMATIS_OK;
  hipStream_t s = (hipStream_t)hs;
  // speculative rounds when every stream's tables fit the probe kernel's LDS
  // (no HBM workspace); TOMATIS_MH_SERIAL keeps the one-CU-per-stream loop
  const bool spec = !p->mh_serial && p->mh_bs && p->mh_gtf;
  if (spec) {
    const int ns = p->n_streams, P = p->mh_parts, mh = p->d.min_hold_frames;
    hipLaunchKernelGGL(k_mh_init, dim3((ns + 255) / 256), dim3(256), 0, s, p->st, ns, tlh,
                       p->mh_bs);
    for (int r = 0; r < 10; ++r)  // 30 bisection steps, three per launch
      hipLaunchKernelGGL(k_mh_probe, dim3(ns, kMhProbes, P), dim3(1024), 0, s, levels, p->st,
                         target_c2, hyst_db, mh, p->mh_bs, p->mh_pc, p->mh_gtf, p->mh_gcnt,
                         p->mh_goff, p->mh_arr, 0);
    hipLaunchKernelGGL(k_mh_probe, dim3(ns, 1, P), dim3(1024), 0, s, levels, p->st, target_c2,
                       hyst_db, mh, p->mh_bs, p->mh_pc, p->mh_gtf, p->mh_gcnt, p->mh_goff,
                       p->mh_arr, 1);
  }
  hipLaunchKernelGGL(k_minhold, dim3(p->n_streams), dim3(1024), 0, s, levels, p->st, tlh,
                     target_c2, hyst_db, p->d.min_hold_frames, p->d.xfade_frames, 1, p->mh_tf,
                     p->mh_cnt, p->mh_off, p->mh_sym, p->mh_soff, t_out, states, rows, alpha_out,
                     spec ? p->mh_bs : nullptr, p->mh_gtf, p->mh_gcnt, p->mh_goff);
  return launch_check();
}

// in-kernel levels + gate outputs (tomatis_stft_ola_gated)
struct GateOut {
  float* r;
  uint8_t* states;
  bool lookback_done;  // tomatis_gate_lookback ran for this input on this stream
};

// per-run carry-in state id of the fused gate (k_gate_carry)
static int gate_lookback(tomatis_plan_s* p, const float* x, hipStream_t s) {
  const int nst = p->d.up_delay_frames + 2;
  const bool chain = nst <= kGateChainStates;
  const bool xa = p->d.alpha_mode == 1;
  if (p->n_runs > p->gate_cap) {
    dfree(p->gate_carry);
    dfree(p->gate_tf);
    dfree(p->gate_acarry);
    p->gate_carry = nullptr;
    p->gate_tf = nullptr;
    p->gate_acarry = nullptr;
    p->gate_cap = 0;
    if (hipMalloc(reinterpret_cast<void**>(&p->gate_carry), (size_t)p->n_runs * sizeof(int32_t)))
      return TOMATIS_E_NOMEM;
    if (chain && hipMalloc(reinterpret_cast<void**>(&p->gate_tf),
                           (size_t)p->n_runs * nst * sizeof(uint16_t)))
      return TOMATIS_E_NOMEM;
    if (xa && hipMalloc(reinterpret_cast<void**>(&p->gate_acarry), (size_t)p->n_runs * sizeof(double)))
      return TOMATIS_E_NOMEM;
    p->gate_cap = p->n_runs;
  }
  p->gl_x = x;
  p->gl_gen = p->runs_gen;
  if (p->n_runs == 0) return TOMATIS_OK;
  MainArgs A{};
  A.x = x;
  A.st = p->st;
  A.runs = p->runs;
  A.n_runs = p->n_runs;
  A.rmax = p->rmax;
  A.hop = p->d.hop;
  A.ch = p->d.ch;
  A.gate_D = p->d.up_delay_frames;
  A.gate_xf = xa ? p->d.xfade_frames : -1;
  A.gate_astep = (xa && p->d.xfade_frames > 0) ? 1.0 / p->d.xfade_frames : 1.0;
  launch_gate_carry(A, p->P, p->SH, p->d.ch, p->gate_carry, (chain && !xa) ? p->gate_tf : nullptr,
                    p->gate_acarry, s);
  return launch_check();
}

// the previous batch of a pipelined call (tomatis_stft_ola_gated_pipelined)
struct PrevBatch {
  float* y;               // its unscaled output (nullptr: first batch)
  const uint32_t* peaks;  // its final chunk peaks
  const tomatis_plan_s* plan;  // its plan (this plan, or one of the same shape)
};

// piece lists of the pipelined partner rescale: every run's own emitted blocks
static int xs_pieces_alloc(tomatis_plan_s* p) {
  if (p->xs_pieces) return TOMATIS_OK;
  int mp = 1;
  for (const Run& R : p->hruns)
    mp = std::max<int>(mp, (int)(R.kb - std::max<int64_t>(0, R.ka - (p->rmax - 1))));
  if (hipMalloc(reinterpret_cast<void**>(&p->xs_pieces),
                (size_t)std::max(1, p->n_runs) * 2 * (mp + 1) * sizeof(uint32_t)))
    return TOMATIS_E_NOMEM;
  p->xs_max_pieces = mp;
  return TOMATIS_OK;
}

static int stft_ola_impl(tomatis_plan_t p, const float* x, const float* gains, int32_t n_rows,
                         const uint16_t* rows, float* y, uint32_t* peaks, float limit,
                         void* hs, const GateOut* gate = nullptr,
                         const PrevBatch* prev = nullptr) {
  if (!p || !x || !gains || (!rows && !gate) || !y || !peaks || n_rows < 1) return TOMATIS_E_ARG;
  if (p->n_runs == 0) return TOMATIS_OK;
  hipStream_t s = (hipStream_t)hs;
  const int N = p->d.n_fft;
  if (p->lds) {
    LdsArgs L;
    L.x = x;
    L.st = p->st;
    L.n_streams = p->n_streams;
    L.gains = gains;
    L.rows = rows;
    L.win = p->win;
    L.win2 = p->win2;
    L.tw = p->twL;
    L.blue_b = p->blue_b;
    L.blue_h = p->blue_h;
    L.work = p->glb_work;
    L.M = p->lds_M;
    L.blue = p->blue ? 1 : 0;
    L.work_blocks = p->glb_blocks;
    L.scratch = reinterpret_cast<float*>(p->scratch);
    L.y = y;
    L.peaks = peaks;
    L.pos_base = p->pos_base;
    L.total_frames = p->total_frames;
    L.total_out = p->total_out;
    L.n_fft = N;
    L.hop = p->d.hop;
    L.ch = p->d.ch;
    L.n_bins = N / 2 + 1;
    L.norm_mode = p->d.norm_mode;
    if (p->total_frames > 0) {
      launch_lds_frames(L, s);
      const int rc = launch_check();
      if (rc) return rc;
    }
    if (p->total_out == 0) return TOMATIS_OK;
    launch_lds_gather(L, s);
    return launch_check();
  }
  if (n_rows > p->gperm_rows) {  // grows only; reuse across calls (graph-safe after first call)
    dfree(p->gperm);
    p->gperm = nullptr;
    if (hipMalloc(reinterpret_cast<void**>(&p->gperm), (size_t)n_rows * N * sizeof(float)))
      return TOMATIS_E_NOMEM;
    p->gperm_rows = n_rows;
  }
  MainArgs A;
  A.x = x;
  A.y = y;
  A.gains = p->gperm;
  A.rows = rows;
  A.peaks = peaks;
  A.st = p->st;
  A.runs = p->runs;
  A.win = p->win;
  A.winS = p->winS;
  A.win2 = p->win2;
  A.twN = p->twN;
  A.twP = p->twP;
  A.winv = p->winv;
  A.scratch = p->scratch;
  A.n_runs = p->n_runs;
  A.hop = p->d.hop;
  A.n_bins = N / 2 + 1;
  A.ch = p->d.ch;
  A.norm_mode = p->d.norm_mode;
  A.rmax = p->generic ? 1 : p->rmax;
  A.inv_n = 1.0f / (float)N;
  A.n_rows_lds = (n_rows <= 2 && N <= 2048) ? n_rows : 0;
  A.lds_mixed = 0;
  A.edge_mask = p->edge_mask;
  A.lds_row[0] = 0;
  A.lds_row[1] = 1;
  if (n_rows > 2 && N <= 2048 && p->d.alpha_mode != 0 && dev_opt(TOMATIS_DEV_GAIN_LDS, 1) != 0) {
    // cross-fade tables: the pure rows (alpha 0 and 1) carry most frames
    // (xfade: rows 0/1; adaptive: rows 2 and 2 + xfade_frames = n_rows - 1)
    A.n_rows_lds = 2;
    A.lds_mixed = 1;
    if (p->d.alpha_mode == 2) {
      A.lds_row[0] = 2;
      A.lds_row[1] = n_rows - 1;
    }
  }
  {  // every row in LDS (gm 1): the kernel prologue permutes the caller's rows
    const bool in_lds = !p->generic && !(p->P == 128 && p->NR == 32) && A.n_rows_lds == n_rows &&
                        !A.lds_mixed;
    A.graw = in_lds ? gains : nullptr;
    A.g_nb = N / 2 + 1;
    if (!in_lds) launch_gain_perm(p->P, p->NR, p->fx, gains, n_rows, N / 2 + 1, p->gperm, s);
  }
  A.limit = limit;
  A.chunk_done = p->chunk_done;
  A.chunk_need = p->chunk_need;
  A.chunk_rng = p->chunk_rng;
  A.err = p->err;
  A.lim_spin = p->lim_spin;
  A.prof = nullptr;
  A.run_base = 0;
  A.defer_self = 0;
  A.pieces = nullptr;
  A.max_pieces = 0;
  A.gated = 0;
  A.gate_D = p->d.up_delay_frames;
  A.r_out = nullptr;
  A.st_out = nullptr;
  A.gcarry = nullptr;
  A.gtf = nullptr;
  A.gate_xf = -1;
  A.a_out = nullptr;
  A.gacarry = nullptr;
  A.yprev = nullptr;
  A.peaks_prev = nullptr;
  A.runs_prev = p->runs;
  A.st_prev = p->st;
  A.chunk_rng_prev = p->chunk_rng;
  A.n_runs_prev = p->n_runs;
  if (gate) {
    // per run: the carry-in state id and leaf window (k_gate_carry), then the
    // transform computes every frame's r and state from the input it loads
    // (re-run a look-back made for another input or run layout: the caller's
    // tomatis_gate_lookback must match this call, the ABI does not assume it)
    if (!gate->lookback_done || p->n_runs > p->gate_cap || p->gl_x != x || p->gl_gen != p->runs_gen) {
      const int rc = gate_lookback(p, x, s);
      if (rc) return rc;
    }
    A.gated = 1;
    A.r_out = gate->r;
    A.st_out = gate->states;
    A.gcarry = p->gate_carry;
    A.gtf = (p->d.up_delay_frames + 2 <= kGateChainStates) ? p->gate_tf : nullptr;
    if (p->d.alpha_mode == 1) {  // cross-fade (n_fft 4096): alpha in-kernel
      A.gate_xf = p->d.xfade_frames;
      A.gate_astep = p->d.xfade_frames > 0 ? 1.0 / p->d.xfade_frames : 1.0;
      A.a_out = p->gate_aout;
      A.gacarry = p->gate_acarry;
      A.gtf = nullptr;
    }
  }
  if (limit > 0.f) {
    if (!p->chunk_done) return TOMATIS_E_UNSUPPORTED;
    // flush counters of the in-launch limiter (a pipelined batch counts none)
    if (!prev && hipMemsetAsync(p->chunk_done, 0, (size_t)p->total_chunks * 4, s))
      return TOMATIS_E_HIP;
  }
  const int nseq = 256 / p->P;
  const int blocks = (p->n_runs + nseq - 1) / nseq;
  const int ch = p->d.ch;
  if (p->generic) {
    launch_frames(A, p->P, p->NR, blocks, s);
    int rc = launch_check();
    if (rc || p->total_out == 0) return rc;
    launch_ola_gather(A, p->n_streams, p->pos_base, p->total_out, N, s);
    return launch_check();
  }
  if (prev) {
    // pipelined batch: this output stays unscaled for the next batch (its peaks
    // complete when the launch does); the previous batch's output, complete,
    // is limited block by block inside this launch's frame loops (k_r2_plan
    // lists each run's blocks of chunks over the limit), the rest in the runs'
    // tails -- no wave waits, and the rescale traffic overlaps the transform
    A.defer_self = 1;
    if (prev->y) {
      int rc = xs_pieces_alloc(p);
      if (rc) return rc;
      A.yprev = prev->y;
      A.peaks_prev = prev->peaks;
      A.runs_prev = prev->plan->runs;
      A.st_prev = prev->plan->st;
      A.chunk_rng_prev = prev->plan->chunk_rng;
      A.n_runs_prev = prev->plan->n_runs;
      A.pieces = p->xs_pieces;
      A.max_pieces = p->xs_max_pieces;
      launch_r2_plan(A, p->xs_pieces, p->total_chunks, p->P, s);  // (zeroes this launch's peaks)
      if ((rc = launch_check())) return rc;
    } else if (hipMemsetAsync(peaks, 0, (size_t)p->total_chunks * 4, s)) {
      return TOMATIS_E_HIP;
    }
    launch_transform(A, p->P, p->NR, p->SH, ch, transform_wg(p->P, p->NR), s);
    int rc = launch_check();
    if (rc) return rc;
    launch_prev_runs(A, N, s);  // the previous plan's runs this launch has no partner for
    return launch_check();
  }
#ifdef TM_PROFILE
  static unsigned long long* prof = nullptr;
  if (!prof) (void)hipMalloc(reinterpret_cast<void**>(&prof), 16 * sizeof(unsigned long long));
  (void)hipMemsetAsync(prof, 0, 16 * sizeof(unsigned long long), s);
  A.prof = prof;
  launch_transform(A, p->P, p->NR, p->SH, ch, transform_wg(p->P, p->NR), s);
  {
    unsigned long long h[16];
    (void)hipMemcpyAsync(h, prof, sizeof(h), hipMemcpyDeviceToHost, s);
    (void)hipStreamSynchronize(s);
    const double fr = h[15] ? (double)h[15] : 1.0;
    fprintf(stderr, "[tm_profile] frames %llu cycles/frame: top %.0f win %.0f fwd %.0f gain %.0f inv %.0f synth %.0f emit %.0f\n",
            h[15], h[0] / fr, h[1] / fr, h[2] / fr, h[3] / fr, h[4] / fr, h[5] / fr, h[6] / fr);
    const double nw = h[10] ? (double)h[10] : 1.0;
    fprintf(stderr, "[tm_profile] waves %llu prologue %.0f lifetime %.0f cycles, %.1f us, clock %.2f GHz, loop share %.3f\n",
            h[10], h[7] / nw, h[8] / nw, h[9] / nw / 100.0, h[9] ? (double)h[8] / (double)h[9] * 0.1 : 0.0,
            (h[0] + h[1] + h[2] + h[3] + h[4] + h[5] + h[6]) / (double)(h[8] ? h[8] : 1));
  }
  return launch_check();
#endif
  launch_transform(A, p->P, p->NR, p->SH, ch, transform_wg(p->P, p->NR), s);
  return launch_check();
}

int tomatis_stft_ola(tomatis_plan_t p, const float* x, const float* gains, int32_t n_rows,
                     const uint16_t* rows, float* y, uint32_t* peaks, void* hs) {
  return stft_ola_impl(p, x, gains, n_rows, rows, y, peaks, 0.f, hs);
}

// chunks whose flushes come from at most this many consecutive runs are limited
// inside the main kernel (waves wait only on near neighbours).
// Runs are dispatched in order and a wave waits only for runs of its own
// chunks, so at most one chunk is partly dispatched while its waves wait: any
// span up to the resident slots progresses; half of them keeps a margin.
constexpr int kFuseMaxSpan = 64;
static int64_t fuse_max_span(const tomatis_plan_s* p) {
  return std::max<int64_t>(kFuseMaxSpan, p->run_slots / 2);
}

static int limiter_launch(tomatis_plan_t p, float* y, const uint32_t* peaks, float limit,
                          int sel, int edge_mask, void* hs) {
  if (!p || !y || !peaks) return TOMATIS_E_ARG;
  if (p->n_chunkdesc == 0) return TOMATIS_OK;
  const int64_t per = p->max_chunk * p->d.ch;
  // ~2 float4 per thread per chunk
  const unsigned gx = (unsigned)std::min<int64_t>(std::max<int64_t>(1, (per + 2047) / 2048), 4096);
  hipLaunchKernelGGL(k_limiter, dim3(gx, p->n_chunkdesc), dim3(256), 0, (hipStream_t)hs, y, p->st,
                     p->chunks, peaks, limit, p->d.ch, sel, edge_mask);
  return launch_check();
}

int tomatis_stft_ola_limited_edges(tomatis_plan_t p, const float* x, const float* gains,
                                   int32_t n_rows, const uint16_t* rows, float* y,
                                   uint32_t* peaks, float limit, int32_t edge_mask, void* hs) {
  if (!p || !(limit > 0.f) || edge_mask < 0 || edge_mask > 3) return TOMATIS_E_ARG;
  const bool fuse = !p->generic && p->chunk_done && p->fuse_span > 0 && p->fuse_enabled &&
                    p->fuse_span <= fuse_max_span(p) && dev_opt(TOMATIS_DEV_FUSE_LIMITER, 1) != 0;
  p->edge_mask = edge_mask;
  int rc;
  if (fuse) {
    rc = stft_ola_impl(p, x, gains, n_rows, rows, y, peaks, limit, hs);
  } else {
    rc = stft_ola_impl(p, x, gains, n_rows, rows, y, peaks, 0.f, hs);
    if (!rc) rc = limiter_launch(p, y, peaks, limit, edge_mask ? 1 : 0, edge_mask, hs);
  }
  p->edge_mask = 0;
  return rc;
}

// tomatis_stft_ola_gated eligibility: the fused kernel's interior loop at
// n_fft 2048 with hop 256 / 512 (the 16-leaf window spans whole hop blocks)
// and the standard gate (two rows), or its two-wave frames at n_fft 4096 with
// hop 1024 and the standard gate or the cross-fade (alpha in-kernel); float
// input used as is, and every stream addressable by the 31-bit buffer offsets
// of k_gate_carry's loads
static bool gated_eligible(const tomatis_plan_s* p) {
  const TomatisPlanDesc& d = p->d;
  if (dev_opt(TOMATIS_DEV_FUSED_LEVELS, 1) == 0) return false;
  if (p->generic || p->lds || p->NR != 32 || d.ch < 1 || d.ch > 2) return false;
  const bool f2048 = p->P == 64 && d.n_fft == 2048 && (p->SH == 4 || p->SH == 8) && d.alpha_mode == 0;
  // (n_fft 4096: measured slower than the two-pass chain -- the level pass's
  // HBM read costs less than the level arithmetic inside the two-wave frame
  // loop, DESIGN.md §6 "Fused levels at 4096" -- so opt-in)
  const bool f4096 = dev_opt(TOMATIS_DEV_FUSED_4096, 0) != 0 &&
                     p->P == 128 && d.n_fft == 4096 && p->SH == 8 && kFftX &&
                     (d.alpha_mode == 0 || d.alpha_mode == 1) &&
                     transform_wg(p->P, p->NR) == 512;
  if (!(f2048 || f4096)) return false;
  for (int s = 0; s < p->n_streams; ++s) {
    const TomatisStream& S = p->hs[s];
    if (S.in_scale != 1.f || S.n * d.ch * 4 > 0x7fffffffll) return false;
  }
  return true;
}

int tomatis_plan_set_gate_alpha(tomatis_plan_t p, double* alpha_out) {
  if (!p) return TOMATIS_E_ARG;
  p->gate_aout = alpha_out;
  return TOMATIS_OK;
}

int tomatis_gate_lookback(tomatis_plan_t p, const float* x, void* hs) {
  if (!p || !x) return TOMATIS_E_ARG;
  if (!gated_eligible(p)) return TOMATIS_E_UNSUPPORTED;
  return gate_lookback(p, x, (hipStream_t)hs);
}

// gain rows of a gated call: g1, g2 (standard); cross-fade: g1, g2 and the
// alpha lattice 0, 1/xf, ..., 1 (rows 2 + m), with the caller's alpha output set
static bool gated_rows_ok(const tomatis_plan_s* p, int32_t n_rows) {
  if (p->d.alpha_mode != 1) return n_rows == 2;
  return p->gate_aout && n_rows >= 2 + std::max(2, p->d.xfade_frames + 1);
}

static int stft_ola_gated(tomatis_plan_t p, const float* x, const float* gains, int32_t n_rows,
                          float* y, uint32_t* peaks, float limit, float* r_out,
                          uint8_t* states_out, bool lookback_done, void* hs) {
  if (!p || !x || !gains || !y || !peaks || !r_out || !states_out || limit < 0.f)
    return TOMATIS_E_ARG;
  if (!gated_eligible(p)) return TOMATIS_E_UNSUPPORTED;
  if (!gated_rows_ok(p, n_rows)) return TOMATIS_E_ARG;
  const GateOut g{r_out, states_out, lookback_done};
  if (!(limit > 0.f)) return stft_ola_impl(p, x, gains, n_rows, nullptr, y, peaks, 0.f, hs, &g);
  const bool fuse = p->chunk_done && p->fuse_span > 0 && p->fuse_enabled &&
                    p->fuse_span <= fuse_max_span(p) && dev_opt(TOMATIS_DEV_FUSE_LIMITER, 1) != 0;
  if (fuse) return stft_ola_impl(p, x, gains, n_rows, nullptr, y, peaks, limit, hs, &g);
  int rc = stft_ola_impl(p, x, gains, n_rows, nullptr, y, peaks, 0.f, hs, &g);
  if (!rc) rc = limiter_launch(p, y, peaks, limit, 0, 0, hs);
  return rc;
}

int tomatis_stft_ola_gated(tomatis_plan_t p, const float* x, const float* gains, int32_t n_rows,
                           float* y, uint32_t* peaks, float limit, float* r_out,
                           uint8_t* states_out, void* hs) {
  return stft_ola_gated(p, x, gains, n_rows, y, peaks, limit, r_out, states_out, false, hs);
}

int tomatis_stft_ola_gated_after_lookback(tomatis_plan_t p, const float* x, const float* gains,
                                          int32_t n_rows, float* y, uint32_t* peaks, float limit,
                                          float* r_out, uint8_t* states_out, void* hs) {
  return stft_ola_gated(p, x, gains, n_rows, y, peaks, limit, r_out, states_out, true, hs);
}

// a previous batch another plan wrote can be limited by this plan's launch
// when the partner rescale's block geometry is the same (n_fft, hop, channels,
// kernel shape) and that plan has per-chunk output ranges
static bool prev_plan_ok(const tomatis_plan_s* p, const tomatis_plan_s* q) {
  if (q == p) return true;
  return q->d.n_fft == p->d.n_fft && q->d.hop == p->d.hop && q->d.ch == p->d.ch && q->P == p->P &&
         q->NR == p->NR && q->SH == p->SH && !q->generic && !q->lds && q->chunk_rng &&
         q->total_chunks > 0;
}

int tomatis_stft_ola_gated_pipelined_after(tomatis_plan_t p, const float* x, const float* gains,
                                           int32_t n_rows, float* y, uint32_t* peaks, float limit,
                                           float* r_out, uint8_t* states_out, tomatis_plan_t prev_plan,
                                           float* prev_y, const uint32_t* prev_peaks, void* hs) {
  if (!p || !x || !gains || !y || !peaks || !r_out || !states_out ||
      !(limit > 0.f) || (prev_y && (!prev_peaks || prev_y == y || prev_peaks == peaks)))
    return TOMATIS_E_ARG;
  // the kernel's partner-rescale instantiations (gated_eligible): n_fft 2048
  // interior loop, two LDS gain rows, hop <= 512; n_fft 4096, hop 1024;
  // per-chunk accounting
  if (!gated_eligible(p) || p->total_chunks <= 0 || !p->chunk_need || p->SH > 8)
    return TOMATIS_E_UNSUPPORTED;
  if (!gated_rows_ok(p, n_rows)) return TOMATIS_E_ARG;
  const tomatis_plan_s* q = prev_plan ? prev_plan : p;
  if (prev_y && !prev_plan_ok(p, q)) return TOMATIS_E_UNSUPPORTED;
  const GateOut g{r_out, states_out, true};
  const PrevBatch pb{prev_y, prev_peaks, q};
  return stft_ola_impl(p, x, gains, n_rows, nullptr, y, peaks, limit, hs, &g, &pb);
}

int tomatis_stft_ola_gated_pipelined(tomatis_plan_t p, const float* x, const float* gains,
                                     int32_t n_rows, float* y, uint32_t* peaks, float limit,
                                     float* r_out, uint8_t* states_out, float* prev_y,
                                     const uint32_t* prev_peaks, void* hs) {
  return tomatis_stft_ola_gated_pipelined_after(p, x, gains, n_rows, y, peaks, limit, r_out,
                                                states_out, nullptr, prev_y, prev_peaks, hs);
}

int tomatis_stft_ola_pipelined(tomatis_plan_t p, const float* x, const float* gains,
                               int32_t n_rows, const uint16_t* rows, float* y, uint32_t* peaks,
                               float limit, float* prev_y, const uint32_t* prev_peaks, void* hs) {
  return tomatis_stft_ola_pipelined_after(p, x, gains, n_rows, rows, y, peaks, limit, nullptr,
                                          prev_y, prev_peaks, hs);
}

int tomatis_stft_ola_pipelined_after(tomatis_plan_t p, const float* x, const float* gains,
                                     int32_t n_rows, const uint16_t* rows, float* y,
                                     uint32_t* peaks, float limit, tomatis_plan_t prev_plan,
                                     float* prev_y, const uint32_t* prev_peaks, void* hs) {
  if (!p || !x || !gains || !rows || !y || !peaks || n_rows < 1 || !(limit > 0.f) ||
      (prev_y && (!prev_peaks || prev_y == y || prev_peaks == peaks)))
    return TOMATIS_E_ARG;
  // the partner-rescale instantiations: n_fft 2048 interior loop, hop <= 512,
  // gain rows in LDS (one or two rows; the cross-fade lattice's pure rows at
  // hop 512); n_fft 4096 (two-wave frames, gain rows in L2, partner blocks
  // through VGPRs), hop <= 1024 at the 512-thread launch; per-chunk accounting
  const TomatisPlanDesc& d = p->d;
  const bool lds_rows = n_rows <= 2 ||
                        (d.alpha_mode != 0 && p->SH == 8 && dev_opt(TOMATIS_DEV_GAIN_LDS, 1) != 0);
  const bool p64 = p->P == 64 && lds_rows;
  const bool p128 = p->P == 128 && transform_wg(p->P, p->NR) == 512;
  if (p->generic || p->lds || p->NR != 32 || p->SH > 8 || !(p64 || p128) ||
      p->total_chunks <= 0 || !p->chunk_need)
    return TOMATIS_E_UNSUPPORTED;
  const tomatis_plan_s* q = prev_plan ? prev_plan : p;
  if (prev_y && !prev_plan_ok(p, q)) return TOMATIS_E_UNSUPPORTED;
  const PrevBatch pb{prev_y, prev_peaks, q};
  return stft_ola_impl(p, x, gains, n_rows, rows, y, peaks, limit, hs, nullptr, &pb);
}

int tomatis_stft_ola_limited(tomatis_plan_t p, const float* x, const float* gains,
                             int32_t n_rows, const uint16_t* rows, float* y, uint32_t* peaks,
                             float limit, void* hs) {
  return tomatis_stft_ola_limited_edges(p, x, gains, n_rows, rows, y, peaks, limit, 0, hs);
}

int tomatis_plan_error(tomatis_plan_t p, void* hs) {
  uint32_t e = 0;
  const int rc = tomatis_plan_error_bits(p, &e, 0, hs);
  if (rc) return rc;
  return e ? TOMATIS_E_HIP : TOMATIS_OK;
}

int tomatis_plan_error_bits(tomatis_plan_t p, uint32_t* bits, int32_t reset, void* hs) {
  if (!p || !p->err || !bits) return TOMATIS_E_ARG;
  uint32_t e = 0;
  if (hipMemcpyAsync(&e, p->err, 4, hipMemcpyDeviceToHost, (hipStream_t)hs)) return TOMATIS_E_HIP;
  if (hipStreamSynchronize((hipStream_t)hs)) return TOMATIS_E_HIP;
  *bits = e;
  if (reset && e) {
    if (hipMemsetAsync(p->err, 0, 4, (hipStream_t)hs)) return TOMATIS_E_HIP;
    if (hipStreamSynchronize((hipStream_t)hs)) return TOMATIS_E_HIP;
  }
  return TOMATIS_OK;
}

int tomatis_plan_set_option(tomatis_plan_t p, int32_t option, int64_t value) {
  if (!p) return TOMATIS_E_ARG;
  switch (option) {
    case TOMATIS_OPT_FUSE_LIMITER: p->fuse_enabled = value != 0; return TOMATIS_OK;
    case TOMATIS_OPT_LIMITER_SPIN:
      if (value < 0 || value > (1 << 24)) return TOMATIS_E_ARG;
      p->lim_spin = (int)value;
      return TOMATIS_OK;
    case TOMATIS_OPT_MINHOLD_SERIAL: p->mh_serial = value != 0; return TOMATIS_OK;
    default: return TOMATIS_E_ARG;
  }
}

int tomatis_set_dev_option(int32_t key, int32_t value) {
  if (key <= 0 || key >= tshared::kDevKeys) return TOMATIS_E_ARG;
  tshared::g_dev[key] = value < 0 ? -1 : value;
  return TOMATIS_OK;
}

int32_t tomatis_get_dev_option(int32_t key) {
  if (key <= 0 || key >= tshared::kDevKeys) return -1;
  return tshared::g_dev[key];
}


int tomatis_apply_limiter(tomatis_plan_t p, float* y, const uint32_t* peaks, float limit, void* hs) {
  return limiter_launch(p, y, peaks, limit, 0, 0, hs);
}

int tomatis_apply_limiter_edges(tomatis_plan_t p, float* y, const uint32_t* peaks, float limit,
                                int32_t edge_mask, void* hs) {
  if (edge_mask == 0) return p && y && peaks ? TOMATIS_OK : TOMATIS_E_ARG;
  return limiter_launch(p, y, peaks, limit, 2, edge_mask & 3, hs);
}

int tomatis_absmax(const float* x, int64_t n, uint32_t* out, void* hs) {
  if (!x || !out || n < 0) return TOMATIS_E_ARG;
  if (n == 0) return TOMATIS_OK;
  const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>(512, (n + 4095) / 4096));
  hipLaunchKernelGGL(k_absmax, dim3(g), dim3(256), 0, (hipStream_t)hs, x, n, out);
  return launch_check();
}

int tomatis_absmax_streams(tomatis_plan_t p, const float* x, uint32_t* out, void* hs) {
  if (!p || !x || !out) return TOMATIS_E_ARG;
  if (p->n_streams == 0) return TOMATIS_OK;
  int64_t nmax = 0;
  for (const auto& S : p->hs) nmax = std::max<int64_t>(nmax, S.n * p->d.ch);
  if (nmax == 0) return TOMATIS_OK;
  const unsigned gx = (unsigned)std::max<int64_t>(
      1, std::min<int64_t>(std::max(8, 1024 / p->n_streams), (nmax + 4095) / 4096));
  hipLaunchKernelGGL(k_absmax_streams, dim3(gx, p->n_streams), dim3(256), 0, (hipStream_t)hs, x,
                     p->st, p->d.ch, out);
  return launch_check();
}

int tomatis_scale_copy(const float* x, float* y, int64_t n, float scale, void* hs) {
  if (!x || !y || n < 0) return TOMATIS_E_ARG;
  if (n == 0) return TOMATIS_OK;
  const unsigned g = (unsigned)std::min<int64_t>(4096, (n + 1023) / 1024);
  hipLaunchKernelGGL(k_scale_copy, dim3(g), dim3(256), 0, (hipStream_t)hs, x, y, n, scale);
  return launch_check();
}

int tomatis_copy_probe(const float* x, float* y, int64_t n, void* hs) {
  if (!x || !y || n < 0 || (n & 3) || ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) & 15))
    return TOMATIS_E_ARG;
  const int64_t n4 = n / 4;
  if (n4 == 0) return TOMATIS_OK;
  if (n4 > (int64_t)0x7fffffff * 256) return TOMATIS_E_ARG;
  const unsigned g = (unsigned)((n4 + 255) / 256);
  hipLaunchKernelGGL(k_copy_probe, dim3(g), dim3(256), 0, (hipStream_t)hs,
                     reinterpret_cast<const float4*>(x), reinterpret_cast<float4*>(y), n4);
  return launch_check();
}

int tomatis_pcm_to_float(const int32_t* pcm, int64_t n, int32_t bps, float* out, void* hs) {
  if (!pcm || !out || n < 0 || bps < 2 || bps > 32) return TOMATIS_E_ARG;
  if (n == 0) return TOMATIS_OK;
  // x / 2^(bps-1): the reciprocal is a power of two, so the product is exact in double
  const double inv = 1.0 / (double)(1ll << (bps - 1));
  const unsigned g = (unsigned)std::min<int64_t>(8192, (n + 1023) / 1024);
  hipLaunchKernelGGL(k_pcm_to_float, dim3(g), dim3(256), 0, (hipStream_t)hs, pcm, n, inv, out);
  return launch_check();
}

int tomatis_float_to_pcm(const float* x, int64_t n, int32_t bps, int32_t* out, void* hs) {
  if (!x || !out || n < 0 || bps < 2 || bps > 32) return TOMATIS_E_ARG;
  if (n == 0) return TOMATIS_OK;
  const double top = (double)((1ll << (bps - 1)) - 1);
  const unsigned g = (unsigned)std::min<int64_t>(8192, (n + 1023) / 1024);
  hipLaunchKernelGGL(k_float_to_pcm, dim3(g), dim3(256), 0, (hipStream_t)hs, x, n, top,
                     -top - 1.0, top, out);
  return launch_check();
}

int tomatis_synth_fill(float* x, int64_t n, int32_t ch, int32_t sr, uint32_t seed, int64_t start,
                       void* hs) {
  if (!x || n < 0 || ch < 1 || sr < 1) return TOMATIS_E_ARG;
  if (n == 0) return TOMATIS_OK;
  const unsigned g = (unsigned)std::min<int64_t>(8192, (n * ch + 1023) / 1024);
  hipLaunchKernelGGL(k_synth, dim3(g), dim3(256), 0, (hipStream_t)hs, x, n, ch, sr, seed, start);
  return launch_check();
}

}  // extern "C"
