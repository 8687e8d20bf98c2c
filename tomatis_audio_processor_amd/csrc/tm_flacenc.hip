// tm_flacenc.hip — FLAC frames encoded on the device (SURVEY.md §8 row f1,
// the egress of src/process_tomatis.py:242-251,357: sf.SoundFile(...,
// format="FLAC", subtype="PCM_24") chunk writes).
//
// Byte for byte the frames of the host encoder (csrc/tm_flac.cpp,
// encode_blocks): 4096-sample blocks; per channel the cheapest of CONSTANT,
// FIXED (order = first minimum of the five sum |d_o| from sample 4; Rice /
// Rice2 partition order and parameters from partition sums, the libFLAC-style
// estimate c (k + 1) + (sum >> k), every tie resolved as the host loop resolves
// it) and VERBATIM; stereo picks the cheapest of independent, left/side,
// side/right and mid/side by the same estimates.  1-2 channels, 4-24 bits (the
// side channel's 25 bits and every fixed residual fit int32).
//
// Two launches per stream, one 256-thread workgroup per block:
//   k_fd_plan   the block's plan (assignment, per channel kind / order /
//               partition order / parameters) and the exact frame size in
//               bytes (the written residual is sum (u >> k) + c (k + 1) bits,
//               at most the estimate);
//   (host)      prefix sum of the sizes -> frame byte offsets, STREAMINFO;
//   k_fd_write  the frame in LDS (every field OR-ed into 32-bit LDS words at
//               its bit position: sample i's Rice code at the block-wide
//               exclusive scan of the code lengths), CRC-8 of the header,
//               CRC-16 of the frame (per-thread chunk CRCs shifted to the
//               frame end with x^(8 * 2^j) matrices and XOR-reduced), then out
//               to HBM as whole words (the two edge words shared with the
//               neighbouring frames OR-ed into the zeroed output).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tomatis_hip.h"

namespace {

constexpr int kFdBlock = 4096;       // samples per FLAC block (tm_flac.cpp kBlock)
constexpr int kFdThreads = 256;
constexpr int kFdMaxPart = 8;        // tm_flac.cpp kMaxPart
constexpr int kFdParts = 1 << kFdMaxPart;
// frame bytes bound: 2 channels x (8 + 4096 x 25) bits + header + CRC (a FIXED
// subframe is chosen only when its estimate, an upper bound of its size, is
// below VERBATIM's)
constexpr int kFdFrameWords = (2 * (8 + kFdBlock * 25) / 8 + 64) / 4 + 2;

struct FdChan {
  uint8_t sig, kind, order, porder, method, pad[3];
  uint8_t k[kFdParts];
};
struct FdPlan {
  uint32_t assign;
  uint32_t bits[2];   // exact subframe bits per channel
  FdChan c[2];
};

// ---------------------------------------------------------------------------
// block reductions (256 threads = 4 waves)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ uint32_t wave_or_u32(uint32_t v) {
  for (int o = 32; o > 0; o >>= 1) v |= __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ uint32_t wave_xor_u32(uint32_t v) {
  for (int o = 32; o > 0; o >>= 1) v ^= __shfl_xor(v, o, 64);
  return v;
}
// sum over the workgroup (every thread gets it); red: 4 slots
__device__ uint64_t block_sum_u64(uint64_t v, uint64_t* red) {
  v = wave_sum_u64(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

// ---------------------------------------------------------------------------
// signals: 0 left (or mono), 1 right, 2 side = L - R, 3 mid = (L + R) >> 1
// ---------------------------------------------------------------------------
__device__ __forceinline__ int32_t sig_at(const int32_t* sL, const int32_t* sR, int sig, int i) {
  switch (sig) {
    case 0: return sL[i];
    case 1: return sR[i];
    case 2: return sL[i] - sR[i];
    default: return (sL[i] + sR[i]) >> 1;
  }
}

__device__ __forceinline__ int32_t fixed_res(const int32_t* sL, const int32_t* sR, int sig,
                                             int order, int i) {
  const int32_t s0 = sig_at(sL, sR, sig, i);
  switch (order) {
    case 0: return s0;
    case 1: return s0 - sig_at(sL, sR, sig, i - 1);
    case 2: return s0 - 2 * sig_at(sL, sR, sig, i - 1) + sig_at(sL, sR, sig, i - 2);
    case 3:
      return s0 - 3 * sig_at(sL, sR, sig, i - 1) + 3 * sig_at(sL, sR, sig, i - 2) -
             sig_at(sL, sR, sig, i - 3);
    default:
      return s0 - 4 * sig_at(sL, sR, sig, i - 1) + 6 * sig_at(sL, sR, sig, i - 2) -
             4 * sig_at(sL, sR, sig, i - 3) + sig_at(sL, sR, sig, i - 4);
  }
}
__device__ __forceinline__ uint32_t zz32(int32_t r) {
  return ((uint32_t)r << 1) ^ (uint32_t)(r >> 31);
}

// largest partition order (tm_flac.cpp plan_rice)
__device__ __forceinline__ int fd_pmax(int n, int order) {
  int pmax = 0;
  while (pmax < kFdMaxPart && n % (1 << (pmax + 1)) == 0 && (n >> (pmax + 1)) > order) ++pmax;
  return pmax;
}
__device__ __forceinline__ int part_lo(int p, int ps, int order) { return p == 0 ? order : p * ps; }

struct FdShared {
  uint64_t sum[kFdParts];
  uint32_t mx[kFdParts];
  int cnt[kFdParts];
  uint64_t red[4];
  uint32_t redu[4];
  int flag;
};

// plan of one signal (every thread; result valid in every thread)
struct SigPlan {
  int kind, order, porder, method;
  uint64_t bits;
};
__device__ SigPlan plan_signal(const int32_t* sL, const int32_t* sR, int sig, int n, int bps,
                               FdShared& S, uint8_t* kout) {
  const int t = threadIdx.x;
  SigPlan best{1, 0, 0, 0, 8 + (uint64_t)n * bps};
  // CONSTANT
  const int32_t v0 = sig_at(sL, sR, sig, 0);
  int same = 1;
  for (int i = t; i < n; i += kFdThreads) same &= sig_at(sL, sR, sig, i) == v0;
  if (__syncthreads_and(same)) {
    best.kind = 0;
    best.bits = 8 + bps;
    return best;
  }
  // fixed order: first minimum of sum |d_o|, o = 0..4, over samples 4..n-1
  int bo = 0;
  if (n > 4) {
    uint64_t e[5] = {0, 0, 0, 0, 0};
    for (int i = 4 + t; i < n; i += kFdThreads) {
#pragma unroll
      for (int o = 0; o < 5; ++o) {
        const int32_t d = fixed_res(sL, sR, sig, o, i);
        e[o] += (uint64_t)(d < 0 ? -(int64_t)d : (int64_t)d);
      }
    }
    uint64_t tot[5];
#pragma unroll
    for (int o = 0; o < 5; ++o) tot[o] = block_sum_u64(e[o], S.red);
    for (int o = 1; o < 5; ++o)
      if (tot[o] < tot[bo]) bo = o;
  }
  // finest partitions: zigzag sums, maxima, counts
  const int pmax = fd_pmax(n, bo);
  const int np = 1 << pmax, ps = n >> pmax;
  __syncthreads();
  if (t < np) {
    const int a = part_lo(t, ps, bo), b = (t + 1) * ps;
    uint64_t sm = 0;
    uint32_t m = 0;
    for (int i = a; i < b; ++i) {
      const uint32_t u = zz32(fixed_res(sL, sR, sig, bo, i));
      sm += u;
      m = max(m, u);
    }
    S.sum[t] = sm;
    S.mx[t] = m;
    S.cnt[t] = b - a;
  }
  __syncthreads();
  // partition orders pmax .. 0 (the host's loop and tie rule: strictly smaller)
  uint64_t best_rice = ~0ull;
  int best_po = 0, best_method = 0;
  for (int po = pmax; po >= 0; --po) {
    const int parts = 1 << po;
    uint64_t bb = 0;
    uint32_t k5 = 0;
    int k = 0;
    if (t < parts) {
      const uint64_t sm = S.sum[t];
      const uint32_t m = S.mx[t];
      const int c = S.cnt[t];
      if (c > 0) {
        const uint64_t mean = sm / (uint64_t)c;
        while (k < 30 && (1ull << (k + 1)) <= mean) ++k;
      }
      bb = (uint64_t)c * (k + 1) + (sm >> k);
      if (((uint64_t)m >> k) >= (1ull << 24)) bb = 1ull << 60;
      k5 = k > 14 ? 1u : 0u;
    }
    uint64_t tot = block_sum_u64(bb, S.red);  // wraps as the host's uint64 sum
    const uint32_t w5 = wave_or_u32(k5);
    __syncthreads();
    if ((t & 63) == 0) S.redu[t >> 6] = w5;
    __syncthreads();
    const bool need5 = (S.redu[0] | S.redu[1] | S.redu[2] | S.redu[3]) != 0;
    tot += 2 + 4;
    tot += (uint64_t)parts * (need5 ? 5 : 4);
    if (tot < best_rice) {
      best_rice = tot;
      best_po = po;
      best_method = need5 ? 1 : 0;
      if (t < parts) kout[t] = (uint8_t)k;
    }
    // merge pairs for the next coarser order
    uint64_t s2 = 0;
    uint32_t m2 = 0;
    int c2 = 0;
    if (t < parts / 2) {
      s2 = S.sum[2 * t] + S.sum[2 * t + 1];
      m2 = max(S.mx[2 * t], S.mx[2 * t + 1]);
      c2 = S.cnt[2 * t] + S.cnt[2 * t + 1];
    }
    __syncthreads();
    if (t < parts / 2) {
      S.sum[t] = s2;
      S.mx[t] = m2;
      S.cnt[t] = c2;
    }
    __syncthreads();
  }
  const uint64_t bits = 8 + (uint64_t)bo * bps + best_rice;
  if (bits < best.bits) {
    best.kind = 2;
    best.order = bo;
    best.porder = best_po;
    best.method = best_method;
    best.bits = bits;
  }
  return best;
}

// exact size of a planned subframe (bits); k: the partition parameters (LDS)
__device__ uint64_t subframe_bits(const int32_t* sL, const int32_t* sR, int sig, const SigPlan& c,
                                  const uint8_t* k, int n, int sbps, FdShared& S) {
  if (c.kind == 0) return 8 + (uint64_t)sbps;
  if (c.kind == 1) return 8 + (uint64_t)n * sbps;
  const int ps = n >> c.porder, parts = 1 << c.porder;
  uint64_t acc = 0;
  for (int i = c.order + threadIdx.x; i < n; i += kFdThreads) {
    const int kp = k[i / ps];
    acc += (uint64_t)(zz32(fixed_res(sL, sR, sig, c.order, i)) >> kp) + 1 + kp;
  }
  const uint64_t codes = block_sum_u64(acc, S.red);
  return 8 + (uint64_t)c.order * sbps + 6 + (uint64_t)parts * (c.method ? 5 : 4) + codes;
}

__device__ __forceinline__ int utf8_bytes(uint64_t v) {
  if (v < 0x80) return 1;
  int nb = 2;
  while (nb < 7 && v >= (1ull << (5 * nb + 1))) ++nb;
  return nb;
}
__device__ __forceinline__ int header_bits(int64_t fn, int n) {
  return 32 + 8 * utf8_bytes((uint64_t)fn) + (n == kFdBlock ? 0 : 16) + 8;
}

__device__ __forceinline__ void load_block(const int32_t* __restrict__ pcm, int64_t f0, int n,
                                           int ch, int32_t* sL, int32_t* sR, int bps,
                                           int* bad) {
  const int64_t lim = (1ll << (bps - 1)) - 1;
  int b = 0;
  for (int i = threadIdx.x; i < n; i += kFdThreads) {
    const int32_t l = pcm[(f0 + i) * ch];
    const int32_t r = ch == 2 ? pcm[(f0 + i) * ch + 1] : 0;
    b |= (l > lim || l < -lim - 1) || (ch == 2 && (r > lim || r < -lim - 1));
    sL[i] = l;
    sR[i] = r;
  }
  if (__syncthreads_or(b) && threadIdx.x == 0) *bad = 1;
  __syncthreads();
}

template <int CH>
__global__ __launch_bounds__(kFdThreads) void k_fd_plan(const int32_t* __restrict__ pcm,
                                                        int64_t frames, int bps,
                                                        FdPlan* __restrict__ plans,
                                                        uint32_t* __restrict__ frame_bytes) {
  __shared__ int32_t sL[kFdBlock], sR[kFdBlock];
  __shared__ FdShared S;
  __shared__ uint8_t kk[4][kFdParts];
  __shared__ int bad;
  const int64_t fn = blockIdx.x;
  const int64_t f0 = fn * kFdBlock;
  const int n = (int)min<int64_t>(kFdBlock, frames - f0);
  if (threadIdx.x == 0) bad = 0;
  __syncthreads();
  load_block(pcm, f0, n, CH, sL, sR, bps, &bad);
  if (bad) {
    if (threadIdx.x == 0) frame_bytes[fn] = 0xFFFFFFFFu;
    return;
  }
  SigPlan sp[4];
  const int nsig = CH == 2 ? 4 : 1;
  for (int s = 0; s < nsig; ++s) sp[s] = plan_signal(sL, sR, s, n, s == 2 ? bps + 1 : bps, S, kk[s]);
  __syncthreads();
  int assign = CH - 1, c0 = 0, c1 = 1;
  if (CH == 2) {
    const uint64_t c_ind = sp[0].bits + sp[1].bits, c_ls = sp[0].bits + sp[2].bits,
                   c_sr = sp[2].bits + sp[1].bits, c_ms = sp[3].bits + sp[2].bits;
    const uint64_t m = min(min(c_ind, c_ls), min(c_sr, c_ms));
    if (m == c_ind) {
      assign = 1, c0 = 0, c1 = 1;
    } else if (m == c_ls) {
      assign = 8, c0 = 0, c1 = 2;
    } else if (m == c_sr) {
      assign = 9, c0 = 2, c1 = 1;
    } else {
      assign = 10, c0 = 3, c1 = 2;
    }
  }
  FdPlan& P = plans[fn];
  const int sel[2] = {c0, c1};
  uint64_t bits = header_bits(fn, n);
  for (int c = 0; c < CH; ++c) {
    const int s = sel[c];
    const SigPlan& q = sp[s];
    if (threadIdx.x == 0) {
      P.c[c].sig = (uint8_t)s;
      P.c[c].kind = (uint8_t)q.kind;
      P.c[c].order = (uint8_t)q.order;
      P.c[c].porder = (uint8_t)q.porder;
      P.c[c].method = (uint8_t)q.method;
    }
    if (threadIdx.x < (1 << q.porder)) P.c[c].k[threadIdx.x] = kk[s][threadIdx.x];
    // exact size (the written residual: sum (u >> k) + c (k + 1) <= the estimate)
    const uint64_t b = subframe_bits(sL, sR, s, q, kk[s], n, bps + (s == 2 ? 1 : 0), S);
    if (threadIdx.x == 0) P.bits[c] = (uint32_t)b;
    bits += b;
  }
  if (threadIdx.x == 0) {
    P.assign = (uint32_t)assign;
    const uint64_t bytes = (bits + 7) / 8 + 2;
    // beyond the writer's LDS frame (a wrapped partition estimate): host encoder
    frame_bytes[fn] = bytes > (uint64_t)(kFdFrameWords - 2) * 4 ? 0xFFFFFFFEu : (uint32_t)bytes;
  }
}

// ---------------------------------------------------------------------------
// writer
// ---------------------------------------------------------------------------
// OR the n-bit field v (n <= 32, MSB first) at frame bit position pos
__device__ __forceinline__ void put_bits(uint32_t* buf, uint64_t pos, uint32_t v, int n) {
  if (n <= 0) return;
  const int off = (int)(pos & 7);
  const uint64_t img = (n == 32 ? (uint64_t)v : ((uint64_t)v & ((1ull << n) - 1))) << (64 - off - n);
  const uint64_t B0 = pos >> 3;
  const int nb = (off + n + 7) >> 3;
  uint32_t w[3] = {0, 0, 0};
  const uint64_t W0 = B0 >> 2;
  for (int t = 0; t < nb; ++t) {
    const uint64_t B = B0 + t;
    const uint32_t byte = (uint32_t)(img >> (56 - 8 * t)) & 0xFFu;
    w[(B >> 2) - W0] |= byte << (8 * (B & 3));
  }
  for (int i = 0; i < 3; ++i)
    if (w[i]) atomicOr(buf + W0 + i, w[i]);
}
__device__ __forceinline__ uint32_t get_byte(const uint32_t* buf, uint64_t b) {
  return (buf[b >> 2] >> (8 * (b & 3))) & 0xFFu;
}

struct FdCrc {
  uint16_t t16[256];
  uint16_t mat[16][16];  // mat[j][b]: 2^j zero bytes appended to the CRC 1 << b
  uint8_t t8[256];
};

__device__ void crc_tables(FdCrc& C) {
  const int t = threadIdx.x;
  if (t < 256) {
    uint16_t d = (uint16_t)(t << 8);
    for (int b = 0; b < 8; ++b) d = (uint16_t)((d & 0x8000) ? (d << 1) ^ 0x8005 : (d << 1));
    C.t16[t] = d;
    uint8_t c = (uint8_t)t;
    for (int b = 0; b < 8; ++b) c = (uint8_t)((c & 0x80) ? (c << 1) ^ 0x07 : (c << 1));
    C.t8[t] = c;
  }
  __syncthreads();
  if (t < 16) {  // one zero byte
    const uint16_t c = (uint16_t)(1u << t);
    C.mat[0][t] = (uint16_t)((uint16_t)(c << 8) ^ C.t16[c >> 8]);
  }
  __syncthreads();
  for (int j = 1; j < 16; ++j) {  // M_j = M_{j-1} o M_{j-1}
    uint16_t r = 0;
    if (t < 16) {
      const uint16_t x = C.mat[j - 1][t];
      for (int b = 0; b < 16; ++b)
        if ((x >> b) & 1) r ^= C.mat[j - 1][b];
    }
    __syncthreads();
    if (t < 16) C.mat[j][t] = r;
    __syncthreads();
  }
}
// c x^(8 m) mod P: m zero bytes appended
__device__ __forceinline__ uint16_t crc_shift(const FdCrc& C, uint16_t c, uint32_t m) {
  for (int j = 0; m && j < 16; ++j, m >>= 1) {
    if (m & 1) {
      uint16_t r = 0;
      for (int b = 0; b < 16; ++b)
        if ((c >> b) & 1) r ^= C.mat[j][b];
      c = r;
    }
  }
  return c;
}

template <int CH>
__global__ __launch_bounds__(kFdThreads) void k_fd_write(const int32_t* __restrict__ pcm,
                                                         int64_t frames, int bps,
                                                         const FdPlan* __restrict__ plans,
                                                         const int64_t* __restrict__ frame_off,
                                                         uint8_t* __restrict__ out) {
  __shared__ int32_t sL[kFdBlock], sR[kFdBlock];
  __shared__ uint32_t fb[kFdFrameWords];
  __shared__ FdCrc C;
  __shared__ uint64_t red[4];
  __shared__ uint32_t scan[kFdThreads];
  __shared__ FdPlan P;
  __shared__ int bad;
  const int t = threadIdx.x;
  const int64_t fn = blockIdx.x;
  const int64_t f0 = fn * kFdBlock;
  const int n = (int)min<int64_t>(kFdBlock, frames - f0);
  if (t == 0) bad = 0;
  for (int i = t; i < kFdFrameWords; i += kFdThreads) fb[i] = 0;
  {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(plans + fn);
    uint32_t* dst = reinterpret_cast<uint32_t*>(&P);
    for (int i = t; i < (int)(sizeof(FdPlan) / 4); i += kFdThreads) dst[i] = src[i];
  }
  crc_tables(C);
  load_block(pcm, f0, n, CH, sL, sR, bps, &bad);
  if (bad) return;
  // ---- frame header (thread 0) ----
  uint64_t pos = 0;
  if (t == 0) {
    put_bits(fb, 0, 0x3FFE, 14);
    put_bits(fb, 14, 0, 2);
    put_bits(fb, 16, n == kFdBlock ? 12 : 7, 4);
    put_bits(fb, 20, 0, 4);
    put_bits(fb, 24, P.assign, 4);
    const int ssc = bps == 8 ? 1 : bps == 12 ? 2 : bps == 16 ? 4 : bps == 20 ? 5 : bps == 24 ? 6 : 0;
    put_bits(fb, 28, (uint32_t)ssc, 3);
    put_bits(fb, 31, 0, 1);
    uint64_t p = 32;
    const uint64_t v = (uint64_t)fn;
    const int nb = utf8_bytes(v);
    if (nb == 1) {
      put_bits(fb, p, (uint32_t)v, 8);
      p += 8;
    } else {
      put_bits(fb, p, ((0xFF00u >> nb) & 0xFF) | (uint32_t)(v >> (6 * (nb - 1))), 8);
      p += 8;
      for (int i = nb - 2; i >= 0; --i) {
        put_bits(fb, p, 0x80u | (uint32_t)((v >> (6 * i)) & 0x3F), 8);
        p += 8;
      }
    }
    if (n != kFdBlock) {
      put_bits(fb, p, (uint32_t)(n - 1), 16);
      p += 16;
    }
    uint8_t c8 = 0;
    for (uint64_t b = 0; b < p / 8; ++b) c8 = C.t8[c8 ^ get_byte(fb, b)];
    put_bits(fb, p, c8, 8);
  }
  pos = (uint64_t)header_bits(fn, n);
  // ---- subframes ----
  for (int c = 0; c < CH; ++c) {
    const FdChan& K = P.c[c];  // (LDS)
    const int sbps = bps + (K.sig == 2 ? 1 : 0);
    const uint32_t smask = sbps >= 32 ? 0xFFFFFFFFu : ((1u << sbps) - 1);
    if (K.kind == 0) {
      if (t == 0) {
        put_bits(fb, pos, 0, 8);
        put_bits(fb, pos + 8, (uint32_t)sig_at(sL, sR, K.sig, 0) & smask, sbps);
      }
    } else if (K.kind == 1) {
      if (t == 0) put_bits(fb, pos, 2, 8);
      for (int i = t; i < n; i += kFdThreads)
        put_bits(fb, pos + 8 + (uint64_t)i * sbps, (uint32_t)sig_at(sL, sR, K.sig, i) & smask, sbps);
    } else {
      const int order = K.order, ps = n >> K.porder, pb = K.method ? 5 : 4;
      if (t == 0) {
        put_bits(fb, pos, (uint32_t)((8 | order) << 1), 8);
        for (int i = 0; i < order; ++i)
          put_bits(fb, pos + 8 + (uint64_t)i * sbps, (uint32_t)sig_at(sL, sR, K.sig, i) & smask,
                   sbps);
        put_bits(fb, pos + 8 + (uint64_t)order * sbps, K.method, 2);
        put_bits(fb, pos + 8 + (uint64_t)order * sbps + 2, K.porder, 4);
      }
      const uint64_t base = pos + 8 + (uint64_t)order * sbps + 6;
      // code lengths of samples [order, n): thread t owns a contiguous range
      const int m = n - order;
      const int per = (m + kFdThreads - 1) / kFdThreads;
      const int i0 = order + min(m, t * per), i1 = order + min(m, (t + 1) * per);
      uint32_t local = 0;
      for (int i = i0; i < i1; ++i) {
        const int p = i / ps;
        const int k = K.k[p];
        const uint32_t u = zz32(fixed_res(sL, sR, K.sig, order, i));
        local += (u >> k) + 1 + k + (i == part_lo(p, ps, order) ? pb : 0);
      }
      // exclusive scan of the per-thread totals
      scan[t] = local;
      __syncthreads();
      for (int o = 1; o < kFdThreads; o <<= 1) {
        const uint32_t add = t >= o ? scan[t - o] : 0;
        __syncthreads();
        scan[t] += add;
        __syncthreads();
      }
      uint64_t q = base + (scan[t] - local);
      for (int i = i0; i < i1; ++i) {
        const int p = i / ps;
        const int k = K.k[p];
        const uint32_t u = zz32(fixed_res(sL, sR, K.sig, order, i));
        if (i == part_lo(p, ps, order)) {
          put_bits(fb, q, (uint32_t)k, pb);
          q += pb;
        }
        const uint32_t hi = u >> k;
        put_bits(fb, q + hi, (k >= 31 ? 0u : (1u << k)) | (k == 0 ? 0u : (u & ((1u << k) - 1))),
                 k + 1);
        q += hi + 1 + k;
      }
      __syncthreads();
    }
    pos += P.bits[c];
  }
  __syncthreads();
  // ---- CRC-16 of the frame up to the padding, then the CRC ----
  const uint32_t body = (uint32_t)((pos + 7) / 8);
  const uint32_t per = (body + kFdThreads - 1) / kFdThreads;
  const uint32_t a = min(body, t * per), b = min(body, (t + 1) * per);
  uint16_t c16 = 0;
  for (uint32_t i = a; i < b; ++i) c16 = (uint16_t)((c16 << 8) ^ C.t16[(c16 >> 8) ^ get_byte(fb, i)]);
  c16 = crc_shift(C, c16, body - b);
  uint32_t x = wave_xor_u32(c16);
  __syncthreads();
  if ((t & 63) == 0) red[t >> 6] = x;
  __syncthreads();
  if (t == 0) put_bits(fb, (uint64_t)body * 8, (uint32_t)(red[0] ^ red[1] ^ red[2] ^ red[3]), 16);
  __syncthreads();
  // ---- out: whole words, the shared edge words OR-ed ----
  const int64_t O = frame_off[fn];
  const int64_t len = (int64_t)body + 2;
  const int64_t W0 = O >> 2, W1 = (O + len - 1) >> 2;
  uint32_t* ow = reinterpret_cast<uint32_t*>(out);
  for (int64_t W = W0 + t; W <= W1; W += kFdThreads) {
    uint32_t v = 0;
    bool full = true;
    for (int j = 0; j < 4; ++j) {
      const int64_t B = 4 * W + j - O;
      if (B >= 0 && B < len) v |= get_byte(fb, (uint64_t)B) << (8 * j);
      else full = false;
    }
    if (full) ow[W] = v;
    else if (v) atomicOr(ow + W, v);
  }
}

}  // namespace

extern "C" {

int64_t tomatis_flacd_workspace_bytes(int64_t frames, int32_t ch) {
  if (frames < 0 || ch < 1 || ch > 2) return -1;
  const int64_t nblk = (frames + kFdBlock - 1) / kFdBlock;
  return nblk * (int64_t)sizeof(FdPlan);
}

int tomatis_flacd_plan(const int32_t* pcm, int64_t frames, int32_t ch, int32_t bps, void* ws,
                       uint32_t* frame_bytes, void* hs) {
  if (frames < 0 || (frames > 0 && (!pcm || !ws || !frame_bytes))) return TOMATIS_E_ARG;
  if (ch < 1 || ch > 2 || bps < 4 || bps > 24) return TOMATIS_E_UNSUPPORTED;
  const int64_t nblk = (frames + kFdBlock - 1) / kFdBlock;
  if (nblk == 0) return TOMATIS_OK;
  if (nblk > 0x7FFFFFFF) return TOMATIS_E_ARG;
  hipStream_t s = (hipStream_t)hs;
  if (ch == 2)
    hipLaunchKernelGGL(k_fd_plan<2>, dim3((unsigned)nblk), dim3(kFdThreads), 0, s, pcm, frames,
                       (int)bps, (FdPlan*)ws, frame_bytes);
  else
    hipLaunchKernelGGL(k_fd_plan<1>, dim3((unsigned)nblk), dim3(kFdThreads), 0, s, pcm, frames,
                       (int)bps, (FdPlan*)ws, frame_bytes);
  return hipGetLastError() == hipSuccess ? TOMATIS_OK : TOMATIS_E_HIP;
}

int tomatis_flacd_write(const int32_t* pcm, int64_t frames, int32_t ch, int32_t bps,
                        const void* ws, const int64_t* frame_off, uint8_t* out, void* hs) {
  if (frames < 0 || (frames > 0 && (!pcm || !ws || !frame_off || !out))) return TOMATIS_E_ARG;
  if (ch < 1 || ch > 2 || bps < 4 || bps > 24) return TOMATIS_E_UNSUPPORTED;
  const int64_t nblk = (frames + kFdBlock - 1) / kFdBlock;
  if (nblk == 0) return TOMATIS_OK;
  hipStream_t s = (hipStream_t)hs;
  if (ch == 2)
    hipLaunchKernelGGL(k_fd_write<2>, dim3((unsigned)nblk), dim3(kFdThreads), 0, s, pcm, frames,
                       (int)bps, (const FdPlan*)ws, frame_off, out);
  else
    hipLaunchKernelGGL(k_fd_write<1>, dim3((unsigned)nblk), dim3(kFdThreads), 0, s, pcm, frames,
                       (int)bps, (const FdPlan*)ws, frame_off, out);
  return hipGetLastError() == hipSuccess ? TOMATIS_OK : TOMATIS_E_HIP;
}

}  // extern "C"
