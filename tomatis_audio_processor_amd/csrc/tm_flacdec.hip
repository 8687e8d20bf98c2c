// tm_flacdec.hip — FLAC frames decoded on the device (SURVEY.md §8 row f1,
// the ingest of src/process_tomatis.py:225-235: sf.read / sf.blocks of the
// input through libsndfile).
//
// The same grammar and checks as the host decoder (csrc/tm_flac.cpp,
// decode_frame): CONSTANT, VERBATIM, FIXED and LPC subframes, wasted bits,
// Rice / Rice2 partitions with escapes, every stereo assignment, fixed or
// variable block size headers, header CRC-8 and frame CRC-16.  Frames are
// independent once their start is known, so the file is decoded in three
// launches over its bytes (resident in HBM):
//   k_fdd_find    every byte position holding a frame sync code whose header
//                 parses and matches its CRC-8 -> candidate list;
//   k_fdd_scan    one thread per candidate walks its frame's bits (no
//                 samples): frame length, CRC-16, sample range;
//   (host)        the verified frames must chain from the first frame to the
//                 end of the stream, each starting where the previous one ended
//                 and covering consecutive samples (else the host decoder runs);
//   k_fdd_decode  one thread per chained frame decodes its samples into the
//                 interleaved int32 PCM at the frame's sample offset.
// 1-2 channels, 4-24 bits (side channel 25 bits; LPC sums in int64).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tomatis_hip.h"

namespace {

__device__ __forceinline__ uint8_t crc8_byte(uint8_t c, uint8_t b) {
  c ^= b;
#pragma unroll
  for (int i = 0; i < 8; ++i) c = (uint8_t)((c & 0x80) ? (c << 1) ^ 0x07 : (c << 1));
  return c;
}

// bit reader over the file bytes d[0, len), MSB first; 64-bit window refilled
// from aligned 32-bit words (the device copy of the file is 4-byte aligned)
struct BR {
  const uint32_t* w;
  int64_t nbits;   // len * 8
  int64_t pos;     // next bit
  uint64_t win;    // bits [pos, pos + avail) left-aligned
  int avail;
  int64_t nw;      // next word to load
  int64_t nwords;
  bool bad;
  __device__ void init(const uint8_t* d, int64_t len, int64_t bitpos) {
    w = reinterpret_cast<const uint32_t*>(d);
    nbits = len * 8;
    nwords = (len + 3) / 4;
    pos = bitpos;
    nw = bitpos >> 5;
    win = 0;
    avail = 0;
    bad = false;
    refill();
    const int skip = (int)(bitpos & 31);
    win <<= skip;
    avail -= skip;
    refill();
  }
  __device__ __forceinline__ void refill() {
    while (avail <= 32) {
      uint32_t x = 0;
      if (nw < nwords) x = __builtin_bswap32(w[nw]);
      ++nw;
      win |= (uint64_t)x << (32 - avail);
      avail += 32;
    }
  }
  __device__ __forceinline__ uint32_t get(int n) {  // n <= 32
    if (n == 0) return 0;
    if (avail < n) refill();
    const uint32_t v = (uint32_t)(win >> (64 - n));
    win <<= n;
    avail -= n;
    pos += n;
    if (pos > nbits) bad = true;
    return v;
  }
  __device__ __forceinline__ int32_t get_signed(int n) {  // n <= 32
    if (n == 0) return 0;
    const uint32_t v = get(n);
    return n == 32 ? (int32_t)v : (int32_t)(v << (32 - n)) >> (32 - n);
  }
  __device__ __forceinline__ uint32_t unary() {  // zeros before the next one
    uint32_t q = 0;
    while (true) {
      if (avail <= 32) refill();
      if (win != 0) {
        const int z = __builtin_clzll(win);
        // (a shift by 64 is not 0 on the hardware: the amount wraps mod 64)
        win = z >= 63 ? 0ull : win << (z + 1);
        avail -= z + 1;
        pos += z + 1;
        q += z;
        if (pos > nbits) bad = true;
        return q;
      }
      q += avail;
      pos += avail;
      win = 0;
      avail = 0;
      if (pos > nbits || q > (1u << 30)) {
        bad = true;
        return q;
      }
    }
  }
  __device__ __forceinline__ void align() {
    const int r = (int)(pos & 7);
    if (r) get(8 - r);
  }
  __device__ __forceinline__ uint8_t byte_at(int64_t b) const {
    const uint32_t x = w[b >> 2];
    return (uint8_t)(x >> (8 * (b & 3)));
  }
};

struct FHdr {
  int strategy, n, asg, nch, bps;
  uint64_t num;
  int hbytes;  // header bytes before the CRC-8
};

// header at byte p (tm_flac.cpp decode_frame's checks); false: not a frame
__device__ bool parse_header(BR& r, int64_t p, int ch0, int bps0, FHdr& h) {
  r.init(reinterpret_cast<const uint8_t*>(r.w), r.nbits / 8, p * 8);
  if (r.get(14) != 0x3FFE) return false;
  if (r.get(1)) return false;
  h.strategy = (int)r.get(1);
  const int bsc = (int)r.get(4), src = (int)r.get(4), asg = (int)r.get(4), ssc = (int)r.get(3);
  if (r.get(1)) return false;
  uint64_t num = r.get(8);
  if (num & 0x80) {
    int extra = 0;
    while (extra < 7 && (num & (0x40u >> extra))) ++extra;
    if (extra == 0) return false;
    num &= (0x3Fu >> extra);
    for (int i = 0; i < extra; ++i) {
      const uint32_t c = r.get(8);
      if ((c & 0xC0) != 0x80) return false;
      num = (num << 6) | (c & 0x3F);
    }
  }
  int n;
  if (bsc == 1) n = 192;
  else if (bsc >= 2 && bsc <= 5) n = 576 << (bsc - 2);
  else if (bsc == 6) n = (int)r.get(8) + 1;
  else if (bsc == 7) n = (int)r.get(16) + 1;
  else if (bsc >= 8) n = 256 << (bsc - 8);
  else return false;
  if (src == 12) r.get(8);
  else if (src == 13 || src == 14) r.get(16);
  else if (src == 15) return false;
  const int ss_tab[8] = {0, 8, 12, 0, 16, 20, 24, 32};
  const int bps = ssc == 0 ? bps0 : ss_tab[ssc];
  if (bps == 0) return false;
  h.hbytes = (int)((r.pos - p * 8) / 8);
  const uint32_t hcrc = r.get(8);
  if (r.bad) return false;
  uint8_t c8 = 0;
  for (int i = 0; i < h.hbytes; ++i) c8 = crc8_byte(c8, r.byte_at(p + i));
  if (c8 != hcrc) return false;
  const int nch = asg < 8 ? asg + 1 : 2;
  if (asg > 10 || nch != ch0) return false;
  h.n = n;
  h.asg = asg;
  h.nch = nch;
  h.bps = bps;
  h.num = num;
  return true;
}

// The frame's subframes (after parse_header): DEC = false only walks the bits;
// DEC = true also writes channel c's samples to out[(i) * ostride + c] for
// i < take (predicted, wasted bits restored; stereo decorrelated by the caller)
template <bool DEC>
__device__ bool walk_subframes(BR& r, const FHdr& h, int32_t* out, int ostride, int take) {
  const int n = h.n;
  for (int c = 0; c < h.nch; ++c) {
    int sb = h.bps;
    if ((h.asg == 8 && c == 1) || (h.asg == 9 && c == 0) || (h.asg == 10 && c == 1)) ++sb;
    if (r.get(1) != 0) return false;
    const int type = (int)r.get(6);
    int wasted = 0;
    if (r.get(1)) wasted = (int)r.unary() + 1;
    sb -= wasted;
    if (sb <= 0 || sb > 32) return false;
    int32_t* o = out + c;
    auto put = [&](int i, int32_t v) {
      if (DEC && i < take) o[(int64_t)i * ostride] = v;
    };
    if (type == 0) {
      const int32_t c0 = r.get_signed(sb);
      if (DEC)
        for (int i = 0; i < n; ++i) put(i, (int32_t)((uint32_t)c0 << wasted));
    } else if (type == 1) {
      for (int i = 0; i < n; ++i) {
        const int32_t v = r.get_signed(sb);
        put(i, (int32_t)((uint32_t)v << wasted));
      }
    } else if ((type & 0x38) == 0x08 || (type & 0x20)) {
      const bool lpc = (type & 0x20) != 0;
      const int order = lpc ? (type & 0x1F) + 1 : (type & 7);
      if ((!lpc && order > 4) || order > n) return false;
      // LPC predicts from its own output read back: only a frame that lies
      // wholly inside the PCM buffer (take == n) may be decoded here; one that
      // reaches past the stream's sample count goes to the host decoder (no
      // read outside the frame's written samples)
      if (DEC && lpc && take < n) return false;
      // warm-up samples (unshifted values kept for the prediction)
      int32_t hist[4] = {0, 0, 0, 0};  // FIXED: last samples, hist[0] newest
      for (int i = 0; i < order; ++i) {
        const int32_t v = r.get_signed(sb);
        if (DEC) {
          if (i < take) o[(int64_t)i * ostride] = v;  // unshifted until the end
          if (!lpc) {
            hist[3] = hist[2];
            hist[2] = hist[1];
            hist[1] = hist[0];
            hist[0] = v;
          }
        }
      }
      int32_t coef[32];
      int shift = 0;
      if (lpc) {
        const int prec = (int)r.get(4) + 1;
        if (prec == 16) return false;
        shift = r.get_signed(5);
        if (shift < 0) return false;
        for (int i = 0; i < order; ++i) coef[i] = r.get_signed(prec);
      }
      const int method = (int)r.get(2);
      if (method > 1) return false;
      const int po = (int)r.get(4);
      const int ps = n >> po;
      if ((ps << po) != n || ps < order) return false;
      const int pbits = method ? 5 : 4, esc = method ? 31 : 15;
      int i = order;
      for (int part = 0; part < (1 << po); ++part) {
        const int k = (int)r.get(pbits);
        const int end = (part + 1) * ps;
        const int nb = k == esc ? (int)r.get(5) : 0;
        for (; i < end; ++i) {
          int32_t res;
          if (k == esc) {
            res = r.get_signed(nb);
          } else {
            const uint32_t q = r.unary();
            const uint32_t u = (q << k) | r.get(k);
            res = (int32_t)(u >> 1) ^ -(int32_t)(u & 1);
          }
          if (DEC) {
            int32_t s;
            if (lpc) {
              int64_t acc = 0;
              for (int j = 0; j < order; ++j)
                acc += (int64_t)coef[j] * (int64_t)o[(int64_t)(i - 1 - j) * ostride];
              s = (int32_t)((uint32_t)res + (uint32_t)(acc >> shift));
            } else {
              int32_t pr;
              switch (order) {
                case 0: pr = 0; break;
                case 1: pr = hist[0]; break;
                case 2: pr = 2 * hist[0] - hist[1]; break;
                case 3: pr = 3 * hist[0] - 3 * hist[1] + hist[2]; break;
                default: pr = 4 * hist[0] - 6 * hist[1] + 4 * hist[2] - hist[3]; break;
              }
              s = (int32_t)((uint32_t)res + (uint32_t)pr);
              hist[3] = hist[2];
              hist[2] = hist[1];
              hist[1] = hist[0];
              hist[0] = s;
            }
            if (i < take) o[(int64_t)i * ostride] = s;
          }
        }
        if (r.bad) return false;
      }
      if (DEC && wasted)
        for (int t = 0; t < min(n, take); ++t)
          o[(int64_t)t * ostride] = (int32_t)((uint32_t)o[(int64_t)t * ostride] << wasted);
    } else {
      return false;
    }
    if (r.bad) return false;
  }
  r.align();
  return true;
}

__device__ uint16_t crc16_range(const BR& r, int64_t a, int64_t b) {
  uint16_t c = 0;
  for (int64_t i = a; i < b; ++i) {
    c ^= (uint16_t)r.byte_at(i) << 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) c = (uint16_t)((c & 0x8000) ? (c << 1) ^ 0x8005 : (c << 1));
  }
  return c;
}

__global__ __launch_bounds__(256) void k_fdd_find(const uint8_t* __restrict__ d, int64_t len,
                                                  int64_t first, int ch0, int bps0,
                                                  int64_t* __restrict__ cand, int cap,
                                                  int* __restrict__ count) {
  const int64_t p = first + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool hit = false;
  if (p + 1 < len) {
    const uint8_t b0 = d[p], b1 = d[p + 1];
    if (b0 == 0xFF && (b1 & 0xFE) == 0xF8) {
      BR r;
      r.w = reinterpret_cast<const uint32_t*>(d);
      r.nbits = len * 8;
      FHdr h;
      hit = parse_header(r, p, ch0, bps0, h);
    }
  }
  if (hit) {
    const int slot = atomicAdd(count, 1);
    if (slot < cap) cand[slot] = p;
  }
}

// per candidate: info[4 * i] = frame bytes (0: not a frame), [+1] first sample
// (frame number x nominal for fixed-blocksize frames), [+2] block size,
// [+3] blocking strategy (1: variable, the coded number is the first sample)
__global__ __launch_bounds__(64) void k_fdd_scan(const uint8_t* __restrict__ d, int64_t len,
                                                 const int64_t* __restrict__ cand, int nc,
                                                 int ch0, int bps0, int64_t nominal,
                                                 int64_t* __restrict__ info) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nc) return;
  const int64_t p = cand[i];
  BR r;
  r.w = reinterpret_cast<const uint32_t*>(d);
  r.nbits = len * 8;
  FHdr h{0, 0, 0, 0, 0, 0, 0};
  int64_t bytes = 0;
  if (parse_header(r, p, ch0, bps0, h) &&
      walk_subframes<false>(r, h, nullptr, 0, 0)) {
    const int64_t fb = r.pos / 8 - p;
    const uint32_t fcrc = r.get(16);
    if (!r.bad && crc16_range(r, p, p + fb) == fcrc) bytes = fb + 2;
  }
  info[4 * (int64_t)i] = bytes;
  info[4 * (int64_t)i + 1] = h.strategy ? (int64_t)h.num : (int64_t)h.num * nominal;
  info[4 * (int64_t)i + 2] = h.n;
  info[4 * (int64_t)i + 3] = h.strategy;
}

__global__ __launch_bounds__(64) void k_fdd_decode(const uint8_t* __restrict__ d, int64_t len,
                                                   const int64_t* __restrict__ frames, int nf,
                                                   int ch0, int bps0, int64_t nominal,
                                                   int32_t* __restrict__ pcm, int64_t max_frames,
                                                   int* __restrict__ err) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nf) return;
  const int64_t p = frames[i];
  BR r;
  r.w = reinterpret_cast<const uint32_t*>(d);
  r.nbits = len * 8;
  FHdr h;
  if (!parse_header(r, p, ch0, bps0, h)) {
    atomicOr(err, 1);
    return;
  }
  const int64_t off = h.strategy ? (int64_t)h.num : (int64_t)h.num * nominal;
  const int take = (int)min<int64_t>(h.n, max<int64_t>(0, max_frames - off));
  int32_t* o = pcm + max<int64_t>(0, off) * h.nch;
  if (!walk_subframes<true>(r, h, o, h.nch, take)) {
    atomicOr(err, 1);
    return;
  }
  if (h.nch == 2 && h.asg >= 8) {
    for (int t = 0; t < take; ++t) {
      int32_t a = o[2 * t], b = o[2 * t + 1];
      if (h.asg == 8) {
        b = a - b;  // left, side -> right
      } else if (h.asg == 9) {
        a = a + b;  // side, right -> left
      } else {     // mid, side
        const int64_t m = (int64_t)(((uint64_t)(int64_t)a << 1) | (uint64_t)(b & 1));
        a = (int32_t)((m + b) >> 1);
        b = (int32_t)((m - b) >> 1);
      }
      o[2 * t] = a;
      o[2 * t + 1] = b;
    }
  }
}

}  // namespace

extern "C" {

int tomatis_flacd_find(const uint8_t* d, int64_t len, int64_t first, int32_t ch, int32_t bps,
                       int64_t* cand, int32_t cap, int32_t* count, void* hs) {
  if (!d || !cand || !count || len < 0 || first < 0 || cap < 0) return TOMATIS_E_ARG;
  if (ch < 1 || ch > 2 || bps < 4 || bps > 24) return TOMATIS_E_UNSUPPORTED;
  const int64_t span = len - first;
  if (span <= 1) return TOMATIS_OK;
  const int64_t blocks = (span + 255) / 256;
  if (blocks > 0x7FFFFFFF) return TOMATIS_E_ARG;
  hipLaunchKernelGGL(k_fdd_find, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)hs, d, len,
                     first, (int)ch, (int)bps, cand, (int)cap, count);
  return hipGetLastError() == hipSuccess ? TOMATIS_OK : TOMATIS_E_HIP;
}

int tomatis_flacd_scan(const uint8_t* d, int64_t len, const int64_t* cand, int32_t nc, int32_t ch,
                       int32_t bps, int64_t nominal, int64_t* info, void* hs) {
  if (!d || (nc > 0 && (!cand || !info)) || nc < 0) return TOMATIS_E_ARG;
  if (ch < 1 || ch > 2 || bps < 4 || bps > 24) return TOMATIS_E_UNSUPPORTED;
  if (nc == 0) return TOMATIS_OK;
  hipLaunchKernelGGL(k_fdd_scan, dim3((unsigned)((nc + 63) / 64)), dim3(64), 0, (hipStream_t)hs,
                     d, len, cand, (int)nc, (int)ch, (int)bps, nominal, info);
  return hipGetLastError() == hipSuccess ? TOMATIS_OK : TOMATIS_E_HIP;
}

int tomatis_flacd_decode(const uint8_t* d, int64_t len, const int64_t* frames, int32_t nf,
                         int32_t ch, int32_t bps, int64_t nominal, int32_t* pcm,
                         int64_t max_frames, int32_t* err, void* hs) {
  if (!d || (nf > 0 && (!frames || !pcm || !err)) || nf < 0) return TOMATIS_E_ARG;
  if (ch < 1 || ch > 2 || bps < 4 || bps > 24) return TOMATIS_E_UNSUPPORTED;
  if (nf == 0) return TOMATIS_OK;
  hipLaunchKernelGGL(k_fdd_decode, dim3((unsigned)((nf + 63) / 64)), dim3(64), 0,
                     (hipStream_t)hs, d, len, frames, (int)nf, (int)ch, (int)bps, nominal, pcm,
                     max_frames, err);
  return hipGetLastError() == hipSuccess ? TOMATIS_OK : TOMATIS_E_HIP;
}

}  // extern "C"
