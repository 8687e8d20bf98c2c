// tm_flac.cpp — native FLAC codec for the file boundary.
//
// The reference reads its inputs and writes its outputs through libsndfile
// (`sf.read`, `sf.write(..., format="FLAC", subtype="PCM_24")`,
// src/process_tomatis.py:225,243-251, src/layer2_apply_eq.py:88-93,215-233);
// libsndfile is not in this image, so this host library encodes and decodes
// FLAC directly (C ABI in include/tomatis_flac.h).  FLAC is lossless: the
// decoded integers equal the encoded ones, so the float conversion around it
// (libsndfile's PCM_24 normalisation, done by the Python caller) is the only
// arithmetic that touches sample values.
//
// Encoder: fixed 4096-sample blocks, per channel the cheapest of CONSTANT,
// FIXED (order by the smallest |residual| sum; Rice / Rice2 partitioned
// residual, partition order and parameters from partition sums) and VERBATIM; stereo also tries the
// left/side, side/right and mid/side decorrelations.  STREAMINFO carries
// min/max block and frame sizes and total samples; MD5 is left zero
// ("unknown", allowed by the format).  Decoder: the full frame/subframe
// grammar (CONSTANT, VERBATIM, FIXED, LPC, wasted bits, Rice/Rice2 with escape
// partitions, every channel assignment, variable block size headers), CRC-8
// and CRC-16 verified per frame.  Bit depths 4..32 (integer path is int64).
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <thread>
#include <vector>

#include "../../include/tomatis_flac.h"

namespace {

// ---------------------------------------------------------------------------
// CRCs
// ---------------------------------------------------------------------------
struct Crc {
  uint8_t t8[256];
  uint16_t t16[256];
  Crc() {
    for (int i = 0; i < 256; ++i) {
      uint8_t c = (uint8_t)i;
      for (int b = 0; b < 8; ++b) c = (uint8_t)((c & 0x80) ? (c << 1) ^ 0x07 : (c << 1));
      t8[i] = c;
      uint16_t d = (uint16_t)(i << 8);
      for (int b = 0; b < 8; ++b) d = (uint16_t)((d & 0x8000) ? (d << 1) ^ 0x8005 : (d << 1));
      t16[i] = d;
    }
  }
  uint8_t crc8(const uint8_t* p, size_t n) const {
    uint8_t c = 0;
    for (size_t i = 0; i < n; ++i) c = t8[c ^ p[i]];
    return c;
  }
  uint16_t crc16(const uint8_t* p, size_t n) const {
    uint16_t c = 0;
    for (size_t i = 0; i < n; ++i) c = (uint16_t)((c << 8) ^ t16[(c >> 8) ^ p[i]]);
    return c;
  }
};
const Crc& crc() {
  static const Crc c;
  return c;
}

// ---------------------------------------------------------------------------
// bit writer / reader (MSB first)
// ---------------------------------------------------------------------------
struct BitWriter {
  std::vector<uint8_t> buf;
  uint64_t acc = 0;
  int nacc = 0;
  void put(uint64_t v, int n) {  // n <= 32
    if (n == 0) return;
    v &= (n == 64) ? ~0ull : ((1ull << n) - 1);
    acc = (acc << n) | v;
    nacc += n;
    while (nacc >= 8) {
      nacc -= 8;
      buf.push_back((uint8_t)(acc >> nacc));
    }
  }
  void put_signed(int64_t v, int n) { put((uint64_t)v, n); }
  void unary(uint32_t q) {  // q zeros then a one
    while (q >= 32) {
      put(0, 32);
      q -= 32;
    }
    put(1, (int)q + 1);
  }
  void align() {
    if (nacc) put(0, 8 - nacc);
  }
  size_t bytes() const { return buf.size(); }
};

struct BitReader {
  const uint8_t* p;
  size_t len, pos = 0;  // pos in bits
  bool bad = false;
  BitReader(const uint8_t* d, size_t n) : p(d), len(n) {}
  uint64_t get(int n) {  // n <= 57
    if (n == 0) return 0;
    if (pos + n > len * 8) {
      bad = true;
      pos = len * 8;
      return 0;
    }
    uint64_t v = 0;
    size_t byte = pos >> 3;
    int off = (int)(pos & 7);
    int need = off + n;
    for (int i = 0; i < (need + 7) / 8; ++i) v = (v << 8) | p[byte + i];
    v >>= ((need + 7) / 8) * 8 - need;
    pos += n;
    return v & ((n == 64) ? ~0ull : ((1ull << n) - 1));
  }
  int64_t get_signed(int n) {
    if (n == 0) return 0;
    uint64_t v = get(n);
    if (n < 64 && (v >> (n - 1)) & 1) v |= ~0ull << n;
    return (int64_t)v;
  }
  uint32_t unary() {
    uint32_t q = 0;
    while (true) {
      if (pos >= len * 8) {
        bad = true;
        return 0;
      }
      const uint8_t b = (uint8_t)(p[pos >> 3] << (pos & 7));
      if (b) {
        const int lz = __builtin_clz((uint32_t)b) - 24;
        q += lz;
        pos += lz + 1;
        return q;
      }
      const int rem = 8 - (int)(pos & 7);
      q += rem;
      pos += rem;
    }
  }
  void align() { pos = (pos + 7) & ~(size_t)7; }
};

// ---------------------------------------------------------------------------
// encoder
// ---------------------------------------------------------------------------
constexpr int kBlock = 4096;
constexpr int kMaxPart = 8;

// zigzag (the shift in unsigned arithmetic: left-shifting a negative value is
// undefined before C++20; found by the UBSan sweep, tools/flac_sanitize.cpp)
inline uint64_t zz(int64_t r) { return ((uint64_t)r << 1) ^ (uint64_t)(r >> 63); }

void fixed_residual(const int64_t* s, int n, int order, int64_t* r) {
  for (int i = order; i < n; ++i) {
    int64_t p;
    switch (order) {
      case 0: p = 0; break;
      case 1: p = s[i - 1]; break;
      case 2: p = 2 * s[i - 1] - s[i - 2]; break;
      case 3: p = 3 * s[i - 1] - 3 * s[i - 2] + s[i - 3]; break;
      default: p = 4 * s[i - 1] - 6 * s[i - 2] + 4 * s[i - 3] - s[i - 4]; break;
    }
    r[i] = s[i] - p;
  }
}

struct RicePlan {
  int porder = 0;
  int method = 0;  // 0: 4-bit params, 1: 5-bit params
  int k[1 << kMaxPart];
  uint64_t bits = ~0ull;
};

// Rice partition order / parameters from per-partition sums of the zigzag
// residual (libFLAC-style estimate: bits(k) ~ cnt*(k+1) + (sum >> k)); sums of
// the finest partitions are computed once and merged for coarser orders.
RicePlan plan_rice(const int64_t* r, int n, int order) {
  RicePlan best;
  int pmax = 0;
  while (pmax < kMaxPart && n % (1 << (pmax + 1)) == 0 && (n >> (pmax + 1)) > order) ++pmax;
  const int np = 1 << pmax, ps = n >> pmax;
  uint64_t sum[1 << kMaxPart], mx[1 << kMaxPart];
  int cnt[1 << kMaxPart];
  for (int p = 0; p < np; ++p) {
    const int a = p == 0 ? order : p * ps, b = (p + 1) * ps;
    uint64_t sm = 0, m = 0;
    for (int i = a; i < b; ++i) {
      const uint64_t u = zz(r[i]);
      sm += u;
      m = std::max(m, u);
    }
    sum[p] = sm;
    mx[p] = m;
    cnt[p] = b - a;
  }
  for (int po = pmax; po >= 0; --po) {
    const int parts = 1 << po;
    RicePlan pl;
    pl.porder = po;
    uint64_t tot = 2 + 4;
    bool need5 = false;
    for (int p = 0; p < parts; ++p) {
      const uint64_t sm = sum[p], m = mx[p];
      const int c = cnt[p];
      int k = 0;
      if (c > 0) {
        const uint64_t mean = sm / (uint64_t)c;
        while (k < 30 && (1ull << (k + 1)) <= mean) ++k;
      }
      uint64_t bb = (uint64_t)c * (k + 1) + (sm >> k);
      if ((m >> k) >= (1ull << 24)) bb = 1ull << 60;  // absurd quotient: never chosen
      pl.k[p] = k;
      need5 |= k > 14;
      tot += bb;
    }
    pl.method = need5 ? 1 : 0;
    tot += (uint64_t)parts * (need5 ? 5 : 4);
    pl.bits = tot;
    if (tot < best.bits) best = pl;
    // merge pairs for the next coarser order
    for (int p = 0; p < parts / 2; ++p) {
      sum[p] = sum[2 * p] + sum[2 * p + 1];
      mx[p] = std::max(mx[2 * p], mx[2 * p + 1]);
      cnt[p] = cnt[2 * p] + cnt[2 * p + 1];
    }
  }
  return best;
}

void write_residual(BitWriter& w, const int64_t* r, int n, int order, const RicePlan& pl) {
  w.put(pl.method, 2);
  w.put(pl.porder, 4);
  const int ps = n >> pl.porder;
  for (int p = 0; p < (1 << pl.porder); ++p) {
    const int k = pl.k[p];
    w.put(k, pl.method ? 5 : 4);
    const int a = p == 0 ? order : p * ps, b = (p + 1) * ps;
    for (int i = a; i < b; ++i) {
      const uint64_t v = zz(r[i]);
      w.unary((uint32_t)(v >> k));
      w.put(v & ((1ull << k) - 1), k);
    }
  }
}

// cheapest subframe for one channel; bits = its size (excluding frame header)
struct SubPlan {
  int kind = 0;  // 0 constant, 1 verbatim, 2 fixed
  int order = 0;
  RicePlan rice;
  uint64_t bits = ~0ull;
};

SubPlan plan_subframe(const int64_t* s, int n, int bps, std::vector<int64_t>& res) {
  SubPlan best;
  bool constant = true;
  for (int i = 1; i < n && constant; ++i) constant = s[i] == s[0];
  if (constant) {
    best.kind = 0;
    best.bits = 8 + bps;
    return best;
  }
  best.kind = 1;
  best.bits = 8 + (uint64_t)n * bps;
  res.resize(n);
  // fixed order by the smallest sum |residual| (one pass per order), then the
  // Rice plan of that order only
  // (all five orders in one pass over successive differences, from sample 4)
  int bo = 0;
  if (n > 4) {
    uint64_t e[5] = {0, 0, 0, 0, 0};
    int64_t d1p = s[3] - s[2], d2p = d1p - (s[2] - s[1]);
    int64_t d3p = d2p - ((s[2] - s[1]) - (s[1] - s[0]));
    for (int i = 4; i < n; ++i) {
      const int64_t d0 = s[i], d1 = s[i] - s[i - 1], d2 = d1 - d1p, d3 = d2 - d2p, d4 = d3 - d3p;
      e[0] += (uint64_t)(d0 < 0 ? -d0 : d0);
      e[1] += (uint64_t)(d1 < 0 ? -d1 : d1);
      e[2] += (uint64_t)(d2 < 0 ? -d2 : d2);
      e[3] += (uint64_t)(d3 < 0 ? -d3 : d3);
      e[4] += (uint64_t)(d4 < 0 ? -d4 : d4);
      d1p = d1;
      d2p = d2;
      d3p = d3;
    }
    for (int o = 1; o < 5; ++o)
      if (e[o] < e[bo]) bo = o;
  }
  fixed_residual(s, n, bo, res.data());
  RicePlan rp = plan_rice(res.data(), n, bo);
  const uint64_t bits = 8 + (uint64_t)bo * bps + rp.bits;
  if (bits < best.bits) {
    best.kind = 2;
    best.order = bo;
    best.rice = rp;
    best.bits = bits;
  }
  return best;
}

void write_subframe(BitWriter& w, const int64_t* s, int n, int bps, const SubPlan& sp,
                    std::vector<int64_t>& res) {
  if (sp.kind == 0) {
    w.put(0, 8);
    w.put_signed(s[0], bps);
  } else if (sp.kind == 1) {
    w.put(1 << 1, 8);  // 0 000001 0
    for (int i = 0; i < n; ++i) w.put_signed(s[i], bps);
  } else {
    w.put((uint64_t)((8 | sp.order) << 1), 8);  // 0 001xxx 0
    for (int i = 0; i < sp.order; ++i) w.put_signed(s[i], bps);
    res.resize(n);
    fixed_residual(s, n, sp.order, res.data());
    write_residual(w, res.data(), n, sp.order, sp.rice);
  }
}

void put_utf8(BitWriter& w, uint64_t v) {
  if (v < 0x80) {
    w.put(v, 8);
    return;
  }
  int nb = 2;
  while (nb < 7 && v >= (1ull << (5 * nb + 1))) ++nb;
  w.put(((0xFF00u >> nb) & 0xFF) | (v >> (6 * (nb - 1))), 8);
  for (int i = nb - 2; i >= 0; --i) w.put(0x80 | ((v >> (6 * i)) & 0x3F), 8);
}

int ss_code(int bps) {
  switch (bps) {
    case 8: return 1;
    case 12: return 2;
    case 16: return 4;
    case 20: return 5;
    case 24: return 6;
    case 32: return 7;
    default: return 0;  // from STREAMINFO
  }
}

// Encode blocks [b0, b1) (frame numbers = block indices) into w; frames are
// byte-aligned, so per-thread outputs concatenate into the stream.
struct EncStats {
  uint32_t min_fs = ~0u, max_fs = 0;
  int min_bs = kBlock, max_bs = 0;
  int rc = TOMATIS_FLAC_OK;
};

// pcm holds frames [base, base + ...) of the stream (streaming encoder segments)
void encode_blocks(const int32_t* pcm, int64_t base, int64_t frames, int ch, int bps, int64_t b0,
                   int64_t b1, BitWriter& w, EncStats& st) {
  const int64_t lim = bps == 32 ? INT32_MAX : (1ll << (bps - 1)) - 1;
  std::vector<int64_t> s[8], side, mid, res;
  uint32_t& min_fs = st.min_fs;
  uint32_t& max_fs = st.max_fs;
  int& min_bs = st.min_bs;
  int& max_bs = st.max_bs;
  const Crc& C = crc();
  for (int64_t fn = b0; fn < b1; ++fn) {
    const int64_t f0 = fn * kBlock;
    const int n = (int)std::min<int64_t>(kBlock, frames - f0);
    for (int c = 0; c < ch; ++c) {
      s[c].resize(n);
      for (int i = 0; i < n; ++i) {
        const int64_t v = pcm[(f0 - base + i) * ch + c];
        if (v > lim || v < -lim - 1) {
          st.rc = TOMATIS_FLAC_E_ARG;
          return;
        }
        s[c][i] = v;
      }
    }
    // channel assignment: independent, or the best stereo decorrelation
    int assign = ch - 1;
    SubPlan plans[8];
    if (ch == 2) {
      side.resize(n);
      mid.resize(n);
      for (int i = 0; i < n; ++i) {
        side[i] = s[0][i] - s[1][i];
        mid[i] = (s[0][i] + s[1][i]) >> 1;
      }
      const SubPlan pl = plan_subframe(s[0].data(), n, bps, res);
      const SubPlan pr = plan_subframe(s[1].data(), n, bps, res);
      const SubPlan ps = plan_subframe(side.data(), n, bps + 1, res);
      const SubPlan pm = plan_subframe(mid.data(), n, bps, res);
      const uint64_t c_ind = pl.bits + pr.bits, c_ls = pl.bits + ps.bits,
                     c_sr = ps.bits + pr.bits, c_ms = pm.bits + ps.bits;
      const uint64_t m = std::min(std::min(c_ind, c_ls), std::min(c_sr, c_ms));
      if (m == c_ind) {
        assign = 1;
        plans[0] = pl;
        plans[1] = pr;
      } else if (m == c_ls) {
        assign = 8;
        plans[0] = pl;
        plans[1] = ps;
      } else if (m == c_sr) {
        assign = 9;
        plans[0] = ps;
        plans[1] = pr;
      } else {
        assign = 10;
        plans[0] = pm;
        plans[1] = ps;
      }
    } else {
      for (int c = 0; c < ch; ++c) plans[c] = plan_subframe(s[c].data(), n, bps, res);
    }
    // frame header
    const size_t h0 = w.bytes();
    w.put(0x3FFE, 14);
    w.put(0, 1);
    w.put(0, 1);  // fixed block size
    const int bs_code = n == kBlock ? 12 : 7;
    w.put(bs_code, 4);
    w.put(0, 4);  // sample rate from STREAMINFO
    w.put(assign, 4);
    w.put(ss_code(bps), 3);
    w.put(0, 1);
    put_utf8(w, (uint64_t)fn);
    if (bs_code == 7) w.put(n - 1, 16);
    w.put(C.crc8(w.buf.data() + h0, w.bytes() - h0), 8);
    for (int c = 0; c < ch; ++c) {
      const int64_t* src;
      int sbps = bps;
      if (assign == 8) {
        src = c == 0 ? s[0].data() : side.data();
        sbps += c == 1;
      } else if (assign == 9) {
        src = c == 0 ? side.data() : s[1].data();
        sbps += c == 0;
      } else if (assign == 10) {
        src = c == 0 ? mid.data() : side.data();
        sbps += c == 1;
      } else {
        src = s[c].data();
      }
      write_subframe(w, src, n, sbps, plans[c], res);
    }
    w.align();
    const uint16_t c16 = C.crc16(w.buf.data() + h0, w.bytes() - h0);
    w.put(c16, 16);
    const uint32_t fs = (uint32_t)(w.bytes() - h0);
    min_fs = std::min(min_fs, fs);
    max_fs = std::max(max_fs, fs);
    min_bs = std::min(min_bs, n);
    max_bs = std::max(max_bs, n);
    }
}

// One frame at d[p]: decoded into pcm at its own sample offset (frame number x
// nominal block size for fixed-blocksize streams, the coded sample number
// otherwise).  *consumed = frame bytes, *end = offset + block size.
int decode_frame(const uint8_t* d, size_t len, size_t p, int ch0, int bps0, int64_t nominal,
                 int32_t* pcm, int64_t max_frames, std::vector<int64_t>* sub, size_t* consumed,
                 int64_t* end, int64_t* start = nullptr) {
  const Crc& C = crc();
  BitReader r(d + p, len - p);
  if (r.get(14) != 0x3FFE) return TOMATIS_FLAC_E_FORMAT;
  if (r.get(1)) return TOMATIS_FLAC_E_FORMAT;
  const int strategy = (int)r.get(1);
  const int bsc = (int)r.get(4), src = (int)r.get(4), asg = (int)r.get(4), ssc = (int)r.get(3);
  if (r.get(1)) return TOMATIS_FLAC_E_FORMAT;
  // UTF-8 coded frame / sample number
  uint64_t num = r.get(8);
  if (num & 0x80) {
    int extra = 0;
    while (extra < 7 && (num & (0x40 >> extra))) ++extra;
    if (extra == 0) return TOMATIS_FLAC_E_FORMAT;
    num &= (0x3Fu >> extra);
    for (int i = 0; i < extra; ++i) {
      const uint64_t c = r.get(8);
      if ((c & 0xC0) != 0x80) return TOMATIS_FLAC_E_FORMAT;
      num = (num << 6) | (c & 0x3F);
    }
  }
  int n;
  if (bsc == 1) n = 192;
  else if (bsc >= 2 && bsc <= 5) n = 576 << (bsc - 2);
  else if (bsc == 6) n = (int)r.get(8) + 1;
  else if (bsc == 7) n = (int)r.get(16) + 1;
  else if (bsc >= 8) n = 256 << (bsc - 8);
  else return TOMATIS_FLAC_E_FORMAT;
  if (src == 12) r.get(8);
  else if (src == 13 || src == 14) r.get(16);
  else if (src == 15) return TOMATIS_FLAC_E_FORMAT;
  static const int ss_tab[8] = {0, 8, 12, 0, 16, 20, 24, 32};
  const int bps = ssc == 0 ? bps0 : ss_tab[ssc];
  if (bps == 0) return TOMATIS_FLAC_E_FORMAT;
  const size_t hbytes = r.pos / 8;
  const uint8_t hcrc = (uint8_t)r.get(8);
  if (r.bad || C.crc8(d + p, hbytes) != hcrc) return TOMATIS_FLAC_E_CRC;
    const int nch = asg < 8 ? asg + 1 : 2;
    if (asg > 10 || nch != ch0) return TOMATIS_FLAC_E_FORMAT;
    for (int c = 0; c < nch; ++c) {
      std::vector<int64_t>& s = sub[c];
      s.assign(n, 0);
      int sb = bps;
      if ((asg == 8 && c == 1) || (asg == 9 && c == 0) || (asg == 10 && c == 1)) ++sb;
      if (r.get(1) != 0) return TOMATIS_FLAC_E_FORMAT;
      const int type = (int)r.get(6);
      int wasted = 0;
      if (r.get(1)) wasted = (int)r.unary() + 1;
      sb -= wasted;
      if (sb <= 0) return TOMATIS_FLAC_E_FORMAT;
      int order = 0;
      if (type == 0) {
        const int64_t c0 = r.get_signed(sb);
        std::fill(s.begin(), s.end(), c0);
      } else if (type == 1) {
        for (int i = 0; i < n; ++i) s[i] = r.get_signed(sb);
      } else if ((type & 0x38) == 0x08 || (type & 0x20)) {
        const bool lpc = (type & 0x20) != 0;
        order = lpc ? (type & 0x1F) + 1 : (type & 7);
        if ((!lpc && order > 4) || order > n) return TOMATIS_FLAC_E_FORMAT;
        for (int i = 0; i < order; ++i) s[i] = r.get_signed(sb);
        int64_t coef[32] = {0};
        int shift = 0;
        if (lpc) {
          const int prec = (int)r.get(4) + 1;
          if (prec == 16) return TOMATIS_FLAC_E_FORMAT;
          shift = (int)r.get_signed(5);
          if (shift < 0) return TOMATIS_FLAC_E_FORMAT;
          for (int i = 0; i < order; ++i) coef[i] = r.get_signed(prec);
        }
        // residual
        const int method = (int)r.get(2);
        if (method > 1) return TOMATIS_FLAC_E_FORMAT;
        const int po = (int)r.get(4);
        const int ps = n >> po;
        if ((ps << po) != n || ps < order) return TOMATIS_FLAC_E_FORMAT;
        const int pbits = method ? 5 : 4, esc = method ? 31 : 15;
        int i = order;
        for (int part = 0; part < (1 << po); ++part) {
          const int k = (int)r.get(pbits);
          const int end = (part + 1) * ps;
          if (k == esc) {
            const int nb = (int)r.get(5);
            for (; i < end; ++i) s[i] = r.get_signed(nb);
          } else {
            for (; i < end; ++i) {
              const uint64_t q = r.unary();
              const uint64_t u = (q << k) | r.get(k);
              s[i] = (int64_t)(u >> 1) ^ -(int64_t)(u & 1);
            }
          }
          if (r.bad) return TOMATIS_FLAC_E_FORMAT;
        }
        // prediction, in wrapping unsigned arithmetic: a valid stream never
        // overflows (same results), a corrupt one (rejected by the CRC-16 below)
        // must not reach signed-overflow UB first (UBSan sweep,
        // tools/flac_sanitize.cpp)
        if (lpc) {
          for (int t = order; t < n; ++t) {
            uint64_t acc = 0;
            for (int j = 0; j < order; ++j) acc += (uint64_t)coef[j] * (uint64_t)s[t - 1 - j];
            s[t] = (int64_t)((uint64_t)s[t] + (uint64_t)((int64_t)acc >> shift));
          }
        } else {
          for (int t = order; t < n; ++t) {
            uint64_t pr;
            const uint64_t a1 = (uint64_t)s[t - (order > 0 ? 1 : 0)];
            switch (order) {
              case 0: pr = 0; break;
              case 1: pr = a1; break;
              case 2: pr = 2 * a1 - (uint64_t)s[t - 2]; break;
              case 3: pr = 3 * a1 - 3 * (uint64_t)s[t - 2] + (uint64_t)s[t - 3]; break;
              default:
                pr = 4 * a1 - 6 * (uint64_t)s[t - 2] + 4 * (uint64_t)s[t - 3] - (uint64_t)s[t - 4];
                break;
            }
            s[t] = (int64_t)((uint64_t)s[t] + pr);
          }
        }
      } else {
        return TOMATIS_FLAC_E_FORMAT;
      }
      if (wasted)
        for (auto& x : s) x = (int64_t)((uint64_t)x << wasted);
      if (r.bad) return TOMATIS_FLAC_E_FORMAT;
    }
    r.align();
  const size_t fbytes = r.pos / 8;
  const uint16_t fcrc = (uint16_t)r.get(16);
  if (r.bad || C.crc16(d + p, fbytes) != fcrc) return TOMATIS_FLAC_E_CRC;
  const int64_t off = strategy ? (int64_t)num : (int64_t)num * nominal;
  // decorrelate and store
  const int64_t take = std::min<int64_t>(n, std::max<int64_t>(0, max_frames - off));
  for (int64_t i = 0; i < take; ++i) {
    int64_t a = sub[0][i], b = nch > 1 ? sub[1][i] : 0;
    if (asg == 8) b = a - b;                 // left, side -> right
    else if (asg == 9) a = a + b;            // side, right -> left
    else if (asg == 10) {                    // mid, side
      const int64_t m = (int64_t)(((uint64_t)a << 1) | (uint64_t)(b & 1));
      a = (m + b) >> 1;
      b = (m - b) >> 1;
    }
    int32_t* o = pcm + (off + i) * nch;
    o[0] = (int32_t)a;
    if (nch > 1) o[1] = (int32_t)b;
    for (int c = 2; c < nch; ++c) o[c] = (int32_t)sub[c][i];
  }
  *consumed = fbytes + 2;
  *end = off + n;
  if (start) *start = off;
  return TOMATIS_FLAC_OK;
}

// true when no frame that verifies (header CRC-8 and frame CRC-16) starts in
// [p, len): the bytes there are not audio (an ID3v1 'TAG' block, padding)
bool no_frame_after(const uint8_t* d, size_t len, size_t p, int ch0, int bps0, int64_t nominal,
                    std::vector<int64_t>* sub) {
  for (; p + 1 < len; ++p) {
    if (!(d[p] == 0xFF && (d[p + 1] & 0xFE) == 0xF8)) continue;
    size_t used;
    int64_t e;
    if (decode_frame(d, len, p, ch0, bps0, nominal, nullptr, 0, sub, &used, &e) ==
        TOMATIS_FLAC_OK)
      return false;
  }
  return true;
}

// Frames whose first byte lies in [lo, hi): the first one is found by sync
// search (0xFFF8/0xFFF9 with a valid header and frame CRC), the rest follow.
// Bytes that fail to decode end the stream (no error) when the decoded end
// has reached STREAMINFO's total, or, for a stream of unknown total, when they
// do not start with a frame sync code and no verified frame follows them:
// trailing non-audio bytes (an ID3v1 tag), which libsndfile accepts.  A frame
// that starts with a sync code and fails its CRC stays an error.
void decode_range(const uint8_t* d, size_t len, size_t lo, size_t hi, bool exact_start, int ch0,
                  int bps0, int64_t nominal, int64_t total, int32_t* pcm, int64_t max_frames,
                  int* rc, int64_t* end, int64_t* begin = nullptr) {
  std::vector<int64_t> sub[8];
  size_t p = lo;
  *rc = TOMATIS_FLAC_OK;
  *end = 0;
  if (begin) *begin = INT64_MAX;
  if (!exact_start) {
    while (true) {
      while (p + 1 < hi && !(d[p] == 0xFF && (d[p + 1] & 0xFE) == 0xF8)) ++p;
      if (p + 1 >= hi) return;  // no frame starts in this range
      size_t used;
      int64_t e;
      int64_t b;
      if (decode_frame(d, len, p, ch0, bps0, nominal, pcm, max_frames, sub, &used, &e, &b) ==
          TOMATIS_FLAC_OK) {
        *end = std::max(*end, e);
        if (begin) *begin = std::min(*begin, b);
        p += used;
        break;
      }
      ++p;
    }
  }
  while (p < hi && p + 2 <= len) {
    size_t used;
    int64_t e;
    int64_t b;
    const int r = decode_frame(d, len, p, ch0, bps0, nominal, pcm, max_frames, sub, &used, &e, &b);
    if (r) {
      const bool sync = d[p] == 0xFF && (d[p + 1] & 0xFE) == 0xF8;
      if ((total > 0 && *end >= total) ||
          (total == 0 && !sync && no_frame_after(d, len, p + 1, ch0, bps0, nominal, sub)))
        return;
      *rc = r;
      return;
    }
    *end = std::max(*end, e);
    if (begin) *begin = std::min(*begin, b);
    p += used;
  }
}

// The threads' frame ranges must tile the decoded samples: every non-empty
// thread's first frame starts where the previous non-empty thread's last frame
// ended.  A thread's sync search skips a frame that starts with a sync code but
// fails its CRC; without this check that frame's samples would be a silent gap
// (left as whatever the output buffer held).
int check_contiguous(int nt, const std::vector<int64_t>& begs, const std::vector<int64_t>& ends) {
  int64_t prev_end = -1;
  for (int t = 0; t < nt; ++t) {
    if (ends[t] <= 0) continue;  // no frame starts in this thread's range
    if (prev_end >= 0 && begs[t] != prev_end) return TOMATIS_FLAC_E_CRC;
    prev_end = ends[t];
  }
  return TOMATIS_FLAC_OK;
}

}  // namespace

extern "C" {

int tomatis_flac_encode(const int32_t* pcm, int64_t frames, int32_t ch, int32_t sr, int32_t bps,
                        uint8_t** out, int64_t* out_len) {
  if (!out || !out_len || (frames > 0 && !pcm) || frames < 0 || ch < 1 || ch > 8 || sr < 1 ||
      sr > 655350 || bps < 4 || bps > 32 || frames >= (1ll << 36))
    return TOMATIS_FLAC_E_ARG;
  // blocks are independent: contiguous block ranges on host threads
  const int64_t nblk = (frames + kBlock - 1) / kBlock;
  int nt = (int)std::min<int64_t>(std::max(1u, std::thread::hardware_concurrency()), 16);
  if (const char* e = getenv("TOMATIS_FLAC_THREADS")) nt = std::max(1, atoi(e));
  nt = (int)std::max<int64_t>(1, std::min<int64_t>(nt, nblk / 8));
  std::vector<BitWriter> ws(nt);
  std::vector<EncStats> sts(nt);
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t) {
    const int64_t b0 = nblk * t / nt, b1 = nblk * (t + 1) / nt;
    if (t == nt - 1)
      encode_blocks(pcm, 0, frames, ch, bps, b0, b1, ws[t], sts[t]);
    else
      th.emplace_back(encode_blocks, pcm, (int64_t)0, frames, ch, bps, b0, b1, std::ref(ws[t]),
                      std::ref(sts[t]));
  }
  for (auto& x : th) x.join();
  EncStats tot;
  size_t body = 0;
  for (int t = 0; t < nt; ++t) {
    if (sts[t].rc) return sts[t].rc;
    tot.min_fs = std::min(tot.min_fs, sts[t].min_fs);
    tot.max_fs = std::max(tot.max_fs, sts[t].max_fs);
    tot.min_bs = std::min(tot.min_bs, sts[t].min_bs);
    tot.max_bs = std::max(tot.max_bs, sts[t].max_bs);
    body += ws[t].bytes();
  }
  uint32_t min_fs = tot.min_fs, max_fs = tot.max_fs;
  int min_bs = tot.min_bs, max_bs = tot.max_bs;
  if (frames == 0) min_fs = max_fs = 0, min_bs = max_bs = kBlock;
  // STREAMINFO (the min block size of a stream whose last block is short is
  // the nominal block size, as the format requires for fixed-blocksize streams)
  BitWriter si;
  si.put(frames > kBlock ? kBlock : (uint32_t)std::max(16, min_bs), 16);
  si.put(std::max(16, max_bs), 16);
  si.put(min_fs, 24);
  si.put(max_fs, 24);
  si.put((uint32_t)sr, 20);
  si.put(ch - 1, 3);
  si.put(bps - 1, 5);
  si.put((uint64_t)frames >> 32, 4);
  si.put((uint64_t)frames & 0xFFFFFFFFu, 32);
  for (int i = 0; i < 16; ++i) si.put(0, 8);
  const size_t hdr = 4 + 4 + 34;
  uint8_t* o = (uint8_t*)malloc(hdr + body);
  if (!o) return TOMATIS_FLAC_E_NOMEM;
  memcpy(o, "fLaC", 4);
  o[4] = 0x80;  // last metadata block, STREAMINFO, length 34
  o[5] = 0;
  o[6] = 0;
  o[7] = 34;
  memcpy(o + 8, si.buf.data(), 34);
  size_t pos = hdr;
  for (int t = 0; t < nt; ++t) {
    memcpy(o + pos, ws[t].buf.data(), ws[t].bytes());
    pos += ws[t].bytes();
  }
  *out = o;
  *out_len = (int64_t)(hdr + body);
  return TOMATIS_FLAC_OK;
}

void tomatis_flac_free(uint8_t* p) { free(p); }

int tomatis_flac_enc_finish(tomatis_flac_enc_t e, uint8_t** out, int64_t* out_len);

struct tomatis_flac_enc_s {
  int ch = 0, sr = 0, bps = 0;
  int64_t frames = 0;  // pushed so far (always a multiple of kBlock until the last push)
  bool closed = false;
  std::vector<uint8_t> body;
  EncStats tot;
};

int tomatis_flac_enc_open(int32_t ch, int32_t sr, int32_t bps, tomatis_flac_enc_t* out) {
  if (!out || ch < 1 || ch > 8 || sr < 1 || sr > 655350 || bps < 4 || bps > 32)
    return TOMATIS_FLAC_E_ARG;
  auto* e = new (std::nothrow) tomatis_flac_enc_s();
  if (!e) return TOMATIS_FLAC_E_NOMEM;
  e->ch = ch;
  e->sr = sr;
  e->bps = bps;
  *out = e;
  return TOMATIS_FLAC_OK;
}

int tomatis_flac_enc_push(tomatis_flac_enc_t e, const int32_t* pcm, int64_t frames) {
  if (!e || frames < 0 || (frames > 0 && !pcm) || e->closed) return TOMATIS_FLAC_E_ARG;
  if (frames == 0) return TOMATIS_FLAC_OK;
  if (e->frames + frames >= (1ll << 36)) return TOMATIS_FLAC_E_ARG;
  // blocks of this segment on host threads, appended in block order
  const int64_t base = e->frames, end = base + frames;
  const int64_t b0 = base / kBlock, b1 = (end + kBlock - 1) / kBlock;
  const int64_t nblk = b1 - b0;
  int nt = (int)std::min<int64_t>(std::max(1u, std::thread::hardware_concurrency()), 16);
  if (const char* ev = getenv("TOMATIS_FLAC_THREADS")) nt = std::max(1, atoi(ev));
  nt = (int)std::max<int64_t>(1, std::min<int64_t>(nt, nblk / 8));
  std::vector<BitWriter> ws(nt);
  std::vector<EncStats> sts(nt);
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t) {
    const int64_t c0 = b0 + nblk * t / nt, c1 = b0 + nblk * (t + 1) / nt;
    if (t == nt - 1)
      encode_blocks(pcm, base, end, e->ch, e->bps, c0, c1, ws[t], sts[t]);
    else
      th.emplace_back(encode_blocks, pcm, base, end, e->ch, e->bps, c0, c1, std::ref(ws[t]),
                      std::ref(sts[t]));
  }
  for (auto& x : th) x.join();
  for (int t = 0; t < nt; ++t) {
    if (sts[t].rc) return sts[t].rc;
    e->tot.min_fs = std::min(e->tot.min_fs, sts[t].min_fs);
    e->tot.max_fs = std::max(e->tot.max_fs, sts[t].max_fs);
    e->tot.min_bs = std::min(e->tot.min_bs, sts[t].min_bs);
    e->tot.max_bs = std::max(e->tot.max_bs, sts[t].max_bs);
    e->body.insert(e->body.end(), ws[t].buf.begin(), ws[t].buf.end());
  }
  e->frames = end;
  if (end % kBlock) e->closed = true;  // a short block ends the stream
  return TOMATIS_FLAC_OK;
}

// the 42-byte stream header ("fLaC" + STREAMINFO) alone, for a caller that
// wrote the frames itself (tomatis_flac_enc_take) after a 42-byte placeholder
int tomatis_flac_enc_header(tomatis_flac_enc_t e, uint8_t* hdr42) {
  if (!e || !hdr42) return TOMATIS_FLAC_E_ARG;
  std::vector<uint8_t> keep;
  keep.swap(e->body);
  uint8_t* o = nullptr;
  int64_t n = 0;
  const int rc = tomatis_flac_enc_finish(e, &o, &n);
  keep.swap(e->body);
  if (rc) return rc;
  memcpy(hdr42, o, 42);
  free(o);
  return TOMATIS_FLAC_OK;
}

int tomatis_flac_enc_finish(tomatis_flac_enc_t e, uint8_t** out, int64_t* out_len) {
  if (!e || !out || !out_len) return TOMATIS_FLAC_E_ARG;
  const int64_t frames = e->frames;
  uint32_t min_fs = e->tot.min_fs, max_fs = e->tot.max_fs;
  int min_bs = e->tot.min_bs, max_bs = e->tot.max_bs;
  if (frames == 0) min_fs = max_fs = 0, min_bs = max_bs = kBlock;
  BitWriter si;
  si.put(frames > kBlock ? kBlock : (uint32_t)std::max(16, min_bs), 16);
  si.put(std::max(16, max_bs), 16);
  si.put(min_fs, 24);
  si.put(max_fs, 24);
  si.put((uint32_t)e->sr, 20);
  si.put(e->ch - 1, 3);
  si.put(e->bps - 1, 5);
  si.put((uint64_t)frames >> 32, 4);
  si.put((uint64_t)frames & 0xFFFFFFFFu, 32);
  for (int i = 0; i < 16; ++i) si.put(0, 8);
  const size_t hdr = 4 + 4 + 34;
  uint8_t* o = (uint8_t*)malloc(hdr + e->body.size());
  if (!o) return TOMATIS_FLAC_E_NOMEM;
  memcpy(o, "fLaC", 4);
  o[4] = 0x80;
  o[5] = 0;
  o[6] = 0;
  o[7] = 34;
  memcpy(o + 8, si.buf.data(), 34);
  if (!e->body.empty()) memcpy(o + hdr, e->body.data(), e->body.size());
  *out = o;
  *out_len = (int64_t)(hdr + e->body.size());
  return TOMATIS_FLAC_OK;
}

int tomatis_flac_enc_take(tomatis_flac_enc_t e, uint8_t** out, int64_t* out_len) {
  if (!e || !out || !out_len) return TOMATIS_FLAC_E_ARG;
  *out = nullptr;
  *out_len = (int64_t)e->body.size();
  if (e->body.empty()) return TOMATIS_FLAC_OK;
  uint8_t* o = (uint8_t*)malloc(e->body.size());
  if (!o) return TOMATIS_FLAC_E_NOMEM;
  memcpy(o, e->body.data(), e->body.size());
  e->body.clear();
  *out = o;
  return TOMATIS_FLAC_OK;
}

void tomatis_flac_enc_close(tomatis_flac_enc_t e) { delete e; }

int tomatis_flac_info(const uint8_t* d, int64_t len, int32_t* sr, int32_t* ch, int32_t* bps,
                      int64_t* frames) {
  if (!d || len < 42 || memcmp(d, "fLaC", 4) != 0) return TOMATIS_FLAC_E_FORMAT;
  if ((d[4] & 0x7F) != 0) return TOMATIS_FLAC_E_FORMAT;  // first block must be STREAMINFO
  BitReader r(d + 8, 34);
  r.get(16);
  r.get(16);
  r.get(24);
  r.get(24);
  const int s = (int)r.get(20), c = (int)r.get(3) + 1, b = (int)r.get(5) + 1;
  const int64_t n = (int64_t)r.get(36);
  if (sr) *sr = s;
  if (ch) *ch = c;
  if (bps) *bps = b;
  if (frames) *frames = n;
  return TOMATIS_FLAC_OK;
}

int64_t tomatis_flac_first_frame(const uint8_t* d, int64_t len) {
  if (!d || len < 42 || memcmp(d, "fLaC", 4) != 0) return -1;
  size_t p = 4;
  while (true) {
    if (p + 4 > (size_t)len) return -1;
    const bool last = d[p] & 0x80;
    const size_t bl = ((size_t)d[p + 1] << 16) | ((size_t)d[p + 2] << 8) | d[p + 3];
    p += 4 + bl;
    if (last) break;
  }
  return (int64_t)p;
}

int tomatis_flac_decode_bytes(const uint8_t* d, int64_t len, int64_t lo, int64_t hi,
                              int32_t* pcm, int64_t max_frames, int64_t* s_lo, int64_t* s_hi) {
  int32_t sr0, ch0, bps0;
  int64_t total;
  int rc = tomatis_flac_info(d, len, &sr0, &ch0, &bps0, &total);
  if (rc) return rc;
  const int64_t first = tomatis_flac_first_frame(d, len);
  if (first < 0) return TOMATIS_FLAC_E_FORMAT;
  if (!pcm || !s_lo || !s_hi || lo < 0 || hi < lo) return TOMATIS_FLAC_E_ARG;
  lo = std::max(lo, first);
  hi = std::min(hi, len);
  *s_lo = *s_hi = 0;
  if (hi <= lo) return TOMATIS_FLAC_OK;
  const int64_t nominal = ((int64_t)d[10] << 8) | d[11];
  const size_t body = (size_t)(hi - lo);
  int nt = (int)std::min<unsigned>(std::max(1u, std::thread::hardware_concurrency()), 16);
  if (const char* e = getenv("TOMATIS_FLAC_THREADS")) nt = std::max(1, atoi(e));
  nt = (int)std::max<size_t>(1, std::min<size_t>(nt, body / (1u << 18)));
  std::vector<int> rcs(nt);
  std::vector<int64_t> ends(nt), begs(nt);
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t) {
    const size_t a = lo + body * t / nt, b = lo + body * (t + 1) / nt;
    const bool exact = t == 0 && lo == first;
    const size_t bhi = (t == nt - 1 && hi == len) ? (size_t)len : b;
    if (t == nt - 1)
      decode_range(d, (size_t)len, a, bhi, exact, ch0, bps0, nominal, total, pcm, max_frames,
                   &rcs[t], &ends[t], &begs[t]);
    else
      th.emplace_back(decode_range, d, (size_t)len, a, bhi, exact, ch0, bps0, nominal, total, pcm,
                      max_frames, &rcs[t], &ends[t], &begs[t]);
  }
  for (auto& x : th) x.join();
  int64_t b = INT64_MAX, e = 0;
  for (int t = 0; t < nt; ++t)
    if (rcs[t]) return rcs[t];
  if ((rc = check_contiguous(nt, begs, ends))) return rc;
  for (int t = 0; t < nt; ++t) {
    if (ends[t] > 0) {
      e = std::max(e, ends[t]);
      b = std::min(b, begs[t]);
    }
  }
  if (e == 0) return TOMATIS_FLAC_OK;  // no frame starts in [lo, hi)
  if (total) e = std::min(e, total);
  *s_lo = std::min(b, max_frames);
  *s_hi = std::min(e, max_frames);
  return TOMATIS_FLAC_OK;
}

int tomatis_flac_decode(const uint8_t* d, int64_t len, int32_t* pcm, int64_t max_frames,
                        int64_t* frames_out) {
  int32_t sr0, ch0, bps0;
  int64_t total;
  int rc = tomatis_flac_info(d, len, &sr0, &ch0, &bps0, &total);
  if (rc) return rc;
  if (!pcm && max_frames > 0) return TOMATIS_FLAC_E_ARG;
  const int64_t nominal = ((int64_t)d[10] << 8) | d[11];  // STREAMINFO max block size
  // skip metadata blocks
  size_t p = 4;
  while (true) {
    if (p + 4 > (size_t)len) return TOMATIS_FLAC_E_FORMAT;
    const bool last = d[p] & 0x80;
    const size_t bl = ((size_t)d[p + 1] << 16) | ((size_t)d[p + 2] << 8) | d[p + 3];
    p += 4 + bl;
    if (last) break;
  }
  // frames are independent: byte ranges on host threads (thread 0 starts at
  // the first frame, the others at the first verified frame in their range)
  const size_t body = (size_t)len > p ? (size_t)len - p : 0;
  int nt = (int)std::min<unsigned>(std::max(1u, std::thread::hardware_concurrency()), 16);
  if (const char* e = getenv("TOMATIS_FLAC_THREADS")) nt = std::max(1, atoi(e));
  nt = (int)std::max<size_t>(1, std::min<size_t>(nt, body / (1u << 20)));
  std::vector<int> rcs(nt);
  std::vector<int64_t> ends(nt), begs(nt);
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t) {
    const size_t lo = p + body * t / nt, hi = p + body * (t + 1) / nt;
    if (t == nt - 1)
      decode_range(d, (size_t)len, lo, (size_t)len, t == 0, ch0, bps0, nominal, total, pcm,
                   max_frames, &rcs[t], &ends[t], &begs[t]);
    else
      th.emplace_back(decode_range, d, (size_t)len, lo, hi, t == 0, ch0, bps0, nominal, total,
                      pcm, max_frames, &rcs[t], &ends[t], &begs[t]);
  }
  for (auto& x : th) x.join();
  int64_t done = 0;
  for (int t = 0; t < nt; ++t)
    if (rcs[t]) return rcs[t];
  if ((rc = check_contiguous(nt, begs, ends))) return rc;
  for (int t = 0; t < nt; ++t) done = std::max(done, ends[t]);
  if (total) done = std::min(done, total);
  // counting mode (pcm == NULL, max_frames == 0): the decoded length
  if (frames_out) *frames_out = pcm ? std::min(done, max_frames) : done;
  return TOMATIS_FLAC_OK;
}

}  // extern "C"
