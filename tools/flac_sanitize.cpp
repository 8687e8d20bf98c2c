// flac_sanitize.cpp -- CPU-only corruption sweep of the host FLAC codec
// (csrc/tm_flac.cpp, include/tomatis_flac.h), built with AddressSanitizer and
// UndefinedBehaviorSanitizer by tests/test_flac_sanitize.py (never on the GPU
// box).  The codec parses untrusted file bytes on every CLI ingest: it stands in
// for libsndfile behind the reference's sf.read / sf.write
// (src/process_tomatis.py:225-251).
//
// For every stream (encoded here, plus files given on the command line, which
// the test writes with its independent Python FLAC writer: LPC subframes,
// wasted bits, escape-coded and Rice2 partitions, side/mid channel modes):
//   * lossless round trip (encoded streams);
//   * bit flips in every byte of the header and metadata, in the first bytes
//     of every frame (frame header, subframe headers, residual partition
//     headers), around every multi-thread decode range boundary, and at
//     pseudo-random body positions;
//   * truncations at every frame boundary and pseudo-random lengths;
// each corrupted stream through tomatis_flac_info / _decode / _first_frame /
// _decode_bytes (whole range and the thread-split ranges).  A flip inside an
// audio frame must return an error status (CRC-8 / CRC-16 / format); a flip in
// STREAMINFO may decode (MD5 and frame-size bounds are not verified) but must
// not produce a sanitizer report.  Exit status 0 = clean.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../include/tomatis_flac.h"

namespace {

struct Rng {
  uint64_t s;
  uint32_t next() {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    return (uint32_t)(s >> 33);
  }
};

int g_fail = 0;
long g_trials = 0;

void fail(const char* what, const char* name, long pos, int rc) {
  if (g_fail < 20) fprintf(stderr, "FAIL %s: %s at %ld (rc %d)\n", what, name, pos, rc);
  ++g_fail;
}

// decode the whole stream every way the pipeline does; returns the first
// non-OK status (or OK)
int decode_all(const std::vector<uint8_t>& b, int64_t frames, int ch) {
  ++g_trials;
  int32_t sr = 0, c = 0, bps = 0;
  int64_t total = 0;
  const int64_t len = (int64_t)b.size();
  int rc = tomatis_flac_info(b.data(), len, &sr, &c, &bps, &total);
  if (rc) return rc;
  int64_t n = 0;
  rc = tomatis_flac_decode(b.data(), len, nullptr, 0, &n);  // count pass
  if (rc) return rc;
  const int64_t cap = std::max<int64_t>(frames, 1) + 65536;
  std::vector<int32_t> pcm((size_t)cap * (size_t)std::max(c, ch));
  int64_t got = 0;
  rc = tomatis_flac_decode(b.data(), len, pcm.data(), cap, &got);
  if (rc) return rc;
  const int64_t p0 = tomatis_flac_first_frame(b.data(), len);
  if (p0 < 0) return TOMATIS_FLAC_E_FORMAT;
  // the file pipeline's byte ranges: 1, 3 and 7 consecutive pieces
  for (int parts : {1, 3, 7}) {
    int64_t prev = 0;
    for (int t = 0; t < parts; ++t) {
      const int64_t lo = p0 + (len - p0) * t / parts, hi = p0 + (len - p0) * (t + 1) / parts;
      int64_t s_lo = 0, s_hi = 0;
      rc = tomatis_flac_decode_bytes(b.data(), len, lo, hi, pcm.data(), cap, &s_lo, &s_hi);
      if (rc) return rc;
      if (s_lo != prev && s_hi > s_lo) return TOMATIS_FLAC_E_FORMAT;  // ranges must tile
      if (s_hi > s_lo) prev = s_hi;
    }
  }
  return TOMATIS_FLAC_OK;
}

// candidate frame starts: 14-bit sync 0b11111111111110 + reserved 0
std::vector<int64_t> frame_starts(const std::vector<uint8_t>& b, int64_t p0) {
  std::vector<int64_t> v;
  for (int64_t i = p0; i + 1 < (int64_t)b.size(); ++i)
    if (b[i] == 0xFF && (b[i + 1] & 0xFE) == 0xF8) v.push_back(i);
  return v;
}

void sweep(const char* name, const std::vector<uint8_t>& blob, int64_t frames, int ch,
           int max_frame_flips, int body_flips, int max_nt, int truncs) {
  if (decode_all(blob, frames, ch) != TOMATIS_FLAC_OK) {
    fail("clean stream does not decode", name, -1, -9);
    return;
  }
  const int64_t len = (int64_t)blob.size();
  const int64_t p0 = tomatis_flac_first_frame(blob.data(), len);
  std::vector<uint8_t> b = blob;
  auto flip = [&](int64_t pos, uint8_t mask, bool must_fail) {
    if (pos < 0 || pos >= len) return;
    b[pos] ^= mask;
    const int rc = decode_all(b, frames, ch);
    if (must_fail && rc == TOMATIS_FLAC_OK) fail("undetected flip", name, (long)pos, rc);
    b[pos] ^= mask;
  };
  // header + metadata: every byte, three masks (may decode: MD5, size bounds)
  for (int64_t i = 0; i < p0 + 4 && i < len; ++i)
    for (uint8_t m : {(uint8_t)0x01, (uint8_t)0x80, (uint8_t)0xFF}) flip(i, m, false);
  // every frame's first 24 bytes: frame header, subframe / partition headers
  const std::vector<int64_t> fs = frame_starts(blob, p0);
  int nf = 0;
  for (int64_t f : fs) {
    if (nf++ >= max_frame_flips) break;
    for (int64_t i = f; i < f + 24 && i < len; ++i) flip(i, 0x10, i >= p0);
  }
  // multi-thread decode boundaries (body split into nt pieces, 2..16 threads)
  const int64_t body = len - p0;
  for (int nt = 2; nt <= max_nt; nt *= 2)
    for (int t = 1; t < nt; ++t) {
      const int64_t c = p0 + body * t / nt;
      for (int64_t i = c - 48; i < c + 48; i += 3) flip(i, 0x04, i >= p0);
    }
  // pseudo-random body positions
  Rng r{(uint64_t)len * 2654435761ull + 17};
  for (int k = 0; k < body_flips && body > 0; ++k) {
    const int64_t i = p0 + (int64_t)(r.next() % (uint64_t)body);
    flip(i, (uint8_t)(1u << (r.next() & 7)), true);
  }
  // truncations: at / around frame starts and pseudo-random lengths (the last
  // frame cut short must be an error; a cut exactly at a frame start may decode)
  for (size_t k = 0; k < fs.size() && (int)k < truncs; ++k)
    for (int64_t d : {-1, 0, 1, 7}) {
      const int64_t cut = fs[k] + d;
      if (cut <= 0 || cut >= len) continue;
      std::vector<uint8_t> tb(blob.begin(), blob.begin() + cut);
      (void)decode_all(tb, frames, ch);
    }
  for (int k = 0; k < truncs; ++k) {
    const int64_t cut = (int64_t)(r.next() % (uint64_t)len);
    std::vector<uint8_t> tb(blob.begin(), blob.begin() + cut);
    (void)decode_all(tb, frames, ch);
  }
}

std::vector<int32_t> make_pcm(int64_t n, int ch, int bps, uint64_t seed) {
  std::vector<int32_t> x((size_t)(n * ch));
  Rng r{seed};
  const int64_t top = (bps == 32) ? 0x7FFFFFFFll : ((1ll << (bps - 1)) - 1);
  for (int64_t i = 0; i < n; ++i)
    for (int c = 0; c < ch; ++c) {
      // a slow sine plus noise: smooth enough for FIXED predictors, noisy
      // enough for large Rice parameters; a constant stretch and full scale
      double v = 0.5 * __builtin_sin(0.001 * (double)i * (c + 1)) +
                 0.01 * ((double)(r.next() & 0xFFFF) / 65536.0 - 0.5);
      if ((i / 9000) % 7 == 3) v = 0.25;
      if (i % 50000 == 7) v = (c & 1) ? -1.0 : 1.0;
      int64_t q = (int64_t)(v * (double)top);
      if (q > top) q = top;
      if (q < -top - 1) q = -top - 1;
      x[(size_t)(i * ch + c)] = (int32_t)q;
    }
  return x;
}

bool encode_checked(const char* name, int64_t n, int ch, int sr, int bps, uint64_t seed,
                    std::vector<uint8_t>& blob) {
  const std::vector<int32_t> x = make_pcm(n, ch, bps, seed);
  uint8_t* out = nullptr;
  int64_t out_len = 0;
  int rc = tomatis_flac_encode(x.data(), n, ch, sr, bps, &out, &out_len);
  if (rc) {
    fail("encode", name, -1, rc);
    return false;
  }
  blob.assign(out, out + out_len);
  tomatis_flac_free(out);
  // streaming encoder: byte-identical
  tomatis_flac_enc_t e = nullptr;
  rc = tomatis_flac_enc_open(ch, sr, bps, &e);
  if (rc) {
    fail("enc_open", name, -1, rc);
    return false;
  }
  const int64_t seg = 4096 * 37;
  for (int64_t a = 0; a < n && !rc; a += seg)
    rc = tomatis_flac_enc_push(e, x.data() + a * ch, std::min<int64_t>(seg, n - a));
  uint8_t* o2 = nullptr;
  int64_t l2 = 0;
  if (!rc) rc = tomatis_flac_enc_finish(e, &o2, &l2);
  tomatis_flac_enc_close(e);
  if (rc || l2 != out_len || memcmp(o2, blob.data(), (size_t)l2) != 0)
    fail("streaming encoder differs", name, -1, rc);
  tomatis_flac_free(o2);
  // lossless
  std::vector<int32_t> y((size_t)(n * ch) + 1);
  int64_t got = 0;
  rc = tomatis_flac_decode(blob.data(), (int64_t)blob.size(), y.data(), n, &got);
  if (rc || got != n || memcmp(y.data(), x.data(), (size_t)n * ch * 4) != 0) {
    fail("round trip", name, -1, rc);
    return false;
  }
  return true;
}

std::vector<uint8_t> read_file(const char* path) {
  std::vector<uint8_t> v;
  FILE* f = fopen(path, "rb");
  if (!f) return v;
  uint8_t buf[1 << 16];
  size_t k;
  while ((k = fread(buf, 1, sizeof buf, f)) > 0) v.insert(v.end(), buf, buf + k);
  fclose(f);
  return v;
}

}  // namespace

int main(int argc, char** argv) {
  struct Cfg {
    const char* name;
    int64_t n;
    int ch, sr, bps, frame_flips, body_flips, max_nt, truncs;
  };
  // the first stream is long enough for a 4-way threaded decode (>= 4 MiB of
  // frames); the rest are swept densely
  const Cfg cfgs[] = {
      {"st24_threaded", 1200000, 2, 48000, 24, 8, 100, 4, 12},
      {"mono16", 70000, 1, 44100, 16, 100000, 2000, 16, 64},
      {"six20", 30000, 6, 96000, 20, 100000, 1000, 16, 64},
      {"st8_short", 5000, 2, 8000, 8, 100000, 1000, 16, 64},
      {"st32", 20000, 2, 192000, 32, 100000, 1000, 16, 64},
      {"one_frame", 4096, 2, 44100, 16, 100000, 500, 16, 64},
      {"tiny", 17, 1, 44100, 12, 100000, 200, 16, 64},
  };
  for (const Cfg& c : cfgs) {
    std::vector<uint8_t> blob;
    if (!encode_checked(c.name, c.n, c.ch, c.sr, c.bps, 0x9E3779B9ull + (uint64_t)c.n, blob))
      continue;
    sweep(c.name, blob, c.n, c.ch, c.frame_flips, c.body_flips, c.max_nt, c.truncs);
    fprintf(stderr, "%s: %zu bytes swept\n", c.name, blob.size());
  }
  // streams from the independent Python writer (argv: path frames ch ...)
  for (int i = 1; i + 2 < argc; i += 3) {
    const std::vector<uint8_t> blob = read_file(argv[i]);
    if (blob.empty()) {
      fail("read", argv[i], -1, -8);
      continue;
    }
    sweep(argv[i], blob, atoll(argv[i + 1]), atoi(argv[i + 2]), 100000, 1000, 16, 64);
    fprintf(stderr, "%s: %zu bytes swept\n", argv[i], blob.size());
  }
  fprintf(stderr, "trials %ld, failures %d\n", g_trials, g_fail);
  return g_fail ? 1 : 0;
}
