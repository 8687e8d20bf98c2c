// tm_analysis.hip — analysis spectra on the device.
//
// The reference's validators and calibration tools run the same framing + real
// FFT as the processors, then reduce over frames:
//   compare_audio.stft_mag_avg                 src/compare_audio.py:12-24
//       mean over frames of |rfft(win * x)|    -> k_an_spec<MAG>, k_an_frame_mean
//   layer2_analyze_eq.stft_logpower_median     src/layer2_analyze_eq.py:54-88
//       frames with rms_dbfs(power_mono) > music_dbfs, median over frames of
//       10 log10(|rfft(win * power_mono)|^2 + EPS)
//                                              -> k_an_frame_r, k_an_select,
//                                                 k_an_spec<LOGPOW>, median kernels
//   validate_layer1.compute_conditional_spectrum  src/validate_layer1.py:261-389
//       stable C1/C2 frames with level >= threshold, median over frames of
//       mean_c|Y_c| / max(mean_c|X_c|, 1e-10)  -> k_an_frame_r, k_an_select,
//                                                 k_an_spec<RATIO>, median kernels
//
// Frames: f = 0 .. F-1 start at f*hop, F = 1 + (n - n_fft) / hop (every frame
// lies inside the signal, as in all three reference loops).
//
// Layout and kernels (HBM-bound streaming work, no MFMA):
//  * k_an_spec: one 256-thread workgroup per frame PAIR (MAG/LOGPOW: the two
//    real frames are packed as a + ib into one complex FFT and split with
//    Z[k] +- conj(Z[n-k])) or per frame (RATIO: x_c + i y_c per channel, so one
//    complex FFT yields X_c and Y_c).  Frame staged in LDS (coalesced loads of
//    the hop-strided PCM), Stockham autosort FFT in LDS (one radix-2 stage when
//    log2 n is odd, then radix-4 stages; every stage reads its butterflies into
//    registers, barrier, writes, barrier), twiddles from a float table built in
//    double precision once per size.  Any n_fft >= 16 (as np.fft.rfft): powers
//    of two up to 16384 directly, other lengths up to 8192 by Bluestein's
//    chirp-z over M = 2^k >= 2n - 1 in the same LDS buffer (tlds::lds_dft,
//    tables per n from tm_host_dsp.h).  Output rows [F][n/2+1] f32.
//  * k_an_frame_r: numpy's pairwise mean of m^2 per frame, restated exactly
//    (128-sample leaves of 8 sequential chains, fixed 8-chain tree, perfect tree
//    over leaves; correctly rounded sqrtf, -ffp-contract=off) so level gating is
//    decided on the bit pattern of r, like the processors' gate.  Other frame
//    lengths take k_an_frame_r_pw: numpy's tree for that length (leaves +
//    postfix program, NPY_BUFSIZE chunks) built on the host.
//  * median: per-bin radix select over the frame axis on order-preserving u32
//    keys, 8-bit digits, 4 passes (+1 min pass for even counts); each pass is a
//    grid of (64-bin group x frame split) workgroups building LDS histograms
//    (digit-major, lane = bin: conflict-free) flushed with global atomics, then
//    a per-bin pick.  numpy's even-count rule: fl32(fl32(v_lo + v_hi) / 2).
//  * k_an_frame_mean: per-bin sequential float32 sum over frames then / F —
//    numpy's axis-0 reduction order of np.stack(rows).mean(axis=0).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <type_traits>
#include <vector>

#include "../../include/tomatis_hip.h"
#include "tm_host_dsp.h"
#include "tm_lds_fft.h"

namespace {

constexpr int kT = 256;                // threads per spectrum workgroup
constexpr int kMaxTreeN = 8192;        // k_an_frame_r: powers of two in [256, 8192]
constexpr int kMaxM = 16384;           // largest FFT in LDS (128 KiB of float2)
constexpr int kMinN = 16;              // smallest spectrum n_fft
constexpr int kPwMax = 256;            // k_an_frame_r_pw leaves (n_fft <= 16384)
constexpr float kEps = 1e-12f;

int an_fail(hipError_t e) { return e == hipSuccess ? TOMATIS_OK : TOMATIS_E_HIP; }
int an_launch() { return an_fail(hipGetLastError()); }

bool is_pow2(int n) { return n > 0 && (n & (n - 1)) == 0; }

// FFT size in LDS for a length-n DFT (0: unsupported)
int dft_m(int n) {
  if (n < kMinN) return 0;
  const int M = is_pow2(n) ? n : thost::bluestein_m(n);
  return M <= kMaxM ? M : 0;
}

// ---------------------------------------------------------------------------
// twiddle table tw[t] = exp(-2 pi i t / n), computed in double, cached per n
// ---------------------------------------------------------------------------
__global__ void k_an_twiddle(float2* tw, int n) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  double s, c;
  sincospi(-2.0 * (double)t / (double)n, &s, &c);
  tw[t] = make_float2((float)c, (float)s);
}

std::mutex g_tw_mu;
std::map<std::pair<int, int>, float2*> g_tw;  // (device, n) -> table (process lifetime)

template <typename T>
int upload(const std::vector<T>& v, T** out) {
  T* p = nullptr;
  if (hipMalloc(&p, sizeof(T) * v.size()) != hipSuccess) return TOMATIS_E_NOMEM;
  if (hipMemcpy(p, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipFree(p);
    return TOMATIS_E_HIP;
  }
  *out = p;
  return TOMATIS_OK;
}

struct Chirp {  // Bluestein tables for one n (tm_host_dsp.h bluestein_tables)
  float2* b = nullptr;
  float2* h = nullptr;
};
std::map<std::pair<int, int>, Chirp> g_chirp;  // (device, n), process lifetime

int chirp_tables(int n, int M, Chirp* out) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return TOMATIS_E_HIP;
  std::lock_guard<std::mutex> lk(g_tw_mu);
  auto it = g_chirp.find({dev, n});
  if (it != g_chirp.end()) {
    *out = it->second;
    return TOMATIS_OK;
  }
  std::vector<float2> bf, hf;
  thost::bluestein_tables(n, M, bf, hf);
  Chirp c;
  int rc = upload(bf, &c.b);
  if (rc == TOMATIS_OK && (rc = upload(hf, &c.h)) != TOMATIS_OK) (void)hipFree(c.b);
  if (rc != TOMATIS_OK) return rc;
  g_chirp[{dev, n}] = c;
  *out = c;
  return TOMATIS_OK;
}

struct PwProg {  // numpy's pairwise tree over one frame length
  int2* leaf = nullptr;
  int16_t* prog = nullptr;
  int n_leaf = 0, n_prog = 0;
};
std::map<std::pair<int, int>, PwProg> g_pw;  // (device, n), process lifetime

int pw_program(int n, PwProg* out) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return TOMATIS_E_HIP;
  std::lock_guard<std::mutex> lk(g_tw_mu);
  auto it = g_pw.find({dev, n});
  if (it != g_pw.end()) {
    *out = it->second;
    return TOMATIS_OK;
  }
  std::vector<int2> lv;
  std::vector<int16_t> prog;
  thost::pw_program(n, lv, prog);
  if ((int)lv.size() > kPwMax) return TOMATIS_E_UNSUPPORTED;
  PwProg q;
  q.n_leaf = (int)lv.size();
  q.n_prog = (int)prog.size();
  int rc = upload(lv, &q.leaf);
  if (rc == TOMATIS_OK && (rc = upload(prog, &q.prog)) != TOMATIS_OK) (void)hipFree(q.leaf);
  if (rc != TOMATIS_OK) return rc;
  g_pw[{dev, n}] = q;
  *out = q;
  return TOMATIS_OK;
}

int twiddles(int n, hipStream_t s, const float2** out) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return TOMATIS_E_HIP;
  std::lock_guard<std::mutex> lk(g_tw_mu);
  auto it = g_tw.find({dev, n});
  if (it != g_tw.end()) {
    *out = it->second;
    return TOMATIS_OK;
  }
  float2* p = nullptr;
  if (hipMalloc(&p, sizeof(float2) * n) != hipSuccess) return TOMATIS_E_NOMEM;
  hipLaunchKernelGGL(k_an_twiddle, dim3((n + 255) / 256), dim3(256), 0, s, p, n);
  int rc = an_launch();
  if (rc == TOMATIS_OK) rc = an_fail(hipStreamSynchronize(s));  // visible to every stream
  if (rc != TOMATIS_OK) {
    (void)hipFree(p);
    return rc;
  }
  g_tw[{dev, n}] = p;
  *out = p;
  return TOMATIS_OK;
}

// ---------------------------------------------------------------------------
// per-sample mono values
// ---------------------------------------------------------------------------
// validate_layer1.py:304-306 / process_tomatis.py:369-371:
//   mono = sqrt(mean(frame**2, axis=1)); rms uses mono*mono
template <int CH>
__device__ __forceinline__ float m2_chmean(const float* __restrict__ x, int64_t p, float sc) {
  float acc = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const float v = x[p * CH + c] * sc;
    acc = acc + v * v;
  }
  const float mean = (CH == 1) ? acc : acc * 0.5f;
  const float m = sqrtf(mean);
  return m * m;
}
// compare_audio.py:7-10 / layer2_analyze_eq.py:71:
//   power_mono = sqrt(0.5 * (L**2 + R**2) + EPS)
__device__ __forceinline__ float power_mono(const float* __restrict__ x, int64_t p, float sc) {
  const float2 u = reinterpret_cast<const float2*>(x)[p];
  const float l = u.x * sc, r = u.y * sc;
  const float s = l * l + r * r;
  return sqrtf(0.5f * s + kEps);
}

// ---------------------------------------------------------------------------
// per-frame r (numpy pairwise mean, restated exactly)
// ---------------------------------------------------------------------------
template <int MODE, int CH>  // MODE: TOMATIS_AN_LEVEL_CHMEAN / _POWER_MONO
__global__ __launch_bounds__(256) void k_an_frame_r(const float* __restrict__ x, int n_fft,
                                                    int hop, int n_frames, float sc,
                                                    float* __restrict__ r_out) {
  __shared__ float lv[4][kMaxTreeN / 128];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int f = blockIdx.x * 4 + w;
  const bool live = f < n_frames;  // wave-uniform
  const int64_t p0 = (int64_t)f * hop;
  const int nl = n_fft >> 7;
  const int b = lane >> 3, c = lane & 7;
  for (int g = 0; g < nl; g += 8) {
    const int L = g + b;
    float acc = 0.f;
    if (live && L < nl) {
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const int64_t p = p0 + 128 * L + c + 8 * t;
        float m2;
        if constexpr (MODE == TOMATIS_AN_LEVEL_POWER_MONO) {
          const float m = power_mono(x, p, sc);
          m2 = m * m;
        } else {
          m2 = m2_chmean<CH>(x, p, sc);
        }
        acc = (t == 0) ? m2 : acc + m2;
      }
    }
    // numpy's 8-chain tree ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)); IEEE add commutes
    acc = acc + __shfl_xor(acc, 1, 64);
    acc = acc + __shfl_xor(acc, 2, 64);
    acc = acc + __shfl_xor(acc, 4, 64);
    if (c == 0 && L < nl) lv[w][L] = acc;
  }
  __syncthreads();
  if (live && lane == 0) {
    float* t = lv[w];
    for (int width = nl; width > 1; width >>= 1)
      for (int i = 0; i < width / 2; ++i) t[i] = t[2 * i] + t[2 * i + 1];
    r_out[f] = sqrtf(t[0] / (float)n_fft + kEps);
  }
}

// any frame length: numpy's pairwise tree from the host program (leaf >= 0
// pushes that leaf's sum, -1 adds the top two); leaves follow numpy's block rule
// (sequential below 8, else 8 accumulators + fixed tree + sequential remainder)
template <int MODE, int CH>
__device__ __forceinline__ float m2_at(const float* __restrict__ x, int64_t p, float sc) {
  if constexpr (MODE == TOMATIS_AN_LEVEL_POWER_MONO) {
    const float m = power_mono(x, p, sc);
    return m * m;
  } else {
    return m2_chmean<CH>(x, p, sc);
  }
}

template <int MODE, int CH>
__global__ __launch_bounds__(256) void k_an_frame_r_pw(const float* __restrict__ x, int n_fft,
                                                       int hop, float sc,
                                                       const int2* __restrict__ leaf, int n_leaf,
                                                       const int16_t* __restrict__ prog,
                                                       int n_prog, float* __restrict__ r_out) {
  __shared__ float ls[kPwMax];
  const int f = blockIdx.x;
  const int64_t p0 = (int64_t)f * hop;
  for (int l = threadIdx.x; l < n_leaf; l += blockDim.x) {
    const int2 lf = leaf[l];
    const int64_t q = p0 + lf.x;
    const int len = lf.y;
    float res;
    if (len < 8) {
      res = 0.f;
      for (int i = 0; i < len; ++i) res = res + m2_at<MODE, CH>(x, q + i, sc);
    } else {
      float r[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] = m2_at<MODE, CH>(x, q + j, sc);
      int i = 8;
      for (; i < len - (len % 8); i += 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] = r[j] + m2_at<MODE, CH>(x, q + i + j, sc);
      }
      res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
      for (; i < len; ++i) res = res + m2_at<MODE, CH>(x, q + i, sc);
    }
    ls[l] = res;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float stk[32];
    int sp = 0;
    for (int i = 0; i < n_prog; ++i) {
      const int op = prog[i];
      if (op >= 0) {
        stk[sp++] = ls[op];
      } else {
        const float b = stk[--sp];
        stk[sp - 1] = stk[sp - 1] + b;
      }
    }
    r_out[f] = sqrtf(stk[0] / (float)n_fft + kEps);
  }
}

// ---------------------------------------------------------------------------
// frame selection on r bit patterns (exact level predicates, dsp.gate_bits)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_an_select(const float* __restrict__ r, int n_frames,
                                                   uint32_t thr, uint4 exc, int n_exc,
                                                   int keep_above, const int8_t* __restrict__ cls,
                                                   int cls_want, uint8_t* __restrict__ mask,
                                                   int32_t* __restrict__ count) {
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  bool keep = false;
  if (f < n_frames) {
    const float rv = r[f];
    const uint32_t b = __float_as_uint(rv);
    const uint32_t e[4] = {exc.x, exc.y, exc.z, exc.w};
    bool hit = false;
    for (int i = 0; i < n_exc; ++i) hit |= (b == e[i]);
    if (rv == rv) {
      // keep_above: level >= T  <=> (b >= thr) xor exc     (gate "on" form)
      // else:       level >  T  <=> !((b <= thr) xor exc)  (not the "off" form)
      keep = keep_above ? ((b >= thr) != hit) : !((b <= thr) != hit);
    }
    if (cls) keep = keep && (cls[f] == cls_want);
    mask[f] = keep ? 1 : 0;
  }
  const unsigned long long bal = __ballot(keep);
  if ((threadIdx.x & 63) == 0 && bal) atomicAdd(count, (int32_t)__popcll(bal));
}

using tlds::cadd;
using tlds::cmul;
using tlds::csub;
using tlds::lds_dft;

// ---------------------------------------------------------------------------
// spectra
// ---------------------------------------------------------------------------
struct SpecArgs {
  const float* x;
  const float* y;
  const float* win;
  const float2* tw;  // exp(-2 pi i t / M)
  const float2* bb;  // Bluestein chirp b (n_fft), BLUE kernels only
  const float2* bh;  // Bluestein kernel spectrum H (M)
  float* out;
  int n_fft, M, hop, n_frames, n_bins;
  float sc;
  int band[4];  // TOMATIS_AN_BAND: bins [band0, band1) and [band2, band3)
};

template <int SIG>  // TOMATIS_AN_SIG_RAW (ch 1) / TOMATIS_AN_SIG_POWER_MONO (ch 2)
__device__ __forceinline__ float sig_at(const float* __restrict__ x, int64_t p, float sc) {
  if constexpr (SIG == TOMATIS_AN_SIG_POWER_MONO) return power_mono(x, p, sc);
  else return x[p] * sc;
}

// DFT bin mirrored for the two-real-frames split: (n - k) mod n
__device__ __forceinline__ int mirror(int k, int n) { return k == 0 ? 0 : n - k; }

// MAG / LOGPOW: workgroup per frame pair (2g, 2g+1) packed as a + ib
template <int KIND, int SIG, int M, bool BLUE>
__global__ __launch_bounds__(kT) void k_an_spec_pair(SpecArgs A) {
  __shared__ float2 buf[M];
  const int f0 = blockIdx.x * 2, f1 = f0 + 1;
  const bool has1 = f1 < A.n_frames;
  const int n = BLUE ? A.n_fft : M;  // constant for powers of two
  const int64_t p0 = (int64_t)f0 * A.hop, p1 = (int64_t)f1 * A.hop;
  for (int i = threadIdx.x; i < n; i += kT) {
    const float w = A.win[i];
    const float a = sig_at<SIG>(A.x, p0 + i, A.sc) * w;
    const float b = has1 ? sig_at<SIG>(A.x, p1 + i, A.sc) * w : 0.f;
    buf[i] = make_float2(a, b);
  }
  __syncthreads();
  lds_dft<M, BLUE>(buf, n, A.tw, A.bb, A.bh);
  float* o0 = A.out + (int64_t)f0 * A.n_bins;
  float* o1 = A.out + (int64_t)f1 * A.n_bins;
  for (int k = threadIdx.x; k < A.n_bins; k += kT) {
    const float2 zk = buf[k], zm = buf[mirror(k, n)];
    // A = (Z[k] + conj Z[n-k]) / 2, B = (Z[k] - conj Z[n-k]) / 2i
    const float2 fa = make_float2(0.5f * (zk.x + zm.x), 0.5f * (zk.y - zm.y));
    const float2 fb = make_float2(0.5f * (zk.y + zm.y), -0.5f * (zk.x - zm.x));
    if constexpr (KIND == TOMATIS_AN_MAG) {
      o0[k] = hypotf(fa.x, fa.y);
      if (has1) o1[k] = hypotf(fb.x, fb.y);
    } else {  // 10 log10(re^2 + im^2 + EPS), float32 (layer2_analyze_eq.py:78-79)
      const float pa = fa.x * fa.x + fa.y * fa.y;
      o0[k] = 10.0f * log10f(pa + kEps);
      if (has1) {
        const float pb = fb.x * fb.x + fb.y * fb.y;
        o1[k] = 10.0f * log10f(pb + kEps);
      }
    }
  }
}

// BAND (stft_band_tilt, calibrate_to_baseline_v2.py:17-31): per frame of the
// pair the float32 power re^2 + im^2 of rfft(win * power_mono) summed over two
// bin ranges; workgroup per frame pair as k_an_spec_pair, block reduction.
template <int M, bool BLUE>
__global__ __launch_bounds__(kT) void k_an_band_pair(SpecArgs A) {
  __shared__ float2 buf[M];
  const int N = BLUE ? A.n_fft : M;
  __shared__ float red[kT / 64][4];
  const int f0 = blockIdx.x * 2, f1 = f0 + 1;
  const bool has1 = f1 < A.n_frames;
  const int64_t p0 = (int64_t)f0 * A.hop, p1 = (int64_t)f1 * A.hop;
  for (int i = threadIdx.x; i < N; i += kT) {
    const float w = A.win[i];
    const float a = power_mono(A.x, p0 + i, A.sc) * w;
    const float b = has1 ? power_mono(A.x, p1 + i, A.sc) * w : 0.f;
    buf[i] = make_float2(a, b);
  }
  __syncthreads();
  lds_dft<M, BLUE>(buf, N, A.tw, A.bb, A.bh);
  float acc[4] = {0.f, 0.f, 0.f, 0.f};  // (frame a, band lo), (a, hi), (b, lo), (b, hi)
  for (int k = threadIdx.x; k < A.n_bins; k += kT) {
    const bool lo = k >= A.band[0] && k < A.band[1], hi = k >= A.band[2] && k < A.band[3];
    if (!lo && !hi) continue;
    const float2 zk = buf[k], zm = buf[mirror(k, N)];
    const float2 fa = make_float2(0.5f * (zk.x + zm.x), 0.5f * (zk.y - zm.y));
    const float2 fb = make_float2(0.5f * (zk.y + zm.y), -0.5f * (zk.x - zm.x));
    const float pa = fa.x * fa.x + fa.y * fa.y, pb = fb.x * fb.x + fb.y * fb.y;
    acc[hi ? 1 : 0] += pa;
    acc[hi ? 3 : 2] += pb;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float v = acc[j];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if (lane == 0) red[w][j] = v;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    float v = 0.f;
    for (int i = 0; i < kT / 64; ++i) v += red[i][threadIdx.x];
    const int j = threadIdx.x;
    if (j < 2) A.out[(int64_t)f0 * 2 + j] = v;
    else if (has1) A.out[(int64_t)f1 * 2 + (j - 2)] = v;
  }
}

// Gate-calibration grid (calibrate_to_baseline_v2.py:84-109 simulate_state,
// :241-265 the search): one lane per candidate runs the standard automaton
// (hysteresis + up-delay on frame starts) over the fitted frames and counts
// mismatches against the target states and state switches.  Levels are
// float32 and compared with the float32 thresholds exactly as numpy compares
// an np.float32 level with a Python float (NEP 50: in float32).
__global__ __launch_bounds__(256) void k_cal_gate_grid(const float* __restrict__ levels,
                                                       int n_fit,
                                                       const int64_t* __restrict__ starts,
                                                       const int32_t* __restrict__ target,
                                                       const TomatisGateCand* __restrict__ cands,
                                                       int n_cand, int32_t* __restrict__ out,
                                                       uint8_t* __restrict__ states) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n_cand) return;  // no barriers below
  const TomatisGateCand C = cands[c];
  const float* lv = levels + (int64_t)C.level_row * n_fit;
  int state = 1, prev = 1, mism = 0, sw = 0;
  bool pend = false;
  int64_t pending = 0;
  for (int i = 0; i < n_fit; ++i) {
    const float l = lv[i];
    const int64_t st = starts[i];
    if (state == 1) {
      if (l >= C.t_on) {
        if (!pend) {
          pend = true;
          pending = st + C.up_delay;
        }
      } else {
        pend = false;
      }
      if (pend && st >= pending) {
        state = 2;
        pend = false;
      }
    } else if (l <= C.t_off) {
      state = 1;
      pend = false;
    }
    if (states) states[(int64_t)c * n_fit + i] = (uint8_t)state;
    if (target) mism += state != target[i];
    sw += (i > 0) & (state != prev);
    prev = state;
  }
  out[2 * c] = mism;
  out[2 * c + 1] = sw;
}

// RATIO: workgroup per frame; per channel one FFT of x_c + i y_c
template <int CH, int M, bool BLUE>
__global__ __launch_bounds__(kT) void k_an_spec_ratio(SpecArgs A) {
  __shared__ float2 buf[M];
  constexpr int kMaxUB = (M / 2 + 1 + kT - 1) / kT;  // bins per thread (n/2+1 <= M/2+1)
  const int f = blockIdx.x;
  const int n = BLUE ? A.n_fft : M;  // constant for powers of two
  const int64_t p0 = (int64_t)f * A.hop;
  float ax[kMaxUB], ay[kMaxUB];
#pragma unroll
  for (int u = 0; u < kMaxUB; ++u) ax[u] = ay[u] = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    for (int i = threadIdx.x; i < n; i += kT) {
      const float w = A.win[i];
      const int64_t q = (p0 + i) * CH + c;
      buf[i] = make_float2(A.x[q] * w, A.y[q] * w);
    }
    __syncthreads();
    lds_dft<M, BLUE>(buf, n, A.tw, A.bb, A.bh);
#pragma unroll
    for (int u = 0; u < kMaxUB; ++u) {
      const int k = threadIdx.x + u * kT;
      if (k < A.n_bins) {
        const float2 zk = buf[k], zm = buf[mirror(k, n)];
        const float xr = 0.5f * (zk.x + zm.x), xi = 0.5f * (zk.y - zm.y);
        const float yr = 0.5f * (zk.y + zm.y), yi = -0.5f * (zk.x - zm.x);
        ax[u] = ax[u] + hypotf(xr, xi);  // X += |rfft(x_c * win)|
        ay[u] = ay[u] + hypotf(yr, yi);
      }
    }
    __syncthreads();  // buf reused by the next channel
  }
  float* o = A.out + (int64_t)f * A.n_bins;
#pragma unroll
  for (int u = 0; u < kMaxUB; ++u) {
    const int k = threadIdx.x + u * kT;
    if (k < A.n_bins) {
      float X = (CH == 1) ? ax[u] : ax[u] * 0.5f;  // X /= ch
      const float Y = (CH == 1) ? ay[u] : ay[u] * 0.5f;
      X = fmaxf(X, 1e-10f);                        // np.maximum(X, 1e-10)
      o[k] = Y / X;
    }
  }
}

// ---------------------------------------------------------------------------
// reductions over frames
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_an_frame_mean(const float* __restrict__ spec,
                                                       int n_frames, int n_bins,
                                                       float* __restrict__ out) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n_bins) return;
  // The sum is one dependent chain per bin (numpy's order); its loads are not:
  // batches of kB frames are loaded one batch ahead so the chain never waits on
  // HBM latency (indices clamped: the last batch re-reads valid rows).
  constexpr int kB = 32;
  float cur[kB], nxt[kB];
  const int last = n_frames - 1;
#pragma unroll
  for (int u = 0; u < kB; ++u) cur[u] = spec[(int64_t)min(u, last) * n_bins + k];
  float s = 0.f;  // numpy's add.reduce starts from the identity (-0 sums to +0)
  for (int f0 = 0; f0 < n_frames; f0 += kB) {
#pragma unroll
    for (int u = 0; u < kB; ++u) nxt[u] = spec[(int64_t)min(f0 + kB + u, last) * n_bins + k];
#pragma unroll
    for (int u = 0; u < kB; ++u)
      if (f0 + u < n_frames) s = s + cur[u];
#pragma unroll
    for (int u = 0; u < kB; ++u) cur[u] = nxt[u];
  }
  out[k] = s / (float)n_frames;
}

__device__ __forceinline__ uint32_t fkey(float v) {
  const uint32_t u = __float_as_uint(v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float fval(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k ^ 0x80000000u) : ~k);
}

struct MedState {  // per bin
  uint32_t prefix;  // key bits fixed so far
  uint32_t rank;    // rank still to find inside the current prefix
  uint32_t cnt;     // elements equal to the selected key (after the last pass)
  uint32_t key2;    // min key > prefix (even counts)
};

__global__ void k_an_med_init(MedState* __restrict__ st, int n_bins, uint32_t k1) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < n_bins) st[b] = MedState{0u, k1, 0u, 0xFFFFFFFFu};
}

// pass p (0..3): histogram of digit (key >> (24 - 8p)) & 255 over selected
// frames whose higher digits equal the prefix; p == 4: min key > prefix
__global__ __launch_bounds__(256) void k_an_med_hist(const float* __restrict__ spec,
                                                     int n_frames, int n_bins,
                                                     const uint8_t* __restrict__ mask,
                                                     const MedState* __restrict__ st,
                                                     uint32_t* __restrict__ ghist, int pass,
                                                     int per_split) {
  __shared__ uint32_t h[256 * 64];  // [digit][lane]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int b = blockIdx.x * 64 + lane;
  const int fa = blockIdx.y * per_split;
  const int fb = min(n_frames, fa + per_split);
  const bool vb = b < n_bins;
  const uint32_t prefix = vb ? st[b].prefix : 0u;
  const int shift = 24 - 8 * pass;
  if (pass < 4) {
    for (int i = threadIdx.x; i < 256 * 64; i += 256) h[i] = 0u;
    __syncthreads();
    const uint32_t hm = pass == 0 ? 0u : (0xFFFFFFFFu << (32 - 8 * pass));
    if (vb) {
      for (int f = fa + w; f < fb; f += 4) {
        if (mask && !mask[f]) continue;
        const uint32_t key = fkey(spec[(int64_t)f * n_bins + b]);
        if ((key & hm) == prefix) atomicAdd(&h[((key >> shift) & 255u) * 64 + lane], 1u);
      }
    }
    __syncthreads();
    if (vb) {
      for (int d = w; d < 256; d += 4) {
        const uint32_t c = h[d * 64 + lane];
        if (c) atomicAdd(&ghist[(int64_t)b * 256 + d], c);
      }
    }
  } else {
    uint32_t m = 0xFFFFFFFFu;
    if (vb) {
      for (int f = fa + w; f < fb; f += 4) {
        if (mask && !mask[f]) continue;
        const uint32_t key = fkey(spec[(int64_t)f * n_bins + b]);
        if (key > prefix) m = min(m, key);
      }
    }
    h[w * 64 + lane] = m;
    __syncthreads();
    if (w == 0 && vb) {
      m = min(min(h[lane], h[64 + lane]), min(h[128 + lane], h[192 + lane]));
      if (m != 0xFFFFFFFFu) atomicMin(&ghist[(int64_t)b * 256], m);
    }
  }
}

__global__ void k_an_med_pick(MedState* __restrict__ st, const uint32_t* __restrict__ ghist,
                              int n_bins, int pass) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n_bins) return;
  MedState s = st[b];
  const uint32_t* hh = ghist + (int64_t)b * 256;
  if (pass < 4) {
    uint32_t r = s.rank, d = 0, c = 0;
    for (; d < 256; ++d) {
      c = hh[d];
      if (r < c) break;
      r -= c;
    }
    s.prefix |= (d & 255u) << (24 - 8 * pass);
    s.rank = r;
    s.cnt = c;
  } else {
    s.key2 = hh[0];
  }
  st[b] = s;
}

__global__ void k_an_med_final(const MedState* __restrict__ st, int n_bins, int even,
                               float* __restrict__ out) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n_bins) return;
  const MedState s = st[b];
  const float v1 = fval(s.prefix);
  // np.median = mean of the middle element(s): add.reduce from the identity 0
  if (!even) {
    out[b] = 0.f + v1;
    return;
  }
  // the upper middle equals v1 if another copy of v1 follows it
  const float v2 = (s.rank + 1 < s.cnt) ? v1 : fval(s.key2);
  out[b] = ((0.f + v1) + v2) / 2.0f;
}

// SpecArgs' FFT tables for n_fft: M, twiddles of M, Bluestein tables
int dft_args(int n_fft, hipStream_t s, SpecArgs* A) {
  A->M = dft_m(n_fft);
  if (A->M == 0) return TOMATIS_E_UNSUPPORTED;
  int rc = twiddles(A->M, s, &A->tw);
  if (rc != TOMATIS_OK || A->M == n_fft) return rc;
  Chirp c;
  if ((rc = chirp_tables(n_fft, A->M, &c)) != TOMATIS_OK) return rc;
  A->bb = c.b;
  A->bh = c.h;
  return TOMATIS_OK;
}

// calls f(integral_constant<M>, bool_constant<BLUE>) for the args' FFT size
// (M = 16 .. 16384; Bluestein sizes start at M = 32 since n_fft >= 16)
template <int M, typename L>
void launch_m(bool blue, L& f) {
  if constexpr (M >= 32) {
    if (blue) {
      f(std::integral_constant<int, M>{}, std::true_type{});
      return;
    }
  }
  f(std::integral_constant<int, M>{}, std::false_type{});
}

template <typename L>
int dispatch_m(const SpecArgs& A, L&& f) {
  const bool blue = A.M != A.n_fft;
  switch (A.M) {
    case 16: launch_m<16>(blue, f); break;
    case 32: launch_m<32>(blue, f); break;
    case 64: launch_m<64>(blue, f); break;
    case 128: launch_m<128>(blue, f); break;
    case 256: launch_m<256>(blue, f); break;
    case 512: launch_m<512>(blue, f); break;
    case 1024: launch_m<1024>(blue, f); break;
    case 2048: launch_m<2048>(blue, f); break;
    case 4096: launch_m<4096>(blue, f); break;
    case 8192: launch_m<8192>(blue, f); break;
    case 16384: launch_m<16384>(blue, f); break;
    default: return TOMATIS_E_UNSUPPORTED;
  }
  return an_launch();
}

}  // namespace

extern "C" {

int tomatis_an_frame_r(const float* x, int64_t n, int32_t ch, int32_t n_fft, int32_t hop,
                       int32_t level_mode, float scale, float* r_out, void* hs) {
  if (!x || !r_out || hop < 1 || ch < 1 || n_fft < 1) return TOMATIS_E_ARG;
  if (n_fft > kMaxM) return TOMATIS_E_UNSUPPORTED;
  if (level_mode == TOMATIS_AN_LEVEL_POWER_MONO) {
    if (ch != 2) return TOMATIS_E_ARG;
  } else if (level_mode == TOMATIS_AN_LEVEL_CHMEAN) {
    if (ch != 1 && ch != 2) return TOMATIS_E_UNSUPPORTED;
  } else {
    return TOMATIS_E_ARG;
  }
  if (n < n_fft) return TOMATIS_OK;
  const int64_t F = 1 + (n - n_fft) / hop;
  if (F > INT32_MAX) return TOMATIS_E_UNSUPPORTED;
  hipStream_t s = (hipStream_t)hs;
  const bool pm = level_mode == TOMATIS_AN_LEVEL_POWER_MONO;
  if (is_pow2(n_fft) && n_fft >= 256 && n_fft <= kMaxTreeN) {
    // perfect tree over 128-sample leaves
    const dim3 g((unsigned)((F + 3) / 4));
    if (pm)
      hipLaunchKernelGGL((k_an_frame_r<TOMATIS_AN_LEVEL_POWER_MONO, 2>), g, dim3(256), 0, s, x,
                         n_fft, hop, (int)F, scale, r_out);
    else if (ch == 1)
      hipLaunchKernelGGL((k_an_frame_r<TOMATIS_AN_LEVEL_CHMEAN, 1>), g, dim3(256), 0, s, x,
                         n_fft, hop, (int)F, scale, r_out);
    else
      hipLaunchKernelGGL((k_an_frame_r<TOMATIS_AN_LEVEL_CHMEAN, 2>), g, dim3(256), 0, s, x,
                         n_fft, hop, (int)F, scale, r_out);
    return an_launch();
  }
  PwProg q;
  int rc = pw_program(n_fft, &q);
  if (rc != TOMATIS_OK) return rc;
  const dim3 g((unsigned)F);
  if (pm)
    hipLaunchKernelGGL((k_an_frame_r_pw<TOMATIS_AN_LEVEL_POWER_MONO, 2>), g, dim3(256), 0, s, x,
                       n_fft, hop, scale, q.leaf, q.n_leaf, q.prog, q.n_prog, r_out);
  else if (ch == 1)
    hipLaunchKernelGGL((k_an_frame_r_pw<TOMATIS_AN_LEVEL_CHMEAN, 1>), g, dim3(256), 0, s, x,
                       n_fft, hop, scale, q.leaf, q.n_leaf, q.prog, q.n_prog, r_out);
  else
    hipLaunchKernelGGL((k_an_frame_r_pw<TOMATIS_AN_LEVEL_CHMEAN, 2>), g, dim3(256), 0, s, x,
                       n_fft, hop, scale, q.leaf, q.n_leaf, q.prog, q.n_prog, r_out);
  return an_launch();
}

int tomatis_an_select(const float* r, int32_t n_frames, uint32_t thr_bits,
                      const uint32_t* exc_host, int32_t n_exc, int32_t keep_above,
                      const int8_t* cls, int32_t cls_want, uint8_t* mask, int32_t* count,
                      void* hs) {
  if (!r || !mask || !count || n_frames < 0 || n_exc < 0 || n_exc > 4 || (n_exc && !exc_host))
    return TOMATIS_E_ARG;
  hipStream_t s = (hipStream_t)hs;
  int rc = an_fail(hipMemsetAsync(count, 0, sizeof(int32_t), s));
  if (rc != TOMATIS_OK || n_frames == 0) return rc;
  uint32_t e[4] = {0u, 0u, 0u, 0u};
  for (int i = 0; i < n_exc; ++i) e[i] = exc_host[i];
  hipLaunchKernelGGL(k_an_select, dim3((n_frames + 255) / 256), dim3(256), 0, s, r, n_frames,
                     thr_bits, make_uint4(e[0], e[1], e[2], e[3]), n_exc, keep_above, cls,
                     cls_want, mask, count);
  return an_launch();
}

int tomatis_an_spectra(const float* x, const float* y, int64_t n, int32_t ch, int32_t n_fft,
                       int32_t hop, int32_t kind, int32_t sig_mode, float scale,
                       const float* win, float* out, void* hs) {
  if (!x || !win || !out || hop < 1 || ch < 1 || n_fft < 1) return TOMATIS_E_ARG;
  if (dft_m(n_fft) == 0) return TOMATIS_E_UNSUPPORTED;
  if (kind == TOMATIS_AN_RATIO) {
    if (!y) return TOMATIS_E_ARG;
    if (ch != 1 && ch != 2) return TOMATIS_E_UNSUPPORTED;
  } else if (kind == TOMATIS_AN_MAG || kind == TOMATIS_AN_LOGPOW) {
    if (sig_mode == TOMATIS_AN_SIG_RAW) {
      if (ch != 1) return TOMATIS_E_ARG;
    } else if (sig_mode == TOMATIS_AN_SIG_POWER_MONO) {
      if (ch != 2) return TOMATIS_E_ARG;
    } else {
      return TOMATIS_E_ARG;
    }
  } else {
    return TOMATIS_E_ARG;
  }
  if (n < n_fft) return TOMATIS_OK;
  const int64_t F = 1 + (n - n_fft) / hop;
  if (F > INT32_MAX) return TOMATIS_E_UNSUPPORTED;
  hipStream_t s = (hipStream_t)hs;
  SpecArgs A{x, y, win, nullptr, nullptr, nullptr, out, n_fft, 0, hop, (int)F, n_fft / 2 + 1,
             scale};
  int rc = dft_args(n_fft, s, &A);
  if (rc != TOMATIS_OK) return rc;
  if (kind == TOMATIS_AN_RATIO) {
    const dim3 g((unsigned)F);
    return dispatch_m(A, [&](auto m, auto b) {
      constexpr int MM = decltype(m)::value;
      constexpr bool BL = decltype(b)::value;
      if (ch == 1) hipLaunchKernelGGL((k_an_spec_ratio<1, MM, BL>), g, dim3(kT), 0, s, A);
      else hipLaunchKernelGGL((k_an_spec_ratio<2, MM, BL>), g, dim3(kT), 0, s, A);
    });
  }
  const dim3 g((unsigned)((F + 1) / 2));
  const bool raw = sig_mode == TOMATIS_AN_SIG_RAW;
  return dispatch_m(A, [&](auto m, auto b) {
    constexpr int MM = decltype(m)::value;
    constexpr bool BL = decltype(b)::value;
    constexpr int MAG = TOMATIS_AN_MAG, LOGP = TOMATIS_AN_LOGPOW;
    constexpr int RAW = TOMATIS_AN_SIG_RAW, PM = TOMATIS_AN_SIG_POWER_MONO;
    if (kind == MAG && raw) hipLaunchKernelGGL((k_an_spec_pair<MAG, RAW, MM, BL>), g, dim3(kT), 0, s, A);
    else if (kind == MAG) hipLaunchKernelGGL((k_an_spec_pair<MAG, PM, MM, BL>), g, dim3(kT), 0, s, A);
    else if (raw) hipLaunchKernelGGL((k_an_spec_pair<LOGP, RAW, MM, BL>), g, dim3(kT), 0, s, A);
    else hipLaunchKernelGGL((k_an_spec_pair<LOGP, PM, MM, BL>), g, dim3(kT), 0, s, A);
  });
}

int tomatis_an_band_energy(const float* x, int64_t n, int32_t n_fft, int32_t hop,
                           int32_t lo0, int32_t lo1, int32_t hi0, int32_t hi1,
                           const float* win, float* out, void* hs) {
  if (!x || !win || !out || hop < 1 || n_fft < 1) return TOMATIS_E_ARG;
  if (dft_m(n_fft) == 0) return TOMATIS_E_UNSUPPORTED;
  const int nb = n_fft / 2 + 1;
  if (lo0 < 0 || lo1 < lo0 || lo1 > nb || hi0 < 0 || hi1 < hi0 || hi1 > nb) return TOMATIS_E_ARG;
  if (lo1 > hi0 && hi1 > lo0) return TOMATIS_E_ARG;  // bands must not overlap
  if (n < n_fft) return TOMATIS_OK;
  const int64_t F = 1 + (n - n_fft) / hop;
  if (F > INT32_MAX) return TOMATIS_E_UNSUPPORTED;
  hipStream_t s = (hipStream_t)hs;
  SpecArgs A{x, nullptr, win, nullptr, nullptr, nullptr, out, n_fft, 0, hop, (int)F, nb, 1.0f,
             {lo0, lo1, hi0, hi1}};
  int rc = dft_args(n_fft, s, &A);
  if (rc != TOMATIS_OK) return rc;
  const dim3 g((unsigned)((F + 1) / 2));
  return dispatch_m(A, [&](auto m, auto b) {
    hipLaunchKernelGGL((k_an_band_pair<decltype(m)::value, decltype(b)::value>), g, dim3(kT), 0,
                       s, A);
  });
}

int tomatis_cal_gate_grid(const float* levels, int32_t n_fit, const int64_t* starts,
                          const int32_t* target, const TomatisGateCand* cands, int32_t n_cand,
                          int32_t* out, uint8_t* states, void* hs) {
  if (n_fit < 0 || n_cand < 0 || (n_cand && (!cands || !out)) || (n_fit && (!levels || !starts)))
    return TOMATIS_E_ARG;
  if (n_cand == 0) return TOMATIS_OK;
  hipLaunchKernelGGL(k_cal_gate_grid, dim3((n_cand + 255) / 256), dim3(256), 0,
                     (hipStream_t)hs, levels, n_fit, starts, target, cands, n_cand, out, states);
  return an_launch();
}

int tomatis_an_frame_mean(const float* spec, int32_t n_frames, int32_t n_bins, float* out,
                          void* hs) {
  if (!spec || !out || n_frames < 1 || n_bins < 1) return TOMATIS_E_ARG;
  // one wave per 64 bins: spread the (latency-bound) chains over many CUs
  hipLaunchKernelGGL(k_an_frame_mean, dim3((n_bins + 63) / 64), dim3(64), 0,
                     (hipStream_t)hs, spec, n_frames, n_bins, out);
  return an_launch();
}

int64_t tomatis_an_median_work_words(int32_t n_bins) {
  return n_bins < 1 ? 0 : (int64_t)n_bins * (4 + 256);
}

int tomatis_an_frame_median(const float* spec, int32_t n_frames, int32_t n_bins,
                            const uint8_t* mask, int32_t n_sel, uint32_t* work, float* out,
                            void* hs) {
  if (!spec || !out || !work || n_frames < 1 || n_bins < 1 || n_sel < 1 || n_sel > n_frames)
    return TOMATIS_E_ARG;
  hipStream_t s = (hipStream_t)hs;
  MedState* st = reinterpret_cast<MedState*>(work);
  uint32_t* gh = work + (int64_t)n_bins * 4;
  const int even = (n_sel % 2) == 0;
  const uint32_t k1 = even ? (uint32_t)(n_sel / 2 - 1) : (uint32_t)(n_sel / 2);
  const dim3 gb((n_bins + 255) / 256);
  hipLaunchKernelGGL(k_an_med_init, gb, dim3(256), 0, s, st, n_bins, k1);
  // frame splits: enough workgroups to cover the chip, >= 1024 frames each
  const int groups = (n_bins + 63) / 64;
  int splits = (n_frames + 1023) / 1024;
  splits = std::max(1, std::min(splits, std::max(1, 2048 / groups)));
  const int per = (n_frames + splits - 1) / splits;
  const size_t gh_bytes = sizeof(uint32_t) * (size_t)n_bins * 256;
  for (int pass = 0; pass < 4 + even; ++pass) {
    int rc = (pass < 4) ? an_fail(hipMemsetAsync(gh, 0, gh_bytes, s))
                        : an_fail(hipMemsetAsync(gh, 0xFF, gh_bytes, s));
    if (rc != TOMATIS_OK) return rc;
    hipLaunchKernelGGL(k_an_med_hist, dim3(groups, splits), dim3(256), 0, s, spec, n_frames,
                       n_bins, mask, st, gh, pass, per);
    hipLaunchKernelGGL(k_an_med_pick, gb, dim3(256), 0, s, st, gh, n_bins, pass);
    rc = an_launch();
    if (rc != TOMATIS_OK) return rc;
  }
  hipLaunchKernelGGL(k_an_med_final, gb, dim3(256), 0, s, st, n_bins, even, out);
  return an_launch();
}

}  // extern "C"
