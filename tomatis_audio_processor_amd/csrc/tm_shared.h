// tm_shared.h — types shared by the two translation units of libtomatis_hip:
// tm_kernels.hip (levels, gate, limiter, plan, C ABI) and tm_transform.hip
// (the fused transform kernels, compiled with the max-ILP scheduler).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tm_common.h"
#include "../../include/tomatis_hip.h"

namespace tshared {
using tdsp::cf;

constexpr float kEps32 = 1e-12f;  // EPS as the reference adds it to float32 arrays
constexpr double kEps64 = 1e-12;

struct Run {          // main-kernel work item: emit frames [ka, kb) of stream s
  int32_t s;
  int32_t last;       // bit 0: kb is the stream's last frame + 1; bit 1: kRunInterior
  int64_t ka, kb;
};
// interior run: frames [max(0, ka - rmax + 1), kb) all read full frames and every
// emitted hop block is a full interior block (fast loop of the fused kernel)
constexpr int32_t kRunInterior = 2;

__device__ __forceinline__ int64_t floordiv(int64_t a, int64_t b) {
  int64_t q = a / b;
  return (q * b > a) ? q - 1 : q;
}

struct MainArgs {
  const float* x;
  float* y;
  const float* gains;   // [rows][N] gain per (lane, register) in bin layout (see gain_perm)
  const uint16_t* rows;
  uint32_t* peaks;
  const TomatisStream* st;
  const Run* runs;
  const float* win;     // [N]
  const float* winS;    // [N] synthesis window x the inverse FFT's output scales (register FFT)
  const float* win2;    // [N] win*win (f32)
  const cf* twN;        // [32][P]
  const cf* twP;        // [P]
  const float* winv;    // [hop] 1/(interior wsum) (already normalisation-rule applied)
  cf* scratch;          // generic path: [frames][N]
  int n_runs, hop, n_bins, ch, norm_mode, rmax, n_rows_lds;
  int lds_row[2];       // GM 2: the rows held in LDS (others read from global)
  int lds_mixed;        // 1: n_rows > 2, only lds_row[] in LDS
  int edge_mask;        // fused limiter skips chunk 0 (bit 0) / the last chunk (bit 1)
  float inv_n;
  // fused limiter (limit > 0): per-chunk flush counters, flushes expected,
  // output ranges; every wave rescales its own output once its chunks are final
  float limit;
  uint32_t* chunk_done;
  const uint32_t* chunk_need;
  const int64_t* chunk_rng;  // [2 * chunk]: output-relative [p0, p1)
  uint32_t* err;        // TOMATIS_ERR_* bits
  int lim_spin;         // fused-limiter wait bound (polls of the chunk counter)
  unsigned long long* prof;  // TM_PROFILE builds only: per-phase wave cycles
  // Pipelined batches (tomatis_stft_ola_gated_pipelined / _pipelined): runs
  // [run_base, run_base + n_runs); defer_self leaves this launch's output
  // unscaled; per launched run 2 * (max_pieces + 1) words of k_r2_plan output:
  // {count, first block left to the tail}, then count x {block, scale bits}
  int run_base;
  int defer_self;
  const uint32_t* pieces;
  int max_pieces;
  // Pipelined batches (tomatis_stft_ola_gated_pipelined): the partner of every
  // run is the same run of the PREVIOUS batch of this plan, whose unscaled
  // output yprev and final chunk peaks peaks_prev are complete (no waits); the
  // kernel's own output stays unscaled (defer_self) for the next batch.
  float* yprev;
  const uint32_t* peaks_prev;
  // the previous batch's plan (tomatis_stft_ola_*_pipelined_after: any plan of
  // the same n_fft / hop / channels; else this plan's own arrays): its runs,
  // stream table and chunk output ranges.  Run r's partner is run r of that
  // plan when r < n_runs_prev; partner runs >= n_runs are limited by
  // launch_prev_runs after the transform
  const Run* runs_prev;
  const TomatisStream* st_prev;
  const int64_t* chunk_rng_prev;
  int n_runs_prev;
  // gain rows as the caller passed them ([rows][n_bins], not permuted): when
  // set, the LDS-gain prologue (all rows in LDS) permutes them itself and the
  // host launches no k_gain_perm
  const float* graw;
  int g_nb;
  // in-kernel levels + gate (tomatis_stft_ola_gated, DESIGN.md §5 "Fused
  // levels"): every frame's r (numpy pairwise order) and gate state are computed
  // from the input the transform loads and written here; each run starts from
  // k_gate_carry's carry-in state id and 16-leaf window
  int gated;
  int gate_D;           // up-delay frames
  float* r_out;
  uint8_t* st_out;
  const int32_t* gcarry;  // per run: state id before its first frame (< 0: unresolved,
                          // kGateChained: compose gtf from the nearest resolved run)
  const uint16_t* gtf;    // chained runs' transfer tables [run][gate_D + 2]
  // cross-fade gate (alpha mode 1, n_fft 4096): gate_xf >= 0 cross-fade frames
  // (-1: standard gate, gain row = state); every frame's alpha (float64,
  // process_tomatis_xfade.py:251-274) to a_out, the gain row from alpha; each
  // run starts from k_gate_carry's alpha before its first frame (gacarry)
  int gate_xf;
  double gate_astep;    // 1.0 / gate_xf (gate_xf > 0), computed once on the host
  double* a_out;
  const double* gacarry;
};
// (also zeroes A.peaks[0, n_zero): this pipelined launch's chunk peaks)
void launch_r2_plan(const MainArgs& A, uint32_t* pieces, int n_zero, int P, hipStream_t s);
// pipelined batches: the limiter on runs [A.n_runs, A.n_runs_prev) of the
// previous batch's plan (partners no run of this launch has), one wave each
void launch_prev_runs(const MainArgs& A, int N, hipStream_t s);
// k_gate_carry over every run of A (A.run_base = 0): carry-in state id per
// run; kGateLookback frames of look-back (kGateLookbackMax back to the
// previous run's start when gtf is given) before a run is left unresolved.
// gtf (optional): per-run transfer tables [n_runs][gate_D + 2] for chained
// runs, composed in the transform's prologue (gate_chain_carry)
// n_fft 2048 (P 64, NR 32) and 4096 (P 128, NR 32; A.gate_xf >= 0: also the
// alpha before each run's first frame into gacarry, no chaining)
void launch_gate_carry(const MainArgs& A, int P, int SH, int ch, int32_t* gcarry,
                       uint16_t* gtf, double* gacarry, hipStream_t s);
constexpr int kGateLookback = 512;       // look-back limit of a run that cannot chain
constexpr int kGateLookbackMax = 4096;   // chained runs: frames back to the previous run's start
constexpr int kGateChainStates = 1024;   // chaining needs gate_D + 2 <= this (transfer tables)
constexpr int kGateChained = -2;         // k_gate_carry -> k_gate_chain marker

// Any-size path (any n_fft in [2, kMaxNfft], any hop, 1..kMaxCh channels): per
// (frame, channel pair) a Stockham FFT of length M (n_fft when it is a power
// of two, else Bluestein's power of two >= 2 n_fft - 1) in LDS (M <= kLdsMaxM)
// or in per-block HBM buffers, windowed frames to scratch float
// [frame][n_fft][ch], then a per-position gather in frame order.
constexpr int kMaxNfft = 1 << 16;
constexpr int kMaxCh = 128;
constexpr int kLdsMaxM = 16384;
struct LdsArgs {
  const float* x;
  const TomatisStream* st;
  int n_streams;
  const float* gains;   // [rows][n_fft/2+1] natural bin order (the caller's table)
  const uint16_t* rows;
  const float* win;     // [N]
  const float* win2;    // [N]
  const float2* tw;     // [M] exp(-2 pi i t / M)
  const float2* blue_b; // Bluestein: [N] chirp exp(i pi n^2 / N)
  const float2* blue_h; // Bluestein: [M] FFT_M(chirp filter) / M
  float2* work;         // M > kLdsMaxM: [gridDim.x][2][M] per-block buffers
  float* scratch;       // [total_frames][N][ch]
  float* y;
  uint32_t* peaks;
  const int64_t* pos_base;  // output position prefix per stream
  int64_t total_frames, total_out;
  int n_fft, hop, ch, n_bins, norm_mode;
  int M, blue, work_blocks;
};
void launch_lds_frames(const LdsArgs& A, hipStream_t s);
void launch_lds_gather(const LdsArgs& A, hipStream_t s);

// n_fft 2048 register kernels (P = 64) run the single-exchange FFT (tm_fft.h
// fftx_*; its bin layout in the gain rows, its output scales in winS); the
// two-exchange form stays for n_fft 4096 and for -DTM_DEV_NOFX A/B builds
#ifdef TM_DEV_NOFX
constexpr bool kFftX = false;
#else
constexpr bool kFftX = true;
#endif

// launchers (tm_transform.hip); kernels stay private to that unit
int transform_wg(int P, int NR);  // workgroup size of the fused kernel
int transform_slots_per_cu(int P, int NR);  // resident sequences per CU
void launch_transform(const MainArgs& A, int P, int NR, int SH, int ch, int wg, hipStream_t s);
void launch_frames(const MainArgs& A, int P, int NR, int blocks, hipStream_t s);
void launch_gain_perm(int P, int NR, bool fx, const float* gains, int n_rows, int n_bins,
                      float* out, hipStream_t s);
void launch_ola_gather(const MainArgs& A, int n_streams, const int64_t* pos_base, int64_t total,
                       int N, hipStream_t s);
int dev_opt(int key, int dflt);  // tomatis_set_dev_option (default when unset)

}  // namespace tshared
