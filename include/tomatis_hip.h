/*
 * tomatis_hip.h — C ABI of the MI355X (gfx950) STFT-gate-OLA engine.
 *
 * Drop-in boundary for the per-frame loop of the reference
 * (xyjk0511/tomatis-audio-processor).  The reference has no FFI: its
 * "operator API" is the set of Python functions below, each of which the
 * Python host layer (tomatis_audio_processor_amd/) re-exposes under the same
 * name and semantics and implements with these entry points:
 *
 *   reference                                   replaced by
 *   ------------------------------------------- -------------------------------
 *   src/process_tomatis.py:359-371 (frame loop:  tomatis_levels
 *       power-mono RMS per frame, rms_dbfs
 *       src/process_tomatis.py:43-52)
 *   src/process_tomatis_adaptive.py:57-84        tomatis_levels
 *       (compute_frame_levels)
 *   src/process_tomatis.py:373-385 (gate)        tomatis_gate_std
 *   src/process_tomatis.py:369-406 (levels,      tomatis_stft_ola_gated
 *       gate and transform in one pass)           (+ tomatis_gate_lookback)
 *   src/process_tomatis_xfade.py:237-274         tomatis_gate_std (+alpha rows)
 *   src/process_tomatis_adaptive.py:87-154       tomatis_minhold_bisect
 *       (simulate_gate, find_optimal_threshold)
 *   src/process_tomatis_adaptive.py:253-265      tomatis_minhold_bisect (alpha)
 *   src/process_tomatis.py:394-406,419-426,451   tomatis_stft_ola
 *       (rfft*gain, irfft*win, OLA, normalise)
 *   src/process_tomatis_xfade.py:277-290         tomatis_stft_ola
 *   src/process_tomatis_adaptive.py:298-338      tomatis_stft_ola
 *   src/layer2_apply_eq.py:143-214               tomatis_stft_ola
 *   src/layer2b_apply_residual_eq.py:120-160     tomatis_stft_ola
 *   src/process_tomatis.py:331-357 (limiter),    tomatis_apply_limiter,
 *                                                 tomatis_stft_ola_limited
 *   src/process_tomatis_adaptive.py:340-345
 *   np.max(np.abs(x)) (adaptive :201,          tomatis_absmax
 *       layer2 gain protect :178,213)
 *   src/compare_audio.py:12-24 (stft_mag_avg)    tomatis_an_spectra(MAG),
 *                                                 tomatis_an_frame_mean
 *   src/layer2_analyze_eq.py:54-88               tomatis_an_frame_r, tomatis_an_select,
 *       (stft_logpower_median)                    tomatis_an_spectra(LOGPOW),
 *                                                 tomatis_an_frame_median
 *   src/validate_layer1.py:261-389               tomatis_an_frame_r, tomatis_an_select,
 *       (compute_conditional_spectrum)            tomatis_an_spectra(RATIO),
 *                                                 tomatis_an_frame_median
 *   src/calibrate_to_baseline_v2.py:192-198      tomatis_an_frame_r (POWER_MONO levels),
 *       (orig/base levels, stft_band_tilt :17-31)  tomatis_an_band_energy
 *   src/calibrate_to_baseline_v2.py:84-109,      tomatis_cal_gate_grid
 *       231-265 (simulate_state x the gain /
 *       up-delay / hysteresis / T search grid)
 *
 * Conventions: every call is asynchronous on the given hipStream_t and returns
 * an int status (0 = ok, <0 = error, see TOMATIS_E_*); no exceptions cross the
 * ABI.  The caller owns every data buffer (device pointers, e.g. torch tensors'
 * data_ptr()).  The library owns only the plan (host tables + small device
 * workspace).  One plan per host thread / stream.  Layouts are documented in
 * DESIGN.md ("Data layout in HBM").
 */
#ifndef TOMATIS_HIP_H
#define TOMATIS_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TOMATIS_ABI_VERSION 11

#define TOMATIS_OK 0
#define TOMATIS_E_ARG (-1)        /* bad argument */
#define TOMATIS_E_UNSUPPORTED (-2)/* shape/config not built for gfx950 here */
#define TOMATIS_E_HIP (-3)        /* a HIP runtime call failed */
#define TOMATIS_E_NOMEM (-4)

/* OLA normalisation rule */
#define TOMATIS_NORM_EPS 0        /* y = ola / (wsum + 1e-12f)   (standard, xfade, layer2, layer2b) */
#define TOMATIS_NORM_MAX 1        /* y = ola / max(wsum, 1e-8f)  (adaptive) */

/* Per-frame level precision (reference dtype) */
#define TOMATIS_F32 0
#define TOMATIS_F64 1

/* Per-stream geometry + gate parameters.  All positions are in samples of the
 * stream's own time axis, where samples [0, n) are the input and everything
 * outside is zero (the reference's padding).  Frame k covers
 * [first_start + k*hop, first_start + k*hop + n_fft). */
typedef struct TomatisStream {
    int64_t in_off;       /* float index of sample 0 / channel 0 in x          */
    int64_t out_off;      /* float index of output sample 0 / channel 0 in y   */
    int64_t n;            /* input samples per channel                          */
    int64_t first_start;  /* position of frame 0                                */
    int64_t n_frames;     /* frames of this stream                              */
    int64_t out_begin;    /* position of output sample 0                        */
    int64_t out_len;      /* output samples per channel                         */
    int64_t chunk_first;  /* position where limiter chunk 1 starts              */
    int64_t chunk_len;    /* length of chunks 1..n_chunks-2 (last runs to end)  */
    int32_t n_chunks;     /* limiter chunks (>=1)                               */
    float in_scale;       /* x is multiplied by this (f32) before framing       */
    float out_scale;      /* y is multiplied by this (f32) before the peak      */
    /* standard gate on float32 r bit patterns:
     *   on  = (bits >= on_bits)  XOR (bits in on_exc[0..n_on_exc))
     *   off = (bits <= off_bits) XOR (bits in off_exc[0..n_off_exc))
     * NaN r -> both false. */
    uint32_t on_bits, off_bits;
    uint32_t on_exc[4], off_exc[4];
    int32_t n_on_exc, n_off_exc;
    /* f64 thresholds (min-hold gate on f64 levels) */
    double t_on, t_off;
    /* filled by tomatis_plan_create: */
    int64_t frame_base;   /* index of frame 0 in per-frame arrays               */
    int32_t chunk_base;   /* index of chunk 0 in per-chunk arrays               */
    int32_t _pad;
} TomatisStream;

typedef struct TomatisPlanDesc {
    int32_t n_fft;        /* 2048 or 4096 on the fast path                      */
    int32_t hop;          /* any 1..n_fft; fast OLA when hop % (n_fft/32) == 0  */
    int32_t ch;           /* 1 or 2                                             */
    int32_t norm_mode;    /* TOMATIS_NORM_*                                     */
    int32_t up_delay_frames; /* ceil(up_delay_samples/hop), >=0 (standard gate) */
    int32_t min_hold_frames; /* adaptive min-hold                               */
    int32_t xfade_frames;    /* xfade / adaptive alpha step = 1/xfade_frames    */
    int32_t alpha_mode;      /* 0 none, 1 xfade (python-float start), 2 adaptive */
} TomatisPlanDesc;

typedef struct tomatis_plan_s* tomatis_plan_t;

/* Library / device info */
int tomatis_abi_version(void);
const char* tomatis_status_string(int status);

/* Plan: copies the stream table (host array) to the device, assigns
 * frame_base / chunk_base, builds window / twiddle / pairwise-sum tables and
 * the work decompositions.  Returns TOMATIS_E_UNSUPPORTED for shapes the
 * gfx950 kernels are not built for. */
int tomatis_plan_create(tomatis_plan_t* plan, const TomatisPlanDesc* desc,
                        const float* window /* host, n_fft floats: np.hanning(n_fft) as f32 */,
                        TomatisStream* streams /* in/out, host */, int32_t n_streams);
int tomatis_plan_destroy(tomatis_plan_t plan);
int64_t tomatis_plan_total_frames(tomatis_plan_t plan);
int32_t tomatis_plan_total_chunks(tomatis_plan_t plan);
/* Re-upload per-stream gate / scale fields after the host changed them
 * (adaptive thresholds, attenuation).  Geometry must be unchanged. */
int tomatis_plan_update_streams(tomatis_plan_t plan, const TomatisStream* streams,
                                void* hip_stream);

/* Per-frame RMS r (reference rms_dbfs before the log10): float32 (prec=F32)
 * or float64 (prec=F64) per frame, frame-major over all streams. */
int tomatis_levels(tomatis_plan_t plan, const float* x, void* r_out, int32_t prec,
                   void* hip_stream);

/* Standard / xfade gate: states (1=C1, 2=C2) per frame and the gain-row index
 * per frame for tomatis_stft_ola.  Rows: 0 = g1, 1 = g2, 2+m = mixed gain at
 * alpha = m/xfade_frames (alpha_mode 1).  alpha_out (optional, f64 per frame). */
int tomatis_gate_std(tomatis_plan_t plan, const float* r, uint8_t* states,
                     uint16_t* rows, double* alpha_out, void* hip_stream);

/* Time sharding of one stream across ranks (host side:
 * tomatis_audio_processor_amd/timeshard.py).  The standard gate's run-scan form
 * (plans whose thresholds admit no float32 r that is both "on" and "off",
 * i.e. hysteresis > 0) is an associative scan over per-segment summaries:
 *   summary (5 int32): all_on, not_on (last not-on frame), l_end (last frame
 *     of the leading on-run), e_int (last gate entry after the first not-on
 *     frame), off (last off frame); frame indices stream-local,
 *     TOMATIS_GATE_NONE for none;
 *   carry (3 int32): a (last not-on frame), e (last entry), f (last off);
 *     C1 idle before frame 0 = (-1, NONE, NONE); state(k) = C2 iff e > f.
 * A rank composes its predecessors' summaries into its carry-in (one
 * all_gather of 5 ints per rank) and resolves its own frames from it.
 * Replaces the sequential automaton src/process_tomatis.py:373-385 across a
 * shard boundary. */
#define TOMATIS_GATE_SEGMENT 1024          /* frames per gate segment */
#define TOMATIS_GATE_NONE (-536870912)     /* INT_MIN / 4 */
int32_t tomatis_plan_gate_segments(tomatis_plan_t plan);
/* Synchronous: per-segment summaries of every stream (segments in stream order,
 * TOMATIS_GATE_SEGMENT frames each, the last one partial), 5 int32 each, into
 * sums_host.  TOMATIS_E_UNSUPPORTED when the gate is not in run-scan form. */
int tomatis_gate_segment_sums(tomatis_plan_t plan, const float* r, int32_t* sums_host,
                              void* hip_stream);
/* tomatis_gate_std (standard gate, alpha_mode 0) starting every stream from
 * carry_host[3*s .. 3*s+2] instead of C1 idle.  Synchronous. */
int tomatis_gate_std_carry(tomatis_plan_t plan, const float* r, const int32_t* carry_host,
                           uint8_t* states, uint16_t* rows, void* hip_stream);

/* Device-resident time-shard step (timeshard.py; single-stream plans):
 * tomatis_ts_summary: the gate summary (5 int32, TOMATIS_GATE_NONE for none)
 *   of the plan's first n_seg gate segments re-indexed by +shift frames, into
 *   device memory (the all_gather input).  Replaces timeshard.summarize/gs_cat
 *   on the host.
 * tomatis_ts_gate: the carry-in composed from sums_all[5*q..] of ranks
 *   q < rank, re-indexed by shift, then the standard gate from it (as
 *   tomatis_gate_std_carry, asynchronous, no host data). */
int tomatis_ts_summary(tomatis_plan_t plan, const float* r, int32_t n_seg, int32_t shift,
                       int32_t* sum_out, void* hip_stream);
int tomatis_ts_gate(tomatis_plan_t plan, const float* r, const int32_t* sums_all, int32_t rank,
                    int32_t shift, uint8_t* states, uint16_t* rows, void* hip_stream);

/* Adaptive: per stream, t_lo_hi_med[3*s..3*s+2] = (np.percentile(v, 5),
 * np.percentile(v, 95), np.median(v)) of v = the stream's levels > -70, or
 * (NaN, NaN, np.median(levels)) when none is valid, (NaN, NaN, 0) for a stream
 * without frames -- bit-identical to numpy (exact selection + numpy's linear
 * interpolation).  Replaces src/process_tomatis_adaptive.py:123-131. */
int tomatis_level_stats(tomatis_plan_t plan, const double* levels, double* t_lo_hi_med,
                        void* hip_stream);

/* Adaptive: bisection for the min-hold threshold per stream
 * (find_optimal_threshold), final states, alpha and gain rows (2+m).
 * levels: f64 per frame; t_lo_hi_med: 3 doubles per stream (p5, p95, median of
 * valid levels; n_valid==0 streams pass NaN and get t = median(levels) in
 * t_lo_hi_med[2]); target_c2, hyst_db as in the reference. */
int tomatis_minhold_bisect(tomatis_plan_t plan, const double* levels,
                           const double* t_lo_hi_med, double target_c2, double hyst_db,
                           double* t_out, uint8_t* states, uint16_t* rows,
                           double* alpha_out, void* hip_stream);

/* Fused framing -> window -> FFT -> gain row -> IFFT -> window -> OLA ->
 * normalise -> out_scale, plus per-chunk |y| maxima as float bits
 * (chunk_peak_bits must be zeroed by the caller; uint32 per chunk).
 * rows: one uint16 gain-row id per frame; the kernel reads it through the
 * scalar cache in aligned 4-byte words, so the allocation must cover
 * total_frames rounded up to an even count. */
int tomatis_stft_ola(tomatis_plan_t plan, const float* x, const float* gain_rows,
                     int32_t n_rows, const uint16_t* rows, float* y,
                     uint32_t* chunk_peak_bits, void* hip_stream);

/* Limiter fix-up: chunk j of every stream is multiplied by limit/peak_j
 * (float32 division, as the reference) when peak_j > limit. */
int tomatis_apply_limiter(tomatis_plan_t plan, float* y, const uint32_t* chunk_peak_bits,
                          float limit, void* hip_stream);

/* tomatis_stft_ola followed by tomatis_apply_limiter(limit), with the limiter
 * done inside the transform kernel when every chunk's samples come from a few
 * neighbouring runs (each wave rescales its own samples once its chunks are
 * complete); otherwise the two launches.  Same results as the pair. */
int tomatis_stft_ola_limited(tomatis_plan_t plan, const float* x, const float* gain_rows,
                             int32_t n_rows, const uint16_t* rows, float* y,
                             uint32_t* chunk_peak_bits, float limit, void* hip_stream);
/* As tomatis_stft_ola_limited, except that the first (edge_mask bit 0) and/or
 * last (bit 1) limiter chunk of every stream is left unscaled: a time shard's
 * chunks shared with its neighbours, scaled by tomatis_apply_limiter_edges once
 * their peaks are all-reduced (src/process_tomatis.py:331-357 per global chunk). */
int tomatis_stft_ola_limited_edges(tomatis_plan_t plan, const float* x, const float* gain_rows,
                                   int32_t n_rows, const uint16_t* rows, float* y,
                                   uint32_t* chunk_peak_bits, float limit, int32_t edge_mask,
                                   void* hip_stream);
/* tomatis_levels(F32) + tomatis_gate_std + tomatis_stft_ola_limited in one
 * pass over the input (standard mode): a small pre-kernel finds every run's
 * gate state before its first frame (a look-back to the nearest frame that
 * fixes the automaton's state: one not "on" and "off", or up_delay_frames + 1
 * consecutive "on" and not "off"), then the transform kernel computes each
 * frame's r (numpy's pairwise order, bit-identical to tomatis_levels) and
 * state from the samples it loads for the FFT and picks the gain row from it.
 * r_out (f32) and states_out (1 = C1, 2 = C2) per frame as tomatis_levels /
 * tomatis_gate_std write them; n_rows must be 2 (rows C1, C2); limit 0 = no
 * limiter.  TOMATIS_E_UNSUPPORTED unless n_fft 2048 with hop 256 or 512 and
 * alpha_mode 0, or (dev option TOMATIS_DEV_FUSED_4096 set: measured slower than
 * the two-pass chain) n_fft 4096 with hop 1024 and alpha_mode 0 or 1, <= 2
 * channels, in_scale 1 and every stream below 2^31 bytes (the caller runs the
 * two-pass chain).  alpha_mode 1 (cross-fade, src/process_tomatis_xfade.py:
 * 237-278): the rows are tomatis_gate_std's (0 = g1, 1 = g2, 2 + m = alpha
 * m / xfade_frames) and every frame's alpha goes to the array set by
 * tomatis_plan_set_gate_alpha (as tomatis_gate_std's alpha_out).  When a run's look-back does not resolve
 * within 512 frames the launch sets TOMATIS_ERR_GATE_CARRY and its outputs are
 * invalid: the caller re-runs the two-pass chain.  Replaces
 * src/process_tomatis.py:373-385 (levels + gate loop) feeding :391-400. */
int tomatis_stft_ola_gated(tomatis_plan_t plan, const float* x, const float* gain_rows,
                           int32_t n_rows, float* y, uint32_t* chunk_peak_bits, float limit,
                           float* r_out, uint8_t* states_out, void* hip_stream);
/* Cross-fade plans (alpha_mode 1): the float64 per-frame alpha output of the
 * gated calls (required before one; frame-major as tomatis_gate_std's).  ABI 11. */
int tomatis_plan_set_gate_alpha(tomatis_plan_t plan, double* alpha_out);
/* The two launches of tomatis_stft_ola_gated separately (the caller times the
 * transform alone): tomatis_gate_lookback runs the look-back pre-kernel on x;
 * tomatis_stft_ola_gated_after_lookback then runs the transform on the same x,
 * on the same stream, with no other gated call of this plan in between. */
int tomatis_gate_lookback(tomatis_plan_t plan, const float* x, void* hip_stream);
int tomatis_stft_ola_gated_after_lookback(tomatis_plan_t plan, const float* x,
                                          const float* gain_rows, int32_t n_rows, float* y,
                                          uint32_t* chunk_peak_bits, float limit, float* r_out,
                                          uint8_t* states_out, void* hip_stream);
/* Pipelined batches of one plan (batch k+1's transform limits batch k's
 * output): as tomatis_stft_ola_gated_after_lookback with limit > 0, except that
 * y is left UNSCALED (chunk_peak_bits complete when the launch does) and, when
 * prev_y is given, the previous batch's unscaled output prev_y (written by the
 * previous call with this plan, its peaks prev_peak_bits) gets the per-chunk
 * limiter of src/process_tomatis.py:331-357 inside this launch's frame loops --
 * so the rescale's HBM traffic overlaps the transform instead of being a tail.
 * The last batch's output is limited by tomatis_apply_limiter(plan, y,
 * chunk_peak_bits, limit).  Results are bit-identical to the unpipelined call.
 * y, chunk_peak_bits must not alias prev_y, prev_peak_bits.  The call zeroes
 * chunk_peak_bits itself (inside the launch sequence; the caller need not).
 * TOMATIS_E_UNSUPPORTED where tomatis_stft_ola_gated is, or without limiter
 * chunks (the caller runs the unpipelined call). */
int tomatis_stft_ola_gated_pipelined(tomatis_plan_t plan, const float* x,
                                     const float* gain_rows, int32_t n_rows, float* y,
                                     uint32_t* chunk_peak_bits, float limit, float* r_out,
                                     uint8_t* states_out, float* prev_y,
                                     const uint32_t* prev_peak_bits, void* hip_stream);
/* The same batch pipeline for the two-pass chain (gain-row ids from the
 * caller: the adaptive processor's min-hold states, src/process_tomatis_adaptive.py
 * :298-345, whose global limiter is one chunk per stream): as
 * tomatis_stft_ola_limited except that y is left unscaled and prev_y (the
 * previous call's output with this plan, peaks prev_peak_bits) is limited
 * inside this launch; chunk_peak_bits zeroed by the call as above.
 * TOMATIS_E_UNSUPPORTED unless n_fft 2048, hop <= 512
 * (hop 512 for cross-fade row tables) and limiter chunks exist. */
int tomatis_stft_ola_pipelined(tomatis_plan_t plan, const float* x, const float* gain_rows,
                               int32_t n_rows, const uint16_t* rows, float* y,
                               uint32_t* chunk_peak_bits, float limit, float* prev_y,
                               const uint32_t* prev_peak_bits, void* hip_stream);
/* Batch pipelines over DIFFERENT plans (a multi-file job: batch k+1's files
 * are not batch k's): as tomatis_stft_ola_gated_pipelined /
 * tomatis_stft_ola_pipelined, with prev_y / prev_peak_bits written by the
 * previous call with prev_plan (NULL: this plan).  prev_plan must have this
 * plan's n_fft, hop and channel count (else TOMATIS_E_UNSUPPORTED: the caller
 * limits prev_y with tomatis_apply_limiter(prev_plan, ...) and runs this batch
 * unpipelined).  Run r of this launch scales run r of prev_plan's output in its
 * frame loop; prev_plan's runs beyond this plan's run count are limited by a
 * short launch after the transform.  prev_plan must stay alive until the call's
 * work has completed.  Results are bit-identical to limiting each batch with
 * its own plan (src/process_tomatis.py:331-357, per file). */
int tomatis_stft_ola_gated_pipelined_after(tomatis_plan_t plan, const float* x,
                                           const float* gain_rows, int32_t n_rows, float* y,
                                           uint32_t* chunk_peak_bits, float limit, float* r_out,
                                           uint8_t* states_out, tomatis_plan_t prev_plan,
                                           float* prev_y, const uint32_t* prev_peak_bits,
                                           void* hip_stream);
int tomatis_stft_ola_pipelined_after(tomatis_plan_t plan, const float* x, const float* gain_rows,
                                     int32_t n_rows, const uint16_t* rows, float* y,
                                     uint32_t* chunk_peak_bits, float limit,
                                     tomatis_plan_t prev_plan, float* prev_y,
                                     const uint32_t* prev_peak_bits, void* hip_stream);
/* The limiter on the edge chunks of edge_mask only. */
int tomatis_apply_limiter_edges(tomatis_plan_t plan, float* y, const uint32_t* chunk_peak_bits,
                                float limit, int32_t edge_mask, void* hip_stream);

/* Device-side consistency checks of the plan's kernels (bits of the plan's
 * error word):
 *   TOMATIS_ERR_LIMITER_WAIT  a fused-limiter wave gave up waiting for its
 *       chunk's flushes (bounded spin) and left its samples of that chunk
 *       unscaled: the launch's output is incomplete; re-run it with
 *       TOMATIS_OPT_FUSE_LIMITER = 0 (transform, then tomatis_apply_limiter).
 *   TOMATIS_ERR_PAIR_BARRIER  a two-wave (n_fft 4096) exchange barrier timed
 *       out: that launch's FFTs are wrong; no retry makes it safe.
 *   TOMATIS_ERR_GATE_CARRY  tomatis_stft_ola_gated could not resolve a run's
 *       gate carry-in within its look-back (the level stayed between the two
 *       thresholds, never D + 1 frames above): that launch's states and output
 *       are invalid; re-run the two-pass path (tomatis_levels, tomatis_gate_std,
 *       tomatis_stft_ola_limited), which has no look-back limit.
 * Synchronous: tomatis_plan_error returns TOMATIS_E_HIP if any bit is set
 * since creation (or the last reset), else OK; tomatis_plan_error_bits returns
 * the bits and clears them when reset != 0.  Replaces nothing in the
 * reference (its loop has no asynchronous device work to check). */
#define TOMATIS_ERR_LIMITER_WAIT 1u
#define TOMATIS_ERR_PAIR_BARRIER 2u
#define TOMATIS_ERR_GATE_CARRY 4u
int tomatis_plan_error(tomatis_plan_t plan, void* hip_stream);
int tomatis_plan_error_bits(tomatis_plan_t plan, uint32_t* bits, int32_t reset,
                            void* hip_stream);

/* Plan options (synchronous, host-side):
 *   TOMATIS_OPT_FUSE_LIMITER (1 default / 0): limiter inside the transform
 *       kernel where eligible, or always the separate tomatis_apply_limiter.
 *   TOMATIS_OPT_LIMITER_SPIN: polls a fused-limiter wave makes before it gives
 *       up (default 2^18; 0 forces TOMATIS_ERR_LIMITER_WAIT: fault-injection
 *       tests of the host's recovery path).
 *   TOMATIS_OPT_MINHOLD_SERIAL (0 default / 1): how tomatis_minhold_bisect runs
 *       the bisection (same result bit for bit).  0: three steps per launch as
 *       the 7 midpoints of their tree, 7 workgroups per stream over the chip,
 *       when every stream's tables fit the LDS (else serial); 1: the 30 steps
 *       in one workgroup per stream -- the small footprint to prefer when the
 *       call overlaps another stream group's transform.
 * (Option 4, the two-round fused limiter of ABI <= 7, is withdrawn: the
 * pipelined calls apply a batch's limiter inside the next batch's transform.) */
#define TOMATIS_OPT_FUSE_LIMITER 1
#define TOMATIS_OPT_LIMITER_SPIN 2
#define TOMATIS_OPT_MINHOLD_SERIAL 3
int tomatis_plan_set_option(tomatis_plan_t plan, int32_t option, int64_t value);

/* Development overrides (tests and A/B experiments only).  Process-wide,
 * explicit: the library reads no environment variable.  value < 0 restores the
 * default.  Read at plan creation: FORCE_LDS, P64 (n_fft 2048 as one wave per
 * frame), FAST_LOOP (interior loop), RUN_FRAMES (frames per run, 0 auto),
 * RUN_ROUNDS, LEVELS_LEGACY, GATE_TF (transfer-function gate scan), MH_PARTS,
 * SLOTS (resident run slots: few slots make long runs on small inputs);
 * at launch: GATE_TF, ALPHA_SEQ (sequential xfade alpha), GAIN_LDS,
 * FUSE_LIMITER, WG (transform workgroup size), FUSED_LEVELS.  Standard-mode
 * plans at n_fft 2048 cut runs of at most 4096 frames whatever RUN_FRAMES
 * says (the in-kernel gate's chained look-back).  Results are bit-identical
 * under every value (the decomposition tests vary them). */
#define TOMATIS_DEV_FAST_LOOP 1
#define TOMATIS_DEV_RUN_ROUNDS 2
#define TOMATIS_DEV_RUN_FRAMES 3
#define TOMATIS_DEV_LEVELS_LEGACY 4
#define TOMATIS_DEV_GATE_TF 5
#define TOMATIS_DEV_MH_PARTS 6
#define TOMATIS_DEV_FORCE_LDS 7
#define TOMATIS_DEV_P64 8
#define TOMATIS_DEV_ALPHA_SEQ 9
#define TOMATIS_DEV_GAIN_LDS 10
#define TOMATIS_DEV_FUSE_LIMITER 11
#define TOMATIS_DEV_WG 12
#define TOMATIS_DEV_SLOTS 13           /* resident run slots assumed by the plan (0: the device's) */
#define TOMATIS_DEV_FUSED_LEVELS 14    /* 0: tomatis_stft_ola_gated declines (host two-pass) */
#define TOMATIS_DEV_FUSED_4096 15      /* 1: the gated calls take n_fft 4096 / hop 1024 (slower) */
int tomatis_set_dev_option(int32_t key, int32_t value);
/* The current override of key (-1: default, or an unknown key). */
int32_t tomatis_get_dev_option(int32_t key);

/* FLAC frames encoded on the device (row f1 egress; src/process_tomatis.py:
 * 242-251,357 write the output through libsndfile's FLAC PCM_24 encoder).
 * Byte for byte the frames tomatis_flac_encode (include/tomatis_flac.h) writes
 * for the same interleaved int32 PCM: 4096-sample blocks, frame number = block
 * index.  1-2 channels, 4-24 bits (TOMATIS_E_UNSUPPORTED otherwise).
 *   tomatis_flacd_workspace_bytes: device workspace for `frames` (plans).
 *   tomatis_flacd_plan: per block its plan (into ws) and frame size in bytes
 *     into frame_bytes[block] (device, uint32); 0xFFFFFFFF marks a block with a
 *     sample outside the bit depth, 0xFFFFFFFE one the device writer cannot
 *     hold (encode the stream on the host then).
 *   tomatis_flacd_write: every frame at byte frame_off[block] (device, int64,
 *     the exclusive prefix sum of the sizes) of `out`, which the caller zeroes
 *     and sizes to the total rounded up to a multiple of 4 bytes.
 * The caller writes "fLaC" + STREAMINFO (block / frame size extremes, total
 * samples, MD5 zero) in front, as tomatis_flac_encode does. */
int64_t tomatis_flacd_workspace_bytes(int64_t frames, int32_t ch);
int tomatis_flacd_plan(const int32_t* pcm, int64_t frames, int32_t ch, int32_t bps, void* ws,
                       uint32_t* frame_bytes, void* hip_stream);
int tomatis_flacd_write(const int32_t* pcm, int64_t frames, int32_t ch, int32_t bps,
                        const void* ws, const int64_t* frame_off, uint8_t* out,
                        void* hip_stream);

/* FLAC frames decoded on the device (row f1 ingest; src/process_tomatis.py:
 * 225-235 read the input through libsndfile).  The grammar and checks of
 * tomatis_flac_decode (include/tomatis_flac.h), for 1-2 channels and 4-24 bits
 * (TOMATIS_E_UNSUPPORTED otherwise).  d: the file's bytes in device memory,
 * 4-byte aligned, followed by >= 8 zero bytes; ch / bps from STREAMINFO.
 *   tomatis_flacd_find: every byte position in [first, len) with a frame sync
 *     code whose header parses and matches its CRC-8, appended (unordered) to
 *     cand (int64 offsets, at most cap; *count = all found, device int32,
 *     zeroed by the caller).
 *   tomatis_flacd_scan: per candidate (sorted or not) info[4i..4i+3] = frame
 *     bytes (0: no frame: a sub-frame, residual or CRC-16 check failed), first
 *     sample (frame number x nominal for fixed-blocksize frames), block size,
 *     blocking strategy bit.
 *   tomatis_flacd_decode: the frames at byte offsets frames[0, nf) (verified,
 *     chained: the caller checks that they tile the stream) into interleaved
 *     int32 pcm (samples >= max_frames dropped; an LPC frame reaching past
 *     max_frames is not decoded: it predicts from its own output); *err
 *     (device, zeroed by the caller) != 0 if a frame was not decoded. */
int tomatis_flacd_find(const uint8_t* d, int64_t len, int64_t first, int32_t ch, int32_t bps,
                       int64_t* cand, int32_t cap, int32_t* count, void* hip_stream);
int tomatis_flacd_scan(const uint8_t* d, int64_t len, const int64_t* cand, int32_t nc,
                       int32_t ch, int32_t bps, int64_t nominal, int64_t* info,
                       void* hip_stream);
int tomatis_flacd_decode(const uint8_t* d, int64_t len, const int64_t* frames, int32_t nf,
                         int32_t ch, int32_t bps, int64_t nominal, int32_t* pcm,
                         int64_t max_frames, int32_t* err, void* hip_stream);

/* max |x| over n floats as float bits (out zeroed by caller). */
int tomatis_absmax(const float* x, int64_t n, uint32_t* out_bits, void* hip_stream);

/* max |x| of every stream of the plan (stream table in_off / n * ch), one
 * launch: out_bits[s] as float bits (zeroed by caller).  Replaces the per-file
 * np.max(np.abs(x)) of src/process_tomatis_adaptive.py:201 for a batch. */
int tomatis_absmax_streams(tomatis_plan_t plan, const float* x, uint32_t* out_bits,
                           void* hip_stream);

/* HBM bandwidth probe: y = x for n floats (n % 4 == 0, both 16-byte aligned)
 * with 16-byte streaming loads and stores -- bench.py times it to report the
 * roofline against a measured copy bandwidth beside the 8 TB/s spec.  Replaces
 * nothing in the reference. */
int tomatis_copy_probe(const float* x, float* y, int64_t n, void* hip_stream);

/* y[i] = x[i] * scale (float32), n floats (layer-2 gain-protect copy). */
int tomatis_scale_copy(const float* x, float* y, int64_t n, float scale, void* hip_stream);

/* File-boundary sample conversion (libsndfile's
 * normalisation, src/process_tomatis.py:225-251 reads float32 and writes
 * PCM_24): out = pcm / 2^(bps-1) (float32, correctly rounded), and
 * out = clip(rint(x * (2^(bps-1) - 1)), -2^(bps-1), 2^(bps-1) - 1). */
int tomatis_pcm_to_float(const int32_t* pcm, int64_t n, int32_t bps, float* out, void* hip_stream);
int tomatis_float_to_pcm(const float* x, int64_t n, int32_t bps, int32_t* out, void* hip_stream);

/* Deterministic synthetic PCM (twin of tomatis_audio_processor_amd/synth.py):
 * samples [start, start+n) of stream `seed`, ch channels, interleaved. */
int tomatis_synth_fill(float* x, int64_t n, int32_t ch, int32_t sr, uint32_t seed,
                       int64_t start, void* hip_stream);

/* ---------------------------------------------------------------------------
 * Analysis spectra (tm_analysis.hip).  Frames
 * f = 0 .. F-1 start at sample f*hop, F = 1 + (n - n_fft) / hop (n >= n_fft);
 * x (and y) float32 [n][ch] interleaved.  n_fft: spectra take powers of two
 * in [16, 16384] and other lengths in [16, 8192] (Bluestein's chirp-z over a
 * power of two >= 2 n_fft - 1, in LDS); tomatis_an_frame_r any n_fft in
 * [1, 16384].  Outside: TOMATIS_E_UNSUPPORTED.
 * ------------------------------------------------------------------------- */
#define TOMATIS_AN_LEVEL_CHMEAN 0     /* mono = sqrt(mean_c x_c^2)        validate_layer1.py:304-306 */
#define TOMATIS_AN_LEVEL_POWER_MONO 1 /* mono = sqrt(0.5(L^2+R^2)+1e-12)  layer2_analyze_eq.py:71, compare_audio.py:7-10 */
#define TOMATIS_AN_SIG_RAW 0          /* spectrum of x itself (ch must be 1)                    */
#define TOMATIS_AN_SIG_POWER_MONO 1   /* spectrum of power_mono(x) (ch must be 2)               */
#define TOMATIS_AN_MAG 0              /* |rfft(win*s)|                    compare_audio.py:16-21 */
#define TOMATIS_AN_LOGPOW 1           /* 10 log10(|rfft(win*s)|^2+1e-12)  layer2_analyze_eq.py:76-79 */
#define TOMATIS_AN_RATIO 2            /* mean_c|Y_c| / max(mean_c|X_c|, 1e-10)  validate_layer1.py:340-355 */

/* Per-frame r = sqrt(mean(mono^2) + 1e-12) in numpy's pairwise order
 * (bit-exact); x scaled by `scale` first.  r_out: F floats. */
int tomatis_an_frame_r(const float* x, int64_t n, int32_t ch, int32_t n_fft, int32_t hop,
                       int32_t level_mode, float scale, float* r_out, void* hip_stream);

/* mask[f] = level predicate on r bits (dsp.gate_bits form) && (cls == NULL ||
 * cls[f] == cls_want); keep_above = 1: level >= T <=> (b >= thr) xor b in exc;
 * keep_above = 0: level > T <=> !((b <= thr) xor b in exc).  exc_host: up to 4
 * host words.  count (device int32): number of kept frames. */
int tomatis_an_select(const float* r, int32_t n_frames, uint32_t thr_bits,
                      const uint32_t* exc_host, int32_t n_exc, int32_t keep_above,
                      const int8_t* cls, int32_t cls_want, uint8_t* mask, int32_t* count,
                      void* hip_stream);

/* Per-frame spectra rows out[F][n_fft/2+1] (TOMATIS_AN_MAG / _LOGPOW of the
 * signal chosen by sig_mode, scaled by `scale`; TOMATIS_AN_RATIO of y over x). */
int tomatis_an_spectra(const float* x, const float* y, int64_t n, int32_t ch, int32_t n_fft,
                       int32_t hop, int32_t kind, int32_t sig_mode, float scale,
                       const float* win, float* out, void* hip_stream);

/* out[k] = (sum over f in order of spec[f][k]) / F, float32 (np.mean(axis=0)). */
int tomatis_an_frame_mean(const float* spec, int32_t n_frames, int32_t n_bins, float* out,
                          void* hip_stream);

/* Workspace (uint32 words) for tomatis_an_frame_median. */
int64_t tomatis_an_median_work_words(int32_t n_bins);

/* out[k] = np.median over the n_sel frames with mask[f] != 0 (mask NULL: all
 * frames, n_sel = F) of spec[f][k]; even counts average the two middle values
 * in float32 like numpy. */
int tomatis_an_frame_median(const float* spec, int32_t n_frames, int32_t n_bins,
                            const uint8_t* mask, int32_t n_sel, uint32_t* work, float* out,
                            void* hip_stream);

/* ---------------------------------------------------------------------------
 * Gate calibration (src/calibrate_to_baseline_v2.py).
 * ------------------------------------------------------------------------- */

/* Per-frame band energies of rfft(win * power_mono(x)) for stereo x
 * (stft_band_tilt, calibrate_to_baseline_v2.py:17-31): out[f][0] = sum of the
 * float32 power re^2+im^2 over bins [lo0, lo1), out[f][1] over [hi0, hi1).
 * Frames and n_fft as tomatis_an_spectra. */
int tomatis_an_band_energy(const float* x, int64_t n, int32_t n_fft, int32_t hop,
                           int32_t lo0, int32_t lo1, int32_t hi0, int32_t hi1,
                           const float* win, float* out, void* hip_stream);

/* One candidate of the gate-calibration grid: thresholds already rounded to
 * float32 (numpy compares an np.float32 level with a Python float in float32),
 * up-delay in samples (int(round(sr * up_ms / 1000))), level row index. */
typedef struct TomatisGateCand {
    int32_t level_row;    /* row of `levels` (one per searched gain)          */
    float t_on, t_off;    /* float32(T + hyst/2), float32(T - hyst/2)         */
    int32_t pad_;
    int64_t up_delay;     /* samples                                          */
} TomatisGateCand;

/* For every candidate c: the standard gate automaton of simulate_state
 * (calibrate_to_baseline_v2.py:84-109) over frames i < n_fit with levels
 * levels[c.level_row * n_fit + i] (float32) and frame starts starts[i];
 * out[2c] = #frames whose state != target[i] (1/2; 0 if target is NULL),
 * out[2c+1] = #switches; states (optional, [n_cand][n_fit] u8) = the state
 * sequence itself.  All buffers device-resident; cands: n_cand records. */
int tomatis_cal_gate_grid(const float* levels, int32_t n_fit, const int64_t* starts,
                          const int32_t* target, const TomatisGateCand* cands, int32_t n_cand,
                          int32_t* out, uint8_t* states, void* hip_stream);

#ifdef __cplusplus
}
#endif
#endif /* TOMATIS_HIP_H */
