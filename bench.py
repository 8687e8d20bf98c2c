#!/usr/bin/env python3
"""Benchmark: Msamples/s of the end-to-end STFT-gate-OLA hot path on MI355X.

Default workload (BASELINE.json configs[1], "C2"): one 60-min stereo 44.1 kHz
stream per GPU, standard mode (process_tomatis), n_fft=2048, hop=512, Hann,
gate_ui=50 (log_percent, -40 dBFS), +-15 dB tilt.  A step = one pass of the
whole device chain over the resident input: the gate look-back pre-kernel, then
the fused levels -> gate -> STFT-gain-ISTFT-OLA-normalise -> per-chunk limiter
kernel (tomatis_stft_ola_gated; shapes it declines run levels -> gate scan ->
fused transform + limiter).  Input is seeded synthetic PCM generated on the
device before timing.

Contract: `python bench.py --gpus N --steps K --warmup W`; for N > 1 launched
by torch.distributed.run (one rank per GPU, RCCL).  Multi-GPU = weak scaling:
each rank owns its own stream(s); the only collective is an all_gather of the
per-stream manifest records (after the timed region).  Rank 0 prints ONE JSON
line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0         # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP32_PEAK_TFLOPS = 157.3      # MI355X vector FP32 (no packed-math doubling on gfx950)

WORKLOADS = {
    # name: (streams per GPU, seconds, sr, ch, mode, n_fft, hop, description)
    "c2": (1, 3600, 44100, 2, "standard", 2048, 512,
           "C2: 1 x 60 min stereo 44.1 kHz per GPU, standard mode, n_fft 2048 hop 512, "
           "gate_ui 50 (log_percent)"),
    "c4": (64, 300, 48000, 2, "standard", 2048, 512,
           "C4: 64 x 5 min stereo 48 kHz per GPU (512 over 8 GPUs), standard, 2048/512"),
    # C4 with stream 17 a sine hovering at the gate threshold for all 5 minutes
    # (every run of it chains its look-back: no two-pass fallback)
    "c4h": (64, 300, 48000, 2, "standard", 2048, 512,
            "C4 + one hovering stream: 64 x 5 min stereo 48 kHz per GPU, stream 17 a "
            "1 kHz sine at the gate threshold (-40 dBFS), standard, 2048/512"),
    # the whole 512-stream C4 batch on ONE GPU (14.4 M frames: more than the
    # 2048 resident run slots x 4096 frames, so runs take two rounds and every
    # look-back still chains), clean and with the hovering stream 17
    "c4all": (512, 300, 48000, 2, "standard", 2048, 512,
              "C4 whole batch on one GPU: 512 x 5 min stereo 48 kHz, standard, 2048/512"),
    "c4allh": (512, 300, 48000, 2, "standard", 2048, 512,
               "C4 whole batch on one GPU + one hovering stream: 512 x 5 min stereo 48 kHz, "
               "stream 17 a 1 kHz sine at the gate threshold (-40 dBFS), standard, 2048/512"),
    "c5x": (16, 300, 96000, 2, "xfade", 4096, 1024,
            "C5 stage 1: 16 x 5 min stereo 96 kHz per GPU, xfade 500 ms, 4096/1024"),
    "c3": (64, 300, 44100, 2, "adaptive", 2048, 512,
           "C3: 64 x 5 min stereo 44.1 kHz per GPU, adaptive (bisection threshold, min-hold "
           "250 ms, xfade 500 ms), 2048/512"),
    "c5": (16, 300, 96000, 2, "chain", 4096, 1024,
           "C5: 16 x 5 min stereo 96 kHz per GPU (128 over 8 GPUs), xfade 500 ms -> layer2b "
           "residual EQ, 4096/1024"),
    # strong scaling: ONE 60-min stream time-sharded over all ranks
    "c2ts": (1, 3600, 44100, 2, "timeshard", 2048, 512,
             "C2 time-sharded: one 60 min stereo 44.1 kHz stream split over all ranks, "
             "standard mode, n_fft 2048 hop 512 (gate-summary all_gather + chunk-peak "
             "all_reduce)"),
}


def flops_per_ch_sample(n_fft: int, hop: int) -> float:
    """per frame-channel 2*2.5*n*log2(n) + 2n + 2(n/2+1) + n."""
    n = n_fft
    per_frame_ch = 2 * 2.5 * n * np.log2(n) + 2 * n + 2 * (n // 2 + 1) + n
    return per_frame_ch / hop


class ChainC5:
    """C5 per step: xfade (500 ms, linear gate at -40 dBFS) then the layer-2b
    residual EQ (src/layer2b_apply_residual_eq.py:99-160: no pad, static row)
    on the stage-1 output, all device-resident.  The residual curve is a fixed
    synthetic diff spectrum (+-4 dB ripple), smoothed and clamped by the
    reference's own rules (dsp.smooth_on_logfreq / build_eq_from_residual).
    ``marks`` time the stage-1 transform (the dominant launch).

    ``pipelined``: stage 1 is a batch pipeline (pass k's transform limits pass
    k-1's output), so stage 2 of pass k-1 runs after stage 1 of pass k, on
    that pass's (alternating) output buffer; flush() limits the last stage-1
    output and runs its stage 2.  K steps + flush = K passes of both stages."""

    def __init__(self, engine, ss, sr, n_fft, hop, pipelined=True):
        from tomatis_audio_processor_amd import dsp
        self.s1 = engine.GatePipeline(ss, gate_ui=50, gate_offset=-90, n_fft=n_fft, hop=hop,
                                      xfade_ms=500.0, pipelined=pipelined)
        res = self.s1.result()
        rf = np.geomspace(20.0, sr / 2, 400)
        rd = 4.0 * np.sin(np.log2(rf / 20.0) * 1.7) * np.exp(-rf / 12000.0)
        res_s = dsp.smooth_on_logfreq(rf, rd, win=41)
        lin, _ = dsp.build_eq_from_residual(np.fft.rfftfreq(n_fft, 1.0 / sr), rf, res_s)
        bufs = self.s1._ys if self.s1.pipelined else [self.s1.y]
        self.s2 = {}
        for y in bufs:  # one stage-2 pipeline per stage-1 output buffer
            ss2 = engine.StreamSet(x=y, offs=res.out_offs, lens=res.out_lens, ch=ss.ch, sr=sr)
            self.s2[y.data_ptr()] = engine.StaticEqPipeline(ss2, lin, n_fft=n_fft, hop=hop,
                                                            pad=False)
        self.pending2 = None  # stage-1 buffer whose stage 2 waits for its limiter

    @property
    def pipelined(self):
        return self.s1.pipelined

    def run(self, marks=None, check_device=True):
        prev = self.s1.y if self.s1.pending else None
        self.s1.run(marks=marks, check_device=check_device)
        if not self.s1.pending:  # unpipelined: stage 2 on this pass at once
            return self.s2[self.s1.y.data_ptr()].run(check_device=check_device)
        if prev is not None:     # pass k-1's output is final now
            self.s2[prev.data_ptr()].run(check_device=check_device)
        return None

    def flush(self):
        """the last pass: stage 1's limiter, then its stage 2 (that result)"""
        if self.s1.pending:
            y = self.s1.y
            self.s1.flush()
            return self.s2[y.data_ptr()].run(check_device=False)
        return None

    def finish(self):
        bits = self.s1.finish()
        for p in self.s2.values():  # (error bits OR together: distinct bits survive)
            bits |= p.finish()
        return bits

    def result(self):
        return self.s1.result()


def plans_of(pipe):
    """Every tomatis plan a bench pipeline launches on."""
    if isinstance(pipe, ChainC5):
        return [pipe.s1.plan] + [p.plan for p in pipe.s2.values()]
    if hasattr(pipe, "pipes"):          # AdaptiveGroups
        return [p.plan for p in pipe.pipes]
    if hasattr(pipe, "rn"):             # timeshard.RankStep
        return [pipe.rn.pipe.plan]
    return [pipe.plan]


def dist_init():
    import torch
    import torch.distributed as dist
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if ws > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend="nccl", rank=rank, world_size=ws,
                                device_id=torch.device("cuda", local))
    return rank, ws, local


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def _host_cores() -> int:
    """Cores this process may use: the affinity mask, capped at the GPU box's
    per-GPU CPU share (16)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def _pool_task(args):
    """One stream through the oracle in a worker process (1 BLAS/OMP thread)."""
    seed, n, ch, sr, n_fft, hop = args
    from oracle import tomatis_oracle as orc
    from tomatis_audio_processor_amd.synth import synth_stream
    x = synth_stream(seed, n, ch, sr)
    t0 = time.perf_counter()
    orc.process_standard(x, sr, gate_ui=50, n_fft=n_fft, hop=hop)
    return time.perf_counter() - t0


def _file_task(args):
    """The CPU file -> file path for one FLAC PCM_24 file in a worker process
    (one thread, codec included): host FLAC decode -> the oracle's
    process_standard (levels, gate, STFT filter, OLA, per-chunk limiter) ->
    PCM_24 quantisation + host FLAC encode -> write; the reference's own file
    path, src/process_tomatis.py:225-251,433-457, with the package's codec in
    place of libsndfile (absent here)."""
    src, dst, n_fft, hop = args
    os.environ["TOMATIS_FLAC_THREADS"] = "1"
    from oracle import tomatis_oracle as orc
    from tomatis_audio_processor_amd import audio_io
    t0 = time.perf_counter()
    x, sr = audio_io.read(src)
    ref = orc.process_standard(x, sr, gate_ui=50, n_fft=n_fft, hop=hop)
    audio_io.write(dst, ref["y"], sr, "FLAC", "PCM_24")
    return time.perf_counter() - t0


def cpu_file_baseline(file_s: int, sr: int, n_fft: int, hop: int, ch: int):
    """CPU file -> file (BASELINE.md §4.5's separate end-to-end number): FLAC
    PCM_24 files of ``file_s`` s (seeds 1000..; written by the host codec
    before timing), one process on one core, then P = host cores processes
    with one file each (aggregate = all channel-samples / the slowest worker).
    The GPU's file -> file rate is tools/bench_file.py's."""
    import multiprocessing as mp
    import tempfile
    from tomatis_audio_processor_amd import audio_io
    from tomatis_audio_processor_amd.synth import synth_stream
    P = _host_cores()
    n = file_s * sr
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as d:
        srcs = []
        for i in range(P):
            f = os.path.join(d, f"in{i}.flac")
            audio_io.write(f, synth_stream(1000 + i, n, ch, sr), sr, "FLAC", "PCM_24")
            srcs.append(f)
        dt1 = _file_task((srcs[0], os.path.join(d, "one.flac"), n_fft, hop))
        pool_val = None
        if P > 1:
            tasks = [(f, os.path.join(d, f"out{i}.flac"), n_fft, hop) for i, f in enumerate(srcs)]
            with mp.get_context("spawn").Pool(P) as pool:
                dts = pool.map(_file_task, tasks, chunksize=1)
            pool_val = round(P * n * ch / max(dts) / 1e6, 3)
    return {"value": pool_val if pool_val is not None else round(n * ch / dt1 / 1e6, 3),
            "unit": "Msamples/s", "cores": P if pool_val is not None else 1,
            "single_core": round(n * ch / dt1 / 1e6, 3),
            "sample": f"{P} FLAC PCM_24 files of {file_s} s stereo {sr} Hz: host FLAC decode -> "
                      f"oracle process_standard -> PCM_24 FLAC encode -> write, one thread per "
                      f"process ({P} processes, one file each); single_core: one of them alone"}


def cpu_baseline(sample_s: int, sr: int, n_fft: int, hop: int, ch: int, x_host=None,
                 pool_s: int = 300):
    """The oracle (a 'port' of the reference loop) on the host:
    (1) one core over the first ``sample_s`` s of the bench stream; (2) file-
    parallel over P = host cores, one process per core, P streams of ``pool_s``
    s each (seeds 1000..), aggregate = all channel-samples / the slowest
    worker's busy time."""
    import multiprocessing as mp
    from oracle import tomatis_oracle as orc
    from tomatis_audio_processor_amd.synth import synth_stream
    n = sample_s * sr
    x = x_host if x_host is not None else synth_stream(1000, n, ch, sr)
    t0 = time.perf_counter()
    orc.process_standard(x, sr, gate_ui=50, n_fft=n_fft, hop=hop)
    dt = time.perf_counter() - t0
    one = round(n * ch / dt / 1e6, 3)
    P = _host_cores()
    pool_val, pool_note = None, ""
    if P > 1 and pool_s > 0:
        for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS"):
            os.environ[k] = "1"
        npool = pool_s * sr
        tasks = [(1000 + i, npool, ch, sr, n_fft, hop) for i in range(P)]
        with mp.get_context("spawn").Pool(P) as pool:
            dts = pool.map(_pool_task, tasks, chunksize=1)
        pool_val = round(P * npool * ch / max(dts) / 1e6, 3)
        pool_note = (f"; {P} processes x one {pool_s} s stream each (seeds 1000..{999 + P}), "
                     f"slowest worker {max(dts):.2f} s")
    return {"value": pool_val if pool_val is not None else one, "unit": "Msamples/s",
            "cores": P if pool_val is not None else 1, "kind": "port",
            "single_core": one, "cpu_model": _cpu_model(), "numpy": np.__version__,
            "sample": f"oracle/tomatis_oracle.process_standard (numpy {np.__version__}) on "
                      f"{_cpu_model()}: 1 core over the first {sample_s} s of stream seed 1000 "
                      f"({n} x {ch} ch, {sr} Hz) in {dt:.2f} s = {one} Msamples/s" + pool_note}


def load_traffic(workload: str):
    """HBM bytes per launch of the fused kernel from the committed rocprofv3 PMC
    summary (profiles/pmc_traffic.json), corrected as MI355X_MICROARCH.md
    prescribes (FETCH_SIZE x 2 for wide streaming reads).  None if absent."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            return json.load(f).get(workload, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def relaunch(n: int) -> int:
    """``--gpus N`` without a launcher: start torch.distributed.run with N
    ranks as a CHILD process (nothing here has touched the GPU) and relay its
    output and exit code."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # (40 passes: a batch pipeline's drain -- the last pass's standalone limiter,
    # ~0.6 ms on C2 -- is inside the timed region, amortised as in a real job)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--cpu-sample-s", type=int, default=3600,
                    help="seconds of audio for the 1-core CPU baseline (0 disables the baseline)")
    ap.add_argument("--input-gain", type=float, default=1.0,
                    help="scale the synthetic input (e.g. 0.05: no limiter chunk engages; "
                         "PMC traffic runs)")
    ap.add_argument("--cpu-pool-s", type=int, default=300,
                    help="seconds of audio per worker for the all-cores CPU baseline")
    ap.add_argument("--cpu-file-s", type=int, default=120,
                    help="seconds per FLAC file of the CPU file->file baseline (0 disables)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="standard / adaptive: every pass applies its own limiter (no batch "
                         "pipeline: tomatis_stft_ola_gated / _limited instead of _pipelined)")
    ap.add_argument("--inputs", type=int, default=2,
                    help="distinct synthetic inputs of the workload's shape, used in turn by the "
                         "passes (a pipeline of different files, not one file re-processed)")
    ap.add_argument("--single-steps", type=int, default=10,
                    help="also time this many unpipelined passes (a job of ONE file: the limiter "
                         "ends the pass) with their own pipeline; 0 disables")
    ap.add_argument("--dev", action="append", default=[], metavar="NAME=VALUE",
                    help="development override (TOMATIS_DEV_<NAME>, A/B experiments); "
                         "recorded in the JSON line's config")
    a = ap.parse_args()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        raise SystemExit(relaunch(a.gpus))
    ws_env = int(os.environ.get("WORLD_SIZE", "1"))
    if ws_env != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={ws_env}: launch one rank per GPU")

    import torch
    import torch.distributed as dist
    rank, ws, local = dist_init()
    from tomatis_audio_processor_amd import engine
    from tomatis_audio_processor_amd._lib import set_dev_option
    for kv in a.dev:
        k, v = kv.split("=", 1)
        set_dev_option(k.upper(), int(v))

    nstr, secs, sr, ch, mode, n_fft, hop, desc = WORKLOADS[a.workload]
    n = secs * sr
    if mode == "timeshard":
        from tomatis_audio_processor_amd import timeshard
        from tomatis_audio_processor_amd._lib import check, lib, ptr, stream_handle
        sh = timeshard.plan_shards(n, n_fft, hop, ws)[rank]
        xs = torch.empty((sh.hi - sh.lo) * ch, dtype=torch.float32, device="cuda")
        check(lib().tomatis_synth_fill(ptr(xs), sh.hi - sh.lo, ch, sr, 1000, sh.lo,
                                       stream_handle()), "synth_fill")
        pipe = timeshard.RankStep(xs, sr, n, rank, ws, ch=ch, gate_ui=50, n_fft=n_fft, hop=hop)
        ss = pipe.rn.pipe.ss
    else:
        ss = engine.StreamSet.synthetic(nstr, n, ch, sr, seed0=1000 + rank * nstr)
        if a.input_gain != 1.0:
            ss.x = engine.scale_copy(ss.x, a.input_gain)
        if a.workload in ("c4h", "c4allh"):
            o, amp = ss.offs[17], np.sqrt(2.0) * 10.0 ** (-40.0 / 20.0)
            t = torch.arange(n, dtype=torch.float64, device="cuda") / sr
            s = (amp * torch.sin(2 * np.pi * 1000.0 * t)).to(torch.float32)
            ss.x[o:o + 2 * n] = torch.stack([s, s], 1).reshape(-1)
    # the passes take distinct inputs in turn (seeds differ): input 0 is the one
    # generated above, the others fresh buffers of the same geometry.  HBM
    # budget (80 % of the device): inputs + two pipelined outputs + the one-file
    # pipeline's output; the extras go first when a workload does not fit
    set_bytes = 4 * n * ch * nstr
    budget = 0.8 * torch.cuda.get_device_properties(torch.cuda.current_device()).total_memory
    if (a.inputs + 3) * set_bytes > budget:
        a.single_steps = 0
    a.inputs = int(max(1, min(a.inputs, budget // set_bytes - (3 if a.single_steps else 2))))
    inputs = [ss.x]
    if mode != "timeshard":
        for j in range(1, max(1, a.inputs)):
            o = engine.StreamSet.synthetic(nstr, n, ch, sr, seed0=1000 + rank * nstr + 7919 * j)
            inputs.append(engine.scale_copy(o.x, a.input_gain) if a.input_gain != 1.0 else o.x)
            if a.workload in ("c4h", "c4allh"):
                inputs[-1][ss.offs[17]:ss.offs[17] + 2 * n] = ss.x[ss.offs[17]:ss.offs[17] + 2 * n]
    stages = 2 if mode == "chain" else 1

    def make_pipe(pipelined):
        if mode == "standard":
            # batch pipeline: pass k+1's transform applies pass k's limiter in its
            # frame loops; the timed region ends with flush() (the last pass's limiter)
            return engine.GatePipeline(ss, gate_ui=50, n_fft=n_fft, hop=hop, pipelined=pipelined)
        if mode == "xfade":
            # batch pipeline (two-pass chain, n_fft 4096: the partner blocks through
            # VGPRs); the timed region ends with flush()
            return engine.GatePipeline(ss, gate_ui=50, gate_offset=-90, n_fft=n_fft, hop=hop,
                                       xfade_ms=500.0, pipelined=pipelined)
        if mode == "adaptive":
            # two stream groups: one group's host phase overlaps the other's device
            # work (batch pipeline as in standard mode: the global limiter of pass k
            # in pass k+1's transforms)
            return engine.AdaptiveGroups(ss, groups=int(os.environ.get("TOMATIS_C3_GROUPS", "2")),
                                         n_fft=n_fft, hop=hop, pipelined=pipelined)
        if mode == "chain":
            return ChainC5(engine, ss, sr, n_fft, hop, pipelined=pipelined)
        return pipe  # timeshard: built above

    pipe = make_pipe(not a.no_pipeline)
    torch.cuda.synchronize()

    def set_input(p, k):
        """pass k of pipeline p reads input k mod len(inputs)"""
        if len(inputs) < 2:
            return
        for q in getattr(p, "pipes", None) or [getattr(p, "s1", p)]:
            q.ss.x = inputs[k % len(inputs)]

    for w in range(a.warmup):
        set_input(pipe, w)
        pipe.run()          # device error word checked after every warm-up pass
    if hasattr(pipe, "flush"):
        pipe.flush()        # pipelined: the timed region starts with nothing pending
    torch.cuda.synchronize()
    if ws > 1:
        dist.barrier()
    # live kernel timing on every 4th step from the second (steady state of a
    # batch pipeline: the first timed pass has no previous batch to limit): a
    # timing event's record stalls the queue for ~6 us, which is measurement
    # overhead, not the workload's
    every = 4 if a.steps >= 8 else 1
    marks = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
             if k % every == min(1, every - 1) else None for k in range(a.steps)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(a.steps):
        set_input(pipe, k)
        pipe.run(marks=marks[k], check_device=False)
    if hasattr(pipe, "flush"):
        pipe.flush()        # pipelined: the last pass's limiter, inside the timed region
    torch.cuda.synchronize()
    if ws > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    # the timed passes' device error word, read once after the timed region: a
    # fired check (fused-limiter wait / exchange barrier) invalidates the line
    dev_err = 0
    for pl in plans_of(pipe):
        dev_err |= pl.error_bits()
    kern_ms = float(np.mean([m[0].elapsed_time(m[1]) for m in marks if m is not None]))
    if ws > 1:
        tt = torch.tensor([elapsed, kern_ms, dev_err], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed, kern_ms, dev_err = float(tt[0]), float(tt[1]), int(tt[2])

    # HBM copy bandwidth measured in this process (roofline.achievable_peak,
    # SURVEY §8(d)): the timed launch's input copied by tomatis_copy_probe
    from tomatis_audio_processor_amd._lib import check as _check, lib as _lib, ptr as _ptr, stream_handle
    cp_src = inputs[0][: min(inputs[0].numel() // 4, 1 << 27) * 4]  # <= 2 GiB, >> the MALL
    cp_dst = torch.empty_like(cp_src)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for j in range(7):
        if j == 2:
            ev[0].record()
        _check(_lib().tomatis_copy_probe(_ptr(cp_src), _ptr(cp_dst), cp_src.numel(), stream_handle()),
               "copy_probe")
    ev[1].record()
    torch.cuda.synchronize()
    copy_gbs = 2.0 * 4.0 * cp_src.numel() * 5 / (ev[0].elapsed_time(ev[1]) * 1e-3) / 1e9
    del cp_dst

    # a job of ONE file: unpipelined passes of the same workload (each ends with
    # its own limiter), their own pipeline; the headline above is a pipeline of
    # distinct files (pass k+1 limits pass k inside its transform), as batch.py
    # runs a multi-file job
    one = None
    if a.single_steps > 0 and mode != "timeshard" and not a.no_pipeline:
        p1 = make_pipe(False)
        for w in range(2):
            set_input(p1, w)
            p1.run()
        torch.cuda.synchronize()
        if ws > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for k in range(a.single_steps):
            set_input(p1, k)
            p1.run(check_device=False)
        torch.cuda.synchronize()
        if ws > 1:
            dist.barrier()
        el1 = time.perf_counter() - t0
        for pl in plans_of(p1):
            dev_err |= pl.error_bits()
        if ws > 1:
            tt = torch.tensor([el1], dtype=torch.float64, device="cuda")
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el1 = float(tt[0])
        one = {"ms_per_step": round(el1 / a.single_steps * 1e3, 4),
               "value": round(n * ch * nstr * ws * a.single_steps / el1 / 1e6, 1),
               "unit": "Msamples/s", "steps": a.single_steps,
               "what": "one file per job: unpipelined passes (each pass applies its own "
                       "limiter), no previous file to overlap with"}
        del p1

    # per-stream manifest: (rank, stream, frames, C2 frames, max chunk peak bits)
    res = pipe.result()
    recs = []
    for i in range(nstr):
        st = res.states[res.frame_base[i]:res.frame_base[i] + res.n_frames[i]]
        pk = res.chunk_peaks[res.chunk_base[i]:res.chunk_base[i] + res.n_chunks[i]].max()
        recs.append(torch.stack([torch.tensor(rank, device="cuda"), torch.tensor(i, device="cuda"),
                                 torch.tensor(res.n_frames[i], device="cuda"),
                                 (st == 2).sum(), pk.to(torch.int64)]))
    man = torch.stack(recs).to(torch.int64)
    if ws > 1:
        allm = [torch.empty_like(man) for _ in range(ws)]
        dist.all_gather(allm, man)
        man = torch.cat(allm)
    man = man.cpu().numpy()

    strong = mode == "timeshard"
    samples_per_step = n * ch * nstr * (1 if strong else ws)
    value = samples_per_step * a.steps / elapsed / 1e6
    ms_per_step = elapsed / a.steps * 1e3
    # roofline of the dominant kernel (fused STFT-OLA), per launch on this rank
    alg_bytes = 8.0 * (ss.lens[0] * ch if strong else n * ch * nstr)  # the timed launch
    achieved_gbs = alg_bytes / (kern_ms * 1e-3) / 1e9
    traffic = load_traffic(a.workload)
    flops = flops_per_ch_sample(n_fft, hop) * alg_bytes / 8.0
    tflops = flops / (kern_ms * 1e-3) / 1e12

    if rank == 0:
        cpu = None
        if a.cpu_sample_s > 0 and mode == "standard" and not strong:
            xs = ss.x[:a.cpu_sample_s * sr * ch].cpu().numpy().reshape(-1, ch)
            cpu = cpu_baseline(a.cpu_sample_s, sr, n_fft, hop, ch, x_host=xs, pool_s=a.cpu_pool_s)
            if a.cpu_file_s > 0:
                cpu["file_to_file"] = cpu_file_baseline(a.cpu_file_s, sr, n_fft, hop, ch)
        out = {
            "metric": "Msamples/s (44.1 kHz stereo) end-to-end STFT-gate-OLA; % HBM roofline",
            "value": round(value, 1), "unit": "Msamples/s", "n_gpus": ws, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "strong" if strong else "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (seeded device-generated noise, -20/-60 dBFS alternating 1.5 s)"
                    + (f", x{a.input_gain:g}" if a.input_gain != 1.0 else "")
                    + (f"; {len(inputs)} distinct inputs taken in turn by the passes"
                       if len(inputs) > 1 else ""),
            "config": {"workload": desc, "streams_per_gpu": nstr, "samples_per_channel": n,
                       "channels": ch, "sr": sr, "mode": mode, "n_fft": n_fft, "hop": hop,
                       "parallelism": (f"time-sharded x{ws} (RCCL gate all_gather + peak "
                                       f"all_reduce)" if strong else
                                       f"file-parallel x{ws} (RCCL manifest all_gather)"),
                       "fused_levels": bool(getattr(pipe, "gated_used", False)),
                       "pipelined": bool(getattr(pipe, "pipelined", False)),
                       "gate_fallbacks": int(getattr(pipe, "gate_fallbacks", 0)),
                       **({"dev_overrides": a.dev} if a.dev else {})},
            "roofline": {"bound": "hbm", "achieved": round(achieved_gbs, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved_gbs / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "achievable_peak": round(copy_gbs, 1),
                         "frac_achievable": round(achieved_gbs / copy_gbs, 4),
                         "achievable_how": "tomatis_copy_probe (16-byte streaming copy) of the "
                                           "launch's input in this process, read + write bytes",
                         "kernel": "k_stft_ola (fused frame/window/FFT/gain/IFFT/OLA/normalise + per-chunk limiter)",
                         "kernel_ms": round(kern_ms, 4),
                         "alg_bytes_per_launch": alg_bytes},
            "compute": {"bound": "valu-fp32", "achieved": round(tflops, 2),
                        "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                        "frac": round(tflops / FP32_PEAK_TFLOPS, 4),
                        "flop_per_ch_sample": round(flops_per_ch_sample(n_fft, hop), 1)},
            "device_error": dev_err,
            "one_file_job": one,
            "cpu_baseline": cpu,
            "manifest": {"streams": int(man.shape[0]),
                         "c2_fraction": round(float(man[:, 3].sum() / max(1, man[:, 2].sum())), 4)},
        }
        print(json.dumps(out), flush=True)
    if ws > 1:
        dist.barrier()
        dist.destroy_process_group()
    if dev_err:
        raise SystemExit(f"device error bits {dev_err:#x} during the timed passes: "
                         "the measurement is invalid")


if __name__ == "__main__":
    main()
