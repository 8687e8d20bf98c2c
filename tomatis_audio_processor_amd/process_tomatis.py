"""Tomatis gate-controlled C1/C2 tilt processor — MI355X drop-in for
src/process_tomatis.py (``process()`` signature :160-178, CLI :481-544).

Same flags, defaults, guard errors, state-CSV format and FLAC->WAV fallback as
the reference; the per-frame loop (levels, gate, rfft*gain/irfft, OLA,
normalise, per-chunk limiter) runs in the HIP library through
``engine.GatePipeline``.  Extension: ``allow_any_format`` /
``--allow_any_format`` lifts the reference's 48 kHz / stereo guard
 for sample rates and mono/stereo the kernels support.
"""
from __future__ import annotations

import argparse
import csv

import numpy as np

from . import audio_io, dsp

EPS = dsp.EPS
PEAK_LIMIT = dsp.PEAK_LIMIT
rms_dbfs = dsp.rms_dbfs
gate_ui_to_dbfs = dsp.gate_ui_to_dbfs
gate_ui_to_dbfs_log_percent = dsp.gate_ui_to_dbfs_log_percent
db_to_lin = dsp.db_to_lin
build_tilt_gain_db = dsp.build_tilt_gain_db


def check_format(sr: int, ch: int, allow_any_format: bool):
    """The reference's guard (src/process_tomatis.py:234-237)."""
    if allow_any_format:
        return
    if sr != 48000:
        raise ValueError(f"期望 48kHz，实际 {sr} Hz")
    if ch != 2:
        raise ValueError(f"期望双声道，实际 {ch} 声道")


def run_gate_file(x, sr, *, xfade_ms=None, **params):
    """Run one in-memory stream through the GPU pipeline; returns (y, result, pipe)."""
    from . import engine
    import torch
    ss = engine.StreamSet.from_arrays([x], sr)
    pipe = engine.GatePipeline(ss, xfade_ms=xfade_ms, **params)
    res = pipe.run()
    torch.cuda.synchronize()
    return res.output(0), res, pipe


def run_gate_path(in_path, out_path, *, xfade_ms=None, timer=None, **params):
    """File -> file through the device (fileio: FLAC decoded into page-locked
    memory and streamed to HBM, PCM_24 quantised on the device and encoded
    while the next segment is copied back).  Returns (result, written, is_flac, N)."""
    from . import engine, fileio
    import time
    import torch
    x, n, ch, sr = fileio.read_device(in_path, timer)
    t0 = time.perf_counter()
    ss = fileio.device_stream_set(x, n, ch, sr)
    pipe = engine.GatePipeline(ss, xfade_ms=xfade_ms, **params)
    if timer is not None:
        timer.add("plan", t0)
    t0 = time.perf_counter()
    res = pipe.run()
    torch.cuda.synchronize()
    if timer is not None:
        timer.add("process", t0)
    y = res.y[res.out_offs[0]:res.out_offs[0] + res.out_lens[0] * ch]
    written, is_flac = fileio.write_device(out_path, y, res.out_lens[0], ch, sr, timer=timer)
    return res, written, is_flac, n


def process(
    in_path,
    out_path,
    gate_ui=50,
    gate_mode="log_percent",
    dynamic_range=80.0,
    gate_scale=1.0,
    gate_offset=-100,
    hysteresis_db=3.0,
    fc=1000.0,
    slope=12.0,
    c1_low=+15.0, c1_high=-15.0,
    c2_low=-15.0, c2_high=+15.0,
    up_delay_ms=250.0,
    n_fft=4096,
    hop=2048,
    state_csv_path=None,
    output_gain_db=0.0,
    allow_any_format=False,
):
    """Apply the gate-controlled C1/C2 tilt filter to ``in_path`` -> ``out_path``."""
    print("=" * 70)
    print("Tomatis 音频处理器 (MI355X)")
    print("=" * 70)
    print(f"\n输入文件: {in_path}\n输出文件: {out_path}")
    if gate_mode == "log_percent":
        T = gate_ui_to_dbfs_log_percent(gate_ui, dynamic_range)
        print(f"  Gate UI: {gate_ui} (模式: 对数百分比, 阈值: {T:.1f} dBFS)")
    else:
        T = gate_ui_to_dbfs(gate_ui, gate_scale, gate_offset)
        print(f"  Gate UI: {gate_ui} (模式: 线性, 阈值: {T:.1f} dBFS)")
    print(f"  FFT 参数: n_fft={n_fft}, hop={hop}\n")

    sr, ch, frames = audio_io.info(in_path)
    print(f"[OK] 采样率: {sr} Hz\n[OK] 声道数: {ch}\n[OK] 总长度: {frames} 采样点 "
          f"({frames / sr:.2f} 秒)")
    check_format(sr, ch, allow_any_format)
    res, written, is_flac, N = run_gate_path(
        in_path, out_path, gate_ui=gate_ui, gate_mode=gate_mode, dynamic_range=dynamic_range,
        gate_scale=gate_scale, gate_offset=gate_offset, hysteresis_db=hysteresis_db, fc=fc,
        slope=slope, c1_low=c1_low, c1_high=c1_high, c2_low=c2_low, c2_high=c2_high,
        up_delay_ms=up_delay_ms, n_fft=n_fft, hop=hop, output_gain_db=output_gain_db)
    states = res.stream_states(0)

    if state_csv_path:
        starts = res.first_start[0] + hop * np.arange(len(states), dtype=np.int64)
        levels = dsp.r_to_level(res.stream_r(0))
        write_state_csv(state_csv_path, starts, levels, states, sr, N)
        print(f"[OK] 状态记录: {state_csv_path}")

    F = len(states)
    c1 = int(np.count_nonzero(states == 1))
    c2 = F - c1
    print("=" * 70 + "\n处理完成！\n" + "=" * 70)
    print(f"\n统计信息:\n  总帧数: {F}")
    print(f"  C1 帧数: {c1} ({c1 / F * 100:.1f}%)")
    print(f"  C2 帧数: {c2} ({c2 / F * 100:.1f}%)")
    print(f"\n输出文件: {written}\n  输出长度: {N} 采样点 (与输入一致)")
    if not is_flac:
        print("\n[WARN] 注意: 已输出 WAV 格式（因 FLAC 写入失败）")
    return None


def write_state_csv(path, starts, levels, states, sr, N):
    """frame_idx,time_sec,level_dbfs,state rows for frames starting in [0, N)
    (src/process_tomatis.py:300-307,408-409; floats written with repr)."""
    with open(path, "w", newline="", encoding="utf-8") as f:
        w = csv.writer(f)
        w.writerow(["frame_idx", "time_sec", "level_dbfs", "state"])
        for k in np.nonzero((starts >= 0) & (starts < N))[0].tolist():
            s = int(starts[k])
            w.writerow([k, s / sr, float(levels[k]), "C1" if states[k] == 1 else "C2"])


def build_parser():
    ap = argparse.ArgumentParser(
        description="Tomatis 音频处理器 - Gate 控制的 C1/C2 倾斜滤波器 (MI355X)",
        formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    ap.add_argument("-i", "--input", required=True, help="输入 FLAC 文件")
    ap.add_argument("-o", "--output", required=True, help="输出 FLAC 文件")
    ap.add_argument("--gate_ui", type=float, default=50, help="Gate UI 值 (0-100)")
    ap.add_argument("--gate_mode", choices=["linear", "log_percent"], default="log_percent",
                    help="门控换算模式: linear=线性公式, log_percent=对数百分比(推荐)")
    ap.add_argument("--dynamic_range", type=float, default=80.0,
                    help="动态范围(dB)，用于log_percent模式")
    ap.add_argument("--gate_scale", type=float, default=1.0, help="Gate 缩放系数(linear模式)")
    ap.add_argument("--gate_offset", type=float, default=-100, help="Gate 偏移量(linear模式)")
    ap.add_argument("--hyst_db", type=float, default=3.0, help="回差（dB）")
    ap.add_argument("--up_delay_ms", type=float, default=250.0, help="C1→C2 上行延迟（ms）")
    ap.add_argument("--fc", type=float, default=1000.0, help="中心频率（Hz）")
    ap.add_argument("--slope", type=float, default=12.0, help="坡度（dB/octave）")
    ap.add_argument("--c1_low", type=float, default=15.0, help="C1 低频增益（dB）")
    ap.add_argument("--c1_high", type=float, default=-15.0, help="C1 高频增益（dB）")
    ap.add_argument("--c2_low", type=float, default=-15.0, help="C2 低频增益（dB）")
    ap.add_argument("--c2_high", type=float, default=15.0, help="C2 高频增益（dB）")
    ap.add_argument("--n_fft", type=int, default=4096, help="FFT 窗长")
    ap.add_argument("--hop", type=int, default=2048, help="跳步长度")
    ap.add_argument("--state_csv", default=None, help="输出状态 CSV 文件路径")
    ap.add_argument("--output_gain_db", type=float, default=0.0, help="输出增益补偿（dB）")
    ap.add_argument("--allow_any_format", action="store_true",
                    help="(MI355X build) accept sample rates other than 48 kHz and mono input")
    return ap


def main(argv=None):
    args = build_parser().parse_args(argv)
    try:
        process(args.input, args.output, gate_ui=args.gate_ui, gate_mode=args.gate_mode,
                dynamic_range=args.dynamic_range, gate_scale=args.gate_scale,
                gate_offset=args.gate_offset, hysteresis_db=args.hyst_db, fc=args.fc,
                slope=args.slope, c1_low=args.c1_low, c1_high=args.c1_high,
                c2_low=args.c2_low, c2_high=args.c2_high, up_delay_ms=args.up_delay_ms,
                n_fft=args.n_fft, hop=args.hop, state_csv_path=args.state_csv,
                output_gain_db=args.output_gain_db, allow_any_format=args.allow_any_format)
    except Exception as e:
        print(f"\n[ERR] 错误: {e}")
        import traceback
        traceback.print_exc()
        return 1
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
