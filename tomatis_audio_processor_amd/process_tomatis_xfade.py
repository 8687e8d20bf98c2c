"""Tomatis processor with C1/C2 cross-fade — MI355X drop-in for
src/process_tomatis_xfade.py (``process()`` :55-71, CLI :362-417).

Linear gate mapping only (as the reference); per-frame alpha moves by
1/xfade_frames towards the gate target and, while 0 < alpha < 1, the gain is
the dB-domain mix of C1/C2 (src/process_tomatis_xfade.py:251-274).  Alpha is
scanned on the device in float64 with the reference's exact update rule.
"""
from __future__ import annotations

import argparse
import csv

import numpy as np

from . import audio_io, dsp
from .process_tomatis import check_format, run_gate_path

EPS = dsp.EPS
PEAK_LIMIT = dsp.PEAK_LIMIT
rms_dbfs = dsp.rms_dbfs
gate_ui_to_dbfs = dsp.gate_ui_to_dbfs
db_to_lin = dsp.db_to_lin
build_tilt_gain_db = dsp.build_tilt_gain_db


def process(
    in_path,
    out_path,
    gate_ui=50,
    gate_scale=1.0,
    gate_offset=-100,
    hysteresis_db=3.0,
    fc=1000.0,
    slope=12.0,
    c1_low=+15.0, c1_high=-15.0,
    c2_low=-15.0, c2_high=+15.0,
    up_delay_ms=250.0,
    xfade_ms=0.0,
    n_fft=4096,
    hop=2048,
    state_csv_path=None,
    allow_any_format=False,
):
    """Gate-controlled C1/C2 tilt filter with optional cross-fade."""
    print("=" * 70 + "\nTomatis 音频处理器 (Crossfade 版, MI355X)\n" + "=" * 70)
    T = gate_ui_to_dbfs(gate_ui, gate_scale, gate_offset)
    print(f"\n输入文件: {in_path}\n输出文件: {out_path}")
    print(f"  Gate UI: {gate_ui} (阈值: {T:.1f} dBFS)\n  Crossfade: {xfade_ms} ms")
    sr, ch, frames = audio_io.info(in_path)
    print(f"✓ 采样率: {sr} Hz\n✓ 声道数: {ch}\n✓ 总长度: {frames} 采样点 ({frames / sr:.2f} 秒)")
    check_format(sr, ch, allow_any_format)
    res, written, is_flac, N = run_gate_path(
        in_path, out_path, xfade_ms=xfade_ms, gate_ui=gate_ui, gate_scale=gate_scale,
        gate_offset=gate_offset, hysteresis_db=hysteresis_db, fc=fc, slope=slope,
        c1_low=c1_low, c1_high=c1_high, c2_low=c2_low, c2_high=c2_high,
        up_delay_ms=up_delay_ms, n_fft=n_fft, hop=hop)
    states = res.stream_states(0)
    alpha = res.stream_alpha(0)
    if state_csv_path:
        starts = res.first_start[0] + hop * np.arange(len(states), dtype=np.int64)
        levels = dsp.r_to_level(res.stream_r(0))
        with open(state_csv_path, "w", newline="", encoding="utf-8") as f:
            w = csv.writer(f)
            w.writerow(["frame_idx", "time_sec", "level_dbfs", "state", "alpha"])
            for k in np.nonzero((starts >= 0) & (starts < N))[0].tolist():
                w.writerow([k, int(starts[k]) / sr, f"{levels[k]:.2f}",
                            "C1" if states[k] == 1 else "C2", f"{alpha[k]:.3f}"])
        print(f"状态记录: {state_csv_path}")
    F = len(states)
    c1 = int(np.count_nonzero(states == 1))
    print("=" * 70 + "\n处理完成！\n" + "=" * 70)
    print(f"\n统计信息:\n  总帧数: {F}\n  C1 帧数: {c1} ({c1 / F * 100:.1f}%)")
    print(f"  C2 帧数: {F - c1} ({(F - c1) / F * 100:.1f}%)")
    if xfade_ms > 0:
        print(f"  Crossfade: {xfade_ms} ms ({res.extra['xfade_frames']} 帧)")
    print(f"\n输出文件: {written}")
    return None


def build_parser():
    ap = argparse.ArgumentParser(
        description="Tomatis 音频处理器 - Gate 控制的 C1/C2 倾斜滤波器 (带 Crossfade, MI355X)",
        formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    ap.add_argument("-i", "--input", required=True, help="输入 FLAC 文件")
    ap.add_argument("-o", "--output", required=True, help="输出 FLAC 文件")
    ap.add_argument("--gate_ui", type=float, default=50, help="Gate UI 值 (0-100)")
    ap.add_argument("--gate_scale", type=float, default=1.0, help="Gate 缩放系数")
    ap.add_argument("--gate_offset", type=float, default=-100, help="Gate 偏移量")
    ap.add_argument("--hyst_db", type=float, default=3.0, help="回差（dB）")
    ap.add_argument("--up_delay_ms", type=float, default=250.0, help="C1→C2 上行延迟（ms）")
    ap.add_argument("--xfade_ms", type=float, default=0.0,
                    help="Crossfade 过渡时间（ms），0=硬切换")
    ap.add_argument("--fc", type=float, default=1000.0, help="中心频率（Hz）")
    ap.add_argument("--slope", type=float, default=12.0, help="坡度（dB/octave）")
    ap.add_argument("--c1_low", type=float, default=15.0, help="C1 低频增益（dB）")
    ap.add_argument("--c1_high", type=float, default=-15.0, help="C1 高频增益（dB）")
    ap.add_argument("--c2_low", type=float, default=-15.0, help="C2 低频增益（dB）")
    ap.add_argument("--c2_high", type=float, default=15.0, help="C2 高频增益（dB）")
    ap.add_argument("--n_fft", type=int, default=4096, help="FFT 窗长")
    ap.add_argument("--hop", type=int, default=2048, help="跳步长度")
    ap.add_argument("--state_csv", default=None, help="输出状态 CSV 文件路径")
    ap.add_argument("--allow_any_format", action="store_true",
                    help="(MI355X build) accept sample rates other than 48 kHz and mono input")
    return ap


def main(argv=None):
    args = build_parser().parse_args(argv)
    try:
        process(args.input, args.output, gate_ui=args.gate_ui, gate_scale=args.gate_scale,
                gate_offset=args.gate_offset, hysteresis_db=args.hyst_db, fc=args.fc,
                slope=args.slope, c1_low=args.c1_low, c1_high=args.c1_high,
                c2_low=args.c2_low, c2_high=args.c2_high, up_delay_ms=args.up_delay_ms,
                xfade_ms=args.xfade_ms, n_fft=args.n_fft, hop=args.hop,
                state_csv_path=args.state_csv, allow_any_format=args.allow_any_format)
    except Exception as e:
        print(f"\n✗ 错误: {e}")
        import traceback
        traceback.print_exc()
        return 1
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
