"""The gate-calibration golden case (tools/make_calib_goldens.py): inputs are
regenerated from seeds, the base through the oracle's standard processor (test
infrastructure only) with a known gate, gain and delay."""
import numpy as np

CASE = dict(sr=48000, secs=60, seed=61, n_fft=4096, hop=2048, max_minutes=1.0,
            gate=dict(gate_ui=50, gate_mode="linear", gate_offset=-92, hysteresis_db=2.0,
                      up_delay_ms=100.0, n_fft=4096, hop=2048),
            gain_db=-2.5, delay=1234, argv=["--max_minutes", "1"])


def make_inputs():
    from oracle import tomatis_oracle as orc
    from tomatis_audio_processor_amd.synth import synth_stream
    sr, n = CASE["sr"], CASE["secs"] * CASE["sr"]
    xo = synth_stream(CASE["seed"], n, 2, sr)
    y = orc.process_standard(xo, sr, **CASE["gate"])["y"]
    y = (y * np.float32(10 ** (CASE["gain_db"] / 20))).astype(np.float32)
    d = CASE["delay"]
    xb = np.concatenate([np.zeros((d, 2), np.float32), y[:n - d]]).astype(np.float32)
    return xo, xb
