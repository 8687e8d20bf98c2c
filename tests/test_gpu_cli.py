"""GPU end-to-end: the drop-in CLIs (file -> file) and the batch runner.

Outputs go through the WAV PCM_24 fallback (no libsndfile in the image), so the
sample tolerance is 1e-4 plus one 24-bit LSB.  State CSVs are compared as text
with the CSV the reference would write for the same frames (levels / states
from the oracle, which is bit-exact with the reference, formatted like the
reference).
"""
import csv
import io
import os

import numpy as np
import pytest

from oracle import tomatis_oracle as orc
from tomatis_audio_processor_amd import audio_io
from tomatis_audio_processor_amd.synth import synth_stream

pytestmark = pytest.mark.gpu
LSB = 1.0 / 8388607


def _gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _written(out):
    """The processors write FLAC (native codec); the reference's WAV fallback
    name is used only if FLAC encoding failed."""
    return out if os.path.exists(out) else out.replace(".flac", ".wav")


def _wav(tmp_path, name, x, sr):
    p = str(tmp_path / name)
    audio_io.write(p, x, sr, "WAV", "FLOAT")
    return p


def _cmp(y, ref, mask, tol=1e-4 + LSB):
    err = np.abs(np.asarray(y, np.float64) - np.asarray(ref, np.float64))[mask]
    assert float(err.max(initial=0)) <= tol, float(err.max())


def test_process_tomatis_cli(tmp_path):
    _gpu()
    from tomatis_audio_processor_amd import process_tomatis
    sr, N = 48000, 48000 * 6 + 123
    x = synth_stream(101, N, 2, sr)
    inp = _wav(tmp_path, "in.wav", x, sr)
    out = str(tmp_path / "out.flac")
    st_csv = str(tmp_path / "st.csv")
    rc = process_tomatis.main(["-i", inp, "-o", out, "--n_fft", "2048", "--hop", "512",
                               "--state_csv", st_csv])
    assert rc == 0
    y, sr2 = audio_io.read(_written(out))
    ref = orc.process_standard(x, sr, gate_ui=50, n_fft=2048, hop=512)
    m = (ref["wsum"][ref["pad"]:ref["pad"] + N] >= 1e-3)
    _cmp(y, ref["y"], m)
    # state CSV text as the reference writes it (csv module, repr floats)
    buf = io.StringIO(newline="")
    w = csv.writer(buf)
    w.writerow(["frame_idx", "time_sec", "level_dbfs", "state"])
    for k in np.nonzero((ref["starts"] >= 0) & (ref["starts"] < N))[0]:
        w.writerow([int(k), int(ref["starts"][k]) / sr, float(ref["levels"][k]),
                    "C1" if ref["states"][k] == 1 else "C2"])
    assert open(st_csv, newline="", encoding="utf-8").read() == buf.getvalue()


def test_process_tomatis_guard(tmp_path):
    _gpu()
    from tomatis_audio_processor_amd import process_tomatis
    x = synth_stream(102, 44100, 2, 44100)
    inp = _wav(tmp_path, "in44.wav", x, 44100)
    assert process_tomatis.main(["-i", inp, "-o", str(tmp_path / "o.flac")]) == 1
    assert process_tomatis.main(["-i", inp, "-o", str(tmp_path / "o.flac"), "--n_fft", "2048",
                                 "--hop", "512", "--allow_any_format"]) == 0


def test_xfade_and_adaptive_cli(tmp_path):
    _gpu()
    from tomatis_audio_processor_amd import process_tomatis_xfade, process_tomatis_adaptive
    sr, N = 48000, 48000 * 5
    x = synth_stream(103, N, 2, sr)
    inp = _wav(tmp_path, "in.wav", x, sr)
    out = str(tmp_path / "xf.wav")
    assert process_tomatis_xfade.main(["-i", inp, "-o", out, "--gate_offset", "-90",
                                       "--xfade_ms", "500", "--n_fft", "2048", "--hop", "512",
                                       "--state_csv", str(tmp_path / "xf.csv")]) == 0
    ref = orc.process_standard(x, sr, gate_ui=50, gate_offset=-90, n_fft=2048, hop=512,
                               xfade_ms=500.0)
    y, _ = audio_io.read(out)
    _cmp(y, ref["y"], ref["wsum"][ref["pad"]:ref["pad"] + N] >= 1e-3)
    rows = list(csv.reader(open(tmp_path / "xf.csv", newline="", encoding="utf-8")))[1:]
    m = (ref["starts"] >= 0) & (ref["starts"] < N)
    assert [r[4] for r in rows] == [f"{a:.3f}" for a in ref["alpha"][m]]
    assert [r[2] for r in rows] == [f"{v:.2f}" for v in ref["levels"][m]]
    out2 = str(tmp_path / "ad.wav")
    assert process_tomatis_adaptive.main(["-i", inp, "-o", out2, "--n_fft", "2048", "--hop",
                                          "512", "--state_csv", str(tmp_path / "ad.csv")]) == 0
    ra = orc.process_adaptive(x, sr, n_fft=2048, hop=512)
    y2, _ = audio_io.read(out2)
    _cmp(y2, ra["y"], ra["wsum"] >= 1e-3)
    rows = list(csv.reader(open(tmp_path / "ad.csv", newline="", encoding="utf-8")))[1:]
    assert [r[3] for r in rows] == ["C1" if s == 1 else "C2" for s in ra["states"]]
    assert [r[4] for r in rows] == [f"{a:.4f}" for a in ra["alpha"]]


def test_layer2_cli_gain_protect(tmp_path):
    _gpu()
    from tomatis_audio_processor_amd import layer2_apply_eq
    from tests.golden.cases import eq_csv_rows
    from tests.golden_util import parse_eq_csv
    sr, N = 48000, 100000
    x = synth_stream(104, N, 2, sr)
    inp = _wav(tmp_path, "in.wav", x, sr)
    eq = str(tmp_path / "eq.csv")
    open(eq, "w").write(eq_csv_rows())
    out = str(tmp_path / "l2.flac")
    # FLAC in: the device file path end to end (fileio ingest and egress)
    inp_flac = str(tmp_path / "in.flac")
    audio_io.write(inp_flac, x, sr, "FLAC", "PCM_24")
    layer2_apply_eq.main(["-i", inp_flac, "-o", out, "--eq_csv", eq, "--n_fft", "2048",
                          "--hop", "512"])
    fr, db = parse_eq_csv(eq_csv_rows())
    xq, _ = audio_io.read(inp_flac)
    ref = orc.apply_eq_stft(xq, sr, fr, db, n_fft=2048, hop=512)
    y, _ = audio_io.read(_written(out))
    assert y.shape == ref["y"].shape
    # PCM_24 clips the reference's ill-conditioned head samples (F7): compare the rest
    m = (ref["wsum"] >= 1e-3)[:, None] & (np.abs(ref["y"]) < 0.99)
    _cmp(y, ref["y"], m)
    # gain protect: the reference re-reads its PCM_24 output and writes
    # float32(x * scale) as PCM_24 (src/layer2_apply_eq.py:220-231); bit-exact
    # given the device's peak
    r = layer2_apply_eq.apply_eq_stft(inp_flac, str(tmp_path / "l2b.flac"), eq, n_fft=2048,
                                      hop=512)
    assert r["peak_seen"] > 0.99, "the case is meant to engage gain protection"
    scale = np.float32(0.99 / max(r["peak_seen"], 1e-12))
    y2, _ = audio_io.read(str(tmp_path / "l2b.flac"))
    np.testing.assert_array_equal(y2, y)
    gp, _ = audio_io.read(str(tmp_path / "l2b_gp.flac"))
    v = np.clip(np.rint((y2 * scale).astype(np.float32).astype(np.float64) * 8388607.0),
                -8388608, 8388607)
    np.testing.assert_array_equal(gp, (v / 8388608.0).astype(np.float32))


def test_batch_runner_single_process(tmp_path):
    _gpu()
    from tomatis_audio_processor_amd import batch
    import json
    sr = 48000
    files = []
    for i in range(3):
        x = synth_stream(200 + i, sr * (2 + i), 2, sr)
        files.append(_wav(tmp_path, f"f{i}.wav", x, sr))
    od = str(tmp_path / "out")
    assert batch.main(["-i", *files, "--out_dir", od, "--n_fft", "2048", "--hop", "512"]) == 0
    man = json.load(open(os.path.join(od, "manifest.json")))
    assert [s["stream"] for s in man["streams"]] == [0, 1, 2]
    for i in range(3):
        x = synth_stream(200 + i, sr * (2 + i), 2, sr)
        ref = orc.process_standard(x, sr, gate_ui=50, n_fft=2048, hop=512)
        y, _ = audio_io.read(os.path.join(od, f"f{i}_tomatis.wav"))
        N = len(x)
        _cmp(y, ref["y"], ref["wsum"][ref["pad"]:ref["pad"] + N] >= 1e-3)
        assert man["streams"][i]["c2_frames"] == int(np.count_nonzero(ref["states"] == 2))


def test_process_tomatis_flac_in_flac_out(tmp_path):
    """FLAC PCM_24 in -> FLAC PCM_24 out through the native codec (row f1)."""
    _gpu()
    from tomatis_audio_processor_amd import process_tomatis
    sr, N = 48000, 48000 * 4 + 77
    x = synth_stream(105, N, 2, sr)
    inp = str(tmp_path / "in.flac")
    audio_io.write(inp, x, sr, "FLAC", "PCM_24")
    xq, _ = audio_io.read(inp)  # what the processor sees (PCM_24 values)
    out = str(tmp_path / "out.flac")
    assert process_tomatis.main(["-i", inp, "-o", out, "--n_fft", "2048", "--hop", "512"]) == 0
    assert os.path.exists(out) and not os.path.exists(out.replace(".flac", ".wav"))
    y, sr2 = audio_io.read(out)
    assert sr2 == sr and y.shape == (N, 2)
    ref = orc.process_standard(xq, sr, gate_ui=50, n_fft=2048, hop=512)
    m = ref["wsum"][ref["pad"]:ref["pad"] + N] >= 1e-3
    _cmp(y, ref["y"], m)


@pytest.mark.parametrize("mode,extra", [("standard", []), ("xfade", []),
                                        ("adaptive", ["--n_fft", "2048", "--hop", "512"])])
def test_batch_runner_pipelined_batches(tmp_path, mode, extra):
    """A rank's files as a pipeline of >= 3 batches of different geometry
    (--batch_gb small: batch k+1's transform limits batch k's output,
    tomatis_stft_ola_*_pipelined_after): every output file and the manifest
    byte-identical to --no_pipeline (each batch limited by itself)."""
    _gpu()
    from tomatis_audio_processor_amd import batch
    import json
    sr = 48000
    # 7 files of different lengths, some loud (limited chunks), one short
    lens = [sr * 9 + 17, sr * 4 + 3, 3000, sr * 12 + 5, sr * 6, sr * 2 + 999, sr * 8 + 1]
    files = []
    for i, n in enumerate(lens):
        x = synth_stream(300 + i, n, 2, sr) * (1.0, 0.3, 1.2)[i % 3]
        files.append(_wav(tmp_path, f"g{i}.wav", x.astype(np.float32), sr))
    # ~ 2 files per batch: 14 s of 48 kHz stereo float
    gb = 14 * sr * 2 * 4 / 2 ** 30
    args = ["-i", *files, "--mode", mode, "--batch_gb", f"{gb:.9f}", *extra]
    if mode != "adaptive":
        args += ["--n_fft", "2048", "--hop", "512"]
    od1, od2 = str(tmp_path / "p"), str(tmp_path / "u")
    assert batch.main(args + ["--out_dir", od1]) == 0
    assert batch.main(args + ["--out_dir", od2, "--no_pipeline"]) == 0
    ids = list(range(len(lens)))
    sizes = {i: lens[i] * 2 for i in ids}
    assert len(batch.split_batches(ids, sizes, int(gb * 2 ** 30 / 4))) >= 3
    for i in ids:
        a = open(os.path.join(od1, f"g{i}_tomatis.wav"), "rb").read()
        b = open(os.path.join(od2, f"g{i}_tomatis.wav"), "rb").read()
        assert a == b, f"file {i} differs ({mode})"
    m1 = json.load(open(os.path.join(od1, "manifest.json")))
    m2 = json.load(open(os.path.join(od2, "manifest.json")))
    assert m1 == m2
    if mode == "standard":  # and the oracle on a limited file of the middle batch
        x = (synth_stream(303, lens[3], 2, sr) * 1.0).astype(np.float32)  # (FLOAT WAV: exact)
        y, _ = audio_io.read(os.path.join(od1, "g3_tomatis.wav"))
        ref = orc.process_standard(x, sr, gate_ui=50, n_fft=2048, hop=512)
        N = lens[3]
        _cmp(y, ref["y"], ref["wsum"][ref["pad"]:ref["pad"] + N] >= 1e-3)
