"""Time sharding host logic (no GPU): the run-scan algebra composed over shard
summaries reproduces the sequential gate, and the shard geometry tiles the
stream (timeshard.py)."""
import numpy as np
import pytest

from oracle import tomatis_oracle as orc
from tomatis_audio_processor_amd import dsp, timeshard as T


def _seq_gate(pred, D):
    """The reference automaton (src/process_tomatis.py:373-385) in frame units:
    pending set at the first 'on' frame of a run, entry when the run has lasted
    D further frames; C2 leaves on an 'off' frame."""
    st, pend = 1, None
    out = []
    for k, p in enumerate(pred):
        if st == 1:
            if p & 1:
                if pend is None:
                    pend = k + D
                if k >= pend:
                    st, pend = 2, None
            else:
                pend = None
        elif p & 2:
            st = 1
        out.append(st)
    return np.asarray(out, np.uint8)


@pytest.mark.parametrize("seed", range(6))
def test_sharded_composition_matches_sequential_gate(seed):
    rng = np.random.default_rng(seed)
    n = 3000
    # runs of on / off / neither, exclusive predicates (hysteresis > 0)
    pred = np.zeros(n, np.uint8)
    k = 0
    while k < n:
        L = int(rng.integers(1, 60))
        pred[k:k + L] = rng.choice([0, 1, 2], p=[0.2, 0.5, 0.3])
        k += L
    for D in (0, 1, 5, 22):
        ref = _seq_gate(pred, D)
        assert np.array_equal(T.resolve(pred, D), ref)
        cuts = sorted(set(int(c) for c in rng.integers(1, n - 1, 5)))
        bs = [0] + cuts + [n]
        sums = [T.summarize(pred[a:b], D, k0=a) for a, b in zip(bs, bs[1:])]
        got = np.concatenate([T.resolve(pred[a:b], D, T.carry_in(sums, r, D), k0=a)
                              for r, (a, b) in enumerate(zip(bs, bs[1:]))])
        assert np.array_equal(got, ref)
        # local-index summaries shifted to global ones compose the same way
        loc = [T.gs_shift(T.summarize(pred[a:b], D), a) for a, b in zip(bs, bs[1:])]
        assert loc == sums


def test_gate_matches_oracle_on_levels():
    sr, n_fft, hop = 44100, 2048, 512
    from tomatis_audio_processor_amd.synth import synth_stream
    x = synth_stream(11, sr * 20, 2, sr)
    ref = orc.process_standard(x, sr, gate_ui=50, n_fft=n_fft, hop=hop)
    lv = orc.r_to_level(ref["r"])
    T_db = dsp.gate_ui_to_dbfs_log_percent(50)
    Ton, Toff = T_db + 1.5, T_db - 1.5
    pred = ((lv >= Ton).astype(np.uint8) | ((lv <= Toff).astype(np.uint8) << 1))
    D = -(-int(sr * 250 / 1000) // hop)
    assert np.array_equal(T.resolve(pred, D), ref["states"])


@pytest.mark.parametrize("N,n_fft,hop,world", [(158_760_000, 2048, 512, 8), (441_000 * 3 + 17, 2048, 512, 3),
                                               (96000 * 300, 4096, 1024, 8), (48000 * 61, 4096, 2048, 4)])
def test_shard_geometry_tiles_the_stream(N, n_fft, hop, world):
    sh = T.plan_shards(N, n_fft, hop, world)
    pad, pe, F, s0 = dsp.std_schedule(N, n_fft, hop)
    W = -(-n_fft // hop) - 1
    assert sh[0].p0 == 0 and sh[-1].p1 == N and sh[0].k0 == 0 and sh[-1].k1 == F
    for a, b in zip(sh, sh[1:]):
        assert a.p1 == b.p0 and a.k1 == b.k0 and b.b == a.b + a.tf_frames
        assert a.tf_frames % T.GATE_SEGMENT == 0 and b.k0 - b.b == W
    G = T.n_chunks_global(N, n_fft, hop)
    covered = set()
    for s in sh:
        g = s.geometry
        assert g["out_len"] == s.p1 - s.p0 and 0 <= g["out_begin"]
        assert s.lo + g["first_start"] == s0 + s.b * hop
        covered |= set(range(s.chunk_lo, s.chunk_lo + g["n_chunks"]))
    assert covered == set(range(G))
