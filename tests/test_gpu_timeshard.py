"""GPU: one stream time-sharded over W ranks (emulated in one process, the two
exchanges done on the host) is bit-identical to the unsharded run: samples,
gate states and limiter chunk peaks (timeshard.py)."""
import numpy as np
import pytest

from tomatis_audio_processor_amd.synth import synth_stream

pytestmark = pytest.mark.gpu


def _engine():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from tomatis_audio_processor_amd import engine, timeshard
    return torch, engine, timeshard


@pytest.mark.parametrize("secs,sr,n_fft,hop,world", [(150, 44100, 2048, 512, 2),
                                                     (150, 44100, 2048, 512, 8),
                                                     (97, 48000, 4096, 1024, 3),
                                                     (300, 48000, 4096, 2048, 4)])
def test_timeshard_bit_identical(secs, sr, n_fft, hop, world):
    torch, E, T = _engine()
    N = sr * secs + 123
    x = synth_stream(31, N, 2, sr)
    params = dict(gate_ui=50, n_fft=n_fft, hop=hop)
    ss = E.StreamSet.from_arrays([x], sr)
    pipe = E.GatePipeline(ss, **params)
    res = pipe.run()
    torch.cuda.synchronize()
    y_ref, st_ref, pk_ref = res.output(0), res.stream_states(0), res.stream_peaks(0)
    y, st, pk = T.run_emulated(x, sr, world, **params)
    assert np.array_equal(st, st_ref)
    assert pk.tobytes() == pk_ref.tobytes()
    assert y.shape == y_ref.shape
    assert y.tobytes() == y_ref.tobytes()


@pytest.mark.parametrize("secs,sr,n_fft,hop,world", [(150, 44100, 2048, 512, 4),
                                                     (97, 48000, 4096, 1024, 3)])
def test_timeshard_vs_oracle(secs, sr, n_fft, hop, world):
    """The concatenated shards against the oracle directly (not only against the
    unsharded GPU run): states bit-exact, chunk scales and masked samples."""
    torch, E, T = _engine()
    from oracle import tomatis_oracle as orc
    N = sr * secs + 777
    x = synth_stream(41, N, 2, sr)
    params = dict(gate_ui=50, n_fft=n_fft, hop=hop)
    y, st, pk = T.run_emulated(x, sr, world, **params)
    ref = orc.process_standard(x, sr, **params)
    assert np.array_equal(st, ref["states"])
    m = ref["wsum"][ref["pad"]:ref["pad"] + N] >= 1e-3
    b = ref["bounds"]
    assert len(pk) == len(b) - 1
    for c in range(len(b) - 1):
        lo, hi = max(0, int(b[c])), min(N, int(b[c + 1]))
        gs = float(np.float32(0.999) / np.float32(pk[c])) if pk[c] > 0.999 else 1.0
        rs = ref["scales"][c] or 1.0
        mm = m[lo:hi]
        err = np.abs(y[lo:hi][mm] / gs - ref["y"][lo:hi][mm] / rs) * min(gs, rs)
        assert err.max() <= 1e-4
        if c < len(b) - 2:   # interior chunks: no ill-conditioned sample in them
            assert abs(gs / rs - 1) <= 5e-5


def _rank_worker(rank, ws, port, secs, sr, q):
    """One rank of a real 2-process run: RankStep.run with its device-resident
    collectives (int32 gate-summary all_gather, chunk-peak all_reduce MAX) over
    gloo on CUDA tensors (two ranks share the box's one GPU, which RCCL does
    not allow)."""
    import os
    import torch
    import torch.distributed as dist
    from tomatis_audio_processor_amd import timeshard as T
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        N = sr * secs + 123
        x = synth_stream(31, N, 2, sr)
        sh = T.plan_shards(N, 2048, 512, ws)[rank]
        xs = torch.from_numpy(x[sh.lo:sh.hi].reshape(-1).copy()).cuda()
        step = T.RankStep(xs, sr, N, rank, ws, ch=2, gate_ui=50, n_fft=2048, hop=512)
        res = step.run()
        torch.cuda.synchronize()
        st = res.stream_states(0)[sh.k0 - sh.b:sh.k1 - sh.b]
        q.put((rank, res.output(0).copy(), st.copy(), res.stream_peaks(0).copy()))
    finally:
        dist.destroy_process_group()


def test_rankstep_two_processes_gloo():
    """RankStep.run in 2 real ranks: concatenated outputs and
    states equal run_emulated's, which equals the unsharded run."""
    torch, E, T = _engine()
    import socket
    import torch.multiprocessing as mp
    secs, sr, ws = 150, 44100, 2
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_worker, args=(r, ws, port, secs, sr, q)) for r in range(ws)]
    for p in procs:
        p.start()
    try:
        out = sorted([q.get(timeout=240) for _ in range(ws)], key=lambda t: t[0])
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    N = sr * secs + 123
    x = synth_stream(31, N, 2, sr)
    y_em, st_em, pk_em = T.run_emulated(x, sr, ws, gate_ui=50, n_fft=2048, hop=512)
    y = np.concatenate([o[1] for o in out])
    st = np.concatenate([o[2] for o in out])
    assert y.tobytes() == y_em.tobytes()
    assert np.array_equal(st, st_em)
