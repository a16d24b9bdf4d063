"""Time-sharded smoothing (eks_amd.timeshard, eks_smooth_seg / eks_seg_combine).

CPU: the frame split and the aggregate sizes.  GPU: the segmented smooth
(phases 1-3 with the two combines) against the one-piece eks_smooth on the
same inputs, in one process and over a 2-rank gloo group sharing cuda:0.
The segments re-associate the scan, so outputs agree to rounding
(|d| < 1e-8 px, the same bar as algo 2 vs algo 1); the north-star tolerance
vs the reference (1e-5 px) is covered by eks_smooth's own parity tests.
"""
import os
import socket

import numpy as np
import pytest


def test_split_frames_partitions():
    from eks_amd.timeshard import split_frames
    for T, nseg in [(10, 1), (10, 3), (50000, 8), (7, 7), (101, 4)]:
        spans = [split_frames(T, nseg, k) for k in range(nseg)]
        assert spans[0][0] == 0
        for (a, la), (b, _) in zip(spans, spans[1:]):
            assert a + la == b
        assert spans[-1][0] + spans[-1][1] == T
        sizes = [t for _, t in spans]
        assert max(sizes) - min(sizes) <= 1 and min(sizes) >= 1
    with pytest.raises(ValueError):
        split_frames(3, 4, 0)


def test_aggregate_sizes_match_header():
    """The header documents EL = R*R + 2R + R(R+1) (A, b, C, eta, J)."""
    from eks_amd import timeshard
    assert timeshard.elem_len(2) == 4 + 4 + 6
    assert timeshard.elem_len(3) == 9 + 6 + 12
    assert timeshard.map_len(3) == 12 and timeshard.state_len(3) == 9


def _problem(kind, B, T, seed=5):
    from eks_amd import batch, synthetic
    from oracle import eks_oracle as O
    rng = np.random.default_rng(seed)
    E = 5
    if kind == "singleview":
        st = synthetic.singleview_obs(rng, E, T, K=B).transpose(2, 0, 1, 3).astype(np.float64)
        r, n = 2, 2
    else:
        st = synthetic.multiview_obs(rng, 4, E, T, K=B).transpose(2, 0, 1, 3).astype(np.float64)
        r, n = 3, 8
    models = []
    for b in range(B):
        preds, ev = O.ensemble_array(st[b])
        p = (O.singleview_params(preds, ev, 0.01, 25) if r == 2
             else O.multicam_params(preds, ev, 0.01, 25))
        p["offset"] = p["means"]
        models.append(p)
    stackp = lambda k: np.stack([m[k] for m in models])  # noqa: E731
    params = batch.pack_params(stackp("m0"), stackp("S0"), stackp("A"), stackp("Q"), stackp("C"),
                               stackp("offset"))
    flags = batch.model_flags(stackp("A"), stackp("C"))
    return st, params, flags, r, n


@pytest.mark.gpu
@pytest.mark.parametrize("kind,B,T,nseg", [
    ("singleview", 3, 20000, 2),
    ("singleview", 3, 20000, 7),      # uneven segments
    ("multiview", 2, 12000, 4),
    ("singleview", 2, 900, 5),        # segments shorter than one chunk
    ("singleview", 2, 40, 40),        # one frame per segment
    ("multiview", 1, 40000, 8),
])
def test_segments_match_one_piece(kind, B, T, nseg):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from eks_amd import batch, timeshard
    st, params, flags, r, n = _problem(kind, B, T)
    d = batch.make_time_major(st, dtype=np.float32)
    ref = batch.smooth(d, params, n=n, r=r, flags=flags, algo=1, want_nll=True, want_ms=True,
                       check=True)
    seg = timeshard.smooth_segments(d, params, n=n, r=r, nseg=nseg, flags=flags, want_ms=True)
    assert int((seg["status"] != 0).sum()) == 0
    o1, o2 = ref["out"].cpu().numpy(), seg["out"].cpu().numpy()
    assert np.isfinite(o1).all() and np.isfinite(o2).all()
    assert np.abs(o1 - o2).max() < 1e-8
    assert float((seg["ms"] - ref["ms"]).abs().max()) < 1e-8
    np.testing.assert_allclose(seg["nll"].cpu().numpy(), ref["nll"].cpu().numpy(), rtol=1e-10)
    # filter only (phases 1-2): the NLL shares sum to eks_smooth's filter-only NLL
    fo = timeshard.smooth_segments(d, params, n=n, r=r, nseg=nseg, flags=flags, want_out=False)
    assert fo["out"] is None
    np.testing.assert_allclose(fo["nll"].cpu().numpy(), ref["nll"].cpu().numpy(), rtol=1e-10)


@pytest.mark.gpu
def test_segment_argument_errors():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from eks_amd import _lib, batch, timeshard
    st, params, flags, r, n = _problem("singleview", 1, 200)
    d = batch.make_time_major(st, dtype=np.float32)
    s = timeshard.Segment(d[:, 100:], params, n=n, r=r, t_base=100, T_total=200, flags=flags)
    with pytest.raises(_lib.EksError):
        s.phase(2)  # a later segment needs the entering state
    with pytest.raises(ValueError):
        timeshard.Segment(d[:, 100:], params, n=n, r=r, t_base=150, T_total=200)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    from eks_amd import batch, timeshard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        st, params, flags, r, n = _problem("multiview", 2, 9000)
        T = st.shape[2]
        t0, tk = timeshard.split_frames(T, world, rank)
        d = batch.make_time_major(st[:, :, t0:t0 + tk], dtype=np.float32)
        res = timeshard.smooth_time_sharded(d, params, n=n, r=r, t_base=t0, T_total=T,
                                            flags=flags, want_nll=True)
        full = batch.make_time_major(st, dtype=np.float32)
        ref = batch.smooth(full, params, n=n, r=r, flags=flags, algo=1, want_nll=True)
        err = float((res["out"] - ref["out"][:, t0:t0 + tk]).abs().max())
        nerr = float(((res["nll"] - ref["nll"]) / ref["nll"]).abs().max())
        fo = timeshard.smooth_time_sharded(d, params, n=n, r=r, t_base=t0, T_total=T,
                                           flags=flags, want_out=False)
        nerr = max(nerr, float(((fo["nll"] - ref["nll"]) / ref["nll"]).abs().max()))
        q.put((rank, err, nerr, int((res["status"] != 0).sum())))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_gloo_world2_time_sharded():
    """Two ranks on cuda:0 exchange the aggregates over gloo (host copies)."""
    import torch
    import torch.multiprocessing as mp
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, err, nerr, bad in got:
        assert bad == 0
        assert err < 1e-8, (rank, err)
        assert nerr < 1e-10, (rank, nerr)
