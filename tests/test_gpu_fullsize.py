"""Parity at BASELINE.json's full config-4 size (1024 videos x 17 keypoints
x 5 members x 10 000 frames, 1.74e8 keypoint-timesteps):

* the CPU oracle (oracle/eks_oracle.py singleview_smooth: ensemble ->
  single-view fit -> filtering_pass -> smooth_backward -> projection, the
  reference's recursions restated) on 8 trajectories spread over the whole
  batch at full T = 10 000 (a few seconds of numpy) against the GPU fit +
  smooth of the whole batch: algo 3 (the default here) and algo 2 within
  1e-5 px (BASELINE.json's tolerance);
* the time-parallel algorithms (algo 2, 16 chunks per trajectory; algo 3,
  625 chunks of 16 frames) equal the sequential recursion (algo 1) on every
  trajectory (max|d| < 1e-8 px);
* translation equivariance: shifting every member by (dx, dy) shifts the
  model offsets and the smoothed outputs by exactly that (to rounding);
* the device fit + hand-off path equals fit + smooth on the members."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def work():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import bench
    from eks_amd import batch
    K, E, T = 17, 5, 10000
    obs_tm = bench.gen_videos(torch, range(1024), K, E, T, 4, torch.device("cuda"))
    obs = obs_tm.permute(3, 0, 1, 2)                            # (B, T, E, 2) view
    params, _ = batch.fit(obs, kind="singleview", n=2, r=2, smooth_param=0.01,
                          quantile_keep=25)
    return torch, obs_tm, obs, params


# 8 trajectories spread over the 17 408 of the batch (first, last, and
# keypoints of videos in between)
ORACLE_SAMPLE = (0, 2175, 4351, 6530, 8703, 10884, 13059, 17407)


def test_oracle_sample_full_size(work):
    torch, obs_tm, obs, params = work
    from eks_amd import _lib, batch
    from oracle import eks_oracle as O
    flags = _lib.EKS_MODEL_A_IDENTITY | _lib.EKS_MODEL_C_IDENTITY
    B, T = obs.shape[0], obs.shape[1]
    assert _lib.load().eks_smooth_algo(B, T, 2, 2, 5, 0) == 3
    outs = {algo: batch.smooth(obs, params, n=2, r=2, algo=algo, flags=flags, check=True)["out"]
            for algo in (0, 2)}
    for b in ORACLE_SAMPLE:
        st = obs_tm[..., b].permute(1, 0, 2).double().cpu().numpy()   # (E, T, 2)
        ref, _, _ = O.singleview_smooth(st, 0.01, 25)
        for algo, out in outs.items():
            d = float(np.abs(out[b].cpu().numpy() - ref).max())
            assert d < 1e-5, (b, algo, d)


def test_algo2_equals_sequential_full_size(work):
    torch, _, obs, params = work
    from eks_amd import _lib, batch
    flags = _lib.EKS_MODEL_A_IDENTITY | _lib.EKS_MODEL_C_IDENTITY
    a2 = batch.smooth(obs, params, n=2, r=2, algo=2, flags=flags, check=True)["out"]
    assert _lib.load().eks_smooth_chunk_len(obs.shape[0], obs.shape[1], 2) > 0
    a1 = batch.smooth(obs, params, n=2, r=2, algo=1, flags=flags, check=True)["out"]
    d = (a2 - a1).abs().max().item()
    assert d < 1e-8, d
    del a2
    r3 = batch.smooth(obs, params, n=2, r=2, algo=3, flags=flags)
    assert (r3["status"] == 0).all()
    d3 = (r3["out"] - a1).abs().max().item()
    assert d3 < 1e-8, d3


def test_translation_equivariance(work):
    torch, obs_tm, _, _ = work
    from eks_amd import _lib, batch
    B = 256 * 17
    x = obs_tm[..., :B].to(torch.float64)                       # (T, E, 2, B), exact copy
    shift = torch.tensor([64.0, -32.0], dtype=torch.float64, device=x.device)
    xs = x + shift[None, None, :, None]                         # exact in float64
    flags = _lib.EKS_MODEL_A_IDENTITY | _lib.EKS_MODEL_C_IDENTITY
    outs, offs = [], []
    for v in (x, xs):
        o = v.permute(3, 0, 1, 2)
        p, _ = batch.fit(o, kind="singleview", n=2, r=2, smooth_param=0.01, quantile_keep=25)
        outs.append(batch.smooth(o, p, n=2, r=2, flags=flags, check=True)["out"])
        offs.append(p[:, -2:])
    assert (offs[1] - offs[0] - shift).abs().max().item() < 1e-9
    assert (outs[1] - outs[0] - shift).abs().max().item() < 1e-8


def test_handoff_full_size(work):
    torch, _, obs, params = work
    from eks_amd import _lib, batch
    flags = _lib.EKS_MODEL_A_IDENTITY | _lib.EKS_MODEL_C_IDENTITY
    p1, _, yev = batch.fit(obs, kind="singleview", n=2, r=2, smooth_param=0.01,
                           quantile_keep=25, keep_yev=True)
    assert torch.equal(p1, params)
    a = batch.smooth(obs, params, n=2, r=2, flags=flags)["out"]
    b = batch.smooth(yev, p1, n=2, r=2, flags=flags)["out"]
    assert torch.equal(a, b)
