"""Parity at BASELINE.json's full sizes for the long-trajectory configurations
(configs 2, 3 and 5; config 4 is tests/test_gpu_fullsize.py), with the bench's
own synthetic generators:

* config 2: single-view, 1 video x 17 keypoints x 5 members x 100 000 frames;
* config 3: multiview PCA, 4 cameras (n = 8, r = 3) x 17 keypoints x 5
  members x 50 000 frames;
* config 5: IBL pupil (n = 8, r = 3), 1 000 000 frames x 5 members, the
  NLL sweep over 64 (diameter_s, com_s) models, then smoothing the argmin.

On every trajectory the time-parallel algorithms (2, and 3 where it
applies) equal the sequential recursion (algo 1) to < 1e-8 px and their NLL
to rtol 1e-10; the CPU oracle (oracle/eks_oracle.py, the reference's
algorithm: eks/ensemble_kalman.py:4-164, eks/multiview_pca_smoother.py:
684-767, eks/pupil_smoother.py:101-223) is run on a bounded sample (2
trajectories x 100k frames; 2 keypoints x 50k frames; a 200k-frame prefix)
and must agree to max|d| < 1e-5 px (north_star's tolerance)."""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

PX_ALGO = 1e-8      # time-parallel vs sequential, pixels
NLL_RTOL = 1e-10    # time-parallel vs sequential NLL
PX_CPU = 1e-5       # GPU vs CPU oracle (north_star)


@pytest.fixture(scope="module")
def torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    return torch


def _algos_agree(torch, obs, params, n, r, flags, algos):
    """Every algo in ``algos`` against algo 1 on all trajectories (outputs
    and NLL).  Returns algo 1's output (B, T, n) on the device."""
    from eks_amd import batch
    ref = batch.smooth(obs, params, n=n, r=r, algo=1, flags=flags, want_nll=True, check=True)
    for al in algos:
        got = batch.smooth(obs, params, n=n, r=r, algo=al, flags=flags, want_nll=True, check=True)
        d = float((got["out"] - ref["out"]).abs().max())
        assert d < PX_ALGO, (al, d)
        rel = float(((got["nll"] - ref["nll"]) / ref["nll"].abs()).abs().max())
        assert rel < NLL_RTOL, (al, rel)
        del got
    return ref["out"]


# ------------------------------------------------------------------ config 2
def test_config2_singleview_17x100k(torch):
    import bench
    from eks_amd import _lib, batch
    from oracle import eks_oracle as O
    K, E, T = 17, 5, 100000
    dev = torch.device("cuda", 0)
    obs_tm = bench.gen_videos(torch, range(1), K, E, T, 2, dev)       # (T, E, 2, K)
    obs = obs_tm.permute(3, 0, 1, 2)
    params, _ = batch.fit(obs, kind="singleview", n=2, r=2, smooth_param=0.01, quantile_keep=25)
    flags = _lib.EKS_MODEL_A_IDENTITY | _lib.EKS_MODEL_C_IDENTITY
    auto = int(_lib.load().eks_smooth_algo(K, T, 2, 2, E, 0))
    assert auto in (2, 3)
    ref = _algos_agree(torch, obs, params, 2, 2, flags, sorted({2, 3, auto}))
    host = obs_tm[..., :2].cpu().numpy().astype(np.float64)          # (T, E, 2, 2)
    for b in range(2):
        out, _, _ = O.singleview_smooth(np.ascontiguousarray(host[..., b].transpose(1, 0, 2)),
                                        0.01, 25)
        d = float(np.abs(ref[b].cpu().numpy() - out).max())
        assert d < PX_CPU, (b, d)


# ------------------------------------------------------------------ config 3
def test_config3_multiview_4cams_17x50k(torch):
    from eks_amd import _lib, batch, synthetic
    from oracle import eks_oracle as O
    K, E, T, V = 17, 5, 50000, 4
    n = 2 * V
    st = synthetic.multiview_obs(np.random.default_rng(3), V, E, T, K=K)   # (E, T, K, 8) f32
    obs = torch.from_numpy(np.ascontiguousarray(st.transpose(1, 0, 3, 2))).cuda()
    obs = obs.permute(3, 0, 1, 2)                                          # (K, T, E, 8) view
    params, _ = batch.fit(obs, kind="multicam", n=n, r=3, smooth_param=0.01, quantile_keep=25)
    flags = _lib.EKS_MODEL_A_IDENTITY
    ref = _algos_agree(torch, obs, params, n, 3, flags, [2, 3])
    for k in range(2):
        cams = [st[:, :, k, 2 * c:2 * c + 2].astype(np.float64) for c in range(V)]
        out, _, _ = O.multicam_smooth(cams, 0.01, 25)
        d = float(np.abs(ref[k].cpu().numpy() - out).max())
        assert d < PX_CPU, (k, d)


# ------------------------------------------------------------------ config 5
def _pupil_candidates(preds):
    from eks_amd import fit
    grid = 1.0 - np.geomspace(1e-4, 1e-1, 8)
    base = fit.pupil_model(preds, np.diag([0.99, 0.99, 0.99]))
    var0 = np.diag(base["S0"])
    cands = []
    for d in grid:
        for c in grid:
            A = np.diag([d, c, c])
            cands.append(dict(base, A=A, Q=np.diag(var0 * (1 - np.diag(A) ** 2))))
    return cands


def test_config5_pupil_1M_sweep_and_smooth(torch):
    from eks_amd import batch, fit, synthetic
    from oracle import eks_oracle as O
    E, T = 5, 1000000
    st = synthetic.pupil_obs(np.random.default_rng(5), E, T, a=0.99)       # (E, T, 8) f32
    obs = torch.from_numpy(np.ascontiguousarray(st.transpose(1, 0, 2))).cuda().unsqueeze(0)
    preds = O.ensemble_array(st.astype(np.float64))[0]
    cands = _pupil_candidates(preds)
    stk = lambda key: np.stack([m[key] for m in cands])  # noqa: E731
    params = batch.pack_params(stk("m0"), stk("S0"), stk("A"), stk("Q"), stk("C"), stk("offset"))
    cobs = obs.expand(len(cands), -1, -1, -1)          # batch stride 0: shared members
    s_auto = batch.nll(cobs, params, n=8, r=3)
    s_seq = batch.nll(cobs, params, n=8, r=3, algo=1)
    rel = float(((s_auto - s_seq) / s_seq.abs()).abs().max())
    assert rel < NLL_RTOL, rel
    assert bool(torch.isfinite(s_auto).all())
    best = int(torch.argmin(s_auto))
    assert best == int(torch.argmin(s_seq))
    # the kernels the bench times: EKS_MODEL_PUPIL (sparse pupil rows, folded
    # equal rows, diagonal A / Q)
    from eks_amd import _lib
    flags = batch.model_flags(stk("A"), stk("C"), stk("Q"))
    assert flags & _lib.EKS_MODEL_PUPIL
    s_pup = batch.nll(cobs, params, n=8, r=3, flags=flags)
    rel = float(((s_pup - s_seq) / s_seq.abs()).abs().max())
    assert rel < NLL_RTOL, rel
    assert int(torch.argmin(s_pup)) == best
    p_best = params[best:best + 1].contiguous()
    ref = _algos_agree(torch, obs, p_best, 8, 3, 0, [2])
    # oracle: the chosen model refitted on a 200k-frame prefix, smoothed on both sides
    Tc = 200000
    A = cands[best]["A"]
    markers, _, _, _ = O.pupil_smooth(st[:, :Tc].astype(np.float64), A)
    pm = fit.pupil_model(O.ensemble_array(st[:, :Tc].astype(np.float64))[0], A)
    pb = batch.pack_params(pm["m0"], pm["S0"], pm["A"], pm["Q"], pm["C"], pm["offset"])
    g = batch.smooth(obs[:, :Tc], pb, n=8, r=3, check=True)["out"][0].cpu().numpy()
    d = float(np.abs(g - markers).max())
    assert d < PX_CPU, d
    fb = batch.model_flags(pm["A"][None], pm["C"][None], pm["Q"][None])
    assert fb & _lib.EKS_MODEL_PUPIL
    gp = batch.smooth(obs[:, :Tc], pb, n=8, r=3, flags=fb, check=True)["out"][0].cpu().numpy()
    d = float(np.abs(gp - markers).max())
    assert d < PX_CPU, d
    # the sweep's NLL against the oracle's definition on a 20k-frame prefix
    Tn = 20000
    pre = st[:, :Tn].astype(np.float64)
    pp, ev = O.ensemble_array(pre)
    for i in (0, best):
        c = cands[i]
        want = O.compute_nll(pp - c["offset"], c["m0"], c["S0"], c["C"], c["A"], c["Q"], ev)
        got = float(batch.nll(obs[:, :Tn], params[i:i + 1].contiguous(), n=8, r=3)[0])
        assert math.isclose(got, want, rel_tol=1e-9), (i, got, want)
        got = float(batch.nll(obs[:, :Tn], params[i:i + 1].contiguous(), n=8, r=3,
                              flags=flags)[0])
        assert math.isclose(got, want, rel_tol=1e-9), (i, got, want)
    del ref
