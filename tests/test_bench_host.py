"""Host logic of bench.py that needs no GPU: the all-core CPU baseline
(one spawned process per core, numpy oracle, BLAS single-threaded) gives
the same outputs as the in-process 1-core run, tasks in order; the N-rank
self-launch builds a torch.distributed.run command."""
import os
import sys

import numpy as np
import pytest

import bench
from eks_amd import synthetic


def _tasks(n, T=400):
    st = synthetic.singleview_obs(np.random.default_rng(7), 5, T, K=n).astype(np.float64)
    return [("singleview", np.ascontiguousarray(st[:, :, k, :]), (0.01, 25.0)) for k in range(n)]


def test_cpu_all_cores_matches_one_core():
    tasks = _tasks(5)
    before = os.environ.get("OPENBLAS_NUM_THREADS")
    _, hot, outs1 = bench.cpu_one_core(tasks)
    assert len(hot) == 5 and all(h > 0 for h in hot)
    wall, outs = bench.cpu_all_cores(tasks, 2)
    assert wall > 0
    for a, b in zip(outs1, outs):
        assert a.shape == (400, 2)
        np.testing.assert_array_equal(a, b)
    # the environment of this process is restored
    assert os.environ.get("OPENBLAS_NUM_THREADS") == before


def test_cpu_nll_task_is_oracle_nll():
    from oracle import eks_oracle as O
    t = _tasks(1)[0]
    preds, ev = O.ensemble_array(t[1])
    p = O.singleview_params(preds, ev, 0.01, 25.0)
    task = ("nll", t[1], p)
    _, _, outs = bench.cpu_one_core([task])
    ref = O.compute_nll(preds - p["means"], p["m0"], p["S0"], p["C"], p["A"], p["Q"], ev)
    assert outs[0] == ref


def test_cpu_cores_respects_cap(monkeypatch):
    monkeypatch.setenv("EKS_CPU_CORES", "1")
    assert bench.cpu_cores() == 1
    monkeypatch.delenv("EKS_CPU_CORES")
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    assert bench.cpu_cores() == min(3, len(os.sched_getaffinity(0)))


def test_launch_ranks_command(monkeypatch):
    seen = {}

    def fake_call(cmd, env):
        seen["cmd"], seen["env"] = cmd, env
        return 0

    import subprocess
    monkeypatch.setattr(subprocess, "call", fake_call)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3"])
    a = bench.parse()
    assert bench.launch_ranks(a) == 0
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"]
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_cpu_task_kinds_match_oracle_smoothers():
    """Each task kind's untimed fit + timed hot path equals the oracle's
    whole-path function for that kind."""
    from oracle import eks_oracle as O
    rng = np.random.default_rng(11)
    st_p = synthetic.pupil_obs(rng, 5, 300).astype(np.float64)               # (E, T, 8)
    A = np.diag([0.99, 0.98, 0.98])
    st_m = synthetic.multiview_obs(rng, 3, 5, 300, K=1)[:, :, 0].astype(np.float64)  # (E, T, 6)
    tasks = [("pupil", st_p, (A,)), ("multicam", st_m, (0.01, 25.0)), _tasks(1)[0]]
    _, _, outs = bench.cpu_one_core(tasks)
    np.testing.assert_array_equal(outs[0], O.pupil_smooth(st_p, A)[0])
    cams = [st_m[:, :, 2 * c:2 * c + 2] for c in range(3)]
    np.testing.assert_allclose(outs[1], O.multicam_smooth(cams, 0.01, 25.0)[0], rtol=0, atol=1e-9)
    np.testing.assert_array_equal(outs[2], O.singleview_smooth(tasks[2][1], 0.01, 25.0)[0])


def test_multi_rank_line_schema(tmp_path, monkeypatch):
    """An N > 1 line (the driver's SCALE runs) carries the CPU baseline (rank
    0's shard), the PMC traffic of one rank's launch (looked up by the
    per-rank shard key, i.e. the entry an N = 1 run of that shard size
    wrote), the distributed block and the timed RCCL gather."""
    import json
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8"])
    a = bench.parse()
    assert bench.runs_cpu_baseline(0, a) and not bench.runs_cpu_baseline(1, a)
    key = "config4-singleview-v128-k17-e5-t10000-a3"
    pmc = tmp_path / "bench_pmc.json"
    pmc.write_text(json.dumps({"entries": {key: {"hbm_bytes_per_launch": 2.5e9}}}))
    w = dict(key=key, desc="config 4 shard", cfg=dict(videos=1024, trajectories_per_rank=2176),
             bytes_per_unit=56, units=2176 * 10000)
    cpu = dict(value=1e5, unit="kp-ts/s", cores=16, kind="port", sample="...")
    line = bench.make_line(a, w, 8, 3, 2176 * 10000, 17408 * 10000, 0.01 * a.steps,
                           [("k3_fwd", 0.2), ("k3_bwd", 0.3)], 0.5, cpu, 1e-11, None, None,
                           3.2, 2.79e9, 1.0, True, "nccl", pmc_path=str(pmc))
    assert line["n_gpus"] == 8 and line["scaling"] == "strong"
    assert line["cpu_baseline"] is cpu
    assert line["roofline"]["traffic"] == 2.5e9
    assert line["distributed"]["world_size"] == 8 and line["distributed"]["backend"] == "nccl"
    assert line["gather_ms"] == 3.2 and line["gather_bytes"] == 2.79e9
    # the gather priced into the rate: kp-ts over (step time + gather time)
    assert line["value_with_gather"] == pytest.approx(17408 * 10000 / (0.01 + 3.2e-3))
    assert line["value"] == 17408 * 10000 / 0.01
    # the N = 1 line of the full batch looks up its own entry
    assert bench.load_pmc("config4-singleview-v1024-k17-e5-t10000-a3", str(pmc)) is None
