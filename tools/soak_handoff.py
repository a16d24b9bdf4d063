"""Soak run of the in-launch hand-offs on the GPU: the chained passes (algo 3,
algo 2's chained scans) called REPS times on one input, every result compared
bit for bit with the first call's, and once with algo 1 (sequential kernels,
no hand-offs).  A race in the publish / poll protocol (handoff.hpp) would
show as a differing call.  Prints one line per case; exit status 1 on any
mismatch.

    python tools/soak_handoff.py [REPS]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(reps):
    import torch
    from eks_amd import _lib, batch, synthetic
    flags = _lib.EKS_MODEL_A_IDENTITY | _lib.EKS_MODEL_C_IDENTITY
    bad = 0
    # (algo, trajectories, frames): the 8-GPU shard of config 4 (34 trajectory
    # groups, long chains), a quarter of config 4 at 2 000 frames, config 2's
    # geometry through algo 2's chained group scans
    for algo, B, T in ((3, 2176, 10000), (3, 4352, 2000), (2, 17, 100000)):
        rng = np.random.default_rng(B + T)
        st = synthetic.singleview_obs(rng, 5, T, K=B).transpose(2, 0, 1, 3).astype(np.float32)
        d = batch.make_time_major(st, dtype=np.float32)
        params = batch.fit(d, kind="singleview", n=2, r=2, smooth_param=0.01, quantile_keep=25)[0]
        ref1 = batch.smooth(d, params, n=2, r=2, algo=1, flags=flags, want_nll=True)
        first = batch.smooth(d, params, n=2, r=2, algo=algo, flags=flags, want_nll=True)
        diff = 0
        t0 = time.time()
        for _ in range(reps):
            r = batch.smooth(d, params, n=2, r=2, algo=algo, flags=flags, want_nll=True)
            same = (torch.equal(r["out"], first["out"]) and torch.equal(r["nll"], first["nll"])
                    and int(r["status"].abs().sum()) == 0)
            diff += 0 if same else 1
        torch.cuda.synchronize()
        dt = time.time() - t0
        vs1 = float((first["out"] - ref1["out"]).abs().max())
        print(f"algo {algo} B={B} T={T}: {reps} calls in {dt:.1f} s, {diff} differing from the "
              f"first; max|algo {algo} - algo 1| = {vs1:.2e}", flush=True)
        bad += diff + (vs1 > 1e-8)
        del d, params, ref1, first
        torch.cuda.empty_cache()
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(int(sys.argv[1]) if len(sys.argv) > 1 else 200))
