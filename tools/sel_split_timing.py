"""Device-fit time by selection form (EKS_DBG_FIT_SELECT: 0 automatic, 1
one block per row, 2 split over row segments) across trajectory counts B and row lengths
T, to place the automatic switch (eks_fit.hip sel_split_auto).  Prints the
median ms of 10 timed fits (hand-off planes written) per (B, T, form).

    python tools/sel_split_timing.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from eks_amd import _lib, batch, synthetic
    prev = _lib.debug_set(_lib.EKS_DBG_FIT_SELECT, 0)
    try:
        for T in (10000, 50000):
            for B in (64, 128, 256, 512):
                rng = np.random.default_rng(B + T)
                st = synthetic.singleview_obs(rng, 5, T, K=B).transpose(2, 0, 1, 3).astype(np.float32)
                d = batch.make_time_major(st, dtype=np.float32)
                kw = dict(kind="singleview", n=2, r=2, smooth_param=0.01, quantile_keep=25,
                          check=False, keep_yev=True)
                res = {}
                for sel in (0, 1, 2):
                    _lib.debug_set(_lib.EKS_DBG_FIT_SELECT, sel)
                    for _ in range(3):
                        batch.fit(d, **kw)
                    ts = []
                    for _ in range(10):
                        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        a.record()
                        out = batch.fit(d, **kw)
                        b.record()
                        torch.cuda.synchronize()
                        ts.append(a.elapsed_time(b))
                    res[sel] = (float(np.median(ts)), out[0])
                same = torch.equal(res[1][1], res[2][1])
                same = same and torch.equal(res[0][1], res[1][1])
                print(f"T={T} B={B}: one block per row {res[1][0]:.4f} ms, split {res[2][0]:.4f} ms, "
                      f"automatic {res[0][0]:.4f} ms; parameters identical: {same}", flush=True)
                del d
                torch.cuda.empty_cache()
    finally:
        _lib.debug_set(_lib.EKS_DBG_FIT_SELECT, prev)


if __name__ == "__main__":
    main()
