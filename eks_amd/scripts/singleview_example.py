"""Single-view EKS for one or many videos from the command line.

    python -m eks_amd.scripts.singleview_example --csv-dir VIDEO_DIR [VIDEO_DIR ...] \
        [--bodypart-list kp1 kp2 ...] [--save-dir OUT] [--s 0.01] [--quantile_keep_pca 25] \
        [--ensembling-mode median]

Each VIDEO_DIR holds the E ensemble members' DLC/LP CSVs of one video (the
layout of the reference's examples, scripts/multicam_example.py:83-94).
The reference snapshot has no single-view script; this is the build's, with
the multicam script's flags and output format: per video
<save-dir>/eks.csv (or <save-dir>/<video dir name>/eks.csv for several
videos), scorer 'ensemble-kalman_tracker', likelihood 1.0.

All (video, body part) trajectories with the same frame count and member
count are smoothed in one batched GPU pass: ensemble (eks_ensemble), model
fit on the device (eks_amd.batch.fit -> eks_fit), fused smoother
(eks_smooth with the A = C = I kernels).
"""
from __future__ import annotations

import argparse
import os
import sys
from collections import defaultdict

import numpy as np


def build_parser():
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument('--csv-dir', required=True, nargs='+', type=str,
                   help='one directory of model prediction csv files per video')
    p.add_argument('--bodypart-list', nargs='+', default=None,
                   help='body parts to smooth (default: all)')
    p.add_argument('--save-dir', default=None, type=str,
                   help='save directory for outputs (default is ./outputs)')
    p.add_argument('--s', default=.01, type=float,
                   help='smoothing parameter (smaller values = more smoothing)')
    p.add_argument('--quantile_keep_pca', default=25, type=float,
                   help='percentage of lowest-variance frames used to fit the model')
    p.add_argument('--ensembling-mode', default='median', choices=['median', 'mean'])
    return p


def run(args):
    import torch

    from eks_amd import _lib, batch, io
    from eks_amd.scripts._common import resolve_save_dir
    from eks_amd.utils import TRACKER

    _lib.require_gpu()
    save_dir = resolve_save_dir(args.save_dir)
    videos = []
    for vd in args.csv_dir:
        markers_list, kps, raw = io.load_markers_dir(os.path.abspath(vd))
        bps = args.bodypart_list or kps
        stack = np.stack([io.member_stack(markers_list, [f'{kp}_x', f'{kp}_y']) for kp in bps])
        videos.append(dict(dir=vd, bps=bps, raw=raw, stack=stack))  # stack (K, E, T, 2)
    groups = defaultdict(list)
    for i, v in enumerate(videos):
        groups[v["stack"].shape[1:]].append(i)
    files = []
    for (E, T, _), members in groups.items():
        stacks = np.concatenate([videos[i]["stack"] for i in members])  # (B, E, T, 2)
        d = torch.from_numpy(np.ascontiguousarray(stacks, dtype=np.float64)).to("cuda")
        obs = d.permute(0, 2, 1, 3)                                      # (B, T, E, 2) view
        params, _ = batch.fit(obs, kind="singleview", n=2, r=2, smooth_param=args.s,
                              quantile_keep=args.quantile_keep_pca, mode=args.ensembling_mode)
        res = batch.smooth(obs, params, n=2, r=2, mode=args.ensembling_mode,
                           flags=_lib.EKS_MODEL_A_IDENTITY | _lib.EKS_MODEL_C_IDENTITY,
                           check=True)
        out = res["out"].cpu().numpy()
        row = 0
        for i in members:
            v = videos[i]
            eks = io.output_template(v["raw"])
            for kp in v["bps"]:
                eks.loc[:, (TRACKER, kp, 'x')] = out[row, :, 0]
                eks.loc[:, (TRACKER, kp, 'y')] = out[row, :, 1]
                row += 1
            sub = save_dir if len(videos) == 1 else os.path.join(
                save_dir, os.path.basename(os.path.normpath(v["dir"])))
            os.makedirs(sub, exist_ok=True)
            f = os.path.join(sub, 'eks.csv')
            eks.to_csv(f)
            files.append(f)
    torch.cuda.synchronize()
    print(f'saved {len(files)} EKS output file(s) under {save_dir}')
    return files


def main(argv=None) -> int:
    run(build_parser().parse_args(argv))
    return 0


if __name__ == "__main__":
    sys.exit(main())
