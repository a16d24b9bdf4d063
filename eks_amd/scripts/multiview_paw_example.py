"""Asynchronous two-camera paw EKS from the command line -- same flags,
inputs and output files as the reference's scripts/multiview_paw_example.py.

    python -m eks_amd.scripts.multiview_paw_example --csv-dir DIR [--save-dir OUT] \
        [--s 1] [--quantile_keep_pca 25] --eks_version {opti,standard}

DIR holds the left / right camera member CSVs ('left' / other in the file
name) and one '*timestamps*left*.npy' and one '*timestamps*.npy' for the right
camera.  The right camera's paws are swapped on load, as in the reference
script.  Writes kalman_smoothed_paw_traces.{left,right}.csv (or
eks_opti_smoothed_paw_traces.{left,right}.csv).  Timestamps are read with
numpy.load(allow_pickle=False).
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

SWAP = {'paw_l_x': 'paw_r_x', 'paw_l_y': 'paw_r_y', 'paw_l_likelihood': 'paw_r_likelihood',
        'paw_r_x': 'paw_l_x', 'paw_r_y': 'paw_l_y', 'paw_r_likelihood': 'paw_l_likelihood'}


def build_parser():
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument('--csv-dir', required=True, type=str, help='directory of models for ensembling')
    p.add_argument('--save-dir', default=None, type=str,
                   help='save directory for outputs (default is ./outputs)')
    p.add_argument('--s', default=1, type=float,
                   help='smoothing parameter ranges from .01-2 (smaller values = more smoothing)')
    p.add_argument('--quantile_keep_pca', default=25, type=float,
                   help='percentage of the points are kept for multi-view PCA '
                        '(lowest ensemble variance)')
    p.add_argument('--eks_version', required=True, type=str,
                   help='choose eks version: "opti" (Newton filter) or anything else (standard)')
    return p


def run(args):
    from eks_amd import io
    from eks_amd.scripts._common import resolve_save_dir
    from eks_amd.smoothers import (ensemble_kalman_smoother_paw_asynchronous,
                                   eks_opti_smoother_paw_asynchronous)
    from eks_amd.utils import convert_lp_dlc

    csv_dir = os.path.abspath(args.csv_dir)
    if not os.path.isdir(csv_dir):
        raise ValueError('csv-dir must be a valid path to a directory')
    save_dir = resolve_save_dir(args.save_dir)
    left, right, tl, tr, keypoint_names = [], [], None, None, None
    for filename in os.listdir(csv_dir):  # the reference's loop (:70-97)
        path = os.path.join(csv_dir, filename)
        if 'timestamps' not in filename:
            raw = io.read_dlc_csv(path)
            keypoint_names = [c[1] for c in raw.columns[::3]]
            fmt = convert_lp_dlc(raw, keypoint_names, model_name=raw.columns[0][0])
            if 'left' in filename:
                left.append(fmt)
            else:
                right.append(fmt.rename(columns=SWAP).loc[:, list(SWAP.keys())])
        elif 'left' in filename:
            tl = np.load(path, allow_pickle=False)
        else:
            tr = np.load(path, allow_pickle=False)
    if tl is None or tr is None:
        raise ValueError('Need timestamps for both cameras')
    if len(right) != len(left) or len(left) == 0:
        raise ValueError('There must be the same number of left and right camera models and '
                         '>=1 model for each.')
    kw = dict(markers_list_left_cam=left, markers_list_right_cam=right, timestamps_left_cam=tl,
              timestamps_right_cam=tr, keypoint_names=keypoint_names, smooth_param=args.s,
              quantile_keep_pca=args.quantile_keep_pca)
    if args.eks_version == "opti":
        d = eks_opti_smoother_paw_asynchronous(**kw)
        prefix = 'eks_opti_smoothed_paw_traces'
    else:
        d = ensemble_kalman_smoother_paw_asynchronous(**kw)
        prefix = 'kalman_smoothed_paw_traces'
    files = []
    for view in ('left', 'right'):
        f = os.path.join(save_dir, f'{prefix}.{view}.csv')
        d[f'{view}_df'].to_csv(f)
        files.append(f)
    print(f'saved {files}')
    return files


def main(argv=None) -> int:
    run(build_parser().parse_args(argv))
    return 0


if __name__ == "__main__":
    sys.exit(main())
