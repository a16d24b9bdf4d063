"""Multi-camera EKS from the command line -- same flags, inputs and output
files as the reference's scripts/multicam_example.py:13-201.

    python -m eks_amd.scripts.multicam_example --csv-dir DIR \
        --bodypart-list paw1LH paw2LF --camera-names top bot \
        [--save-dir OUT] [--s 0.01] [--quantile_keep_pca 25] --eks_version {opti,standard}

Writes <save-dir>/eks.csv (or eks_opti.csv for --eks_version opti) in the
input CSVs' 3-row header format with scorer 'ensemble-kalman_tracker' and
likelihood 1.0, plus the example plot.  Differences from the reference
script, all additive: the CSVs are parsed by the native reader
(eks_amd.io), every body part is smoothed in ONE batched GPU call
(eks_amd.smoothers.multi_cam_batch), and --no-plot skips the PDF.  The
column selection keeps the reference's substring rule (:112-117).
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np


def build_parser():
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument('--csv-dir', required=True, type=str,
                   help='directory of model prediction csv files')
    p.add_argument('--bodypart-list', required=True, nargs='+',
                   help='the list of body parts to be ensembled and smoothed')
    p.add_argument('--camera-names', required=True, nargs='+', help='the camera names')
    p.add_argument('--save-dir', default=None, type=str,
                   help='save directory for outputs (default is ./outputs)')
    p.add_argument('--s', default=.01, type=float,
                   help='smoothing parameter ranges from .01-2 (smaller values = more smoothing)')
    p.add_argument('--quantile_keep_pca', default=25, type=float,
                   help='percentage of the points are kept for multi-view PCA '
                        '(lowest ensemble variance)')
    p.add_argument('--eks_version', required=True, type=str,
                   help='choose eks version: "opti" (Newton filter) or anything else (standard)')
    p.add_argument('--no-plot', action='store_true', help='do not write the example plot')
    return p


def select_columns(markers, camera_name, keypoint):
    """scripts/multicam_example.py:112-117: keys containing the camera name
    and the keypoint name (substrings) and not 'likelihood'."""
    return [k for k in markers.keys()
            if camera_name in k and 'likelihood' not in k and keypoint in k]


def run(args) -> str:
    from eks_amd import io
    from eks_amd.scripts._common import example_plot, resolve_save_dir
    from eks_amd.smoothers import multi_cam_batch
    from eks_amd.utils import TRACKER

    csv_dir = os.path.abspath(args.csv_dir)
    if not os.path.isdir(csv_dir):
        raise ValueError('--csv-dir must be a valid directory containing prediction csv files')
    save_dir = resolve_save_dir(args.save_dir)
    markers_list, _, raw = io.load_markers_dir(csv_dir)
    markers_eks = io.output_template(raw)
    cams = args.camera_names
    stacks = []
    for kp in args.bodypart_list:
        per_cam = []
        for cam in cams:
            cols = []
            for m in markers_list:
                keys = select_columns(m, cam, kp)
                if len(keys) < 2:
                    raise KeyError(f"no x/y columns for body part {kp!r} in camera {cam!r}")
                cols.append(m[keys].to_numpy()[:, :2])  # positional, as the reference
            per_cam.append(np.stack(cols))  # (E, T, 2)
        stacks.append(np.concatenate(per_cam, axis=2))  # (E, T, 2V)
    opti = args.eks_version == "opti"
    out = multi_cam_batch(np.stack(stacks), args.s, args.quantile_keep_pca,
                          version="opti" if opti else "standard")
    for k, kp in enumerate(args.bodypart_list):
        for c, cam in enumerate(cams):
            for j, coord in enumerate(('x', 'y')):
                markers_eks.loc[:, (TRACKER, f'{kp}_{cam}', coord)] = out[k, :, 2 * c + j]
    save_file = os.path.join(save_dir, 'eks_opti.csv' if opti else 'eks.csv')
    markers_eks.to_csv(save_file)
    print(f'saved EKS output to {save_file}')
    if not args.no_plot:
        kp, cam = args.bodypart_list[0], cams[0]
        pdf = example_plot(markers_list, lambda c: f'{kp}_{cam}_{c}', markers_eks,
                           lambda c: (TRACKER, f'{kp}_{cam}', c),
                           f'EKS results for {kp} ({cam} view)',
                           os.path.join(save_dir, 'example_eks_opti_result.pdf' if opti
                                        else 'example_eks_result.pdf'))
        if pdf:
            print(f'see example EKS output at {pdf}')
    return save_file


def main(argv=None) -> int:
    run(build_parser().parse_args(argv))
    return 0


if __name__ == "__main__":
    sys.exit(main())
