"""IBL pupil EKS from the command line -- same flags, inputs and output
files as the reference's scripts/pupil_example.py:12-152.

    python -m eks_amd.scripts.pupil_example --csv-dir DIR [--save-dir OUT] \
        [--diameter-s .9999] [--com-s .999] --eks_version {opti,standard}

standard: kalman_smoothed_pupil_traces.csv + kalman_smoothed_latents.csv;
opti:     opti_eks_pupil_traces.csv + opti_eks_latents.csv;
plus example_eks_result.pdf (skip with --no-plot).  Additive option
--sweep D1,D2,... C1,C2,...: choose (diameter_s, com_s) from the grid by
innovation likelihood (eks_amd.smoothers.pupil_smoothing_sweep, one batched
filter-only GPU call) instead of taking --diameter-s/--com-s.
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np


def build_parser():
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument('--csv-dir', required=True, type=str, help='directory of models for ensembling')
    p.add_argument('--save-dir', default=None, type=str,
                   help='save directory for outputs (default is ./outputs)')
    p.add_argument('--diameter-s', default=.9999, type=float,
                   help='smoothing parameter for diameter (closer to 1 = more smoothing)')
    p.add_argument('--com-s', default=.999, type=float,
                   help='smoothing parameter for center of mass (closer to 1 = more smoothing)')
    p.add_argument('--eks_version', required=True, type=str,
                   help='choose eks version: "opti" (Newton filter) or anything else (standard)')
    p.add_argument('--sweep', nargs=2, default=None, metavar=('DIAMETER_S_LIST', 'COM_S_LIST'),
                   help='comma-separated grids; pick the pair with the lowest NLL (standard only)')
    p.add_argument('--no-plot', action='store_true', help='do not write the example plot')
    return p


def run(args):
    from eks_amd import io
    from eks_amd.scripts._common import example_plot, resolve_save_dir
    from eks_amd.smoothers import (ensemble_kalman_smoother_pupil, eks_opti_smoother_pupil,
                                   pupil_smoothing_sweep)
    from eks_amd.utils import TRACKER

    csv_dir = os.path.abspath(args.csv_dir)
    if not os.path.isdir(csv_dir):
        raise ValueError('--csv-dir must be a valid path to a directory')
    save_dir = resolve_save_dir(args.save_dir)
    markers_list, keypoint_names, _ = io.load_markers_dir(csv_dir)
    A = np.asarray([[args.diameter_s, 0, 0], [0, args.com_s, 0], [0, 0, args.com_s]])
    print(f'Smoothing matrix: {A}')
    kw = dict(markers_list=markers_list, keypoint_names=keypoint_names, tracker_name=TRACKER)
    if args.eks_version == "opti":
        d = eks_opti_smoother_pupil(state_transition_matrix=A, **kw)
        names = ('opti_eks_pupil_traces.csv', 'opti_eks_latents.csv')
    else:
        if args.sweep:
            dg = [float(x) for x in args.sweep[0].split(',')]
            cg = [float(x) for x in args.sweep[1].split(',')]
            d = pupil_smoothing_sweep(markers_list, keypoint_names, TRACKER, dg, cg)
            print(f'chosen (diameter_s, com_s) = {d["best"]}')
        else:
            d = ensemble_kalman_smoother_pupil(state_transition_matrix=A, **kw)
        names = ('kalman_smoothed_pupil_traces.csv', 'kalman_smoothed_latents.csv')
    files = []
    for key, name in zip(('markers_df', 'latents_df'), names):
        f = os.path.join(save_dir, name)
        print(f'saving {"smoothed predictions" if key == "markers_df" else "latents"} to {f}')
        d[key].to_csv(f)
        files.append(f)
    if not args.no_plot:
        kp = keypoint_names[0]
        pdf = example_plot(markers_list, lambda c: f'{kp}_{c}', d['markers_df'],
                           lambda c: (TRACKER, kp, c), f'EKS results for {kp}',
                           os.path.join(save_dir, 'example_eks_result.pdf'))
        if pdf:
            print(f'see example EKS output at {pdf}')
    return files


def main(argv=None) -> int:
    run(build_parser().parse_args(argv))
    return 0


if __name__ == "__main__":
    sys.exit(main())
