"""Shared pieces of the CLI scripts: save-dir handling and the example plot
(scripts/multicam_example.py:156-201, scripts/pupil_example.py:117-152)."""
from __future__ import annotations

import os


def resolve_save_dir(save_dir):
    """The reference's default: ./outputs (created), else the given path."""
    if save_dir is None:
        save_dir = os.path.join(os.getcwd(), 'outputs')
        os.makedirs(save_dir, exist_ok=True)
    return save_dir


def example_plot(markers_list, member_col, eks_df, eks_col, title, save_file):
    """Members (grey) and EKS (black) for frames 0-500 of one keypoint, three
    panels x / y / likelihood, saved as PDF.  Skipped without matplotlib."""
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except ImportError:  # pragma: no cover
        print("matplotlib not available: no example plot")
        return None
    idxs = (0, 500)
    fig, axes = plt.subplots(3, 1, figsize=(9, 6))
    for ax, coord in zip(axes, ['x', 'y', 'likelihood']):
        for m, markers_curr in enumerate(markers_list):
            ax.plot(markers_curr.loc[slice(*idxs), member_col(coord)], color=[0.5, 0.5, 0.5],
                    label='Individual models' if m == 0 else None)
        ax.set_ylabel(coord, fontsize=12)
        ax.set_xlabel('Time (frames)', fontsize=12)
        if coord == 'likelihood':
            continue
        ax.plot(eks_df.loc[slice(*idxs), eks_col(coord)], color='k', linewidth=2, label='EKS')
        if coord == 'x':
            ax.legend()
    plt.suptitle(title, fontsize=14)
    plt.tight_layout()
    plt.savefig(save_file)
    plt.close()
    return save_file
