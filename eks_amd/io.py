"""DLC / Lightning-Pose CSV I/O on the native reader (F1).

    read_csv_array(path)      native parse -> (header rows, index, data (T, C))
    read_dlc_csv(path)        the DataFrame pd.read_csv(path, header=[0, 1, 2],
                              index_col=0) returns (scripts/multicam_example.py:88)
    load_markers_dir(csv_dir) the scripts' directory loop
                              (scripts/multicam_example.py:83-94,
                              scripts/pupil_example.py:63-74)
    member_stack(...)         (E, T, n) float64 member array for chosen columns,
                              straight from the parsed arrays (no DataFrames)
    output_template(raw)      the scripts' output frame: scorer renamed to
                              'ensemble-kalman_tracker', likelihood 1.0, the
                              rest NaN (scripts/multicam_example.py:96-103)

The parse itself (eks_csv_probe / eks_csv_read in include/eks_io.h) is
multi-threaded C++ with correctly rounded float conversion; pandas is used
only to wrap the arrays into the reference's DataFrame shapes and to write.
"""
from __future__ import annotations

import csv
import ctypes as C
import io as _io
import os

import numpy as np
import pandas as pd

from . import _lib
from .utils import TRACKER, convert_lp_dlc


class CsvError(RuntimeError):
    pass


def _check(code: int, what: str) -> None:
    if code != 0:
        msg = _lib.load().eks_io_last_error().decode(errors="replace")
        raise CsvError(f"{what}: {msg}")


def read_csv_array(path: str, header_rows: int = 3, nthreads: int = 0):
    """-> (header: list of header rows (list of cells), index (T,) float64,
    data (T, C) float64 without the index column)."""
    lib = _lib.load()
    bpath = os.fsencode(path)
    rows, cols, hb = C.c_int64(), C.c_int64(), C.c_int64()
    _check(lib.eks_csv_probe(bpath, header_rows, C.byref(rows), C.byref(cols), C.byref(hb)), path)
    data = np.empty((rows.value, cols.value), dtype=np.float64)
    index = np.empty(rows.value, dtype=np.float64)
    hbuf = C.create_string_buffer(hb.value)
    _check(lib.eks_csv_read(bpath, header_rows, data.ctypes.data, rows.value, cols.value,
                            index.ctypes.data, hbuf, hb.value, nthreads), path)
    header = list(csv.reader(_io.StringIO(hbuf.value.decode())))
    return header, index, data


def read_dlc_csv(path: str) -> pd.DataFrame:
    """Same frame as pd.read_csv(path, header=[0, 1, 2], index_col=0)."""
    header, index, data = read_csv_array(path, 3)
    names = [h[0] if h else None for h in header]
    tuples = list(zip(*[h[1:] for h in header]))
    if len(tuples) != data.shape[1]:
        raise CsvError(f"{path}: {len(tuples)} header columns but {data.shape[1]} data columns")
    columns = pd.MultiIndex.from_tuples(tuples, names=names)
    if np.all(np.isfinite(index)) and np.all(index == np.round(index)):
        idx = pd.Index(index.astype(np.int64))
    else:
        idx = pd.Index(index)
    return pd.DataFrame(data, index=idx, columns=columns)


def load_markers_dir(csv_dir: str):
    """The scripts' loader: every '*csv' file of csv_dir in os.listdir order
    (as the reference), parsed and flattened with convert_lp_dlc.  Returns
    (markers_list, keypoint_names, last_raw_frame)."""
    if not os.path.isdir(csv_dir):
        raise ValueError('--csv-dir must be a valid directory containing prediction csv files')
    markers_list, keypoint_names, raw = [], None, None
    for f in os.listdir(csv_dir):
        if not f.endswith('csv'):
            continue
        raw = read_dlc_csv(os.path.join(csv_dir, f))
        keypoint_names = [c[1] for c in raw.columns[::3]]
        markers_list.append(convert_lp_dlc(raw, keypoint_names, model_name=raw.columns[0][0]))
    if not markers_list:
        raise FileNotFoundError(f'No marker csv files found in {csv_dir}')
    return markers_list, keypoint_names, raw


def member_stack(markers_list, columns) -> np.ndarray:
    """(E, T, len(columns)) float64 array of the members' chosen columns."""
    return np.stack([np.stack([np.asarray(m[c], dtype=np.float64) for c in columns], axis=1)
                     for m in markers_list])


def output_template(raw: pd.DataFrame) -> pd.DataFrame:
    """scripts/multicam_example.py:96-103: copy of the last input frame with
    scorer 'ensemble-kalman_tracker', likelihood columns 1.0, others NaN."""
    out = raw.copy()
    out.columns = out.columns.set_levels([TRACKER], level=0)
    lik = np.array([c[-1] == 'likelihood' for c in out.columns])
    vals = np.where(lik[None, :], 1.0, np.nan) * np.ones((len(out), 1))
    return pd.DataFrame(vals, index=out.index, columns=out.columns)
