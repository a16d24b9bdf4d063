"""F1: native DLC/LP CSV reader and the script-level loader, on the
committed fixtures (first 300 frames of the reference's example data).
CPU only: the reader is host code in libeks_hip.so."""
import glob
import os

import numpy as np
import pandas as pd
import pytest

from eks_amd import io
from eks_amd.utils import convert_lp_dlc
from tests.conftest import GOLDEN

CSV = os.path.join(GOLDEN, "csv")
FILES = sorted(glob.glob(os.path.join(CSV, "mirror-mouse", "*.csv")) +
               glob.glob(os.path.join(CSV, "ibl-pupil", "*.csv")))


@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(p) for p in FILES])
def test_read_dlc_csv_matches_pandas(path):
    ours = io.read_dlc_csv(path)
    ref = pd.read_csv(path, header=[0, 1, 2], index_col=0, float_precision="round_trip")
    assert list(ours.columns) == list(ref.columns)
    assert list(ours.columns.names) == list(ref.columns.names)
    assert (ours.index == ref.index).all()
    # bit-exact against the correctly rounded parse
    assert np.array_equal(ours.to_numpy(), ref.to_numpy(), equal_nan=True)
    # and within an ulp of pandas' default parser (what the reference uses)
    dflt = pd.read_csv(path, header=[0, 1, 2], index_col=0)
    np.testing.assert_allclose(ours.to_numpy(), dflt.to_numpy(), rtol=4e-16, atol=0)
    assert ours.to_csv() == ref.to_csv()


def test_threads_do_not_change_result(tmp_path):
    rng = np.random.default_rng(0)
    T, K = 20000, 7
    cols = pd.MultiIndex.from_product([["m"], [f"k{i}" for i in range(K)], ["x", "y", "likelihood"]],
                                      names=["scorer", "bodyparts", "coords"])
    df = pd.DataFrame(rng.normal(size=(T, 3 * K)) * 100, columns=cols)
    df.iloc[5, 3] = np.nan
    p = tmp_path / "big.csv"
    df.to_csv(p)
    h1, i1, d1 = io.read_csv_array(str(p), 3, nthreads=1)
    h8, i8, d8 = io.read_csv_array(str(p), 3, nthreads=8)
    assert np.array_equal(d1, d8, equal_nan=True) and np.array_equal(i1, i8)
    assert np.array_equal(d1, df.to_numpy(), equal_nan=True)  # to_csv writes repr -> exact
    assert h1[1][1] == "k0" and h1[0][0] == "scorer"


def test_na_blank_and_crlf(tmp_path):
    p = tmp_path / "na.csv"
    p.write_bytes(b"scorer,s,s\r\nbodyparts,a,a\r\ncoords,x,y\r\n0,1.5,\r\n1,NaN,nan\r\n\r\n"
                  b"2, 3e2 ,N/A\r\n")
    ours = io.read_dlc_csv(str(p))
    ref = pd.read_csv(p, header=[0, 1, 2], index_col=0)
    np.testing.assert_array_equal(ours.to_numpy(), ref.to_numpy())
    assert list(ours.index) == [0, 1, 2]


def test_errors(tmp_path):
    with pytest.raises(io.CsvError, match="cannot open"):
        io.read_csv_array(str(tmp_path / "missing.csv"))
    p = tmp_path / "bad.csv"
    p.write_text("a,b\nc,d\ne,f\n0,1.0\n1,abc\n")
    with pytest.raises(io.CsvError, match="non-numeric"):
        io.read_csv_array(str(p))
    p.write_text("a,b\nc,d\ne,f\n0,1.0\n1,2.0,3.0\n")
    with pytest.raises(io.CsvError, match="number of fields"):
        io.read_csv_array(str(p))
    p.write_text("a,b\n")
    with pytest.raises(io.CsvError, match="header"):
        io.read_csv_array(str(p))


def test_load_markers_dir_and_template():
    d = os.path.join(CSV, "mirror-mouse")
    ml, kps, raw = io.load_markers_dir(d)
    assert len(ml) == 5 and kps[0] == "paw1LH_top"
    # same flattening as the scripts' pd.read_csv + convert_lp_dlc
    f = os.path.join(d, sorted(os.listdir(d))[0])
    ref_raw = pd.read_csv(f, header=[0, 1, 2], index_col=0)
    ref = convert_lp_dlc(ref_raw, kps, model_name=ref_raw.columns[0][0])
    ours = convert_lp_dlc(io.read_dlc_csv(f), kps, model_name=ref_raw.columns[0][0])
    assert list(ours.columns) == list(ref.columns)
    np.testing.assert_allclose(ours.to_numpy(), ref.to_numpy(), rtol=4e-16)
    tpl = io.output_template(raw)
    assert set(tpl.columns.get_level_values(0)) == {"ensemble-kalman_tracker"}
    lik = [c[-1] == "likelihood" for c in tpl.columns]
    assert (tpl.loc[:, lik].to_numpy() == 1.0).all()
    assert np.isnan(tpl.loc[:, [not x for x in lik]].to_numpy()).all()
    st = io.member_stack(ml, ["paw2LF_top_x", "paw2LF_top_y"])
    assert st.shape == (5, 300, 2)
    with pytest.raises(ValueError):
        io.load_markers_dir(os.path.join(CSV, "nope"))
