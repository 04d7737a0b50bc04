"""gm2.data.read_matrix_csv: the numpy parse of the pan-genome CSV must give exactly what
pd.read_csv(path, index_col=0, header=0) gives (data_exploration.py:54-107 reads it that way) --
values, dtypes, index and column labels -- on the reference's layout, and fall back to pandas on
every other form. Also load_and_validate_data's three frames through both readers."""
import os

import numpy as np
import pandas as pd
import pytest


def _check(path):
    from gm2.data import read_matrix_csv
    got = read_matrix_csv(path)
    want = pd.read_csv(path, index_col=0, header=0)
    pd.testing.assert_frame_equal(got, want, check_exact=True)
    return got


def test_reference_layout_fast_path(tmp_path, monkeypatch):
    from gm2 import data
    from gm2.data import load_and_validate_data, write_synthetic_csvs
    root = str(tmp_path)
    write_synthetic_csvs(root, 37, 211, seed=9)
    path = os.path.join(root, "data", "F4_complete_presence_absence.csv")
    # the fast path is taken (pandas' reader is not called) and equals pandas
    calls = []
    real = pd.read_csv
    monkeypatch.setattr(pd, "read_csv", lambda *a, **k: calls.append(a) or real(*a, **k))
    got = data.read_matrix_csv(path)
    assert calls == []
    monkeypatch.setattr(pd, "read_csv", real)
    pd.testing.assert_frame_equal(got, real(path, index_col=0, header=0), check_exact=True)
    phylo = os.path.join(root, "data", "accessionID_phylogroup_BD.csv")
    a = load_and_validate_data(path, phylo)
    monkeypatch.setattr(data, "read_matrix_csv", lambda p: real(p, index_col=0, header=0))
    b = load_and_validate_data(path, phylo)
    for x, y in zip(a, b):
        pd.testing.assert_frame_equal(x, y, check_exact=True)


@pytest.mark.parametrize("case", ["lineage_ints", "other_ints", "crlf", "quoted", "na_cell", "numeric_names",
                                  "na_name", "dup_cols", "blank_col", "index_name", "space_cell", "ragged"])
def test_other_forms_equal_pandas(tmp_path, case):
    rng = np.random.default_rng(3)
    n, g = 6, 9
    x = (rng.random((g, n)) < 0.4).astype(int)
    cols = [f"s{i}" for i in range(n)]
    names = [f"g{i}" for i in range(g)]
    lineage = [3, 1, 12, 7, 2, 40]
    rows = [["Lineage"] + [str(v) for v in lineage]] + [[nm] + [str(v) for v in r] for nm, r in zip(names, x)]
    head = [""] + cols
    nl = "\n"
    if case == "other_ints":
        rows[3][2] = "2"
    elif case == "crlf":
        nl = "\r\n"
    elif case == "quoted":
        rows[2][0] = '"g1"'
    elif case == "na_cell":
        rows[4][3] = "NA"
    elif case == "numeric_names":
        rows[5][0] = "123"
    elif case == "na_name":
        rows[5][0] = "NA"
    elif case == "dup_cols":
        head[2] = head[1]
    elif case == "blank_col":
        head[3] = ""
    elif case == "index_name":
        head[0] = "gene"
    elif case == "space_cell":
        rows[2][2] = " 1"
    elif case == "ragged":
        rows[3] = rows[3][:-1]
    p = tmp_path / "m.csv"
    p.write_text(nl.join(",".join(r) for r in [head] + rows) + nl)
    if case == "ragged":
        from gm2.data import read_matrix_csv
        try:
            want = pd.read_csv(p, index_col=0, header=0)
        except Exception as e:  # pandas' own error, raised by the fallback as well
            with pytest.raises(type(e)):
                read_matrix_csv(p)
            return
        pd.testing.assert_frame_equal(read_matrix_csv(p), want, check_exact=True)
        return
    _check(p)
