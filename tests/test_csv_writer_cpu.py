"""Genes x samples CSV writer (gm2.extras.write_samples_to_dataframe) byte-identical to the
reference's own function (extras.py:31-39), pinned by tests/golden/csv_writer.npz: the bytes that
function wrote for each sample matrix (tests/golden/make_golden_csv.py runs it, extracted with `ast`,
in the build container)."""
import os

import numpy as np
import pytest

from gm2.extras import write_samples_to_dataframe

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "csv_writer.npz")


def _golden():
    return np.load(GOLD, allow_pickle=False)


@pytest.mark.parametrize("dtype", ["float64", "float32", "uint8", "int64", "bool"])
@pytest.mark.parametrize("n", [1, 7, 300])
@pytest.mark.parametrize("chunk", [64, None])
def test_csv_matches_reference_bytes(tmp_path, dtype, n, chunk):
    z = _golden()
    tag = f"{dtype}_{n}"
    m = z[f"{tag}_samples"]
    assert m.dtype == np.dtype(dtype)
    out = tmp_path / "a.csv"
    kw = {"max_chunk_bytes": chunk} if chunk else {}
    write_samples_to_dataframe(m, [str(g) for g in z["genes37"]], out, **kw)  # 64: several gene blocks
    assert out.read_bytes() == z[f"{tag}_csv"].tobytes()


def test_csv_non_binary_matches_reference_bytes(tmp_path):
    z = _golden()
    out = tmp_path / "a.csv"
    write_samples_to_dataframe(z["frac_samples"], [str(g) for g in z["frac_genes"]], out)
    assert out.read_bytes() == z["frac_csv"].tobytes()
