"""Genes x samples CSV writer (gm2.extras.write_samples_to_dataframe) byte-identical to the
reference's pandas route (extras.py:31-39, restated inline here as the checker)."""
import numpy as np
import pandas as pd
import pytest

from gm2.extras import write_samples_to_dataframe


def reference_csv(samples, genes, path):
    df = pd.DataFrame(samples, columns=genes)
    df.index = [f"Sample_{i+1}" for i in range(df.shape[0])]
    df = df.transpose()
    df.columns = [f"Sample_{i+1}" for i in range(df.shape[1])]
    df = df.reset_index()
    df = df.rename(columns={'index': 'Gene'})
    df.to_csv(path, index=False)


@pytest.mark.parametrize("dtype", [np.float64, np.float32, np.uint8, np.int64])
@pytest.mark.parametrize("n", [1, 7, 300])
def test_csv_matches_pandas(tmp_path, dtype, n):
    rng = np.random.default_rng(n)
    G = 37
    genes = [f"g{i}" for i in range(G)]
    genes[3], genes[5], genes[9] = "a,b", 'q"uote', "group_1234"
    m = (rng.random((n, G)) < 0.4).astype(dtype)
    a, b = tmp_path / "a.csv", tmp_path / "b.csv"
    write_samples_to_dataframe(m, genes, a, max_chunk_bytes=64)  # several gene blocks
    reference_csv(m, genes, b)
    assert a.read_bytes() == b.read_bytes()


def test_csv_non_binary_falls_back(tmp_path):
    m = np.array([[0.25, 1.0], [0.0, 0.5]])
    a, b = tmp_path / "a.csv", tmp_path / "b.csv"
    write_samples_to_dataframe(m, ["x", "y"], a)
    reference_csv(m, ["x", "y"], b)
    assert a.read_bytes() == b.read_bytes()
