"""count_essential_genes (utils/extras.py:49-87) pinned to the reference's own function: goldens in
tests/golden/essential.npz were produced by running the reference's count_essential_genes
(tests/golden/make_golden_essential.py). Host path of gm2.extras and the oracle's loop restatement.
The device path (packed masks, gm2_mask_count_groups) is checked against the same goldens in
tests/test_gpu_masks.py."""
import numpy as np
import pytest

from golden_io import load

G_ = load("essential")
CASES = [str(c) for c in G_["cases"]]


def _dict(name):
    offs, pos = G_[f"{name}_offsets"], G_[f"{name}_positions"]
    return {f"g{i}": [int(p) for p in pos[offs[i]:offs[i + 1]]] for i in range(len(offs) - 1)}


@pytest.mark.parametrize("name", CASES)
def test_host_count_matches_reference(name):
    from gm2.extras import count_essential_genes
    got = count_essential_genes(G_[f"{name}_masks"], _dict(name))
    np.testing.assert_array_equal(got, G_[f"{name}_counts"])


@pytest.mark.parametrize("name", CASES)
def test_oracle_loop_matches_reference(name):
    from oracle import vae_oracle as O
    got = O.count_essential_genes_loop(G_[f"{name}_masks"], _dict(name))
    np.testing.assert_array_equal(got, G_[f"{name}_counts"])


def test_essential_groups_csr():
    from gm2.masks import essential_groups
    offs, pos = essential_groups({"a": [1, 9, 3], "b": [12], "c": [-2, 40]}, 10)
    assert offs.tolist() == [0, 3, 3, 4] and pos.tolist() == [1, 9, 3, 8]
    with pytest.raises(IndexError):
        essential_groups({"a": [-11]}, 10)
