"""`--mode convert-samples`: gm2.binary_converter against golden outputs of the
reference's explore_data/binary_converter.py (tests/golden/converter.json, made by
tests/golden/make_golden_converter.py), and main.py's convert-samples route end to end. CPU only."""
import json
import os

import numpy as np
import pandas as pd
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = json.load(open(os.path.join(ROOT, "tests", "golden", "converter.json")))["cases"]


def _as_lists(arr):
    return [list(map(str, row)) for row in arr]


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_converter_matches_reference(case, tmp_path):
    from gm2 import binary_converter as bc
    mpath = tmp_path / "masks.npy"
    np.save(mpath, np.asarray(case["masks"], dtype=case["mask_dtype"]))
    out = str(tmp_path / "ids.npy")
    cols = pd.Index(case["cols"])
    if "error" in case:
        with pytest.raises(ValueError) as e:
            bc.masks_to_gene_lists(str(mpath), cols, out)
        assert str(e.value) == case["error"]
        return
    bc.masks_to_gene_lists(str(mpath), cols, out)
    ids = np.load(out, allow_pickle=True)  # written by our own code just above
    assert _as_lists(ids) == case["ids"]
    assert ids.ndim == case["ids_ndim"] and list(ids.shape) == case["ids_shape"]
    epath = tmp_path / "ess.csv"
    pd.DataFrame({case["ess_col"]: case["essentials"]}).to_csv(epath, index=False)
    ess, id_lists = bc.load_files(str(epath), out)
    filled = bc.check_essential_genes(ess, id_lists, out)
    assert os.path.basename(filled) == case["filled_name"]
    f = np.load(filled, allow_pickle=True)
    assert _as_lists(f) == case["filled"]
    assert f.ndim == case["filled_ndim"] and list(f.shape) == case["filled_shape"]


def test_cli_convert_samples(tmp_path):
    import main as cli
    from gm2.data import write_synthetic_csvs
    root = str(tmp_path)
    write_synthetic_csvs(root, 20, 50, seed=3)
    rng = np.random.Generator(np.random.PCG64(1))
    masks = (rng.random((6, 50)) < 0.4).astype(np.uint8)
    mpath = os.path.join(root, "masks.npy")
    np.save(mpath, masks)
    out = os.path.join(root, "out", "ids.npy")
    assert cli.main(["--mode", "convert-samples", "--genes-path", mpath, "--output-file", out,
                     "--project-root", root]) == 0
    ids = np.load(out, allow_pickle=True)
    genes = [f"gene{i:05d}" for i in range(50)]
    assert _as_lists(ids) == [[genes[j] for j in np.flatnonzero(r)] for r in masks]
    filled = np.load(os.path.join(root, "out", "ids_with_essentials.npy"), allow_pickle=True)
    ess = set(genes[: max(1, 50 // 20)])
    assert all(ess <= set(r) and list(r) == sorted(r) for r in filled)
    assert cli.main(["--mode", "convert-samples", "--genes-path", os.path.join(root, "nope.npy"),
                     "--project-root", root]) == 1
