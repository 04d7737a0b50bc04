#!/usr/bin/env python3
"""Golden vectors for `--mode convert-samples` by IMPORTING the reference's
explore_data/binary_converter.py (masks_to_gene_lists :19-76, load_files :11-17,
check_essential_genes :78-121). Run here only (the reference is absent on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_converter.py

Writes tests/golden/converter.json: inputs (gene columns, masks, essential genes) and the
reference's outputs (gene-id lists before and after the essential-gene fill, the saved arrays'
ndim/shape, or the error raised). Data only."""
import importlib.util
import json
import os
import sys
import tempfile

import numpy as np
import pandas as pd

sys.dont_write_bytecode = True
REF = "/root/reference/src/genome_minimizer_2/explore_data/binary_converter.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "converter.json")

spec = importlib.util.spec_from_file_location("ref_binary_converter", REF)
bc = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bc)


def to_json(arr):
    return [list(map(str, row)) for row in arr]


def run_case(name, cols, masks, essentials, ess_col="gene", mask_dtype="float64"):
    case = {"name": name, "cols": list(map(str, cols)), "masks": np.asarray(masks).tolist(),
            "mask_dtype": mask_dtype, "essentials": essentials, "ess_col": ess_col}
    with tempfile.TemporaryDirectory() as d:
        mpath = os.path.join(d, "masks.npy")
        np.save(mpath, np.asarray(masks, dtype=mask_dtype))
        out = os.path.join(d, "ids.npy")
        try:
            bc.masks_to_gene_lists(masks_npy_path=mpath, cols=pd.Index(cols), out_ids_npy=out)
        except ValueError as e:
            case["error"] = str(e)
            return case
        ids = np.load(out, allow_pickle=True)  # written by the reference function just above
        case["ids"] = to_json(ids)
        case["ids_ndim"], case["ids_shape"] = int(ids.ndim), list(ids.shape)
        epath = os.path.join(d, "ess.csv")
        pd.DataFrame({ess_col: essentials}).to_csv(epath, index=False)
        ess_set, id_lists = bc.load_files(epath, out)
        filled = bc.check_essential_genes(ess_set, id_lists, out)
        f = np.load(filled, allow_pickle=True)
        case["filled"] = to_json(f)
        case["filled_ndim"], case["filled_shape"] = int(f.ndim), list(f.shape)
        case["filled_name"] = os.path.basename(filled)
    return case


def main():
    rng = np.random.Generator(np.random.PCG64(7))
    cols = [f"g{i:03d}" for i in range(12)]
    m = rng.random((5, 12))
    m[0, 3], m[1, 4], m[2, 5] = 0.5, 0.49999999, 1.0
    m[3] = 0.0
    cases = [
        run_case("float_masks", cols, m, ["g001", "g007", "zzz_missing"]),
        run_case("uint8_masks", cols, (m >= 0.5).astype(np.uint8), ["g002", "g011"], mask_dtype="uint8"),
        run_case("equal_length_rows", cols, np.tile((np.arange(12) % 3 == 0).astype(float), (4, 1)),
                 ["g000", "g003"], ess_col="# gene"),
        run_case("duplicate_columns", cols[:11] + ["g004"], m, ["g001"]),
    ]
    json.dump({"meta": {"generator": "tests/golden/make_golden_converter.py", "numpy": np.__version__,
                        "pandas": pd.__version__}, "cases": cases}, open(OUT, "w"), indent=0)
    print("wrote", OUT, [c["name"] + (" (error)" if "error" in c else "") for c in cases])


if __name__ == "__main__":
    main()
