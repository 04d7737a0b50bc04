#!/usr/bin/env python3
"""Golden vectors for the genes x samples CSV writer, produced by the
REFERENCE'S OWN FUNCTION: utils/extras.py imports matplotlib / seaborn and the reference's model
module at import time, so this script parses it with `ast`, takes exactly
`write_samples_to_dataframe` (extras.py:31-39), compiles it alone with pandas as its only global,
and runs it on synthetic sample matrices. Nothing else of extras.py runs and no stand-in module is
written. Run here only (the reference is absent on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_csv.py

Writes tests/golden/csv_writer.npz: per case the sample matrix, the gene names and the bytes of the
CSV file the reference wrote. Data only."""
import ast
import json
import os
import sys
import tempfile

import numpy as np
import pandas as pd

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/src/genome_minimizer_2/utils/extras.py"
OUT = os.path.join(HERE, "csv_writer.npz")

tree = ast.parse(open(REF).read(), filename=REF)
fns = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "write_samples_to_dataframe"]
assert len(fns) == 1
mod = ast.fix_missing_locations(ast.Module(body=fns, type_ignores=[]))
ns = {"pd": pd}
exec(compile(mod, REF, "exec"), ns)
ref_write = ns["write_samples_to_dataframe"]


def genes_for(G):
    genes = [f"g{i}" for i in range(G)]
    genes[3], genes[5], genes[9] = "a,b", 'q"uote', "group_1234"
    return genes


out, cases = {}, []
with tempfile.TemporaryDirectory() as tmp:
    for dtype in ("float64", "float32", "uint8", "int64", "bool"):
        for n in (1, 7, 300):
            rng = np.random.default_rng(n)
            G = 37
            m = (rng.random((n, G)) < 0.4).astype(dtype)
            path = os.path.join(tmp, "out.csv")
            ref_write(m, genes_for(G), path)
            tag = f"{dtype}_{n}"
            out[f"{tag}_samples"] = m
            out[f"{tag}_csv"] = np.frombuffer(open(path, "rb").read(), dtype=np.uint8)
            cases.append(tag)
    # non-binary values (the writer's fallback route)
    m = np.array([[0.25, 1.0], [0.0, 0.5]])
    path = os.path.join(tmp, "out.csv")
    ref_write(m, ["x", "y"], path)
    out["frac_samples"] = m
    out["frac_csv"] = np.frombuffer(open(path, "rb").read(), dtype=np.uint8)
    out["frac_genes"] = np.array(["x", "y"])
    cases.append("frac")
np.savez_compressed(OUT, cases=np.array(cases), genes37=np.array(genes_for(37)),
                    meta=json.dumps({"generator": "tests/golden/make_golden_csv.py", "reference": "extras.py:31-39",
                                     "pandas": pd.__version__}), **out)
print(OUT, os.path.getsize(OUT), len(cases), "cases")
