#!/usr/bin/env python3
"""Golden vectors for count_essential_genes (utils/extras.py:49-87), produced by
the REFERENCE'S OWN FUNCTION: extras.py cannot be imported whole here (its plotting helpers import
seaborn, absent from the image), so this script parses extras.py with `ast`, takes exactly the
`count_essential_genes` FunctionDef (it only uses numpy), compiles it and runs it. No stand-in
module is written; nothing else of extras.py runs. Run here only (the reference is absent on the
GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_essential.py

Writes tests/golden/essential.npz: per case the masks, the essential-position dict flattened as
(gene offsets, positions) in dict order, G, and the reference's counts. Data only."""
import ast
import os
import sys

import numpy as np

sys.dont_write_bytecode = True
REF = "/root/reference/src/genome_minimizer_2/utils/extras.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "essential.npz")

tree = ast.parse(open(REF).read(), filename=REF)
fn = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "count_essential_genes"]
assert len(fn) == 1
mod = ast.Module(body=fn, type_ignores=[])
ns = {"np": np}
exec(compile(mod, REF, "exec"), ns)
ref_count = ns["count_essential_genes"]


def positions_dict(rng, G, n_genes):
    """gene -> positions: mostly single columns, some multi-position genes, some positions beyond G
    (the reference's `pos < G` filter), a few negative (numpy wrap-around in the reference)."""
    d = {}
    for i in range(n_genes):
        k = rng.choice([1, 1, 1, 2, 3, 5])
        pos = list(rng.integers(0, G, size=k))
        if rng.random() < 0.1:
            pos.append(int(G + rng.integers(0, 50)))
        if rng.random() < 0.05:
            pos.insert(0, int(-rng.integers(1, G)))
        d[f"gene{i}"] = [int(p) for p in pos]
    d["all_beyond"] = [G + 3, G + 7]
    return d


out = {}
rng = np.random.Generator(np.random.PCG64(2718))
cases = [("u8", 300, 517, 60, np.uint8), ("f64", 200, 1000, 120, np.float64),
         ("frac", 150, 333, 40, np.float64), ("bool", 64, 129, 25, bool)]
for name, n, G, ng, dt in cases:
    if name == "frac":  # astype(int) truncation: 0.7 counts as absent, 1.3 as present
        m = rng.choice([0.0, 0.3, 0.7, 1.0, 1.3], size=(n, G))
    else:
        m = (rng.random((n, G)) < 0.4).astype(dt)
    d = positions_dict(rng, G, ng)
    counts = np.asarray(ref_count(m.copy(), d))
    offs, pos = [0], []
    for _, p in d.items():
        pos += p
        offs.append(len(pos))
    out[f"{name}_masks"] = m
    out[f"{name}_offsets"] = np.asarray(offs, np.int64)
    out[f"{name}_positions"] = np.asarray(pos, np.int64)
    out[f"{name}_G"] = np.int64(G)
    out[f"{name}_counts"] = counts.astype(np.int64)
out["cases"] = np.array([c[0] for c in cases])
np.savez_compressed(OUT, **out)
print("wrote", OUT, {c[0]: int(out[f"{c[0]}_counts"].sum()) for c in cases})
