#!/usr/bin/env python3
"""Golden vectors for the genome minimizer, produced by the REFERENCE'S OWN
METHODS: minimizer_2.py imports Biopython (absent from this image), so this script parses it with
`ast`, takes exactly the three methods of GenomeMinimiser that do the work --
`_extract_non_essential_genes`, `_get_positions_to_remove`, `_create_minimized_sequence`
(minimizer_2.py:50-101) -- compiles them into a bare class and runs them on synthetic records. Those
methods read only `record.features` (feature.type, feature.qualifiers, feature.location.start/end),
`record.seq` and `needed_genes`; the records are the build's own gm2.minimizer.GenBankRecord /
Feature objects (the attribute surface of Biopython's SeqRecord / SeqFeature those lines use). No
stand-in module is written; nothing else of minimizer_2.py runs. Run here only (the reference is
absent on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_minimizer.py

Writes tests/golden/minimizer.npz: per case the record (sequence bytes, feature type / start / end /
gene name), the needed-gene list, and the reference's outputs (indices of the removed features in
record.features, the sorted removed positions, the minimized sequence bytes). Data only."""
import ast
import json
import logging
import os
import sys

import numpy as np

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "genome-minimizer-2_amd"))
from gm2.minimizer import Feature, GenBankRecord  # noqa: E402

REF = "/root/reference/src/genome_minimizer_2/minimizer/minimizer_2.py"
OUT = os.path.join(HERE, "minimizer.npz")
METHODS = ("_extract_non_essential_genes", "_get_positions_to_remove", "_create_minimized_sequence")

tree = ast.parse(open(REF).read(), filename=REF)
cls = [n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "GenomeMinimiser"]
assert len(cls) == 1
fns = [n for n in cls[0].body if isinstance(n, ast.FunctionDef) and n.name in METHODS]
assert sorted(f.name for f in fns) == sorted(METHODS)
body = ast.ClassDef(name="RefMinimiser", bases=[], keywords=[], body=fns, decorator_list=[])
mod = ast.fix_missing_locations(ast.Module(body=[body], type_ignores=[]))
ns = {"logging": logging}
exec(compile(mod, REF, "exec"), ns)
RefMinimiser = ns["RefMinimiser"]


def synth_record(rng, L, n_genes):
    """Random genome with overlapping / nested / duplicated gene spans, genes without a /gene
    qualifier, non-gene features (CDS, source, misc) spanning genes, and a gene at each end."""
    seq = "".join(rng.choice(list("ACGT"), size=L))
    feats = [Feature("source", 0, L, 1, {"organism": ["Synthetic"]})]
    for i in range(n_genes):
        a = int(rng.integers(0, L - 50))
        b = min(L, a + int(rng.integers(1, 600)))
        q = {} if i % 13 == 0 else {"gene": [f"g{i % (n_genes - 7)}"], "locus_tag": [f"b{i:04d}"]}
        feats.append(Feature("gene", a, b, 1 if i % 3 else -1, q))
        if i % 4 == 0:
            feats.append(Feature("CDS", a, b, 1, dict(q)))
    feats.append(Feature("gene", 0, 17, 1, {"gene": ["first"]}))
    feats.append(Feature("gene", L - 9, L, -1, {"gene": ["last"]}))
    feats.append(Feature("misc_feature", 10, L - 10, 1, {"note": ["spans everything"]}))
    return GenBankRecord(seq, feats, id="SYN", name="SYN")


def run_reference(rec, needed):
    m = RefMinimiser.__new__(RefMinimiser)
    m.record, m.needed_genes, m.idx = rec, needed, 0
    m.features = m._extract_non_essential_genes()
    m.positions_to_remove = m._get_positions_to_remove()
    return m.features, m.positions_to_remove, m._create_minimized_sequence()


out = {}
cases = []
rng = np.random.Generator(np.random.PCG64(31415))
for ci, (L, n_genes) in enumerate([(5000, 40), (20000, 150), (1200, 60)]):
    rec = synth_record(rng, L, n_genes)
    names = sorted({f.qualifiers["gene"][0] for f in rec.features if f.type == "gene" and "gene" in f.qualifiers})
    needed_sets = [[], names, list(rng.choice(names, size=len(names) // 2, replace=False)), ["", "first", "zzz"]]
    for ni, needed in enumerate(needed_sets):
        tag = f"c{ci}n{ni}"
        feats, pos, red = run_reference(rec, [str(x) for x in needed])
        idx = [rec.features.index(f) for f in feats]
        out[f"{tag}_seq"] = np.frombuffer(rec.seq.encode(), dtype=np.uint8)
        out[f"{tag}_ftype"] = np.array([f.type for f in rec.features])
        out[f"{tag}_fspan"] = np.array([[f.start, f.end, f.strand] for f in rec.features], dtype=np.int64)
        out[f"{tag}_fgene"] = np.array([f.qualifiers["gene"][0] if "gene" in f.qualifiers else "\x00"
                                        for f in rec.features])
        out[f"{tag}_needed"] = np.array([str(x) for x in needed] + ["\x00"])[:-1] if needed else np.array([], dtype="<U1")
        out[f"{tag}_removed_features"] = np.array(idx, dtype=np.int64)
        out[f"{tag}_positions"] = np.array(sorted(pos), dtype=np.int64)
        out[f"{tag}_reduced"] = np.frombuffer(red.encode(), dtype=np.uint8)
        cases.append(tag)
np.savez_compressed(OUT, cases=np.array(cases), meta=json.dumps({"generator": "tests/golden/make_golden_minimizer.py",
                                                                   "reference": "minimizer_2.py:50-101"}), **out)
print(OUT, os.path.getsize(OUT), len(cases), "cases")
