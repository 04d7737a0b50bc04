"""Genome minimizer host rewrite (gm2.minimizer) vs the reference's per-base algorithm
(oracle/minimizer_oracle.py, minimizer_2.py:54-103) on synthetic GenBank records, plus the GenBank
location semantics the reference inherits from Biopython (hand-written cases; Biopython itself is
not installed, so the parser is pinned by these cases only)."""
import os

import numpy as np
import pytest

from gm2 import minimizer as M
from oracle import minimizer_oracle as O


@pytest.mark.parametrize("loc,span", [
    ("190..255", (189, 255, 1)),
    ("complement(190..255)", (189, 255, -1)),
    ("<1..206", (0, 206, 1)),
    ("4500..>4641", (4499, 4641, 1)),
    ("467", (466, 467, 1)),
    ("467^468", (467, 467, 1)),
    ("join(10..20,30..40)", (9, 40, 1)),
    ("complement(join(10..20,30..40))", (9, 40, -1)),
    ("join(complement(30..40),complement(10..20))", (9, 40, -1)),
    ("order(5..8, 100..120)", (4, 120, 1)),
    ("join(4600..4641,1..50)", (0, 4641, 1)),   # origin-spanning: Biopython's min start .. max end
])
def test_parse_location(loc, span):
    assert M.parse_location(loc) == span


def write_genbank(path, seq, genes, extra_features=()):
    """genes: [(name or None, location string)]"""
    lines = [f"LOCUS       SYNTH {len(seq)} bp    DNA     circular BCT 01-JAN-2024",
             "DEFINITION  synthetic test genome.", "VERSION     SYN_000001.1",
             "FEATURES             Location/Qualifiers",
             f"     source          1..{len(seq)}", '                     /organism="Synthetic"']
    for name, loc in genes:
        if len(loc) > 50:  # wrap long locations onto continuation lines as GenBank does
            lines.append(f"     gene            {loc[:50]}")
            lines.append(f"                     {loc[50:]}")
        else:
            lines.append(f"     gene            {loc}")
        if name is not None:
            lines.append(f'                     /gene="{name}"')
        lines.append(f'                     /locus_tag="b{abs(hash(loc)) % 10000:04d}"')
        lines.append(f"     CDS             {loc[:40] if len(loc) <= 40 else loc[:40]}")
        if name is not None:
            lines.append(f'                     /gene="{name}"')
        lines.append('                     /note="a long free-text note that wraps onto a second line of the')
        lines.append('                     qualifier block"')
    lines.extend(extra_features)
    lines.append("ORIGIN")
    s = seq.lower()
    for i in range(0, len(s), 60):
        chunk = " ".join(s[j:j + 10] for j in range(i, min(i + 60, len(s)), 10))
        lines.append(f"{i + 1:>9} {chunk}")
    lines.append("//")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def synth(tmp_path, n_genes=120, L=20000, seed=0):
    rng = np.random.default_rng(seed)
    seq = "".join(rng.choice(list("ACGT"), size=L))
    genes = []
    for i in range(n_genes):
        a = int(rng.integers(1, L - 400))
        b = a + int(rng.integers(50, 400))   # overlapping intervals are common
        kind = rng.integers(0, 5)
        if kind == 0:
            loc = f"complement({a}..{b})"
        elif kind == 1:
            c = min(L, b + int(rng.integers(10, 200)))
            loc = f"join({a}..{b},{b + 5}..{c})"
        elif kind == 2:
            loc = f"<{a}..{b}"
        else:
            loc = f"{a}..{b}"
        genes.append((f"g{i}" if i % 17 else None, loc))   # some genes without a /gene name
    genes.append(("span", f"join({L - 100}..{L},1..30)"))
    p = os.path.join(tmp_path, "synth.gb")
    write_genbank(p, seq, genes)
    return p, seq, genes


def test_read_genbank(tmp_path):
    p, seq, genes = synth(tmp_path)
    rec = M.read_genbank(p)
    assert rec.seq == seq and len(rec) == len(seq)
    g = [f for f in rec.features if f.type == "gene"]
    assert len(g) == len(genes)
    for f, (name, loc) in zip(g, genes):
        assert (f.start, f.end, f.strand) == M.parse_location(loc)
        assert f.qualifiers.get("gene", [""])[0] == (name or "")
    cds = [f for f in rec.features if f.type == "CDS"]
    assert cds[0].qualifiers["note"][0].endswith("second line of the qualifier block")


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_minimizer_matches_reference_algorithm(tmp_path, seed):
    p, seq, genes = synth(tmp_path, seed=seed)
    rec = M.read_genbank(p)
    rng = np.random.default_rng(100 + seed)
    names = [n for n, _ in genes if n is not None]
    for needed in ([], names, list(rng.choice(names, size=len(names) // 2, replace=False)), ["", "g1"]):
        gm = M.GenomeMinimiser(record=rec, needed_genes_list=needed, idx=3, model_name="t")
        ref, feats, pos = O.minimize(rec, needed)
        assert gm.reduced_genome_str == ref
        assert [(f.start, f.end) for f in gm.features] == [(f.start, f.end) for f in feats]
        assert gm.positions_to_remove == pos
        st = gm.get_reduction_stats()
        assert st["positions_removed"] == len(pos) and st["reduced_length"] == len(ref)
        assert st["genes_removed"] == len(feats)


def test_batch_drivers(tmp_path, capsys):
    p, seq, genes = synth(tmp_path, n_genes=60, L=6000)
    names = [n for n, _ in genes if n is not None]
    rng = np.random.default_rng(5)
    # "span" (the origin-spanning join covers the whole genome) is kept in every list
    lists = [list(rng.choice(names, size=int(rng.integers(5, len(names))), replace=False)) + ["span"]
             for _ in range(12)]
    lists[7] = list(lists[3])  # a duplicate
    gpath = os.path.join(tmp_path, "ids.npy")
    np.save(gpath, np.array(lists, dtype=object), allow_pickle=True)
    rec = M.read_genbank(p)
    out = os.path.join(tmp_path, "one.fasta")
    r = M.process_multiple_genomes_single_file(p, gpath, "v1", output_file=out)
    text = open(out).read().split("\n")
    assert text[0] == "# Minimized genomes generated using model: v1" and text[1] == "# Total genomes: 12"
    recs = [(text[i], text[i + 1]) for i in range(3, len(text) - 1, 2)]
    assert len(recs) == 12
    printed_red, printed_len = 0.0, 0
    for idx, (hdr, body) in enumerate(recs):
        assert hdr == f">Minimized_E_coli_K12_MG1655_{idx + 1}"
        ref = O.minimize(rec, lists[idx])[0]
        assert body == ref
        if idx <= 9 or (idx + 1) % 100 == 0:  # what the reference accumulates (minimizer_2.py:468-472)
            printed_red += (len(seq) - len(ref)) / len(seq) * 100.0
            printed_len += len(ref)
    assert r["genome_count"] == 12
    assert abs(r["average_reduction_pct"] - printed_red / 12) < 1e-9
    assert abs(r["average_length_bp"] - printed_len / 12) < 1e-9
    d = os.path.join(tmp_path, "many")
    r2 = M.process_multiple_genomes_multiple_files(p, gpath, "v1", output_dir=d)
    # this driver accumulates every sample (minimizer_2.py:545-546)
    lens = [len(b) for _, b in recs]
    assert r2["genome_count"] == 12 and abs(r2["average_length_bp"] - sum(lens) / 12) < 1e-9
    assert abs(r2["average_reduction_pct"] - sum((len(seq) - n) / len(seq) * 100.0 for n in lens) / 12) < 1e-9
    assert open(os.path.join(d, "minimized_v1_0003.fasta")).read() == f">Minimized_E_coli_K12_MG1655_4\n{recs[3][1]}\n"
    dup = M.check_sequence_duplicates({h: b for h, b in recs})
    assert dup["total_sequences"] == 12 and dup["duplicate_groups"] >= 1 and dup["duplicated_sequences"] >= 2


def test_load_errors(tmp_path):
    with pytest.raises(FileNotFoundError):
        M.GenomeMinimiser(record_path=os.path.join(tmp_path, "none.gb"), needed_genes_list=[])
    bad = os.path.join(tmp_path, "x.fasta")
    open(bad, "w").write(">x\nACGT\n")
    with pytest.raises(ValueError):
        M.GenomeMinimiser(record_path=bad, needed_genes_list=[])


def test_cli_minimizer(tmp_path):
    import main as cli
    p, seq, genes = synth(tmp_path, n_genes=30, L=3000)
    names = [n for n, _ in genes if n is not None]
    gpath = os.path.join(tmp_path, "ids.npy")
    np.save(gpath, np.array([names[:10] + ["span"], names[5:] + ["span"]], dtype=object), allow_pickle=True)
    out = os.path.join(tmp_path, "o", "all.fasta")
    assert cli.main(["--mode", "minimizer", "--genome-path", p, "--genes-path", gpath, "--output-file", out,
                     "--model-name", "v1"]) == 0
    rec = M.read_genbank(p)
    body = open(out).read().split("\n")
    assert body[4] == O.minimize(rec, names[:10] + ["span"])[0]
    assert cli.main(["--mode", "minimizer", "--genome-path", p, "--genes-path", os.path.join(tmp_path, "no.npy")]) == 1


def _golden_record(g, tag):
    seq = bytes(g[f"{tag}_seq"]).decode()
    feats = []
    for t, (a, b, st), gene in zip(g[f"{tag}_ftype"], g[f"{tag}_fspan"], g[f"{tag}_fgene"]):
        q = {} if gene == "\x00" else {"gene": [str(gene)]}
        feats.append(M.Feature(str(t), int(a), int(b), int(st), q))
    return M.GenBankRecord(seq, feats)


def test_minimizer_matches_reference_goldens():
    """gm2.minimizer (interval union + slice join) and the oracle's per-base restatement against the
    outputs of the REFERENCE'S OWN methods (minimizer_2.py:50-101, run by
    tests/golden/make_golden_minimizer.py on synthetic records: overlapping / nested / duplicated
    gene spans, genes without a /gene qualifier, non-gene features, genes at both ends)."""
    from golden_io import load
    g = load("minimizer")
    for tag in g["cases"]:
        rec = _golden_record(g, tag)
        needed = [str(x) for x in g[f"{tag}_needed"]]
        ref_red = bytes(g[f"{tag}_reduced"]).decode()
        ref_pos = set(int(p) for p in g[f"{tag}_positions"])
        ref_feat = [int(i) for i in g[f"{tag}_removed_features"]]
        gm = M.GenomeMinimiser(record=rec, needed_genes_list=needed, idx=0, model_name="golden")
        assert gm.reduced_genome_str == ref_red, tag
        assert [rec.features.index(f) for f in gm.features] == ref_feat, tag
        assert gm.positions_to_remove == ref_pos, tag
        o_red, o_feats, o_pos = O.minimize(rec, needed)
        assert o_red == ref_red and o_pos == ref_pos and [rec.features.index(f) for f in o_feats] == ref_feat, tag
