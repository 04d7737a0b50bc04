"""TEST INFRASTRUCTURE ONLY (imported by tests/, never by the product path).

Restatement of the reference genome minimizer's per-sample algorithm, literally as written in
/root/reference/src/genome_minimizer_2/minimizer/minimizer_2.py:
  _extract_non_essential_genes (:54-70): gene features whose first /gene value is not needed;
  _get_positions_to_remove   (:72-86): the set of every position in range(start, end) of them;
  _create_minimized_sequence (:88-103): the bases whose index is not in that set, in order.
It works on any record exposing .seq and .features with .type / .qualifiers / .location.start/.end
(gm2.minimizer.read_genbank's records). Parity status: PINNED -- both this restatement and
gm2.minimizer are checked against tests/golden/minimizer.npz, the outputs of the reference's own
three methods run on synthetic records (tests/golden/make_golden_minimizer.py). Biopython (the
reference's GenBank reader) is absent here, so the GenBank PARSING is pinned only by hand-written
location cases in tests/test_minimizer_cpu.py ("parity unpinned" against Biopython's own parser).
"""


def minimize(record, needed):
    feats = [f for f in record.features
             if f.type == "gene" and f.qualifiers.get("gene", [""])[0] not in needed]
    positions = set()
    for f in feats:
        positions.update(range(int(f.location.start), int(f.location.end)))
    out = []
    for i, base in enumerate(record.seq):
        if i not in positions:
            out.append(base)
    return "".join(out), feats, positions
