"""Genome minimizer: the consumer of the per-sample gene lists that
`convert-samples` writes. Mirror of minimizer/minimizer_2.py: GenomeMinimiser (:19-254),
check_sequence_duplicates (:257-287), generate_summary_file (:326-424) and the two batch drivers
process_multiple_genomes_single_file / _multiple_files (:427-560), with the same file names, FASTA
headers, statistics and printed lines.

What changes is the algorithm, not the result. The reference builds, per sample, a Python set of
every removed base position and then walks the whole genome base by base testing membership
(minimizer_2.py:67-101): O(genome length) Python work per sample. Here the removed regions are the
union of the non-essential gene intervals, merged once per sample with numpy (sort + running max),
and the minimized sequence is the concatenation of the kept slices of the sequence string: O(genes)
numpy work plus one string join. The gene-name test is one vectorised `isin` over the record's gene
features, shared by every sample.

GenBank input: Biopython (the reference's `SeqIO.read(path, "genbank")`) is not a dependency here;
`read_genbank` parses the subset the minimizer uses -- the sequence (ORIGIN, upper-cased as
Biopython returns it) and each feature's key, `/qualifier` values and location, with Biopython's
start / end semantics (0-based start, exclusive end; a join/order spans min start .. max end;
fuzzy `<` / `>` ends taken at their position; `a^b` between-positions are empty).
"""
from __future__ import annotations

import logging
import os
import re
from collections import defaultdict

import numpy as np

logger = logging.getLogger(__name__)

PROJECT_ROOT = os.environ.get("GM2_PROJECT_ROOT", os.getcwd())

__all__ = ["Feature", "GenBankRecord", "read_genbank", "parse_location", "GenomeMinimiser",
           "check_sequence_duplicates", "print_duplicate_statistics", "generate_summary_file",
           "process_multiple_genomes_single_file", "process_multiple_genomes_multiple_files"]


# --------------------------------------------------------------------------------------------------
# GenBank subset reader
# --------------------------------------------------------------------------------------------------
class Feature:
    """A feature table entry: `type`, `qualifiers` (name -> list of values, as Biopython) and the
    location span `start` (0-based) / `end` (exclusive)."""
    __slots__ = ("type", "start", "end", "strand", "qualifiers")

    def __init__(self, type_, start, end, strand, qualifiers):
        self.type, self.start, self.end, self.strand, self.qualifiers = type_, start, end, strand, qualifiers

    @property
    def location(self):  # feature.location.start / .end as the reference reads them
        return self

    def __repr__(self):
        return f"Feature({self.type!r}, {self.start}..{self.end}, {self.qualifiers.get('gene', [''])[0]!r})"


class GenBankRecord:
    """The parts of a Biopython SeqRecord the minimizer reads: `seq` (str), `features`, `id`."""

    def __init__(self, seq: str, features: list, id: str = "", name: str = ""):
        self.seq, self.features, self.id, self.name = seq, features, id, name

    def __len__(self):
        return len(self.seq)


_SPAN = re.compile(r"^<?(\d+)\.\.>?(\d+)$")


def parse_location(text: str):
    """(start, end, strand) of a GenBank location string, Biopython's span semantics."""
    t = text.replace(" ", "")
    strand = 1
    if t.startswith("complement(") and t.endswith(")"):
        s, e, st = parse_location(t[len("complement("):-1])
        return s, e, -st
    for op in ("join(", "order("):
        if t.startswith(op) and t.endswith(")"):
            parts, depth, cur = [], 0, ""
            for ch in t[len(op):-1]:
                if ch == "," and depth == 0:
                    parts.append(cur)
                    cur = ""
                    continue
                depth += ch == "("
                depth -= ch == ")"
                cur += ch
            parts.append(cur)
            spans = [parse_location(p) for p in parts if p]
            strands = {sp[2] for sp in spans}
            return min(sp[0] for sp in spans), max(sp[1] for sp in spans), strands.pop() if len(strands) == 1 else 0
    if ":" in t:
        raise ValueError(f"remote location not supported: {text}")
    m = _SPAN.match(t)
    if m:
        return int(m.group(1)) - 1, int(m.group(2)), strand
    if "^" in t:  # between two bases: an empty span after the first
        a = int(t.split("^")[0].lstrip("<>"))
        return a, a, strand
    m = re.match(r"^[<>]?(\d+)$", t)
    if m:
        p = int(m.group(1))
        return p - 1, p, strand
    raise ValueError(f"unsupported GenBank location: {text}")


def _parse_qualifier_value(v: str):
    v = v.strip()
    if len(v) >= 2 and v[0] == '"' and v[-1] == '"':
        return v[1:-1].replace('""', '"')
    return v


def read_genbank(path: str) -> GenBankRecord:
    """One-record GenBank file -> GenBankRecord (see module docstring)."""
    features, seq_chunks = [], []
    rec_id = name = ""
    state = "header"
    key = loc = None
    quals: dict = {}
    qname = qval = None

    def flush_qual():
        nonlocal qname, qval
        if qname is not None:
            quals.setdefault(qname, []).append(_parse_qualifier_value(qval) if qval is not None else "")
        qname = qval = None

    def flush_feature():
        nonlocal key, loc, quals
        flush_qual()
        if key is not None:
            s, e, st = parse_location(loc)
            features.append(Feature(key, s, e, st, quals))
        key, loc, quals = None, None, {}

    with open(path) as fh:
        for line in fh:
            line = line.rstrip("\n\r")
            if state == "header":
                if line.startswith("LOCUS"):
                    f = line.split()
                    name = f[1] if len(f) > 1 else ""
                elif line.startswith("VERSION"):
                    f = line.split()
                    rec_id = f[1] if len(f) > 1 else name
                elif line.startswith("FEATURES"):
                    state = "features"
                elif line.startswith("ORIGIN"):
                    state = "origin"
                continue
            if state == "features":
                if line.startswith("ORIGIN") or line.startswith("CONTIG") or line.startswith("BASE COUNT"):
                    flush_feature()
                    state = "origin" if line.startswith("ORIGIN") else "tail"
                    continue
                if len(line) > 5 and line[5] != " " and line.startswith("     "):  # new feature key
                    flush_feature()
                    key = line[5:21].strip()
                    loc = line[21:].strip()
                    continue
                body = line[21:] if len(line) > 21 else ""
                if body.startswith("/"):
                    flush_qual()
                    q = body[1:]
                    if "=" in q:
                        qname, qval = q.split("=", 1)
                    else:
                        qname, qval = q, None
                elif qname is not None and qval is not None:
                    # continuation of a quoted value (free text keeps a space, sequences do not)
                    sep = "" if qname == "translation" else " "
                    qval = qval + sep + body.strip()
                elif key is not None and qname is None:
                    loc += body.strip()
                continue
            if state == "tail":
                if line.startswith("ORIGIN"):
                    state = "origin"
                continue
            if state == "origin":
                if line.startswith("//"):
                    break
                seq_chunks.append("".join(line.split()[1:]))
    if state == "features":
        flush_feature()
    return GenBankRecord("".join(seq_chunks).upper(), features, rec_id or name, name)


# --------------------------------------------------------------------------------------------------
# interval helpers
# --------------------------------------------------------------------------------------------------
def _merged(starts: np.ndarray, ends: np.ndarray):
    """Union of [start, end) intervals -> disjoint sorted (starts, ends); empty intervals dropped."""
    keep = ends > starts
    s, e = starts[keep], ends[keep]
    if s.size == 0:
        return s, e
    o = np.argsort(s, kind="stable")
    s, e = s[o], e[o]
    run_end = np.maximum.accumulate(e)
    new = np.ones(s.size, dtype=bool)
    new[1:] = s[1:] > run_end[:-1]
    grp = np.cumsum(new) - 1
    ms = s[new]
    me = np.zeros(ms.size, dtype=e.dtype)
    np.maximum.at(me, grp, e)
    return ms, me


class _GeneTable:
    """The record's gene features as arrays (shared by every sample of a batch run)."""

    def __init__(self, record):
        genes = [f for f in record.features if f.type == "gene"]
        self.features = genes
        self.names = np.array([f.qualifiers.get("gene", [""])[0] for f in genes], dtype=object)
        self.starts = np.array([int(f.location.start) for f in genes], dtype=np.int64)
        self.ends = np.array([int(f.location.end) for f in genes], dtype=np.int64)

    def removed(self, needed):
        """mask of the gene features whose name is not in `needed` (minimizer_2.py:54-65)."""
        need = set(needed.tolist() if isinstance(needed, np.ndarray) else needed)
        return np.fromiter((n not in need for n in self.names), dtype=bool, count=self.names.size)


class GenomeMinimiser:
    """Same constructor, attributes and methods as the reference (minimizer_2.py:19-254)."""

    def __init__(self, record_path: str = None, needed_genes_path: str = None, idx: int = 0, model_name: str = "",
                 record=None, all_needed_gene_lists: list = None, needed_genes_list: list = None,
                 _table: _GeneTable = None):
        self.idx = idx
        self.model_name = model_name
        self.record = record if record is not None else self.load_genome(record_path)
        self.wildtype_sequence = self.record
        self.original_genome_length = len(self.record.seq)
        if needed_genes_list is not None:
            self.needed_genes = needed_genes_list
        elif all_needed_gene_lists is not None:
            self.needed_genes = all_needed_gene_lists[idx]
        else:
            self.needed_genes = self.get_needed_genes(needed_genes_path)[idx]
        table = _table if _table is not None else _GeneTable(self.record)
        rm = table.removed(self.needed_genes)
        self.features = [f for f, r in zip(table.features, rm) if r]
        self._rs, self._re = _merged(table.starts[rm], table.ends[rm])
        self.reduced_genome_str = self._create_minimized_sequence()

    # reference method names ------------------------------------------------------------------
    def _extract_non_essential_genes(self) -> list:
        return list(self.features)

    @property
    def positions_to_remove(self) -> set:
        """The reference's set of removed positions (built on demand; the minimizer itself works
        on the merged intervals)."""
        out = set()
        for s, e in zip(self._rs.tolist(), self._re.tolist()):
            out.update(range(s, e))
        return out

    def _get_positions_to_remove(self) -> set:
        return self.positions_to_remove

    @property
    def positions_removed_count(self) -> int:
        return int((self._re - self._rs).sum())

    def _create_minimized_sequence(self) -> str:
        seq = str(self.record.seq)
        L = len(seq)
        rs = np.clip(self._rs, 0, L).tolist()
        re_ = np.clip(self._re, 0, L).tolist()
        pieces, cur = [], 0
        for s, e in zip(rs, re_):
            if s > cur:
                pieces.append(seq[cur:s])
            cur = max(cur, e)
        if cur < L:
            pieces.append(seq[cur:])
        return "".join(pieces)

    def save_minimized_genome(self, file_path: str):
        try:
            os.makedirs(os.path.join(PROJECT_ROOT, "minimized_genomes"), exist_ok=True)
            with open(file_path, "w") as output_file:
                output_file.write(f">Minimized_E_coli_K12_MG1655_{self.idx + 1}\n")
                output_file.write(str(self.reduced_genome_str))
                logger.info(f"Successfully saved reduced genome: {file_path}")
        except IOError as e:
            logger.error(f"\n✗ Could not write to file: {file_path} - {e}")
            raise

    def load_genome(self, file_path: str):
        if file_path is None or not os.path.isfile(file_path):
            raise FileNotFoundError(f"The file {file_path} does not exist.")
        if not file_path.endswith((".gb", ".genbank", ".gbff")):
            raise ValueError(f"The file {file_path} could not be read.\nEnsure the file holds a GenBank format.")
        rec = read_genbank(file_path)
        logger.info(f"✓ Successfully loaded genome from {file_path}")
        return rec

    def get_needed_genes(self, file_path: str) -> list:
        if file_path is None or not os.path.isfile(file_path):
            raise FileNotFoundError(f"The file {file_path} does not exist.")
        if not file_path.endswith(".npy"):
            raise ValueError(f"Invalid file format. Expected .npy file, got: {os.path.splitext(file_path)[1]}")
        # object arrays of gene-name lists (written by convert-samples) need the pickle loader, as in
        # the reference (minimizer_2.py:184)
        return np.load(file_path, allow_pickle=True).tolist()

    def get_reduction_stats(self) -> dict:
        reduced_length = len(self.reduced_genome_str)
        return {"original_length": self.original_genome_length, "reduced_length": reduced_length,
                "reduction_percentage": (self.original_genome_length - reduced_length) / self.original_genome_length
                * 100, "genes_removed": len(self.features), "positions_removed": self.positions_removed_count}


def check_sequence_duplicates(sequences_dict: dict) -> dict:
    """minimizer_2.py:257-287."""
    groups = defaultdict(list)
    for seq_id, sequence in sequences_dict.items():
        groups[sequence].append(seq_id)
    duplicates = {s: ids for s, ids in groups.items() if len(ids) > 1}
    unique = {s: ids for s, ids in groups.items() if len(ids) == 1}
    return {"total_sequences": len(sequences_dict), "unique_sequences": len(groups),
            "duplicate_groups": len(duplicates), "duplicated_sequences": sum(len(i) for i in duplicates.values()),
            "unique_only_sequences": len(unique), "duplicates_detail": duplicates,
            "compression_ratio": len(groups) / len(sequences_dict) if sequences_dict else 0}


def print_duplicate_statistics(d: dict):
    """minimizer_2.py:290-323."""
    print("\n" + "=" * 80)
    print("SEQUENCE DUPLICATION ANALYSIS")
    print("=" * 80)
    print(" Overview:")
    print(f"- Total sequences generated: {d['total_sequences']:,}")
    print(f"- Unique sequences: {d['unique_sequences']:,}")
    print(f"- Duplicate groups: {d['duplicate_groups']:,}")
    print(f"- Sequences with duplicates: {d['duplicated_sequences']:,}")
    print(f"- Truly unique sequences: {d['unique_only_sequences']:,}")
    print(f"- Percentage of unique sequences: {d['compression_ratio']:.2%}")
    if d["duplicate_groups"] > 0:
        print("\n Duplicate Details:")
        dups = sorted(d["duplicates_detail"].items(), key=lambda x: len(x[1]), reverse=True)
        for i, (sequence, ids) in enumerate(dups[:10]):
            print(f"Group {i + 1}: {len(ids)} identical sequences")
            print(f"- Sequence: {sequence[:50]}{'...' if len(sequence) > 50 else ''}")
            print(f"- IDs: {', '.join(ids[:5])}{'...' if len(ids) > 5 else ''}")
            print()
        if len(dups) > 10:
            print(f"  ... and {len(dups) - 10} more duplicate groups")
    else:
        print("\n✓ No duplicate sequences found!")
    print("=" * 80)


def generate_summary_file(output_file: str, model_name: str, genome_path: str, genes_path: str,
                          original_length: int, minimised_sizes: list, duplicate_stats: dict):
    """minimizer_2.py:326-424 (same report layout)."""
    try:
        out_dir = os.path.join(PROJECT_ROOT, "minimized_genomes")
        os.makedirs(out_dir, exist_ok=True)
        summary_file = os.path.join(out_dir, os.path.basename(output_file).replace(".fasta", "_summary.txt"))
        n = len(minimised_sizes)
        mean = np.mean(minimised_sizes) if minimised_sizes else 0
        med = np.median(minimised_sizes) if minimised_sizes else 0
        mn = np.min(minimised_sizes) if minimised_sizes else 0
        mx = np.max(minimised_sizes) if minimised_sizes else 0
        sd = np.std(minimised_sizes) if minimised_sizes else 0
        with open(summary_file, "w") as f:
            f.write("=" * 80 + "\n" + "GENOME MINIMIZATION SUMMARY REPORT\n" + "=" * 80 + "\n\n")
            f.write("GENERATION INFORMATION\n" + "-" * 40 + "\n")
            f.write(f"Model Name: {model_name}\n")
            f.write(f"Generated on: {np.datetime64('now')}\n")
            f.write(f"Output FASTA file: {os.path.basename(output_file)}\n")
            f.write(f"Summary file: {os.path.basename(summary_file)}\n\n")
            f.write("INPUT FILES\n" + "-" * 40 + "\n")
            f.write(f"Genome template: {os.path.basename(genome_path)}\n")
            f.write(f"Gene lists file: {os.path.basename(genes_path)}\n")
            f.write(f"Original genome length: {original_length:,} bp\n\n")
            f.write("PROCESSING STATISTICS\n" + "-" * 40 + "\n")
            f.write(f"Successfully processed: {n:,}\n\n")
            f.write("MINIMIZED GENOME SIZE STATISTICS\n" + "-" * 40 + "\n")
            f.write(f"Mean size: {mean:.3f} Mbp ({mean * 1e6:,.0f} bp)\n")
            f.write(f"Median size: {med:.3f} Mbp ({med * 1e6:,.0f} bp)\n")
            f.write(f"Minimum size: {mn:.3f} Mbp ({mn * 1e6:,.0f} bp)\n")
            f.write(f"Maximum size: {mx:.3f} Mbp ({mx * 1e6:,.0f} bp)\n")
            f.write(f"Standard deviation: {sd:.3f} Mbp\n")
            f.write(f"Size range: {mx - mn:.3f} Mbp\n\n")
            if original_length > 0:
                f.write("GENOME REDUCTION STATISTICS\n" + "-" * 40 + "\n")
                f.write(f"Mean reduction: {(original_length - mean * 1e6) / original_length * 100:.2f}%\n")
                f.write(f"Minimum reduction: {(original_length - mx * 1e6) / original_length * 100:.2f}% "
                        "(largest genome)\n")
                f.write(f"Maximum reduction: {(original_length - mn * 1e6) / original_length * 100:.2f}% "
                        "(smallest genome)\n\n")
            f.write("SEQUENCE DUPLICATION ANALYSIS\n" + "-" * 40 + "\n")
            f.write(f"Total sequences: {duplicate_stats['total_sequences']:,}\n")
            f.write(f"Unique sequences: {duplicate_stats['unique_sequences']:,}\n")
            f.write(f"Duplicate groups: {duplicate_stats['duplicate_groups']:,}\n")
            f.write(f"Sequences with duplicates: {duplicate_stats['duplicated_sequences']:,}\n")
            f.write(f"Uniqueness ratio: {duplicate_stats['compression_ratio']:.2%}\n")
            if minimised_sizes:
                f.write("\nSIZE DISTRIBUTION SUMMARY\n" + "-" * 40 + "\n")
                bins = np.linspace(mn, mx, 6)
                hist, _ = np.histogram(minimised_sizes, bins=bins)
                for i in range(len(hist)):
                    f.write(f"{bins[i]:.2f} - {bins[i + 1]:.2f} Mbp: {hist[i]:,} genomes "
                            f"({hist[i] / len(minimised_sizes) * 100:.1f}%)\n")
        logger.info(f"✓ Summary file saved: {summary_file}")
    except Exception as e:  # the reference logs and carries on
        logger.error(f"✗ Failed to generate summary file: {e}")


def _load_batch(genome_path, genes_path):
    record = read_genbank(genome_path)
    return record, np.load(genes_path, allow_pickle=True).tolist(), _GeneTable(record)


def process_multiple_genomes_single_file(genome_path: str, genes_path: str, model_name: str, output_file: str = None):
    """All minimized genomes into one FASTA file (minimizer_2.py:427-478): same header lines, record
    ids, progress lines and returned averages (the reference averages the reductions it printed --
    samples 1-10 and every 100th -- over all samples; kept as is)."""
    if not output_file:
        output_file = os.path.join(PROJECT_ROOT, "minimized_genomes", f"minimized_genomes_{model_name}.fasta")
    os.makedirs(os.path.dirname(output_file) or ".", exist_ok=True)
    record, all_lists, table = _load_batch(genome_path, genes_path)
    original_length = len(record.seq)
    tot_red_pct, total_length_bp, n = 0.0, 0, len(all_lists)
    with open(output_file, "w") as out:
        out.write(f"# Minimized genomes generated using model: {model_name}\n")
        out.write(f"# Total genomes: {n}\n")
        out.write(f"# Generated on: {np.datetime64('now')}\n")
        for idx, needed in enumerate(all_lists):
            print(f"[{idx + 1}/{n}] genes present: {len(needed)}")
            gm = GenomeMinimiser(record=record, needed_genes_list=needed, idx=idx, model_name=model_name, _table=table)
            out.write(f">Minimized_E_coli_K12_MG1655_{idx + 1}\n{gm.reduced_genome_str}\n")
            length = len(gm.reduced_genome_str)
            if idx <= 9 or (idx + 1) % 100 == 0:
                red = (original_length - length) / original_length * 100.0
                print(f"  → {length:,} bp ({red:.1f}% reduction)")
                tot_red_pct += red
                total_length_bp += length
    return {"genome_count": n, "average_reduction_pct": tot_red_pct / n, "average_length_bp": total_length_bp / n}


def process_multiple_genomes_multiple_files(genome_path: str, genes_path: str, model_name: str, output_dir: str = None,
                                            filename_template: str = "minimized_{model}_{idx:04d}.fasta"):
    """One FASTA file per minimized genome (minimizer_2.py:482-560)."""
    if output_dir is None:
        output_dir = os.path.join(PROJECT_ROOT, "minimized_genomes")
    os.makedirs(output_dir, exist_ok=True)
    record, all_lists, table = _load_batch(genome_path, genes_path)
    original_length = len(record.seq)
    n = len(all_lists)
    tot_red_pct, total_length = 0.0, 0
    print(f"Writing {n} individual FASTA files to: {output_dir}")
    for idx, needed in enumerate(all_lists):
        print(f"[{idx + 1}/{n}] genes present: {len(needed)}")
        gm = GenomeMinimiser(record=record, needed_genes_list=needed, idx=idx, model_name=model_name, _table=table)
        genome_str = gm.reduced_genome_str
        length = len(genome_str)
        red = (original_length - length) / original_length * 100.0
        out_path = os.path.join(output_dir, filename_template.format(model=model_name, idx=idx))
        with open(out_path, "w") as fh:
            fh.write(f">Minimized_E_coli_K12_MG1655_{idx + 1}\n{genome_str}\n")
        tot_red_pct += red
        total_length += length
        if idx <= 9 or (idx + 1) % 100 == 0:
            print(f"  → saved {os.path.basename(out_path)} | {length:,} bp ({red:.1f}% reduction)")
    return {"genome_count": n, "average_reduction_pct": tot_red_pct / n, "average_length_bp": total_length / n}
