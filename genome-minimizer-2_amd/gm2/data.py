"""Data side of the hot path: the presence/absence matrix resident in HBM, and a DataLoader mirror
that yields strain-row index batches with the reference's RNG consumption.

Reference: data ingest `load_and_validate_data` (explore_data/data_exploration.py:54-107), the split
+ loaders of `create_dataloaders` (utils/experiments.py:225-252), DataLoader/RandomSampler semantics
of torch (one int64 base-seed draw per iterator, one seed draw + randperm per shuffled epoch).
"""
from __future__ import annotations

import math
import os
import re

import numpy as np
import torch


def _pad_cols(G):
    return int(math.ceil(G / 128) * 128)


class ResidentMatrix:
    """0/1 matrix [n, G] stored once in HBM as u8 rows of ld = roundup(G, 128) bytes (zero pad).
    1 byte per gene: the F4 matrix (10k x 55k) is 0.55 GB; batches are gathered by row index."""

    def __init__(self, x, device=None):
        if isinstance(x, ResidentMatrix):
            self.__dict__.update(x.__dict__)
            return
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        t = torch.as_tensor(np.asarray(x) if not torch.is_tensor(x) else x)
        if t.dim() != 2:
            raise ValueError("presence/absence matrix must be 2-D [strains, genes]")
        self.n, self.G = int(t.shape[0]), int(t.shape[1])
        self.ld = _pad_cols(self.G)
        if t.dtype != torch.uint8:
            tf = t.to(torch.float32)
            bad = ((tf != 0) & (tf != 1)).any().item() if tf.numel() else False
            if bad:
                raise ValueError("the fused BCE path needs a binary 0/1 matrix (reference data is 0/1)")
            t = tf.to(torch.uint8)
        buf = torch.zeros(max(self.n, 1), self.ld, dtype=torch.uint8)
        buf[: self.n, : self.G] = t.cpu()
        self.data = buf.to(device)

    def operands(self, prec):
        """The matrix as GEMM operands for `prec` (native.ResidentOperands), built on first use and
        kept: training steps then read their rows in place instead of gathering them."""
        from . import native
        cache = self.__dict__.setdefault("_operands", {})
        if prec not in cache:
            cache[prec] = native.ResidentOperands(self.data, self.ld, self.n, self.G, prec)
        return cache[prec]

    def __len__(self):
        return self.n


class _Subset:
    """`len(loader.dataset)` for the epoch averages (trainer.py:127, :152)."""

    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n


class StrainLoader:
    """DataLoader(TensorDataset(X[idx]), batch_size, shuffle) mirror: iterates device int32 row
    indices into a ResidentMatrix. RNG use is the torch DataLoader's: each iterator draws an int64
    base seed from the global CPU generator; a shuffled one then draws its sampler seed and runs
    randperm on a private generator (so the global stream advances exactly as in the reference)."""

    def __init__(self, matrix: ResidentMatrix, rows=None, batch_size=32, shuffle=False, drop_last=False):
        self.matrix = matrix
        rows = np.arange(matrix.n) if rows is None else np.asarray(rows)
        self.rows_host = torch.as_tensor(rows, dtype=torch.int64)
        self.rows = self.rows_host.to(torch.int32).to(matrix.data.device)
        self.batch_size = int(batch_size)
        self.shuffle = bool(shuffle)
        self.drop_last = bool(drop_last)
        self.dataset = _Subset(len(rows))

    def __len__(self):
        n = len(self.dataset)
        return n // self.batch_size if self.drop_last else (n + self.batch_size - 1) // self.batch_size

    def __iter__(self):
        n = len(self.dataset)
        torch.empty((), dtype=torch.int64).random_()  # _BaseDataLoaderIter._base_seed
        if self.shuffle:
            seed = int(torch.empty((), dtype=torch.int64).random_().item())
            g = torch.Generator()
            g.manual_seed(seed)
            perm = torch.randperm(n, generator=g).to(torch.int32).to(self.rows.device)
            order = self.rows[perm.long()]
        else:
            order = self.rows
        for s in range(0, n, self.batch_size):
            e = min(n, s + self.batch_size)
            if self.drop_last and e - s < self.batch_size:
                break
            yield order[s:e]


def as_strain_loader(loader, device=None):
    """Accept a reference-style torch DataLoader(TensorDataset(X), batch_size, shuffle) too."""
    if isinstance(loader, StrainLoader):
        return loader
    ds = loader.dataset
    x = ds.tensors[0] if hasattr(ds, "tensors") else torch.stack([ds[i][0] for i in range(len(ds))])
    from torch.utils.data import RandomSampler
    shuffle = isinstance(loader.sampler, RandomSampler)
    return StrainLoader(ResidentMatrix(x, device=device), None, loader.batch_size, shuffle, loader.drop_last)


def split_indices(n, test_size=0.3, val_ratio=0.3333, random_state=12345):
    """create_dataloaders' two train_test_split calls (experiments.py:232-237) on row indices."""
    from sklearn.model_selection import train_test_split
    idx = np.arange(n)
    tr, tmp = train_test_split(idx, test_size=test_size, random_state=random_state)
    va, te = train_test_split(tmp, test_size=val_ratio, random_state=random_state)
    return tr, va, te


_INT_CELL = re.compile(rb"-?[0-9]+\Z")


def read_matrix_csv(path):
    """pd.read_csv(path, index_col=0, header=0) for the pan-genome table's own form, parsed with
    numpy over the file's bytes (pandas' tokenizer takes ~10 s at F4 width, 55,039 x 7,512): a
    header row of distinct non-empty strain IDs after an empty first cell, then one row per gene
    (and the 'Lineage' row) of plain integer cells -- the gene rows' single-digit 0 / 1 cells taken
    by one vectorised check per row. Any other form (quotes, CR line ends, blanks or NA markers,
    numeric-looking gene names, other cell text) returns pandas' own parse of the file, so the
    result is always what pandas gives (int64 cells, object index and columns)."""
    import pandas as pd

    def fallback():
        return pd.read_csv(path, index_col=0, header=0)

    with open(path, "rb") as f:
        raw = f.read()
    if b'"' in raw or b"\r" in raw:
        return fallback()
    lines = raw.split(b"\n")
    if lines and lines[-1] == b"":
        lines.pop()
    head = lines[0].split(b",") if lines else []
    cols = [h.decode() for h in head[1:]]
    n = len(cols)
    if len(lines) < 2 or head[0] != b"" or n == 0 or "" in cols or len(set(cols)) != n:
        return fallback()
    names, vals = [], np.empty((len(lines) - 1, n), dtype=np.int64)
    for i, ln in enumerate(lines[1:]):
        k = ln.find(b",")
        name = ln[:k]
        if k <= 0 or _INT_CELL.match(name) or name.strip() != name or name.upper() in _NA_NAMES:
            return fallback()
        names.append(name.decode())
        body = np.frombuffer(ln, dtype=np.uint8)[k + 1:]
        if body.size == 2 * n - 1 and (body[1::2] == 44).all():
            d = body[0::2] - 48  # (uint8: any byte below '0' wraps above 1)
            if (d <= 1).all():
                vals[i] = d
                continue
        parts = ln[k + 1:].split(b",")
        if len(parts) != n or not all(_INT_CELL.match(c) for c in parts):
            return fallback()
        vals[i] = [int(c) for c in parts]
    return pd.DataFrame(vals, index=pd.Index(names, dtype=object), columns=pd.Index(cols, dtype=object))


# pandas' default NA markers (read_csv na_values), upper-cased: an index cell equal to one is NaN there
_NA_NAMES = {b"", b"#N/A", b"#N/A N/A", b"#NA", b"-1.#IND", b"-1.#QNAN", b"-NAN", b"1.#IND", b"1.#QNAN",
             b"<NA>", b"N/A", b"NA", b"NULL", b"NAN", b"NONE"}


def load_and_validate_data(dataset_csv, phylogroups_csv):
    """(large_data, merged_df, data_without_lineage) as data_exploration.py:54-107: genes x strains
    CSV (index_col=0), strain IDs upper-cased, 'Lineage' row dropped, transposed and inner-merged
    with the phylogroup table on ID."""
    import pandas as pd
    large = read_matrix_csv(dataset_csv)
    large.columns = large.columns.str.upper()
    phylo = pd.read_csv(phylogroups_csv, index_col=0, header=0)
    without = large.drop(index=["Lineage"], errors="ignore")
    merged = pd.merge(without.transpose(), phylo, how="inner", left_index=True, right_on="ID")
    if merged.empty:
        raise ValueError("Merged dataset is empty - check ID matching between datasets")
    if "Phylogroup" not in merged.columns:
        raise ValueError("Phylogroup column not found in merged data")
    return large, merged, without


def synthetic_pangenome(n, g, seed=12345, core_frac=0.15, core_freq=0.98):
    """Synthetic binary pan-genome: 15% core genes at f=0.98, accessory genes
    f ~ Beta(0.1, 1); X[s, g] ~ Bernoulli(f_g). numpy PCG64(seed). Returns u8 [n, g]."""
    rng = np.random.Generator(np.random.PCG64(seed))
    f = rng.beta(0.1, 1.0, size=g)
    core = rng.random(g) < core_frac
    f[core] = core_freq
    out = np.empty((n, g), dtype=np.uint8)
    step = max(1, (1 << 26) // max(g, 1))
    for s in range(0, n, step):
        e = min(n, s + step)
        out[s:e] = rng.random((e - s, g), dtype=np.float32) < f[None, :]
    return out


def write_synthetic_csvs(root, n, g, seed=12345):
    """Write a synthetic data/ tree in the reference's on-disk layout (genes x strains CSV with a
    'Lineage' row, ID,Phylogroup CSV, essential genes CSV) for CLI runs without the private data."""
    import pandas as pd
    x = synthetic_pangenome(n, g, seed)
    genes = [f"gene{i:05d}" for i in range(g)]
    strains = [f"S{i:06d}" for i in range(n)]
    df = pd.DataFrame(x.T, index=genes, columns=strains)
    lineage = pd.DataFrame([[1] * n], index=["Lineage"], columns=strains)
    os.makedirs(os.path.join(root, "data"), exist_ok=True)
    pd.concat([lineage, df]).to_csv(os.path.join(root, "data", "F4_complete_presence_absence.csv"))
    groups = np.array(list("ABCDEFG"))[np.arange(n) % 7]
    pd.DataFrame({"ID": strains, "Phylogroup": groups}).to_csv(
        os.path.join(root, "data", "accessionID_phylogroup_BD.csv"), index=False)
    pd.DataFrame({"gene": genes[: max(1, g // 20)]}).to_csv(os.path.join(root, "data", "essential_genes.csv"),
                                                           index=False)
    return x
