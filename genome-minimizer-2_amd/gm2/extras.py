"""Sampling / checkpoint utilities — mirror of src/genome_minimizer_2/utils/extras.py:
load_model (:166-189), sample_from_model (:192-203), get_latent_variables (:205-228),
count_essential_genes (:49-87), write_samples_to_dataframe (:31-39). Plots are out of scope."""
from __future__ import annotations

import numpy as np
import torch

from . import native
from .data import ResidentMatrix, as_strain_loader
from .model import VAE


def load_model(input_dim, hidden_dim, latent_dim, path_to_model, precision=native.GM2_BF16):
    """VAE(...) + load_state_dict(torch.load(path, weights_only=True)) + eval() (extras.py:185-187)."""
    model = VAE(input_dim, hidden_dim, latent_dim, precision=precision, init=False)
    model.load_state_dict(torch.load(path_to_model, weights_only=True, map_location="cpu"))
    model.eval()
    return model


def sample_from_model(model, latent_dim, num_samples, device, binary_dtype=np.float64, return_probs=True,
                      chunk=65536, stats=None):
    """z ~ N(0, I) drawn with torch.randn(num_samples, latent_dim, device=device) exactly as the
    reference, decoded with eval-mode BatchNorm (hidden layers in fp32; with probs requested, the
    reference's default, the output layer in exact fp32 too, else gated per tile between bf16x3 and
    fp32 with the certified band recomputed in fp64: gm2.h GM2_OPT_SAMPLE_SPLIT), thresholded at
    sigmoid > 0.5. Returns (binary [N,G] as `binary_dtype` (reference: float64), probs fp32 [N,G] or
    None, z). `stats` (a dict, optional) receives this call's decode counters (VAE.decode_stats:
    tiles per path, band elements recomputed in fp64, bits flipped)."""
    with torch.no_grad():
        z = torch.randn(num_samples, latent_dim, device=device)
    before = model.decode_stats() if stats is not None else None
    mask, probs = model.decode_mask(z, want_probs=return_probs, chunk=chunk)
    if stats is not None:
        after = model.decode_stats()
        stats.update({k: after[k] - before[k] for k in after})
    binary = mask.cpu().numpy()
    if binary_dtype is not None and binary_dtype != np.uint8:
        binary = binary.astype(binary_dtype)
    return binary, (probs.cpu().numpy() if probs is not None else None), z


def get_latent_variables(model, data_loader, device=None):
    """Encoder means of every row of `data_loader`, in loader order (extras.py:205-228)."""
    model.eval()
    loader = as_strain_loader(data_loader, model.device)
    mat = loader.matrix
    out = []
    ws = model.workspace(model.precision, loader.batch_size)
    for rows in loader:
        n = rows.shape[0]
        mu = torch.empty(n, model.latent_dim, device=model.device)
        native.encode(ws, native.make_batch(mat.data, mat.ld, rows, n, None), model.params, model.bn, mu, None)
        out.append(mu)
    if not out:
        return np.zeros((0, model.latent_dim), np.float32)
    return torch.cat(out).cpu().numpy()


def count_essential_genes(binary_generated_samples, essential_gene_positions):
    """Per sample, how many essential genes are present: a gene counts when ANY of its column
    positions (< G; negative positions index from the end, as numpy does there) is non-zero after
    `astype(int)` (extras.py:65-85). Packed device masks (gm2.masks.PackedMasks, what --mode sample
    produces) are counted on the GPU (gm2_mask_count_groups); a host array keeps the reference's
    host semantics, vectorised over samples instead of the per-sample loop."""
    from .masks import PackedMasks
    if isinstance(binary_generated_samples, PackedMasks):
        return binary_generated_samples.count_groups(essential_gene_positions)
    b = np.asarray(binary_generated_samples)
    G = b.shape[1]
    # the reference tests `astype(int) != 0` (truncation: 0.7 counts as absent)
    present = b if b.dtype == bool else (b != 0 if b.dtype.kind in "iu" else b.astype(int) != 0)
    counts = np.zeros(b.shape[0], dtype=int)
    for _, positions in essential_gene_positions.items():
        cols = [p for p in positions if p < G]
        if cols:
            counts += present[:, cols].any(axis=1)
    return counts


def _csv_field(s) -> str:
    """One field as pandas' to_csv writes it (csv.QUOTE_MINIMAL, ',' separator, '"' quote)."""
    s = str(s)
    if any(ch in s for ch in ',"\n\r'):
        return '"' + s.replace('"', '""') + '"'
    return s


def write_samples_to_dataframe(binary_generated_samples, all_genes, output_file, max_chunk_bytes=1 << 26):
    """Genes x samples CSV with a leading 'Gene' column (extras.py:31-39).

    The reference builds a DataFrame, transposes it and calls to_csv, which formats every cell in
    Python (tens of MB/s; hours at 1e5 samples x 55k genes). For 0/1 masks -- what sampling
    produces -- this writes the same bytes directly: each cell is one of two fixed tokens ("0.0" /
    "1.0" for float masks, "0" / "1" for integer ones, as pandas formats them), so a block of genes
    is one lookup-table gather over the transposed mask and one write per gene row. Any other
    input (fractional values, bool, non-2-D) goes through the reference's pandas path."""
    m = np.asarray(binary_generated_samples)
    genes = list(all_genes)
    fast = m.ndim == 2 and m.shape[1] == len(genes) and m.dtype.kind in "fiu"
    if fast:
        fast = bool(((m == 0) | (m == 1)).all())
    if not fast:
        import pandas as pd
        df = pd.DataFrame(binary_generated_samples, columns=all_genes)
        df.index = [f"Sample_{i+1}" for i in range(df.shape[0])]
        df = df.transpose()
        df.columns = [f"Sample_{i+1}" for i in range(df.shape[1])]
        df = df.reset_index().rename(columns={"index": "Gene"})
        df.to_csv(output_file, index=False)
        return
    n = m.shape[0]
    toks = (b"0.0,", b"1.0,") if m.dtype.kind == "f" else (b"0,", b"1,")
    w = len(toks[0])
    lut = np.frombuffer(toks[0] + toks[1], dtype=np.uint8).reshape(2, w)
    gchunk = max(1, min(len(genes), max_chunk_bytes // max(1, n * w)))
    with open(output_file, "wb") as f:
        f.write(("Gene" + "".join(f",Sample_{i + 1}" for i in range(n)) + "\n").encode())
        for g0 in range(0, len(genes), gchunk):
            g1 = min(len(genes), g0 + gchunk)
            block = lut[(m[:, g0:g1].T != 0).view(np.uint8)]  # [genes, n, w] tokens
            block = block.reshape(g1 - g0, n * w)
            if n:
                block[:, -1] = ord("\n")  # the last token's comma ends the row
            for j in range(g1 - g0):
                f.write((_csv_field(genes[g0 + j]) + ("," if n else "\n")).encode())
                f.write(block[j].tobytes())


def as_matrix(x, device=None):
    return x if isinstance(x, ResidentMatrix) else ResidentMatrix(x, device=device)
