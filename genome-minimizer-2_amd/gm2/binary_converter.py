"""Mask -> gene-list conversion, the consumer of the sampled masks: mirror of
explore_data/binary_converter.py (load_files :11-17, masks_to_gene_lists :19-76,
check_essential_genes :78-121) with the same files, names, ordering and errors.

The reference thresholds and compacts one Python row at a time. Here a 2-D mask array is
thresholded in one vectorised pass (the same float64 `>= threshold`) and, on a GPU box, packed 8 genes
per byte, uploaded and compacted on the device (gm2.masks: gm2_mask_row_offsets + gm2_mask_compact,
a row-popcount scan and a wave-parallel bit compaction) into a CSR of column indices that the host
turns into name lists; without a GPU the same CSR comes from numpy. Outputs are the same object
arrays (`np.array(list_of_lists, dtype=object)`, so equal-length rows become a 2-D object array
exactly as there).
"""
from __future__ import annotations

import logging
import os

import numpy as np

logger = logging.getLogger(__name__)


def load_files(essentials_csv_path: str, ids_npy_path: str):
    """(set of essential gene names, id lists) -- column '# gene' if present, else 'gene'."""
    import pandas as pd
    essential_genes = pd.read_csv(essentials_csv_path)
    col = "# gene" if "# gene" in essential_genes.columns else "gene"
    essential_set = set(essential_genes[col].astype(str).str.strip())
    # object arrays of Python lists (written by masks_to_gene_lists) need the pickle loader
    id_lists = np.load(ids_npy_path, allow_pickle=True)
    return essential_set, id_lists


def _threshold_rows(masks, P, threshold):
    if masks.dtype != object and masks.ndim == 2:
        if masks.shape[1] != P:
            msg = f"Mask row 0 has length {masks.shape[1]}, but dataset has {P} gene columns."
            logger.error(msg)
            raise ValueError(msg)
        # the same float64 comparison as the reference's per-row np.asarray(row, float) >= t
        # (exact for every integer / float32 / float64 mask), without an N x G float copy
        return masks >= threshold
    rows = []
    for i, row in enumerate(masks):
        r = np.asarray(row, dtype=float)
        if r.size != P:
            msg = f"Mask row {i} has length {r.size}, but dataset has {P} gene columns."
            logger.error(msg)
            raise ValueError(msg)
        rows.append(r >= threshold)
    return np.stack(rows, axis=0) if rows else np.zeros((0, P), dtype=bool)


def gene_index_csr(M):
    """(row offsets, ascending column indices) of a boolean [N, P] mask: on the device when one is
    visible (packed upload + gm2 compaction), else numpy."""
    import torch
    if M.shape[0] and torch.cuda.is_available():
        from .masks import PackedMasks
        return PackedMasks.from_host(M, threshold=True).gene_index_csr()
    nz = np.nonzero(M)
    offsets = np.zeros(M.shape[0] + 1, dtype=np.int64)
    np.cumsum(np.bincount(nz[0], minlength=M.shape[0]), out=offsets[1:])
    return offsets, nz[1].astype(np.int32)


def gene_lists_from_csr(offsets, idx, names):
    from .masks import gene_lists_from_csr as f
    return f(offsets, idx, names)


def masks_to_gene_lists(masks_npy_path: str, cols, out_ids_npy: str, threshold: float = 0.5):
    """Threshold each mask row (>= threshold) and list the present genes' names in column order;
    duplicate gene names keep their first occurrence (binary_converter.py:29-36)."""
    cols = np.asarray(cols)
    P = len(cols)
    uniq, first_idx = np.unique(cols, return_index=True)
    if len(uniq) != P:
        logger.warning(f"{P - len(uniq)} duplicate gene names detected; keeping first occurrences")
        keep = np.zeros(P, dtype=bool)
        keep[np.sort(first_idx)] = True
        cols = cols[keep]
        P = len(cols)
    masks = np.load(masks_npy_path, allow_pickle=True)
    if masks.dtype == np.uint8 and masks.ndim == 2 and P > 8 and masks.shape[1] == (P + 7) // 8:
        # `main.py --mode sample --mask-dtype bits`: numpy packbits(bitorder='little') rows
        masks = np.unpackbits(masks, axis=1, count=P, bitorder="little")
    if masks.ndim == 1:
        if len(masks) and isinstance(masks[0], (list, np.ndarray)):
            masks = np.array([np.asarray(row) for row in masks], dtype=object)
        else:
            masks = masks[None, :]
    M = _threshold_rows(masks, P, threshold)
    N = M.shape[0]
    offsets, idx = gene_index_csr(M)
    id_lists = gene_lists_from_csr(offsets, idx, cols)
    if out_ids_npy:
        os.makedirs(os.path.dirname(out_ids_npy) or ".", exist_ok=True)
        np.save(out_ids_npy, np.array(id_lists, dtype=object))
    sizes = np.fromiter((len(x) for x in id_lists), dtype=int, count=N)
    print(f"✓ Number of samples processed = {N} | Average gene count = {sizes.mean() if N else float('nan'):.1f}")
    return id_lists


def check_essential_genes(essential_set, id_lists, out_ids_npy):
    """Add every missing essential gene to each sample, sort, save `<base>_with_essentials<ext>`."""
    updated, n_fixed, n_ok = [], 0, 0
    for gene_list in id_lists:
        if isinstance(gene_list, np.ndarray):
            gene_list = gene_list.tolist()
        gene_set = set(gene_list)
        missing = essential_set - gene_set
        if missing:
            gene_set.update(missing)
            n_fixed += 1
        else:
            n_ok += 1
        updated.append(sorted(gene_set))
    base, ext = os.path.splitext(out_ids_npy)
    out_path = base + "_with_essentials" + ext
    np.save(out_path, np.array(updated, dtype=object))
    print(f"✓ Verified {len(id_lists)} samples | already OK: {n_ok} | fixed: {n_fixed}")
    return out_path
