"""Packed sampled masks and their consumers on the device.

A sampled mask set lives in HBM as numpy packbits(bitorder='little') rows (bit g & 7 of byte g // 8 =
gene g; row pitch native.packed_row_bytes(G), a multiple of 16; bits beyond G zero): 1e6 F4-shaped
genomes are 6.9 GB instead of 55 GB of u8 or 440 GB of the reference's float64. The reference's
consumers run on it without leaving the device:
  * count_essential_genes (utils/extras.py:49-87)        -> PackedMasks.count_groups
  * genome sizes (main.py:376-380 statistics)             -> PackedMasks.row_sizes
  * masks_to_gene_lists (explore_data/binary_converter.py:19-76) -> PackedMasks.gene_index_csr
and `to_host` returns the packed rows (8x less PCIe than u8) for the .npy writers.
"""
from __future__ import annotations

import numpy as np
import torch

from . import native


def essential_groups(essential_gene_positions, G):
    """The pickle dict {gene: [column, ...]} as CSR (group offsets, positions) of valid columns, in
    dict order. The reference tests `pos < G` (extras.py:71-82); a negative position indexes from
    the end as numpy does there (and raises where numpy would)."""
    offs, pos = [0], []
    for _, positions in essential_gene_positions.items():
        for p in positions:
            p = int(p)
            if p < G:
                if p < 0:
                    if p < -G:
                        raise IndexError(f"index {p} is out of bounds for axis 1 with size {G}")
                    p += G
                pos.append(p)
        offs.append(len(pos))
    return np.asarray(offs, dtype=np.int32), np.asarray(pos, dtype=np.int32)


class PackedMasks:
    """n x G packed masks on the device (a [n, ld] uint8 tensor)."""

    def __init__(self, bits: torch.Tensor, G: int):
        self.bits, self.G = bits, int(G)
        self.n, self.ld = int(bits.shape[0]), int(bits.shape[1])
        if self.ld % 16 or self.ld * 8 < self.G:
            raise ValueError("packed mask rows: pitch must be a multiple of 16 bytes covering G")

    @staticmethod
    def empty(n, G, device):
        ld = native.packed_row_bytes(G)
        return PackedMasks(torch.zeros(n, ld, dtype=torch.uint8, device=device), G)

    @staticmethod
    def from_host(mask, threshold=0.5, device=None):
        """Threshold a host [n, G] mask (any numeric dtype; `>= threshold` as binary_converter.py:55)
        and upload it packed."""
        m = np.asarray(mask)
        n, G = m.shape
        ld = native.packed_row_bytes(G)
        packed = np.zeros((n, ld), dtype=np.uint8)
        packed[:, : (G + 7) // 8] = np.packbits(m >= threshold, axis=1, bitorder="little")
        dev = device or torch.device("cuda", torch.cuda.current_device())
        return PackedMasks(torch.from_numpy(packed).to(dev), G)

    def to_host(self):
        """numpy packbits rows [n, ceil(G/8)] (bitorder 'little')."""
        return self.bits[:, : (self.G + 7) // 8].cpu().numpy()

    def unpack(self, dtype=np.uint8):
        """The [n, G] 0/1 mask on the host in `dtype` (the reference's float64 with dtype=float)."""
        u = np.unpackbits(self.to_host(), axis=1, count=self.G, bitorder="little")
        return u if dtype == np.uint8 else u.astype(dtype)

    def count_groups(self, essential_gene_positions):
        """count_essential_genes(binary, positions) on the device -> int64 numpy [n]."""
        offs, pos = essential_groups(essential_gene_positions, self.G)
        dev = self.bits.device
        counts = torch.empty(self.n, dtype=torch.int32, device=dev)
        go = torch.from_numpy(offs).to(dev)
        po = torch.from_numpy(pos if len(pos) else np.zeros(1, np.int32)).to(dev)
        native.mask_count_groups(self.bits, self.n, self.ld, go, len(offs) - 1, po, counts)
        return counts.cpu().numpy().astype(np.int64)

    def _keep(self, keep_cols):
        if keep_cols is None:
            return None
        k = np.zeros(self.ld, dtype=np.uint8)
        k[: (self.G + 7) // 8] = np.packbits(np.asarray(keep_cols, dtype=bool), bitorder="little")
        return torch.from_numpy(k).to(self.bits.device)

    def row_offsets(self, keep_cols=None):
        offsets = torch.empty(self.n + 1, dtype=torch.int64, device=self.bits.device)
        native.mask_row_offsets(self.bits, self.n, self.ld, self._keep(keep_cols), offsets)
        return offsets

    def row_sizes(self):
        """Genes per sample (binary.sum(axis=1)) -> int64 numpy [n]."""
        return np.diff(self.row_offsets().cpu().numpy())

    def gene_index_csr(self, keep_cols=None):
        """(offsets int64 [n+1], column indices int32) of the set genes of every row, ascending;
        keep_cols (bool [G]) restricts to the kept columns."""
        keep = self._keep(keep_cols)
        offsets = torch.empty(self.n + 1, dtype=torch.int64, device=self.bits.device)
        native.mask_row_offsets(self.bits, self.n, self.ld, keep, offsets)
        total = int(offsets[-1].item())
        idx = torch.empty(max(total, 1), dtype=torch.int32, device=self.bits.device)
        native.mask_compact(self.bits, self.n, self.ld, keep, offsets, idx)
        return offsets.cpu().numpy(), idx[:total].cpu().numpy()


def gene_lists_from_csr(offsets, idx, names):
    """[[names[i] for the row's indices] for every row] (binary_converter.py:64-66)."""
    names = np.asarray(names)
    sel = names[idx].tolist()
    return [sel[offsets[i]:offsets[i + 1]] for i in range(len(offsets) - 1)]
