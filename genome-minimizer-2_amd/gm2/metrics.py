"""Test-set reconstruction metrics — mirror of src/genome_minimizer_2/training/evaluation/metrics.py
calculate_reconstruction_metrics (:19-64) on libgm2.

The reference collects model(batch) for the whole test split, thresholds recon > threshold and
asks sklearn for F1 / accuracy, overall (flattened) and per sample. Here each batch's eval-mode
forward ends in gm2_recon_counts, whose epilogue compares the thresholded reconstruction with the
strain's genes and keeps only (TP, FP, FN) per strain: the [N, G] reconstruction never leaves the
GPU or even HBM. The sklearn formulas then follow exactly: F1 = 2TP / (2TP + FP + FN) (0 when the
denominator is 0: sklearn's zero_division default), accuracy = (G - FP - FN) / G. The forward is
exact fp32 (as the reference's) whatever the model's training precision."""
from __future__ import annotations

from typing import List, Tuple

import numpy as np
import torch

from . import native
from .data import as_strain_loader


def reconstruction_counts(model, test_loader, threshold: float = 0.5, eps_rng="device"):
    """int64 [N, 3] = (TP, FP, FN) per strain in loader order; eps drawn per batch like the
    reference's randn_like inside model(batch)."""
    model.eval()
    loader = as_strain_loader(test_loader, model.device)
    mat = loader.matrix
    ws = model.workspace(native.GM2_F32, loader.batch_size)
    out = []
    for rows in loader:
        n = rows.shape[0]
        eps = (torch.randn(n, model.latent_dim) if eps_rng == "cpu"
               else torch.randn(n, model.latent_dim, device=model.device)).to(model.device)
        counts = torch.empty(n, 3, dtype=torch.int32, device=model.device)
        native.recon_counts(ws, native.make_batch(mat.data, mat.ld, rows, n, eps), model.params, model.bn, threshold,
                            counts)
        out.append(counts)
    if not out:
        return np.zeros((0, 3), np.int64)
    return torch.cat(out).cpu().numpy().astype(np.int64)


def _f1(tp, fp, fn):
    den = 2 * tp + fp + fn
    return np.where(den > 0, 2 * tp / np.maximum(den, 1), 0.0)


def calculate_reconstruction_metrics(model, test_loader, threshold: float = 0.5,
                                     eps_rng="device") -> Tuple[float, float, List[float], List[float]]:
    """(overall_f1, overall_accuracy, per_sample_f1_scores, per_sample_accuracy_scores), metrics.py:19-64."""
    c = reconstruction_counts(model, test_loader, threshold, eps_rng)
    G = model.input_dim
    tp, fp, fn = c[:, 0], c[:, 1], c[:, 2]
    T, Fp, Fn = int(tp.sum()), int(fp.sum()), int(fn.sum())
    total = c.shape[0] * G
    overall_f1 = float(_f1(np.int64(T), np.int64(Fp), np.int64(Fn)))
    overall_acc = float((total - Fp - Fn) / total) if total else 0.0
    f1s = [float(v) for v in _f1(tp, fp, fn)]
    accs = [float(v) for v in (G - fp - fn) / G]
    return overall_f1, overall_acc, f1s, accs


__all__ = ["calculate_reconstruction_metrics", "reconstruction_counts"]
