"""bench.py host logic (no GPU): the per-step scalar tables of the preset lines (round 6) follow the
reference's schedules -- v0/v1 linear KL beta at epoch 0 of a 10000-epoch run, v2/v3 cosine beta
advancing its counter once per batch (loss_components.py:76-91, 187-202), gene abundance w*gamma
(loss_components.py:111-115: v1/v2 gamma 1.0, v3 gamma 2.0 with weight 1), L1 lambda 0.01 for
v1-v3 (experiments.py:42-114, trainer.py:193-257) -- and the Adam constants of torch.optim.Adam
at lr 1e-3 (bias corrections per step)."""
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_preset_scalar_tables():
    import bench
    from gm2 import native
    n = 25
    t0, t1, t2, t3 = (bench.scalar_table(n, p) for p in ("v0", "v1", "v2", "v3"))
    for t in (t0, t1):
        assert np.allclose(t[:, native.S_BETA], 0.1)
    cos = lambda k, T, lo, hi: lo + (hi - lo) / 2 * (1 + math.cos(math.pi * (k % T) / T))  # noqa: E731
    assert np.allclose(t2[:, native.S_BETA], [cos(k, 10, 0.0, 1.0) for k in range(n)])
    assert np.allclose(t3[:, native.S_BETA], [cos(k, 50, 0.1, 1.0) for k in range(n)])
    assert t2[10, native.S_BETA] == t2[0, native.S_BETA] == 1.0 and t2[5, native.S_BETA] < 0.51
    assert np.all(t0[:, native.S_WGAMMA] == 0) and np.all(t0[:, native.S_LAMBDA] == 0)
    assert np.allclose(t1[:, native.S_WGAMMA], 1.0) and np.allclose(t2[:, native.S_WGAMMA], 1.0)
    assert np.allclose(t3[:, native.S_WGAMMA], 2.0)
    for t in (t1, t2, t3):
        assert np.allclose(t[:, native.S_LAMBDA], 0.01)
    for t in (t0, t1, t2, t3):
        k = np.arange(1, n + 1)
        assert np.allclose(t[:, native.S_NEG_STEP], -(1e-3 / (1 - 0.9 ** k)))
        assert np.allclose(t[:, native.S_BC2_SQRT], np.sqrt(1 - 0.999 ** k))
        assert np.all(t[:, native.S_MAX_NORM] == 1.0)
    # the train FLOP count of SURVEY.md 8(d) at the bench's dims
    assert bench.train_flops_per_vector(55039, 1024, 64) == 2 * (3 * (2 * 55039 * 1024 + 4 * 1024 ** 2 + 3 * 1024 * 64)
                                                                  - 55039 * 1024)
    assert abs(bench.train_flops_per_vector(55039, 1024, 64) / 1e6 - 589.9) < 0.1
    assert abs(bench.train_flops_per_vector(55039, 512, 32) / 1e6 - 288.4) < 0.1
