#!/usr/bin/env python3
"""Host-side enqueue time of one training step vs its GPU wall time (is the step host-bound?),
for libgm2 option values: python3 tools/host_probe.py OPTION v1 v2 ..."""
import os
import sys
import time

import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "tools"))
import recon_ab as R  # noqa: E402  (builds the C2 model / workspace at import)
from gm2 import native  # noqa: E402

opt = sys.argv[1] if len(sys.argv) > 1 else "bn_epilogue"
vals = [int(v) for v in sys.argv[2:]] or [1, 0]
key = R.KEYS[opt]
for rnd in range(2):
    for v in vals:
        native.set_option(key, v)
        for i in range(3):
            R.step(i)
        torch.cuda.synchronize()
        host = []
        t0 = time.perf_counter()
        for i in range(10):
            a = time.perf_counter()
            R.step(i)
            host.append(time.perf_counter() - a)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"{opt}={v}: host enqueue/step {1e3 * sorted(host)[5]:.3f} ms (first {1e3 * host[0]:.3f}), "
              f"loop {1e3 * (t1 - t0) / 10:.3f} ms/step, wall incl. drain {1e3 * (t2 - t0) / 10:.3f} ms/step")
