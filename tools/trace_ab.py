#!/usr/bin/env python3
"""Per-kernel median durations (us) of the 256-tile GEMMs in tools/trace_ab.sh runs: python3 tools/trace_ab.py TAG"""
import collections
import csv
import glob
import re
import sys

tag = sys.argv[1]
res = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sorted(glob.glob(f"gpurun_out/tab_{tag}_*_*/")):
    var = re.search(rf"tab_{tag}_(\d+)_\d+", d).group(1)
    for f in glob.glob(d + "**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if "Cfg<256" not in n and "k_adam" not in n and "k_fwd_tail" not in n:
                continue
            key = (n[n.find("k_"):n.find("<")] + " " + n[n.find("unsigned"):n.find(">(")])[:60]
            g = r.get("Grid_Size_X", r.get("Grid_Size"))
            res[(key, g)][var].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k in sorted(res):
    line = f"{k[0]:62s} grid={k[1]:>8s}"
    for var in sorted(res[k]):
        v = sorted(res[k][var])
        line += f"  v{var}: {v[len(v) // 2]:7.1f} (n={len(v)})"
    print(line)
