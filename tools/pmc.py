#!/usr/bin/env python3
"""Summarise two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) into per-launch HBM traffic.

MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE
reports half the bytes of a wide coalesced streaming read, so it is doubled here. Values are the
median over the launches of each (kernel, grid) pair. Usage:
    python3 tools/pmc.py gpurun_out/pmc_fetch_TAG gpurun_out/pmc_write_TAG profiles/rNN_pmc_traffic.json
"""
import collections
import csv
import json
import re
import sys


def short(name):
    n = re.sub(r"\(gm2::.*$", "", name)
    return n.replace("void ", "").replace("gm2::(anonymous namespace)::", "")


def load(d):
    out = collections.defaultdict(list)
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        out[(short(r["Kernel_Name"]), int(r["Grid_Size"]))].append(float(r["Counter_Value"]))
    return out


def med(v):
    v = sorted(v)
    return v[len(v) // 2]


def main(fetch_dir, write_dir, dst):
    f, w = load(fetch_dir), load(write_dir)
    rows = []
    for key in sorted(f, key=lambda k: -med(f[k])):
        fb = 2.0 * med(f[key]) * 1024
        wb = med(w[key]) * 1024 if key in w else None
        rows.append({"kernel": key[0], "grid": key[1], "launches": len(f[key]),
                     "fetch_bytes": fb, "write_bytes": wb,
                     "traffic_bytes": fb + (wb or 0.0)})
    json.dump({"source": [fetch_dir, write_dir], "correction": "FETCH_SIZE x2 (gfx950), KiB -> bytes",
               "kernels": rows}, open(dst, "w"), indent=1)
    for r in rows:
        print(f"{r['traffic_bytes'] / 1e6:10.1f} MB  (fetch {r['fetch_bytes'] / 1e6:9.1f}, write "
              f"{(r['write_bytes'] or 0) / 1e6:9.1f})  x{r['launches']:<3d} {r['kernel']} grid={r['grid']}")


if __name__ == "__main__":
    main(*sys.argv[1:4])
