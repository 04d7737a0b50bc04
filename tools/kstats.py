#!/usr/bin/env python3
"""Per-kernel summary of rocprofv3 runs of bench.py (tools/prof.sh):

  * time per training step by kernel (kernel trace of the timed steps: every dispatch between the
    first and last gm2 recon-loss launch, divided by the number of steps);
  * MFMA utilisation per kernel from SQ_VALU_MFMA_BUSY_CYCLES over the kernel's SIMD-cycles,
    SIMD-cycles = GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs) x 256 CUs x 4 SIMDs
    (MI355X_MICROARCH.md DVFS item: GRBM_GUI_ACTIVE is the sum over XCDs), cross-checked against
    the kernel's algorithmic MFMA count where it is known;
  * HBM bytes per launch from separate FETCH_SIZE / WRITE_SIZE passes (FETCH_SIZE x2 on gfx950).

Usage: python3 tools/kstats.py TAG [out.json|-] [timed steps]   (reads gpurun_out/{prof,pmc_mfma,pmc_fetch,pmc_write}_TAG)
"""
import collections
import csv
import json
import re
import sys


def short(name):
    n = re.sub(r"\(gm2::.*$|\(int, at::.*$", "", name)
    n = n.replace("void ", "").replace("gm2::(anonymous namespace)::", "")
    return re.sub(r"\(.*$", "", n)


def trace(d):
    rows = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    return rows


def counters(d, with_grid=False):
    out = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        out[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        k = short(r["Kernel_Name"])
        names[int(r["Dispatch_Id"])] = (k, int(r["Grid_Size"])) if with_grid else k
    return out, names


def step_breakdown(tag, steps):
    rows = trace(f"gpurun_out/prof_{tag}")
    recon = [i for i, r in enumerate(rows) if "k_gemm_recon_loss" in r["Kernel_Name"]]
    # the timed steps of a C2-only run (bench.py --no-c5): from the `steps`-th last gather (a step's
    # first kernel) to the end of the last Adam launch (the final join's deferred output-layer update)
    gath = [i for i, r in enumerate(rows) if "k_gather" in r["Kernel_Name"] or "k_resident_rows" in r["Kernel_Name"]]
    adam = [i for i, r in enumerate(rows) if "k_adam_fused" in r["Kernel_Name"]]
    lo = gath[-steps]
    hi = adam[-1] + 1
    agg = collections.defaultdict(lambda: [0, 0.0])
    grids = {}
    for r in rows[lo:hi]:
        k = short(r["Kernel_Name"])
        agg[k][0] += 1
        agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
        grids.setdefault(k, int(r["Grid_Size_X"]) * int(r.get("Grid_Size_Y", 1) or 1) * int(r.get("Grid_Size_Z", 1) or 1))
    wall = (int(rows[hi - 1]["End_Timestamp"]) - int(rows[lo]["Start_Timestamp"])) * 1e-3 / steps
    return wall, {k: (v[0] / steps, v[1] / steps) for k, v in agg.items()}, grids


def mfma(tag):
    try:
        c, names = counters(f"gpurun_out/pmc_mfma_{tag}")
    except FileNotFoundError:
        return {}
    per = collections.defaultdict(list)
    for d, v in c.items():
        if v.get("GRBM_GUI_ACTIVE", 0) <= 0:
            continue
        simd_cycles = v["GRBM_GUI_ACTIVE"] / 8 * 256 * 4
        per[names[d]].append((v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / simd_cycles, v["GRBM_GUI_ACTIVE"] / 8))
    return {k: (sorted(x[0] for x in v)[len(v) // 2], len(v)) for k, v in per.items()}


def traffic(tag):
    out = {}
    for kind, scale in (("fetch", 2.0), ("write", 1.0)):
        try:
            c, names = counters(f"gpurun_out/pmc_{kind}_{tag}", with_grid=True)
        except FileNotFoundError:
            continue
        per = collections.defaultdict(list)
        for d, v in c.items():
            per[names[d]].append(scale * 1024 * sum(v.values()))
        for k, v in per.items():
            out.setdefault(k, {})[kind] = sorted(v)[len(v) // 2]
    return out


def main(tag, dst=None, steps=6):
    wall, brk, grids = step_breakdown(tag, steps)
    util = mfma(tag)
    tr = traffic(tag)
    rows = []
    print(f"step wall (a step's gather -> the last Adam end, per step): {wall:.1f} us")
    for k, (n, us) in sorted(brk.items(), key=lambda kv: -kv[1][1]):
        u = util.get(k, (None, 0))[0]
        t = tr.get((k, grids.get(k)), {})
        rows.append({"kernel": k, "launches_per_step": n, "us_per_step": round(us, 1),
                     "mfma_busy": None if u is None else round(u, 4),
                     "fetch_bytes": t.get("fetch"), "write_bytes": t.get("write")})
        print(f"{us:9.1f} us  x{n:<4.0f} mfma {'-' if u is None else f'{u:6.3f}'}  "
              f"fetch {t.get('fetch', 0) / 1e6:9.1f} MB  write {t.get('write', 0) / 1e6:8.1f} MB  {k}")
    if dst:
        json.dump({"tag": tag, "step_wall_us": round(wall, 1), "kernels": rows,
                   "notes": "us_per_step = summed kernel durations per training step (side-stream kernels overlap); "
                            "mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 * 1024 SIMDs), median launch; "
                            "fetch = 2 x FETCH_SIZE (gfx950), per launch, median"}, open(dst, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 and sys.argv[2] != "-" else None,
         int(sys.argv[3]) if len(sys.argv) > 3 else 6)
