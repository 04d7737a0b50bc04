#!/usr/bin/env python3
"""Print the kernel timeline of the last full training step of a rocprofv3 kernel trace
(gpurun_out/prof_TAG/run_kernel_trace.csv): start/end relative to the step, queue, grid, name."""
import csv
import re
import sys

rows = list(csv.DictReader(open(f"gpurun_out/prof_{sys.argv[1]}/run_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
gath = [i for i, r in enumerate(rows) if "k_gather" in r["Kernel_Name"] or "k_resident_rows" in r["Kernel_Name"]]
lo, hi = gath[-2], gath[-1]
t0 = int(rows[lo]["Start_Timestamp"])


def short(n):
    n = re.sub(r"\(gm2::.*$", "", n).replace("void ", "").replace("gm2::(anonymous namespace)::", "")
    return re.sub(r"\(.*$", "", n)[:72]


for r in rows[lo - 3:hi]:
    s = (int(r["Start_Timestamp"]) - t0) / 1e3
    e = (int(r["End_Timestamp"]) - t0) / 1e3
    print(f"{s:8.1f} {e:8.1f} {e - s:7.1f} q{r['Queue_Id']} g{r['Grid_Size_X']:>8} {short(r['Kernel_Name'])}")
print("step (gather to gather):", (int(rows[hi]["Start_Timestamp"]) - t0) / 1e3, "us")
