#!/usr/bin/env python3
"""Per-kernel register / spill table from hipcc's `-Rpass-analysis=kernel-resource-usage` remarks.

    hipcc ... -Rpass-analysis=kernel-resource-usage -c gemm.hip 2> remarks.txt
    python3 tools/kres.py remarks.txt [--grep SUBSTR]
"""
import re
import subprocess
import sys

KEYS = {"VGPRs": "vgpr", "AGPRs": "agpr", "ScratchSize [bytes/lane]": "scratch", "Occupancy [waves/SIMD]": "occ",
        "SGPRs Spill": "sspill", "VGPRs Spill": "vspill"}


def parse(path):
    rows, cur, d = [], None, {}
    for line in open(path):
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            if cur:
                rows.append((cur, d))
            cur, d = m.group(1), {}
            continue
        m = re.search(r"remark:\s+([A-Za-z][A-Za-z /\[\]]*?): (\d+)", line)
        if m and m.group(1) in KEYS:
            d[KEYS[m.group(1)]] = int(m.group(2))
    if cur:
        rows.append((cur, d))
    names = subprocess.run(["c++filt"], input="\n".join(r[0] for r in rows), capture_output=True, text=True).stdout.split("\n")
    out = []
    for (raw, d), dn in zip(rows, names):
        dn = dn.replace("gm2::(anonymous namespace)::", "").replace("unsigned short", "bf16")
        dn = re.sub(r"\(gm2::.*$", "", dn)
        out.append((dn, d))
    return out


if __name__ == "__main__":
    flt = sys.argv[sys.argv.index("--grep") + 1] if "--grep" in sys.argv else ""
    print(f"{'vgpr':>5} {'agpr':>5} {'vspill':>6} {'scratch':>7} {'occ':>3}  kernel")
    for dn, d in parse(sys.argv[1]):
        if flt in dn:
            print(f"{d.get('vgpr', 0):5d} {d.get('agpr', 0):5d} {d.get('vspill', 0):6d} {d.get('scratch', 0):7d} "
                  f"{d.get('occ', 0):3d}  {dn}")
