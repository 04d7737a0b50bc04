#!/usr/bin/env python3
"""End-to-end run of the reference's own command line at F4 width on one MI355X: a synthetic
F4-shaped data/ tree (genes x strains CSV with the 'Lineage' row, ID/Phylogroup CSV; N = 7,512
strains as SURVEY.md's split probe, G = 55,039 genes), then
  main.py --mode training --preset v0 --epochs E          (CLI default batch 32, bf16)
  main.py --mode sample --model-path <that checkpoint> --num-samples S --mask-dtype bits --no-csv
each as a child process, with its wall time (CSV parse, model setup and process start included).
Usage: python3 tools/e2e_cli.py [root] [epochs] [samples]"""
import glob
import os
import pickle
import subprocess
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.join(HERE, "..")
sys.path.insert(0, os.path.join(REPO, "genome-minimizer-2_amd"))
from gm2.data import synthetic_pangenome  # noqa: E402

root = sys.argv[1] if len(sys.argv) > 1 else "/tmp/gm2_e2e"
epochs = int(sys.argv[2]) if len(sys.argv) > 2 else 2
samples = int(sys.argv[3]) if len(sys.argv) > 3 else 100000
N, G = int(os.environ.get("GM2_E2E_N", 7512)), int(os.environ.get("GM2_E2E_G", 55039))


def write_csvs():
    """The reference's on-disk layout (as gm2.data.write_synthetic_csvs), the big CSV written as
    bytes (pandas.to_csv takes minutes at this size)."""
    x = synthetic_pangenome(N, G, seed=12345)
    d = os.path.join(root, "data")
    os.makedirs(d, exist_ok=True)
    strains = [f"S{i:06d}" for i in range(N)]
    with open(os.path.join(d, "F4_complete_presence_absence.csv"), "wb") as f:
        f.write(("," + ",".join(strains) + "\n").encode())
        f.write(("Lineage," + ",".join(["1"] * N) + "\n").encode())
        row = np.empty(2 * N, dtype=np.uint8)
        row[0::2] = ord(",")
        xt = np.ascontiguousarray(x.T)
        for g in range(G):
            row[1::2] = xt[g] + ord("0")
            f.write(f"gene{g:05d}".encode() + row.tobytes() + b"\n")
    groups = np.array(list("ABCDEFG"))[np.arange(N) % 7]
    with open(os.path.join(d, "accessionID_phylogroup_BD.csv"), "w") as f:
        f.write("ID,Phylogroup\n" + "".join(f"{s},{p}\n" for s, p in zip(strains, groups)))
    with open(os.path.join(d, "essential_genes.csv"), "w") as f:
        f.write("gene\n" + "".join(f"gene{g:05d}\n" for g in range(G // 20)))
    # the sampling mode's essential-gene positions (the user's preprocessing output): 300 genes, some
    # at several positions
    rng = np.random.default_rng(7)
    pos = {f"ess{i}": sorted(rng.choice(G, size=1 + (i % 3 == 0), replace=False).tolist()) for i in range(300)}
    with open(os.path.join(root, "ess.pkl"), "wb") as f:
        pickle.dump(pos, f)


def run(args, tag):
    """The child's output streamed through (a long CSV parse must not look like a hang)."""
    t = time.perf_counter()
    p = subprocess.Popen([sys.executable, "-u", os.path.join(REPO, "main.py")] + args, cwd=REPO,
                         stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    for ln in p.stdout:
        if ln.strip() and "amdgpu.ids" not in ln:
            print(f"[{time.perf_counter() - t:7.1f} s] {ln.rstrip()}", flush=True)
    rc = p.wait()
    dt = time.perf_counter() - t
    print(f"--- {tag}: rc {rc}, {dt:.1f} s wall", flush=True)
    if rc != 0:
        sys.exit(rc)
    return dt


t0 = time.perf_counter()
write_csvs()
print(f"--- synthetic F4-shaped data/ ({N} strains x {G} genes) written in {time.perf_counter() - t0:.1f} s",
      flush=True)
run(["--mode", "training", "--preset", "v0", "--epochs", str(epochs), "--project-root", root], "training")
ckpt = glob.glob(os.path.join(root, "models", "**", "saved_VAE_v0.pt"), recursive=True)[0]
run(["--mode", "sample", "--model-path", ckpt, "--genes-path", os.path.join(root, "ess.pkl"), "--num-samples",
     str(samples), "--project-root", root, "--mask-dtype", "bits", "--no-csv"], "sampling")
