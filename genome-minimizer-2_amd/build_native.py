#!/usr/bin/env python3
"""Build libgm2.so (HIP, gfx950) in-tree: csrc/*.hip -> build/*.o -> gm2/libgm2.so.

Plain hipcc, no CMake: `python genome-minimizer-2_amd/build_native.py [--force] [-j N]`.
Objects are rebuilt when their source or any header is newer. The .so is git-ignored but
travels to the GPU box with the gpurun snapshot.
"""
import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "build")
OUT = os.path.join(HERE, "gm2", "libgm2.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-function",
         "-I" + CSRC, "-I" + os.path.join(ROOT, "include")]


def _newer(src, dst, deps):
    if not os.path.exists(dst):
        return True
    t = os.path.getmtime(dst)
    return any(os.path.getmtime(p) > t for p in [src] + deps)


def build(force=False, jobs=None, verbose=False):
    os.makedirs(BUILD, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    deps = glob.glob(os.path.join(CSRC, "*.hpp")) + glob.glob(os.path.join(ROOT, "include", "*.h"))
    objs, todo = [], []
    for s in srcs:
        o = os.path.join(BUILD, os.path.basename(s)[:-4] + ".o")
        objs.append(o)
        if force or _newer(s, o, deps):
            todo.append((s, o))

    def cc(so):
        s, o = so
        cmd = [HIPCC] + FLAGS + ["-c", s, "-o", o]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {s}:\n{r.stdout}\n{r.stderr}")
        if verbose and r.stderr.strip():
            print(r.stderr, file=sys.stderr)
        return o

    jobs = jobs or min(8, max(1, len(todo)))
    with cf.ThreadPoolExecutor(jobs) as ex:
        list(ex.map(cc, todo))
    if todo or force or not os.path.exists(OUT) or any(os.path.getmtime(o) > os.path.getmtime(OUT) for o in objs):
        cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", OUT] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    return OUT


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    a = ap.parse_args()
    print(build(force=a.force, jobs=a.j, verbose=True))
