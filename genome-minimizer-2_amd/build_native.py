#!/usr/bin/env python3
"""Build libgm2 (HIP, gfx950) in-tree: csrc/*.hip -> build*/ objects -> the variant's output.

Plain hipcc, no CMake: `python genome-minimizer-2_amd/build_native.py [--variant V] [--force] [-j N]`.
Variants:
  release  gm2/libgm2.so        the product library
  debug    gm2/libgm2_debug.so  -DGM2_DEBUG: device-side bounds checks of the index data the kernels
                                follow + host layout checks (include/gm2_debug.h); same results
  asan     build_asan/gm2_host_asan  a host executable (tools/asan/host_asan.cpp) linked with every
                                source built -DGM2_DEBUG and AddressSanitizer on the HOST code only
                                (-Xarch_host -fsanitize=address); it drives the C-ABI's host-side
                                logic (layouts, options, argument and error paths) with no GPU
Objects are rebuilt when their source or any header is newer. Outputs are git-ignored but travel to
the GPU box with the gpurun snapshot.
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


VARIANTS = {
    "release": dict(build=BUILD, out=OUT, flags=[], link=["-shared"]),
    "debug": dict(build=os.path.join(HERE, "build_debug"), out=os.path.join(HERE, "gm2", "libgm2_debug.so"),
                  flags=["-DGM2_DEBUG"], link=["-shared"]),
    "asan": dict(build=os.path.join(HERE, "build_asan"), out=os.path.join(HERE, "build_asan", "gm2_host_asan"),
                 flags=["-DGM2_DEBUG", "-g", "-fno-omit-frame-pointer", "-Xarch_host", "-fsanitize=address"],
                 link=["-Xarch_host", "-fsanitize=address"],
                 extra=[os.path.join(ROOT, "tools", "asan", "host_asan.cpp")]),
    # the second build of a same-box A/B (tools/ab_lib.sh; GM2_LIB_PATH selects it; not part of
    # build()): an experiment's code sits behind #ifdef GM2_AB
    "ab": dict(build=os.path.join(HERE, "build_ab"), out=os.path.join(HERE, "gm2", "libgm2_ab.so"),
               flags=["-DGM2_AB"], link=["-shared"]),
}


def build(force=False, jobs=None, verbose=False, variant="release"):
    v = VARIANTS[variant]
    bdir, out = v["build"], v["out"]
    os.makedirs(bdir, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip"))) + v.get("extra", [])
    deps = glob.glob(os.path.join(CSRC, "*.hpp")) + glob.glob(os.path.join(ROOT, "include", "*.h"))
    objs, todo = [], []
    for s in srcs:
        o = os.path.join(bdir, os.path.splitext(os.path.basename(s))[0] + ".o")
        objs.append(o)
        if force or _newer(s, o, deps):
            todo.append((s, o))

    def cc(so):
        s, o = so
        lang = ["-x", "hip"] if s.endswith(".cpp") else []
        cmd = [HIPCC] + FLAGS + v["flags"] + lang + ["-c", s, "-o", o]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {s}:\n{r.stdout}\n{r.stderr}")
        if verbose and r.stderr.strip():
            print(r.stderr, file=sys.stderr)
        return o

    jobs = jobs or min(8, max(1, len(todo)))
    with cf.ThreadPoolExecutor(jobs) as ex:
        list(ex.map(cc, todo))
    if todo or force or not os.path.exists(out) or any(os.path.getmtime(o) > os.path.getmtime(out) for o in objs):
        cmd = [HIPCC, "--offload-arch=gfx950"] + v["link"] + ["-fPIC", "-o", out] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("--variant", choices=sorted(VARIANTS), default="release")
    a = ap.parse_args()
    print(build(force=a.force, jobs=a.j, verbose=True, variant=a.variant))
