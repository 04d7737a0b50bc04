#!/bin/bash
# incremental build of the three libgm2 variants (release, debug, asan) before a GPU run
cd "$(dirname "$0")/.." || exit 2
for v in release debug asan; do
  timeout 1200 python3 genome-minimizer-2_amd/build_native.py --variant $v -j 6 > /tmp/build_$v.log 2>&1 || { echo "build $v failed"; tail -20 /tmp/build_$v.log; exit 1; }
done
echo "built release debug asan"
