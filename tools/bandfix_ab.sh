#!/bin/bash
# Same-box A/B of k_band_fix's tile order (XCD-aware default vs GM2_BANDFIX_LINEAR=1) on the bench's
# sample leg (trained v1 checkpoint, 1e6 genomes): R alternating runs of genomes/s, then one kernel
# trace per order for k_band_fix's duration.      bash tools/bandfix_ab.sh TAG R
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
T=$1; R=${2:-2}
out=gpurun_out/bandfix_$T.log
: > $out
B="--steps 3 --warmup 1 --no-cpu-baseline --no-f32-line --no-c5 --no-presets --no-c1"
for r in $(seq 1 $R); do
  for lin in 0 1; do
    if [ $lin = 1 ]; then export GM2_BANDFIX_LINEAR=1; else unset GM2_BANDFIX_LINEAR; fi
    res=$(timeout -k 10 300 python3 bench.py $B 2>/dev/null | tail -1)
    rc=$?
    [ $rc -ne 0 ] && { echo "linear $lin rc=$rc" >> $out; exit $rc; }
    echo "linear $lin $(echo "$res" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["sample"]; print("genomes/s", s["genomes_per_s"], "band", s["band_elements"], "flips", s["band_flips"])')" >> $out
  done
done
unset GM2_BANDFIX_LINEAR
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bfx_$T -o run --output-format csv -- python3 bench.py $B --sample-genomes 262144 > gpurun_out/prof_bfx_$T.log 2>&1 || exit $?
export GM2_BANDFIX_LINEAR=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bfl_$T -o run --output-format csv -- python3 bench.py $B --sample-genomes 262144 > gpurun_out/prof_bfl_$T.log 2>&1
exit $?
