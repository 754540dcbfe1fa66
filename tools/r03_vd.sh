#!/bin/bash
# A/B of the per-tile value dictionaries on the whole V-cycle (same box, same binary).
set -euo pipefail
export TMPDIR=/tmp
TAG=${1:-r03_vd}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in 1 2; do
  timeout -k 10 300 python3 -u bench.py --cpu-baseline off --pcg-rtol 0 > "$OUT/bench_vd0_$rep.json" 2> "$OUT/bench_vd0_$rep.log"
  echo "vd0 $rep done"
  timeout -k 10 300 python3 -u bench.py --cpu-baseline off --pcg-rtol 0 --value-dict > "$OUT/bench_vd1_$rep.json" 2> "$OUT/bench_vd1_$rep.log"
  echo "vd1 $rep done"
done
