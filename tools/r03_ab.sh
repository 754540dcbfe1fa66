#!/bin/bash
# Layout defaults check: the parity tests touching the tile layouts, then two bench lines.
set -euo pipefail
export TMPDIR=/tmp
TAG=${1:-r03_ab}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "dictionary or tile_configs or vcycle or stream_bytes or layouts_agree or restriction" > "$OUT/tests.log" 2>&1
echo "tests ok"
for r in 1 2; do
  timeout -k 10 300 python3 -u bench.py --cpu-baseline off --pcg-rtol 0 > "$OUT/bench_$r.json" 2> "$OUT/bench_$r.log"
  echo "bench $r ok"
done
