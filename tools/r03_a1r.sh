#!/bin/bash
# A1 at 2048-nonzero tiles (long_tiles_min rule): the full-size long-row test, the 512^3
# config tests, then the default bench line.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03_a1r}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_configs.py -m gpu > "$OUT/tests.log" 2>&1
echo "tests ok"
timeout -k 10 400 python3 -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.log"
echo "bench ok"
