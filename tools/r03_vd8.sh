#!/bin/bash
# 8-bit per-tile value dictionaries for tile-major sets (the 512^3 level-1 operator): parity
# tests, the A1 kernels, and the bench line. Each GPU step has its own time limit.
set -euo pipefail
export TMPDIR=/tmp
TAG=${1:-r03_vd8}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "value_dictionary or column_dictionary or tile_configs or vcycle_bit_exact or stream_bytes" > "$OUT/tests.log" 2>&1
echo "tests ok"
timeout -k 10 400 python3 -u tools/kbench.py --n 512 --levels 2 --mats A1 --ops 1,2 --reps 10 --configs 1024:1,1024:1:1:0 > "$OUT/kb_a1.jsonl" 2> "$OUT/kb.err"
echo "kbench ok"
timeout -k 10 300 python3 -u bench.py --cpu-baseline off --pcg-rtol 0 > "$OUT/bench.json" 2> "$OUT/bench.log"
echo "bench ok"
