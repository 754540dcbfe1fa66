#!/bin/bash
# Temporally blocked level-0 sweeps (k_sym_tb): parity tests, the kernel micro-benchmark
# (ops 4 / 5 beside the separate sweeps) and the default bench line. Each GPU step has its own
# time limit; the first failure ends the script.
set -euo pipefail
export TMPDIR=/tmp
TAG=${1:-r03_tb}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k "jacobi_residual_op or fused_jacobi or pipelined_cycles" > "$OUT/tests_fused.log" 2>&1
echo "fused tests ok"
timeout -k 10 300 python3 -u tools/kbench.py --n 512 --levels 1 --ops 1,2,4,5 --reps 10 --configs 1024 > "$OUT/kbench.jsonl" 2> "$OUT/kbench.err"
echo "kbench ok"
timeout -k 10 300 python3 -u bench.py --cpu-baseline off --pcg-rtol 0 > "$OUT/bench.json" 2> "$OUT/bench.log"
echo "bench ok"
