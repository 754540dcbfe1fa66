#!/bin/bash
# Round-3 symmetric diagonal-class layout check: parity tests, then same-box A0 kbench (sym on /
# off), then the default bench line. Every GPU step under its own time limit.
set -euo pipefail
export TMPDIR=/tmp
TAG=${1:-r03_sym}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py ${TESTSEL:+-k "$TESTSEL"} > "$OUT/tests.log" 2>&1
echo "tests ok"
timeout -k 10 300 python3 -u tools/kbench.py --n 512 --levels 1 --ops 0,1,2 --reps 10 --configs 1024 --set sym_dia=1 > "$OUT/kb_sym1.jsonl" 2> "$OUT/kb_sym1.err"
timeout -k 10 300 python3 -u tools/kbench.py --n 512 --levels 1 --ops 0,1,2 --reps 10 --configs 1024 --set sym_dia=0 > "$OUT/kb_sym0.jsonl" 2> "$OUT/kb_sym0.err"
echo "kbench ok"
timeout -k 10 400 python3 -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.log"
echo "bench ok"
