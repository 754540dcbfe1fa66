#!/bin/bash
# Jacobi with stored diagonals in the tile kernels (jacobi_diag 0/1 on the same upload, A1 / A2
# at 4096- and 2048-nonzero tiles), then the parity file with the new default.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03_jdiag}
mkdir -p "$OUT"
timeout -k 10 600 python3 -u tools/kbench.py --n 512 --levels 3 --mats A1,A2 --ops 1,2 --reps 20 --ab jacobi_diag \
    --configs 1024,2048,3072 > "$OUT/kb.jsonl" 2> "$OUT/kb.err"
echo "kbench ok"
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_parity.py -m gpu > "$OUT/parity.log" 2>&1
echo "parity ok"
