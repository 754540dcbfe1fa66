#!/bin/bash
# A1 / A2 / R1 tile budgets with 8-bit value dictionaries (round-3 default layout): 4096 (the
# long-row default), 2048, 1024, and 4096 again (drift). Same box, same upload path.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03_a1tile}
mkdir -p "$OUT"
timeout -k 10 600 python3 -u tools/kbench.py --n 512 --levels 3 --mats A1,A2,R1 --ops 1,2,0 --reps 20 \
    --configs 1024,2048,1024:1:1:1:0,1024 > "$OUT/kb.jsonl" 2> "$OUT/kb.err"
echo "kbench ok"
