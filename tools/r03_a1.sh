#!/bin/bash
# Level-1 operator A1 at 512^3 (a third of the V-cycle): its row kernels under the layout
# variants — default, value dictionaries, no tile-major — for the residual and Jacobi sweeps.
set -euo pipefail
export TMPDIR=/tmp
TAG=${1:-r03_a1}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python3 -u tools/kbench.py --n 512 --levels 2 --mats A1,P0,R0 --ops 0,1,2,3 --reps 10 \
    --configs 1024:1,1024:1:1:1,1024:1:1:1:1:1:1:0,2048:1:1:1,4096:1:1:1 > "$OUT/kb_a1.jsonl" 2> "$OUT/kb.err"
echo "kbench done"
