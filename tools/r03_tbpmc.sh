#!/bin/bash
# HBM traffic of the temporally blocked passes (k_sym_tb<2>, <3>) beside the separate sweeps:
# two PMC passes (FETCH_SIZE, WRITE_SIZE; MI355X_MICROARCH.md §HBM) and an L2 hit-rate pass over
# tools/kbench.py ops 1, 2, 4, 5 on the 512^3 fine operator.
set -euo pipefail
export TMPDIR=/tmp
TAG=${1:-r03_tbpmc}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
KB="tools/kbench.py --n 512 --levels 1 --ops 1,2,4,5 --reps 3 --configs 1024"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o fetch --output-format csv -- python3 -u $KB > "$OUT/fetch.jsonl" 2> "$OUT/fetch.err"
echo "fetch done"
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o write --output-format csv -- python3 -u $KB > "$OUT/write.jsonl" 2> "$OUT/write.err"
echo "write done"
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$OUT/pmc_hit" -o hit --output-format csv -- python3 -u $KB > "$OUT/hit.jsonl" 2> "$OUT/hit.err"
echo "hit done"
