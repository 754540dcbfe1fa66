#!/bin/bash
# Memory-request anatomy of the level-0/1 row kernels (is R0's PMC excess real?):
# two rocprofv3 --pmc passes (separate runs, <= 4 TCC counters each) over tools/kbench.py at
# 512^3 — read requests by size (32/64/128 B) and total, then DRAM-bound reads, L2 hits /
# misses and write requests. tools/pmc_requests.py turns them into bytes per launch.
#
#   gpurun -- 'bash tools/pmc_requests.sh r02_req'
set -euo pipefail
export TMPDIR=/tmp
TAG=${1:-r02_req}
MATS=${MATS:-A0,R0,P0,A1}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
KB="tools/kbench.py --n 512 --levels ${LEVELS:-2} --mats $MATS --ops ${OPS:-0,2,3} --reps 2 --configs 1024"
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
    -d "$OUT/pass1" -o p1 --output-format csv -- python3 -u $KB > "$OUT/pass1.jsonl" 2> "$OUT/pass1.err"
echo "pass 1 done"
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum \
    -d "$OUT/pass2" -o p2 --output-format csv -- python3 -u $KB > "$OUT/pass2.jsonl" 2> "$OUT/pass2.err"
echo "pass 2 done"
python3 tools/pmc_requests.py "$OUT/pass1" "$OUT/pass2" > "$OUT/requests.json"
echo "requests.json written"
