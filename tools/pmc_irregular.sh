#!/bin/bash
# Counter anatomy of the irregular-numbering path (VERDICT r2 "profile the irregular path"):
# per level-0/1 row operation of a randomly renumbered problem — times (HIP events), HBM
# traffic (FETCH_SIZE / WRITE_SIZE, MI355X_MICROARCH.md §HBM) and TCC read requests by size,
# DRAM-bound requests and L2 hit rate (tools/pmc_requests.py). One counter group per pass,
# each pass a separate run under its own time limit.
#
#   gpurun -- 'bash tools/pmc_irregular.sh r03_irr "--kind elastic3d --n 80 --permute 1"'
set -euo pipefail
export TMPDIR=/tmp
TAG=${1:-irr}
PROB=${2:---kind elastic3d --n 80 --permute 1}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
KB="tools/kbench.py $PROB --levels 2 --ops 0,1,2,3 --reps 3 --configs 1024 ${KBEXTRA:-}"
timeout -k 10 300 python3 -u $KB > "$OUT/times.jsonl" 2> "$OUT/times.err"
echo "times done"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o fetch --output-format csv \
    -- python3 -u $KB > "$OUT/pmc_fetch.jsonl" 2> "$OUT/pmc_fetch.err"
echo "fetch pass done"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o write --output-format csv \
    -- python3 -u $KB > "$OUT/pmc_write.jsonl" 2> "$OUT/pmc_write.err"
echo "write pass done"
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
    -d "$OUT/pass1" -o p1 --output-format csv -- python3 -u $KB > "$OUT/pass1.jsonl" 2> "$OUT/pass1.err"
echo "request pass 1 done"
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum \
    -d "$OUT/pass2" -o p2 --output-format csv -- python3 -u $KB > "$OUT/pass2.jsonl" 2> "$OUT/pass2.err"
echo "request pass 2 done"
python3 tools/pmc_traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" --kernel "k_rows" --workload "${WKEY:-irregular}" > "$OUT/traffic_all.json"
python3 tools/pmc_requests.py "$OUT/pass1" "$OUT/pass2" > "$OUT/requests.json"
echo "records in $OUT"
