#!/bin/bash
# HBM traffic (rocprofv3 FETCH_SIZE / WRITE_SIZE passes, MI355X_MICROARCH.md §HBM) and times of
# every level-0 / level-1 row operation at 512^3, for the per-kernel table in DESIGN.md. Run on
# the MI355X box (gpurun); one counter per pass, each pass under its own time limit.
#
#   gpurun -- 'bash tools/pmc_levels.sh r02_levels'
set -euo pipefail
export TMPDIR=/tmp
TAG=${1:-levels}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
KB="tools/kbench.py --n 512 --levels 2 --ops 0,1,2,3 --reps 3 --configs 1024"
timeout -k 10 400 python3 -u $KB > "$OUT/times.jsonl" 2> "$OUT/times.err"
echo "times done"
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o fetch --output-format csv \
    -- python3 -u $KB > "$OUT/pmc_fetch.jsonl" 2> "$OUT/pmc_fetch.err"
echo "fetch pass done"
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o write --output-format csv \
    -- python3 -u $KB > "$OUT/pmc_write.jsonl" 2> "$OUT/pmc_write.err"
echo "write pass done"
python3 tools/pmc_traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" --kernel "k_rows" > "$OUT/traffic_all.json"
echo "traffic in $OUT/traffic_all.json"
