#!/bin/bash
# Profiles of a round, run on the MI355X box (gpurun): the default bench line (with the CPU
# baseline), a rocprofv3 kernel trace + stats of bench.py, and the two PMC passes
# (FETCH_SIZE, WRITE_SIZE; separate runs, MI355X_MICROARCH.md §HBM) of the level-0 SpMV and
# Jacobi kernels through tools/kbench.py. Every GPU step has its own time limit; the first
# failure ends the script (set -e).
#
#   gpurun -- 'bash tools/profile_round.sh r01_v9'
set -euo pipefail
export TMPDIR=/tmp
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python3 -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.log"
echo "bench done"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o bench --output-format csv \
    -- python3 -u bench.py --steps 5 --cpu-baseline off > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.log"
echo "kernel trace done"
KB="tools/kbench.py --n 512 --levels 1 --ops 0,2,5 --reps 3 --configs 1024"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o fetch --output-format csv \
    -- python3 -u $KB > "$OUT/pmc_fetch.jsonl" 2> "$OUT/pmc_fetch.err"
echo "fetch pass done"
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o write --output-format csv \
    -- python3 -u $KB > "$OUT/pmc_write.jsonl" 2> "$OUT/pmc_write.err"
echo "write pass done"
mkdir -p "$OUT/pmc"
# the level-0 kernel of the default layout: the symmetric diagonal-class kernel (r03; the
# tile-major one before)
K=${PMCKERNEL:-k_rows_sym2}
python3 tools/pmc_traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" --kernel "$K<2" > "$OUT/pmc/traffic_jacobi.json"
python3 tools/pmc_traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" --kernel "$K<0" > "$OUT/pmc/traffic_spmv.json"
# the pipelined cycles' level-0 chain (k_sym_tb<3>, the timed region's dominant kernel)
python3 tools/pmc_traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" --kernel "k_sym_tb<3>" > "$OUT/pmc/traffic_chain.json"
echo "traffic records in $OUT/pmc (copy to profiles/pmc/ to let bench.py report them)"
