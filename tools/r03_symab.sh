#!/bin/bash
# Same-box A/B of the symmetric layout's kernels at 512^3 (A0 SpMV / residual / Jacobi):
# rows per lane 1 / 2, XCD-banded / natural block order, tile kernel for reference; then
# PMC traffic (FETCH_SIZE / WRITE_SIZE) and read-request anatomy of the default.
set -euo pipefail
export TMPDIR=/tmp
TAG=${1:-r03_symab}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "sym" > "$OUT/tests.log" 2>&1
echo "tests ok"
KB="tools/kbench.py --n 512 --levels 1 --ops 0,1,2 --reps 10"
for cfg in "--configs 1024:1 --set sym_rows=1" "--configs 1024:1 --set sym_rows=2" "--configs 1024:0 --set sym_rows=1" "--configs 1024:0 --set sym_rows=2" "--configs 1024:1 --set sym_dia=0"; do
    timeout -k 10 300 python3 -u $KB $cfg >> "$OUT/kb.jsonl" 2>> "$OUT/kb.err"
done
echo "kbench ok"
KP="tools/kbench.py --n 512 --levels 1 --ops 0,2 --reps 3 --configs 1024:1 ${PMCSET:-}"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o fetch --output-format csv -- python3 -u $KP > "$OUT/pmc_fetch.jsonl" 2> "$OUT/pmc_fetch.err"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o write --output-format csv -- python3 -u $KP > "$OUT/pmc_write.jsonl" 2> "$OUT/pmc_write.err"
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
    -d "$OUT/pass1" -o p1 --output-format csv -- python3 -u $KP > "$OUT/pass1.jsonl" 2> "$OUT/pass1.err"
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum \
    -d "$OUT/pass2" -o p2 --output-format csv -- python3 -u $KP > "$OUT/pass2.jsonl" 2> "$OUT/pass2.err"
echo "pmc ok"
python3 tools/pmc_traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" --kernel "k_rows_sym" > "$OUT/traffic.json"
python3 tools/pmc_requests.py "$OUT/pass1" "$OUT/pass2" > "$OUT/requests.json"
echo "records ok"
