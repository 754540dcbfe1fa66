#!/bin/bash
# Fused level-0 Jacobi -> residual (jr_fuse): parity tests, then same-box bench lines with the
# fusion on and off. Each GPU step under its own time limit; the first failure ends the script.
set -euo pipefail
export TMPDIR=/tmp
TAG=${1:-r03_jr}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
rc=0
timeout -k 10 400 python -u -m pytest -v --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k "jacobi_residual_op or fused_jacobi or pipelined_cycles" > "$OUT/tests_fused.log" 2>&1 || rc=$?
echo "fused tests rc=$rc"
# a failed parity test still leaves the speed of the path worth measuring; a crash / hang does not
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 -u bench.py --cpu-baseline off --pcg-rtol 0 --set jr_fuse=1 > "$OUT/bench_jr1.json" 2> "$OUT/bench_jr1.log"
echo "bench jr1 ok"
timeout -k 10 300 python3 -u bench.py --cpu-baseline off --pcg-rtol 0 --set jr_fuse=0 > "$OUT/bench_jr0.json" 2> "$OUT/bench_jr0.log"
echo "bench jr0 ok"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_configs.py -k "not eight_parts" > "$OUT/tests.log" 2>&1
echo "tests ok"
