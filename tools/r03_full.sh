#!/bin/bash
# The whole GPU suite (as the driver runs it at round end) in three time-limited steps, then
# smoke(). The first failure ends the script.
set -euo pipefail
export TMPDIR=/tmp
TAG=${1:-r03_full}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_configs.py -m gpu > "$OUT/tests_a.log" 2>&1
echo "parity/fullsize/configs ok"
timeout -k 10 900 python -u -m pytest -x -q --timeout 700 --timeout-method thread tests -m gpu --deselect tests/test_gpu_parity.py --deselect tests/test_gpu_fullsize.py --deselect tests/test_gpu_configs.py > "$OUT/tests_b.log" 2>&1
echo "other gpu tests ok"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
echo "smoke ok"
