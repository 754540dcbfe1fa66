#!/bin/bash
# Final check of the round-3 tree: parity + full-size GPU tests, then the profile round (bench
# line, kernel trace, PMC traffic of the chain kernel for the current kernels.hip).
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03_full4
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu > "$OUT/tests_a.log" 2>&1
echo "parity/fullsize ok"
bash tools/profile_round.sh r03_final4
