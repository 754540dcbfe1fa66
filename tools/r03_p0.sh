#!/bin/bash
# P0 with 8-bit row lengths beside its 4-bit value dictionaries (row_len8 on / off, same box),
# the parity file, and the default bench line with the upload phases traced.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03_p0}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_parity.py -m gpu > "$OUT/parity.log" 2>&1
echo "parity ok"
timeout -k 10 400 python3 -u tools/kbench.py --n 512 --levels 2 --mats P0 --ops 3 --reps 20 \
    --configs 1024:1:1:1:1:1,1024:1:1:1:1:0,1024:1:1:1:1:1,1024:1:1:1:1:0 > "$OUT/kb.jsonl" 2> "$OUT/kb.err"
echo "kbench ok"
PAMG_TRACE_UPLOAD=1 timeout -k 10 400 python3 -u bench.py --cpu-baseline off > "$OUT/bench.json" 2> "$OUT/bench.log"
echo "bench ok"
