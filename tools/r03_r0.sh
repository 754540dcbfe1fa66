#!/bin/bash
# R0 / P0 (512^3) under the value-dictionary variants: 4-bit in descriptor tiles (value_dict 1)
# vs 8-bit in tile-major slots (value_dict 2; tile_major 2 lets P0 take slots too).
set -euo pipefail
export TMPDIR=/tmp
TAG=${1:-r03_r0}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
KB="python3 -u tools/kbench.py --n 512 --levels 2 --mats R0,P0 --ops 0,3 --reps 10"
timeout -k 10 400 $KB --configs 1024:1:1:1,1024:1:1:2,1024:1:1:2:1:1:1:2,2048:1:1:2,4096:1:1:2 > "$OUT/kb.jsonl" 2> "$OUT/kb.err"; echo "kb done"
