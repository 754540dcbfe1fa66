#!/bin/bash
# R0 / P0 under the banded XCD order's band scale (band_pct_restrict 25 / 50 (default) / 100 /
# 200) and the natural order, in the round-3 default layout, one box.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03_r0band}
mkdir -p "$OUT"
for bp in 50 25 100 200; do
  timeout -k 10 300 python3 -u tools/kbench.py --n 512 --levels 2 --mats R0 --ops 0 --reps 20 \
      --set band_pct_restrict=$bp --configs 1024,1024:0 >> "$OUT/kb.jsonl" 2>> "$OUT/kb.err"
  echo "band $bp ok"
done
