#!/bin/bash
# R1 (level-1 restriction at 512^3) experiments: request anatomy by size and
# L2 hit rate of R1 / P1 / A1, then same-box kbench of R1 over band scales and tile budgets.
set -euo pipefail
export TMPDIR=/tmp
TAG=${1:-r03_r1}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
KB="tools/kbench.py --n 512 --levels 2 --mats R1 --ops 0 --reps 10"
for bp in 25 50 100 200; do
  timeout -k 10 300 python3 -u $KB --configs 1024:1,2048:1,4096:1 --set band_pct_restrict=$bp >> "$OUT/kb_r1.jsonl" 2>> "$OUT/kb.err"
  echo "band $bp done"
done
timeout -k 10 300 python3 -u $KB --configs 1024:0 >> "$OUT/kb_r1.jsonl" 2>> "$OUT/kb.err"
echo "natural order done"
MATS=R1,P1,A1 timeout -k 10 700 bash tools/pmc_requests.sh $TAG/req
echo "requests done"
# the temporally blocked level-0 passes beside the separate sweeps: DRAM reads vs fabric reads
MATS=A0 LEVELS=1 OPS=1,2,4,5 timeout -k 10 400 bash tools/pmc_requests.sh $TAG/req_tb
echo "tb requests done"
