#!/bin/bash
# Same-box A/B of the 512^3 restriction R0's group processing order (Options::ell_yblock, an
# upload-time option: one kbench per value). Output: gpurun_out/${1:-r05_r0}/yb<N>.jsonl
set -euo pipefail
O=gpurun_out/${1:-r05_r0}
mkdir -p $O
KB="python3 -u tools/kbench.py --n 512 --levels 2 --mats R0 --ops 0 --reps 5 --configs 1024"
for YB in ${YBS:-0 16 32 64}; do
  timeout -k 10 300 $KB --set ell_yblock=$YB > $O/yb$YB.jsonl 2> $O/yb$YB.err
  echo yb$YB
done
