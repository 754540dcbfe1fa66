#!/bin/bash
# Counter anatomy of the level-0 z-marching kernels (k_sym_zm one-sweep ops, k_sym_zc blocked
# passes) on the 512^3 fine operator: kernel trace + SQ instruction / wait split + LDS + HBM
# traffic, one rocprofv3 pass per counter group. Output: gpurun_out/$1/.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-zm}
mkdir -p $O
KB="python3 -u tools/kbench.py ${KB_ARGS:---n 512 --levels 1 --ops ${OPS:-0,2,4,5} --reps 3 --configs 1024}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- $KB > $O/kt.jsonl 2> $O/kt.err
echo "trace done"
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
         "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_MISC" \
         "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --pmc $C -d $O/p$i -o p --output-format csv -- $KB > $O/p$i.jsonl 2> $O/p$i.err
    echo "pmc $i done"
done
