#!/bin/bash
# Rehearsal of bench.py's N>1 path on ONE GPU: N ranks (torch.distributed.run, gloo rendezvous)
# share the card through the host debug transport (RCCL refuses two ranks on one device), so
# the 8-slab partition, distributed setup, agglomeration and the JSON line are exercised end
# to end before the driver's multi-GPU run. Not a performance mode.
#
#   gpurun -- 'bash tools/multirank_rehearsal.sh r01_v11'
#   gpurun -- 'GRID=512 NS=8 bash tools/multirank_rehearsal.sh r02_512'   # the metric's size
set -euo pipefail
export TMPDIR=/tmp
TAG=${1:-r01}
GRID=${GRID:-128}
NS=${NS:-"2 4 8"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for N in $NS; do
    timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
        --master-addr 127.0.0.1 --master-port $((29500 + N)) bench.py --gpus $N --steps 5 --warmup 2 \
        --samples 2 --grid $GRID --transport host > "$OUT/rehearsal_n${N}_g$GRID.json" 2> "$OUT/rehearsal_n${N}_g$GRID.log"
    echo "N=$N: $(tail -1 "$OUT/rehearsal_n${N}_g$GRID.json" | cut -c1-160)"
done
