#!/bin/bash
# The other BASELINE.json configs with the round-3 defaults (one bench line each, no CPU baseline)
# and the 8-rank 512^3 rehearsal through the host transport. Each step has its own time limit.
set -euo pipefail
export TMPDIR=/tmp
TAG=${1:-r03_cfg}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
B="python3 -u bench.py --cpu-baseline off"
timeout -k 10 200 $B --grid 128 --steps 50 > "$OUT/p128.json" 2> "$OUT/p128.log"; echo "p128 done"
timeout -k 10 300 $B --kind aniso3d --grid 256 > "$OUT/a256.json" 2> "$OUT/a256.log"; echo "a256 done"
timeout -k 10 200 $B --kind elastic3d --grid 80 --steps 50 > "$OUT/e80.json" 2> "$OUT/e80.log"; echo "e80 done"
timeout -k 10 200 $B --kind elastic3d --grid 80 --steps 50 --permute 7 > "$OUT/e80_perm.json" 2> "$OUT/e80_perm.log"; echo "e80 perm done"
timeout -k 10 600 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 8 --steps 3 --warmup 1 --transport host --cpu-baseline off \
    > "$OUT/p512_n8_host.json" 2> "$OUT/p512_n8_host.log"; echo "n8 host done"
