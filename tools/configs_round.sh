#!/bin/bash
# One-GPU bench lines of the other BASELINE.json configs (parity configs, not the metric's):
# 128^3 Poisson, anisotropic 256^3, elastic3d 80^3 (the Flan_1565 stand-in), each with the
# default layout and with x staging off (A/B). Run on the MI355X box (gpurun).
#
#   gpurun -- 'bash tools/configs_round.sh r01_v10'
set -euo pipefail
export TMPDIR=/tmp
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
run() {  # name, bench args...
    local name=$1; shift
    timeout -k 10 240 python3 -u bench.py --cpu-baseline off --steps 50 "$@" > "$OUT/cfg_$name.json" 2> "$OUT/cfg_$name.log"
    echo "$name: $(python3 -c "import json,sys; print(json.loads(open('$OUT/cfg_$name.json').read().strip().splitlines()[-1])['value'])")"
}
run p128 --grid 128
run p128_xs0 --grid 128 --set x_stage=0
run a256 --kind aniso3d --grid 256
run a256_xs0 --kind aniso3d --grid 256 --set x_stage=0
run e80 --kind elastic3d --grid 80
run e80_xs0 --kind elastic3d --grid 80 --set x_stage=0
# the Flan_1565 proxy: elastic3d renumbered at random (no column dictionary, no banded order)
run e80_perm --kind elastic3d --grid 80 --permute 1
run p128_perm --grid 128 --permute 1
# the graph partitioner on the renumbered elastic operator
run e80_perm_rcm --kind elastic3d --grid 80 --permute 1 --rcm
