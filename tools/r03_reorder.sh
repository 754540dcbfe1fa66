set -o pipefail
mkdir -p gpurun_out/r03_reorder
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "upload_perm or reorder or permuted or vcycle_bit_exact" > gpurun_out/r03_reorder/tests.log 2>&1 && echo tests ok &&
timeout -k 10 300 python3 -u bench.py --kind elastic3d --grid 80 --permute 1 --cpu-baseline off --steps 50 > gpurun_out/r03_reorder/e80_perm.json 2> gpurun_out/r03_reorder/e80_perm.log && echo e80 perm ok &&
timeout -k 10 300 python3 -u bench.py --kind elastic3d --grid 80 --permute 1 --reorder off --cpu-baseline off --steps 50 > gpurun_out/r03_reorder/e80_perm_off.json 2> gpurun_out/r03_reorder/e80_perm_off.log && echo e80 perm off ok &&
timeout -k 10 300 python3 -u bench.py --grid 128 --permute 1 --cpu-baseline off --steps 50 > gpurun_out/r03_reorder/p128_perm.json 2> gpurun_out/r03_reorder/p128_perm.log && echo p128 perm ok &&
timeout -k 10 300 python3 -u bench.py --kind elastic3d --grid 80 --cpu-baseline off --steps 50 > gpurun_out/r03_reorder/e80.json 2> gpurun_out/r03_reorder/e80.log && echo e80 ok
