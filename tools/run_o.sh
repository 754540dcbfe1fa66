set -e
SUB_K="ell or vcycle or restriction or prolongat" bash tools/gpu_steps.sh r05_o sub
KB_ARGS="--n 512 --levels 2 --mats R0,R1 --ops 0 --reps 10 --configs 1024" bash tools/gpu_steps.sh r05_o kbench
timeout -k 10 400 python3 -u bench.py --cpu-baseline off --pmc off --pcg-rtol 0 > gpurun_out/r05_o/b.json 2> gpurun_out/r05_o/b.log
