set -e
SUB_K="absent_in_grid or sym_zm or jacobi_residual_op or pipelined_cycles or chain_two or aggregate_order" bash tools/gpu_steps.sh r05_k sub
KB_ARGS="--n 512 --levels 1 --ops 0,1,2,4,5 --reps 10 --configs 1024" bash tools/gpu_steps.sh r05_k kbench
timeout -k 10 400 python3 -u bench.py --cpu-baseline off --pmc off --pcg-rtol 0 > gpurun_out/r05_k/b_auto.json 2> gpurun_out/r05_k/b_auto.log
echo auto done
timeout -k 10 400 python3 -u bench.py --cpu-baseline off --pmc off --pcg-rtol 0 --reorder agg > gpurun_out/r05_k/b_agg.json 2> gpurun_out/r05_k/b_agg.log
echo agg done
