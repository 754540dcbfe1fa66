set -e
SUB_K="ell or absent_in_grid or vcycle" bash tools/gpu_steps.sh r05_m sub
KB_ARGS="--n 512 --levels 2 --mats A1 --ops 0,1,2 --reps 10 --configs 1024 --ab ell" bash tools/gpu_steps.sh r05_m kbench
