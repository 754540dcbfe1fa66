set -e
mkdir -p gpurun_out/r05_l
timeout -k 10 300 python3 -u tools/kbench.py --n 512 --levels 1 --ops 4,5 --reps 10 --configs 1024 --ab tb_xfast > gpurun_out/r05_l/kb_tb.jsonl 2> gpurun_out/r05_l/kb_tb.err
echo tb done
timeout -k 10 300 python3 -u tools/kbench.py --n 512 --levels 1 --ops 0,1,2 --reps 10 --configs 1024 --ab zm_xfast > gpurun_out/r05_l/kb_zm.jsonl 2> gpurun_out/r05_l/kb_zm.err
echo zm done
