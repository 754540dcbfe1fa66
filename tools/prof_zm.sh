set -e
export TMPDIR=/tmp
O=gpurun_out/r05_e
mkdir -p $O
KB="python3 -u tools/kbench.py --n 512 --levels 1 --ops 0 --reps 5 --configs 1024"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- $KB > $O/kt.jsonl 2> $O/kt.err
echo "trace done"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $O/p1 -o p --output-format csv -- $KB > $O/p1.jsonl 2> $O/p1.err
echo "pmc1 done"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM -d $O/p2 -o p --output-format csv -- $KB > $O/p2.jsonl 2> $O/p2.err
echo "pmc2 done"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD -d $O/p3 -o p --output-format csv -- tools/stencil_ceiling 512 3 > $O/p3.jsonl 2> $O/p3.err
echo "pmc3 done"
