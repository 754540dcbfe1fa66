#!/bin/bash
# GPU-box steps of a round (run through gpurun), one launcher instead of per-experiment scripts:
#
#   gpurun -- 'bash tools/gpu_steps.sh TAG step [step ...]'
#
# steps (each GPU step under its own time limit; the first failure ends the script):
#   tests      the whole -m gpu suite (one process)
#   timed      the 512^3 timed-path tests + the parity file (faster than `tests`)
#   tp         the 512^3 timed-path tests alone (oracle parity at the benchmarked size, setup included)
#   p8         configs[2]: the 512^3 8-part test against the oracle's 8-part setup
#   bench      the default bench line (live PMC passes included) -> TAG/bench.json, bench.log
#   trace      rocprofv3 --kernel-trace --stats of bench.py (5 steps, no CPU leg, no PMC)
#   anatomy    counter anatomy of the level-0/1 row operators (A0 chain/SpMV, R0, P0, A1, R1, P1):
#              three --pmc passes (requests by size; DRAM / L2 hits / writes; SQ wave-cycle split)
#   part       tools/part_bench.py: one part (3 of 8 z-slabs of 512^3) timed alone (the T_8 model)
#   gen        the general-matrix path: elastic3d 80^3 natural / permuted, 512^3 with sym_vd=0 (bench lines)
#   cfgs       bench lines of configs[1] (128^3) and configs[3]'s operator (aniso 256^3) on one GPU
#   gentrace   rocprofv3 kernel stats of the same three runs
#   calib      counter calibration: tools/fetch_calib (known bytes per access width) and the row kernels
#              (kbench) under FETCH_SIZE / WRITE_SIZE / request-size / DRAM passes -> calib.json
#   chainpmc   SQ instruction / LDS counters of the chain and the fine SpMV (one pass)
#   r1band     R1 with its restriction band swept (tile order A/B)
#   kbench     tools/kbench.py --n 512 --levels 2 timings (KB_ARGS overrides)
#   world      the in-process device-world tests (tests/test_gpu_local_world.py)
#   stream / chain / sub   parity subsets: streamed sweeps; chain variants; -k "$SUB_K"
#   cab        tools/cycle_ab.py: same-box A/B of a cycle-level option (CAB_ARGS overrides)
# Output: gpurun_out/TAG/.
set -euo pipefail
export TMPDIR=/tmp
TAG=$1
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
PYT="python -u -m pytest -x -q --timeout 600 --timeout-method thread"
KBA=${KB_ARGS:-"--n 512 --levels 2 --mats A0,R0,P0,A1,R1,P1 --ops 0,1,2,3,5 --reps 3 --configs 1024"}
for step in "$@"; do
    case $step in
    tests)
        timeout -k 10 1000 $PYT tests -m gpu > "$OUT/tests.log" 2>&1
        ;;
    timed)
        timeout -k 10 800 $PYT tests/test_gpu_timed_path.py tests/test_gpu_parity.py tests/test_gpu_local_world.py -m gpu > "$OUT/timed.log" 2>&1
        ;;
    tp)
        timeout -k 10 900 $PYT -s --durations=10 tests/test_gpu_timed_path.py -m gpu > "$OUT/tp.log" 2>&1
        ;;
    p8)
        timeout -k 10 1100 $PYT -s --durations=5 tests/test_gpu_configs.py -k eight_parts -m gpu > "$OUT/p8.log" 2>&1
        ;;
    stream)
        timeout -k 10 300 $PYT tests/test_gpu_parity.py -k "sym_zm or symd_units" -m gpu > "$OUT/stream.log" 2>&1
        ;;
    chain)
        timeout -k 10 400 $PYT tests/test_gpu_parity.py -k "chain_variants or jacobi_residual_op or pipelined_cycles" -m gpu > "$OUT/chain.log" 2>&1
        ;;
    cab)
        timeout -k 10 500 python3 -u tools/cycle_ab.py ${CAB_ARGS:---ab chain_store_x=1,0} > "$OUT/cycle_ab.jsonl" 2> "$OUT/cycle_ab.err"
        ;;
    sub)
        timeout -k 10 400 $PYT tests/test_gpu_parity.py -k "${SUB_K:-prolongator}" -m gpu > "$OUT/sub.log" 2>&1
        ;;
    world)
        timeout -k 10 600 $PYT tests/test_gpu_local_world.py -m gpu > "$OUT/world.log" 2>&1
        ;;
    bench)
        timeout -k 10 700 python3 -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.log"
        ;;
    trace)
        timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o bench --output-format csv \
            -- python3 -u bench.py --steps 5 --cpu-baseline off --pmc off > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.log"
        ;;
    anatomy)
        timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
            -d "$OUT/an1" -o p --output-format csv -- python3 -u tools/kbench.py $KBA > "$OUT/an1.jsonl" 2> "$OUT/an1.err"
        echo "anatomy pass 1 done"
        timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum \
            -d "$OUT/an2" -o p --output-format csv -- python3 -u tools/kbench.py $KBA > "$OUT/an2.jsonl" 2> "$OUT/an2.err"
        echo "anatomy pass 2 done"
        timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
            SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS \
            -d "$OUT/an3" -o p --output-format csv -- python3 -u tools/kbench.py $KBA > "$OUT/an3.jsonl" 2> "$OUT/an3.err"
        echo "anatomy pass 3 done"
        timeout -s KILL 300 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum \
            -d "$OUT/an4" -o p --output-format csv -- python3 -u tools/kbench.py $KBA > "$OUT/an4.jsonl" 2> "$OUT/an4.err"
        echo "anatomy pass 4 done"
        python3 tools/pmc_anatomy.py "$OUT/an1" "$OUT/an2" "$OUT/an3" "$OUT/an4" > "$OUT/anatomy.json"
        ;;
    part)
        timeout -k 10 600 python3 -u tools/part_bench.py ${PART_ARGS:---n 512 --parts 8 --part 3} > "$OUT/part.json" 2> "$OUT/part.err"
        ;;
    gen)
        # the general-matrix path: the elastic3d stand-in for Flan_1565 in natural
        # and randomly renumbered order, and 512^3 without the row-class dictionary
        timeout -k 10 400 python3 -u bench.py --kind elastic3d --grid 80 --pcg-rtol 0 > "$OUT/gen_e80.json" 2> "$OUT/gen_e80.log"
        echo "gen e80 done"
        timeout -k 10 400 python3 -u bench.py --kind elastic3d --grid 80 --permute 1 --pcg-rtol 0 > "$OUT/gen_e80p.json" 2> "$OUT/gen_e80p.log"
        echo "gen e80p done"
        timeout -k 10 600 python3 -u bench.py --set sym_vd=0 --cpu-baseline off --pcg-rtol 0 > "$OUT/gen_svd0.json" 2> "$OUT/gen_svd0.log"
        echo "gen svd0 done"
        ;;
    cfgs)
        # the other BASELINE configs at one GPU (bench lines with their oracle parity and CPU baseline)
        timeout -k 10 300 python3 -u bench.py --grid 128 > "$OUT/cfg_p128.json" 2> "$OUT/cfg_p128.log"
        echo "cfg p128 done"
        timeout -k 10 500 python3 -u bench.py --kind aniso3d --grid 256 > "$OUT/cfg_a256.json" 2> "$OUT/cfg_a256.log"
        echo "cfg a256 done"
        ;;
    gentrace)
        for spec in "e80:--kind elastic3d --grid 80" "e80p:--kind elastic3d --grid 80 --permute 1" "svd0:--set sym_vd=0"; do
            tag=${spec%%:*}
            timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$tag" -o bench --output-format csv \
                -- python3 -u bench.py ${spec#*:} --steps 5 --samples 1 --cpu-baseline off --pmc off --pcg-rtol 0 \
                > "$OUT/prof_$tag.json" 2> "$OUT/prof_$tag.log"
            echo "gentrace $tag done"
        done
        ;;
    calib)
        # known-byte kernels under each counter pass, then the row kernels under
        # the same passes; tools/calib_analysis.py turns both into per-width factors and traffic
        test -x tools/fetch_calib || hipcc --offload-arch=gfx950 -O3 -o tools/fetch_calib tools/fetch_calib.hip
        i=0
        for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" \
                    "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_DRAM_32B_sum"; do
            i=$((i + 1))
            timeout -s KILL 120 rocprofv3 --pmc $pass -d "$OUT/cal$i" -o p --output-format csv -- tools/fetch_calib \
                > "$OUT/cal$i.jsonl" 2> "$OUT/cal$i.err"
            echo "calib pass $i done"
            timeout -s KILL 300 rocprofv3 --pmc $pass -d "$OUT/kb$i" -o p --output-format csv -- python3 -u tools/kbench.py $KBA \
                > "$OUT/kb$i.jsonl" 2> "$OUT/kb$i.err"
            echo "kbench pass $i done"
        done
        python3 tools/calib_analysis.py "$OUT" > "$OUT/calib.json"
        ;;
    chainpmc)
        # where the level-0 chain and the fine SpMV spend their issue slots: LDS vs VALU vs memory (one pass)
        timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
            SQ_WAIT_INST_LDS SQ_INSTS_LDS_LOAD_BANDWIDTH SQ_LDS_BANK_CONFLICT \
            -d "$OUT/chainpmc" -o p --output-format csv -- python3 -u tools/kbench.py --n 512 --levels 1 --mats A0 \
            --ops 0,5 --reps 3 --configs 1024 > "$OUT/chainpmc.jsonl" 2> "$OUT/chainpmc.err"
        python3 tools/pmc_anatomy.py "$OUT/chainpmc" > "$OUT/chainpmc.json"
        ;;
    r1band)
        # R1's tile order: the XCD band of the restriction tiles swept (read at upload), natural order beside it
        timeout -k 10 500 python3 -u tools/kbench.py --n 512 --levels 2 --mats R1 --ops 0 --reps 10 --configs 1024:1,1024:0 \
            --sweep band_pct_restrict=6,12,25,50,100,200 > "$OUT/r1band.jsonl" 2> "$OUT/r1band.err"
        ;;
    kbench)
        timeout -k 10 400 python3 -u tools/kbench.py $KBA > "$OUT/kbench.jsonl" 2> "$OUT/kbench.err"
        ;;
    *)
        echo "unknown step $step" >&2
        exit 2
        ;;
    esac
    echo "$step done"
done
