#!/bin/bash
# One parameterised runner for every GPU-box measurement (replaces the
# per-session gpu_r3*.sh scripts and the single-use A/B scripts of rounds
# 1-3, which git history keeps).  Steps run in order; the first failure ends
# the call (no GPU step after a failed one).  Output under gpurun_out/ (or
# $OUT); each GPU step under its own time limit.
#
#   tools/gpu_run.sh STEP [STEP ...]
#     suite                 the whole GPU suite as the driver runs it (gpu_suite.txt)
#     tests:<-k expr>       a subset of the GPU suite
#     smoke                 __graft_entry__.smoke()
#     bench1                N=1 line (bench_n1.json) + rocprofv3 --kernel-trace --stats of the same command
#     benchN:<n>[:args]     N-rank line, ranks sharing the GPU (bench_n<n>.txt); args: bench.py flags, ',' = ' '
#     pmc1                  N=1 k_reduce HBM counters (FETCH_SIZE, WRITE_SIZE passes) -> traffic.json
#     pmc0:<algo>:<n>:<B>   rank 0 of an n-rank allreduce under --pmc, the others unprofiled
#     ktrace0:<algo>:<n>:<B> rank 0 of an n-rank bench under --kernel-trace --stats, the others unprofiled
#     ab:<name>:<envA>:<envB>[:args]
#                           bench.py N=2 alternated A B A B with two env settings (',' separates
#                           VAR=value pairs; '-' = none), e.g. ab:tile:RDC_TILE_BYTES=256K:-
#     hostab:<name>:<envA>:<envB>:<bytes>:<calls>
#                           tools/host_path.py (host-buffer RdcAllreduce, n = 2) alternated A B A B
#     py:<name>:<env>:<script>:<args>
#                           one python process (a script that starts its own ranks), stdout to <name>.txt
#     run:<name>:<env>:<n>:<script>:<args>
#                           any script as n torch.distributed ranks with env (',' separates), stdout
#                           to <name>.txt, stderr to <name>.err
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname $0)/..}
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out}
mkdir -p $OUT
port=$((20000 + RANDOM % 20000))

envset() {  # "A=1,B=2" or "-" -> "A=1 B=2"
    [ "$1" = "-" ] && return 0
    echo "$1" | tr ',' ' '
}

run_bench_n() {  # n log args...
    local n=$1 log=$2
    shift 2
    port=$((port + 11))
    timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
        --master-port $port bench.py --gpus $n "$@" > $log 2> $log.err
}

for step in "$@"; do
    IFS=':' read -r kind a1 a2 a3 a4 a5 <<< "$step"
    echo "== $step"
    case $kind in
    suite)
        timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
            > $OUT/gpu_suite.txt 2>&1 || { tail -30 $OUT/gpu_suite.txt; exit 1; }
        tail -1 $OUT/gpu_suite.txt ;;
    tests)
        timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$a1" \
            > $OUT/gpu_tests.txt 2>&1 || { tail -30 $OUT/gpu_tests.txt; exit 1; }
        tail -1 $OUT/gpu_tests.txt ;;
    smoke)
        timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 \
            || { tail -20 $OUT/smoke.txt; exit 1; }
        tail -1 $OUT/smoke.txt ;;
    bench1)
        timeout -k 10 300 python3 bench.py > $OUT/bench_n1.json 2> $OUT/bench_n1.err \
            || { tail -20 $OUT/bench_n1.err; exit 1; }
        cat $OUT/bench_n1.json
        rm -rf $OUT/prof_n1
        timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_n1 -o bench_n1 --output-format csv -- \
            python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $OUT/prof_n1.log 2>&1 \
            || { tail -20 $OUT/prof_n1.log; exit 1; }
        cp $(find $OUT/prof_n1 -name "*kernel_stats.csv" | head -1) $OUT/bench_n1_kernel_stats.csv
        head -3 $OUT/bench_n1_kernel_stats.csv ;;
    benchN)
        tagged=$OUT/bench_n$a1$(echo "${a2:+_$a2}" | tr ',-' '__').txt   # one file per (n, args)
        run_bench_n $a1 $tagged $(echo "$a2" | tr ',' ' ') || { tail -20 $tagged.err; exit 1; }
        [ "$tagged" = "$OUT/bench_n$a1.txt" ] || cp $tagged $OUT/bench_n$a1.txt
        grep '^{' $tagged | head -c 400; echo ;;
    pmc1)
        P=$OUT/pmc_n1
        rm -rf $P && mkdir -p $P
        for c in FETCH_SIZE WRITE_SIZE; do
            timeout -s KILL 120 rocprofv3 --pmc $c -d $P/$c -o $c --output-format csv -- \
                python3 bench.py --steps 5 --warmup 1 --cpu-seconds 0 --no-check > $P/$c.log 2>&1 \
                || { tail -20 $P/$c.log; exit 1; }
            cp $(find $P/$c -name "*counter_collection.csv" | head -1) $P/${c}_counter_collection.csv
        done
        python3 tools/pmc_traffic.py $P/FETCH_SIZE_counter_collection.csv $P/WRITE_SIZE_counter_collection.csv \
            "k_reduce<2, float" reduce_sum_f32_1073741824 $P/traffic.json ;;
    pmc0)
        bash tools/pmc_rank0.sh $a1 $a2 $a3 $OUT/pmc_rank0_${a1}_n${a2} || exit 1 ;;
    ktrace0)
        bash tools/ktrace_rank0.sh $a1 $a2 $a3 $OUT/ktrace_rank0_${a1}_n${a2} || exit 1 ;;
    ab)
        extra=$(echo "${a4:-}" | tr ',' ' ')
        for v in A B A B; do
            e=$([ $v = A ] && envset "$a2" || envset "$a3")
            port=$((port + 11))
            env $e timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
                --master-addr 127.0.0.1 --master-port $port bench.py --gpus 2 --steps 30 --extra-steps 0 \
                --rccl-steps 0 --cpu-seconds 0 --no-check --autotune-reps 0 --extras-budget-s 30 $extra \
                > $OUT/ab_${a1}_$v.$port.txt 2>&1 || { tail -20 $OUT/ab_${a1}_$v.$port.txt; exit 1; }
            echo "$v $(grep '^{' $OUT/ab_${a1}_$v.$port.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], (d.get("ring_schedule") or {}).get("ms_per_step"))')"
        done ;;
    hostab)
        for v in A B A B; do
            e=$([ $v = A ] && envset "$a2" || envset "$a3")
            port=$((port + 11))
            env $e timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
                --master-addr 127.0.0.1 --master-port $port tools/host_path.py $a4 $a5 \
                > $OUT/hostab_${a1}_$v.$port.txt 2>&1 || { tail -20 $OUT/hostab_${a1}_$v.$port.txt; exit 1; }
            echo "$v $(grep -o '"ms_per_call": [0-9.]*' $OUT/hostab_${a1}_$v.$port.txt | head -1)"
        done ;;
    py)
        env $(envset "$a2") timeout -k 10 300 python3 $a3 $(echo "$a4" | tr ',' ' ') \
            > $OUT/$a1.txt 2> $OUT/$a1.err || { tail -20 $OUT/$a1.err; exit 1; }
        tail -c 600 $OUT/$a1.txt; echo ;;
    run)
        port=$((port + 11))
        env $(envset "$a2") timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $a3 \
            --master-addr 127.0.0.1 --master-port $port $a4 $(echo "$a5" | tr ',' ' ') \
            > $OUT/$a1.txt 2> $OUT/$a1.err || { tail -20 $OUT/$a1.err; exit 1; }
        tail -c 600 $OUT/$a1.txt; echo ;;
    *)
        echo "unknown step $step"; exit 2 ;;
    esac
done
