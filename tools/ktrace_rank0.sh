#!/bin/bash
# Kernel-trace summary of ONE rank of an N-rank bench on the 1-GPU box: rank 0
# runs under rocprofv3 --kernel-trace --stats, ranks 1..N-1 unprofiled (as
# tools/pmc_rank0.sh does for counters).  The per-kernel average of rank 0's
# collective should agree with the bench line's HIP-event kernel_avg_ms.
#   tools/ktrace_rank0.sh <algo|auto> <world> <bytes> [out-dir]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
algo=${1:-auto}; world=${2:-2}; bytes=${3:-1073741824}
out=${4:-gpurun_out/ktrace_rank0_${algo}_n${world}}
rm -rf $out && mkdir -p $out
args="--gpus $world --algo $algo --bytes $bytes --steps 20 --warmup 5 --cpu-seconds 0 --no-check --extras-budget-s 0"
port=$((20000 + RANDOM % 20000))
pids=()
for ((r = 1; r < world; ++r)); do
    RANK=$r LOCAL_RANK=$r WORLD_SIZE=$world LOCAL_WORLD_SIZE=$world MASTER_ADDR=127.0.0.1 MASTER_PORT=$port \
        timeout -s KILL 240 python3 bench.py $args > $out/rank$r.log 2>&1 &
    pids+=($!)
done
RANK=0 LOCAL_RANK=0 WORLD_SIZE=$world LOCAL_WORLD_SIZE=$world MASTER_ADDR=127.0.0.1 MASTER_PORT=$port \
    timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $out/prof -o ktrace --output-format csv -- \
    python3 bench.py $args > $out/rank0.log 2>&1
rc=$?
for p in "${pids[@]}"; do wait $p || rc=1; done
if [ $rc -ne 0 ]; then tail -20 $out/rank0.log; exit 1; fi
cp $(find $out/prof -name "*kernel_stats.csv" | head -1) $out/kernel_stats.csv
head -4 $out/kernel_stats.csv
grep '^{' $out/rank0.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("bench line:", d["ms_per_step"], "ms/step, kernel_avg_ms", r["kernel_avg_ms"], r["kernel"])'
