#!/bin/bash
# HBM-side counters of ONE rank of an N-rank allreduce on the 1-GPU box:
# rank 0 runs under rocprofv3 --pmc, ranks 1..N-1 run unprofiled (profiling
# every rank inflated the counts 1.6-2.0x; one profiled process
# beside unprofiled ones counts its own requests exactly, profiles/r02/
# pmc_uc_ipc/).  One counter group per pass (MI355X_MICROARCH.md: FETCH_SIZE
# and WRITE_SIZE do not fit one TCC pass), then tools/pmc_traffic.py.
#   tools/pmc_rank0.sh <ring|mesh|mesh_pull|oneshot> <world> <bytes> [out-dir]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
algo=${1:-ring}; world=${2:-2}; bytes=${3:-1073741824}
out=${4:-gpurun_out/pmc_rank0_${algo}_n${world}}
rm -rf $out && mkdir -p $out
args="--gpus $world --algo $algo --bytes $bytes --steps 5 --warmup 1 --cpu-seconds 0 --no-check --autotune-reps 0 --extras-budget-s 0"
pass() {  # $1 = pass name, $2 = counters
    local port=$((20000 + RANDOM % 20000)) pids=() r
    for ((r = 1; r < world; ++r)); do
        RANK=$r LOCAL_RANK=$r WORLD_SIZE=$world LOCAL_WORLD_SIZE=$world MASTER_ADDR=127.0.0.1 MASTER_PORT=$port \
            timeout -s KILL 150 python3 bench.py $args > $out/$1_rank$r.log 2>&1 &
        pids+=($!)
    done
    RANK=0 LOCAL_RANK=0 WORLD_SIZE=$world LOCAL_WORLD_SIZE=$world MASTER_ADDR=127.0.0.1 MASTER_PORT=$port \
        timeout -s KILL 150 rocprofv3 --pmc $2 -d $out/$1 -o $1 --output-format csv -- python3 bench.py $args \
        > $out/$1_rank0.log 2>&1
    local rc=$?
    for p in "${pids[@]}"; do wait $p || rc=1; done
    if [ $rc -ne 0 ]; then tail -20 $out/$1_rank0.log; return 1; fi
    cp $(find $out/$1 -name "*counter_collection.csv" | head -1) $out/$1_counter_collection.csv
}
pass fetch FETCH_SIZE && pass write WRITE_SIZE && pass l2 "TCC_HIT_sum TCC_MISS_sum" || exit 1
kern="k_${algo}<"
[ "$algo" = mesh_pull ] && kern="k_mesh<"   # the pull mesh is k_mesh with a.pull set
python3 tools/pmc_traffic.py $out/fetch_counter_collection.csv $out/write_counter_collection.csv "$kern" \
    "${algo}_f32_n${world}_${bytes}" $out/traffic.json
