#!/bin/bash
# tools/rotate_litmus as P concurrent IPC pairs (owner + writer process each),
# every process holding Q hardware queues (GPU_MAX_HW_QUEUES=Q plus Q-1 extra
# streams): with 2P x Q queues beyond the GPU's queue slots the scheduler
# time-slices.  Each process under its own time limit.
set -o pipefail
P=${1:-5}; Q=${2:-3}; MEM=${3:-1}; LOAD=${4:-1}; IT=${5:-20000}
O=gpurun_out/rotate_os
mkdir -p $O
pids=()
for p in $(seq 1 $P); do
  d=$(mktemp -d)
  GPU_MAX_HW_QUEUES=$Q LITMUS_EXTRA_STREAMS=$((Q-1)) timeout -k 10 150 tools/rotate_litmus owner $d $MEM $LOAD $IT > $O/owner$p.json 2>&1 &
  pids+=($!)
  GPU_MAX_HW_QUEUES=$Q LITMUS_EXTRA_STREAMS=$((Q-1)) timeout -k 10 150 tools/rotate_litmus writer $d > $O/writer$p.txt 2>&1 &
  pids+=($!)
done
rc=0
for pid in "${pids[@]}"; do wait $pid || rc=$?; done
cat $O/owner*.json
exit $rc
