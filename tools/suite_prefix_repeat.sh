#!/bin/bash
# The driver's -m gpu suite up to and including the round-4 red test
# (test_gpu_allreduce.py through test_group_graph_capture_replay), run K
# times in separate processes; an assertion failure goes on, anything else
# (timeout, abort, fault) ends the call.
set -o pipefail
K=${1:-8}
mkdir -p gpurun_out/prefix
for i in $(seq 1 $K); do
  timeout -k 10 240 python3 -u -m pytest tests/test_gpu_allreduce.py -m gpu -x -q --timeout 120 --timeout-method thread \
     -k "group3_all_types or tree_order_all_types or tree_multi_piece or group_multi_piece or tuned_mesh or tune_rejects or repeated_calls or far_past or graph_capture" \
     -p no:cacheprovider > gpurun_out/prefix/run$i.txt 2>&1
  rc=$?
  echo "[$i] rc=$rc $(tail -1 gpurun_out/prefix/run$i.txt)"
  [ $rc -le 1 ] || exit $rc
done
