#!/bin/bash
# Round 3: unit-table ring + service/channel/tune-file changes under the GPU
# suite's coalesced / service / mixed tests; data sensitivity of the timing;
# an N=2 rehearsal (cfg5 through the tuned schedule).  Stops at the first failure.
set -e -o pipefail
out=gpurun_out/r3b
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_allreduce.py tests/test_gpu_mixed.py \
  -k "coalesced or order_violation or host_small_service or named or tune or cfg5 or mixed or subset or full_grid" \
  > $out/tests.log 2>&1
echo tests-ok
for a in 1 2; do
  ALGO=$a timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 2962$a tools/data_sensitivity.py 1024 > $out/data_sensitivity_n2_algo$a.log 2>&1
done
echo sens-ok
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus 2 > $out/bench_n2.log 2>&1
echo bench-ok
