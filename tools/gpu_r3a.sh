#!/bin/bash
# Round-3 GPU check: new parity / Python-surface / order / autotune / custom-reducer tests,
# an N=2 bench rehearsal, and the custom-reducer A/B.  Stops at the first failing step.
set -e -o pipefail
out=gpurun_out/r3a
mkdir -p $out
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_entrypoints.py tests/test_gpu_allreduce.py \
  -k "python_surface or bench or order_violation or autotune or buffer_surface" > $out/tests.log 2>&1
echo tests-ok
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus 2 > $out/bench_n2.log 2>&1
echo bench-ok
bash tools/custom_reducer_ab.sh 4 64 $out/custom_reducer
echo ab-ok
