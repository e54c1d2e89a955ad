#!/bin/bash
# Round 3, session 3: the fuzz suite with registered host ranges in the mix,
# then 40 more stress seeds (tools/fuzz_stress.py 400 40).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 500 python -u -m pytest tests/test_gpu_allreduce.py -k "random_sizes_fuzz or host_registered" -x -v \
  --timeout 300 --timeout-method thread > gpurun_out/fuzz_registered.log 2>&1 || { tail -40 gpurun_out/fuzz_registered.log; exit 1; }
tail -4 gpurun_out/fuzz_registered.log
timeout -k 10 600 python -u tools/fuzz_stress.py 400 40 > gpurun_out/fuzz_stress_400.log 2>&1 || { tail -30 gpurun_out/fuzz_stress_400.log; exit 1; }
tail -5 gpurun_out/fuzz_stress_400.log
