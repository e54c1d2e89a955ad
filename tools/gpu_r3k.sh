#!/bin/bash
# Round 3, session 3: the registered-buffer host path (GPU test at n = 2 / 3,
# then the pageable vs registered A/B), then the whole GPU suite + final.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_allreduce.py -k "host_registered" -x -v --timeout 300 \
  --timeout-method thread > gpurun_out/registered_tests.log 2>&1 || { tail -40 gpurun_out/registered_tests.log; exit 1; }
tail -5 gpurun_out/registered_tests.log
bash tools/host_registered_ab.sh gpurun_out/host_registered_ab || exit 1
