#!/bin/bash
# The whole GPU suite as the driver runs it, then smoke + N=1 line + rocprofv3 stats.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_suite.log 2>&1 || { tail -30 gpurun_out/gpu_suite.log; exit 1; }
tail -3 gpurun_out/gpu_suite.log
bash tools/gpu_final.sh
