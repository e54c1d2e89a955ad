#!/bin/bash
# Round 3, session 3 final: N=8 / N=4 rehearsals with the queue budget, then
# the whole GPU suite + smoke + N=1 line + rocprofv3 (tools/gpu_suite.sh).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
set -o pipefail
bash tools/gpu_rehearse.sh 8 gpurun_out/rehearse/n8_q.txt || exit 1
bash tools/gpu_rehearse.sh 4 gpurun_out/rehearse/n4_q.txt || exit 1
bash tools/gpu_suite.sh || exit 1
