#!/bin/bash
# Round 3, session 3: registered-buffer A/B (tools/host_registered_ab2.sh),
# then the whole GPU suite + smoke + N=1 line + rocprofv3 (tools/gpu_suite.sh).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
set -o pipefail
bash tools/host_registered_ab2.sh gpurun_out/host_registered_ab2 || exit 1
bash tools/gpu_suite.sh || exit 1
