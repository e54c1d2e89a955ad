#!/bin/bash
# Round 3, session 2: the whole GPU suite at HEAD, smoke + N=1 line + rocprofv3
# stats, then the streaming-store host copy A/B (tools/host_nt_ab.sh).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
set -o pipefail
bash tools/gpu_suite.sh || exit 1
bash tools/host_nt_ab.sh gpurun_out/host_nt_ab || exit 1
