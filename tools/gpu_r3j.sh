#!/bin/bash
# Host path by dtype and size: which (dtype, size) disagree with the oracle.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/diag2
set -o pipefail
D=gpurun_out/diag2
for cnt in 100003 3145731 41943043 100667395; do
  timeout -k 10 200 python tools/diag_host_windows.py $cnt 2 0 1 2 6 > $D/c$cnt.log 2>&1 || { tail -20 $D/c$cnt.log; exit 1; }
  grep "^count\|^dtype" $D/c$cnt.log | head -30
done
