#!/bin/bash
# Bisect the >2^31 host_allreduce mismatch: per-window report at a small and
# the full size, streaming-store copy on/off, ramp on/off.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/diag
set -o pipefail
D=gpurun_out/diag
timeout -k 10 200 python tools/diag_host_windows.py 100667395 > $D/small_default.log 2>&1 && tail -3 $D/small_default.log &&
RDC_HOST_NT_COPY=0 timeout -k 10 200 python tools/diag_host_windows.py 100667395 > $D/small_nt0.log 2>&1 && tail -3 $D/small_nt0.log &&
timeout -k 10 300 python tools/diag_host_windows.py 2147487747 > $D/big_default.log 2>&1 && tail -8 $D/big_default.log &&
RDC_HOST_NT_COPY=0 timeout -k 10 300 python tools/diag_host_windows.py 2147487747 > $D/big_nt0.log 2>&1 && tail -8 $D/big_nt0.log &&
RDC_HOST_PIECE_RAMP=0 timeout -k 10 300 python tools/diag_host_windows.py 2147487747 > $D/big_ramp0.log 2>&1 && tail -8 $D/big_ramp0.log
