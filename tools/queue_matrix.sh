#!/bin/bash
# tools/host_sweep_repro.py over (world, hardware queues per process) pairs at
# one block per CU (RDC_DEBUG_LDS_PAD=96K): "W:Q:K" arguments.  A wrong or
# timed-out collective (exit 1) goes on; anything else ends the call.
set -o pipefail
mkdir -p gpurun_out/qm
for spec in "$@"; do
  IFS=':' read -r W Q K <<< "$spec"
  GPU_MAX_HW_QUEUES=$Q RDC_TEST_KEEP_QUEUES=1 RDC_DEBUG_LDS_PAD=${PAD:-98304} RDC_TIMEOUT=15 \
    timeout -k 10 400 python3 -u tools/host_sweep_repro.py $W $K > gpurun_out/qm/w${W}q${Q}.txt 2>&1
  rc=$?
  cut -c1-300 gpurun_out/qm/w${W}q${Q}.txt
  [ $rc -le 1 ] || exit $rc
done
