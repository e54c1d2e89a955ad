#!/bin/bash
# Rehearsal of round 4's lost one-shot hand-off: the 5-process host size sweep
# on one GPU at the launcher's queue budget (3 per process), every collective
# held to one block per CU (RDC_DEBUG_LDS_PAD), with the device-side
# launch-number check on.  K runs; a test failure goes on, anything else ends.
set -o pipefail
K=${1:-6}
PAD=${2:-98304}
SEL=${3:-"host_size_sweep and 5-0"}
O=gpurun_out/repro
mkdir -p $O
for i in $(seq 1 $K); do
  RDC_DEBUG_LDS_PAD=$PAD RDC_SEQ_CHECK=1 RDC_TIMEOUT=20 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_allreduce.py \
      -m gpu -x -q --timeout 280 --timeout-method thread -k "$SEL" -p no:cacheprovider \
      > $O/run$i.txt 2>&1
  rc=$?
  echo "[$i] rc=$rc $(tail -1 $O/run$i.txt)"; grep -h "device collective failed" $O/run$i.txt | sed 's/.*failed on//' | cut -c1-400 | head -5
  [ $rc -le 1 ] || exit $rc
done
