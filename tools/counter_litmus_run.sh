#!/bin/bash
# tools/counter_litmus in one process and in 5 concurrent processes with 3
# hardware queues each (round 4's 5 x 3 configuration).  A mismatch exits 1
# and the script goes on; anything else ends it.
set -o pipefail
O=gpurun_out/counter
mkdir -p $O
run1() {  # name args...
  local name=$1; shift
  timeout -k 10 120 tools/counter_litmus "$@" > $O/$name.json 2>&1; local rc=$?
  echo "$name rc=$rc $(cat $O/$name.json)"; [ $rc -le 1 ] || exit $rc
}
run1 single_g256 256 20000 1 0 0
run1 single_g40 40 20000 1 0 0
run1 single_3streams 256 20000 3 0 0
run1 single_uc 256 20000 1 1 0
for variant in "40 10000 3 0 2" "256 10000 3 0 2" "40 10000 1 0 0"; do
  pids=()
  for p in 1 2 3 4 5; do
    GPU_MAX_HW_QUEUES=3 timeout -k 10 240 tools/counter_litmus $variant > $O/mp_$p.json 2>&1 &
    pids+=($!)
  done
  for p in 1 2 3 4 5; do
    wait ${pids[$((p-1))]}; rc=$?
    echo "mp[$variant] proc $p rc=$rc $(cat $O/mp_$p.json)"
    [ $rc -le 1 ] || exit $rc
  done
done
