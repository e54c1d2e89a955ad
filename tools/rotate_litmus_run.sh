#!/bin/bash
# tools/rotate_litmus: one process (every memory kind x load kind) and IPC
# (writers in a second process) — each step under its own time limit.
set -o pipefail
O=gpurun_out/rotate
mkdir -p $O
: > $O/results.jsonl
for mem in 1 0 2; do for load in 1 3 0; do
  timeout -k 10 60 tools/rotate_litmus local $mem $load 4000 >> $O/results.jsonl 2>&1 || exit 1
done; done
for mem in 1 0; do for load in 1 3; do
  d=$(mktemp -d)
  timeout -k 10 90 tools/rotate_litmus owner $d $mem $load 4000 >> $O/results.jsonl 2>&1 &
  op=$!
  timeout -k 10 90 tools/rotate_litmus writer $d >> $O/results.jsonl 2>&1 || { kill $op; exit 1; }
  wait $op || exit 1
done; done
cat $O/results.jsonl
