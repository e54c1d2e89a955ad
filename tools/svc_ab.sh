#!/bin/bash
# tools/small_latency.py alternated between two env settings (A B A B ...):
#   tools/svc_ab.sh "ENV_A" "ENV_B" ROUNDS [small_latency args]
set -o pipefail
A=$1; B=$2; R=${3:-3}; shift 3
mkdir -p gpurun_out/svc_ab
for i in $(seq 1 $R); do
  for v in A B; do
    e=$A; [ $v = B ] && e=$B
    env $(echo "$e" | tr ',' ' ') timeout -k 10 120 python3 -u tools/small_latency.py "$@" > gpurun_out/svc_ab/$v$i.txt 2>&1 \
      || { tail -5 gpurun_out/svc_ab/$v$i.txt; exit 1; }
    echo "$v$i [$e] $(grep -h '^{' gpurun_out/svc_ab/$v$i.txt | tail -1 | cut -c1-400)"
  done
done
