#!/bin/bash
# Runs tools/graph_eager_stress.py variants; a wrong-result exit (1) goes on,
# anything else (timeout, abort, fault) ends the call.
set -o pipefail
mkdir -p gpurun_out/stress
i=0
for spec in "$@"; do
  i=$((i+1))
  IFS='|' read -r envs args <<< "$spec"
  env $(echo "$envs" | tr ',' ' ') timeout -k 10 180 python3 -u tools/graph_eager_stress.py $args \
      > gpurun_out/stress/s$i.json 2> gpurun_out/stress/s$i.err
  rc=$?
  echo "[$i] rc=$rc env=$envs args=$args"; head -c 1500 gpurun_out/stress/s$i.json; echo
  [ $rc -le 1 ] || { tail -5 gpurun_out/stress/s$i.err; exit $rc; }
done
