#!/bin/bash
# Timeline of the registered host path at 64 MiB, n = 2 on one GPU: each rank
# under its own rocprofv3 (kernel + memory-copy trace), started directly (no
# launcher between the profiler and python).
out=${1:-gpurun_out/host_registered_trace}
mkdir -p $out
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1 MASTER_PORT=30700 WORLD_SIZE=2 LOCAL_RANK=0
S=${2:-67108864}
for pin in 1 0; do
  pids=""
  for r in 0 1; do
    RDC_BENCH_PINNED=$pin RANK=$r timeout -k 10 150 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
      -d $out/pin${pin}_r$r -o trace -- python3 tools/host_path.py $S 6 > $out/pin${pin}_r$r.log 2>&1 &
    pids="$pids $!"
  done
  for p in $pids; do wait $p || exit 1; done
  grep host_path $out/pin${pin}_r0.log
  export MASTER_PORT=30701
done
