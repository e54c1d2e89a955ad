#!/bin/bash
# A/B of hand-off fence variants on one box: N=2 (two processes on one GPU),
# 1 GiB fp32 mesh + ring, the main line only.  Usage: tools/ab_n2.sh OUTDIR
out=${1:-gpurun_out/ab}
mkdir -p $out
port=29700
for v in default strict default strict; do
  port=$((port+10))
  if [ $v = strict ]; then export RDC_STRICT_FENCES=1; else unset RDC_STRICT_FENCES; fi
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus 2 --steps 30 --extra-steps 0 --rccl-steps 0 --cpu-seconds 0 --ring-steps 10 \
    --no-check > $out/n2_$v.$port.log 2>&1 || exit 1
  echo "$v $(grep '^{' $out/n2_$v.$port.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["ring_schedule"]["ms_per_step"])')"
done
