#!/bin/bash
# A/B of two builds of librdc_amd.so on one box: N=2 (two processes on one
# GPU), 1 GiB fp32 mesh + ring + link probe.  ab_old/librdc_amd.so (A) vs
# ab_old/librdc_amd_new.so (B), alternated.  Usage: tools/ab_lib.sh OUTDIR
out=${1:-gpurun_out/ab_lib}
mkdir -p $out
port=29800
for v in new old new old; do
  port=$((port+10))
  if [ $v = new ]; then cp ab_old/librdc_amd_new.so rdc_amd/librdc_amd.so; else cp ab_old/librdc_amd.so rdc_amd/librdc_amd.so; fi
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus 2 --steps 30 --extra-steps 0 --rccl-steps 0 --cpu-seconds 0 --ring-steps 10 \
    --no-check > $out/n2_$v.$port.log 2>&1 || exit 1
  echo "$v $(grep '^{' $out/n2_$v.$port.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["ms_per_step"], d["ring_schedule"]["ms_per_step"], r["xgmi_probe"])')"
done
cp ab_old/librdc_amd_new.so rdc_amd/librdc_amd.so
