#!/bin/bash
# A/B of two builds on one box for the cfg5 shape (1024 x 1 MiB fp32, one
# coalesced call) and the plain 1 GiB buffer, N=2 (two processes on one GPU):
# ab_old/librdc_amd.so (A) vs ab_old/librdc_amd_new.so (B), alternated.
out=${1:-gpurun_out/ab_cfg5}
mkdir -p $out
port=29900
for v in new old new old; do
  port=$((port+10))
  if [ $v = new ]; then cp ab_old/librdc_amd_new.so rdc_amd/librdc_amd.so; else cp ab_old/librdc_amd.so rdc_amd/librdc_amd.so; fi
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus 2 --steps 20 --buckets 1024 --autotune-reps 0 --no-check --cpu-seconds 0 \
    > $out/cfg5_$v.$port.log 2>&1 || exit 1
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $((port+1)) bench.py --gpus 2 --steps 20 --algo mesh --autotune-reps 0 --extra-steps 0 \
    --ring-steps 0 --rccl-steps 0 --no-check --cpu-seconds 0 > $out/mesh_$v.$port.log 2>&1 || exit 1
  echo "$v cfg5 $(grep '^{' $out/cfg5_$v.$port.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])') mesh $(grep '^{' $out/mesh_$v.$port.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done
cp ab_old/librdc_amd_new.so rdc_amd/librdc_amd.so
