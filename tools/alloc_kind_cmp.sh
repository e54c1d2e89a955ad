# scratch memory kind (RDC_ALLOC = uncached | fine | coarse), 2 ranks as processes on ONE GPU:
# probe push rate and 1 GiB allreduce time (correctness across GPUs needs uncached)
cd $GRAFT_REPO_ROOT
port=29900
for k in uncached fine coarse; do
  port=$((port+5))
  RDC_ALLOC=$k timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus 2 --steps 10 --warmup 3 --ring-steps 5 --extra-steps 0 --rccl-steps 0 2>&1 | grep '^{' \
    | python -c "import sys,json; d=json.loads(sys.stdin.read()); p=d['roofline']['xgmi_probe']; print('$k mesh %.3f ms ring %.3f ms probe one-link %.0f all-links %.0f GB/s' % (d['ms_per_step'], d['ring_schedule']['ms_per_step'], p['one_link_one_direction_GBps'], p['all_links_egress_GBps']))" || exit 1
done
