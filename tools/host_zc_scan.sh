# small host-buffer allreduce: zero-copy on pinned memory vs H2D/allreduce/D2H,
# per-call latency at n = 2 and 3 ranks (processes sharing ONE GPU)
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
for n in 2 3; do
  for zc in 0 1048576; do
    for spec in "4096 2000" "16384 2000" "65536 1000" "262144 500" "1048576 300"; do
      set -- $spec
      RDC_HOST_ZC_BYTES=$zc timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
        --master-addr 127.0.0.1 --master-port $((29600 + n * 10 + ${#1})) tools/host_path.py $1 $2 2>&1 \
        | grep host_path | sed "s/^/zc=$zc /" || exit 1
    done
  done
done
