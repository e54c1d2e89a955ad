# host-buffer allreduce: parity cases, then per-call rates at 4 KiB / 1 MiB / 256 MiB
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -k "mp_allreduce or cpp" > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for n in 2 3; do
  for spec in "4096 500" "1048576 100" "268435456 12"; do
    set -- $spec
    timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29700 + n * 10 + ${#1})) tools/host_path.py $1 $2 2>&1 | grep host_path || exit 1
  done
done
