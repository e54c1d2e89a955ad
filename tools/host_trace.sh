cd $GRAFT_REPO_ROOT
RDC_HOST_TRACE=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29811 tools/host_path.py 268435456 2 > gpurun_out/host_trace.log 2>&1
rc=$?; grep -E "host_path" gpurun_out/host_trace.log; grep "\[host" gpurun_out/host_trace.log | tail -60; exit $rc
