# round 6: which dma-bufs come out smaller than the allocation (realloc replay at n = 2 with the direct log)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6c19; mkdir -p $O
RDC_DIRECT_LOG=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 tools/direct_check.py 16,64,256 6,10 realloc > $O/realloc_n2.log 2>&1; rc=$?; echo "realloc n2 rc $rc"
grep -E "dma-buf|, fallback" $O/realloc_n2.log | head -20
