# round 6: the exporter's checks (ROCr pointer info, dma-buf size and inode): realloc replays at n = 2 and 3 with the direct log, after-free once
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6c20; mkdir -p $O
( while true; do date +%s >> $O/heartbeat.txt; sleep 45; done ) & hb=$!
RDC_DIRECT_LOG=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 tools/direct_check.py 16,64,256 6,10 realloc > $O/realloc_n2.log 2>&1; rc=$?; echo "realloc n2 rc $rc"
grep -E "dma-buf export|, fallback" $O/realloc_n2.log | cut -c1-220 | head -10
if [ $rc -eq 0 ]; then
  RDC_DIRECT_LOG=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29611 tools/direct_check.py 16,64,256 6,10 realloc > $O/realloc_n3.log 2>&1; rc=$?; echo "realloc n3 rc $rc"
  echo "bad0 $(grep -c '"bad": 0' $O/realloc_n3.log) of $(grep -c '"bad"' $O/realloc_n3.log)"
  grep -E "dma-buf export|, fallback" $O/realloc_n3.log | cut -c1-220 | head -10
fi
if [ $rc -eq 0 ]; then
  RDC_DIRECT_LOG=1 RDC_TEST_MP_LOGDIR=$O/logs RDC_TEST_MP_TIMEOUT=200 timeout -k 10 500 python -u -m pytest tests/test_gpu_allreduce.py -m gpu -x -v --timeout 250 --timeout-method thread -p no:cacheprovider -k "direct_after_free" > $O/after_free.log 2>&1; rc=$?; echo "after_free rc $rc"; tail -1 $O/after_free.log
fi
kill $hb
