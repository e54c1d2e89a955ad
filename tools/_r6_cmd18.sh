# round 6: direct schedule with peers imported at chosen addresses (dma-buf + ROCr vmem): every direct test, after-free three times, realloc replay at n = 3 and n = 2
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6c18; mkdir -p $O
( while true; do date +%s >> $O/heartbeat.txt; sleep 45; done ) & hb=$!
rc=0
RDC_DIRECT_LOG=1 RDC_TEST_MP_LOGDIR=$O/logs0 RDC_TEST_MP_TIMEOUT=120 timeout -k 10 400 python -u -m pytest tests/test_gpu_allreduce.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "untuned_default" > $O/untuned.log 2>&1; rc=$?; echo "untuned rc $rc"; tail -1 $O/untuned.log
for k in 1 2 3; do
  if [ $rc -eq 0 ]; then
    RDC_DIRECT_LOG=1 RDC_TEST_MP_LOGDIR=$O/logs$k RDC_TEST_MP_TIMEOUT=200 timeout -k 10 500 python -u -m pytest tests/test_gpu_allreduce.py -m gpu -x -v --timeout 250 --timeout-method thread -p no:cacheprovider -k "direct_after_free" > $O/after_free$k.log 2>&1; rc=$?; echo "after_free run $k rc $rc"; tail -1 $O/after_free$k.log
  fi
done
if [ $rc -eq 0 ]; then
  RDC_TEST_MP_TIMEOUT=200 timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "direct" > $O/direct_tests.log 2>&1; rc=$?; echo "direct tests rc $rc"; tail -1 $O/direct_tests.log
fi
if [ $rc -eq 0 ]; then
  RDC_DIRECT_LOG=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29611 tools/direct_check.py 16,64,256 6,10 realloc > $O/realloc_n3.log 2>&1; rc=$?; echo "realloc n3 rc $rc"
  echo "lines $(grep -c '"bad"' $O/realloc_n3.log) bad0 $(grep -c '"bad": 0' $O/realloc_n3.log) fallback $(grep -c ', fallback' $O/realloc_n3.log) direct $(grep -c ', direct$' $O/realloc_n3.log) unmaps $(grep -c 'close peer' $O/realloc_n3.log)"
fi
if [ $rc -eq 0 ]; then
  RDC_DIRECT_LOG=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 tools/direct_check.py 16,64,256 6,10 realloc > $O/realloc_n2.log 2>&1; rc=$?; echo "realloc n2 rc $rc"
  echo "lines $(grep -c '"bad"' $O/realloc_n2.log) bad0 $(grep -c '"bad": 0' $O/realloc_n2.log) fallback $(grep -c ', fallback' $O/realloc_n2.log) direct $(grep -c ', direct$' $O/realloc_n2.log)"
fi
kill $hb
