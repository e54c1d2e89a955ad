# round 6: the canary check of new peer mappings — after-free (ipc and vmem, n = 2 and 3) three times, every direct test, realloc replay n = 3 (HIP IPC)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6c24; mkdir -p $O
( while true; do date +%s >> $O/heartbeat.txt; sleep 45; done ) & hb=$!
rc=0
for k in 1 2 3; do
  if [ $rc -eq 0 ]; then
    RDC_DIRECT_LOG=1 RDC_TEST_MP_LOGDIR=$O/logs$k RDC_TEST_MP_TIMEOUT=200 timeout -k 10 600 python -u -m pytest tests/test_gpu_allreduce.py -m gpu -x -v --timeout 250 --timeout-method thread -p no:cacheprovider -k "direct_after_free" > $O/after_free$k.log 2>&1; rc=$?; echo "after_free run $k rc $rc"; tail -1 $O/after_free$k.log
  fi
done
if [ $rc -eq 0 ]; then
  RDC_TEST_MP_TIMEOUT=200 timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "direct" > $O/direct_tests.log 2>&1; rc=$?; echo "direct tests rc $rc"; tail -1 $O/direct_tests.log
fi
if [ $rc -eq 0 ]; then
  RDC_DIRECT_LOG=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29611 tools/direct_check.py 16,64,256 6,10 realloc > $O/realloc_n3.log 2>&1; rc=$?; echo "realloc n3 rc $rc"
  echo "bad0 $(grep -c '"bad": 0' $O/realloc_n3.log) of $(grep -c '"bad"' $O/realloc_n3.log) canary-mismatch $(grep -c 'canary .*expected' $O/realloc_n3.log)"
fi
echo "canary mismatches in the test logs: $(cat $O/logs*/*.log 2>/dev/null | grep -c 'canary .*expected')"
kill $hb
