# round 6: the HSA-attach fallback test (timed out once in r6c6, passed alone in r6c14) eight times with the library's debug lines; stops at the first failure
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6c16; mkdir -p $O
( while true; do date +%s >> $O/heartbeat.txt; sleep 45; done ) & hb=$!
rc=0
for k in 1 2 3 4 5 6 7 8; do
  if [ $rc -eq 0 ]; then
    RDC_DEBUG=1 RDC_TEST_MP_TIMEOUT=60 RDC_TEST_MP_LOGDIR=$O/logs$k timeout -k 10 200 python -u -m pytest tests/test_gpu_allreduce.py -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider -k "uncached_flags_fall_back" > $O/run$k.log 2>&1; rc=$?; echo "run $k rc $rc $(tail -1 $O/run$k.log)"
  fi
done
if [ $rc -eq 0 ]; then
  RDC_TEST_MP_TIMEOUT=200 timeout -k 10 600 python -u -m pytest tests/test_gpu_allreduce.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "direct_after_free or freed_memory_returned" > $O/direct_tests.log 2>&1; rc=$?; echo "direct tests rc $rc"; tail -1 $O/direct_tests.log
fi
kill $hb
