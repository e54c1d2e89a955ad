# round 6: RDC_DIRECT_IMPORT=vmem opt-in, HIP IPC default: after-free (ipc and vmem, n = 2 and 3) twice, every direct test, the HSA-attach fallback test
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6c21; mkdir -p $O
( while true; do date +%s >> $O/heartbeat.txt; sleep 45; done ) & hb=$!
rc=0
for k in 1 2; do
  if [ $rc -eq 0 ]; then
    RDC_DIRECT_LOG=1 RDC_TEST_MP_LOGDIR=$O/logs$k RDC_TEST_MP_TIMEOUT=200 timeout -k 10 600 python -u -m pytest tests/test_gpu_allreduce.py -m gpu -x -v --timeout 250 --timeout-method thread -p no:cacheprovider -k "direct_after_free" > $O/after_free$k.log 2>&1; rc=$?; echo "after_free run $k rc $rc"; tail -1 $O/after_free$k.log
  fi
done
if [ $rc -eq 0 ]; then
  RDC_TEST_MP_TIMEOUT=200 timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "direct or uncached_flags" > $O/direct_tests.log 2>&1; rc=$?; echo "direct tests rc $rc"; tail -1 $O/direct_tests.log
fi
kill $hb
