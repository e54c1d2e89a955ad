# round 6: refusal only (plug retry reverted): the after-free and memory-returned tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6c12; mkdir -p $O
( while true; do date +%s >> $O/heartbeat.txt; sleep 45; done ) & hb=$!
rc=0
if [ $rc -eq 0 ]; then
  RDC_TEST_MP_TIMEOUT=240 timeout -k 10 600 python -u -m pytest tests/test_gpu_allreduce.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "direct_after_free or freed_memory_returned or untuned_default" > $O/tests.log 2>&1; rc=$?; echo "tests rc $rc"; tail -3 $O/tests.log
fi

# last (a hang ends the call): the HSA-attach fallback test that timed out in r6c6, with the library's and the workers' debug lines
if [ $rc -eq 0 ]; then
  RDC_DEBUG=1 RDC_LAUNCH_TIMES=1 RDC_TEST_MP_TIMEOUT=150 RDC_TEST_MP_LOGDIR=$O/fallback timeout -k 10 300 python -u -m pytest tests/test_gpu_allreduce.py -m gpu -x -v --timeout 250 --timeout-method thread -p no:cacheprovider -k "uncached_flags_fall_back" > $O/fallback.log 2>&1; echo "fallback rc $?"; tail -3 $O/fallback.log
fi
kill $hb
