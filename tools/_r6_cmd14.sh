# round 6: fallback accounting (direct_fallback / direct_map_failed / reason) — test_mp_direct_after_free three times with the direct log, then the HSA-attach fallback test with debug lines
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6c14; mkdir -p $O
( while true; do date +%s >> $O/heartbeat.txt; sleep 45; done ) & hb=$!
rc=0
for k in 1 2 3; do
  if [ $rc -eq 0 ]; then
    RDC_DIRECT_LOG=1 RDC_TEST_MP_LOGDIR=$O/logs$k RDC_TEST_MP_TIMEOUT=200 timeout -k 10 500 python -u -m pytest tests/test_gpu_allreduce.py -m gpu -v --timeout 250 --timeout-method thread -p no:cacheprovider -k "direct_after_free" > $O/tests$k.log 2>&1; rc=$?; echo "after_free run $k rc $rc"; tail -1 $O/tests$k.log
  fi
done
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  RDC_DEBUG=1 RDC_LAUNCH_TIMES=1 RDC_TEST_MP_TIMEOUT=150 RDC_TEST_MP_LOGDIR=$O/fallback timeout -k 10 300 python -u -m pytest tests/test_gpu_allreduce.py -m gpu -x -v --timeout 250 --timeout-method thread -p no:cacheprovider -k "uncached_flags_fall_back" > $O/fallback.log 2>&1; echo "fallback rc $?"; tail -3 $O/fallback.log
fi
kill $hb
