# round 6: test_mp_direct_after_free with the direct log (a fallback at case 11 with no refusal counted)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6c13; mkdir -p $O
( while true; do date +%s >> $O/heartbeat.txt; sleep 45; done ) & hb=$!
RDC_DIRECT_LOG=1 RDC_TEST_MP_LOGDIR=$O/logs RDC_TEST_MP_TIMEOUT=200 timeout -k 10 500 python -u -m pytest tests/test_gpu_allreduce.py -m gpu -v --timeout 250 --timeout-method thread -p no:cacheprovider -k "direct_after_free" > $O/tests.log 2>&1; echo "tests rc $?"; tail -3 $O/tests.log
kill $hb
