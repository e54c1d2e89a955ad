# round 6: test_mp_direct_after_free[3] hung in one suite run: the same test with every rank's rendezvous log, 3 times
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6c8; mkdir -p $O
( while true; do date +%s >> $O/heartbeat.txt; sleep 45; done ) & hb=$!
for i in 1 2 3 4 5; do
  RDC_TEST_MP_LOGDIR=$O/mplogs_$i RDC_DIRECT_LOG=1 RDC_DEBUG=1 RDC_TIMEOUT=30 RDC_TEST_MP_TIMEOUT=140 timeout -k 10 170 python -u -m pytest -x -v --timeout 160 --timeout-method thread -m gpu -p no:cacheprovider tests/test_gpu_allreduce.py -k "direct_after_free and 3" > $O/after_free_$i.log 2>&1; rc=$?
  echo "run $i rc $rc" | tee -a $O/progress.txt
  [ $rc -eq 0 ] || break
done
kill $hb
