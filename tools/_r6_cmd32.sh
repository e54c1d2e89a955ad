# round 6, re-entry: test_mp_uncached_flags_fall_back_together N times at HEAD (default 8) (timed out once in 11 runs before the detach-before-free barrier); stops at the first failure
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6c32${TAG:-}; mkdir -p $O
T=tests/test_gpu_allreduce.py::test_mp_uncached_flags_fall_back_together
for i in $(seq 1 ${N:-8}); do
  RDC_TEST_MP_TIMEOUT=90 timeout -k 10 150 python -u -m pytest $T -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/run$i.log 2>&1 || { echo "run $i failed"; tail -40 $O/run$i.log; exit 1; }
  echo "run $i: $(tail -1 $O/run$i.log)" | tee -a $O/progress.txt
done
