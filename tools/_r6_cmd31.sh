# round 6, re-entry: the whole GPU suite, smoke, N = 1 bench + rocprofv3 with libraries rebuilt in the re-created container
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6c31; mkdir -p $O
( while true; do date +%s >> $O/heartbeat.txt; sleep 45; done ) & hb=$!
RDC_TEST_MP_TIMEOUT=240 RDC_DIRECT_LOG=1 timeout -k 10 1300 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > $O/gpu_suite.log 2>&1; rc=$?; echo "suite rc $rc"; tail -3 $O/gpu_suite.log
if [ $rc -eq 0 ]; then
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; echo "smoke rc $?"; tail -1 $O/smoke.log
  timeout -k 10 300 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err; echo "bench n1 rc $?"; cut -c1-400 $O/bench_n1.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_n1 -o n1 -- python3 bench.py --steps 25 --warmup 3 --cpu-seconds 0 --no-check > $O/bench_n1_prof.json 2> $O/bench_n1_prof.err; echo "rocprof rc $?"
fi
kill $hb
