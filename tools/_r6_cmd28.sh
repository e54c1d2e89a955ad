# round 6: more evidence for the canary at HEAD — after-free (ipc and vmem, n = 2 and 3) three times, the memory-returned tests, realloc replay n = 3 (HIP IPC) twice
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6c28; mkdir -p $O
( while true; do date +%s >> $O/heartbeat.txt; sleep 45; done ) & hb=$!
rc=0
for k in 1 2 3; do
  if [ $rc -eq 0 ]; then
    RDC_DIRECT_LOG=1 RDC_TEST_MP_LOGDIR=$O/logs$k RDC_TEST_MP_TIMEOUT=200 timeout -k 10 600 python -u -m pytest tests/test_gpu_allreduce.py -m gpu -x -v --timeout 250 --timeout-method thread -p no:cacheprovider -k "direct_after_free or freed_memory_returned" > $O/tests$k.log 2>&1; rc=$?; echo "run $k rc $rc $(tail -1 $O/tests$k.log)"
  fi
done
for k in 1 2; do
  if [ $rc -eq 0 ]; then
    RDC_DIRECT_LOG=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 2961$k tools/direct_check.py 16,64,256 6,10 realloc > $O/realloc_n3_$k.log 2>&1; rc=$?
    echo "realloc n3 run $k rc $rc bad0 $(grep -c '"bad": 0' $O/realloc_n3_$k.log) of $(grep -c '"bad"' $O/realloc_n3_$k.log) canary-mismatch $(grep -c 'canary .*expected' $O/realloc_n3_$k.log) fallback $(grep -c ', fallback' $O/realloc_n3_$k.log) direct $(grep -c ', direct$' $O/realloc_n3_$k.log)"
  fi
done
echo "canary mismatches in the test logs: $(cat $O/logs*/*.log 2>/dev/null | grep -c 'canary .*expected')"
kill $hb
