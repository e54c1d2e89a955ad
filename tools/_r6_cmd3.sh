# round 6: new life cycle (refuse partly-overlapping mappings), UC flags check, 5 x 3 repro with launch timelines, realloc replay
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6c3; mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider"
timeout -k 10 600 $T tests/test_gpu_allreduce.py -k "untuned_default or freed_memory or direct_after_free" > $O/tests.log 2>&1; echo "tests rc $?"; grep -E "PASSED|FAILED" $O/tests.log
export GPU_MAX_HW_QUEUES=3 RDC_TEST_KEEP_QUEUES=1 RDC_LAUNCH_TIMES=1
bash tools/repro_5x3.sh 1 > $O/repro_uc_times.txt 2>&1; echo "repro rc $?"; head -12 $O/repro_uc_times.txt | cut -c1-1500
cp gpurun_out/repro/run1.txt $O/repro_uc_times_run1.txt 2>/dev/null
unset GPU_MAX_HW_QUEUES RDC_TEST_KEEP_QUEUES RDC_LAUNCH_TIMES
RDC_DIRECT_LOG=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29611 tools/direct_check.py 16,64,256 6,10 realloc > $O/realloc_n3_refuse.log 2>&1; echo "realloc n3 rc $?"
grep -c '"bad": 0' $O/realloc_n3_refuse.log; grep -c "close peer" $O/realloc_n3_refuse.log; grep -c "refused" $O/realloc_n3_refuse.log; grep -c "fallback" $O/realloc_n3_refuse.log
