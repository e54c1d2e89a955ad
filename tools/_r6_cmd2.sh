# round 6: HSA-uncached flags (MTYPE UC) against the 5 x 3 repro, and the remap record at n = 3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6c2; mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider"
timeout -k 10 600 $T tests/test_gpu_allreduce.py -k "direct_registered_buffers or freed_memory or fuzz and 2-21 or many_ranks and 8 or host_size_sweep and 3-0" > $O/tests.log 2>&1; echo "tests rc $?"; tail -3 $O/tests.log
# the lost hand-off: 5 processes x 3 hardware queues, one block per CU; flags CC (rounds 1-5), then UC (round 6)
export GPU_MAX_HW_QUEUES=3 RDC_TEST_KEEP_QUEUES=1
RDC_FLAGS_MEM=cc bash tools/repro_5x3.sh 1 > $O/repro_cc.txt 2>&1; echo "repro cc rc $?"; cat $O/repro_cc.txt | head -8
mkdir -p gpurun_out/repro_cc && cp -r gpurun_out/repro/* gpurun_out/repro_cc/ 2>/dev/null
bash tools/repro_5x3.sh 2 > $O/repro_uc.txt 2>&1; echo "repro uc rc $?"; cat $O/repro_uc.txt | head -8
unset GPU_MAX_HW_QUEUES RDC_TEST_KEEP_QUEUES
# round 5's fault record, replayed with the round-6 life cycle (close after the previous direct launch, closed ranges held reserved)
RDC_DIRECT_LOG=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29611 tools/direct_check.py 16,64,256 6,10 realloc > $O/realloc_n3_quarantine.log 2>&1; echo "realloc n3 rc $?"
grep -c '"bad": 0' $O/realloc_n3_quarantine.log; grep -c "close peer" $O/realloc_n3_quarantine.log; grep -c "fallback" $O/realloc_n3_quarantine.log
