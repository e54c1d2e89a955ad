# round 6: the 5 x 3 and 6 x 3 configs at HEAD (slack from 5 ranks per GPU, canary in), one block per CU
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6c30; mkdir -p $O
( while true; do date +%s >> $O/heartbeat.txt; sleep 45; done ) & hb=$!
GPU_MAX_HW_QUEUES=3 RDC_TEST_KEEP_QUEUES=1 RDC_LAUNCH_TIMES=1 bash tools/repro_5x3.sh 3 > $O/repro_5x3.txt 2>&1
echo "5x3: $(grep -c 'rc=0' $O/repro_5x3.txt) of 3 passed" | tee -a $O/progress.txt
RDC_LAUNCH_TIMES=1 bash tools/queue_matrix.sh 6:3:2 > $O/qm.txt 2>&1; echo "6x3 rc $?" | tee -a $O/progress.txt
cp gpurun_out/qm/w6q3.txt $O/ 2>/dev/null; head -3 $O/w6q3.txt | cut -c1-200 | tee -a $O/progress.txt
kill $hb
