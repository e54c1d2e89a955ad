# round 6: how much CU slack removes the 5 x 3 starvation (one block per CU, 5 ranks, 3 queues each)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6c5; mkdir -p $O
export GPU_MAX_HW_QUEUES=3 RDC_TEST_KEEP_QUEUES=1 RDC_LAUNCH_TIMES=1
for nb in 40 32; do
  RDC_NBLOCKS=$nb bash tools/repro_5x3.sh 1 > $O/repro_nblocks$nb.txt 2>&1; echo "repro nblocks$nb rc $?"; head -2 $O/repro_nblocks$nb.txt | cut -c1-200
  cp gpurun_out/repro/run1.txt $O/repro_nblocks${nb}_run1.txt 2>/dev/null
done
