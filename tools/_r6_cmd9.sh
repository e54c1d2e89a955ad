# round 6: is the 5 x 3 starvation a matter of grid size? 3 runs each at 32 and 48 blocks per rank (one block per CU)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6c9; mkdir -p $O
( while true; do date +%s >> $O/heartbeat.txt; sleep 45; done ) & hb=$!
export GPU_MAX_HW_QUEUES=3 RDC_TEST_KEEP_QUEUES=1 RDC_LAUNCH_TIMES=1
for nb in 32 48; do
  RDC_NBLOCKS=$nb bash tools/repro_5x3.sh 3 > $O/repro_nblocks$nb.txt 2>&1
  echo "nblocks $nb: $(grep -c 'rc=0' $O/repro_nblocks$nb.txt) of 3 passed" | tee -a $O/progress.txt
done
kill $hb
