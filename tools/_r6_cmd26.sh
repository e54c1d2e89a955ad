# round 6: N = 2 / 4 / 8 rehearsals on one GPU (bench.py self-launches its ranks); heartbeat keeps the run visible
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6c26; mkdir -p $O
( while true; do date +%s >> $O/heartbeat.txt; sleep 45; done ) & hb=$!
for n in ${NS:-2 4 8}; do
  timeout -k 10 900 python bench.py --gpus $n > $O/bench_n$n.json 2> $O/bench_n$n.err; rc=$?
  echo "bench n$n rc $rc" | tee -a $O/progress.txt
  [ $rc -eq 0 ] || break
done
kill $hb
