# round 6, re-entry: N = 2 and 8 rehearsals at HEAD (ranks on one GPU), launched the way the driver launches them
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6c34; mkdir -p $O
( while true; do date +%s >> $O/heartbeat.txt; sleep 45; done ) & hb=$!
for n in 2 8; do
  timeout -k 10 540 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2977$n bench.py --gpus $n > $O/bench_n$n.json 2> $O/bench_n$n.err; brc=$?
  echo "bench n$n rc $brc" | tee -a $O/progress.txt; grep '^{' $O/bench_n$n.json | cut -c1-300
  [ $brc -eq 0 ] || break
done
kill $hb
