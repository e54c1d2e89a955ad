cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 ./tools/bench_reduce > gpurun_out/sweep3.log 2>&1; echo "sweep rc=$?"
awk '{for(i=1;i<=NF;i++) if($i=="GB/s") print $(i-1), $0}' gpurun_out/sweep3.log | sort -n -r | head -25
