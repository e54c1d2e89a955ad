# GPU session: reduce parity, bench N=1, rocprofv3 kernel trace + PMC traffic (round 1 profile set)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_reduce.py -q -x > gpurun_out/t_red.log 2>&1; echo "reduce tests rc=$?"; tail -1 gpurun_out/t_red.log
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1; echo "bench rc=$?"
grep '^{' gpurun_out/bench.log
P=$GRAFT_REPO_ROOT/gpurun_out/prof
rm -rf $P
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/trace -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/prof_trace.log 2>&1; echo "trace rc=$?"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $P/fetch -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --cpu-seconds 0 > gpurun_out/prof_fetch.log 2>&1; echo "fetch rc=$?"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $P/write -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --cpu-seconds 0 > gpurun_out/prof_write.log 2>&1; echo "write rc=$?"
cat $P/trace/run_kernel_stats.csv
