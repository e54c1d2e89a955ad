# One GPU call: smoke, N=1 bench line, rocprofv3 kernel stats of the same command.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err || { tail -20 gpurun_out/bench_n1.err; exit 1; }
cat gpurun_out/bench_n1.json
P=gpurun_out/prof_n1
rm -rf $P
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P -o bench_n1 --output-format csv -- python bench.py --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/prof_n1.log 2>&1 || { tail -20 gpurun_out/prof_n1.log; exit 1; }
find $P -name "*kernel_stats.csv" -exec cat {} \;
