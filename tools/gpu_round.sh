# One GPU call: parity suite, N=1 bench lines (fp32 headline + cfg4 fp16/bf16),
# cfg5 fused-vs-separate, and a rocprofv3 kernel trace of the coalesced path.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
  tail -2 gpurun_out/gpu_tests.log
fi
timeout -k 10 200 python bench.py > gpurun_out/bench_f32.json 2> gpurun_out/bench_f32.err || exit 1
timeout -k 10 200 python bench.py --dtype float16 --cpu-seconds 0 > gpurun_out/bench_f16.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --dtype bfloat16 --cpu-seconds 0 > gpurun_out/bench_bf16.json 2>gpurun_out/bench_bf16.err || { tail gpurun_out/bench_bf16.err; exit 1; }
cat gpurun_out/bench_f32.json gpurun_out/bench_f16.json gpurun_out/bench_bf16.json
bash tools/cfg5_compare.sh 2 > gpurun_out/cfg5.log 2>&1 || exit 1
cat gpurun_out/cfg5.log
P=gpurun_out/prof_coal
rm -rf $P
GP_BUCKETS=256 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P -o coal --output-format csv -- python tools/group_perf.py 2 256e6 > gpurun_out/prof_coal.log 2>&1 || exit 1
grep "n=2" gpurun_out/prof_coal.log
find $P -name "*kernel_stats.csv" -exec cat {} \;
