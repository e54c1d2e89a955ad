cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
P=$GRAFT_REPO_ROOT/gpurun_out/profc
rm -rf $P
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P -o group2 --output-format csv -- python tools/group_perf.py 2 1e6 16e6 256e6 > gpurun_out/profc.log 2>&1; echo "rc=$?"
grep -v amdgpu gpurun_out/profc.log | grep "n=2"
cat $P/group2_kernel_stats.csv
