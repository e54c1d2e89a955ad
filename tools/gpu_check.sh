cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_entrypoints.py -q > gpurun_out/t_entry.log 2>&1; echo "rc=$?"
grep -E "^--- rank|rdc|mismatch|OK|passed|failed" gpurun_out/t_entry.log | head -40
