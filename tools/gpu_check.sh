cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/t_gpu.log 2>&1; echo "rc=$?"
grep -E "^E  |passed|failed" gpurun_out/t_gpu.log | head -30
timeout -k 10 120 python tools/group_perf.py 3 1e6 16e6 64e6 256e6 2>&1 | grep -v amdgpu.ids
