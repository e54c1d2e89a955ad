cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/t_gpu.log 2>&1; echo "rc=$?"
grep -E "^E  |passed|failed|Error" gpurun_out/t_gpu.log | head -30
