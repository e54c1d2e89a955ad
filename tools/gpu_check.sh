cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_allreduce.py -q -x -k many_ranks > gpurun_out/t_many.log 2>&1; echo "rc=$?"
grep -E "^E  |passed|failed|Error" gpurun_out/t_many.log | head -30
