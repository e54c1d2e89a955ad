cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/o
export TMPDIR=/tmp
python - > gpurun_out/cases.json <<'PY'
import json; print(json.dumps([{"count": 1024, "dtype": 6, "op": 2, "algo": 2}]))
PY
export RDC_DEBUG=1 RDC_NBLOCKS=64 RDC_DEVICE=0 RDC_TIMEOUT=20 RDC_BOOTSTRAP_TIMEOUT=30
port=29700
for sz in 3G 4080M; do
  port=$((port+1))
  echo "=== scratch $sz"
  RDC_SCRATCH_BYTES=$sz timeout -k 5 40 python tests/mp_worker.py 0 2 $port gpurun_out/o gpurun_out/cases.json > gpurun_out/w0.log 2>&1 &
  RDC_SCRATCH_BYTES=$sz timeout -k 5 40 python tests/mp_worker.py 1 2 $port gpurun_out/o gpurun_out/cases.json > gpurun_out/w1.log 2>&1 &
  wait
  cat gpurun_out/w0.log gpurun_out/w1.log | grep -v amdgpu.ids | grep -E "mapped|done|Error|error"
done
unset RDC_DEBUG RDC_NBLOCKS RDC_DEVICE RDC_TIMEOUT RDC_BOOTSTRAP_TIMEOUT
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/t_gpu.log 2>&1; echo "gpu tests rc=$?"
tail -15 gpurun_out/t_gpu.log
