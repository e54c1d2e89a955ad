set -o pipefail
mkdir -p gpurun_out/litmus
timeout -k 10 120 tools/handoff_litmus local 3000 > gpurun_out/litmus/local.jsonl 2>&1 || exit 1
for load in 4 5 3 0; do
  d=$(mktemp -d)
  timeout -k 10 60 tools/handoff_litmus owner $d 1 $load 3000 >> gpurun_out/litmus/ipc.jsonl 2>&1 &
  op=$!
  timeout -k 10 60 tools/handoff_litmus writer $d >> gpurun_out/litmus/ipc.jsonl 2>&1 || { kill $op; exit 1; }
  wait $op || exit 1
done
cat gpurun_out/litmus/local.jsonl gpurun_out/litmus/ipc.jsonl
