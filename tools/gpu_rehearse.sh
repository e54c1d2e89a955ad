#!/bin/bash
# bench.py as the driver runs it for N > 1, with N processes sharing this
# box's one GPU (a protocol rehearsal: every byte moves through one HBM).
# Usage: tools/gpu_rehearse.sh N OUTFILE [extra bench args]
n=$1; out=$2; shift 2
mkdir -p "$(dirname "$out")"
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" --master-addr 127.0.0.1 \
  --master-port $((29700 + n)) bench.py --gpus "$n" "$@" > "$out" 2>&1
rc=$?
grep '^{' "$out" | python -c '
import json, sys
d = json.loads(sys.stdin.read())
print("N=%d value %.2f ms/step %.4f kernel %.4f launch %s" % (d["n_gpus"], d["value"], d["ms_per_step"],
      d["roofline"]["kernel_avg_ms"], d["config"].get("launch")))
print("autotune chosen", (d.get("autotune") or {}).get("chosen"))
print("checks", d.get("oracle_check"))
print("extras", d.get("extras_wall_s"), "skipped", d.get("extras_skipped"), "errors", d.get("extras_error"))
' || true
exit $rc
