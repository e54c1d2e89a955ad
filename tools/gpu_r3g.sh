#!/bin/bash
# Unit-cache ring + contiguous host pieces: coalesced GPU tests, host piece
# sweep (twice, alternating order), copy-only pipeline by piece size, then
# the r3f batch (cfg5 vs one buffer, N = 4 / N = 8 rehearsals).
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_allreduce.py \
  -k "coalesced or cfg5" > gpurun_out/r3g_tests.log 2>&1 || exit 1
echo tests-ok
PIECES="2097152 4194304 8388608" bash tools/host_piece_sweep.sh gpurun_out/r3g_piece_a || exit 1
PIECES="8388608 4194304 2097152" bash tools/host_piece_sweep.sh gpurun_out/r3g_piece_b || exit 1
for P in 2097152 4194304 8388608; do
  for S in 67108864 268435456; do
    timeout -k 10 120 tools/pcie_pipeline_bench $S $P 10 > gpurun_out/r3g_copy_only_${P}_$S.json || exit 1
  done
done
echo sweep-ok
bash tools/gpu_r3f.sh
