#!/bin/bash
# Runs tools/ipc_mtype_probe: the per-MTYPE request counters of every
# (memory kind, side) kernel in separate rocprofv3 --pmc passes (both
# processes profiled, their kernels never overlap), then the alias trials.
# Output: gpurun_out/mtype/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/mtype
mkdir -p $out
pass() {  # pass NAME COUNTERS...
  local tag=$1; shift
  local name="p$tag.$$"
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d $out/$tag/owner -o owner -- tools/ipc_mtype_probe owner "$name" mtype > $out/$tag.owner.log 2>&1 &
  local op=$!
  sleep 2
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d $out/$tag/peer -o peer -- tools/ipc_mtype_probe peer "$name" mtype > $out/$tag.peer.log 2>&1
  local prc=$?
  wait $op
  local orc=$?
  rm -f /dev/shm/rdc_mtype_$name
  echo "pass $tag: owner rc $orc peer rc $prc"
  [ $prc -eq 0 ] && [ $orc -eq 0 ]
}
pass read TCP_TCC_UC_READ_REQ_sum TCP_TCC_NC_READ_REQ_sum TCP_TCC_RW_READ_REQ_sum TCP_TCC_CC_READ_REQ_sum &&
pass write TCP_TCC_UC_WRITE_REQ_sum TCP_TCC_NC_WRITE_REQ_sum TCP_TCC_RW_WRITE_REQ_sum TCP_TCC_CC_WRITE_REQ_sum &&
pass atomic TCP_TCC_UC_ATOMIC_REQ_sum TCP_TCC_NC_ATOMIC_REQ_sum TCP_TCC_RW_ATOMIC_REQ_sum TCP_TCC_CC_ATOMIC_REQ_sum &&
pass hit TCC_HIT_sum TCC_MISS_sum || exit 1
name="alias.$$"
timeout -k 10 120 tools/ipc_mtype_probe owner "$name" alias ${TRIALS:-50} > $out/alias.owner.jsonl 2>&1 &
op=$!
sleep 1
timeout -k 10 120 tools/ipc_mtype_probe peer "$name" alias ${TRIALS:-50} > $out/alias.peer.jsonl 2>&1
prc=$?
wait $op
orc=$?
rm -f /dev/shm/rdc_mtype_$name
echo "alias: owner rc $orc peer rc $prc"
[ $prc -eq 0 ] && [ $orc -eq 0 ]
