set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/ipc_remap_run.sh > gpurun_out/remap_run2.log 2>&1; echo remap rc $?
out=gpurun_out/mtype2; mkdir -p $out
for tag in read hit; do
  if [ $tag = read ]; then C="TCP_TCC_UC_READ_REQ_sum TCP_TCC_NC_READ_REQ_sum TCP_TCC_RW_READ_REQ_sum TCP_TCC_CC_READ_REQ_sum"; else C="TCC_HIT_sum TCC_MISS_sum"; fi
  n="m2$tag.$$"
  timeout -s KILL 90 rocprofv3 --pmc $C -d $out/$tag/owner -o owner -- tools/ipc_mtype_probe owner $n mtype > $out/$tag.owner.log 2>&1 &
  op=$!
  sleep 2
  timeout -s KILL 90 rocprofv3 --pmc $C -d $out/$tag/peer -o peer -- tools/ipc_mtype_probe peer $n mtype > $out/$tag.peer.log 2>&1; prc=$?
  wait $op; orc=$?
  echo "mtype $tag owner $orc peer $prc"
  rm -f /dev/shm/rdc_mtype_$n
  [ $prc -eq 0 ] && [ $orc -eq 0 ] || exit 1
done
timeout -k 10 500 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_allreduce.py -k "direct_after_free or freed_memory or untuned_default" -p no:cacheprovider > gpurun_out/t_direct_new.log 2>&1; echo tests rc $?
tail -5 gpurun_out/t_direct_new.log
