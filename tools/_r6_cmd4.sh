# round 6: per-size schedule sweep with the direct rendezvous cost (N = 2 and 8 on one GPU), default vs RDC_DIRECT_BYTES=0
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6c4; mkdir -p $O
S="0.00390625,0.0625,0.25,1,4,16,64,256,1024"
for n in 2 8; do
  q=4; [ $n -gt 4 ] && q=2
  GPU_MAX_HW_QUEUES=$q SWEEP_ALGOS=0/1/2/3/5/6 timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2962$n tools/algo_sweep.py $S 20 > $O/sweep_n$n.txt 2>&1; echo "sweep n$n rc $?"
  grep algo_sweep $O/sweep_n$n.txt | cut -c1-400
done
GPU_MAX_HW_QUEUES=2 RDC_DIRECT_BYTES=0 SWEEP_ALGOS=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29631 tools/algo_sweep.py $S 20 > $O/sweep_n8_nodirect.txt 2>&1; echo "sweep n8 nodirect rc $?"
# flag words HSA-uncached (default) vs hipDeviceMallocUncached (CC): small-size latency at N = 8 and 2
for n in 8 2; do
  q=4; [ $n -gt 4 ] && q=2
  GPU_MAX_HW_QUEUES=$q RDC_FLAGS_MEM=cc SWEEP_ALGOS=0/2/3/5/6 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2964$n tools/algo_sweep.py 0.00390625,0.0625,1,16,256 20 > $O/sweep_n${n}_flags_cc.txt 2>&1; echo "sweep n$n cc rc $?"
  GPU_MAX_HW_QUEUES=$q SWEEP_ALGOS=0/2/3/5/6 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2965$n tools/algo_sweep.py 0.00390625,0.0625,1,16,256 20 > $O/sweep_n${n}_flags_uc.txt 2>&1; echo "sweep n$n uc rc $?"
done
# the 5 x 3 starvation with a small grid (8 blocks per rank: 40 of 256 CUs): CU capacity or queue scheduling?
export GPU_MAX_HW_QUEUES=3 RDC_TEST_KEEP_QUEUES=1 RDC_LAUNCH_TIMES=1 RDC_NBLOCKS=8
bash tools/repro_5x3.sh 1 > $O/repro_nblocks8.txt 2>&1; echo "repro nblocks8 rc $?"; head -3 $O/repro_nblocks8.txt | cut -c1-300
cp gpurun_out/repro/run1.txt $O/repro_nblocks8_run1.txt 2>/dev/null
