# N = 1 HBM traffic of k_reduce<Sum,float> on 1 GiB: FETCH_SIZE and WRITE_SIZE in separate rocprofv3 --pmc passes
# (MI355X_MICROARCH.md HBM section), summarised per launch by tools/pmc_traffic.py into $O/traffic.json
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${O:-gpurun_out/pmc_n1}; mkdir -p $O
B="python3 bench.py --steps 5 --warmup 1 --cpu-seconds 0 --no-check"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o f -- $B > $O/fetch.json 2> $O/fetch.err && echo "fetch pass ok" &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o w -- $B > $O/write.json 2> $O/write.err && echo "write pass ok" &&
python3 tools/pmc_traffic.py $(ls $O/fetch/*counter_collection.csv $O/fetch/*/*counter_collection.csv 2>/dev/null | head -1) \
    $(ls $O/write/*counter_collection.csv $O/write/*/*counter_collection.csv 2>/dev/null | head -1) \
    "k_reduce<2, float" reduce_sum_f32_1073741824 $O/traffic.json && cat $O/traffic.json
