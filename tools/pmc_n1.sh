#!/bin/bash
# HBM traffic of the N=1 bench's k_reduce: FETCH_SIZE and WRITE_SIZE in
# separate rocprofv3 --pmc passes (MI355X_MICROARCH.md HBM section), then
# tools/pmc_traffic.py applies the gfx950 correction and writes the
# per-launch bytes into profiles/traffic.json (copied back by the caller).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/pmc_n1
rm -rf $out && mkdir -p $out
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $out/fetch -o fetch --output-format csv -- \
  python3 bench.py --steps 5 --warmup 1 --cpu-seconds 0 --no-check > $out/fetch.log 2>&1 || { tail -20 $out/fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $out/write -o write --output-format csv -- \
  python3 bench.py --steps 5 --warmup 1 --cpu-seconds 0 --no-check > $out/write.log 2>&1 || { tail -20 $out/write.log; exit 1; }
f=$(find $out/fetch -name "*counter_collection.csv" | head -1)
w=$(find $out/write -name "*counter_collection.csv" | head -1)
cp $f $out/fetch_counter_collection.csv && cp $w $out/write_counter_collection.csv
python3 tools/pmc_traffic.py $out/fetch_counter_collection.csv $out/write_counter_collection.csv "k_reduce<2, float" \
  reduce_sum_f32_1073741824 $out/traffic.json
