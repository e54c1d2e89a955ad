# mesh/ring medium sizes, 2 ranks of one process on ONE GPU: tile-size sweep
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
for tile in 0 32K 64K 128K 256K 512K; do
  RDC_TILE_BYTES=$tile timeout -k 10 120 python tools/group_perf.py 2 4e6 16e6 64e6 2>&1 | grep "n=2" | sed "s/^/tile=$tile /" || exit 1
done
