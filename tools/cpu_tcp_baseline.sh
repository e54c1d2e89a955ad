# The reference's CPU ring allreduce over loopback TCP (oracle/tcp_ring, a C
# restatement — the reference does not build as shipped) on this host's cores,
# at the BASELINE configs' shapes.  One JSON line per (n, size).
cd ${GRAFT_REPO_ROOT:-.}
[ -x oracle/tcp_ring ] || make -s -C oracle
echo "{\"host\": \"$(grep -m1 'model name' /proc/cpuinfo | cut -d: -f2 | sed 's/^ *//')\", \"nproc\": $(nproc)}"
run() { timeout -k 5 600 ./oracle/tcp_ring "$@" || exit 1; }
run -n 2 -c 1024 -i 500 -w 10                     # cfg1: 4 KiB fp32, 2 ranks
for n in 2 4 8; do run -n $n -c 262144 -i 20 -w 2; done      # 1 MiB (cfg5's bucket)
for n in 2 4 8; do run -n $n -c 67108864 -i 3 -w 1; done     # 256 MiB (cfg2 at n=2)
run -n 8 -c 268435456 -i 2 -w 1                   # cfg3: 1 GiB fp32, 8 ranks
