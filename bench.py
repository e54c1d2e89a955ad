#!/usr/bin/env python
"""Benchmark of the MI355X rdc allreduce path (BASELINE.json metric:
"allreduce GB/s (device-resident fp32) at 1/2/4/8 GPUs; % xGMI roofline").

    python bench.py --gpus N --steps K --warmup W
    (N>1 under a launcher: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...;
     N>1 without one, WORLD_SIZE unset: bench.py starts that launcher itself as a child process)

Workload: a 1 GiB fp32 buffer per GPU (the cfg3 buffer), synthetic data
from the device generator, resident in HBM before timing starts.
  N = 1 : one "step" = the reduce kernel alone (op::Reducer<Sum,float>,
          include/core/mpi.h:113-120): dst += src over the 1 GiB buffer —
          the north star's 1-GPU data point (an allreduce over one rank moves
          nothing).  HBM-bound: 3 x S algorithmic bytes per launch.
  N > 1 : one step = one in-place allreduce of the buffer across the N ranks
          (one process per GPU, HIP IPC over xGMI), bit-identical to the
          reference's ring.  xGMI-bound: 2(N-1)/N x S egress bytes per GPU.
value: N = 1 -> S / t of the reduce kernel (algbw of dst += src);
       N > 1 -> busbw = S / t x 2(N-1)/N (nccl-tests convention, SURVEY.md
       8(d)), with algbw = S / t beside it
(t = wall time of the K timed steps, max over ranks, barrier+sync brackets).
When ranks share a GPU (rehearsals on a 1-GPU box) every byte moves through
one HBM and no xGMI link is exercised: the roofline is reported as
bound "shared-hbm" with frac null.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md)
XGMI_LINK_DIR_GBPS = 76.8     # one xGMI link, one direction (153.6 GB/s bidirectional)
BIDIR_RING_GBPS = 153.6       # north-star roofline: two counter-rotating rings (busbw)
DTYPES = {"float32": (6, 4), "float16": (10, 2), "bfloat16": (11, 2), "float64": (7, 8)}
DT_SHORT = {"float32": "f32", "float16": "f16", "bfloat16": "bf16", "float64": "f64"}
CXX_TYPE = {"float32": "float", "float16": "_Float16", "bfloat16": "bf16_t", "float64": "double"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--bytes", type=int, default=1 << 30, help="buffer size per GPU")
    ap.add_argument("--dtype", default="float32", choices=sorted(DTYPES))
    ap.add_argument("--algo", default="auto", choices=["auto", "mesh", "mesh_pull", "ring", "oneshot", "direct"])
    ap.add_argument("--buckets", type=int, default=1,
                    help="N>1: split the buffer into this many equal buckets (cfg5: --buckets 1024)")
    ap.add_argument("--unfused", action="store_true", help="buckets as separate allreduce calls (no coalescing)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget (0 = skip)")
    ap.add_argument("--no-check", action="store_true", help="skip the post-run oracle spot check")
    ap.add_argument("--rccl-steps", type=int, default=10,
                    help="N>1: also time RCCL's allreduce of the same buffer (child processes, 0 = skip)")
    ap.add_argument("--extra-steps", type=int, default=5,
                    help="N>1: also time cfg4 (fp16) and cfg5 (1024 buckets) this many steps after the timed region")
    ap.add_argument("--ring-steps", type=int, default=5,
                    help="N>1: also time the reference's ring schedule this many steps after the timed region")
    ap.add_argument("--extras-budget-s", type=float, default=200.0,
                    help="N>1: wall-clock budget (s) of everything after the timed region, agreed across ranks; "
                         "extras that do not fit are skipped and listed in extras_skipped")
    ap.add_argument("--autotune-reps", type=int, default=3,
                    help="N>1: before the warm-up, RdcCommAutotune times the launch shapes (role split, grid, "
                         "tile) for this buffer size on this node and keeps the fastest (0 = library defaults)")
    return ap.parse_args()


def load_traffic(kernel_key):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (or None).
    The summary lives at the top of the tree (traffic.json), not under
    profiles/, which .gpurunignore keeps off the GPU box (the
    round-4 bench line's traffic was null for that reason)."""
    path = os.path.join(ROOT, "traffic.json")
    try:
        with open(path) as f:
            return json.load(f).get(kernel_key)
    except (OSError, ValueError):
        return None


def hbm_model(lib, world, count, dt_enum, algo_name):
    """RdcPlanHbmBytes for the schedule the timed launches used: per-rank
    (max) and all-rank loads / stores of one allreduce, or None."""
    algo = {"ring": 1, "mesh": 2, "oneshot": 3, "tree": 4, "mesh_pull": 5, "direct": 6}.get(algo_name)
    if algo is None:
        return None
    out = (ctypes.c_uint64 * 5)()
    if lib.RdcPlanHbmBytes(world, count, dt_enum, algo, out) != 0:
        return None
    return {"read": int(out[0]), "write": int(out[1]), "read_sum": int(out[2]), "write_sum": int(out[3]),
            "egress": int(out[4])}


def cpu_baseline(nbytes_workload, seconds):
    """Reference op::Reducer<Sum,float> (oracle/_ref, the reference's own header
    compiled -O2) or, if absent, the C oracle port, single thread, on a bounded
    256 MiB sample of the same dst += src workload."""
    import numpy as np
    from oracle import oracle as O
    if seconds <= 0:
        return None
    n = min(nbytes_workload, 256 << 20) // 4
    dst = np.ones(n, dtype=np.float32)
    src = np.full(n, 0.5, dtype=np.float32)
    ref = O.ref() if O.ref_available() else None
    fn = (lambda: ref.ref_reducer(dst.ctypes.data, src.ctypes.data, n, 6, 2)) if ref else \
        (lambda: O.lib().rdc_oracle_reducer(dst.ctypes.data, src.ctypes.data, n, 6, 2))
    fn()  # page in
    reps, t0 = 0, time.perf_counter()
    while True:
        fn()
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {
        "value": round(n * 4 * reps / el / 1e9, 3),
        "unit": "GB/s",
        "cores": 1,
        "kind": "reference" if ref else "port",
        "sample": "op::Reducer<Sum,float> dst += src over a %d MiB fp32 buffer, %d reps in %.1f s, 1 thread "
                  "(value = buffer bytes / time, same unit as the GPU line; HBM-equivalent traffic 3x)"
                  % (n * 4 >> 20, reps, el),
    }


def sync_check(comm, sp, dist, torch):
    """Synchronise, read this rank's device error word, and agree over the CPU
    process group: every rank raises if any rank failed, so all ranks leave a
    failed step together (no rank waits in a barrier its peers never reach)."""
    err = ""
    try:
        torch.cuda.synchronize()
        comm.check(sp)
    except Exception as e:  # noqa: BLE001 - re-raised below on every rank
        err = str(e)[:300] or "error"
    f = torch.tensor([1.0 if err else 0.0], dtype=torch.float64)
    dist.all_reduce(f, op=dist.ReduceOp.MAX)
    if float(f[0]) > 0:
        raise RuntimeError(err or "failed on another rank")


def timed_ms(one, comm, sp, dist, torch, steps, warm=2, synchronous=False):
    """ms per call of one(), max over ranks, after `warm` checked calls.
    synchronous: one() has completed when it returns (host-buffer calls), so
    the clock stops at the end of the loop; otherwise after a device sync and
    a barrier (stream-ordered launches)."""
    for _ in range(warm):
        one()
    sync_check(comm, sp, dist, torch)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        one()
    if not synchronous:
        torch.cuda.synchronize()
        dist.barrier()
    t = torch.tensor([(time.perf_counter() - t0) / steps], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    sync_check(comm, sp, dist, torch)
    return float(t[0]) * 1e3


def time_ring(lib, comm, buf, count, dt_enum, sp, dist, torch, steps):
    """ms per in-place allreduce with the reference's ring schedule (k_ring),
    max over ranks, after 2 warm-up launches."""
    from rdc_amd._lib import check_call

    def one():
        check_call(lib.RdcCommAllreduceEx(comm.handle, ctypes.c_void_p(buf.data_ptr()), count, dt_enum, 2, 1, sp))
    return timed_ms(one, comm, sp, dist, torch, steps)


def time_extra_configs(lib, comm, S, world, rank, sp, dist, torch, steps, out, autotune_reps=0, budget=None):
    """The other BASELINE.json configs on the same communicator, after the
    timed region (informational): cfg4 = fp16 allreduce of a buffer of S
    bytes, cfg5 = 1024 buckets of S/1024 bytes fp32 in one coalesced call,
    cfg1 = a 4 KiB fp32 allreduce of HOST memory through the reference's own
    entry point (RdcAllreduce on a numpy array: pinned zero-copy launch, the
    real host path) and cfg2's 256 MiB fp32 buffer, with a device size curve
    4 KiB - 256 MiB (`sizes_fp32`: the automatic rule's schedule and shape,
    then, with autotune on, the same size after RdcCommAutotune for its size
    class).  ms per step = max over ranks of the wall time of `steps` calls.
    Fills `out` as it goes."""
    from rdc_amd._lib import check_call
    import numpy as np
    import rdc_amd

    def timed(one, nsteps=steps):
        return timed_ms(one, comm, sp, dist, torch, nsteps)

    def entry(ms, nbytes, what, nsteps=steps, device=True):
        bb = nbytes / (ms * 1e-3) / 1e9 * 2 * (world - 1) / world
        e = {"workload": what, "bytes_per_gpu": nbytes, "ms_per_step": round(ms, 4), "busbw_GBps": round(bb, 2),
             "steps": nsteps}
        if device:  # the schedule the last timed call launched (RdcCommLastLaunch)
            ll = (ctypes.c_uint64 * 6)()
            check_call(lib.RdcCommLastLaunch(comm.handle, ll))
            e["schedule"] = {1: "ring", 2: "mesh", 3: "oneshot", 4: "tree", 5: "mesh_pull", 6: "direct"}.get(int(ll[5]))
        return e

    h = torch.empty(S // 2, dtype=torch.float16, device="cuda")
    rdc_amd.fill_(h, 0x5EED0000, rank)
    ms = timed(lambda: check_call(lib.RdcCommAllreduceEx(comm.handle, ctypes.c_void_p(h.data_ptr()), h.numel(),
                                                         10, 2, 0, sp)))
    out["cfg4_fp16"] = entry(ms, S, "in-place allreduce(sum) of a %d MiB float16 buffer (packed half "
                                    "reduce kernel)" % (S >> 20))
    del h
    K = 1024
    per = S // 4 // K
    bks = [torch.empty(per, dtype=torch.float32, device="cuda") for _ in range(K)]
    for b, t in enumerate(bks):
        rdc_amd.fill_(t, 0x5EED0000 + b, rank)
    ptrs = (ctypes.c_void_p * K)(*[t.data_ptr() for t in bks])
    cnts = (ctypes.c_size_t * K)(*([per] * K))
    ms = timed(lambda: check_call(lib.RdcCommAllreduceCoalesced(comm.handle, ptrs, cnts, K, 6, 2, 0, sp)))
    out["cfg5_buckets"] = entry(ms, per * 4 * K, "%d x %d KiB float32 buckets, one coalesced call "
                                                 "(test/mallreduce.cc shape)" % (K, per * 4 >> 10))
    del bks
    # cfg1 on the real path: 4 KiB of fp32 in pageable host memory through
    # RdcAllreduce (rdc/core.py's entry point), synchronous per call
    a = np.ones(1024, dtype=np.float32)
    pa = ctypes.c_void_p(a.ctypes.data)
    ms = timed_ms(lambda: check_call(lib.RdcAllreduce(pa, 1024, 6, 2, None, None)), comm, sp, dist, torch,
                  max(steps, 2000), warm=20, synchronous=True)
    e = entry(ms, 4096, "4 KiB float32 allreduce of HOST memory via RdcAllreduce (cfg1 shape, synchronous; "
              "clock stops when the last call returns, max over ranks)", max(steps, 2000), device=False)
    e["us_per_call"] = round(ms * 1e3, 2)
    out["cfg1_host_4KiB"] = e
    # the PCIe-inclusive rate (north star: rdc buffers begin and end in host
    # memory): 64 MiB of fp32 in pageable host memory through RdcAllreduce,
    # i.e. the host pipeline (copy in, H2D, allreduce, D2H) with each rank on
    # its own link when ranks have a GPU each
    if budget is None or budget.left() >= 15:
        hb = np.ones(16 << 20, dtype=np.float32)
        ph = ctypes.c_void_p(hb.ctypes.data)
        ms = timed_ms(lambda: check_call(lib.RdcAllreduce(ph, hb.size, 6, 2, None, None)), comm, sp, dist, torch, 5,
                      warm=2, synchronous=True)
        e = entry(ms, hb.nbytes, "64 MiB float32 allreduce of HOST (pageable) memory via RdcAllreduce: copy in, "
                  "H2D, allreduce, D2H, pipelined (PCIe-inclusive; synchronous, max over ranks)", 5, device=False)
        e["algbw_GBps_pcie_inclusive"] = round(hb.nbytes / (ms * 1e-3) / 1e9, 2)
        out["host_64MiB"] = e
        del hb
    else:
        out.setdefault("skipped", []).append("host_64MiB")
    # the same 64 MiB in a registered RdcNewBuffer(pinned=1) range: the DMA
    # engines read and write the caller's pages in place (no copy in)
    if budget is None or budget.left() >= 15:
        import mmap
        mm = mmap.mmap(-1, 64 << 20)
        hb = np.frombuffer(mm, dtype=np.float32)
        hb[:] = 1.0
        reg = ctypes.c_void_p()
        check_call(lib.RdcNewBuffer(ctypes.byref(reg), ctypes.c_void_p(hb.ctypes.data), hb.nbytes, 1))
        try:
            ph = ctypes.c_void_p(hb.ctypes.data)
            ms = timed_ms(lambda: check_call(lib.RdcAllreduce(ph, hb.size, 6, 2, None, None)), comm, sp, dist, torch,
                          5, warm=2, synchronous=True)
        finally:
            check_call(lib.RdcDelBuffer(reg))
        e = entry(ms, hb.nbytes, "64 MiB float32 allreduce of HOST memory registered with RdcNewBuffer(pinned=1) "
                  "via RdcAllreduce: H2D, allreduce, D2H in place, pipelined (PCIe-inclusive; synchronous, max "
                  "over ranks)", 5, device=False)
        e["algbw_GBps_pcie_inclusive"] = round(hb.nbytes / (ms * 1e-3) / 1e9, 2)
        out["host_64MiB_registered"] = e
        del hb
    else:
        out.setdefault("skipped", []).append("host_64MiB_registered")
    # the north star's host-inclusive rate at cfg3's size: 1 GiB of fp32 in
    # pageable host memory through RdcAllreduce (copy in, H2D, allreduce, D2H,
    # pipelined in 16 MiB pieces), one warm-up and two timed calls
    if budget is None or budget.left() >= 40:
        hb = np.ones(S // 4, dtype=np.float32)
        ph = ctypes.c_void_p(hb.ctypes.data)
        ms = timed_ms(lambda: check_call(lib.RdcAllreduce(ph, hb.size, 6, 2, None, None)), comm, sp, dist, torch, 2,
                      warm=1, synchronous=True)
        e = entry(ms, hb.nbytes, "%d MiB float32 allreduce of HOST (pageable) memory via RdcAllreduce: copy in, "
                  "H2D, allreduce, D2H, pipelined (PCIe-inclusive; synchronous, max over ranks)" % (S >> 20), 2,
                  device=False)
        e["algbw_GBps_pcie_inclusive"] = round(hb.nbytes / (ms * 1e-3) / 1e9, 2)
        out["host_1GiB"] = e
        del hb
    else:
        out.setdefault("skipped", []).append("host_1GiB")
    # cfg2's 256 MiB fp32 buffer and the sizes below it (prefixes of one
    # buffer): where the mesh's per-launch fill / drain and the one-shot
    # hand-off decide the rate, for the size thresholds at this rank count
    big = min(S, 256 << 20)
    f = torch.empty(big // 4, dtype=torch.float32, device="cuda")
    rdc_amd.fill_(f, 0x5EED0000, rank)
    sizes = {}
    out["sizes_fp32"] = sizes
    for nb in (4 << 10, 64 << 10, 1 << 20, 4 << 20, 16 << 20, 64 << 20, big):
        if nb > big:
            continue
        if budget is not None and budget.left() < 8:
            out.setdefault("skipped", []).append("sizes_fp32[%d]" % nb)
            continue
        # small calls: enough of them that the closing device sync + barrier
        # (~1 ms with gloo) is noise (50 calls made it 20 us of a 4 KiB call)
        ns = max(steps, 2000 if nb <= (64 << 10) else 400 if nb <= (1 << 20) else 50 if nb <= (16 << 20) else 0)
        def one():
            check_call(lib.RdcCommAllreduceEx(comm.handle, ctypes.c_void_p(f.data_ptr()), nb // 4, 6, 2, 0, sp))
        ms = timed(one, ns)
        e = entry(ms, nb, "in-place allreduce(sum) of %d KiB float32" % (nb >> 10), ns)
        sizes[str(nb)] = {k: e[k] for k in ("ms_per_step", "busbw_GBps", "steps", "schedule")}
        if autotune_reps > 0 and nb < S:
            t = comm.autotune(nb, 6, reps=autotune_reps, stream=sp)
            if t["chosen"] is not None:
                ms_t = timed(one, ns)
                sizes[str(nb)].update({"tuned_ms_per_step": round(ms_t, 4),
                                       "tuned_busbw_GBps": round(nb / (ms_t * 1e-3) / 1e9 * 2 * (world - 1)
                                                                 / world, 2),
                                       "tuned": {k: t["chosen"][k] for k in ("schedule", "split", "grid",
                                                                             "tiles_per_block")}})
        if nb == (256 << 20):
            e.update({k: v for k, v in sizes[str(nb)].items() if k.startswith("tuned")})
            out["cfg2_256MiB"] = e
    del f
    return out


class Budget(object):
    """Wall-clock budget of the informational extras after the timed region,
    agreed across ranks: left() is the same number on every rank (the
    slowest rank's elapsed time, MAX over the CPU process group), so every
    rank takes the same skip decision and no rank waits in a collective its
    peers skipped."""

    def __init__(self, seconds, dist, torch, world):
        self.limit, self.dist, self.torch, self.world = float(seconds), dist, torch, world
        self.t0 = time.perf_counter()

    def elapsed(self):
        el = time.perf_counter() - self.t0
        if self.world > 1:
            t = self.torch.tensor([el], dtype=self.torch.float64)
            self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
            el = float(t[0])
        return el

    def left(self):
        return self.limit - self.elapsed()


def parity_checks(lib, comm, S, world, rank, sp, dist, torch, out, budget=None):
    """Bit-exact checks at the bench's own shapes (after all timing), each on
    fresh synthetic inputs, every key its own boolean (AND over ranks):

    * cfg3_direct / cfg3_mesh / cfg3_ring / cfg3_mesh_pull / cfg4_fp16: ONE allreduce of the whole S-byte
      buffer.  Every rank hashes its WHOLE result (sha256) and the ranks
      compare digests; rank r compares Split chunk r of its result, every
      element, with the oracle's ring order.  Identical digests + every chunk
      verified on some rank = every byte of every rank's buffer verified:
      every tile of every chunk, i.e. every hand-off the schedule made.
    * cfg5_buckets: 1024 buckets in one coalesced call; digests over all
      buckets compared across ranks, rank r verifies buckets b = r mod n
      whole (so every bucket, every chunk boundary).
    * oneshot_512KiB: four back-to-back one-shot launches (no host sync in
      between: the slot halves are reused while peers may still read), every
      result whole on every rank.
    * service_host_4KiB: eight synchronous 4 KiB fp32 HOST-buffer allreduces
      through RdcAllreduce (the small-allreduce service's LL-word exchange
      where it runs, the launch path otherwise), every result whole.
    * tree_order: a 64 KiB + 12 B fp32 buffer in the reference's tree order
      (algo 4 = what rdc_reduce_ring_mincount selects), against the oracle's
      restated tree.
    * broadcast_nonzero_root: 8 MiB + 12 B from root n-1 (forwarded through
      the other ranks at n >= 3), every byte on every rank.
    * allgather_varsize: per-rank sizes 1 MiB + c x 4100 B, every buffer on
      every rank.
    """
    from rdc_amd._lib import check_call
    import hashlib
    from oracle import oracle as O

    t_start = time.perf_counter()
    wall = {}

    def agree(ok):
        f = torch.tensor([0.0 if ok else 1.0], dtype=torch.float64)
        dist.all_reduce(f, op=dist.ReduceOp.MAX)
        return float(f[0]) == 0.0

    def identical(host_bytes):
        """Every rank holds the same bytes (sha256 compared over gloo)."""
        d = hashlib.sha256(host_bytes).hexdigest()
        ds = [None] * world
        dist.all_gather_object(ds, d)
        return all(x == d for x in ds)

    def host_u8(t):
        return t.cpu().contiguous().view(torch.uint8).numpy()

    def verify_range(u8, total, lo, hi, dt, seed, esz, block=1 << 20):
        """Elements [lo, hi) of a `total`-element result vs the oracle's ring
        order, block by block (the oracle computes each window alone)."""
        for st in range(lo, hi, block):
            m = min(block, hi - st)
            want = O.expected_window(total, st, m, world, dt, 2, seed)
            if u8[st * esz:(st + m) * esz].tobytes() != want.tobytes():
                return False
        return True

    def fill(t, count, dt, seed, r):
        check_call(lib.RdcFill(ctypes.c_void_p(t.data_ptr()), count, dt, seed, r, sp))

    def should_run(name, need_s):
        if budget is not None and budget.left() < need_s:
            out.setdefault("skipped", []).append(name)
            return False
        return True

    for name, dt, algo, tdt in (("cfg3_direct", 6, 6, torch.float32), ("cfg3_mesh", 6, 2, torch.float32),
                                ("cfg3_ring", 6, 1, torch.float32), ("cfg3_mesh_pull", 6, 5, torch.float32),
                                ("cfg4_fp16", 10, 0, torch.float16)):
        if not should_run(name, 20):
            continue
        t0 = time.perf_counter()
        esz = 4 if dt == 6 else 2
        count = S // esz
        t = torch.empty(count, dtype=tdt, device="cuda")
        seed = 0x5EED1000 + dt * 16 + algo
        fill(t, count, dt, seed, rank)
        check_call(lib.RdcCommAllreduceEx(comm.handle, ctypes.c_void_p(t.data_ptr()), count, dt, 2, algo, sp))
        sync_check(comm, sp, dist, torch)
        ll = (ctypes.c_uint64 * 6)()
        check_call(lib.RdcCommLastLaunch(comm.handle, ll))
        out.setdefault("schedule", {})[name] = {1: "ring", 2: "mesh", 3: "oneshot", 4: "tree", 5: "mesh_pull",
                                                6: "direct"}.get(int(ll[5]), int(ll[5]))
        u8 = host_u8(t)
        del t
        lo, hi = O.split(count, world)[rank]
        ok = verify_range(u8, count, lo, hi, dt, seed, esz)
        out[name] = agree(ok) and identical(u8.data)
        del u8
        wall[name] = round(time.perf_counter() - t0, 2)
    if should_run("cfg5_buckets", 20):
        t0 = time.perf_counter()
        K = 1024
        per = S // 4 // K
        bks = [torch.empty(per, dtype=torch.float32, device="cuda") for _ in range(K)]
        for b, t in enumerate(bks):
            fill(t, per, 6, 0x5EED2000 + b, rank)
        ptrs = (ctypes.c_void_p * K)(*[t.data_ptr() for t in bks])
        cnts = (ctypes.c_size_t * K)(*([per] * K))
        check_call(lib.RdcCommAllreduceCoalesced(comm.handle, ptrs, cnts, K, 6, 2, 0, sp))
        sync_check(comm, sp, dist, torch)
        u8 = host_u8(torch.cat(bks))
        del bks
        ok = all(verify_range(u8[b * per * 4:(b + 1) * per * 4], per, 0, per, 6, 0x5EED2000 + b, 4)
                 for b in range(rank, K, world))
        out["cfg5_buckets"] = agree(ok) and identical(u8.data)
        del u8
        wall["cfg5_buckets"] = round(time.perf_counter() - t0, 2)
    if should_run("oneshot_512KiB", 5):
        t0 = time.perf_counter()
        count = (512 << 10) // 4
        ts = [torch.empty(count, dtype=torch.float32, device="cuda") for _ in range(4)]
        for k, t in enumerate(ts):
            fill(t, count, 6, 0x5EED4000 + k, rank)
        for t in ts:  # back to back on one stream: consecutive launches alternate slot halves
            check_call(lib.RdcCommAllreduceEx(comm.handle, ctypes.c_void_p(t.data_ptr()), count, 6, 2, 3, sp))
        sync_check(comm, sp, dist, torch)
        ok = all(host_u8(t).tobytes() == O.expected_window(count, 0, count, world, 6, 2, 0x5EED4000 + k).tobytes()
                 for k, t in enumerate(ts))
        out["oneshot_512KiB"] = agree(ok)
        wall["oneshot_512KiB"] = round(time.perf_counter() - t0, 2)
    if should_run("service_host_4KiB", 5):
        t0 = time.perf_counter()
        ok = True
        g = torch.empty(1024, dtype=torch.float32, device="cuda")
        for k in range(8):
            fill(g, 1024, 6, 0x5EED5000 + k, rank)  # the device generator: same values as the oracle's
            torch.cuda.synchronize()
            a = g.cpu().numpy().copy()             # pageable host memory, as rdc/core.py passes it
            check_call(lib.RdcAllreduce(ctypes.c_void_p(a.ctypes.data), 1024, 6, 2, None, None))
            ok = ok and a.tobytes() == O.expected_window(1024, 0, 1024, world, 6, 2, 0x5EED5000 + k).tobytes()
        out["service_host_4KiB"] = agree(ok)
        wall["service_host_4KiB"] = round(time.perf_counter() - t0, 2)
    if should_run("tree_order", 5):
        t0 = time.perf_counter()
        count = (64 << 10) // 4 + 3
        t = torch.empty(count, dtype=torch.float32, device="cuda")
        fill(t, count, 6, 0x5EED6000, rank)
        check_call(lib.RdcCommAllreduceEx(comm.handle, ctypes.c_void_p(t.data_ptr()), count, 6, 2, 4, sp))
        sync_check(comm, sp, dist, torch)
        want = O.expected_tree([O.fill(count, 6, 0x5EED6000, r) for r in range(world)], 6, 2)
        out["tree_order"] = agree(host_u8(t).tobytes() == want.tobytes())
        wall["tree_order"] = round(time.perf_counter() - t0, 2)
    if should_run("broadcast_nonzero_root", 5):
        t0 = time.perf_counter()
        root = world - 1
        count = (8 << 20) // 4 + 3
        t = torch.empty(count, dtype=torch.float32, device="cuda")
        fill(t, count, 6, 0x5EED7000 if rank == root else 0x5EED7001, rank)
        check_call(lib.RdcCommBroadcast(comm.handle, ctypes.c_void_p(t.data_ptr()), count * 4, root, sp))
        sync_check(comm, sp, dist, torch)
        out["broadcast_nonzero_root"] = agree(host_u8(t).tobytes() == O.fill(count, 6, 0x5EED7000, root).tobytes())
        wall["broadcast_nonzero_root"] = round(time.perf_counter() - t0, 2)
    if should_run("allgather_varsize", 5):
        t0 = time.perf_counter()
        counts = [(1 << 18) + 1025 * c for c in range(world)]
        bufs = [torch.zeros(c, dtype=torch.float32, device="cuda") for c in counts]
        fill(bufs[rank], counts[rank], 6, 0x5EED8000, rank)
        ptrs = (ctypes.c_void_p * world)(*[b.data_ptr() for b in bufs])
        sizes = (ctypes.c_size_t * world)(*[4 * c for c in counts])
        check_call(lib.RdcCommAllgather(comm.handle, ptrs, sizes, sp))
        sync_check(comm, sp, dist, torch)
        ok = all(host_u8(b).tobytes() == O.fill(counts[c], 6, 0x5EED8000, c).tobytes() for c, b in enumerate(bufs))
        out["allgather_varsize"] = agree(ok)
        wall["allgather_varsize"] = round(time.perf_counter() - t0, 2)
    out["wall_s"] = wall
    out["method"] = ("fresh synthetic inputs per check.  cfg3/cfg4: one allreduce of the whole buffer; rank r "
                     "compares every element of Split chunk r with the oracle's ring order and the ranks compare "
                     "sha256 digests of their whole results (identical digests + every chunk verified on some "
                     "rank = every byte of every rank verified).  cfg5: the same over 1024 buckets (rank r "
                     "verifies buckets r mod n whole).  oneshot / service / tree / broadcast / allgather: every "
                     "result whole on every rank.  Each key is the AND over ranks.")
    out["seconds"] = round(time.perf_counter() - t_start, 2)
    return out


def rccl_compare(S, world, rank, local, dist, torch, steps, limit_s=150.0):
    """The same allreduce through RCCL (torch.distributed nccl backend), one
    child process per rank (tools/rccl_allreduce.py), after every rdc
    measurement and under a time limit inside the extras budget:
    informational, never costs the line.
    Skipped when ranks share a GPU (RCCL needs one rank per device)."""
    import subprocess
    if torch.cuda.device_count() < world:
        return {"skipped": "ranks share a GPU (RCCL needs one GPU per rank)"}
    addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = int(os.environ.get("MASTER_PORT", "29500")) + 7
    dist.barrier()
    cmd = [sys.executable, os.path.join(ROOT, "tools", "rccl_allreduce.py"), str(rank), str(world), str(local), addr,
           str(port), str(S), str(steps)]
    res = {"error": "no result"}
    try:
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=max(10.0, limit_s))
        lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
        if lines:
            res = json.loads(lines[-1])
        elif p.returncode != 0:
            res = {"error": "rc=%d: %s" % (p.returncode, p.stderr[-300:])}
    except subprocess.TimeoutExpired:
        res = {"error": "timed out after %.0f s" % max(10.0, limit_s)}
    except Exception as e:  # noqa: BLE001 - informational only
        res = {"error": str(e)}
    dist.barrier()
    return res


def cpu_tcp_ring(S, world, rank, dist):
    """A PORT of the reference's CPU ring allreduce over loopback TCP
    (oracle/tcp_ring: a C restatement of TryAllreduceRing's schedule and
    op::Reducer over one TCP socket per ring link, without the reference's
    epoll poller, thread pool or its partial-write liveness bug - the shipped
    reference does not build, SURVEY finding 1) at this run's
    rank count, on a bounded 64 MiB fp32 sample, rank 0 only, after every GPU
    measurement (a reported baseline, informational)."""
    import subprocess
    res = None
    if rank == 0:
        exe = os.path.join(ROOT, "oracle", "tcp_ring")
        nb = min(S, 64 << 20)
        try:
            p = subprocess.run([exe, "-n", str(world), "-c", str(nb // 4), "-i", "3", "-w", "1"], capture_output=True,
                               text=True, timeout=120)
            lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
            res = json.loads(lines[-1]) if lines else {"error": "rc=%d: %s" % (p.returncode, p.stderr[-300:])}
            res["sample"] = "%d ranks as processes, one thread each, %d MiB fp32, median of 3 calls" % (world, nb >> 20)
            res["kind"] = "port"
            res["cores"] = world
        except Exception as e:  # noqa: BLE001 - informational only
            res = {"error": str(e)}
    dist.barrier()
    return res


def trace_roles(lib, comm, buf, count, dt_enum, sp, dist, torch):
    """One traced allreduce (RdcCommTraceNext) after the timed region: when
    each block role started and finished, relative to the launch's first
    block (max over ranks), in microseconds (wall_clock64 = 100 MHz).  Tells
    which role bounds the schedule on real links."""
    import numpy as np
    from rdc_amd._lib import check_call
    words = 2 * 8192
    tr = torch.zeros(words, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    dist.barrier()
    check_call(lib.RdcCommTraceNext(comm.handle, ctypes.c_void_p(tr.data_ptr()), words))
    check_call(lib.RdcCommAllreduceEx(comm.handle, ctypes.c_void_p(buf.data_ptr()), count, dt_enum, 2, 0, sp))
    sync_check(comm, sp, dist, torch)
    ll = (ctypes.c_uint64 * 6)()
    check_call(lib.RdcCommLastLaunch(comm.handle, ll))
    grid, s, r, g, tile, algo = [int(x) for x in ll]
    t = tr[:2 * grid].cpu().numpy().view(np.uint64).reshape(grid, 2).astype(np.float64)
    t0 = t[:, 0].min()
    dump = os.environ.get("RDC_BENCH_TRACE_DUMP")  # per-rank raw {start, end} ticks per block
    if dump:
        np.save("%s.rank%d.npy" % (dump, dist.get_rank()), np.concatenate([[grid, s, r, g, tile, algo], t.ravel()]))
    names = {1: "ring", 2: "mesh", 3: "oneshot", 5: "mesh_pull", 6: "direct"}
    roles = {"all": (0, grid)} if algo not in (2, 5) else {"scatter": (0, s), "reduce": (s, s + r),
                                                           "gather": (s + r, grid)}
    vals = []
    for lo, hi in roles.values():
        seg = t[lo:hi]
        vals += [(seg[:, 0].min() - t0) / 100.0, (seg[:, 1].max() - t0) / 100.0, float(np.mean(seg[:, 1] - seg[:, 0])) / 100.0]
    v = torch.tensor(vals, dtype=torch.float64)
    dist.all_reduce(v, op=dist.ReduceOp.MAX)
    out = {"schedule": names.get(algo, str(algo)), "grid": grid, "tile_bytes": tile,
           "blocks": {"scatter": s, "reduce": r, "gather": g} if algo in (2, 5) else {"all": grid}}
    for i, k in enumerate(roles):
        out[k + "_us"] = {"first_start": round(float(v[3 * i]), 1), "last_end": round(float(v[3 * i + 1]), 1),
                          "mean_block_busy": round(float(v[3 * i + 2]), 1)}
    return out


def xgmi_probe(lib, comm, sp, dist, torch, nbytes=256 << 20, reps=5):
    """Measured link rates (outside the timed region, every rank idle): the
    copy kernel the collectives use pushes nbytes from each GPU into
    (a) rank+1 only - one link, one direction, every link busy in a ring;
    (b) every peer at once - all n-1 links out of each GPU (the mesh's egress);
    then the same two reading instead (pull: remote loads into local scratch),
    the data for choosing push or pull hand-offs on real xGMI.
    Slowest rank's rate.  On a 1-GPU box the ranks share one HBM."""
    out = {}
    for mode, key in ((0, "one_link_one_direction_GBps"), (1, "all_links_egress_GBps"),
                      (2, "pull_one_link_GBps"), (3, "pull_all_links_GBps")):
        ms, used = ctypes.c_double(), ctypes.c_size_t()
        rc = lib.RdcCommProbe(comm.handle, mode, nbytes, reps, sp, ctypes.byref(ms), ctypes.byref(used))
        err = lib.RdcGetLastError().decode() if rc != 0 else ""
        per_target = used.value
        t = torch.tensor([ms.value, 1.0 if rc != 0 else 0.0], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)  # every rank leaves together on a failure
        if float(t[1]) > 0:
            return {"error": err or "failed on another rank"}
        ntarget = 1 if mode in (0, 2) else int(os.environ.get("WORLD_SIZE", "1")) - 1
        out[key] = round(per_target * ntarget / (float(t[0]) * 1e-3) / 1e9, 2)
        dist.barrier()
    out["bytes_per_target"] = per_target
    out["kernel"] = "k_push (block_copy, 16-B lanes; push = write-through (sc0 sc1) remote stores, pull = remote loads)"
    return out


# Keys every N > 1 line carries, null where ranks share a
# GPU (no link timed) but always present, so an 8-GPU run is decisive:
REQUIRED_MULTI_KEYS = (
    "direct_selfcheck",                      # the channel's self-check at creation (passed / failed / not run)
    "cfg3_schedule.untuned.schedule",        # what a drop-in call gets with no tuning ...
    "cfg3_schedule.untuned.ms_per_step",
    "cfg3_schedule.tuned.schedule",          # ... and what the timed region ran after Autotune
    "cfg3_schedule.tuned.ms_per_step",
    "roofline.frac_of_bidir_ring_roofline",  # north star: >= 0.70 at n = 8
    "roofline.frac_of_measured",             # against this line's own link probe
    "xgmi_link_rates.one_link_one_direction_GBps",
    "xgmi_link_rates.all_links_egress_GBps",
    "host_inclusive_1GiB.algbw_GBps_pcie_inclusive",  # H2D + allreduce + D2H of 1 GiB of host memory
)


def missing_multi_keys(line, need_values=False):
    """REQUIRED_MULTI_KEYS absent from `line` (dotted paths); need_values: also
    the ones whose value is null (a line measured with one rank per GPU)."""
    miss = []
    for path in REQUIRED_MULTI_KEYS:
        cur, ok = line, True
        for part in path.split("."):
            if not isinstance(cur, dict) or part not in cur:
                ok = False
                break
            cur = cur[part]
        if not ok or (need_values and cur is None):
            miss.append(path)
    return miss


def compose_multi(lib, ctx):
    """The N > 1 line's roofline and decisive keys from the run's measurements
    (ctx: world, S, count, esz, dtype, dt_enum, buckets, unfused, algo, steps,
    wall, kern_ms, timed_algo, gpus_here, probe, tuned, direct_selfcheck,
    untuned = {schedule, ms_per_step} or None, host_1g = extra_configs'
    host_1GiB entry or None).  Pure function of ctx (lib only for the HBM
    byte model), so tests/test_bench_line.py checks a mocked 8-GPU line."""
    world, S = ctx["world"], ctx["S"]
    steps, wall, kern_ms = ctx["steps"], ctx["wall"], ctx["kern_ms"]
    gpus_here = ctx["gpus_here"]
    shared = gpus_here < world
    algbw = S / (kern_ms * 1e-3) / 1e9
    busbw = algbw * 2 * (world - 1) / world
    algo_name = ctx["algo"]
    if algo_name == "auto":  # the schedule the library launched in the timed region (RdcCommLastLaunch)
        algo_name = ctx["timed_algo"] or "mesh"
    peak = XGMI_LINK_DIR_GBPS * (1 if algo_name == "ring" else (world - 1))  # mesh / mesh_pull / direct: every link
    probe = ctx["probe"]
    roof = {"bound": "xgmi", "achieved": round(busbw, 2), "peak": round(peak, 1), "unit": "GB/s",
            "frac": round(busbw / peak, 4), "traffic": None,
            "kernel": "k_%s<Sum,%s>" % (algo_name, ctx["dtype"]),
            "algorithmic_bytes_per_launch": int(2 * (world - 1) * S // world), "kernel_avg_ms": round(kern_ms, 4),
            "frac_of_bidir_ring_roofline": round(busbw / BIDIR_RING_GBPS, 4),
            "peak_measured": None, "frac_of_measured": None,
            "xgmi_probe": probe}
    if isinstance(probe, dict) and probe.get("all_links_egress_GBps"):
        meas = probe["one_link_one_direction_GBps"] if algo_name == "ring" else probe["all_links_egress_GBps"]
        roof["peak_measured"] = meas
        roof["frac_of_measured"] = round(busbw / meas, 4)
    # HBM side of the same launches: the committed byte model of the
    # schedule (RdcPlanHbmBytes = rdc_plan.cpp ModelHbmBytes: bytes the
    # kernels load and store, per rank) over the kernel time
    count = ctx["count"] if ctx["buckets"] == 1 else S // ctx["esz"]
    hm = hbm_model(lib, world, count, ctx["dt_enum"], algo_name)
    if hm is not None:
        per_gpu = -(-world // max(1, gpus_here)) if shared else 1   # ranks on one GPU
        moved = hm["read_sum"] + hm["write_sum"] if (shared and gpus_here == 1) else \
            per_gpu * (hm["read"] + hm["write"])
        ach = moved / (kern_ms * 1e-3) / 1e9
        hb = {"model": "rdc_plan.cpp ModelHbmBytes (RdcPlanHbmBytes): loads + stores the schedule's kernels "
                       "issue, remote stores counted at the issuing rank",
              "read_bytes_per_rank": hm["read"], "write_bytes_per_rank": hm["write"], "ranks_on_gpu": per_gpu,
              "bytes_per_step": int(moved), "achieved": round(ach, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
              "frac": round(ach / HBM_PEAK_GBPS, 4)}
        # rank 0's own L2-to-memory bytes (rocprofv3 PMC, FETCH_SIZE x 2 +
        # WRITE_SIZE, the other ranks unprofiled: tools/pmc_rank0.sh),
        # committed per (schedule, dtype, n, S) in traffic.json
        tr = load_traffic("%s_%s_n%d_%d" % (algo_name, DT_SHORT[ctx["dtype"]], world, S))
        hb["traffic_per_rank"] = tr
        hb["traffic_over_model"] = round(tr / (hm["read"] + hm["write"]), 4) if tr else None
        roof["shared_hbm" if shared else "hbm"] = hb
    if shared:
        # every rank's bytes move through ONE HBM: no xGMI link is timed,
        # so no xGMI fraction is meaningful (round 1 printed 7.996 here)
        roof.update({"bound": "shared-hbm", "peak": None, "frac": None, "frac_of_bidir_ring_roofline": None,
                     "frac_of_measured": None,
                     "note": "%d ranks share %d GPU(s): rehearsal of the protocol, not an xGMI measurement; "
                             "roofline.shared_hbm is the one HBM all ranks' bytes move through"
                             % (world, gpus_here)})
    keys = {}
    keys["direct_selfcheck"] = ctx["direct_selfcheck"]
    unt = ctx.get("untuned")
    tuned = ctx.get("tuned")
    tuned_ok = isinstance(tuned, dict) and tuned.get("chosen") is not None
    keys["cfg3_schedule"] = {
        "untuned": {"schedule": unt.get("schedule") if unt else None,
                    "ms_per_step": unt.get("ms_per_step") if unt else None,
                    "busbw_GBps": round(S / (unt["ms_per_step"] * 1e-3) / 1e9 * 2 * (world - 1) / world, 2)
                    if unt and unt.get("ms_per_step") else None,
                    "note": "the library's default for this buffer with no RdcCommAutotune (what rdc::Allreduce / "
                            "rdc.allreduce get), timed before the autotune"},
        "tuned": {"schedule": algo_name, "ms_per_step": round(wall / steps * 1e3, 4),
                  "busbw_GBps": round(S / (wall / steps) / 1e9 * 2 * (world - 1) / world, 2),
                  "source": "RdcCommAutotune on this node" if tuned_ok else "library defaults (no autotune)"},
    }
    rates = probe if isinstance(probe, dict) else {}
    keys["xgmi_link_rates"] = {k: rates.get(k) for k in ("one_link_one_direction_GBps", "all_links_egress_GBps",
                                                          "pull_one_link_GBps", "pull_all_links_GBps")}
    keys["xgmi_link_rates"]["note"] = ("slowest rank, k_push copy kernel, %s" % (
        "ranks share one GPU: HBM, not xGMI" if shared else "one rank per GPU")) if rates else \
        (probe.get("error") if isinstance(probe, dict) else "not measured")
    h1 = ctx.get("host_1g")
    keys["host_inclusive_1GiB"] = {
        "algbw_GBps_pcie_inclusive": h1.get("algbw_GBps_pcie_inclusive") if isinstance(h1, dict) else None,
        "ms_per_step": h1.get("ms_per_step") if isinstance(h1, dict) else None,
        "workload": "1 GiB float32 of pageable HOST memory through RdcAllreduce (copy in, H2D, allreduce, D2H); "
                    "never the headline value (DESIGN.md 7.5)"}
    return roof, algo_name, keys


def free_port():
    import socket
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def self_launch_cmd(gpus, argv, port):
    """The child command that runs `bench.py argv` as `gpus` ranks, one process
    per GPU, exactly as the driver's N>1 form does (torch.distributed.run,
    one node, rendezvous on 127.0.0.1) — the reference's harness likewise
    spawns its own workers (tracker/launcher_local.py:63-100)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(gpus),
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def maybe_self_launch(args, argv):
    """`python bench.py --gpus N` (N > 1) started without a launcher: start the
    N ranks as ONE child process tree (torch.distributed.run), forward its
    output (inherited stdout/stderr: the ranks' JSON line is the only line
    rank 0 prints) and return its exit code.  None when this process is
    already a rank (WORLD_SIZE set) or N = 1.  Runs before torch or the HIP
    library is loaded and never execs (a child, so nothing that touched the
    GPU is replaced)."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(self_launch_cmd(args.gpus, argv, free_port()), env=env)


def main():
    args = parse()
    rc = maybe_self_launch(args, sys.argv[1:])
    if rc is not None:
        sys.exit(rc)
    # a rehearsal of N > 4 ranks on a 1-GPU box: fewer hardware queues per
    # process, as rdc_amd.launcher gives workers that share a GPU (the GPU's
    # scheduler otherwise time-slices 4 x N queues, ~10 ms per slice;
    # profiles/r03/host_n8_queues/).  Before HIP starts (launcher.py is loaded by
    # path: importing the package would load the HIP library); never with a GPU per rank.
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "_rdc_launcher", os.path.join(os.path.dirname(os.path.abspath(__file__)), "rdc_amd", "launcher.py"))
    launcher = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(launcher)
    q = launcher.hw_queues_per_process(int(os.environ.get("LOCAL_WORLD_SIZE", "1")))
    if q is not None and launcher.visible_gpu_count() == 1 and \
            launcher.queues_over_budget(os.environ.get("GPU_MAX_HW_QUEUES"), q):
        os.environ["GPU_MAX_HW_QUEUES"] = str(q)
    import torch
    import rdc_amd
    from rdc_amd._lib import _LIB, check_call

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        raise SystemExit("--gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    dt_enum, esz = DTYPES[args.dtype]
    count = args.bytes // esz
    S = count * esz
    torch.cuda.set_device(local % torch.cuda.device_count())
    tdtype = getattr(torch, args.dtype)
    stream = torch.cuda.current_stream()
    sp = ctypes.c_void_p(stream.cuda_stream)
    dist = None
    if world > 1:
        import torch.distributed as dist
        # a 1 GiB allreduce takes milliseconds: give up on a missing peer fast
        os.environ.setdefault("RDC_TIMEOUT", "30")
        dist.init_process_group("gloo")
        rdc_amd.init([])          # RANK/WORLD_SIZE + MASTER_ADDR:MASTER_PORT+1 bootstrap
        comm = rdc_amd.get_comm("main")
        algo = {"auto": 0, "ring": 1, "mesh": 2, "oneshot": 3, "mesh_pull": 5, "direct": 6}[args.algo]
        K = max(1, args.buckets)
        if K == 1:
            buf = torch.empty(count, dtype=tdtype, device="cuda")
            rdc_amd.fill_(buf, 0x5EED0000, rank)

            def step():
                check_call(_LIB.RdcCommAllreduceEx(comm.handle, ctypes.c_void_p(buf.data_ptr()), count, dt_enum, 2,
                                                   algo, sp))
        else:
            # cfg5 shape: K separate buckets (own allocations), one coalesced call per step
            per = count // K
            count = per * K
            S = count * esz
            bks = [torch.empty(per, dtype=tdtype, device="cuda") for _ in range(K)]
            for b, t in enumerate(bks):
                rdc_amd.fill_(t, 0x5EED0000 + b, rank)
            ptrs = (ctypes.c_void_p * K)(*[t.data_ptr() for t in bks])
            cnts = (ctypes.c_size_t * K)(*([per] * K))

            if args.unfused:
                def step():
                    for t in bks:
                        check_call(_LIB.RdcCommAllreduceEx(comm.handle, ctypes.c_void_p(t.data_ptr()), per, dt_enum,
                                                           2, algo, sp))
            else:
                def step():
                    check_call(_LIB.RdcCommAllreduceCoalesced(comm.handle, ptrs, cnts, K, dt_enum, 2, algo, sp))
    else:
        dst = torch.empty(count, dtype=tdtype, device="cuda")
        src = torch.empty(count, dtype=tdtype, device="cuda")
        rdc_amd.fill_(dst, 0x5EED0000, 0)
        rdc_amd.fill_(src, 0x5EED0000, 1)

        def step():
            check_call(_LIB.RdcReduce(ctypes.c_void_p(dst.data_ptr()), ctypes.c_void_p(src.data_ptr()), count,
                                      dt_enum, 2, sp))

    # first step checked on its own: a broken peer path fails in seconds
    # (RDC_TIMEOUT) instead of once per warm-up launch
    step()
    torch.cuda.synchronize()
    if world > 1:
        sync_check(comm, sp, dist, torch)
    tuned = untuned = direct_selfcheck = None
    if world > 1:
        # the direct schedule's self-check, run by the library when the channel
        # was created (round 6): 1 passed, 2 failed, 0 not run
        dc = ctypes.c_uint64()
        check_call(_LIB.RdcCommGetParam(comm.handle, b"direct_check", ctypes.byref(dc)))
        direct_selfcheck = {0: "not run", 1: "passed", 2: "failed"}.get(int(dc.value), int(dc.value))
    if world > 1 and args.autotune_reps > 0 and args.algo == "auto" and args.buckets == 1:
        # what a drop-in caller gets: the untuned default for this buffer,
        # timed (a few steps, max over ranks) before the autotune replaces it
        ms_u = timed_ms(step, comm, sp, dist, torch, max(3, min(args.steps, 10)), warm=1)
        llu = (ctypes.c_uint64 * 6)()
        check_call(_LIB.RdcCommLastLaunch(comm.handle, llu))
        untuned = {"schedule": {1: "ring", 2: "mesh", 3: "oneshot", 4: "tree", 5: "mesh_pull", 6: "direct"}.get(
            int(llu[5])), "ms_per_step": round(ms_u, 4)}
    if world > 1 and args.autotune_reps > 0:
        # launch-shape autotuning on THIS node (outside the timed region; the
        # defaults were tuned where every rank shares one HBM).  Every rank
        # keeps the same winner (times agreed by a MAX allreduce in the
        # library); a failure is recorded and the defaults kept.
        try:
            if os.environ.get("RDC_BENCH_FAIL_AUTOTUNE") == str(rank):  # test hook: this rank fails
                raise RuntimeError("injected autotune failure (RDC_BENCH_FAIL_AUTOTUNE)")
            tuned = comm.autotune(S, dt_enum, reps=args.autotune_reps, stream=sp)
            # the direct schedule's self-check (run by Autotune before it times
            # that schedule): 1 passed, 2 failed (then not a candidate), 0 not run
            dc = ctypes.c_uint64()
            check_call(_LIB.RdcCommGetParam(comm.handle, b"direct_check", ctypes.byref(dc)))
            tuned["direct_selfcheck"] = {0: "not run", 1: "passed", 2: "failed"}.get(int(dc.value), int(dc.value))
            failed = 0.0
        except Exception as e:  # noqa: BLE001 - recorded in the line
            tuned, failed = {"error": str(e)[:300]}, 1.0
        f = torch.tensor([failed], dtype=torch.float64)
        dist.all_reduce(f, op=dist.ReduceOp.MAX)
        if float(f[0]) > 0:
            if "error" not in tuned:
                tuned = {"error": "failed on another rank"}
            # A candidate that failed on the device (a wait timed out) leaves
            # its channel unusable: every later launch on it skips its body
            # and reports the error.  Every rank (the failure is agreed above)
            # moves to a fresh communicator with a channel of its own and the
            # library's default shape; `step` and the extras use it.
            os.environ["RDC_SHARE_SCRATCH"] = "0"
            comm = rdc_amd.new_comm("bench_after_autotune_failure")
            tuned["timed_on"] = "a fresh communicator (own channel, default shape) after the failure"
            step()
            torch.cuda.synchronize()
        sync_check(comm, sp, dist, torch)
    for _ in range(max(0, args.warmup - 1)):
        step()
    torch.cuda.synchronize()
    probe = None
    if world > 1:
        sync_check(comm, sp, dist, torch)
        dist.barrier()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(args.steps):
        step()
    e1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    if world > 1:
        sync_check(comm, sp, dist, torch)
    wall = t1 - t0
    kern_ms = e0.elapsed_time(e1) / args.steps
    timed_algo = timed_launch = None
    if world > 1:  # the schedule and launch shape the library used for the timed launches
        ll = (ctypes.c_uint64 * 6)()
        if _LIB.RdcCommLastLaunch(comm.handle, ll) == 0:
            timed_algo = {1: "ring", 2: "mesh", 3: "oneshot", 4: "tree", 5: "mesh_pull", 6: "direct"}.get(int(ll[5]))
            timed_launch = {"schedule": timed_algo, "grid": int(ll[0]), "scatter_blocks": int(ll[1]),
                            "reduce_blocks": int(ll[2]), "gather_blocks": int(ll[3]), "tile_bytes": int(ll[4])}
    if world > 1:
        tt = torch.tensor([wall, kern_ms], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        wall, kern_ms = float(tt[0]), float(tt[1])

    # Everything after the timed region is informational.  A failure there
    # (e.g. a device wait timing out) must not cost the headline line: every
    # extra runs guarded; inside, every step agrees on failure over the CPU
    # process group (sync_check), so all ranks leave a failed extra together;
    # once one has failed the communicator is unusable, and the remaining
    # extras that need it are skipped.  Partial results are kept.
    #
    # The extras share one wall-clock budget (--extras-budget-s), agreed
    # across ranks before each one: an extra that needs more than what is
    # left is skipped (`extras_skipped`), so the line is printed well inside
    # the driver's limit however slow the node is.  Each extra's wall
    # seconds are in `extras_wall_s`.  Order = value of the evidence: the
    # parity checks (every hand-off verified over the real links) first.
    extras_error = {}
    extras_skipped = []
    extras_wall = {}
    budget = Budget(args.extras_budget_s, dist, torch, world)

    def guarded(name, fn, needs_comm=True, partial=None, need_s=10.0):
        if needs_comm and extras_error:
            return None
        if budget.left() < need_s:
            extras_skipped.append(name)
            return None
        t_x = time.perf_counter()
        res, failed = None, 0.0
        try:
            res = fn()
        except Exception as e:  # noqa: BLE001 - diagnostics only
            extras_error[name] = str(e)[:300]
            failed = 1.0
        if world > 1:
            f = torch.tensor([failed], dtype=torch.float64)
            dist.all_reduce(f, op=dist.ReduceOp.MAX)
            if float(f[0]) > 0 and name not in extras_error:
                extras_error[name] = "failed on another rank"
        extras_wall[name] = round(time.perf_counter() - t_x, 2)
        if name in extras_error:
            return partial if partial else None
        return res

    multi = world > 1 and args.buckets == 1 and args.algo == "auto"
    f32 = args.dtype == "float32"
    roles = ring_cmp = extra = rccl = tcp = checks = None
    if world > 1:
        # the measured link rates (every rank idle), after the timed region so
        # that a failure here cannot cost the headline
        probe = guarded("xgmi_probe", lambda: xgmi_probe(_LIB, comm, sp, dist, torch), need_s=5)
    if multi:
        roles = guarded("role_timeline", lambda: trace_roles(_LIB, comm, buf, count, dt_enum, sp, dist, torch),
                        need_s=2)
    if multi and f32 and not args.no_check:
        # before the timed buffer is freed: the direct schedule does not
        # export an address it exported for another allocation (a freed
        # buffer's address handed out again falls back to the scratch
        # schedules), so the direct check's buffer must be a fresh address
        part_c = {}
        checks = guarded("parity_checks", lambda: parity_checks(_LIB, comm, S, world, rank, sp, dist, torch, part_c,
                                                                budget),
                         partial=part_c, need_s=30)
    if multi:
        # back to torch's caching allocator, NOT to HIP (no empty_cache): the
        # later configs' buffers come out of the same allocations, which the
        # direct schedule has mapped already; a freed allocation's address
        # handed out again would not be exported (AllreduceDirect)
        del buf
    if multi and args.ring_steps > 0:
        # the reference's own schedule on a buffer of the same size (same
        # bits, one link direction per GPU).  Grids are clamped to what stays
        # resident next to the ranks sharing a GPU, so this runs in rehearsals.
        def ring_leg():
            rbuf = torch.empty(count, dtype=tdtype, device="cuda")
            rdc_amd.fill_(rbuf, 0x5EED0000, rank)
            ms = time_ring(_LIB, comm, rbuf, count, dt_enum, sp, dist, torch, args.ring_steps)
            del rbuf
            return ms
        ring_cmp = guarded("ring_schedule", ring_leg, need_s=5)
    if multi and f32 and args.extra_steps > 0:
        part = {}
        extra = guarded("extra_configs", lambda: time_extra_configs(_LIB, comm, S, world, rank, sp, dist, torch,
                                                                    args.extra_steps, part, args.autotune_reps,
                                                                    budget),
                        partial=part, need_s=20)
    if multi and f32 and args.rccl_steps > 0:
        rccl = guarded("rccl_comparison", lambda: rccl_compare(S, world, rank, local, dist, torch, args.rccl_steps,
                                                               limit_s=min(150.0, budget.left() - 15)),
                       need_s=45)
    if world > 1 and args.cpu_seconds > 0:
        tcp = guarded("cpu_tcp_ring", lambda: cpu_tcp_ring(S, world, rank, dist), needs_comm=False, need_s=20)

    # spot check (outside the timed region): N=1 reduce result vs oracle on a slice
    check = None
    if world == 1 and not args.no_check:
        from oracle import oracle as O
        m = min(count, 1 << 16)
        d0 = O.fill(m, dt_enum, 0x5EED0000, 0)  # the generator is position-keyed: first m elements
        s0 = O.fill(m, dt_enum, 0x5EED0000, 1)
        acc = d0.copy()
        for _ in range(args.warmup + args.steps):
            O.reducer(s0, acc, dt_enum, 2)
        got = dst[:m].cpu().view(torch.uint8).numpy()  # bytes (numpy has no bfloat16)
        check = bool(got.tobytes() == acc.tobytes())

    if rank != 0:
        dist.barrier()
        _finalize(rdc_amd, extras_error)
        return
    algbw = S / (kern_ms * 1e-3) / 1e9
    gpus_here = torch.cuda.device_count()
    shared = world > 1 and gpus_here < world
    if world == 1:
        value = S / wall * args.steps / 1e9
        achieved = 3 * S / (kern_ms * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": load_traffic("reduce_sum_%s_%d" % (DT_SHORT[args.dtype], S)),
                "kernel": "k_reduce<Sum,%s>" % CXX_TYPE[args.dtype],
                "algorithmic_bytes_per_launch": 3 * S, "kernel_avg_ms": round(kern_ms, 4)}
        workload = "reduce kernel alone (n=1): dst += src, %s, %d MiB per buffer" % (args.dtype, S >> 20)
        par = "single GPU"
    else:
        # busbw of the whole job: S / t x 2(n-1)/n, t = the
        # wall time per step (max over ranks, barrier-bracketed)
        value = S / (wall / args.steps) / 1e9 * 2 * (world - 1) / world
        ctx = {"world": world, "S": S, "count": count, "esz": esz, "dtype": args.dtype, "dt_enum": dt_enum,
               "buckets": args.buckets, "unfused": args.unfused, "algo": args.algo, "steps": args.steps,
               "wall": wall, "kern_ms": kern_ms, "timed_algo": timed_algo, "gpus_here": gpus_here, "probe": probe,
               "tuned": tuned, "direct_selfcheck": direct_selfcheck, "untuned": untuned,
               "host_1g": extra.get("host_1GiB") if isinstance(extra, dict) else None}
        roof, algo_name, multi_keys = compose_multi(_LIB, ctx)
        workload = "in-place allreduce(sum) of a %d MiB %s buffer per GPU, %s schedule" % (S >> 20, args.dtype,
                                                                                        algo_name)
        if args.buckets > 1:
            workload = "%d x %d KiB %s buckets per GPU (%d MiB), %s, %s schedule" % (
                args.buckets, (S // args.buckets) >> 10, args.dtype, S >> 20,
                "separate calls" if args.unfused else "one coalesced call", algo_name)
        par = "dp%d (one process per GPU, xGMI P2P)" % world
        if timed_launch is not None:
            timed_launch["note"] = "last launch of the timed region (RdcCommLastLaunch)"
            timed_launch["source"] = ("RdcCommAutotune on this node before the warm-up (see `autotune`)"
                                      if isinstance(tuned, dict) and tuned.get("chosen") else
                                      "library defaults (automatic rule)")
    out = {
        "metric": "allreduce GB/s (device-resident fp32) at 1/2/4/8 GPUs; % xGMI roofline",
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": DT_SHORT[args.dtype],
        "data": "synthetic (splitmix64 device generator, seed 0x5EED0000)",
        "config": dict({"workload": workload, "bytes_per_gpu": S, "parallelism": par},
                       **({"launch": timed_launch} if timed_launch is not None else {})),
        "value_definition": "reduce kernel alone: S / t" if world == 1 else
                            "busbw = S / t x 2(n-1)/n (algbw_GBps = S / t)",
        "algbw_GBps": round(S / (wall / args.steps) / 1e9, 2),
        "roofline": roof,
        "cpu_baseline": cpu_baseline(S, args.cpu_seconds) if world == 1 else None,
    }
    if world > 1:
        out.update(multi_keys)
        out["busbw_GBps"] = round(value, 2)
        out["ranks_share_gpu"] = shared
        out["gpu_max_hw_queues"] = os.environ.get("GPU_MAX_HW_QUEUES")  # None: HIP's default (4)
    if ring_cmp is not None:
        rb = S / (ring_cmp * 1e-3) / 1e9 * 2 * (world - 1) / world
        out["ring_schedule"] = {"ms_per_step": round(ring_cmp, 4), "busbw_GBps": round(rb, 2),
                                "frac_of_one_link_peak": None if shared else round(rb / XGMI_LINK_DIR_GBPS, 4),
                                "note": "reference ring schedule (k_ring) on the same buffer, timed after the "
                                        "main region; bit-identical result"}
        hm = hbm_model(_LIB, world, count, dt_enum, "ring")
        if hm is not None:
            moved = hm["read_sum"] + hm["write_sum"] if (shared and gpus_here == 1) else hm["read"] + hm["write"]
            ach = moved / (ring_cmp * 1e-3) / 1e9
            out["ring_schedule"]["shared_hbm" if shared else "hbm"] = {
                "bytes_per_step": int(moved), "achieved": round(ach, 1), "frac": round(ach / HBM_PEAK_GBPS, 4),
                "traffic_per_rank": load_traffic("ring_%s_n%d_%d" % (DT_SHORT[args.dtype], world, S))}
    if tuned is not None:
        out["autotune"] = tuned
    if roles is not None:
        out["role_timeline"] = roles
    if extra is not None:
        out["extra_configs"] = extra
    if checks is not None:
        out["oracle_check"] = checks
    if rccl is not None:
        out["rccl_comparison"] = rccl
    if tcp is not None:
        out["cpu_tcp_ring"] = tcp
    if check is not None:
        out["oracle_check"] = check
    if extras_error:
        out["extras_error"] = extras_error
    if world > 1:
        out["extras_budget_s"] = args.extras_budget_s
        out["extras_wall_s"] = extras_wall
        out["extras_skipped"] = extras_skipped
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        _finalize(rdc_amd, extras_error)


def _finalize(rdc_amd, extras_error):
    """Tear the communicators down; after a failed extra the library may
    refuse, which must not turn a printed line into a failed run."""
    try:
        rdc_amd.finalize()
    except Exception as e:  # noqa: BLE001
        if not extras_error:
            raise
        print("bench: finalize after a failed extra: %s" % e, file=sys.stderr)


if __name__ == "__main__":
    main()
