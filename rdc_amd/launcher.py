"""Single-node launcher — the counterpart of the reference's
``python -m tracker.launcher_local -n N prog args`` (tracker/launcher_local.py,
tracker/args.py) for the MI355X path:

    python -m rdc_amd.launcher -n 8 ./test_allreduce 1024
    python -m rdc_amd.launcher -n 8 python train.py

Starts N worker processes on this node, one per GPU (rank r -> GPU
r % #GPUs via LOCAL_RANK), with the reference's environment contract
(tracker/tracker.py:467-477): RDC_TRACKER_URI / RDC_TRACKER_PORT (here the
rendezvous of rank 0's TCP bootstrap, which exchanges HIP IPC handles — no
Python tracker process and no data over TCP), RDC_HEARTBEAT_INTERVAL,
plus RDC_RANK / RDC_WORLD_SIZE so ranks are fixed up front.  Like
launcher_local's keepalive loop (launcher_local.py:17-27), a worker that
exits with code 254 is restarted with RDC_NUM_ATTEMPT incremented (before the
rendezvous completes; rejoining a running job is the tracker's recovery
protocol, out of scope like checkpointing).  Unlike
it, the first worker that fails for good stops the others and its exit code
is returned (the reference raises inside a daemon thread and hangs).

--numa-bind confines each worker to the CPUs of its GPU's NUMA node (read
from sysfs before the worker starts; the launcher never touches the GPU).
Host buffers are copied into pinned memory and DMA'd from there: at n = 2
on one GPU, 16 MiB host allreduces ran 1.52-1.54 ms on the GPU's node vs
1.67-1.76 ms on the other one, little difference above (DESIGN.md §5.3,
profiles/r03/host_numa_ab2/).
"""
import argparse
import os
import socket
import subprocess
import sys
import threading
import time

RESTART_RC = 254
HEARTBEAT_INTERVAL_MS = 5000  # tracker/tracker.py HEARTBEAT_INTERVAL_MS (accepted, unused on the device path)


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="launch rdc workers on this node (one process per GPU)")
    p.add_argument("-n", "--num-workers", type=int, required=True, help="number of worker processes")
    p.add_argument("--host-ip", default="127.0.0.1", help="address rank 0's bootstrap listens on")
    p.add_argument("--port", type=int, default=0, help="bootstrap port (0 = pick a free one)")
    p.add_argument("--gpus", type=int, default=0, help="GPUs to spread ranks over (0 = all visible)")
    p.add_argument("--max-attempts", type=int, default=10, help="restarts per worker on exit code 254")
    p.add_argument("--numa-bind", action="store_true",
                   help="confine each worker to the CPUs of its GPU's NUMA node")
    p.add_argument("command", nargs=argparse.REMAINDER, help="command for launching the program")
    args, unknown = p.parse_known_args(argv)
    # the reference appends unknown options to the command (launcher_local.py:34)
    args.command = list(args.command) + list(unknown)
    if not args.command:
        p.error("missing command")
    if args.num_workers < 1:
        p.error("--num-workers must be >= 1")
    return args


def free_port(host):
    s = socket.socket()
    s.bind((host, 0))
    port = s.getsockname()[1]
    s.close()
    return port


def count_gpus():
    """GPUs visible to the workers, without initialising HIP in this process."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v:
            return len([x for x in v.split(",") if x.strip()])
    try:
        return len([d for d in os.listdir("/dev/dri") if d.startswith("renderD")]) or 1
    except OSError:
        return 1


def _read(path):
    try:
        with open(path) as f:
            return f.read()
    except OSError:
        return None


def parse_cpulist(text):
    """'0-63,128-191' -> {0..63, 128..191}"""
    cpus = set()
    for part in text.strip().split(","):
        if not part:
            continue
        lo, _, hi = part.partition("-")
        cpus.update(range(int(lo), int(hi or lo) + 1))
    return cpus


def _visible_count():
    """Devices *_VISIBLE_DEVICES leaves to HIP (None when none is set)."""
    n = None
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v:
            k = len([x for x in v.split(",") if x.strip()])
            n = k if n is None else min(n, k)
    return n


def visible_gpu_count(dev="/dev/dri"):
    """GPUs this process may use, without initialising HIP: the
    *_VISIBLE_DEVICES list when one is set, else the render nodes under
    /dev/dri; None when neither tells."""
    n = _visible_count()
    if n is not None:
        return n
    try:
        return len([d for d in os.listdir(dev) if d.startswith("renderD")]) or None
    except OSError:
        return None


def kfd_gpu_count(sysfs="/sys"):
    """GPUs in the KFD topology this process can read (None when unreadable)."""
    base = os.path.join(sysfs, "class", "kfd", "kfd", "topology", "nodes")
    try:
        nodes = [x for x in os.listdir(base) if x.isdigit()]
    except OSError:
        return None
    n = 0
    for nd in nodes:
        props = _read(os.path.join(base, nd, "properties")) or ""
        for line in props.splitlines():
            kv = line.split(None, 1)
            if len(kv) == 2 and kv[0] == "simd_count" and kv[1].strip().isdigit() and int(kv[1]) > 0:
                n += 1
    return n or None


# Hardware queues the GPU's scheduler maps at once, summed over the processes
# on it.  HIP gives every process GPU_MAX_HW_QUEUES (default 4) queues; with 8
# processes on one GPU (32 queues) the scheduler time-slices them, and a
# collective spinning on a peer whose queue is not mapped waits ~10 ms for the
# next slice: host allreduces of 4 KiB took 10.7 ms per call and of 64 MiB
# 253 ms, against 62 us and 18.4 ms with 2 queues per process
# (profiles/r03/host_n8_queues/).
QUEUE_BUDGET = 16


def hw_queues_per_process(ranks_per_gpu):
    """GPU_MAX_HW_QUEUES for a process that shares its GPU with
    ranks_per_gpu - 1 others (None: leave HIP's default of 4): the budget's
    share rounded down to a power of two, so never 3.  With three queues per
    process and 5 or more processes on one GPU, the GPU's scheduler left one
    rank's next collective kernel undispatched for as long as its peers'
    kernels spun waiting for it (device launch timelines, the
    late rank's kernel started exactly when the waiters timed out; round 6).
    At one block per CU (RDC_DEBUG_LDS_PAD=96K) 5 x 3 and 6 x 3 failed every
    run, 5 x 1, 5 x 2, 5 x 4, 6 x 2, 8 x 2, 4 x 2, 4 x 3 and 3 x 3 never
    (profiles/r05/queues/).  Round 6 found it depends on how full the XCDs
    are: ResidentGrid now keeps 3/8 of every XCD free for ranks sharing a GPU
    at one block per CU, and 5 x 3 and 6 x 3 then pass every run — this
    budget is kept, no longer load-bearing.  One rank per GPU is not
    affected."""
    if ranks_per_gpu * 4 <= QUEUE_BUDGET:
        return None
    q = max(1, QUEUE_BUDGET // ranks_per_gpu)
    while q & (q - 1):
        q &= q - 1
    return q


def queues_over_budget(current, q):
    """True when GPU_MAX_HW_QUEUES (unset = HIP's 4) exceeds the budget q: a
    value above it only buys the scheduler's time slices, so it is lowered
    (GPU boxes may export the default 4 explicitly)."""
    try:
        return int(current) > q if current not in (None, "") else 4 > q
    except ValueError:
        return True


def gpu_local_cpus(ordinal, sysfs="/sys"):
    """CPUs local to HIP device `ordinal`: the KFD topology's GPU nodes this
    process can read, in node order (HIP's device order); a node's
    drm_render_minor names its render device, whose PCI function lists its
    local CPUs.  When *_VISIBLE_DEVICES is set, only if it leaves exactly the
    readable GPUs (a container that exposes just its own); otherwise, or when
    sysfs cannot be read, None."""
    base = os.path.join(sysfs, "class", "kfd", "kfd", "topology", "nodes")
    try:
        nodes = sorted(int(x) for x in os.listdir(base) if x.isdigit())
    except OSError:
        return None
    minors = []
    for nd in nodes:
        props = _read(os.path.join(base, str(nd), "properties")) or ""
        kv = dict(line.split(None, 1) for line in props.splitlines() if len(line.split(None, 1)) == 2)
        try:
            if int(kv.get("simd_count", "0")) > 0 and "drm_render_minor" in kv:
                minors.append(int(kv["drm_render_minor"]))
        except ValueError:
            return None
    vis = _visible_count()
    if (vis is not None and vis != len(minors)) or ordinal >= len(minors):
        return None
    text = _read(os.path.join(sysfs, "class", "drm", "renderD%d" % minors[ordinal], "device", "local_cpulist"))
    if not text:
        return None
    try:
        cpus = parse_cpulist(text)
    except ValueError:
        return None
    return cpus or None


def worker_env(args, rank, port, ngpu):
    env = dict(os.environ)
    env.update({
        "RDC_TRACKER_URI": args.host_ip,
        "RDC_TRACKER_PORT": str(port),
        "RDC_HEARTBEAT_INTERVAL": str(HEARTBEAT_INTERVAL_MS),
        "RDC_RANK": str(rank),
        "RDC_WORLD_SIZE": str(args.num_workers),
        "LOCAL_RANK": str(rank % max(1, ngpu)),
    })
    # several workers on one GPU: fewer hardware queues each, so the GPU's
    # scheduler maps every worker's queues at once (a lower setting is kept)
    q = hw_queues_per_process(-(-args.num_workers // max(1, ngpu)))
    if q is not None and queues_over_budget(os.environ.get("GPU_MAX_HW_QUEUES"), q):
        env["GPU_MAX_HW_QUEUES"] = str(q)
    # torchrun-style names would override the rdc ones inside RdcInit's
    # fallbacks only where rdc names are absent; drop stale ones anyway
    for k in ("RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def run(args):
    port = args.port or free_port(args.host_ip)
    ngpu = args.gpus or count_gpus()
    procs = [None] * args.num_workers
    rcs = [None] * args.num_workers
    lock = threading.Lock()
    stop = threading.Event()
    first_fail = []  # exit code of the worker that failed first

    def keepalive(rank):
        env = worker_env(args, rank, port, ngpu)
        if args.numa_bind:
            local = gpu_local_cpus(rank % max(1, ngpu))
            allowed = os.sched_getaffinity(0)
            cpus = (local & allowed) if local else None
            if cpus:
                # this keepalive thread only (Linux: pid 0 = the calling
                # thread); the worker forked from it inherits the mask
                os.sched_setaffinity(0, cpus)
            else:
                print("rdc_amd.launcher: --numa-bind: no CPU list for GPU %d, worker %d unbound"
                      % (rank % max(1, ngpu), rank), file=sys.stderr)
        attempt = 0
        while not stop.is_set():
            env["RDC_NUM_ATTEMPT"] = str(attempt)
            with lock:
                if stop.is_set():
                    return
                procs[rank] = subprocess.Popen(args.command, env=env)
            rc = procs[rank].wait()
            if rc == RESTART_RC and attempt + 1 < args.max_attempts:
                attempt += 1
                continue
            rcs[rank] = rc
            if rc != 0:
                with lock:
                    if not stop.is_set():
                        first_fail.append(rc)
                    stop.set()
            return

    threads = [threading.Thread(target=keepalive, args=(r,), daemon=True) for r in range(args.num_workers)]
    for t in threads:
        t.start()
    try:
        while any(t.is_alive() for t in threads):
            if stop.is_set():
                break
            time.sleep(0.05)
    except KeyboardInterrupt:
        stop.set()
    if stop.is_set():
        # one worker failed for good: stop the rest (they would wait on it)
        with lock:
            live = [p for p in procs if p is not None and p.poll() is None]
        for p in live:
            p.terminate()
        deadline = time.time() + 10
        for p in live:
            try:
                p.wait(timeout=max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
    for t in threads:
        t.join(timeout=15)
    if first_fail:
        return first_fail[0]
    if any(rc is None for rc in rcs):
        return 1
    return 0


def main(argv=None):
    return run(parse_args(argv))


if __name__ == "__main__":
    sys.exit(main())
