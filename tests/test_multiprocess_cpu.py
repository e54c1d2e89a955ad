"""CPU, world size > 1.

* the native TCP bootstrap (tracker replacement, rdc_amd/csrc/rdc_bootstrap.cpp):
  rank/world from env or argv key=val, barrier, connect timeout;
* the mesh decomposition under torch.distributed gloo (world size 2 and 3):
  each rank folds ONLY its own Split chunk in the reference ring's order from
  all ranks' inputs, then the owners' chunks are gathered — exactly the work
  split k_mesh performs — and must equal the oracle's ring allreduce
  bit-for-bit on every rank.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import oracle as O
from tests.conftest import ROOT, free_port


def clean_env():
    e = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    return e


BOOT = r'''
import sys, rdc_amd as r
r.init(sys.argv[1:])
for _ in range(5):
    r.barrier()
print("rank %d/%d ok" % (r.get_rank(), r.get_world_size()), flush=True)
r.finalize()
'''


@pytest.mark.parametrize("world", [2, 3, 5])
def test_tcp_bootstrap(world):
    port = free_port()
    procs = [subprocess.Popen([sys.executable, "-c", BOOT, "RDC_RANK=%d" % r, "rdc_world_size=%d" % world,
                               "RDC_TRACKER_URI=127.0.0.1", "RDC_TRACKER_PORT=%d" % port],
                              cwd=ROOT, env=clean_env(), stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for r in range(world)]
    outs = [p.communicate(timeout=120)[0] for p in procs]
    for r, (p, o) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, o
        assert "rank %d/%d ok" % (r, world) in o


def test_torchrun_env_fallback():
    """RANK/WORLD_SIZE/MASTER_ADDR/MASTER_PORT (+1 = tracker port) as under torchrun."""
    port = free_port()
    procs = []
    for r in range(2):
        env = clean_env()
        env.update(RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port - 1))
        procs.append(subprocess.Popen([sys.executable, "-c", BOOT], cwd=ROOT, env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = [p.communicate(timeout=120)[0] for p in procs]
    assert all(p.returncode == 0 for p in procs), outs


def test_bootstrap_timeout_is_an_error():
    code = r'''
import rdc_amd as r
from rdc_amd._lib import RdcError
try:
    r.init(["RDC_RANK=1", "RDC_WORLD_SIZE=2", "RDC_TRACKER_PORT=%d", "RDC_BOOTSTRAP_TIMEOUT=1"])
except RdcError as e:
    assert "connect" in str(e); print("OK")
''' % free_port()
    p = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=clean_env(), capture_output=True, text=True,
                       timeout=60)
    assert "OK" in p.stdout, p.stdout + p.stderr


def fold_chunk(parts, c, dtype, op):
    """Chunk c's ring order: s = x[c-1]; s = OP(x[c-2], s); ...; s = OP(x[c], s)
    (OP(dst, src) = op::Reducer with dst the rank's own value)."""
    n = len(parts)
    acc = parts[(c - 1) % n].copy()
    for k in range(2, n + 1):
        dst = parts[(c - k) % n].copy()
        O.reducer(acc, dst, dtype, op)
        acc = dst
    return acc


def _gloo_worker(rank, world, port, count, dtype, op, q):
    try:
        _gloo_body(rank, world, port, count, dtype, op, q)
    except Exception as e:  # report instead of leaving the parent waiting
        q.put((rank, repr(e)))


def _gloo_body(rank, world, port, count, dtype, op, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    x = O.fill(count, dtype, 0x5EED0000, rank)
    # exchange inputs (stand-in for the scatter stage's pushes)
    xs = [torch.empty(count, dtype=torch.from_numpy(x).dtype) for _ in range(world)]
    dist.all_gather(xs, torch.from_numpy(x))
    inputs = [t.numpy() for t in xs]
    # owner computes its chunk in ring order (k_mesh's reduce role)
    b, e = O.split(count, world)[rank]
    part = [np.ascontiguousarray(v[b:e]) for v in inputs]
    mine = fold_chunk(part, rank, dtype, op)
    # gather the owners' results (k_mesh's allgather role); gloo wants equal
    # sizes, so pad every chunk to the first (longest) one and trim after
    sizes = [e2 - b2 for b2, e2 in O.split(count, world)]
    padded = np.zeros(sizes[0], dtype=x.dtype)
    padded[: mine.size] = mine
    outs = [torch.empty(sizes[0], dtype=torch.from_numpy(x).dtype) for _ in sizes]
    dist.all_gather(outs, torch.from_numpy(padded))
    got = np.concatenate([t.numpy()[:s] for t, s in zip(outs, sizes)])
    want = O.expected_allreduce(inputs, dtype, op)
    q.put((rank, got.tobytes() == want.tobytes()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("count,dtype,op", [(1001, O.DT_FLOAT32, O.OP_SUM), (4099, O.DT_FLOAT64, O.OP_MAX),
                                            (7, O.DT_INT32, O.OP_SUM)])
def test_gloo_owner_computes_matches_ring(world, count, dtype, op):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_gloo_worker, args=(r, world, port, count, dtype, op, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    assert all(res[r] is True for r in range(world)), res


# ------------------------------------------------------------- launcher ---
LAUNCHED = r'''
import os, sys
att = int(os.environ["RDC_NUM_ATTEMPT"])
if sys.argv[1] == "restart" and os.environ["RDC_RANK"] == "1" and att == 0:
    sys.exit(254)                # asks the keepalive loop for a restart (launcher_local.py:17-27)
import rdc_amd as r
r.init([])                       # rank / world / rendezvous from the launcher's env
if sys.argv[1] == "fail" and r.get_rank() == 2:
    sys.exit(3)
r.barrier()
print("rank %d/%d attempt %d local %s ok" % (r.get_rank(), r.get_world_size(), att, os.environ["LOCAL_RANK"]),
      flush=True)
r.finalize()
'''


def launch(n, mode, timeout=180):
    return subprocess.run([sys.executable, "-m", "rdc_amd.launcher", "-n", str(n), "--gpus", "2",
                           sys.executable, "-c", LAUNCHED, mode],
                          cwd=ROOT, env=clean_env(), capture_output=True, text=True, timeout=timeout)


def test_launcher_runs_workers_with_reference_env():
    p = launch(3, "ok")
    assert p.returncode == 0, p.stdout + p.stderr
    for r in range(3):
        assert "rank %d/3 attempt 0 local %d ok" % (r, r % 2) in p.stdout, p.stdout


def test_launcher_restarts_on_254():
    """A worker that exits 254 before the rendezvous is restarted and joins
    (mid-job recovery is the tracker's fault-tolerance protocol: out of scope)."""
    p = launch(2, "restart")
    assert p.returncode == 0, p.stdout + p.stderr
    assert "rank 1/2 attempt 1" in p.stdout and "rank 0/2 attempt 0" in p.stdout, p.stdout


def test_launcher_stops_all_on_failure():
    """rank 2 exits 3: the others (blocked in the bootstrap) are stopped and
    the launcher returns 3 instead of hanging."""
    p = launch(3, "fail", timeout=120)
    assert p.returncode == 3, p.stdout + p.stderr


BUDGET = r'''
import os, sys, time, json
sys.path.insert(0, os.environ["ROOT"])
import torch, torch.distributed as dist
dist.init_process_group("gloo")
import bench
rank = dist.get_rank()
b = bench.Budget(1.0, dist, torch, dist.get_world_size())
out = []
for step in range(4):
    time.sleep(0.05 * (rank + 1) * (step + 1))   # rank 1 falls behind more each step
    out.append(round(b.left(), 6))
print("LEFT", rank, json.dumps(out), flush=True)
'''


def test_bench_extras_budget_agreed_across_ranks():
    """bench.py's extras budget: every rank computes the same time left (the
    slowest rank's elapsed time, MAX over the CPU group), so every rank takes
    the same skip decision even when one rank runs behind."""
    port = free_port()
    procs = []
    for r in range(2):
        env = clean_env()
        env.update(RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), ROOT=ROOT)
        procs.append(subprocess.Popen([sys.executable, "-c", BUDGET], cwd=ROOT, env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = [p.communicate(timeout=120)[0] for p in procs]
    import json
    lefts = []
    for p, o in zip(procs, outs):
        assert p.returncode == 0, o
        line = [l for l in o.splitlines() if l.startswith("LEFT")][0]
        lefts.append(json.loads(line.split(" ", 2)[2]))
    assert lefts[0] == lefts[1], lefts
    assert lefts[0][-1] < 0 < lefts[0][0] and lefts[0] == sorted(lefts[0], reverse=True), lefts


def _fake_sysfs(root, gpus):
    """KFD topology with a CPU node and one GPU node per (render minor,
    local_cpulist) in `gpus`, plus the render devices' local_cpulist."""
    nodes = root / "class" / "kfd" / "kfd" / "topology" / "nodes"
    (nodes / "0").mkdir(parents=True)
    (nodes / "0" / "properties").write_text("cpu_cores_count 64\nsimd_count 0\n")
    for i, (minor, cpus) in enumerate(gpus, start=1):
        (nodes / str(i)).mkdir()
        (nodes / str(i) / "properties").write_text("simd_count 1024\ndrm_render_minor %d\n" % minor)
        dev = root / "class" / "drm" / ("renderD%d" % minor) / "device"
        dev.mkdir(parents=True)
        (dev / "local_cpulist").write_text(cpus + "\n")


def test_launcher_numa_cpus_from_sysfs(tmp_path, monkeypatch):
    """--numa-bind's lookup (rdc_amd/launcher.py gpu_local_cpus): HIP device
    k = the k-th readable KFD GPU node, its render device's local_cpulist;
    none when *_VISIBLE_DEVICES remaps the readable GPUs or the topology is
    missing."""
    from rdc_amd.launcher import gpu_local_cpus, parse_cpulist
    for v in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    assert parse_cpulist("0-3,8,10-11") == {0, 1, 2, 3, 8, 10, 11}
    _fake_sysfs(tmp_path, [(128, "0-63,128-191"), (136, "64-127,192-255")])
    assert gpu_local_cpus(0, str(tmp_path)) == set(range(0, 64)) | set(range(128, 192))
    assert gpu_local_cpus(1, str(tmp_path)) == set(range(64, 128)) | set(range(192, 256))
    assert gpu_local_cpus(2, str(tmp_path)) is None
    assert gpu_local_cpus(0, str(tmp_path / "missing")) is None
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "1")          # remaps 2 readable GPUs: unknown
    assert gpu_local_cpus(0, str(tmp_path)) is None
    one = tmp_path / "one"                                    # a container exposing only its GPU
    _fake_sysfs(one, [(168, "0-63,128-191")])
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "0")
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0")
    assert gpu_local_cpus(0, str(one)) == set(range(0, 64)) | set(range(128, 192))


def test_launcher_numa_bind_confines_workers(tmp_path):
    """With --numa-bind every worker starts inside this process's allowed
    CPUs (here no GPU topology: workers run unbound with a warning, and the
    run still succeeds)."""
    prog = tmp_path / "aff.py"
    prog.write_text("import os\nprint('cpus', len(os.sched_getaffinity(0)))\n")
    p = subprocess.run([sys.executable, "-m", "rdc_amd.launcher", "-n", "2", "--numa-bind", sys.executable,
                        str(prog)], cwd=ROOT, capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr
    assert p.stdout.count("cpus") == 2


def test_launcher_queue_budget(tmp_path, monkeypatch):
    """Workers sharing a GPU get fewer hardware queues each (rdc_amd/launcher.py
    hw_queues_per_process): up to 4 per GPU keep HIP's default, 8 get 2, 16 get
    1; a GPU_MAX_HW_QUEUES above the budget is lowered, one below it kept; the KFD GPU count from sysfs."""
    import argparse
    from rdc_amd.launcher import hw_queues_per_process, kfd_gpu_count, visible_gpu_count, worker_env
    assert [hw_queues_per_process(k) for k in (1, 2, 4, 5, 8, 16, 32)] == [None, None, None, 2, 2, 1, 1]
    # never 3 queues per process (5 x 3 and 6 x 3 lose hand-offs)
    assert all(hw_queues_per_process(k) in (None, 1, 2, 4) for k in range(1, 65))
    monkeypatch.delenv("GPU_MAX_HW_QUEUES", raising=False)
    a = argparse.Namespace(host_ip="127.0.0.1", num_workers=8)
    assert worker_env(a, 3, 1234, 1)["GPU_MAX_HW_QUEUES"] == "2"
    assert "GPU_MAX_HW_QUEUES" not in worker_env(a, 3, 1234, 8)
    assert "GPU_MAX_HW_QUEUES" not in worker_env(argparse.Namespace(host_ip="127.0.0.1", num_workers=4), 0, 1, 1)
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")             # a box exporting HIP's default: lowered
    assert worker_env(a, 3, 1234, 1)["GPU_MAX_HW_QUEUES"] == "2"
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "1")             # a lower choice is kept
    assert worker_env(a, 3, 1234, 1)["GPU_MAX_HW_QUEUES"] == "1"
    _fake_sysfs(tmp_path, [(128, "0-3"), (136, "4-7")])
    assert kfd_gpu_count(str(tmp_path)) == 2 and kfd_gpu_count(str(tmp_path / "missing")) is None
    for v in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    dri = tmp_path / "dri"
    dri.mkdir()
    for name in ("card1", "renderD128", "renderD136"):
        (dri / name).write_text("")
    assert visible_gpu_count(str(dri)) == 2 and visible_gpu_count(str(tmp_path / "none")) is None
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "3")
    assert visible_gpu_count(str(dri)) == 1


def test_bench_self_launch_command(monkeypatch):
    """`python bench.py --gpus N` without a launcher: the
    child it starts is the driver's own N > 1 form — torch.distributed.run,
    one node, N processes, rendezvous on 127.0.0.1 — running this bench.py
    with the same arguments; nothing is started at N = 1 or inside a rank."""
    import argparse
    import bench
    cmd = bench.self_launch_cmd(8, ["--gpus", "8", "--steps", "20"], 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert cmd[3:10] == ["--nnodes=1", "--nproc-per-node", "8", "--master-addr", "127.0.0.1", "--master-port",
                         "29555"]
    assert cmd[10] == os.path.join(ROOT, "bench.py") and cmd[11:] == ["--gpus", "8", "--steps", "20"]
    monkeypatch.setenv("WORLD_SIZE", "8")
    assert bench.maybe_self_launch(argparse.Namespace(gpus=8), []) is None   # already a rank
    monkeypatch.delenv("WORLD_SIZE")
    assert bench.maybe_self_launch(argparse.Namespace(gpus=1), []) is None   # N = 1 runs in place


def test_bench_self_launch_forwards_exit_code():
    """The self-launched ranks' exit status is bench.py's: here (no GPU) both
    ranks fail, so bench.py fails and prints no JSON line."""
    env = clean_env()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup",
                        "1", "--bytes", "4096"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode != 0
    assert not [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert "torch.distributed" in p.stderr or "ChildFailedError" in p.stderr or "local_rank" in p.stderr, p.stderr[-2000:]


def test_bench_traffic_file_reaches_the_gpu_box():
    """bench.py's roofline.traffic comes from the committed PMC summary
    (it was null in BENCH_r04 because the summary sat under
    profiles/, which .gpurunignore keeps off the GPU box).  The file must
    exist at the path bench.py reads, hold the N = 1 kernel's bytes, and no
    .gpurunignore pattern may exclude it."""
    import fnmatch
    import bench
    path = os.path.join(ROOT, "traffic.json")
    assert os.path.exists(path)
    # measured HBM bytes of one 1 GiB launch: 3 x S within 0.1 % (round 6: 3,221,259,392)
    t = bench.load_traffic("reduce_sum_f32_1073741824")
    assert t is not None and abs(t / (3 * 2**30) - 1) < 1e-3, t
    rel = "traffic.json"
    with open(os.path.join(ROOT, ".gpurunignore")) as f:
        pats = [ln.strip() for ln in f if ln.strip() and not ln.startswith("#")]
    for p in pats:
        anchored = p.startswith("./")
        q = p[2:] if anchored else p
        assert not fnmatch.fnmatch(rel, q), (p, "excludes traffic.json from the GPU box")
        assert not (not anchored and fnmatch.fnmatch(os.path.basename(rel), q)), p
