"""GPU: the reference-shaped entry points end to end.

* the C++ header (include/rdc.h) known-answer program — test/allreduce.cc's
  checks — as 2 and 3 processes on GPU 0, host buffers staged through HBM;
* bench.py launched exactly as the driver launches it for N > 1
  (torch.distributed.run, one process per rank; here all ranks share GPU 0).
"""
import json
import os
import subprocess
import sys

import pytest

from tests.conftest import ROOT, free_port

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def known_answer_exe(tmp_path_factory):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    exe = str(tmp_path_factory.mktemp("cpp") / "known_answer")
    subprocess.check_call(["g++", "-std=c++11", "-O1", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "cpp", "known_answer.cc"), "-o", exe,
                           "-L", os.path.join(ROOT, "rdc_amd"), "-lrdc_amd",
                           "-Wl,-rpath," + os.path.join(ROOT, "rdc_amd")])
    return exe


@pytest.mark.parametrize("world,N", [(2, 3), (3, 1024), (3, 100003)])
def test_cpp_known_answer(known_answer_exe, world, N):
    port = free_port()
    env = dict(os.environ, RDC_DEVICE="0", RDC_SCRATCH_BYTES="64M")
    procs = [subprocess.Popen([known_answer_exe, str(N), "RDC_RANK=%d" % r, "rdc_world_size=%d" % world,
                               "RDC_TRACKER_URI=127.0.0.1", "RDC_TRACKER_PORT=%d" % port],
                              env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for r in range(world)]
    outs = [p.communicate(timeout=180)[0] for p in procs]
    report = "\n".join("--- rank %d rc=%s\n%s" % (r, p.returncode, o[-1500:]) for r, (p, o) in enumerate(zip(procs, outs)))
    for r, (p, o) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, report
        assert "rank %d: known-answer OK" % r in o, report


def test_bench_torchrun_two_ranks():
    """bench.py exactly as the driver launches it for N > 1, with every extra:
    value = busbw; ranks sharing a GPU report bound "shared-hbm" and no
    fraction; the CPU TCP ring is labelled a port; the cfg1 host-buffer line,
    the reference ring schedule and the bit-exact checks at the bench's own
    shapes are present; no extra failed."""
    port = free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--bytes", str(64 << 20), "--extra-steps", "2",
           "--ring-steps", "2", "--cpu-seconds", "1"]
    p = subprocess.run(cmd, cwd=ROOT, env=dict(os.environ), capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["value"] > 0
    assert out["value"] == out["busbw_GBps"] and out["value"] == pytest.approx(out["algbw_GBps"], rel=0.02)
    assert out["config"]["bytes_per_gpu"] == 64 << 20
    assert "extras_error" not in out, out.get("extras_error")
    roof = out["roofline"]
    if torch.cuda.device_count() < 2:
        assert out["ranks_share_gpu"] is True
        assert roof["bound"] == "shared-hbm" and roof["frac"] is None and roof["frac_of_measured"] is None
    else:
        assert roof["bound"] == "xgmi" and 0 < roof["frac"] < 1.5
    probe = roof["xgmi_probe"]
    assert probe["one_link_one_direction_GBps"] > 0 and probe["all_links_egress_GBps"] > 0, probe
    assert probe["pull_one_link_GBps"] > 0 and probe["pull_all_links_GBps"] > 0, probe
    assert out["cpu_tcp_ring"]["kind"] == "port" and out["cpu_tcp_ring"]["median_ms"] > 0
    assert out["ring_schedule"]["ms_per_step"] > 0
    ex = out["extra_configs"]
    assert ex["cfg1_host_4KiB"]["us_per_call"] > 0 and ex["cfg5_buckets"]["ms_per_step"] > 0
    assert ex["host_64MiB"]["algbw_GBps_pcie_inclusive"] > 0, ex.get("host_64MiB")
    assert ex["host_64MiB_registered"]["algbw_GBps_pcie_inclusive"] > 0, ex.get("host_64MiB_registered")
    chk = out["oracle_check"]
    assert all(chk.get(k) is True for k in PARITY_KEYS), chk
    assert chk["schedule"]["cfg3_direct"] == "direct", chk  # a fresh buffer: the registered-buffer schedule ran
    assert out["extras_skipped"] == [] and "parity_checks" in out["extras_wall_s"], out["extras_wall_s"]


# every hand-off kind the timed lines use, verified bit-exact in bench.py's
# parity_checks
PARITY_KEYS = ("cfg3_direct", "cfg3_mesh", "cfg3_ring", "cfg3_mesh_pull", "cfg4_fp16", "cfg5_buckets", "oneshot_512KiB", "service_host_4KiB",
               "tree_order", "broadcast_nonzero_root", "allgather_varsize")


def test_bench_self_launches_its_ranks():
    """`python bench.py --gpus 2` with no launcher (WORLD_SIZE unset) starts
    its two ranks itself (a torch.distributed.run child): exactly one JSON
    line, n_gpus 2, and every bit-exact check after the timed region true —
    so a driver that starts the N-GPU bench like the N = 1 one still
    measures N ranks."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--bytes", str(16 << 20), "--extra-steps", "0", "--rccl-steps", "0", "--cpu-seconds", "0",
           "--autotune-reps", "0"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["value"] > 0 and out["config"]["bytes_per_gpu"] == 16 << 20
    chk = out["oracle_check"]
    assert all(chk.get(k) is True for k in PARITY_KEYS), chk


def test_bench_tiny_extras_budget():
    """--extras-budget-s bounds everything after the timed region: with a
    1-second budget the headline line is still printed, every extra is listed
    in extras_skipped and none ran."""
    port = free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--bytes", str(16 << 20), "--extras-budget-s", "1",
           "--autotune-reps", "0"]
    p = subprocess.run(cmd, cwd=ROOT, env=dict(os.environ), capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["value"] > 0 and out["extras_budget_s"] == 1
    assert set(out["extras_skipped"]) >= {"parity_checks", "ring_schedule", "extra_configs", "cpu_tcp_ring"}, out
    assert out["extras_wall_s"].get("role_timeline") is not None or "role_timeline" in out["extras_skipped"]
    assert "extra_configs" not in out and "oracle_check" not in out


def test_bench_recovers_from_autotune_failure():
    """An autotune that fails on one rank (injected on rank 1, whose absence
    then times out rank 0's candidates on the device) is agreed by every
    rank, which then time the region on a fresh communicator with a channel
    of its own (a device-side failure leaves the old channel unusable): the
    line is printed, records the failure, and every parity check after the
    timed region passes on the new communicator."""
    port = free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "2", "--bytes", str(16 << 20), "--autotune-reps", "1",
           "--extra-steps", "0", "--ring-steps", "0", "--rccl-steps", "0", "--cpu-seconds", "0"]
    # rank 1 skips autotune: rank 0's candidates wait for it until RDC_TIMEOUT,
    # so rank 0's channel really fails on the device
    env = dict(os.environ, RDC_BENCH_FAIL_AUTOTUNE="1", RDC_TIMEOUT="8")
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["value"] > 0
    assert "error" in out["autotune"] and "fresh communicator" in out["autotune"]["timed_on"], out["autotune"]
    assert out["config"]["launch"]["source"] == "library defaults (automatic rule)", out["config"]
    chk = out["oracle_check"]
    assert all(chk.get(k) is True for k in PARITY_KEYS), chk


def test_launcher_cpp_known_answer(known_answer_exe):
    """The reference's workflow (launcher -n N prog args) with rdc_amd's
    launcher: the C++ known-answer program at 3 ranks, rendezvous from env."""
    env = dict(os.environ, RDC_SCRATCH_BYTES="64M")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, "-m", "rdc_amd.launcher", "-n", "3", "--gpus", "1", known_answer_exe, "4099"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    for r in range(3):
        assert "rank %d: known-answer OK" % r in p.stdout, p.stdout


@pytest.mark.parametrize("world", [2, 3])
def test_python_surface_across_ranks(world):
    """rdc_amd's Python surface at world size > 1, launched as the reference
    launches pytest/allreduce.py (launcher -n N python script): the harness's
    MAX/SUM known answers, allreduce's copy rule on owning / 2-D / view /
    non-contiguous arrays, prepare_fun inside RdcAllreduce, pickled broadcast
    from non-zero roots, and collectives on new_comm("x") / get_comm("x")
    handles (host allreduce, isend/irecv ring, device allreduce)
    (tests/py_surface_worker.py)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, RDC_SCRATCH_BYTES="64M")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, "-m", "rdc_amd.launcher", "-n", str(world), "--gpus", "1", sys.executable,
                        os.path.join(ROOT, "tests", "py_surface_worker.py")],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    for r in range(world):
        assert "rank %d: python surface OK" % r in p.stdout, p.stdout + p.stderr[-2000:]


@pytest.fixture(scope="module")
def buffer_api_exe(tmp_path_factory):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    exe = str(tmp_path_factory.mktemp("cpp2") / "buffer_api")
    subprocess.check_call(["g++", "-std=c++11", "-O1", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "cpp", "buffer_api.cc"), "-o", exe,
                           "-L", os.path.join(ROOT, "rdc_amd"), "-lrdc_amd",
                           "-Wl,-rpath," + os.path.join(ROOT, "rdc_amd")])
    return exe


@pytest.mark.parametrize("world,mincount", [(2, None), (3, None), (4, "4K")])
def test_cpp_buffer_surface(buffer_api_exe, tmp_path, world, mincount):
    """include/rdc.h's Buffer-typed and custom-reducer surface end to end as
    `world` processes: rdc::Buffer (Slice/Count/As/Alloc), Allreduce<OP>(Buffer&),
    Broadcast(Buffer&), Send/Recv(Buffer[, size]), ISend/IRecv(Buffer),
    Allgather(vector<Buffer>&), virtual ICommunicator::Allreduce(Buffer,
    ReduceFunction), Reducer<DType,freduce> (float and struct items),
    SerializeReducer<DType> (variable-length objects) and CreateGroup.  The
    program checks integer known answers itself; its float results are
    compared here with the oracle (ring order; the tree order when
    rdc_reduce_ring_mincount=4K covers the 4004-byte buffers)."""
    import numpy as np
    from oracle import oracle as O
    port = free_port()
    env = dict(os.environ, RDC_DEVICE="0", RDC_SCRATCH_BYTES="64M")
    extra = ["rdc_reduce_ring_mincount=%s" % mincount] if mincount else []
    procs = [subprocess.Popen([buffer_api_exe, str(tmp_path), "RDC_RANK=%d" % r, "rdc_world_size=%d" % world,
                               "RDC_TRACKER_URI=127.0.0.1", "RDC_TRACKER_PORT=%d" % port] + extra,
                              env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for r in range(world)]
    outs = [p.communicate(timeout=240)[0] for p in procs]
    report = "\n".join("--- rank %d rc=%s\n%s" % (r, p.returncode, o[-1500:]) for r, (p, o) in enumerate(zip(procs, outs)))
    for r, p in enumerate(procs):
        assert p.returncode == 0 and "rank %d: buffer api OK" % r in outs[r], report
    tree = mincount is not None
    N = 1001
    for name, seed, op in (("typed_sum", 0x5EED3000, O.OP_SUM), ("custom_sum", 0x5EED3100, O.OP_SUM),
                           ("reducer_sum", 0x5EED3200, O.OP_SUM), ("op_reducer_sum", 0x5EED3400, O.OP_SUM),
                           ("op_reducer_max", 0x5EED3500, O.OP_MAX)):
        xs = [O.fill(N, O.DT_FLOAT32, seed, r) for r in range(world)]
        want = (O.expected_tree if tree else O.expected_allreduce)(xs, O.DT_FLOAT32, op)
        for r in range(world):
            got = np.fromfile(str(tmp_path / ("%s_rank%d.bin" % (name, r))), dtype=np.float32)
            assert got.tobytes() == want.tobytes(), (name, r)
    for M in (1, 2, 3, (1 << 18) + 3):  # custom reducer: empty chunks (M < world), ragged Split
        xs = [O.fill(M, O.DT_FLOAT32, 0x5EED3100 + M, r) for r in range(world)]
        want = (O.expected_tree if tree and 4 * M <= 4096 else O.expected_allreduce)(xs, O.DT_FLOAT32, O.OP_SUM)
        for r in range(world):
            got = np.fromfile(str(tmp_path / ("custom_sum_%d_rank%d.bin" % (M, r))), dtype=np.float32)
            assert got.tobytes() == want.tobytes(), ("custom_sum", M, r)
    members = [q for q in range(world - 1, -1, -1) if q % 2 == 0]
    xs = [O.fill(N, O.DT_FLOAT32, 0x5EED3300, i) for i in range(len(members))]
    want = (O.expected_tree if tree else O.expected_allreduce)(xs, O.DT_FLOAT32, O.OP_SUM)
    for q in members:
        got = np.fromfile(str(tmp_path / ("group_sum_rank%d.bin" % q)), dtype=np.float32)
        assert got.tobytes() == want.tobytes(), ("group", q)


def test_rccl_comparison_child_one_rank():
    """tools/rccl_allreduce.py, the RCCL comparison child bench.py starts per
    rank on a node with one GPU per rank (never run in the one-GPU
    rehearsals, where ranks share the GPU): one rank, 64 MiB, a JSON line."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import json
    port = free_port()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "rccl_allreduce.py"), "0", "1", "0", "127.0.0.1",
                        str(port), str(64 << 20), "5"], capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    line = [l for l in p.stdout.splitlines() if l.startswith("{")][-1]
    d = json.loads(line)
    assert d["rccl"] is True and d["ms_per_step"] > 0 and d["bytes_per_gpu"] == 64 << 20, d
