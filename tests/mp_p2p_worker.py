"""One rank of a multi-process point-to-point run (spawned by tests/test_gpu_p2p.py).

argv: rank world port mode.  All ranks share GPU 0 (RDC_DEVICE=0).
  hello   — test/sendrecv.cc (rdc::Send / rdc::Recv of "hello world %u ",
            100 messages, the receiver sleeping before the first) and
            pytest/comm.py (Buffer(b'hello') -> Buffer(b'00000'))
  ring    — send a multi-piece device buffer to rank+1, receive from rank-1
  fuzz    — a seeded list of messages between random pairs, random sizes,
            device or host memory on either side, up to 8 in flight
  timeout — rank 1 receives a message rank 0 never sends: an error, not a hang
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    rank, world, port, mode = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    import torch
    import rdc_amd
    rdc_amd.init(["RDC_RANK=%d" % rank, "RDC_WORLD_SIZE=%d" % world, "RDC_TRACKER_PORT=%d" % port,
                  "RDC_TRACKER_URI=127.0.0.1", "RDC_DEVICE=0"])
    torch.cuda.set_device(0)
    comm = rdc_amd.new_comm("main")
    if mode == "hello":
        for i in range(100):
            s = ("hello world %u " % i).encode()
            if rank == 0:
                rdc_amd.send(rdc_amd.Buffer(s), 1)
            else:
                if i == 0:
                    time.sleep(1.0)
                buf = rdc_amd.Buffer(bytearray(16))
                # the reference receives str.size() bytes into a 16-byte buffer
                b = rdc_amd.Buffer(addr=buf.addr, size=len(s))
                rdc_amd.recv(b, 0)
                got = buf.bytes()[:len(s)]
                assert got == s, (i, got, s)
        # pytest/comm.py
        if rank == 0:
            comm.send(rdc_amd.Buffer(b"hello"), 1)
        else:
            buf = rdc_amd.Buffer(b"00000")
            comm.recv(buf, 0)
            assert buf.bytes() == b"hello", buf.bytes()
    elif mode == "ring":
        nxt, prv = (rank + 1) % world, (rank - 1 + world) % world
        for rnd in range(4):
            n = (9 << 20) + 1000 * rnd + 3
            x = torch.from_numpy(np.random.default_rng(rank * 100 + rnd).integers(0, 256, n, dtype=np.uint8)).cuda()
            want = np.random.default_rng(prv * 100 + rnd).integers(0, 256, n, dtype=np.uint8)
            y = torch.zeros(n, dtype=torch.uint8, device="cuda")
            ws = comm.isend(x, nxt)
            wr = comm.irecv(y, prv)
            ws.wait()
            wr.wait()
            assert np.array_equal(y.cpu().numpy(), want), "round %d differs" % rnd
        # host ndarrays through the Buffer path, float payload
        f = np.arange(12345, dtype=np.float64) + rank
        g = np.zeros_like(f)
        ws = comm.isend(f, nxt)
        wr = comm.irecv(g, prv)
        ws.wait(), wr.wait()
        assert np.array_equal(g, np.arange(12345, dtype=np.float64) + prv)
    elif mode == "fuzz":
        # a seeded global list of messages (source, destination, size 0 B ..
        # ~24 MiB, device or host memory); every rank walks it in order,
        # posting its own sends and receives non-blocking with up to 8 in
        # flight, so each pair's messages are matched in list order
        rng = np.random.default_rng(777 + world)
        msgs = []
        for i in range(60):
            s = int(rng.integers(world))
            d = int((s + 1 + rng.integers(world - 1)) % world)
            n = 0 if rng.random() < 0.05 else int(2 ** rng.uniform(0, 24.5))
            msgs.append((i, s, d, n, bool(rng.random() < 0.3), bool(rng.random() < 0.3)))
        pend, checks = [], []
        for i, s, d, n, host_s, host_r in msgs:
            if rank == s:
                x = np.random.default_rng(1000 + i).integers(0, 256, n, dtype=np.uint8)
                t = x if host_s else torch.from_numpy(x).cuda()
                pend.append((comm.isend(t, d), t))
            if rank == d:
                y = np.zeros(n, np.uint8) if host_r else torch.zeros(n, dtype=torch.uint8, device="cuda")
                pend.append((comm.irecv(y, s), y))
                checks.append((i, n, y))
            while len(pend) > 8:
                pend.pop(0)[0].wait()
        for w, _ in pend:
            w.wait()
        for i, n, y in checks:
            got = y if isinstance(y, np.ndarray) else y.cpu().numpy()
            want = np.random.default_rng(1000 + i).integers(0, 256, n, dtype=np.uint8)
            assert np.array_equal(got, want), "message %d (%d B) differs" % (i, n)
    elif mode == "timeout":
        if rank == 1:
            y = torch.zeros(100, dtype=torch.uint8, device="cuda")
            t0 = time.time()
            try:
                comm.irecv(y, 0).wait()
                raise AssertionError("receive from a silent peer completed")
            except rdc_amd.RdcError as e:
                assert "no progress" in str(e), str(e)
            assert time.time() - t0 < 30
    else:
        raise SystemExit("unknown mode " + mode)
    rdc_amd.barrier()
    print("rank %d: %s OK" % (rank, mode), flush=True)
    rdc_amd.finalize()


if __name__ == "__main__":
    main()
