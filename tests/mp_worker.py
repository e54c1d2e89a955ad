"""One rank of a multi-process GPU parity run (spawned by tests/test_gpu_allreduce.py).

argv: rank world port outdir cases_json.  Every case: device-side synthetic
input (RdcFill, seed/rank) -> collective on the given communicator ->
bytes saved to outdir/case<i>_rank<r>.npy for the parent to check against
the CPU oracle.  All ranks share GPU 0 (RDC_DEVICE=0) on the 1-GPU box.
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def log(*a):
    if os.environ.get("RDC_DEBUG"):
        import time
        print("[%.3f]" % time.time(), *a, flush=True)


def main():
    rank, world, port, outdir, cases = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], sys.argv[5]
    cases = json.loads(open(cases).read())
    import torch
    import rdc_amd
    from rdc_amd._lib import _LIB, check_call
    # RDC_DEVICE=rank: rank r on GPU r % #GPUs (a node with several GPUs);
    # otherwise every rank on that one device (the 1-GPU box: GPU 0)
    dev_env = os.environ.get("RDC_DEVICE", "0")
    device = rank % max(1, torch.cuda.device_count()) if dev_env == "rank" else int(dev_env)
    rdc_amd.init(["RDC_RANK=%d" % rank, "RDC_WORLD_SIZE=%d" % world, "RDC_TRACKER_PORT=%d" % port,
                  "RDC_TRACKER_URI=127.0.0.1", "RDC_DEVICE=%d" % device])
    torch.cuda.set_device(device)
    log("rank", rank, "init done")
    comms = {}
    esz = {0: 1, 1: 1, 2: 4, 3: 4, 4: 8, 5: 8, 6: 4, 7: 8, 8: 8, 9: 8, 10: 2, 11: 2}
    stream = torch.cuda.current_stream()
    sp = ctypes.c_void_p(stream.cuda_stream)
    for i, c in enumerate(cases):
        name = c.get("comm", "main")
        if name not in comms:
            comms[name] = rdc_amd.new_comm(name) if name != "main" else rdc_amd.get_comm("main")
            log("rank", rank, "comm", name, "ready")
        comm = comms[name]
        kind = c.get("kind", "allreduce")
        count, dtype = c["count"], c["dtype"]
        pad = c.get("pad", 0) + rank * c.get("pad_per_rank", 0)
        nbytes = count * esz[dtype]
        if kind == "allgather":
            nbytes = 0
        if c.get("empty_cache"):  # the freed blocks go back to HIP: a new allocation may reuse their addresses
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
        buf = torch.zeros(nbytes + pad + 64, dtype=torch.uint8, device="cuda")
        p = buf.data_ptr() + pad
        check_call(_LIB.RdcFill(ctypes.c_void_p(p), count, dtype, c.get("seed", 0x5EED0000), rank, sp))
        log("rank", rank, "case", i, "filled")
        if kind == "allgather":
            # test/allgather.cc shape: buffer i has i + N int32 items, owner fills a[i][j] = i + j
            N = c["count"]
            ts = [torch.zeros(i + N, dtype=torch.int32, device="cuda") for i in range(world)]
            ts[rank].copy_(torch.arange(rank, rank + rank + N, dtype=torch.int32, device="cuda"))
            torch.cuda.synchronize()
            comm.allgather(ts, stream=sp)
            comm.check(sp)
            out = torch.cat(ts).cpu().numpy().view(np.uint8)
            np.save(os.path.join(outdir, "case%d_rank%d.npy" % (i, rank)), out)
            print("rank %d case %d ok" % (rank, i), flush=True)
            continue
        if kind == "host_mix":
            # small synchronous HOST allreduces through the resident service
            # (rdc_service.h): (dtype, op) switches relaunch it, sleeps longer
            # than its idle time let it exit between calls, device-resident
            # collectives run in between; every result saved
            import time as _time
            outs = []
            dev = torch.zeros(20011, dtype=torch.float32, device="cuda")
            for j, (cnt, dt, op, sleep_ms) in enumerate(c["ops"]):
                t = torch.zeros(cnt * esz[dt] + 16, dtype=torch.uint8, device="cuda")
                check_call(_LIB.RdcFill(ctypes.c_void_p(t.data_ptr()), cnt, dt, 0x5EED6000 + j, rank, sp))
                torch.cuda.synchronize()
                h = t[: cnt * esz[dt]].cpu().numpy().copy()
                if sleep_ms:
                    _time.sleep(sleep_ms / 1000.0)
                check_call(_LIB.RdcAllreduce(ctypes.c_void_p(h.ctypes.data), cnt, dt, op, None, None))
                outs.append(h)
                if j % 3 == 2:  # a device collective between service calls
                    check_call(_LIB.RdcFill(ctypes.c_void_p(dev.data_ptr()), dev.numel(), 6, 0x5EED6500 + j, rank, sp))
                    check_call(_LIB.RdcCommAllreduceEx(comm.handle, ctypes.c_void_p(dev.data_ptr()), dev.numel(), 6,
                                                       2, 0, sp))
                    comm.check(sp)
                    outs.append(dev.cpu().numpy().view(np.uint8).copy())
            np.save(os.path.join(outdir, "case%d_rank%d.npy" % (i, rank)), np.concatenate(outs))
            print("rank %d case %d ok" % (rank, i), flush=True)
            continue
        if kind == "shared_comms":
            # named communicators over the same ranks share one scratch channel:
            # memory cost, and launches of different communicators issued on
            # different streams without host syncs (the channel orders them)
            free0 = torch.cuda.mem_get_info()[0]
            extra = [rdc_amd.new_comm("shared_%d_%d" % (i, k)) for k in range(2)]
            free1 = torch.cuda.mem_get_info()[0]
            shares = [comm.get_param("shares_scratch")] + [e.get_param("shares_scratch") for e in extra]
            streams = [torch.cuda.Stream() for _ in range(3)]
            bufs = [torch.zeros(count, dtype=torch.float32, device="cuda") for _ in range(3)]
            torch.cuda.synchronize()
            for j, (cm, st, b) in enumerate(zip([comm] + extra, streams, bufs)):
                check_call(_LIB.RdcFill(ctypes.c_void_p(b.data_ptr()), count, 6, 0x5EED4000 + j, rank,
                                        ctypes.c_void_p(st.cuda_stream)))
            for rep in range(c.get("reps", 1)):
                for j, (cm, st, b) in enumerate(zip([comm] + extra, streams, bufs)):
                    algo = (rep + j) % 4
                    check_call(_LIB.RdcCommAllreduceEx(cm.handle, ctypes.c_void_p(b.data_ptr()), count, 6, 2, algo,
                                                       ctypes.c_void_p(st.cuda_stream)))
            torch.cuda.synchronize()
            for cm, st in zip([comm] + extra, streams):
                cm.check(ctypes.c_void_p(st.cuda_stream))
            out = torch.cat(bufs).cpu().numpy().view(np.uint8)
            np.save(os.path.join(outdir, "case%d_rank%d.npy" % (i, rank)), out)
            open(os.path.join(outdir, "case%d_rank%d.json" % (i, rank)), "w").write(
                json.dumps({"shares": shares, "bytes_used_by_two_comms": free0 - free1}))
            for e in extra:
                e.destroy()
            print("rank %d case %d ok" % (rank, i), flush=True)
            continue
        if kind == "order_violation":
            # two communicators sharing one channel issued in DIFFERENT orders
            # on different ranks (rank 0: main then x; the others: x then
            # main): the launches with equal sequence numbers belong to
            # different communicators, which the tagged hand-off flags turn
            # into an error on every rank instead of folding unrelated buffers
            other = rdc_amd.new_comm("order_%d" % i)
            info = {"shares": [comm.get_param("shares_scratch"), other.get_param("shares_scratch")]}
            a = torch.zeros(count, dtype=torch.float32, device="cuda")
            b = torch.zeros(count, dtype=torch.float32, device="cuda")
            torch.cuda.synchronize()
            order = [(comm, a), (other, b)] if rank == 0 else [(other, b), (comm, a)]
            err = ""
            import time as _time
            t_start = _time.time()
            try:
                for cm, t in order:
                    check_call(_LIB.RdcCommAllreduceEx(cm.handle, ctypes.c_void_p(t.data_ptr()), count, 6, 2,
                                                       c.get("algo", 0), sp))
                comm.check(sp)
            except Exception as e:  # noqa: BLE001 - the expected outcome
                err = str(e)
            info["error"] = err
            info["seconds"] = round(_time.time() - t_start, 3)
            open(os.path.join(outdir, "case%d_rank%d.json" % (i, rank)), "w").write(json.dumps(info))
            print("rank %d case %d ok" % (rank, i), flush=True)
            # the channel is unusable now: leave without finalizing collectives
            os._exit(0)
        if kind == "mem_return":
            # the direct schedule's mapping life cycle (round 6): a big buffer
            # goes through the direct schedule, is freed back to HIP, and the
            # next direct call (a small new buffer) makes every peer close its
            # mapping of it — the freed memory must come back to the device
            # (round 5 kept peer mappings, so a freed allocation stayed alive)
            def stat(k):
                v = ctypes.c_uint64()
                check_call(_LIB.RdcCommGetParam(comm.handle, k.encode(), ctypes.byref(v)))
                return int(v.value)
            def vram_used():  # device-wide bytes in use (driver sysfs), -1 if unreadable
                try:
                    hip = ctypes.CDLL("libamdhip64.so")
                    b = ctypes.create_string_buffer(64)
                    hip.hipDeviceGetPCIBusId(b, 63, device)
                    with open("/sys/bus/pci/devices/%s/mem_info_vram_used" % b.value.decode().lower()) as f:
                        return int(f.read().split()[0])
                except Exception:  # noqa: BLE001
                    return -1
            big = torch.empty(count, dtype=torch.float32, device="cuda")
            check_call(_LIB.RdcFill(ctypes.c_void_p(big.data_ptr()), count, 6, c.get("seed", 0x5EED0000), rank, sp))
            check_call(_LIB.RdcCommAllreduceEx(comm.handle, ctypes.c_void_p(big.data_ptr()), count, 6, 2, 6, sp))
            comm.check(sp)
            ll = (ctypes.c_uint64 * 6)()
            check_call(_LIB.RdcCommLastLaunch(comm.handle, ll))
            first_algo = int(ll[5])
            got = big[:1024].cpu().numpy().view(np.uint8).copy()  # the first 4 KiB
            del big
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
            free0 = torch.cuda.mem_get_info()[0]
            used0 = vram_used()
            closed0 = stat("direct_closed")
            # second_pad: the second buffer sits rank x 4 bytes into its allocation, so the ranks'
            # buffers differ mod 16 and that call cannot run direct — the peers must close the
            # freed buffer's mappings in its rendezvous all the same
            sp_pad = rank * 4 if c.get("second_pad") else 0
            small_alloc = torch.empty(c["small"] + 4 * world, dtype=torch.float32, device="cuda")
            small = small_alloc[sp_pad // 4: sp_pad // 4 + c["small"]]
            check_call(_LIB.RdcFill(ctypes.c_void_p(small.data_ptr()), c["small"], 6, 0x5EEDB000, rank, sp))
            check_call(_LIB.RdcCommAllreduceEx(comm.handle, ctypes.c_void_p(small.data_ptr()), c["small"], 6, 2, 6, sp))
            comm.check(sp)
            check_call(_LIB.RdcCommLastLaunch(comm.handle, ll))
            torch.cuda.synchronize()
            free1 = torch.cuda.mem_get_info()[0]
            used1 = vram_used()
            info = {"first_algo": first_algo, "second_algo": int(ll[5]), "free_before": free0, "free_after": free1,
                    "vram_used_before": used0, "vram_used_after": used1,
                    "closed": stat("direct_closed") - closed0, "retired": stat("direct_retired"),
                    "maps": stat("direct_maps"), "refused": stat("direct_refused")}
            open(os.path.join(outdir, "case%d_rank%d.json" % (i, rank)), "w").write(json.dumps(info))
            out = np.concatenate([got, small.cpu().numpy().view(np.uint8)])
            np.save(os.path.join(outdir, "case%d_rank%d.npy" % (i, rank)), out)
            del small, small_alloc
            print("rank %d case %d ok" % (rank, i), flush=True)
            continue
        if kind == "bcast_chain":
            # stream-ordered chain without host syncs: refill, broadcast from a
            # rotating root, accumulate — exposes a root overwriting a peer's
            # scratch before the peer consumed the previous broadcast
            acc = torch.zeros(count, dtype=torch.int32, device="cuda")
            for k in range(c["steps"]):
                root = (k * 3 + 1) % world
                check_call(_LIB.RdcFill(ctypes.c_void_p(p), count, 2, c.get("seed", 0x5EED0000) + k, rank, sp))
                check_call(_LIB.RdcCommBroadcast(comm.handle, ctypes.c_void_p(p), count * 4, root, sp))
                check_call(_LIB.RdcReduce(ctypes.c_void_p(acc.data_ptr()), ctypes.c_void_p(p), count, 2, 2, sp))
            comm.check(sp)
            np.save(os.path.join(outdir, "case%d_rank%d.npy" % (i, rank)), acc.cpu().numpy().view(np.uint8))
            print("rank %d case %d ok" % (rank, i), flush=True)
            continue
        if kind == "coalesced":
            # bucketed allreduce: buffer b filled with seed + b, one fused call per rep
            counts = c["counts"]
            # pads differ per rank unless "same_pads" (the direct schedule needs every
            # buffer congruent mod 16 across ranks)
            pads = [((0 if c.get("same_pads") else rank * 3) + b) % 5 * esz[dtype] for b in range(len(counts))]
            bufs = [torch.zeros(k * esz[dtype] + pd + 64, dtype=torch.uint8, device="cuda")
                    for k, pd in zip(counts, pads)]
            ptrs = [t.data_ptr() + pd for t, pd in zip(bufs, pads)]
            for b, k in enumerate(counts):
                check_call(_LIB.RdcFill(ctypes.c_void_p(ptrs[b]), k, dtype, c.get("seed", 0x5EED0000) + b, rank, sp))
            arr = (ctypes.c_void_p * len(counts))(*ptrs)
            cnt = (ctypes.c_size_t * len(counts))(*counts)
            for _ in range(c.get("reps", 1)):
                if c.get("host"):
                    hosts = [t[pd: pd + k * esz[dtype]].cpu().numpy().copy() for t, pd, k in zip(bufs, pads, counts)]
                    harr = (ctypes.c_void_p * len(counts))(*[h.ctypes.data for h in hosts])
                    check_call(_LIB.RdcAllreduceCoalesced(harr, cnt, len(counts), dtype, c["op"]))
                    for t, pd, h in zip(bufs, pads, hosts):
                        if h.size:
                            t[pd: pd + h.size] = torch.from_numpy(h).cuda()
                else:
                    check_call(_LIB.RdcCommAllreduceCoalesced(comm.handle, arr, cnt, len(counts), dtype, c["op"],
                                                              c.get("algo", 0), sp))
            comm.check(sp)
            if c.get("last_launch"):
                ll = (ctypes.c_uint64 * 6)()
                check_call(_LIB.RdcCommLastLaunch(comm.handle, ll))
                open(os.path.join(outdir, "case%d_rank%d.launch" % (i, rank)), "w").write(
                    json.dumps([int(x) for x in ll]))
            if c.get("digest"):  # full-size lists: sha256 over the buckets in order
                import hashlib
                h = hashlib.sha256()
                for t, pd, k in zip(bufs, pads, counts):
                    h.update(t[pd: pd + k * esz[dtype]].cpu().numpy().tobytes())
                open(os.path.join(outdir, "case%d_rank%d.sha" % (i, rank)), "w").write(h.hexdigest())
            else:
                out = np.concatenate([t[pd: pd + k * esz[dtype]].cpu().numpy()
                                      for t, pd, k in zip(bufs, pads, counts)])
                np.save(os.path.join(outdir, "case%d_rank%d.npy" % (i, rank)), out)
            del bufs
            print("rank %d case %d ok" % (rank, i), flush=True)
            continue
        if c.get("autotune"):  # RdcCommAutotune for this many bytes, then the case runs on the chosen shape
            res = comm.autotune(c["autotune"], dtype, reps=2, stream=sp)
            dc = ctypes.c_uint64()
            check_call(_LIB.RdcCommGetParam(comm.handle, b"direct_check", ctypes.byref(dc)))
            res["direct_check"] = int(dc.value)  # the direct schedule's self-check (1 = passed)
            open(os.path.join(outdir, "case%d_rank%d.tune" % (i, rank)), "w").write(json.dumps(res))
        if c.get("last_launch"):  # record the launch shape the library chose (grid clamp checks)
            ll = (ctypes.c_uint64 * 6)()
        if c.get("direct_release"):  # RdcCommDirectRelease: mappings closed, the direct schedule off
            comm.direct_release()
        reps = c.get("reps", 1)
        for _ in range(reps):
            if c.get("warm_l2"):  # every XCD's L2 holds the buffer's lines before peers overwrite them
                buf.sum()
            if kind == "allreduce":
                check_call(_LIB.RdcCommAllreduceEx(comm.handle, ctypes.c_void_p(p), count, dtype, c["op"],
                                                   c.get("algo", 0), sp))
            elif kind == "algo_chain":
                for algo in c["algos"]:
                    check_call(_LIB.RdcCommAllreduceEx(comm.handle, ctypes.c_void_p(p), count, dtype, c["op"], algo,
                                                       sp))
            elif kind == "broadcast":
                check_call(_LIB.RdcCommBroadcast(comm.handle, ctypes.c_void_p(p), nbytes, c["root"], sp))
            elif kind == "host_allreduce":
                # host_offset: the host buffer starts that many bytes past an
                # aligned allocation (element-aligned, not 16-B aligned)
                ho = c.get("host_offset", 0)
                # pinned: True = every rank's buffer lies in a registered
                # RdcNewBuffer(pinned=1) range (DMA in place), "even" = even
                # ranks only (registered and staged ranks in one collective)
                pin = c.get("pinned")
                bh = None
                if pin is True or (pin == "even" and rank % 2 == 0):
                    import mmap
                    span = (nbytes + ho + mmap.PAGESIZE - 1) // mmap.PAGESIZE * mmap.PAGESIZE
                    backing = np.frombuffer(mmap.mmap(-1, span), dtype=np.uint8)
                    bh = ctypes.c_void_p()
                    check_call(_LIB.RdcNewBuffer(ctypes.byref(bh), backing.ctypes.data_as(ctypes.c_void_p), span, 1))
                    reg0 = ctypes.c_uint64()
                    check_call(_LIB.RdcCommGetParam(comm.handle, b"host_registered_calls", ctypes.byref(reg0)))
                else:
                    backing = np.empty(nbytes + ho + 64, dtype=np.uint8)
                host = backing[ho: ho + nbytes]
                host[:] = buf[pad: pad + nbytes].cpu().numpy()
                check_call(_LIB.RdcAllreduce(host.ctypes.data_as(ctypes.c_void_p), count, dtype, c["op"], None,
                                             None))
                buf[pad: pad + nbytes] = torch.from_numpy(host.copy()).cuda()
                if bh is not None:
                    reg1 = ctypes.c_uint64()
                    check_call(_LIB.RdcCommGetParam(comm.handle, b"host_registered_calls", ctypes.byref(reg1)))
                    open(os.path.join(outdir, "case%d_rank%d.reg" % (i, rank)), "w").write(
                        str(reg1.value - reg0.value))
                    check_call(_LIB.RdcDelBuffer(bh))
        log("rank", rank, "case", i, "launched")
        comm.check(sp)
        if c.get("last_launch"):
            check_call(_LIB.RdcCommLastLaunch(comm.handle, ll))
            open(os.path.join(outdir, "case%d_rank%d.launch" % (i, rank)), "w").write(json.dumps([int(x) for x in ll]))
        if c.get("direct_stats"):  # the direct schedule's rendezvous / mapping counters after this case
            st = {}
            for k in ("direct_check", "direct_calls", "direct_retired", "direct_closed", "direct_maps", "flags_kind",
                      "direct_exports", "direct_refused", "direct_rendezvous_ns", "direct_export_ns",
                      "direct_fallback", "direct_unusable", "direct_map_failed", "direct_fail_reason",
                      "direct_export_failed", "direct_export_error", "direct_import", "direct_pending", "direct_canary"):
                v = ctypes.c_uint64()
                check_call(_LIB.RdcCommGetParam(comm.handle, k.encode(), ctypes.byref(v)))
                st[k] = int(v.value)
            open(os.path.join(outdir, "case%d_rank%d.stats" % (i, rank)), "w").write(json.dumps(st))
        log("rank", rank, "case", i, "done")
        # warm_l2: the result read back by a copy KERNEL (through the L2s), not by a DMA copy
        out = (buf[pad: pad + nbytes].clone() if c.get("warm_l2") else buf[pad: pad + nbytes]).cpu().numpy()
        del buf
        if c.get("windows"):  # huge buffers: the listed element windows + a digest of the whole result
            import hashlib
            e = esz[dtype]
            win = np.concatenate([out[st * e:(st + m) * e] for st, m in c["windows"]])
            np.save(os.path.join(outdir, "case%d_rank%d.npy" % (i, rank)), win)
            open(os.path.join(outdir, "case%d_rank%d.sha" % (i, rank)), "w").write(
                hashlib.sha256(out.data).hexdigest())
        elif c.get("digest"):
            import hashlib
            open(os.path.join(outdir, "case%d_rank%d.sha" % (i, rank)), "w").write(
                hashlib.sha256(out.tobytes()).hexdigest())
        else:
            np.save(os.path.join(outdir, "case%d_rank%d.npy" % (i, rank)), out)
        print("rank %d case %d ok" % (rank, i), flush=True)
    rdc_amd.finalize()


if __name__ == "__main__":
    main()
