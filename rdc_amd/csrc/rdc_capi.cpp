// C ABI of librdc_amd.so (include/rdc_amd.h) and the process-wide manager —
// the counterpart of comm::CommunicatorManager (src/comm/communicator_manager.cc)
// for the device path: parameters from env + argv (:87-115, :140-162), the
// communicator registry (:164-193), and the host-memory entry points the
// reference's Python package binds (rdc/core.py).
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/rdc_amd.h"
#include "rdc_bootstrap.h"
#include "rdc_comm.h"
#include "rdc_host.h"
#include "rdc_p2p.h"

using namespace rdc_amd;

namespace {

thread_local std::string g_last_error;

struct Manager {
    std::recursive_mutex mu;
    bool inited = false;
    bool env_loaded = false;  // environment parameters applied (RdcSetParam overrides them afterwards)
    int rank = 0, world = 1, device = -1;
    std::string tracker_uri = "127.0.0.1";
    int tracker_port = 29571;
    double bootstrap_timeout_s = 300.0;
    size_t host_zc_bytes = (size_t)1 << 20;  // host buffers up to this run zero-copy on pinned memory
    CommConfig cfg;
    std::unique_ptr<Bootstrap> bs;
    std::map<std::string, std::unique_ptr<Communicator>> comms;
    std::map<Communicator*, std::unique_ptr<Communicator>> groups;  // RdcCommInitAll handles
    void* stage = nullptr;
    size_t stage_bytes = 0;
    hipStream_t stream = nullptr;
    std::unique_ptr<HostPath> host;  // pipelined host-buffer allreduce (rdc_host.h)
    int group_counter = 0;           // unnamed CreateGroup communicators: "group<k>" (same k on every rank)
};

Manager& M() {
    static Manager* m = new Manager();  // never destroyed: may outlive HIP teardown
    return *m;
}

// ParseUnit (src/comm/communicator_manager.cc:14-42): {integer}{B,K,M,G}
size_t parse_unit(const char* v) {
    char unit = 0;
    unsigned long amt = 0;
    int k = sscanf(v, "%lu%c", &amt, &unit);
    if (k == 2) {
        switch (unit) {
            case 'B': return amt;
            case 'K': return (size_t)amt << 10;
            case 'M': return (size_t)amt << 20;
            case 'G': return (size_t)amt << 30;
            default: throw std::invalid_argument(std::string("rdc: bad size ") + v);
        }
    }
    if (k == 1) return amt;
    throw std::invalid_argument(std::string("rdc: bad size ") + v);
}

void set_param(Manager& m, const char* name, const char* val) {
    std::string k(name);
    if (k == "RDC_TRACKER_URI") m.tracker_uri = val;
    else if (k == "RDC_TRACKER_PORT") m.tracker_port = atoi(val);
    else if (k == "rdc_world_size" || k == "RDC_WORLD_SIZE") m.world = atoi(val);
    else if (k == "RDC_RANK" || k == "rdc_rank") m.rank = atoi(val);
    else if (k == "rdc_reduce_ring_mincount") m.cfg.ring_mincount = parse_unit(val);
    else if (k == "RDC_DEVICE") m.device = atoi(val);
    else if (k == "RDC_SCRATCH_BYTES" || k == "rdc_reduce_buffer") m.cfg.scratch_bytes = parse_unit(val);
    else if (k == "RDC_ALGO") {
        std::string v(val);
        m.cfg.algo = v == "ring" ? RDC_ALGO_RING : v == "mesh" ? RDC_ALGO_MESH : v == "mesh_pull" ? RDC_ALGO_MESH_PULL
                     : v == "direct" ? RDC_ALGO_DIRECT
                     : v == "oneshot" ? RDC_ALGO_ONESHOT : RDC_ALGO_AUTO;
        // (the tree is chosen by size through rdc_reduce_ring_mincount, as in the reference)
    } else if (k == "RDC_NBLOCKS") m.cfg.max_blocks = atoi(val);
    else if (k == "RDC_TILE_BYTES") m.cfg.tile_bytes = parse_unit(val);
    else if (k == "RDC_TIMEOUT") m.cfg.timeout_s = atof(val);
    else if (k == "RDC_ONESHOT_BYTES") m.cfg.oneshot_push_max = parse_unit(val);
    else if (k == "RDC_FUSE_BYTES") m.cfg.fuse_bytes = std::max<size_t>(parse_unit(val), 1);
    else if (k == "RDC_BOOTSTRAP_TIMEOUT") m.bootstrap_timeout_s = atof(val);
    else if (k == "RDC_HOST_ZC_BYTES") m.host_zc_bytes = parse_unit(val);
    else if (k == "RDC_COALESCE_FUSED") m.cfg.coalesce_fused = atoi(val) != 0;
    else if (k == "RDC_BCAST_SPLIT_BYTES") m.cfg.bcast_split_bytes = parse_unit(val);
    else if (k == "RDC_MESH_SPLIT") {
        int s = 0, r = 0;
        if (sscanf(val, "%d,%d", &s, &r) != 2 || s < 1 || r < 1 || s + r > 15)
            throw std::invalid_argument(std::string("rdc: RDC_MESH_SPLIT wants s,r sixteenths (s+r<=15), got ") + val);
        m.cfg.mesh_split.s16 = s;
        m.cfg.mesh_split.r16 = r;
    }
    else if (k == "RDC_FUSE_BYTES_DIRECT") m.cfg.fuse_bytes_direct = std::max<size_t>(parse_unit(val), 1);
    else if (k == "RDC_POISON_SCRATCH") m.cfg.poison = atoi(val) != 0 ? 1 : 0;
    else if (k == "RDC_DIRECT_BYTES") m.cfg.direct_min = strcmp(val, "auto") == 0 ? kDirectMinAuto : parse_unit(val);
    else if (k == "RDC_P2P_SLOT_BYTES") m.cfg.p2p_slot_bytes = std::max<size_t>(parse_unit(val) / 4096 * 4096, 4096);
    // other reference keys (RDC_HEARTBEAT_INTERVAL, RDC_RESTART, ...) belong
    // to subsystems outside the device path and are accepted silently
}

void env_param(Manager& m, const char* name) {
    const char* v = getenv(name);
    if (v && *v) set_param(m, name, v);
}

template <typename F>
int guard(F&& f) {
    try {
        f();
        g_last_error.clear();
        return 0;
    } catch (const std::exception& e) {
        g_last_error = e.what();
    } catch (...) {
        g_last_error = "rdc: unknown error";
    }
    return 1;
}

void require_init(Manager& m) {
    if (!m.inited) throw std::runtime_error("rdc: RdcInit has not been called");
}

int pick_device(Manager& m) {
    if (m.device >= 0) return m.device;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        throw std::runtime_error("rdc: no HIP device visible (the MI355X path has no CPU fallback)");
    const char* lr = getenv("LOCAL_RANK");
    int d = lr ? atoi(lr) : m.rank;
    m.device = d % ndev;
    return m.device;
}

Communicator* get_comm(Manager& m, const std::string& name, bool create) {
    auto it = m.comms.find(name);
    if (it != m.comms.end()) return it->second.get();
    if (!create) throw std::runtime_error("rdc: communicator '" + name + "' does not exist");
    require_init(m);
    Communicator* c = Communicator::Create(name, m.bs.get(), m.world == 1 ? std::max(m.device, 0) : pick_device(m),
                                           m.cfg);
    m.comms[name].reset(c);
    return c;
}

Communicator* as_comm(void* h) {
    if (!h) throw std::invalid_argument("rdc: null communicator handle");
    return static_cast<Communicator*>(h);
}

bool is_device_pointer(const void* p) {
    hipPointerAttribute_t attr;
    memset(&attr, 0, sizeof(attr));
    hipError_t e = hipPointerGetAttributes(&attr, p);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged;
}

hipStream_t manager_stream(Manager& m, int device) {
    if (!m.stream) {
        // a blocking stream: synchronous calls on device memory are ordered
        // after the work the caller queued on the null (default) stream
        if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&m.stream, hipStreamDefault) != hipSuccess)
            throw std::runtime_error("rdc: cannot create stream");
    }
    return m.stream;
}

void* staging(Manager& m, size_t bytes, int device) {
    if (bytes > m.stage_bytes) {
        if (m.stage) (void)hipFree(m.stage);
        m.stage = nullptr;
        m.stage_bytes = 0;
        (void)hipSetDevice(device);
        if (hipMalloc(&m.stage, bytes) != hipSuccess) throw std::runtime_error("rdc: cannot allocate staging buffer");
        m.stage_bytes = bytes;
    }
    return m.stage;
}

void hcheck(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string("rdc: ") + what + ": " + hipGetErrorString(e));
}

}  // namespace

extern "C" {

int RdcInit(int argc, char** argv) {
    Manager& m = M();
    std::lock_guard<std::recursive_mutex> lk(m.mu);
    if (m.inited) return 0;
    return guard([&] {
        // torchrun-style fallbacks first, rdc names override, argv overrides all
        if (const char* v = getenv("RANK")) m.rank = atoi(v);
        if (const char* v = getenv("WORLD_SIZE")) m.world = atoi(v);
        if (const char* v = getenv("MASTER_ADDR")) m.tracker_uri = v;
        if (const char* v = getenv("MASTER_PORT")) m.tracker_port = atoi(v) + 1;
        static const char* keys[] = {"RDC_TRACKER_URI", "RDC_TRACKER_PORT", "RDC_WORLD_SIZE", "rdc_world_size",
                                     "RDC_RANK", "rdc_reduce_ring_mincount", "RDC_DEVICE", "RDC_SCRATCH_BYTES",
                                     "RDC_ALGO", "RDC_NBLOCKS", "RDC_TILE_BYTES", "RDC_TIMEOUT",
                                     "RDC_BOOTSTRAP_TIMEOUT", "RDC_ONESHOT_BYTES", "RDC_FUSE_BYTES",
                                     "RDC_P2P_SLOT_BYTES", "RDC_COALESCE_FUSED", "RDC_HOST_ZC_BYTES",
                                     "RDC_FUSE_BYTES_DIRECT", "RDC_BCAST_SPLIT_BYTES", "RDC_MESH_SPLIT",
                                     "RDC_POISON_SCRATCH", "RDC_DIRECT_BYTES"};
        for (const char* k : keys) env_param(m, k);
        m.env_loaded = true;
        for (int i = 0; i < argc; ++i) {
            if (!argv || !argv[i]) continue;
            char name[256], val[256];
            if (sscanf(argv[i], "%255[^=]=%255s", name, val) == 2) set_param(m, name, val);
        }
        if (m.world < 1 || m.rank < 0 || m.rank >= m.world)
            throw std::invalid_argument("rdc: bad rank " + std::to_string(m.rank) + " / world " +
                                        std::to_string(m.world));
        if (m.world > RDC_MAX_RANKS) throw std::invalid_argument("rdc: world size exceeds 16");
        m.bs.reset(new TcpBootstrap(m.rank, m.world, m.tracker_uri, m.tracker_port, m.bootstrap_timeout_s));
        m.inited = true;
    });
}

int RdcFinalize(void) {
    Manager& m = M();
    std::lock_guard<std::recursive_mutex> lk(m.mu);
    if (!m.inited) return 0;
    return guard([&] {
        m.host.reset();
        m.comms.clear();  // collective destroys (barriers) in name order on every rank
        if (m.stage) (void)hipFree(m.stage);
        m.stage = nullptr;
        m.stage_bytes = 0;
        if (m.stream) (void)hipStreamDestroy(m.stream);
        m.stream = nullptr;
        if (m.bs) m.bs->barrier();
        m.bs.reset();
        m.inited = false;
        m.rank = 0;
        m.world = 1;
    });
}

int RdcGetRank(void) { return M().rank; }
int RdcGetWorldSize(void) { return M().world; }
int RdcIsDistributed(void) { return M().world > 1 ? 1 : 0; }

int RdcTrackerPrint(const char* msg) {
    fprintf(stderr, "[rdc rank %d] %s\n", M().rank, msg ? msg : "");
    fflush(stderr);
    return 0;
}

int RdcGetProcessorName(char* buf, unsigned long* out_len, unsigned long max_len) {
    return guard([&] {
        if (!buf || max_len == 0) throw std::invalid_argument("rdc: bad buffer");
        char host[256] = {0};
        gethostname(host, sizeof(host) - 1);
        size_t n = strnlen(host, sizeof(host));
        if (n >= max_len) n = max_len - 1;
        memcpy(buf, host, n);
        buf[n] = 0;
        if (out_len) *out_len = n;
    });
}

int RdcBarrier(void) {
    Manager& m = M();
    std::lock_guard<std::recursive_mutex> lk(m.mu);
    return guard([&] {
        require_init(m);
        m.bs->barrier();
    });
}

int RdcNewCommunicator(void** out, const char* name) {
    Manager& m = M();
    std::lock_guard<std::recursive_mutex> lk(m.mu);
    return guard([&] {
        if (!out || !name) throw std::invalid_argument("rdc: null argument");
        *out = get_comm(m, name, true);
    });
}

int RdcCreateGroup(void** out, void* parent, const int* ranks, int nranks, const char* name) {
    Manager& m = M();
    std::lock_guard<std::recursive_mutex> lk(m.mu);
    return guard([&] {
        if (!out || (nranks > 0 && !ranks) || nranks < 1) throw std::invalid_argument("rdc: bad CreateGroup arguments");
        *out = nullptr;
        require_init(m);
        Communicator* p = parent ? as_comm(parent) : get_comm(m, "main", true);
        const std::string nm = name && *name ? std::string(name) : "group" + std::to_string(m.group_counter);
        ++m.group_counter;
        if (!p->bootstrap()) throw std::runtime_error("rdc: CreateGroup needs a multi-process communicator");
        // the name must be free on every member (checked collectively: a
        // member that refused alone would leave the others waiting)
        std::vector<int> rs(ranks, ranks + nranks);
        char taken = 0;
        for (int r : rs)
            if (r == p->rank() && m.comms.count(nm)) taken = 1;
        std::vector<char> all((size_t)p->size());
        p->bootstrap()->allgather(&taken, 1, all.data());
        for (char t : all)
            if (t) throw std::invalid_argument("rdc: communicator '" + nm + "' already exists on a member");
        Communicator* c = Communicator::CreateSubset(nm, p, rs, p->config());
        if (c) m.comms[nm].reset(c);
        *out = c;
    });
}

int RdcGetCommunicator(void** out, const char* name) {
    Manager& m = M();
    std::lock_guard<std::recursive_mutex> lk(m.mu);
    return guard([&] {
        if (!out) throw std::invalid_argument("rdc: null argument");
        // the reference aborts on a missing name (communicator_manager.cc:190-193);
        // "main" is created on first use instead
        std::string n = name ? name : "main";
        *out = get_comm(m, n, n == "main");
    });
}

namespace {

void check_dtype_op(int dtype, int op) {
    if (rdc_dtype_size(dtype) == 0) throw std::invalid_argument("rdc: bad dtype " + std::to_string(dtype));
    if (op < 0 || op >= RDC_OP_COUNT) throw std::invalid_argument("rdc: bad op " + std::to_string(op));
    if (op == RDC_OP_BITOR && rdc_dtype_is_float(dtype))
        throw std::invalid_argument("rdc: BITOR needs an integer dtype");
}

// synchronous allreduce of host or device memory on communicator c
void allreduce_sync(Manager& m, Communicator* c, void* sendrecv, size_t count, int dtype, int op) {
    check_dtype_op(dtype, op);
    if (c->size() == 1 || count == 0) return;
    hipStream_t s = manager_stream(m, c->device());
    if (is_device_pointer(sendrecv)) {
        // the manager's stream is ordered after the caller's null-stream
        // work; completion is the launch's own token (no stream sync)
        const uint32_t token = c->ArmNotify();
        try {
            c->Allreduce(sendrecv, count, dtype, op, s);
        } catch (...) {
            c->WaitNotify(token, s);  // disarms
            throw;
        }
        c->WaitNotify(token, s);
        return;
    }
    // host-resident buffer: pieces of every chunk through pinned slots, H2D /
    // allreduce / D2H overlapped on three streams
    if (!m.host) m.host.reset(new HostPath(c->device(), m.host_zc_bytes));
    // the copy path comes up only for buffers that use it (the service and
    // the zero-copy path below HostPath::kSmall never DMA)
    if (count * rdc_dtype_size(dtype) > HostPath::kSmall) m.host->Warm(s);
    m.host->Allreduce(c, sendrecv, count, dtype, op, s);
}

// synchronous coalesced allreduce of host or device buffers (all of one kind)
void allreduce_coalesced_sync(Manager& m, Communicator* c, void** bufs, const size_t* counts, int nbuf, int dtype,
                              int op) {
    check_dtype_op(dtype, op);
    if (nbuf < 0 || (nbuf > 0 && (!bufs || !counts))) throw std::invalid_argument("rdc: bad buffer list");
    if (c->size() == 1 || nbuf == 0) return;
    hipStream_t s = manager_stream(m, c->device());
    int ndev = 0, nhost = 0;
    for (int b = 0; b < nbuf; ++b)
        if (counts[b]) (is_device_pointer(bufs[b]) ? ndev : nhost)++;
    if (nhost == 0) {
        c->AllreduceCoalesced(bufs, counts, nbuf, dtype, op, s);
        c->Check(s);
        return;
    }
    if (ndev) throw std::invalid_argument("rdc: coalesced allreduce needs all-host or all-device buffers");
    // host buffers: one HBM image (256-B aligned per buffer), H2D, device path, D2H
    const size_t esz = rdc_dtype_size(dtype);
    std::vector<size_t> at((size_t)nbuf);
    size_t total = 0;
    for (int b = 0; b < nbuf; ++b) {
        at[(size_t)b] = total;
        total += (counts[b] * esz + 255) / 256 * 256;
    }
    char* d = static_cast<char*>(staging(m, std::max<size_t>(total, 256), c->device()));
    std::vector<void*> dbufs((size_t)nbuf);
    for (int b = 0; b < nbuf; ++b) {
        dbufs[(size_t)b] = d + at[(size_t)b];
        if (counts[b]) hcheck(hipMemcpyAsync(dbufs[(size_t)b], bufs[b], counts[b] * esz, hipMemcpyHostToDevice, s), "H2D");
    }
    c->AllreduceCoalesced(dbufs.data(), counts, nbuf, dtype, op, s);
    for (int b = 0; b < nbuf; ++b)
        if (counts[b]) hcheck(hipMemcpyAsync(bufs[b], dbufs[(size_t)b], counts[b] * esz, hipMemcpyDeviceToHost, s), "D2H");
    c->Check(s);
}

void broadcast_sync(Manager& m, Communicator* c, void* sendrecv, size_t size, int root) {
    if (root < 0 || root >= c->size()) throw std::invalid_argument("rdc: broadcast root out of range");
    if (c->size() == 1 || size == 0) return;
    hipStream_t s = manager_stream(m, c->device());
    if (is_device_pointer(sendrecv)) {
        c->Broadcast(sendrecv, size, root, s);
        c->Check(s);
        return;
    }
    void* d = staging(m, size, c->device());
    if (c->rank() == root) hcheck(hipMemcpyAsync(d, sendrecv, size, hipMemcpyHostToDevice, s), "H2D");
    c->Broadcast(d, size, root, s);
    if (c->rank() != root) hcheck(hipMemcpyAsync(sendrecv, d, size, hipMemcpyDeviceToHost, s), "D2H");
    c->Check(s);
}

void allgather_sync(Manager& m, Communicator* c, void** bufs, const size_t* sizes) {
    if (!bufs || !sizes) throw std::invalid_argument("rdc: null argument");
    const int n = c->size();
    if (n == 1) return;
    std::vector<uint64_t> sz((size_t)n);
    for (int i = 0; i < n; ++i) sz[(size_t)i] = sizes[i];
    hipStream_t s = manager_stream(m, c->device());
    if (is_device_pointer(bufs[c->rank()]) || sz[(size_t)c->rank()] == 0) {
        bool dev = true;
        for (int i = 0; i < n; ++i)
            if (sz[(size_t)i] && !is_device_pointer(bufs[i])) dev = false;
        if (dev) {
            c->Allgather(bufs, sz.data(), s);
            c->Check(s);
            return;
        }
    }
    // host buffers: one staging image in HBM (256-B aligned per rank)
    std::vector<size_t> at((size_t)n);
    size_t total = 0;
    for (int i = 0; i < n; ++i) {
        at[(size_t)i] = total;
        total += (sz[(size_t)i] + 255) / 256 * 256;
    }
    char* d = static_cast<char*>(staging(m, std::max<size_t>(total, 256), c->device()));
    std::vector<void*> dbufs((size_t)n);
    for (int i = 0; i < n; ++i) dbufs[(size_t)i] = d + at[(size_t)i];
    const int r = c->rank();
    if (sz[(size_t)r])
        hcheck(hipMemcpyAsync(dbufs[(size_t)r], bufs[r], sz[(size_t)r], hipMemcpyHostToDevice, s), "H2D");
    c->Allgather(dbufs.data(), sz.data(), s);
    for (int i = 0; i < n; ++i)
        if (i != r && sz[(size_t)i])
            hcheck(hipMemcpyAsync(bufs[i], dbufs[(size_t)i], sz[(size_t)i], hipMemcpyDeviceToHost, s), "D2H");
    c->Check(s);
}

}  // namespace

int RdcAllgather(void** bufs, const size_t* sizes) {
    Manager& m = M();
    std::lock_guard<std::recursive_mutex> lk(m.mu);
    return guard([&] {
        require_init(m);
        if (m.world == 1) return;
        allgather_sync(m, get_comm(m, "main", true), bufs, sizes);
    });
}

int RdcAllgatherOn(void* comm, void** bufs, const size_t* sizes) {
    Manager& m = M();
    std::lock_guard<std::recursive_mutex> lk(m.mu);
    return guard([&] { allgather_sync(m, as_comm(comm), bufs, sizes); });
}

int RdcCommAllgather(void* comm, void** dev_bufs, const size_t* sizes, void* stream) {
    return guard([&] {
        Communicator* c = as_comm(comm);
        if (!dev_bufs || !sizes) throw std::invalid_argument("rdc: null argument");
        std::vector<uint64_t> sz((size_t)c->size());
        for (int i = 0; i < c->size(); ++i) sz[(size_t)i] = sizes[i];
        c->Allgather(dev_bufs, sz.data(), static_cast<hipStream_t>(stream));
    });
}

int RdcAllreduce(void* sendrecv, size_t count, int dtype, int op, void (*prepare_fun)(void*), void* prepare_arg) {
    Manager& m = M();
    std::lock_guard<std::recursive_mutex> lk(m.mu);
    return guard([&] {
        require_init(m);
        if (prepare_fun) prepare_fun(prepare_arg);
        check_dtype_op(dtype, op);
        // world size 1: Communicator::Allreduce returns at once (communicator_base.h:133-138)
        if (m.world == 1 || count == 0) return;
        allreduce_sync(m, get_comm(m, "main", true), sendrecv, count, dtype, op);
    });
}

int RdcAllreduceCoalesced(void** bufs, const size_t* counts, int nbuf, int dtype, int op) {
    Manager& m = M();
    std::lock_guard<std::recursive_mutex> lk(m.mu);
    return guard([&] {
        require_init(m);
        check_dtype_op(dtype, op);
        if (m.world == 1 || nbuf == 0) return;
        allreduce_coalesced_sync(m, get_comm(m, "main", true), bufs, counts, nbuf, dtype, op);
    });
}

int RdcAllreduceCoalescedOn(void* comm, void** bufs, const size_t* counts, int nbuf, int dtype, int op) {
    Manager& m = M();
    std::lock_guard<std::recursive_mutex> lk(m.mu);
    return guard([&] { allreduce_coalesced_sync(m, as_comm(comm), bufs, counts, nbuf, dtype, op); });
}

int RdcCommAllreduceCoalesced(void* comm, void* const* dev_bufs, const size_t* counts, int nbuf, int dtype, int op,
                              int algo, void* stream) {
    return guard([&] {
        if (algo < RDC_ALGO_AUTO || algo > RDC_ALGO_DIRECT) throw std::invalid_argument("rdc: bad algo");
        as_comm(comm)->AllreduceCoalesced(dev_bufs, counts, nbuf, dtype, op, static_cast<hipStream_t>(stream), algo);
    });
}

int RdcBroadcast(void* sendrecv, unsigned long size, int root) {
    Manager& m = M();
    std::lock_guard<std::recursive_mutex> lk(m.mu);
    return guard([&] {
        require_init(m);
        if (root < 0 || root >= m.world) throw std::invalid_argument("rdc: broadcast root out of range");
        if (m.world == 1 || size == 0) return;
        broadcast_sync(m, get_comm(m, "main", true), sendrecv, size, root);
    });
}

int RdcAllreduceOn(void* comm, void* sendrecv, size_t count, int dtype, int op) {
    Manager& m = M();
    std::lock_guard<std::recursive_mutex> lk(m.mu);
    return guard([&] { allreduce_sync(m, as_comm(comm), sendrecv, count, dtype, op); });
}

int RdcBroadcastOn(void* comm, void* sendrecv, size_t size, int root) {
    Manager& m = M();
    std::lock_guard<std::recursive_mutex> lk(m.mu);
    return guard([&] { broadcast_sync(m, as_comm(comm), sendrecv, size, root); });
}

int RdcCommAllreduce(void* comm, void* dev_buf, size_t count, int dtype, int op, void* stream) {
    return RdcCommAllreduceEx(comm, dev_buf, count, dtype, op, RDC_ALGO_AUTO, stream);
}

int RdcCommAllreduceEx(void* comm, void* dev_buf, size_t count, int dtype, int op, int algo, void* stream) {
    return guard([&] {
        if (algo < RDC_ALGO_AUTO || algo > RDC_ALGO_DIRECT) throw std::invalid_argument("rdc: bad algo");
        as_comm(comm)->Allreduce(dev_buf, count, dtype, op, static_cast<hipStream_t>(stream), algo);
    });
}

int RdcCommBroadcast(void* comm, void* dev_buf, size_t bytes, int root, void* stream) {
    return guard([&] { as_comm(comm)->Broadcast(dev_buf, bytes, root, static_cast<hipStream_t>(stream)); });
}

int RdcCommCheck(void* comm, void* stream) {
    return guard([&] { as_comm(comm)->Check(static_cast<hipStream_t>(stream)); });
}

int RdcCommTune(void* comm, int mesh_s16, int mesh_r16, int max_blocks, size_t tile_bytes) {
    return guard([&] { as_comm(comm)->Tune(mesh_s16, mesh_r16, max_blocks, tile_bytes); });
}

int RdcCommSetPoison(void* comm, int on) {
    return guard([&] { as_comm(comm)->SetPoison(on != 0); });
}

int RdcCommDirectRelease(void* comm) {
    return guard([&] { as_comm(comm)->DirectUnmapAll(); });
}

int RdcCommAutotune(void* comm, size_t bytes, int dtype, int reps, void* stream, RdcTuneCand* cand, int max_cand,
                    int* ncand, int* best) {
    return guard([&] {
        if (!cand || !ncand || !best || max_cand <= 0) throw std::invalid_argument("rdc: null argument");
        std::vector<rdc_amd::Communicator::TuneCand> c((size_t)max_cand);
        int b = -1;
        const int k = as_comm(comm)->Autotune(bytes, dtype, reps, static_cast<hipStream_t>(stream), c.data(),
                                              max_cand, &b);
        for (int i = 0; i < k; ++i) cand[i] = RdcTuneCand{c[i].algo, c[i].s16, c[i].r16, c[i].grid, c[i].tpb, c[i].ms, c[i].ms_min,
                                                     c[i].ms_max};
        *ncand = k;
        *best = b;
    });
}

int RdcCommProbe(void* comm, int mode, size_t bytes, int reps, void* stream, double* ms_out, size_t* bytes_out) {
    return guard([&] {
        if (!ms_out) throw std::invalid_argument("rdc: null argument");
        *ms_out = as_comm(comm)->Probe(mode, &bytes, reps, static_cast<hipStream_t>(stream));
        if (bytes_out) *bytes_out = bytes;
    });
}

int RdcCommTraceNext(void* comm, void* dev_words, size_t nwords) {
    return guard([&] { as_comm(comm)->TraceNext(static_cast<uint64_t*>(dev_words), dev_words ? nwords : 0); });
}

int RdcCommLastLaunch(void* comm, uint64_t* out6) {
    return guard([&] {
        if (!out6) throw std::invalid_argument("rdc: null argument");
        as_comm(comm)->LastLaunch(out6);
    });
}

int RdcCommLaunchCounter(void* comm, uint64_t* value) {
    return guard([&] {
        if (!value) throw std::invalid_argument("rdc: null argument");
        *value = as_comm(comm)->LaunchCounter();
    });
}

int RdcCommSetLaunchCounter(void* comm, uint64_t value) {
    return guard([&] { as_comm(comm)->SetLaunchCounter(value); });
}

int RdcCommGetParam(void* comm, const char* key, uint64_t* value) {
    return guard([&] {
        if (!key || !value) throw std::invalid_argument("rdc: null argument");
        Communicator* c = as_comm(comm);
        const CommConfig& g = c->config();
        const std::string k(key);
        if (k == "rdc_reduce_ring_mincount") *value = g.ring_mincount;
        else if (k == "RDC_SCRATCH_BYTES") *value = g.scratch_bytes;
        else if (k == "RDC_TILE_BYTES") *value = g.tile_bytes;
        else if (k == "RDC_NBLOCKS") *value = (uint64_t)g.max_blocks;
        else if (k == "RDC_ONESHOT_BYTES") *value = g.oneshot_push_max;
        else if (k == "slot_bytes") *value = c->slot_bytes();
        else if (k == "ranks_per_gpu") *value = (uint64_t)c->ranks_per_gpu();
        else if (k == "coalesced_misaligned") *value = (uint64_t)c->coalesced_misaligned_;
        else if (k == "shares_scratch") *value = c->shares_channel() ? 1 : 0;
        else if (k == "host_registered_calls") *value = HostRegisteredCalls();
        else if (k == "direct_check") *value = (uint64_t)c->DirectCheckResult();
        else if (k == "flags_kind") *value = (uint64_t)c->region_kind(2);    // 3 = HSA-uncached (MTYPE UC)
        else if (k == "scratch_kind") *value = (uint64_t)c->region_kind(0);
        else if (k.compare(0, 7, "direct_") == 0) *value = c->DirectStat(k);
        else if (k == "RDC_DIRECT_BYTES") *value = g.direct_min;
        else throw std::invalid_argument("rdc: unknown parameter " + k);
    });
}

int RdcCommRank(void* comm) { return comm ? static_cast<Communicator*>(comm)->rank() : -1; }
int RdcCommSize(void* comm) { return comm ? static_cast<Communicator*>(comm)->size() : -1; }
int RdcCommDevice(void* comm) { return comm ? static_cast<Communicator*>(comm)->device() : -1; }
int RdcCommAllocKind(void* comm) { return comm ? static_cast<Communicator*>(comm)->alloc_kind() : -1; }

int RdcCommInitAll(void** comms, int n, const int* devices, size_t scratch_bytes) {
    Manager& m = M();
    std::lock_guard<std::recursive_mutex> lk(m.mu);
    return guard([&] {
        if (!comms || !devices) throw std::invalid_argument("rdc: null argument");
        // parameters from the environment even without RdcInit
        static const char* keys[] = {"RDC_SCRATCH_BYTES", "RDC_ALGO", "RDC_NBLOCKS", "RDC_TILE_BYTES",
                                     "RDC_TIMEOUT", "RDC_ONESHOT_BYTES", "RDC_FUSE_BYTES", "RDC_P2P_SLOT_BYTES",
                                     "RDC_COALESCE_FUSED", "RDC_FUSE_BYTES_DIRECT",
                                     "RDC_BCAST_SPLIT_BYTES", "RDC_MESH_SPLIT", "rdc_reduce_ring_mincount",
                                     "RDC_POISON_SCRATCH"};
        if (!m.inited && !m.env_loaded) {
            for (const char* k : keys) env_param(m, k);
            m.env_loaded = true;
        }
        CommConfig cfg = m.cfg;
        if (scratch_bytes) cfg.scratch_bytes = scratch_bytes;
        std::vector<Communicator*> out;
        Communicator::CreateGroup("group", n, devices, cfg, &out);
        for (int i = 0; i < n; ++i) {
            m.groups[out[(size_t)i]].reset(out[(size_t)i]);
            comms[i] = out[(size_t)i];
        }
    });
}

int RdcCommDestroy(void* comm) {
    Manager& m = M();
    std::lock_guard<std::recursive_mutex> lk(m.mu);
    return guard([&] {
        Communicator* c = as_comm(comm);
        auto g = m.groups.find(c);
        if (g != m.groups.end()) {
            m.groups.erase(g);
            return;
        }
        for (auto it = m.comms.begin(); it != m.comms.end(); ++it) {
            if (it->second.get() == c) {
                m.comms.erase(it);
                return;
            }
        }
        throw std::invalid_argument("rdc: unknown communicator handle");
    });
}

int RdcReduce(void* dst, const void* src, size_t count, int dtype, int op, void* stream) {
    return guard([&] { DeviceReduce(dst, src, count, dtype, op, static_cast<hipStream_t>(stream)); });
}

int RdcMemcpy(void* dst, const void* src, size_t bytes) {
    return guard([&] {
        if (bytes == 0) return;
        if (!dst || !src) throw std::invalid_argument("rdc: null argument");
        if (!is_device_pointer(dst) && !is_device_pointer(src)) {
            memcpy(dst, src, bytes);
            return;
        }
        hcheck(hipMemcpy(dst, src, bytes, hipMemcpyDefault), "copy");
    });
}

int RdcFill(void* dev_buf, size_t count, int dtype, uint64_t seed, int rank, void* stream) {
    return guard([&] { DeviceFill(dev_buf, count, dtype, seed, rank, static_cast<hipStream_t>(stream)); });
}

int RdcPlanTree(int n, int* dst, int* src) {
    if (n < 1 || n > RDC_MAX_RANKS || !dst || !src) return -1;
    return PlanTreeProgram(n, dst, src);
}

int RdcPlanResidentGrid(int want, int blocks_per_cu, int cus, int ranks_per_gpu) {
    return ResidentGrid(want, blocks_per_cu, cus, ranks_per_gpu);
}

int RdcPlanResidentGridXcd(int want, int blocks_per_cu, int cus, int ranks_per_gpu, int xcds, int reserve_cus) {
    return ResidentGrid(want, blocks_per_cu, cus, ranks_per_gpu, xcds, reserve_cus);
}

int RdcPlanLayout(int n, size_t scratch_bytes, uint64_t* out4) {
    return guard([&] {
        if (n < 1 || n > RDC_MAX_RANKS || !out4) throw std::invalid_argument("rdc: bad argument");
        const Layout L = MakeLayout(n, scratch_bytes ? scratch_bytes : CommConfig().scratch_bytes);
        out4[0] = L.slot_bytes;
        out4[1] = L.region_bytes;
        out4[2] = L.max_tiles;
        out4[3] = L.flag_bytes;
    });
}

int RdcPlanAutoAlgo(int n, size_t bytes, size_t scratch_bytes, size_t oneshot_bytes) {
    int algo = -1;
    const int rc = guard([&] {
        if (n < 1 || n > RDC_MAX_RANKS) throw std::invalid_argument("rdc: bad argument");
        const Layout L = MakeLayout(n, scratch_bytes ? scratch_bytes : CommConfig().scratch_bytes);
        algo = AutoAlgo(n, bytes, L, oneshot_bytes);
    });
    return rc != 0 ? rc : algo;
}

int RdcPlanDirectAuto(int n, size_t bytes, size_t scratch_bytes, size_t oneshot_bytes, uint64_t direct_min) {
    int on = -1;
    const int rc = guard([&] {
        if (n < 1 || n > RDC_MAX_RANKS) throw std::invalid_argument("rdc: bad argument");
        const Layout L = MakeLayout(n, scratch_bytes ? scratch_bytes : CommConfig().scratch_bytes);
        on = DirectAuto(n, bytes, L, oneshot_bytes, direct_min) ? 1 : 0;
    });
    return rc != 0 ? rc : on;
}

int RdcPlanHbmBytes(int n, size_t count, int dtype, int algo, uint64_t* out5) {
    return guard([&] {
        const size_t esz = rdc_dtype_size(dtype);
        if (n < 1 || n > RDC_MAX_RANKS || esz == 0 || !out5 ||
            (algo != RDC_ALGO_RING && algo != RDC_ALGO_MESH && algo != RDC_ALGO_ONESHOT && algo != RDC_ALGO_TREE &&
             algo != RDC_ALGO_MESH_PULL && algo != RDC_ALGO_DIRECT))
            throw std::invalid_argument("rdc: bad argument");
        const HbmBytes h = ModelHbmBytes(n, count, esz, algo);
        out5[0] = h.read_max;
        out5[1] = h.write_max;
        out5[2] = h.read_sum;
        out5[3] = h.write_sum;
        out5[4] = h.egress_max;
    });
}

int RdcPlanHostPieceRanges(int n, size_t count, int dtype, uint64_t lo, uint64_t hi, int balanced, uint64_t* off,
                           uint64_t* len, int* fold) {
    return guard([&] {
        const size_t esz = rdc_dtype_size(dtype);
        if (n < 1 || n > RDC_MAX_RANKS || esz == 0 || !off || !len || !fold || lo > hi || hi > (uint64_t)count * esz ||
            lo % esz || hi % esz)
            throw std::invalid_argument("rdc: bad argument");
        int64_t cb[RDC_MAX_RANKS], ce[RDC_MAX_RANKS];
        SplitRanges((int64_t)count, n, cb, ce);
        int8_t f[RDC_MAX_RANKS];
        HostPieceRanges(lo, hi, n, cb, ce, esz, balanced != 0, off, len, f);
        for (int q = 0; q < n; ++q) fold[q] = f[q];
    });
}

int RdcPlanHostPieces(size_t bytes, uint64_t* bounds, int max_bounds, int* out_n) {
    return guard([&] {
        if (!bounds || !out_n || max_bounds < 2) throw std::invalid_argument("rdc: bad argument");
        const std::vector<uint64_t> b = rdc_amd::HostPieceBounds(bytes);
        *out_n = (int)b.size();
        for (size_t i = 0; i < b.size() && i < (size_t)max_bounds; ++i) bounds[i] = b[i];
    });
}

int RdcPlanAllreduce(int n, size_t count, int dtype, size_t scratch_bytes, int algo, size_t tile_bytes,
                     int max_blocks, uint64_t* out, int max_pieces, int* out_pieces) {
    return guard([&] {
        const size_t esz = rdc_dtype_size(dtype);
        if (n < 1 || n > RDC_MAX_RANKS || esz == 0 || !out_pieces) throw std::invalid_argument("rdc: bad argument");
        if (algo == RDC_ALGO_AUTO) algo = RDC_ALGO_MESH;
        const Layout L = MakeLayout(n, scratch_bytes ? scratch_bytes : CommConfig().scratch_bytes);
        const std::vector<Piece> plan = PlanAllreduce(n, count, esz, L, algo, tile_bytes, max_blocks > 0 ? max_blocks : 256);
        *out_pieces = (int)plan.size();
        for (int k = 0; k < (int)plan.size() && k < max_pieces && out; ++k) {
            uint64_t* o = out + (size_t)k * RDC_PLAN_WORDS;
            const Piece& p = plan[(size_t)k];
            o[0] = p.tile_bytes;
            o[1] = (uint64_t)p.nb_scatter;
            o[2] = (uint64_t)p.nb_reduce;
            o[3] = (uint64_t)p.nb_gather;
            for (int c = 0; c < RDC_MAX_RANKS; ++c) {
                o[4 + c] = p.off[c];
                o[20 + c] = p.len[c];
                o[36 + c] = p.mis[c];
                o[52 + c] = (uint64_t)p.tiles[c];
            }
        }
    });
}

int RdcPlanDirectItems(int n, int rank, const size_t* counts, int nbuf, int dtype, uint64_t tile, uint64_t* out,
                       int max_items, int* out_items) {
    return guard([&] {
        const size_t esz = rdc_dtype_size(dtype);
        if (n < 1 || n > RDC_MAX_RANKS || rank < 0 || rank >= n || esz == 0 || nbuf < 0 || (nbuf && !counts) ||
            tile == 0 || !out_items)
            throw std::invalid_argument("rdc: bad argument");
        std::vector<uint64_t> bytes((size_t)nbuf);
        for (int b = 0; b < nbuf; ++b) bytes[(size_t)b] = (uint64_t)counts[b] * esz;
        const std::vector<uint64_t> items = PlanDirectItems(n, rank, bytes.data(), nbuf, esz, tile);
        *out_items = (int)(items.size() / 3);
        for (size_t i = 0; i < items.size() && out && (int)(i / 3) < max_items; ++i) out[i] = items[i];
    });
}

int RdcPlanCoalesced(int n, const size_t* counts, int nbuf, int dtype, uint64_t* chunk_out, uint64_t* units_out,
                     int max_units, int* out_units) {
    return guard([&] {
        const size_t esz = rdc_dtype_size(dtype);
        if (n < 1 || n > RDC_MAX_RANKS || esz == 0 || nbuf < 0 || (nbuf && !counts) || !out_units)
            throw std::invalid_argument("rdc: bad argument");
        std::vector<uint64_t> cnt((size_t)nbuf);
        for (int b = 0; b < nbuf; ++b) cnt[(size_t)b] = counts[b];
        const CoalescedPlan P = PlanCoalesced(n, cnt.data(), nbuf, esz);
        if (chunk_out) {
            for (int c = 0; c < RDC_MAX_RANKS; ++c) {
                chunk_out[c] = P.off[c];
                chunk_out[RDC_MAX_RANKS + c] = P.len[c];
            }
            chunk_out[2 * RDC_MAX_RANKS] = P.total;
        }
        *out_units = (int)P.units.size();
        for (int i = 0; i < (int)P.units.size() && i < max_units && units_out; ++i) {
            units_out[4 * i + 0] = P.units[(size_t)i].buf;
            units_out[4 * i + 1] = P.units[(size_t)i].buf_off;
            units_out[4 * i + 2] = P.units[(size_t)i].packed;
            units_out[4 * i + 3] = P.units[(size_t)i].len;
        }
    });
}

int RdcPlanFuseGroups(const size_t* counts, int nbuf, int dtype, size_t fuse_bytes, int* bounds_out, int max_bounds,
                      int* out_n) {
    return guard([&] {
        const size_t esz = rdc_dtype_size(dtype);
        if (esz == 0 || nbuf < 0 || (nbuf && !counts) || !out_n) throw std::invalid_argument("rdc: bad argument");
        std::vector<uint64_t> cnt((size_t)nbuf);
        for (int b = 0; b < nbuf; ++b) cnt[(size_t)b] = counts[b];
        const std::vector<int> g = GroupCoalesced(cnt.data(), nbuf, esz, fuse_bytes ? fuse_bytes : CommConfig().fuse_bytes);
        *out_n = (int)g.size();
        for (int i = 0; i < (int)g.size() && i < max_bounds && bounds_out; ++i) bounds_out[i] = g[(size_t)i];
    });
}

// ------------------------------------------------------- point-to-point --
namespace {
struct BufferH {  // rdc::Buffer (include/transport/buffer.h:15-66): a view, not an owner
    void* addr = nullptr;
    size_t size = 0;
    bool registered = false;  // pinned: hipHostRegister'ed by RdcNewBuffer
};
BufferH* as_buffer(void* h) {
    if (!h) throw std::invalid_argument("rdc: null buffer handle");
    return static_cast<BufferH*>(h);
}
WorkComp* as_wc(void* h) {
    if (!h) throw std::invalid_argument("rdc: null work completion handle");
    return static_cast<WorkComp*>(h);
}
}  // namespace

int RdcNewBuffer(void** out, void* addr, size_t size, int pinned) {
    return guard([&] {
        if (!out) throw std::invalid_argument("rdc: null argument");
        if (size && !addr) throw std::invalid_argument("rdc: null buffer address");
        std::unique_ptr<BufferH> b(new BufferH());
        b->addr = addr;
        b->size = size;
        const uintptr_t page = (uintptr_t)sysconf(_SC_PAGESIZE);
        if (pinned && size && !is_device_pointer(addr) && (uintptr_t)addr % page == 0 && size % page == 0) {
            // a performance hint: an unregistrable range stays pageable.  Whole
            // pages only: a registration covers whole pages, and pages shared
            // with unrelated heap objects can be pinned and unpinned by the
            // runtime's own copies behind this registration's back
            b->registered = hipHostRegister(addr, size, hipHostRegisterDefault) == hipSuccess;
            (void)hipGetLastError();
            // host allreduces inside the range DMA straight from / into it
            // (HostPath::AllreduceRegistered)
            if (b->registered) {
                HostRegistryAdd(addr, size);
                // the copy path that will DMA this range comes up now, not
                // inside the first allreduce of it (HostPath::Warm)
                Manager& m = M();
                std::lock_guard<std::recursive_mutex> lk(m.mu);
                auto it = m.comms.find("main");
                if (m.inited && it != m.comms.end() && it->second->size() > 1) {
                    Communicator* c = it->second.get();
                    if (!m.host) m.host.reset(new HostPath(c->device(), m.host_zc_bytes));
                    // the path's own copy streams, not the manager stream
                    // (which may hold queued collectives: ADVICE r4)
                    if (size > HostPath::kSmall) m.host->Warm(nullptr);
                }
            }
        }
        *out = b.release();
    });
}

int RdcDelBuffer(void* buf) {
    return guard([&] {
        if (!buf) return;
        BufferH* b = static_cast<BufferH*>(buf);
        if (b->registered) {
            HostRegistryRemove(b->addr);
            (void)hipHostUnregister(b->addr);
        }
        delete b;
    });
}

int RdcCommISend(void** wc, void* comm, const void* buf, size_t bytes, int dest, void* stream) {
    return guard([&] {
        if (!wc) throw std::invalid_argument("rdc: null argument");
        *wc = as_comm(comm)->ISend(buf, bytes, dest, static_cast<hipStream_t>(stream));
    });
}

int RdcCommIRecv(void** wc, void* comm, void* buf, size_t bytes, int src, void* stream) {
    return guard([&] {
        if (!wc) throw std::invalid_argument("rdc: null argument");
        *wc = as_comm(comm)->IRecv(buf, bytes, src, static_cast<hipStream_t>(stream));
    });
}

int RdcISend(void** wc, void* comm, void* buf, int dest) {
    return guard([&] {
        if (!wc) throw std::invalid_argument("rdc: null argument");
        BufferH* b = as_buffer(buf);
        *wc = as_comm(comm)->ISend(b->addr, b->size, dest, nullptr);
    });
}

void* RdcIRecv(void* comm, void* buf, int src) {
    void* wc = nullptr;
    guard([&] {
        BufferH* b = as_buffer(buf);
        wc = as_comm(comm)->IRecv(b->addr, b->size, src, nullptr);
    });
    return wc;
}

int RdcWorkCompletionWait(void* wc) {
    int rc = 1;
    if (guard([&] { rc = as_wc(wc)->Wait(); }) != 0) return 1;
    if (rc != 0) g_last_error = static_cast<WorkComp*>(wc)->error();
    return rc;
}

int RdcWorkCompletionStatus(void* wc) { return wc ? static_cast<WorkComp*>(wc)->Status() : RDC_WS_ERROR; }

const char* RdcWorkCompletionError(void* wc) {
    thread_local std::string s;
    s = wc ? static_cast<WorkComp*>(wc)->error() : std::string("rdc: null work completion handle");
    return s.c_str();
}

int RdcDelWorkCompletion(void* wc) {
    return guard([&] {
        if (wc) static_cast<WorkComp*>(wc)->Release();
    });
}

namespace {
void p2p_sync(bool send, void* buf, size_t size, int peer) {
    Manager& m = M();
    Communicator* c;
    {
        std::lock_guard<std::recursive_mutex> lk(m.mu);
        require_init(m);
        c = get_comm(m, "main", true);
    }
    WorkComp* w = send ? c->ISend(buf, size, peer, nullptr) : c->IRecv(buf, size, peer, nullptr);
    const int rc = w->Wait();
    const std::string err = rc ? w->error() : std::string();
    w->Release();
    if (rc) throw std::runtime_error(err);
}
}  // namespace

int RdcSend(void* buf, size_t size, int dest) { return guard([&] { p2p_sync(true, buf, size, dest); }); }
int RdcRecv(void* buf, size_t size, int src) { return guard([&] { p2p_sync(false, buf, size, src); }); }

int RdcSetParam(const char* name, const char* value) {
    Manager& m = M();
    std::lock_guard<std::recursive_mutex> lk(m.mu);
    return guard([&] {
        if (!name || !value) throw std::invalid_argument("rdc: null argument");
        set_param(m, name, value);
    });
}

const char* RdcGetLastError(void) { return g_last_error.c_str(); }

const char* RdcVersion(void) { return "rdc_amd 0.1 (gfx950)"; }

}  // extern "C"
