// Device communicator (see rdc_comm.h).
#include "rdc_comm.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <errno.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <random>
#include <unordered_map>
#include <new>
#include <stdexcept>
#include <string>

#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include "rdc_kernels.h"
#include "rdc_p2p.h"
#include "rdc_plan.h"
#include "rdc_host.h"
#include "rdc_service.h"

namespace rdc_amd {

namespace {

void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string("rdc: ") + what + ": " + hipGetErrorString(e));
}

// Region kinds of a channel (Channel::region_kind): 0 hipExtMallocWithFlags(
// hipDeviceMallocUncached), 1 fine-grained, 2 coarse (hipMalloc), 3 the GPU's
// coarse HSA pool allocated with HSA_AMD_MEMORY_POOL_UNCACHED_FLAG and shared
// through HSA IPC (kKindHsaUC).
//
// What the L2s make of them (round 6, tools/ipc_mtype_probe.hip, per-request
// MTYPE counters TCP_TCC_{UC,NC,RW,CC}_READ_REQ, profiles/r06/mtype/): kind 0
// is NOT uncached on gfx950 — every request is MTYPE CC (cached in the
// reader XCD's L2, kept coherent by the hardware's invalidations), in the
// allocating process and in every hipIpcOpenMemHandle importer alike; kinds 1
// and 2 are RW; kind 3 is UC in both (every access goes to memory).  With CC,
// every device read kind — plain, sc1, nt, atomic, after a system acquire —
// of a line is served by that XCD's L2, so a line whose invalidation was lost
// stays stale for all of them while memory (and the host) hold the new value:
// the record of round 5's lost 5 x 3 hand-off.  The flag words
// of multi-process channels are therefore kind 3 (RDC_FLAGS_MEM=cc: kind 0).
constexpr int kKindHsaUC = 3;

// RDC_ALLOC: the data regions' kind ("fine", "coarse", "uc"; default 0)
int env_alloc_kind() {
    const char* v = getenv("RDC_ALLOC");
    if (!v) return 0;
    if (!strcmp(v, "fine")) return 1;
    if (!strcmp(v, "coarse")) return 2;
    if (!strcmp(v, "uc")) return kKindHsaUC;
    return 0;
}

// RDC_FLAGS_MEM: the flag words' kind on multi-process channels ("uc", the
// default, or "cc" = kind 0 as in rounds 1-5)
int env_flags_kind() {
    const char* v = getenv("RDC_FLAGS_MEM");
    return v && !strcmp(v, "cc") ? 0 : kKindHsaUC;
}

// the HSA agent of HIP device `device` (matched by PCI location) and its
// coarse-grained global pool; cached per device
struct HsaDev {
    bool ok = false;
    hsa_agent_t agent{};
    hsa_amd_memory_pool_t pool{};
    uint32_t want_bdf = 0, want_domain = 0;
    bool have_agent = false;
};
hsa_status_t hsa_pick_agent(hsa_agent_t a, void* d) {
    HsaDev* h = static_cast<HsaDev*>(d);
    hsa_device_type_t t;
    if (h->have_agent || hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS ||
        t != HSA_DEVICE_TYPE_GPU)
        return HSA_STATUS_SUCCESS;
    uint32_t bdf = 0, dom = 0;
    hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf);
    hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom);
    if ((bdf >> 3) == (h->want_bdf >> 3) && dom == h->want_domain) {
        h->agent = a;
        h->have_agent = true;
    }
    return HSA_STATUS_SUCCESS;
}
hsa_status_t hsa_pick_coarse(hsa_amd_memory_pool_t pool, void* d) {
    HsaDev* h = static_cast<HsaDev*>(d);
    hsa_amd_segment_t seg;
    uint32_t flags = 0;
    if (h->ok || hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg) != HSA_STATUS_SUCCESS)
        return HSA_STATUS_SUCCESS;
    hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
    if (seg == HSA_AMD_SEGMENT_GLOBAL && (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED)) {
        h->pool = pool;
        h->ok = true;
    }
    return HSA_STATUS_SUCCESS;
}
const HsaDev& hsa_dev(int device) {
    static std::mutex mu;
    static std::map<int, HsaDev> cache;
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(device);
    if (it != cache.end()) return it->second;
    HsaDev h;
    int bus = 0, dev = 0, dom = 0;
    if (hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, device) == hipSuccess &&
        hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, device) == hipSuccess &&
        hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, device) == hipSuccess &&
        hsa_init() == HSA_STATUS_SUCCESS) {  // reference-counted; HIP holds it already (never shut down here)
        h.want_bdf = ((uint32_t)bus << 8) | ((uint32_t)dev << 3);
        h.want_domain = (uint32_t)dom;
        if (hsa_iterate_agents(hsa_pick_agent, &h) == HSA_STATUS_SUCCESS && h.have_agent)
            hsa_amd_agent_iterate_memory_pools(h.agent, hsa_pick_coarse, &h);
    }
    (void)hipGetLastError();
    return cache.emplace(device, h).first->second;
}

// One region of a channel: `want` = a kind from the list above; kind 3 falls
// back to 0 where the HSA pool refuses (and kinds 0 / 1 fall back as before:
// fine-grained, then coarse).  Kind 3 memory is zeroed here.
void* alloc_shared(size_t bytes, int* kind, int device, int want) {
    void* p = nullptr;
    if (want == kKindHsaUC) {
        const HsaDev& h = hsa_dev(device);
        if (h.ok && hsa_amd_memory_pool_allocate(h.pool, bytes, HSA_AMD_MEMORY_POOL_UNCACHED_FLAG, &p) ==
                        HSA_STATUS_SUCCESS) {
            if (hsa_amd_memory_fill(p, 0, bytes / 4) == HSA_STATUS_SUCCESS) {
                *kind = kKindHsaUC;
                return p;
            }
            hsa_amd_memory_pool_free(p);
            p = nullptr;
        }
        want = 0;
    }
    if (want <= 0 && hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached) == hipSuccess) {
        *kind = 0;
        return p;
    }
    (void)hipGetLastError();
    if (want <= 1 && hipExtMallocWithFlags(&p, bytes, hipDeviceMallocFinegrained) == hipSuccess) {
        *kind = 1;
        return p;
    }
    (void)hipGetLastError();
    hip_check(hipMalloc(&p, bytes), "hipMalloc scratch");
    *kind = 2;
    return p;
}
void free_shared(void* p, int kind) {
    if (!p) return;
    if (kind == kKindHsaUC) hsa_amd_memory_pool_free(p);
    else (void)hipFree(p);
}

// one region's IPC handle (HIP's for kinds 0-2, HSA's for kind 3)
struct RegionHandle {
    int32_t kind;
    int32_t pad_;
    uint64_t bytes;
    hipIpcMemHandle_t hip;
    hsa_amd_ipc_memory_t hsa;
};
void export_region(void* p, size_t bytes, int kind, RegionHandle* h, const char* what) {
    memset(h, 0, sizeof(*h));
    h->kind = kind;
    h->bytes = bytes;
    if (kind == kKindHsaUC) {
        if (hsa_amd_ipc_memory_create(p, bytes, &h->hsa) != HSA_STATUS_SUCCESS)
            throw std::runtime_error(std::string("rdc: hsa_amd_ipc_memory_create(") + what + ") failed");
    } else {
        hip_check(hipIpcGetMemHandle(&h->hip, p), what);
    }
}
void* import_region(const RegionHandle& h, int device, const char* what) {
    void* p = nullptr;
    if (h.kind == kKindHsaUC) {
        const HsaDev& d = hsa_dev(device);
        if (!d.have_agent || hsa_amd_ipc_memory_attach(&h.hsa, h.bytes, 1, &d.agent, &p) != HSA_STATUS_SUCCESS || !p)
            throw std::runtime_error(std::string("rdc: hsa_amd_ipc_memory_attach(") + what + ") failed");
        return p;
    }
    hip_check(hipIpcOpenMemHandle(&p, h.hip, hipIpcMemLazyEnablePeerAccess), what);
    return p;
}
void close_region(void* p, int kind) {
    if (!p) return;
    if (kind == kKindHsaUC) hsa_amd_ipc_memory_detach(p);
    else (void)hipIpcCloseMemHandle(p);
}

void dbg(const char* fmt, int rank, const char* what) {
    static const bool on = getenv("RDC_DEBUG") != nullptr;
    if (on) {
        fprintf(stderr, fmt, rank, what);
        fflush(stderr);
    }
}

constexpr int kPlanKeys = 20;  // PlanKey below; sizes PeerInfo::plan

struct PeerInfo {
    uint64_t channel;   // id of the live channel this rank would share (0 = none)
    int32_t device;
    int32_t pid;
    int32_t alloc_kind;
    int32_t svc_ok;  // a new channel may run the small-allreduce service here
    uint64_t slot_bytes;
    uint64_t max_tiles;
    uint64_t p2p_slot_bytes;
    int32_t num_cus;
    int32_t num_xcds;  // hipDeviceAttributeNumberOfXccs (dispatch round-robins workgroups over them)
    uint64_t plan[kPlanKeys];  // PlanKey: the parameters that shape a launch plan (must agree)
    char host[64];
    char pci[32];  // physical GPU (ranks may share one: tests, emulation)
};

struct Handles {  // round 2 of Create: IPC handles (the channel's regions only for a new channel)
    RegionHandle region[4];  // scratch, ag, flags, service slots
    hipIpcMemHandle_t p2p;
};

// Launch plans are made on each host; flags are matched by tile index while
// data lands by byte offset, so ranks that planned differently would read
// contributions that have not landed (silent wrong bits, not a timeout).
// Every parameter a plan depends on is exchanged at creation and compared.
// The small-allreduce service's switches too: a rank that serves a small host
// buffer through it while a peer launches a kernel would wait out RDC_TIMEOUT.
void PlanKey(const CommConfig& c, uint64_t tune_hash, uint64_t (&k)[kPlanKeys]) {
    const uint64_t v[kPlanKeys] = {(uint64_t)c.algo, (uint64_t)c.max_blocks, (uint64_t)c.tile_bytes,
                                   (uint64_t)c.oneshot_push_max, (uint64_t)c.fuse_bytes, (uint64_t)c.coalesce_fused,
                                   (uint64_t)c.fuse_bytes_direct, (uint64_t)c.bcast_split_bytes,
                                   (uint64_t)c.mesh_split.s16, (uint64_t)c.mesh_split.r16, (uint64_t)c.ring_mincount,
                                   (uint64_t)c.scratch_bytes, (uint64_t)SmallService::Enabled(),
                                   (uint64_t)SmallService::ShareMax(),
                                   (uint64_t)HostPieceBytes() | ((uint64_t)HostPieceRamp() << 63), tune_hash,
                                   (uint64_t)HostInlineBytes(), (uint64_t)(HostBalanceSetting() + 1),
                                   SmallService::HxBytes(), (uint64_t)c.direct_min};
    memcpy(k, v, sizeof(v));
}
const char* kPlanKeyNames[kPlanKeys] = {"RDC_ALGO", "RDC_NBLOCKS", "RDC_TILE_BYTES", "RDC_ONESHOT_BYTES",
                                        "RDC_FUSE_BYTES", "RDC_COALESCE_FUSED", "RDC_FUSE_BYTES_DIRECT",
                                        "RDC_BCAST_SPLIT_BYTES", "RDC_MESH_SPLIT", "RDC_MESH_SPLIT",
                                        "rdc_reduce_ring_mincount", "RDC_SCRATCH_BYTES", "RDC_HOST_SERVICE",
                                        "RDC_HOST_SERVICE_SHARE_MAX", "RDC_HOST_PIECE_BYTES / RDC_HOST_PIECE_RAMP",
                                        "RDC_TUNE_FILE (set or not)", "RDC_HOST_INLINE_BYTES", "RDC_HOST_BALANCE",
                                        "RDC_HOST_SERVICE_HX_BYTES", "RDC_DIRECT_BYTES"};

// Autotune results kept across runs (RDC_TUNE_FILE): one line per winner,
// "rdc-tune 2 <ranks> <cus> <ranks per gpu> <size class> <algo> <s16> <r16>
// <grid> <tpb> <ms>", later lines overriding earlier ones.  Rank 0 alone
// reads the file at communicator creation and broadcasts the parsed entries,
// so every rank plans from the same table even while another job appends to
// the file; only rank 0 appends (Communicator::Autotune).  Entries apply to
// communicators of the same rank count, fewest CUs and ranks per GPU (a shape
// tuned with ranks sharing a GPU says nothing about one rank per GPU).
struct TuneEntry {
    int32_t n, cus, rpg, cls, algo, s16, r16, grid, tpb;
};
constexpr int kTuneEntriesMax = 256;  // the latest ones are kept
std::string tune_file() {
    const char* e = getenv("RDC_TUNE_FILE");
    return e && *e ? std::string(e) : std::string();
}
std::vector<TuneEntry> read_tune_file(const std::string& path) {
    std::vector<TuneEntry> out;
    if (path.empty()) return out;
    FILE* f = fopen(path.c_str(), "r");
    if (!f) return out;  // no table yet: nothing tuned
    char line[256];
    while (fgets(line, sizeof(line), f)) {
        TuneEntry e;
        int ver = 0;
        double ms = 0;
        if (sscanf(line, "rdc-tune %d %d %d %d %d %d %d %d %d %d %lf", &ver, &e.n, &e.cus, &e.rpg, &e.cls, &e.algo,
                   &e.s16, &e.r16, &e.grid, &e.tpb, &ms) == 11 &&
            ver == 2 && e.rpg >= 1 && e.cls >= 0 && e.cls < 64 &&
            (e.algo == RDC_ALGO_RING || e.algo == RDC_ALGO_MESH || e.algo == RDC_ALGO_MESH_PULL ||
             e.algo == RDC_ALGO_ONESHOT || e.algo == RDC_ALGO_DIRECT) && e.s16 >= 1 &&
            e.r16 >= 1 && e.s16 + e.r16 <= 15 && e.grid >= 0 && e.tpb >= 0)
            out.push_back(e);
    }
    fclose(f);
    if (out.size() > (size_t)kTuneEntriesMax) out.erase(out.begin(), out.end() - kTuneEntriesMax);
    return out;
}
// rank 0's table on every rank (collective over bs)
std::vector<TuneEntry> shared_tune_table(Bootstrap* bs) {
    struct {
        int32_t count;
        TuneEntry e[kTuneEntriesMax];
    } msg;
    memset(&msg, 0, sizeof(msg));
    if (bs->rank() == 0) {
        const std::vector<TuneEntry> t = read_tune_file(tune_file());
        msg.count = (int32_t)t.size();
        if (!t.empty()) memcpy(msg.e, t.data(), t.size() * sizeof(TuneEntry));
    }
    bs->broadcast(&msg, sizeof(msg), 0);
    return std::vector<TuneEntry>(msg.e, msg.e + std::max(0, std::min(msg.count, kTuneEntriesMax)));
}

size_t round_up_bytes(size_t v, size_t a) { return (v + a - 1) / a * a; }

// `bytes` of POSIX shared memory every rank of bs maps and registers for its
// device (hipHostRegister `flags`): rank 0 creates it, every rank maps it,
// rank 0 unlinks the name once all mapped (nothing is left in /dev/shm).
// Collective over bs.  Zero-filled.
std::shared_ptr<char> map_shared_host(Bootstrap* bs, size_t bytes, const char* what, unsigned flags) {
    char name[64];
    memset(name, 0, sizeof(name));
    int fd = -1;
    std::string err;
    if (bs->rank() == 0) {
        static std::atomic<int> counter{0};
        snprintf(name, sizeof(name), "/rdc_%s_%d_%d", what, (int)getpid(), counter++);
        fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
        if (fd < 0 || ftruncate(fd, (off_t)bytes) != 0) {
            err = std::string("rdc: cannot create shared memory ") + name + ": " + strerror(errno);
            if (fd >= 0) {
                close(fd);
                shm_unlink(name);
            }
            fd = -1;
            memset(name, 0, sizeof(name));  // tells the others
        }
    }
    bs->broadcast(name, sizeof(name), 0);
    if (!name[0])
        throw std::runtime_error(err.empty() ? std::string("rdc: rank 0 could not create shared memory for ") + what
                                             : err);
    if (bs->rank() != 0) {
        fd = shm_open(name, O_RDWR, 0600);
        if (fd < 0) throw std::runtime_error(std::string("rdc: cannot open shared memory ") + name + ": " + strerror(errno));
    }
    void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) throw std::runtime_error(std::string("rdc: cannot map shared memory: ") + strerror(errno));
    if (hipHostRegister(p, bytes, flags) != hipSuccess) {
        (void)hipGetLastError();
        munmap(p, bytes);
        throw std::runtime_error(std::string("rdc: cannot register shared memory for ") + what + " for device access");
    }
    std::shared_ptr<char> mem(static_cast<char*>(p), [bytes](char* q) {
        (void)hipHostUnregister(q);
        munmap(q, bytes);
    });
    bs->barrier();
    if (bs->rank() == 0) shm_unlink(name);
    return mem;
}

// The point-to-point control block (rdc_p2p.h), registered for device access:
// the p2p copy kernels publish posted / consumed themselves
std::shared_ptr<P2PCtl> map_p2p_ctl(Bootstrap* bs) {
    std::shared_ptr<char> mem =
        map_shared_host(bs, sizeof(P2PCtl), "p2p", hipHostRegisterMapped | hipHostRegisterPortable);
    return std::shared_ptr<P2PCtl>(mem, reinterpret_cast<P2PCtl*>(mem.get()));
}

// the small-allreduce service's host exchange region (rdc_service.h); MTYPE
// UC on the GPU side like the mailbox, so the block's loads see the hosts' stores
size_t svc_hx_bytes(int n) { return (size_t)2 * (size_t)n * RDC_SVC_HX_RANK_BYTES; }

}  // namespace

Communicator::Communicator() {}

// ------------------------------------------------------------------ Channel --
namespace {
// live channels per bootstrap, and how many each bootstrap has created (the
// id every rank gives its k-th channel on that bootstrap)
std::mutex g_reg_mu;
std::map<Bootstrap*, std::vector<std::weak_ptr<Channel>>> g_channels;
std::map<Bootstrap*, uint64_t> g_channel_count;
// channels of this process whose small-allreduce service may run, per device:
// at most one (Communicator::Create), so at most one persistent service block
// per process and GPU is resident — what LaunchGrid's one-CU-per-rank
// reservation assumes
// (leaked: channels may be destroyed from other translation units' static
// destructors at exit)
struct SvcRegistry {
    std::mutex mu;
    std::map<int, int> channels;
};
SvcRegistry& svc_registry() {
    static SvcRegistry* r = new SvcRegistry();
    return *r;
}

// RDC_STRICT_FENCES=1: keep the system-scope release fences on every hand-off
// even with uncached scratch (diagnostics; rdc_device.h block_publish)
bool strict_fences() {
    static const bool on = [] {
        const char* v = getenv("RDC_STRICT_FENCES");
        return v && *v && atoi(v) != 0;
    }();
    return on;
}

// RDC_LAUNCH_LOG=<prefix>: every collective launch appended to <prefix>.<pid>
// (communicator, launch number, kind, bytes, grid, tile) — diagnostics for
// ranks whose launch sequences diverge
void log_launch(const Communicator* c, uint32_t seq, int kind, uint64_t bytes, int grid, uint64_t tile) {
    static const char* prefix = getenv("RDC_LAUNCH_LOG");
    if (!prefix || !*prefix) return;
    static std::mutex mu;
    std::lock_guard<std::mutex> lk(mu);
    static FILE* f = [] {
        char path[512];
        snprintf(path, sizeof(path), "%s.%d", getenv("RDC_LAUNCH_LOG"), (int)getpid());
        return fopen(path, "a");
    }();
    if (!f) return;
    // the device's block-arrival and completed-launch counters before this
    // launch (a synchronous read: waits for this rank's earlier launches)
    uint32_t w[16] = {0};
    uint64_t ctr = 0;
    if (c->err_words()) {
        (void)hipMemcpy(w, c->err_words() + 16, sizeof(uint32_t), hipMemcpyDeviceToHost);
        (void)hipMemcpy(&ctr, c->err_words() + 32, sizeof(ctr), hipMemcpyDeviceToHost);
    }
    fprintf(f, "%s rank %d launch %u kind %d bytes %llu grid %d tile %llu | arrivals %u completed %llu\n",
            c->name().c_str(), c->rank(), seq, kind, (unsigned long long)bytes, grid, (unsigned long long)tile, w[0],
            (unsigned long long)ctr);
    fflush(f);
}

bool share_enabled() {
    const char* v = getenv("RDC_SHARE_SCRATCH");
    return !(v && *v && atoi(v) == 0);
}
}  // namespace

Channel::~Channel() {
    svc.reset();  // the resident service block leaves first
    if (svc_counted) {
        std::lock_guard<std::mutex> lk(svc_registry().mu);
        --svc_registry().channels[device];
    }
    (void)hipSetDevice(device);
    (void)hipDeviceSynchronize();
    if (ipc && bs) {
        try {
            bs->barrier();  // nobody still pushes into my scratch
        } catch (...) {
        }
        for (int p = 0; p < n; ++p)
            if (p != rank) {
                close_region(peer_scratch[p], peer_kind[0][p]);
                close_region(peer_ag[p], peer_kind[1][p]);
                close_region(peer_flags[p], peer_kind[2][p]);
                close_region(peer_svc_region[p], peer_kind[3][p]);
            }
        for (auto& m : dmaps) {  // registered peers' buffers
            if (vmem) vmem->Unmap(m.second.ptr);
            else (void)hipIpcCloseMemHandle(m.second.ptr);
        }
        dmaps.clear();
        try {
            bs->barrier();  // every importer closed its mapping
        } catch (...) {
        }
        vmem.reset();
    }
    if (dlast) (void)hipEventDestroy(dlast);
    if (last_ev) (void)hipEventDestroy(last_ev);
    if (tune_buf) (void)hipFree(tune_buf);
    for (void* p : tune_old) (void)hipFree(p);
    free_shared(scratch, region_kind[0]);
    free_shared(scratch_ag, region_kind[1]);
    free_shared(flags, region_kind[2]);
    free_shared(svc_region, region_kind[3]);
    if (err) (void)hipFree(err);
    if (tlog) (void)hipFree(tlog);
    if (err_host) (void)hipHostFree(err_host);
    if (dpeek_stream) (void)hipStreamDestroy(dpeek_stream);
    if (dpeek_host) (void)hipHostFree(dpeek_host);
}

void Channel::Order(hipStream_t s) {
    std::lock_guard<std::mutex> lk(mu);
    if (users > 1 && have_last && last_stream != s) hip_check(hipStreamWaitEvent(s, last_ev, 0), "order channel");
}

void Channel::Mark(hipStream_t s) {
    std::lock_guard<std::mutex> lk(mu);
    if (users <= 1) return;
    if (!last_ev) hip_check(hipEventCreateWithFlags(&last_ev, hipEventDisableTiming), "channel event");
    hip_check(hipEventRecord(last_ev, s), "record channel event");
    last_stream = s;
    have_last = true;
}

namespace {
// a collective call on a channel: ordered behind the channel's previous call
// (when another communicator may have issued it on another stream), and
// recorded as the latest one when it returns
struct ChannelCall {
    Channel* ch;
    hipStream_t s;
    ChannelCall(Channel* c, hipStream_t st) : ch(c), s(st) {
        if (ch) ch->Order(s);
    }
    ~ChannelCall() {
        try {
            if (ch) ch->Mark(s);
        } catch (...) {
        }
    }
};
}  // namespace

bool Communicator::shares_channel() const {
    if (!ch_) return false;
    std::lock_guard<std::mutex> lk(ch_->mu);
    return ch_->users > 1;
}

// this rank's scratch regions, flags and error words (uncached, IPC-exportable)
void Communicator::AllocChannel() {
    hip_check(hipSetDevice(device_), "hipSetDevice");
    std::shared_ptr<Channel> ch = std::make_shared<Channel>();
    ch->rank = rank_;
    ch->n = n_;
    ch->device = device_;
    ch->bs = bs_;
    ch->L = MakeLayout(n_, cfg_.scratch_bytes);
    int k1 = 0, k2 = 0, k3 = 0;
    // HSA-uncached regions (kind 3) only where peers import them through HSA
    // IPC: multi-process channels.  Single-process groups keep HIP memory.
    const int data_want = bs_ ? env_alloc_kind() : std::min(env_alloc_kind(), 2);
    const int flags_want = bs_ ? std::max(env_flags_kind(), data_want) : data_want;
    ch->scratch = static_cast<char*>(alloc_shared(ch->L.region_bytes, &k1, device_, data_want));
    ch->scratch_ag = static_cast<char*>(alloc_shared(ch->L.region_bytes, &k3, device_, data_want));
    ch->flags = static_cast<uint64_t*>(alloc_shared(ch->L.flag_bytes, &k2, device_, flags_want));
    int k5 = 0;  // service LL slots [2][n] x RDC_SVC_SLOT_BYTES; zero: no sequence number matches
    const size_t svc_bytes = (size_t)2 * n_ * RDC_SVC_SLOT_BYTES;
    ch->svc_region = static_cast<char*>(alloc_shared(svc_bytes, &k5, device_, flags_want));
    if (k5 != kKindHsaUC) hip_check(hipMemset(ch->svc_region, 0, svc_bytes), "memset service slots");
    ch->region_kind[0] = k1;
    ch->region_kind[1] = k3;
    ch->region_kind[2] = k2;
    ch->region_kind[3] = k5;
    ch->region_bytes[0] = ch->region_bytes[1] = ch->L.region_bytes;
    ch->region_bytes[2] = ch->L.flag_bytes;
    ch->region_bytes[3] = svc_bytes;
    // 0 = the uncached class for the fences' choice (rdc_device.h): CC and UC alike
    auto cls = [](int k) { return k == kKindHsaUC ? 0 : k; };
    ch->alloc_kind = std::max(std::max(std::max(cls(k1), cls(k2)), cls(k3)), cls(k5));
    // [0] error word, [16] block arrival counter, [32] completed-launch counter, [48] last kind.
    // [64..] the first timed-out wait (rdc_device.h block_wait: seq, flag value,
    // flag address).  Plain device memory, read and written with agent-scope
    // atomics (sc1) only.  RDC_COUNTERS_UNCACHED=1 allocates it uncached like
    // the flags; tried in round 4 while chasing the 5 x 3-queue hand-off loss,
    // it did not change that, and small launches measured the same or a
    // little slower (one-shot 4 B at n = 2 back to back: 7.54 vs 6.99-7.35 us
    // per launch, profiles/r04/counters_ab/).
    static const bool uc_counters = getenv("RDC_COUNTERS_UNCACHED") && atoi(getenv("RDC_COUNTERS_UNCACHED")) != 0;
    if (!uc_counters ||
        hipExtMallocWithFlags(reinterpret_cast<void**>(&ch->err), 512, hipDeviceMallocUncached) != hipSuccess) {
        (void)hipGetLastError();
        hip_check(hipMalloc(&ch->err, 512), "hipMalloc err");
    }
    if (k2 != kKindHsaUC) hip_check(hipMemset(ch->flags, 0, ch->L.flag_bytes), "memset flags");
    hip_check(hipMemset(ch->err, 0, 512), "memset err");
    if (getenv("RDC_LAUNCH_TIMES") && atoi(getenv("RDC_LAUNCH_TIMES")) != 0) {
        hip_check(hipMalloc(reinterpret_cast<void**>(&ch->tlog), 64 * 4 * sizeof(uint64_t)), "launch log");
        hip_check(hipMemset(ch->tlog, 0, 64 * 4 * sizeof(uint64_t)), "launch log");
    }
    hip_check(hipHostMalloc(reinterpret_cast<void**>(&ch->err_host), 64, hipHostMallocCoherent), "hipHostMalloc err");
    memset(ch->err_host, 0, 64);
    hip_check(hipHostGetDevicePointer(reinterpret_cast<void**>(&ch->err_host_dev), ch->err_host, 0),
              "err device pointer");
    hip_check(hipDeviceSynchronize(), "sync after alloc");
    ch->peer_scratch[rank_] = ch->scratch;
    ch->peer_ag[rank_] = ch->scratch_ag;
    ch->peer_flags[rank_] = ch->flags;
    ch->peer_svc_region[rank_] = ch->svc_region;
    if (bs_) {
        std::lock_guard<std::mutex> lk(g_reg_mu);
        ch->id = ++g_channel_count[bs_];
        g_channels[bs_].push_back(ch);
    }
    Attach(ch);
}

void Communicator::AllocP2P() {
    int k4 = 0;
    p2p_ = static_cast<char*>(alloc_shared((size_t)n_ * kP2PSlots * cfg_.p2p_slot_bytes, &k4, device_,
                                           std::min(env_alloc_kind(), 2)));  // HIP IPC
    alloc_kind_ = std::max(alloc_kind_, k4);
    peer_p2p_[rank_] = p2p_;
}

// join a channel as one more user
void Communicator::Attach(const std::shared_ptr<Channel>& ch) {
    ch_ = ch;
    {
        std::lock_guard<std::mutex> lk(ch->mu);
        ++ch->users;
        // communicators attach to a channel in creation order, which is
        // collective: the k-th user's tag is k on every rank (rdc_device.h kTagBits)
        tag_ = ch->attached++ & 0xFFu;
    }
    Alias();
}

// the channel's resources under this communicator's (non-owning) names
void Communicator::Alias() {
    Channel* ch = ch_.get();
    const Layout& L = ch->L;
    slot_bytes_ = L.slot_bytes;
    region_bytes_ = L.region_bytes;
    max_tiles_ = L.max_tiles;
    flag_bytes_ = L.flag_bytes;
    alloc_kind_ = ch->alloc_kind;
    scratch_ = ch->scratch;
    scratch_ag_ = ch->scratch_ag;
    flags_ = ch->flags;
    err_ = ch->err;
    err_host_ = ch->err_host;
    err_host_dev_ = ch->err_host_dev;
    for (int p = 0; p < n_; ++p) {
        peer_scratch_[p] = ch->peer_scratch[p];
        peer_ag_[p] = ch->peer_ag[p];
        peer_flags_[p] = ch->peer_flags[p];
    }
}

namespace {
int device_xcds(int device) {
    int x = 0;
    if (hipDeviceGetAttribute(&x, hipDeviceAttributeNumberOfXccs, device) != hipSuccess || x < 1) {
        (void)hipGetLastError();
        x = 1;
    }
    return x;
}
}  // namespace

void Communicator::AllocLocal() {
    hip_check(hipSetDevice(device_), "hipSetDevice");
    AllocChannel();
    AllocP2P();
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device_) == hipSuccess && cus > 0)
        num_cus_ = cus;
    num_xcds_ = device_xcds(device_);
    int wclk = 0;  // kHz
    if (hipDeviceGetAttribute(&wclk, hipDeviceAttributeWallClockRate, device_) != hipSuccess || wclk <= 0)
        wclk = 100000;
    wall_khz_ = wclk;
    tree_len_ = PlanTreeProgram(n_, tree_dst_, tree_src_);
}

Communicator* Communicator::Create(const std::string& name, Bootstrap* bs, int device, const CommConfig& cfg) {
    std::unique_ptr<Communicator> c(new Communicator());
    c->name_ = name;
    c->rank_ = bs->rank();
    c->n_ = bs->size();
    c->device_ = device;
    c->cfg_ = cfg;
    c->bs_ = bs;
    if (c->n_ > RDC_MAX_RANKS) throw std::runtime_error("rdc: world size exceeds RDC_MAX_RANKS");
    // world size 1 moves no data (Communicator::Allreduce returns at once,
    // communicator_base.h:133-138): no device resources, no GPU needed
    if (c->n_ == 1) return c.release();
    hip_check(hipSetDevice(device), "hipSetDevice");
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
        c->num_cus_ = cus;
    c->num_xcds_ = device_xcds(device);
    c->xcds_max_ = c->num_xcds_;
    int wclk = 0;  // kHz
    if (hipDeviceGetAttribute(&wclk, hipDeviceAttributeWallClockRate, device) != hipSuccess || wclk <= 0) wclk = 100000;
    c->wall_khz_ = wclk;
    c->tree_len_ = PlanTreeProgram(c->n_, c->tree_dst_, c->tree_src_);
    const Layout L = MakeLayout(c->n_, cfg.scratch_bytes);

    // round 1: the facts every rank must agree on, and the channel this rank
    // could share (a live channel of this bootstrap with the same geometry)
    PeerInfo mine;
    memset(&mine, 0, sizeof(mine));
    mine.p2p_slot_bytes = cfg.p2p_slot_bytes;
    mine.device = device;
    mine.pid = (int32_t)getpid();
    mine.slot_bytes = L.slot_bytes;
    mine.max_tiles = L.max_tiles;
    mine.num_cus = c->num_cus_;
    mine.num_xcds = c->num_xcds_;
    PlanKey(cfg, tune_file().empty() ? 0 : 1, mine.plan);
    std::shared_ptr<Channel> cand;
    if (share_enabled()) {
        std::lock_guard<std::mutex> lk(g_reg_mu);
        std::vector<std::weak_ptr<Channel>>& live = g_channels[bs];
        live.erase(std::remove_if(live.begin(), live.end(),
                                  [](const std::weak_ptr<Channel>& w) { return w.expired(); }),
                   live.end());
        for (auto& w : live) {
            std::shared_ptr<Channel> ch = w.lock();
            if (ch && ch->device == device && ch->n == c->n_ && ch->L.slot_bytes == L.slot_bytes &&
                ch->L.max_tiles == L.max_tiles && ch->ipc)
                cand = ch;
        }
    }
    mine.channel = cand ? cand->id : 0;
    // a NEW channel may run the small-allreduce service only if no other
    // channel of this process on this device may (one resident service block
    // per process and GPU, LaunchGrid); agreed below (AND over ranks).  The
    // slot is reserved under the lock when it is offered, so two threads
    // creating communicators on one device at once cannot both take it; the
    // reservation passes to the new channel, or is released (shared channel,
    // a rank without the slot, an error on the way).
    struct SvcSlot {
        int device;
        bool held = false;
        explicit SvcSlot(int d) : device(d) {}
        void release() {
            if (!held) return;
            std::lock_guard<std::mutex> lk(svc_registry().mu);
            --svc_registry().channels[device];
            held = false;
        }
        ~SvcSlot() { release(); }
    } svc_slot(device);
    {
        std::lock_guard<std::mutex> lk(svc_registry().mu);
        int& used = svc_registry().channels[device];
        if (SmallService::Enabled() && used == 0) {
            ++used;
            svc_slot.held = true;
        }
        mine.svc_ok = svc_slot.held ? 1 : 0;
    }
    gethostname(mine.host, sizeof(mine.host) - 1);
    if (hipDeviceGetPCIBusId(mine.pci, sizeof(mine.pci) - 1, device) != hipSuccess) {
        (void)hipGetLastError();
        snprintf(mine.pci, sizeof(mine.pci), "device-%d", device);
    }
    std::vector<PeerInfo> all((size_t)c->n_);
    bs->allgather(&mine, sizeof(mine), all.data());
    bool share = mine.channel != 0;
    bool svc_all = true;
    for (int p = 0; p < c->n_; ++p) {
        const PeerInfo& q = all[(size_t)p];
        svc_all = svc_all && q.svc_ok != 0;
        if (q.slot_bytes != mine.slot_bytes || q.max_tiles != mine.max_tiles ||
            q.p2p_slot_bytes != mine.p2p_slot_bytes)
            throw std::runtime_error("rdc: ranks disagree on scratch size (set RDC_SCRATCH_BYTES identically)");
        for (int k = 0; k < kPlanKeys; ++k)
            if (q.plan[k] != mine.plan[k])
                throw std::runtime_error(std::string("rdc: rank ") + std::to_string(p) + " and rank " +
                                         std::to_string(c->rank_) + " disagree on " + kPlanKeyNames[k] + " (" +
                                         std::to_string(q.plan[k]) + " vs " + std::to_string(mine.plan[k]) +
                                         "): every rank must plan launches identically");
        if (strncmp(q.host, mine.host, sizeof(mine.host)) != 0)
            throw std::runtime_error("rdc: xGMI path needs every rank on one node (rank " + std::to_string(p) +
                                     " is on " + q.host + ")");
        share = share && q.channel == mine.channel;  // every rank holds the same channel
    }
    // grids are planned from values every rank sees: the fewest CUs of any
    // rank's GPU and the most ranks sharing one physical GPU (ResidentGrid)
    c->cus_min_ = c->num_cus_;
    c->share_max_ = 1;
    for (int p = 0; p < c->n_; ++p) {
        c->cus_min_ = std::min(c->cus_min_, std::max(1, (int)all[(size_t)p].num_cus));
        c->xcds_max_ = std::max(c->xcds_max_, std::max(1, (int)all[(size_t)p].num_xcds));
        int same = 0;
        for (int q = 0; q < c->n_; ++q) same += strncmp(all[(size_t)p].pci, all[(size_t)q].pci, sizeof(mine.pci)) == 0;
        c->share_max_ = std::max(c->share_max_, same);
    }
    {   // more than 16 hardware queues on one GPU are time-sliced by its
        // scheduler (~10 ms slices): a collective spinning on a peer whose
        // queue is not mapped waits a slice (DESIGN.md §4, round 3 session 3)
        // The advice is rdc_amd.launcher's budget (hw_queues_per_process): the
        // share of 16 rounded down to a power of two — with 3 queues per
        // process at 5-6 ranks per GPU the GPU left one rank's kernel
        // undispatched behind its peers' spinning kernels
        const char* q = getenv("GPU_MAX_HW_QUEUES");
        const int per = q && *q ? atoi(q) : 4;
        static bool warned = false;
        int want = 1;
        while (want * 2 <= std::max(1, 16 / c->share_max_)) want *= 2;
        const bool pow2 = per > 0 && (per & (per - 1)) == 0;
        if (c->rank_ == 0 && !warned && c->share_max_ > 1 && (c->share_max_ * per > 16 || !pow2)) {
            warned = true;
            fprintf(stderr,
                    "rdc: %d ranks share one GPU with GPU_MAX_HW_QUEUES=%d each; set GPU_MAX_HW_QUEUES=%d "
                    "(rdc_amd.launcher does): more than 16 queues are time-sliced (~10 ms per slice) and with "
                    "3 per process at 5-6 ranks per GPU one rank's kernel went undispatched while its peers "
                    "waited\n",
                    c->share_max_, per, want);
        }
    }
    // schedules and shapes an earlier Autotune of this node measured for this
    // rank count, CU count and ranks per GPU (RDC_TUNE_FILE, rank 0's table)
    const std::vector<TuneEntry> tuned = tune_file().empty() ? std::vector<TuneEntry>() : shared_tune_table(bs);
    if (cfg.algo == RDC_ALGO_AUTO)
        for (const TuneEntry& e : tuned) {
            if (e.n != c->n_ || e.cus != c->cus_min_ || e.rpg != c->share_max_) continue;
            Shape s;
            s.split.s16 = e.s16;
            s.split.r16 = e.r16;
            s.split.tpb = e.tpb;
            s.max_blocks = e.grid;
            c->tuned_[e.cls * 8 + e.algo] = s;
            c->tuned_algo_[e.cls] = e.algo;
        }
    // direct peer access between distinct devices (xGMI); IPC mapping with
    // hipIpcMemLazyEnablePeerAccess covers the rest.
    for (int p = 0; p < c->n_; ++p) {
        int d = all[(size_t)p].device;
        if (d == device) continue;
        int can = 0;
        if (hipDeviceCanAccessPeer(&can, device, d) == hipSuccess && can) {
            hipError_t e = hipDeviceEnablePeerAccess(d, 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
        }
    }
    (void)hipGetLastError();

    // round 2: IPC handles of a new channel (unless shared) and of this
    // communicator's point-to-point region
    dbg("[rdc %d] %s\n", c->rank_, share ? "sharing the channel" : "alloc");
    if (share || !svc_all) svc_slot.release();
    if (share) {
        c->Attach(cand);
    } else {
        c->AllocChannel();
        if (svc_all) {  // the reserved slot now belongs to the channel (released by ~Channel)
            svc_slot.held = false;
            c->ch_->svc_enabled = true;
            c->ch_->svc_counted = true;
        }
    }
    c->AllocP2P();
    Handles h;
    memset(&h, 0, sizeof(h));
    if (!share) {
        Channel* mc = c->ch_.get();
        void* const own[4] = {mc->scratch, mc->scratch_ag, mc->flags, mc->svc_region};
        const char* what[4] = {"IPC handle (scratch)", "IPC handle (ag)", "IPC handle (flags)",
                               "IPC handle (service)"};
        for (int r = 0; r < 4; ++r) export_region(own[r], mc->region_bytes[r], mc->region_kind[r], &h.region[r], what[r]);
    }
    hip_check(hipIpcGetMemHandle(&h.p2p, c->p2p_), "hipIpcGetMemHandle(p2p)");
    std::vector<Handles> hs((size_t)c->n_);
    bs->allgather(&h, sizeof(h), hs.data());
    dbg("[rdc %d] %s\n", c->rank_, "handles exchanged");
    Channel* ch = c->ch_.get();
    // the channel's regions of every peer; an HSA-uncached region (kind 3)
    // that cannot be attached here is reported, not thrown: the ranks agree
    // below and, if any attach failed anywhere, every kind-3 region becomes
    // kind 0 on every rank and the regions are exchanged again
    const char* rwhat[4] = {"import (scratch)", "import (ag)", "import (flags)", "import (service)"};
    // test hook: RDC_TEST_FAIL_HSA_ATTACH=<rank> makes that rank's kind-3 attaches fail
    const char* fail_env = getenv("RDC_TEST_FAIL_HSA_ATTACH");
    const bool fail_here = fail_env && *fail_env && atoi(fail_env) == c->rank_;
    auto import_all = [&](const std::vector<Handles>& hv) -> bool {
        bool ok = true;
        for (int p = 0; p < c->n_; ++p) {
            if (p == c->rank_) continue;
            const RegionHandle* rh = hv[(size_t)p].region;
            void* got[4] = {nullptr, nullptr, nullptr, nullptr};
            for (int r = 0; r < 4; ++r) {
                ch->peer_kind[r][p] = (int8_t)rh[r].kind;
                if (rh[r].kind == kKindHsaUC) {
                    try {
                        if (fail_here) throw std::runtime_error("injected attach failure");
                        got[r] = import_region(rh[r], device, rwhat[r]);
                    } catch (const std::exception&) {
                        ok = false;
                    }
                } else {
                    got[r] = import_region(rh[r], device, rwhat[r]);
                }
            }
            ch->peer_scratch[p] = static_cast<char*>(got[0]);
            ch->peer_ag[p] = static_cast<char*>(got[1]);
            ch->peer_flags[p] = static_cast<uint64_t*>(got[2]);
            ch->peer_svc_region[p] = static_cast<char*>(got[3]);
        }
        return ok;
    };
    if (!share) {
        ch->ipc = true;
        const bool ok = import_all(hs);
        int32_t mine_ok = ok ? 1 : 0;
        std::vector<int32_t> oks((size_t)c->n_);
        bs->allgather(&mine_ok, sizeof(mine_ok), oks.data());
        bool all_ok = true;
        for (int32_t v : oks) all_ok = all_ok && v != 0;
        if (!all_ok) {
            if (c->rank_ == 0)
                fprintf(stderr, "rdc: an HSA-uncached channel region could not be attached on some rank; every "
                                "rank falls back to hipDeviceMallocUncached regions (RDC_FLAGS_MEM=cc)\n");
            for (int p = 0; p < c->n_; ++p) {
                if (p == c->rank_) continue;
                close_region(ch->peer_scratch[p], ch->peer_kind[0][p]);
                close_region(ch->peer_ag[p], ch->peer_kind[1][p]);
                close_region(ch->peer_flags[p], ch->peer_kind[2][p]);
                close_region(ch->peer_svc_region[p], ch->peer_kind[3][p]);
                ch->peer_scratch[p] = ch->peer_ag[p] = nullptr;
                ch->peer_flags[p] = nullptr;
                ch->peer_svc_region[p] = nullptr;
            }
            // every rank has let go of its peers' kind-3 regions before any
            // exporter frees its own (no detach racing the free in the runtime)
            dbg("[rdc %d] %s\n", c->rank_, "fallback: peers' regions detached");
            bs->barrier();
            void** own[4] = {reinterpret_cast<void**>(&ch->scratch), reinterpret_cast<void**>(&ch->scratch_ag),
                             reinterpret_cast<void**>(&ch->flags), reinterpret_cast<void**>(&ch->svc_region)};
            for (int r = 0; r < 4; ++r) {
                if (ch->region_kind[r] != kKindHsaUC) continue;
                free_shared(*own[r], kKindHsaUC);
                int k = 0;
                *own[r] = alloc_shared(ch->region_bytes[r], &k, device, 0);
                ch->region_kind[r] = k;
                hip_check(hipMemset(*own[r], 0, ch->region_bytes[r]), "memset channel region");
            }
            hip_check(hipDeviceSynchronize(), "sync after fallback alloc");
            dbg("[rdc %d] %s\n", c->rank_, "fallback: own regions reallocated");
            ch->peer_scratch[c->rank_] = ch->scratch;
            ch->peer_ag[c->rank_] = ch->scratch_ag;
            ch->peer_flags[c->rank_] = ch->flags;
            ch->peer_svc_region[c->rank_] = ch->svc_region;
            const char* what[4] = {"IPC handle (scratch)", "IPC handle (ag)", "IPC handle (flags)",
                                   "IPC handle (service)"};
            for (int r = 0; r < 4; ++r)
                export_region(*own[r], ch->region_bytes[r], ch->region_kind[r], &h.region[r], what[r]);
            bs->allgather(&h, sizeof(h), hs.data());
            if (!import_all(hs)) throw std::runtime_error("rdc: channel regions could not be mapped");
            dbg("[rdc %d] %s\n", c->rank_, "fallback: regions exchanged again");
        }
    }
    for (int p = 0; p < c->n_; ++p) {
        if (p == c->rank_) continue;
        void* pp = nullptr;
        hip_check(hipIpcOpenMemHandle(&pp, hs[(size_t)p].p2p, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle(p2p)");
        c->peer_p2p_[p] = static_cast<char*>(pp);
    }
    if (!share) c->Alias();  // the aliases now include the peers' mappings
    c->p2p_ctl_ = map_p2p_ctl(bs);
    if (!share)  // registered-buffer rendezvous slots, [2 parities][n]
        ch->dreg = map_shared_host(bs, round_up_bytes(2 * (size_t)c->n_ * sizeof(DirectDesc), 4096), "direct",
                                   hipHostRegisterDefault);
    if (!share && svc_all && SmallService::HxBytes() > 0)  // the same branch on every rank (agreed above)
        ch->svc_hx = map_shared_host(bs, svc_hx_bytes(c->n_), "svc",
                                     hipHostRegisterMapped | hipHostRegisterPortable | hipExtHostRegisterUncached);
    // Round 6: RDC_DIRECT_IMPORT=vmem imports peers' allocations at addresses
    // this process chooses (rdc_vmem.h) instead of through HIP IPC.  Opt-in:
    // shown on one GPU only (ranks sharing it), never across devices, and the
    // runtime's dma-buf export of a reused base can name an earlier buffer
    // object.  Collective on every rank of a new
    // multi-process channel (share and dreg are agreed); a rank that does not
    // ask for it, or cannot set it up, keeps HIP IPC everywhere.
    if (!share && ch->dreg) {
        const char* im = getenv("RDC_DIRECT_IMPORT");
        const HsaDev& hd = hsa_dev(device);
        int32_t want = im && !strcmp(im, "vmem") && hd.have_agent ? 1 : 0;
        std::vector<int32_t> wants((size_t)c->n_);
        bs->allgather(&want, sizeof(want), wants.data());
        bool all = true;
        for (int32_t v : wants) all = all && v != 0;
        std::string why;
        if (all) ch->vmem = VmemImporter::Create(bs, c->rank_, c->n_, hd.agent, std::max(30.0, cfg.timeout_s), &why);
        if (all && !ch->vmem && c->rank_ == 0)
            fprintf(stderr, "rdc: the direct schedule maps peers through HIP IPC (%s)\n", why.c_str());
    }
    dbg("[rdc %d] %s\n", c->rank_, "peers mapped");
    c->owns_peers_ipc_ = true;
    bs->barrier();
    // Round 6: the direct schedule's self-check runs once
    // per channel here, not only before Autotune, so that untuned automatic
    // calls may take the schedule (DirectEligible).  Collective: share, dreg,
    // RDC_ALGO and RDC_DIRECT_BYTES are the same on every rank (plan keys).
    if (!share && ch->dreg && cfg.algo == RDC_ALGO_AUTO && cfg.direct_min != 0) {
        dbg("[rdc %d] %s\n", c->rank_, "direct self-check");
        hipStream_t s = nullptr;
        hip_check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "self-check stream");
        try {
            c->DirectSelfCheck(s);
        } catch (...) {
            (void)hipStreamDestroy(s);
            throw;
        }
        (void)hipStreamSynchronize(s);
        (void)hipStreamDestroy(s);
        dbg("[rdc %d] %s\n", c->rank_, ch->direct_check == 1 ? "direct self-check passed" : "direct self-check failed");
    }
    return c.release();
}

Communicator* Communicator::CreateSubset(const std::string& name, Communicator* parent, const std::vector<int>& ranks,
                                         const CommConfig& cfg) {
    if (!parent->bs_)
        throw std::runtime_error("rdc: CreateGroup needs a communicator of separate processes (not RdcCommInitAll)");
    std::unique_ptr<Bootstrap> bs(ShmBootstrap::CreateGroup(parent->bs_, ranks, std::max(60.0, 4 * cfg.timeout_s)));
    if (!bs) return nullptr;
    Communicator* c = Create(name, bs.get(), parent->device_, cfg);
    c->owned_bs_ = std::move(bs);
    return c;
}

void Communicator::CreateGroup(const std::string& name, int n, const int* devices, const CommConfig& cfg,
                               std::vector<Communicator*>* out) {
    if (n < 1 || n > RDC_MAX_RANKS) throw std::runtime_error("rdc: bad group size");
    std::vector<std::unique_ptr<Communicator>> cs;
    for (int i = 0; i < n; ++i) {
        std::unique_ptr<Communicator> c(new Communicator());
        c->name_ = name;
        c->rank_ = i;
        c->n_ = n;
        c->device_ = devices[i];
        c->cfg_ = cfg;
        c->AllocLocal();
        c->ch_->svc_enabled = SmallService::Enabled();  // one process drives every rank: all or none
        cs.push_back(std::move(c));
    }
    int share = 1, cus = cs[0]->num_cus_, xcds = 1;
    for (int i = 0; i < n; ++i) {
        int same = 0;
        for (int j = 0; j < n; ++j) same += devices[i] == devices[j];
        share = std::max(share, same);
        cus = std::min(cus, cs[(size_t)i]->num_cus_);
        xcds = std::max(xcds, cs[(size_t)i]->num_xcds_);
    }
    for (auto& c : cs) {
        c->share_max_ = share;
        c->cus_min_ = cus;
        c->xcds_max_ = xcds;
    }
    if (SmallService::Enabled() && SmallService::HxBytes() > 0) {  // one exchange region every rank uses
        void* hx = nullptr;
        if (hipHostMalloc(&hx, svc_hx_bytes(n), hipHostMallocUncached | hipHostMallocMapped | hipHostMallocPortable) !=
            hipSuccess) {
            (void)hipGetLastError();
            throw std::runtime_error("rdc: cannot allocate the service's host exchange region");
        }
        memset(hx, 0, svc_hx_bytes(n));
        std::shared_ptr<char> mem(static_cast<char*>(hx), [](char* q) { (void)hipHostFree(q); });
        for (auto& c : cs) c->ch_->svc_hx = mem;
    }
    // Pinned coherent pages of its own, not a registered heap object: a
    // registration covers whole pages, and a heap object shares its first and
    // last page with unrelated allocations that the runtime may pin and unpin
    // for its own copies (see rdc_p2p.h, "Control block").
    void* mem = nullptr;
    if (hipHostMalloc(&mem, sizeof(P2PCtl), hipHostMallocCoherent | hipHostMallocMapped | hipHostMallocPortable) !=
        hipSuccess) {
        (void)hipGetLastError();
        throw std::runtime_error("rdc: cannot allocate the p2p control block in pinned host memory");
    }
    memset(mem, 0, sizeof(P2PCtl));
    std::shared_ptr<P2PCtl> ctl(new (mem) P2PCtl(), [](P2PCtl* q) {
        q->~P2PCtl();
        (void)hipHostFree(q);
    });
    for (int i = 0; i < n; ++i) {
        Communicator* ci = cs[(size_t)i].get();
        ci->p2p_ctl_ = ctl;
        for (int j = 0; j < n; ++j) {
            ci->ch_->peer_scratch[j] = cs[(size_t)j]->scratch_;
            ci->ch_->peer_ag[j] = cs[(size_t)j]->scratch_ag_;
            ci->ch_->peer_flags[j] = cs[(size_t)j]->flags_;
            ci->ch_->peer_svc_region[j] = cs[(size_t)j]->ch_->svc_region;
            ci->peer_p2p_[j] = cs[(size_t)j]->p2p_;
            if (devices[i] != devices[j]) {
                int can = 0;
                (void)hipSetDevice(devices[i]);
                if (hipDeviceCanAccessPeer(&can, devices[i], devices[j]) == hipSuccess && can)
                    (void)hipDeviceEnablePeerAccess(devices[j], 0);
                (void)hipGetLastError();
            }
        }
    }
    for (auto& c : cs) c->Alias();  // the aliases now include the peers
    out->clear();
    for (auto& c : cs) out->push_back(c.release());
}

Communicator::~Communicator() {
    if (n_ == 1 && scratch_ == nullptr) return;  // trivial communicator
    p2p_engine_.reset();  // joins the progress thread; pending requests end in error
    (void)hipSetDevice(device_);
    (void)hipDeviceSynchronize();
    if (owns_peers_ipc_ && bs_) {
        try {
            bs_->barrier();  // nobody still pushes into my p2p slots
        } catch (...) {
        }
        for (int p = 0; p < n_; ++p)
            if (p != rank_ && peer_p2p_[p]) (void)hipIpcCloseMemHandle(peer_p2p_[p]);
        try {
            bs_->barrier();  // every importer closed its mapping
        } catch (...) {
        }
    }
    for (auto& kv : pack_cache_)
        if (kv.second.dtable) (void)hipFreeAsync(kv.second.dtable, nullptr);
    for (auto& kv : direct_tables_)
        if (kv.second.dtable) (void)hipFreeAsync(kv.second.dtable, nullptr);
    if (image_) (void)hipFreeAsync(image_, nullptr);
    (void)hipStreamSynchronize(nullptr);
    for (auto& r : retired_) (void)hipEventDestroy(r.first);
    for (auto& r : direct_retired_) (void)hipEventDestroy(r.first);
    if (p2p_) (void)hipFree(p2p_);
    if (ch_) {
        {
            std::lock_guard<std::mutex> lk(ch_->mu);
            --ch_->users;
        }
        ch_.reset();  // the last user frees the channel (collective over its bootstrap)
    }
}

P2PEngine* Communicator::P2P() {
    std::lock_guard<std::mutex> lk(p2p_mu_);
    if (n_ == 1 || !p2p_) throw std::runtime_error("rdc: point-to-point needs a communicator of 2 or more ranks");
    if (!p2p_engine_)
        p2p_engine_.reset(new P2PEngine(rank_, n_, device_, cfg_.p2p_slot_bytes, p2p_, peer_p2p_, p2p_ctl_.get(),
                                        cfg_.timeout_s));
    return p2p_engine_.get();
}

WorkComp* Communicator::ISend(const void* buf, size_t bytes, int dest, hipStream_t after) {
    return P2P()->ISend(buf, bytes, dest, after);
}

WorkComp* Communicator::IRecv(void* buf, size_t bytes, int src, hipStream_t after) {
    return P2P()->IRecv(buf, bytes, src, after);
}

int Communicator::PickAlgo(int algo) const {
    if (algo == RDC_ALGO_AUTO) algo = cfg_.algo;
    if (algo == RDC_ALGO_AUTO || algo == RDC_ALGO_DIRECT) algo = RDC_ALGO_MESH;
    return algo;
}

int Communicator::PickAlgo(int algo, uint64_t bytes) const {
    if (algo == RDC_ALGO_AUTO) algo = cfg_.algo;
    // the registered-buffer schedule is taken before any plan (DirectEligible /
    // AllreduceDirect); here it means "not possible for this call"
    if (algo == RDC_ALGO_DIRECT) algo = RDC_ALGO_AUTO;
    if (algo == RDC_ALGO_AUTO) {
        algo = AutoAlgo(n_, bytes, layout(), cfg_.oneshot_push_max);
        // a schedule Autotune measured for this size class replaces the
        // rule's mesh / ring / one-shot choice (never a tree-order size; a
        // one-shot that does not fit half a slot falls back below)
        if (algo == RDC_ALGO_MESH || algo == RDC_ALGO_RING || algo == RDC_ALGO_ONESHOT) {
            const auto it = tuned_algo_.find(SizeClass(bytes));  // may be RDC_ALGO_MESH_PULL
            if (it != tuned_algo_.end() && it->second != RDC_ALGO_DIRECT) algo = it->second;
        }
    }
    if (algo == RDC_ALGO_ONESHOT && !OneshotEligible(n_, bytes, layout(), (uint64_t)-1))
        algo = RDC_ALGO_MESH;  // does not fit half a slot
    return algo;
}

void Communicator::FillArgsCommon(CollArgs* a) const {
    memset(a, 0, sizeof(*a));
    a->n = n_;
    a->rank = rank_;
    for (int c = 0; c < RDC_MAX_RANKS; ++c) a->fold[c] = (int8_t)c;
    a->slot_bytes = slot_bytes_;
    a->max_tiles = max_tiles_;
    for (int p = 0; p < n_; ++p) {
        a->rs[p] = peer_scratch_[p];
        a->ag[p] = peer_ag_[p];
        a->flags[p] = peer_flags_[p];
    }
    a->err = err_;
    a->err_mirror = err_host_dev_;
    a->done_ctr = err_ + 16;
    a->launch_ctr = reinterpret_cast<uint64_t*>(err_ + 32);  // bytes 128-135
    a->launch_kind = err_ + 48;
    a->tag = tag_;
    a->half_bytes = OneshotHalfBytes(layout());
    a->timeout_ticks = (uint64_t)(cfg_.timeout_s * (double)wall_khz_ * 1000.0);
    a->uc = (alloc_kind_ == 0 && !strict_fences()) ? 1 : 0;
    static const bool seq_check = getenv("RDC_SEQ_CHECK") && atoi(getenv("RDC_SEQ_CHECK")) != 0;
    a->seq_check = seq_check ? 1 : 0;  // device-side: blocks of one launch agree (graph replays included)
    a->poison = cfg_.poison;
    static const bool verify = getenv("RDC_VERIFY_PUBLISH") && atoi(getenv("RDC_VERIFY_PUBLISH")) != 0;
    a->verify = verify ? err_ + 84 : nullptr;
    static const bool poll_rmw = getenv("RDC_POLL_RMW") && atoi(getenv("RDC_POLL_RMW")) != 0;
    a->poll_rmw = poll_rmw ? 1 : 0;
    a->tlog = ch_ ? ch_->tlog : nullptr;
}

Layout Communicator::layout() const {
    Layout L;
    L.slot_bytes = slot_bytes_;
    L.region_bytes = region_bytes_;
    L.max_tiles = max_tiles_;
    L.flag_bytes = flag_bytes_;
    return L;
}

int Communicator::max_blocks() const { return cfg_.max_blocks > 0 ? cfg_.max_blocks : cus_min_; }

int Communicator::SizeClass(uint64_t bytes) {
    int k = 0;
    while (k < 63 && (bytes >> (k + 1)) != 0) ++k;
    return k;
}

Communicator::Shape Communicator::ShapeFor(uint64_t total, int algo) const {
    const auto it = tuned_.find(SizeClass(total) * 8 + algo);
    if (it != tuned_.end()) return it->second;
    Shape s;
    s.split = cfg_.mesh_split;
    s.max_blocks = cfg_.max_blocks;
    s.tile_bytes = cfg_.tile_bytes;
    return s;
}

// The mesh keeps more remote stores in flight with two blocks per CU (k_mesh:
// 100 VGPRs, 4 blocks per CU fit): 1 GiB on 2 ranks 1.86 -> 1.65-1.69 ms at
// 384-512 blocks (round-1 sweeps, profiles/r01/; tools/gpu_run.sh ab:).  Ranks sharing a GPU get their share
// of the resident blocks through LaunchGrid.
int Communicator::mesh_blocks() const { return cfg_.max_blocks > 0 ? cfg_.max_blocks : 2 * cus_min_; }

// One CU per rank on the GPU is left out of the resident budget: the
// small-allreduce service (rdc_service.h) keeps one persistent block per rank
// resident, and its registers (k_svc: 512 threads, ~208 VGPRs) leave no room
// for a collective block on its CU.  A grid sized to every CU would then not
// be co-resident while the service runs (RDC_NBLOCKS / Tune / Autotune can
// ask for 4 blocks per CU) and its waits would time out.
// The reservation applies only where a service can run at all: the channel's
// agreed svc_enabled and ranks per GPU within RDC_HOST_SERVICE_SHARE_MAX (both
// the same on every rank, so every rank still computes the same grid) —
// otherwise (RDC_HOST_SERVICE=0, more ranks per GPU) the CUs stay in the
// grid (8 ranks on one GPU held back 64 of 256 CUs for nothing).
int Communicator::LaunchGrid(int want, int blocks_per_cu) const {
    const bool svc = ch_ && ch_->svc_enabled && share_max_ <= SmallService::ShareMax();
    return ResidentGrid(want, blocks_per_cu, cus_min_, share_max_, xcds_max_, svc ? share_max_ : 0);
}

void Communicator::Allreduce(void* buf, size_t count, int dtype, int op, hipStream_t stream, int algo) {
    KernelSet ks;
    if (!get_kernels(dtype, op, &ks))
        throw std::invalid_argument("rdc: unsupported (dtype, op) = (" + std::to_string(dtype) + ", " +
                                    std::to_string(op) + ")");
    const size_t esz = rdc_dtype_size(dtype);
    if ((uintptr_t)buf % esz) throw std::invalid_argument("rdc: buffer not aligned to its element size");
    // Communicator::Allreduce returns at world size 1 (communicator_base.h:133-138)
    if (n_ == 1 || count == 0) return;
    if (buf == nullptr) throw std::invalid_argument("rdc: null buffer");
    hip_check(hipSetDevice(device_), "hipSetDevice");
    ChannelCall call(ch_.get(), stream);
    // TryAllreduce (communicator_collective.cc:6-13): the ring for buffers of
    // more than rdc_reduce_ring_mincount bytes, the tree's order otherwise
    if ((uint64_t)count * esz <= cfg_.ring_mincount || algo == RDC_ALGO_TREE) {
        LaunchTree(ks, static_cast<char*>(buf), (uint64_t)count * esz, stream);
        return;
    }
    if (DirectEligible(algo, (uint64_t)count * esz, stream)) {
        char* b0 = static_cast<char*>(buf);
        const uint64_t nb = (uint64_t)count * esz;
        if (AllreduceDirect(ks, &b0, &nb, 1, esz, stream)) return;
    }
    if (algo == RDC_ALGO_DIRECT) algo = RDC_ALGO_AUTO;  // not registrable here: the scratch schedules
    int64_t cb[RDC_MAX_RANKS], ce[RDC_MAX_RANKS];
    SplitRanges((int64_t)count, n_, cb, ce);  // utils::Split (include/utils/utils.h:59-70)
    uint64_t off[RDC_MAX_RANKS] = {0}, len[RDC_MAX_RANKS] = {0};
    for (int c = 0; c < n_; ++c) {
        off[c] = (uint64_t)cb[c] * esz;
        len[c] = (uint64_t)(ce[c] - cb[c]) * esz;
    }
    LaunchRanges(ks, static_cast<char*>(buf), off, len, (uint64_t)count * esz, esz, algo, stream);
}

// ------------------------------------------------- registered buffers ----
// Every check here uses values identical on every rank (the schedule asked
// for, the byte count, the channel kind, whether the stream is being
// captured — ranks capture alike), so either all ranks rendezvous or none.
//
// An automatic call (algo and RDC_ALGO auto) takes the schedule only on a
// channel whose self-check passed (DirectSelfCheck, run at channel creation:
// direct_check is agreed by a MAX allreduce, so it is rank-uniform), and then
// where Autotune / RDC_TUNE_FILE chose it for the size class, or — untuned —
// by the rule DirectAuto (RDC_DIRECT_BYTES; rdc_plan.h).  A tune file written
// on a node where the check passed therefore never turns it on where it did
// not.  An explicit algo 6 or RDC_ALGO=direct is taken as asked.
bool Communicator::DirectEligible(int algo, uint64_t bytes, hipStream_t stream) const {
    if (!ch_ || !ch_->dreg || n_ < 2) return false;  // multi-process channels only
    bool want = algo == RDC_ALGO_DIRECT || (algo == RDC_ALGO_AUTO && cfg_.algo == RDC_ALGO_DIRECT);
    if (algo == RDC_ALGO_AUTO && cfg_.algo == RDC_ALGO_AUTO) {
        if (ch_->direct_check != 1) return false;
        const auto it = tuned_algo_.find(SizeClass(bytes));
        want = it != tuned_algo_.end() ? it->second == RDC_ALGO_DIRECT
                                       : DirectAuto(n_, bytes, layout(), cfg_.oneshot_push_max, cfg_.direct_min);
    }
    if (!want) return false;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(stream, &cs) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return cs == hipStreamCaptureStatusNone;  // a rendezvous per replay is not possible
}

namespace {
// RDC_DIRECT_LOG=1: one stderr line per export and mapping of the direct
// schedule, for debugging the mapping cache
// RDC_DIRECT_ROTATE=0: every owner walks its chunk from tile 0 (A/B knob)
bool direct_rotate() {
    static const bool on = [] {
        const char* e = getenv("RDC_DIRECT_ROTATE");
        return !(e && *e == '0');
    }();
    return on;
}

// RDC_DIRECT_OVERLAP=1: use a new peer mapping even where it lands partly
// over address ranges this process unmapped before (A/B knob for the remap
// fault; off: such calls take the scratch schedules)
bool direct_overlap_ok() {
    static const bool on = [] {
        const char* e = getenv("RDC_DIRECT_OVERLAP");
        return e && *e == '1';
    }();
    return on;
}

// [b, b + n) lies partly over a range of `closed` (an exact match of base and
// size — a new allocation at an old one's place, which never faulted — is not
// an overlap)
bool partly_over(const std::vector<std::pair<uintptr_t, size_t>>& closed, uintptr_t b, size_t n) {
    for (const auto& c : closed)
        if (b < c.first + c.second && c.first < b + n && !(c.first == b && c.second == n)) return true;
    return false;
}

constexpr size_t kDirectExportsMax = 4096;  // allocations one rank exports over a channel's life
constexpr size_t kDirectMapsMax = 16384;    // peer allocations one rank maps

bool direct_log() {
    static const bool on = [] {
        const char* e = getenv("RDC_DIRECT_LOG");
        return e && *e && *e != '0';
    }();
    return on;
}

// spin until every slot of `slots` carries `stamp` in the field `field`
// (release-stored last by its owner); false on timeout
bool rendezvous_wait(DirectDesc* slots, int n, uint64_t DirectDesc::*field, uint64_t stamp, double timeout_s) {
    const auto t0 = std::chrono::steady_clock::now();
    for (int p = 0; p < n; ++p) {
        uint32_t spins = 0;
        while (__atomic_load_n(&(slots[p].*field), __ATOMIC_ACQUIRE) != stamp) {
            __builtin_ia32_pause();
            if ((++spins & 1023) == 0 &&
                std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s)
                return false;
        }
    }
    return true;
}
}  // namespace

// Step 1 of AllreduceDirect: this rank's buffers as (allocation, offset)
// and the allocations' IPC handles, into its rendezvous slot `me`; false when
// any buffer cannot be exported (the call then falls back on every rank).
// own_base[i] = the base of me.alloc[i] in this process.
//
// Mapping life cycle (round 6; round 5's rule kept every mapping for the
// channel's life).  A HIP IPC handle names an allocation by (exporting
// process, base address), and an importer that still holds a mapping of an
// earlier allocation at the same base gets that old mapping back — stale
// memory — when it opens the new handle (round 5, profiles/r05/direct/).  So
// this rank RETIRES every allocation it exported that is gone (its buffer id
// at the base changed or the base is no longer allocated): the ones that
// overlap a buffer of this call always (before that buffer's allocation is
// exported, possibly at the same base), and up to kRetireScan others per call
// round-robin.  The retired ids ride in this rank's slot; every peer closes
// its mapping of them (DirectMapPeers) BEFORE it opens anything in the same
// rendezvous, so the old mapping is never handed back, and the exporter's
// freed memory is released once every peer closed.
namespace {
constexpr size_t kRetireScan = 16;  // exports checked per call beyond this call's own ranges

// the allocation that now holds `base` in this process, if any
uint64_t live_buffer_id(uintptr_t base) {
    unsigned long long id = 0;
    if (hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)base) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return (uint64_t)id;
}
}  // namespace

bool Communicator::DirectExport(DirectDesc& me, char* const* bufs, const uint64_t* bytes, int nbuf, uint64_t call,
                                std::vector<char*>* own_base,
                                std::vector<std::pair<uint32_t, std::pair<char*, uint32_t>>>* fresh) {
    fresh->clear();
    Channel& ch = *ch_;
    me.nalloc = 0;
    me.nretired = 0;
    me.nbuf = (uint32_t)nbuf;
    if (ch.direct_off || nbuf < 1 || nbuf > kDirectBufsMax) return false;
    // vmem: the dma-bufs of the allocations retired in this call close when
    // this function returns — after this call's new exports, which must not
    // get one of them back (VmemImporter::Export)
    struct ReleaseAtExit {
        VmemImporter* v;
        std::vector<uint64_t> ids;
        ~ReleaseAtExit() {
            if (v)
                for (uint64_t id : ids) v->Release(id);
        }
    } release_at_exit{ch.vmem.get(), {}};
    auto retire = [&](std::map<uintptr_t, Channel::DirectExport>::iterator it) -> bool {
        if (me.nretired >= (uint32_t)kDirectRetireMax) return false;
        me.retired[me.nretired++] = it->second.id;
        release_at_exit.ids.push_back(it->second.id);
        ch.dclosed.emplace_back(it->first, it->second.size);
        if (direct_log())
            fprintf(stderr, "rdc-direct r%d call %llu: retire id %llu (base %p)\n", rank_, (unsigned long long)call,
                    (unsigned long long)it->second.id, (void*)it->first);
        if (ch.dscan == it->first) ch.dscan = it->first + 1;
        ch.dexports.erase(it);
        ++ch.dstat_retired;
        return true;
    };
    std::unordered_map<uint64_t, uint32_t> alloc_index;  // allocation id -> index in me.alloc
    for (int b = 0; b < nbuf; ++b) {
        char* buf = bufs[b];
        unsigned long long id = 0;
        hipDeviceptr_t base = nullptr;
        size_t size = 0;
        hipPointerAttribute_t at;
        const bool dev = hipPointerGetAttributes(&at, buf) == hipSuccess && at.type == hipMemoryTypeDevice &&
                         hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)buf) ==
                             hipSuccess &&
                         hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)buf) == hipSuccess && base != nullptr &&
                         buf + bytes[b] <= (char*)base + size;
        (void)hipGetLastError();
        if (!dev) {
            if (direct_log())
                fprintf(stderr, "rdc-direct r%d call %llu: buffer %d %p is not exportable device memory\n", rank_,
                        (unsigned long long)call, b, (void*)buf);
            return false;
        }
        auto ix = alloc_index.find((uint64_t)id);
        const uint32_t ai = ix != alloc_index.end() ? ix->second : me.nalloc;
        if (ai == me.nalloc) {  // this call's first buffer in that allocation: export it
            const uintptr_t bs = (uintptr_t)base;
            const char* why = nullptr;
            // every earlier export overlapping [bs, bs + size) under another id
            // belongs to a dead allocation (live ones do not overlap): retire it
            auto nx = ch.dexports.upper_bound(bs);
            if (nx != ch.dexports.begin()) --nx;
            while (!why && nx != ch.dexports.end() && nx->first < bs + size) {
                auto cur = nx++;
                if (cur->first + cur->second.size <= bs || cur->second.id == (uint64_t)id) continue;
                if (!retire(cur)) why = "retire list full";
            }
            // hipIpcOpenMemHandle of an allocation of 2 GiB or more never
            // returns on this stack (rdc_plan.h kMaxRegionBytes): such a
            // buffer takes the scratch schedules (round 6: the untuned default
            // sent test_mp_count_beyond_int32's 2 GiB buffer here and hung)
            if (!why && size > kMaxRegionBytes) why = "allocation of 2 GiB or more (HIP IPC cannot map it)";
            auto it = ch.dexports.find(bs);
            if (!why && it == ch.dexports.end()) {
                if (ch.dexports.size() >= kDirectExportsMax)
                    why = "export table full";
                else {
                    Channel::DirectExport ex;
                    ex.id = (uint64_t)id;
                    ex.size = size;
                    std::string xw;
                    const hipError_t ge = ch.vmem ? (ch.vmem->Export(base, size, (uint64_t)id, &xw)
                                                         ? hipSuccess
                                                         : hipErrorInvalidValue)
                                                  : hipIpcGetMemHandle(&ex.handle, base);
                    (void)hipGetLastError();
                    if (ch.vmem) memset(&ex.handle, 0, sizeof(ex.handle));
                    if (ge == hipSuccess) {
                        it = ch.dexports.emplace(bs, ex).first;
                    } else {
                        why = "no IPC handle";
                        ch.dexport_err = (uint64_t)ge;
                        ++ch.dstat_exportfail;
                        if (direct_log())
                            fprintf(stderr, "rdc-direct r%d call %llu: %s(%p): %s (%d), %u retired in this call\n",
                                    rank_, (unsigned long long)call, ch.vmem ? "dma-buf export" : "hipIpcGetMemHandle",
                                    (void*)base, ch.vmem ? xw.c_str() : hipGetErrorName(ge), (int)ge, me.nretired);
                    }
                }
            }
            if (!why && me.nalloc >= (uint32_t)kDirectAllocsMax) why = "too many allocations in one call";
            // a new export is checked by its importers through a canary in
            // this buffer's first (up to 8) bytes
            const bool is_new = !why && it != ch.dexports.end() && !it->second.verified;
            const uint32_t canary_len = (uint32_t)std::min<uint64_t>(8, bytes[b]);
            if (direct_log())
                fprintf(stderr, "rdc-direct r%d call %llu: buffer %d %p id %llu base %p size %zu%s%s\n", rank_,
                        (unsigned long long)call, b, (void*)buf, id, (void*)base, size,
                        why ? ": not exported, " : "", why ? why : "");
            if (why) return false;
            me.alloc[ai].id = (uint64_t)id;
            me.alloc[ai].handle = it->second.handle;
            me.alloc[ai].nonce = 0;
            me.alloc[ai].canary_off = 0;
            me.alloc[ai].canary_len = 0;
            if (is_new && canary_len) fresh->emplace_back(ai, std::make_pair(buf, canary_len));
            alloc_index.emplace((uint64_t)id, ai);
            own_base->push_back((char*)base);
            ++me.nalloc;
        }
        me.buf[b].alloc = ai;
        me.buf[b].mis16 = (uint32_t)((uintptr_t)buf & 15);
        me.buf[b].off = (uint64_t)(buf - (char*)base);
        me.buf[b].bytes = bytes[b];
    }
    // round-robin check of the other exports: allocations freed since
    if (!ch.dexports.empty()) {
        auto it = ch.dexports.lower_bound(ch.dscan);
        for (size_t k = 0; k < std::min(kRetireScan, ch.dexports.size()) && me.nretired < (uint32_t)kDirectRetireMax;
             ++k) {
            if (it == ch.dexports.end()) it = ch.dexports.begin();
            auto cur = it++;
            if (alloc_index.count(cur->second.id)) continue;  // in use by this call
            if (live_buffer_id(cur->first) != cur->second.id) retire(cur);
        }
        ch.dscan = it == ch.dexports.end() ? 0 : it->first;
    }
    return true;
}

// Step 2: every rank's allocations as mapped in this process (*amap, indexed
// q * kDirectAllocsMax + i; this rank's own from own_base), opening the ones
// not mapped yet; false when one cannot be mapped.  Before it (every call,
// usable or not: DirectCloseRetired), the mappings of allocations the peers
// retired are closed — after this rank's previous direct launch (the last
// one that may read through them) has completed
// (hipIpcCloseMemHandle also waits for the device: 250 ms for a kernel
// spinning 250 ms, tools/ipc_remap_probe.hip "inflight").  A new mapping that
// lands partly over a range this process unmapped or retired is closed again
// unused and the call falls back on every rank (the peer allocation stays
// refused): the first launch through such a mapping faulted the GPU in round
// 5 and, with those ranges held by hipMemAddressReserve, again in round 6
// (profiles/r06/remap/).
void Communicator::DirectCloseRetired(const DirectDesc* slots, uint64_t call) {
    Channel& ch = *ch_;
    bool waited = false;
    if (ch.vmem) ch.vmem->Drain();  // the dma-bufs the peers sent before this rendezvous
    for (int p = 0; p < n_; ++p) {
        if (p == rank_) continue;
        const uint32_t nr = std::min<uint32_t>(slots[p].nretired, (uint32_t)kDirectRetireMax);
        if (ch.vmem)
            for (uint32_t k = 0; k < nr; ++k) ch.vmem->Forget(p, slots[p].retired[k]);  // received, never mapped
        for (uint32_t k = 0; k < nr; ++k) {
            auto it = ch.dmaps.find(std::make_pair(p, slots[p].retired[k]));
            if (it == ch.dmaps.end()) continue;
            if (!waited && ch.dlast) {
                const auto t0 = std::chrono::steady_clock::now();
                hip_check(hipEventSynchronize(ch.dlast), "wait for the previous direct launch");
                ch.dstat_close_wait_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                                              std::chrono::steady_clock::now() - t0)
                                              .count();
                waited = true;
            }
            const Channel::DirectMap m = it->second;
            ch.dmaps.erase(it);
            hipError_t e = hipSuccess;
            if (ch.vmem) {
                ch.vmem->Unmap(m.ptr);  // its range is only ever handed out again whole
            } else {
                e = hipIpcCloseMemHandle(m.ptr);
                (void)hipGetLastError();
                if (m.size) ch.dclosed.emplace_back((uintptr_t)m.ptr, m.size);
            }
            ++ch.dstat_closed;
            if (direct_log())
                fprintf(stderr, "rdc-direct r%d call %llu: close peer %d id %llu at %p (%zu B)%s\n", rank_,
                        (unsigned long long)call, p, (unsigned long long)slots[p].retired[k], (void*)m.ptr, m.size,
                        e == hipSuccess ? "" : " FAILED");
            // device tables naming that allocation can never match a later call
            // (buffer ids are not reused); they age out of the LRU
        }
        for (uint32_t k = 0; k < nr; ++k) ch.drefused.erase(std::make_pair(p, slots[p].retired[k]));
    }
}

// A new peer mapping is that peer's current allocation only if it shows the
// nonce the exporter wrote for this rendezvous (DirectAlloc::nonce).
bool Communicator::CanaryOk(const DirectAlloc& al, char* mapped, size_t size, int p, uint64_t call) {
    if (al.canary_len == 0) return true;
    Channel& ch = *ch_;
    if (al.canary_len > 8 || (size && al.canary_off + al.canary_len > size)) return false;
    if (!ch.dpeek_stream) {
        hip_check(hipStreamCreateWithFlags(&ch.dpeek_stream, hipStreamNonBlocking), "direct canary stream");
        hip_check(hipHostMalloc(reinterpret_cast<void**>(&ch.dpeek_host), 64, hipHostMallocCoherent),
                  "direct canary word");
    }
    *ch.dpeek_host = 0;
    hip_check(Peek(mapped + al.canary_off, (uint32_t)al.canary_len, ch.dpeek_host, ch.dpeek_stream),
              "direct canary read");
    hip_check(hipStreamSynchronize(ch.dpeek_stream), "direct canary read done");
    const uint64_t got = __atomic_load_n(ch.dpeek_host, __ATOMIC_ACQUIRE);
    ++ch.dstat_canary;
    if (got != al.nonce && direct_log())
        fprintf(stderr, "rdc-direct r%d call %llu: peer %d id %llu: canary %016llx, expected %016llx\n", rank_,
                (unsigned long long)call, p, (unsigned long long)al.id, (unsigned long long)got,
                (unsigned long long)al.nonce);
    return got == al.nonce;
}

bool Communicator::DirectMapPeers(const DirectDesc* slots, const std::vector<char*>& own_base, uint64_t call,
                                  std::vector<char*>* amap) {
    Channel& ch = *ch_;
    amap->assign((size_t)n_ * kDirectAllocsMax, nullptr);
    for (int p = 0; p < n_; ++p)
        for (uint32_t i = 0; i < slots[p].nalloc; ++i) {
            char*& dst = (*amap)[(size_t)p * kDirectAllocsMax + i];
            if (p == rank_) {
                dst = own_base[i];
                continue;
            }
            auto key = std::make_pair(p, slots[p].alloc[i].id);
            auto it = ch.dmaps.find(key);
            if (it == ch.dmaps.end()) {
                auto fail = [&](int code, const char* why) {
                    ch.dfail_reason = code;
                    ++ch.dstat_mapfail;
                    if (direct_log())
                        fprintf(stderr, "rdc-direct r%d call %llu: peer %d id %llu not mapped: %s\n", rank_,
                                (unsigned long long)call, p, (unsigned long long)slots[p].alloc[i].id, why);
                    return false;
                };
                if (ch.dmaps.size() >= kDirectMapsMax) return fail(1, "mapping table full");
                if (ch.vmem) {  // at an address this process chose: no placement to refuse
                    Channel::DirectMap dm;
                    std::string w;
                    if (!ch.vmem->Map(p, slots[p].alloc[i].id, &dm.ptr, &dm.size, &w)) return fail(3, w.c_str());
                    if (direct_log())
                        fprintf(stderr, "rdc-direct r%d call %llu: map peer %d id %llu -> %p (%zu B)\n", rank_,
                                (unsigned long long)call, p, (unsigned long long)slots[p].alloc[i].id,
                                (void*)dm.ptr, dm.size);
                    if (!CanaryOk(slots[p].alloc[i], dm.ptr, dm.size, p, call)) {
                        ch.vmem->Unmap(dm.ptr);  // read once by the check, never by a collective
                        ch.drefused.insert(key);
                        ++ch.dstat_refused;
                        return fail(6, "maps another buffer object (canary)");
                    }
                    it = ch.dmaps.emplace(key, dm).first;
                    dst = it->second.ptr;
                    continue;
                }
                if (ch.drefused.count(key)) {  // counted per call that falls back for it
                    ++ch.dstat_refused;
                    return fail(2, "refused earlier (landed over unmapped ranges)");
                }
                void* m = nullptr;
                const hipError_t oe = hipIpcOpenMemHandle(&m, slots[p].alloc[i].handle, hipIpcMemLazyEnablePeerAccess);
                if (oe != hipSuccess || !m) {
                    (void)hipGetLastError();
                    return fail(3, oe != hipSuccess ? hipGetErrorString(oe) : "null mapping");
                }
                // a pointer this rank already holds for another allocation
                // would be the stale mapping described above: never use it
                bool dup = false;
                for (auto& o : ch.dmaps) dup = dup || o.second.ptr == (char*)m;
                Channel::DirectMap dm;
                dm.ptr = static_cast<char*>(m);
                hipDeviceptr_t mb = nullptr;
                if (hipMemGetAddressRange(&mb, &dm.size, (hipDeviceptr_t)m) != hipSuccess || mb != m) dm.size = 0;
                (void)hipGetLastError();
                const bool over = !dup && !direct_overlap_ok() &&
                                  partly_over(ch.dclosed, (uintptr_t)m, dm.size ? dm.size : 1);
                if (direct_log())
                    fprintf(stderr, "rdc-direct r%d call %llu: open peer %d id %llu -> %p (%zu B)%s\n", rank_,
                            (unsigned long long)call, p, (unsigned long long)slots[p].alloc[i].id, m, dm.size,
                            dup ? " (a mapping already held: not used)"
                                : over ? " (lands partly over unmapped ranges: closed unused, refused)" : "");
                if (dup) {
                    ch.dfail_reason = 4;
                    ++ch.dstat_mapfail;
                    return false;
                }
                if (over) {  // never touched by a kernel: close it again and fall back
                    (void)hipIpcCloseMemHandle(m);
                    (void)hipGetLastError();
                    ch.drefused.insert(key);
                    ++ch.dstat_refused;
                    ch.dfail_reason = 5;
                    ++ch.dstat_mapfail;
                    return false;
                }
                if (!CanaryOk(slots[p].alloc[i], dm.ptr, dm.size, p, call)) {
                    (void)hipIpcCloseMemHandle(m);  // read once by the check, never by a collective
                    (void)hipGetLastError();
                    if (dm.size) ch.dclosed.emplace_back((uintptr_t)m, dm.size);
                    ch.drefused.insert(key);
                    ++ch.dstat_refused;
                    return fail(6, "maps another buffer object (canary)");
                }
                it = ch.dmaps.emplace(key, dm).first;
            }
            dst = it->second.ptr;
        }
    return true;
}

// The device table of a coalesced direct launch: this owner's items (chunk
// rank_ of every buffer in pieces of at most `tile`: {buffer, byte offset,
// length} as 3 words), then every rank's buffer addresses as mapped here
// (ptr[q * nbuf + b]).  Cached by the layout (every rank's allocations and
// offsets), so a repeated bucket list uploads nothing; evicted tables are
// freed stream-ordered and their host copies kept until the upload is done.
const Communicator::DirectTable& Communicator::DirectTableFor(const DirectDesc* slots, const uint64_t* bytes,
                                                              int nbuf, size_t esz, uint64_t tile,
                                                              const std::vector<char*>& amap, hipStream_t stream) {
    std::vector<uint64_t> key;
    key.reserve(2 + (size_t)nbuf * (1 + 2 * (size_t)n_));
    key.push_back(esz);
    key.push_back(tile);
    for (int b = 0; b < nbuf; ++b) key.push_back(bytes[b]);
    for (int p = 0; p < n_; ++p)
        for (int b = 0; b < nbuf; ++b) {
            key.push_back(slots[p].alloc[slots[p].buf[b].alloc].id);
            key.push_back(slots[p].buf[b].off);
        }
    auto it = direct_tables_.find(key);
    if (it == direct_tables_.end()) {
        if (direct_tables_.size() >= 16) {  // evict the least recently used layout
            auto lru = direct_tables_.begin();
            for (auto j = direct_tables_.begin(); j != direct_tables_.end(); ++j)
                if (j->second.last_use < lru->second.last_use) lru = j;
            if (lru->second.dtable) hip_check(hipFreeAsync(lru->second.dtable, stream), "release direct table");
            hipEvent_t ev = nullptr;
            hip_check(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "event");
            hip_check(hipEventRecord(ev, stream), "record");
            direct_retired_.emplace_back(ev, lru->second.host);
            direct_tables_.erase(lru);
        }
        for (size_t i = 0; i < direct_retired_.size();) {  // host copies whose upload has surely finished
            if (hipEventQuery(direct_retired_[i].first) == hipSuccess) {
                (void)hipEventDestroy(direct_retired_[i].first);
                direct_retired_[i] = direct_retired_.back();
                direct_retired_.pop_back();
            } else {
                (void)hipGetLastError();
                ++i;
            }
        }
        auto host = std::make_shared<std::vector<uint64_t>>(PlanDirectItems(n_, rank_, bytes, nbuf, esz, tile));
        const int nitems = (int)(host->size() / 3);
        for (int p = 0; p < n_; ++p)
            for (int b = 0; b < nbuf; ++b)
                host->push_back((uint64_t)(uintptr_t)(amap[(size_t)p * kDirectAllocsMax + slots[p].buf[b].alloc] +
                                                      slots[p].buf[b].off));
        DirectTable t;
        t.nitems = nitems;
        t.tile = tile;
        t.host = host;
        const size_t tb = host->size() * sizeof(uint64_t);
        hip_check(hipMallocAsync(&t.dtable, tb, stream), "allocate direct table");
        hip_check(hipMemcpyAsync(t.dtable, host->data(), tb, hipMemcpyHostToDevice, stream), "upload direct table");
        it = direct_tables_.emplace(std::move(key), t).first;
    }
    it->second.last_use = ++direct_tick_;
    return it->second;
}

bool Communicator::AllreduceDirect(const KernelSet& ks, char* const* bufs, const uint64_t* bytes, int nbuf,
                                   size_t esz, hipStream_t stream) {
    Channel& ch = *ch_;
    const uint64_t call = ++ch.dcalls;  // the same on every rank (DirectEligible)
    DirectDesc* slots = reinterpret_cast<DirectDesc*>(ch.dreg.get()) + (call & 1) * (uint64_t)n_;
    DirectDesc& me = slots[rank_];
    const auto t0 = std::chrono::steady_clock::now();
    // 1) publish this rank's buffers
    std::vector<char*> own_base;
    std::vector<std::pair<uint32_t, std::pair<char*, uint32_t>>> fresh;
    me.valid = DirectExport(me, bufs, bytes, nbuf, call, &own_base, &fresh) ? 1 : 0;
    // The canary (round 6): after an allocation was exported and freed, the
    // runtime can resolve a new allocation at the same base to the earlier
    // buffer object, and a peer mapping that object reads and writes memory
    // that is not this buffer (test_mp_direct_after_free[3-ipc] read one wrong
    // chunk once; profiles/r06/canary/).  So each allocation this rank
    // exports carries, until every importer has read it through its new
    // mapping, a random nonce in 8 bytes of one of this call's buffers; the
    // original bytes go back, stream-ordered before any launch, after the
    // second rendezvous stamp.  Only calls with new allocations pay for it.
    struct Saved {
        char* at;
        uint32_t len;
        uint64_t orig, nonce;
    };
    std::vector<Saved> saved;  // canary address and length, original bytes, nonce
    if (me.valid && !fresh.empty()) {
        hip_check(hipStreamSynchronize(stream), "direct canary: inputs ready");
        saved.resize(fresh.size());
        static thread_local std::mt19937_64 rng(std::random_device{}() ^ ((uint64_t)getpid() << 32));
        for (size_t k = 0; k < fresh.size(); ++k) {
            Saved& sv = saved[k];
            const uint32_t ai = fresh[k].first;
            sv.at = fresh[k].second.first;
            sv.len = fresh[k].second.second;
            sv.orig = 0;
            hip_check(hipMemcpyAsync(&sv.orig, sv.at, sv.len, hipMemcpyDeviceToHost, stream), "direct canary: save");
            hip_check(hipStreamSynchronize(stream), "direct canary: saved");
            do {  // differs from the bytes it replaces
                sv.nonce = rng();
                if (sv.len < 8) sv.nonce &= (1ull << (8 * sv.len)) - 1;
            } while (sv.nonce == sv.orig);
            hip_check(Poke(sv.at, sv.len, sv.nonce, stream), "direct canary: write");
            me.alloc[ai].nonce = sv.nonce;
            me.alloc[ai].canary_off = (uint64_t)(sv.at - own_base[ai]);
            me.alloc[ai].canary_len = sv.len;
        }
        hip_check(hipStreamSynchronize(stream), "direct canary: written");
    }
    const double export_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    __atomic_store_n(&me.stamp0, call, __ATOMIC_RELEASE);
    if (!rendezvous_wait(slots, n_, &DirectDesc::stamp0, call, cfg_.timeout_s))
        throw std::runtime_error("rdc: registered-buffer rendezvous timed out (a peer did not join the allreduce)");
    // the peers' retired allocations: closed whether or not this call runs
    // direct (an exporter announces each retirement once)
    DirectCloseRetired(slots, call);
    // 2) every rank's list usable and alike (same buffers' sizes, each buffer
    // congruent mod 16 on every rank)?  Then map the peers' allocations
    bool usable = true;
    for (int p = 0; p < n_ && usable; ++p) {
        usable = slots[p].valid && slots[p].nbuf == (uint32_t)nbuf;
        for (int b = 0; b < nbuf && usable; ++b)
            usable = slots[p].buf[b].bytes == bytes[b] && slots[p].buf[b].mis16 == me.buf[b].mis16;
    }
    std::vector<char*> amap;  // rank q's allocation i as mapped here, at q * kDirectAllocsMax + i
    me.ok = usable && DirectMapPeers(slots, own_base, call, &amap) ? 1 : 0;
    __atomic_store_n(&me.stamp1, call, __ATOMIC_RELEASE);
    if (!rendezvous_wait(slots, n_, &DirectDesc::stamp1, call, cfg_.timeout_s))
        throw std::runtime_error("rdc: registered-buffer rendezvous timed out (a peer did not join the allreduce)");
    if (!usable) ++ch.dstat_unusable;  // some rank's list not exportable, or the lists differ
    for (int p = 0; p < n_; ++p) usable = usable && slots[p].ok;
    if (!usable) ++ch.dstat_fallback;
    if (!saved.empty()) {  // every importer has read the canaries: the inputs go back
        // stream-ordered before this call's kernel, whose ready signal (a
        // system-scope release) publishes these bytes to the peers' reads
        for (auto& sv : saved) hip_check(Poke(sv.at, sv.len, sv.orig, stream), "direct canary: restore");
        if (usable)
            for (auto& f : fresh) {
                auto ex = ch.dexports.find((uintptr_t)own_base[f.first]);
                if (ex != ch.dexports.end()) ex->second.verified = true;
            }
    }
    ++ch.dstat_calls;
    ch.dstat_export_ns += (uint64_t)(export_us * 1e3);
    ch.dstat_rdv_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                           std::chrono::steady_clock::now() - t0)
                           .count();
    if (direct_log())
        fprintf(stderr, "rdc-direct r%d call %llu: %d buffers in %u allocations, export %.1f us, total %.1f us, %s\n",
                rank_, (unsigned long long)call, nbuf, me.nalloc, export_us,
                std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count(),
                usable ? "direct" : "fallback");
    if (!usable) return false;  // every rank saw the same slots: all fall back together
    // 3) one launch: owner r folds chunk r of every buffer in place
    uint64_t total = 0;
    for (int b = 0; b < nbuf; ++b) total += bytes[b];
    CollArgs a;
    FillArgsCommon(&a);
    a.kind = RDC_KIND_DIRECT;
    a.rotate = direct_rotate() ? 1 : 0;
    const Shape sh = ShapeFor(total, RDC_ALGO_DIRECT);  // an Autotune'd grid, else the mesh's
    const int grid_cap = LaunchGrid(sh.max_blocks > 0 ? sh.max_blocks : mesh_blocks(),
                                    ks.occupancy(RDC_KIND_DIRECT, n_));
    // ~2 tiles (items) per block, 64 KiB .. 4 MiB, a multiple of 256 B
    uint64_t tile = total / n_ / (2 * (uint64_t)grid_cap) + 1;
    tile = std::min<uint64_t>(std::max<uint64_t>(tile, 64 << 10), 4 << 20);
    tile = (tile + 255) & ~(uint64_t)255;
    int grid = 1;
    if (nbuf == 1) {
        int64_t cb[RDC_MAX_RANKS], ce[RDC_MAX_RANKS];
        SplitRanges((int64_t)(bytes[0] / esz), n_, cb, ce);
        a.user = bufs[0];
        for (int c = 0; c < n_; ++c) {
            a.off[c] = (uint64_t)cb[c] * esz;
            a.len[c] = (uint64_t)(ce[c] - cb[c]) * esz;
            a.cbuf[c] = amap[(size_t)c * kDirectAllocsMax + slots[c].buf[0].alloc] + slots[c].buf[0].off;
        }
        const int tiles = (int)std::max<uint64_t>(1, (a.len[rank_] + tile - 1) / tile);
        a.tile_bytes = tile;
        a.tiles[rank_] = a.len[rank_] ? tiles : 0;
        grid = std::max(1, std::min(tiles, grid_cap));
    } else {
        const DirectTable& t = DirectTableFor(slots, bytes, nbuf, esz, tile, amap, stream);
        a.user = bufs[0];
        a.units = t.dtable;
        a.nunits = t.nitems;
        a.dnbuf = nbuf;
        a.tile_bytes = tile;
        grid = std::max(1, std::min(t.nitems, grid_cap));
    }
    if (notify_) {
        a.notify = notify_;
        a.notify_val = notify_val_;
        notify_ = nullptr;
    }
    last_launch_[0] = (uint64_t)grid;
    last_launch_[1] = last_launch_[2] = last_launch_[3] = 0;
    last_launch_[4] = tile;
    last_launch_[5] = RDC_ALGO_DIRECT;
    ++seq_;
    log_launch(this, seq_, RDC_ALGO_DIRECT, total, grid, tile);
    hip_check(ks.direct(a, grid, stream), "launch direct allreduce");
    // the last launch that may read through this rank's peer mappings: a
    // later rendezvous that closes one of them waits for it first
    if (!ch.dlast) hip_check(hipEventCreateWithFlags(&ch.dlast, hipEventDisableTiming), "direct event");
    hip_check(hipEventRecord(ch.dlast, stream), "record direct launch");
    trace_ = nullptr;
    return true;
}

// The channel's own hipMalloc buffer of at least `bytes` (Autotune, the
// direct self-check): peers map it, so an outgrown one is kept, not freed.
void Communicator::TuneBuffer(size_t bytes) {
    Channel& ch = *ch_;
    if (ch.tune_bytes >= bytes) return;
    if (ch.tune_buf) ch.tune_old.push_back(ch.tune_buf);
    ch.tune_buf = nullptr;
    ch.tune_bytes = 0;
    hip_check(hipMalloc(&ch.tune_buf, bytes), "autotune buffer");
    ch.tune_bytes = bytes;
}

// One int32 BitOR allreduce of 4 MiB by the direct schedule and one by the
// ring on the same input (the ring's result is the reference: every schedule
// gives the same bits).  The direct result is then read by a KERNEL
// (k_reduce: 0 | x) so that it comes through the caches of this GPU, where a
// line written by another GPU could be stale, not through a DMA engine.  Both
// land on the host, every rank compares, and the ranks agree (MAX) before
// anyone uses the answer.  A failure is reported on stderr and the direct
// schedule is left out of every Autotune on this channel.
int Communicator::DirectSelfCheck(hipStream_t stream) {
    Channel& ch = *ch_;
    if (ch.direct_check) return ch.direct_check;
    KernelSet ks;
    if (!get_kernels(RDC_DT_INT32, RDC_OP_BITOR, &ks)) throw std::logic_error("rdc: no int32 BitOR kernels");
    const size_t count = (size_t)1 << 20, nb = count * sizeof(int32_t);
    hip_check(hipSetDevice(device_), "hipSetDevice");
    TuneBuffer(3 * nb);
    char* x = static_cast<char*>(ch.tune_buf);
    char* y = x + nb;
    char* z = y + nb;
    DeviceFill(x, count, RDC_DT_INT32, 0x5EEDC4ECull, rank_, stream);
    hip_check(hipMemcpyAsync(y, x, nb, hipMemcpyDeviceToDevice, stream), "self-check copy");
    hip_check(hipMemsetAsync(z, 0, nb, stream), "self-check zero");
    Allreduce(y, count, RDC_DT_INT32, RDC_OP_BITOR, stream, RDC_ALGO_RING);
    Allreduce(x, count, RDC_DT_INT32, RDC_OP_BITOR, stream, RDC_ALGO_DIRECT);
    const bool took = last_launch_[5] == RDC_ALGO_DIRECT;
    hip_check(ks.reduce(z, x, nb, 2 * cus_min_, stream), "self-check read-back");
    std::vector<char> hy(nb), hz(nb);
    hip_check(hipMemcpyAsync(hy.data(), y, nb, hipMemcpyDeviceToHost, stream), "D2H");
    hip_check(hipMemcpyAsync(hz.data(), z, nb, hipMemcpyDeviceToHost, stream), "D2H");
    Check(stream);
    int32_t bad = (!took || memcmp(hy.data(), hz.data(), nb) != 0) ? 1 : 0;
    // agree: every rank's flag, MAX over ranks (a scratch schedule: 4 bytes)
    hip_check(hipMemcpyAsync(z, &bad, sizeof(bad), hipMemcpyHostToDevice, stream), "H2D");
    Allreduce(z, 1, RDC_DT_INT32, RDC_OP_MAX, stream, RDC_ALGO_AUTO);
    hip_check(hipMemcpyAsync(&bad, z, sizeof(bad), hipMemcpyDeviceToHost, stream), "D2H");
    Check(stream);
    ch.direct_check = bad ? 2 : 1;
    if (bad && rank_ == 0 && !ch.direct_off)
        fprintf(stderr, "rdc: the direct schedule failed its self-check on this node (%s); Autotune leaves it out\n",
                took ? "results differ from the ring's" : "it did not run");
    return ch.direct_check;
}

uint64_t Communicator::DirectStat(const std::string& k) const {
    if (!ch_) return 0;
    const Channel& ch = *ch_;
    if (k == "direct_calls") return ch.dstat_calls;
    if (k == "direct_rendezvous_ns") return ch.dstat_rdv_ns;
    if (k == "direct_export_ns") return ch.dstat_export_ns;
    if (k == "direct_retired") return ch.dstat_retired;
    if (k == "direct_closed") return ch.dstat_closed;
    if (k == "direct_refused") return ch.dstat_refused;
    if (k == "direct_fallback") return ch.dstat_fallback;
    if (k == "direct_unusable") return ch.dstat_unusable;
    if (k == "direct_map_failed") return ch.dstat_mapfail;
    if (k == "direct_fail_reason") return ch.dfail_reason;
    if (k == "direct_export_failed") return ch.dstat_exportfail;
    if (k == "direct_export_error") return ch.dexport_err;
    if (k == "direct_import") return ch.vmem ? 1 : 0;
    if (k == "direct_canary") return ch.dstat_canary;
    if (k == "direct_pending") return ch.vmem ? ch.vmem->pending() : 0;
    if (k == "direct_close_wait_ns") return ch.dstat_close_wait_ns;
    if (k == "direct_maps") return ch.dmaps.size();
    if (k == "direct_exports") return ch.dexports.size();
    throw std::invalid_argument("rdc: unknown parameter " + k);
}

// Closes every peer-buffer mapping of the direct schedule and turns the
// schedule off for the channel (re-mapping into just-unmapped address ranges
// faulted the GPU in round 5's tests, so nothing is mapped again).  A mapping
// keeps the peer's allocation alive after the peer frees it: this releases
// them.  Every rank should call it (a rank that has it off makes every call
// fall back anyway).
// direct_check stays as agreed (a release on a subset of ranks
// must not make the ranks' Autotune candidate lists or self-check collectives
// differ); direct_off alone makes this rank publish valid = 0 at every later
// rendezvous, so every rank falls back together.
void Communicator::DirectUnmapAll() {
    if (!ch_) return;
    if (!ch_->dmaps.empty()) (void)hipDeviceSynchronize();  // no launch still reads through them
    for (auto& m : ch_->dmaps) {
        if (ch_->vmem) ch_->vmem->Unmap(m.second.ptr);
        else (void)hipIpcCloseMemHandle(m.second.ptr);
    }
    ch_->dmaps.clear();
    ch_->direct_off = true;
    (void)hipGetLastError();
}

void Communicator::AllreduceRanges(void* buf, const uint64_t* off, const uint64_t* len, int dtype, int op,
                                   hipStream_t stream, const int8_t* fold) {
    KernelSet ks;
    if (!get_kernels(dtype, op, &ks))
        throw std::invalid_argument("rdc: unsupported (dtype, op) = (" + std::to_string(dtype) + ", " +
                                    std::to_string(op) + ")");
    if (n_ == 1) return;
    const size_t esz = rdc_dtype_size(dtype);
    uint64_t total = 0, sum = 0, first = ~0ull;
    for (int c = 0; c < n_; ++c) {
        if (off[c] % esz || len[c] % esz) throw std::invalid_argument("rdc: range not element-aligned");
        if (len[c]) {
            total = std::max<uint64_t>(total, off[c] + len[c]);
            first = std::min<uint64_t>(first, off[c]);
            sum += len[c];
        }
    }
    if (total == 0) return;
    hip_check(hipSetDevice(device_), "hipSetDevice");
    ChannelCall call(ch_.get(), stream);
    // the one-shot pushes all of [0, total): only for ranges that tile it
    // (disjoint chunk ranges starting at 0 with no gap); otherwise the mesh
    const bool contiguous = first == 0 && sum == total;
    int algo = contiguous ? PickAlgo(RDC_ALGO_AUTO, total) : PickAlgo(RDC_ALGO_AUTO);
    if (algo == RDC_ALGO_ONESHOT && !contiguous) algo = RDC_ALGO_MESH;
    bool identity = true;
    if (fold)
        for (int c = 0; c < n_; ++c) {
            if (fold[c] < 0 || fold[c] >= n_) throw std::invalid_argument("rdc: fold chunk out of range");
            identity = identity && fold[c] == c;
        }
    if (!identity && algo == RDC_ALGO_RING) algo = RDC_ALGO_MESH;  // the ring's order is its schedule
    LaunchRanges(ks, static_cast<char*>(buf), off, len, total, esz, algo, stream, nullptr, 0, identity ? nullptr : fold);
}

// The reference's small-buffer path (TryAllreduceTree: TryReduceTree to rank
// 0, TryBroadcast from it, communicator_collective.cc:14-78) as ONE hand-off:
// every rank pushes its buffer into every peer's one-shot slot, then folds the
// n inputs in the tree's order (PlanTreeProgram) — the root's bits, which the
// reference's broadcast gives every rank.  Buffers above half a slot go in
// pieces (the fold is per element).  Uses the one-shot's slot halves and gates.
void Communicator::LaunchTree(const KernelSet& ks, char* buf, uint64_t total, hipStream_t stream) {
    if (total == 0) return;
    const uint64_t cap = OneshotHalfBytes(layout());
    const int grid_cap = LaunchGrid(max_blocks(), ks.occupancy(RDC_KIND_TREE, n_));
    const uint64_t zero[RDC_MAX_RANKS] = {0};
    for (uint64_t off = 0; off < total; off += cap) {
        const uint64_t len = std::min<uint64_t>(cap, total - off);
        const Piece p = PlanOneshotRanges(n_, zero, zero, len, layout(), cfg_.tile_bytes, grid_cap);
        CollArgs a;
        FillArgsCommon(&a);
        a.kind = RDC_KIND_ONESHOT;  // same slot protocol: the next mesh / ring launch gates on it
        a.user = buf + off;
        a.tiles[0] = p.tiles[0];
        a.tile_bytes = p.tile_bytes;
        a.total_bytes = len;
        a.tree_len = tree_len_;
        for (int i = 0; i < tree_len_; ++i) {
            a.tree_dst[i] = (int8_t)tree_dst_[i];
            a.tree_src[i] = (int8_t)tree_src_[i];
        }
        if (off + len >= total) {
            a.notify = notify_;
            a.notify_val = notify_val_;
            notify_ = nullptr;
        }
        last_launch_[0] = last_launch_[1] = (uint64_t)p.nb_scatter;
        last_launch_[2] = last_launch_[3] = 0;
        last_launch_[4] = p.tile_bytes;
        last_launch_[5] = RDC_ALGO_TREE;
        ++seq_;
        log_launch(this, seq_, RDC_ALGO_TREE, len, p.nb_scatter, p.tile_bytes);
        hip_check(ks.tree(a, p.nb_scatter, stream), "launch tree allreduce");
    }
    trace_ = nullptr;
}

// The schedule over explicit chunk byte ranges of `buf` (chunk c = [off[c],
// off[c]+len[c]), folded in the ring order of c).
void Communicator::LaunchRanges(const KernelSet& ks, char* buf, const uint64_t* off, const uint64_t* len,
                                uint64_t total, size_t esz, int algo, hipStream_t stream, const PackUnit* units,
                                int nunits, const int8_t* fold) {
    algo = PickAlgo(algo, total);
    if (fold && algo == RDC_ALGO_RING) throw std::logic_error("rdc: a fold order needs an owner-computes schedule");
    const bool mesh_like = algo == RDC_ALGO_MESH || algo == RDC_ALGO_MESH_PULL;
    if (units && !mesh_like && algo != RDC_ALGO_RING)
        throw std::logic_error("rdc: unit-table launch needs the mesh or ring schedule");
    if (algo == RDC_ALGO_ONESHOT) {
        const Piece p = PlanOneshotRanges(n_, off, len, total, layout(), cfg_.tile_bytes,
                                          LaunchGrid(max_blocks(), ks.occupancy(RDC_KIND_ONESHOT, n_)));
        CollArgs a;
        FillArgsCommon(&a);
        a.kind = RDC_KIND_ONESHOT;
        a.user = buf;
        if (fold) memcpy(a.fold, fold, (size_t)n_);
        memcpy(a.off, p.off, sizeof(a.off));
        memcpy(a.len, p.len, sizeof(a.len));
        memcpy(a.tiles, p.tiles, sizeof(a.tiles));
        a.tile_bytes = p.tile_bytes;
        a.total_bytes = total;
        a.notify = notify_;
        a.notify_val = notify_val_;
        notify_ = nullptr;
        trace_ = nullptr;  // one-shot launches are not traced
        last_launch_[0] = (uint64_t)p.nb_scatter;
        last_launch_[1] = (uint64_t)p.nb_scatter;
        last_launch_[2] = last_launch_[3] = 0;
        last_launch_[4] = p.tile_bytes;
        last_launch_[5] = RDC_ALGO_ONESHOT;
        ++seq_;
        log_launch(this, seq_, RDC_ALGO_ONESHOT, total, p.nb_scatter, p.tile_bytes);
        hip_check(ks.oneshot(a, p.nb_scatter, stream), "launch one-shot allreduce");
        return;
    }
    const Shape sh = ShapeFor(total, algo);
    const int grid_cap =
        mesh_like ? LaunchGrid(sh.max_blocks > 0 ? sh.max_blocks : 2 * cus_min_, ks.occupancy(RDC_KIND_MESH, n_))
                  : LaunchGrid(sh.max_blocks > 0 ? sh.max_blocks : cus_min_, ks.occupancy(RDC_KIND_RING, n_));
    // the pull mode plans exactly as the push mode (same roles, same tiles)
    const std::vector<Piece> plan = PlanAllreduceRanges(n_, off, len, esz, layout(), mesh_like ? RDC_ALGO_MESH : algo,
                                                        sh.tile_bytes, grid_cap, sh.split);
    for (const Piece& p : plan) {
        CollArgs a;
        FillArgsCommon(&a);
        if (&p == &plan.back()) {
            a.notify = notify_;
            a.notify_val = notify_val_;
            notify_ = nullptr;
        }
        a.user = buf;
        if (fold) memcpy(a.fold, fold, (size_t)n_);
        memcpy(a.off, p.off, sizeof(a.off));
        memcpy(a.len, p.len, sizeof(a.len));
        memcpy(a.mis, p.mis, sizeof(a.mis));
        memcpy(a.tiles, p.tiles, sizeof(a.tiles));
        a.tile_bytes = p.tile_bytes;
        ++seq_;
        const int grid = algo == RDC_ALGO_RING ? p.nb_scatter : p.nb_scatter + p.nb_reduce + p.nb_gather;
        if (trace_ && trace_words_ >= 2 * (size_t)grid) a.trace = trace_;
        last_launch_[0] = (uint64_t)grid;
        last_launch_[1] = (uint64_t)p.nb_scatter;
        last_launch_[2] = (uint64_t)(algo == RDC_ALGO_RING ? 0 : p.nb_reduce);
        last_launch_[3] = (uint64_t)(algo == RDC_ALGO_RING ? 0 : p.nb_gather);
        last_launch_[4] = p.tile_bytes;
        last_launch_[5] = (uint64_t)algo;
        log_launch(this, seq_, algo, total, grid, p.tile_bytes);
        a.units = units;
        a.nunits = nunits;
        if (algo == RDC_ALGO_RING) {
            a.kind = RDC_KIND_RING;
            hip_check(ks.ring(a, grid, stream), "launch ring allreduce");
        } else {
            a.nb_scatter = p.nb_scatter;
            a.nb_reduce = p.nb_reduce;
            a.nb_gather = p.nb_gather;
            a.kind = RDC_KIND_MESH;
            a.pull = algo == RDC_ALGO_MESH_PULL ? 1 : 0;
            hip_check(ks.mesh(a, grid, stream), "launch mesh allreduce");
        }
    }
    trace_ = nullptr;  // one call only
}

// Staging image of the coalesced path, grown on demand (never shrinks).  The
// old image is released stream-ordered (hipFreeAsync): launches already queued
// may still read it, and a device-wide sync here would wait on kernels that
// wait for ranks a single-process group has not launched yet.  Callers size it
// once per call, before the call's first launch.
char* Communicator::Image(uint64_t bytes, hipStream_t stream) {
    if (bytes > image_bytes_) {
        if (image_) {
            hip_check(hipFreeAsync(image_, stream), "release coalesced image");
            image_ = nullptr;
            image_bytes_ = 0;
        }
        const uint64_t want = (bytes + ((uint64_t)1 << 20) - 1) & ~(((uint64_t)1 << 20) - 1);
        hip_check(hipMallocAsync(reinterpret_cast<void**>(&image_), want, stream), "allocate coalesced image");
        image_bytes_ = want;
    }
    return image_;
}

// Unit table of one fusion group, cached by (dtype size, buffers, counts) so
// repeated buckets (every training step) launch with no host->device traffic
// and can be captured in a hipGraph once warm.  Tables are stream-ordered
// allocations uploaded on `stream` (no host sync: in a single-process group
// a sync here would wait on kernels waiting for ranks not launched yet); an
// evicted table is freed stream-ordered after the launches that read it, and
// its host copy (the upload's source) is kept until an event says the stream
// passed that point.
const Communicator::PackEntry& Communicator::PackTable(void* const* bufs, const size_t* counts, int nbuf,
                                                         size_t esz, hipStream_t stream) {
    std::vector<uint64_t> key;
    key.reserve(2 + 2 * (size_t)nbuf);
    key.push_back(esz);
    key.push_back((uint64_t)nbuf);
    for (int b = 0; b < nbuf; ++b) {
        key.push_back((uint64_t)(uintptr_t)bufs[b]);
        key.push_back((uint64_t)counts[b]);
    }
    auto it = pack_cache_.find(key);
    if (it != pack_cache_.end()) {
        it->second.last_use = ++pack_tick_;
        return it->second;
    }
    if (pack_cache_.size() >= kPackCacheMax) {  // evict the least recently used group
        auto lru = pack_cache_.begin();
        for (auto j = pack_cache_.begin(); j != pack_cache_.end(); ++j)
            if (j->second.last_use < lru->second.last_use) lru = j;
        if (lru->second.dtable) hip_check(hipFreeAsync(lru->second.dtable, stream), "release pack table");
        hipEvent_t ev = nullptr;
        hip_check(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "event");
        hip_check(hipEventRecord(ev, stream), "record");
        retired_.emplace_back(ev, lru->second.host);
        pack_cache_.erase(lru);
    }
    for (size_t i = 0; i < retired_.size();) {  // host copies whose upload has surely finished
        if (hipEventQuery(retired_[i].first) == hipSuccess) {
            (void)hipEventDestroy(retired_[i].first);
            retired_[i] = retired_.back();
            retired_.pop_back();
        } else {
            (void)hipGetLastError();
            ++i;
        }
    }
    std::vector<uint64_t> cnt((size_t)nbuf);
    for (int b = 0; b < nbuf; ++b) cnt[(size_t)b] = counts[b];
    CoalescedPlan P = PlanCoalesced(n_, cnt.data(), nbuf, esz);
    for (PackUnit& u : P.units) {  // buffer index -> user address
        u.buf = (uint64_t)(uintptr_t)bufs[u.buf] + u.buf_off;
        u.buf_off = 0;
    }
    PackEntry e;
    memcpy(e.off, P.off, sizeof(e.off));
    memcpy(e.len, P.len, sizeof(e.len));
    e.total = P.total;
    e.nunits = (int)P.units.size();
    if (e.nunits > 0) {
        e.host = std::make_shared<std::vector<PackUnit>>(std::move(P.units));
        const size_t tb = e.host->size() * sizeof(PackUnit);
        hip_check(hipMallocAsync(reinterpret_cast<void**>(&e.dtable), tb, stream), "allocate pack table");
        hip_check(hipMemcpyAsync(e.dtable, e.host->data(), tb, hipMemcpyHostToDevice, stream), "upload pack table");
    }
    e.last_use = ++pack_tick_;
    return pack_cache_.emplace(std::move(key), e).first->second;
}

void Communicator::AllreduceCoalesced(void* const* bufs, const size_t* counts, int nbuf, int dtype, int op,
                                      hipStream_t stream, int algo) {
    KernelSet ks;
    if (!get_kernels(dtype, op, &ks))
        throw std::invalid_argument("rdc: unsupported (dtype, op) = (" + std::to_string(dtype) + ", " +
                                    std::to_string(op) + ")");
    if (nbuf < 0 || (nbuf > 0 && (!bufs || !counts))) throw std::invalid_argument("rdc: bad buffer list");
    const size_t esz = rdc_dtype_size(dtype);
    int misaligned = 0;
    for (int b = 0; b < nbuf; ++b) {
        if (counts[b] && bufs[b] == nullptr) throw std::invalid_argument("rdc: null buffer in coalesced allreduce");
        if ((uintptr_t)bufs[b] % esz) throw std::invalid_argument("rdc: buffer not aligned to its element size");
        misaligned += counts[b] != 0 && ((uintptr_t)bufs[b] & 15) != 0;
    }
    coalesced_misaligned_ = misaligned;
    if (n_ == 1 || nbuf == 0) return;
    hip_check(hipSetDevice(device_), "hipSetDevice");
    ChannelCall call(ch_.get(), stream);
    if (algo == RDC_ALGO_TREE || cfg_.ring_mincount >= esz) {
        // buffers of <= rdc_reduce_ring_mincount bytes take the tree's order
        // (TryAllreduce per buffer, communicator_collective.cc:6-13); the
        // tree fold is the same for every element, so they are packed into
        // the staging image together and folded in ONE tree launch
        std::vector<void*> sb, lb;
        std::vector<size_t> sc, lc;
        for (int b = 0; b < nbuf; ++b) {
            if (counts[b] == 0) continue;
            const bool small = algo == RDC_ALGO_TREE || (uint64_t)counts[b] * esz <= cfg_.ring_mincount;
            (small ? sb : lb).push_back(bufs[b]);
            (small ? sc : lc).push_back(counts[b]);
        }
        if (!sb.empty()) CoalescedTree(ks, sb.data(), sc.data(), (int)sb.size(), esz, stream);
        if (!sb.empty() && !lb.empty())
            AllreduceCoalesced(lb.data(), lc.data(), (int)lb.size(), dtype, op, stream, algo);
        if (!sb.empty()) return;
    }
    {
        // registered buffers (k_direct over the list): every buffer mapped
        // into every peer, one launch for the whole list, no scratch
        std::vector<char*> db;
        std::vector<uint64_t> dn;
        uint64_t total = 0;
        for (int b = 0; b < nbuf; ++b)
            if (counts[b]) {
                db.push_back(static_cast<char*>(bufs[b]));
                dn.push_back((uint64_t)counts[b] * esz);
                total += (uint64_t)counts[b] * esz;
            }
        if (!db.empty() && DirectEligible(algo, total, stream) &&
            AllreduceDirect(ks, db.data(), dn.data(), (int)db.size(), esz, stream))
            return;
        if (algo == RDC_ALGO_DIRECT) algo = RDC_ALGO_AUTO;  // not registrable here: the scratch schedules
    }
    std::vector<uint64_t> cnt((size_t)nbuf);
    for (int b = 0; b < nbuf; ++b) cnt[(size_t)b] = counts[b];
    // The unit-table mesh needs no staging memory, so its groups are large
    // (one launch sequence for the whole list: 1024 x 1 MiB on 2 ranks, 1.85 ms
    // as one group vs 2.25 ms as 256 MiB groups); whatever is too small for the
    // mesh, or runs another schedule, goes through the staging image in groups
    // of fuse_bytes.
    if (cfg_.coalesce_fused) {
        const std::vector<int> big = GroupCoalesced(cnt.data(), nbuf, esz, cfg_.fuse_bytes_direct);
        for (size_t g = 0; g + 1 < big.size(); ++g) {
            const int b0 = big[g], b1 = big[g + 1];
            uint64_t bytes = 0;
            int live = 0;
            for (int b = b0; b < b1; ++b) {
                bytes += (uint64_t)counts[b] * esz;
                live += counts[b] != 0;
            }
            // the schedule (and, via ShapeFor, the launch shape) a single
            // buffer of the list's size class gets — the automatic rule or
            // what Autotune measured — run over the unit table: mesh and ring
            // read and write the user buffers in place, no staging image
            const int pick = PickAlgo(algo, bytes);
            if (live >= 2 && (pick == RDC_ALGO_MESH || pick == RDC_ALGO_MESH_PULL || pick == RDC_ALGO_RING)) {
                const PackEntry& e = PackTable(bufs + b0, counts + b0, b1 - b0, esz, stream);
                LaunchRanges(ks, nullptr, e.off, e.len, e.total, esz, pick, stream, e.dtable, e.nunits);
            } else {
                CoalescedStaged(ks, bufs + b0, counts + b0, b1 - b0, dtype, op, esz, algo, stream);
            }
        }
        return;
    }
    CoalescedStaged(ks, bufs, counts, nbuf, dtype, op, esz, algo, stream);
}

// tree-order buffers: pack into the staging image, one tree launch over the
// packed bytes (padding between segments is folded too, never unpacked), unpack
void Communicator::CoalescedTree(const KernelSet& ks, void* const* bufs, const size_t* counts, int nbuf, size_t esz,
                                 hipStream_t stream) {
    if (nbuf == 1) {
        LaunchTree(ks, static_cast<char*>(bufs[0]), (uint64_t)counts[0] * esz, stream);
        return;
    }
    uint64_t need = (uint64_t)RDC_SLOT_ALIGN * (uint64_t)n_;
    for (int b = 0; b < nbuf; ++b) need += (uint64_t)n_ * 16 + ((uint64_t)counts[b] * esz + 15) / 16 * 16;
    char* img = Image(need, stream);
    const PackEntry& e = PackTable(bufs, counts, nbuf, esz, stream);
    const int grid = std::max(1, std::min(e.nunits, 2 * num_cus_));
    hip_check(launch_pack(e.dtable, e.nunits, img, 0, grid, stream), "launch pack");
    LaunchTree(ks, img, e.total, stream);
    hip_check(launch_pack(e.dtable, e.nunits, img, 1, grid, stream), "launch unpack");
}

// pack -> schedule on the staging image -> unpack, in groups of fuse_bytes
void Communicator::CoalescedStaged(const KernelSet& ks, void* const* bufs, const size_t* counts, int nbuf, int dtype,
                                   int op, size_t esz, int algo, hipStream_t stream) {
    std::vector<uint64_t> cnt((size_t)nbuf);
    for (int b = 0; b < nbuf; ++b) cnt[(size_t)b] = counts[b];
    const std::vector<int> bounds = GroupCoalesced(cnt.data(), nbuf, esz, cfg_.fuse_bytes);
    // the image is sized once, for the largest group, before the first launch
    // (an upper bound of PlanCoalesced's total: 16-B segments, 256-B chunks)
    uint64_t need = 0;
    for (size_t g = 0; g + 1 < bounds.size(); ++g) {
        uint64_t bytes = (uint64_t)RDC_SLOT_ALIGN * (uint64_t)n_;
        int live = 0;
        for (int b = bounds[g]; b < bounds[g + 1]; ++b)
            if (counts[b]) {
                ++live;
                bytes += (uint64_t)n_ * 16 + ((uint64_t)counts[b] * esz + 15) / 16 * 16;
            }
        if (live >= 2) need = std::max(need, bytes);
    }
    char* img = need ? Image(need, stream) : nullptr;
    for (size_t g = 0; g + 1 < bounds.size(); ++g) {
        const int b0 = bounds[g], b1 = bounds[g + 1];
        int live = 0, last = -1;
        for (int b = b0; b < b1; ++b)
            if (counts[b]) ++live, last = b;
        if (live == 0) continue;
        if (live == 1) {  // nothing to fuse: the buffer's own schedule, no staging
            Allreduce(bufs[last], counts[last], dtype, op, stream, algo);
            continue;
        }
        const PackEntry& e = PackTable(bufs + b0, counts + b0, b1 - b0, esz, stream);
        if (e.total > image_bytes_) throw std::logic_error("rdc: coalesced image smaller than its group");
        const int grid = std::max(1, std::min(e.nunits, 2 * num_cus_));
        hip_check(launch_pack(e.dtable, e.nunits, img, 0, grid, stream), "launch pack");
        LaunchRanges(ks, img, e.off, e.len, e.total, esz, algo, stream);
        hip_check(launch_pack(e.dtable, e.nunits, img, 1, grid, stream), "launch unpack");
    }
}

void Communicator::Broadcast(void* buf, size_t bytes, int root, hipStream_t stream) {
    if (root < 0 || root >= n_) throw std::invalid_argument("rdc: broadcast root out of range");
    if (n_ == 1 || bytes == 0) return;
    if (buf == nullptr) throw std::invalid_argument("rdc: null buffer");
    hip_check(hipSetDevice(device_), "hipSetDevice");
    ChannelCall call(ch_.get(), stream);
    for (const Piece& p :
         PlanBroadcast(bytes, layout(), cfg_.tile_bytes, LaunchGrid(max_blocks(), occupancy_bcast()))) {
        CollArgs a;
        FillArgsCommon(&a);
        a.user = static_cast<char*>(buf);
        a.root = root;
        a.kind = RDC_KIND_BCAST;
        a.off[0] = p.off[0];
        a.len[0] = p.len[0];
        a.mis[0] = p.mis[0];
        a.tiles[0] = p.tiles[0];
        a.tile_bytes = p.tile_bytes;
        // large pieces: root -> one forwarder per tile -> the other ranks (k_bcast)
        a.bcast_split = (n_ >= 3 && p.len[0] >= cfg_.bcast_split_bytes && p.tiles[0] >= n_ - 1) ? 1 : 0;
        ++seq_;
        log_launch(this, seq_, 100, p.len[0], p.nb_scatter, p.tile_bytes);
        hip_check(launch_bcast(a, p.nb_scatter, stream), "launch broadcast");
    }
}

void Communicator::Tune(int s16, int r16, int max_blocks, size_t tile_bytes) {
    if (s16 < 1 || r16 < 1 || s16 + r16 > 15 || max_blocks < 0)
        throw std::invalid_argument("rdc: mesh split wants s,r sixteenths with s+r <= 15 and a grid >= 0");
    if (tile_bytes % RDC_SLOT_ALIGN) throw std::invalid_argument("rdc: tile bytes must be a multiple of 256");
    cfg_.mesh_split.s16 = s16;
    cfg_.mesh_split.r16 = r16;
    cfg_.mesh_split.tpb = 0;
    cfg_.max_blocks = max_blocks;
    cfg_.tile_bytes = tile_bytes;
    tuned_.clear();  // an explicit shape replaces every autotuned one (and schedule)
    tuned_algo_.clear();
}

// Schedule and launch-shape autotuning for one buffer size (rdc_comm.h).
// Stage 0 times the ring, the mesh and (where it fits) the one-shot — all
// bit-identical; the rule picks among them on byte counts alone.  The defaults
// (4 / 8 / 4 split, 2 blocks per CU, ~2 tiles per reduce block) were tuned on
// one GPU where HBM is the bound; over xGMI the balance between the copy
// roles and the reduce role, the number of remote stores in flight and the
// tile granularity (the ring: 2(n-1) hand-offs per tile) can differ, so a
// node measures its own.  Coordinate descent, every stage
// agreed across ranks before the next one is built from its winner.
int Communicator::Autotune(size_t bytes, int dtype, int reps, hipStream_t stream, TuneCand* cand, int max_cand,
                           int* best) {
    if (!cand || !best || max_cand <= 0 || reps <= 0) throw std::invalid_argument("rdc: autotune needs reps and room");
    *best = -1;
    const size_t esz = rdc_dtype_size(dtype);
    if (esz == 0) throw std::invalid_argument("rdc: unsupported dtype");
    const size_t count = bytes / esz;
    const uint64_t total = (uint64_t)count * esz;
    if (n_ == 1 || count == 0 || total <= cfg_.ring_mincount || cfg_.algo != RDC_ALGO_AUTO) return 0;
    const int rule = AutoAlgo(n_, total, layout(), cfg_.oneshot_push_max);
    if (rule != RDC_ALGO_MESH && rule != RDC_ALGO_RING && rule != RDC_ALGO_ONESHOT) return 0;  // (never pull)
    const bool oneshot_fits = OneshotEligible(n_, total, layout(), (uint64_t)-1);
    hip_check(hipSetDevice(device_), "hipSetDevice");
    void* buf = nullptr;
    double* dms = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    const int cls = SizeClass(total);
    // state to restore on failure: the class's schedule and both shapes
    const std::map<int, Shape> saved_shapes = tuned_;
    const std::map<int, int> saved_algos = tuned_algo_;
    int nc = 0;
    // the direct schedule maps every rank's buffer into its peers: then the
    // buffer is the channel's own hipMalloc allocation (stream-ordered pool
    // memory has no IPC handle), kept for later autotunes — freed, it would
    // stay alive in the peers' mappings and its address could not be
    // exported again (AllreduceDirect)
    // (the same on every rank: not direct_off, which RdcCommDirectRelease
    // sets per rank — the self-check then fails on every rank alike)
    const bool direct_cand = ch_ && ch_->dreg;
    // the direct schedule is a candidate only where it passed its self-check
    const bool direct_ok = direct_cand && DirectSelfCheck(stream) == 1;
    auto release = [&] {
        if (buf && !direct_cand) (void)hipFreeAsync(buf, stream);
        if (dms) (void)hipFreeAsync(dms, stream);
        if (e0) (void)hipEventDestroy(e0);
        if (e1) (void)hipEventDestroy(e1);
        (void)hipStreamSynchronize(stream);
    };
    try {
        if (direct_cand) {
            TuneBuffer(count * esz);
            buf = ch_->tune_buf;
        } else {
            hip_check(hipMallocAsync(&buf, count * esz, stream), "autotune buffer");
        }
        // per-round times of one stage, agreed across ranks
        constexpr int kStageMax = 16;
        hip_check(hipMallocAsync(reinterpret_cast<void**>(&dms), sizeof(double) * kStageMax * kTuneRounds, stream),
                  "autotune times");
        // synthetic full-entropy values, reduced with Max so they stay that way:
        // the timing depends on the data (1 GiB ring, n = 2 on one GPU: zeros
        // 1.42 ms, random 1.51 ms under Max or Sum; tools/data_sensitivity.py,
        // profiles/r03/data_sensitivity_*), and Sum would drive them to inf
        DeviceFill(buf, count, dtype, 0x5EED7E57ull, rank_, stream);
        hip_check(hipEventCreate(&e0), "event");
        hip_check(hipEventCreate(&e1), "event");
        // a candidate = schedule + shape, installed where PickAlgo / ShapeFor
        // look them up for this size class
        auto set_shape = [&](const TuneCand& c) {
            Shape s;
            s.split.s16 = c.s16;
            s.split.r16 = c.r16;
            s.split.tpb = c.tpb;
            s.max_blocks = c.grid;
            tuned_[cls * 8 + c.algo] = s;
            tuned_algo_[cls] = c.algo;
        };
        auto add = [&](int algo, int s16, int r16, int grid, int tpb) {
            if (nc < max_cand) cand[nc++] = TuneCand{algo, s16, r16, grid, tpb, 0.0, 0.0, 0.0};
        };
        // one round of one candidate: ms per allreduce on this rank
        auto measure = [&](const TuneCand& c, bool warm) {
            set_shape(c);
            if (warm) Allreduce(buf, count, dtype, RDC_OP_MAX, stream, RDC_ALGO_AUTO);  // first-use work
            hip_check(hipEventRecord(e0, stream), "record");
            for (int i = 0; i < reps; ++i) Allreduce(buf, count, dtype, RDC_OP_MAX, stream, RDC_ALGO_AUTO);
            hip_check(hipEventRecord(e1, stream), "record");
            hip_check(hipEventSynchronize(e1), "sync");
            float ms = 0;
            hip_check(hipEventElapsedTime(&ms, e0, e1), "elapsed");
            return (double)ms / reps;
        };
        // a stage = candidates [lo, nc), cand[lo] the incumbent.  kTuneRounds
        // rounds, each timing every candidate once (round-robin: a slow spell
        // of the node hits the whole stage, not one candidate); the slowest
        // rank's time per (candidate, round) by a MAX allreduce — identical on
        // every rank — then each candidate's median over its rounds.  The
        // incumbent stays unless another median beats it by > kTuneMargin.
        auto stage = [&](int lo) {
            const int k = nc - lo;
            if (k <= 0) throw std::runtime_error("rdc: autotune ran out of candidate room");
            if (k > kStageMax) throw std::logic_error("rdc: autotune stage too large");
            double h[kStageMax * kTuneRounds];
            for (int r = 0; r < kTuneRounds; ++r)
                for (int i = 0; i < k; ++i) h[i * kTuneRounds + r] = measure(cand[lo + i], r == 0);
            const size_t m = (size_t)k * kTuneRounds;
            hip_check(hipMemcpyAsync(dms, h, sizeof(double) * m, hipMemcpyHostToDevice, stream), "H2D");
            Allreduce(dms, m, RDC_DT_FLOAT64, RDC_OP_MAX, stream, RDC_ALGO_AUTO);
            hip_check(hipMemcpyAsync(h, dms, sizeof(double) * m, hipMemcpyDeviceToHost, stream), "D2H");
            Check(stream);
            int fastest = lo;
            for (int i = 0; i < k; ++i) {
                double* t = h + (size_t)i * kTuneRounds;
                std::sort(t, t + kTuneRounds);
                TuneCand& c = cand[lo + i];
                c.ms = t[kTuneRounds / 2];
                c.ms_min = t[0];
                c.ms_max = t[kTuneRounds - 1];
                if (c.ms < cand[fastest].ms) fastest = lo + i;
            }
            return cand[fastest].ms < cand[lo].ms * (1.0 - kTuneMargin) ? fastest : lo;
        };
        const int cus = cus_min_;
        const int s0 = cfg_.mesh_split.s16, r0 = cfg_.mesh_split.r16;
        const int g0 = cfg_.max_blocks, t0 = cfg_.mesh_split.tpb;
        // stage 0: the schedule (all bit-identical) with the configured shape,
        // the automatic rule's choice first (the incumbent); the one-shot
        // (one hand-off, (n-1) x the egress) where it fits
        int lo = nc;
        add(rule, s0, r0, g0, t0);
        // (the mesh twice: pushed by remote stores and pulled by remote loads —
        // which direction the links serve faster is this node's answer)
        // (and the direct schedule on registered buffers where the ranks are
        // processes: no scratch, each buffer read and written once)
        for (int a : {RDC_ALGO_RING, RDC_ALGO_MESH, RDC_ALGO_MESH_PULL, RDC_ALGO_ONESHOT, RDC_ALGO_DIRECT})
            if (a != rule && (a != RDC_ALGO_ONESHOT || oneshot_fits) && (a != RDC_ALGO_DIRECT || direct_ok))
                add(a, s0, r0, g0, t0);
        int w = stage(lo);
        if (cand[w].algo == RDC_ALGO_ONESHOT) {
            // no roles or tiles to shape: the schedule is the result
        } else if (cand[w].algo == RDC_ALGO_DIRECT) {
            lo = nc;
            add(RDC_ALGO_DIRECT, s0, r0, cand[w].grid, cand[w].tpb);
            for (int bpc : {1, 2, 3, 4})  // (grid 0 = automatic = 2 per CU)
                if (bpc * cus != (cand[lo].grid ? cand[lo].grid : 2 * cus)) add(RDC_ALGO_DIRECT, s0, r0, bpc * cus, 0);
            w = stage(lo);
        } else if (cand[w].algo == RDC_ALGO_MESH || cand[w].algo == RDC_ALGO_MESH_PULL) {
            static const int kSplits[][2] = {{4, 8}, {3, 9}, {5, 8}, {6, 6}, {3, 10}, {2, 10}, {5, 7}};
            const int ma = cand[w].algo;
            lo = nc;
            add(ma, cand[w].s16, cand[w].r16, cand[w].grid, cand[w].tpb);
            for (const auto& sp : kSplits)
                if (sp[0] != cand[lo].s16 || sp[1] != cand[lo].r16) add(ma, sp[0], sp[1], cand[lo].grid, 0);
            w = stage(lo);
            const int s16 = cand[w].s16, r16 = cand[w].r16;
            lo = nc;
            add(ma, s16, r16, cand[w].grid, cand[w].tpb);
            for (int bpc : {1, 2, 3, 4})  // (grid 0 = automatic = 2 per CU)
                if (bpc * cus != (cand[lo].grid ? cand[lo].grid : 2 * cus)) add(ma, s16, r16, bpc * cus, 0);
            w = stage(lo);
            const int grid = cand[w].grid;
            lo = nc;
            add(ma, s16, r16, grid, cand[w].tpb);
            for (int tpb : {1, 2, 4, 8})  // (tpb 0 = the default, 2 per reduce block)
                if (tpb != (cand[lo].tpb ? cand[lo].tpb : 2)) add(ma, s16, r16, grid, tpb);
            w = stage(lo);
        } else {
            lo = nc;
            add(RDC_ALGO_RING, s0, r0, cand[w].grid, cand[w].tpb);
            for (int bpc : {1, 2})  // (grid 0 = automatic = 1 per CU)
                if (bpc * cus != (cand[lo].grid ? cand[lo].grid : cus)) add(RDC_ALGO_RING, s0, r0, bpc * cus, 0);
            w = stage(lo);
            const int grid = cand[w].grid;
            lo = nc;
            add(RDC_ALGO_RING, s0, r0, grid, cand[w].tpb);
            for (int tpb : {1, 4, 8, 16, 32})  // (tpb 0 = the default, 1 per block)
                if (tpb != (cand[lo].tpb ? cand[lo].tpb : 1)) add(RDC_ALGO_RING, s0, r0, grid, tpb);
            w = stage(lo);
        }
        set_shape(cand[w]);
        const std::string tf = tune_file();
        if (!tf.empty()) {
            // rank 0 records the winner; the closing collective keeps every
            // rank from reading the table (a new communicator) before it has
            if (rank_ == 0) {
                FILE* f = fopen(tf.c_str(), "a");
                if (!f) throw std::runtime_error("rdc: cannot append to RDC_TUNE_FILE " + tf);
                fprintf(f, "rdc-tune 2 %d %d %d %d %d %d %d %d %d %.4f\n", n_, cus_min_, share_max_, cls, cand[w].algo,
                        cand[w].s16, cand[w].r16, cand[w].grid, cand[w].tpb, cand[w].ms);
                fclose(f);
            }
            hip_check(hipMemsetAsync(dms, 0, sizeof(double), stream), "memset");
            Allreduce(dms, 1, RDC_DT_FLOAT64, RDC_OP_MAX, stream, RDC_ALGO_AUTO);
            Check(stream);
        }
        *best = w;
    } catch (...) {
        tuned_ = saved_shapes;
        tuned_algo_ = saved_algos;
        release();
        throw;
    }
    release();
    return nc;
}

uint64_t Communicator::LaunchCounter() {
    if (err_ == nullptr) return 0;  // world size 1: nothing is ever launched
    hip_check(hipSetDevice(device_), "hipSetDevice");
    hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    uint64_t v = 0;
    hip_check(hipMemcpy(&v, err_ + 32, sizeof(v), hipMemcpyDeviceToHost), "read launch counter");
    return v;
}

void Communicator::SetLaunchCounter(uint64_t value) {
    if (err_ == nullptr) return;
    if (value >> 55) throw std::invalid_argument("rdc: launch counter is 56 bits");
    hip_check(hipSetDevice(device_), "hipSetDevice");
    hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    hip_check(hipMemcpy(err_ + 32, &value, sizeof(value), hipMemcpyHostToDevice), "write launch counter");
}

double Communicator::Probe(int mode, size_t* bytes_io, int reps, hipStream_t stream) {
    size_t bytes = *bytes_io;
    if (n_ == 1) throw std::invalid_argument("rdc: probe needs 2 or more ranks");
    if (mode < 0 || mode > 3)
        throw std::invalid_argument("rdc: probe mode is 0 / 1 (push to next rank / all peers), 2 / 3 (pull)");
    bytes = std::min(bytes, region_bytes_ - (size_t)RDC_SLOT_ALIGN);  // source: an AG region
    if (mode == 1 || mode == 3) bytes = std::min(bytes, slot_bytes_ - (size_t)RDC_SLOT_ALIGN);
    bytes &= ~(size_t)255;
    if (bytes == 0 || reps <= 0) throw std::invalid_argument("rdc: probe needs bytes and reps");
    *bytes_io = bytes;
    hip_check(hipSetDevice(device_), "hipSetDevice");
    ChannelCall call(ch_.get(), stream);
    PushTargets t;
    memset(&t, 0, sizeof(t));
    int nd = 0;
    if (mode == 0) {
        t.dst[nd++] = peer_scratch_[(rank_ + 1) % n_];  // the whole RS region of the next rank
    } else if (mode == 1) {
        for (int k = 1; k < n_; ++k)  // my slot in every peer's RS region
            t.dst[nd++] = peer_scratch_[(rank_ + k) % n_] + (size_t)rank_ * slot_bytes_;
    } else if (mode == 2) {  // the next rank's AG region into my RS region (reads over one link)
        t.src[nd] = peer_ag_[(rank_ + 1) % n_];
        t.dst[nd++] = scratch_;
    } else {  // every peer's AG region into my RS slots (reads over all n-1 links)
        for (int k = 1; k < n_; ++k) {
            const int p = (rank_ + k) % n_;
            t.src[nd] = peer_ag_[p] + (size_t)rank_ * slot_bytes_;
            t.dst[nd++] = scratch_ + (size_t)p * slot_bytes_;
        }
    }
    hipEvent_t e0, e1;
    hip_check(hipEventCreate(&e0), "event");
    hip_check(hipEventCreate(&e1), "event");
    const int grid = 2 * num_cus_;
    hip_check(launch_push(t, nd, scratch_ag_, bytes, grid, stream), "launch push");  // warm
    hip_check(hipEventRecord(e0, stream), "record");
    for (int i = 0; i < reps; ++i) hip_check(launch_push(t, nd, scratch_ag_, bytes, grid, stream), "launch push");
    hip_check(hipEventRecord(e1, stream), "record");
    hip_check(hipEventSynchronize(e1), "sync");
    float ms = 0;
    hip_check(hipEventElapsedTime(&ms, e0, e1), "elapsed");
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return ms / reps;
}

void Communicator::Allgather(void* const* bufs, const uint64_t* sizes, hipStream_t stream) {
    if (n_ == 1) return;
    for (int c = 0; c < n_; ++c)
        if (sizes[c] && bufs[c] == nullptr) throw std::invalid_argument("rdc: null allgather buffer");
    hip_check(hipSetDevice(device_), "hipSetDevice");
    ChannelCall call(ch_.get(), stream);
    for (const Piece& p :
         PlanAllgather(n_, sizes, layout(), cfg_.tile_bytes, LaunchGrid(max_blocks(), occupancy_allgather()))) {
        CollArgs a;
        FillArgsCommon(&a);
        for (int c = 0; c < n_; ++c) a.cbuf[c] = static_cast<char*>(bufs[c]);
        memcpy(a.off, p.off, sizeof(a.off));
        memcpy(a.len, p.len, sizeof(a.len));
        memcpy(a.mis, p.mis, sizeof(a.mis));
        memcpy(a.tiles, p.tiles, sizeof(a.tiles));
        a.tile_bytes = p.tile_bytes;
        a.nb_scatter = p.nb_scatter;
        a.nb_gather = p.nb_gather;
        a.kind = RDC_KIND_ALLGATHER;
        ++seq_;
        log_launch(this, seq_, 101, 0, p.nb_scatter + p.nb_gather, p.tile_bytes);
        hip_check(launch_allgather(a, p.nb_scatter + p.nb_gather, stream), "launch allgather");
    }
}

bool Communicator::SmallHostAllreduce(void* host, size_t count, int dtype, int op) {
    const size_t esz = rdc_dtype_size(dtype);
    const uint64_t bytes = (uint64_t)count * esz;
    // a persistent block per rank: with many ranks on one GPU their queues
    // outnumber what the hardware scheduler keeps mapped and it time-slices
    // them (measured: 8 ranks on one MI355X, ~10 ms per call), so past
    // RDC_HOST_SERVICE_SHARE_MAX ranks per GPU (default 4) the launch path runs
    if (n_ == 1 || bytes == 0 || bytes > RDC_SVC_MAX_BYTES || !ch_ || !ch_->svc_region || !ch_->svc_enabled ||
        share_max_ > SmallService::ShareMax())
        return false;
    KernelSet ks;
    if (!get_kernels(dtype, op, &ks))
        throw std::invalid_argument("rdc: unsupported (dtype, op) = (" + std::to_string(dtype) + ", " +
                                    std::to_string(op) + ")");
    SmallService* svc;
    {
        std::lock_guard<std::mutex> lk(ch_->mu);
        if (!ch_->svc)
            ch_->svc.reset(new SmallService(rank_, n_, device_, ch_->peer_svc_region, err_ + 56,
                                            tree_len_, tree_dst_, tree_src_, cfg_.timeout_s, wall_khz_,
                                            ch_->svc_hx.get()));
        svc = ch_->svc.get();
    }
    // every rank allocates the same way on one machine image; a rank without
    // the uncached mailbox would leave its peers waiting, so that is an error
    if (!svc->Usable())
        throw std::runtime_error("rdc: small-allreduce service mailbox (hipHostMallocUncached) unavailable; "
                                 "set RDC_HOST_SERVICE=0 on every rank");
    svc->Allreduce(ks, dtype * 8 + op, static_cast<char*>(host), bytes, bytes <= cfg_.ring_mincount);
    return true;
}

void Communicator::Check(hipStream_t stream) {
    if (err_ == nullptr) return;  // world size 1: nothing was ever launched
    hip_check(hipSetDevice(device_), "hipSetDevice");
    hip_check(hipStreamSynchronize(stream), "stream sync");
    RaiseIfError(HostErrorWord());
}

// pinned words: err_host_[0] = error mirror, err_host_[4] = notify token
uint32_t Communicator::ArmNotify() {
    if (err_host_dev_ == nullptr) return 0;
    notify_ = err_host_dev_ + 4;
    {
        std::lock_guard<std::mutex> lk(ch_->mu);  // tokens unique across the channel's communicators
        notify_val_ = ++ch_->notify_token;
    }
    return notify_val_;
}

void Communicator::WaitNotify(uint32_t token, hipStream_t stream) {
    if (err_host_ == nullptr) return;
    if (notify_ != nullptr) {  // nothing was launched (empty buffer, world size 1, or an error before launch)
        notify_ = nullptr;
        return;
    }
    const uint32_t* w = err_host_ + 4;
    const auto t0 = std::chrono::steady_clock::now();
    const double limit = cfg_.timeout_s * 2 + 10;  // the kernels themselves give up after timeout_s
    uint32_t spins = 0;
    while (__atomic_load_n(w, __ATOMIC_ACQUIRE) != token) {
        __builtin_ia32_pause();
        if ((++spins & 4095) == 0 &&
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit) {
            hip_check(hipStreamSynchronize(stream), "stream sync");  // surfaces a launch failure
            if (__atomic_load_n(w, __ATOMIC_ACQUIRE) != token)
                throw std::runtime_error("rdc: collective did not complete on rank " + std::to_string(rank_));
        }
    }
    RaiseIfError(HostErrorWord());
}

uint32_t Communicator::HostErrorWord() const {
    if (err_host_ == nullptr) return RDC_KERR_NONE;
    return __atomic_load_n(err_host_, __ATOMIC_ACQUIRE);
}

void Communicator::RaiseIfError(uint32_t e) const {
    if (e != RDC_KERR_NONE) {
        static const char* names[] = {"none", "reduce-scatter wait timed out", "allgather wait timed out",
                                      "broadcast wait timed out", "ring step wait timed out",
                                      "allgather (buffers) wait timed out",
                                      "a peer's hand-off belongs to another communicator's collective",
                                      "blocks of one launch read different launch numbers (RDC_SEQ_CHECK)"};
        if (e == RDC_KERR_ORDER)
            throw std::runtime_error(std::string("rdc: device collective failed on rank ") + std::to_string(rank_) +
                                     ": " + names[e] +
                                     " (communicators sharing a scratch channel were used in different orders "
                                     "on different ranks; issue them in one order everywhere or set "
                                     "RDC_SHARE_SCRATCH=0; communicator is now unusable)");
        static const char* algos[] = {"auto", "ring", "mesh", "one-shot", "tree", "pull mesh"};
        const uint64_t al = last_launch_[5];
        // the first timed-out wait (rdc_device.h block_wait): which flag, the
        // launch number it waited for and the value it last saw
        std::string waited;
        uint32_t diag[8] = {0};
        if (err_ && hipMemcpy(diag, err_ + 64, sizeof(diag), hipMemcpyDeviceToHost) == hipSuccess && diag[0] == 1) {
            uint64_t d[3];
            memcpy(d, diag + 2, sizeof(d));
            const uint64_t at = (d[2] - (uint64_t)(uintptr_t)flags_) / (sizeof(uint64_t) * RDC_FLAG_STRIDE);
            const uint64_t mt = max_tiles_ ? max_tiles_ : 1;
            char buf[200];
            snprintf(buf, sizeof(buf), "; waited for launch %llu (tag %llu) at flag row %llu tile %llu, saw launch %llu "
                     "(tag %llu)", (unsigned long long)(d[0] >> 8), (unsigned long long)(d[0] & 255),
                     (unsigned long long)(at / mt), (unsigned long long)(at % mt), (unsigned long long)(d[1] >> 8),
                     (unsigned long long)(d[1] & 255));
            waited = buf;
            uint64_t pr[5] = {0};
            uint64_t host = 0;
            if (hipMemcpy(pr, err_ + 96, sizeof(pr), hipMemcpyDeviceToHost) == hipSuccess &&
                hipMemcpy(&host, reinterpret_cast<void*>((uintptr_t)d[2]), 8, hipMemcpyDeviceToHost) == hipSuccess) {
                snprintf(buf, sizeof(buf), " [after giving up, the flag read by the device: load %llu, atomic %llu, "
                         "after acquire %llu, nt %llu (XCC %llu); by the host: %llu]",
                         (unsigned long long)(pr[0] >> 8), (unsigned long long)(pr[1] >> 8),
                         (unsigned long long)(pr[2] >> 8), (unsigned long long)(pr[3] >> 8), (unsigned long long)pr[4],
                         (unsigned long long)(host >> 8));
                waited += buf;
            } else {
                (void)hipGetLastError();
            }
        } else {
            (void)hipGetLastError();
        }
        waited += "; flags kind " + std::to_string(region_kind(2)) + " (3 = HSA-uncached, MTYPE UC)";
        if (ch_ && ch_->tlog) {
            // RDC_LAUNCH_TIMES: this rank's last launches as {launch, block 0
            // start, latest block start, end} in ms of the GPU's wall clock
            // (100 MHz, one clock for every process on the GPU)
            uint64_t lg[64 * 4];
            if (hipMemcpy(lg, ch_->tlog, sizeof(lg), hipMemcpyDeviceToHost) == hipSuccess) {
                uint64_t top = 0;
                for (int i = 0; i < 64; ++i) top = std::max(top, lg[i * 4]);
                waited += "; launch log (launch: block0 start / last block start / end, ms):";
                for (uint64_t k = top > 5 ? top - 5 : 1; k <= top; ++k) {
                    const uint64_t* e = lg + (k & 63) * 4;
                    if (e[0] != k) continue;
                    char b[160];
                    snprintf(b, sizeof(b), " %llu: %.3f / %.3f / %s", (unsigned long long)k, (double)e[1] / 1e5,
                             (double)e[2] / 1e5, e[3] >= e[1] && e[3] ? std::to_string((double)e[3] / 1e5).c_str() : "-");
                    waited += b;
                }
            } else {
                (void)hipGetLastError();
            }
        }
        if (getenv("RDC_FLAG_DUMP") && atoi(getenv("RDC_FLAG_DUMP")) != 0) {
            // debug: the reduce-scatter rows as this rank sees them, in its own
            // flag array (row q: written by rank q) and, through its mappings,
            // its own row in every peer's array (what it wrote there), as
            // launch numbers, first 48 tiles; read by the host (hipMemcpy)
            const uint32_t T = std::min<uint32_t>(max_tiles_, 48);
            std::vector<uint64_t> w((size_t)T * RDC_FLAG_STRIDE);
            auto row = [&](const uint64_t* base, int r) {
                std::string out;
                if (hipMemcpy(w.data(), base + (uint64_t)r * max_tiles_ * RDC_FLAG_STRIDE, w.size() * 8,
                              hipMemcpyDeviceToHost) != hipSuccess) {
                    (void)hipGetLastError();
                    return std::string("?");
                }
                for (uint32_t t = 0; t < T; ++t) out += std::to_string(w[(size_t)t * RDC_FLAG_STRIDE] >> 8) + " ";
                return out;
            };
            std::string d = "; flag dump:";
            for (int q = 0; q < n_; ++q)
                if (q != rank_) d += " [own row " + std::to_string(q) + ": " + row(flags_, q) + "]";
            for (int p = 0; p < n_; ++p)
                if (p != rank_ && peer_flags_[p])
                    d += " [rank " + std::to_string(p) + "'s row " + std::to_string(rank_) + ": " +
                         row(peer_flags_[p], rank_) + "]";
            waited += d;
        }
        uint32_t vr[4] = {0};
        if (err_ && hipMemcpy(vr, err_ + 84, sizeof(vr), hipMemcpyDeviceToHost) == hipSuccess && vr[0] != 0) {
            uint64_t va;
            memcpy(&va, vr + 2, sizeof(va));
            char buf[160];
            snprintf(buf, sizeof(buf), "; RDC_VERIFY_PUBLISH: %u flag stores this rank never read back (last at %#llx)",
                     vr[0], (unsigned long long)va);
            waited += buf;
        }
        if (err_ && hipMemcpy(diag, err_ + 72, sizeof(diag), hipMemcpyDeviceToHost) == hipSuccess && diag[0] == 1) {
            uint64_t d[3];
            memcpy(d, diag + 2, sizeof(d));
            char buf[160];
            snprintf(buf, sizeof(buf), "; the launch's first block read launch number %llu, block %llu of %llu read %llu",
                     (unsigned long long)d[1], (unsigned long long)(d[2] & 0xffffffffu),
                     (unsigned long long)(d[2] >> 32), (unsigned long long)d[0]);
            waited += buf;
        } else {
            (void)hipGetLastError();
        }
        throw std::runtime_error(std::string("rdc: device collective failed on rank ") + std::to_string(rank_) +
                                 ": " + (e < 8 ? names[e] : "unknown") +
                                 " (a peer did not join the collective; communicator is now unusable; this "
                                 "rank's last launch: " + (al < 6 ? algos[al] : "?") + ", grid " +
                                 std::to_string(last_launch_[0]) + ", tile " + std::to_string(last_launch_[4]) +
                                 " B, launches issued " + std::to_string(seq_) + ", scratch kind " +
                                 std::to_string(alloc_kind_) + waited + ")");
    }
}

void DeviceReduce(void* dst, const void* src, size_t count, int dtype, int op, hipStream_t stream, int grid) {
    KernelSet ks;
    if (!get_kernels(dtype, op, &ks))
        throw std::invalid_argument("rdc: unsupported (dtype, op) = (" + std::to_string(dtype) + ", " +
                                    std::to_string(op) + ")");
    const size_t esz = rdc_dtype_size(dtype);
    if ((uintptr_t)dst % esz || (uintptr_t)src % esz)
        throw std::invalid_argument("rdc: buffer not aligned to its element size");
    if (count == 0) return;
    const uint64_t nbytes = (uint64_t)count * esz;
    if (grid <= 0) {  // one block per CU (k_reduce's 2 MiB sweep window), fewer for small buffers
        static int cu_cache[64] = {0};  // per device, filled on first use
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
        int cus = cu_cache[dev];
        if (cus <= 0) {
            if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
                cus = 256;
            cu_cache[dev] = cus;
        }
        const uint64_t want = (nbytes + 8191) / 8192;  // >= 8 KiB per block
        grid = (int)std::max<uint64_t>(1, std::min<uint64_t>(want, (uint64_t)cus));
    }
    hip_check(ks.reduce(static_cast<char*>(dst), static_cast<const char*>(src), nbytes, grid, stream),
              "launch reduce");
}

void DeviceFill(void* buf, size_t count, int dtype, uint64_t seed, int rank, hipStream_t stream) {
    if (rdc_dtype_size(dtype) == 0) throw std::invalid_argument("rdc: bad dtype");
    hip_check(launch_fill(buf, count, dtype, seed, rank, stream), "launch fill");
}

}  // namespace rdc_amd
