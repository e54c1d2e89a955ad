// Device communicator (see rdc_comm.h).
#include "rdc_comm.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <stdexcept>
#include <string>

#include "rdc_kernels.h"

namespace rdc_amd {

namespace {

void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string("rdc: ") + what + ": " + hipGetErrorString(e));
}

size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }
size_t round_down(size_t x, size_t a) { return x / a * a; }

// utils::Split (include/utils/utils.h:59-70) in 64-bit: same ranges for every
// count the reference's int version can represent.
void split(int64_t count, int n, int64_t* b, int64_t* e) {
    const int64_t k = count / n, m = count % n;
    for (int i = 0; i < n; ++i) {
        b[i] = (int64_t)i * k + std::min<int64_t>(i, m);
        e[i] = (int64_t)(i + 1) * k + std::min<int64_t>(i + 1, m);
    }
}

int env_alloc_kind() {
    const char* v = getenv("RDC_ALLOC");
    if (!v) return 0;
    if (!strcmp(v, "fine")) return 1;
    if (!strcmp(v, "coarse")) return 2;
    return 0;
}

// Cross-GPU scratch: uncached (MTYPE UC) so that remote stores landing in
// this HBM are never shadowed by a stale line in any XCD's L2, and remote
// readers never cache it either.  Falls back to fine-grained, then coarse.
void* alloc_shared(size_t bytes, int* kind) {
    void* p = nullptr;
    int want = env_alloc_kind();
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

void dbg(const char* fmt, int rank, const char* what) {
    static const bool on = getenv("RDC_DEBUG") != nullptr;
    if (on) {
        fprintf(stderr, fmt, rank, what);
        fflush(stderr);
    }
}

struct PeerInfo {
    hipIpcMemHandle_t scratch;
    hipIpcMemHandle_t ag;
    hipIpcMemHandle_t flags;
    int32_t device;
    int32_t pid;
    int32_t alloc_kind;
    int32_t pad;
    uint64_t slot_bytes;
    uint64_t max_tiles;
    char host[64];
};

}  // namespace

void Communicator::AllocLocal() {
    hip_check(hipSetDevice(device_), "hipSetDevice");
    // RS and AG regions are separate allocations, each below 2 GiB: on ROCm
    // 7.2 (dmabuf IPC) hipIpcOpenMemHandle of an allocation >= 2 GiB never
    // returns (measured: 2044 MiB opens, 2048 MiB hangs).
    size_t region = std::min<size_t>(cfg_.scratch_bytes / 2, kMaxRegionBytes);
    size_t slot = round_down(region / (size_t)n_, 4096);
    if (slot < 64 * 1024 || n_ == 1) slot = 64 * 1024;  // world size 1 never moves data
    slot_bytes_ = slot;
    region_bytes_ = slot * (size_t)n_;
    max_tiles_ = (uint32_t)(region_bytes_ / RDC_MIN_TILE + 2);
    flag_bytes_ = round_up((size_t)2 * n_ * max_tiles_ * sizeof(uint32_t), 4096);
    int k1 = 0, k2 = 0, k3 = 0;
    scratch_ = static_cast<char*>(alloc_shared(region_bytes_, &k1));
    scratch_ag_ = static_cast<char*>(alloc_shared(region_bytes_, &k3));
    flags_ = static_cast<uint32_t*>(alloc_shared(flag_bytes_, &k2));
    alloc_kind_ = std::max(std::max(k1, k2), k3);
    hip_check(hipMalloc(&err_, 64), "hipMalloc err");
    hip_check(hipMemset(flags_, 0, flag_bytes_), "memset flags");
    hip_check(hipMemset(err_, 0, 64), "memset err");
    hip_check(hipDeviceSynchronize(), "sync after alloc");
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device_) == hipSuccess && cus > 0)
        num_cus_ = cus;
    int wclk = 0;  // kHz
    if (hipDeviceGetAttribute(&wclk, hipDeviceAttributeWallClockRate, device_) != hipSuccess || wclk <= 0)
        wclk = 100000;
    wall_khz_ = wclk;
    peer_scratch_[rank_] = scratch_;
    peer_ag_[rank_] = scratch_ag_;
    peer_flags_[rank_] = flags_;
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
    dbg("[rdc %d] %s\n", c->rank_, "alloc");
    c->AllocLocal();
    dbg("[rdc %d] %s\n", c->rank_, "alloc done");

    PeerInfo mine;
    memset(&mine, 0, sizeof(mine));
    hip_check(hipIpcGetMemHandle(&mine.scratch, c->scratch_), "hipIpcGetMemHandle(scratch)");
    hip_check(hipIpcGetMemHandle(&mine.ag, c->scratch_ag_), "hipIpcGetMemHandle(ag)");
    hip_check(hipIpcGetMemHandle(&mine.flags, c->flags_), "hipIpcGetMemHandle(flags)");
    mine.device = device;
    mine.pid = (int32_t)getpid();
    mine.alloc_kind = c->alloc_kind_;
    mine.slot_bytes = c->slot_bytes_;
    mine.max_tiles = c->max_tiles_;
    gethostname(mine.host, sizeof(mine.host) - 1);
    std::vector<PeerInfo> all((size_t)c->n_);
    dbg("[rdc %d] %s\n", c->rank_, "handles exported");
    bs->allgather(&mine, sizeof(mine), all.data());
    dbg("[rdc %d] %s\n", c->rank_, "handles exchanged");
    for (int p = 0; p < c->n_; ++p) {
        if (all[(size_t)p].slot_bytes != mine.slot_bytes || all[(size_t)p].max_tiles != mine.max_tiles)
            throw std::runtime_error("rdc: ranks disagree on scratch size (set RDC_SCRATCH_BYTES identically)");
        if (strncmp(all[(size_t)p].host, mine.host, sizeof(mine.host)) != 0)
            throw std::runtime_error("rdc: xGMI path needs every rank on one node (rank " + std::to_string(p) +
                                     " is on " + all[(size_t)p].host + ")");
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
    for (int p = 0; p < c->n_; ++p) {
        if (p == c->rank_) continue;
        void* ps = nullptr;
        void* pa = nullptr;
        void* pf = nullptr;
        hip_check(hipIpcOpenMemHandle(&ps, all[(size_t)p].scratch, hipIpcMemLazyEnablePeerAccess),
                  "hipIpcOpenMemHandle(scratch)");
        hip_check(hipIpcOpenMemHandle(&pa, all[(size_t)p].ag, hipIpcMemLazyEnablePeerAccess),
                  "hipIpcOpenMemHandle(ag)");
        c->peer_ag_[p] = static_cast<char*>(pa);
        hip_check(hipIpcOpenMemHandle(&pf, all[(size_t)p].flags, hipIpcMemLazyEnablePeerAccess),
                  "hipIpcOpenMemHandle(flags)");
        c->peer_scratch_[p] = static_cast<char*>(ps);
        c->peer_flags_[p] = static_cast<uint32_t*>(pf);
    }
    dbg("[rdc %d] %s\n", c->rank_, "peers mapped");
    c->owns_peers_ipc_ = true;
    bs->barrier();
    return c.release();
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
        cs.push_back(std::move(c));
    }
    for (int i = 0; i < n; ++i) {
        for (int j = 0; j < n; ++j) {
            cs[(size_t)i]->peer_scratch_[j] = cs[(size_t)j]->scratch_;
            cs[(size_t)i]->peer_ag_[j] = cs[(size_t)j]->scratch_ag_;
            cs[(size_t)i]->peer_flags_[j] = cs[(size_t)j]->flags_;
            if (devices[i] != devices[j]) {
                int can = 0;
                (void)hipSetDevice(devices[i]);
                if (hipDeviceCanAccessPeer(&can, devices[i], devices[j]) == hipSuccess && can)
                    (void)hipDeviceEnablePeerAccess(devices[j], 0);
                (void)hipGetLastError();
            }
        }
    }
    out->clear();
    for (auto& c : cs) out->push_back(c.release());
}

Communicator::~Communicator() {
    (void)hipSetDevice(device_);
    (void)hipDeviceSynchronize();
    if (owns_peers_ipc_ && bs_) {
        try {
            bs_->barrier();  // nobody still pushes into my scratch
        } catch (...) {
        }
        for (int p = 0; p < n_; ++p)
            if (p != rank_) {
                if (peer_scratch_[p]) (void)hipIpcCloseMemHandle(peer_scratch_[p]);
                if (peer_ag_[p]) (void)hipIpcCloseMemHandle(peer_ag_[p]);
                if (peer_flags_[p]) (void)hipIpcCloseMemHandle(peer_flags_[p]);
            }
        try {
            bs_->barrier();  // every importer closed its mapping
        } catch (...) {
        }
    }
    if (scratch_) (void)hipFree(scratch_);
    if (scratch_ag_) (void)hipFree(scratch_ag_);
    if (flags_) (void)hipFree(flags_);
    if (err_) (void)hipFree(err_);
}

int Communicator::PickAlgo(int algo) const {
    if (algo == RDC_ALGO_AUTO) algo = cfg_.algo;
    if (algo == RDC_ALGO_AUTO) algo = RDC_ALGO_MESH;
    return algo;
}

void Communicator::FillArgsCommon(CollArgs* a) const {
    memset(a, 0, sizeof(*a));
    a->n = n_;
    a->rank = rank_;
    a->slot_bytes = slot_bytes_;
    a->max_tiles = max_tiles_;
    for (int p = 0; p < n_; ++p) {
        a->rs[p] = peer_scratch_[p];
        a->ag[p] = peer_ag_[p];
        a->flags[p] = peer_flags_[p];
    }
    a->err = err_;
    a->timeout_ticks = (uint64_t)(cfg_.timeout_s * (double)wall_khz_ * 1000.0);
}

void Communicator::Plan(size_t chunk_bytes, int algo, size_t* tile, int* nb_s, int* nb_r, int* nb_g) const {
    algo = PickAlgo(algo);
    size_t t = cfg_.tile_bytes;
    if (t == 0) {
        // mesh: ~64 tiles per chunk keeps every reduce block busy; ring: each
        // block walks 2(n-1) hand-offs per tile, so aim for one tile per block.
        const size_t want = algo == RDC_ALGO_RING ? chunk_bytes / (size_t)num_cus_ : chunk_bytes / 64;
        t = std::min<size_t>(std::max<size_t>(want, RDC_MIN_TILE), (size_t)1 << 20);
    }
    t = std::max<size_t>(round_up(t, RDC_SLOT_ALIGN), RDC_MIN_TILE);
    *tile = t;
    const int T = (int)((chunk_bytes + t - 1) / t);
    const int G = cfg_.max_blocks > 0 ? cfg_.max_blocks : num_cus_;
    if (algo == RDC_ALGO_RING) {
        *nb_s = std::max(1, std::min(T, G));
        *nb_r = *nb_g = 0;
        return;
    }
    const int items_s = (n_ - 1) * T;
    int s = std::max(1, std::min(items_s, G * 3 / 8));
    int r = std::max(1, std::min(T, G * 3 / 8));
    int g = std::max(1, std::min(items_s, G - s - r));
    *nb_s = s;
    *nb_r = r;
    *nb_g = g;
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
    algo = PickAlgo(algo);
    hip_check(hipSetDevice(device_), "hipSetDevice");
    int64_t cb[RDC_MAX_RANKS], ce[RDC_MAX_RANKS];
    split((int64_t)count, n_, cb, ce);
    const int64_t maxlen = ce[0] - cb[0];  // first chunk is never shorter
    const int64_t pe = (int64_t)(round_down(slot_bytes_ - RDC_SLOT_ALIGN, RDC_SLOT_ALIGN) / esz);
    const int64_t npieces = (maxlen + pe - 1) / pe;
    char* user = static_cast<char*>(buf);
    for (int64_t k = 0; k < npieces; ++k) {
        CollArgs a;
        FillArgsCommon(&a);
        a.user = user;
        size_t chunk_max = 0;
        for (int c = 0; c < n_; ++c) {
            const int64_t b0 = cb[c] + k * pe;
            const int64_t e0 = std::min(ce[c], b0 + pe);
            if (e0 > b0) {
                a.off[c] = (uint64_t)b0 * esz;
                a.len[c] = (uint64_t)(e0 - b0) * esz;
            } else {
                a.off[c] = 0;
                a.len[c] = 0;
            }
            // buffer-relative: every rank places chunk c's bytes identically
            a.mis[c] = (uint32_t)(a.off[c] % 16);
            chunk_max = std::max<size_t>(chunk_max, a.len[c]);
        }
        size_t tile;
        int nb_s, nb_r, nb_g;
        Plan(chunk_max, algo, &tile, &nb_s, &nb_r, &nb_g);
        a.tile_bytes = tile;
        for (int c = 0; c < n_; ++c) a.tiles[c] = (int)((a.len[c] + tile - 1) / tile);
        a.seq = ++seq_;
        if (algo == RDC_ALGO_RING) {
            hip_check(ks.ring(a, nb_s, stream), "launch ring allreduce");
        } else {
            a.nb_scatter = nb_s;
            a.nb_reduce = nb_r;
            a.nb_gather = nb_g;
            hip_check(ks.mesh(a, nb_s + nb_r + nb_g, stream), "launch mesh allreduce");
        }
    }
}

void Communicator::Broadcast(void* buf, size_t bytes, int root, hipStream_t stream) {
    if (root < 0 || root >= n_) throw std::invalid_argument("rdc: broadcast root out of range");
    if (n_ == 1 || bytes == 0) return;
    if (buf == nullptr) throw std::invalid_argument("rdc: null buffer");
    hip_check(hipSetDevice(device_), "hipSetDevice");
    const size_t cap = round_down(region_bytes_ - RDC_SLOT_ALIGN, RDC_SLOT_ALIGN);
    char* user = static_cast<char*>(buf);
    const int G = cfg_.max_blocks > 0 ? cfg_.max_blocks : num_cus_;
    for (size_t off = 0; off < bytes; off += cap) {
        CollArgs a;
        FillArgsCommon(&a);
        a.user = user;
        a.root = root;
        a.off[0] = off;
        a.len[0] = std::min(cap, bytes - off);
        a.mis[0] = (uint32_t)(off % 16);
        size_t tile = cfg_.tile_bytes ? cfg_.tile_bytes
                                      : std::min<size_t>(std::max<size_t>(a.len[0] / (size_t)G, RDC_MIN_TILE),
                                                         (size_t)1 << 20);
        tile = std::max<size_t>(round_up(tile, RDC_SLOT_ALIGN), RDC_MIN_TILE);
        a.tile_bytes = tile;
        a.tiles[0] = (int)((a.len[0] + tile - 1) / tile);
        a.seq = ++seq_;
        hip_check(launch_bcast(a, std::max(1, std::min(a.tiles[0], G)), stream), "launch broadcast");
    }
}

void Communicator::Check(hipStream_t stream) {
    hip_check(hipSetDevice(device_), "hipSetDevice");
    hip_check(hipStreamSynchronize(stream), "stream sync");
    uint32_t e = 0;
    hip_check(hipMemcpy(&e, err_, sizeof(e), hipMemcpyDeviceToHost), "read error word");
    if (e != RDC_KERR_NONE) {
        static const char* names[] = {"none", "reduce-scatter wait timed out", "allgather wait timed out",
                                      "broadcast wait timed out", "ring step wait timed out"};
        throw std::runtime_error(std::string("rdc: device collective failed on rank ") + std::to_string(rank_) +
                                 ": " + (e < 5 ? names[e] : "unknown") +
                                 " (a peer did not join the collective; communicator is now unusable)");
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
    if (grid <= 0) {  // >= 4 KiB per block, at most 4096 blocks (16 per CU)
        const uint64_t want = (nbytes + 4095) / 4096;
        grid = (int)std::max<uint64_t>(1, std::min<uint64_t>(want, 4096));
    }
    hip_check(ks.reduce(static_cast<char*>(dst), static_cast<const char*>(src), nbytes, grid, stream),
              "launch reduce");
}

void DeviceFill(void* buf, size_t count, int dtype, uint64_t seed, int rank, hipStream_t stream) {
    if (rdc_dtype_size(dtype) == 0) throw std::invalid_argument("rdc: bad dtype");
    hip_check(launch_fill(buf, count, dtype, seed, rank, stream), "launch fill");
}

}  // namespace rdc_amd
