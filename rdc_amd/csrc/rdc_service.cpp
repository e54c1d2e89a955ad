// Small-allreduce service (see rdc_service.h).
#include "rdc_service.h"

#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <stdexcept>
#include <string>

namespace rdc_amd {

namespace {
void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string("rdc service: ") + what + ": " + hipGetErrorString(e));
}
double env_double(const char* name, double dflt) {
    const char* v = getenv(name);
    return v && *v ? atof(v) : dflt;
}
uint32_t host_load(const uint32_t* p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }
void host_store(uint32_t* p, uint32_t v) { __atomic_store_n(p, v, __ATOMIC_SEQ_CST); }
}  // namespace

bool SmallService::Enabled() {
    static const bool on = [] {
        const char* v = getenv("RDC_HOST_SERVICE");
        return !(v && *v && atoi(v) == 0);
    }();
    return on;
}

namespace {
// sfence: orders and drains stores to write-combining memory (the BAR mapping
// of a VRAM mailbox); on write-back memory it costs a few cycles
inline void wc_flush() { __builtin_ia32_sfence(); }

struct PoolPick {
    hsa_agent_t gpu{}, cpu{};
    uint32_t want_bdf = 0, want_domain = 0;
    bool have_gpu = false, have_cpu = false, have_pool = false;
    hsa_amd_memory_pool_t pool{};
};
hsa_status_t pick_agent(hsa_agent_t a, void* d) {
    PoolPick* p = static_cast<PoolPick*>(d);
    hsa_device_type_t t;
    if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
    if (t == HSA_DEVICE_TYPE_CPU && !p->have_cpu) {
        p->cpu = a;
        p->have_cpu = true;
    } else if (t == HSA_DEVICE_TYPE_GPU && !p->have_gpu) {
        uint32_t bdf = 0, dom = 0;
        hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf);
        hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom);
        if ((bdf >> 3) == (p->want_bdf >> 3) && dom == p->want_domain) {
            p->gpu = a;
            p->have_gpu = true;
        }
    }
    return HSA_STATUS_SUCCESS;
}
hsa_status_t pick_pool(hsa_amd_memory_pool_t pool, void* d) {
    PoolPick* p = static_cast<PoolPick*>(d);
    hsa_amd_segment_t seg;
    uint32_t flags = 0;
    if (hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg) != HSA_STATUS_SUCCESS)
        return HSA_STATUS_SUCCESS;
    hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
    if (seg == HSA_AMD_SEGMENT_GLOBAL && (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_FINE_GRAINED) && !p->have_pool) {
        p->pool = pool;
        p->have_pool = true;
    }
    return HSA_STATUS_SUCCESS;
}
}  // namespace

// Device memory of HIP device `device` that this process's CPU can write
// through the PCIe BAR (the GPU's fine-grained pool, uncached, CPU given
// access), or null when the runtime refuses any step (small BAR, no such
// pool).  The HSA runtime is the one HIP runs on.  Opt-in
// (RDC_HOST_SERVICE_VRAM=1): a bare word round trip through it is faster
// (1.8 vs 2.6 us, tools/mailbox_rtt.hip), but the service with its request
// side in VRAM measured slower on one shared GPU — n = 2, 4 B 10.4-11.4 vs
// 6.4-6.5 us, 4 KiB 11.8-12.8 vs 8.2 us, also without eager data reads
// (profiles/r05/svc_vram/).
void* AllocVramMailbox(int device, size_t bytes) {
    const char* e = getenv("RDC_HOST_SERVICE_VRAM");
    if (!(e && *e && atoi(e) != 0)) return nullptr;
    int bus = 0, dev = 0, dom = 0;
    if (hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, device) != hipSuccess ||
        hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, device) != hipSuccess ||
        hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, device) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    if (hsa_init() != HSA_STATUS_SUCCESS) return nullptr;  // reference-counted; HIP holds it already
    PoolPick p;
    p.want_bdf = ((uint32_t)bus << 8) | ((uint32_t)dev << 3);
    p.want_domain = (uint32_t)dom;
    void* mem = nullptr;
    if (hsa_iterate_agents(pick_agent, &p) == HSA_STATUS_SUCCESS && p.have_gpu && p.have_cpu &&
        hsa_amd_agent_iterate_memory_pools(p.gpu, pick_pool, &p) == HSA_STATUS_SUCCESS && p.have_pool &&
        hsa_amd_memory_pool_allocate(p.pool, bytes, HSA_AMD_MEMORY_POOL_UNCACHED_FLAG, &mem) == HSA_STATUS_SUCCESS) {
        hsa_agent_t both[2] = {p.gpu, p.cpu};
        if (hsa_amd_agents_allow_access(2, both, nullptr, mem) != HSA_STATUS_SUCCESS) {
            hsa_amd_memory_pool_free(mem);
            mem = nullptr;
        }
    }
    hsa_shut_down();  // drops this call's reference only
    return mem;
}

void FreeVramMailbox(void* p) {
    if (p) hsa_amd_memory_pool_free(p);
}

uint64_t SmallService::HxBytes() {
    // off by default: on one shared GPU it measured no faster at n = 2 and
    // slower at n = 4; opt in per node
    static const uint64_t v = (uint64_t)std::max(0.0, env_double("RDC_HOST_SERVICE_HX_BYTES", 0));
    return v;
}

SmallService::SmallService(int rank, int n, int device, char* const* region, uint32_t* derr,
                           int tree_len, const int* tree_dst, const int* tree_src, double timeout_s, int wall_khz,
                           char* hx)
    : rank_(rank), device_(device), timeout_s_(timeout_s), n_(n) {
    memset(&args_, 0, sizeof(args_));
    for (int p = 0; p < n; ++p) args_.region[p] = region[p];
    args_.derr = derr;
    args_.n = n;
    args_.rank = rank;
    args_.strict = getenv("RDC_STRICT_FENCES") && atoi(getenv("RDC_STRICT_FENCES")) != 0;
    args_.trace = getenv("RDC_SVC_TRACE") && atoi(getenv("RDC_SVC_TRACE")) != 0;
    // LL mode up to RDC_HOST_SERVICE_LL_BYTES (default and most RDC_SVC_LL_MAX);
    // RDC_HOST_SERVICE_EAGER_BYTES of LL input (default 4 KiB) read by every poll round
    ll_bytes_ = (uint64_t)std::min(env_double("RDC_HOST_SERVICE_LL_BYTES", RDC_SVC_LL_MAX), (double)RDC_SVC_LL_MAX);
    // LL result up to RDC_HOST_SERVICE_LL_OUT_BYTES (default 256: measured faster
    // than a drained result + `done` up to 256 B, slower from 1 KiB)
    ll_out_bytes_ = (uint64_t)std::min(env_double("RDC_HOST_SERVICE_LL_OUT_BYTES", 256), (double)RDC_SVC_LL_MAX);
    const int block = n <= 8 ? 512 : 256;  // Kernels::svc's block size
    args_.eager = std::max(0, std::min(block, (int)(env_double("RDC_HOST_SERVICE_EAGER_BYTES", 4096) / 16)));
    args_.pipe = env_double("RDC_HOST_SERVICE_PIPELINE", 0) != 0 ? 1 : 0;  // two poll rounds in flight (k_svc)
    args_.hx_eager =
        std::max(0, std::min(block, (int)(env_double("RDC_HOST_SERVICE_HX_EAGER_BYTES", 8192) / (16.0 * n))));
    wall_khz_ = wall_khz;
    args_.idle_ticks = (uint64_t)(env_double("RDC_HOST_SERVICE_IDLE_US", 1000.0) * (double)wall_khz / 1000.0);
    args_.timeout_ticks = (uint64_t)(timeout_s * (double)wall_khz * 1000.0);
    args_.tree_len = tree_len;
    for (int i = 0; i < tree_len; ++i) {
        args_.tree_dst[i] = (int8_t)tree_dst[i];
        args_.tree_src[i] = (int8_t)tree_src[i];
    }
    hip_check(hipSetDevice(device_), "hipSetDevice");
    // MTYPE UC host memory: the kernel's plain loads and stores of `data` bypass
    // every GPU cache (k_svc); without it there is no service
    if (hipHostMalloc(reinterpret_cast<void**>(&box_), sizeof(SvcBox), hipHostMallocUncached | hipHostMallocMapped) !=
        hipSuccess) {
        (void)hipGetLastError();
        box_ = nullptr;
        return;
    }
    memset(static_cast<void*>(box_), 0, sizeof(SvcBox));
    void* d = nullptr;
    hip_check(hipHostGetDevicePointer(&d, box_, 0), "mailbox device address");
    args_.box = static_cast<SvcBox*>(d);
    // the request side: VRAM the CPU writes through the BAR, else pinned host memory
    in_ = static_cast<SvcIn*>(AllocVramMailbox(device_, sizeof(SvcIn)));
    in_vram_ = in_ != nullptr;
    if (in_vram_) {
        args_.in = in_;  // one address for the CPU and the GPU
    } else {
        if (hipHostMalloc(reinterpret_cast<void**>(&in_), sizeof(SvcIn), hipHostMallocUncached | hipHostMallocMapped) !=
            hipSuccess) {
            (void)hipGetLastError();
            (void)hipHostFree(box_);
            box_ = nullptr;
            in_ = nullptr;
            return;
        }
        hip_check(hipHostGetDevicePointer(&d, in_, 0), "mailbox device address");
        args_.in = static_cast<SvcIn*>(d);
    }
    memset(static_cast<void*>(in_), 0, sizeof(SvcIn));
    wc_flush();
    if (hx && HxBytes() > 0) {
        void* hd = nullptr;
        hip_check(hipHostGetDevicePointer(&hd, hx, 0), "host exchange device address");
        hx_ = hx;
        args_.hx = static_cast<char*>(hd);
    }
    hip_check(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "service stream");
}

int SmallService::ShareMax() {
    static const int v = [] {
        const char* e = getenv("RDC_HOST_SERVICE_SHARE_MAX");
        return e && *e ? atoi(e) : 4;
    }();
    return v;
}

bool SmallService::Usable() const { return box_ != nullptr; }

SmallService::~SmallService() {
    if (args_.trace && traced_ > 0) {
        const double us = 1000.0 / (double)wall_khz_, k = 1.0 / (double)traced_;
        fprintf(stderr,
                "[rdc service] rank %d: %ld requests: host post->done %.2f us; device: seen->sent %.2f, "
                "sent->peers in %.2f, peers in->result out %.2f us; poll + done visibility %.2f us\n",
                rank_, traced_, tr_[0] * k, tr_[1] * k * us, tr_[2] * k * us, tr_[3] * k * us,
                (tr_[0] - (tr_[1] + tr_[2] + tr_[3]) * us) * k);
        fprintf(stderr, "[rdc service] rank %d host: LL encode + copy in %.2f us\n", rank_, ht_[0] * k);
    }
    try {
        Stop();
    } catch (...) {
    }
    if (stream_) (void)hipStreamDestroy(stream_);
    if (box_) (void)hipHostFree(box_);
    if (in_ && in_vram_) FreeVramMailbox(in_);
    else if (in_) (void)hipHostFree(in_);
}

// the kernel leaves at its next poll (or when a request it serves completes
// or times out); the stream sync makes sure it is gone
void SmallService::Stop() {
    if (!launched_) return;
    host_store(&in_->stop, 1);
    wc_flush();
    (void)hipSetDevice(device_);
    hip_check(hipStreamSynchronize(stream_), "stop service");
    host_store(&in_->stop, 0);
    wc_flush();
    launched_ = false;
}

void SmallService::EnsureRunning(const KernelSet& ks, int kind) {
    if (launched_) {
        uint32_t st = host_load(&box_->state);
        // leaving: it either saw our request (RUNNING again) or it is gone
        while (st == RDC_SVC_EXITING) {
            __builtin_ia32_pause();
            st = host_load(&box_->state);
        }
        if (st != RDC_SVC_EXITED) return;  // RUNNING (or not started yet: it will read `req` when it does)
        hip_check(hipStreamSynchronize(stream_), "service exit");
        launched_ = false;
    }
    host_store(&box_->state, RDC_SVC_NEVER);
    hip_check(hipSetDevice(device_), "hipSetDevice");
    hip_check(ks.svc(args_, stream_), "launch service");
    launched_ = true;
    kind_ = kind;
}

void SmallService::Allreduce(const KernelSet& ks, int kind, char* host, uint64_t bytes, bool tree) {
    std::lock_guard<std::mutex> lk(mu_);
    if (broken_) throw std::runtime_error("rdc service: unusable after an earlier failure");
    if (bytes > RDC_SVC_MAX_BYTES) throw std::logic_error("rdc service: buffer too large");
    if (launched_ && kind != kind_) Stop();  // another (dtype, op) needs another kernel
    const uint32_t r = ++req_;
    // host exchange: the same choice on every rank — it depends only on n,
    // bytes, the LL limit and the budget (a plan key), never on this
    // process's RDC_HOST_SERVICE_LL_BYTES (ranks that set that
    // differently would write to different places and wait on words never
    // written); it carries its input as LL words, so it forces LL input
    const bool hx = hx_ != nullptr && bytes <= RDC_SVC_LL_MAX && bytes * (uint64_t)n_ <= HxBytes();
    const bool ll = hx || bytes <= ll_bytes_;
    const uint64_t nwords = ((bytes + 15) / 16) * 4;  // whole 16-byte vectors of 4-byte LL payloads
    const auto t0 = std::chrono::steady_clock::now();
    if (ll) {
        // LL words {4 payload bytes, r}, built in host memory and copied in
        // whole; the device takes a word once it carries r, so the order in
        // which they land does not matter.  Planar (k_svc): payload word j of
        // vector j / 4 goes to plane (j / 2) % 2.
        const uint64_t tag = (uint64_t)r << 32, full = bytes / 4;
        auto put = [&](uint64_t j, uint32_t v) { stage_[ll_index(j)] = tag | v; };
        for (uint64_t j = 0; j < full; ++j) {
            uint32_t v;
            memcpy(&v, host + 4 * j, 4);
            put(j, v);
        }
        for (uint64_t j = full; j < nwords; ++j) {
            uint32_t v = 0;
            if (4 * j < bytes) memcpy(&v, host + 4 * j, bytes - 4 * j);
            put(j, v);
        }
        const uint64_t plane_words = nwords / 2;  // nwords is a multiple of 4
        // each 8-byte {payload, r} word must become visible whole: a word
        // whose r landed before its payload would be taken with stale data.
        // memcpy gives no such guarantee (rep movsb, overlapping vector
        // stores); aligned 8-byte atomic stores do.
        char* dst = hx ? hx_ + ((uint64_t)(r & 1u) * (uint64_t)n_ + (uint64_t)rank_) * RDC_SVC_HX_RANK_BYTES
                       : in_->data;
        uint64_t* p0 = reinterpret_cast<uint64_t*>(dst);
        uint64_t* p1 = reinterpret_cast<uint64_t*>(dst + RDC_SVC_LL_MAX);
        const uint64_t* s0 = stage_.data();
        const uint64_t* s1 = stage_.data() + RDC_SVC_LL_MAX / 8;
        for (uint64_t j = 0; j < plane_words; ++j) {
            __atomic_store_n(p0 + j, s0[j], __ATOMIC_RELAXED);
            __atomic_store_n(p1 + j, s1[j], __ATOMIC_RELAXED);
        }
        if (args_.trace) ht_[0] += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    } else {
        memcpy(in_->data, host, bytes);
    }
    // the header, after the data: x86 stores to write-back host memory stay in
    // order, stores to the write-combining BAR mapping of VRAM only behind an
    // sfence (wc_flush), which also sends them out at once
    wc_flush();
    const bool ll_out = bytes <= ll_out_bytes_;
    __atomic_store_n(&in_->hdr,
                     ((uint64_t)r << 32) | (tree ? 1ull << 31 : 0ull) | (ll ? 1ull << 30 : 0ull) |
                         (ll_out ? 1ull << 29 : 0ull) | (hx ? 1ull << 28 : 0ull) | bytes,
                     __ATOMIC_SEQ_CST);
    wc_flush();
    EnsureRunning(ks, kind);
    const double limit = timeout_s_ * 2 + 10;
    auto check = [&](uint32_t spins) {
        if ((spins & 4095) != 0) return;
        if (host_load(&box_->err) != 0) {
            broken_ = true;
            (void)hipStreamSynchronize(stream_);
            launched_ = false;
            throw std::runtime_error("rdc service: a peer did not join request " + std::to_string(r) + " on rank " +
                                     std::to_string(rank_) + " (communicator is now unusable)");
        }
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit) {
            broken_ = true;
            throw std::runtime_error("rdc service: request " + std::to_string(r) + " did not complete on rank " +
                                     std::to_string(rank_));
        }
    };
    uint32_t spins = 0;
    if (ll_out) {  // every result word as it lands, decoded in place
        const uint64_t* o = reinterpret_cast<const uint64_t*>(box_->out);
        const uint64_t used = (bytes + 3) / 4;
        // the last word first: spinning on word 0 while the device's 16-byte
        // stores land line by line pulls every line into this core's cache and
        // loses it again to the next store into it (each re-read a memory
        // round trip); once the last word is in, most lines are complete
        if (used > 64) {
            while ((uint32_t)(__atomic_load_n(o + ll_index(used - 1), __ATOMIC_ACQUIRE) >> 32) != r) {
                __builtin_ia32_pause();
                check(++spins);
            }
        }
        for (uint64_t j = 0; j < used; ++j) {
            uint64_t v;
            while ((uint32_t)((v = __atomic_load_n(o + ll_index(j), __ATOMIC_ACQUIRE)) >> 32) != r) {
                __builtin_ia32_pause();
                check(++spins);
            }
            const uint32_t x = (uint32_t)v;
            memcpy(host + 4 * j, &x, std::min<uint64_t>(4, bytes - 4 * j));
        }
    } else {
        while ((int32_t)(host_load(&box_->done) - r) < 0) {
            __builtin_ia32_pause();
            check(++spins);
        }
    }
    if (args_.trace) {
        while ((int32_t)(host_load(&box_->done) - r) < 0) __builtin_ia32_pause();  // the stamps
        const double host_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        const uint64_t* t = box_->trace;
        tr_[0] += host_us;
        tr_[1] += (double)(t[1] - t[0]);
        tr_[2] += (double)(t[2] - t[1]);
        tr_[3] += (double)(t[3] - t[2]);
        ++traced_;
    }
    if (host_load(&box_->err) != 0) {
        broken_ = true;
        (void)hipStreamSynchronize(stream_);
        launched_ = false;
        throw std::runtime_error("rdc service: a peer did not join request " + std::to_string(r) + " on rank " +
                                 std::to_string(rank_) + " (communicator is now unusable)");
    }
    if (!ll_out) memcpy(host, box_->out, bytes);
}

}  // namespace rdc_amd
