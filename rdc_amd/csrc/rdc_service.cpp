// Small-allreduce service (see rdc_service.h).
#include "rdc_service.h"

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
}

// the kernel leaves at its next poll (or when a request it serves completes
// or times out); the stream sync makes sure it is gone
void SmallService::Stop() {
    if (!launched_) return;
    host_store(&box_->stop, 1);
    (void)hipSetDevice(device_);
    hip_check(hipStreamSynchronize(stream_), "stop service");
    host_store(&box_->stop, 0);
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
                       : box_->data;
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
        memcpy(box_->data, host, bytes);
    }
    // the header, after the data (x86 stores stay in order)
    const bool ll_out = bytes <= ll_out_bytes_;
    __atomic_store_n(&box_->hdr,
                     ((uint64_t)r << 32) | (tree ? 1ull << 31 : 0ull) | (ll ? 1ull << 30 : 0ull) |
                         (ll_out ? 1ull << 29 : 0ull) | (hx ? 1ull << 28 : 0ull) | bytes,
                     __ATOMIC_SEQ_CST);
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
