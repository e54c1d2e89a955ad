// Small-allreduce service (see rdc_service.h).
#include "rdc_service.h"

#include <stdlib.h>
#include <string.h>

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

SmallService::SmallService(int rank, int n, int device, char* const* region, uint32_t* const* sflags, uint32_t* derr,
                           int tree_len, const int* tree_dst, const int* tree_src, double timeout_s, int wall_khz)
    : rank_(rank), device_(device), timeout_s_(timeout_s) {
    memset(&args_, 0, sizeof(args_));
    for (int p = 0; p < n; ++p) {
        args_.region[p] = region[p];
        args_.sflags[p] = sflags[p];
    }
    args_.derr = derr;
    args_.n = n;
    args_.rank = rank;
    args_.strict = getenv("RDC_STRICT_FENCES") && atoi(getenv("RDC_STRICT_FENCES")) != 0;
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
    hip_check(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "service stream");
}

bool SmallService::Usable() const { return box_ != nullptr; }

SmallService::~SmallService() {
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
    hip_check(ks.svc(args_, stream_), "launch service");
    launched_ = true;
    kind_ = kind;
}

void SmallService::Allreduce(const KernelSet& ks, int kind, char* host, uint64_t bytes, bool tree) {
    std::lock_guard<std::mutex> lk(mu_);
    if (broken_) throw std::runtime_error("rdc service: unusable after an earlier failure");
    if (bytes > RDC_SVC_MAX_BYTES) throw std::logic_error("rdc service: buffer too large");
    hip_check(hipSetDevice(device_), "hipSetDevice");
    if (launched_ && kind != kind_) Stop();  // another (dtype, op) needs another kernel
    memcpy(box_->data, host, bytes);
    const uint32_t r = ++req_;
    // the whole request in one word, stored after the data (x86 stores stay in order)
    __atomic_store_n(&box_->req, ((uint64_t)r << 32) | (tree ? 1ull << 31 : 0ull) | bytes, __ATOMIC_SEQ_CST);
    EnsureRunning(ks, kind);
    const auto t0 = std::chrono::steady_clock::now();
    const double limit = timeout_s_ * 2 + 10;
    for (uint32_t spins = 0; (int32_t)(host_load(&box_->done) - r) < 0;) {
        __builtin_ia32_pause();
        if ((++spins & 4095) == 0 &&
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit) {
            broken_ = true;
            throw std::runtime_error("rdc service: request " + std::to_string(r) + " did not complete on rank " +
                                     std::to_string(rank_));
        }
    }
    if (host_load(&box_->err) != 0) {
        broken_ = true;
        (void)hipStreamSynchronize(stream_);
        launched_ = false;
        throw std::runtime_error("rdc service: a peer did not join request " + std::to_string(r) + " on rank " +
                                 std::to_string(rank_) + " (communicator is now unusable)");
    }
    memcpy(host, box_->data, bytes);
}

}  // namespace rdc_amd
