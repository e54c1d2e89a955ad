// Pipelined host-resident allreduce (see rdc_host.h).
#include "rdc_host.h"

#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <stdexcept>
#include <string>

#include "rdc_plan.h"

namespace rdc_amd {

namespace {
void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string("rdc host path: ") + what + ": " + hipGetErrorString(e));
}
int env_int(const char* name, int dflt) {
    const char* v = getenv(name);
    return v && *v ? atoi(v) : dflt;
}
constexpr size_t kPieceTarget = (size_t)16 << 20;  // bytes of all chunks' slices per piece
constexpr size_t kParallelMin = (size_t)1 << 20;   // below this a copy runs on the caller alone
}  // namespace

// ---------------------------------------------------------------- CopyPool --
CopyPool::CopyPool(int threads) {
    for (int i = 0; i < threads; ++i) th_.emplace_back([this] { Loop(); });
}

CopyPool::~CopyPool() {
    {
        std::lock_guard<std::mutex> lk(mu_);
        stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
}

void CopyPool::Loop() {
    uint64_t seen = 0;
    for (;;) {
        const std::function<void(int)>* job;
        {
            std::unique_lock<std::mutex> lk(mu_);
            cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
            if (stop_) return;
            seen = gen_;
            job = job_;
        }
        for (;;) {
            int i;
            {
                std::lock_guard<std::mutex> lk(mu_);
                if (next_ >= total_) break;
                i = next_++;
            }
            (*job)(i);
            std::lock_guard<std::mutex> lk(mu_);
            if (++finished_ == total_) done_cv_.notify_all();
        }
    }
}

void CopyPool::Run(int n, const std::function<void(int)>& f) {
    if (n <= 0) return;
    if (th_.empty() || n == 1) {
        for (int i = 0; i < n; ++i) f(i);
        return;
    }
    {
        std::lock_guard<std::mutex> lk(mu_);
        job_ = &f;
        next_ = 0;
        total_ = n;
        finished_ = 0;
        ++gen_;
    }
    cv_.notify_all();
    for (;;) {  // the caller works too
        int i;
        {
            std::lock_guard<std::mutex> lk(mu_);
            if (next_ >= total_) break;
            i = next_++;
        }
        f(i);
        std::lock_guard<std::mutex> lk(mu_);
        if (++finished_ == total_) done_cv_.notify_all();
    }
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return finished_ == total_; });
    job_ = nullptr;
}

// ---------------------------------------------------------------- HostPath --
HostPath::HostPath(int device) : device_(device), pool_(std::max(0, env_int("RDC_HOST_THREADS", 4) - 1)) {
    hip_check(hipSetDevice(device_), "hipSetDevice");
    hip_check(hipStreamCreateWithFlags(&h2d_, hipStreamNonBlocking), "stream");
    hip_check(hipStreamCreateWithFlags(&d2h_, hipStreamNonBlocking), "stream");
    for (int i = 0; i < kSlots; ++i) {
        hip_check(hipEventCreateWithFlags(&in_done_[i], hipEventDisableTiming), "event");
        hip_check(hipEventCreateWithFlags(&ar_done_[i], hipEventDisableTiming), "event");
        hip_check(hipEventCreateWithFlags(&out_done_[i], hipEventDisableTiming), "event");
    }
}

HostPath::~HostPath() {
    (void)hipSetDevice(device_);
    (void)hipDeviceSynchronize();
    for (int i = 0; i < kSlots; ++i) {
        if (pin_in_[i]) (void)hipHostFree(pin_in_[i]);
        if (pin_out_[i]) (void)hipHostFree(pin_out_[i]);
        (void)hipEventDestroy(in_done_[i]);
        (void)hipEventDestroy(ar_done_[i]);
        (void)hipEventDestroy(out_done_[i]);
    }
    if (dev_) (void)hipFree(dev_);
    if (h2d_) (void)hipStreamDestroy(h2d_);
    if (d2h_) (void)hipStreamDestroy(d2h_);
}

void HostPath::Reserve(size_t piece_bytes, size_t total_bytes) {
    if (piece_bytes > slot_bytes_) {
        hip_check(hipDeviceSynchronize(), "sync before regrow");
        for (int i = 0; i < kSlots; ++i) {
            if (pin_in_[i]) (void)hipHostFree(pin_in_[i]);
            if (pin_out_[i]) (void)hipHostFree(pin_out_[i]);
            pin_in_[i] = pin_out_[i] = nullptr;
        }
        slot_bytes_ = 0;
        for (int i = 0; i < kSlots; ++i) {
            hip_check(hipHostMalloc(reinterpret_cast<void**>(&pin_in_[i]), piece_bytes, hipHostMallocDefault),
                      "hipHostMalloc");
            hip_check(hipHostMalloc(reinterpret_cast<void**>(&pin_out_[i]), piece_bytes, hipHostMallocDefault),
                      "hipHostMalloc");
        }
        slot_bytes_ = piece_bytes;
    }
    if (total_bytes > dev_bytes_) {
        if (dev_) {
            hip_check(hipDeviceSynchronize(), "sync before regrow");
            (void)hipFree(dev_);
            dev_ = nullptr;
            dev_bytes_ = 0;
        }
        hip_check(hipMalloc(reinterpret_cast<void**>(&dev_), total_bytes), "hipMalloc host-path image");
        dev_bytes_ = total_bytes;
    }
}

void HostPath::Copy(char* dst, const char* src, size_t bytes) {
    if (bytes < kParallelMin) {
        memcpy(dst, src, bytes);
        return;
    }
    const int parts = (int)std::min<size_t>(16, bytes / (kParallelMin / 2));
    const size_t per = (bytes / (size_t)parts + 4095) & ~(size_t)4095;
    pool_.Run(parts, [&](int i) {
        const size_t lo = (size_t)i * per;
        if (lo >= bytes) return;
        memcpy(dst + lo, src + lo, std::min(per, bytes - lo));
    });
}

void HostPath::Allreduce(Communicator* c, void* host, size_t count, int dtype, int op, hipStream_t comm_stream) {
    const int n = c->size();
    if (n == 1 || count == 0) return;
    const size_t esz = rdc_dtype_size(dtype);
    const size_t S = count * esz;
    char* h = static_cast<char*>(host);
    hip_check(hipSetDevice(device_), "hipSetDevice");

    int64_t cb[RDC_MAX_RANKS], ce[RDC_MAX_RANKS];
    SplitRanges((int64_t)count, n, cb, ce);
    const uint64_t maxlen = (uint64_t)(ce[0] - cb[0]) * esz;  // the first chunk is never shorter
    // slice length per chunk and piece: a multiple of 4 KiB (hence of esz)
    const uint64_t K0 = std::max<uint64_t>(1, (S + kPieceTarget - 1) / kPieceTarget);
    const uint64_t sl = std::max<uint64_t>(4096, ((maxlen + K0 - 1) / K0 + 4095) & ~(uint64_t)4095);
    const int K = (int)((maxlen + sl - 1) / sl);
    Reserve((size_t)sl * (size_t)n, S);

    struct Slice {
        uint64_t off[RDC_MAX_RANKS], len[RDC_MAX_RANKS], pos[RDC_MAX_RANKS];  // pos: offset in the pinned slot
        uint64_t bytes;
    };
    auto slice = [&](int k) {
        Slice s;
        memset(&s, 0, sizeof(s));
        for (int q = 0; q < n; ++q) {
            const uint64_t lo = (uint64_t)cb[q] * esz + (uint64_t)k * sl;
            const uint64_t hi = std::min<uint64_t>((uint64_t)ce[q] * esz, lo + sl);
            s.pos[q] = s.bytes;
            if (hi > lo && (uint64_t)k * sl < (uint64_t)(ce[q] - cb[q]) * esz) {
                s.off[q] = lo;
                s.len[q] = hi - lo;
                s.bytes += hi - lo;
            }
        }
        return s;
    };
    auto drain = [&](int k) {  // D2H of piece k landed: copy its slices back into the user buffer
        const int slot = k % kSlots;
        hip_check(hipEventSynchronize(out_done_[slot]), "wait D2H");
        const Slice s = slice(k);
        for (int q = 0; q < n; ++q)
            if (s.len[q]) Copy(h + s.off[q], pin_out_[slot] + s.pos[q], s.len[q]);
    };
    for (int k = 0; k < K; ++k) {
        const int slot = k % kSlots;
        const Slice s = slice(k);
        // the slot's previous H2D has been consumed before we overwrite it
        if (k >= kSlots) hip_check(hipEventSynchronize(in_done_[slot]), "wait H2D slot");
        for (int q = 0; q < n; ++q)
            if (s.len[q]) Copy(pin_in_[slot] + s.pos[q], h + s.off[q], s.len[q]);
        for (int q = 0; q < n; ++q)
            if (s.len[q])
                hip_check(hipMemcpyAsync(dev_ + s.off[q], pin_in_[slot] + s.pos[q], s.len[q], hipMemcpyHostToDevice,
                                         h2d_),
                          "H2D");
        hip_check(hipEventRecord(in_done_[slot], h2d_), "record");
        hip_check(hipStreamWaitEvent(comm_stream, in_done_[slot], 0), "wait");
        c->AllreduceRanges(dev_, s.off, s.len, dtype, (int)op, comm_stream);
        hip_check(hipEventRecord(ar_done_[slot], comm_stream), "record");
        hip_check(hipStreamWaitEvent(d2h_, ar_done_[slot], 0), "wait");
        // pin_out_[slot] was drained at iteration k-1 (piece k - kSlots)
        for (int q = 0; q < n; ++q)
            if (s.len[q])
                hip_check(hipMemcpyAsync(pin_out_[slot] + s.pos[q], dev_ + s.off[q], s.len[q], hipMemcpyDeviceToHost,
                                         d2h_),
                          "D2H");
        hip_check(hipEventRecord(out_done_[slot], d2h_), "record");
        if (k - (kSlots - 1) >= 0) drain(k - (kSlots - 1));
    }
    for (int k = std::max(0, K - (kSlots - 1)); k < K; ++k) drain(k);
    c->Check(comm_stream);  // a device-side failure surfaces here
}

}  // namespace rdc_amd
