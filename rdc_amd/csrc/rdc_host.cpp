// Pipelined host-resident allreduce (see rdc_host.h).
#include "rdc_host.h"
#include "rdc_kernels.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <map>
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
// Buffers up to HostInlineBytes() go as ONE piece on the caller's thread;
// larger ones through the pipeline in pieces of piece_target() bytes
// (RDC_HOST_PIECE_BYTES, default 16 MiB since round 4: with contiguous pieces
// and the ramp, n = 2 on one GPU, staged 64 MiB 5.16-5.21 vs 5.64 ms with
// 8 MiB pieces and 256 MiB 20.8-20.9 vs 21.6-21.7 ms, registered 13.4 vs
// 15.9 ms; 32 MiB within noise of 16; profiles/r04/host_gap/.  Round 2's
// pipeline, before contiguous pieces, measured 8 MiB faster.)
size_t piece_target() { return HostPieceBytes(); }
constexpr size_t kParallelMin = (size_t)512 << 10;  // below this a copy runs on the caller alone (waking the pool costs more)
// RDC_HOST_TRACE=1: per-piece timeline on stderr (diagnostics)
double trace_now() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e3 + t.tv_nsec * 1e-6;
}
bool tracing() {
    static const bool on = getenv("RDC_HOST_TRACE") != nullptr;
    return on;
}
}  // namespace

// {integer}{B,K,M,G} as the reference's ParseUnit (communicator_manager.cc:14-42)
// into *out; false when unset or malformed (a warning names a malformed value)
static bool env_bytes_parse(const char* name, size_t* out) {
    const char* e = getenv(name);
    if (!e || !*e) return false;
    unsigned long long amt = 0;
    char unit = 0, extra = 0;
    const int k = sscanf(e, "%llu%c%c", &amt, &unit, &extra);
    bool ok = k == 1 || (k == 2 && (unit == 'B' || unit == 'K' || unit == 'M' || unit == 'G'));
    if (ok) {
        const int shift = k == 1 || unit == 'B' ? 0 : unit == 'K' ? 10 : unit == 'M' ? 20 : 30;
        *out = (size_t)amt << shift;
    } else {
        fprintf(stderr, "rdc: ignoring malformed %s=%s (expected an integer with an optional B/K/M/G unit)\n",
                name, e);
    }
    return ok;
}
// 0 when unset or malformed
static size_t env_bytes(const char* name) {
    size_t v = 0;
    return env_bytes_parse(name, &v) ? v : 0;
}

int HostBalanceSetting() {
    static const int v = env_int("RDC_HOST_BALANCE", -1);
    return v < 0 ? -1 : (v != 0 ? 1 : 0);
}

size_t HostPieceBytes() {
    static const size_t v = [] {
        const size_t x = env_bytes("RDC_HOST_PIECE_BYTES");
        return x >= ((size_t)1 << 20) ? x : (size_t)16 << 20;
    }();
    return v;
}

// inline (one piece on the caller) up to 16 MiB by default: pipelining 4-16
// MiB in 1-2 MiB pieces measured no better (n = 2 on one GPU, alternating:
// 16 MiB 1.55-1.61 ms inline vs 1.53-1.65 with 2 MiB pieces, 2.8-3.1 with
// 1 MiB; 4 MiB 0.46-0.49 vs 0.50-0.51; profiles/r03/host_inline_ab/)
size_t HostInlineBytes() {
    static const size_t v = [] {
        size_t x = 0;  // an explicit 0 keeps every host buffer in the pipeline; malformed = the default
        return env_bytes_parse("RDC_HOST_INLINE_BYTES", &x) ? x : (size_t)16 << 20;
    }();
    return v;
}

bool HostPieceRamp() {
    static const bool v = [] {
        const char* e = getenv("RDC_HOST_PIECE_RAMP");
        return !(e && *e && atoi(e) == 0);
    }();
    return v;
}

// Contiguous pieces of about HostPieceBytes() P (multiples of 4 KiB).  With
// the ramp (RDC_HOST_PIECE_RAMP, default on; buffers of at least 8 P: n = 2
// on one GPU, same box, alternating, 64 MiB 5.0 / 5.1 vs 5.7 / 6.1 ms without,
// but 32 MiB 2.7 / 3.1 vs 2.5 / 2.5 ms — profiles/r03/host_ramp/) the
// first three pieces are P/8, P/4, P/2 and the last three P/2, P/4, P/8: the
// first H2D starts after an eighth of a piece's copy-in and the last D2H
// moves an eighth of a piece, so the pipeline fills and drains in small steps.
std::vector<uint64_t> HostPieceBounds(uint64_t S) {
    const uint64_t P = piece_target();
    auto up4k = [](uint64_t x) { return std::max<uint64_t>(4096, (x + 4095) & ~(uint64_t)4095); };
    std::vector<uint64_t> b{0};
    if (S <= HostInlineBytes()) {
        b.push_back(S);
        return b;
    }
    uint64_t ramp[3] = {0, 0, 0}, ramp_sum = 0;
    if (HostPieceRamp() && S >= 8 * P) {
        for (int i = 0; i < 3; ++i) {
            ramp[i] = up4k(P >> (3 - i));  // P/8, P/4, P/2
            ramp_sum += ramp[i];
        }
    }
    for (int i = 0; i < 3; ++i)
        if (ramp[i]) b.push_back(b.back() + ramp[i]);
    // the tail ramp starts on a 4 KiB boundary; the last piece takes the rest
    const uint64_t mid_end = ramp_sum ? (S - ramp_sum) & ~(uint64_t)4095 : S;
    const uint64_t mid = mid_end - b.back();
    const uint64_t K0 = std::max<uint64_t>(1, (mid + P - 1) / P);
    const uint64_t sl = up4k((mid + K0 - 1) / K0);
    for (uint64_t x = b.back() + sl; x < mid_end; x += sl) b.push_back(x);
    b.push_back(mid_end);
    if (ramp_sum) {
        b.push_back(b.back() + ramp[2]);
        b.push_back(b.back() + ramp[1]);
        b.push_back(S);
    }
    return b;  // b.back() == S
}

// ------------------------------------------------------ registered ranges --
namespace {
std::mutex g_reg_mu;
std::map<uintptr_t, size_t> g_reg;  // start -> bytes, non-overlapping (hipHostRegister refuses overlaps)
std::atomic<uint64_t> g_reg_calls{0};
}  // namespace

void HostRegistryAdd(const void* p, size_t bytes) {
    std::lock_guard<std::mutex> lk(g_reg_mu);
    g_reg[(uintptr_t)p] = bytes;
}

void HostRegistryRemove(const void* p) {
    std::lock_guard<std::mutex> lk(g_reg_mu);
    g_reg.erase((uintptr_t)p);
}

bool HostRegistryCovers(const void* p, size_t bytes, const void** base) {
    const uintptr_t a = (uintptr_t)p;
    std::lock_guard<std::mutex> lk(g_reg_mu);
    auto it = g_reg.upper_bound(a);  // the first range starting after a
    if (it == g_reg.begin()) return false;
    --it;
    const bool in = a - it->first <= it->second && bytes <= it->second - (a - it->first);
    if (in && base) *base = reinterpret_cast<const void*>(it->first);
    return in;
}

uint64_t HostRegisteredCalls() { return g_reg_calls.load(std::memory_order_relaxed); }

// ---------------------------------------------------------------- HostPath --
// wait for an event by polling it: a blocking synchronisation may sleep and
// pay a wake-up on every piece
void HostPath::SpinEvent(hipEvent_t e, const char* what) {
    for (;;) {
        const hipError_t q = hipEventQuery(e);
        if (q == hipSuccess) return;
        if (q != hipErrorNotReady) hip_check(q, what);
        __builtin_ia32_pause();
    }
}

HostPath::HostPath(int device, size_t zc_max)
    : device_(device), zc_max_(zc_max), pool_(std::max(0, env_int("RDC_HOST_THREADS", 4) - 1)) {
    hip_check(hipSetDevice(device_), "hipSetDevice");
    hip_check(hipStreamCreateWithFlags(&h2d_, hipStreamNonBlocking), "stream");
    hip_check(hipStreamCreateWithFlags(&d2h_, hipStreamNonBlocking), "stream");
    for (int i = 0; i < kSlots; ++i) hip_check(hipEventCreateWithFlags(&in_done_[i], hipEventDisableTiming), "event");
    drain_ = std::thread([this] { DrainLoop(); });
}

HostPath::~HostPath() {
    {
        std::lock_guard<std::mutex> lk(dmu_);
        dstop_ = true;
    }
    dcv_.notify_all();
    drain_.join();
    (void)hipSetDevice(device_);
    (void)hipDeviceSynchronize();
    for (int i = 0; i < kSlots; ++i) {
        if (pin_in_[i]) (void)hipHostFree(pin_in_[i]);
        (void)hipEventDestroy(in_done_[i]);
    }
    for (hipEvent_t e : ar_done_) (void)hipEventDestroy(e);
    for (hipEvent_t e : h2d_done_) (void)hipEventDestroy(e);
    if (pin_small_) (void)hipHostFree(pin_small_);
    if (small_done_) (void)hipEventDestroy(small_done_);
    if (dev_small_) (void)hipFree(dev_small_);
    if (dev_) (void)hipFree(dev_);
    if (h2d_) (void)hipStreamDestroy(h2d_);
    if (d2h_) (void)hipStreamDestroy(d2h_);
}

void HostPath::Warm(hipStream_t comm_stream) {
    if (warm_ || env_int("RDC_HOST_WARM", 1) == 0) return;
    warm_ = true;
    hip_check(hipSetDevice(device_), "hipSetDevice");
    constexpr size_t kMax = (size_t)16 << 20;
    Reserve(0, kMax, 0, comm_stream);
    char* pin = nullptr;
    hip_check(hipHostMalloc(reinterpret_cast<void**>(&pin), kMax, hipHostMallocDefault), "hipHostMalloc");
    try {
        // comm_stream null (RdcNewBuffer): the path's own copy streams only —
        // never a sync of a stream that may hold queued collectives
        for (hipStream_t s : {h2d_, d2h_, comm_stream}) {
            if (!s) continue;
            for (size_t b : {(size_t)64 << 10, (size_t)1 << 20, kMax}) {
                hip_check(hipMemcpyAsync(dev_, pin, b, hipMemcpyHostToDevice, s), "warm H2D");
                hip_check(hipMemcpyAsync(pin, dev_, b, hipMemcpyDeviceToHost, s), "warm D2H");
                hip_check(hipStreamSynchronize(s), "warm sync");
            }
        }
    } catch (...) {
        (void)hipHostFree(pin);
        throw;
    }
    hip_check(hipHostFree(pin), "hipHostFree");
}

// Growing waits only for this path's own streams and the communicator's
// stream (the previous call's copies and launches that may still use the old
// buffers), never for the whole device: in a single-process group the other
// ranks' launches may be waiting on this rank's next one.
void HostPath::QuiesceForRegrow(hipStream_t comm_stream) {
    hip_check(hipStreamSynchronize(h2d_), "sync before regrow");
    hip_check(hipStreamSynchronize(d2h_), "sync before regrow");
    if (comm_stream) hip_check(hipStreamSynchronize(comm_stream), "sync before regrow");
}

void HostPath::Reserve(size_t piece_bytes, size_t total_bytes, int pieces, hipStream_t comm_stream) {
    if (piece_bytes > slot_bytes_) {
        QuiesceForRegrow(comm_stream);
        for (int i = 0; i < kSlots; ++i) {
            if (pin_in_[i]) (void)hipHostFree(pin_in_[i]);
            pin_in_[i] = nullptr;
        }
        slot_bytes_ = 0;
        for (int i = 0; i < kSlots; ++i)
            hip_check(hipHostMalloc(reinterpret_cast<void**>(&pin_in_[i]), piece_bytes, hipHostMallocDefault),
                      "hipHostMalloc");
        slot_bytes_ = piece_bytes;
    }
    if (total_bytes > dev_bytes_) {
        if (dev_) {
            QuiesceForRegrow(comm_stream);
            (void)hipFree(dev_);
            dev_ = nullptr;
            dev_bytes_ = 0;
        }
        hip_check(hipMalloc(reinterpret_cast<void**>(&dev_), total_bytes), "hipMalloc host-path image");
        dev_bytes_ = total_bytes;
    }
    while ((int)ar_done_.size() < pieces) {
        hipEvent_t e;
        hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "event");
        ar_done_.push_back(e);
    }
}

namespace {
// RDC_HOST_NT_COPY=0: plain memcpy into the pinned slots (rdc_copypool.h StreamCopy)
bool nt_copy_enabled() {
    static const bool v = [] {
        const char* e = getenv("RDC_HOST_NT_COPY");
        return !(e && *e && atoi(e) == 0) && __builtin_cpu_supports("avx2");
    }();
    return v;
}
}  // namespace

void HostPath::Copy(char* dst, const char* src, size_t bytes, bool to_pinned) {
    ParallelCopy(pool_, dst, src, bytes, to_pinned && nt_copy_enabled(), kParallelMin);
}

void HostPath::DrainLoop() {
    for (;;) {
        Drain d;
        char* dst;
        {
            std::unique_lock<std::mutex> lk(dmu_);
            dcv_.wait(lk, [&] { return dstop_ || qhead_ < queue_.size(); });
            if (dstop_) return;
            d = queue_[qhead_++];
            dst = dst_;
        }
        std::string err;
        try {
            hip_check(hipSetDevice(device_), "hipSetDevice");
            const double t0 = tracing() ? trace_now() : 0;
            // blocking waits here: a spinning drain thread competes with the
            // copy threads for cores and measured no faster (2-16 MiB)
            hip_check(hipEventSynchronize(d.ready), "wait allreduce");
            const double t1 = tracing() ? trace_now() : 0;
            for (int q = 0; q < d.nslice; ++q)
                if (d.len[q])
                    hip_check(hipMemcpyAsync(dst + d.off[q], dev_ + d.off[q], d.len[q], hipMemcpyDeviceToHost, d2h_),
                              "D2H");
            hip_check(hipStreamSynchronize(d2h_), "D2H sync");
            if (tracing())
                fprintf(stderr, "[host %.3f] drain: waited AR %.3f ms, D2H %.3f ms\n", t1, t1 - t0, trace_now() - t1);
        } catch (const std::exception& e) {
            err = e.what();
        }
        std::lock_guard<std::mutex> lk(dmu_);
        if (!err.empty() && derr_.empty()) derr_ = err;
        ++drained_;
        ddone_cv_.notify_all();
    }
}

// Small buffers are latency-bound.  Up to zc_max bytes the collective runs
// zero-copy on the pinned staging buffer itself (the kernel reads and writes
// host memory over PCIe): memcpy in, ONE kernel, one sync, memcpy out.  Larger
// ones: H2D, allreduce, D2H on the communicator's stream, one sync.  The
// error word needs no copy (the kernel mirrors it into pinned memory).
void HostPath::AllreduceSmall(Communicator* c, char* h, size_t count, size_t S, int dtype, int op,
                              hipStream_t comm_stream) {
    if (!pin_small_) {
        hip_check(hipHostMalloc(reinterpret_cast<void**>(&pin_small_), kSmall + 64, hipHostMallocCoherent),
                  "hipHostMalloc");
        hip_check(hipHostGetDevicePointer(reinterpret_cast<void**>(&pin_small_dev_), pin_small_, 0),
                  "hipHostGetDevicePointer");
        hip_check(hipMalloc(reinterpret_cast<void**>(&dev_small_), kSmall), "hipMalloc");
    }
    Copy(pin_small_, h, S);
    if (S <= zc_max_) {
        // the launch's last block stores a token into pinned memory: spin on
        // it instead of a stream sync (Communicator::ArmNotify / WaitNotify)
        const uint32_t token = c->ArmNotify();
        try {
            c->Allreduce(pin_small_dev_, count, dtype, op, comm_stream);
        } catch (...) {
            c->WaitNotify(token, comm_stream);  // disarms
            throw;
        }
        c->WaitNotify(token, comm_stream);
        Copy(h, pin_small_, S);
        return;
    }
    hip_check(hipMemcpyAsync(dev_small_, pin_small_, S, hipMemcpyHostToDevice, comm_stream), "H2D");
    c->Allreduce(dev_small_, count, dtype, op, comm_stream);
    hip_check(hipMemcpyAsync(pin_small_, dev_small_, S, hipMemcpyDeviceToHost, comm_stream), "D2H");
    // spin on the D2H's completion (a blocking synchronisation may sleep and
    // pay a wake-up per call)
    if (!small_done_) hip_check(hipEventCreateWithFlags(&small_done_, hipEventDisableTiming), "event");
    hip_check(hipEventRecord(small_done_, comm_stream), "record");
    SpinEvent(small_done_, "D2H completion");
    c->RaiseIfError(c->HostErrorWord());
    Copy(h, pin_small_, S);
}

namespace {
// RDC_HOST_BALANCE=1 / 0 forces balanced / chunk-owned piece ranges; by
// default balanced with one rank per GPU (each rank's own links and HBM),
// chunk-owned where ranks share a GPU (the one-GPU rehearsals measured that
// layout, profiles/r03/host_contiguous_pieces/)
bool balance_pieces(const Communicator* c) {
    const int env = HostBalanceSetting();
    return env >= 0 ? env != 0 : c->ranks_per_gpu() == 1;
}

void host_piece_ranges(const Communicator* c, uint64_t lo, uint64_t hi, const int64_t* cb, const int64_t* ce,
                       size_t esz, uint64_t* roff, uint64_t* rlen, int8_t* fold) {
    HostPieceRanges(lo, hi, c->size(), cb, ce, esz, balance_pieces(c), roff, rlen, fold);
}
}  // namespace

namespace {
// the device address of registered host bytes [h, h + bytes)
char* registered_device_address(char* h, uint64_t bytes) {
    const void* base = nullptr;
    if (!HostRegistryCovers(h, bytes, &base)) throw std::logic_error("rdc: device address of an unregistered range");
    void* dbase = nullptr;
    hip_check(hipHostGetDevicePointer(&dbase, const_cast<void*>(base), 0), "hipHostGetDevicePointer");
    return static_cast<char*>(dbase) + (h - static_cast<const char*>(base));
}
}  // namespace

// A registered buffer is DMA-able in place (57 GB/s either way on the box,
// the rate of hipHostMalloc memory): no pinned slots, no copy pool, no drain
// thread.  Every piece's H2D, allreduce and D2H is queued up front on the
// three streams, chained by per-piece events, and the caller spins once on the
// last D2H.  Pieces and collectives are the pipeline's (HostPieceBounds, the
// same AllreduceRanges calls), so ranks with and without a registered buffer
// issue matching collectives and every element is folded in its chunk's ring
// order either way.
void HostPath::AllreduceRegistered(Communicator* c, char* h, size_t count, int dtype, int op,
                                   hipStream_t comm_stream, const std::vector<uint64_t>& bounds, const int64_t* cb,
                                   const int64_t* ce) {
    const size_t esz = rdc_dtype_size(dtype);
    const size_t S = count * esz;
    const int K = (int)bounds.size() - 1;
    Reserve(0, S, K, comm_stream);
    while ((int)h2d_done_.size() < K) {
        hipEvent_t e;
        hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "event");
        h2d_done_.push_back(e);
    }
    g_reg_calls.fetch_add(1, std::memory_order_relaxed);
    if (RegisteredZeroCopy()) {
        AllreduceRegisteredZeroCopy(c, h, count, dtype, op, comm_stream, bounds, cb, ce);
        return;
    }
    // the copies: DMA, or kernels on the caller's pages' device mapping
    char* const hd = RegisteredKernelCopy() ? registered_device_address(h, S) : nullptr;
    auto h2d = [&](uint64_t lo, uint64_t len, hipStream_t s) {
        if (hd) hip_check(launch_copy(dev_ + lo, hd + lo, len, s), "H2D kernel");
        else hip_check(hipMemcpyAsync(dev_ + lo, h + lo, len, hipMemcpyHostToDevice, s), "H2D");
    };
    auto d2h = [&](uint64_t lo, uint64_t len, hipStream_t s) {
        if (hd) hip_check(launch_copy(hd + lo, dev_ + lo, len, s), "D2H kernel");
        else hip_check(hipMemcpyAsync(h + lo, dev_ + lo, len, hipMemcpyDeviceToHost, s), "D2H");
    };
    if (K == 1) {  // the inline piece's collective: the whole buffer
        h2d(0, S, comm_stream);
        hip_check(hipEventRecord(h2d_done_[0], comm_stream), "record");
        try {
            c->Allreduce(dev_, count, dtype, op, comm_stream);
        } catch (...) {
            (void)hipEventSynchronize(h2d_done_[0]);  // the H2D still reads the caller's buffer
            throw;
        }
        try {
            d2h(0, S, comm_stream);
            hip_check(hipEventRecord(in_done_[0], comm_stream), "record");
            SpinEvent(in_done_[0], "host allreduce");
        } catch (...) {
            (void)hipStreamSynchronize(comm_stream);  // no DMA into the caller's buffer outlives the call
            throw;
        }
        c->RaiseIfError(c->HostErrorWord());
        return;
    }
    // RDC_HOST_REG_AHEAD=a > 0: piece k's H2D waits for piece k-a's allreduce
    // (stream-ordered), so the input DMA runs at most a pieces ahead
    static const int ahead = env_int("RDC_HOST_REG_AHEAD", 0);
    static const bool etrace = env_int("RDC_HOST_EVENT_TRACE", 0) != 0;
    const auto h0 = std::chrono::steady_clock::now();
    if (etrace)
        while ((int)tev_.size() < 6 * K) {
            hipEvent_t e;
            hip_check(hipEventCreate(&e), "event");
            tev_.push_back(e);
        }
    auto mark = [&](int k, int what, hipStream_t s) {
        if (etrace) hip_check(hipEventRecord(tev_[(size_t)(6 * k + what)], s), "record");
    };
    try {
        for (int k = 0; k < K; ++k) {
            const uint64_t lo = bounds[(size_t)k], hi = bounds[(size_t)k + 1];
            uint64_t roff[RDC_MAX_RANKS], rlen[RDC_MAX_RANKS];
            int8_t fold[RDC_MAX_RANKS];
            host_piece_ranges(c, lo, hi, cb, ce, esz, roff, rlen, fold);
            if (ahead > 0 && k >= ahead)
                hip_check(hipStreamWaitEvent(h2d_, ar_done_[(size_t)(k - ahead)], 0), "wait");
            mark(k, 0, h2d_);
            h2d(lo, hi - lo, h2d_);
            hip_check(hipEventRecord(h2d_done_[(size_t)k], h2d_), "record");
            mark(k, 1, h2d_);
            hip_check(hipStreamWaitEvent(comm_stream, h2d_done_[(size_t)k], 0), "wait");
            mark(k, 2, comm_stream);
            c->AllreduceRanges(dev_ + lo, roff, rlen, dtype, op, comm_stream, fold);
            hip_check(hipEventRecord(ar_done_[(size_t)k], comm_stream), "record");
            mark(k, 3, comm_stream);
            hip_check(hipStreamWaitEvent(d2h_, ar_done_[(size_t)k], 0), "wait");
            mark(k, 4, d2h_);
            d2h(lo, hi - lo, d2h_);
            mark(k, 5, d2h_);
        }
        hip_check(hipEventRecord(in_done_[0], d2h_), "record");
        SpinEvent(in_done_[0], "host allreduce");
    } catch (...) {
        // no DMA into or out of the caller's buffer may outlive the call
        (void)hipStreamSynchronize(h2d_);
        (void)hipStreamSynchronize(d2h_);
        throw;
    }
    if (etrace)
        TraceRegistered(K, bounds, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - h0)
                                       .count());
    c->Check(comm_stream);  // a device-side failure surfaces here
}

// RDC_HOST_REG_ZC=1: the registered path runs every piece's collective on
// the caller's pages themselves (the kernels load their inputs from and store
// their results to host memory over PCIe): no device image, no H2D / D2H
// DMA.  The pieces and their collectives are the staged path's (the same
// AllreduceRanges calls), so zero-copy, registered-DMA and staged ranks still
// meet in one call; each rank may choose for itself.
bool RegisteredZeroCopy() {
    static const bool on = env_int("RDC_HOST_REG_ZC", 0) != 0;
    return on;
}

// RDC_HOST_REG_KCOPY (default 1): the registered path's H2D / D2H copies are
// kernels (launch_copy: up to 128 blocks loading from / storing to the
// caller's pages through their device mapping, 53-57 GB/s either way,
// tools/zc_bw.hip) instead of the DMA engines.  DMA copies from and into
// registered pages are faster back to back (64 MiB 3.8 vs 4.8 ms, n = 2 on one
// GPU) but stall on the first calls (14-17 ms) and slow down whenever the
// host idled before the call (20 ms idle: 5.0-7.1 ms per 64 MiB call, kernel
// copies 4.6-5.2; profiles/r04/host_gap/) — as it does between the
// allreduces of a training step.  The same pieces and collectives either
// way; a rank's own choice (0 = DMA).
bool RegisteredKernelCopy() {
    static const bool on = env_int("RDC_HOST_REG_KCOPY", 1) != 0;
    return on;
}


void HostPath::AllreduceRegisteredZeroCopy(Communicator* c, char* h, size_t count, int dtype, int op,
                                           hipStream_t comm_stream, const std::vector<uint64_t>& bounds,
                                           const int64_t* cb, const int64_t* ce) {
    const size_t esz = rdc_dtype_size(dtype);
    const int K = (int)bounds.size() - 1;
    // the device address of the caller's pages: the registration's, plus the offset
    char* hd = registered_device_address(h, count * esz);
    uint32_t token = 0;
    try {
        for (int k = 0; k < K; ++k) {
            const uint64_t lo = bounds[(size_t)k], hi = bounds[(size_t)k + 1];
            if (k == K - 1) token = c->ArmNotify();  // the call's last launch signals the host
            if (K == 1) {
                c->Allreduce(hd, count, dtype, op, comm_stream);
            } else {
                uint64_t roff[RDC_MAX_RANKS], rlen[RDC_MAX_RANKS];
                int8_t fold[RDC_MAX_RANKS];
                host_piece_ranges(c, lo, hi, cb, ce, esz, roff, rlen, fold);
                c->AllreduceRanges(hd + lo, roff, rlen, dtype, op, comm_stream, fold);
            }
        }
    } catch (...) {
        if (token) c->WaitNotify(token, comm_stream);  // disarms
        (void)hipStreamSynchronize(comm_stream);      // no kernel still touches the caller's pages
        throw;
    }
    c->WaitNotify(token, comm_stream);
}

// One line per call: the span from the first H2D's start to the last D2H's
// end, each engine's busy time (sum of its pieces) and its idle time inside
// the span, the allreduce time per piece, and the host's wall time for the
// call — JSON after the tag, for tools to parse.
void HostPath::TraceRegistered(int K, const std::vector<uint64_t>& bounds, double host_ms) {
    hip_check(hipEventSynchronize(tev_[(size_t)(6 * K - 1)]), "trace sync");
    auto at = [&](int k, int w) {
        float ms = 0;
        hip_check(hipEventElapsedTime(&ms, tev_[0], tev_[(size_t)(6 * k + w)]), "elapsed");
        return (double)ms;
    };
    double busy[3] = {0, 0, 0};
    std::string pieces;
    for (int k = 0; k < K; ++k) {
        const double t[6] = {at(k, 0), at(k, 1), at(k, 2), at(k, 3), at(k, 4), at(k, 5)};
        for (int e = 0; e < 3; ++e) busy[e] += t[2 * e + 1] - t[2 * e];
        char buf[160];
        snprintf(buf, sizeof(buf), "%s[%llu,%.3f,%.3f,%.3f,%.3f,%.3f,%.3f]", k ? "," : "",
                 (unsigned long long)(bounds[(size_t)k + 1] - bounds[(size_t)k]), t[0], t[1], t[2], t[3], t[4], t[5]);
        pieces += buf;
    }
    const double span = at(K - 1, 5);
    fprintf(stderr,
            "[rdc host-reg] {\"pieces\": %d, \"span_ms\": %.3f, \"host_ms\": %.3f, \"busy_ms\": {\"h2d\": %.3f, "
            "\"allreduce\": %.3f, \"d2h\": %.3f}, \"piece\": [%s]}\n",
            K, span, host_ms, busy[0], busy[1], busy[2], pieces.c_str());
}

void HostPath::Allreduce(Communicator* c, void* host, size_t count, int dtype, int op, hipStream_t comm_stream) {
    const int n = c->size();
    if (n == 1 || count == 0) return;
    const size_t esz = rdc_dtype_size(dtype);
    const size_t S = count * esz;
    char* h = static_cast<char*>(host);
    // the resident service (rdc_service.h) needs no HIP call per request
    if (S <= kSmall && c->SmallHostAllreduce(h, count, dtype, op)) return;
    hip_check(hipSetDevice(device_), "hipSetDevice");
    if (S <= kSmall) {
        AllreduceSmall(c, h, count, S, dtype, op, comm_stream);
        return;
    }
    if (S <= c->config().ring_mincount) {
        // the tree's order (rdc_reduce_ring_mincount) is per element, but the
        // pipeline below cuts the buffer by Split chunk for the ring: stage
        // the whole buffer instead (raised thresholds are for small buffers)
        Reserve(0, S, 0, comm_stream);
        hip_check(hipMemcpyAsync(dev_, h, S, hipMemcpyHostToDevice, comm_stream), "H2D");
        c->Allreduce(dev_, count, dtype, op, comm_stream);
        hip_check(hipMemcpyAsync(h, dev_, S, hipMemcpyDeviceToHost, comm_stream), "D2H");
        c->Check(comm_stream);
        return;
    }

    int64_t cb[RDC_MAX_RANKS], ce[RDC_MAX_RANKS];
    SplitRanges((int64_t)count, n, cb, ce);
    // pieces are contiguous byte ranges of the buffer, a multiple of 4 KiB
    // (hence of esz) long: one copy in, one H2D, one D2H each (the first
    // version cut piece k from the k-th slice of EVERY chunk — n copies each
    // way per piece).  Every element is still folded in its own Split chunk's
    // ring order: a piece's allreduce gets the chunk ranges it intersects.
    const std::vector<uint64_t> bounds = HostPieceBounds(S);
    const int K = (int)bounds.size() - 1;
    if (HostRegistryCovers(h, S)) {
        AllreduceRegistered(c, h, count, dtype, op, comm_stream, bounds, cb, ce);
        return;
    }
    uint64_t sl = 0;  // the largest piece: the pinned slot size
    for (int k = 0; k < K; ++k) sl = std::max<uint64_t>(sl, bounds[(size_t)k + 1] - bounds[(size_t)k]);
    Reserve((size_t)sl, S, K, comm_stream);
    if (K == 1) {
        // one piece (up to the piece target): nothing to overlap, so no drain
        // thread hand-off either — the slices of one piece are the chunks in
        // order, i.e. the whole buffer: pool copy into a pinned slot, H2D,
        // allreduce, pageable D2H straight into the caller's buffer, all on
        // the communicator's stream, and the caller spins on the end
        const double t0 = tracing() ? trace_now() : 0;
        Copy(pin_in_[0], h, S, true);
        const double t1 = tracing() ? trace_now() : 0;
        hip_check(hipMemcpyAsync(dev_, pin_in_[0], S, hipMemcpyHostToDevice, comm_stream), "H2D");
        c->Allreduce(dev_, count, dtype, op, comm_stream);
        hip_check(hipMemcpyAsync(h, dev_, S, hipMemcpyDeviceToHost, comm_stream), "D2H");
        hip_check(hipEventRecord(in_done_[0], comm_stream), "record");
        SpinEvent(in_done_[0], "host allreduce");
        if (tracing())
            fprintf(stderr, "[host %.3f] one piece: copy-in %.3f ms, H2D+allreduce+D2H %.3f ms (%llu B)\n", t0,
                    t1 - t0, trace_now() - t1, (unsigned long long)S);
        c->RaiseIfError(c->HostErrorWord());
        return;
    }
    {
        std::lock_guard<std::mutex> lk(dmu_);
        queue_.clear();
        qhead_ = drained_ = 0;
        dst_ = h;
        derr_.clear();
    }
    int issued = 0;
    std::string err;
    try {
        for (int k = 0; k < K; ++k) {
            const int slot = k % kSlots;
            Drain d;
            d.ready = ar_done_[(size_t)k];
            d.nslice = 1;
            const uint64_t lo = bounds[(size_t)k], hi = bounds[(size_t)k + 1], bytes = hi - lo;
            d.off[0] = lo;
            d.len[0] = bytes;
            uint64_t roff[RDC_MAX_RANKS], rlen[RDC_MAX_RANKS];
            int8_t fold[RDC_MAX_RANKS];
            host_piece_ranges(c, lo, hi, cb, ce, esz, roff, rlen, fold);
            // the slot's previous H2D has been consumed before we overwrite it
            const double t0 = tracing() ? trace_now() : 0;
            if (k >= kSlots) hip_check(hipEventSynchronize(in_done_[slot]), "wait H2D slot");
            const double t1 = tracing() ? trace_now() : 0;
            Copy(pin_in_[slot], h + lo, bytes, true);
            if (tracing())
                fprintf(stderr, "[host %.3f] piece %d: slot wait %.3f ms, copy-in %.3f ms (%llu B)\n", t0, k, t1 - t0,
                        trace_now() - t1, (unsigned long long)bytes);
            hip_check(hipMemcpyAsync(dev_ + lo, pin_in_[slot], bytes, hipMemcpyHostToDevice, h2d_), "H2D");
            hip_check(hipEventRecord(in_done_[slot], h2d_), "record");
            hip_check(hipStreamWaitEvent(comm_stream, in_done_[slot], 0), "wait");
            c->AllreduceRanges(dev_ + lo, roff, rlen, dtype, op, comm_stream, fold);
            hip_check(hipEventRecord(d.ready, comm_stream), "record");
            {
                std::lock_guard<std::mutex> lk(dmu_);
                queue_.push_back(d);
            }
            dcv_.notify_all();
            ++issued;
        }
    } catch (const std::exception& e) {
        err = e.what();
    }
    {   // every issued piece drained (the drain thread owns the user buffer until then)
        std::unique_lock<std::mutex> lk(dmu_);
        ddone_cv_.wait(lk, [&] { return (int)drained_ == issued; });
        if (err.empty()) err = derr_;
        dst_ = nullptr;
    }
    if (!err.empty()) throw std::runtime_error(err);
    c->Check(comm_stream);  // a device-side failure surfaces here
}

}  // namespace rdc_amd
