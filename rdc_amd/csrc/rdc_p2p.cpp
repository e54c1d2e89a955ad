// Point-to-point engine (see rdc_p2p.h).
#include "rdc_p2p.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <stdexcept>

#include "rdc_kernels.h"

namespace rdc_amd {

namespace {
// RDC_P2P_TRACE=1: timeline of the first pieces on stderr (diagnostics)
double trace_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
bool trace_on() {
    static const bool on = getenv("RDC_P2P_TRACE") != nullptr;
    return on;
}
#define P2P_TRACE(...)                                          \
    do {                                                        \
        if (trace_on()) {                                       \
            fprintf(stderr, "[p2p %.1f] ", trace_us());         \
            fprintf(stderr, __VA_ARGS__);                       \
            fputc('\n', stderr);                               \
        }                                                       \
    } while (0)

void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string("rdc p2p: ") + what + ": " + hipGetErrorString(e));
}
// The control block must sit on pages of its own, wholly inside ONE device
// mapping (round 1's illegal address, DESIGN.md §4 "Point-to-point": the
// only host memory a copy kernel touches is this block, and a block that
// shared pages with heap objects could lose its GPU mapping when the runtime
// pinned and unpinned those pages for an unrelated copy).  Returns the block's
// device address; throws if any of that does not hold.
char* checked_ctl_mapping(const P2PCtl* ctl) {
    const uintptr_t page = 4096;
    if ((uintptr_t)ctl % page != 0)
        throw std::logic_error("rdc p2p: control block not page-aligned (it must own its pages)");
    void* d0 = nullptr;
    hip_check(hipHostGetDevicePointer(&d0, const_cast<P2PCtl*>(ctl), 0), "control block device address");
    const char* last = reinterpret_cast<const char*>(ctl) + sizeof(P2PCtl) - 1;
    hipPointerAttribute_t a0, a1;
    memset(&a0, 0, sizeof(a0));
    memset(&a1, 0, sizeof(a1));
    hip_check(hipPointerGetAttributes(&a0, ctl), "control block attributes");
    hip_check(hipPointerGetAttributes(&a1, last), "control block attributes (last byte)");
    const bool mapped = a0.type == hipMemoryTypeHost && a1.type == hipMemoryTypeHost && a0.devicePointer &&
                        a1.devicePointer &&
                        static_cast<char*>(a1.devicePointer) - static_cast<char*>(a0.devicePointer) ==
                            (ptrdiff_t)(sizeof(P2PCtl) - 1) &&
                        a0.devicePointer == d0;
    if (!mapped) throw std::logic_error("rdc p2p: control block is not one contiguous device-mapped host range");
    return static_cast<char*>(d0);
}

bool is_host(const void* p) {
    hipPointerAttribute_t a;
    memset(&a, 0, sizeof(a));
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return true;
    }
    return !(a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged);
}
}  // namespace

// ---------------------------------------------------------------- WorkComp --
int WorkComp::Wait() {
    for (int i = 0; i < 20000; ++i) {  // short transfers finish within microseconds: spin first
        const int s = status_.load(std::memory_order_acquire);
        if (s == RDC_WS_FINISHED || s == RDC_WS_ERROR) {
            std::lock_guard<std::mutex> lk(mu_);  // Finish() has released the lock: err_ is final
            return s == RDC_WS_FINISHED ? 0 : 1;
        }
        __builtin_ia32_pause();
    }
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return status_.load() == RDC_WS_FINISHED || status_.load() == RDC_WS_ERROR; });
    return status_.load() == RDC_WS_FINISHED ? 0 : 1;
}

std::string WorkComp::error() {
    std::lock_guard<std::mutex> lk(mu_);
    return err_;
}

void WorkComp::Finish(int status, const std::string& err) {
    {
        std::lock_guard<std::mutex> lk(mu_);
        err_ = err;
        status_.store(status);
        cv_.notify_all();
    }
    Release();  // the engine's reference
}

void WorkComp::Release() {
    if (refs_.fetch_sub(1) == 1) delete this;
}

// --------------------------------------------------------------- P2PEngine --
P2PEngine::P2PEngine(int rank, int n, int device, size_t slot_bytes, char* local, char* const* peers, P2PCtl* ctl,
                     double timeout_s)
    : rank_(rank), n_(n), device_(device), slot_bytes_(slot_bytes), timeout_s_(timeout_s), local_(local), ctl_(ctl) {
    for (int p = 0; p < RDC_MAX_RANKS; ++p) peers_[p] = p < n ? peers[p] : nullptr;
    hip_check(hipSetDevice(device_), "hipSetDevice");
    ctl_dev_ = checked_ctl_mapping(ctl_);
    hip_check(hipMalloc(&arrive_, 2 * RDC_MAX_RANKS * sizeof(uint32_t)), "hipMalloc arrival counters");
    // zeroed on a private stream: the engine starts on first use, possibly
    // while collectives of other ranks of a single-process group are waiting
    // on this one, so nothing here may wait for the whole device
    hipStream_t s = nullptr;
    hip_check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "stream");
    const hipError_t e = hipMemsetAsync(arrive_, 0, 2 * RDC_MAX_RANKS * sizeof(uint32_t), s);
    const hipError_t w = e == hipSuccess ? hipStreamSynchronize(s) : e;
    (void)hipStreamDestroy(s);
    hip_check(w, "memset arrival counters");
    th_ = std::thread([this] { Loop(); });
}

P2PEngine::~P2PEngine() {
    {
        std::lock_guard<std::mutex> lk(mu_);
        stop_ = true;
    }
    cv_.notify_all();
    th_.join();
    (void)hipSetDevice(device_);
    for (int p = 0; p < n_; ++p) {
        for (Lane* L : {&send_[p], &recv_[p]}) {
            if (L->stream) (void)hipStreamSynchronize(L->stream);
            Fail(*L, "rdc p2p: communicator destroyed with the request pending");
            if (L->stream) (void)hipStreamDestroy(L->stream);
            if (L->bounce) (void)hipFree(L->bounce);
        }
    }
    for (hipEvent_t e : free_events_) (void)hipEventDestroy(e);
    if (arrive_) (void)hipFree(arrive_);
}

uint64_t* P2PEngine::DevWord(const std::atomic<uint64_t>& w) const {
    const ptrdiff_t off = reinterpret_cast<const char*>(&w) - reinterpret_cast<const char*>(ctl_);
    if (off < 0 || off % 8 != 0 || (size_t)off + sizeof(uint64_t) > sizeof(P2PCtl))
        throw std::logic_error("rdc p2p: control word outside the control block");
    return reinterpret_cast<uint64_t*>(ctl_dev_ + off);
}

// every address a copy kernel will touch, checked before the launch
void P2PEngine::CheckLaunch(const char* slot_base, size_t slot_off, size_t len, const uint32_t* arrive) const {
    const size_t region = (size_t)n_ * kP2PSlots * slot_bytes_;
    if (slot_base == nullptr || slot_off + len > region || len > slot_bytes_ || (slot_off % slot_bytes_) != 0)
        throw std::logic_error("rdc p2p: piece outside the slot region");
    if (arrive < arrive_ || arrive >= arrive_ + 2 * RDC_MAX_RANKS)
        throw std::logic_error("rdc p2p: arrival counter outside its allocation");
}

WorkComp* P2PEngine::Post(Lane& L, char* buf, size_t bytes, hipStream_t after) {
    if (bytes && !buf) throw std::invalid_argument("rdc p2p: null buffer");
    WorkComp* wc = new WorkComp();
    if (bytes == 0) {
        wc->Finish(RDC_WS_FINISHED, "");
        return wc;
    }
    Req r;
    r.wc = wc;
    r.buf = buf;
    r.bytes = bytes;
    r.host = is_host(buf);
    P2P_TRACE("post %p %zu B host=%d", (void*)buf, bytes, (int)r.host);
    {
        std::lock_guard<std::mutex> lk(mu_);
        if (!r.host) {
            // order the engine's copies after the caller's queued work on `after`
            (void)hipSetDevice(device_);
            r.ready = Event();
            if (hipEventRecord(r.ready, after) != hipSuccess) {
                (void)hipGetLastError();
                free_events_.push_back(r.ready);
                delete wc;
                throw std::runtime_error("rdc p2p: cannot record the caller's stream");
            }
        }
        if (L.q.empty()) L.last = std::chrono::steady_clock::now();
        L.q.push_back(std::move(r));
        ++pending_;
    }
    cv_.notify_all();
    P2P_TRACE("posted");
    return wc;
}

WorkComp* P2PEngine::ISend(const void* buf, size_t bytes, int dest, hipStream_t after) {
    if (dest < 0 || dest >= n_ || dest == rank_) throw std::invalid_argument("rdc p2p: bad destination rank");
    return Post(send_[dest], const_cast<char*>(static_cast<const char*>(buf)), bytes, after);
}

WorkComp* P2PEngine::IRecv(void* buf, size_t bytes, int src, hipStream_t after) {
    if (src < 0 || src >= n_ || src == rank_) throw std::invalid_argument("rdc p2p: bad source rank");
    return Post(recv_[src], static_cast<char*>(buf), bytes, after);
}

hipEvent_t P2PEngine::Event() {
    if (!free_events_.empty()) {
        hipEvent_t e = free_events_.back();
        free_events_.pop_back();
        return e;
    }
    hipEvent_t e;
    hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "event");
    return e;
}

void P2PEngine::Fail(Lane& L, const std::string& err) {
    for (Req& r : L.q) {
        if (r.ready) free_events_.push_back(r.ready);
        r.wc->Finish(RDC_WS_ERROR, err);
        --pending_;
    }
    L.q.clear();
}

// the request's first piece waits for the caller's stream
void P2PEngine::Ready(Lane& L, Req& r) {
    if (!L.stream) hip_check(hipStreamCreateWithFlags(&L.stream, hipStreamNonBlocking), "stream");
    if (r.ready) {
        hip_check(hipStreamWaitEvent(L.stream, r.ready, 0), "stream wait");
        free_events_.push_back(r.ready);  // the wait captured the event's state
        r.ready = nullptr;
    }
}

// retire finished pieces of the front requests: `word` (posted for a send
// lane, consumed for a recv lane) is advanced by the copy kernels themselves
bool P2PEngine::Complete(Lane& L, const std::atomic<uint64_t>& word) {
    bool moved = false;
    const uint64_t now = word.load(std::memory_order_acquire);
    while (!L.q.empty()) {
        Req& r = L.q.front();
        while (!r.inflight.empty() && r.inflight.front().first <= now) {
            r.done += r.inflight.front().second;
            r.inflight.pop_front();
            ++L.seq_done;
            P2P_TRACE("piece %llu complete", (unsigned long long)L.seq_done);
            moved = true;
        }
        if (r.done < r.bytes) break;
        r.wc->Finish(RDC_WS_FINISHED, "");
        L.q.pop_front();
        --pending_;
        moved = true;
    }
    return moved;
}

// Sender: piece seq goes to slot (seq-1) % kP2PSlots of the peer's region
// row for this rank once the peer consumed piece seq - kP2PSlots.
bool P2PEngine::StepSend(int dest, Lane& L) {
    bool moved = Complete(L, ctl_->posted[rank_][dest].v);
    for (Req& r : L.q) {
        while (r.issued < r.bytes) {
            const uint64_t seq = L.seq_issued + 1;
            if (seq > (uint64_t)kP2PSlots &&
                ctl_->consumed[rank_][dest].v.load(std::memory_order_acquire) < seq - kP2PSlots)
                return moved;
            const int s = (int)((seq - 1) % kP2PSlots);
            const size_t len = std::min(slot_bytes_, r.bytes - r.issued);
            Ready(L, r);
            const char* src = r.buf + r.issued;
            if (r.host) {
                if (!L.bounce) hip_check(hipMalloc(&L.bounce, slot_bytes_ * kP2PSlots), "hipMalloc bounce");
                hip_check(hipMemcpyAsync(L.bounce + (size_t)s * slot_bytes_, src, len, hipMemcpyHostToDevice, L.stream),
                          "H2D");
                src = L.bounce + (size_t)s * slot_bytes_;
            }
            const size_t slot_off = ((size_t)rank_ * kP2PSlots + s) * slot_bytes_;
            CheckLaunch(peers_[dest], slot_off, len, arrive_ + dest);
            char* dst = peers_[dest] + slot_off;
            ctl_->len[rank_][dest][s].v.store(len, std::memory_order_relaxed);  // published by posted's release
            hip_check(launch_copy(dst, src, len, L.stream, arrive_ + dest, DevWord(ctl_->posted[rank_][dest].v), seq),
                      "launch copy");
            P2P_TRACE("send piece %llu launched", (unsigned long long)seq);
            r.inflight.emplace_back(seq, len);
            r.issued += len;
            L.seq_issued = seq;
            moved = true;
        }
    }
    return moved;
}

// Receiver: piece seq is readable once posted >= seq; after the copy out,
// consumed = seq frees the slot for the sender.
bool P2PEngine::StepRecv(int src, Lane& L) {
    bool moved = Complete(L, ctl_->consumed[src][rank_].v);
    for (Req& r : L.q) {
        while (r.issued < r.bytes) {
            const uint64_t seq = L.seq_issued + 1;
            if (ctl_->posted[src][rank_].v.load(std::memory_order_acquire) < seq) return moved;
            const int s = (int)((seq - 1) % kP2PSlots);
            const size_t len = std::min(slot_bytes_, r.bytes - r.issued);
            const size_t sent = ctl_->len[src][rank_][s].v.load(std::memory_order_relaxed);
            if (sent != len) {
                Fail(L, "rdc p2p: message size mismatch with rank " + std::to_string(src) + " (piece of " +
                            std::to_string(sent) + " B sent, " + std::to_string(len) + " B expected)");
                return true;
            }
            Ready(L, r);
            const size_t slot_off = ((size_t)src * kP2PSlots + s) * slot_bytes_;
            CheckLaunch(local_, slot_off, len, arrive_ + RDC_MAX_RANKS + src);
            const char* from = local_ + slot_off;
            char* to = r.buf + r.issued;
            uint64_t* word = DevWord(ctl_->consumed[src][rank_].v);
            if (r.host) {  // DMA, then a signal-only launch (stream order: after the copy landed)
                hip_check(hipMemcpyAsync(to, from, len, hipMemcpyDeviceToHost, L.stream), "D2H");
                hip_check(launch_copy(nullptr, nullptr, 0, L.stream, arrive_ + RDC_MAX_RANKS + src, word, seq),
                          "launch signal");
            } else {
                hip_check(launch_copy(to, from, len, L.stream, arrive_ + RDC_MAX_RANKS + src, word, seq),
                          "launch copy");
            }
            P2P_TRACE("recv piece %llu launched", (unsigned long long)seq);
            r.inflight.emplace_back(seq, len);
            r.issued += len;
            L.seq_issued = seq;
            moved = true;
        }
    }
    return moved;
}

bool P2PEngine::Progress() {
    bool moved = false;
    const auto now = std::chrono::steady_clock::now();
    for (int p = 0; p < n_; ++p) {
        if (p == rank_) continue;
        for (int dir = 0; dir < 2; ++dir) {
            Lane& L = dir == 0 ? send_[p] : recv_[p];
            if (L.q.empty()) continue;
            bool m = false;
            try {
                m = dir == 0 ? StepSend(p, L) : StepRecv(p, L);
            } catch (const std::exception& e) {
                Fail(L, e.what());
                m = true;
            }
            if (m) {
                L.last = now;
                moved = true;
            } else if (std::chrono::duration<double>(now - L.last).count() > timeout_s_) {
                Fail(L, std::string("rdc p2p: ") + (dir == 0 ? "send to" : "receive from") + " rank " +
                            std::to_string(p) + " made no progress for " + std::to_string(timeout_s_) + " s");
                moved = true;
            }
        }
    }
    return moved;
}

void P2PEngine::Loop() {
    (void)hipSetDevice(device_);
    std::unique_lock<std::mutex> lk(mu_);
    int idle = 0, quiet = 0;
    while (!stop_) {
        if (pending_ == 0) {
            // stay hot for ~2 ms after the last request: the next message of
            // an exchange usually follows within microseconds, and a wake
            // from the condition variable costs 5-10 us
            if (quiet < 4096) {
                ++quiet;
                lk.unlock();
                for (int i = 0; i < 32; ++i) __builtin_ia32_pause();
                lk.lock();
                continue;
            }
            cv_.wait(lk, [&] { return stop_ || pending_ > 0; });
            idle = quiet = 0;
            continue;
        }
        quiet = 0;
        if (Progress()) {
            idle = 0;
            continue;
        }
        // nothing moved: spin (a hand-off is a few microseconds away) for
        // ~10 ms of idle polls, then back off to sleeps of up to 50 us
        lk.unlock();
        if (++idle < 8192) {
            for (int i = 0; i < 32; ++i) __builtin_ia32_pause();
        } else {
            std::this_thread::sleep_for(std::chrono::microseconds(std::min(50, (idle - 8192) / 64 + 1)));
        }
        lk.lock();
    }
}

}  // namespace rdc_amd
