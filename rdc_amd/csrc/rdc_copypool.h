// A small pool of host threads that run the items 0..n-1 of a job together
// with the caller (the host path's pageable <-> pinned copies, rdc_host.cpp).
// Standard C++ only, so tests/cpp/copypool_stress.cc builds it without HIP.
#pragma once
#include <immintrin.h>
#include <string.h>

#include <algorithm>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace rdc_amd {

class CopyPool {
public:
    explicit CopyPool(int threads);
    ~CopyPool();
    // runs f(0) .. f(n-1) on the pool and the caller; returns when all are done
    void Run(int n, const std::function<void(int)>& f);

private:
    void Loop();
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(int)>* job_ = nullptr;
    int next_ = 0, total_ = 0, finished_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

inline CopyPool::CopyPool(int threads) {
    for (int i = 0; i < threads; ++i) th_.emplace_back([this] { Loop(); });
}

inline CopyPool::~CopyPool() {
    {
        std::lock_guard<std::mutex> lk(mu_);
        stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
}

inline void CopyPool::Loop() {
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
                // claim only items of the generation whose job we hold: a
                // thread that woke late may find the caller already returned
                // (its job destroyed) and the next Run's items on offer
                std::lock_guard<std::mutex> lk(mu_);
                if (gen_ != seen || next_ >= total_) break;
                i = next_++;
            }
            (*job)(i);
            std::lock_guard<std::mutex> lk(mu_);
            if (++finished_ == total_) done_cv_.notify_all();
        }
    }
}

inline void CopyPool::Run(int n, const std::function<void(int)>& f) {
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
    job_ = nullptr;  // under the lock: no thread takes it once this returns
}

// Copies into a pinned staging slot are read by the DMA engine, never by
// this CPU: streaming (non-temporal) stores skip the read-for-ownership of
// every destination line and leave the caches to the source.  glibc's memcpy
// only streams above a size threshold the pool's 512 KiB parts stay under.
// Streaming stores are weakly ordered: the sfence drains them before the
// thread reports its part done (the DMA that follows must see every byte).
__attribute__((target("avx2"))) inline void StreamCopy(char* dst, const char* src, size_t bytes) {
    size_t head = (32 - ((uintptr_t)dst & 31)) & 31;
    if (head > bytes) head = bytes;
    memcpy(dst, src, head);
    size_t i = head;
    for (; i + 128 <= bytes; i += 128) {
        const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i));
        const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 32));
        const __m256i c = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 64));
        const __m256i d = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 96));
        _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i), a);
        _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i + 32), b);
        _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i + 64), c);
        _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i + 96), d);
    }
    memcpy(dst + i, src + i, bytes - i);
    _mm_sfence();
}

// Bytes per part when a copy of `bytes` is cut into `parts` (4 KiB multiples,
// parts * per >= bytes).  Rounding the FLOOR of bytes / parts up to 4 KiB
// loses the last bytes % parts bytes whenever that floor is already a 4 KiB
// multiple (e.g. 4 x 256 KiB + 3 B); round the ceiling instead.
inline size_t CopyPartBytes(size_t bytes, int parts) {
    const size_t q = (bytes + (size_t)parts - 1) / (size_t)parts;
    return (q + 4095) & ~(size_t)4095;
}

// dst <- src over the pool: below min_parallel on the caller alone, else in
// up to 16 parts of at least min_parallel / 2.  stream: streaming stores.
inline void ParallelCopy(CopyPool& pool, char* dst, const char* src, size_t bytes, bool stream,
                         size_t min_parallel) {
    if (bytes < min_parallel) {
        if (stream) StreamCopy(dst, src, bytes);
        else memcpy(dst, src, bytes);
        return;
    }
    const int parts = (int)std::min<size_t>(16, bytes / (min_parallel / 2));
    const size_t per = CopyPartBytes(bytes, parts);
    pool.Run(parts, [&](int i) {
        const size_t lo = (size_t)i * per;
        if (lo >= bytes) return;
        if (stream) StreamCopy(dst + lo, src + lo, std::min(per, bytes - lo));
        else memcpy(dst + lo, src + lo, std::min(per, bytes - lo));
    });
}

}  // namespace rdc_amd
