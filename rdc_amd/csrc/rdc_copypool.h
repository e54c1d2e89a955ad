// A small pool of host threads that run the items 0..n-1 of a job together
// with the caller (the host path's pageable <-> pinned copies, rdc_host.cpp).
// Standard C++ only, so tests/cpp/copypool_stress.cc builds it without HIP.
#pragma once
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

}  // namespace rdc_amd
