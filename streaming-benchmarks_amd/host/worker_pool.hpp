// worker_pool.hpp -- threads that stay up for the owner's lifetime (the file source's readers,
// the streaming job's slot fillers): run(n, f) calls f(t) for t in [0, n) on n threads (the
// caller's is t = 0) and returns when all are done.
#pragma once

#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace ysb {
namespace topology {

class WorkerPool {
public:
    explicit WorkerPool(unsigned n) {
        for (unsigned t = 1; t < n; ++t) th_.emplace_back([this, t] { loop(t); });
    }
    ~WorkerPool() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& x : th_) x.join();
    }
    unsigned size() const { return (unsigned)th_.size() + 1; }
    // f(t) for t in [0, n), n <= size(); t = 0 on the calling thread
    void run(unsigned n, const std::function<void(unsigned)>& f) {
        if (n <= 1) { f(0u); return; }
        {
            std::lock_guard<std::mutex> g(m_);
            job_ = &f;
            active_ = n;
            left_ = n - 1;
            ++gen_;
        }
        cv_.notify_all();
        f(0u);
        std::unique_lock<std::mutex> g(m_);
        done_.wait(g, [this] { return left_ == 0; });
        job_ = nullptr;
    }

private:
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    const std::function<void(unsigned)>* job_ = nullptr;
    unsigned active_ = 0, left_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
    void loop(unsigned t) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(unsigned)>* f;
            {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                if (t >= active_) continue;
                f = job_;
            }
            (*f)(t);
            std::lock_guard<std::mutex> g(m_);
            if (--left_ == 0) done_.notify_all();
        }
    }
};

}  // namespace topology
}  // namespace ysb
