// A fixed set of host worker threads that run one indexed job at a time (the uploader's gather,
// seedgen.hip upload_pack). Spawning the gather threads per frame started the last of them ~0.15 ms after
// the first; parked workers are woken together.
#pragma once
#include <sched.h>

#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace aos {

// CPUs of the calling thread's affinity set (read once: the first call comes from the thread that created the
// handle); the library sizes its host thread pools to at most this (a bench that pins its CPU baseline child to one of
// the process's cores leaves the process one core fewer: 16 gather threads on 15 cores stretched the upload's tail).
inline int host_cpu_share() {
    static const int n = [] {
        cpu_set_t set;
        CPU_ZERO(&set);
        if (sched_getaffinity(0, sizeof(set), &set) != 0) return 16;
        return CPU_COUNT(&set) > 0 ? CPU_COUNT(&set) : 1;
    }();
    return n;
}

class HostPool {
  public:
    HostPool() = default;
    HostPool(const HostPool &) = delete;
    HostPool &operator=(const HostPool &) = delete;
    ~HostPool() { stop(); }

    // f(0 .. n - 1): f(0) on the calling thread, f(i) on worker i; returns when every call has returned.
    // One caller at a time. f must not throw (callers catch per index).
    void run(int n, const std::function<void(int)> &f) {
        if (n <= 1) { if (n == 1) f(0); return; }
        ensure(n - 1);
        {
            std::lock_guard<std::mutex> lk(mu_);
            job_ = &f;
            n_ = n;
            pending_ = n - 1;
            ++gen_;
        }
        cv_.notify_all();
        f(0);
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [&] { return pending_ == 0; });
        job_ = nullptr;
    }

    void stop() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            quit_ = true;
        }
        cv_.notify_all();
        for (std::thread &t : th_) t.join();
        th_.clear();
        quit_ = false;
    }

  private:
    void ensure(int workers) {
        while ((int)th_.size() < workers) {
            const int id = (int)th_.size() + 1;
            th_.emplace_back([this, id] { loop(id); });
        }
    }
    void loop(int id) {
        uint64_t seen = 0;
        {
            std::lock_guard<std::mutex> lk(mu_);
            seen = gen_;   // (a worker created for this job is counted in pending_ and catches up below)
            if (job_ && id < n_) seen = gen_ - 1;
        }
        for (;;) {
            const std::function<void(int)> *f;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return quit_ || gen_ != seen; });
                if (quit_) return;
                seen = gen_;
                if (id >= n_) continue;
                f = job_;
            }
            (*f)(id);
            {
                std::lock_guard<std::mutex> lk(mu_);
                if (--pending_ == 0) done_.notify_one();
            }
        }
    }

    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    const std::function<void(int)> *job_ = nullptr;
    int n_ = 0, pending_ = 0;
    uint64_t gen_ = 0;
    bool quit_ = false;
};

}  // namespace aos
