// hvws_hostpool.cpp -- a small host thread pool for the byte copies around
// the batched drop-in (hvws_feed_many's gather into / scatter out of the
// pinned stage, hvws_rx_batch's pageable-buffer staging).  One core moves
// ~8-10 GB/s through memcpy; at thousands of 8 KiB reads per poll iteration
// those copies, not the GPU, set the iteration time (profiles/r2aa_raw).
//
// One pool per process, shared by every thread context: a caller that finds
// it busy copies on its own thread instead of queueing.  $HVWS_COPY_THREADS
// sets the width (default 8, 1 = always serial).
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "hvws_internal.h"

namespace hvws {
namespace {

class host_pool {
  public:
    explicit host_pool(int width) : width_(width) {
        for (int t = 1; t < width_; ++t) threads_.emplace_back([this] { worker(); });
        for (std::thread& t : threads_) t.detach();   // parked on cv_ until the process ends
    }
    int width() const { return width_; }

    // false when another caller holds the pool: the caller runs serially.
    bool run(int n, const std::function<void(int)>& fn) {
        std::unique_lock<std::mutex> own(busy_, std::try_to_lock);
        if (!own.owns_lock()) return false;
        {
            std::lock_guard<std::mutex> lk(m_);
            job_ = &fn;
            njob_ = n;
            next_.store(0);
            active_ = (int)threads_.size();
            ++gen_;
        }
        cv_.notify_all();
        drain(fn, n);
        std::unique_lock<std::mutex> lk(m_);
        done_.wait(lk, [this] { return active_ == 0; });
        job_ = nullptr;
        return true;
    }

  private:
    void drain(const std::function<void(int)>& fn, int n) {
        for (int i = next_.fetch_add(1); i < n; i = next_.fetch_add(1)) fn(i);
    }
    void worker() {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(int)>* fn;
            int n;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return gen_ != seen; });
                seen = gen_;
                fn = job_;
                n = njob_;
            }
            drain(*fn, n);
            std::lock_guard<std::mutex> lk(m_);
            if (--active_ == 0) done_.notify_one();
        }
    }

    const int width_;
    std::vector<std::thread> threads_;
    std::mutex busy_, m_;
    std::condition_variable cv_, done_;
    const std::function<void(int)>* job_ = nullptr;
    int njob_ = 0;
    int active_ = 0;
    uint64_t gen_ = 0;
    std::atomic<int> next_{0};
};

std::mutex g_pool_m;
host_pool* g_pool = nullptr;   // leaked on purpose: workers stay parked until exit
pid_t g_pool_pid = 0;

host_pool* pool() {
    std::lock_guard<std::mutex> lk(g_pool_m);
    if (!g_pool || g_pool_pid != getpid()) {   // a forked child has none of the parent's threads
        int w = 8;
        if (const char* e = getenv("HVWS_COPY_THREADS")) w = atoi(e);
        w = w < 1 ? 1 : (w > 64 ? 64 : w);
        g_pool = new host_pool(w);
        g_pool_pid = getpid();
    }
    return g_pool;
}

}  // namespace

int copy_width() { return pool()->width(); }

void par_for(int n, const std::function<void(int)>& fn) {
    if (n <= 0) return;
    if (n == 1 || pool()->width() == 1 || !pool()->run(n, fn))
        for (int i = 0; i < n; ++i) fn(i);
}

void par_memcpy(void* dst, const void* src, uint64_t n) {
    const int w = n >= kParCopyMin ? copy_width() : 1;
    if (w <= 1) {
        memcpy(dst, src, n);
        return;
    }
    const uint64_t piece = ((n + w - 1) / w + 4095) & ~4095ull;
    const int parts = (int)((n + piece - 1) / piece);
    par_for(parts, [&](int i) {
        const uint64_t o = (uint64_t)i * piece;
        memcpy((char*)dst + o, (const char*)src + o, n - o < piece ? n - o : piece);
    });
}

}  // namespace hvws
