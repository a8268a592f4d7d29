// Host side of the row digests (include/mcroute.h mc_host_digest / mc_host_digest2): the same
// sum the device forms for every fetched row (kernels.hip row_digests), so the drop-in API can
// tell whether a yielded array was edited in place.  Host-only code, built by the host C++
// compiler (its inner loop multiversioned for the widest vector unit of the machine).
#include "digest.hpp"

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <mutex>
#include <thread>
#include <vector>

namespace mcr {
namespace {

// Host row digests (mc_host_digest): the device's row_digests sum, formed over column blocks
// by a small persistent pool.  The drop-in API checks two Texas rows (3 MB) after every yielded
// step; workers spin briefly between jobs (the next step's check follows within ~0.1 ms), then
// sleep on a condition variable.
class DigestPool {
  public:
    static DigestPool& get() {
        static DigestPool pool;
        return pool;
    }
    // rows given by pointers (the drop-in API checks a step's outflow and inflow rows, which
    // live in different fetched blocks, in one call)
    void run_rows(const double* const* rows, int64_t nrows, int64_t n, uint64_t* out) {
        std::lock_guard<std::mutex> call(call_mu_);
        const int parts = (nrows * n < (1 << 15) || workers_.empty())
                              ? 1 : (int)workers_.size() + 1;
        rows_ = rows;
        nrows_ = nrows;
        n_ = n;
        parts_ = parts;
        partial_.assign((size_t)parts * (size_t)nrows, 0);
        if (parts > 1) {
            pending_.store(parts - 1, std::memory_order_relaxed);
            {
                std::lock_guard<std::mutex> lk(mu_);
                gen_.fetch_add(1, std::memory_order_release);
            }
            cv_.notify_all();
        }
        block(0);
        while (parts > 1 && pending_.load(std::memory_order_acquire) != 0) {
        }
        for (int64_t r = 0; r < nrows; ++r) {
            uint64_t h = 0;
            for (int p = 0; p < parts; ++p) h += partial_[(size_t)p * nrows + r];
            out[r] = h;
        }
    }
    ~DigestPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
            gen_.fetch_add(1, std::memory_order_release);
        }
        cv_.notify_all();
        for (std::thread& t : workers_) t.join();
    }

  private:
    DigestPool() {
        int want = 8;
        if (const char* e = std::getenv("MCR_DIGEST_THREADS")) want = std::atoi(e);
        else if (const char* e2 = std::getenv("OMP_NUM_THREADS")) want = std::min(8, std::atoi(e2));
        const int hw = (int)std::thread::hardware_concurrency();
        want = std::max(1, std::min(want, hw > 0 ? hw : 1));
        for (int t = 1; t < want; ++t) workers_.emplace_back([this, t] { work(t); });
    }
    void block(int p) {
        const int64_t j0 = n_ * p / parts_, j1 = n_ * (p + 1) / parts_;
        for (int64_t r = 0; r < nrows_; ++r)
            partial_[(size_t)p * nrows_ + r] =
                digest_span(reinterpret_cast<const uint64_t*>(rows_[r]), j0, j1);
    }
    // the inner sum, compiled for the host's widest vector unit (64-bit multiplies: AVX-512DQ
    // has them natively) and picked once at load time
    template <int V>
    static uint64_t span_impl(const uint64_t* row, int64_t j0, int64_t j1) {
        uint64_t h = 0, jk = (uint64_t)j0 * kDigestK1;   // j * K1, strength-reduced
        for (int64_t j = j0; j < j1; ++j, jk += kDigestK1) {
            uint64_t t = (row[j] ^ jk) * kDigestK2;
            h += t ^ (t >> 29);
        }
        return h;
    }
    __attribute__((target("avx512f,avx512dq,avx512vl")))
    static uint64_t span_avx512(const uint64_t* row, int64_t j0, int64_t j1) {
        uint64_t h = 0, jk = (uint64_t)j0 * kDigestK1;   // j * K1, strength-reduced
        for (int64_t j = j0; j < j1; ++j, jk += kDigestK1) {
            uint64_t t = (row[j] ^ jk) * kDigestK2;
            h += t ^ (t >> 29);
        }
        return h;
    }
    __attribute__((target("avx2")))
    static uint64_t span_avx2(const uint64_t* row, int64_t j0, int64_t j1) {
        uint64_t h = 0, jk = (uint64_t)j0 * kDigestK1;   // j * K1, strength-reduced
        for (int64_t j = j0; j < j1; ++j, jk += kDigestK1) {
            uint64_t t = (row[j] ^ jk) * kDigestK2;
            h += t ^ (t >> 29);
        }
        return h;
    }
    using SpanFn = uint64_t (*)(const uint64_t*, int64_t, int64_t);
    static SpanFn pick_span() {
        __builtin_cpu_init();
        if (__builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512dq") &&
            __builtin_cpu_supports("avx512vl"))
            return &span_avx512;
        if (__builtin_cpu_supports("avx2")) return &span_avx2;
        return &span_impl<0>;
    }
    static uint64_t digest_span(const uint64_t* row, int64_t j0, int64_t j1) {
        static const SpanFn fn = pick_span();
        return fn(row, j0, j1);
    }
    void work(int p) {
        uint64_t seen = 0;
        for (;;) {
            uint64_t g = gen_.load(std::memory_order_acquire);
            if (g == seen) {
                const auto t0 = std::chrono::steady_clock::now();
                while ((g = gen_.load(std::memory_order_acquire)) == seen &&
                       std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(300)) {
                }
                if (g == seen) {
                    std::unique_lock<std::mutex> lk(mu_);
                    cv_.wait(lk, [&] { return gen_.load(std::memory_order_acquire) != seen; });
                    g = gen_.load(std::memory_order_acquire);
                }
            }
            seen = g;
            if (stop_) return;
            if (p < parts_) block(p);
            pending_.fetch_sub(1, std::memory_order_acq_rel);
        }
    }
    std::mutex call_mu_, mu_;
    std::condition_variable cv_;
    std::vector<std::thread> workers_;
    std::atomic<uint64_t> gen_{0};
    std::atomic<int> pending_{0};
    bool stop_ = false;
    const double* const* rows_ = nullptr;
    int64_t nrows_ = 0, n_ = 0;
    int parts_ = 1;
    std::vector<uint64_t> partial_;
};

}  // namespace

void host_digest_rows(const double* const* rows, int64_t nrows, int64_t n, uint64_t* out) {
    DigestPool::get().run_rows(rows, nrows, n, out);
}

}  // namespace mcr
