// Error handling and device-buffer helpers shared by the C ABI translation units
// (capi.cpp: routing sessions; kalman.cpp: covariance propagation and the Kalman update).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <utility>
#include <new>
#include <stdexcept>
#include <string>

#include "mcroute.h"

namespace mcr {
namespace capi {

// message of the last failed call on this thread (mc_last_error)
inline thread_local std::string g_err;

struct Fail : std::runtime_error {
    int code;
    Fail(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define HIPC(expr)                                                                   \
    do {                                                                             \
        hipError_t e_ = (expr);                                                      \
        if (e_ != hipSuccess)                                                        \
            throw Fail(e_ == hipErrorOutOfMemory ? MC_E_NOMEM : MC_E_HIP,            \
                       std::string(#expr) + ": " + hipGetErrorString(e_));           \
    } while (0)

#define REQUIRE(cond, msg)                                                           \
    do {                                                                             \
        if (!(cond)) throw Fail(MC_E_INVALID, msg);                                  \
    } while (0)

template <class F>
int guarded(F&& f) {
    try {
        f();
        return MC_OK;
    } catch (const Fail& e) {
        g_err = e.what();
        return e.code;
    } catch (const std::bad_alloc&) {
        g_err = "host allocation failed";
        return MC_E_NOMEM;
    } catch (const std::exception& e) {
        g_err = e.what();
        return MC_E_INVALID;
    } catch (...) {
        g_err = "unknown error";
        return MC_E_INVALID;
    }
}

template <class T>
struct DBuf {
    T* p = nullptr;
    size_t cap = 0;
    DBuf() = default;
    DBuf(const DBuf&) = delete;
    DBuf& operator=(const DBuf&) = delete;
    ~DBuf() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    void reserve(size_t k) {
        if (k <= cap && p) return;
        release();
        HIPC(hipMalloc(reinterpret_cast<void**>(&p), std::max<size_t>(k, 1) * sizeof(T)));
        cap = std::max<size_t>(k, 1);
    }
    void upload(const T* src, size_t k, hipStream_t s) {
        reserve(k);
        if (k) HIPC(hipMemcpyAsync(p, src, k * sizeof(T), hipMemcpyHostToDevice, s));
    }
    void swap(DBuf& o) {
        std::swap(p, o.p);
        std::swap(cap, o.cap);
    }
};


}  // namespace capi
}  // namespace mcr
