// common.hpp -- error state, HIP checks, device buffers for libspimdecon.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/spimdecon.h"

namespace spimdecon {

// Error carried through the C++ layer; converted to a status code at the C-ABI.
struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

void set_last_error(const std::string& msg);
void clear_last_error();

[[noreturn]] inline void fail(int code, const std::string& msg) { throw Error(code, msg); }

#define SD_HIP(expr)                                                                   \
    do {                                                                               \
        hipError_t _e = (expr);                                                        \
        if (_e != hipSuccess)                                                          \
            ::spimdecon::fail(_e == hipErrorOutOfMemory ? SPIMDECON_ERR_OOM            \
                                                        : SPIMDECON_ERR_HIP,           \
                              std::string(#expr " failed: ") + hipGetErrorString(_e) + \
                                  " (" __FILE__ ":" + std::to_string(__LINE__) + ")"); \
    } while (0)

#define SD_CHECK(cond, code, msg)                     \
    do {                                              \
        if (!(cond)) ::spimdecon::fail((code), (msg)); \
    } while (0)

// Validates a device id (>= 0 and present).  There is no CPU fallback.
void check_device(int dev);

// Scoped hipSetDevice with restore.
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        SD_HIP(hipGetDevice(&prev));
        if (prev != dev) SD_HIP(hipSetDevice(dev));
    }
    ~DeviceGuard() {
        int cur = -1;
        if (hipGetDevice(&cur) == hipSuccess && cur != prev && prev >= 0) (void)hipSetDevice(prev);
    }
};

// Owning device allocation.
template <typename T>
struct DBuf {
    T* p = nullptr;
    size_t n = 0;
    DBuf() = default;
    explicit DBuf(size_t count) { alloc(count); }
    void alloc(size_t count) {
        release();
        n = count;
        if (count) SD_HIP(hipMalloc(reinterpret_cast<void**>(&p), count * sizeof(T)));
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    ~DBuf() { release(); }
    DBuf(const DBuf&) = delete;
    DBuf& operator=(const DBuf&) = delete;
    DBuf(DBuf&& o) noexcept : p(o.p), n(o.n) { o.p = nullptr; o.n = 0; }
    DBuf& operator=(DBuf&& o) noexcept {
        if (this != &o) { release(); p = o.p; n = o.n; o.p = nullptr; o.n = 0; }
        return *this;
    }
    size_t bytes() const { return n * sizeof(T); }
};

// Runs fn() converting exceptions to status codes + last-error message.
template <typename F>
int guarded(F&& fn) {
    try {
        clear_last_error();
        fn();
        return SPIMDECON_OK;
    } catch (const Error& e) {
        set_last_error(e.what());
        std::fprintf(stderr, "[spimdecon] %s\n", e.what());
        return e.code;
    } catch (const std::bad_alloc&) {
        set_last_error("host out of memory");
        return SPIMDECON_ERR_OOM;
    } catch (const std::exception& e) {
        set_last_error(e.what());
        std::fprintf(stderr, "[spimdecon] %s\n", e.what());
        return SPIMDECON_ERR_STATE;
    }
}

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

}  // namespace spimdecon
