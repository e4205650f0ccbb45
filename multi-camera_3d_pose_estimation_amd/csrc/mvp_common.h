// Shared internals of libmvpose.so: error capture across the C-ABI.
// Every exported entry point returns int (0 = OK, <0 = error) and never throws;
// the message of the last failure on the calling thread is kept for
// mvp_last_error().
#pragma once
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdarg>
#include <exception>
#include <string>

#include "../../include/mvpose.h"

namespace mvp {

void set_error(const char* fmt, ...);

struct Error : std::exception {
    int code;
    std::string msg;
    Error(int c, std::string m) : code(c), msg(std::move(m)) {}
    const char* what() const noexcept override { return msg.c_str(); }
};

[[noreturn]] void fail(int code, const char* fmt, ...);

inline void hip_check(hipError_t e, const char* what, const char* file, int line) {
    if (e != hipSuccess) fail(MVP_ERR_HIP, "%s failed at %s:%d: %s", what, file, line, hipGetErrorString(e));
}

}  // namespace mvp

#define MVP_HIP(x) ::mvp::hip_check((x), #x, __FILE__, __LINE__)
#define MVP_REQUIRE(cond, ...)                                   \
    do {                                                         \
        if (!(cond)) ::mvp::fail(MVP_ERR_ARG, __VA_ARGS__);      \
    } while (0)

// Wrap an exported function body: converts exceptions into codes + last error.
#define MVP_ABI_BEGIN try {
#define MVP_ABI_END                                              \
    return MVP_OK;                                               \
    }                                                            \
    catch (const ::mvp::Error& e) {                              \
        ::mvp::set_error("%s", e.msg.c_str());                   \
        return e.code;                                           \
    }                                                            \
    catch (const std::exception& e) {                            \
        ::mvp::set_error("internal error: %s", e.what());        \
        return MVP_ERR_INTERNAL;                                 \
    }                                                            \
    catch (...) {                                                \
        ::mvp::set_error("internal error: unknown exception");   \
        return MVP_ERR_INTERNAL;                                 \
    }
