// Shared helpers for libconfild_hip (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/confild.h"

typedef float f4 __attribute__((ext_vector_type(4)));

namespace cfd {

void set_error(const std::string& msg);

struct Error {
    int code;
    std::string msg;
};

// Throwing check used inside the library; the extern "C" wrappers convert the
// exception into a return code + cfd_last_error() text.
#define CFD_HIP(expr)                                                                  \
    do {                                                                               \
        hipError_t _e = (expr);                                                        \
        if (_e != hipSuccess)                                                          \
            throw ::cfd::Error{CFD_EHIP, std::string(#expr) + ": " + hipGetErrorString(_e)}; \
    } while (0)

#define CFD_REQUIRE(cond, code, msg)                                                   \
    do {                                                                               \
        if (!(cond)) throw ::cfd::Error{code, std::string(msg)};                       \
    } while (0)

template <class F>
int guard(F&& f) {
    try {
        f();
        return CFD_OK;
    } catch (const Error& e) {
        set_error(e.msg);
        return e.code;
    } catch (const std::exception& e) {
        set_error(e.what());
        return CFD_ESTATE;
    }
}

inline void check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) throw Error{CFD_EHIP, std::string(what) + ": " + hipGetErrorString(e)};
}

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Accurate fp32 sine: Cody-Waite reduction by pi in three fma steps (exact for
// |x| < 125), then a degree-9 odd minimax polynomial on [-pi/2, pi/2]
// (~3.5 ulp).  Larger arguments (never produced by SIREN-initialised weights,
// but possible with trained ones) take the library sinf path.
__device__ __forceinline__ float sin_cw(float x) {
    if (__builtin_expect(fabsf(x) >= 125.0f, 0)) return sinf(x);
    const float q = rintf(x * 0.318309886183790671538f);
    float r = fmaf(q, -3.1414794921875f, x);
    r = fmaf(q, -0.00011315941810607910156f, r);
    r = fmaf(q, -1.9841872589410058936e-09f, r);
    const float s = r * r;
    float u = 2.6083159809786593541503e-06f;
    u = fmaf(u, s, -0.0001981069071916863322258f);
    u = fmaf(u, s, 0.00833307858556509017944336f);
    u = fmaf(u, s, -0.166666597127914428710938f);
    float y = fmaf(s, u * r, r);
    const int qi = (int)q;
    return (qi & 1) ? -y : y;
}

}  // namespace cfd
