// Shared helpers for libconfild_hip (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/confild.h"

// Device-side index assertions of the bounds-checked build (make DEBUG=1 ->
// lib/libconfild_hip_debug.so, selected with CFD_LIB=libconfild_hip_debug.so):
// a failing check prints its site and traps the wave (the launch fails, the
// process sees a HIP error).  Compiled out of the shipped library.
#ifdef CFD_DEBUG
#define CFD_DASSERT(cond)                                                                         \
    do {                                                                                          \
        if (!(cond)) {                                                                            \
            printf("CFD_DASSERT failed %s:%d: %s (block %d,%d,%d thread %d)\n", __FILE__, __LINE__, #cond, \
                   (int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z, (int)threadIdx.x);         \
            __builtin_trap();                                                                     \
        }                                                                                         \
    } while (0)
#else
#define CFD_DASSERT(cond) ((void)0)
#endif

// In-kernel timestamps of the development build (make STAMPS=1 ->
// lib/libconfild_hip_stamps.so; tools/dev/stamps.py): wave 0 of a workgroup
// records (realtime, kind/launch/slot, block, shader clock) at named points of
// the small-batch kernels into a buffer set by cfd_stamps_set.  Vector atomics
// and vector stores only.  Compiled out of the shipped library.
#ifdef CFD_STAMPS
__device__ __forceinline__ void cfd_stamp(unsigned long long* buf, unsigned kind, unsigned seq, unsigned slot) {
    if (buf && threadIdx.x == 0) {
        const unsigned long long t = __builtin_amdgcn_s_memrealtime();
        const unsigned long long i = atomicAdd(buf, 1ULL);
        if (i < (1ull << 20)) {
            unsigned long long* r = buf + 8 + 8 * i;
            r[0] = t;
            r[1] = ((unsigned long long)kind << 56) | ((unsigned long long)seq << 24) | slot;
            r[2] = blockIdx.x + ((unsigned long long)blockIdx.y << 20) + ((unsigned long long)blockIdx.z << 40);
            r[3] = __builtin_amdgcn_s_memtime();
            // where the wave runs: HW_ID (hwreg 4: simd, cu, sh, se) and XCC_ID (hwreg 20), read-only
            r[4] = (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4) |
                   ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32);
        }
    }
}
#define CFD_STAMP(buf, kind, seq, slot) cfd_stamp(buf, kind, seq, slot)
#else
#define CFD_STAMP(buf, kind, seq, slot) ((void)0)
#endif

typedef float f4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8v __attribute__((ext_vector_type(8)));

namespace cfd {

// n / d for 0 <= n < 2^24, d >= 1, exact: a float multiply by r = RN(1/d) is
// within one of the quotient, then one correction each way.  ~6 instructions
// instead of the ~40 of an integer division by a runtime value -- the pixel
// tables of the convolution prologues (measured in-kernel: ~1.4 us of a small
// K1s launch was its table's divisions)
__device__ __forceinline__ int fdiv24(int n, int d, float r) {
    int q = (int)((float)n * r);
    const int rm = n - q * d;
    q += rm >= d ? 1 : 0;
    q -= rm < 0 ? 1 : 0;
    return q;
}
// tap / ks for the kernel sizes the convolutions use (3, 1, and the 4x4 and 2x2
// of the input-gradient packs) without an integer division
__device__ __forceinline__ int tap_row(int tap, int ks) {
    return ks == 3 ? (tap * 11) >> 5 : ks == 4 ? tap >> 2 : ks == 2 ? tap >> 1 : ks == 1 ? 0 : tap / ks;
}

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

// Makes `device` current for the scope and restores the caller's device on
// exit, so an entry point never changes the calling process's (or torch's)
// current HIP device.
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int device) {
        CFD_HIP(hipGetDevice(&prev));
        if (prev != device) CFD_HIP(hipSetDevice(device));
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
    DeviceGuard(const DeviceGuard&) = delete;
    DeviceGuard& operator=(const DeviceGuard&) = delete;
};

// fp32 sine, branch-free.  |x| < 39000: Cody-Waite reduction by pi with a
// 4-term split of pi (exact reduction in that range, the SLEEF single-precision
// scheme), then a degree-9 odd minimax polynomial on [-pi/2, pi/2] (~3.5 ulp).
// Beyond that (|w0 * preactivation| >= 39000, i.e. |preactivation| >= 1300,
// three orders of magnitude above what SIREN weights produce) the hardware
// v_sin_f32 result is selected; DESIGN.md states this range.
__device__ __forceinline__ float sin_cw(float x) {
    const float q = rintf(x * 0.318309886183790671538f);
    float r = fmaf(q, -3.140625f, x);
    r = fmaf(q, -0.0009670257568359375f, r);
    r = fmaf(q, -6.2771141529083251953e-07f, r);
    r = fmaf(q, -1.2154201256553420762e-10f, r);
    const float s = r * r;
    float u = 2.6083159809786593541503e-06f;
    u = fmaf(u, s, -0.0001981069071916863322258f);
    u = fmaf(u, s, 0.00833307858556509017944336f);
    u = fmaf(u, s, -0.166666597127914428710938f);
    const float y = fmaf(s, u * r, r);
    const unsigned sgn = ((unsigned)(int)q & 1u) << 31;  // negate for odd q
    const float v = __uint_as_float(__float_as_uint(y) ^ sgn);
    return fabsf(x) < 39000.0f ? v : __builtin_amdgcn_sinf(x * 0.159154943091895335768f);
}

// fp32 cosine, same scheme (SLEEF cosf_u35 reduction): x = r + q*pi/2 with q odd,
// cos(x) = -+sin(r); hardware v_cos_f32 beyond |x| >= 39000.
__device__ __forceinline__ float cos_cw(float x) {
    const float q = fmaf(2.0f, rintf(fmaf(x, 0.318309886183790671538f, -0.5f)), 1.0f);
    float r = fmaf(q, -1.5703125f, x);
    r = fmaf(q, -0.00048351287841796875f, r);
    r = fmaf(q, -3.13855707645416259765625e-07f, r);
    r = fmaf(q, -6.077100628276710381e-11f, r);
    const float s = r * r;
    float u = 2.6083159809786593541503e-06f;
    u = fmaf(u, s, -0.0001981069071916863322258f);
    u = fmaf(u, s, 0.00833307858556509017944336f);
    u = fmaf(u, s, -0.166666597127914428710938f);
    const float y = fmaf(s, u * r, r);
    const unsigned sgn = ((unsigned)(int)q & 2u) ? 0u : (1u << 31);  // q = 1 mod 4: -sin(r)
    const float v = __uint_as_float(__float_as_uint(y) ^ sgn);
    return fabsf(x) < 39000.0f ? v : __builtin_amdgcn_cosf(x * 0.159154943091895335768f);
}

}  // namespace cfd
