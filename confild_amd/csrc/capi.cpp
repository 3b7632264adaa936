// Library-wide C ABI helpers: thread-local error text and the build tag.
#include <string>

#include "common.hpp"

namespace cfd {
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
}  // namespace cfd

extern "C" const char* cfd_last_error(void) { return cfd::g_last_error.c_str(); }

extern "C" const char* cfd_version(void) {
    return "libconfild_hip gfx950 r6 (split-f16 / bf16 / fp32 MFMA; native sampler graphs; planned batch; CU-range streams; split-f16 DPS tape; key-chunked attention)";
}
