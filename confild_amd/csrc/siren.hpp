// Shared pieces of the fused SIREN decoders (siren.hip: exact fp32 MFMA chain;
// siren_split.hip: fp32-accurate split-f16 MFMA chain).
#pragma once
#include <type_traits>
#include <utility>

#include "common.hpp"

namespace cfd {

// Compile-time loop: f(std::integral_constant<int, I>) for I in [0, N).  Keeps
// every register-array index static (a runtime index sends the array to scratch).
template <int N, class F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
    static_for_impl<N>(f, std::make_integer_sequence<int, N>{});
}

struct SirenArgs {
    const float* w0;      // (H, d)            net1.0.weight
    const float* wimg;    // nh * NB blocks of NB*256 floats (packed hidden weights)
    const float* wout;    // (c, H)            net1.{nh+1}.weight
    const float* bout;    // (c)               net1.{nh+1}.bias
    const float* film;    // (b, nh+1, H)      b_i + V_i z
    const float* coords;  // (N, d)
    const float* xmax;
    const float* xmin;
    const float* ymax;
    const float* ymin;
    float* out;           // (b, N, c)
    const float* wscale;  // (nh) power-of-two weight scale of each hidden layer (split-f16 image only)
    const float* wimg_rev; // siren_split32 image of the hidden weights pre-scaled by (w0 / 2pi) s'_i (HWSIN >= 3)
    const float* wrev;     // (2 nh): FiLM scale (w0 / 2pi) s'_i of each hidden layer, then 1 / s'_i
    int64_t N;
    int64_t ystride;
    int64_t b0;           // first latent of this launch (grid.y chunking)
    int d, c, nh;
    float w0f;
    unsigned long long* stamps;   // development (CFD_STAMPS builds): timestamp buffer, else null
};
// Tape kernels of the DPS adjoint and the CNF training backward (siren.hip):
// pre-activations u and deltas of every layer for P = R x Ns (row, sensor) pairs
struct SirenTapeArgs {
    const float* w0;      // (H, d)
    const float* wimg;    // forward weight image (as SirenArgs)
    const float* wimg_t;  // transposed image, layers nh..1: img[j][q][lane][s] = W_i[16q+4g+s][16j+(lane&15)]
    const float* wout;    // (c, H)
    const float* bout;    // (c)
    const float* film;    // (R, nh+1, H)
    const float* coords;  // (Ns, d)
    const float* xmax;
    const float* xmin;
    const float* ymax;
    const float* ymin;
    float* u;             // (P, nh+1, H) tape
    float* delta;         // (P, nh+1, H)
    float* out;           // (P, c)
    const float* gout;    // (P, c)
    const float* wimg16;  // split-f16 image of the hidden weights (pack_split_f16), null: fp32 tape
    const float* wimg16t; // split-f16 image of their transposes, layers nh..1 (pack_split_f16t)
    const float* wscale;  // (nh) the power-of-two scale of both images
    int64_t P;
    int64_t ystride;
    int Ns, d, c, nh;
    float w0f;
};
// the CFD_STAMPS build's timestamp buffer (unet_kernels.hip; null: off)
unsigned long long* stamps_buf();

// LDS-DMA of one weight block (NB pieces of 1 KiB) into an LDS ring slot: one
// global_load_lds_dwordx4 wave-instruction per piece, pieces spread over the waves.
template <int NB, int WAVES>
__device__ __forceinline__ void siren_issue_block(const float* __restrict__ wimg, int J, float* dst,
                                                  int wave, int lane) {
    constexpr int BLK = NB * 256;
    // J through readfirstlane: keeps the block base a scalar (else the compiler
    // precomputes one 64-bit VGPR address per unrolled block)
    const float* src = wimg + (int64_t)__builtin_amdgcn_readfirstlane(J) * BLK;
    for (int piece = wave; piece < NB; piece += WAVES) {
        __builtin_amdgcn_global_load_lds((const void*)(src + piece * 256 + lane * 4),
                                         (__attribute__((address_space(3))) void*)(dst + piece * 256),
                                         16, 0, 0);
    }
}

// The same with the piece loop unrolled (NB % WAVES == 0: NB / WAVES pieces per
// wave, a compile-time count, so the compiler's vmcnt accounting stays exact
// across the issue instead of falling back to vmcnt(0) at the next use of an
// earlier load)
template <int NB, int WAVES>
__device__ __forceinline__ void siren_issue_block_u(const float* __restrict__ wimg, int J, float* dst,
                                                    int wave, int lane) {
    static_assert(NB % WAVES == 0, "whole pieces per wave");
    constexpr int BLK = NB * 256;
    const float* src = wimg + (int64_t)__builtin_amdgcn_readfirstlane(J) * BLK;
    static_for<NB / WAVES>([&](auto mc) {
        constexpr int m = decltype(mc)::value;
        const int piece = wave + m * WAVES;
        __builtin_amdgcn_global_load_lds((const void*)(src + piece * 256 + lane * 4),
                                         (__attribute__((address_space(3))) void*)(dst + piece * 256), 16, 0, 0);
    });
}

// Split-f16 chain (siren_split.hip).  Defined for even NB (H a multiple of 32).
bool siren_split_supported(int NB);
void launch_siren_split(int NB, SirenArgs a, int b, hipStream_t st);
// 32x32x16 form of the chain (K7t, image from pack_split_f16_32)
bool siren_split32_supported(int H, int nh);
void launch_siren_split32(int H, SirenArgs a, int b, hipStream_t st);
// split-f16 K-split tape kernels (K9t, siren_split.hip): null when NB has no form
bool tape_split_supported(int NB);
void launch_tape_split(int NB, const SirenTapeArgs& a, bool bwd, hipStream_t st);

}  // namespace cfd
