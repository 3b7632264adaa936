// Launch interface of the U-Net kernels (unet_kernels.hip).
#pragma once
#include "common.hpp"

namespace cfd {

struct GnArgs {
    const float* src1;
    const float* src2;  // second (concatenated) source or null
    const float* gamma;
    const float* beta;
    double* part;       // (B, nchunks, 32, 2) partial sums
    float* ss;          // (B, Ctot, 2) scale / shift
    float* out;         // (B, HW, Ctot) normalised (+ SiLU) activation
    int C1, C2, Ctot, HW;
    float eps;
    int silu;
    int nchunks;
    int B;
};

struct ConvArgs {
    const float* src1;
    const float* src2;   // concat-free second source (channels C1..C1+C2) or null
    const float* w;      // packed (Cout, ks*ks, Ctot)
    const float* bias;   // (Cout)
    const float* emb;    // (B, emb_stride) slice, or null
    const float* res;    // (M, Cout) residual, or null
    float* out;          // (M, Cout)
    float* part;         // split-K partial slab (splits, M, Cout), or null
    int C1, C2, Ctot;
    int Hin, Win, Hout, Wout;
    int stride, ks, pad, up;
    int Cout;
    int emb_stride;
    int M, K;
};

struct AttnArgs {
    const float* qkv;  // (B, T, 3C)
    float* out;        // (B, T, C)
    int T, C;
    float scale;       // 1/sqrt(sqrt(ch)), applied to q and k separately
};

struct ConvPlan {
    int bm = 128, bn = 128, splits = 1;
};

int gn_chunks(int HW);
// GroupNorm statistics + normalise (+SiLU) into a.out
void launch_gn(const GnArgs& a, int B, hipStream_t st);
ConvPlan plan_conv(const ConvArgs& a, size_t part_cap_floats);
void launch_conv(const ConvArgs& a, const ConvPlan& p, hipStream_t st);
void launch_conv_in(const ConvArgs& a, hipStream_t st);
void launch_conv_out(const ConvArgs& a, hipStream_t st);
void launch_attention(const AttnArgs& a, int CH, int heads, int B, hipStream_t st);
void launch_temb(const int64_t* t, const float* freqs, float* out, int dim, int B, hipStream_t st);
void launch_linear(const float* x, const float* W, const float* bias, float* y, int B, int K, int N, int act,
                   hipStream_t st);

}  // namespace cfd
