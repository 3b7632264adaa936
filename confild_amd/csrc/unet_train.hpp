// Launch interface of the U-Net parameter-gradient kernels (unet_train.hip, K11).
#pragma once
#include "common.hpp"

namespace cfd {

// convolution weight gradient: dY (P = B Hout Wout, Cout) against the im2col of
// the forward input (two sources; optional GroupNorm affine (+ SiLU) from ss)
struct WgradArgs {
    const float* dy;
    const float* src1;
    const float* src2;
    const float* ss;     // (B, Ctot, 2) forward GroupNorm scale / shift, or null (raw input)
    float* part;         // scratch: wgrad_part_floats(a) floats (<= part_cap)
    float* act;          // scratch (B, Hin, Win, Ctot) for the activated input of the 128-tile path, or null
    int64_t P, kspan, part_cap;
    int C1, C2, Ctot, Cout;
    int Hin, Win, Hout, Wout;
    int ks, stride, pad, up, silu;
    // split-f16 kernel: the two operand ranges (max |dY|, max |X| as float bits),
    // each in a zeroed slot of its own (null: the exact fp32 kernel).  ymax_known:
    // amax_y already holds max |dY| (written by the pass that produced dY), so no
    // range pass over dY runs.  amax_out: where gn_act reduces max |X| (internal)
    unsigned* amax_y;
    unsigned* amax_x;
    int ymax_known;
    int xmax_known;   // amax_x already holds max |X| (the forward GroupNorm kept X and its range)
    unsigned* amax_out;
    // optional: the bias gradient (sum of dY over the pixels) from the split
    // product kernel's dY loads -- bpart scratch (slices x Cout floats), Gb += it.
    // launch_conv_wgrad returns whether it took it (else the caller sums dY)
    float* bpart;
    int64_t bpart_cap;
    float* Gb;
};


// pixel slice of one block (P, Cout, Ctot, ks and part_cap of a set)
int64_t wgrad_kspan(const WgradArgs& a);
size_t wgrad_part_floats(const WgradArgs& a);
// G (Cout, Ctot, ks, ks) += dW; returns true when it also added the bias gradient
// into a.Gb (the split kernel with a.bpart / a.Gb set)
bool launch_conv_wgrad(WgradArgs a, float* G, hipStream_t st);
size_t colsum_part_floats(int64_t n, int64_t F, int R);
// out (R, F) = per-row-group column sums of X (R groups of n rows of F)
void launch_colsum(const float* X, int64_t n, int64_t F, int R, float* part, float* out, hipStream_t st);
// G (F) += sum of the R rows of rows (R, F)
void launch_rows_accum(const float* rows, int R, int64_t F, float* G, hipStream_t st);
// dgamma / dbeta += the (nparts, Ctot, 2) partials in part order (gn_bwd_partial's PP form)
void launch_gn_param_accum(const float* part, int nparts, int Ctot, float* dgamma, float* dbeta, hipStream_t st);
void launch_linear_wgrad(const float* d, const float* a, int B, int K, int N, int act, float* GW, float* Gb,
                         hipStream_t st);
void launch_linear_dgrad(const float* d, const float* W, const float* x, int B, int K, int N, int act, int accumulate,
                         float* da, hipStream_t st);

}  // namespace cfd
