// K11: parameter gradients of the latent U-Net (the diffusion TrainLoop's
// backward, U/src/train_util.py:196-240 -> loss.backward() through
// UNetModel.forward, U/src/unet.py:634-663), fp32, on the tape of
// cfd_unet_forward_tape and the input-gradient walk of unet.hip:
//   conv_wgrad_kernel   dW[co][ci][tap] = sum over output pixels p of
//                       dY[p][co] * act(X[src(p, tap)][ci]) -- the convolution's
//                       weight gradient as a "TN" product over pixels with the
//                       im2col operand gathered on the fly (stride-2 / nearest-2x
//                       addressing, two concat sources, the GroupNorm affine
//                       (+ SiLU) of the forward's normalised input recomputed from
//                       the raw input and its scale / shift), fp32 MFMA 16x16x4,
//                       k (pixels) split into fixed slices added in order;
//   colsum_kernel       per-(sample) column sums (bias and emb gradients);
//   gn_param_kernel     GroupNorm gamma / beta gradients;
//   linear_*_kernel     time_embed / emb_layers (B rows);
//   ema_kernel          update_ema (U/src/nn.py:71-80).
// Every reduction runs in a fixed order: the gradients are deterministic.
#include <algorithm>

#include "unet_kernels.hpp"
#include "unet_train.hpp"

namespace cfd {

__device__ __forceinline__ float sigm_t(float x) {   // the forward SiLU's sigmoid (silu_f, unet_kernels.hip)
    return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * -1.44269504088896340736f));
}
__device__ __forceinline__ float silu_f(float x) { return x * sigm_t(x); }   // silu_f's exact arithmetic

// ---------------------------------------------------------------------------
// conv weight gradient, C[z][co][tap * Ctot + ci] over the slice z of pixels
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void conv_wgrad_kernel(WgradArgs a) {
    constexpr int T = 64;
    __shared__ float Xs[16][T + 4];
    __shared__ float Ys[16][T + 4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int m0 = blockIdx.y * T, n0 = blockIdx.x * T;
    const int N = a.ks * a.ks * a.Ctot, M = a.Cout;
    const int64_t kbeg = (int64_t)blockIdx.z * a.kspan, kend = min(a.P, kbeg + a.kspan);
    const int HWo = a.Hout * a.Wout;
    f4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    const int kr = tid >> 4, c4 = (tid & 15) * 4;
    for (int64_t k0 = kbeg; k0 < kend; k0 += 16) {
        const int64_t k = k0 + kr;
        const bool kin = k < kend;
        int b = 0, oy = 0, ox = 0;
        if (kin) {
            b = (int)(k / HWo);
            const int rem = (int)(k - (int64_t)b * HWo);
            oy = rem / a.Wout;
            ox = rem - oy * a.Wout;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int m = m0 + c4 + j, n = n0 + c4 + j;
            Xs[kr][c4 + j] = kin && m < M ? a.dy[k * M + m] : 0.f;
            float y = 0.f;
            if (kin && n < N) {
                const int tap = n / a.Ctot, ci = n - tap * a.Ctot;
                const int ty = tap / a.ks, tx = tap - ty * a.ks;
                int iy, ix;
                bool ok;
                if (a.up) {   // nearest-2x input: upsampled coordinate, then halved
                    iy = oy - a.pad + ty;
                    ix = ox - a.pad + tx;
                    ok = iy >= 0 && iy < 2 * a.Hin && ix >= 0 && ix < 2 * a.Win;
                    iy >>= 1;
                    ix >>= 1;
                } else {
                    iy = oy * a.stride - a.pad + ty;
                    ix = ox * a.stride - a.pad + tx;
                    ok = iy >= 0 && iy < a.Hin && ix >= 0 && ix < a.Win;
                }
                if (ok) {
                    const int64_t pix = ((int64_t)b * a.Hin + iy) * a.Win + ix;
                    float v = ci < a.C1 ? a.src1[pix * a.C1 + ci] : a.src2[pix * a.C2 + (ci - a.C1)];
                    if (a.ss) {   // the forward's GroupNorm affine (gn_apply_kernel's arithmetic) (+ SiLU)
                        const float* s = a.ss + ((int64_t)b * a.Ctot + ci) * 2;
                        v = v * s[0] + s[1];
                        if (a.silu) v = silu_f(v);
                    }
                    y = v;
                }
            }
            Ys[kr][c4 + j] = y;
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < 16; kk += 4) {
            float fa[2], fb[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) fa[i] = Xs[kk + (lane >> 4)][wm * 32 + 16 * i + (lane & 15)];
#pragma unroll
            for (int j = 0; j < 2; ++j) fb[j] = Ys[kk + (lane >> 4)][wn * 32 + 16 * j + (lane & 15)];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i], fb[j], acc[i][j], 0, 0, 0);
        }
        __syncthreads();
    }
    float* Cz = a.part + (int64_t)blockIdx.z * M * N;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int n = n0 + wn * 32 + 16 * j + (lane & 15);
            if (n >= N) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + wm * 32 + 16 * i + 4 * (lane >> 4) + r;
                if (m < M) Cz[(int64_t)m * N + n] = acc[i][j][r];
            }
        }
}

// The same product on 128 x 128 tiles when the tile's 128 columns lie in one tap
// (Ctot % 128 == 0, every level of the recipe U-Nets): the pixel decode is per
// row (32-bit), the input quads are float4 loads of one source (the activated copy
// `act` when the forward applied GroupNorm (+ SiLU), else the raw sources), the
// next 32-pixel slice is prefetched into registers while the MFMAs run on this one.
__global__ __launch_bounds__(256) void conv_wgrad128_kernel(WgradArgs a, const float* __restrict__ act) {
    constexpr int T = 128, KS = 32, RW = KS / 8;   // rows a thread stages: rq + 8 r
    __shared__ __attribute__((aligned(16))) float Xs[KS][T + 4];
    __shared__ __attribute__((aligned(16))) float Ys[KS][T + 4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int m0 = blockIdx.y * T, n0 = blockIdx.x * T;
    const int M = a.Cout, N = a.ks * a.ks * a.Ctot;
    const int tap = n0 / a.Ctot, ci0 = n0 - tap * a.Ctot;
    const int ty = tap / a.ks, tx = tap - ty * a.ks;
    const int kbeg = (int)(blockIdx.z * a.kspan), kend = (int)min(a.P, (int64_t)kbeg + a.kspan);   // P < 2^31
    const int HWo = a.Hout * a.Wout;
    const int cq = (tid & 31) * 4, rq = tid >> 5;   // column quad; rows rq + 8 r
    f4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    f4 xv[RW], yv[RW];
    auto load = [&](int k0) {
#pragma unroll
        for (int hh = 0; hh < RW; ++hh) {
            const int k = k0 + rq + 8 * hh;
            f4 x = f4{0.f, 0.f, 0.f, 0.f}, y = f4{0.f, 0.f, 0.f, 0.f};
            if (k < kend) {
                if (m0 + cq < M) x = *(const f4*)(a.dy + (int64_t)k * M + m0 + cq);
                const int b = k / HWo;
                const int rem = k - b * HWo;
                const int oy = rem / a.Wout, ox = rem - oy * a.Wout;
                int iy, ix;
                bool ok;
                if (a.up) {
                    iy = oy - a.pad + ty;
                    ix = ox - a.pad + tx;
                    ok = iy >= 0 && iy < 2 * a.Hin && ix >= 0 && ix < 2 * a.Win;
                    iy >>= 1;
                    ix >>= 1;
                } else {
                    iy = oy * a.stride - a.pad + ty;
                    ix = ox * a.stride - a.pad + tx;
                    ok = iy >= 0 && iy < a.Hin && ix >= 0 && ix < a.Win;
                }
                if (ok) {
                    const int64_t pix = ((int64_t)b * a.Hin + iy) * a.Win + ix;
                    const int ci = ci0 + cq;
                    if (act)
                        y = *(const f4*)(act + pix * a.Ctot + ci);
                    else
                        y = ci < a.C1 ? *(const f4*)(a.src1 + pix * a.C1 + ci)
                                      : *(const f4*)(a.src2 + pix * a.C2 + (ci - a.C1));
                }
            }
            xv[hh] = x;
            yv[hh] = y;
        }
    };
    load(kbeg);
    for (int k0 = kbeg; k0 < kend; k0 += KS) {
#pragma unroll
        for (int hh = 0; hh < RW; ++hh) {
            *(f4*)&Xs[rq + 8 * hh][cq] = xv[hh];
            *(f4*)&Ys[rq + 8 * hh][cq] = yv[hh];
        }
        __syncthreads();
        if (k0 + KS < kend) load(k0 + KS);
#pragma unroll
        for (int kk = 0; kk < KS; kk += 4) {
            float fa[4], fb[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) fa[i] = Xs[kk + (lane >> 4)][wm * 64 + 16 * i + (lane & 15)];
#pragma unroll
            for (int j = 0; j < 4; ++j) fb[j] = Ys[kk + (lane >> 4)][wn * 64 + 16 * j + (lane & 15)];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i], fb[j], acc[i][j], 0, 0, 0);
        }
        __syncthreads();
    }
    float* Cz = a.part + (int64_t)blockIdx.z * M * N;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int n = n0 + wn * 64 + 16 * j + (lane & 15);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + wm * 64 + 16 * i + 4 * (lane >> 4) + r;
                if (m < M) Cz[(int64_t)m * N + n] = acc[i][j][r];
            }
        }
}

// ---------------------------------------------------------------------------
// Split-f16 weight gradient (default where the 128-tile kernel applies): the same
// product dW[m][n] = sum over pixels k of dY[k][m] * X[k][n], on f16 matrix cores
// at fp32-level accuracy, as the forward convolutions run it:
// both operands are scaled by a power of two into the f16 range -- s_y from
// max|dY| and s_x from max|X| over the whole tensors (absmax_kernel, atomicMax of
// non-negative float bits: exact and order-free) -- and split x = hi + lo (hi =
// f16(x), lo = f16(x - hi), RNE); each product runs as lo.hi + hi.lo + hi.hi on
// v_mfma_f32_16x16x32_f16 with fp32 accumulation, and the sums are multiplied
// back by 1 / (s_x s_y) (exact).  Operands below 2^-14 of their tensor's maximum
// keep fewer bits in their halves, but their absolute error stays at the 2^-25
// level of the largest product they are summed with.
// Tiles: 128 output rows (Cout) x 128 columns (one tap's channels) per block, 4
// waves of 64 x 64; pixels in steps of 32 (one MFMA depth).  The operands are
// staged transposed, [row][pixel] f16 rows of 64 B (a thread: 4 rows x 4 pixels),
// in the K1s fragment layout; the next step's loads are in flight during the
// MFMAs.  Partial slabs and wgrad_accum_kernel as in the fp32 kernel.
// ---------------------------------------------------------------------------
// LDS byte offset of 16-B chunk `chunk` of operand row `row`: rows are permuted
// within each group of 16 (bits 0-1 <-> bits 2-3) and the chunk is XOR-swizzled by
// the row's low bits, so that both the transposing stores (a lane: rows 4q+i, one
// 8-B half-chunk) and the fragment reads (16 rows x one chunk) spread over all banks
__device__ __forceinline__ int wg_swz(int row, int chunk) {
    const int P = (row & ~15) | ((row & 3) << 2) | ((row >> 2) & 3);
    return P * 64 + ((chunk ^ row) & 3) * 16;
}
// hi = f16(s x), lo = f16(s x - hi) of 4 values, packed as 2 x (2 halfs)
__device__ __forceinline__ void wg_split4(f4 x, float s, uint2& hi, uint2& lo) {
    typedef _Float16 h2_ __attribute__((ext_vector_type(2)));
    typedef float f2_ __attribute__((ext_vector_type(2)));
    x *= s;
    hi.x = __builtin_bit_cast(unsigned, __builtin_convertvector((f2_){x[0], x[1]}, h2_));
    hi.y = __builtin_bit_cast(unsigned, __builtin_convertvector((f2_){x[2], x[3]}, h2_));
    asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=&v"(lo.x) : "v"(x[0]), "v"(hi.x));
    asm("v_fma_mixhi_f16 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "+v"(lo.x) : "v"(x[1]), "v"(hi.x));
    asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=&v"(lo.y) : "v"(x[2]), "v"(hi.y));
    asm("v_fma_mixhi_f16 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "+v"(lo.y) : "v"(x[3]), "v"(hi.y));
}
// power of two s with max * s in [2^14, 2^15) (1 for an all-zero tensor): the top
// of the f16 range, so the bulk of a heavy-tailed operand stays above the f16
// normal limit (2^-14) down to 2^-28 of its maximum -- hi.hi products reach 2^30
// and fp32 sums over P < 2^24 pixels 2^54, far inside fp32.  The exponent is
// clamped so s and 1/s stay normal (a tensor below 2^-111 keeps s = 2^126).
__device__ __forceinline__ float wg_scale(unsigned amax_bits) {
    const float m = __uint_as_float(amax_bits);
    if (!(m > 0.f) || !(m < 3.0e38f)) return 1.f;
    int e;
    (void)frexpf(m, &e);
    return ldexpf(1.f, min(15 - e, 126));
}

// max |x| over n floats (n % 4 == 0) into *out (atomicMax of the float bits)
__global__ __launch_bounds__(256) void absmax_kernel(const float* __restrict__ x, int64_t n4, unsigned* out) {
    float m = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
        const f4 v = *(const f4*)(x + 4 * i);
        m = fmaxf(m, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    __shared__ float wm[4];
    if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(out, __float_as_uint(fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]))));
}

// UP: the forward input was nearest-2x upsampled.  The block's 128 columns lie in
// one source (launch_conv_wgrad: act, or C1 % 128 == 0), chosen once per block;
// a thread's 4 pixels of a step are consecutive, decoded once and stepped; 32-bit
// element offsets (launch_conv_wgrad checks P * Cout and the sources' sizes).
template <bool UP>
__global__ __launch_bounds__(256) void conv_wgrad128_split_kernel(WgradArgs a, const float* __restrict__ act) {
    constexpr int T = 128, KS = 32;
    constexpr int PLANE = T * KS * 2;   // bytes of one f16 [128][32] plane
    __shared__ __attribute__((aligned(16))) char lds[2][4 * PLANE];   // stage: dY hi, dY lo, X hi, X lo
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int m0 = blockIdx.y * T, n0 = blockIdx.x * T;
    const int M = a.Cout, N = a.ks * a.ks * a.Ctot;
    const int tap = n0 / a.Ctot, ci0 = n0 - tap * a.Ctot;
    const int ty = tap / a.ks, tx = tap - ty * a.ks;
    const int kbeg = (int)(blockIdx.z * a.kspan), kend = (int)min(a.P, (int64_t)kbeg + a.kspan);   // P < 2^31
    const int HWo = a.Hout * a.Wout, Wo = a.Wout, Ho = a.Hout;
    const float sy = wg_scale(*a.amax_y), sx = wg_scale(*a.amax_x);
    const int q = tid >> 3, ko = tid & 7;   // rows 4q..4q+3 (both operands), pixels 4ko..4ko+3 of a step
    const float rhw = 1.0f / (float)HWo, rw = 1.0f / (float)Wo;   // fdiv24: P < 2^24 (launch_conv_wgrad)
    // this block's X columns: one source, its row stride and channel offset
    const float* xs;
    int xld, xc;
    if (act) {
        xs = act, xld = a.Ctot, xc = ci0;
    } else if (ci0 < a.C1) {
        xs = a.src1, xld = a.C1, xc = ci0;
    } else {
        xs = a.src2, xld = a.C2, xc = ci0 - a.C1;
    }
    xs += xc + 4 * q;
    const bool yrow = m0 + 4 * q < M;
    const float* ys = a.dy + m0 + 4 * q;
    const int iyo = UP ? ty - a.pad : ty - a.pad, ixo = UP ? tx - a.pad : tx - a.pad;
    const int Hlim = UP ? 2 * a.Hin : a.Hin, Wlim = UP ? 2 * a.Win : a.Win;
    f4 yv[4], xv[4];   // [pixel]: 4 rows each
    // bias gradient (a.bpart, the tap-0 column blocks): this thread's rows summed
    // over its pixels in load order, fp32
    const bool bias = a.bpart && blockIdx.x == 0;
    f4 bsum = f4{0.f, 0.f, 0.f, 0.f};
    auto load = [&](int k0) {
        const int kb = k0 + 4 * ko;          // the thread's first pixel; the next 3 follow it
        int b = fdiv24(kb, HWo, rhw);
        const int rem = kb - b * HWo;
        int oy = fdiv24(rem, Wo, rw), ox = rem - oy * Wo;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const int k = kb + p;
            if (p > 0) {                      // step to the next output pixel
                if (++ox == Wo) {
                    ox = 0;
                    if (++oy == Ho) oy = 0, ++b;
                }
            }
            f4 y = f4{0.f, 0.f, 0.f, 0.f}, x = f4{0.f, 0.f, 0.f, 0.f};
            if (k < kend) {
                if (yrow) y = *(const f4*)(ys + (unsigned)k * (unsigned)M);
                int iy = UP ? oy + iyo : oy * a.stride + iyo, ix = UP ? ox + ixo : ox * a.stride + ixo;
                if (iy >= 0 && iy < Hlim && ix >= 0 && ix < Wlim) {
                    if (UP) iy >>= 1, ix >>= 1;
                    const unsigned pix = ((unsigned)b * a.Hin + iy) * a.Win + ix;
                    x = *(const f4*)(xs + pix * (unsigned)xld);
                }
            }
            yv[p] = y;
            xv[p] = x;
        }
        if (bias) bsum = ((bsum + yv[0]) + yv[1]) + (yv[2] + yv[3]);
    };
    // transpose in registers: row r = 4q + i gets pixels 4ko..4ko+3 of both operands
    auto store = [&](int buf) {
        char* base = lds[buf];
        const int off0 = (ko & 1) * 8;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int off = wg_swz(4 * q + i, ko >> 1) + off0;
            uint2 hy, ly, hx, lx;
            wg_split4(f4{yv[0][i], yv[1][i], yv[2][i], yv[3][i]}, sy, hy, ly);
            wg_split4(f4{xv[0][i], xv[1][i], xv[2][i], xv[3][i]}, sx, hx, lx);
            *(uint2*)(base + off) = hy;
            *(uint2*)(base + PLANE + off) = ly;
            *(uint2*)(base + 2 * PLANE + off) = hx;
            *(uint2*)(base + 3 * PLANE + off) = lx;
        }
    };
    f4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    const int li = lane & 15, g = lane >> 4;
    if (kbeg < kend) {
        load(kbeg);
        store(0);
        __syncthreads();
        int cur = 0;
        for (int k0 = kbeg; k0 < kend; k0 += KS) {
            const bool more = k0 + KS < kend;
            if (more) load(k0 + KS);
            const char* base = lds[cur];
            h8v ah[4], al[4], bh[4], bl[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int off = wg_swz(wm * 64 + 16 * i + li, g);
                ah[i] = *(const h8v*)(base + off);
                al[i] = *(const h8v*)(base + PLANE + off);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int off = wg_swz(wn * 64 + 16 * j + li, g);
                bh[j] = *(const h8v*)(base + 2 * PLANE + off);
                bl[j] = *(const h8v*)(base + 3 * PLANE + off);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
                }
            if (more) store(cur ^ 1);
            __syncthreads();
            cur ^= 1;
        }
    }
    if (bias) {   // the 8 pixel lanes of a row quad (consecutive lanes) in lane order
#pragma unroll
        for (int o = 1; o < 8; o <<= 1) {
            f4 t;
#pragma unroll
            for (int e = 0; e < 4; ++e) t[e] = __shfl_xor(bsum[e], o);
            bsum = (ko & o) ? t + bsum : bsum + t;
        }
        if (ko == 0)
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (m0 + 4 * q + e < M) a.bpart[(int64_t)blockIdx.z * M + m0 + 4 * q + e] = bsum[e];
    }
    // 1/s_x and 1/s_y applied one after the other (each exact, a power of two in
    // the normal range): their product could leave the fp32 range where s_x s_y
    // does, and a flushed unscale would zero the gradient
    const float usx = 1.f / sx, usy = 1.f / sy;
    float* Cz = a.part + (int64_t)blockIdx.z * M * N;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int n = n0 + wn * 64 + 16 * j + li;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + wm * 64 + 16 * i + 4 * g + r;
                if (m < M) Cz[(int64_t)m * N + n] = (acc[i][j][r] * usx) * usy;
            }
        }
}

// act (B, Hin, Win, Ctot) = the forward's GroupNorm affine (+ SiLU) of the two
// sources, once per layer for conv_wgrad128_kernel (conv_wgrad_kernel's arithmetic)
__global__ __launch_bounds__(256) void gn_act_kernel(WgradArgs a, int64_t nquads) {
    float m = 0.f;
    const int cqn = a.Ctot / 4;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nquads; i += (int64_t)gridDim.x * 256) {
        const int64_t pix = i / cqn;
        const int c = (int)(i - pix * cqn) * 4;
        const int64_t b = pix / ((int64_t)a.Hin * a.Win);
        f4 v = c < a.C1 ? *(const f4*)(a.src1 + pix * a.C1 + c) : *(const f4*)(a.src2 + pix * a.C2 + (c - a.C1));
        const float* s = a.ss + (b * a.Ctot + c) * 2;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float x = v[j] * s[2 * j] + s[2 * j + 1];
            if (a.silu) x = silu_f(x);
            v[j] = x;
        }
        *(f4*)(a.act + pix * a.Ctot + c) = v;
        m = fmaxf(m, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
    }
    if (a.amax_out) {   // the split weight gradient's operand range: one atomic per workgroup
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
        __shared__ float wm[4];
        if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
        __syncthreads();
        if (threadIdx.x == 0) atomicMax(a.amax_out, __float_as_uint(fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]))));
    }
}

// Thin layers (the U-Net's 1-channel input and output convolutions: Ctot or
// Cout <= 4, 3x3 stride 1): the 64x64 tiles would be 1/16 to 1/64 occupied.
// Here a workgroup is 64 channels of the wide side x 16 pixel lanes; a thread
// keeps the narrow side's <= 4 x 9 sums in registers and walks every 16th pixel
// of the slice, four pixels' loads issued before their FMAs.  WIDE_OUT (input
// conv, Cout wide): the pixels are output pixels, dY read once and coalesced, the
// taps' narrow inputs broadcast.  Otherwise (output conv, Ctot wide): the pixels
// are INPUT pixels, X read once and coalesced, the <= 4 dY values of the output
// pixels each feeds broadcast.  The 16 lanes' sums are added in lane order, the
// slices by wgrad_accum_kernel in slice order (deterministic).
template <bool WIDE_OUT, int NN>
__global__ __launch_bounds__(1024) void conv_wgrad_thin_kernel(WgradArgs a) {
    constexpr int NPL = 16, U = NN == 1 ? 4 : 1;   // U: pixels whose loads are in flight together
    const int w = blockIdx.x * 64 + (threadIdx.x & 63), pl = threadIdx.x >> 6;   // wide channel, pixel lane
    const int wide = WIDE_OUT ? a.Cout : a.Ctot, narrow = WIDE_OUT ? a.Ctot : a.Cout;
    const int ks = a.ks, taps = ks * ks;
    const int N = taps * a.Ctot;
    const int64_t MN = (int64_t)a.Cout * N;
    const int64_t kbeg = (int64_t)blockIdx.z * a.kspan, kend = min(a.P, kbeg + a.kspan);
    const int H = a.Hout, W = a.Wout, HW = H * W;   // stride 1, no upsample: input = output geometry
    float acc[NN][9];
#pragma unroll
    for (int n = 0; n < NN; ++n)
#pragma unroll
        for (int t = 0; t < 9; ++t) acc[n][t] = 0.f;
    auto xval = [&](int64_t pix, int64_t b, int ci) -> float {   // the forward input (GroupNorm affine / SiLU)
        float v = ci < a.C1 ? a.src1[pix * a.C1 + ci] : a.src2[pix * a.C2 + (ci - a.C1)];
        if (a.ss) {
            const float* s = a.ss + (b * a.Ctot + ci) * 2;
            v = v * s[0] + s[1];
            if (a.silu) v = silu_f(v);
        }
        return v;
    };
    const bool on = w < wide;
    for (int64_t k0 = kbeg + pl; k0 < kend; k0 += NPL * U) {
        float wv[U];                 // the wide-side value of each pixel (dY or X)
        float nv[U][NN][9];          // the narrow-side value of each (pixel, narrow index, tap), 0 off-image
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t k = k0 + (int64_t)u * NPL;
            const bool kin = on && k < kend;
            const int64_t b = kin ? k / HW : 0;
            const int rem = (int)(k - b * HW), y = rem / W, x = rem - y * W;
            wv[u] = 0.f;
            if (kin) wv[u] = WIDE_OUT ? a.dy[k * a.Cout + w] : xval(k, b, w);
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                const int ty = t / 3, tx = t - 3 * ty;   // ks == 3 (ks == 1: t == 0 only, tap (0, 0))
                const int dy_ = ks == 3 ? ty - a.pad : 0, dx_ = ks == 3 ? tx - a.pad : 0;
                const int yy = WIDE_OUT ? y + dy_ : y - dy_, xx = WIDE_OUT ? x + dx_ : x - dx_;
                const bool ok = kin && t < taps && yy >= 0 && yy < H && xx >= 0 && xx < W;
                const int64_t q = (b * H + yy) * W + xx;
#pragma unroll
                for (int n = 0; n < NN; ++n)
                    nv[u][n][t] = ok && n < narrow ? (WIDE_OUT ? xval(q, b, n) : a.dy[q * a.Cout + n]) : 0.f;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int n = 0; n < NN; ++n)
#pragma unroll
                for (int t = 0; t < 9; ++t) acc[n][t] = fmaf(wv[u], nv[u][n][t], acc[n][t]);
    }
    // the 16 pixel lanes' sums, added in lane order.  NN = 4 makes this 144 KiB of
    // static LDS: it fits gfx950's 160 KiB per workgroup only (the library is built
    // for gfx950 alone; an older target's 64 KiB would fail to compile here)
    static_assert(sizeof(float) * NPL * 64 * NN * 9 <= 160 * 1024, "thin wgrad: LDS beyond gfx950's 160 KiB");
    __shared__ float red[NPL][64][NN * 9];
#pragma unroll
    for (int n = 0; n < NN; ++n)
#pragma unroll
        for (int t = 0; t < 9; ++t) red[pl][threadIdx.x & 63][n * 9 + t] = acc[n][t];
    __syncthreads();
    if (pl == 0 && on) {
        float* part = a.part + (int64_t)blockIdx.z * MN;
#pragma unroll
        for (int n = 0; n < NN; ++n)
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                if (n >= narrow || t >= taps) continue;
                float v = red[0][threadIdx.x][n * 9 + t];
                for (int l = 1; l < NPL; ++l) v += red[l][threadIdx.x][n * 9 + t];
                const int co = WIDE_OUT ? w : n, ci = WIDE_OUT ? n : w;
                part[(int64_t)co * N + t * a.Ctot + ci] = v;
            }
    }
}

// G[co][ci][tap] (the reference weight layout) += sum_z part[z][co][tap * Ctot + ci]
__global__ __launch_bounds__(256) void wgrad_accum_kernel(const float* __restrict__ part, int Cout, int Ctot, int taps,
                                                          int splits, float* __restrict__ G,
                                                          const float* __restrict__ bpart, float* __restrict__ Gb) {
    const int64_t MN = (int64_t)Cout * Ctot * taps;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // index in G
    if (bpart && i < Cout) {   // the bias gradient's slices in slice order
        float sb = bpart[i];
        for (int z = 1; z < splits; ++z) sb += bpart[(int64_t)z * Cout + i];
        Gb[i] = Gb[i] + sb;
    }
    if (i >= MN) return;
    const int64_t co = i / ((int64_t)Ctot * taps);
    const int rem = (int)(i - co * Ctot * taps), ci = rem / taps, tap = rem - ci * taps;
    const int64_t j = co * ((int64_t)taps * Ctot) + (int64_t)tap * Ctot + ci;
    float s = part[j];
    for (int z = 1; z < splits; ++z) s += part[z * MN + j];
    G[i] = G[i] + s;
}

// part[z][r][f] = sum over rows [z span, (z+1) span) of X[(r n + s) F + f]: a
// block per (slice, row group), threads over (row lane, column group of VW), the
// row lanes combined in order through LDS
template <int VW>
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ X, float* __restrict__ part, int64_t n,
                                                     int64_t F, int R, int64_t span) {
    typedef float vt __attribute__((ext_vector_type(VW)));
    const int z = blockIdx.x, r = blockIdx.y;
    const int G = (int)(F / VW);
    const int64_t s0 = (int64_t)z * span, s1 = min(n, s0 + span);
    const float* src = X + (int64_t)r * n * F;
    float* dst = part + ((int64_t)z * R + r) * F;
    if (G >= 256) {   // one row lane: every thread walks whole columns
        for (int cg = threadIdx.x; cg < G; cg += 256) {
            vt a0 = (vt)0.f, a1 = (vt)0.f;
            int64_t s = s0;
            for (; s + 1 < s1; s += 2) {
                a0 += *(const vt*)(src + s * F + cg * VW);
                a1 += *(const vt*)(src + (s + 1) * F + cg * VW);
            }
            if (s < s1) a0 += *(const vt*)(src + s * F + cg * VW);
            *(vt*)(dst + cg * VW) = a0 + a1;
        }
        return;
    }
    const int L = 256 / G, rl = threadIdx.x / G, cg = threadIdx.x - rl * G;
    __shared__ float red[256 * VW];
    vt a0 = (vt)0.f, a1 = (vt)0.f;
    if (rl < L) {
        int64_t s = s0 + rl;
        for (; s + L < s1; s += 2 * L) {
            a0 += *(const vt*)(src + s * F + cg * VW);
            a1 += *(const vt*)(src + (s + L) * F + cg * VW);
        }
        if (s < s1) a0 += *(const vt*)(src + s * F + cg * VW);
        *(vt*)(red + (rl * G + cg) * VW) = a0 + a1;
    }
    __syncthreads();
    for (int f = threadIdx.x; f < G * VW; f += 256) {
        float t = 0.f;
        for (int l = 0; l < L; ++l) t += red[l * G * VW + f];
        dst[f] = t;
    }
}

// out[r][f] = sum_z part[z][r][f] (a block per 64 columns of a row, 4 slice lanes
// combined in order)
__global__ __launch_bounds__(256) void colsum_reduce_kernel(const float* __restrict__ part, int R, int64_t F,
                                                            int splits, float* __restrict__ out) {
    const int r = blockIdx.y, zl = threadIdx.x >> 6;
    const int64_t f = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
    __shared__ float red[4][64];
    float a0 = 0.f, a1 = 0.f;
    if (f < F) {
        int z = zl;
        for (; z + 4 < splits; z += 8) {
            a0 += part[((int64_t)z * R + r) * F + f];
            a1 += part[((int64_t)(z + 4) * R + r) * F + f];
        }
        if (z < splits) a0 += part[((int64_t)z * R + r) * F + f];
    }
    red[zl][threadIdx.x & 63] = a0 + a1;
    __syncthreads();
    if (threadIdx.x < 64 && f < F)
        out[(int64_t)r * F + f] = (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
}
__global__ __launch_bounds__(256) void rows_accum_kernel(const float* __restrict__ rows, int R, int64_t F,
                                                         float* __restrict__ G) {
    const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= F) return;
    float s = rows[f];
    for (int r = 1; r < R; ++r) s += rows[r * F + f];
    G[f] = G[f] + s;
}

// dgamma[c] += sum over (sample, chunk) of part, dbeta likewise: a block per 32
// channels, 8 part lanes combined in order
__global__ __launch_bounds__(256) void gn_param_accum_kernel(const float* __restrict__ part, int nparts, int Ctot,
                                                             float* __restrict__ dgamma, float* __restrict__ dbeta) {
    const int pl = threadIdx.x >> 5, c = blockIdx.x * 32 + (threadIdx.x & 31);
    __shared__ float red[8][32][2];
    float s1 = 0.f, s2 = 0.f;
    if (c < Ctot)
        for (int k = pl; k < nparts; k += 8) {
            s1 += part[((int64_t)k * Ctot + c) * 2];
            s2 += part[((int64_t)k * Ctot + c) * 2 + 1];
        }
    red[pl][threadIdx.x & 31][0] = s1;
    red[pl][threadIdx.x & 31][1] = s2;
    __syncthreads();
    if (threadIdx.x < 32 && c < Ctot) {
        float t1 = 0.f, t2 = 0.f;
        for (int l = 0; l < 8; ++l) {
            t1 += red[l][threadIdx.x][0];
            t2 += red[l][threadIdx.x][1];
        }
        dgamma[c] = dgamma[c] + t1;
        dbeta[c] = dbeta[c] + t2;
    }
}

// Linear(K -> N) of B rows, backward: GW[n][k] += sum_b d[b][n] f(a[b][k]),
// Gb[n] += sum_b d[b][n]; f = SiLU when act (the layer's input is SiLU(a))
__global__ __launch_bounds__(256) void linear_wgrad_kernel(const float* __restrict__ d, const float* __restrict__ a,
                                                           int B, int K, int N, int act, float* __restrict__ GW,
                                                           float* __restrict__ Gb) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)N * K) return;
    const int n = (int)(i / K), k = (int)(i - (int64_t)n * K);
    float s = 0.f;
    for (int b = 0; b < B; ++b) {
        const float x = a[(int64_t)b * K + k];
        s += d[(int64_t)b * N + n] * (act ? silu_f(x) : x);
    }
    GW[i] = GW[i] + s;
    if (k == 0 && Gb) {
        float t = 0.f;
        for (int b = 0; b < B; ++b) t += d[(int64_t)b * N + n];
        Gb[n] = Gb[n] + t;
    }
}

// da[b][k] (+)= (sum_n d[b][n] W[n][k]) * (act ? SiLU'(x[b][k]) : 1): a block per
// (sample, 32 columns k), 8 lanes over n (coalesced rows of W) combined in order
__global__ __launch_bounds__(256) void linear_dgrad_kernel(const float* __restrict__ d, const float* __restrict__ W,
                                                           const float* __restrict__ x, int B, int K, int N, int act,
                                                           int accumulate, float* __restrict__ da) {
    const int b = blockIdx.y, nl = threadIdx.x >> 5, k = blockIdx.x * 32 + (threadIdx.x & 31);
    __shared__ float red[8][32];
    float s0 = 0.f, s1 = 0.f;
    if (k < K) {
        const float* dr = d + (int64_t)b * N;
        int n = nl;
        for (; n + 8 < N; n += 16) {
            s0 += dr[n] * W[(int64_t)n * K + k];
            s1 += dr[n + 8] * W[(int64_t)(n + 8) * K + k];
        }
        if (n < N) s0 += dr[n] * W[(int64_t)n * K + k];
    }
    red[nl][threadIdx.x & 31] = s0 + s1;
    __syncthreads();
    if (threadIdx.x < 32 && k < K) {
        float s = 0.f;
        for (int l = 0; l < 8; ++l) s += red[l][threadIdx.x];
        const int64_t i = (int64_t)b * K + k;
        if (act) {
            const float z = x[i], sg = sigm_t(z);
            s = s * (sg * (1.0f + z * (1.0f - sg)));
        }
        da[i] = accumulate ? da[i] + s : s;
    }
}

// update_ema: targ = targ * rate + src * (1 - rate)  (targ.mul_(rate).add_(src, alpha=1 - rate))
__global__ void ema_kernel(float* __restrict__ targ, const float* __restrict__ src, int64_t n, float rate,
                           float omr) {
#pragma clang fp contract(off)
    // update_ema's targ.mul_(rate).add_(src, alpha=1 - rate): torch's add-with-alpha
    // is one fused multiply-add on the rounded product (GPU and CPU kernels alike)
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) targ[i] = __builtin_fmaf(src[i], omr, targ[i] * rate);
}

// diffusion training loss (GaussianDiffusion.training_losses, MSE on eps,
// gaussian_diffusion.py:775-853): x_t = sqrt(abar_t) x0 + sqrt(1 - abar_t) noise is
// formed by the caller's q_sample; here d_eps = scale w[b] (eps - noise) with scale =
// 2 / numel (mean_flat then the batch mean), w the schedule sampler's importance
// weights (train_util.py:210, null = 1), and per-sample sums of squares
__global__ __launch_bounds__(256) void eps_mse_kernel(const float* __restrict__ eps, const float* __restrict__ noise,
                                                      const float* __restrict__ weights, float* __restrict__ d_eps,
                                                      int64_t n_per, float scale, float* __restrict__ sse) {
    const int64_t b = blockIdx.x;
    __shared__ float red[256];
    const float sw = weights ? scale * weights[b] : scale;
    float s = 0.f;
    for (int64_t i = threadIdx.x; i < n_per; i += 256) {
        const int64_t j = b * n_per + i;
        const float d = eps[j] - noise[j];
        d_eps[j] = d * sw;
        s += d * d;
    }
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) sse[b] = red[0];
}

// ---------------------------------------------------------------------------
namespace {
bool wgrad_fast(const WgradArgs& a) {
    return a.Ctot % 128 == 0 && a.Cout % 4 == 0 && a.C1 % 4 == 0 && a.C2 % 4 == 0;
}
// conv_wgrad_thin_kernel's shapes (the 1- to 4-channel convolutions)
bool wgrad_thin(const WgradArgs& a) {
    return !wgrad_fast(a) && (a.Ctot <= 4 || a.Cout <= 4) && a.stride == 1 && !a.up && a.ks <= 3 &&
           a.Hin == a.Hout && a.Win == a.Wout;
}
}  // namespace

// pixel slices: the 64-tile kernel >= 256 pixels a slice, at most 16 slices; the
// 128-tile kernel enough slices for <= 512 blocks (<= 64, >= 256 pixels a slice,
// partials within part_cap)
int64_t wgrad_kspan(const WgradArgs& a) {
    int64_t splits;
    if (wgrad_fast(a)) {
        const int64_t N = (int64_t)a.ks * a.ks * a.Ctot, MN = (int64_t)a.Cout * N;
        const int64_t tiles = ceil_div(N, 128) * ceil_div(a.Cout, 128);
        // as many slices as fill whole rounds of resident blocks: 512 = two 64-KB-LDS
        // blocks per CU, so a launch has no partial last round (576 blocks, 9 tiles
        // x 64 slices, ran as two rounds, the second one eighth full); at most 64 slices
        splits = std::min<int64_t>({(int64_t)64, std::max<int64_t>(1, 512 / tiles), ceil_div(a.P, 256),
                                    std::max<int64_t>(1, a.part_cap / MN)});
        splits = std::max<int64_t>(1, splits);
        const int64_t span = ceil_div(a.P, splits);
        return (span + 31) / 32 * 32;
    }
    if (wgrad_thin(a)) {   // ~512 blocks of 64 wide-side channels x 16 pixel lanes, slices of >= 512 pixels
        const int64_t MN = (int64_t)a.Cout * a.ks * a.ks * a.Ctot;
        const int64_t blocks = ceil_div(a.Ctot <= 4 ? a.Cout : a.Ctot, 64);
        splits = std::min<int64_t>({ceil_div(512, blocks), ceil_div(a.P, 512), std::max<int64_t>(1, a.part_cap / MN)});
        splits = std::max<int64_t>(1, splits);
        return ceil_div(a.P, splits);
    }
    // 64-tile kernel (narrow test topologies): ~1024 blocks, <= 128 slices of >= 256 pixels
    const int64_t N = (int64_t)a.ks * a.ks * a.Ctot, MN = (int64_t)a.Cout * N;
    const int64_t tiles = ceil_div(N, 64) * ceil_div(a.Cout, 64);
    splits = std::min<int64_t>({128, ceil_div(1024, tiles), ceil_div(a.P, 256), std::max<int64_t>(1, a.part_cap / MN)});
    splits = std::max<int64_t>(1, splits);
    const int64_t span = ceil_div(a.P, splits);
    return (span + 15) / 16 * 16;
}

size_t wgrad_part_floats(const WgradArgs& a) {
    const int64_t span = wgrad_kspan(a);
    return (size_t)((a.P + span - 1) / span) * a.Cout * a.Ctot * a.ks * a.ks;
}

bool launch_conv_wgrad(WgradArgs a, float* G, hipStream_t st) {
    a.kspan = wgrad_kspan(a);
    const int splits = (int)((a.P + a.kspan - 1) / a.kspan);
    bool bias_fused = false;
    const int N = a.ks * a.ks * a.Ctot;
    CFD_REQUIRE(wgrad_part_floats(a) <= (size_t)a.part_cap, CFD_ESTATE, "internal: weight-gradient scratch");
    if (wgrad_fast(a)) {
        CFD_REQUIRE(a.P < (int64_t)1 << 31, CFD_ESHAPE, "weight gradient over 2^31 or more pixels");
        // split-f16 products where the operand ranges are known (else the exact
        // fp32-MFMA kernel); fdiv24 pixel decode; 32-bit element offsets; one source
        // per 128-column tile
        const int64_t srows0 = (int64_t)(a.P / ((int64_t)a.Hout * a.Wout)) * a.Hin * a.Win;
        const bool split = a.amax_y && a.amax_x && a.P < (1 << 24) && a.P * a.Cout < (1ll << 31) &&
                           srows0 * a.Ctot < (1ll << 31) && (a.ss || a.C2 == 0 || a.C1 % 128 == 0);
        auto absmax = [&](const float* x, int64_t n, unsigned* out) {
            const int64_t n4 = n / 4;
            hipLaunchKernelGGL(absmax_kernel, dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>(1024, ceil_div(n4, 256)))),
                               dim3(256), 0, st, x, n4, out);
            check_launch("absmax_kernel");
        };
        // the range slots arrive zeroed (the caller zeroes its slot array once per
        // backward and gives every range a slot of its own)
        if (split && !a.ymax_known) absmax(a.dy, a.P * a.Cout, a.amax_y);
        const int64_t srows = (int64_t)(a.P / ((int64_t)a.Hout * a.Wout)) * a.Hin * a.Win;
        const float* act = nullptr;
        WgradArgs b = a;
        b.amax_out = nullptr;
        if (a.ss) {
            CFD_REQUIRE(a.act, CFD_ESTATE, "internal: activation scratch");
            const int64_t nq = srows * (a.Ctot / 4);
            WgradArgs g = a;
            g.amax_out = split ? a.amax_x : nullptr;
            hipLaunchKernelGGL(gn_act_kernel, dim3((unsigned)std::min<int64_t>(4096, ceil_div(nq, 256))), dim3(256), 0, st,
                               g, nq);
            check_launch("gn_act_kernel");
            act = a.act;
        } else if (split && !a.xmax_known) {
            absmax(a.src1, srows * a.C1, a.amax_x);
            if (a.src2 && a.C2) absmax(a.src2, srows * a.C2, a.amax_x);
        }
        const dim3 grid((unsigned)(N / 128), (unsigned)ceil_div(a.Cout, 128), (unsigned)splits);
        if (!split || !a.Gb || (int64_t)splits * a.Cout > a.bpart_cap) b.bpart = nullptr;
        bias_fused = b.bpart != nullptr;
        if (split) {
            if (a.up)
                hipLaunchKernelGGL(conv_wgrad128_split_kernel<true>, grid, dim3(256), 0, st, b, act);
            else
                hipLaunchKernelGGL(conv_wgrad128_split_kernel<false>, grid, dim3(256), 0, st, b, act);
            check_launch("conv_wgrad128_split_kernel");
        } else {
            hipLaunchKernelGGL(conv_wgrad128_kernel, grid, dim3(256), 0, st, b, act);
            check_launch("conv_wgrad128_kernel");
        }
    } else if (wgrad_thin(a)) {
        const bool wide_out = a.Ctot <= 4;
        const int narrow = wide_out ? a.Ctot : a.Cout;
        const dim3 grid((unsigned)ceil_div(wide_out ? a.Cout : a.Ctot, 64), 1, (unsigned)splits);
        if (wide_out) {
            if (narrow == 1) hipLaunchKernelGGL((conv_wgrad_thin_kernel<true, 1>), grid, dim3(1024), 0, st, a);
            else hipLaunchKernelGGL((conv_wgrad_thin_kernel<true, 4>), grid, dim3(1024), 0, st, a);
        } else {
            if (narrow == 1) hipLaunchKernelGGL((conv_wgrad_thin_kernel<false, 1>), grid, dim3(1024), 0, st, a);
            else hipLaunchKernelGGL((conv_wgrad_thin_kernel<false, 4>), grid, dim3(1024), 0, st, a);
        }
        check_launch("conv_wgrad_thin_kernel");
    } else {
        const dim3 grid((unsigned)ceil_div(N, 64), (unsigned)ceil_div(a.Cout, 64), (unsigned)splits);
        hipLaunchKernelGGL(conv_wgrad_kernel, grid, dim3(256), 0, st, a);
        check_launch("conv_wgrad_kernel");
    }
    const int64_t MN = (int64_t)a.Cout * N;
    hipLaunchKernelGGL(wgrad_accum_kernel, dim3((unsigned)ceil_div(std::max<int64_t>(MN, a.Cout), 256)), dim3(256), 0, st,
                       a.part, a.Cout, a.Ctot, a.ks * a.ks, splits, G, bias_fused ? a.bpart : nullptr, a.Gb);
    check_launch("wgrad_accum_kernel");
    return bias_fused;
}

namespace {
int colsum_splits(int64_t n, int R) {
    return (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(256, R), ceil_div(n, 64)));
}
}  // namespace

size_t colsum_part_floats(int64_t n, int64_t F, int R) { return (size_t)colsum_splits(n, R) * R * F; }

void launch_colsum(const float* X, int64_t n, int64_t F, int R, float* part, float* out, hipStream_t st) {
    const int splits = colsum_splits(n, R);
    const int64_t span = ceil_div(n, splits);
    const bool v4 = F % 4 == 0 && ((uintptr_t)X & 15) == 0;
    if (v4)
        hipLaunchKernelGGL(colsum_kernel<4>, dim3(splits, R), dim3(256), 0, st, X, part, n, F, R, span);
    else
        hipLaunchKernelGGL(colsum_kernel<1>, dim3(splits, R), dim3(256), 0, st, X, part, n, F, R, span);
    check_launch("colsum_kernel");
    hipLaunchKernelGGL(colsum_reduce_kernel, dim3((unsigned)ceil_div(F, 64), R), dim3(256), 0, st, part, R, F,
                       splits, out);
    check_launch("colsum_reduce_kernel");
}

void launch_rows_accum(const float* rows, int R, int64_t F, float* G, hipStream_t st) {
    hipLaunchKernelGGL(rows_accum_kernel, dim3((unsigned)ceil_div(F, 256)), dim3(256), 0, st, rows, R, F, G);
    check_launch("rows_accum_kernel");
}

void launch_gn_param_accum(const float* part, int nparts, int Ctot, float* dgamma, float* dbeta, hipStream_t st) {
    hipLaunchKernelGGL(gn_param_accum_kernel, dim3((unsigned)ceil_div(Ctot, 32)), dim3(256), 0, st, part, nparts, Ctot,
                       dgamma, dbeta);
    check_launch("gn_param_accum_kernel");
}

void launch_linear_wgrad(const float* d, const float* a, int B, int K, int N, int act, float* GW, float* Gb,
                         hipStream_t st) {
    hipLaunchKernelGGL(linear_wgrad_kernel, dim3((unsigned)ceil_div((int64_t)N * K, 256)), dim3(256), 0, st, d, a, B,
                       K, N, act, GW, Gb);
    check_launch("linear_wgrad_kernel");
}

void launch_linear_dgrad(const float* d, const float* W, const float* x, int B, int K, int N, int act, int accumulate,
                         float* da, hipStream_t st) {
    hipLaunchKernelGGL(linear_dgrad_kernel, dim3((unsigned)ceil_div(K, 32), B), dim3(256), 0, st, d, W, x, B, K, N,
                       act, accumulate, da);
    check_launch("linear_dgrad_kernel");
}

}  // namespace cfd

namespace cfd {
// q_sample (gaussian_diffusion.py:188-206): x_t = a[b] x0 + s[b] noise, a / s the
// fp32 casts of sqrt(abar_t) / sqrt(1 - abar_t) gathered per sample
__global__ void q_sample_kernel(const float* __restrict__ x0, const float* __restrict__ noise,
                                const float* __restrict__ a, const float* __restrict__ s, float* __restrict__ xt,
                                int64_t n_per, int64_t n) {
#pragma clang fp contract(off)   // torch's two rounded products and a rounded sum: bit-exact x_t
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t b = i / n_per;
    xt[i] = a[b] * x0[i] + s[b] * noise[i];
}
}  // namespace cfd

extern "C" int cfd_q_sample(const float* x0, const float* noise, const float* coef_a, const float* coef_s, float* x_t,
                            int64_t n_per_sample, int B, void* stream) {
    return cfd::guard([&] {
        CFD_REQUIRE(x0 && noise && coef_a && coef_s && x_t && n_per_sample > 0 && B > 0, CFD_EARG, "bad argument");
        const int64_t n = n_per_sample * B;
        hipLaunchKernelGGL(cfd::q_sample_kernel, dim3((unsigned)cfd::ceil_div(n, 256)), dim3(256), 0,
                           (hipStream_t)stream, x0, noise, coef_a, coef_s, x_t, n_per_sample, n);
        cfd::check_launch("q_sample_kernel");
    });
}

extern "C" int cfd_ema_update(float* target, const float* source, int64_t n, double rate, void* stream) {
    return cfd::guard([&] {
        CFD_REQUIRE(target && source && n >= 0 && rate >= 0 && rate <= 1, CFD_EARG, "bad argument");
        if (n == 0) return;
        hipLaunchKernelGGL(cfd::ema_kernel, dim3((unsigned)cfd::ceil_div(n, 256)), dim3(256), 0, (hipStream_t)stream,
                           target, source, n, (float)rate, (float)(1.0 - rate));
        cfd::check_launch("ema_kernel");
    });
}

extern "C" int cfd_eps_mse(const float* eps, const float* noise, const float* weights, float* d_eps,
                           int64_t n_per_sample, int B, float scale, float* sse, void* stream) {
    return cfd::guard([&] {
        CFD_REQUIRE(eps && noise && d_eps && sse && n_per_sample > 0 && B > 0, CFD_EARG, "bad argument");
        hipLaunchKernelGGL(cfd::eps_mse_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, eps, noise, weights,
                           d_eps, n_per_sample, scale, sse);
        cfd::check_launch("eps_mse_kernel");
    });
}
