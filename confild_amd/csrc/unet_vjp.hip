// Backward (input-gradient) kernels of the latent U-Net, for the DPS adjoint
// (grad_and_value, condition_methods.py:31-47, takes
// d||y - A(x0_hat(x_t))|| / d x_t through the U-Net; no weight gradients).
//
//   gn_bwd_partial/finalize/apply  GroupNorm(32) (+SiLU) backward, float64 group
//                                  sums, dx split over the two forward sources
//                                  (the concat-free skip input);
//   attn_bwd_dq / attn_bwd_dkv     QKVAttentionLegacy backward, flash-style: P is
//                                  recomputed from the forward's log-sum-exp, all
//                                  products on fp32 MFMA 16x16x4 with the same
//                                  accumulator-as-operand layouts as the forward;
//   add_kernel                     y += x (skip-gradient merge).
// The convolution input-gradients reuse conv_gemm (unet_kernels.hip) with
// transposed weight packs and TMODE addressing.
#include "unet_kernels.hpp"

namespace cfd {

__device__ __forceinline__ float sigmoid_f(float x) {   // the forward's SiLU form (unet_kernels.hip silu_f)
    return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * -1.44269504088896340736f));
}
// e^x for the recomputed attention probabilities (x = S - lse <= ~0): one multiply
// and v_exp_f32 instead of ocml's ~11-instruction expf; the rounding of x log2(e)
// is 2^-24 relative to |x|, below the split-f16 forward's own S error
__device__ __forceinline__ float exp_nat(float x) { return __builtin_amdgcn_exp2f(x * 1.44269504088896340736f); }

// Per-thread constants of a channel quad c0..c0+3 of sample b: forward scale /
// shift, gamma, group mean / rstd (loaded once, not per pixel).
struct GnbQuad {
    f4 sc, sh, gm, mean, rstd;
};
__device__ __forceinline__ GnbQuad gnb_quad(const GnbArgs& a, int64_t b, int c0) {
    GnbQuad k;
    const int cpg = a.Ctot / 32;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int c = c0 + j, grp = c / cpg;
        k.sc[j] = a.ss[(b * a.Ctot + c) * 2 + 0];
        k.sh[j] = a.ss[(b * a.Ctot + c) * 2 + 1];
        k.gm[j] = a.gamma[c];
        k.mean[j] = a.stats[(b * 32 + grp) * 2 + 0];
        k.rstd[j] = a.stats[(b * 32 + grp) * 2 + 1];
    }
    return k;
}

// dz_eff = dz * SiLU'(z) (or dz), g = gamma * dz_eff, xhat = (x - mean) * rstd, for 4 channels
__device__ __forceinline__ void gnb_load_d(const GnbArgs& a, const GnbQuad& k, int64_t pix, int c0, f4& d, f4& xh) {
    const f4 x = c0 < a.C1 ? *(const f4*)(a.x1 + pix * a.C1 + c0) : *(const f4*)(a.x2 + pix * a.C2 + (c0 - a.C1));
    const f4 dz = *(const f4*)(a.dz + pix * a.Ctot + c0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        float dj = dz[j];
        if (a.silu) {
            const float z = x[j] * k.sc[j] + k.sh[j];
            const float sg = sigmoid_f(z);
            dj = dj * (sg * (1.0f + z * (1.0f - sg)));
        }
        d[j] = dj;
        xh[j] = (x[j] - k.mean[j]) * k.rstd[j];
    }
}
__device__ __forceinline__ void gnb_load(const GnbArgs& a, const GnbQuad& k, int64_t pix, int c0, f4& g, f4& xh) {
    f4 d;
    gnb_load_d(a, k, pix, c0, d, xh);
#pragma unroll
    for (int j = 0; j < 4; ++j) g[j] = d[j] * k.gm[j];
}

// PP (training): the per-channel sums are of dz_eff, not g = gamma dz_eff, so the
// same pass also yields the parameter-gradient partials (sum dz_eff xhat, sum
// dz_eff) per (chunk, channel) -- gn_param_part's pass over the same data folded
// in; the group sums are then sum_c gamma_c (per-channel sum), in float64
template <bool PP, int NT = 256>
__global__ __launch_bounds__(NT) void gn_bwd_partial_kernel(GnbArgs a) {
    static_assert(!PP || NT == 256, "parameter partials: 256 threads");
    const int chunk = blockIdx.x;
    const int64_t b = blockIdx.y;
    const int Ctot = a.Ctot, cq = Ctot / 4, cpg = Ctot / 32;
    const int HW = a.HW;
    const int p0 = (int)((int64_t)HW * chunk / a.nchunks), p1 = (int)((int64_t)HW * (chunk + 1) / a.nchunks);
    const int rows = NT / cq;
    const int q = threadIdx.x % cq, r0 = threadIdx.x / cq;
    __shared__ double red[2][4 * NT];   // rows * Ctot = 4 NT
    if (r0 < rows) {
        double s[4] = {0, 0, 0, 0}, s2[4] = {0, 0, 0, 0};
        const int c0 = 4 * q;
        const GnbQuad k = gnb_quad(a, b, c0);
        constexpr int U = 4;   // pixel rows in flight per thread (the sums stay in pixel order)
        for (int pb = p0 + r0; pb < p1; pb += U * rows) {
            f4 g[U], xh[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int p = pb + u * rows;
                if (p < p1) {
                    if constexpr (PP)
                        gnb_load_d(a, k, b * HW + p, c0, g[u], xh[u]);
                    else
                        gnb_load(a, k, b * HW + p, c0, g[u], xh[u]);
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (pb + u * rows >= p1) break;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    s[j] += g[u][j];
                    s2[j] += (double)g[u][j] * xh[u][j];
                }
            }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            red[0][r0 * Ctot + c0 + j] = s[j];
            red[1][r0 * Ctot + c0 + j] = s2[j];
        }
    }
    __syncthreads();
    if constexpr (PP) {
        if (threadIdx.x < 32) {
            const int grp = threadIdx.x;
            double ts = 0, ts2 = 0;
            for (int r = 0; r < rows; ++r)
                for (int c = grp * cpg; c < (grp + 1) * cpg; ++c) {
                    const double gm = (double)a.gamma[c];
                    ts += gm * red[0][r * Ctot + c];
                    ts2 += gm * red[1][r * Ctot + c];
                }
            double* dst = a.part + ((b * a.nchunks + chunk) * 32 + grp) * 2;
            dst[0] = ts;
            dst[1] = ts2;
        }
        // rows in order, per channel: (sum dz_eff xhat, sum dz_eff)
        for (int c = threadIdx.x; c < Ctot; c += 256) {
            double t1 = 0, t2 = 0;
            for (int r = 0; r < rows; ++r) {
                t1 += red[1][r * Ctot + c];
                t2 += red[0][r * Ctot + c];
            }
            float* dst = a.ppart + ((b * a.nchunks + chunk) * (int64_t)Ctot + c) * 2;
            dst[0] = (float)t1;
            dst[1] = (float)t2;
        }
    } else {   // per group: GL lanes over its (row, channel) sums, then an xor butterfly
        constexpr int GL = NT / 32;
        const int grp = threadIdx.x / GL, sub = threadIdx.x % GL;
        double ts = 0, ts2 = 0;
        for (int e = sub; e < rows * cpg; e += GL) {
            const int r = e / cpg, c = grp * cpg + (e - r * cpg);
            ts += red[0][r * Ctot + c];
            ts2 += red[1][r * Ctot + c];
        }
#pragma unroll
        for (int o = 1; o < GL; o <<= 1) {
            ts += __shfl_xor(ts, o);
            ts2 += __shfl_xor(ts2, o);
        }
        if (sub == 0) {
            double* dst = a.part + ((b * a.nchunks + chunk) * 32 + grp) * 2;
            dst[0] = ts;
            dst[1] = ts2;
        }
    }
}

// the input-gradient pass over one pixel chunk of a sample (grid (chunks, B)),
// the statistics finalised by every workgroup itself from the sample's chunk
// partials (GL lanes per group, fixed order, xor butterfly: the same value on every
// workgroup) -- no finalize launch.  gn2's layout: NT = 1024 with kGn2BigChunks
// chunks beyond 128^2 (one round of partial loads), 256 threads below
template <int NT>
__global__ __launch_bounds__(NT) void gn_bwd_apply2_kernel(GnbArgs a) {
    const int chunk = blockIdx.x;
    const int64_t b = blockIdx.y;
    const int NC = gridDim.x, Ctot = a.Ctot, cq = Ctot / 4, cpg = Ctot / 32, HW = a.HW;
    __shared__ float fsh[2][32];
    {
        constexpr int GL = NT / 32;
        const int grp = threadIdx.x / GL, sub = threadIdx.x % GL;
        double S = 0, S2 = 0;
        for (int k = sub; k < NC; k += GL) {
            const double2 v = *(const double2*)(a.part + ((b * NC + k) * 32 + grp) * 2);
            S += v.x;
            S2 += v.y;
        }
#pragma unroll
        for (int o = 1; o < GL; o <<= 1) {
            S += __shfl_xor(S, o);
            S2 += __shfl_xor(S2, o);
        }
        if (sub == 0) {
            const double n = (double)HW * cpg;
            fsh[0][grp] = (float)(S / n);
            fsh[1][grp] = (float)(S2 / n);
        }
    }
    __syncthreads();
    const int p0 = (int)((int64_t)HW * chunk / NC), p1 = (int)((int64_t)HW * (chunk + 1) / NC);
    const int rows = NT / cq, q = threadIdx.x % cq, r0 = threadIdx.x / cq, c0 = 4 * q;
    float mx = 0.f;
    if (r0 < rows) {
        const GnbQuad k = gnb_quad(a, b, c0);
        f4 mg, mgx;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            mg[j] = fsh[0][(c0 + j) / cpg];
            mgx[j] = fsh[1][(c0 + j) / cpg];
        }
        constexpr int U = 4;
        for (int pb = p0 + r0; pb < p1; pb += U * rows) {
            f4 g[U], xh[U], ad[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t pix = b * HW + pb + u * rows;
                if (pb + u * rows < p1) {
                    gnb_load(a, k, pix, c0, g[u], xh[u]);
                    if (a.addsrc) ad[u] = *(const f4*)(a.addsrc + pix * Ctot + c0);
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (pb + u * rows >= p1) break;
                const int64_t pix = b * HW + pb + u * rows;
                f4 dx;
#pragma unroll
                for (int j = 0; j < 4; ++j) dx[j] = k.rstd[j] * (g[u][j] - mg[j] - xh[u][j] * mgx[j]);
                if (a.addsrc) dx += ad[u];
                if (c0 < a.C1) {
                    f4* o = (f4*)(a.out1 + pix * a.C1 + c0);
                    const f4 v = a.acc1 ? *o + dx : dx;
                    *o = v;
                    mx = fmaxf(mx, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
                } else {
                    f4* o = (f4*)(a.out2 + pix * a.C2 + (c0 - a.C1));
                    *o = a.acc2 ? *o + dx : dx;
                }
            }
        }
    }
    if (a.amax_out) {   // block-uniform
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
        __shared__ float wm[NT / 64];
        if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = mx;
        __syncthreads();
        if (threadIdx.x == 0) {
            float m = 0.f;
            for (int w = 0; w < NT / 64; ++w) m = fmaxf(m, wm[w]);
            atomicMax(a.amax_out, __float_as_uint(m));
        }
    }
}

// 32 threads per group, each summing every 32nd chunk, then a fixed-order tree
__global__ __launch_bounds__(1024) void gn_bwd_finalize_kernel(GnbArgs a) {
    const int64_t b = blockIdx.x;
    __shared__ double red[2][1024];
    const int grp = threadIdx.x >> 5, sub = threadIdx.x & 31;
    {
        double s = 0, s2 = 0;
        for (int ch = sub; ch < a.nchunks; ch += 32) {
            const double* src = a.part + ((b * a.nchunks + ch) * 32 + grp) * 2;
            s += src[0];
            s2 += src[1];
        }
        red[0][threadIdx.x] = s;
        red[1][threadIdx.x] = s2;
    }
    __syncthreads();
    for (int w = 16; w > 0; w >>= 1) {
        if (sub < w) {
            red[0][threadIdx.x] += red[0][threadIdx.x + w];
            red[1][threadIdx.x] += red[1][threadIdx.x + w];
        }
        __syncthreads();
    }
    if (sub == 0) {
        const double n = (double)a.HW * (a.Ctot / 32);
        a.fin[(b * 32 + grp) * 2 + 0] = (float)(red[0][threadIdx.x] / n);
        a.fin[(b * 32 + grp) * 2 + 1] = (float)(red[1][threadIdx.x] / n);
    }
}

// thread = (channel quad, pixel); GNB_PIX pixels per thread at a stride of the
// grid's pixel rows, so the per-channel constants load once per GNB_PIX pixels
constexpr int GNB_PIX = 4;
__global__ __launch_bounds__(256) void gn_bwd_apply_kernel(GnbArgs a) {
    const int cq = a.Ctot / 4;
    const int64_t npix = (int64_t)a.B * a.HW;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // over (pixel row, quad)
    const int64_t prow = i / cq;
    const int c0 = (int)(i - prow * cq) * 4;
    const int64_t nrow = (npix + GNB_PIX - 1) / GNB_PIX;
    const int cpg = a.Ctot / 32;
    int64_t bcur = -1;
    GnbQuad k;
    f4 mg, mgx;
    float mx = 0.f;   // max |stored out1| of this thread (a.amax_out)
#pragma unroll
    for (int e = 0; e < GNB_PIX; ++e) {
        const int64_t pix = prow + e * nrow;
        if (prow >= nrow || pix >= npix) break;
        const int64_t b = pix / a.HW;
        if (b != bcur) {
            bcur = b;
            k = gnb_quad(a, b, c0);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int grp = (c0 + j) / cpg;
                mg[j] = a.fin[(b * 32 + grp) * 2 + 0];
                mgx[j] = a.fin[(b * 32 + grp) * 2 + 1];
            }
        }
        f4 g, xh;
        gnb_load(a, k, pix, c0, g, xh);
        f4 dx;
#pragma unroll
        for (int j = 0; j < 4; ++j) dx[j] = k.rstd[j] * (g[j] - mg[j] - xh[j] * mgx[j]);
        if (a.addsrc) dx += *(const f4*)(a.addsrc + pix * a.Ctot + c0);
        if (c0 < a.C1) {
            f4* o = (f4*)(a.out1 + pix * a.C1 + c0);
            const f4 v = a.acc1 ? *o + dx : dx;
            *o = v;
            mx = fmaxf(mx, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
        } else {
            f4* o = (f4*)(a.out2 + pix * a.C2 + (c0 - a.C1));
            *o = a.acc2 ? *o + dx : dx;
        }
    }
    if (a.amax_out) {   // block-uniform
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
        __shared__ float wm[4];
        if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = mx;
        __syncthreads();
        if (threadIdx.x == 0) atomicMax(a.amax_out, __float_as_uint(fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]))));
    }
}

__global__ void add_kernel(float* __restrict__ y, const float* __restrict__ x, int64_t n4) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n4) ((f4*)y)[i] += ((const f4*)x)[i];
}

// ---------------------------------------------------------------------------
// Attention backward.  With s = scale, S = (s q)(s k)^T, P = softmax_rows(S),
// O = P V, D_q = sum_d dO[q][d] O[q][d]:
//   dS = P * (dO V^T - D),  dq = s^2 dS k,  dk = s^2 dS^T q,  dv = P^T dO.
// attn_bwd_dq  : one wave per 16 queries, loop over 16-key blocks; S^T / dP^T
//                blocks have lane = query, so dS^T feeds dQ^T = K^T dS^T as the
//                MFMA B operand in place (same as O^T = V^T P^T in the forward).
// attn_bwd_dkv : one wave per 16 keys, loop over 16-query blocks; S / dP blocks
//                have lane = key, so P and dS feed dV^T = dO^T P and
//                dK^T = Q^T dS directly.
// ---------------------------------------------------------------------------
template <int CH>
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(AttnBwdArgs a) {
    constexpr int KQ = CH / 4;
    constexpr int ND = CH / 16;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane >> 4, li = lane & 15;
    const int h = blockIdx.y, heads = gridDim.y;
    const int64_t b = blockIdx.z;
    const int T = a.T;
    const int q0 = blockIdx.x * 64 + wave * 16;
    if (q0 >= T) return;
    const int C3 = 3 * a.C;
    const float* base = a.qkv + b * (int64_t)T * C3 + (int64_t)h * 3 * CH;
    const float scale = a.scale;
    const int tq = q0 + li;
    const float* dop = a.dout + (b * (int64_t)T + tq) * a.C + (int64_t)h * CH + KQ * g;
    const float* opp = a.o + (b * (int64_t)T + tq) * a.C + (int64_t)h * CH + KQ * g;

    float qf[KQ], df[KQ];
    float dsum = 0.f;
    {
        const float* qp = base + (int64_t)tq * C3 + KQ * g;
#pragma unroll
        for (int s = 0; s < KQ; s += 4) {
            const f4 v = *(const f4*)(qp + s);
            const f4 dv = *(const f4*)(dop + s);
            const f4 ov = *(const f4*)(opp + s);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                qf[s + u] = v[u] * scale;
                df[s + u] = dv[u];
                dsum = fmaf(dv[u], ov[u], dsum);
            }
        }
    }
    dsum += __shfl_xor(dsum, 16);
    dsum += __shfl_xor(dsum, 32);
    const int64_t row = (b * heads + h) * (int64_t)T;
    if (g == 0) a.dd[row + tq] = dsum;
    const float lse = a.lse[row + tq];

    f4 dQ[ND];
#pragma unroll
    for (int d = 0; d < ND; ++d) dQ[d] = f4{0.f, 0.f, 0.f, 0.f};
    for (int kb = 0; kb < T; kb += 16) {
        f4 st = {0.f, 0.f, 0.f, 0.f}, dpt = {0.f, 0.f, 0.f, 0.f};
        {
            const float* kp = base + (int64_t)(kb + li) * C3 + CH + KQ * g;
            const float* vp = kp + CH;
#pragma unroll
            for (int s = 0; s < KQ; s += 4) {
                const f4 kv = *(const f4*)(kp + s);
                const f4 vv = *(const f4*)(vp + s);
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    st = __builtin_amdgcn_mfma_f32_16x16x4f32(kv[u] * scale, qf[s + u], st, 0, 0, 0);
                    dpt = __builtin_amdgcn_mfma_f32_16x16x4f32(vv[u], df[s + u], dpt, 0, 0, 0);
                }
            }
        }
        // lane (g, li): S[query li][key kb + 4g + r], dP likewise
        float ds[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) ds[r] = exp_nat(st[r] - lse) * (dpt[r] - dsum);
        // dQ^T[d][query] += K^T[d][key] dS^T[key][query]
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float* kp = base + (int64_t)(kb + 4 * g + r) * C3 + CH + li;
#pragma unroll
            for (int d = 0; d < ND; ++d) dQ[d] = __builtin_amdgcn_mfma_f32_16x16x4f32(kp[16 * d], ds[r], dQ[d], 0, 0, 0);
        }
    }
    const float s2 = scale * scale;
    float* out = a.dqkv + (b * (int64_t)T + tq) * C3 + (int64_t)h * 3 * CH;
#pragma unroll
    for (int d = 0; d < ND; ++d) *(f4*)(out + 16 * d + 4 * g) = dQ[d] * s2;
}

template <int CH>
__global__ __launch_bounds__(256) void attn_bwd_dkv_kernel(AttnBwdArgs a) {
    constexpr int KQ = CH / 4;
    constexpr int ND = CH / 16;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane >> 4, li = lane & 15;
    const int h = blockIdx.y, heads = gridDim.y;
    const int64_t b = blockIdx.z;
    const int T = a.T;
    const int k0 = blockIdx.x * 64 + wave * 16;
    if (k0 >= T) return;
    const int C3 = 3 * a.C;
    const float* base = a.qkv + b * (int64_t)T * C3 + (int64_t)h * 3 * CH;
    const float* dbase = a.dout + b * (int64_t)T * a.C + (int64_t)h * CH;
    const float scale = a.scale;
    const int64_t row = (b * heads + h) * (int64_t)T;

    float kf[KQ], vf[KQ];
    {
        const float* kp = base + (int64_t)(k0 + li) * C3 + CH + KQ * g;
#pragma unroll
        for (int s = 0; s < KQ; s += 4) {
            const f4 kv = *(const f4*)(kp + s);
            const f4 vv = *(const f4*)(kp + CH + s);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                kf[s + u] = kv[u] * scale;
                vf[s + u] = vv[u];
            }
        }
    }
    f4 dK[ND], dV[ND];
#pragma unroll
    for (int d = 0; d < ND; ++d) dK[d] = dV[d] = f4{0.f, 0.f, 0.f, 0.f};
    for (int qb = 0; qb < T; qb += 16) {
        f4 st = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
        {
            const float* qp = base + (int64_t)(qb + li) * C3 + KQ * g;
            const float* dop = dbase + (int64_t)(qb + li) * a.C + KQ * g;
#pragma unroll
            for (int s = 0; s < KQ; s += 4) {
                const f4 qv = *(const f4*)(qp + s);
                const f4 dv = *(const f4*)(dop + s);
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    st = __builtin_amdgcn_mfma_f32_16x16x4f32(qv[u] * scale, kf[s + u], st, 0, 0, 0);
                    dp = __builtin_amdgcn_mfma_f32_16x16x4f32(dv[u], vf[s + u], dp, 0, 0, 0);
                }
            }
        }
        // lane (g, li): S[query qb + 4g + r][key li]
        float p[4], ds[4];
        {
            const f4 l4 = *(const f4*)(a.lse + row + qb + 4 * g);
            const f4 d4 = *(const f4*)(a.dd + row + qb + 4 * g);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                p[r] = exp_nat(st[r] - l4[r]);
                ds[r] = p[r] * (dp[r] - d4[r]);
            }
        }
        // dV^T[d][key] += dO^T[d][q] P[q][key];  dK^T[d][key] += Q^T[d][q] dS[q][key]
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int tq = qb + 4 * g + r;
            const float* dop = dbase + (int64_t)tq * a.C + li;
            const float* qp = base + (int64_t)tq * C3 + li;
#pragma unroll
            for (int d = 0; d < ND; ++d) {
                dV[d] = __builtin_amdgcn_mfma_f32_16x16x4f32(dop[16 * d], p[r], dV[d], 0, 0, 0);
                dK[d] = __builtin_amdgcn_mfma_f32_16x16x4f32(qp[16 * d], ds[r], dK[d], 0, 0, 0);
            }
        }
    }
    const float s2 = scale * scale;
    float* out = a.dqkv + (b * (int64_t)T + k0 + li) * C3 + (int64_t)h * 3 * CH;
#pragma unroll
    for (int d = 0; d < ND; ++d) {
        *(f4*)(out + CH + 16 * d + 4 * g) = dK[d] * s2;
        *(f4*)(out + 2 * CH + 16 * d + 4 * g) = dV[d];
    }
}

// ---------------------------------------------------------------------------
// K9s: the attention backward at fp32 accuracy on f16 MFMA (split compute), the
// backward of K4s / K4d.  Every product is three v_mfma_f32_16x16x32_f16 on hi/lo
// halves (lo*hi + hi*lo + hi*hi, fp32 accumulate), as in the forward.
//   attn_bwd_prep : per (sample, head) D = rowsum(dO * O) and a power-of-two
//                   gradient scale sig: max |sig dO| < 1 and CH max|sig dO| max|V|
//                   < 2^14, so sig dP, sig D and sig dS = P (sig dP - sig D) fit f16
//                   with full hi/lo precision (the gradient's own scale, e.g. 1e-4,
//                   would leave the lo halves subnormal).  Per (sample, head): a
//                   sample's bits do not depend on the batch.
//   attn_bwd_pack : hi/lo fragments of seven operands, keys / queries padded to 32:
//                   row packs (token-row MFMA A operand, attn_kv_split's K layout)
//                   Kr = K kln2(s), Vr = V, Qr = Q s, dOr = sig dO; column packs
//                   (channel-row, tokens in kmap order, its V layout) Kt = K,
//                   dOt = sig dO, Qt = Q.
//   attn_bwd_dq   : a wave per 16 queries, 32-key blocks of Kr / Vr / Kt staged by
//                   LDS-DMA into a ring shared by the workgroup (K4d's scheme):
//                   S^T = Kr Q^T (base 2, the forward's bits), dP^T = Vr dO^T,
//                   dS^T = P^T (dP^T - D), dQ^T += Kt dS^T (dS^T feeds the B operand
//                   in kmap order straight from the accumulator layout).
//   attn_bwd_dkv  : a wave per 16 keys, 32-query blocks of Qr / dOr / dOt / Qt and
//                   the block's log-sum-exp / D (one dword DMA piece): S = Qr K^T,
//                   dP = dOr V^T, dV^T += dOt P, dK^T += Qt dS.
// Outputs: dq = s^2 dS k, dk = s^2 dS^T q, dv = P^T dO, each times 1/sig (exact).
// ---------------------------------------------------------------------------
enum { AB_KR = 0, AB_VR, AB_QR, AB_DOR, AB_KT, AB_DOT, AB_QT, AB_NPACK };

// x materialised as an fp32 register value: the backend otherwise folds a product
// into its f16 conversion (v_fma_mixlo_f16 x, y, 0: one rounding of the exact
// product instead of fp32 then f16), in some kernel variants and not in others
__device__ __forceinline__ float ab_f32(float x) {
    asm("" : "+v"(x));
    return x;
}

size_t attention_bwd_split_floats(int T, int C) {
    const size_t T32 = (size_t)(T + 31) / 32 * 32;
    // packs (hi + lo: a float per value), then 2 maxima per (head, 32-token block):
    // heads <= C / 32 (head channels >= 32)
    return (size_t)AB_NPACK * T32 * C + T32 * C / 512 + 2;
}

bool attention_bwd_split_ok(int T, int CH) { return (CH == 32 || CH == 64 || CH == 128) && T % 16 == 0; }

// the gradient scale of a (sample, head) from its per-block maxima (AttnBwdArgs::
// amax: (max |dO|, max |V|) of each 32-token block, reduced here by every wave --
// a max is order-free, so every reader gets the same value): 2^-e with max |dO| <
// 2^e, lowered until CH max|dO| max|V| sig < 2^14 (which bounds |sig dP| and
// |sig D|: |O| <= max |V|)
__device__ __forceinline__ float ab_sigma(const float* bm, int nblk, int CH) {
    float mdo = 0.f, mv = 0.f;
    for (int k = threadIdx.x & 63; k < nblk; k += 64) {
        mdo = fmaxf(mdo, bm[2 * k]);
        mv = fmaxf(mv, bm[2 * k + 1]);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        mdo = fmaxf(mdo, __shfl_xor(mdo, off));
        mv = fmaxf(mv, __shfl_xor(mv, off));
    }
    float sg = 1.f;
    if (mdo > 0.f && isfinite(mdo)) {
        int e = 0;
        frexpf(mdo, &e);
        sg = ldexpf(1.f, -e);
        const float bound = (float)CH * mdo * mv;
        if (bound > 0.f && isfinite(bound)) {
            int e2 = 0;
            frexpf(bound, &e2);
            sg = fminf(sg, ldexpf(1.f, 14 - e2));
        }
    }
    return sg;
}

// hi/lo fragments of one 32-token block from an LDS tile [32][CH + 4] (zero rows
// past T): the row pack's two 16-token tiles (slot e < 2 NJ 64) or the column
// pack (slot e < ND 64), times sc
template <int CH>
__device__ __forceinline__ void ab_frag_row(const float (*tile)[CH + 4], int e, float sc, h8v* dst0, int64_t tile0) {
#pragma clang fp contract(off)
    constexpr int NJ = CH / 32;
    const int lane = e & 63, f = e >> 6, u = f / NJ, j = f - u * NJ, g = lane >> 4, li = lane & 15;
    float v[8];
    const float* sp = &tile[16 * u + li][32 * j + 8 * g];
#pragma unroll
    for (int t = 0; t < 8; ++t) v[t] = ab_f32(sp[t] * sc);
    h8v hi, lo;
    split8_f16(v, hi, lo);
    h8v* d = dst0 + ((tile0 + u) * NJ + j) * 128 + lane;
    d[0] = hi;
    d[64] = lo;
}
template <int CH>
__device__ __forceinline__ void ab_frag_col(const float (*tile)[CH + 4], int e, float sc, h8v* dst0, int64_t blk) {
#pragma clang fp contract(off)
    constexpr int ND = CH / 16;
    const int lane = e & 63, dd = e >> 6, g = lane >> 4, li = lane & 15;
    float v[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) v[t] = ab_f32(tile[t < 4 ? 4 * g + t : 16 + 4 * g + t - 4][16 * dd + li] * sc);
    h8v hi, lo;
    split8_f16(v, hi, lo);
    h8v* d = dst0 + (blk * ND + dd) * 128 + lane;
    d[0] = hi;
    d[64] = lo;
}

// one 32-token block of a (sample, head): D = rowsum(dO * O) (unscaled), the
// maxima of |dO| and |V| (atomic max on float bits: order-free, so deterministic),
// and the five packs that need no gradient scale (Kr, Vr, Qr, Kt, Qt), from an LDS
// copy of the block's q / k / v rows
template <int CH>
__global__ __launch_bounds__(256) void attn_bwd_prep_kernel(AttnBwdArgs a) {
#pragma clang fp contract(off)
    constexpr int NJ = CH / 32, ND = CH / 16, CQ = CH / 4;
    __shared__ __attribute__((aligned(16))) float tile[3][32][CH + 4];   // q, k, v
    const int kb = blockIdx.x;
    const int64_t bh = blockIdx.y;
    const int heads = a.heads, B = gridDim.y / heads;
    const int64_t b = bh / heads;
    const int h = (int)(bh - b * heads);
    const int T = a.T, T32 = (T + 31) / 32 * 32, C = a.C, C3 = 3 * a.C;
    const float* qb = a.qkv + b * (int64_t)T * C3 + (int64_t)h * 3 * CH;
    float mv = 0.f, mdo = 0.f;
    for (int e = threadIdx.x; e < 3 * 32 * CQ; e += 256) {
        const int ts = e / (32 * CQ), rem = e - ts * 32 * CQ, tk = rem / CQ, c4 = rem - tk * CQ;
        const int tok = 32 * kb + tk;
        const f4 v = tok < T ? *(const f4*)(qb + (int64_t)tok * C3 + ts * CH + 4 * c4) : f4{0.f, 0.f, 0.f, 0.f};
        *(f4*)&tile[ts][tk][4 * c4] = v;
        if (ts == 2) mv = fmaxf(mv, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
    }
    // D: a token's CQ lanes are consecutive and all active (32 CQ is a multiple of 64
    // for CH >= 8), so the xor partners stay within the token
    for (int e = threadIdx.x; e < 32 * CQ; e += 256) {
        const int tk = e / CQ, c4 = e - tk * CQ, tok = 32 * kb + tk;
        f4 d = {0.f, 0.f, 0.f, 0.f}, o = {0.f, 0.f, 0.f, 0.f};
        if (tok < T) {
            const int64_t off = (b * (int64_t)T + tok) * C + (int64_t)h * CH + 4 * c4;
            d = *(const f4*)(a.dout + off);
            o = *(const f4*)(a.o + off);
        }
        float sm = d[0] * o[0];
#pragma unroll
        for (int jj = 1; jj < 4; ++jj) sm = fmaf(d[jj], o[jj], sm);
        for (int off = 1; off < CQ; off <<= 1) sm += __shfl_xor(sm, off);
        if (c4 == 0 && tok < T) a.dd[bh * T + tok] = sm;
        mdo = fmaxf(mdo, fmaxf(fmaxf(fabsf(d[0]), fabsf(d[1])), fmaxf(fabsf(d[2]), fabsf(d[3]))));
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        mdo = fmaxf(mdo, __shfl_xor(mdo, off));
        mv = fmaxf(mv, __shfl_xor(mv, off));
    }
    __shared__ float wm[2][4];
    if ((threadIdx.x & 63) == 0) {
        wm[0][threadIdx.x >> 6] = mdo;
        wm[1][threadIdx.x >> 6] = mv;
    }
    __syncthreads();
    if (threadIdx.x == 0) {   // this block's maxima (no atomics: the readers reduce the blocks)
        a.amax[(bh * (T32 / 32) + kb) * 2 + 0] = fmaxf(fmaxf(wm[0][0], wm[0][1]), fmaxf(wm[0][2], wm[0][3]));
        a.amax[(bh * (T32 / 32) + kb) * 2 + 1] = fmaxf(fmaxf(wm[1][0], wm[1][1]), fmaxf(wm[1][2], wm[1][3]));
    }
    const int64_t PB = (int64_t)B * heads * T32 * CH / 4;
    const int64_t rt = bh * (T32 / 16) + 2 * kb, cbk = bh * (T32 / 32) + kb;
    for (int e = threadIdx.x; e < 3 * 2 * NJ * 64; e += 256) {   // Kr, Vr, Qr
        const int kind = e / (2 * NJ * 64), r = e - kind * 2 * NJ * 64;
        const int ts = kind == 0 ? 1 : kind == 1 ? 2 : 0;
        const float sc = kind == 0 ? kln2(a.scale) : kind == 1 ? 1.f : a.scale;
        ab_frag_row<CH>(tile[ts], r, sc, a.packs + (AB_KR + kind) * PB, rt);
    }
    for (int e = threadIdx.x; e < 2 * ND * 64; e += 256) {   // Kt, Qt
        const int kind = e / (ND * 64), r = e - kind * ND * 64;
        ab_frag_col<CH>(tile[kind == 0 ? 1 : 0], r, 1.f, a.packs + (kind == 0 ? AB_KT : AB_QT) * PB, cbk);
    }
}

// the two gradient packs of one 32-token block (dOr, dOt), times the scale
template <int CH>
__global__ __launch_bounds__(256) void attn_bwd_pack_do_kernel(AttnBwdArgs a) {
#pragma clang fp contract(off)
    constexpr int NJ = CH / 32, ND = CH / 16, CQ = CH / 4;
    __shared__ __attribute__((aligned(16))) float tile[32][CH + 4];
    const int kb = blockIdx.x;
    const int64_t bh = blockIdx.y;
    const int heads = a.heads, B = gridDim.y / heads;
    const int64_t b = bh / heads;
    const int h = (int)(bh - b * heads);
    const int T = a.T, T32 = (T + 31) / 32 * 32, C = a.C;
    for (int e = threadIdx.x; e < 32 * CQ; e += 256) {
        const int tk = e / CQ, c4 = e - tk * CQ, tok = 32 * kb + tk;
        *(f4*)&tile[tk][4 * c4] = tok < T ? *(const f4*)(a.dout + (b * (int64_t)T + tok) * C + (int64_t)h * CH + 4 * c4)
                                          : f4{0.f, 0.f, 0.f, 0.f};
    }
    const float sg = ab_sigma(a.amax + bh * (T32 / 32) * 2, T32 / 32, CH);
    __syncthreads();
    const int64_t PB = (int64_t)B * heads * T32 * CH / 4;
    for (int e = threadIdx.x; e < 2 * NJ * 64; e += 256)
        ab_frag_row<CH>(tile, e, sg, a.packs + AB_DOR * PB, bh * (T32 / 16) + 2 * kb);
    for (int e = threadIdx.x; e < ND * 64; e += 256)
        ab_frag_col<CH>(tile, e, sg, a.packs + AB_DOT * PB, bh * (T32 / 32) + kb);
}

// the workgroup's (query / key tile, head, sample), with the K4d XCD map: the
// tiles of one (sample, head) on one XCD, so its packed blocks are fetched into
// one L2 (a schedule change only)
__device__ __forceinline__ void ab_tile(const AttnBwdArgs& a, int& tile, int& h, int64_t& b) {
    tile = blockIdx.x;
    h = blockIdx.y;
    b = blockIdx.z;
    if (a.xcdmap) {
        const int nt = gridDim.x, heads = gridDim.y;
        const int L = blockIdx.x + nt * (blockIdx.y + heads * blockIdx.z);
        const int r = L >> 3, grp = (r / nt) * 8 + (L & 7);
        tile = r - (r / nt) * nt;
        h = grp % heads;
        b = grp / heads;
    }
}

template <int CH, int WAVES, int NS>
__global__ __launch_bounds__(64 * WAVES) void attn_bwd_dq_split_kernel(AttnBwdArgs a) {
    // contraction off: every product rounds to fp32 before its f16 split (a fused
    // v_fma_mix round would vary with the variant the compiler schedules, and the
    // W = 4 / W = 8 variants -- chosen from the batch -- must give the same bits)
#pragma clang fp contract(off)
    constexpr int NJ = CH / 32, ND = CH / 16;
    constexpr int KP = 4 * NJ, VP = 4 * NJ, TP = 2 * ND, NP = KP + VP + TP;   // 1-KiB pieces per block
    constexpr int PPW = NP / WAVES;
    static_assert(NP % WAVES == 0 && NS >= 2 && NS <= 3, "piece split");
    __shared__ __attribute__((aligned(16))) h8v ring[NS][NP * 64];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = lane >> 4, li = lane & 15;
    int qt, h;
    int64_t b;
    ab_tile(a, qt, h, b);
    const int heads = gridDim.y, B = gridDim.z;
    const int T = a.T, T32 = (T + 31) / 32 * 32;
    const int q0 = (qt * WAVES + wave) * 16;
    const bool active = q0 < T;   // wave-uniform; an idle wave still stages and syncs
    const int64_t bh = b * heads + h;
    const int64_t PB = (int64_t)B * heads * T32 * CH / 4;
    const h8v* kr = a.packs + AB_KR * PB + bh * (T32 / 16) * NJ * 128;
    const h8v* vr = a.packs + AB_VR * PB + bh * (T32 / 16) * NJ * 128;
    const h8v* kt = a.packs + AB_KT * PB + bh * (T32 / 32) * ND * 128;
    auto issue = [&](int ib, int stage) {
#pragma unroll
        for (int i = 0; i < PPW; ++i) {
            const int piece = wave + WAVES * i;
            const h8v* src = piece < KP        ? kr + (int64_t)ib * KP * 64 + piece * 64
                             : piece < KP + VP ? vr + (int64_t)ib * VP * 64 + (piece - KP) * 64
                                               : kt + (int64_t)ib * TP * 64 + (piece - KP - VP) * 64;
            __builtin_amdgcn_global_load_lds((const void*)(src + lane),
                                             (__attribute__((address_space(3))) void*)&ring[stage][piece * 64], 16, 0, 0);
        }
    };
    const int nblk = T32 / 32;
#pragma unroll
    for (int i = 0; i < NS - 1; ++i)
        if (i < nblk) issue(i, i);

    const int C3 = 3 * a.C;
    const int tq = min(q0 + li, T - 1);
    const float sg = ab_sigma(a.amax + bh * (T32 / 32) * 2, T32 / 32, CH);
    h8v qh[NJ], ql[NJ], dh[NJ], dl[NJ];
    {
        const float* qp = a.qkv + (b * (int64_t)T + tq) * C3 + (int64_t)h * 3 * CH + 8 * g;
        const float* dp = a.dout + (b * (int64_t)T + tq) * a.C + (int64_t)h * CH + 8 * g;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            float v[8], w[8];
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                v[t] = ab_f32(qp[32 * j + t] * a.scale);
                w[t] = ab_f32(dp[32 * j + t] * sg);
            }
            split8_f16(v, qh[j], ql[j]);
            split8_f16(w, dh[j], dl[j]);
        }
    }
    const float lse2 = a.lse[bh * T + tq] * 1.44269504088896340736f;   // base-2 units, as S
    const float dq = a.dd[bh * T + tq] * sg;
    f4 dQ[ND];
#pragma unroll
    for (int d = 0; d < ND; ++d) dQ[d] = f4{0.f, 0.f, 0.f, 0.f};

    for (int ib = 0; ib < nblk; ++ib) {
        const int kb = 32 * ib, stage = ib % NS;
        if (NS == 3 && ib + 1 < nblk)
            __builtin_amdgcn_s_waitcnt(vmcnt_wait(PPW));
        else
            __builtin_amdgcn_s_waitcnt(vmcnt_wait(0));
        __builtin_amdgcn_s_barrier();
        if (ib + NS - 1 < nblk) issue(ib + NS - 1, (ib + NS - 1) % NS);
        if (!active) continue;
        const h8v* R = &ring[stage][lane];
        f4 st[2], dpt[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            st[u] = dpt[u] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const h8v kh = R[((u * NJ + j) * 2) * 64], kl = R[((u * NJ + j) * 2 + 1) * 64];
                st[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kl, qh[j], st[u], 0, 0, 0);
                st[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kh, ql[j], st[u], 0, 0, 0);
                st[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kh, qh[j], st[u], 0, 0, 0);
                const h8v vh = R[(KP + (u * NJ + j) * 2) * 64], vl = R[(KP + (u * NJ + j) * 2 + 1) * 64];
                dpt[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vl, dh[j], dpt[u], 0, 0, 0);
                dpt[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vh, dl[j], dpt[u], 0, 0, 0);
                dpt[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vh, dh[j], dpt[u], 0, 0, 0);
            }
        }
        // lane (g, li): key kb + 16 u + 4 g + r of query li; element t = 4 u + r of
        // the B operand below is key kmap(g, t), Kt's k order
        float ds[8];
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float p = __builtin_amdgcn_exp2f(st[u][r] - lse2);
                if (kb + 32 > T && kb + 16 * u + 4 * g + r >= T) p = 0.f;   // padded keys (ragged last block)
                ds[4 * u + r] = ab_f32(p * (dpt[u][r] - dq));
            }
        h8v sh, sl;
        split8_f16(ds, sh, sl);
#pragma unroll
        for (int d = 0; d < ND; ++d) {
            const h8v th = R[(KP + VP + 2 * d) * 64], tl = R[(KP + VP + 2 * d + 1) * 64];
            dQ[d] = __builtin_amdgcn_mfma_f32_16x16x32_f16(tl, sh, dQ[d], 0, 0, 0);
            dQ[d] = __builtin_amdgcn_mfma_f32_16x16x32_f16(th, sl, dQ[d], 0, 0, 0);
            dQ[d] = __builtin_amdgcn_mfma_f32_16x16x32_f16(th, sh, dQ[d], 0, 0, 0);
        }
    }
    if (!active || q0 + li >= T) return;
    const float os = a.scale * a.scale / sg;
    float* out = a.dqkv + (b * (int64_t)T + q0 + li) * C3 + (int64_t)h * 3 * CH;
#pragma unroll
    for (int d = 0; d < ND; ++d) *(f4*)(out + 16 * d + 4 * g) = dQ[d] * os;
}

template <int CH, int WAVES, int NS>
__global__ __launch_bounds__(64 * WAVES) void attn_bwd_dkv_split_kernel(AttnBwdArgs a) {
#pragma clang fp contract(off)
    constexpr int NJ = CH / 32, ND = CH / 16;
    constexpr int QP = 4 * NJ, OP = 4 * NJ, TO = 2 * ND, TQ = 2 * ND, NP = QP + OP + TO + TQ;
    constexpr int PPW = NP / WAVES;
    static_assert(NP % WAVES == 0 && NS >= 2 && NS <= 3, "piece split");
    __shared__ __attribute__((aligned(16))) h8v ring[NS][NP * 64];
    __shared__ __attribute__((aligned(16))) float lring[NS][64];   // the block's lse (0-31) and D (32-63)
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = lane >> 4, li = lane & 15;
    int kt, h;
    int64_t b;
    ab_tile(a, kt, h, b);
    const int heads = gridDim.y, B = gridDim.z;
    const int T = a.T, T32 = (T + 31) / 32 * 32;
    const int k0 = (kt * WAVES + wave) * 16;
    const bool active = k0 < T;
    const int64_t bh = b * heads + h;
    const int64_t PB = (int64_t)B * heads * T32 * CH / 4;
    const h8v* qr = a.packs + AB_QR * PB + bh * (T32 / 16) * NJ * 128;
    const h8v* dor = a.packs + AB_DOR * PB + bh * (T32 / 16) * NJ * 128;
    const h8v* dot = a.packs + AB_DOT * PB + bh * (T32 / 32) * ND * 128;
    const h8v* qtp = a.packs + AB_QT * PB + bh * (T32 / 32) * ND * 128;
    const float* lsrc = a.lse + bh * T;
    const float* dsrc = a.dd + bh * T;
    // wave 0 also moves the block's 32 log-sum-exps and 32 D (one dword piece)
    auto issue = [&](int ib, int stage) {
#pragma unroll
        for (int i = 0; i < PPW; ++i) {
            const int piece = wave + WAVES * i;
            const h8v* src = piece < QP             ? qr + (int64_t)ib * QP * 64 + piece * 64
                             : piece < QP + OP      ? dor + (int64_t)ib * OP * 64 + (piece - QP) * 64
                             : piece < QP + OP + TO ? dot + (int64_t)ib * TO * 64 + (piece - QP - OP) * 64
                                                    : qtp + (int64_t)ib * TQ * 64 + (piece - QP - OP - TO) * 64;
            __builtin_amdgcn_global_load_lds((const void*)(src + lane),
                                             (__attribute__((address_space(3))) void*)&ring[stage][piece * 64], 16, 0, 0);
        }
        if (wave == 0) {
            const int q = min(32 * ib + (lane & 31), T - 1);   // clamped: padded queries are masked
            const float* src = lane < 32 ? lsrc + q : dsrc + q;
            __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)&lring[stage][0],
                                             4, 0, 0);
        }
    };
    const int nblk = T32 / 32;
#pragma unroll
    for (int i = 0; i < NS - 1; ++i)
        if (i < nblk) issue(i, i);

    const int C3 = 3 * a.C;
    const int tk = min(k0 + li, T - 1);
    const float sg = ab_sigma(a.amax + bh * (T32 / 32) * 2, T32 / 32, CH);
    h8v kh[NJ], kl[NJ], vh[NJ], vl[NJ];
    {
        const float* kp = a.qkv + (b * (int64_t)T + tk) * C3 + (int64_t)h * 3 * CH + CH + 8 * g;
        const float ks = kln2(a.scale);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            float v[8], w[8];
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                v[t] = ab_f32(kp[32 * j + t] * ks);
                w[t] = kp[CH + 32 * j + t];
            }
            split8_f16(v, kh[j], kl[j]);
            split8_f16(w, vh[j], vl[j]);
        }
    }
    f4 dK[ND], dV[ND];
#pragma unroll
    for (int d = 0; d < ND; ++d) dK[d] = dV[d] = f4{0.f, 0.f, 0.f, 0.f};

    for (int ib = 0; ib < nblk; ++ib) {
        const int qb = 32 * ib, stage = ib % NS;
        if (NS == 3 && ib + 1 < nblk) {
            if (wave == 0)
                __builtin_amdgcn_s_waitcnt(vmcnt_wait(PPW + 1));
            else
                __builtin_amdgcn_s_waitcnt(vmcnt_wait(PPW));
        } else {
            __builtin_amdgcn_s_waitcnt(vmcnt_wait(0));
        }
        __builtin_amdgcn_s_barrier();
        if (ib + NS - 1 < nblk) issue(ib + NS - 1, (ib + NS - 1) % NS);
        if (!active) continue;
        const h8v* R = &ring[stage][lane];
        f4 st[2], dp[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            st[u] = dp[u] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const h8v ah = R[((u * NJ + j) * 2) * 64], al = R[((u * NJ + j) * 2 + 1) * 64];
                st[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, kh[j], st[u], 0, 0, 0);
                st[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, kl[j], st[u], 0, 0, 0);
                st[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, kh[j], st[u], 0, 0, 0);
                const h8v oh = R[(QP + (u * NJ + j) * 2) * 64], ol = R[(QP + (u * NJ + j) * 2 + 1) * 64];
                dp[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ol, vh[j], dp[u], 0, 0, 0);
                dp[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(oh, vl[j], dp[u], 0, 0, 0);
                dp[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(oh, vh[j], dp[u], 0, 0, 0);
            }
        }
        // lane (g, li): query qb + 16 u + 4 g + r of key li (element 4 u + r of the
        // B operands below: query kmap(g, t), the column packs' k order)
        float p[8], ds[8];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const f4 l4 = *(const f4*)&lring[stage][16 * u + 4 * g];
            const f4 d4 = *(const f4*)&lring[stage][32 + 16 * u + 4 * g];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float pv = __builtin_amdgcn_exp2f(st[u][r] - l4[r] * 1.44269504088896340736f);
                if (qb + 32 > T && qb + 16 * u + 4 * g + r >= T) pv = 0.f;
                p[4 * u + r] = pv;
                ds[4 * u + r] = ab_f32(pv * (dp[u][r] - d4[r] * sg));
            }
        }
        h8v ph, pl, sh, sl;
        split8_f16(p, ph, pl);
        split8_f16(ds, sh, sl);
#pragma unroll
        for (int d = 0; d < ND; ++d) {
            const h8v oh = R[(QP + OP + 2 * d) * 64], ol = R[(QP + OP + 2 * d + 1) * 64];
            dV[d] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ol, ph, dV[d], 0, 0, 0);
            dV[d] = __builtin_amdgcn_mfma_f32_16x16x32_f16(oh, pl, dV[d], 0, 0, 0);
            dV[d] = __builtin_amdgcn_mfma_f32_16x16x32_f16(oh, ph, dV[d], 0, 0, 0);
            const h8v qh = R[(QP + OP + TO + 2 * d) * 64], ql = R[(QP + OP + TO + 2 * d + 1) * 64];
            dK[d] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ql, sh, dK[d], 0, 0, 0);
            dK[d] = __builtin_amdgcn_mfma_f32_16x16x32_f16(qh, sl, dK[d], 0, 0, 0);
            dK[d] = __builtin_amdgcn_mfma_f32_16x16x32_f16(qh, sh, dK[d], 0, 0, 0);
        }
    }
    if (!active || k0 + li >= T) return;
    const float ks2 = a.scale * a.scale / sg, vs = 1.f / sg;
    float* out = a.dqkv + (b * (int64_t)T + k0 + li) * C3 + (int64_t)h * 3 * CH;
#pragma unroll
    for (int d = 0; d < ND; ++d) {
        *(f4*)(out + CH + 16 * d + 4 * g) = dK[d] * ks2;
        *(f4*)(out + 2 * CH + 16 * d + 4 * g) = dV[d] * vs;
    }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
int launch_gn_bwd(const GnbArgs& a0, int B, hipStream_t st) {
    CFD_REQUIRE(a0.Ctot % 32 == 0 && a0.C1 % 4 == 0 && a0.C2 % 4 == 0 && a0.Ctot <= 1024, CFD_ESHAPE,
                "GroupNorm32 backward needs channels % 32 == 0 (<= 1024)");
    CFD_REQUIRE(a0.C2 == 0 || a0.out2, CFD_ESTATE, "GroupNorm backward: second-source gradient needs out2");
    GnbArgs a = a0;
    // with parameter partials (training) ~256 blocks over the batch, >= 16 row passes
    // a chunk: the (B x chunks) partials are then few enough for one accumulation
    // block per 32 channels (4096 partial rows at 128^2 took 51 us to accumulate)
    if (a.ppart) {
        const int rows = std::max(1, 256 / (a.Ctot / 4));
        a.nchunks = (int)std::min<int64_t>({kGnMaxChunks, std::max<int64_t>(1, ceil_div(256, B)),
                                            std::max<int64_t>(1, ceil_div(a.HW, 16 * rows))});
    } else {
        // no parameter partials (the DPS adjoint): gn2's chunking, the statistics
        // finalised inside the apply pass (config-D input-VJP -0.1-0.2 ms), with
        // gn2's 256-thread layout (<= 64 chunks: config D's levels).  A small
        // planned batch's 1024-thread chunks (Case4 at one chain: 96^2, 48^2) keep
        // the finalize launch: every apply workgroup re-reading the 256 chunk
        // partials cost more than it (real Case4 18.71 vs 18.55 ms per step, r05o)
        const int nc2 = gn2_chunks(a.HW, a.plan_b);
        if (gn2_threads(nc2) == 256) {
            a.nchunks = nc2;
            a.B = B;
            const dim3 grid((unsigned)a.nchunks, (unsigned)B);
            hipLaunchKernelGGL((gn_bwd_partial_kernel<false, 256>), grid, dim3(256), 0, st, a);
            check_launch("gn_bwd_partial_kernel");
            hipLaunchKernelGGL(gn_bwd_apply2_kernel<256>, grid, dim3(256), 0, st, a);
            check_launch("gn_bwd_apply2_kernel");
            return a.nchunks;
        }
        a.nchunks = gn_chunks(a.HW);
    }
    a.B = B;
    if (a.ppart)
        hipLaunchKernelGGL(gn_bwd_partial_kernel<true>, dim3(a.nchunks, B), dim3(256), 0, st, a);
    else
        hipLaunchKernelGGL(gn_bwd_partial_kernel<false>, dim3(a.nchunks, B), dim3(256), 0, st, a);
    check_launch("gn_bwd_partial_kernel");
    hipLaunchKernelGGL(gn_bwd_finalize_kernel, dim3(B), dim3(1024), 0, st, a);
    check_launch("gn_bwd_finalize_kernel");
    const int64_t nq = ceil_div((int64_t)B * a.HW, GNB_PIX) * (a.Ctot / 4);
    hipLaunchKernelGGL(gn_bwd_apply_kernel, dim3((unsigned)ceil_div(nq, 256)), dim3(256), 0, st, a);
    check_launch("gn_bwd_apply_kernel");
    return a.nchunks;
}

template <int CH>
static void launch_attn_bwd_ch(const AttnBwdArgs& a, dim3 grid, hipStream_t st) {
    hipLaunchKernelGGL(attn_bwd_dq_kernel<CH>, grid, dim3(256), 0, st, a);
    check_launch("attn_bwd_dq_kernel");
    hipLaunchKernelGGL(attn_bwd_dkv_kernel<CH>, grid, dim3(256), 0, st, a);
    check_launch("attn_bwd_dkv_kernel");
}

void launch_attention_bwd(const AttnBwdArgs& a, int CH, int heads, int B, hipStream_t st) {
    CFD_REQUIRE(a.T % 16 == 0, CFD_ESHAPE, "attention backward needs T % 16 == 0");
    const dim3 grid((unsigned)ceil_div(a.T, 64), heads, B);
    switch (CH) {
        case 16: return launch_attn_bwd_ch<16>(a, grid, st);
        case 32: return launch_attn_bwd_ch<32>(a, grid, st);
        case 64: return launch_attn_bwd_ch<64>(a, grid, st);
        case 128: return launch_attn_bwd_ch<128>(a, grid, st);
        default: throw Error{CFD_ESHAPE, "attention head channels must be 16, 32, 64 or 128"};
    }
}

static int vjp_env(const char* name, int dflt) {
    const char* e = getenv(name);
    return e ? atoi(e) : dflt;
}

template <int CH, int WAVES>
static void launch_attn_bwd_split_ch(const AttnBwdArgs& a, dim3 grid, hipStream_t st) {
    constexpr int NJ = CH / 32, ND = CH / 16;
    constexpr int NPQ = 8 * NJ + 2 * ND, NPK = 8 * NJ + 4 * ND;   // KiB per ring stage
    constexpr int NSQ = NPQ * 3 <= 96 ? 3 : 2, NSK = NPK * 3 <= 96 ? 3 : 2;
    hipLaunchKernelGGL((attn_bwd_dq_split_kernel<CH, WAVES, NSQ>), grid, dim3(64 * WAVES), 0, st, a);
    check_launch("attn_bwd_dq_split_kernel");
    hipLaunchKernelGGL((attn_bwd_dkv_split_kernel<CH, WAVES, NSK>), grid, dim3(64 * WAVES), 0, st, a);
    check_launch("attn_bwd_dkv_split_kernel");
}

void launch_attention_bwd_split(const AttnBwdArgs& a0, int CH, int heads, int B, float* ws, hipStream_t st) {
    CFD_REQUIRE(attention_bwd_split_ok(a0.T, CH), CFD_ESHAPE,
                "split attention backward needs head channels 32, 64 or 128 and T % 16 == 0");
    AttnBwdArgs a = a0;
    const int T32 = (a.T + 31) / 32 * 32;
    a.heads = heads;
    a.packs = (h8v*)ws;
    a.amax = ws + (size_t)B * AB_NPACK * T32 * a.C;
    static const int xcd = vjp_env("CFD_ATTN_XCD", 1);
    a.xcdmap = xcd && (heads * B) % 8 == 0 ? 1 : 0;
    const dim3 pgrid((unsigned)(T32 / 32), (unsigned)(B * heads));
    switch (CH) {
        case 32: hipLaunchKernelGGL(attn_bwd_prep_kernel<32>, pgrid, dim3(256), 0, st, a); break;
        case 64: hipLaunchKernelGGL(attn_bwd_prep_kernel<64>, pgrid, dim3(256), 0, st, a); break;
        default: hipLaunchKernelGGL(attn_bwd_prep_kernel<128>, pgrid, dim3(256), 0, st, a); break;
    }
    check_launch("attn_bwd_prep_kernel");
    switch (CH) {
        case 32: hipLaunchKernelGGL(attn_bwd_pack_do_kernel<32>, pgrid, dim3(256), 0, st, a); break;
        case 64: hipLaunchKernelGGL(attn_bwd_pack_do_kernel<64>, pgrid, dim3(256), 0, st, a); break;
        default: hipLaunchKernelGGL(attn_bwd_pack_do_kernel<128>, pgrid, dim3(256), 0, st, a); break;
    }
    check_launch("attn_bwd_pack_do_kernel");
    // 4 waves (64 queries / keys) per workgroup; 8 where that still leaves >= 256 workgroups
    static const int w8 = vjp_env("CFD_ATTN_BWD_W8", 1);
    const bool eight = w8 && CH >= 64 && (int64_t)ceil_div(a.T, 128) * heads * B >= 256;
    const dim3 grid((unsigned)ceil_div(a.T, eight ? 128 : 64), heads, B);
    switch (CH) {
        case 32: return launch_attn_bwd_split_ch<32, 4>(a, grid, st);   // 12 pieces: 4 waves
        case 64: return eight ? launch_attn_bwd_split_ch<64, 8>(a, grid, st) : launch_attn_bwd_split_ch<64, 4>(a, grid, st);
        default: return eight ? launch_attn_bwd_split_ch<128, 8>(a, grid, st) : launch_attn_bwd_split_ch<128, 4>(a, grid, st);
    }
}

void launch_add(float* y, const float* x, int64_t n, hipStream_t st) {
    CFD_REQUIRE(n % 4 == 0, CFD_ESHAPE, "add: n % 4");
    hipLaunchKernelGGL(add_kernel, dim3((unsigned)ceil_div(n / 4, 256)), dim3(256), 0, st, y, x, n / 4);
    check_launch("add_kernel");
}

}  // namespace cfd
