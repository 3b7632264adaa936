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
template <bool PP>
__global__ __launch_bounds__(256) void gn_bwd_partial_kernel(GnbArgs a) {
    const int chunk = blockIdx.x;
    const int64_t b = blockIdx.y;
    const int Ctot = a.Ctot, cq = Ctot / 4, cpg = Ctot / 32;
    const int HW = a.HW;
    const int p0 = (int)((int64_t)HW * chunk / a.nchunks), p1 = (int)((int64_t)HW * (chunk + 1) / a.nchunks);
    const int rows = 256 / cq;
    const int q = threadIdx.x % cq, r0 = threadIdx.x / cq;
    __shared__ double red[2][1024];
    if (r0 < rows) {
        double s[4] = {0, 0, 0, 0}, s2[4] = {0, 0, 0, 0};
        const int c0 = 4 * q;
        const GnbQuad k = gnb_quad(a, b, c0);
        for (int p = p0 + r0; p < p1; p += rows) {
            f4 g, xh;
            if constexpr (PP)
                gnb_load_d(a, k, b * HW + p, c0, g, xh);
            else
                gnb_load(a, k, b * HW + p, c0, g, xh);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                s[j] += g[j];
                s2[j] += (double)g[j] * xh[j];
            }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            red[0][r0 * Ctot + c0 + j] = s[j];
            red[1][r0 * Ctot + c0 + j] = s2[j];
        }
    }
    __syncthreads();
    if (threadIdx.x < 32) {
        const int grp = threadIdx.x;
        double ts = 0, ts2 = 0;
        for (int r = 0; r < rows; ++r)
            for (int c = grp * cpg; c < (grp + 1) * cpg; ++c) {
                if constexpr (PP) {
                    const double gm = (double)a.gamma[c];
                    ts += gm * red[0][r * Ctot + c];
                    ts2 += gm * red[1][r * Ctot + c];
                } else {
                    ts += red[0][r * Ctot + c];
                    ts2 += red[1][r * Ctot + c];
                }
            }
        double* dst = a.part + ((b * a.nchunks + chunk) * 32 + grp) * 2;
        dst[0] = ts;
        dst[1] = ts2;
    }
    if constexpr (PP) {   // rows in order, per channel: (sum dz_eff xhat, sum dz_eff)
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

void launch_add(float* y, const float* x, int64_t n, hipStream_t st) {
    CFD_REQUIRE(n % 4 == 0, CFD_ESHAPE, "add: n % 4");
    hipLaunchKernelGGL(add_kernel, dim3((unsigned)ceil_div(n / 4, 256)), dim3(256), 0, st, y, x, n / 4);
    check_launch("add_kernel");
}

}  // namespace cfd
