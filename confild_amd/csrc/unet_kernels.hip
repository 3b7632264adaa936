// Latent U-Net kernels for gfx950 (K1-K5 of DESIGN.md), fp32, NHWC activations.
//
//   conv_gemm   K1/K2  implicit-GEMM 3x3 / 1x1 convolution on fp32 MFMA 16x16x4,
//                      bias / timestep-embedding / residual fused in the epilogue,
//                      concat-free two-source input (skip connections), stride-2
//                      (Downsample) and nearest-2x (Upsample) addressing, split-K
//                      for the low-resolution levels;
//   gn_partial/apply K3 GroupNorm(32) statistics + normalise (+SiLU), written once;
//   attention   K4     QKVAttentionLegacy (flash-style, fp32 MFMA, online softmax);
//   temb/linear K5     timestep embedding + time_embed MLP + all emb_layers;
//   conv_in / conv_out the 1-channel first/last convolutions (VALU).
#include <algorithm>
#include <cstdlib>

#include "unet_kernels.hpp"

namespace cfd {

// ---------------------------------------------------------------------------
// K3: GroupNorm(32), eps 1e-5, statistics in float64 (nn.py:17-19 computes GN
// in fp32; double accumulation keeps the result within rounding of the exact
// moments).  Two passes over the data:
//   gn_partial  per (pixel chunk, sample): per-group sum and sum of squares of
//               its pixels, read as coalesced full-channel rows (two sources =
//               the concat-free skip input);
//   gn_apply    per-(b, c) scale/shift from the partials (fixed summation order,
//               deterministic), then y = x*scale + shift (+ SiLU) written as one
//               contiguous (B, HW, Ctot) tensor for the next convolution.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void gn_partial_kernel(GnArgs a) {
    const int chunk = blockIdx.x;
    const int64_t b = blockIdx.y;
    const int Ctot = a.Ctot, cq = Ctot / 4, cpg = Ctot / 32;
    const int HW = a.HW;
    const int p0 = (int)((int64_t)HW * chunk / a.nchunks), p1 = (int)((int64_t)HW * (chunk + 1) / a.nchunks);
    // thread t owns channel quad q = t % cq for pixel rows r0 = t / cq (step `rows`);
    // rows * cq <= 256 so rows * Ctot <= 1024 per-channel sums per block
    const int rows = 256 / cq;
    const int q = threadIdx.x % cq, r0 = threadIdx.x / cq;
    __shared__ double red[2][1024];
    if (r0 < rows) {
        double s[4] = {0, 0, 0, 0}, s2[4] = {0, 0, 0, 0};
        const int c0 = 4 * q;
        for (int p = p0 + r0; p < p1; p += rows) {
            const int64_t pix = b * HW + p;
            const f4 v = c0 < a.C1 ? *(const f4*)(a.src1 + pix * a.C1 + c0)
                                   : *(const f4*)(a.src2 + pix * a.C2 + (c0 - a.C1));
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                s[j] += v[j];
                s2[j] += (double)v[j] * v[j];
            }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            red[0][r0 * Ctot + c0 + j] = s[j];
            red[1][r0 * Ctot + c0 + j] = s2[j];
        }
    }
    __syncthreads();
    // one thread per group sums its channels over the rows in a fixed order
    if (threadIdx.x < 32) {
        const int grp = threadIdx.x;
        double ts = 0, ts2 = 0;
        for (int r = 0; r < rows; ++r)
            for (int c = grp * cpg; c < (grp + 1) * cpg; ++c) {
                ts += red[0][r * Ctot + c];
                ts2 += red[1][r * Ctot + c];
            }
        double* dst = a.part + ((b * a.nchunks + chunk) * 32 + grp) * 2;
        dst[0] = ts;
        dst[1] = ts2;
    }
}

// SiLU as x * rcp(1 + 2^(-x log2 e)): v_exp_f32 and v_rcp_f32 (~1 ulp each) instead
// of ocml's expf and an IEEE division (~21 instructions per element in the
// GroupNorm apply loops); the backward's sigmoid (unet_vjp.hip) is the same form
__device__ __forceinline__ float silu_f(float x) {
    return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * -1.44269504088896340736f));
}

// per (b, c): scale = rstd*gamma, shift = beta - mean*scale (ATen CPU GroupNorm
// affine form) from the chunk partials: 32 threads per group each summing every
// 32nd chunk, then a fixed-order tree (up to kGnMaxChunks chunks at large latents).
__global__ __launch_bounds__(1024) void gn_finalize_kernel(GnArgs a) {
    const int64_t b = blockIdx.x;
    const int Ctot = a.Ctot, cpg = Ctot / 32;
    __shared__ float sh_mean[32], sh_rstd[32];
    __shared__ double red[2][1024];
    const int grp = threadIdx.x >> 5, sub = threadIdx.x & 31;
    {
        // every 32nd chunk, four loads in flight, added in chunk order
        double s = 0, s2 = 0;
        for (int ch = sub; ch < a.nchunks; ch += 128) {
            double2 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int c = ch + 32 * u;
                v[u] = c < a.nchunks ? *(const double2*)(a.part + ((b * a.nchunks + c) * 32 + grp) * 2)
                                     : double2{0.0, 0.0};
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                s += v[u].x;
                s2 += v[u].y;
            }
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
        const double n = (double)a.HW * cpg;
        const double mean = red[0][threadIdx.x] / n;
        const double var = fmax(red[1][threadIdx.x] / n - mean * mean, 0.0);
        sh_mean[grp] = (float)mean;
        sh_rstd[grp] = (float)(1.0 / sqrt(var + (double)a.eps));
        if (a.stats) {
            a.stats[(b * 32 + grp) * 2 + 0] = sh_mean[grp];
            a.stats[(b * 32 + grp) * 2 + 1] = sh_rstd[grp];
        }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < Ctot; c += blockDim.x) {
        const int g = c / cpg;
        const float sc = sh_rstd[g] * a.gamma[c];
        a.ss[(b * Ctot + c) * 2 + 0] = sc;
        a.ss[(b * Ctot + c) * 2 + 1] = a.beta[c] - sh_mean[g] * sc;
    }
}

// store 4 consecutive channels of a GroupNorm output at element offset e of a.out:
// fp32, or (a.out_bf16) bf16 by the same RNE conversion K1hb applies when it
// stages an fp32 operand (v_cvt_pk_bf16_f32), so the consumer sees the same bits
__device__ __forceinline__ void gn_store4(const GnArgs& a, int64_t e, const f4& y) {
    if (a.out_bf16)
        *(bf16x4*)((__bf16*)(void*)a.out + e) = __builtin_convertvector(y, bf16x4);
    else
        *(f4*)(a.out + e) = y;
}

// every thread of the workgroup calls it: max of mx over the workgroup, then one
// atomicMax of its float bits (non-negative: the integer order is the float order)
__device__ __forceinline__ void block_amax_atomic(float mx, unsigned* out) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    __shared__ float wmx[16];
    const int nw = (blockDim.x + 63) >> 6;
    if ((threadIdx.x & 63) == 0) wmx[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
        float m = wmx[0];
        for (int w = 1; w < nw; ++w) m = fmaxf(m, wmx[w]);
        atomicMax(out, __float_as_uint(m));
    }
}
__device__ __forceinline__ float amax4(const f4& y) {
    return fmaxf(fmaxf(fabsf(y[0]), fabsf(y[1])), fmaxf(fabsf(y[2]), fabsf(y[3])));
}

// y = x*scale + shift (+ SiLU), one float4 per thread, written as one
// contiguous (B, HW, Ctot) tensor (the concat of two sources materialised here).
__global__ __launch_bounds__(256) void gn_apply_kernel(GnArgs a) {
    const int cq = a.Ctot / 4;
    float mx = 0.f;
    // grid-stride over float4 quads (a bounded grid: one range atomic per workgroup)
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (int64_t)a.B * a.HW * cq;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t pix = i / cq;
        const int c0 = (int)(i - pix * cq) * 4;
        const int64_t b = pix / a.HW;
        f4 v = c0 < a.C1 ? *(const f4*)(a.src1 + pix * a.C1 + c0) : *(const f4*)(a.src2 + pix * a.C2 + (c0 - a.C1));
        const float* ss = a.ss + (b * a.Ctot + c0) * 2;
        const f4 s01 = *(const f4*)ss, s23 = *(const f4*)(ss + 4);
        v[0] = v[0] * s01[0] + s01[1];
        v[1] = v[1] * s01[2] + s01[3];
        v[2] = v[2] * s23[0] + s23[1];
        v[3] = v[3] * s23[2] + s23[3];
        if (a.silu) {
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = silu_f(v[j]);
        }
        gn_store4(a, pix * a.Ctot + c0, v);
        mx = fmaxf(mx, amax4(v));   // every quad of the grid-stride loop, not the last
    }
    if (a.amax_out) block_amax_atomic(mx, a.amax_out);
}

// GroupNorm in one launch, one workgroup per (sample, group), for HW x cpg <=
// NT x IPT x 4: every thread loads its IPT float4 at once (the loads pipeline
// instead of forming a latency chain), a fixed-order float64 tree gives mean /
// rstd, and the same registers are normalised (one HBM read): y = x*scale +
// shift (+ SiLU).  Same statistics, affine form and output as the three-kernel
// path; batch-invariant (a sample's summation order does not depend on B).
template <int IPT, int NT = 512>
__global__ __launch_bounds__(NT) void gn_fused_reg_kernel(GnArgs a) {
    const int L = blockIdx.x;
    const int64_t b = L % a.B;
    const int grp = L / a.B;
    const int Ctot = a.Ctot, cpg = Ctot / 32, nq = cpg / 4;
    const int HW = a.HW;
    const int rows = NT / nq;
    CFD_DASSERT(grp < 32 && nq >= 1 && (HW + rows - 1) / rows <= IPT);   // every pixel has a register slot
    const int t = threadIdx.x;
    CFD_STAMP(a.stamps, 4, a.seq, 0);
    const bool act = t < rows * nq;
    const int q = t % nq, r0 = t / nq;
    const int c = grp * cpg + 4 * q;
    const float* src = c < a.C1 ? a.src1 + b * HW * a.C1 + c : a.src2 + b * HW * a.C2 + (c - a.C1);
    const int ld = c < a.C1 ? a.C1 : a.C2;
    constexpr int NWV = NT / 64;
    __shared__ double wred[2][NWV];
    __shared__ float sh[2][32];
    // this group's gamma / beta, loaded now (the finalize would otherwise wait one
    // more memory latency for them after the reduction)
    float gam = 0.f, bet = 0.f;
    if (t < cpg) {
        gam = a.gamma[grp * cpg + t];
        bet = a.beta[grp * cpg + t];
    }
    f4 v[IPT];
    bool ksrc = false;
    if constexpr (IPT <= 16) ksrc = a.kpart && c < a.C1;  // (gn_takes_splitk: IPT <= 16)
    if (ksrc) {  // constant false for IPT > 16: the branch folds away
        // split-K source (GnArgs::kpart): reduce, epilogue, store x, keep it
        const int64_t slab = (int64_t)a.B * HW * a.C1;
        f4 kb = {0.f, 0.f, 0.f, 0.f}, ke = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (a.kbias) kb[j] = a.kbias[c + j];
            if (a.kemb) ke[j] = a.kemb[b * a.kemb_stride + c + j];
        }
        // every load first (the partials, then the residual), every store after:
        // kx may alias neither input, but the compiler cannot know that, and an
        // interleaved store would serialise the loads behind it
        const float* __restrict__ kpart = a.kpart;
        const float* __restrict__ kres = a.kres;
        float* __restrict__ kx = a.kx;
        const int64_t ib = (b * HW + r0) * a.C1 + c, istep = (int64_t)rows * a.C1;
        // the residual, slab 0 and the first UN slabs are one round of loads in
        // flight (the split-K levels are latency-bound: every dependent round is a
        // memory latency); the slabs are added in split order, as splitk_reduce does
        f4 rs[IPT];
#pragma unroll
        for (int k = 0; k < IPT; ++k) {
            const int p = r0 + k * rows;
            rs[k] = kres && act && p < HW ? *(const f4*)(kres + ib + k * istep) : f4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int k = 0; k < IPT; ++k) {
            const int p = r0 + k * rows;
            v[k] = act && p < HW ? *(const f4*)(kpart + ib + k * istep) : f4{0.f, 0.f, 0.f, 0.f};
        }
        // 2 slabs per round in the 1024-thread tier: 55 VGPRs, two workgroups per CU (the
        // 256 launches of a B = 8 32^2 level fit one round on a CU half: pipelined step
        // +0.4 %, whole chip flat, the same bits; profiles/r06v_gn1024_ab.json)
        constexpr int UN = IPT <= 2 ? (NT >= 1024 ? 2 : 8) : IPT <= 4 ? 4 : 1;
        for (int sp = 1; sp < a.ksplits; sp += UN) {
            f4 u[UN][IPT];
#pragma unroll
            for (int q2 = 0; q2 < UN; ++q2)
#pragma unroll
                for (int k = 0; k < IPT; ++k) {
                    const int p = r0 + k * rows;
                    u[q2][k] = sp + q2 < a.ksplits && act && p < HW
                                   ? *(const f4*)(kpart + (sp + q2) * slab + ib + k * istep)
                                   : f4{0.f, 0.f, 0.f, 0.f};
                }
#pragma unroll
            for (int q2 = 0; q2 < UN; ++q2)
                if (sp + q2 < a.ksplits) {
#pragma unroll
                    for (int k = 0; k < IPT; ++k) v[k] += u[q2][k];
                }
        }
#pragma unroll
        for (int k = 0; k < IPT; ++k) {
            const int p = r0 + k * rows;
            if (act && p < HW) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    float y = a.kbias ? v[k][j] + kb[j] : v[k][j];
                    if (a.kemb) y = y + ke[j];
                    if (kres) y = rs[k][j] + y;
                    v[k][j] = y;
                }
                if (kx) *(f4*)(kx + ib + k * istep) = v[k];   // null: nobody reads the raw sum
            }
        }
    } else {
#pragma unroll
        for (int k = 0; k < IPT; ++k) {
            const int p = r0 + k * rows;
            v[k] = act && p < HW ? *(const f4*)(src + (int64_t)p * ld) : f4{0.f, 0.f, 0.f, 0.f};
        }
    }
    CFD_STAMP(a.stamps, 4, a.seq, 1);
    double s = 0, s2 = 0;
#pragma unroll
    for (int k = 0; k < IPT; ++k)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            s += v[k][j];
            s2 += (double)v[k][j] * v[k][j];
        }
    // fixed-order reduction: a butterfly within each wave (lane 0's sum), then
    // the NWV wave sums in wave order -- one barrier instead of a log2(NT)-level
    // LDS tree (measured in-kernel: the tree was ~2-3 us of a 6-10 us GroupNorm)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        s += __shfl_xor(s, o);
        s2 += __shfl_xor(s2, o);
    }
    if ((t & 63) == 0) {
        wred[0][t >> 6] = s;
        wred[1][t >> 6] = s2;
    }
    __syncthreads();
    if (t < cpg) {
        double S = 0.0, S2 = 0.0;
#pragma unroll
        for (int w = 0; w < NWV; ++w) {
            S += wred[0][w];
            S2 += wred[1][w];
        }
        const double n = (double)HW * cpg;
        const double mean = S / n;
        const double var = fmax(S2 / n - mean * mean, 0.0);
        const float mf = (float)mean, rf = (float)(1.0 / sqrt(var + (double)a.eps));
        const int cc = grp * cpg + t;
        const float sc = rf * gam;
        const float sf = bet - mf * sc;
        sh[0][t] = sc;
        sh[1][t] = sf;
        a.ss[(b * Ctot + cc) * 2 + 0] = sc;
        a.ss[(b * Ctot + cc) * 2 + 1] = sf;
        if (a.stats && t == 0) {
            a.stats[(b * 32 + grp) * 2 + 0] = mf;
            a.stats[(b * 32 + grp) * 2 + 1] = rf;
        }
    }
    __syncthreads();
    CFD_STAMP(a.stamps, 4, a.seq, 2);
    float mx = 0.f;
    if (act) {
        f4 sc, sf;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            sc[j] = sh[0][4 * q + j];
            sf[j] = sh[1][4 * q + j];
        }
        const int64_t dst = b * HW * Ctot + c;
#pragma unroll
        for (int k = 0; k < IPT; ++k) {
            const int p = r0 + k * rows;
            if (p < HW) {
                f4 y;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    y[j] = v[k][j] * sc[j] + sf[j];
                    if (a.silu) y[j] = silu_f(y[j]);
                }
                gn_store4(a, dst + (int64_t)p * Ctot, y);
                mx = fmaxf(mx, amax4(y));
            }
        }
    }
    if (a.amax_out) block_amax_atomic(mx, a.amax_out);
#ifdef CFD_STAMPS
    __builtin_amdgcn_s_waitcnt(0);
#endif
    CFD_STAMP(a.stamps, 4, a.seq, 4);
}

// ---------------------------------------------------------------------------
// K3c: GroupNorm(32)(+SiLU) in two launches over pixel chunks, full pixel rows
// (every channel of a pixel: 512-B lines read once, not one 16-B group slice per
// workgroup and line).  gn2_stats: per (chunk, sample) the per-group float64 sum
// and sum of squares of its pixels (a split-K source reduced on the way, as the
// register kernel does, and its sum stored at kx); gn2_apply: every workgroup
// reduces its sample's chunk partials itself (fixed order, identical on every
// workgroup), forms scale / shift and normalises its chunk.  The chunk count is a
// function of HW only, so a sample's statistics do not depend on the batch.  For
// the large latents (config E 128^2) and, with more workgroups than groups, the
// small batches.
// ---------------------------------------------------------------------------
// Up to 128^2 at the default planned batch (8): 256-thread workgroups, up to 64
// chunks (config E, B = 1 64^2); a smaller planned batch (ConvArgs::plan_b, e.g.
// Case4 at one chain) takes up to 64 * 8 / plan_b (<= 256) chunks.  Beyond 128^2
// (Case4's 384^2 / 192^2 levels): kGn2BigChunks chunks.  Above 64 chunks the
// workgroups have 1024 threads (gn2_threads): a batch-1 sample still fills the
// chip (64 KB of loads in flight per CU) and the apply pass reduces the partials
// in one round of loads (32 lanes per group, nchunks / 32 each).
int gn2_chunks(int HW, int plan_b) {
    if (HW > kGn2BigHW) return kGn2BigChunks;
    const int pb = plan_b > 0 ? plan_b : 8;
    const int cap = std::min(kGn2BigChunks, std::max(64, 64 * 8 / pb));
    return (int)std::max<int64_t>(1, std::min<int64_t>(cap, HW / 16));
}

template <int NT>
__global__ __launch_bounds__(NT) void gn2_stats_kernel(GnArgs a) {
    const int chunk = blockIdx.x;
    const int64_t b = blockIdx.y;
    const int Ctot = a.Ctot, cq = Ctot / 4, cpg = Ctot / 32;
    const int HW = a.HW, NC = gridDim.x;
    const int p0 = (int)((int64_t)HW * chunk / NC), p1 = (int)((int64_t)HW * (chunk + 1) / NC);
    const int rows = NT / cq;
    const int q = threadIdx.x % cq, r0 = threadIdx.x / cq;
    const int c0 = 4 * q;
    const bool act = r0 < rows;
    const bool ksrc = a.kpart && c0 < a.C1;
    __shared__ double red[2][4 * NT];   // rows * Ctot = 4 * NT
    double s[4] = {0, 0, 0, 0}, s2[4] = {0, 0, 0, 0};
    f4 kb = {0.f, 0.f, 0.f, 0.f}, ke = {0.f, 0.f, 0.f, 0.f};
    if (ksrc) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (a.kbias) kb[j] = a.kbias[c0 + j];
            if (a.kemb) ke[j] = a.kemb[b * a.kemb_stride + c0 + j];
        }
    }
    const int64_t slab = (int64_t)a.B * HW * a.C1;
    constexpr int U = 4;   // pixel rows in flight per thread
    if (act) {
        for (int pb = p0 + r0; pb < p1; pb += U * rows) {
            f4 v[U];
            if (ksrc) {   // splitk_reduce's order: slab 0, the others in split order, bias, emb, residual
                f4 rs[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int p = pb + u * rows;
                    const int64_t e = (b * HW + p) * a.C1 + c0;
                    rs[u] = a.kres && p < p1 ? *(const f4*)(a.kres + e) : f4{0.f, 0.f, 0.f, 0.f};
                    v[u] = p < p1 ? *(const f4*)(a.kpart + e) : f4{0.f, 0.f, 0.f, 0.f};
                }
                for (int sp = 1; sp < a.ksplits; ++sp) {
                    f4 w[U];
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const int p = pb + u * rows;
                        w[u] = p < p1 ? *(const f4*)(a.kpart + sp * slab + (b * HW + p) * a.C1 + c0)
                                      : f4{0.f, 0.f, 0.f, 0.f};
                    }
#pragma unroll
                    for (int u = 0; u < U; ++u) v[u] += w[u];
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int p = pb + u * rows;
                    if (p >= p1) continue;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        float y = a.kbias ? v[u][j] + kb[j] : v[u][j];
                        if (a.kemb) y = y + ke[j];
                        if (a.kres) y = rs[u][j] + y;
                        v[u][j] = y;
                    }
                    *(f4*)(a.kx + (b * HW + p) * a.C1 + c0) = v[u];
                }
            } else {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int p = pb + u * rows;
                    const int64_t pix = b * HW + p;
                    v[u] = p >= p1 ? f4{0.f, 0.f, 0.f, 0.f}
                         : c0 < a.C1 ? *(const f4*)(a.src1 + pix * a.C1 + c0)
                                     : *(const f4*)(a.src2 + pix * a.C2 + (c0 - a.C1));
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int j = 0; j < 4; ++j) {   // zero padding adds nothing
                    s[j] += v[u][j];
                    s2[j] += (double)v[u][j] * v[u][j];
                }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            red[0][r0 * Ctot + c0 + j] = s[j];
            red[1][r0 * Ctot + c0 + j] = s2[j];
        }
    }
    __syncthreads();
    // per group: its channels over the rows, fixed order (GL lanes per group, then a
    // fixed-order combine of the GL)
    constexpr int GL = NT / 32;
    const int grp = threadIdx.x / GL, sub = threadIdx.x % GL;
    double ts = 0, ts2 = 0;
    for (int e = sub; e < rows * cpg; e += GL) {
        const int r = e / cpg, c = grp * cpg + (e - r * cpg);
        ts += red[0][r * Ctot + c];
        ts2 += red[1][r * Ctot + c];
    }
#pragma unroll
    for (int o = 1; o < GL; o <<= 1) {   // xor butterfly: the same sum on all GL lanes
        ts += __shfl_xor(ts, o);
        ts2 += __shfl_xor(ts2, o);
    }
    if (sub == 0) {
        double* dst = a.part + ((b * NC + chunk) * 32 + grp) * 2;
        dst[0] = ts;
        dst[1] = ts2;
    }
}

template <int NT>
__global__ __launch_bounds__(NT) void gn2_apply_kernel(GnArgs a) {
    const int chunk = blockIdx.x;
    const int64_t b = blockIdx.y;
    const int Ctot = a.Ctot, cq = Ctot / 4, cpg = Ctot / 32;
    const int HW = a.HW, NC = gridDim.x;
    __shared__ float ssh[2][1024];
    {   // the sample's statistics from the chunk partials: GL lanes per group, every
        // GL-th chunk in chunk order, then an xor butterfly (the same value on every lane)
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
        const double n = (double)HW * cpg;
        const double mean = S / n;
        const double var = fmax(S2 / n - mean * mean, 0.0);
        const float mf = (float)mean, rf = (float)(1.0 / sqrt(var + (double)a.eps));
        if (sub < cpg) {   // this group's channels (cpg <= 32: GL lanes, a few each)
            for (int cc = sub; cc < cpg; cc += GL) {
                const int c = grp * cpg + cc;
                const float sc = rf * a.gamma[c];
                const float sf = a.beta[c] - mf * sc;
                ssh[0][c] = sc;
                ssh[1][c] = sf;
                if (chunk == 0) {
                    a.ss[(b * Ctot + c) * 2 + 0] = sc;
                    a.ss[(b * Ctot + c) * 2 + 1] = sf;
                }
            }
        }
        if (a.stats && chunk == 0 && sub == 0) {
            a.stats[(b * 32 + grp) * 2 + 0] = mf;
            a.stats[(b * 32 + grp) * 2 + 1] = rf;
        }
    }
    __syncthreads();
    const int p0 = (int)((int64_t)HW * chunk / NC), p1 = (int)((int64_t)HW * (chunk + 1) / NC);
    const int rows = NT / cq;
    const int q = threadIdx.x % cq, r0 = threadIdx.x / cq;
    const int c0 = 4 * q;
    float mx = 0.f;
    if (r0 < rows) {
        f4 sc, sf;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            sc[j] = ssh[0][c0 + j];
            sf[j] = ssh[1][c0 + j];
        }
        // the raw input: a split-K source was reduced into kx by gn2_stats
        const bool kin = a.kpart && c0 < a.C1;
        const float* xs = kin ? a.kx : c0 < a.C1 ? a.src1 : a.src2;
        const int ld = c0 < a.C1 ? a.C1 : a.C2, cx = c0 < a.C1 ? c0 : c0 - a.C1;
        constexpr int U = 4;
        for (int pb = p0 + r0; pb < p1; pb += U * rows) {
            f4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int p = pb + u * rows;
                v[u] = p < p1 ? *(const f4*)(xs + (b * HW + p) * ld + cx) : f4{0.f, 0.f, 0.f, 0.f};
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int p = pb + u * rows;
                if (p >= p1) continue;
                f4 y;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    y[j] = v[u][j] * sc[j] + sf[j];
                    if (a.silu) y[j] = silu_f(y[j]);
                }
                gn_store4(a, (b * HW + p) * Ctot + c0, y);
                mx = fmaxf(mx, amax4(y));
            }
        }
    }
    if (a.amax_out) block_amax_atomic(mx, a.amax_out);
}

// ---------------------------------------------------------------------------
// K1/K2: implicit-GEMM convolution.  GEMM view: M = B*Hout*Wout output pixels,
// N = Cout, K = ks*ks*Ctot ordered (tap, channel).  Workgroup tile BM x BN x 32,
// 4 waves as 2x2, each wave (BM/2)x(BN/2) of 16x16 fp32 MFMA tiles.
// LDS tiles are [row][32 floats] with the 16-byte chunk index XOR-swizzled by
// (row ^ row>>1) & 7: conflict-free for every ds_read_b128 lane group of the
// fragment reads and for the ds_write_b128 staging (found by exhaustive check).
// Lane group g = lane>>4 owns k in [8g, 8g+8) of every 32-deep tile (the same
// permutation for A and B).  The (tap, channel) position advances incrementally
// (no integer division in the K loop).  Register-staged double buffer.
// Optional split-K (gridDim.z > 1): partial sums go to a (split, M, N) slab and
// splitk_reduce applies the epilogue.
// TMODE: transposed addressing for the input-gradient of a stride-s convolution
// (DPS adjoint): output pixel o gathers dY[(o + pad - tap) / s] where divisible,
// with weights packed (Cin_fwd, tap, Cout_fwd).
// ---------------------------------------------------------------------------
__device__ __forceinline__ int lds_swz(int row, int chunk) { return row * 32 + 4 * (chunk ^ ((row ^ (row >> 1)) & 7)); }

// BF (config E): bf16 operands, fp32 accumulate on v_mfma_f32_16x16x32_bf16.  The
// fp32 activations are rounded to bf16 (RNE, v_cvt_pk_bf16_f32) as the A tile is
// staged; weights come pre-rounded (a.wbf).  An LDS row is 32 bf16 = four 16-B
// chunks, chunk c of row r stored in slot (c + 2 * ((r >> 2) & 1)) & 3: one
// ds_read_b128 per lane (k = 8g..8g+7, the MFMA operand layout), conflict-free.
// Chunk slot (chunk + 2 * bit 2 of the row) & 3: each of ds_read_b128's four
// 16-lane groups ({0-3,12-15,20-27}, {4-11,16-19,28-31}, +32; rows li, chunk
// lane/16) then covers all 64 banks once (the earlier (chunk + row/4) & 3 put
// two lanes of every group on one 16-byte slot: 37% extra LDS cycles measured),
// and a ds_write_b64 pair of rows fills 128 contiguous bytes.
__device__ __forceinline__ int lds_swz_bf(int row, int chunk) {
    return row * 64 + ((chunk + 2 * ((row >> 2) & 1)) & 3) * 16;
}

// hi = f16(x) (RNE), lo = f16(x - hi) for 4 values: two packed converts and four
// v_fma_mix (x - hi is exact in fp32, so lo carries one rounding, as before)
__device__ __forceinline__ void split4_mix(const f4& x, uint2& hi, uint2& lo) {
    typedef _Float16 h2_ __attribute__((ext_vector_type(2)));
    typedef float f2_ __attribute__((ext_vector_type(2)));
    hi.x = __builtin_bit_cast(unsigned, __builtin_convertvector((f2_){x[0], x[1]}, h2_));
    hi.y = __builtin_bit_cast(unsigned, __builtin_convertvector((f2_){x[2], x[3]}, h2_));
    asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=&v"(lo.x) : "v"(x[0]), "v"(hi.x));
    asm("v_fma_mixhi_f16 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "+v"(lo.x) : "v"(x[1]), "v"(hi.x));
    asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=&v"(lo.y) : "v"(x[2]), "v"(hi.y));
    asm("v_fma_mixhi_f16 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "+v"(lo.y) : "v"(x[3]), "v"(hi.y));
}


// SPLIT (MODE 2, default fp32 path): fp32-accurate convolution on f16 MFMA.
// Activations are split as staged, x = xh + xl (xh = f16(x), xl = f16(x - xh),
// RNE); weights come pre-split from the host as (s w) = wh + wl with a
// power-of-two s per convolution (a.wbf = wh, a.wlo = wl, a.acc_scale = 1/s).
// Each product runs as wl xh + wh xl + wh xh on v_mfma_f32_16x16x32_f16 (fp32
// accumulate): 22-bit operands, exact products, the fp32 accumulation order of
// the fp32 kernel -- error against fp64 at the fp32 kernel's level
// (tests/test_gpu_unet_split.py).  hi and lo tiles use the bf16 LDS layout.
// NW waves as (NW/2) x 2; 8 waves with BM = 128 halve the weight-tile reads per
// output pixel at the same per-wave tile.
// PF: K tiles in flight through registers (1: the next tile, the double buffer;
// 2-3: a register ring for the short, latency-bound K chains at small batch --
// the same tiles in the same order, so the same sums)
template <int BM, int BN, bool TMODE, int MODE, int NW = 4, bool BUFA = false, int PF = 1>
__global__ __launch_bounds__(64 * NW, NW == 4 ? 2 : 1) void conv_gemm_kernel(ConvArgs a) {
    constexpr bool BF = MODE == 1, SP = MODE == 2;
    constexpr int BK = 32;
    constexpr int WM = BM / (NW / 2), WN = BN / 2;
    constexpr int TM = WM / 16, TN = WN / 16;
    constexpr int RPP = 8 * NW;                  // staged rows per pass (8 threads per 32-deep row)
    constexpr int AIT = BM / RPP, BIT = BN / RPP;  // float4 (bf16: 4 x bf16) per thread per tile
    static_assert(AIT >= 1 && BIT >= 1 && TM >= 1, "tile too small for the wave count");
    // floats per LDS tile: fp32 BM*BK; bf16 half that; split two f16 tiles (hi, lo)
    constexpr int AFL = BF ? BM * BK / 2 : BM * BK, BFL = BF ? BN * BK / 2 : BN * BK;
    // one array: the epilogue (a.ldsepi) reuses all of it as a BM x BN fp32 tile
    __shared__ __attribute__((aligned(16))) float smem_ab[2 * AFL + 2 * BFL];
    float(*const As)[AFL] = (float(*)[AFL])smem_ab;
    float(*const Bs)[BFL] = (float(*)[BFL])(smem_ab + 2 * AFL);
    // the LDS epilogue parks the BM x BN tile in EPI_PASSES row bands (bf16 tiles
    // leave half the fp32 tile's LDS: two bands of whole wave rows)
    constexpr int EPI_FL = 2 * AFL + 2 * BFL;
    constexpr int EPI_PASSES = (BM * BN + EPI_FL - 1) / EPI_FL;
    constexpr bool LDSEPI_FITS = BM % EPI_PASSES == 0 && (BM / EPI_PASSES) % WM == 0 &&
                                 (BM / EPI_PASSES) * BN <= EPI_FL && (BM / EPI_PASSES) * BN / 4 % (64 * NW) == 0;
    // buffer-addressed forward (a.bufaddr): source pixel of every (tap, tile row),
    // -1 for padding, built once per workgroup; the tile loads then cost one table
    // read, one 24-bit multiply-add and a select per row instead of the 64-bit
    // index arithmetic that made the kernel VALU-issue-bound
    __shared__ int pixtab[BUFA ? 9 * BM : 1];

    CFD_STAMP(a.stamps, 1, a.seq, 0);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    // XCD-contiguous tile order (a.xcd): workgroup L runs on XCD L % 8 (round-robin
    // dispatch); hand XCD x the x-th contiguous run of the (m, n, split) tiles,
    // splits fastest, so the workgroups sharing an XCD's L2 share activation rows
    // (the 3x3 halo and every split of one pixel tile) instead of striding the image.
    int bx, by, bz;
    xcd_tile(a.xcd, bx, by, bz);
    const int m0 = bx * BM, n0 = by * BN;
    const int HWo = a.Hout * a.Wout;
    const int kq = tid & 7, rsub = tid >> 3;  // 8 threads per 32-float row

    int a_b[AIT], a_oy[AIT], a_ox[AIT];
    bool a_ok[AIT];
#pragma unroll
    for (int it = 0; it < AIT; ++it) {
        const int m = m0 + rsub + it * RPP;
        a_ok[it] = m < a.M;
        const int mm = a_ok[it] ? m : 0;
        a_b[it] = mm / HWo;
        const int rem = mm - a_b[it] * HWo;
        a_oy[it] = rem / a.Wout;
        a_ox[it] = rem - a_oy[it] * a.Wout;
        if (TMODE) {
            a_oy[it] += a.pad;
            a_ox[it] += a.pad;
        } else if (!a.up) {
            a_oy[it] = a_oy[it] * a.stride - a.pad;
            a_ox[it] = a_ox[it] * a.stride - a.pad;
        } else {
            a_oy[it] -= a.pad;
            a_ox[it] -= a.pad;
        }
    }
    const float* wrow[BIT];
    const unsigned short* wrow_bf[BIT];
    const unsigned short* wrow_lo[BIT];
    bool b_ok[BIT];
#pragma unroll
    for (int it = 0; it < BIT; ++it) {
        const int n = n0 + rsub + it * RPP;
        b_ok[it] = n < a.Cout;
        if constexpr (BF || SP)
            wrow_bf[it] = (const unsigned short*)a.wbf + (int64_t)(b_ok[it] ? n : 0) * a.K + 4 * kq;
        else
            wrow[it] = a.w + (int64_t)(b_ok[it] ? n : 0) * a.K + 4 * kq;
        if constexpr (SP) wrow_lo[it] = (const unsigned short*)a.wlo + (int64_t)(b_ok[it] ? n : 0) * a.K + 4 * kq;
    }
    const int nkt = a.K / BK;
    const int per = (nkt + gridDim.z - 1) / gridDim.z;
    const int kt0 = bz * per;
    const int kt1 = min(nkt, kt0 + per);
    // wave-uniform K position of tile kt: (dy, dx) tap and channel base, in
    // (tap, chunk) order.  Derived from kt per tile and pinned to SGPRs: a position
    // carried across tiles ended up in scratch and VGPRs, and a VGPR-selected
    // buffer descriptor costs a readfirstlane loop around every load.
    auto kpos_of = [&](int kt, int& cb, int& dy, int& dx) {
        const int kb = kt * BK;
        const int tap = kb / a.Ctot;
        cb = kb - tap * a.Ctot;
        dy = tap / a.ks;
        dx = tap - dy * a.ks;
        cb = __builtin_amdgcn_readfirstlane(cb);
        dy = __builtin_amdgcn_readfirstlane(dy);
        dx = __builtin_amdgcn_readfirstlane(dx);
    };

    const int smask = a.stride - 1, sshift = a.stride >> 1;
    f4 ra[PF][AIT], rb[PF][BIT];
    uint2 rbh[PF][BIT], rbl[PF][BIT];
    // buffer-addressed path: resources, per-row weight offsets, the pixel table
    constexpr int WES = (BF || SP) ? 2 : 4;   // weight element bytes
    const int srows = __builtin_amdgcn_readfirstlane(a.Hin * a.Win * (a.M / HWo));   // SGPR descriptor fields
    const __amdgpu_buffer_rsrc_t rs1 = __builtin_amdgcn_make_buffer_rsrc((void*)a.src1, 0, srows * a.C1 * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t rs2 = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(a.src2 ? a.src2 : a.src1), 0, a.src2 ? srows * a.C2 * 4 : 0, 0x00020000);
    const __amdgpu_buffer_rsrc_t rwh = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((BF || SP) ? (const void*)a.wbf : (const void*)a.w), 0, a.Cout * a.K * WES, 0x00020000);
    const __amdgpu_buffer_rsrc_t rwl = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(SP ? (const void*)a.wlo : (const void*)a.w), 0, a.Cout * a.K * WES, 0x00020000);
    unsigned b_voff[BIT];
    if constexpr (BUFA) {
#pragma unroll
        for (int it = 0; it < BIT; ++it) {
            const int n = n0 + rsub + it * RPP;
            b_voff[it] = n < a.Cout ? (unsigned)((n * a.K + 4 * kq) * WES) : 0x80000000u;
        }
        const int ntap = a.ks * a.ks;
        const float rhw = 1.0f / (float)HWo, rw = 1.0f / (float)a.Wout;   // fdiv24 (M < 2^24: launch_conv)
        for (int e = tid; e < ntap * BM; e += 64 * NW) {
            const int tap = e / BM, r = e - tap * BM;
            const int ty = tap_row(tap, a.ks), tx = tap - ty * a.ks;
            const int m = m0 + r;
            int pix = -1;
            if (m < a.M) {
                const int b = fdiv24(m, HWo, rhw), rem = m - b * HWo;
                const int oy = fdiv24(rem, a.Wout, rw), ox = rem - oy * a.Wout;
                int iy, ix;
                bool ok;
                if (TMODE) {   // transposed addressing: dY[(o + pad - tap) / s] where divisible
                    iy = oy + a.pad - ty;
                    ix = ox + a.pad - tx;
                    ok = iy >= 0 && ix >= 0 && ((iy | ix) & smask) == 0;
                    iy >>= sshift;
                    ix >>= sshift;
                    ok = ok && iy < a.Hin && ix < a.Win;
                } else if (a.up) {
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
                if (ok) pix = (b * a.Hin + iy) * a.Win + ix;
            }
            CFD_DASSERT(pix < srows);
            pixtab[e] = pix;
        }
        __syncthreads();
        CFD_STAMP(a.stamps, 1, a.seq, 1);
    }
    auto load_tile = [&](int kt, int sl) {
        int cb, dy, dx;
        kpos_of(kt, cb, dy, dx);
        const int c0 = cb + 4 * kq;
        const int kpos = (dy * a.ks + dx) * a.Ctot + cb;   // this tile's offset in a (tap, channel) weight row
        if constexpr (BUFA) {
            const int tap = dy * a.ks + dx;
            const bool second = cb >= a.C1;
            const unsigned csrc4 = 4u * (second ? a.C2 : a.C1);
            const unsigned cofs4 = 4u * (second ? c0 - a.C1 : c0);
            const __amdgpu_buffer_rsrc_t rsa = second ? rs2 : rs1;
#pragma unroll
            for (int it = 0; it < AIT; ++it) {
                const int pix = pixtab[tap * BM + rsub + it * RPP];
                const unsigned off = pix >= 0 ? __umul24((unsigned)pix, csrc4) + cofs4 : 0x80000000u;
                ra[sl][it] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rsa, off, 0, 0));
            }
            const int soff = kpos * WES;
#pragma unroll
            for (int it = 0; it < BIT; ++it) {
                if constexpr (BF || SP)
                    rbh[sl][it] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rwh, b_voff[it], soff, 0));
                if constexpr (SP)
                    rbl[sl][it] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rwl, b_voff[it], soff, 0));
                if constexpr (!BF && !SP)
                    rb[sl][it] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rwh, b_voff[it], soff, 0));
            }
        } else {
#pragma unroll
        for (int it = 0; it < AIT; ++it) {
            f4 v = {0.f, 0.f, 0.f, 0.f};
            int iy, ix;
            bool ok = a_ok[it];
            if (TMODE) {
                iy = a_oy[it] - dy;
                ix = a_ox[it] - dx;
                ok = ok && iy >= 0 && ix >= 0 && ((iy | ix) & smask) == 0;
                iy >>= sshift;
                ix >>= sshift;
                ok = ok && iy < a.Hin && ix < a.Win;
            } else if (a.up) {
                iy = a_oy[it] + dy;
                ix = a_ox[it] + dx;
                ok = ok && iy >= 0 && iy < 2 * a.Hin && ix >= 0 && ix < 2 * a.Win;
                iy >>= 1;
                ix >>= 1;
            } else {
                iy = a_oy[it] + dy;
                ix = a_ox[it] + dx;
                ok = ok && iy >= 0 && iy < a.Hin && ix >= 0 && ix < a.Win;
            }
            if (ok) {
                const int64_t pix = ((int64_t)a_b[it] * a.Hin + iy) * a.Win + ix;
                v = c0 < a.C1 ? *(const f4*)(a.src1 + pix * a.C1 + c0)
                              : *(const f4*)(a.src2 + pix * a.C2 + (c0 - a.C1));
            }
            ra[sl][it] = v;
        }
#pragma unroll
        for (int it = 0; it < BIT; ++it) {
            if constexpr (BF || SP)
                rbh[sl][it] = b_ok[it] ? *(const uint2*)(wrow_bf[it] + kpos) : uint2{0u, 0u};
            if constexpr (SP)
                rbl[sl][it] = b_ok[it] ? *(const uint2*)(wrow_lo[it] + kpos) : uint2{0u, 0u};
            if constexpr (!BF && !SP)
                rb[sl][it] = b_ok[it] ? *(const f4*)(wrow[it] + kpos) : f4{0.f, 0.f, 0.f, 0.f};
        }
        }
    };
    auto store_tile = [&](int buf, int sl) {
        if constexpr (SP) {
            // hi tile at [0, BM*BK/2) floats, lo tile after it (same bf16 layout)
#pragma unroll
            for (int it = 0; it < AIT; ++it) {
                // hi = f16(x) (RNE, packed convert), lo = f16(x - hi) in one v_fma_mix per value
                uint2 hv, lv;
                split4_mix(ra[sl][it], hv, lv);
                const int off = lds_swz_bf(rsub + it * RPP, kq >> 1) + (kq & 1) * 8;
                *(uint2*)((char*)As[buf] + off) = hv;
                *(uint2*)((char*)As[buf] + BM * BK * 2 + off) = lv;
            }
#pragma unroll
            for (int it = 0; it < BIT; ++it) {
                const int off = lds_swz_bf(rsub + it * RPP, kq >> 1) + (kq & 1) * 8;
                *(uint2*)((char*)Bs[buf] + off) = rbh[sl][it];
                *(uint2*)((char*)Bs[buf] + BN * BK * 2 + off) = rbl[sl][it];
            }
        } else if constexpr (BF) {
            // thread kq holds k = 4kq..4kq+3: chunk kq/2, half kq%2
#pragma unroll
            for (int it = 0; it < AIT; ++it) {
                const bf16x4 v = __builtin_convertvector(ra[sl][it], bf16x4);
                *(bf16x4*)((char*)As[buf] + lds_swz_bf(rsub + it * RPP, kq >> 1) + (kq & 1) * 8) = v;
            }
#pragma unroll
            for (int it = 0; it < BIT; ++it)
                *(uint2*)((char*)Bs[buf] + lds_swz_bf(rsub + it * RPP, kq >> 1) + (kq & 1) * 8) = rbh[sl][it];
        } else {
#pragma unroll
            for (int it = 0; it < AIT; ++it) *(f4*)(&As[buf][lds_swz(rsub + it * RPP, kq)]) = ra[sl][it];
#pragma unroll
            for (int it = 0; it < BIT; ++it) *(f4*)(&Bs[buf][lds_swz(rsub + it * RPP, kq)]) = rb[sl][it];
        }
    };

    f4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

    const int g2 = 2 * (lane >> 4), li = lane & 15;
    auto compute = [&](int cur) {
            if constexpr (SP) {
                const int g = lane >> 4;
                h8v fah[TM], fal[TM], fbh[TN], fbl[TN];
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    const int off = lds_swz_bf(wm * WM + 16 * i + li, g);
                    fah[i] = *(const h8v*)((const char*)As[cur] + off);
                    fal[i] = *(const h8v*)((const char*)As[cur] + BM * BK * 2 + off);
                }
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int off = lds_swz_bf(wn * WN + 16 * j + li, g);
                    fbh[j] = *(const h8v*)((const char*)Bs[cur] + off);
                    fbl[j] = *(const h8v*)((const char*)Bs[cur] + BN * BK * 2 + off);
                }
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j) {
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fal[i], fbh[j], acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fah[i], fbl[j], acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fah[i], fbh[j], acc[i][j], 0, 0, 0);
                    }
            } else if constexpr (BF) {
                const int g = lane >> 4;
                bf16x8 fa[TM], fb[TN];
#pragma unroll
                for (int i = 0; i < TM; ++i)
                    fa[i] = *(const bf16x8*)((const char*)As[cur] + lds_swz_bf(wm * WM + 16 * i + li, g));
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    fb[j] = *(const bf16x8*)((const char*)Bs[cur] + lds_swz_bf(wn * WN + 16 * j + li, g));
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
            } else
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                f4 fa[TM], fb[TN];
#pragma unroll
                for (int i = 0; i < TM; ++i) fa[i] = *(const f4*)(&As[cur][lds_swz(wm * WM + 16 * i + li, g2 + h)]);
#pragma unroll
                for (int j = 0; j < TN; ++j) fb[j] = *(const f4*)(&Bs[cur][lds_swz(wn * WN + 16 * j + li, g2 + h)]);
#pragma unroll
                for (int s = 0; s < 4; ++s)
#pragma unroll
                    for (int i = 0; i < TM; ++i)
#pragma unroll
                        for (int j = 0; j < TN; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i][s], fb[j][s], acc[i][j], 0, 0, 0);
            }
    };
    if (kt0 < kt1) {
        load_tile(kt0, 0);
#pragma unroll
        for (int p = 1; p < PF; ++p) load_tile(min(kt0 + p, kt1 - 1), p);
        store_tile(0, 0);
        __syncthreads();
        CFD_STAMP(a.stamps, 1, a.seq, 2);
        // step kt: tile kt + PF into the register slot tile kt left (clamped: a
        // repeated last tile keeps every load unconditional, so the wait before a
        // store is a counted vmcnt), MFMAs on LDS stage cur, then tile kt + 1 from
        // its slot into the other stage
        auto step = [&](int kt, int j) {
            const int cur = (kt - kt0) & 1;
            if constexpr (PF == 1) {
                if (kt + 1 < kt1) load_tile(kt + 1, 0);
            } else {
                load_tile(min(kt + PF, kt1 - 1), j);
            }
            compute(cur);
            if (kt + 1 < kt1) store_tile(cur ^ 1, (j + 1) % PF);
            __syncthreads();
        };
        for (int kt = kt0; kt < kt1; kt += PF) {
            step(kt, 0);
            if constexpr (PF > 1)
                if (kt + 1 < kt1) step(kt + 1, 1);
            if constexpr (PF > 2)
                if (kt + 2 < kt1) step(kt + 2, 2);
        }
    }
    CFD_STAMP(a.stamps, 1, a.seq, 3);

    const int g4 = 4 * (lane >> 4);
    if constexpr (SP) {  // undo the power-of-two weight scale (exact)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[i][j] *= a.acc_scale;
    }
    // LDS epilogue (a.ldsepi, Cout % 4 == 0): the accumulators go through LDS
    // (every wave is past its last fragment read: the K loop ends on a barrier)
    // so the stores -- and the residual / bias loads -- are float4 rows of BN
    // channels instead of the 16x16 accumulator layout's 64-B column pieces.
    // Columns XOR-swizzled by 16 ((row >> 2) & 3) so the four row groups of a
    // write land in different banks.  Same values, same rounding.
    if constexpr (LDSEPI_FITS) {
        if (a.ldsepi) {
          constexpr int RB = BM / EPI_PASSES;   // tile rows per band
          for (int band = 0; band < EPI_PASSES; ++band) {
            __syncthreads();
            float* tile = smem_ab;
            auto sw = [](int row, int col) { return row * BN + (col ^ (((row >> 2) & 3) << 4)); };
            if (wm * WM / RB == band) {
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            tile[sw(wm * WM - band * RB + 16 * i + g4 + r, wn * WN + 16 * j + li)] = acc[i][j][r];
            }
            __syncthreads();
            constexpr int NV = RB * BN / 4 / (64 * NW);
            float* part = gridDim.z > 1 ? a.part + (int64_t)bz * a.M * a.Cout : nullptr;
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                const int idx = tid + v * 64 * NW;
                const int row = idx / (BN / 4), c4 = (idx - row * (BN / 4)) * 4;
                const int m = m0 + band * RB + row, n = n0 + c4;
                if (m >= a.M || n >= a.Cout) continue;
                f4 val = *(const f4*)&tile[sw(row, c4)];
                const int64_t o = (int64_t)m * a.Cout + n;
                if (part) {
                    *(f4*)(part + o) = val;
                    continue;
                }
                if (a.bias) val = val + *(const f4*)(a.bias + n);
                if (a.emb) val = val + *(const f4*)(a.emb + (int64_t)(m / HWo) * a.emb_stride + n);
                if (a.res) val = *(const f4*)(a.res + o) + val;
                *(f4*)(a.out + o) = val;
            }
            // qkv convolution: the split attention's K / V fragments from this band of
            // the staged tile, attn_kv_split_kernel's layout and arithmetic -- K =
            // (acc + bias) * scale log2 e, V = acc + bias, each split into f16 hi / lo
            // -- so the same bits, without its launch and its re-read of qkv.
            // T % 32 == 0 (conv_kv_pack_ok) and bands of whole 32-row blocks: a
            // 32-key block never straddles two samples or bands, and T32 = T.
            if constexpr ((SP || BF) && RB % 32 == 0) {
              if (a.kvf && !part) {
                const int CH = a.kv_ch, C3 = 3 * CH, T = a.kv_T, nj = CH >> 5, nd = CH >> 4;
                const float ks = kln2(a.kv_scale);
                // head and sample of a (row, column): fdiv24 (exact below 2^24 pixels,
                // launch_conv's bufaddr bound) instead of two integer divisions per
                // item, which were most of this epilogue's VALU
                const float rc3 = 1.0f / (float)C3, rT = 1.0f / (float)T;
                const bool small = a.M < (1 << 24);
                h8v* kf = (h8v*)a.kvf;
                h8v* vf = kf + a.kv_voff;
                const int mband = m0 + band * RB;
                // K: (key row, 8 channels) -> one lane of fragment (key / 16, j)
                for (int it = tid; it < RB * (BN / 8); it += 64 * NW) {
                    const int row = it / (BN / 8), c8 = (it - row * (BN / 8)) * 8;
                    const int m = mband + row, n = n0 + c8;
                    if (m >= a.M || n >= a.Cout) continue;
                    const int hh = small ? fdiv24(n, C3, rc3) : n / C3, o = n - hh * C3;
                    if (o < CH || o >= 2 * CH) continue;
                    const int b = small ? fdiv24(m, T, rT) : m / T;
                    const int kc = o - CH, key = m - b * T;
                    f4 v0 = *(const f4*)&tile[sw(row, c8)], v1 = *(const f4*)&tile[sw(row, c8 + 4)];
                    v0 = v0 + *(const f4*)(a.bias + n);
                    v1 = v1 + *(const f4*)(a.bias + n + 4);
                    float v[8];
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        v[t] = v0[t] * ks;
                        v[t + 4] = v1[t] * ks;
                    }
                    h8v hi, lo;
                    split8_f16(v, hi, lo);
                    const int64_t bh = (int64_t)b * a.kv_heads + hh;
                    h8v* dst = kf + ((bh * (T >> 4) + (key >> 4)) * nj + (kc >> 5)) * 128 + ((kc & 31) >> 3) * 16 + (key & 15);
                    dst[0] = hi;
                    dst[64] = lo;
                }
                // V: (32-key block, lane group g, channel) -> one lane of fragment (block, channel / 16)
                for (int it = tid; it < (RB / 32) * 4 * BN; it += 64 * NW) {
                    const int col = it % BN, r2 = it / BN, g = r2 & 3, blk = r2 >> 2;
                    const int n = n0 + col, mb = mband + 32 * blk;
                    if (n >= a.Cout || mb >= a.M) continue;
                    const int hh = small ? fdiv24(n, C3, rc3) : n / C3, o = n - hh * C3;
                    if (o < 2 * CH) continue;
                    const int b = small ? fdiv24(mb, T, rT) : mb / T;
                    const int vc = o - 2 * CH, kb = (mb - b * T) >> 5;
                    const float bn = a.bias[n];
                    float v[8];
#pragma unroll
                    for (int t = 0; t < 8; ++t) v[t] = tile[sw(32 * blk + (t < 4 ? 4 * g + t : 12 + 4 * g + t), col)] + bn;
                    h8v hi, lo;
                    split8_f16(v, hi, lo);
                    const int64_t bh = (int64_t)b * a.kv_heads + hh;
                    h8v* dst = vf + ((bh * (T >> 5) + kb) * nd + (vc >> 4)) * 128 + g * 16 + (vc & 15);
                    dst[0] = hi;
                    dst[64] = lo;
                }
              }
            }
          }
#ifdef CFD_STAMPS
            __builtin_amdgcn_s_waitcnt(0);
#endif
            CFD_STAMP(a.stamps, 1, a.seq, 4);
            return;
        }
    }
    if (gridDim.z > 1) {
        float* part = a.part + (int64_t)bz * a.M * a.Cout;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + wm * WM + 16 * i + g4 + r;
                if (m >= a.M) continue;
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int n = n0 + wn * WN + 16 * j + li;
                    if (n < a.Cout) part[(int64_t)m * a.Cout + n] = acc[i][j][r];
                }
            }
        CFD_STAMP(a.stamps, 1, a.seq, 4);
        return;
    }
    // epilogue: (acc + bias) (+ emb[b, n]); residual + h
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = m0 + wm * WM + 16 * i + g4 + r;
            if (m >= a.M) continue;
            const int bb = m / HWo;
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int n = n0 + wn * WN + 16 * j + li;
                if (n >= a.Cout) continue;
                float v = a.bias ? acc[i][j][r] + a.bias[n] : acc[i][j][r];
                if (a.emb) v = v + a.emb[(int64_t)bb * a.emb_stride + n];
                if (a.res) v = a.res[(int64_t)m * a.Cout + n] + v;
                a.out[(int64_t)m * a.Cout + n] = v;
            }
        }
    }
    CFD_STAMP(a.stamps, 1, a.seq, 4);
}

// sum of split-K partials in split order + the conv epilogue
__global__ void splitk_reduce_kernel(ConvArgs a, int splits) {
    const int64_t i4 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total4 = (int64_t)a.M * a.Cout / 4;
    if (i4 >= total4) return;
    const int64_t i = i4 * 4;
    const int64_t slab = (int64_t)a.M * a.Cout;
    // the residual, slab 0 and up to 15 more slabs in one round of loads (each
    // dependent round is a memory latency), added in split order
    const f4 rv = a.res ? *(const f4*)(a.res + i) : f4{0.f, 0.f, 0.f, 0.f};
    f4 s = *(const f4*)(a.part + i);
    constexpr int UN = 15;
    for (int k = 1; k < splits; k += UN) {
        f4 u[UN];
#pragma unroll
        for (int q = 0; q < UN; ++q)
            u[q] = k + q < splits ? *(const f4*)(a.part + (k + q) * slab + i) : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < UN; ++q)
            if (k + q < splits) s += u[q];
    }
    const int64_t m = i / a.Cout;
    const int n = (int)(i - m * a.Cout);
    const int bb = (int)(m / (a.Hout * a.Wout));
    f4 v;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        float y = a.bias ? s[j] + a.bias[n + j] : s[j];
        if (a.emb) y = y + a.emb[(int64_t)bb * a.emb_stride + n + j];
        if (a.res) y = rv[j] + y;
        v[j] = y;
    }
    *(f4*)(a.out + i) = v;
}

// First convolution, in_channels (<= 4) -> Cout, 3x3 pad 1: VALU, one output per thread.
// tmode: the same gather with the taps mirrored (input-gradient of the last
// convolution, weights packed (Cin_fwd, tap, Cout_fwd)); bias may be null.
__global__ void conv_in_kernel(ConvArgs a) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (int64_t)a.M * a.Cout) return;
    const int n = (int)(idx % a.Cout);
    const int m = (int)(idx / a.Cout);
    const int HW = a.Hout * a.Wout;
    const int b = m / HW, rem = m - b * HW, oy = rem / a.Wout, ox = rem - oy * a.Wout;
    float s = 0.f;
    for (int tap = 0; tap < 9; ++tap) {
        const int ty = a.tmode ? 1 - tap / 3 : tap / 3 - 1, tx = a.tmode ? 1 - tap % 3 : tap % 3 - 1;
        const int iy = oy + ty, ix = ox + tx;
        if (iy < 0 || iy >= a.Hin || ix < 0 || ix >= a.Win) continue;
        const float* px = a.src1 + (((int64_t)b * a.Hin + iy) * a.Win + ix) * a.C1;
        for (int c = 0; c < a.C1; ++c) s = fmaf(a.w[((int64_t)n * 9 + tap) * a.C1 + c], px[c], s);
    }
    a.out[idx] = a.bias ? s + a.bias[n] : s;
}

// Last convolution (input already GroupNorm+SiLU'd), Ctot -> Cout (<= 4), 3x3 pad 1.  One wave
// per output pixel; lanes split K = 9*Ctot, wave-reduced.
__global__ void conv_out_kernel(ConvArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t m = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (m >= a.M) return;
    const int HW = a.Hout * a.Wout;
    const int b = (int)(m / HW), rem = (int)(m - (int64_t)b * HW), oy = rem / a.Wout, ox = rem - oy * a.Wout;
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    for (int k = lane; k < a.K; k += 64) {
        const int tap = k / a.Ctot, c = k - tap * a.Ctot;
        const int ty = a.tmode ? 1 - tap / 3 : tap / 3 - 1, tx = a.tmode ? 1 - tap % 3 : tap % 3 - 1;
        const int iy = oy + ty, ix = ox + tx;
        if (iy < 0 || iy >= a.Hin || ix < 0 || ix >= a.Win) continue;
        const float v = a.src1[(((int64_t)b * a.Hin + iy) * a.Win + ix) * a.C1 + c];
        for (int n = 0; n < a.Cout; ++n) s[n] = fmaf(a.w[(int64_t)n * a.K + k], v, s[n]);
    }
    for (int n = 0; n < a.Cout; ++n) {
        float v = s[n];
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        if (lane == 0) {
            const float y = a.bias ? v + a.bias[n] : v;
            a.out[m * a.Cout + n] = y;
            if (a.nonfinite && !isfinite(y)) *a.nonfinite = 1;
        }
    }
}

// Forward last convolution, vectorised: LP = Ctot/4 lanes per output pixel
// (64/LP pixels per wave), each lane a float4 of channels per tap; per-tap
// bounds, no division in the loop; weights (Cout, 9, Ctot) staged in LDS.
// Fixed summation order (lane partial over taps, then a butterfly), so every
// sample's output is independent of the batch.
__global__ __launch_bounds__(256) void conv_out_vec_kernel(ConvArgs a, int LP) {
    extern __shared__ __attribute__((aligned(16))) float wsm[];
    for (int i = threadIdx.x; i < a.Cout * a.K; i += blockDim.x) wsm[i] = a.w[i];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int ppw = 64 / LP;
    const int c = 4 * (lane % LP);
    const int HW = a.Hout * a.Wout;
    // grid-stride over pixel groups (launch_conv_out bounds the grid): the weight
    // table each workgroup stages in LDS serves many pixels, not one wave's ppw
    for (int64_t m0 = ((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * ppw; m0 < a.M;
         m0 += (int64_t)gridDim.x * (blockDim.x >> 6) * ppw) {
    const int64_t m = m0 + lane / LP;
    const int64_t mm = m < a.M ? m : a.M - 1;
    const int b = (int)(mm / HW), rem = (int)(mm - (int64_t)b * HW), oy = rem / a.Wout, ox = rem - oy * a.Wout;
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    for (int tap = 0; tap < 9; ++tap) {
        // tmode: taps mirrored (the input-gradient of the first convolution)
        const int iy = a.tmode ? oy + 1 - tap / 3 : oy + tap / 3 - 1, ix = a.tmode ? ox + 1 - tap % 3 : ox + tap % 3 - 1;
        if (iy < 0 || iy >= a.Hin || ix < 0 || ix >= a.Win) continue;
        const f4 v = *(const f4*)(a.src1 + (((int64_t)b * a.Hin + iy) * a.Win + ix) * a.C1 + c);
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            if (n < a.Cout) {
                const f4 w = *(const f4*)(wsm + (n * 9 + tap) * a.Ctot + c);
                s[n] = fmaf(w[0], v[0], fmaf(w[1], v[1], fmaf(w[2], v[2], fmaf(w[3], v[3], s[n]))));
            }
        }
    }
#pragma unroll
    for (int n = 0; n < 4; ++n) {
        if (n >= a.Cout) break;
        float v = s[n];
        for (int o = LP >> 1; o > 0; o >>= 1) v += __shfl_xor(v, o);
        if (lane % LP == 0 && m < a.M) {
            const float y = a.bias ? v + a.bias[n] : v;
            a.out[m * a.Cout + n] = y;
            // range guard: an activation beyond the f16 range makes a split-f16 hi
            // part infinite, and every such value reaches eps as inf / NaN
            if (a.nonfinite && !isfinite(y)) *a.nonfinite = 1;
        }
    }
    }
}

// Forward first convolution, C1 <= 4 -> Cout: one thread per (pixel, 4 output
// channels), weights staged in LDS as (tap, c, Cout) so a thread reads a float4.
__global__ __launch_bounds__(256) void conv_in_vec_kernel(ConvArgs a) {
    extern __shared__ __attribute__((aligned(16))) float wsm[];  // (9, C1, Cout)
    const int C1 = a.C1, Cout = a.Cout;
    for (int i = threadIdx.x; i < 9 * C1 * Cout; i += blockDim.x) {
        const int n = i % Cout, tc = i / Cout, tap = tc / C1, cc = tc % C1;
        wsm[i] = a.w[((int64_t)n * 9 + tap) * C1 + cc];
    }
    __syncthreads();
    const int nq = Cout / 4;
    // grid-stride (launch_conv_in bounds the grid): the staged weight table serves
    // many pixels per workgroup instead of 256 / nq
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < (int64_t)a.M * nq;
         idx += (int64_t)gridDim.x * blockDim.x) {
    const int n0 = 4 * (int)(idx % nq);
    const int64_t m = idx / nq;
    const int HW = a.Hout * a.Wout;
    const int b = (int)(m / HW), rem = (int)(m - (int64_t)b * HW), oy = rem / a.Wout, ox = rem - oy * a.Wout;
    f4 s = {0.f, 0.f, 0.f, 0.f};
    for (int tap = 0; tap < 9; ++tap) {
        // tmode: taps mirrored (the input-gradient of the last convolution)
        const int iy = a.tmode ? oy + 1 - tap / 3 : oy + tap / 3 - 1, ix = a.tmode ? ox + 1 - tap % 3 : ox + tap % 3 - 1;
        if (iy < 0 || iy >= a.Hin || ix < 0 || ix >= a.Win) continue;
        const float* px = a.src1 + (((int64_t)b * a.Hin + iy) * a.Win + ix) * C1;
        for (int cc = 0; cc < C1; ++cc) {
            const float v = px[cc];
            const f4 w = *(const f4*)(wsm + (tap * C1 + cc) * Cout + n0);
#pragma unroll
            for (int j = 0; j < 4; ++j) s[j] = fmaf(w[j], v, s[j]);
        }
    }
    if (a.bias) {
#pragma unroll
        for (int j = 0; j < 4; ++j) s[j] += a.bias[n0 + j];
    }
    *(f4*)(a.out + m * Cout + n0) = s;
    }
}

// ---------------------------------------------------------------------------
// K4: QKVAttentionLegacy.  qkv (B, T, 3C) with head h's q/k/v at channels
// h*3*CH + {0, CH, 2CH} + i (the legacy "split heads before qkv" order,
// unet.py:337-354).  Each wave owns 16 queries; S^T = K Q^T and O^T = V^T P^T on
// fp32 MFMA 16x16x4 so P stays in registers; online softmax over 16-key blocks.
// ---------------------------------------------------------------------------
template <int CH>
__global__ __launch_bounds__(256) void attention_kernel(AttnArgs a) {
    constexpr int KQ = CH / 4;    // MFMA k-steps over the head dimension
    constexpr int ND = CH / 16;   // 16-wide output blocks
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane >> 4, li = lane & 15;
    const int h = blockIdx.y;
    const int64_t b = blockIdx.z;
    const int T = a.T;
    const int q0 = blockIdx.x * 64 + wave * 16;
    if (q0 >= T) return;  // wave-uniform
    const int C3 = 3 * a.C;
    const float* base = a.qkv + b * (int64_t)T * C3 + (int64_t)h * 3 * CH;
    const float scale = a.scale;

    float qf[KQ];
    {
        const int tq = min(q0 + li, T - 1);
        const float* qp = base + (int64_t)tq * C3 + KQ * g;
#pragma unroll
        for (int s = 0; s < KQ; s += 4) {
            const f4 v = *(const f4*)(qp + s);
            qf[s + 0] = v[0] * scale;
            qf[s + 1] = v[1] * scale;
            qf[s + 2] = v[2] * scale;
            qf[s + 3] = v[3] * scale;
        }
    }
    f4 O[ND];
#pragma unroll
    for (int d = 0; d < ND; ++d) O[d] = f4{0.f, 0.f, 0.f, 0.f};
    float mrun = -INFINITY, lrun = 0.f;

    for (int kb = 0; kb < T; kb += 16) {
        // S^T[key][query]
        f4 st = {0.f, 0.f, 0.f, 0.f};
        {
            const int tk = min(kb + li, T - 1);
            const float* kp = base + (int64_t)tk * C3 + CH + KQ * g;
#pragma unroll
            for (int s = 0; s < KQ; s += 4) {
                const f4 kv = *(const f4*)(kp + s);
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    st = __builtin_amdgcn_mfma_f32_16x16x4f32(kv[u] * scale, qf[s + u], st, 0, 0, 0);
            }
        }
        // lane (g, li) holds S[query li][key kb + 4g + r]
        float mx = -INFINITY;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            if (kb + 4 * g + r >= T) st[r] = -INFINITY;
            mx = fmaxf(mx, st[r]);
        }
        mx = fmaxf(mx, __shfl_xor(mx, 16));
        mx = fmaxf(mx, __shfl_xor(mx, 32));
        const float mnew = fmaxf(mrun, mx);
        const float alpha = expf(mrun - mnew);
        float p[4], ps = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            p[r] = expf(st[r] - mnew);
            ps += p[r];
        }
        ps += __shfl_xor(ps, 16);
        ps += __shfl_xor(ps, 32);
        lrun = lrun * alpha + ps;
        mrun = mnew;
#pragma unroll
        for (int d = 0; d < ND; ++d) O[d] = O[d] * alpha;
        // O^T[d][query] += V^T[d][key] P^T[key][query]
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int tk = min(kb + 4 * g + r, T - 1);
            const float* vp = base + (int64_t)tk * C3 + 2 * CH + li;
#pragma unroll
            for (int d = 0; d < ND; ++d)
                O[d] = __builtin_amdgcn_mfma_f32_16x16x4f32(vp[16 * d], p[r], O[d], 0, 0, 0);
        }
    }
    // lane (g, li) holds O[query li][16 d + 4 g + r]
    const int tq = q0 + li;
    if (a.lse && g == 0 && tq < T) a.lse[((int64_t)b * gridDim.y + h) * T + tq] = mrun + logf(lrun);
    if (tq < T) {
        float* op = a.out + (b * (int64_t)T + tq) * a.C + (int64_t)h * CH;
        const float inv = 1.0f / lrun;
#pragma unroll
        for (int d = 0; d < ND; ++d) {
            f4 v = O[d] * inv;
            *(f4*)(op + 16 * d + 4 * g) = v;
        }
    }
}

// ---------------------------------------------------------------------------
// K4s: the same attention at fp32 accuracy on f16 MFMA (split compute).
// attn_kv_split packs K (times the q/k scale) and V once per call as hi/lo f16
// MFMA fragments (x = hi + lo, 22 significant bits), keys padded to a multiple
// of 32 with zeros:
//   Kf[b][h][kt][j][hl][lane][8]: key 16 kt + lane%16, channel 32 j + 8(lane/16) + t
//   Vf[b][h][kb][dd][hl][lane][8]: channel 16 dd + lane%16, key 32 kb + kmap(lane/16, t)
// with kmap(g, t) = 4g + t (t < 4), 16 + 4g + t - 4 (t >= 4): the keys a lane holds
// of two 16-key S^T tiles, so P^T feeds the P.V MFMA straight from the softmax
// registers.  attention_dma_kernel (K4d) then runs S^T = K Q^T and O^T = V^T P^T as
// three v_mfma_f32_16x16x32_f16 each (lo*hi + hi*lo + hi*hi, fp32 accumulate) over
// 32-key blocks with the fp32 kernel's online softmax.  K carries the q/k scale
// times log2(e) (kln2 below), so S is in base-2 units: every exponential is one
// v_exp_f32 (ocml's expf is ~11 instructions: the softmax was ~1/3 of the loop's
// issue) and the saved log-sum-exp is converted back to natural units.
// ---------------------------------------------------------------------------

__global__ __launch_bounds__(256) void attn_kv_split_kernel(AttnArgs a, int CH, int heads, int B, h8v* kf,
                                                            h8v* vf) {
    const int T = a.T, T32 = (T + 31) / 32 * 32;
    const int nj = CH / 32, nd = CH / 16;
    // slots: K (T32/16 * nj * 64) then V (T32/32 * nd * 64) per (b, h)
    const int64_t kslots = (int64_t)(T32 / 16) * nj * 64, vslots = (int64_t)(T32 / 32) * nd * 64;
    const int64_t per = kslots + vslots;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= per * heads * B) return;
    const int64_t bh = i / per;
    int64_t r = i - bh * per;
    const int64_t b = bh / heads;
    const int h = (int)(bh - b * heads);
    const int C3 = 3 * a.C;
    const float* base = a.qkv + b * (int64_t)T * C3 + (int64_t)h * 3 * CH;
    const int lane = (int)(r & 63), g = lane >> 4, li = lane & 15;
    float v[8];
    h8v* dst;
    int64_t stride;
    if (r < kslots) {
        const int64_t f = r >> 6;  // fragment (kt, j)
        const int kt = (int)(f / nj), j = (int)(f - (int64_t)kt * nj);
        const int key = 16 * kt + li;
        const float* kp = base + (int64_t)min(key, T - 1) * C3 + CH + 32 * j + 8 * g;
        const float ks = kln2(a.scale);
#pragma unroll
        for (int t = 0; t < 8; ++t) v[t] = key < T ? kp[t] * ks : 0.f;
        dst = kf + ((bh * (T32 / 16) + kt) * nj + j) * 128 + lane;
        stride = 64;
    } else {
        r -= kslots;
        const int64_t f = r >> 6;  // fragment (kb, dd)
        const int kb = (int)(f / nd), dd = (int)(f - (int64_t)kb * nd);
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const int key = 32 * kb + (t < 4 ? 4 * g + t : 16 + 4 * g + t - 4);
            v[t] = key < T ? base[(int64_t)key * C3 + 2 * CH + 16 * dd + li] : 0.f;
        }
        dst = vf + ((bh * (T32 / 32) + kb) * nd + dd) * 128 + lane;
        stride = 64;
    }
    h8v hi, lo;
    split8_f16(v, hi, lo);
    dst[0] = hi;
    dst[stride] = lo;
}

// K4d: the split attention, each 32-key block's packed K/V fragments
// (attn_kv_split's layout: K of the block's two 16-key tiles = 4 NJ contiguous
// 1-KiB pieces, V = 2 ND pieces) staged ONCE per workgroup into an NS-stage LDS
// ring by LDS-DMA (global_load_lds_dwordx4: no VGPR staging, no VALU), NS - 1
// blocks in flight, one barrier per block; WAVES waves (16 queries each) share
// one copy.  The round-2 form (K4s, removed in round 6) had every wave stream the
// whole K/V of its (sample, head) from L2 (1 GB of L2 reads per 32^2 attention at
// config B, its bound); K4d computes the same fragments in the same MFMA order
// with the same softmax, bit-identical to it.
template <int CH, int WAVES, int NS = 3, bool SPLIT = false>
__global__ __launch_bounds__(64 * WAVES) void attention_dma_kernel(AttnArgs a, const h8v* __restrict__ kf,
                                                                   const h8v* __restrict__ vf) {
    constexpr int NJ = CH / 32, ND = CH / 16;
    constexpr int KP = 4 * NJ, NP = KP + 2 * ND;   // 1-KiB pieces per block: K, then V
    constexpr int PPW = NP / WAVES;                // pieces per wave and block
    static_assert(NP % WAVES == 0 && NS >= 2 && NS <= 3, "piece split");
    __shared__ __attribute__((aligned(16))) h8v ring[NS][NP * 64];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = lane >> 4, li = lane & 15;
    // linear workgroup L goes to XCD L % 8: with xcdmap the query tiles of one
    // (sample, head) all get L % 8 == that group's XCD (the same queries, the same
    // arithmetic: a schedule change only)
    int qt = blockIdx.x, h = blockIdx.y;
    int64_t b = blockIdx.z;
    const int heads = gridDim.y;
    // SPLIT: grid.z = B x kc, this workgroup's key chunk kc_i of its (sample, head)
    const int kcs = SPLIT ? a.kc : 1;
    const int kc_i = SPLIT ? (int)(blockIdx.z % kcs) : 0;
    if (SPLIT) b = blockIdx.z / kcs;
    if (!SPLIT && a.xcdmap) {
        const int nt = gridDim.x;
        const int L = blockIdx.x + nt * (blockIdx.y + heads * blockIdx.z);
        const int r = L >> 3, grp = (r / nt) * 8 + (L & 7);
        qt = r - (r / nt) * nt;
        h = grp % heads;
        b = grp / heads;
    }
    const int T = a.T, T32 = (T + 31) / 32 * 32;
    const int q0 = (qt * WAVES + wave) * 16;
    const bool active = q0 < T;   // wave-uniform; an idle wave still stages and syncs
    CFD_DASSERT(h * CH + CH <= a.C);
    const int C3 = 3 * a.C;
    const float* base = a.qkv + b * (int64_t)T * C3 + (int64_t)h * 3 * CH;
    const int64_t bh = b * heads + h;
    const h8v* kfb = kf + bh * (T32 / 16) * NJ * 128;
    const h8v* vfb = vf + bh * (T32 / 32) * ND * 128;
    auto issue = [&](int kb, int stage) {
        const h8v* ks = kfb + (int64_t)(kb >> 4) * NJ * 128;
        const h8v* vs = vfb + (int64_t)(kb >> 5) * ND * 128;
#pragma unroll
        for (int i = 0; i < PPW; ++i) {
            const int piece = wave + WAVES * i;
            const h8v* src = piece < KP ? ks + piece * 64 : vs + (piece - KP) * 64;
            __builtin_amdgcn_global_load_lds((const void*)(src + lane),
                                             (__attribute__((address_space(3))) void*)&ring[stage][piece * 64], 16, 0, 0);
        }
    };
    // key blocks [blk0, blk0 + nblk) of this workgroup (all of them unless SPLIT)
    const int nall = T32 / 32, per = (nall + kcs - 1) / kcs;
    const int blk0 = kc_i * per, nblk = min(per, nall - blk0);
#pragma unroll
    for (int i = 0; i < NS - 1; ++i)
        if (i < nblk) issue(32 * (blk0 + i), i);

    h8v qh[NJ], ql[NJ];
    {
        const int tq = min(q0 + li, T - 1);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const float* qp = base + (int64_t)tq * C3 + 32 * j + 8 * g;
            float v[8];
#pragma unroll
            for (int t = 0; t < 8; ++t) v[t] = qp[t] * a.scale;
            split8_f16(v, qh[j], ql[j]);
        }
    }
    f4 O[ND];
#pragma unroll
    for (int d = 0; d < ND; ++d) O[d] = f4{0.f, 0.f, 0.f, 0.f};
    float mrun = -INFINITY, lrun = 0.f;

    for (int ib = 0; ib < nblk; ++ib) {
        const int kb = 32 * (blk0 + ib), stage = ib % NS;
        // this wave's pieces of block ib landed (the blocks issued after it may
        // still fly), then the barrier publishes every wave's pieces and retires
        // every read of the stage refilled below (block ib - 1's)
        if (NS == 3 && ib + 1 < nblk)
            __builtin_amdgcn_s_waitcnt(vmcnt_wait(PPW));
        else
            __builtin_amdgcn_s_waitcnt(vmcnt_wait(0));
        __builtin_amdgcn_s_barrier();
        if (ib + NS - 1 < nblk) issue(kb + 32 * (NS - 1), (ib + NS - 1) % NS);
        if (!active) continue;
        const h8v* kl8 = &ring[stage][lane];
        f4 st[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            st[u] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const h8v kh = kl8[((u * NJ + j) * 2) * 64], kl = kl8[((u * NJ + j) * 2 + 1) * 64];
                st[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kl, qh[j], st[u], 0, 0, 0);
                st[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kh, ql[j], st[u], 0, 0, 0);
                st[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kh, qh[j], st[u], 0, 0, 0);
            }
        }
        float mx = -INFINITY;
        if (kb + 32 > T) {
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (kb + 16 * u + 4 * g + r >= T) st[u][r] = -INFINITY;
        }
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int r = 0; r < 4; ++r) mx = fmaxf(mx, st[u][r]);
        mx = fmaxf(mx, __shfl_xor(mx, 16));
        mx = fmaxf(mx, __shfl_xor(mx, 32));
        const float mnew = fmaxf(mrun, mx);
        const float alpha = __builtin_amdgcn_exp2f(mrun - mnew);
        float p[8], ps = 0.f;
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                p[4 * u + r] = __builtin_amdgcn_exp2f(st[u][r] - mnew);
                ps += p[4 * u + r];
            }
        ps += __shfl_xor(ps, 16);
        ps += __shfl_xor(ps, 32);
        lrun = lrun * alpha + ps;
        mrun = mnew;
#pragma unroll
        for (int d = 0; d < ND; ++d) O[d] = O[d] * alpha;
        h8v ph, pl;
        split8_f16(p, ph, pl);
        const h8v* vl8 = &ring[stage][KP * 64 + lane];
#pragma unroll
        for (int d = 0; d < ND; ++d) {
            const h8v vh = vl8[(2 * d) * 64], vl = vl8[(2 * d + 1) * 64];
            O[d] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vl, ph, O[d], 0, 0, 0);
            O[d] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vh, pl, O[d], 0, 0, 0);
            O[d] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vh, ph, O[d], 0, 0, 0);
        }
    }
    if (!active) return;
    const int tq = q0 + li;
    if constexpr (SPLIT) {   // this chunk's unnormalised O and its (max, sum), for attn_combine_kernel
        if (tq < T) {
            const int64_t row = ((int64_t)kc_i * (gridDim.z / kcs) + b) * heads + h;
            float* op = a.part + (row * T + tq) * CH;
#pragma unroll
            for (int d = 0; d < ND; ++d) *(f4*)(op + 16 * d + 4 * g) = O[d];
            if (g == 0) {
                float* ml = a.part + (int64_t)kcs * (gridDim.z / kcs) * heads * T * CH;
                *(float2*)(ml + 2 * (row * T + tq)) = float2{mrun, lrun};
            }
        }
        return;
    }
    if (a.lse && g == 0 && tq < T)
        a.lse[((int64_t)b * gridDim.y + h) * T + tq] = (mrun + log2f(lrun)) * 0.69314718055994530942f;
    if (tq < T) {
        float* op = a.out + (b * (int64_t)T + tq) * a.C + (int64_t)h * CH;
        const float inv = 1.0f / lrun;
#pragma unroll
        for (int d = 0; d < ND; ++d) {
            f4 v = O[d] * inv;
            *(f4*)(op + 16 * d + 4 * g) = v;
        }
    }
}

// ---------------------------------------------------------------------------
// The key-chunked attention's combine pass: per (sample, head, query) the kc
// chunks' (max m_c, sum l_c, unnormalised O_c) in chunk order, M = max m_c,
// O = sum 2^(m_c - M) O_c / sum 2^(m_c - M) l_c (base 2, as the kernel's softmax);
// the log-sum-exp for the backward where it is kept.  One thread per 4 channels.
template <int CH>
__global__ __launch_bounds__(256) void attn_combine_kernel(AttnArgs a, int heads, int B) {
    constexpr int Q = CH / 4;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t rows = (int64_t)B * heads * a.T;
    if (i >= rows * Q) return;
    const int d4 = (int)(i % Q);
    const int64_t r = i / Q;   // (b, h, q) row
    const int kc = a.kc;
    const float* ml = a.part + (int64_t)kc * rows * CH;
    float M = -INFINITY;
    for (int c = 0; c < kc; ++c) M = fmaxf(M, ml[2 * (c * rows + r)]);
    float L = 0.f;
    f4 o = {0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < kc; ++c) {
        const float w = __builtin_amdgcn_exp2f(ml[2 * (c * rows + r)] - M);
        L += w * ml[2 * (c * rows + r) + 1];
        o += w * *(const f4*)(a.part + (c * rows + r) * CH + 4 * d4);
    }
    const int tq = (int)(r % a.T);
    const int64_t bh = r / a.T;
    const int h = (int)(bh % heads);
    const int64_t b = bh / heads;
    *(f4*)(a.out + (b * (int64_t)a.T + tq) * a.C + (int64_t)h * CH + 4 * d4) = o * (1.0f / L);
    if (a.lse && d4 == 0) a.lse[bh * a.T + tq] = (M + log2f(L)) * 0.69314718055994530942f;
}

// ---------------------------------------------------------------------------
// K5: timestep embedding and small dense layers.
// ---------------------------------------------------------------------------
__global__ void temb_kernel(const int64_t* __restrict__ t, const float* __restrict__ freqs, float* __restrict__ out,
                            int dim) {
    const int b = blockIdx.x;
    const int half = dim / 2;
    const float tf = (float)t[b];
    for (int i = threadIdx.x; i < dim; i += blockDim.x) {
        float v = 0.f;
        if (i < half) {
            v = cosf(tf * freqs[i]);
        } else if (i < 2 * half) {
            v = sinf(tf * freqs[i - half]);
        }
        out[(int64_t)b * dim + i] = v;
    }
}

// y[b][n] = bias[n] + sum_k W[n][k] * act(x[b][k]); one wave per output feature.
// y[b][n] = W[n] . act(x[b]) + bias[n] (time_embed, emb_layers): a bandwidth
// problem (the weights are read once, ~15 MB for all emb_layers at config B).
// One wave per output feature, its weight row held in registers as KW float4s
// per lane (K <= 256 KW); act(x) staged once per workgroup in LDS, 8 samples at
// a time; fixed-order lane reduction per sample (batch-invariant: sample b's
// sum does not depend on B).
template <int KW>
__global__ __launch_bounds__(256) void linear_kernel(const float* __restrict__ x, const float* __restrict__ W,
                                                     const float* __restrict__ bias, float* __restrict__ y, int B,
                                                     int K, int N, int act) {
    constexpr int BC = 8;   // samples per LDS chunk
    extern __shared__ __attribute__((aligned(16))) float xs[];   // BC x K
    const int lane = threadIdx.x & 63;
    const int n = blockIdx.x * 4 + (threadIdx.x >> 6);
    const bool live = n < N;
    CFD_DASSERT(K <= 256 * KW && K % 4 == 0);
    f4 w[KW];
#pragma unroll
    for (int i = 0; i < KW; ++i) {
        const int k = 4 * (lane + 64 * i);
        w[i] = live && k < K ? *(const f4*)(W + (int64_t)n * K + k) : f4{0.f, 0.f, 0.f, 0.f};
    }
    const float bn = live ? bias[n] : 0.f;
    for (int b0 = 0; b0 < B; b0 += BC) {
        const int nb = min(BC, B - b0);
        __syncthreads();   // the previous chunk's readers are done
        for (int i = threadIdx.x; i < nb * K; i += 256) {
            const float v = x[(int64_t)b0 * K + i];
            xs[i] = act ? silu_f(v) : v;
        }
        __syncthreads();
        if (!live) continue;
        for (int bb = 0; bb < nb; ++bb) {
            float s = 0.f;
#pragma unroll
            for (int i = 0; i < KW; ++i) {
                const int k = 4 * (lane + 64 * i);
                if (k < K) {
                    const f4 v = *(const f4*)(xs + bb * K + k);
                    s = fmaf(w[i][0], v[0], s);
                    s = fmaf(w[i][1], v[1], s);
                    s = fmaf(w[i][2], v[2], s);
                    s = fmaf(w[i][3], v[3], s);
                }
            }
            for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
            if (lane == 0) y[(int64_t)(b0 + bb) * N + n] = s + bn;
        }
    }
}

// ---------------------------------------------------------------------------
// host-side launchers
// ---------------------------------------------------------------------------
// Pixel chunks of the three-kernel GroupNorm (forward and backward): a function
// of HW only (batch invariance).  Up to 64 at the config-B sizes; the large
// latents (Case4 384^2, 192^2) take up to kGnMaxChunks so a batch-1 sample still
// spreads its statistics pass over the whole chip.
int gn_chunks(int HW) {
    const int64_t small = std::min<int64_t>(64, HW / 16);
    return (int)std::max<int64_t>(1, std::min<int64_t>(kGnMaxChunks, std::max<int64_t>(HW / 64, small)));
}

static unsigned long long* g_stamps = nullptr;
void stamps_set(unsigned long long* buf) { g_stamps = buf; }
unsigned long long* stamps_buf() { return g_stamps; }
static int g_seq = 0;   // launch sequence number of the U-Net kernels (timestamps)

static int env_int(const char* name, int dflt) {
    const char* e = getenv(name);
    return e ? atoi(e) : dflt;
}

// the two-launch full-row GroupNorm (gn2_*) for this shape (a function of the
// per-sample shape only: batch invariance): from 4096 pixels per sample at the
// default plan.  Measured: B = 1 64^2 -3.5 %, config E -3 %, B = 8 flat; the
// threshold scales with the planned batch (plan_b 2: from 1024 pixels, where the
// one-launch kernels' 32 workgroups per sample leave a batch-1 chip idle)
bool gn2_applies(const GnArgs& a) {
    const int pb = a.plan_b > 0 ? a.plan_b : 8;
    return (int64_t)a.HW * 8 >= (int64_t)4096 * pb && a.Ctot % 4 == 0 && a.C1 % 4 == 0 && a.C2 % 4 == 0 &&
           a.Ctot <= 1024;
}

// rows of the register-resident kernel's (pixel, channel-quad) grid per pass and
// pixels per thread (0: not that kernel's shape)
static int gn_reg_ipt(const GnArgs& a) {
    return a.Ctot % 128 == 0 ? (int)ceil_div(a.HW, 512 / (a.Ctot / 128)) : 0;
}

bool gn_takes_splitk(const GnArgs& a, int B) {
    (void)B;
    if (gn2_applies(a)) return a.C1 % 4 == 0;
    if (a.Ctot % 128 != 0 || a.C1 % 4 != 0) return false;
    return gn_reg_ipt(a) <= 16;
}

void launch_gn(const GnArgs& a0, int B, hipStream_t st) {
    CFD_REQUIRE(a0.Ctot % 32 == 0 && a0.C1 % 4 == 0 && a0.C2 % 4 == 0 && a0.Ctot <= 1024, CFD_ESHAPE,
                "GroupNorm32 needs channels % 32 == 0 (<= 1024)");
    GnArgs a = a0;
    a.nchunks = gn_chunks(a.HW);
    a.B = B;
    a.stamps = g_stamps;
    a.seq = g_seq++;
    CFD_REQUIRE(!a.kpart || gn_takes_splitk(a, B), CFD_ESTATE, "internal: split-K source on a GroupNorm path without it");
    if (gn2_applies(a)) {
        CFD_REQUIRE(!a.kpart || a.kx, CFD_ESTATE, "internal: gn2 needs the split-K sum's destination");
        a.nchunks = gn2_chunks(a.HW, a.plan_b);
        if (gn2_threads(a.nchunks) == 1024) {
            hipLaunchKernelGGL(gn2_stats_kernel<1024>, dim3(a.nchunks, B), dim3(1024), 0, st, a);
            check_launch("gn2_stats_kernel");
            hipLaunchKernelGGL(gn2_apply_kernel<1024>, dim3(a.nchunks, B), dim3(1024), 0, st, a);
        } else {
            hipLaunchKernelGGL(gn2_stats_kernel<256>, dim3(a.nchunks, B), dim3(256), 0, st, a);
            check_launch("gn2_stats_kernel");
            hipLaunchKernelGGL(gn2_apply_kernel<256>, dim3(a.nchunks, B), dim3(256), 0, st, a);
        }
        check_launch("gn2_apply_kernel");
        return;
    }
    // one workgroup per (sample, group), the sample's rows in registers; 1024
    // threads up to 16 pixels per thread (twice the waves, and loads, in flight per
    // CU).  Large latents (ipt > 32) would leave the chip idle at small batch (32
    // workgroups at B = 1, 384^2): they take the three-kernel path below, whose
    // statistics spread over gn_chunks(HW) chunks
    const int ipt = gn_reg_ipt(a);
    if (ipt > 0 && ipt <= 32) {
        const dim3 grid((unsigned)(32 * B));
        // small groups (<= 1024 float4 per (sample, group): the 16^2 / 8^2 levels):
        // 256-thread workgroups, up to 4 float4 per thread -- a quarter of the waves
        // to gather at the statistics barrier
        const int nq = a.Ctot / 128, r256 = 256 / nq, i256 = (a.HW + r256 - 1) / r256;
        if (i256 <= 4) {
            if (i256 <= 1)
                hipLaunchKernelGGL((gn_fused_reg_kernel<1, 256>), grid, dim3(256), 0, st, a);
            else if (i256 <= 2)
                hipLaunchKernelGGL((gn_fused_reg_kernel<2, 256>), grid, dim3(256), 0, st, a);
            else
                hipLaunchKernelGGL((gn_fused_reg_kernel<4, 256>), grid, dim3(256), 0, st, a);
            check_launch("gn_fused_reg_kernel");
            return;
        }
        if (ipt <= 4)
            hipLaunchKernelGGL((gn_fused_reg_kernel<2, 1024>), grid, dim3(1024), 0, st, a);
        else if (ipt <= 8)
            hipLaunchKernelGGL((gn_fused_reg_kernel<4, 1024>), grid, dim3(1024), 0, st, a);
        else if (ipt <= 16)
            hipLaunchKernelGGL((gn_fused_reg_kernel<8, 1024>), grid, dim3(1024), 0, st, a);
        else
            hipLaunchKernelGGL(gn_fused_reg_kernel<32>, grid, dim3(512), 0, st, a);
        check_launch("gn_fused_reg_kernel");
        return;
    }
    hipLaunchKernelGGL(gn_partial_kernel, dim3(a.nchunks, B), dim3(256), 0, st, a);
    check_launch("gn_partial_kernel");
    hipLaunchKernelGGL(gn_finalize_kernel, dim3(B), dim3(1024), 0, st, a);
    check_launch("gn_finalize_kernel");
    const int64_t nq = (int64_t)B * a.HW * a.Ctot / 4;
    hipLaunchKernelGGL(gn_apply_kernel, dim3((unsigned)std::min<int64_t>(4096, ceil_div(nq, 256))), dim3(256), 0, st, a);
    check_launch("gn_apply_kernel");
}


// K1h splits chunk ranges of ceil(nch / splits) chunks: drop the splits that
// would be left with none (they cost a zero partial slab written and read)
static int even_splits(int nch, int splits) {
    if (splits <= 1) return 1;
    const int per = (nch + splits - 1) / splits;
    return (nch + per - 1) / per;
}

ConvPlan plan_conv(const ConvArgs& a, size_t part_cap_floats) {
    // Every choice is made from the per-sample shape at the planned batch (8 unless
    // the model sets another, cfd_unet_set_plan_batch), never from the actual
    // batch: the split-K count fixes each output's summation order, so a sample's
    // eps is then bit-identical whatever batch (or rank shard) it is computed in.
    // part_cap_floats: the split-K slab per planned batch (the caller sizes the
    // real slab as ceil(B / plan_b) of these)
    const int plan_b = a.plan_b > 0 ? a.plan_b : 8;
    ConvPlan p;
    const int64_t mn = (int64_t)plan_b * a.Hout * a.Wout;
    p.bn = a.Cout >= 128 ? 128 : 64;
    auto tiles = [&](int bm) { return ceil_div(mn, bm) * ceil_div(a.Cout, p.bn); };
    // K1s tiles: 8-wave 128x128 for Cout >= 128, counted as 2 workgroups each (r01
    // sweep, B = 8 64^2 forward: 5.51 ms vs 5.88 with 4-wave tiles), else 64x64;
    // split-K up to a 768-workgroup target, >= 4 K tiles per split
    p.bm = 64;
    int wg_per_tile = 1;
    if (p.bn == 128) {
        p.bm = 128;
        p.nw = 8;
        wg_per_tile = 2;
    }
    const int nkt = a.K / 32;
    p.splits = 1;
    while (tiles(p.bm) * wg_per_tile * p.splits < 768 && nkt / (p.splits * 2) >= 4 && p.splits < 16)
        p.splits *= 2;
    // 1x1 convolutions (qkv, proj_out, skip) with >= 128 tiles: no split-K.  Their
    // K is short (256-640), so a split only adds partial slabs and a reduction pass
    // (convbench, reduction included: 1.09-1.72x unsplit on the config-B shapes
    // with 128-256 tiles, 0.5-0.8x below)
    if (a.ks == 1 && !a.tmode && tiles(p.bm) >= 128) p.splits = 1;
    // memory guard, on the nominal shape too
    while (p.splits > 1 && (size_t)p.splits * mn * a.Cout > part_cap_floats) p.splits /= 2;
    // the large-latent levels (Case4's 192^2 / 384^2) with <= 128 input channels
    // stay on the K1s 128x128 8-wave tiles (tools/convbench at one sample: 384^2
    // 128->128 178 vs K1h 199 us, the 2x upsampling 174 vs 197, 192^2 128->128 63
    // vs 74; 256 input channels go to K1h: 344 vs 364 us)
    if (a.wlo && a.ks == 3 && a.stride == 1 && !a.tmode && a.Ctot <= 128 && (int64_t)a.Hout * a.Wout >= 36864)
        return p;
    const int64_t srows = mn / ((int64_t)a.Hout * a.Wout) * a.Hin * a.Win;
    const bool fits32 = srows < (1 << 23) && srows * std::max(a.C1, a.C2) * 4 < (1ll << 30) &&
                        (int64_t)a.Cout * a.K * 2 < (1ll << 31);
    auto halo_splits = [&](int64_t t) {   // K1h / K1hb: split-K over the 32-channel chunks
        const int nch = a.Ctot / 32;
        int sp = 1;
        while (t * sp < 256 && sp * 2 <= nch && sp < 16) sp *= 2;
        while (sp > 1 && (size_t)sp * mn * a.Cout > part_cap_floats) sp /= 2;
        return even_splits(nch, sp);
    };
    // K1hb (conv_x.hip): the bf16-operand 3x3 convolutions (config E) on the halo
    // tiles; the others (8^2, which the 256-pixel tiles do not cover) stay on the
    // K1s bf16 tiles
    if (a.wbf && !a.wlo && !a.tmode && a.ks == 3 && a.stride == 1 && a.Cout >= 128 && fits32 && conv_h_tw(a) > 0) {
        ConvPlan q;
        q.kx = 22;
        q.bm = 256;
        q.bn = 128;
        q.nw = 8;
        q.splits = halo_splits(ceil_div(mn, 256) * ceil_div(a.Cout, 128));
        return q;
    }
    // the split-f16 3x3 stride-1 convolutions: K1h (halo tiles) where a 256-pixel
    // block tiles the image (16x16 and up: each activation fetched once per
    // 32-channel chunk instead of once per tap; tools/convbench, same box:
    // 1.19-1.29x K1x on the config-B 64^2 / 32^2 shapes, 1.04-1.17x at 16^2), else
    // K1x: 64x64 wave tiles on 32x32x16 MFMAs, 256x128 workgroup tiles where the
    // per-sample shape has >= 256 pixels at the planned batch, 128x128 below
    // (1.04-1.17x the K1s tiles).  1x1 and stride-2 convolutions stay on K1s.
    if (a.wbf && a.wlo && !a.tmode && a.ks == 3 && a.stride == 1 && a.Cout >= 128 && fits32) {
        ConvPlan q;
        if (conv_h_tw(a) > 0) {
            q.kx = 20;
            q.bm = 256;
            q.bn = 128;
            q.nw = 8;
            q.splits = halo_splits(ceil_div(mn, 256) * ceil_div(a.Cout, 128));
            return q;
        }
        // at least 4 K tiles per split, at most 32 splits: the small levels (8^2,
        // 4^2) run long K chains on few tiles, and at batch 1 each K tile waits a
        // memory latency (config A 32^2 B = 1 forward 2.78 -> 2.68 ms against 8 / 16)
        q.kx = mn >= 2048 ? 2 : 1;
        q.bm = q.kx == 2 ? 256 : 128;
        q.bn = 128;
        q.nw = q.kx == 2 ? 8 : 4;
        const int64_t t = ceil_div(mn, q.bm) * ceil_div(a.Cout, q.bn);
        q.splits = 1;
        while (t * q.splits < 256 && nkt / (q.splits * 2) >= 4 && q.splits < 32) q.splits *= 2;
        while (q.splits > 1 && (size_t)q.splits * mn * a.Cout > part_cap_floats) q.splits /= 2;
        return q;
    }
    return p;
}

// grid size below which the K1s / K1h forward tiles go 64 channels wide
// (CFD_CONV_SMALLN: 0 never, 1 the default 128 workgroups, n > 1 below n)
int smalln_below() {
    const int v = env_int("CFD_CONV_SMALLN", 1);
    return v == 1 ? 128 : std::max(v, 0);
}

template <bool TMODE, int MODE, bool BUFA>
static void launch_conv_tiles_(const ConvArgs& a, const ConvPlan& p, dim3 grid, hipStream_t st) {
    if constexpr (MODE != 0 && BUFA) {   // the split-f16 / bf16 tiles, forward and transposed
        // small batch (forward): where the 128 x 128 grid leaves most CUs idle (< 128
        // workgroups of 8 waves, two per SIMD), 128 x 64 tiles of 8 waves (32 x 32
        // each) -- twice the workgroups, half the work per wave, the same tiles'
        // sums (CFD_CONV_SMALLN=0 keeps 128 x 128)
        static const int smalln = smalln_below();
        if (!TMODE && p.nw == 8 && p.bm == 128 && p.bn == 128 && (int64_t)grid.x * grid.y * grid.z < smalln &&
            a.Cout % 64 == 0) {
            const dim3 g64(grid.x, (unsigned)ceil_div(a.Cout, 64), grid.z);
            hipLaunchKernelGGL((conv_gemm_kernel<128, 64, false, MODE, 8, true>), g64, dim3(512), 0, st, a);
            return;
        }
        // the register ring of K tiles (p.pf deep; the same tiles in the same order)
        if (p.nw == 8 && p.bm == 128 && p.bn == 128 && p.pf == 2) {
            hipLaunchKernelGGL((conv_gemm_kernel<128, 128, TMODE, MODE, 8, true, 2>), grid, dim3(512), 0, st, a);
            return;
        }
        if (p.nw == 8 && p.bm == 128 && p.bn == 128 && p.pf == 3) {
            hipLaunchKernelGGL((conv_gemm_kernel<128, 128, TMODE, MODE, 8, true, 3>), grid, dim3(512), 0, st, a);
            return;
        }
    }
    if (p.nw == 8 && p.bm == 128 && p.bn == 128)
        hipLaunchKernelGGL((conv_gemm_kernel<128, 128, TMODE, MODE, 8, BUFA>), grid, dim3(512), 0, st, a);
    else if (p.bm == 128 && p.bn == 128)
        hipLaunchKernelGGL((conv_gemm_kernel<128, 128, TMODE, MODE, 4, BUFA>), grid, dim3(256), 0, st, a);
    else if (p.bm == 64 && p.bn == 128)
        hipLaunchKernelGGL((conv_gemm_kernel<64, 128, TMODE, MODE, 4, BUFA>), grid, dim3(256), 0, st, a);
    else if (p.bm == 128 && p.bn == 64)
        hipLaunchKernelGGL((conv_gemm_kernel<128, 64, TMODE, MODE, 4, BUFA>), grid, dim3(256), 0, st, a);
    else
        hipLaunchKernelGGL((conv_gemm_kernel<64, 64, TMODE, MODE, 4, BUFA>), grid, dim3(256), 0, st, a);
}

template <bool TMODE, int MODE>
static void launch_conv_tiles(const ConvArgs& a, const ConvPlan& p, dim3 grid, hipStream_t st) {
    if (a.bufaddr) return launch_conv_tiles_<TMODE, MODE, true>(a, p, grid, st);
    launch_conv_tiles_<TMODE, MODE, false>(a, p, grid, st);
}

void launch_splitk_reduce(const ConvArgs& a, int splits, hipStream_t st) {
    const int64_t total4 = (int64_t)a.M * a.Cout / 4;
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)ceil_div(total4, 256)), dim3(256), 0, st, a, splits);
    check_launch("splitk_reduce_kernel");
}

// K1x / K1h need 32-bit operand offsets at the real batch; else K1s 128x128 tiles of 8
// waves with the same splits (CFD_CONV_FORCE_K1S=1 forces that fallback: tests)
static bool conv_x_falls_back(const ConvArgs& a) {
    static const int force_k1s = env_int("CFD_CONV_FORCE_K1S", 0);
    const int64_t srows = (int64_t)a.Hin * a.Win * (a.M / (a.Hout * a.Wout));
    return force_k1s || !(srows < (1 << 24) && a.M < (1 << 24) && srows * std::max(a.C1, a.C2) * 4 < (1ll << 31));
}

bool conv_runs_k1hb(const ConvArgs& a, const ConvPlan& p) { return p.kx == 22 && !conv_x_falls_back(a); }

bool conv_kv_pack_ok(const ConvArgs& a, const ConvPlan& p, int T) {
    // launch_conv's choices: K1s (a 1x1 never takes K1x), split or bf16 compute
    // (MODE 2 / 1: bands of whole 32-row blocks), the LDS epilogue on, one split
    static const int ldsepi = env_int("CFD_CONV_LDSEPI", 1);
    return ldsepi && p.kx < 0 && p.splits == 1 && a.wbf && !a.tmode && a.ks == 1 && a.bias &&
           !a.emb && !a.res && a.Cout % 8 == 0 && a.emb_stride % 4 == 0 && T % 32 == 0 && a.M % T == 0;
}

int launch_conv(const ConvArgs& a, const ConvPlan& p0, hipStream_t st, bool defer) {
    ConvPlan p = p0;
    if (p.kx >= 0 && conv_x_falls_back(a)) {
        p.kx = -1;
        p.bm = p.bn = 128;
        p.nw = 8;
    }
    CFD_REQUIRE(!a.src_bf16 || p.kx == 22, CFD_ESTATE, "internal: a bf16 convolution source needs the K1hb kernel");
    // K1s register-ring depth (development: CFD_CONV_PF; the tiles and their order,
    // hence the sums, do not depend on it)
    // (round 5 default 2: B = 8 64^2 3.95 -> 3.92 ms per step, others flat, r05as)
    static const int pf = env_int("CFD_CONV_PF", 2);
    if (p.kx < 0) p.pf = pf >= 1 && pf <= 3 ? pf : 1;
    CFD_REQUIRE(a.Ctot % 32 == 0 && a.C1 % 4 == 0 && a.C2 % 4 == 0, CFD_ESHAPE, "conv_gemm needs channels % 32 == 0");
    CFD_REQUIRE(a.K == a.ks * a.ks * a.Ctot, CFD_ESHAPE, "conv K mismatch");
    CFD_REQUIRE(p.splits == 1 || (a.part && a.Cout % 4 == 0), CFD_ESTATE, "split-K needs a partial buffer");
    CFD_REQUIRE(!a.tmode || ((a.stride == 1 || a.stride == 2) && !a.up), CFD_ESHAPE, "transposed conv: stride 1|2");
    const dim3 grid((unsigned)ceil_div(a.M, p.bm), (unsigned)ceil_div(a.Cout, p.bn), p.splits);
    CFD_REQUIRE(!(a.tmode && a.wbf && !a.wlo), CFD_ESTATE, "bf16 input-gradient convolutions are not built");
    static const int xcd = env_int("CFD_CONV_XCD", 4);   // round 5: 3 (PMC: 16^2 K1h L2 hit 0.19-0.27 -> 0.69-0.79), then 4
    static const int ldsepi = env_int("CFD_CONV_LDSEPI", 1);
    ConvArgs b = a;
    b.stamps = g_stamps;
    b.seq = g_seq++;
    // float4 rows need Cout % 4 == 0 and 16-B aligned bias / emb / res / out rows
    b.ldsepi = ldsepi && a.Cout % 4 == 0 && a.emb_stride % 4 == 0;
    // 1: splits-fastest XCD order; 2: m-fastest (weight-sharing) order; 3: order 2 where
    // the per-sample image has <= 256 pixels (the small-M levels), else 1; 4: order 1
    // for the bf16-operand convolutions (config E 4.66 -> 4.62 ms per step; the
    // split-f16 config A is 0.3 % slower with it, r05as), 3 for the others
    const int xo = xcd == 4 ? (a.wbf && !a.wlo ? 1 : 3) : xcd;
    b.xcd = xo == 3 ? ((int64_t)a.Hout * a.Wout <= 256 ? 2 : 1) : xo < 0 || xo > 2 ? 1 : xo;
    {   // 32-bit buffer offsets and 24-bit pixel indices must hold
        const int64_t srows = (int64_t)a.Hin * a.Win * (a.M / (a.Hout * a.Wout));
        const int64_t wes = (a.wbf || a.wlo) ? 2 : 4;
        b.bufaddr = a.ks * a.ks <= 9 && srows < (1 << 24) && a.M < (1 << 24) &&
                    srows * std::max(a.C1, a.C2) * 4 < (1ll << 31) && (int64_t)a.Cout * a.K * wes < (1ll << 31);
    }
    const ConvArgs& a_ = b;
    if (p.kx >= 0) {
        launch_conv_x(a_, p.kx, p.splits, st);
        if (p.splits > 1 && !defer) launch_splitk_reduce(a, p.splits, st);
        return p.splits;
    }
    if (a.tmode && a.wlo)
        launch_conv_tiles<true, 2>(a_, p, grid, st);
    else if (a.tmode)
        launch_conv_tiles<true, 0>(a_, p, grid, st);
    else if (a.wbf && a.wlo)
        launch_conv_tiles<false, 2>(a_, p, grid, st);
    else if (a.wbf)
        launch_conv_tiles<false, 1>(a_, p, grid, st);
    else
        launch_conv_tiles<false, 0>(a_, p, grid, st);
    check_launch("conv_gemm_kernel");
    if (p.splits > 1 && !defer) launch_splitk_reduce(a, p.splits, st);
    return p.splits;
}

void launch_conv_in(const ConvArgs& a, hipStream_t st) {
    if (a.Cout % 4 == 0 && a.C1 <= 4 && (size_t)9 * a.C1 * a.Cout * 4 <= 64 * 1024) {
        const int64_t n = (int64_t)a.M * (a.Cout / 4);
        hipLaunchKernelGGL(conv_in_vec_kernel, dim3((unsigned)std::min<int64_t>(2048, ceil_div(n, 256))), dim3(256),
                           sizeof(float) * 9 * a.C1 * a.Cout, st, a);
        check_launch("conv_in_vec_kernel");
        return;
    }
    const int64_t n = (int64_t)a.M * a.Cout;
    hipLaunchKernelGGL(conv_in_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, st, a);
    check_launch("conv_in_kernel");
}

void launch_conv_out(const ConvArgs& a, hipStream_t st) {
    CFD_REQUIRE(a.Cout <= 4, CFD_ESHAPE, "out_channels must be <= 4");
    const int LP = a.Ctot / 4;
    if (a.Ctot % 4 == 0 && a.C1 == a.Ctot && LP >= 1 && LP <= 64 && (LP & (LP - 1)) == 0 &&
        (size_t)a.Cout * a.K * 4 <= 64 * 1024) {
        const int64_t waves = ceil_div(a.M, 64 / LP);
        hipLaunchKernelGGL(conv_out_vec_kernel, dim3((unsigned)std::min<int64_t>(8192, ceil_div(waves, 4))), dim3(256),
                           sizeof(float) * a.Cout * a.K, st, a, LP);
        check_launch("conv_out_vec_kernel");
        return;
    }
    hipLaunchKernelGGL(conv_out_kernel, dim3((unsigned)ceil_div(a.M, 4)), dim3(256), 0, st, a);
    check_launch("conv_out_kernel");
}

void launch_attention(const AttnArgs& a, int CH, int heads, int B, hipStream_t st) {
    const dim3 grid((unsigned)ceil_div(a.T, 64), heads, B);
    switch (CH) {
        case 16: hipLaunchKernelGGL(attention_kernel<16>, grid, dim3(256), 0, st, a); break;
        case 32: hipLaunchKernelGGL(attention_kernel<32>, grid, dim3(256), 0, st, a); break;
        case 64: hipLaunchKernelGGL(attention_kernel<64>, grid, dim3(256), 0, st, a); break;
        case 128: hipLaunchKernelGGL(attention_kernel<128>, grid, dim3(256), 0, st, a); break;
        default: throw Error{CFD_ESHAPE, "attention head channels must be 16, 32, 64 or 128"};
    }
    check_launch("attention_kernel");
}

size_t attention_split_floats(int T, int C) { return (size_t)(T + 31) / 32 * 32 * C * 2; }

int64_t attention_split_voff(int T, int CH, int heads, int B) {
    const int T32 = (T + 31) / 32 * 32;
    return (int64_t)B * heads * (T32 / 16) * (CH / 32) * 128;
}

// Key chunks: where the planned batch's 4-wave grid has at most 128 workgroups
// (planned batch 1-2 at 32^2 and below), the keys of each (sample, head) are split
// into kc chunks of >= 2 blocks (kc x the grid <= 256), each a workgroup of its own,
// and a combine pass adds the chunks' softmax partials in chunk order.  A function
// of T, heads and the planned batch only (never of the real batch): a sample's bits
// stay batch-invariant for a given plan.  At the default plan (8) every config-B / E
// level keeps kc = 1.  Measured (graph-loop step, same box, r06q): planned batch 1,
// B = 1 64^2 2.60 -> 2.52 ms, config A 2.17 -> 2.09 ms; a 16^2 split at plan 8
// (192 -> 384 workgroups) cost B = 8 +0.7 %, hence the bound.
int attention_kv_chunks(int T, int heads, int plan_b) {
    const int nblk = (T + 31) / 32;
    const int64_t wgs = (int64_t)plan_b * heads * ceil_div(T, 64);
    int kc = 1;
    while (kc * 4 <= nblk && wgs * kc * 2 <= 256) kc *= 2;
    return kc;
}

size_t attention_part_floats(int T, int C, int CH, int plan_b) {
    const int heads = C / CH, kc = attention_kv_chunks(T, heads, plan_b);
    return kc == 1 ? 0 : (size_t)kc * T * (C + 2 * heads);
}

void launch_attention_split(const AttnArgs& a, int CH, int heads, int B, int plan_b, float* kvws, hipStream_t st,
                            bool packed) {
    CFD_REQUIRE(CH == 32 || CH == 64 || CH == 128, CFD_ESHAPE, "split attention needs head channels 32, 64 or 128");
    const int T32 = (a.T + 31) / 32 * 32;
    h8v* kf = (h8v*)kvws;
    h8v* vf = kf + attention_split_voff(a.T, CH, heads, B);
    if (!packed) {   // else the qkv convolution's epilogue wrote them (ConvArgs::kvf)
        const int64_t slots = (int64_t)B * heads * ((T32 / 16) * (CH / 32) * 64 + (T32 / 32) * (CH / 16) * 64);
        hipLaunchKernelGGL(attn_kv_split_kernel, dim3((unsigned)ceil_div(slots, 256)), dim3(256), 0, st, a, CH, heads,
                           B, kf, vf);
        check_launch("attn_kv_split_kernel");
    }
    const int kc = attention_kv_chunks(a.T, heads, plan_b);
    if (kc > 1) {
        CFD_REQUIRE(a.part, CFD_ESTATE, "internal: key-chunked attention without a partial buffer");
        AttnArgs a2 = a;
        a2.kc = kc;
        a2.xcdmap = 0;
        const dim3 grid((unsigned)ceil_div(a.T, 64), heads, B * kc);
        switch (CH) {
            case 32: hipLaunchKernelGGL((attention_dma_kernel<32, 4, 3, true>), grid, dim3(256), 0, st, a2, kf, vf); break;
            case 64: hipLaunchKernelGGL((attention_dma_kernel<64, 4, 3, true>), grid, dim3(256), 0, st, a2, kf, vf); break;
            default: hipLaunchKernelGGL((attention_dma_kernel<128, 4, 3, true>), grid, dim3(256), 0, st, a2, kf, vf); break;
        }
        check_launch("attention_dma_kernel (key chunks)");
        const int64_t n = (int64_t)B * heads * a.T * (CH / 4);
        const dim3 g2((unsigned)ceil_div(n, 256));
        switch (CH) {
            case 32: hipLaunchKernelGGL(attn_combine_kernel<32>, g2, dim3(256), 0, st, a2, heads, B); break;
            case 64: hipLaunchKernelGGL(attn_combine_kernel<64>, g2, dim3(256), 0, st, a2, heads, B); break;
            default: hipLaunchKernelGGL(attn_combine_kernel<128>, g2, dim3(256), 0, st, a2, heads, B); break;
        }
        check_launch("attn_combine_kernel");
        return;
    }
    // K4d: fragments staged per workgroup by LDS-DMA, 8 waves (128 queries) per
    // workgroup where T >= 512 and that still gives >= 256 workgroups, else 4 -- at
    // batch 1 the 64-query workgroups double the parallelism of the 32^2 blocks
    // (the choice changes no result: every query's arithmetic is the same)
    static const int xcdmap = env_int("CFD_ATTN_XCD", 1);   // (sample, head) workgroups on one XCD
    AttnArgs a2 = a;
    a2.xcdmap = xcdmap && (heads * B) % 8 == 0 ? 1 : 0;
    const int w8 = a.T >= 512 && (int64_t)B * heads * ceil_div(a.T, 128) >= 256;
    const dim3 grid((unsigned)ceil_div(a.T, w8 ? 128 : 64), heads, B);
    const dim3 blk(w8 ? 512 : 256);
    switch (CH * 2 + w8) {
        case 64: hipLaunchKernelGGL((attention_dma_kernel<32, 4>), grid, blk, 0, st, a2, kf, vf); break;
        case 65: hipLaunchKernelGGL((attention_dma_kernel<32, 8>), grid, blk, 0, st, a2, kf, vf); break;
        case 128: hipLaunchKernelGGL((attention_dma_kernel<64, 4>), grid, blk, 0, st, a2, kf, vf); break;
        case 129: hipLaunchKernelGGL((attention_dma_kernel<64, 8>), grid, blk, 0, st, a2, kf, vf); break;
        case 256: hipLaunchKernelGGL((attention_dma_kernel<128, 4>), grid, blk, 0, st, a2, kf, vf); break;
        default: hipLaunchKernelGGL((attention_dma_kernel<128, 8>), grid, blk, 0, st, a2, kf, vf); break;
    }
    check_launch("attention_dma_kernel");
}

void launch_temb(const int64_t* t, const float* freqs, float* out, int dim, int B, hipStream_t st) {
    hipLaunchKernelGGL(temb_kernel, dim3(B), dim3(128), 0, st, t, freqs, out, dim);
    check_launch("temb_kernel");
}

void launch_linear(const float* x, const float* W, const float* bias, float* y, int B, int K, int N, int act,
                   hipStream_t st) {
    CFD_REQUIRE(K % 4 == 0 && K <= 2048, CFD_ESHAPE, "linear: K must be a multiple of 4, at most 2048");
    const dim3 g((unsigned)ceil_div(N, 4));
    const size_t lds = sizeof(float) * 8 * K;
    if (K <= 256) hipLaunchKernelGGL(linear_kernel<1>, g, dim3(256), lds, st, x, W, bias, y, B, K, N, act);
    else if (K <= 512) hipLaunchKernelGGL(linear_kernel<2>, g, dim3(256), lds, st, x, W, bias, y, B, K, N, act);
    else if (K <= 1024) hipLaunchKernelGGL(linear_kernel<4>, g, dim3(256), lds, st, x, W, bias, y, B, K, N, act);
    else hipLaunchKernelGGL(linear_kernel<8>, g, dim3(256), lds, st, x, W, bias, y, B, K, N, act);
    check_launch("linear_kernel");
}

}  // namespace cfd

// development hook of the CFD_STAMPS build (not in include/confild.h): the
// buffer the instrumented kernels append their timestamps to (null: off)
extern "C" int cfd_stamps_set(void* buf) {
#ifdef CFD_STAMPS
    cfd::stamps_set((unsigned long long*)buf);
    return CFD_OK;
#else
    (void)buf;
    cfd::set_error("cfd_stamps_set: not a CFD_STAMPS build (make STAMPS=1)");
    return CFD_ESTATE;
#endif
}
