// Latent U-Net kernels for gfx950 (K1-K5 of DESIGN.md), fp32, NHWC activations.
//
//   conv_gemm   K1/K2  implicit-GEMM 3x3 / 1x1 convolution on fp32 MFMA 16x16x4,
//                      GroupNorm(+SiLU) applied while staging the input tile
//                      (prologue), bias / timestep-embedding / residual fused in the
//                      epilogue, concat-free two-source input (skip connections),
//                      stride-2 (Downsample) and nearest-2x (Upsample) addressing;
//   gn_stats    K3     GroupNorm(32) statistics -> per-(b,c) scale/shift;
//   attention   K4     QKVAttentionLegacy (flash-style, fp32 MFMA, online softmax);
//   temb/linear K5     timestep embedding + time_embed MLP + all emb_layers;
//   conv_in / conv_out the 1-channel first/last convolutions (VALU).
#include "unet_kernels.hpp"

namespace cfd {

// ---------------------------------------------------------------------------
// K3: GroupNorm statistics.  One workgroup per (group, sample).  Output, per
// (b, c): scale = rstd*gamma, shift = beta - mean*scale, so the consumer applies
// y = x*scale + shift (the affine form of the ATen CPU GroupNorm kernel).
// ---------------------------------------------------------------------------
__global__ void gn_stats_kernel(GnArgs a) {
    const int grp = blockIdx.x;
    const int64_t b = blockIdx.y;
    const int cpg = a.Ctot / 32;
    const int64_t n = (int64_t)a.HW * cpg;
    const float* s1 = a.src1 + b * (int64_t)a.HW * a.C1;
    const float* s2 = a.src2 ? a.src2 + b * (int64_t)a.HW * a.C2 : nullptr;
    __shared__ double red[8];
    __shared__ double bc_mean, bc_rstd;

    auto load = [&](int64_t idx) -> float {
        const int64_t p = idx / cpg;
        const int c = grp * cpg + (int)(idx - p * cpg);
        return c < a.C1 ? s1[p * a.C1 + c] : s2[p * a.C2 + (c - a.C1)];
    };
    auto block_sum = [&](double v) -> double {
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
        __syncthreads();
        double t = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w];
        __syncthreads();
        return t;
    };
    double s = 0;
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) s += load(i);
    const double mean = block_sum(s) / (double)n;
    double v2 = 0;
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
        const double d = (double)load(i) - mean;
        v2 += d * d;
    }
    const double var = block_sum(v2) / (double)n;
    if (threadIdx.x == 0) {
        bc_mean = mean;
        bc_rstd = 1.0 / sqrt(var + (double)a.eps);
    }
    __syncthreads();
    const float meanf = (float)bc_mean, rstd = (float)bc_rstd;
    for (int j = threadIdx.x; j < cpg; j += blockDim.x) {
        const int c = grp * cpg + j;
        const float sc = rstd * a.gamma[c];
        a.ss[(b * a.Ctot + c) * 2 + 0] = sc;
        a.ss[(b * a.Ctot + c) * 2 + 1] = a.beta[c] - meanf * sc;
    }
}

__device__ __forceinline__ float silu_f(float x) { return x / (1.0f + expf(-x)); }

// ---------------------------------------------------------------------------
// K1/K2: implicit-GEMM convolution.  GEMM view: M = B*Hout*Wout output pixels,
// N = Cout, K = ks*ks*Ctot ordered (tap, channel).  Workgroup tile BM x BN x 16,
// 4 waves as 2x2, each wave (BM/2)x(BN/2) built from 16x16 fp32 MFMA tiles.
// LDS tiles are [row][16 + 4 pad]; lane (g = lane>>4, i = lane&15) reads one
// ds_read_b128 per operand per 4 MFMA k-steps, with physical k = 4g + s.
// ---------------------------------------------------------------------------
template <int BM, int BN>
__global__ __launch_bounds__(256) void conv_gemm_kernel(ConvArgs a) {
    constexpr int LDK = 20;
    constexpr int TM = BM / 32, TN = BN / 32;
    constexpr int AIT = BM / 64, BIT = BN / 64;
    __shared__ __attribute__((aligned(16))) float As[2][BM * LDK];
    __shared__ __attribute__((aligned(16))) float Bs[2][BN * LDK];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
    const int HWo = a.Hout * a.Wout;
    const int kq = tid & 3;

    // per-thread A rows (fixed over the K loop)
    int a_b[AIT], a_oy[AIT], a_ox[AIT];
    bool a_ok[AIT];
#pragma unroll
    for (int it = 0; it < AIT; ++it) {
        const int m = m0 + (tid >> 2) + it * 64;
        a_ok[it] = m < a.M;
        const int mm = a_ok[it] ? m : 0;
        a_b[it] = mm / HWo;
        const int rem = mm - a_b[it] * HWo;
        a_oy[it] = rem / a.Wout;
        a_ox[it] = rem - a_oy[it] * a.Wout;
    }
    const int nK = a.K / 16;

    f4 ra[AIT], rb[BIT];
    auto load_tile = [&](int kt) {
        const int kbase = kt * 16;
        const int tap = kbase / a.Ctot;
        const int c0 = kbase - tap * a.Ctot + 4 * kq;
        const int dy = tap / a.ks, dx = tap - (tap / a.ks) * a.ks;
#pragma unroll
        for (int it = 0; it < AIT; ++it) {
            f4 v = {0.f, 0.f, 0.f, 0.f};
            int iy, ix;
            bool ok = a_ok[it];
            if (a.up) {
                const int iyu = a_oy[it] + dy - a.pad, ixu = a_ox[it] + dx - a.pad;
                ok = ok && iyu >= 0 && iyu < 2 * a.Hin && ixu >= 0 && ixu < 2 * a.Win;
                iy = iyu >> 1;
                ix = ixu >> 1;
            } else {
                iy = a_oy[it] * a.stride + dy - a.pad;
                ix = a_ox[it] * a.stride + dx - a.pad;
                ok = ok && iy >= 0 && iy < a.Hin && ix >= 0 && ix < a.Win;
            }
            if (ok) {
                const int64_t pix = ((int64_t)a_b[it] * a.Hin + iy) * a.Win + ix;
                v = c0 < a.C1 ? *(const f4*)(a.src1 + pix * a.C1 + c0)
                              : *(const f4*)(a.src2 + pix * a.C2 + (c0 - a.C1));
                if (a.act) {
                    const float* ss = a.ss + ((int64_t)a_b[it] * a.Ctot + c0) * 2;
                    const f4 s01 = *(const f4*)ss, s23 = *(const f4*)(ss + 4);
                    v[0] = v[0] * s01[0] + s01[1];
                    v[1] = v[1] * s01[2] + s01[3];
                    v[2] = v[2] * s23[0] + s23[1];
                    v[3] = v[3] * s23[2] + s23[3];
                    if (a.act == 2) {
#pragma unroll
                        for (int j = 0; j < 4; ++j) v[j] = silu_f(v[j]);
                    }
                }
            }
            ra[it] = v;
        }
#pragma unroll
        for (int it = 0; it < BIT; ++it) {
            const int n = n0 + (tid >> 2) + it * 64;
            rb[it] = n < a.Cout ? *(const f4*)(a.w + (int64_t)n * a.K + kbase + 4 * kq) : f4{0.f, 0.f, 0.f, 0.f};
        }
    };
    auto store_tile = [&](int buf) {
#pragma unroll
        for (int it = 0; it < AIT; ++it) *(f4*)(&As[buf][((tid >> 2) + it * 64) * LDK + 4 * kq]) = ra[it];
#pragma unroll
        for (int it = 0; it < BIT; ++it) *(f4*)(&Bs[buf][((tid >> 2) + it * 64) * LDK + 4 * kq]) = rb[it];
    };

    f4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

    load_tile(0);
    store_tile(0);
    __syncthreads();
    const int g4 = 4 * (lane >> 4), li = lane & 15;
    for (int kt = 0; kt < nK; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nK) load_tile(kt + 1);
        f4 fa[TM], fb[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[i] = *(const f4*)(&As[cur][(wm * (BM / 2) + 16 * i + li) * LDK + g4]);
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[j] = *(const f4*)(&Bs[cur][(wn * (BN / 2) + 16 * j + li) * LDK + g4]);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i][s], fb[j][s], acc[i][j], 0, 0, 0);
        if (kt + 1 < nK) store_tile(cur ^ 1);
        __syncthreads();
    }

    // epilogue: + bias (+ emb[b, n]) then residual + h
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = m0 + wm * (BM / 2) + 16 * i + g4 + r;
            if (m >= a.M) continue;
            const int bb = m / HWo;
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int n = n0 + wn * (BN / 2) + 16 * j + li;
                if (n >= a.Cout) continue;
                float v = acc[i][j][r] + a.bias[n];
                if (a.emb) v = v + a.emb[(int64_t)bb * a.emb_stride + n];
                if (a.res) v = a.res[(int64_t)m * a.Cout + n] + v;
                a.out[(int64_t)m * a.Cout + n] = v;
            }
        }
    }
}

// First convolution, in_channels (<= 4) -> Cout, 3x3 pad 1: VALU, one output per thread.
__global__ void conv_in_kernel(ConvArgs a) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (int64_t)a.M * a.Cout) return;
    const int n = (int)(idx % a.Cout);
    const int m = (int)(idx / a.Cout);
    const int HW = a.Hout * a.Wout;
    const int b = m / HW, rem = m - b * HW, oy = rem / a.Wout, ox = rem - oy * a.Wout;
    float s = 0.f;
    for (int tap = 0; tap < 9; ++tap) {
        const int iy = oy + tap / 3 - 1, ix = ox + tap % 3 - 1;
        if (iy < 0 || iy >= a.Hin || ix < 0 || ix >= a.Win) continue;
        const float* px = a.src1 + (((int64_t)b * a.Hin + iy) * a.Win + ix) * a.C1;
        for (int c = 0; c < a.C1; ++c) s = fmaf(a.w[((int64_t)n * 9 + tap) * a.C1 + c], px[c], s);
    }
    a.out[idx] = s + a.bias[n];
}

// Last convolution: GN+SiLU prologue, Ctot -> Cout (<= 4), 3x3 pad 1.  One wave
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
        const int iy = oy + tap / 3 - 1, ix = ox + tap % 3 - 1;
        if (iy < 0 || iy >= a.Hin || ix < 0 || ix >= a.Win) continue;
        float v = a.src1[(((int64_t)b * a.Hin + iy) * a.Win + ix) * a.C1 + c];
        const float* ss = a.ss + ((int64_t)b * a.Ctot + c) * 2;
        v = silu_f(v * ss[0] + ss[1]);
        for (int n = 0; n < a.Cout; ++n) s[n] = fmaf(a.w[(int64_t)n * a.K + k], v, s[n]);
    }
    for (int n = 0; n < a.Cout; ++n) {
        float v = s[n];
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        if (lane == 0) a.out[m * a.Cout + n] = v + a.bias[n];
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
__global__ void linear_kernel(const float* __restrict__ x, const float* __restrict__ W, const float* __restrict__ bias,
                              float* __restrict__ y, int B, int K, int N, int act) {
    const int lane = threadIdx.x & 63;
    const int n = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (n >= N) return;
    const float* wr = W + (int64_t)n * K;
    for (int b = 0; b < B; ++b) {
        const float* xb = x + (int64_t)b * K;
        float s = 0.f;
        for (int k = lane; k < K; k += 64) {
            const float v = act ? silu_f(xb[k]) : xb[k];
            s = fmaf(wr[k], v, s);
        }
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
        if (lane == 0) y[(int64_t)b * N + n] = s + bias[n];
    }
}

// ---------------------------------------------------------------------------
// host-side launchers
// ---------------------------------------------------------------------------
void launch_gn_stats(const GnArgs& a, int B, hipStream_t st) {
    CFD_REQUIRE(a.Ctot % 32 == 0, CFD_ESHAPE, "GroupNorm32 needs channels % 32 == 0");
    hipLaunchKernelGGL(gn_stats_kernel, dim3(32, B), dim3(256), 0, st, a);
    check_launch("gn_stats_kernel");
}

void launch_conv(const ConvArgs& a, hipStream_t st) {
    CFD_REQUIRE(a.Ctot % 16 == 0 && a.C1 % 4 == 0 && a.C2 % 4 == 0, CFD_ESHAPE, "conv_gemm needs channels % 16 == 0");
    CFD_REQUIRE(a.K == a.ks * a.ks * a.Ctot, CFD_ESHAPE, "conv K mismatch");
    const int64_t t128 = ceil_div(a.M, 128) * ceil_div(a.Cout, 128);
    if (t128 >= 256 && a.Cout % 128 == 0) {
        hipLaunchKernelGGL((conv_gemm_kernel<128, 128>), dim3((unsigned)ceil_div(a.M, 128), (unsigned)ceil_div(a.Cout, 128)),
                           dim3(256), 0, st, a);
    } else {
        hipLaunchKernelGGL((conv_gemm_kernel<64, 64>), dim3((unsigned)ceil_div(a.M, 64), (unsigned)ceil_div(a.Cout, 64)),
                           dim3(256), 0, st, a);
    }
    check_launch("conv_gemm_kernel");
}

void launch_conv_in(const ConvArgs& a, hipStream_t st) {
    const int64_t n = (int64_t)a.M * a.Cout;
    hipLaunchKernelGGL(conv_in_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, st, a);
    check_launch("conv_in_kernel");
}

void launch_conv_out(const ConvArgs& a, hipStream_t st) {
    CFD_REQUIRE(a.Cout <= 4, CFD_ESHAPE, "out_channels must be <= 4");
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

void launch_temb(const int64_t* t, const float* freqs, float* out, int dim, int B, hipStream_t st) {
    hipLaunchKernelGGL(temb_kernel, dim3(B), dim3(128), 0, st, t, freqs, out, dim);
    check_launch("temb_kernel");
}

void launch_linear(const float* x, const float* W, const float* bias, float* y, int B, int K, int N, int act,
                   hipStream_t st) {
    hipLaunchKernelGGL(linear_kernel, dim3((unsigned)ceil_div(N, 4)), dim3(256), 0, st, x, W, bias, y, B, K, N, act);
    check_launch("linear_kernel");
}

}  // namespace cfd
