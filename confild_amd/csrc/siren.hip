// Fused SIREN/FiLM conditional-neural-field decoder for gfx950 (K7).
//
// Replaces, per (coordinate, latent) pair, the reference chain
//   Normalizer_ts.normalize(coords)                (N/cnf/utils/normalize.py:100-103)
//   for i < nh+1: x = sin(w0 * (W_i x + b_i + V_i z))  (N/cnf/nf_networks.py:480-495,
//                                                    components.py:19-25,64-76)
//   out = W_last x + b_last
//   Normalizer_ts.denormalize(out)                 (normalize.py:112-114)
// with one launch.  Design (DESIGN.md "K7"):
//   * workgroup = 4 waves x 16 coordinates, one latent (grid.y);
//   * activations never leave registers: each wave holds its 16 coordinates'
//     hidden vector as NB = H/16 fragments of the fp32 MFMA 16x16x4 layout
//     (lane = coord + 16*g, 4 features per fragment).  The accumulator layout of
//     one layer IS the B-operand layout of the next (k order 16q + 4g + s), so
//     no LDS round trip or shuffle between layers;
//   * hidden weights stream through a 2-slot LDS ring by LDS-DMA
//     (global_load_lds_dwordx4, 1 KiB per wave-instruction) from a pre-packed
//     image whose lane-linear order is exactly the A-fragment order, read back
//     with one ds_read_b128 per 4 MFMAs;
//   * the per-latent FiLM vectors F_i = b_i + V_i z (all layers) are computed by
//     siren_film and staged in LDS; they initialise each accumulator;
//   * sin(w0*x) uses a Cody-Waite reduced polynomial (common.hpp sin_cw);
//   * the last (H -> c) layer, the bias and the per-point de-normalisation are
//     fused into the store.
#include <cstdlib>
#include <cstring>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

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

// coordinates per workgroup = 16 * waves (4 waves: 2 workgroups per CU; 8 waves:
// one workgroup per CU, each LDS-DMA'd weight block shared by 128 coordinates)

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
    int64_t N;
    int64_t ystride;
    int64_t b0;           // first latent of this launch (grid.y chunking)
    int d, c, nh;
    float w0f;
};

template <int NB, int WAVES>
__device__ __forceinline__ void siren_issue_block(const float* __restrict__ wimg, int J, float* dst,
                                                  int wave, int lane) {
    constexpr int BLK = NB * 256;
    const float* src = wimg + (int64_t)J * BLK;
    for (int piece = wave; piece < NB; piece += WAVES) {
        __builtin_amdgcn_global_load_lds((const void*)(src + piece * 256 + lane * 4),
                                         (__attribute__((address_space(3))) void*)(dst + piece * 256),
                                         16, 0, 0);
    }
}

// DUAL = false: one accumulation chain per 16-row block, 2 workgroups per CU
//              (256 VGPRs: the partner workgroup hides the MFMA dependency);
// DUAL = true : two interleaved chains, 1 workgroup per CU (512 VGPRs).
template <int NB, bool DUAL, int WAVES>
// 2 waves per SIMD (256 VGPRs each) in both geometries; dual / NB 32: 1 wave per SIMD
__global__ __launch_bounds__(64 * WAVES, (NB <= 24 && !DUAL) ? 2 : 1) void siren_fused(SirenArgs p) {
    constexpr int TILE = 16 * WAVES;
    constexpr int H = NB * 16;
    constexpr int BLK = NB * 256;  // floats in one 16-row weight block image
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* wbuf = smem;            // 2 slots
    float* film = smem + 2 * BLK;  // (nh+1) x H, then w0 as (H, 4)

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int g = lane >> 4;
    const int j16 = lane & 15;
    const int64_t b = p.b0 + blockIdx.y;
    const int64_t n = (int64_t)blockIdx.x * TILE + wave * 16 + j16;
    const int64_t nc = n < p.N ? n : p.N - 1;
    const int nh = p.nh;

    // ---- stage this latent's FiLM rows (no LDS-DMA in flight yet) ----
    {
        const float* fsrc = p.film + b * (int64_t)(nh + 1) * H;
        const int nf = (nh + 1) * H;
        for (int i = threadIdx.x * 4; i < nf; i += 64 * WAVES * 4) *(f4*)(film + i) = *(const f4*)(fsrc + i);
    }
    // ---- layer-0 inputs: normalised coordinates; (H, d) weight staged as (H, 4) ----
    float* w0s = film + (nh + 1) * H;
    for (int f = threadIdx.x; f < H; f += 64 * WAVES) {
        f4 w = {0.f, 0.f, 0.f, 0.f};
        for (int k = 0; k < p.d; ++k) w[k] = p.w0[f * p.d + k];
        *(f4*)(w0s + 4 * f) = w;
    }
    float cn[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (k < p.d) {
            float v = p.coords[nc * p.d + k];
            if (p.xmax) v = (v - p.xmin[k]) / (p.xmax[k] - p.xmin[k]) * 2.0f - 1.0f;
            cn[k] = v;
        }
    }

    __syncthreads();  // film + w0 visible; every ordinary global load above has been consumed
    if (nh > 0) siren_issue_block<NB, WAVES>(p.wimg, 0, wbuf, wave, lane);

    // ---- layer 0: x = sin(w0 * (W0 c + F_0)) ----
    float X[NB][4];
    auto layer0_arg = [&](int q, int r) -> float {
        const f4 fv = *(const f4*)(film + 16 * q + 4 * g);
        const f4 w = *(const f4*)(w0s + 4 * (16 * q + 4 * g + r));
        float a = cn[0] * w[0];
#pragma unroll
        for (int k = 1; k < 4; ++k)
            if (k < p.d) a = fmaf(cn[k], w[k], a);
        return p.w0f * (a + fv[r]);
    };
    static_for<NB>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
#pragma unroll
        for (int r = 0; r < 4; ++r) X[q][r] = sin_cw(layer0_arg(q, r));
    });

    // ---- hidden layers on fp32 MFMA 16x16x4 ----
    const int nblocks = nh * NB;
    int J = 0;
    for (int layer = 1; layer <= nh; ++layer) {
        f4 acc[NB];
        static_for<NB>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            if (J + 1 < nblocks) siren_issue_block<NB, WAVES>(p.wimg, J + 1, wbuf + ((J + 1) & 1) * BLK, wave, lane);
            const float* wb = wbuf + (J & 1) * BLK;
            // two interleaved accumulation chains (even / odd k-steps): the f32
            // 16x16x4 MFMA has a 40-cycle dependent latency vs a 32-cycle issue
            f4 a = *(const f4*)(film + layer * H + 16 * j + 4 * g);
            if constexpr (DUAL) {
                f4 a2 = {0.f, 0.f, 0.f, 0.f};
                static_for<NB>([&](auto qc) {
                    constexpr int q = decltype(qc)::value;
                    const f4 w = *(const f4*)(wb + (q * 64 + lane) * 4);
                    a = __builtin_amdgcn_mfma_f32_16x16x4f32(w.x, X[q][0], a, 0, 0, 0);
                    a2 = __builtin_amdgcn_mfma_f32_16x16x4f32(w.y, X[q][1], a2, 0, 0, 0);
                    a = __builtin_amdgcn_mfma_f32_16x16x4f32(w.z, X[q][2], a, 0, 0, 0);
                    a2 = __builtin_amdgcn_mfma_f32_16x16x4f32(w.w, X[q][3], a2, 0, 0, 0);
                });
                acc[j] = a + a2;
            } else {
                static_for<NB>([&](auto qc) {
                    constexpr int q = decltype(qc)::value;
                    const f4 w = *(const f4*)(wb + (q * 64 + lane) * 4);
                    a = __builtin_amdgcn_mfma_f32_16x16x4f32(w.x, X[q][0], a, 0, 0, 0);
                    a = __builtin_amdgcn_mfma_f32_16x16x4f32(w.y, X[q][1], a, 0, 0, 0);
                    a = __builtin_amdgcn_mfma_f32_16x16x4f32(w.z, X[q][2], a, 0, 0, 0);
                    a = __builtin_amdgcn_mfma_f32_16x16x4f32(w.w, X[q][3], a, 0, 0, 0);
                });
                acc[j] = a;
            }
            // block J+1 landed (this wave's pieces) -> barrier makes every wave's
            // pieces visible and retires all reads of slot J&1 before it is refilled.
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            ++J;
        });
        static_for<NB>([&](auto qc) {
            constexpr int q = decltype(qc)::value;
#pragma unroll
            for (int r = 0; r < 4; ++r) X[q][r] = sin_cw(p.w0f * acc[q][r]);
        });
    }

    // ---- last layer (H -> c) + bias + de-normalisation ----
    float o[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int oc = 0; oc < 4; ++oc) {
        if (oc < p.c) {
            const float* wr = p.wout + oc * H + 4 * g;
            float s = 0.f;
            static_for<NB>([&](auto qc) {
                constexpr int q = decltype(qc)::value;
                const f4 w = *(const f4*)(wr + 16 * q);
                s = fmaf(w.x, X[q][0], s);
                s = fmaf(w.y, X[q][1], s);
                s = fmaf(w.z, X[q][2], s);
                s = fmaf(w.w, X[q][3], s);
            });
            s += __shfl_xor(s, 16);
            s += __shfl_xor(s, 32);
            o[oc] = s + p.bout[oc];
        }
    }
    if (n < p.N && g < p.c) {
        float v = g == 0 ? o[0] : g == 1 ? o[1] : g == 2 ? o[2] : o[3];
        if (p.ymax) {
            const int64_t yi = n * p.ystride + g;
            const float hi = p.ymax[yi], lo = p.ymin[yi];
            v = (v + 1.0f) / 2.0f * (hi - lo) + lo;
        }
        p.out[(b * p.N + n) * p.c + g] = v;
    }
}

// F[b][i][f] = b_i[f] + sum_l V_i[f][l] z[b][l]   (net1[i].bias + net2[i](z))
__global__ void siren_film(const float* __restrict__ V, const float* __restrict__ bias,
                           const float* __restrict__ z, float* __restrict__ F, int H, int L, int nl) {
    const int i = blockIdx.x;   // layer
    const int64_t b = blockIdx.y;
    const float* zb = z + b * L;
    for (int f = threadIdx.x; f < H; f += blockDim.x) {
        const float* vr = V + ((int64_t)i * H + f) * L;
        float s = 0.f;
        for (int l = 0; l < L; ++l) s = fmaf(vr[l], zb[l], s);
        F[(b * nl + i) * H + f] = bias[i * H + f] + s;
    }
}

// ---------------------------------------------------------------------------
// Input-gradient (DPS adjoint): d<g, A(z)>/dz for the
// Case4 measurement operator A = y_norm.denormalize(SIREN(x_norm(sensors), z))
// (measurements.py:219-226).  One workgroup per latent row z, all sensors of the
// row in groups of VJP_SG; thread j owns hidden feature j.  Sensor counts are
// small (10 in the Case4 notebook), so this is VALU work on L2-resident weights:
//   siren_tape_fwd  u_i = W_i x_i + F_i kept for every layer (the tape), x_{i+1} =
//                   sin(w0 u_i); outputs A (coalesced W^T reads, x broadcast from LDS);
//   siren_tape_vjp  delta_i = (W_{i+1}^T delta_{i+1}) * w0 cos(w0 u_i), summed over
//                   sensors per layer, then g_z = sum_i V_i^T (sum_s delta_i).
// ---------------------------------------------------------------------------
constexpr int VJP_SG = 8;

struct SirenVjpArgs {
    const float* w0;     // (H, d)
    const float* wtr;    // (nh, H, H) hidden weights transposed: wtr[i][k][j] = W_{i+1}[j][k]
    const float* wraw;   // (nh, H, H) hidden weights as stored: W_{i+1}[j][k]
    const float* wout;   // (c, H)
    const float* bout;   // (c)
    const float* V;      // (nh+1, H, L)
    const float* film;   // (R, nh+1, H)
    const float* coords; // (Ns, d) raw sensor coordinates
    const float* xmax;
    const float* xmin;
    const float* ymax;
    const float* ymin;
    float* pre;          // (R, Ns, nh+1, H) tape
    float* out;          // (R, Ns, c)  forward output A
    const float* gout;   // (R, Ns, c)  gradient w.r.t. A
    float* gz;           // (R, L)
    int64_t ystride;
    int Ns, d, c, nh, H, L;
    float w0f;
};

__global__ __launch_bounds__(512) void siren_tape_fwd(SirenVjpArgs p) {
    extern __shared__ __attribute__((aligned(16))) float xs[];  // VJP_SG x H
    const int64_t r = blockIdx.x;
    const int j = threadIdx.x;
    const int H = p.H, nl = p.nh + 1;
    const float* film = p.film + r * nl * H;
    for (int s0 = 0; s0 < p.Ns; s0 += VJP_SG) {
        const int ns = min(VJP_SG, p.Ns - s0);
        float* pre = p.pre + ((r * p.Ns + s0) * nl) * (int64_t)H;
        if (j < H) {
            const float f0 = film[j];
#pragma unroll
            for (int s = 0; s < VJP_SG; ++s) {
                if (s < ns) {
                    float a = 0.f;
                    for (int k = 0; k < p.d; ++k) {
                        float v = p.coords[(int64_t)(s0 + s) * p.d + k];
                        if (p.xmax) v = (v - p.xmin[k]) / (p.xmax[k] - p.xmin[k]) * 2.0f - 1.0f;
                        a = k == 0 ? v * p.w0[j * p.d] : fmaf(v, p.w0[j * p.d + k], a);
                    }
                    const float u = a + f0;
                    pre[(int64_t)s * nl * H + j] = u;
                    xs[s * H + j] = sin_cw(p.w0f * u);
                }
            }
        }
        __syncthreads();
        for (int i = 1; i <= p.nh; ++i) {
            float acc[VJP_SG];
            if (j < H) {
                const float fi = film[i * H + j];
#pragma unroll
                for (int s = 0; s < VJP_SG; ++s) acc[s] = fi;
                const float* wt = p.wtr + (int64_t)(i - 1) * H * H + j;
                for (int k = 0; k < H; ++k) {
                    const float w = wt[(int64_t)k * H];
#pragma unroll
                    for (int s = 0; s < VJP_SG; ++s)
                        if (s < ns) acc[s] = fmaf(w, xs[s * H + k], acc[s]);
                }
            }
            __syncthreads();
            if (j < H) {
#pragma unroll
                for (int s = 0; s < VJP_SG; ++s) {
                    if (s < ns) {
                        pre[((int64_t)s * nl + i) * H + j] = acc[s];
                        xs[s * H + j] = sin_cw(p.w0f * acc[s]);
                    }
                }
            }
            __syncthreads();
        }
        if (j < ns * p.c) {
            const int s = j / p.c, oc = j - s * p.c;
            float o = 0.f;
            for (int k = 0; k < H; ++k) o = fmaf(p.wout[oc * H + k], xs[s * H + k], o);
            o += p.bout[oc];
            if (p.ymax) {
                const int64_t yi = (int64_t)(s0 + s) * p.ystride + oc;
                o = (o + 1.0f) / 2.0f * (p.ymax[yi] - p.ymin[yi]) + p.ymin[yi];
            }
            p.out[(r * p.Ns + s0 + s) * p.c + oc] = o;
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(512) void siren_tape_vjp(SirenVjpArgs p) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int64_t r = blockIdx.x;
    const int j = threadIdx.x;
    const int H = p.H, nl = p.nh + 1;
    float* dl = sm;                   // VJP_SG x H: this layer's deltas
    float* dacc = sm + VJP_SG * H;    // nl x H: deltas summed over sensors
    for (int i = j; i < nl * H; i += blockDim.x) dacc[i] = 0.f;
    for (int s0 = 0; s0 < p.Ns; s0 += VJP_SG) {
        const int ns = min(VJP_SG, p.Ns - s0);
        const float* pre = p.pre + ((r * p.Ns + s0) * nl) * (int64_t)H;
        // gradient w.r.t. the last hidden activation: W_out^T (g * dA/dout)
        float gx[VJP_SG];
#pragma unroll
        for (int s = 0; s < VJP_SG; ++s) gx[s] = 0.f;
        if (j < H) {
#pragma unroll
            for (int s = 0; s < VJP_SG; ++s) {
                if (s < ns) {
                    float a = 0.f;
                    for (int oc = 0; oc < p.c; ++oc) {
                        float gy = p.gout[(r * p.Ns + s0 + s) * p.c + oc];
                        if (p.ymax) {
                            const int64_t yi = (int64_t)(s0 + s) * p.ystride + oc;
                            gy = gy * ((p.ymax[yi] - p.ymin[yi]) / 2.0f);
                        }
                        a = fmaf(p.wout[oc * H + j], gy, a);
                    }
                    gx[s] = a;
                }
            }
        }
        for (int i = p.nh; i >= 0; --i) {
            if (j < H) {
                float sum = 0.f;
#pragma unroll
                for (int s = 0; s < VJP_SG; ++s) {
                    if (s < ns) {
                        const float u = pre[((int64_t)s * nl + i) * H + j];
                        const float dlt = gx[s] * (p.w0f * cosf(p.w0f * u));
                        dl[s * H + j] = dlt;
                        sum += dlt;
                    }
                }
                dacc[i * H + j] += sum;
            }
            __syncthreads();
            if (i > 0 && j < H) {
                // gx = W_i^T delta_i  (W_i = hidden layer i, stored at slot i-1)
#pragma unroll
                for (int s = 0; s < VJP_SG; ++s) gx[s] = 0.f;
                const float* w = p.wraw + (int64_t)(i - 1) * H * H + j;
                for (int k = 0; k < H; ++k) {
                    const float wv = w[(int64_t)k * H];
#pragma unroll
                    for (int s = 0; s < VJP_SG; ++s)
                        if (s < ns) gx[s] = fmaf(wv, dl[s * H + k], gx[s]);
                }
            }
            __syncthreads();
        }
    }
    // g_z[l] = sum_i sum_f V_i[f][l] dacc[i][f]
    for (int l = j; l < p.L; l += blockDim.x) {
        float a = 0.f;
        for (int i = 0; i < nl; ++i) {
            const float* v = p.V + (int64_t)i * H * p.L + l;
            for (int f = 0; f < H; ++f) a = fmaf(v[(int64_t)f * p.L], dacc[i * H + f], a);
        }
        p.gz[r * p.L + l] = a;
    }
}

// ---------------------------------------------------------------------------
// handle
// ---------------------------------------------------------------------------
struct SirenParam {
    std::string key;
    std::vector<int64_t> shape;
    bool set = false;
};

}  // namespace cfd

struct cfd_siren {
    cfd_siren_cfg cfg;
    int device = 0;
    int NB = 0;
    std::vector<cfd::SirenParam> params;
    float* w0 = nullptr;    // (H, d)
    float* fbias = nullptr; // (nh+1, H)
    float* V = nullptr;     // (nh+1, H, L)
    float* wimg = nullptr;  // nh * NB * NB*256
    float* wout = nullptr;  // (c, H)
    float* bout = nullptr;  // (c)
    float* wraw = nullptr;  // (nh, H, H) hidden weights (input-gradient path)
    float* wtr = nullptr;   // (nh, H, H) hidden weights transposed
};

namespace {

int siren_variant() {
    static int v = [] {
        const char* e = getenv("CFD_SIREN_VARIANT");
        return e ? atoi(e) : 2;
    }();
    return v;
}

template <int NB>
void launch_siren_nb(const cfd_siren* h, cfd::SirenArgs a, int b, hipStream_t st) {
    const int H = NB * 16;
    const size_t lds = (size_t)(2 * NB * 256 + (h->cfg.num_hidden_layers + 1) * H + 4 * H) * sizeof(float);
    const int v = siren_variant();  // 2 (default): 8 waves/WG, 0: 4 waves/WG, 1: dual chain
    const void* fn = v == 1 ? (const void*)cfd::siren_fused<NB, true, 4>
                   : v == 2 ? (const void*)cfd::siren_fused<NB, false, 8>
                            : (const void*)cfd::siren_fused<NB, false, 4>;
    CFD_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const int waves = v == 2 ? 8 : 4;
    const int64_t tiles = cfd::ceil_div(a.N, 16 * waves);
    for (int64_t b0 = 0; b0 < b; b0 += 65535) {
        a.b0 = b0;
        const int nb = (int)std::min<int64_t>(65535, b - b0);
        const dim3 grid((unsigned)tiles, nb);
        if (v == 1)
            hipLaunchKernelGGL((cfd::siren_fused<NB, true, 4>), grid, dim3(256), lds, st, a);
        else if (v == 2)
            hipLaunchKernelGGL((cfd::siren_fused<NB, false, 8>), grid, dim3(512), lds, st, a);
        else
            hipLaunchKernelGGL((cfd::siren_fused<NB, false, 4>), grid, dim3(256), lds, st, a);
        cfd::check_launch("siren_fused");
    }
}

void launch_siren(const cfd_siren* h, const cfd::SirenArgs& a, int b, hipStream_t st) {
    switch (h->NB) {
        case 1: return launch_siren_nb<1>(h, a, b, st);
        case 2: return launch_siren_nb<2>(h, a, b, st);
        case 3: return launch_siren_nb<3>(h, a, b, st);
        case 4: return launch_siren_nb<4>(h, a, b, st);
        case 6: return launch_siren_nb<6>(h, a, b, st);
        case 8: return launch_siren_nb<8>(h, a, b, st);
        case 12: return launch_siren_nb<12>(h, a, b, st);
        case 16: return launch_siren_nb<16>(h, a, b, st);
        case 24: return launch_siren_nb<24>(h, a, b, st);
        case 32: return launch_siren_nb<32>(h, a, b, st);
        default: throw cfd::Error{CFD_EARG, "hidden_features must be 16*{1,2,3,4,6,8,12,16,24,32}"};
    }
}

}  // namespace

extern "C" int cfd_siren_create(const cfd_siren_cfg* cfg, int device, cfd_siren** out) {
    return cfd::guard([&] {
        CFD_REQUIRE(cfg && out, CFD_EARG, "null argument");
        const int d = cfg->in_coord_features, L = cfg->in_latent_features, c = cfg->out_features;
        const int nh = cfg->num_hidden_layers, H = cfg->hidden_features;
        CFD_REQUIRE(d >= 1 && d <= 4, CFD_EARG, "in_coord_features must be 1..4");
        CFD_REQUIRE(c >= 1 && c <= 4, CFD_EARG, "out_features must be 1..4");
        CFD_REQUIRE(L >= 1 && nh >= 0 && H % 16 == 0 && H >= 16 && H <= 512, CFD_EARG,
                    "hidden_features must be a multiple of 16 in [16, 512]");
        const int NB = H / 16;
        CFD_REQUIRE(NB == 1 || NB == 2 || NB == 3 || NB == 4 || NB == 6 || NB == 8 || NB == 12 || NB == 16 ||
                        NB == 24 || NB == 32,
                    CFD_EARG, "hidden_features must be 16*{1,2,3,4,6,8,12,16,24,32}");
        CFD_HIP(hipSetDevice(device));
        auto* h = new cfd_siren();
        h->cfg = *cfg;
        if (h->cfg.w0 == 0.f) h->cfg.w0 = 30.f;
        h->device = device;
        h->NB = NB;
        for (int i = 0; i < nh + 2; ++i) {
            const int fin = i == 0 ? d : H, fout = i == nh + 1 ? c : H;
            h->params.push_back({"net1." + std::to_string(i) + ".weight", {fout, fin}});
            h->params.push_back({"net1." + std::to_string(i) + ".bias", {fout}});
        }
        for (int i = 0; i < nh + 1; ++i) h->params.push_back({"net2." + std::to_string(i) + ".weight", {H, L}});
        CFD_HIP(hipMalloc(&h->w0, sizeof(float) * H * d));
        CFD_HIP(hipMalloc(&h->fbias, sizeof(float) * (nh + 1) * H));
        CFD_HIP(hipMalloc(&h->V, sizeof(float) * (size_t)(nh + 1) * H * L));
        CFD_HIP(hipMalloc(&h->wimg, sizeof(float) * (size_t)std::max(nh, 1) * NB * NB * 256));
        CFD_HIP(hipMalloc(&h->wout, sizeof(float) * c * H));
        CFD_HIP(hipMalloc(&h->bout, sizeof(float) * 4));
        CFD_HIP(hipMalloc(&h->wraw, sizeof(float) * (size_t)std::max(nh, 1) * H * H));
        CFD_HIP(hipMalloc(&h->wtr, sizeof(float) * (size_t)std::max(nh, 1) * H * H));
        *out = h;
    });
}

extern "C" void cfd_siren_destroy(cfd_siren* h) {
    if (!h) return;
    (void)hipFree(h->w0);
    (void)hipFree(h->fbias);
    (void)hipFree(h->V);
    (void)hipFree(h->wimg);
    (void)hipFree(h->wout);
    (void)hipFree(h->bout);
    (void)hipFree(h->wraw);
    (void)hipFree(h->wtr);
    delete h;
}

extern "C" int cfd_siren_num_params(const cfd_siren* h, int* n) {
    return cfd::guard([&] {
        CFD_REQUIRE(h && n, CFD_EARG, "null argument");
        *n = (int)h->params.size();
    });
}

extern "C" int cfd_siren_param_info(const cfd_siren* h, int idx, const char** key, int* ndim, int64_t shape[4]) {
    return cfd::guard([&] {
        CFD_REQUIRE(h && idx >= 0 && idx < (int)h->params.size(), CFD_EARG, "bad index");
        const auto& p = h->params[idx];
        if (key) *key = p.key.c_str();
        if (ndim) *ndim = (int)p.shape.size();
        if (shape)
            for (size_t i = 0; i < p.shape.size(); ++i) shape[i] = p.shape[i];
    });
}

extern "C" int cfd_siren_set_param(cfd_siren* h, const char* key, const float* host, size_t n) {
    return cfd::guard([&] {
        CFD_REQUIRE(h && key && host, CFD_EARG, "null argument");
        CFD_HIP(hipSetDevice(h->device));
        const std::string k(key);
        cfd::SirenParam* prm = nullptr;
        for (auto& p : h->params)
            if (p.key == k) prm = &p;
        CFD_REQUIRE(prm, CFD_EKEY, "unknown SIREN parameter key: " + k);
        size_t want = 1;
        for (auto s : prm->shape) want *= (size_t)s;
        CFD_REQUIRE(n == want, CFD_ESHAPE, "size mismatch for " + k);
        const int d = h->cfg.in_coord_features, L = h->cfg.in_latent_features, c = h->cfg.out_features;
        const int nh = h->cfg.num_hidden_layers, H = h->cfg.hidden_features, NB = h->NB;
        const bool is_w = k.size() > 7 && k.compare(k.size() - 7, 7, ".weight") == 0;
        const int li = std::stoi(k.substr(5, k.find('.', 5) - 5));
        if (k.rfind("net2.", 0) == 0) {
            CFD_HIP(hipMemcpy(h->V + (size_t)li * H * L, host, n * 4, hipMemcpyHostToDevice));
        } else if (li == nh + 1) {
            CFD_HIP(hipMemcpy(is_w ? h->wout : h->bout, host, n * 4, hipMemcpyHostToDevice));
        } else if (!is_w) {
            CFD_HIP(hipMemcpy(h->fbias + (size_t)li * H, host, n * 4, hipMemcpyHostToDevice));
        } else if (li == 0) {
            CFD_HIP(hipMemcpy(h->w0, host, n * 4, hipMemcpyHostToDevice));
            (void)d;
        } else {
            // pack W_li (H,H) into NB blocks of the A-fragment image:
            // img[j][q][lane][s] = W[16j + (lane&15)][16q + 4(lane>>4) + s]
            std::vector<float> img((size_t)NB * NB * 256);
            for (int j = 0; j < NB; ++j)
                for (int q = 0; q < NB; ++q)
                    for (int lane = 0; lane < 64; ++lane)
                        for (int s = 0; s < 4; ++s)
                            img[(((size_t)j * NB + q) * 64 + lane) * 4 + s] =
                                host[(size_t)(16 * j + (lane & 15)) * H + 16 * q + 4 * (lane >> 4) + s];
            CFD_HIP(hipMemcpy(h->wimg + (size_t)(li - 1) * NB * NB * 256, img.data(), img.size() * 4,
                              hipMemcpyHostToDevice));
            std::vector<float> tr((size_t)H * H);
            for (int a = 0; a < H; ++a)
                for (int bb = 0; bb < H; ++bb) tr[(size_t)bb * H + a] = host[(size_t)a * H + bb];
            CFD_HIP(hipMemcpy(h->wraw + (size_t)(li - 1) * H * H, host, n * 4, hipMemcpyHostToDevice));
            CFD_HIP(hipMemcpy(h->wtr + (size_t)(li - 1) * H * H, tr.data(), n * 4, hipMemcpyHostToDevice));
        }
        (void)c;
        prm->set = true;
    });
}

extern "C" int cfd_siren_ready(const cfd_siren* h) {
    return cfd::guard([&] {
        CFD_REQUIRE(h, CFD_EARG, "null handle");
        for (const auto& p : h->params) CFD_REQUIRE(p.set, CFD_ESTATE, "SIREN parameter not set: " + p.key);
    });
}

extern "C" int cfd_siren_workspace_bytes(const cfd_siren* h, int b, size_t* bytes) {
    return cfd::guard([&] {
        CFD_REQUIRE(h && bytes && b >= 0, CFD_EARG, "bad argument");
        *bytes = sizeof(float) * (size_t)b * (h->cfg.num_hidden_layers + 1) * h->cfg.hidden_features;
    });
}

extern "C" int cfd_siren_forward(cfd_siren* h, const float* coords, int64_t N, const float* latents, int b,
                                 const float* xmax, const float* xmin, const float* ymax, const float* ymin,
                                 int64_t y_stride, float* out, void* ws, size_t ws_bytes, void* stream) {
    return cfd::guard([&] {
        CFD_REQUIRE(h && coords && latents && out, CFD_EARG, "null argument");
        CFD_REQUIRE(N >= 1 && b >= 1, CFD_EARG, "empty decode");
        CFD_REQUIRE((xmax == nullptr) == (xmin == nullptr), CFD_EARG, "xmax/xmin must both be set or both NULL");
        CFD_REQUIRE((ymax == nullptr) == (ymin == nullptr), CFD_EARG, "ymax/ymin must both be set or both NULL");
        size_t need = 0;
        cfd_siren_workspace_bytes(h, b, &need);
        CFD_REQUIRE(ws && ws_bytes >= need, CFD_EARG, "workspace too small");
        const int nh = h->cfg.num_hidden_layers, H = h->cfg.hidden_features, L = h->cfg.in_latent_features;
        auto st = (hipStream_t)stream;
        float* film = (float*)ws;
        hipLaunchKernelGGL(cfd::siren_film, dim3(nh + 1, b), dim3(128), 0, st, h->V, h->fbias, latents, film, H, L,
                           nh + 1);
        cfd::check_launch("siren_film");
        cfd::SirenArgs a{};
        a.w0 = h->w0;
        a.wimg = h->wimg;
        a.wout = h->wout;
        a.bout = h->bout;
        a.film = film;
        a.coords = coords;
        a.xmax = xmax;
        a.xmin = xmin;
        a.ymax = ymax;
        a.ymin = ymin;
        a.out = out;
        a.N = N;
        a.ystride = y_stride;
        a.d = h->cfg.in_coord_features;
        a.c = h->cfg.out_features;
        a.nh = nh;
        a.w0f = h->cfg.w0;
        launch_siren(h, a, b, st);
    });
}

namespace {

void siren_vjp_args(const cfd_siren* h, cfd::SirenVjpArgs& a, int64_t Ns, int R, void* ws) {
    const int nh = h->cfg.num_hidden_layers, H = h->cfg.hidden_features;
    a.w0 = h->w0;
    a.wtr = h->wtr;
    a.wraw = h->wraw;
    a.wout = h->wout;
    a.bout = h->bout;
    a.V = h->V;
    a.film = (float*)ws;
    a.pre = (float*)ws + (size_t)R * (nh + 1) * H;
    a.Ns = (int)Ns;
    a.d = h->cfg.in_coord_features;
    a.c = h->cfg.out_features;
    a.nh = nh;
    a.H = H;
    a.L = h->cfg.in_latent_features;
    a.w0f = h->cfg.w0;
}

int vjp_threads(int H) { return (H + 63) / 64 * 64; }

}  // namespace

extern "C" int cfd_siren_vjp_workspace_bytes(const cfd_siren* h, int64_t Ns, int R, size_t* bytes) {
    return cfd::guard([&] {
        CFD_REQUIRE(h && bytes && Ns >= 0 && R >= 0, CFD_EARG, "bad argument");
        const size_t nl = h->cfg.num_hidden_layers + 1, H = h->cfg.hidden_features;
        *bytes = sizeof(float) * ((size_t)R * nl * H + (size_t)R * Ns * nl * H);
    });
}

extern "C" int cfd_siren_tape_forward(cfd_siren* h, const float* coords, int64_t Ns, const float* latents, int R,
                                      const float* xmax, const float* xmin, const float* ymax, const float* ymin,
                                      int64_t y_stride, float* out, void* ws, size_t ws_bytes, void* stream) {
    return cfd::guard([&] {
        CFD_REQUIRE(h && coords && latents && out && ws, CFD_EARG, "null argument");
        CFD_REQUIRE(Ns >= 1 && Ns <= (1 << 20) && R >= 1, CFD_EARG, "bad sensor / row count");
        CFD_REQUIRE((xmax == nullptr) == (xmin == nullptr) && (ymax == nullptr) == (ymin == nullptr), CFD_EARG,
                    "normaliser bounds must be set in pairs");
        size_t need = 0;
        cfd_siren_vjp_workspace_bytes(h, Ns, R, &need);
        CFD_REQUIRE(ws_bytes >= need, CFD_EARG, "workspace too small");
        const int nh = h->cfg.num_hidden_layers, H = h->cfg.hidden_features, L = h->cfg.in_latent_features;
        auto st = (hipStream_t)stream;
        cfd::SirenVjpArgs a{};
        siren_vjp_args(h, a, Ns, R, ws);
        a.coords = coords;
        a.xmax = xmax;
        a.xmin = xmin;
        a.ymax = ymax;
        a.ymin = ymin;
        a.ystride = y_stride;
        a.out = out;
        hipLaunchKernelGGL(cfd::siren_film, dim3(nh + 1, R), dim3(128), 0, st, h->V, h->fbias, latents, (float*)ws,
                           H, L, nh + 1);
        cfd::check_launch("siren_film");
        hipLaunchKernelGGL(cfd::siren_tape_fwd, dim3(R), dim3(vjp_threads(H)), sizeof(float) * cfd::VJP_SG * H, st,
                           a);
        cfd::check_launch("siren_tape_fwd");
    });
}

extern "C" int cfd_siren_tape_vjp(cfd_siren* h, const float* g_out, int64_t Ns, int R, const float* ymax,
                                  const float* ymin, int64_t y_stride, float* g_latents, void* ws, size_t ws_bytes,
                                  void* stream) {
    return cfd::guard([&] {
        CFD_REQUIRE(h && g_out && g_latents && ws, CFD_EARG, "null argument");
        CFD_REQUIRE(Ns >= 1 && R >= 1, CFD_EARG, "bad sensor / row count");
        CFD_REQUIRE((ymax == nullptr) == (ymin == nullptr), CFD_EARG, "ymax/ymin must both be set or both NULL");
        size_t need = 0;
        cfd_siren_vjp_workspace_bytes(h, Ns, R, &need);
        CFD_REQUIRE(ws_bytes >= need, CFD_EARG, "workspace too small");
        const int nh = h->cfg.num_hidden_layers, H = h->cfg.hidden_features;
        cfd::SirenVjpArgs a{};
        siren_vjp_args(h, a, Ns, R, ws);
        a.ymax = ymax;
        a.ymin = ymin;
        a.ystride = y_stride;
        a.gout = g_out;
        a.gz = g_latents;
        const size_t lds = sizeof(float) * ((size_t)cfd::VJP_SG * H + (size_t)(nh + 1) * H);
        CFD_REQUIRE(lds <= 160 * 1024, CFD_EARG, "SIREN too deep for the input-gradient kernel");
        CFD_HIP(hipFuncSetAttribute((const void*)cfd::siren_tape_vjp, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)lds));
        hipLaunchKernelGGL(cfd::siren_tape_vjp, dim3(R), dim3(vjp_threads(H)), lds, (hipStream_t)stream, a);
        cfd::check_launch("siren_tape_vjp");
    });
}
