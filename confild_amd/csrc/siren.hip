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
#include <cmath>
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "siren.hpp"

namespace cfd {

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
// fp32 GEMM on v_mfma_f32_16x16x4_f32 (exact fp32 products, fp32 accumulation)
// for the two latent-side products of the decoder:
//   FiLM vectors      F (b, nl*H) = z (b, L) . V^T + bias   (V: (nl*H, L), BT)
//   latent gradient   g_z (R, L)  = D (R, nl*H) . V           (V as (K, N))
// C = A . op(B) (+ bias[n]); A (M, K) row-major; B (N, K) (BT) or (K, N).
// 64x64 tiles, 4 waves of 32x32 (2x2 16x16 blocks), K-steps of 16 through LDS
// stored k-major.  Every output's K order is fixed (batch invariant).  The
// per-(latent, layer) VALU dot products it replaces re-read all of V once per
// latent row (2.2 ms per 384-row Case4 film; 1.3 ms per latent gradient).
// ---------------------------------------------------------------------------
template <bool BT>
__global__ __launch_bounds__(256) void gemm_f32_kernel(const float* __restrict__ A, int lda,
                                                       const float* __restrict__ Bm, int ldb,
                                                       const float* __restrict__ bias, float* __restrict__ C, int ldc,
                                                       int M, int N, int K) {
    __shared__ float As[16][64 + 4];
    __shared__ float Bs[16][64 + 4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
    // split-K (gridDim.z > 1): slice z of K, partial sums to C + z * M * ldc
    const int kspan = K / (int)gridDim.z, kbeg = (int)blockIdx.z * kspan;
    A += kbeg;
    Bm += BT ? kbeg : (int64_t)kbeg * ldb;
    K = kspan;
    C += (int64_t)blockIdx.z * M * ldc;
    f4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    const int lr = tid >> 2, lk = (tid & 3) * 4;       // (row, 4 k) of a (64, 16) tile
    const int kr = tid >> 4, kn = (tid & 15) * 4;      // (k, 4 n) of a (16, 64) tile
    for (int k0 = 0; k0 < K; k0 += 16) {
        {
            const int m = m0 + lr;
            f4 v = {0.f, 0.f, 0.f, 0.f};
            if (m < M) v = *(const f4*)(A + (int64_t)m * lda + k0 + lk);
#pragma unroll
            for (int j = 0; j < 4; ++j) As[lk + j][lr] = v[j];
        }
        if constexpr (BT) {
            const int n = n0 + lr;
            f4 v = {0.f, 0.f, 0.f, 0.f};
            if (n < N) v = *(const f4*)(Bm + (int64_t)n * ldb + k0 + lk);
#pragma unroll
            for (int j = 0; j < 4; ++j) Bs[lk + j][lr] = v[j];
        } else {
            f4 v = {0.f, 0.f, 0.f, 0.f};
            if (n0 + kn < N) v = *(const f4*)(Bm + (int64_t)(k0 + kr) * ldb + n0 + kn);
            *(f4*)&Bs[kr][kn] = v;
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < 16; kk += 4) {
            float fa[2], fb[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) fa[i] = As[kk + (lane >> 4)][wm * 32 + 16 * i + (lane & 15)];
#pragma unroll
            for (int j = 0; j < 2; ++j) fb[j] = Bs[kk + (lane >> 4)][wn * 32 + 16 * j + (lane & 15)];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i], fb[j], acc[i][j], 0, 0, 0);
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int n = n0 + wn * 32 + 16 * j + (lane & 15);
            if (n >= N) continue;
            const float bb = bias ? bias[n] : 0.f;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + wm * 32 + 16 * i + 4 * (lane >> 4) + r;
                if (m < M) C[(int64_t)m * ldc + n] = bias ? acc[i][j][r] + bb : acc[i][j][r];
            }
        }
}

// C[m, n] = sum_z part[z][m, n] (+ bias[n]), z in order
__global__ __launch_bounds__(256) void gemm_splitk_reduce_kernel(const float* __restrict__ part, const float* bias,
                                                                float* __restrict__ C, int M, int N, int ldc,
                                                                int splits) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)M * N) return;
    const int64_t m = i / N, n = i - m * N;
    float s = part[m * ldc + n];
    for (int z = 1; z < splits; ++z) s += part[((int64_t)z * M + m) * ldc + n];
    C[m * ldc + n] = bias ? s + bias[n] : s;
}

// split-K count of a latent-side GEMM: a function of K only (never of M, the
// latent rows), so a row's result does not depend on how many rows share the call
static int gemm_splits(int K) {
    int s = 1;
    while (s < 16 && K / (2 * s) >= 256 && K % (32 * s) == 0) s *= 2;
    return s;
}

// part: scratch of gemm_splits(K) * M * ldc floats (used when that is > 1)
static void launch_gemm_f32(bool bt, const float* A, int lda, const float* B, int ldb, const float* bias, float* C,
                            int ldc, int M, int N, int K, hipStream_t st, float* part = nullptr) {
    CFD_REQUIRE(K % 16 == 0 && lda % 4 == 0 && ldb % 4 == 0 && (bt || N % 4 == 0), CFD_ESHAPE,
                "gemm_f32: K % 16, leading dims % 4");
    const int splits = part ? gemm_splits(K) : 1;
    const dim3 grid((unsigned)ceil_div(N, 64), (unsigned)ceil_div(M, 64), (unsigned)splits);
    float* out = splits > 1 ? part : C;
    const float* b = splits > 1 ? nullptr : bias;
    if (bt)
        hipLaunchKernelGGL(gemm_f32_kernel<true>, grid, dim3(256), 0, st, A, lda, B, ldb, b, out, ldc, M, N, K);
    else
        hipLaunchKernelGGL(gemm_f32_kernel<false>, grid, dim3(256), 0, st, A, lda, B, ldb, b, out, ldc, M, N, K);
    check_launch("gemm_f32_kernel");
    if (splits > 1) {
        hipLaunchKernelGGL(gemm_splitk_reduce_kernel, dim3((unsigned)ceil_div((int64_t)M * N, 256)), dim3(256), 0, st,
                           part, bias, C, M, N, ldc, splits);
        check_launch("gemm_splitk_reduce_kernel");
    }
}

// D (R, nf) = sum over the Ns sensors of delta (R, Ns, nf), in sensor order
__global__ __launch_bounds__(256) void sensor_sum_kernel(const float* __restrict__ delta, float* __restrict__ D,
                                                         int Ns, int64_t nf, int64_t R) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= R * nf) return;
    const int64_t r = i / nf, f = i - r * nf;
    const float* src = delta + r * Ns * nf + f;
    float s = 0.f;
    for (int k = 0; k < Ns; ++k) s += src[(int64_t)k * nf];
    D[i] = s;
}

// ---------------------------------------------------------------------------
// K10: CNF autodecoder training step (N/scripts/train.py:392-416, MSELoss): the
// gradients of mean((SIREN(coords, z_rows) - target)^2) w.r.t. every net1 / net2
// parameter and the batch's latent rows, from the DPS tape (pre-activations u_i
// and deltas delta_i per (row, coordinate) pair, siren_tape_fwd / _bwd below).
// Every weight gradient is a "TN" product over the pairs, C[m, n] = sum_k
// X[k, m] Y[k, n] with both operands pair-major (k = pair): X a delta slice,
// Y the previous layer's activation sin(w0 u) recomputed from the tape with the
// forward's own sine (so it is the activation the forward used, bit for bit).
// fp32 MFMA 16x16x4 (exact products), split over k in a fixed slicing and the
// slices added in order: deterministic and independent of the launch.
// ---------------------------------------------------------------------------

// gout = scale * (out - target) (MSELoss 'mean' backward, scale = 2 / numel as
// ATen's mse_loss_backward forms it); per-block sums of (out - target)^2 in double
__global__ __launch_bounds__(256) void mse_grad_kernel(const float* __restrict__ out, const float* __restrict__ target,
                                                       float* __restrict__ gout, int64_t n, float scale,
                                                       double* __restrict__ part) {
    __shared__ double red[256];
    double s = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const float d = out[i] - target[i];
        gout[i] = d * scale;
        s += (double)d * d;
    }
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

// *sse += sum of the block partials, in block order
__global__ void sse_accum_kernel(const double* __restrict__ part, int nb, float* sse) {
    if (threadIdx.x != 0) return;
    double s = 0;
    for (int i = 0; i < nb; ++i) s += part[i];
    *sse += (float)s;
}

// TN product slice: C[z] (M x N) = sum_{k in slice z} X[k * ldx + m] * f(Y[row(k) * ldy + n]),
// row(k) = k % ymod (ymod > 0: the coordinate of pair k) else k; f by YF:
// 0 identity, 1 sin(w0 y) (sin_cw: the tape forward's sine), 2 one (column sums).
// T x T output tiles (T = 64 or 128) over 4 waves (2 x 2, (T/2)^2 each), 16-deep
// k steps staged through LDS, the next step's operands loaded into registers
// while this step's MFMAs run.
template <int YF, int T>
__global__ __launch_bounds__(256) void gemm_tn_kernel(const float* __restrict__ X, int64_t ldx,
                                                      const float* __restrict__ Y, int64_t ldy, int64_t ymod,
                                                      float w0f, float* __restrict__ C, int M, int N, int64_t K,
                                                      int64_t kspan) {
    constexpr int WT = T / 2, NBK = WT / 16;        // wave tile, 16x16 blocks per wave side
    constexpr int PASS = T / 64;                    // (16 x T) tile = PASS x 256 threads x 4 values
    __shared__ float Xs[16][T + 4];
    __shared__ float Ys[16][T + 4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int m0 = blockIdx.y * T, n0 = blockIdx.x * T;
    const int64_t kbeg = (int64_t)blockIdx.z * kspan, kend = min(K, kbeg + kspan);
    f4 acc[NBK][NBK];
#pragma unroll
    for (int i = 0; i < NBK; ++i)
#pragma unroll
        for (int j = 0; j < NBK; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    float xr[PASS][4], yr[PASS][4];
    auto load = [&](int64_t k0) {
#pragma unroll
        for (int ps = 0; ps < PASS; ++ps) {
            const int e = tid + ps * 256;
            const int kr = e / (T / 4), c4 = (e % (T / 4)) * 4;
            const int64_t k = k0 + kr;
            const bool kin = k < kend;
            const int64_t yrow = ymod > 0 ? k % ymod : k;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int m = m0 + c4 + j, n = n0 + c4 + j;
                xr[ps][j] = kin && m < M ? X[k * ldx + m] : 0.f;
                float y = 0.f;
                if (kin && n < N) {
                    if constexpr (YF == 2) y = 1.f;
                    else y = Y[yrow * ldy + n];
                }
                yr[ps][j] = y;
            }
        }
    };
    auto stage = [&]() {
#pragma unroll
        for (int ps = 0; ps < PASS; ++ps) {
            const int e = tid + ps * 256;
            const int kr = e / (T / 4), c4 = (e % (T / 4)) * 4;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                Xs[kr][c4 + j] = xr[ps][j];
                float y = yr[ps][j];
                if constexpr (YF == 1) y = sin_cw(w0f * y);   // padding: sin(0) = 0 (and X is zero there)
                Ys[kr][c4 + j] = y;
            }
        }
    };
    if (kbeg < kend) load(kbeg);
    for (int64_t k0 = kbeg; k0 < kend; k0 += 16) {
        stage();
        __syncthreads();
        if (k0 + 16 < kend) load(k0 + 16);
#pragma unroll
        for (int kk = 0; kk < 16; kk += 4) {
            float fa[NBK], fb[NBK];
#pragma unroll
            for (int i = 0; i < NBK; ++i) fa[i] = Xs[kk + (lane >> 4)][wm * WT + 16 * i + (lane & 15)];
#pragma unroll
            for (int j = 0; j < NBK; ++j) fb[j] = Ys[kk + (lane >> 4)][wn * WT + 16 * j + (lane & 15)];
#pragma unroll
            for (int i = 0; i < NBK; ++i)
#pragma unroll
                for (int j = 0; j < NBK; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i], fb[j], acc[i][j], 0, 0, 0);
        }
        __syncthreads();
    }
    float* Cz = C + (int64_t)blockIdx.z * M * N;
#pragma unroll
    for (int i = 0; i < NBK; ++i)
#pragma unroll
        for (int j = 0; j < NBK; ++j) {
            const int n = n0 + wn * WT + 16 * j + (lane & 15);
            if (n >= N) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + wm * WT + 16 * i + 4 * (lane >> 4) + r;
                if (m < M) Cz[(int64_t)m * N + n] = acc[i][j][r];
            }
        }
}

// G[m * N + n] += sum over the slices of part[z][m, n], z in order (torch's
// gradient accumulation: param.grad + this backward's gradient)
__global__ __launch_bounds__(256) void tn_accum_kernel(const float* __restrict__ part, int64_t MN, int splits,
                                                       float* __restrict__ G) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= MN) return;
    float s = part[i];
    for (int z = 1; z < splits; ++z) s += part[z * MN + i];
    G[i] = G[i] + s;
}

// zr (R, L) = Z[rows[r]] (the batch's latent rows, LatentContainer.forward)
__global__ void gather_rows_kernel(const float* __restrict__ Z, const int64_t* __restrict__ rows, float* __restrict__ zr,
                                   int R, int L) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)R * L) return;
    const int64_t r = i / L, l = i - r * L;
    zr[i] = Z[rows[r] * L + l];
}

// G[rows[r]] += g[r] (distinct rows: the host checks)
__global__ void scatter_add_rows_kernel(const float* __restrict__ g, const int64_t* __restrict__ rows,
                                        float* __restrict__ G, int R, int L) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)R * L) return;
    const int64_t r = i / L, l = i - r * L;
    float* dst = G + rows[r] * L + l;
    *dst = *dst + g[i];
}

// Per-row sums over the coordinates, D[r, f] = sum_s delta[(r Ns + s) nf + f], as
// slice partials: part[z][r][f] over coordinates [z span, (z+1) span) -- every
// thread one column, rows read coalesced (the one-thread-per-column loop over
// all Ns coordinates, sensor_sum_kernel, waited one load per coordinate: 24.6 ms
// for a Case4-width batch of 4 x 65536 pairs).  tn_accum_kernel adds the slices
// in order.
__global__ __launch_bounds__(256) void colsum_part_kernel(const float* __restrict__ delta, float* __restrict__ part,
                                                          int64_t Ns, int64_t nf, int R, int64_t span) {
    const int64_t f = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int r = blockIdx.y, z = blockIdx.z;
    if (f >= nf) return;
    const int64_t s0 = z * span, s1 = min(Ns, s0 + span);
    const float* src = delta + ((int64_t)r * Ns) * nf + f;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;   // four rows in flight, added in row order below
    int64_t s = s0;
    for (; s + 3 < s1; s += 4) {
        const float v0 = src[s * nf], v1 = src[(s + 1) * nf], v2 = src[(s + 2) * nf], v3 = src[(s + 3) * nf];
        a0 += v0;
        a1 += v1;
        a2 += v2;
        a3 += v3;
    }
    for (; s < s1; ++s) a0 += src[s * nf];
    part[((int64_t)z * R + r) * nf + f] = (a0 + a1) + (a2 + a3);
}

// k-slices of a TN product: a function of K only (fixed slicing, deterministic)
static int64_t tn_kspan(int64_t K) {
    const int64_t span = std::max<int64_t>(256, (K + 63) / 64);
    return (span + 15) / 16 * 16;
}

// G (M x N) += TN(X, Y) over K rows; part: scratch of tn_splits * M * N floats
template <int YF>
static void launch_tn(const float* X, int64_t ldx, const float* Y, int64_t ldy, int64_t ymod, float w0f, float* G,
                      int M, int N, int64_t K, float* part, hipStream_t st) {
    const int64_t span = tn_kspan(K);
    const int splits = (int)((K + span - 1) / span);
    if (M >= 128 && N >= 128) {   // the hidden-layer weight gradients: 128 x 128 tiles
        const dim3 grid((unsigned)ceil_div(N, 128), (unsigned)ceil_div(M, 128), (unsigned)splits);
        hipLaunchKernelGGL((gemm_tn_kernel<YF, 128>), grid, dim3(256), 0, st, X, ldx, Y, ldy, ymod, w0f, part, M, N,
                           K, span);
    } else {
        const dim3 grid((unsigned)ceil_div(N, 64), (unsigned)ceil_div(M, 64), (unsigned)splits);
        hipLaunchKernelGGL((gemm_tn_kernel<YF, 64>), grid, dim3(256), 0, st, X, ldx, Y, ldy, ymod, w0f, part, M, N,
                           K, span);
    }
    check_launch("gemm_tn_kernel");
    const int64_t MN = (int64_t)M * N;
    hipLaunchKernelGGL(tn_accum_kernel, dim3((unsigned)ceil_div(MN, 256)), dim3(256), 0, st, part, MN, splits, G);
    check_launch("tn_accum_kernel");
}

// ---------------------------------------------------------------------------
// Latent gradient (DPS adjoint): d<g, A(z)>/dz for the
// Case4 measurement operator A = y_norm.denormalize(SIREN(x_norm(sensors), z))
// (measurements.py:219-226).  The P = R x Ns (latent row, sensor) pairs are the
// "coordinates" of the fused decoder's MFMA chain, each lane carrying its own
// row's FiLM vectors:
//   siren_tape_fwd  forward as siren_fused, also writing every layer's
//                   pre-activation u_i (the tape) and the output A;
//   siren_tape_bwd  delta_nh = (W_out^T g) * w0 cos(w0 u_nh), then
//                   delta_{i-1} = (W_i^T delta_i) * w0 cos(w0 u_{i-1}) on MFMA with a
//                   transposed weight image streamed in reverse layer order;
//                   every delta_i is written out;
//   siren_latent_grad  g_z[r] = sum_i V_i^T (sum_s delta_i[r, s]) in a fixed order
//                   (deterministic, batch invariant).
// ---------------------------------------------------------------------------
// (SirenTapeArgs: siren.hpp)

template <int NB, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void siren_tape_fwd(SirenTapeArgs p) {
    constexpr int TILE = 16 * WAVES;
    constexpr int H = NB * 16;
    constexpr int BLK = NB * 256;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* wbuf = smem;
    float* w0s = smem + 2 * BLK;  // (H, 4)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane >> 4, j16 = lane & 15;
    const int64_t n = (int64_t)blockIdx.x * TILE + wave * 16 + j16;
    const int64_t nc = n < p.P ? n : p.P - 1;
    const int64_t row = nc / p.Ns;
    const int sensor = (int)(nc - row * p.Ns);
    const int nh = p.nh, nl = nh + 1;
    const float* film = p.film + row * nl * H;
    float* ut = p.u + nc * nl * H;
    const bool live = n < p.P;

    for (int f = threadIdx.x; f < H; f += 64 * WAVES) {
        f4 w = {0.f, 0.f, 0.f, 0.f};
        for (int k = 0; k < p.d; ++k) w[k] = p.w0[f * p.d + k];
        *(f4*)(w0s + 4 * f) = w;
    }
    float cn[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (k < p.d) {
            float v = p.coords[(int64_t)sensor * p.d + k];
            if (p.xmax) v = (v - p.xmin[k]) / (p.xmax[k] - p.xmin[k]) * 2.0f - 1.0f;
            cn[k] = v;
        }
    }
    __syncthreads();
    if (nh > 0) siren_issue_block<NB, WAVES>(p.wimg, 0, wbuf, wave, lane);

    float X[NB][4];
    static_for<NB>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        const f4 fv = *(const f4*)(film + 16 * q + 4 * g);
        f4 uu;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const f4 w = *(const f4*)(w0s + 4 * (16 * q + 4 * g + r));
            float a = cn[0] * w[0];
#pragma unroll
            for (int k = 1; k < 4; ++k)
                if (k < p.d) a = fmaf(cn[k], w[k], a);
            uu[r] = a + fv[r];
            X[q][r] = sin_cw(p.w0f * uu[r]);
        }
        if (live) *(f4*)(ut + 16 * q + 4 * g) = uu;
    });

    const int nblocks = nh * NB;
    int J = 0;
    for (int layer = 1; layer <= nh; ++layer) {
        f4 acc[NB];
        static_for<NB>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            if (J + 1 < nblocks) siren_issue_block<NB, WAVES>(p.wimg, J + 1, wbuf + ((J + 1) & 1) * BLK, wave, lane);
            const float* wb = wbuf + (J & 1) * BLK;
            f4 a = *(const f4*)(film + layer * H + 16 * j + 4 * g);
            static_for<NB>([&](auto qc) {
                constexpr int q = decltype(qc)::value;
                const f4 w = *(const f4*)(wb + (q * 64 + lane) * 4);
                a = __builtin_amdgcn_mfma_f32_16x16x4f32(w.x, X[q][0], a, 0, 0, 0);
                a = __builtin_amdgcn_mfma_f32_16x16x4f32(w.y, X[q][1], a, 0, 0, 0);
                a = __builtin_amdgcn_mfma_f32_16x16x4f32(w.z, X[q][2], a, 0, 0, 0);
                a = __builtin_amdgcn_mfma_f32_16x16x4f32(w.w, X[q][3], a, 0, 0, 0);
            });
            acc[j] = a;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            ++J;
        });
        static_for<NB>([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            if (live) *(f4*)(ut + layer * H + 16 * q + 4 * g) = acc[q];
#pragma unroll
            for (int r = 0; r < 4; ++r) X[q][r] = sin_cw(p.w0f * acc[q][r]);
        });
    }

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
    if (live && g < p.c) {
        float v = g == 0 ? o[0] : g == 1 ? o[1] : g == 2 ? o[2] : o[3];
        if (p.ymax) {
            const int64_t yi = (int64_t)sensor * p.ystride + g;
            const float hi = p.ymax[yi], lo = p.ymin[yi];
            v = (v + 1.0f) / 2.0f * (hi - lo) + lo;
        }
        p.out[n * p.c + g] = v;
    }
}

template <int NB, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void siren_tape_bwd(SirenTapeArgs p) {
    constexpr int TILE = 16 * WAVES;
    constexpr int H = NB * 16;
    constexpr int BLK = NB * 256;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* wbuf = smem;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane >> 4, j16 = lane & 15;
    const int64_t n = (int64_t)blockIdx.x * TILE + wave * 16 + j16;
    const int64_t nc = n < p.P ? n : p.P - 1;
    const int sensor = (int)(nc % p.Ns);
    const int nh = p.nh, nl = nh + 1;
    const float* ut = p.u + nc * nl * H;
    float* dt = p.delta + nc * nl * H;
    const bool live = n < p.P;
    const float w0f = p.w0f;

    if (nh > 0) siren_issue_block<NB, WAVES>(p.wimg_t, 0, wbuf, wave, lane);
    // gradient w.r.t. the raw output: g * (ymax - ymin) / 2 (denormalize), then
    // delta_nh = (W_out^T dy) * w0 cos(w0 u_nh) in the B-operand layout
    float dy[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int oc = 0; oc < 4; ++oc) {
        if (oc < p.c) {
            float v = live ? p.gout[nc * p.c + oc] : 0.f;
            if (p.ymax) {
                const int64_t yi = (int64_t)sensor * p.ystride + oc;
                v = v * ((p.ymax[yi] - p.ymin[yi]) / 2.0f);
            }
            dy[oc] = v;
        }
    }
    float X[NB][4];
    static_for<NB>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        const f4 uu = *(const f4*)(ut + nh * H + 16 * q + 4 * g);
        f4 dd;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int f = 16 * q + 4 * g + r;
            float gx = 0.f;
#pragma unroll
            for (int oc = 0; oc < 4; ++oc)
                if (oc < p.c) gx = fmaf(p.wout[oc * H + f], dy[oc], gx);
            dd[r] = gx * (w0f * cos_cw(w0f * uu[r]));
            X[q][r] = dd[r];
        }
        if (live) *(f4*)(dt + nh * H + 16 * q + 4 * g) = dd;
    });

    const int nblocks = nh * NB;
    int J = 0;
    for (int layer = nh; layer >= 1; --layer) {
        // delta_{layer-1} = (W_layer^T delta_layer) * w0 cos(w0 u_{layer-1})
        f4 acc[NB];
        static_for<NB>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            if (J + 1 < nblocks)
                siren_issue_block<NB, WAVES>(p.wimg_t, J + 1, wbuf + ((J + 1) & 1) * BLK, wave, lane);
            const float* wb = wbuf + (J & 1) * BLK;
            f4 a = {0.f, 0.f, 0.f, 0.f};
            static_for<NB>([&](auto qc) {
                constexpr int q = decltype(qc)::value;
                const f4 w = *(const f4*)(wb + (q * 64 + lane) * 4);
                a = __builtin_amdgcn_mfma_f32_16x16x4f32(w.x, X[q][0], a, 0, 0, 0);
                a = __builtin_amdgcn_mfma_f32_16x16x4f32(w.y, X[q][1], a, 0, 0, 0);
                a = __builtin_amdgcn_mfma_f32_16x16x4f32(w.z, X[q][2], a, 0, 0, 0);
                a = __builtin_amdgcn_mfma_f32_16x16x4f32(w.w, X[q][3], a, 0, 0, 0);
            });
            acc[j] = a;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            ++J;
        });
        const int li = layer - 1;
        static_for<NB>([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            const f4 uu = *(const f4*)(ut + li * H + 16 * q + 4 * g);
            f4 dd;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                dd[r] = acc[q][r] * (w0f * cos_cw(w0f * uu[r]));
                X[q][r] = dd[r];
            }
            if (live) *(f4*)(dt + li * H + 16 * q + 4 * g) = dd;
        });
    }
}

// K-split forms of the two tape kernels for small pair counts (a DPS step has
// P = B x rows x sensors pairs, 3840 at Case4 B = 1: 240 waves of 16 pairs, a
// quarter of the chip's SIMDs).  KS waves share one 16-pair tile and split each
// layer's K (input features): wave w multiplies its quarter of the activations by
// its quarter of every weight block (one block per step through the same LDS
// ring) and parks the partial sum in LDS; the wave that owns the block's output
// features (block j belongs to wave j / (NB/KS), which holds exactly those
// features as its next-layer operand) adds the KS partials in wave order, takes
// the sine (forward) or the cos derivative (backward) and writes the tape.  Same
// products as the one-wave kernels, partial sums added in a fixed order
// (deterministic, batch invariant); KS x the waves per pair tile.
template <int NB, int KS>
__global__ __launch_bounds__(64 * KS) void siren_tape_fwd_ks(SirenTapeArgs p) {
    constexpr int H = NB * 16, BLK = NB * 256, QW = NB / KS;
    static_assert(NB % KS == 0, "K split must divide the blocks");
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* wbuf = smem;               // 2 ring slots
    float* w0s = smem + 2 * BLK;      // (H, 4)
    float* red = w0s + 4 * H;         // 2 x KS x 64 lanes x f4 partial sums
    float* osum = red + 2 * KS * 256; // KS x 4 x 16
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = lane >> 4, j16 = lane & 15;
    const int64_t n = (int64_t)blockIdx.x * 16 + j16;
    const int64_t nc = n < p.P ? n : p.P - 1;
    const int64_t row = nc / p.Ns;
    const int sensor = (int)(nc - row * p.Ns);
    const int nh = p.nh, nl = nh + 1;
    const float* film = p.film + row * nl * H;
    float* ut = p.u + nc * nl * H;
    const bool live = n < p.P;
    const int q0 = wave * QW;

    for (int f = threadIdx.x; f < H; f += 64 * KS) {
        f4 w = {0.f, 0.f, 0.f, 0.f};
        for (int k = 0; k < p.d; ++k) w[k] = p.w0[f * p.d + k];
        *(f4*)(w0s + 4 * f) = w;
    }
    float cn[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (k < p.d) {
            float v = p.coords[(int64_t)sensor * p.d + k];
            if (p.xmax) v = (v - p.xmin[k]) / (p.xmax[k] - p.xmin[k]) * 2.0f - 1.0f;
            cn[k] = v;
        }
    }
    __syncthreads();
    if (nh > 0) siren_issue_block<NB, KS>(p.wimg, 0, wbuf, wave, lane);

    float X[QW][4], Xn[QW][4];
    static_for<QW>([&](auto qc) {
        constexpr int qq = decltype(qc)::value;
        const int q = q0 + qq;
        const f4 fv = *(const f4*)(film + 16 * q + 4 * g);
        f4 uu;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const f4 w = *(const f4*)(w0s + 4 * (16 * q + 4 * g + r));
            float a = cn[0] * w[0];
#pragma unroll
            for (int k = 1; k < 4; ++k)
                if (k < p.d) a = fmaf(cn[k], w[k], a);
            uu[r] = a + fv[r];
            X[qq][r] = sin_cw(p.w0f * uu[r]);
        }
        if (live) *(f4*)(ut + 16 * q + 4 * g) = uu;
    });

    const int nblocks = nh * NB;
    int J = 0;
    for (int layer = 1; layer <= nh; ++layer) {
        static_for<NB>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            if (J + 1 < nblocks) siren_issue_block<NB, KS>(p.wimg, J + 1, wbuf + ((J + 1) & 1) * BLK, wave, lane);
            const float* wb = wbuf + (J & 1) * BLK;
            f4 a = wave == 0 ? *(const f4*)(film + layer * H + 16 * j + 4 * g) : f4{0.f, 0.f, 0.f, 0.f};
            static_for<QW>([&](auto qc) {
                constexpr int qq = decltype(qc)::value;
                const f4 w = *(const f4*)(wb + ((q0 + qq) * 64 + lane) * 4);
                a = __builtin_amdgcn_mfma_f32_16x16x4f32(w.x, X[qq][0], a, 0, 0, 0);
                a = __builtin_amdgcn_mfma_f32_16x16x4f32(w.y, X[qq][1], a, 0, 0, 0);
                a = __builtin_amdgcn_mfma_f32_16x16x4f32(w.z, X[qq][2], a, 0, 0, 0);
                a = __builtin_amdgcn_mfma_f32_16x16x4f32(w.w, X[qq][3], a, 0, 0, 0);
            });
            float* rs = red + (j & 1) * KS * 256;
            *(f4*)(rs + (wave * 64 + lane) * 4) = a;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (j / QW == wave) {   // this wave owns output block j: its next-layer features
                constexpr int qq = j % QW;
                f4 acc = *(const f4*)(rs + lane * 4);
#pragma unroll
                for (int w = 1; w < KS; ++w) acc += *(const f4*)(rs + (w * 64 + lane) * 4);
                if (live) *(f4*)(ut + layer * H + 16 * j + 4 * g) = acc;
#pragma unroll
                for (int r = 0; r < 4; ++r) Xn[qq][r] = sin_cw(p.w0f * acc[r]);
            }
            ++J;
        });
        static_for<QW>([&](auto qc) {
            constexpr int qq = decltype(qc)::value;
#pragma unroll
            for (int r = 0; r < 4; ++r) X[qq][r] = Xn[qq][r];
        });
    }

    // output layer: partial sums over this wave's features, combined in wave order
#pragma unroll
    for (int oc = 0; oc < 4; ++oc) {
        if (oc < p.c) {
            const float* wr = p.wout + oc * H + 4 * g;
            float sm = 0.f;
            static_for<QW>([&](auto qc) {
                constexpr int qq = decltype(qc)::value;
                const f4 w = *(const f4*)(wr + 16 * (q0 + qq));
                sm = fmaf(w.x, X[qq][0], sm);
                sm = fmaf(w.y, X[qq][1], sm);
                sm = fmaf(w.z, X[qq][2], sm);
                sm = fmaf(w.w, X[qq][3], sm);
            });
            sm += __shfl_xor(sm, 16);
            sm += __shfl_xor(sm, 32);
            if (g == 0) osum[(wave * 4 + oc) * 16 + j16] = sm;
        }
    }
    __syncthreads();
    if (wave != 0) return;
    float o[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int oc = 0; oc < 4; ++oc) {
        if (oc < p.c) {
            float sm = osum[oc * 16 + j16];
#pragma unroll
            for (int w = 1; w < KS; ++w) sm += osum[(w * 4 + oc) * 16 + j16];
            o[oc] = sm + p.bout[oc];
        }
    }
    if (live && g < p.c) {
        float v = g == 0 ? o[0] : g == 1 ? o[1] : g == 2 ? o[2] : o[3];
        if (p.ymax) {
            const int64_t yi = (int64_t)sensor * p.ystride + g;
            const float hi = p.ymax[yi], lo = p.ymin[yi];
            v = (v + 1.0f) / 2.0f * (hi - lo) + lo;
        }
        p.out[n * p.c + g] = v;
    }
}

template <int NB, int KS>
__global__ __launch_bounds__(64 * KS) void siren_tape_bwd_ks(SirenTapeArgs p) {
    constexpr int H = NB * 16, BLK = NB * 256, QW = NB / KS;
    static_assert(NB % KS == 0, "K split must divide the blocks");
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* wbuf = smem;
    float* red = smem + 2 * BLK;      // 2 x KS x 64 lanes x f4
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = lane >> 4, j16 = lane & 15;
    const int64_t n = (int64_t)blockIdx.x * 16 + j16;
    const int64_t nc = n < p.P ? n : p.P - 1;
    const int sensor = (int)(nc % p.Ns);
    const int nh = p.nh, nl = nh + 1;
    const float* ut = p.u + nc * nl * H;
    float* dt = p.delta + nc * nl * H;
    const bool live = n < p.P;
    const float w0f = p.w0f;
    const int q0 = wave * QW;

    if (nh > 0) siren_issue_block<NB, KS>(p.wimg_t, 0, wbuf, wave, lane);
    float dy[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int oc = 0; oc < 4; ++oc) {
        if (oc < p.c) {
            float v = live ? p.gout[nc * p.c + oc] : 0.f;
            if (p.ymax) {
                const int64_t yi = (int64_t)sensor * p.ystride + oc;
                v = v * ((p.ymax[yi] - p.ymin[yi]) / 2.0f);
            }
            dy[oc] = v;
        }
    }
    float X[QW][4], Xn[QW][4];
    static_for<QW>([&](auto qc) {
        constexpr int qq = decltype(qc)::value;
        const int q = q0 + qq;
        const f4 uu = *(const f4*)(ut + nh * H + 16 * q + 4 * g);
        f4 dd;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int f = 16 * q + 4 * g + r;
            float gx = 0.f;
#pragma unroll
            for (int oc = 0; oc < 4; ++oc)
                if (oc < p.c) gx = fmaf(p.wout[oc * H + f], dy[oc], gx);
            dd[r] = gx * (w0f * cos_cw(w0f * uu[r]));
            X[qq][r] = dd[r];
        }
        if (live) *(f4*)(dt + nh * H + 16 * q + 4 * g) = dd;
    });

    const int nblocks = nh * NB;
    int J = 0;
    for (int layer = nh; layer >= 1; --layer) {
        const int li = layer - 1;
        static_for<NB>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            if (J + 1 < nblocks)
                siren_issue_block<NB, KS>(p.wimg_t, J + 1, wbuf + ((J + 1) & 1) * BLK, wave, lane);
            const float* wb = wbuf + (J & 1) * BLK;
            f4 a = {0.f, 0.f, 0.f, 0.f};
            static_for<QW>([&](auto qc) {
                constexpr int qq = decltype(qc)::value;
                const f4 w = *(const f4*)(wb + ((q0 + qq) * 64 + lane) * 4);
                a = __builtin_amdgcn_mfma_f32_16x16x4f32(w.x, X[qq][0], a, 0, 0, 0);
                a = __builtin_amdgcn_mfma_f32_16x16x4f32(w.y, X[qq][1], a, 0, 0, 0);
                a = __builtin_amdgcn_mfma_f32_16x16x4f32(w.z, X[qq][2], a, 0, 0, 0);
                a = __builtin_amdgcn_mfma_f32_16x16x4f32(w.w, X[qq][3], a, 0, 0, 0);
            });
            float* rs = red + (j & 1) * KS * 256;
            *(f4*)(rs + (wave * 64 + lane) * 4) = a;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (j / QW == wave) {
                constexpr int qq = j % QW;
                f4 acc = *(const f4*)(rs + lane * 4);
#pragma unroll
                for (int w = 1; w < KS; ++w) acc += *(const f4*)(rs + (w * 64 + lane) * 4);
                const f4 uu = *(const f4*)(ut + li * H + 16 * j + 4 * g);
                f4 dd;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    dd[r] = acc[r] * (w0f * cos_cw(w0f * uu[r]));
                    Xn[qq][r] = dd[r];
                }
                if (live) *(f4*)(dt + li * H + 16 * j + 4 * g) = dd;
            }
            ++J;
        });
        static_for<QW>([&](auto qc) {
            constexpr int qq = decltype(qc)::value;
#pragma unroll
            for (int r = 0; r < 4; ++r) X[qq][r] = Xn[qq][r];
        });
    }
}

// g_z[r][l] = sum_i sum_f V_i[f][l] * (sum_s delta[r*Ns + s][i][f])
__global__ __launch_bounds__(256) void siren_latent_grad(const float* __restrict__ delta,
                                                         const float* __restrict__ V, float* __restrict__ gz,
                                                         int Ns, int nl, int H, int L) {
    extern __shared__ __attribute__((aligned(16))) float D[];  // nl * H
    const int64_t r = blockIdx.x;
    const int nf = nl * H;
    const float* dr = delta + r * (int64_t)Ns * nf;
    for (int i = threadIdx.x; i < nf; i += blockDim.x) {
        float s = 0.f;
        for (int k = 0; k < Ns; ++k) s += dr[(int64_t)k * nf + i];
        D[i] = s;
    }
    __syncthreads();
    for (int l = threadIdx.x; l < L; l += blockDim.x) {
        float a = 0.f;
        for (int i = 0; i < nf; ++i) a = fmaf(V[(int64_t)i * L + l], D[i], a);
        gz[r * L + l] = a;
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
    float* wimg_t = nullptr; // transposed weight image, layers nh..1 (latent-gradient path)
    float* wimg16 = nullptr; // split-f16 image (hi, lo) of the scaled hidden weights, same bytes as wimg
    float* wimg16t = nullptr; // the same image of the transposes, layers nh..1 (K9t backward)
    float* wscale = nullptr; // (nh) power-of-two scale of each hidden layer in wimg16
    float* wimg32 = nullptr; // the same split in the 32x32x16 chain's k order (siren_split32)
    float* wimg32r = nullptr; // siren_split32 image of W (w0 / 2pi) s'_i: accumulators in revolutions
    float* wrev = nullptr;    // (2 nh): (w0 / 2pi) s'_i, then 1 / s'_i
    int compute = CFD_SIREN_SPLIT_F16;
};

namespace {

// K7 (fp32 compute): 8 waves per workgroup (the 4-wave and dual-chain variants,
// measured slower, were removed in round 3)
template <int NB>
void launch_siren_nb(const cfd_siren* h, cfd::SirenArgs a, int b, hipStream_t st) {
    const int H = NB * 16;
    const size_t lds = (size_t)(2 * NB * 256 + (h->cfg.num_hidden_layers + 1) * H + 4 * H) * sizeof(float);
    const void* fn = (const void*)cfd::siren_fused<NB, false, 8>;
    CFD_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const int waves = 8;
    const int64_t tiles = cfd::ceil_div(a.N, 16 * waves);
    for (int64_t b0 = 0; b0 < b; b0 += 65535) {
        a.b0 = b0;
        const int nb = (int)std::min<int64_t>(65535, b - b0);
        const dim3 grid((unsigned)tiles, nb);
        hipLaunchKernelGGL((cfd::siren_fused<NB, false, 8>), grid, dim3(512), lds, st, a);
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

namespace {

// Split-f16 image of hidden layer li (siren_split.hip): W s = Wh + Wl with
// s = 2^-e, e = frexp exponent of max|W| (so max|W s| is in [0.5, 1)), both
// halves RNE.  Block j, K-chunk q: 1 KiB of Wh then 1 KiB of Wl, lane-linear,
// lane l element t = W[16j + l%16][16(2q + t/4) + 4(l/16) + t%4] (the A operand
// of v_mfma_f32_16x16x32_f16 in the k order of the accumulator-as-B layout).
void pack_split_f16(cfd_siren* h, int li, const float* W) {
    const int H = h->cfg.hidden_features, NB = h->NB, NQ = NB / 2;
    float amax = 0.f;
    for (size_t i = 0; i < (size_t)H * H; ++i) amax = std::max(amax, std::fabs(W[i]));
    int e = 0;
    if (amax > 0.f) std::frexp(amax, &e);
    const float s = std::ldexp(1.0f, -e);
    std::vector<_Float16> img((size_t)NB * NB * 512);
    for (int j = 0; j < NB; ++j)
        for (int q = 0; q < NQ; ++q)
            for (int l = 0; l < 64; ++l)
                for (int t = 0; t < 8; ++t) {
                    const float v = W[(size_t)(16 * j + l % 16) * H + 16 * (2 * q + t / 4) + 4 * (l / 16) + t % 4] * s;
                    const _Float16 hi = (_Float16)v;
                    const _Float16 lo = (_Float16)(v - (float)hi);
                    const size_t base = ((size_t)j * NB + 2 * q) * 512 + l * 8 + t;
                    img[base] = hi;
                    img[base + 512] = lo;
                }
    CFD_HIP(hipMemcpy(h->wimg16 + (size_t)(li - 1) * NB * NB * 256, img.data(), img.size() * sizeof(_Float16),
                      hipMemcpyHostToDevice));
    // the same image of W^T (same scale), at slot nh - li: the K9t backward's A operand
    for (int j = 0; j < NB; ++j)
        for (int q = 0; q < NQ; ++q)
            for (int l = 0; l < 64; ++l)
                for (int t = 0; t < 8; ++t) {
                    const float v = W[(size_t)(16 * (2 * q + t / 4) + 4 * (l / 16) + t % 4) * H + 16 * j + l % 16] * s;
                    const _Float16 hi = (_Float16)v;
                    const _Float16 lo = (_Float16)(v - (float)hi);
                    const size_t base = ((size_t)j * NB + 2 * q) * 512 + l * 8 + t;
                    img[base] = hi;
                    img[base + 512] = lo;
                }
    CFD_HIP(hipMemcpy(h->wimg16t + (size_t)(h->cfg.num_hidden_layers - li) * NB * NB * 256, img.data(),
                      img.size() * sizeof(_Float16), hipMemcpyHostToDevice));
    // 32x32x16 image: block J (32 rows), K-chunk k = 2 jb + e: 1 KiB of Wh then
    // 1 KiB of Wl, lane-linear, lane l element t =
    // W[32J + l%32][32 jb + 8(2e + t/4) + 4(l/32) + t%4]
    if (H % 32 == 0) {
        const int NB2 = H / 32, NK = H / 16;
        for (int J = 0; J < NB2; ++J)
            for (int k = 0; k < NK; ++k)
                for (int l = 0; l < 64; ++l)
                    for (int t = 0; t < 8; ++t) {
                        const int jb = k / 2, e = k % 2;
                        const float v = W[(size_t)(32 * J + l % 32) * H + 32 * jb + 8 * (2 * e + t / 4) +
                                          4 * (l / 32) + t % 4] * s;
                        const _Float16 hi = (_Float16)v;
                        const _Float16 lo = (_Float16)(v - (float)hi);
                        const size_t base = ((size_t)J * NK + k) * 1024 + l * 8 + t;
                        img[base] = hi;
                        img[base + 512] = lo;
                    }
        CFD_HIP(hipMemcpy(h->wimg32 + (size_t)(li - 1) * NB * NB * 256, img.data(),
                          img.size() * sizeof(_Float16), hipMemcpyHostToDevice));
        // the same image of W (w0 / 2pi) s'_i (s'_i = 2^-e, e the frexp exponent of
        // max|W w0 / 2pi|; scaled and split from float64, both halves RNE): the
        // accumulator of s'_i F_i (w0 / 2pi) + sum is the pre-activation in
        // revolutions times s'_i, so the sine is one multiply by 1/s'_i (exact),
        // a fract and v_sin_f32 (siren_split32, HWSIN >= 3)
        const double kr = (double)h->cfg.w0 / (2.0 * M_PI);
        const double amr = (double)amax * kr;
        int er = 0;
        if (amr > 0.0) std::frexp(amr, &er);
        const double sr = std::ldexp(1.0, -er);
        for (int J = 0; J < NB2; ++J)
            for (int k = 0; k < NK; ++k)
                for (int l = 0; l < 64; ++l)
                    for (int t = 0; t < 8; ++t) {
                        const int jb = k / 2, e = k % 2;
                        const double v = (double)W[(size_t)(32 * J + l % 32) * H + 32 * jb + 8 * (2 * e + t / 4) +
                                                   4 * (l / 32) + t % 4] * kr * sr;
                        const _Float16 hi = (_Float16)v;
                        const _Float16 lo = (_Float16)(v - (double)hi);
                        const size_t base = ((size_t)J * NK + k) * 1024 + l * 8 + t;
                        img[base] = hi;
                        img[base + 512] = lo;
                    }
        CFD_HIP(hipMemcpy(h->wimg32r + (size_t)(li - 1) * NB * NB * 256, img.data(),
                          img.size() * sizeof(_Float16), hipMemcpyHostToDevice));
        const int nh = h->cfg.num_hidden_layers;
        const float fs = (float)(kr * sr), inv = (float)(1.0 / sr);
        CFD_HIP(hipMemcpy(h->wrev + (li - 1), &fs, sizeof(float), hipMemcpyHostToDevice));
        CFD_HIP(hipMemcpy(h->wrev + nh + (li - 1), &inv, sizeof(float), hipMemcpyHostToDevice));
    }
    CFD_HIP(hipMemcpy(h->wscale + (li - 1), &s, sizeof(float), hipMemcpyHostToDevice));
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
        cfd::DeviceGuard dg(device);
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
        CFD_HIP(hipMalloc(&h->wimg_t, sizeof(float) * (size_t)std::max(nh, 1) * NB * NB * 256));
        CFD_HIP(hipMalloc(&h->wimg16, sizeof(float) * (size_t)std::max(nh, 1) * NB * NB * 256));
        CFD_HIP(hipMalloc(&h->wimg16t, sizeof(float) * (size_t)std::max(nh, 1) * NB * NB * 256));
        CFD_HIP(hipMalloc(&h->wscale, sizeof(float) * (size_t)std::max(nh, 1)));
        CFD_HIP(hipMalloc(&h->wimg32, sizeof(float) * (size_t)std::max(nh, 1) * NB * NB * 256));
        CFD_HIP(hipMalloc(&h->wimg32r, sizeof(float) * (size_t)std::max(nh, 1) * NB * NB * 256));
        CFD_HIP(hipMalloc(&h->wrev, sizeof(float) * 2 * (size_t)std::max(nh, 1)));
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
    (void)hipFree(h->wimg_t);
    (void)hipFree(h->wimg16);
    (void)hipFree(h->wimg16t);
    (void)hipFree(h->wscale);
    (void)hipFree(h->wimg32);
    (void)hipFree(h->wimg32r);
    (void)hipFree(h->wrev);
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
        cfd::DeviceGuard dg(h->device);
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
            // transposed image for the backward chain, stored at slot nh - li:
            // img_t[j][q][lane][s] = W[16q + 4(lane>>4) + s][16j + (lane&15)]
            for (int j = 0; j < NB; ++j)
                for (int q = 0; q < NB; ++q)
                    for (int lane = 0; lane < 64; ++lane)
                        for (int s2 = 0; s2 < 4; ++s2)
                            img[(((size_t)j * NB + q) * 64 + lane) * 4 + s2] =
                                host[(size_t)(16 * q + 4 * (lane >> 4) + s2) * H + 16 * j + (lane & 15)];
            CFD_HIP(hipMemcpy(h->wimg_t + (size_t)(nh - li) * NB * NB * 256, img.data(), img.size() * 4,
                              hipMemcpyHostToDevice));
            if (NB % 2 == 0) pack_split_f16(h, li, host);
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

// FiLM vectors F_i = b_i + V_i z of b latent rows, (b, nl, H): one fp32 MFMA GEMM
// (the per-row VALU kernel for latent widths the GEMM tiling does not take)
static void film_vectors(const cfd_siren* h, const float* latents, int b, float* film, hipStream_t st) {
    const int nl = h->cfg.num_hidden_layers + 1, H = h->cfg.hidden_features, L = h->cfg.in_latent_features;
    if (L % 16 == 0) {
        cfd::launch_gemm_f32(true, latents, L, h->V, L, h->fbias, film, nl * H, b, nl * H, L, st);
        return;
    }
    hipLaunchKernelGGL(cfd::siren_film, dim3(nl, b), dim3(128), 0, st, h->V, h->fbias, latents, film, H, L, nl);
    cfd::check_launch("siren_film");
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
        const int nh = h->cfg.num_hidden_layers, H = h->cfg.hidden_features;
        auto st = (hipStream_t)stream;
        float* film = (float*)ws;
        film_vectors(h, latents, b, film, st);
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
        a.stamps = cfd::stamps_buf();
        a.w0f = h->cfg.w0;
        if (h->compute == CFD_SIREN_SPLIT_F16 && nh >= 1 && cfd::siren_split_supported(h->NB)) {
            a.wscale = h->wscale;
            if (cfd::siren_split32_supported(H, nh)) {   // K7t; K7s for the other widths
                a.wimg = h->wimg32;
                a.wimg_rev = h->wimg32r;
                a.wrev = h->wrev;
                cfd::launch_siren_split32(H, a, b, st);
            } else {
                a.wimg = h->wimg16;
                cfd::launch_siren_split(h->NB, a, b, st);
            }
        } else {
            launch_siren(h, a, b, st);
        }
    });
}

extern "C" int cfd_siren_set_compute(cfd_siren* h, int compute) {
    return cfd::guard([&] {
        CFD_REQUIRE(h, CFD_EARG, "null handle");
        CFD_REQUIRE(compute == CFD_SIREN_F32 || compute == CFD_SIREN_SPLIT_F16, CFD_EARG, "unknown SIREN compute mode");
        h->compute = compute;
    });
}

extern "C" int cfd_siren_get_compute(const cfd_siren* h, int* compute) {
    return cfd::guard([&] {
        CFD_REQUIRE(h && compute, CFD_EARG, "null argument");
        const bool split = h->compute == CFD_SIREN_SPLIT_F16 && h->cfg.num_hidden_layers >= 1 &&
                           cfd::siren_split_supported(h->NB);
        *compute = split ? CFD_SIREN_SPLIT_F16 : CFD_SIREN_F32;
    });
}

namespace {

void tape_args(const cfd_siren* h, cfd::SirenTapeArgs& a, int64_t Ns, int R, void* ws) {
    const int nh = h->cfg.num_hidden_layers, H = h->cfg.hidden_features;
    const size_t nl = nh + 1;
    a.w0 = h->w0;
    a.wimg = h->wimg;
    a.wimg_t = h->wimg_t;
    a.wout = h->wout;
    a.bout = h->bout;
    a.film = (float*)ws;
    a.u = (float*)ws + (size_t)R * nl * H;
    a.delta = a.u + (size_t)R * Ns * nl * H;
    a.P = (int64_t)R * Ns;
    a.Ns = (int)Ns;
    a.d = h->cfg.in_coord_features;
    a.c = h->cfg.out_features;
    a.nh = nh;
    a.w0f = h->cfg.w0;
    // K9t (split-f16 tape) in split compute for the widths it has a form for
    if (h->compute == CFD_SIREN_SPLIT_F16 && nh >= 1 && cfd::tape_split_supported(h->NB)) {
        a.wimg16 = h->wimg16;
        a.wimg16t = h->wimg16t;
        a.wscale = h->wscale;
    }
}

// waves per workgroup: 4 when there are enough pairs to fill the chip, else fewer
// (the pair count of a DPS step is small: R * Ns = B * T * 10)
int tape_waves(int64_t P) { return P >= 16 * 4 * 512 ? 4 : P >= 16 * 2 * 256 ? 2 : 1; }

template <int NB, int W>
void launch_tape_w(const cfd::SirenTapeArgs& a, bool bwd, hipStream_t st) {
    const size_t lds = sizeof(float) * (2 * NB * 256 + (bwd ? 0 : 4 * NB * 16));
    const void* fn = bwd ? (const void*)cfd::siren_tape_bwd<NB, W> : (const void*)cfd::siren_tape_fwd<NB, W>;
    CFD_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const dim3 grid((unsigned)cfd::ceil_div(a.P, 16 * W));
    if (bwd)
        hipLaunchKernelGGL((cfd::siren_tape_bwd<NB, W>), grid, dim3(64 * W), lds, st, a);
    else
        hipLaunchKernelGGL((cfd::siren_tape_fwd<NB, W>), grid, dim3(64 * W), lds, st, a);
    cfd::check_launch(bwd ? "siren_tape_bwd" : "siren_tape_fwd");
}

template <int NB, int KS>
void launch_tape_ks(const cfd::SirenTapeArgs& a, bool bwd, hipStream_t st) {
    const size_t lds = sizeof(float) * (2 * NB * 256 + 2 * KS * 256 + (bwd ? 0 : 4 * NB * 16 + KS * 64));
    const void* fn = bwd ? (const void*)cfd::siren_tape_bwd_ks<NB, KS> : (const void*)cfd::siren_tape_fwd_ks<NB, KS>;
    CFD_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const dim3 grid((unsigned)cfd::ceil_div(a.P, 16));
    if (bwd)
        hipLaunchKernelGGL((cfd::siren_tape_bwd_ks<NB, KS>), grid, dim3(64 * KS), lds, st, a);
    else
        hipLaunchKernelGGL((cfd::siren_tape_fwd_ks<NB, KS>), grid, dim3(64 * KS), lds, st, a);
    cfd::check_launch(bwd ? "siren_tape_bwd_ks" : "siren_tape_fwd_ks");
}

template <int NB>
void launch_tape_nb(const cfd::SirenTapeArgs& a, bool bwd, hipStream_t st) {
    // K-split tiles where one wave per 16 pairs leaves most SIMDs idle: K9t in
    // split compute (tape_args set its images), else the fp32 MFMA form
    if constexpr (NB % 4 == 0 && NB <= 24) {
        if (a.P < 16 * 2048) {
            if (a.wimg16) return cfd::launch_tape_split(NB, a, bwd, st);
            return launch_tape_ks<NB, 4>(a, bwd, st);
        }
    }
    switch (tape_waves(a.P)) {
        case 4: return launch_tape_w<NB, 4>(a, bwd, st);
        case 2: return launch_tape_w<NB, 2>(a, bwd, st);
        default: return launch_tape_w<NB, 1>(a, bwd, st);
    }
}

void launch_tape(const cfd_siren* h, const cfd::SirenTapeArgs& a, bool bwd, hipStream_t st) {
    switch (h->NB) {
        case 1: return launch_tape_nb<1>(a, bwd, st);
        case 2: return launch_tape_nb<2>(a, bwd, st);
        case 3: return launch_tape_nb<3>(a, bwd, st);
        case 4: return launch_tape_nb<4>(a, bwd, st);
        case 6: return launch_tape_nb<6>(a, bwd, st);
        case 8: return launch_tape_nb<8>(a, bwd, st);
        case 12: return launch_tape_nb<12>(a, bwd, st);
        case 16: return launch_tape_nb<16>(a, bwd, st);
        case 24: return launch_tape_nb<24>(a, bwd, st);
        case 32: return launch_tape_nb<32>(a, bwd, st);
        default: throw cfd::Error{CFD_EARG, "hidden_features must be 16*{1,2,3,4,6,8,12,16,24,32}"};
    }
}

}  // namespace

extern "C" int cfd_siren_vjp_workspace_bytes(const cfd_siren* h, int64_t Ns, int R, size_t* bytes) {
    return cfd::guard([&] {
        CFD_REQUIRE(h && bytes && Ns >= 0 && R >= 0, CFD_EARG, "bad argument");
        const size_t nl = h->cfg.num_hidden_layers + 1, H = h->cfg.hidden_features;
        // FiLM vectors, the tape (pre-activations and deltas), the sensor-summed deltas,
        // the latent-gradient GEMM's split-K partials
        const size_t L = h->cfg.in_latent_features;
        *bytes = sizeof(float) * (2 * (size_t)R * nl * H + 2 * (size_t)R * Ns * nl * H +
                                  (size_t)cfd::gemm_splits((int)(nl * H)) * R * L);
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
        CFD_REQUIRE(((uintptr_t)ws & 15) == 0, CFD_EARG, "workspace must be 16-byte aligned");
        size_t need = 0;
        cfd_siren_vjp_workspace_bytes(h, Ns, R, &need);
        CFD_REQUIRE(ws_bytes >= need, CFD_EARG, "workspace too small");
        auto st = (hipStream_t)stream;
        cfd::SirenTapeArgs a{};
        tape_args(h, a, Ns, R, ws);
        a.coords = coords;
        a.xmax = xmax;
        a.xmin = xmin;
        a.ymax = ymax;
        a.ymin = ymin;
        a.ystride = y_stride;
        a.out = out;
        film_vectors(h, latents, R, (float*)ws, st);
        launch_tape(h, a, false, st);
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
        const int nh = h->cfg.num_hidden_layers, H = h->cfg.hidden_features, L = h->cfg.in_latent_features;
        auto st = (hipStream_t)stream;
        cfd::SirenTapeArgs a{};
        tape_args(h, a, Ns, R, ws);
        a.ymax = ymax;
        a.ymin = ymin;
        a.ystride = y_stride;
        a.gout = g_out;
        launch_tape(h, a, true, st);
        // g_z = (sum over sensors of delta) . V, as one fp32 MFMA GEMM
        const int64_t nf = (int64_t)(nh + 1) * H;
        if (L % 4 == 0 && nf % 16 == 0) {
            float* D = (float*)ws + (size_t)R * nf + 2 * (size_t)R * Ns * nf;
            hipLaunchKernelGGL(cfd::sensor_sum_kernel, dim3((unsigned)cfd::ceil_div(R * nf, 256)), dim3(256), 0, st,
                               a.delta, D, (int)Ns, nf, (int64_t)R);
            cfd::check_launch("sensor_sum_kernel");
            cfd::launch_gemm_f32(false, D, (int)nf, h->V, L, nullptr, g_latents, L, R, L, (int)nf, st, D + R * nf);
        } else {
            const size_t lds = sizeof(float) * (size_t)(nh + 1) * H;
            CFD_REQUIRE(lds <= 160 * 1024, CFD_EARG, "SIREN too deep for the latent-gradient reduction");
            CFD_HIP(hipFuncSetAttribute((const void*)cfd::siren_latent_grad,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            hipLaunchKernelGGL(cfd::siren_latent_grad, dim3(R), dim3(256), lds, st, a.delta, h->V, g_latents,
                               (int)Ns, nh + 1, H, L);
            cfd::check_launch("siren_latent_grad");
        }
    });
}

// ---------------------------------------------------------------------------
// K10 C ABI: one backward of the CNF autodecoder training loop.
// ---------------------------------------------------------------------------
namespace {

struct TrainWs {
    float *film, *u, *delta, *D, *gpart, *zr, *out, *gout, *gz, *tpart;
    double* sse;
    size_t floats;
};

constexpr int kSseBlocks = 1024;

TrainWs train_ws(const cfd_siren* h, int64_t N, int R, void* base) {
    const size_t nl = h->cfg.num_hidden_layers + 1, H = h->cfg.hidden_features, L = h->cfg.in_latent_features;
    const size_t c = h->cfg.out_features, d = h->cfg.in_coord_features, nf = nl * H, P = (size_t)R * N;
    float* p = (float*)base;
    size_t off = 0;
    auto take = [&](size_t n) {
        float* q = p ? p + off : nullptr;
        off += (n + 63) / 64 * 64;
        return q;
    };
    TrainWs w{};
    // film, u, delta, D back to back: the layout tape_args / the DPS latent gradient use
    w.film = take((size_t)R * nf);
    w.u = p ? w.film + (size_t)R * nf : nullptr;
    off += 2 * P * nf;
    w.delta = p ? w.u + P * nf : nullptr;
    off = (off + 63) / 64 * 64;
    w.D = take((size_t)R * nf);
    w.gpart = take((size_t)cfd::gemm_splits((int)nf) * R * L);
    w.zr = take((size_t)R * L);
    w.out = take(P * c);
    w.gout = take(P * c);
    w.gz = take((size_t)R * L);
    w.sse = (double*)take(2 * kSseBlocks);
    // TN-product slices (<= 64 of the largest gradient) and the column-sum slices (<= 64 x R x nf)
    w.tpart = take((size_t)64 * std::max(std::max(std::max(H * H, H * L), std::max(H * d, c * H)), (size_t)R * nf));
    w.floats = off;
    return w;
}

// the latent-gradient GEMM (launch_gemm_f32) needs these; checked before any
// launch so an unsupported configuration leaves the caller's sums untouched
void train_shape_check(const cfd_siren* h) {
    const int64_t nf = (int64_t)(h->cfg.num_hidden_layers + 1) * h->cfg.hidden_features;
    CFD_REQUIRE(h->cfg.in_latent_features % 4 == 0 && nf % 16 == 0, CFD_ESHAPE,
                "training needs in_latent_features % 4 == 0 and (nh+1)*H % 16 == 0");
}

}  // namespace

extern "C" int cfd_siren_train_workspace_bytes(const cfd_siren* h, int64_t N, int R, size_t* bytes) {
    return cfd::guard([&] {
        CFD_REQUIRE(h && bytes && N >= 0 && R >= 0, CFD_EARG, "bad argument");
        train_shape_check(h);
        *bytes = sizeof(float) * train_ws(h, N, R, nullptr).floats;
    });
}

extern "C" int cfd_siren_train_grad(cfd_siren* h, const float* coords, int64_t N, const float* latents,
                                    const int64_t* rows, int R, const float* target, float scale, float* grad,
                                    float* grad_latents, float* sse, void* ws, size_t ws_bytes, void* stream) {
    return cfd::guard([&] {
        CFD_REQUIRE(h && coords && latents && rows && target && grad && grad_latents && sse && ws, CFD_EARG,
                    "null argument");
        CFD_REQUIRE(N >= 1 && N <= (1 << 20) && R >= 1, CFD_EARG, "bad coordinate / row count");
        CFD_REQUIRE(((uintptr_t)ws & 15) == 0, CFD_EARG, "workspace must be 16-byte aligned");
        train_shape_check(h);
        for (const auto& p : h->params) CFD_REQUIRE(p.set, CFD_ESTATE, "SIREN parameter not set: " + p.key);
        const TrainWs w = train_ws(h, N, R, ws);
        CFD_REQUIRE(ws_bytes >= sizeof(float) * w.floats, CFD_EARG, "workspace too small");
        const int nh = h->cfg.num_hidden_layers, H = h->cfg.hidden_features, L = h->cfg.in_latent_features;
        const int c = h->cfg.out_features, d = h->cfg.in_coord_features;
        const int64_t nf = (int64_t)(nh + 1) * H, P = (int64_t)R * N;
        const float w0f = h->cfg.w0;
        auto st = (hipStream_t)stream;
        // parameter offsets in the flat gradient (cfd_siren_param_info order, reference shapes)
        std::vector<size_t> off;
        size_t o = 0;
        for (const auto& p : h->params) {
            off.push_back(o);
            size_t n = 1;
            for (auto e : p.shape) n *= (size_t)e;
            o += n;
        }
        auto goff = [&](const std::string& key) -> float* {
            for (size_t i = 0; i < h->params.size(); ++i)
                if (h->params[i].key == key) return grad + off[i];
            throw cfd::Error{CFD_ESTATE, "internal: no parameter " + key};
        };
        // forward with tape (LatentContainer rows -> FiLM -> siren_tape_fwd), raw in and out
        hipLaunchKernelGGL(cfd::gather_rows_kernel, dim3((unsigned)cfd::ceil_div((int64_t)R * L, 256)), dim3(256), 0,
                           st, latents, rows, w.zr, R, L);
        cfd::check_launch("gather_rows_kernel");
        film_vectors(h, w.zr, R, w.film, st);
        cfd::SirenTapeArgs a{};
        tape_args(h, a, N, R, ws);
        a.coords = coords;
        a.out = w.out;
        launch_tape(h, a, false, st);
        // loss gradient and sum of squared errors
        const int nb = (int)std::min<int64_t>(kSseBlocks, cfd::ceil_div(P * c, 256));
        hipLaunchKernelGGL(cfd::mse_grad_kernel, dim3(nb), dim3(256), 0, st, w.out, target, w.gout, P * c, scale, w.sse);
        cfd::check_launch("mse_grad_kernel");
        hipLaunchKernelGGL(cfd::sse_accum_kernel, dim3(1), dim3(64), 0, st, w.sse, nb, sse);
        cfd::check_launch("sse_accum_kernel");
        // backward through the chain: every delta_i (P, nl, H)
        a.gout = w.gout;
        launch_tape(h, a, true, st);
        // per-row sums D_i[r] = sum over the coordinates of delta_i = dL/dF_i[r]
        {
            const int64_t span = cfd::tn_kspan(N);
            const int slices = (int)((N + span - 1) / span);
            float* part = slices > 1 ? w.tpart : w.D;
            hipLaunchKernelGGL(cfd::colsum_part_kernel, dim3((unsigned)cfd::ceil_div(nf, 256), R, slices), dim3(256),
                               0, st, w.delta, part, N, nf, R, span);
            cfd::check_launch("colsum_part_kernel");
            if (slices > 1) {
                CFD_HIP(hipMemsetAsync(w.D, 0, sizeof(float) * R * nf, st));
                hipLaunchKernelGGL(cfd::tn_accum_kernel, dim3((unsigned)cfd::ceil_div(R * nf, 256)), dim3(256), 0, st,
                                   part, R * nf, slices, w.D);
                cfd::check_launch("tn_accum_kernel");
            }
        }
        // latent rows: g_z = sum_i D_i V_i, added into grad_latents[rows]
        cfd::launch_gemm_f32(false, w.D, (int)nf, h->V, L, nullptr, w.gz, L, R, L, (int)nf, st, w.gpart);
        hipLaunchKernelGGL(cfd::scatter_add_rows_kernel, dim3((unsigned)cfd::ceil_div((int64_t)R * L, 256)),
                           dim3(256), 0, st, w.gz, rows, grad_latents, R, L);
        cfd::check_launch("scatter_add_rows_kernel");
        // weights: dW_0 = delta_0^T coords, dW_i = delta_i^T sin(w0 u_{i-1}), dW_out = g^T sin(w0 u_nh)
        cfd::launch_tn<0>(w.delta, nf, coords, d, N, w0f, goff("net1.0.weight"), H, d, P, w.tpart, st);
        for (int i = 1; i <= nh; ++i)
            cfd::launch_tn<1>(w.delta + (int64_t)i * H, nf, w.u + (int64_t)(i - 1) * H, nf, 0, w0f,
                              goff("net1." + std::to_string(i) + ".weight"), H, H, P, w.tpart, st);
        const std::string lo = "net1." + std::to_string(nh + 1);
        cfd::launch_tn<1>(w.gout, c, w.u + (int64_t)nh * H, nf, 0, w0f, goff(lo + ".weight"), c, H, P, w.tpart, st);
        cfd::launch_tn<2>(w.gout, c, nullptr, 0, 0, w0f, goff(lo + ".bias"), c, 1, P, w.tpart, st);
        // FiLM side: db_i = sum_r D_i[r], dV_i = D_i^T z
        for (int i = 0; i <= nh; ++i) {
            const std::string k = std::to_string(i);
            cfd::launch_tn<2>(w.D + (int64_t)i * H, nf, nullptr, 0, 0, w0f, goff("net1." + k + ".bias"), H, 1, R,
                              w.tpart, st);
            cfd::launch_tn<0>(w.D + (int64_t)i * H, nf, w.zr, L, 0, w0f, goff("net2." + k + ".weight"), H, L, R,
                              w.tpart, st);
        }
    });
}
