// Fused SIREN/FiLM decoder on f16 MFMA with fp32-level accuracy (K7s).
//
// Same contract and per-(coordinate, latent) arithmetic as siren_fused
// (siren.hip; reference N/cnf/nf_networks.py:480-495, components.py:19-25,64-76,
// normalize.py:100-114), but every hidden-layer product W x runs as three
// v_mfma_f32_16x16x32_f16 on a two-term f16 split of both operands:
//     W s = Wh + Wl,  x = xh + xl   (xh = f16(x), xl = f16(x - xh), RNE)
//     s W x ~= Wl xh + Wh xl + Wh xh          (fp32 accumulate; Wl xl dropped)
// Each split carries 22 significant bits and the products are exact in fp32, so
// the dot product's error is that of an fp32 accumulation (measured against an
// fp64 evaluation: same max / mean error as the fp32 chain).
// s = 2^-e per layer (host, from max|W|) keeps Wh/Wl in f16 normal range;
// the accumulator starts at s F_i (FiLM) and the sine takes (w0/s) acc -- both
// power-of-two rescalings, exact.  The f16 MFMA issues 16x the f32 MFMA rate,
// so three of them cost 3/16 of the f32 chain.
//
// Layout: workgroup = WAVES x 16 coordinates, one latent (grid.y).  The B operand
// of K-chunk q (32 features) is lane-local: lane (n, g) holds features
// 16(2q + t/4) + 4g + t%4, t < 8, which are exactly the accumulator rows of
// output blocks 2q and 2q+1 -- no shuffle between layers.  Hidden weights stream
// through a 2-slot LDS ring by LDS-DMA, one 16-row block (NQ x {hi, lo} x 1 KiB)
// per slot, read with ds_read_b128.  The sine + split of output block j runs
// while block j+1's MFMAs issue (software pipelined, next-layer operands in a
// second register set); the last hidden layer feeds the H -> c output layer in
// fp32 directly.
#include <cstdint>
#include <cstdlib>
#include <algorithm>

#include "siren.hpp"

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef float f2 __attribute__((ext_vector_type(2)));
typedef unsigned u2 __attribute__((ext_vector_type(2)));
typedef unsigned u4 __attribute__((ext_vector_type(4)));

namespace cfd {

// One MFMA operand (8 x f16) as 4 packed 32-bit words, always written whole (a
// partial write of a register tuple makes the allocator copy the tuple around).
struct Frag {
    u4 v;
    __device__ __forceinline__ h8 h() const { return __builtin_bit_cast(h8, v); }
};

__device__ __forceinline__ unsigned pk_f16(float a, float b) {
    return __builtin_bit_cast(unsigned, __builtin_convertvector((f2){a, b}, h2));
}

// Operand split of the 8 values of K-chunk q (x0: output block 2q, x1: block
// 2q+1): hi = f16(x), lo = f16(x - hi), both RNE; written as whole fragments and
// pinned here (IR passes would otherwise sink the split to the fragment's use in
// the next layer, keeping the fp32 values live instead).
__device__ __forceinline__ void split8(const float (&x0)[4], const float (&x1)[4], Frag& hi, Frag& lo) {
    unsigned hw[4], lw[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const float a = w < 2 ? x0[2 * w] : x1[2 * w - 4];
        const float b = w < 2 ? x0[2 * w + 1] : x1[2 * w - 3];
        hw[w] = pk_f16(a, b);
        const f2 hf = __builtin_convertvector(__builtin_bit_cast(h2, hw[w]), f2);
        lw[w] = pk_f16(a - hf.x, b - hf.y);
    }
    hi.v = (u4){hw[0], hw[1], hw[2], hw[3]};
    lo.v = (u4){lw[0], lw[1], lw[2], lw[3]};
    asm volatile("" : "+v"(hi.v), "+v"(lo.v));
}

// sin(x) for two lanes' values on packed fp32 math (v_pk_fma_f32 / v_pk_mul_f32
// do two elements per issue).  Same reduction constants and polynomial as
// sin_cw (common.hpp); the quotient q = rint(x / pi) comes from the 1.5*2^23
// round-to-integer constant (exact for |x| < 2^21 pi), whose low mantissa bit is
// the parity that sets the sign.  The reduction is exact for |x| < 39000 (as
// sin_cw) and degrades gradually beyond (no v_sin_f32 fallback: its valid
// domain ends at 256 revolutions = 1608); q is right for |x| < 2^21 pi.
__device__ __forceinline__ f2 sin2_cw(f2 x) {
    const f2 magic = {12582912.0f, 12582912.0f};
    const f2 t = __builtin_elementwise_fma(x, (f2){0.318309886183790671538f, 0.318309886183790671538f}, magic);
    const f2 q = t - magic;
    f2 r = __builtin_elementwise_fma(q, (f2){-3.140625f, -3.140625f}, x);
    r = __builtin_elementwise_fma(q, (f2){-0.0009670257568359375f, -0.0009670257568359375f}, r);
    r = __builtin_elementwise_fma(q, (f2){-6.2771141529083251953e-07f, -6.2771141529083251953e-07f}, r);
    r = __builtin_elementwise_fma(q, (f2){-1.2154201256553420762e-10f, -1.2154201256553420762e-10f}, r);
    const f2 s = r * r;
    f2 u = (f2){2.6083159809786593541503e-06f, 2.6083159809786593541503e-06f};
    u = __builtin_elementwise_fma(u, s, (f2){-0.0001981069071916863322258f, -0.0001981069071916863322258f});
    u = __builtin_elementwise_fma(u, s, (f2){0.00833307858556509017944336f, 0.00833307858556509017944336f});
    u = __builtin_elementwise_fma(u, s, (f2){-0.166666597127914428710938f, -0.166666597127914428710938f});
    const f2 y = __builtin_elementwise_fma(s, u * r, r);
    // (element-wise scalar bit casts here were miscompiled into a lane copy)
    // adding t << 31 to the bits of y flips exactly the sign bit: one v_lshl_add_u32
    const u2 sg = __builtin_bit_cast(u2, t) << 31;
    return __builtin_bit_cast(f2, __builtin_bit_cast(u2, y) + sg);
}

// Scalar form of sin2_cw (one value; same constants and result bits).  Beside
// MFMAs a packed-fp32 instruction costs more issue than two scalar ones
// (MI355X_MICROARCH.md, one-wave-per-SIMD filler prices), so both are kept.
__device__ __forceinline__ float sin1_cw(float x) {
    const float t = fmaf(x, 0.318309886183790671538f, 12582912.0f);
    const float q = t - 12582912.0f;
    float r = fmaf(q, -3.140625f, x);
    r = fmaf(q, -0.0009670257568359375f, r);
    r = fmaf(q, -6.2771141529083251953e-07f, r);
    r = fmaf(q, -1.2154201256553420762e-10f, r);
    const float s = r * r;
    float u = 2.6083159809786593541503e-06f;
    u = fmaf(u, s, -0.0001981069071916863322258f);
    u = fmaf(u, s, 0.00833307858556509017944336f);
    u = fmaf(u, s, -0.166666597127914428710938f);
    const float y = fmaf(s, u * r, r);
    return __uint_as_float(__float_as_uint(y) + (__float_as_uint(t) << 31));
}

// sin(x) with the hardware sine: x = r + q 2pi (q = rint(x / 2pi), Cody-Waite
// with 2x sin1_cw's pi terms, exact for the same range), then v_sin_f32 on
// r / 2pi revolutions (|r / 2pi| <= 1/2).  7 VALU + one transcendental (2 issue
// slots) against sin1_cw's 13.
__device__ __forceinline__ float sin_hw(float x) {
    const float t = fmaf(x, 0.159154943091895335768f, 12582912.0f);
    const float q = t - 12582912.0f;
    float r = fmaf(q, -6.28125f, x);
    r = fmaf(q, -0.001934051513671875f, r);
    r = fmaf(q, -1.2554228305816650391e-06f, r);
    r = fmaf(q, -2.4308402513106841524e-10f, r);
    return __builtin_amdgcn_sinf(r * 0.159154943091895335768f);
}

// sin(x) with the reduction in revolutions (CFD_SIREN_HWSIN=2; the split32 default before HWSIN 4):
// q = rint(x / 2pi), r = x C_hi - q + x C_lo with 1/2pi = C_hi + C_lo (fma: x C_hi - q
// is exact before its one rounding), then v_sin_f32 on r.  4 VALU + one
// transcendental against sin_hw's 7; two roundings of |r| <= 1/2 (2^-26 rev each)
// instead of one, for any |x| < 2^22 pi (no Cody-Waite range limit).  +2% decoder
// throughput (same-box A/B, 711 -> 697 ms per 256-latent decode).
__device__ __forceinline__ float sin_hw_rev(float x) {
    const float t = fmaf(x, 0.159154943091895335768f, 12582912.0f);
    const float q = t - 12582912.0f;
    float r = fmaf(x, 0.15915493667125701904f, -q);
    r = fmaf(x, 6.4206382432985265041e-09f, r);
    return __builtin_amdgcn_sinf(r);
}

// The hidden-layer sine of siren_split32.  HWSIN 0-2: x is the pre-activation
// w0 u in radians (sin1_cw / sin_hw / sin_hw_rev).  HWSIN 3 and 4: the weights and
// FiLM rows carry w0 / 2pi (wimg_rev), so x = u w0 / 2pi is already in
// revolutions.  4, the default: v_sin_f32 on x as it is -- its input reduction is
// exact (probed over |x| < 1e7 rev: max abs error 1.2e-7, the same as on |x| <= 16;
// test_device_sine_in_revolutions), so the sine costs no VALU besides the
// transcendental (sin_hw_rev: 4 + 1).  3: an explicit r = fract(x) first (fract of a
// small negative x rounds 1 + x to 2^-24: 3.7e-7).
template <int HWSIN>
__device__ __forceinline__ float hidden_sine(float x) {
    if constexpr (HWSIN == 4) return __builtin_amdgcn_sinf(x);
    else if constexpr (HWSIN == 3) return __builtin_amdgcn_sinf(__builtin_amdgcn_fractf(x));
    else if constexpr (HWSIN == 2) return sin_hw_rev(x);
    else if constexpr (HWSIN == 1) return sin_hw(x);
    else return sin1_cw(x);
}

template <bool PK>
__device__ __forceinline__ f2 sin2_sel(f2 x) {
    if constexpr (PK) return sin2_cw(x);
    else return (f2){sin1_cw(x.x), sin1_cw(x.y)};
}

// s_waitcnt immediate waiting for vmcnt <= n only (expcnt, lgkmcnt at their maxima)
constexpr int vmcnt_imm(int n) { return (n & 15) | (7 << 4) | (15 << 8) | (((n >> 4) & 3) << 14); }
// the same with lgkmcnt 0 (the wave's LDS accesses retired too)
constexpr int vm_lgkm0_imm(int n) { return vmcnt_imm(n) & ~(15 << 8); }

// CG column groups of 16 coordinates per wave share every A-fragment read (CG = 2:
// one wave per SIMD, 512 registers; CG = 1: two waves per SIMD, 256 registers).
// RB output blocks (16 rows each) per LDS ring slot: one barrier per RB blocks.
template <int NB, int WAVES, int RING, int CG, int RB = 1, bool NOSYNC = false, bool PKSIN = true>
__global__ __launch_bounds__(64 * WAVES, CG == 1 ? 2 : 1) void siren_fused_split(SirenArgs p) {
    static_assert(NB % 2 == 0, "split-f16 chain needs H % 32 == 0");
    constexpr int NQ = NB / 2;
    constexpr int TILE = 16 * CG * WAVES;
    constexpr int H = NB * 16;
    constexpr int BLK = NB * 256;  // floats per output block: NQ x (hi, lo) x 512 halves
    constexpr int SLOT = RB * BLK;
    static_assert(NB % RB == 0, "ring slots hold whole groups of RB blocks");
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int nh = p.nh;
    float* wbuf = smem;                  // RING slots of RB blocks
    float* film = smem + RING * SLOT;    // (nh+1) x H; hidden layers' rows pre-scaled by s_i
    float* w0s = film + (nh + 1) * H;    // (H, 4)
    float* wos = w0s + 4 * H;            // (4, H) output weights

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int g = lane >> 4;
    const int j16 = lane & 15;
    const int64_t b = p.b0 + blockIdx.y;
    const int64_t n0 = (int64_t)blockIdx.x * TILE + wave * 16 * CG + j16;  // + 16 c

    {
        const float* fsrc = p.film + b * (int64_t)(nh + 1) * H;
        const int nf = (nh + 1) * H;
        for (int i = threadIdx.x * 4; i < nf; i += 64 * WAVES * 4) {
            const int layer = i / H;  // H constexpr
            const float sc = layer == 0 ? 1.0f : p.wscale[layer - 1];
            *(f4*)(film + i) = *(const f4*)(fsrc + i) * sc;  // power-of-two: exact
        }
    }
    for (int f = threadIdx.x; f < H; f += 64 * WAVES) {
        f4 w = {0.f, 0.f, 0.f, 0.f};
        for (int k = 0; k < p.d; ++k) w[k] = p.w0[f * p.d + k];
        *(f4*)(w0s + 4 * f) = w;
    }
    for (int i = threadIdx.x; i < 4 * H; i += 64 * WAVES) wos[i] = i < p.c * H ? p.wout[i] : 0.f;
    float cn[CG][4];
#pragma unroll
    for (int c = 0; c < CG; ++c) {
        const int64_t n = n0 + 16 * c;
        const int64_t nc = n < p.N ? n : p.N - 1;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float v = 0.f;
            if (k < p.d) {
                v = p.coords[nc * p.d + k];
                if (p.xmax) v = (v - p.xmin[k]) / (p.xmax[k] - p.xmin[k]) * 2.0f - 1.0f;
            }
            cn[c][k] = v;
        }
    }

    __syncthreads();
    const int nslots = nh * NB / RB;  // ring fills per decode (nh >= 1, host-checked)
    for (int k = 0; k < RING - 1; ++k)
        if (k < nslots) siren_issue_block<RB * NB, WAVES>(p.wimg, k, wbuf + k * SLOT, wave, lane);
    // LDS-DMA pieces this wave issues per slot (the in-flight count its vmcnt waits see)
    constexpr int PC_LO = RB * NB / WAVES, PC_HI = (RB * NB + WAVES - 1) / WAVES;
    const bool pc_hi = wave < (RB * NB) % WAVES;

    Frag BH[CG][NQ], BL[CG][NQ], NH[CG][NQ], NL[CG][NQ];
    float o[CG][4];
#pragma unroll
    for (int c = 0; c < CG; ++c)
#pragma unroll
        for (int oc = 0; oc < 4; ++oc) o[c][oc] = 0.f;
    // output layer partial sums over this lane's 4 features of block j
    auto out_acc = [&](int c, int j, const float (&x)[4]) __attribute__((always_inline)) {
#pragma unroll
        for (int oc = 0; oc < 4; ++oc) {
            if (oc < p.c) {
                const f4 w = *(const f4*)(wos + oc * H + 16 * j + 4 * g);
                o[c][oc] = fmaf(w.x, x[0], o[c][oc]);
                o[c][oc] = fmaf(w.y, x[1], o[c][oc]);
                o[c][oc] = fmaf(w.z, x[2], o[c][oc]);
                o[c][oc] = fmaf(w.w, x[3], o[c][oc]);
            }
        }
    };

    // ---- layer 0 (d -> H, fp32 VALU): x = sin(w0 (W0 c + F_0)) ----
    static_for<NQ>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
#pragma unroll
        for (int c = 0; c < CG; ++c) {
            float x[2][4];
#pragma unroll
            for (int hb = 0; hb < 2; ++hb) {
                const int blk = 2 * q + hb;
                const f4 fv = *(const f4*)(film + 16 * blk + 4 * g);
                float u[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const f4 w = *(const f4*)(w0s + 4 * (16 * blk + 4 * g + r));
                    float a = cn[c][0] * w[0];
#pragma unroll
                    for (int k = 1; k < 4; ++k)
                        if (k < p.d) a = fmaf(cn[c][k], w[k], a);
                    u[r] = p.w0f * (a + fv[r]);
                }
#pragma unroll
                for (int r = 0; r < 4; r += 2) {
                    const f2 v = sin2_cw((f2){u[r], u[r + 1]});
                    x[hb][r] = v.x;
                    x[hb][r + 1] = v.y;
                }
            }
            split8(x[0], x[1], BH[c][q], BL[c][q]);
        }
    });

    // ---- hidden layers: 3 f16 MFMAs per fp32 product ----
    // Output block j's MFMAs overlap the epilogue of block j-1: its sines in
    // K-chunk 0, and (for odd j-1) the split of blocks (j-2, j-1) into next-layer
    // fragment j/2-1 in K-chunk 1 -- or, in the last layer, the output-layer
    // accumulation.
    int J = 0, slot = 0;
    constexpr int QE = NQ > 1 ? 1 : 0;  // K-chunk of the split / output step
    for (int layer = 1; layer <= nh; ++layer) {
        const bool last = layer == nh;
        const float m = p.w0f / p.wscale[layer - 1];  // power-of-two scale: exact
        float x[CG][4], xs[CG][4];
        auto sines = [&](const f4 (&a)[CG]) __attribute__((always_inline)) {
#pragma unroll
            for (int c = 0; c < CG; ++c) {
                const f2 v0 = sin2_sel<PKSIN>((f2){a[c][0] * m, a[c][1] * m});
                const f2 v1 = sin2_sel<PKSIN>((f2){a[c][2] * m, a[c][3] * m});
                x[c][0] = v0.x;
                x[c][1] = v0.y;
                x[c][2] = v1.x;
                x[c][3] = v1.y;
                asm volatile("" : "+v"(x[c][0]), "+v"(x[c][1]), "+v"(x[c][2]), "+v"(x[c][3]));
            }
        };
        auto epilogue = [&](auto jc) __attribute__((always_inline)) {  // block j's sines are in x
            constexpr int j = decltype(jc)::value;
#pragma unroll
            for (int c = 0; c < CG; ++c) {
                if (last) {
                    out_acc(c, j, x[c]);
                } else if constexpr (j & 1) {
                    split8(xs[c], x[c], NH[c][j / 2], NL[c][j / 2]);
                } else {
#pragma unroll
                    for (int r = 0; r < 4; ++r) xs[c][r] = x[c][r];
                }
            }
        };
        f4 prev[CG];
        static_for<NB>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            // at a slot's first block: refill the slot the previous group used
            // (every wave left it at the last barrier)
            // (one block of the group per output block, spreading the DMA issue)
            const bool steady = J + RING - 1 < nslots;
            {
                const int fill = slot == 0 ? RING - 1 : slot - 1;
                if (steady && !NOSYNC)
                    siren_issue_block<NB, WAVES>(p.wimg, (J + RING - 1) * RB + j % RB,
                                                 wbuf + fill * SLOT + (j % RB) * BLK, wave, lane);
            }
            const float* wb = wbuf + slot * SLOT + (j % RB) * BLK;
            f4 a[CG];
            {
                const f4 f = *(const f4*)(film + layer * H + 16 * j + 4 * g);
#pragma unroll
                for (int c = 0; c < CG; ++c) a[c] = f;
            }
            h8 FH[NQ], FL[NQ];
            FH[0] = *(const h8*)(wb + lane * 4);
            FL[0] = *(const h8*)(wb + 256 + lane * 4);
            static_for<NQ>([&](auto qc) {
                constexpr int q = decltype(qc)::value;
                if constexpr (q + 1 < NQ) {
                    FH[q + 1] = *(const h8*)(wb + (q + 1) * 512 + lane * 4);
                    FL[q + 1] = *(const h8*)(wb + (q + 1) * 512 + 256 + lane * 4);
                }
#pragma unroll
                for (int c = 0; c < CG; ++c)
                    a[c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(FL[q], BH[c][q].h(), a[c], 0, 0, 0);
#pragma unroll
                for (int c = 0; c < CG; ++c)
                    a[c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(FH[q], BL[c][q].h(), a[c], 0, 0, 0);
#pragma unroll
                for (int c = 0; c < CG; ++c)
                    a[c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(FH[q], BH[c][q].h(), a[c], 0, 0, 0);
                if constexpr (j > 0) {
                    if constexpr (q == 0) sines(prev);
                    if constexpr (q == QE) epilogue(std::integral_constant<int, j - 1>{});
                }
                __builtin_amdgcn_sched_barrier(0);
            });
#pragma unroll
            for (int c = 0; c < CG; ++c) prev[c] = a[c];
            // block J+1 landed (this wave's pieces; the RING-2 younger blocks may
            // stay in flight); the barrier publishes every wave's pieces and
            // retires all reads of this slot before its refill.  A bare s_barrier:
            // __syncthreads' LDS release fence would drain every LDS-DMA in flight.
            if constexpr (j % RB == RB - 1) {
                if (NOSYNC) {
                    // timing experiment only (wrong results): no weight streaming, no barrier
                } else if (steady) {
                    if (PC_HI == PC_LO || !pc_hi)
                        __builtin_amdgcn_s_waitcnt(vmcnt_imm((RING - 2) * PC_LO));
                    else
                        __builtin_amdgcn_s_waitcnt(vmcnt_imm((RING - 2) * PC_HI));
                } else {
                    __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));
                }
                if (!NOSYNC) asm volatile("s_barrier" ::: "memory");
                ++J;
                slot = slot == RING - 1 ? 0 : slot + 1;
            }
        });
        sines(prev);
        epilogue(std::integral_constant<int, NB - 1>{});
        static_for<NQ>([&](auto qc) {
            constexpr int q = decltype(qc)::value;
#pragma unroll
            for (int c = 0; c < CG; ++c) {
                BH[c][q] = NH[c][q];
                BL[c][q] = NL[c][q];
            }
        });
    }

    // ---- output layer (H -> c): reduce the 4 lane groups, bias, de-normalise ----
#pragma unroll
    for (int c = 0; c < CG; ++c) {
        float ov[4];
#pragma unroll
        for (int oc = 0; oc < 4; ++oc) {
            float sum = o[c][oc];
            sum += __shfl_xor(sum, 16);
            sum += __shfl_xor(sum, 32);
            ov[oc] = oc < p.c ? sum + p.bout[oc] : 0.f;
        }
        const int64_t n = n0 + 16 * c;
        if (n < p.N && g < p.c) {
            float v = g == 0 ? ov[0] : g == 1 ? ov[1] : g == 2 ? ov[2] : ov[3];
            if (p.ymax) {
                const int64_t yi = n * p.ystride + g;
                const float hi = p.ymax[yi], lo = p.ymin[yi];
                v = (v + 1.0f) / 2.0f * (hi - lo) + lo;
            }
            p.out[(b * p.N + n) * p.c + g] = v;
        }
    }
}

// ---------------------------------------------------------------------------
// K7t: the same split-f16 chain on v_mfma_f32_32x32x16_f16, one wave per SIMD.
//
// Why: the 16x16x32 chain above is issue-bound, not MFMA-bound.  A 16x16x32
// MFMA holds the SIMD's vector issue for 8 of its 16 cycles, and each fp32
// activation needs ~15 VALU instructions (scale, sine, split) -- together more
// issue than the MFMA time they hide behind.  A 32x32x16 MFMA holds issue for 8
// of its 32 cycles at the same FLOP rate, which halves the hold per FLOP.
//
// Layout: workgroup = 4 waves x 32 coordinates, one latent (grid.y).  Output
// block J (32 features) of a layer is one 32x32 accumulator: lane (h = l/32,
// n = l%32) holds features 32J + 8qq + 4h + r at acc[4qq + r] for coordinate n.
// K-chunk 2J + e of the next layer (16 features) is lane-local: lane (h, n)
// element t = acc[8e + t], feature 32J + 8(2e + t/4) + 4h + t%4 -- the weight
// image is packed in that k order (pack_split_f16_32), so no shuffle between
// layers.  Weights stream through a 2-slot LDS ring by LDS-DMA, one 32-row block
// (NK x {hi, lo} x 1 KiB) per slot, issued in the first half of the previous
// block.  Block j's MFMAs overlap block j-1's sines (one value per K-chunk step)
// and its split (v_fma_mix: lo = f16(x - hi) in one instruction per value).
typedef float f16v __attribute__((ext_vector_type(16)));

// hi/lo f16 split of two values: hi = f16(a, b) (RNE), lo = f16(a - hi_a, b - hi_b)
// (a - hi is exact in fp32, so one rounding as in split8).
__device__ __forceinline__ void split2_mix(float a, float b, unsigned& hi, unsigned& lo) {
    hi = pk_f16(a, b);
    asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=&v"(lo) : "v"(a), "v"(hi));
    asm("v_fma_mixhi_f16 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "+v"(lo) : "v"(b), "v"(hi));
}

// chunk e (0, 1) of a 32x32 block's 16 values -> (hi, lo) fragments
__device__ __forceinline__ void split_chunk(const float (&x)[16], int e, Frag& hi, Frag& lo) {
    unsigned hw[4], lw[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) split2_mix(x[8 * e + 2 * w], x[8 * e + 2 * w + 1], hw[w], lw[w]);
    hi.v = (u4){hw[0], hw[1], hw[2], hw[3]};
    lo.v = (u4){lw[0], lw[1], lw[2], lw[3]};
    asm volatile("" : "+v"(hi.v), "+v"(lo.v));
}

// EXP (timing experiments only, wrong results): bit 0 no weight streaming / barrier,
// bit 1 no sine (x = scaled accumulator), bit 2 no per-step A-fragment LDS reads
// (every step reuses the block's first fragments)
template <int NB2, int EXP = 0, int HWSIN = 0>
__global__ __launch_bounds__(256, 1) void siren_split32(SirenArgs p) {
    constexpr int NK = 2 * NB2;    // 16-deep K chunks per layer
    constexpr int H = 32 * NB2;
    constexpr int BLK = NK * 512;  // floats per 32-row block: NK x {hi, lo} x 1 KiB
    constexpr int WAVES = 4, TILE = 128;
    constexpr int NPC = 2 * NK;    // 1-KiB LDS-DMA pieces per block
    constexpr int PPW = NPC / WAVES;
    // K-chunk steps carrying the previous block's 16 sines, and the step that
    // splits them: block 0 reads the chunks it produces at steps NK-2, NK-1
    constexpr int NKS = NK >= 18 ? 16 : NK - 2;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int nh = p.nh;
    float* wbuf = smem;                // 2 ring slots
    float* film = smem + 2 * BLK;      // (nh+1) x H; hidden layers' rows pre-scaled by s_i
    float* w0s = film + (nh + 1) * H;  // (H, 4)
    float* wos = w0s + 4 * H;          // (4, H)

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int h = lane >> 5;
    const int64_t b = p.b0 + blockIdx.y;
    const int64_t n = (int64_t)blockIdx.x * TILE + wave * 32 + (lane & 31);
    CFD_DASSERT(p.d >= 1 && p.d <= 4 && p.c >= 1 && p.c <= 4 && nh >= 1);
#ifdef CFD_STAMPS
    // the in-kernel clock (tools/dev/siren_clock.py): entry / exit stamps of
    // s_memrealtime (100 MHz) and s_memtime (shader cycles) on every 61st tile
    // column, spread over the XCDs (kind 5, launch field = the latent)
    const bool stamped = blockIdx.x % 61 == 0;
    if (stamped) CFD_STAMP(p.stamps, 5, (unsigned)blockIdx.y, 0);
    __builtin_amdgcn_s_waitcnt(0xC07F);
#endif

    {
        const float* fsrc = p.film + b * (int64_t)(nh + 1) * H;
        const int nf = (nh + 1) * H;
        for (int i = threadIdx.x * 4; i < nf; i += 64 * WAVES * 4) {
            const int layer = i / H;
            // HWSIN < 3: power-of-two s_i (exact); HWSIN >= 3: (w0 / 2pi) s'_i
            const float sc = layer == 0 ? 1.0f : HWSIN >= 3 ? p.wrev[layer - 1] : p.wscale[layer - 1];
            *(f4*)(film + i) = *(const f4*)(fsrc + i) * sc;
        }
    }
    for (int f = threadIdx.x; f < H; f += 64 * WAVES) {
        f4 w = {0.f, 0.f, 0.f, 0.f};
        for (int k = 0; k < p.d; ++k) w[k] = p.w0[f * p.d + k];
        *(f4*)(w0s + 4 * f) = w;
    }
    for (int i = threadIdx.x; i < 4 * H; i += 64 * WAVES) wos[i] = i < p.c * H ? p.wout[i] : 0.f;
    float cn[4];
    {
        const int64_t nc = n < p.N ? n : p.N - 1;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float v = 0.f;
            if (k < p.d) {
                v = p.coords[nc * p.d + k];
                if (p.xmax) v = (v - p.xmin[k]) / (p.xmax[k] - p.xmin[k]) * 2.0f - 1.0f;
            }
            cn[k] = v;
        }
    }
    __syncthreads();
    const int nblocks = nh * NB2;
    const __amdgpu_buffer_rsrc_t wrsrc =
        __builtin_amdgcn_make_buffer_rsrc((void*)p.wimg, 0, nblocks * (BLK * 4), 0x00020000);
    siren_issue_block<NPC, WAVES>(p.wimg, 0, wbuf, wave, lane);

    Frag BH[NK], BL[NK], NH[NK], NL[NK];
    float o[4] = {0.f, 0.f, 0.f, 0.f};

    // ---- layer 0 (d -> H, fp32 VALU): x = sin(w0 (W0 c + F_0)), into the split set ----
    static_for<NB2>([&](auto Jc) {
        constexpr int J = decltype(Jc)::value;
        float x[16];
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
            const f4 fv = *(const f4*)(film + 32 * J + 8 * qq + 4 * h);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const f4 w = *(const f4*)(w0s + 4 * (32 * J + 8 * qq + 4 * h + r));
                float a = cn[0] * w[0];
#pragma unroll
                for (int k = 1; k < 4; ++k)
                    if (k < p.d) a = fmaf(cn[k], w[k], a);
                x[4 * qq + r] = hidden_sine<HWSIN >= 2 ? 2 : HWSIN>(p.w0f * (a + fv[r]));
            }
        }
        split_chunk(x, 0, NH[2 * J], NL[2 * J]);
        split_chunk(x, 1, NH[2 * J + 1], NL[2 * J + 1]);
    });

    // ---- hidden layers: 3 f16 MFMAs per fp32 product ----
    // Block j's MFMAs overlap the epilogue (sines, split or output-layer sums) of
    // the block before it -- for j = 0 the previous layer's last block, whose
    // chunks NK-2, NK-1 are produced at steps 16-17 and consumed at steps NK-2,
    // NK-1 of the same block.  Block 0 reads its B operands from the VGPR split
    // set and copies each chunk into the accumulator file for blocks 1.. (the
    // 384 operand registers of two layers do not fit in one file).
    static_assert(NB2 % 2 == 0, "static ring slots need an even block count");
    int J = 0;
    f16v prev;
    float mprev = 0.f;
    float x[16];
    for (int layer = 1; layer <= nh; ++layer) {
        const bool last = layer == nh;
        // power-of-two scales: exact (HWSIN >= 3: 1 / s'_i, the result in revolutions)
        const float m = HWSIN >= 3 ? p.wrev[nh + layer - 1] : p.w0f / p.wscale[layer - 1];
        // output-layer partial sums over the 4 features of part e of block jp (x: its sines)
        auto outsum = [&](int jp, int e) __attribute__((always_inline)) {  // wos rows oc >= c are zero
            const int f = 32 * jp + 8 * e + 4 * h;
#pragma unroll
            for (int oc = 0; oc < 4; ++oc) {
                const f4 w = *(const f4*)(wos + oc * H + f);
#pragma unroll
                for (int r = 0; r < 4; ++r) o[oc] = fmaf(w[r], x[4 * e + r], o[oc]);
            }
        };
        static_for<NB2>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            constexpr int jp = j == 0 ? NB2 - 1 : j - 1;  // block whose epilogue runs here
            const float me = j == 0 ? mprev : m;
            const bool live = j > 0 || layer > 1;        // there is such a block
            // block J+1 into the free slot; past the last block, the last block
            // again (branch-free; that slot is no longer read)
            // NB2 is even, so block j of every layer uses ring slot j % 2 (static
            // LDS offsets off one lane base)
            float* nxt = wbuf + ((j & 1) ^ 1) * BLK;
            const float* wb = wbuf + (j & 1) * BLK;
            const int soff = __builtin_amdgcn_readfirstlane(min(J + 1, nblocks - 1)) * (BLK * 4);
            f16v a;
#pragma unroll
            for (int qq = 0; qq < 4; ++qq) {
                const f4 f = *(const f4*)(film + layer * H + 32 * j + 8 * qq + 4 * h);
#pragma unroll
                for (int r = 0; r < 4; ++r) a[4 * qq + r] = f[r];
            }
            h8 FH = *(const h8*)(wb + lane * 4);
            h8 FL = *(const h8*)(wb + 256 + lane * 4);
            static_for<NK>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                h8 FH1 = FH, FL1 = FL;
                if constexpr (k + 1 < NK && !(EXP & 4)) {
                    FH1 = *(const h8*)(wb + (k + 1) * 512 + lane * 4);
                    FL1 = *(const h8*)(wb + (k + 1) * 512 + 256 + lane * 4);
                }
                if constexpr (k < PPW && !(EXP & 1)) {
                    const int piece = wave + WAVES * k;
                    // buffer form: scalar base + offset, one per-lane VGPR offset (no VALU per piece)
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(
                        wrsrc, (__attribute__((address_space(3))) void*)(nxt + piece * 256), 16, lane * 16,
                        soff + piece * 1024, 0, 0);
                }
                if constexpr (j == 0) {
                    a = __builtin_amdgcn_mfma_f32_32x32x16_f16(FL, NH[k].h(), a, 0, 0, 0);
                    a = __builtin_amdgcn_mfma_f32_32x32x16_f16(FH, NL[k].h(), a, 0, 0, 0);
                    a = __builtin_amdgcn_mfma_f32_32x32x16_f16(FH, NH[k].h(), a, 0, 0, 0);
                    BH[k] = NH[k];
                    BL[k] = NL[k];
                    asm volatile("" : "+a"(BH[k].v), "+a"(BL[k].v));
                } else {
                    a = __builtin_amdgcn_mfma_f32_32x32x16_f16(FL, BH[k].h(), a, 0, 0, 0);
                    a = __builtin_amdgcn_mfma_f32_32x32x16_f16(FH, BL[k].h(), a, 0, 0, 0);
                    a = __builtin_amdgcn_mfma_f32_32x32x16_f16(FH, BH[k].h(), a, 0, 0, 0);
                }
                if constexpr (k < NKS) {
#pragma unroll
                    for (int v = 16 * k / NKS; v < 16 * (k + 1) / NKS; ++v) {
                        x[v] = (EXP & 2) ? prev[v] * me : hidden_sine<HWSIN>(prev[v] * me);
                        asm volatile("" : "+v"(x[v]));  // keep it in this step (no sinking to the split)
                    }
                }
                // split (chunks 2jp, 2jp+1 of the next layer -- or, for j = 0, of this
                // one) or, in the last layer, the output-layer sums
                constexpr int KE = NK >= 18 ? 16 : NKS - 1;
                if constexpr (k == KE || k == (NK >= 18 ? 17 : KE)) {
                    constexpr bool both = NK < 18;
                    constexpr int e0 = (NK >= 18 && k == 17) ? 1 : 0;
                    if (live) {
#pragma unroll
                        for (int e = e0; e < (both ? 2 : e0 + 1); ++e)
                            split_chunk(x, e, NH[2 * jp + e], NL[2 * jp + e]);
                        if (j > 0 && last) {
#pragma unroll
                            for (int e = 2 * e0; e < (both ? 4 : 2 * e0 + 2); ++e) outsum(jp, e);
                        }
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
                FH = FH1;
                FL = FL1;
            });
            prev = a;
            // this wave's pieces of block J+1 landed; the barrier publishes every
            // wave's pieces and retires all reads of this slot before its refill
            // (a bare s_barrier: __syncthreads' fence would add nothing here)
            if constexpr (!(EXP & 1)) {
                __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));
                asm volatile("s_barrier" ::: "memory");
            }
            ++J;
        });
        mprev = m;
    }
    // the last layer's last block
#pragma unroll
    for (int v = 0; v < 16; ++v) x[v] = hidden_sine<HWSIN>(prev[v] * mprev);
    {
        const int f0 = 32 * (NB2 - 1) + 4 * h;
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int oc = 0; oc < 4; ++oc) {
                const f4 w = *(const f4*)(wos + oc * H + f0 + 8 * e);
#pragma unroll
                for (int r = 0; r < 4; ++r) o[oc] = fmaf(w[r], x[4 * e + r], o[oc]);
            }
    }

    // ---- output layer (H -> c): reduce the two lane halves, bias, de-normalise ----
    float ov[4];
#pragma unroll
    for (int oc = 0; oc < 4; ++oc) {
        const float sum = o[oc] + __shfl_xor(o[oc], 32);
        ov[oc] = oc < p.c ? sum + p.bout[oc] : 0.f;
    }
    if (n < p.N) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int oc = 2 * h + i;
            if (oc < p.c) {
                float v = ov[oc];
                if (p.ymax) {
                    const int64_t yi = n * p.ystride + oc;
                    const float hi = p.ymax[yi], lo = p.ymin[yi];
                    v = (v + 1.0f) / 2.0f * (hi - lo) + lo;
                }
                p.out[(b * p.N + n) * p.c + oc] = v;
            }
        }
    }
#ifdef CFD_STAMPS
    if (stamped) CFD_STAMP(p.stamps, 5, (unsigned)blockIdx.y, 4);
#endif
}

namespace {

template <int NB, int RING, int CG, int RB = 1, bool NOSYNC = false, bool PKSIN = true>
void launch_ring(SirenArgs a, int b, hipStream_t st) {
    constexpr int H = NB * 16;
    constexpr int WAVES = CG == 1 ? 8 : 4;
    const size_t lds = sizeof(float) * ((size_t)RING * RB * NB * 256 + (size_t)(a.nh + 1) * H + 8 * H);
    const void* fn = (const void*)siren_fused_split<NB, WAVES, RING, CG, RB, NOSYNC, PKSIN>;
    CFD_REQUIRE(lds <= 160 * 1024, CFD_EARG, "SIREN too deep for the split-f16 decoder's LDS staging");
    CFD_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const int64_t tiles = ceil_div(a.N, 16 * CG * WAVES);
    CFD_REQUIRE(tiles <= 0x7fffffff, CFD_EARG, "too many coordinates for one launch");
    for (int64_t b0 = 0; b0 < b; b0 += 65535) {
        a.b0 = b0;
        const int nb = (int)std::min<int64_t>(65535, b - b0);
        hipLaunchKernelGGL((siren_fused_split<NB, WAVES, RING, CG, RB, NOSYNC, PKSIN>), dim3((unsigned)tiles, nb),
                           dim3(64 * WAVES), lds, st, a);
        check_launch("siren_fused_split");
    }
}

// K7s: 8 waves, one 16-row block per ring slot (the measured variants -- two
// coordinate groups per wave, two blocks per slot, the scalar sine, no barrier
// -- were removed in round 3)
template <int NB>
void launch_nb(SirenArgs a, int b, hipStream_t st) {
    launch_ring<NB, 2, 1, 1>(a, b, st);
}
}  // namespace

template <int NB2, int EXP = 0, int HWSIN = 0>
void launch_split32(SirenArgs a, int b, hipStream_t st) {
    constexpr int H = NB2 * 32;
    const size_t lds = sizeof(float) * ((size_t)2 * 2 * NB2 * 512 + (size_t)(a.nh + 1) * H + 8 * H);
    const void* fn = (const void*)siren_split32<NB2, EXP, HWSIN>;
    CFD_REQUIRE((int64_t)a.nh * H * H * 4 < 0x7fffffffLL, CFD_EARG, "weight image beyond the 2 GiB buffer range");
    CFD_REQUIRE(lds <= 160 * 1024, CFD_EARG, "SIREN too deep for the split-f16 decoder's LDS staging");
    CFD_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const int64_t tiles = ceil_div(a.N, 128);
    CFD_REQUIRE(tiles <= 0x7fffffff, CFD_EARG, "too many coordinates for one launch");
    for (int64_t b0 = 0; b0 < b; b0 += 65535) {
        a.b0 = b0;
        const int nb = (int)std::min<int64_t>(65535, b - b0);
        hipLaunchKernelGGL((siren_split32<NB2, EXP, HWSIN>), dim3((unsigned)tiles, nb), dim3(256), lds, st, a);
        check_launch("siren_split32");
    }
}

bool siren_split32_supported(int H, int nh) {
    const size_t film = (size_t)(nh + 1) * H + 8 * (size_t)H;
    return (H == 64 || H == 128 || H == 256 || H == 384) &&
           sizeof(float) * ((size_t)4 * (H / 32) * 512 + film) <= 160 * 1024;
}

// HWSIN 4: weights pre-scaled by w0/2pi, v_sin_f32 on the revolutions (the
// explicit-fract form, 3, measured the same and was removed in round 6).  The
// radian-domain sines (0: polynomial, 1: 2pi Cody-Waite, 2: reduction in
// revolutions) stay in the sine probe (cfd_sine_probe) and the K7s/K9d kernels;
// their full decoder instantiations were removed in round 3.
void launch_siren_split32(int H, SirenArgs a, int b, hipStream_t st) {
    CFD_REQUIRE(a.wimg_rev && a.wrev, CFD_EARG, "split32 revolution image not set");
    a.wimg = a.wimg_rev;
    switch (H) {
        case 64: return launch_split32<2, 0, 4>(a, b, st);
        case 128: return launch_split32<4, 0, 4>(a, b, st);
        case 256: return launch_split32<8, 0, 4>(a, b, st);
        case 384: return launch_split32<12, 0, 4>(a, b, st);
        default: throw Error{CFD_EARG, "32x32 split-f16 SIREN needs hidden_features in {64, 128, 256, 384}"};
    }
}

bool siren_split_supported(int NB) {
    switch (NB) {
        case 2: case 4: case 6: case 8: case 12: case 16: case 24: return true;
        default: return false;
    }
}

void launch_siren_split(int NB, SirenArgs a, int b, hipStream_t st) {
    switch (NB) {
        case 2: return launch_nb<2>(a, b, st);
        case 4: return launch_nb<4>(a, b, st);
        case 6: return launch_nb<6>(a, b, st);
        case 8: return launch_nb<8>(a, b, st);
        case 12: return launch_nb<12>(a, b, st);
        case 16: return launch_nb<16>(a, b, st);
        case 24: return launch_nb<24>(a, b, st);
        default: throw Error{CFD_EARG, "split-f16 SIREN needs hidden_features = 32*{1,2,3,4,6,8,12,16}"};
    }
}

// ---------------------------------------------------------------------------
// K9t: the tape kernels of the DPS adjoint on split-f16 MFMA (the K-split forms
// of siren_tape_fwd_ks / siren_tape_bwd_ks, siren.hip, with every hidden-layer
// product W x as three v_mfma_f32_16x16x32_f16 on hi/lo halves, K7s's scheme).
// KS waves share one 16-pair tile; wave w owns output blocks [QW w, QW (w + 1))
// and holds exactly those features as its next-layer operand: QW / 2 K-chunks of
// 32 features in the accumulator-as-B k order of pack_split_f16, split once per
// layer.  Per output block every wave multiplies its chunks by the block's
// weights (one block per ring slot, LDS-DMA, fetched one block ahead) and parks
// the partial in LDS.  The epilogue of block j -- the KS partials added in wave
// order (fixed: deterministic, batch invariant), the weight scale undone, the
// FiLM row added, the sine / the cos derivative -- runs in block j + 1 between
// that block's MFMAs (every wave computes it, pinned there; the owner keeps it
// and stores the tape), the FiLM rows / pre-activations of a wave's own blocks
// are loaded once per layer, and each block ends on a bare s_barrier after
// vmcnt(1) -- the tape store stays in flight (memory operations retire in order)
// where __syncthreads' fence would wait for it.
// Operand range: the forward's operands are sines (|x| <= 1).  The backward's
// deltas have no bound, so each wave scales its slice of a pair's deltas by a
// power of two 2^-e (e: exponent of the slice's max |delta|, per pair and per
// wave: a pair's bits never depend on its tile neighbours) before the split and
// multiplies its partial by 2^e -- exact -- so the f16 halves keep 22 bits
// whatever the gradient's scale.
// Lanes past the last pair compute pair P - 1 again (same inputs, same bits), so
// every tape store is issued by every lane and the vmcnt accounting is exact.
// ---------------------------------------------------------------------------
template <int NB, int KS, int RING>
__global__ __launch_bounds__(64 * KS) void siren_tape_fwd_split(SirenTapeArgs p) {
    constexpr int H = NB * 16, BLK = NB * 256, QW = NB / KS, QC = QW / 2;
    static_assert(QW % 2 == 0 && (RING == 2 || RING == 3), "K9t: an even block count per wave");
    extern __shared__ __attribute__((aligned(16))) float smem[];
    // RING ring slots, then 2 x KS x 64 lanes x f4 partial sums: 80 KiB at H = 384, RING = 3
    // (two workgroups per CU)
    float* wbuf = smem;
    float* red = smem + RING * BLK;
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
    const int q0 = wave * QW;
    const int nblocks = nh * NB;

    float cn[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (k < p.d) {
            float v = p.coords[(int64_t)sensor * p.d + k];
            if (p.xmax) v = (v - p.xmin[k]) / (p.xmax[k] - p.xmin[k]) * 2.0f - 1.0f;
            cn[k] = v;
        }
    }
#pragma unroll
    for (int r = 0; r + 1 < RING; ++r)
        if (r < nblocks) siren_issue_block_u<NB, KS>(p.wimg16, r, wbuf + r * BLK, wave, lane);

    float X[QW][4], Xn[QW][4];
    static_for<QW>([&](auto qc) {
        constexpr int qq = decltype(qc)::value;
        const int q = q0 + qq;
        const f4 fv = *(const f4*)(film + 16 * q + 4 * g);
        f4 uu;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float* w = p.w0 + (16 * q + 4 * g + r) * p.d;   // layer 0 (d <= 4 inputs)
            float a = cn[0] * w[0];
#pragma unroll
            for (int k = 1; k < 4; ++k)
                if (k < p.d) a = fmaf(cn[k], w[k], a);
            uu[r] = a + fv[r];
            X[qq][r] = sin_cw(p.w0f * uu[r]);
        }
        *(f4*)(ut + 16 * q + 4 * g) = uu;
    });
    Frag xh[QC], xl[QC];
    auto split_x = [&]() __attribute__((always_inline)) {
        static_for<QC>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            split8(X[2 * i], X[2 * i + 1], xh[i], xl[i]);
        });
    };
    split_x();

    int J = 0;
    for (int layer = 1; layer <= nh; ++layer) {
        const float inv = 1.0f / p.wscale[layer - 1];   // a power of two: exact
        // this wave's FiLM rows of the layer (its own blocks), before the block loop: the
        // loop's only vector-memory operations are then the DMA and the tape store
        f4 fvr[QW];
        static_for<QW>([&](auto qc) {
            constexpr int qq = decltype(qc)::value;
            fvr[qq] = *(const f4*)(film + layer * H + 16 * (q0 + qq) + 4 * g);
        });
        static_for<NB>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            constexpr int jp = j > 0 ? j - 1 : 0;   // the pending block (j > 0)
            const bool own = j > 0 && jp / QW == wave;
            const bool ahead = J + RING - 1 < nblocks;   // block J + RING - 1 fetched now
            if (ahead)
                siren_issue_block_u<NB, KS>(p.wimg16, J + RING - 1, wbuf + ((J + RING - 1) % RING) * BLK, wave, lane);
            const float* wb = wbuf + (J % RING) * BLK;
            h8 wh[QC], wl[QC];
            static_for<QC>([&](auto ic) {
                constexpr int i = decltype(ic)::value;
                const int qg = q0 / 2 + i;
                wh[i] = *(const h8*)(wb + qg * 512 + lane * 4);
                wl[i] = *(const h8*)(wb + qg * 512 + 256 + lane * 4);
            });
            __builtin_amdgcn_sched_barrier(0);
            // the MFMA chain of block j, with the pending block's epilogue between its
            // K-chunks (every wave computes it, the owner keeps it: no branch in the chain)
            f4 a = {0.f, 0.f, 0.f, 0.f}, acc = {0.f, 0.f, 0.f, 0.f};
            float xs[4] = {0.f, 0.f, 0.f, 0.f};
            static_for<QC>([&](auto ic) {
                constexpr int i = decltype(ic)::value;
                a = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl[i], xh[i].h(), a, 0, 0, 0);
                a = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[i], xl[i].h(), a, 0, 0, 0);
                a = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[i], xh[i].h(), a, 0, 0, 0);
                if constexpr (j > 0 && i == 0) {
                    const float* rs = red + (jp & 1) * KS * 256;
                    acc = *(const f4*)(rs + lane * 4);
#pragma unroll
                    for (int w = 1; w < KS; ++w) acc += *(const f4*)(rs + (w * 64 + lane) * 4);
                    asm volatile("" : "+v"(acc));
                }
                if constexpr (j > 0 && i == (QC > 1 ? 1 : 0)) {
                    acc = acc * inv + fvr[jp % QW];
#pragma unroll
                    for (int r = 0; r < 4; ++r) xs[r] = sin_cw(p.w0f * acc[r]);
                    // pinned here, between the MFMAs (else they sink into the owner's branch)
                    asm volatile("" : "+v"(xs[0]), "+v"(xs[1]), "+v"(xs[2]), "+v"(xs[3]), "+v"(acc));
                }
                __builtin_amdgcn_sched_barrier(0);
            });
            if constexpr (j > 0) {
                if (own) {
                    *(f4*)(ut + layer * H + 16 * jp + 4 * g) = acc;
#pragma unroll
                    for (int r = 0; r < 4; ++r) Xn[jp % QW][r] = xs[r];
                }
            }
            *(f4*)(red + (j & 1) * KS * 256 + (wave * 64 + lane) * 4) = a;
            // block J + 1 landed (this wave's pieces; the barrier covers the others') and
            // the partial is in LDS; the owner's tape store may stay in flight.  A bare
            // s_barrier: __syncthreads' fence would wait for that store.
            // in flight at most: the younger block's DMA (RING 3) and the tape store
            if (RING == 3 && ahead) {
                if (own) __builtin_amdgcn_s_waitcnt(vm_lgkm0_imm(QW + 1));
                else __builtin_amdgcn_s_waitcnt(vm_lgkm0_imm(QW));
            } else {
                if (own) __builtin_amdgcn_s_waitcnt(vm_lgkm0_imm(1));
                else __builtin_amdgcn_s_waitcnt(vm_lgkm0_imm(0));
            }
            asm volatile("s_barrier" ::: "memory");
            ++J;
        });
        // the layer's last block, after its barrier
        if ((NB - 1) / QW == wave) {
            constexpr int qq = (NB - 1) % QW;
            const float* rs = red + ((NB - 1) & 1) * KS * 256;
            f4 acc = *(const f4*)(rs + lane * 4);
#pragma unroll
            for (int w = 1; w < KS; ++w) acc += *(const f4*)(rs + (w * 64 + lane) * 4);
            acc = acc * inv + fvr[qq];
            *(f4*)(ut + layer * H + 16 * (NB - 1) + 4 * g) = acc;
#pragma unroll
            for (int r = 0; r < 4; ++r) Xn[qq][r] = sin_cw(p.w0f * acc[r]);
        }
        static_for<QW>([&](auto qc) {
            constexpr int qq = decltype(qc)::value;
#pragma unroll
            for (int r = 0; r < 4; ++r) X[qq][r] = Xn[qq][r];
        });
        if (layer < nh) split_x();
    }

    // output layer in fp32: partial sums over this wave's features, combined in wave order
    // (KS x 4 x 16 sums in the partial-sum slot the last block's epilogue does not read)
    float* osum = red + (NB & 1) * KS * 256;
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
    if (n < p.P && g < p.c) {
        float v = g == 0 ? o[0] : g == 1 ? o[1] : g == 2 ? o[2] : o[3];
        if (p.ymax) {
            const int64_t yi = (int64_t)sensor * p.ystride + g;
            const float hi = p.ymax[yi], lo = p.ymin[yi];
            v = (v + 1.0f) / 2.0f * (hi - lo) + lo;
        }
        p.out[n * p.c + g] = v;
    }
}

template <int NB, int KS, int RING>
__global__ __launch_bounds__(64 * KS) void siren_tape_bwd_split(SirenTapeArgs p) {
    constexpr int H = NB * 16, BLK = NB * 256, QW = NB / KS, QC = QW / 2;
    static_assert(QW % 2 == 0 && (RING == 2 || RING == 3), "K9t: an even block count per wave");
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* wbuf = smem;
    float* red = smem + RING * BLK;      // 2 x KS x 64 lanes x f4
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = lane >> 4, j16 = lane & 15;
    const int64_t n = (int64_t)blockIdx.x * 16 + j16;
    const int64_t nc = n < p.P ? n : p.P - 1;
    const int sensor = (int)(nc % p.Ns);
    const int nh = p.nh, nl = nh + 1;
    const float* ut = p.u + nc * nl * H;
    float* dt = p.delta + nc * nl * H;
    const float w0f = p.w0f;
    const int q0 = wave * QW;
    const int nblocks = nh * NB;

#pragma unroll
    for (int r = 0; r + 1 < RING; ++r)
        if (r < nblocks) siren_issue_block_u<NB, KS>(p.wimg16t, r, wbuf + r * BLK, wave, lane);
    float dy[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int oc = 0; oc < 4; ++oc) {
        if (oc < p.c) {
            float v = p.gout[nc * p.c + oc];
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
        *(f4*)(dt + nh * H + 16 * q + 4 * g) = dd;
    });
    // this wave's slice of a pair's deltas, scaled by 2^-e into [0.5, 1) and split;
    // returns e (0 for an all-zero slice)
    Frag xh[QC], xl[QC];
    auto split_scaled = [&]() __attribute__((always_inline)) -> int {
        float m = 0.f;
        static_for<QW>([&](auto qc) {
            constexpr int qq = decltype(qc)::value;
#pragma unroll
            for (int r = 0; r < 4; ++r) m = fmaxf(m, fabsf(X[qq][r]));
        });
        m = fmaxf(m, __shfl_xor(m, 16));
        m = fmaxf(m, __shfl_xor(m, 32));
        const int e = m > 0.f ? __builtin_amdgcn_frexp_expf(m) : 0;
        static_for<QC>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            float x0[4], x1[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                x0[r] = __builtin_amdgcn_ldexpf(X[2 * i][r], -e);
                x1[r] = __builtin_amdgcn_ldexpf(X[2 * i + 1][r], -e);
            }
            split8(x0, x1, xh[i], xl[i]);
        });
        return e;
    };

    int J = 0;
    for (int layer = nh; layer >= 1; --layer) {
        const int li = layer - 1;
        const int e = split_scaled();
        const float inv = 1.0f / p.wscale[li];   // a power of two: exact
        f4 uur[QW];   // this wave's pre-activations of the layer (its own blocks)
        static_for<QW>([&](auto qc) {
            constexpr int qq = decltype(qc)::value;
            uur[qq] = *(const f4*)(ut + li * H + 16 * (q0 + qq) + 4 * g);
        });
        static_for<NB>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            constexpr int jp = j > 0 ? j - 1 : 0;
            const bool own = j > 0 && jp / QW == wave;
            const bool ahead = J + RING - 1 < nblocks;   // block J + RING - 1 fetched now
            if (ahead)
                siren_issue_block_u<NB, KS>(p.wimg16t, J + RING - 1, wbuf + ((J + RING - 1) % RING) * BLK, wave, lane);
            const float* wb = wbuf + (J % RING) * BLK;
            h8 wh[QC], wl[QC];
            static_for<QC>([&](auto ic) {
                constexpr int i = decltype(ic)::value;
                const int qg = q0 / 2 + i;
                wh[i] = *(const h8*)(wb + qg * 512 + lane * 4);
                wl[i] = *(const h8*)(wb + qg * 512 + 256 + lane * 4);
            });
            __builtin_amdgcn_sched_barrier(0);
            f4 a = {0.f, 0.f, 0.f, 0.f}, acc = {0.f, 0.f, 0.f, 0.f}, dd = {0.f, 0.f, 0.f, 0.f};
            static_for<QC>([&](auto ic) {
                constexpr int i = decltype(ic)::value;
                a = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl[i], xh[i].h(), a, 0, 0, 0);
                a = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[i], xl[i].h(), a, 0, 0, 0);
                a = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[i], xh[i].h(), a, 0, 0, 0);
                if constexpr (j > 0 && i == 0) {
                    const float* rs = red + (jp & 1) * KS * 256;
                    acc = *(const f4*)(rs + lane * 4);
#pragma unroll
                    for (int w = 1; w < KS; ++w) acc += *(const f4*)(rs + (w * 64 + lane) * 4);
                    asm volatile("" : "+v"(acc));
                }
                if constexpr (j > 0 && i == (QC > 1 ? 1 : 0)) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) dd[r] = acc[r] * (w0f * cos_cw(w0f * uur[jp % QW][r]));
                    asm volatile("" : "+v"(dd));
                }
                __builtin_amdgcn_sched_barrier(0);
            });
            if constexpr (j > 0) {
                if (own) {
                    *(f4*)(dt + li * H + 16 * jp + 4 * g) = dd;
#pragma unroll
                    for (int r = 0; r < 4; ++r) Xn[jp % QW][r] = dd[r];
                }
            }
            // back to the deltas' own scale: x 2^e / s (exact)
#pragma unroll
            for (int r = 0; r < 4; ++r) a[r] = __builtin_amdgcn_ldexpf(a[r] * inv, e);
            *(f4*)(red + (j & 1) * KS * 256 + (wave * 64 + lane) * 4) = a;
            // in flight at most: the younger block's DMA (RING 3) and the tape store
            if (RING == 3 && ahead) {
                if (own) __builtin_amdgcn_s_waitcnt(vm_lgkm0_imm(QW + 1));
                else __builtin_amdgcn_s_waitcnt(vm_lgkm0_imm(QW));
            } else {
                if (own) __builtin_amdgcn_s_waitcnt(vm_lgkm0_imm(1));
                else __builtin_amdgcn_s_waitcnt(vm_lgkm0_imm(0));
            }
            asm volatile("s_barrier" ::: "memory");
            ++J;
        });
        if ((NB - 1) / QW == wave) {
            constexpr int qq = (NB - 1) % QW;
            const float* rs = red + ((NB - 1) & 1) * KS * 256;
            f4 acc = *(const f4*)(rs + lane * 4);
#pragma unroll
            for (int w = 1; w < KS; ++w) acc += *(const f4*)(rs + (w * 64 + lane) * 4);
            f4 dd;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                dd[r] = acc[r] * (w0f * cos_cw(w0f * uur[qq][r]));
                Xn[qq][r] = dd[r];
            }
            *(f4*)(dt + li * H + 16 * (NB - 1) + 4 * g) = dd;
        }
        static_for<QW>([&](auto qc) {
            constexpr int qq = decltype(qc)::value;
#pragma unroll
            for (int r = 0; r < 4; ++r) X[qq][r] = Xn[qq][r];
        });
    }
}

namespace {
// RING 3: two blocks' DMA ahead of the MFMAs (80 KiB of LDS at H = 384: still two
// workgroups per CU).  Measured per DPS step (tools/dev/tape_bench.py, one box):
// against RING 2 the VJP 0.41 -> 0.35 ms (config D) and 0.31 -> 0.25 ms (Case4);
// two 16-pair tiles per workgroup (every weight fragment read feeding two MFMA
// chains) measured no faster at D and 25 % slower at Case4 (half the workgroups).
template <int NB, int KS>
void launch_tape_split_nb(const SirenTapeArgs& a, bool bwd, hipStream_t st) {
    constexpr int RING = 3;
    const size_t lds = sizeof(float) * ((size_t)RING * NB * 256 + 2 * KS * 256);
    const void* fn = bwd ? (const void*)siren_tape_bwd_split<NB, KS, RING> : (const void*)siren_tape_fwd_split<NB, KS, RING>;
    CFD_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const dim3 grid((unsigned)ceil_div(a.P, 16));
    if (bwd)
        hipLaunchKernelGGL((siren_tape_bwd_split<NB, KS, RING>), grid, dim3(64 * KS), lds, st, a);
    else
        hipLaunchKernelGGL((siren_tape_fwd_split<NB, KS, RING>), grid, dim3(64 * KS), lds, st, a);
    check_launch(bwd ? "siren_tape_bwd_split" : "siren_tape_fwd_split");
}
}  // namespace

// K9t takes 4 waves per tile where 4 divides the block count into even shares
bool tape_split_supported(int NB) { return NB == 8 || NB == 16 || NB == 24; }

void launch_tape_split(int NB, const SirenTapeArgs& a, bool bwd, hipStream_t st) {
    CFD_REQUIRE(a.wimg16 && a.wimg16t && a.wscale, CFD_ESTATE, "internal: split tape images not set");
    switch (NB) {
        case 8: return launch_tape_split_nb<8, 4>(a, bwd, st);
        case 16: return launch_tape_split_nb<16, 4>(a, bwd, st);
        case 24: return launch_tape_split_nb<24, 4>(a, bwd, st);
        default: throw Error{CFD_EARG, "split-f16 tape needs hidden_features in {128, 256, 384}"};
    }
}

__global__ void sine_probe_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t n, int which) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n)
        y[i] = which == 4   ? hidden_sine<4>(x[i])
               : which == 3 ? hidden_sine<3>(x[i])
               : which == 2 ? sin_hw_rev(x[i])
               : which == 1 ? sin_hw(x[i])
                            : sin1_cw(x[i]);
}

}  // namespace cfd

extern "C" int cfd_sine_probe(const float* x, float* y, int64_t n, int which, void* stream) {
    return cfd::guard([&] {
        CFD_REQUIRE(x && y && n > 0 && which >= 0 && which <= 4, CFD_EARG, "bad argument");
        hipLaunchKernelGGL(cfd::sine_probe_kernel, dim3((unsigned)cfd::ceil_div(n, 256)), dim3(256), 0,
                           (hipStream_t)stream, x, y, n, which);
        cfd::check_launch("sine_probe_kernel");
    });
}
