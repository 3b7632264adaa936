// K1x: split-f16 implicit-GEMM convolution on v_mfma_f32_32x32x16_f16 with
// 64x64 wave tiles and an in-workgroup K split (gfx950).
//
// Same GEMM view, operands and numerics as conv_gemm_kernel<..., MODE=2> (K1s,
// unet_kernels.hip): M = B*Hout*Wout output pixels, N = Cout, K = ks*ks*Ctot
// ordered (tap, channel); activations split x = xh + xl (f16 RNE) as they are
// staged; weights pre-split (s w) = wh + wl; each product as wl.xh + wh.xl +
// wh.xh with fp32 accumulation -- fp32-level error against fp64.
//
// What changes is the shape of the work, for the MFMA/LDS budget of a CU:
//   * 32x32x16 MFMAs on 64x64 wave tiles: per 16-deep K sub-step a wave reads
//     2+2 (hi, lo) A and B fragments (8 ds_read_b128) for 12 MFMAs of 32 cycles;
//     K1s' 16x16x32 on 32x64 tiles reads 12 per 384 MFMA cycles -- 2x the LDS
//     bytes per FLOP, and LDS, not the matrix pipe, bounded it;
//   * KG wave groups split each workgroup's K range (group g takes K tiles
//     g, g+KG, ...) and meet once through LDS at the end: KG x the waves per
//     SIMD for latency hiding without split-K partial slabs in HBM.  The two
//     partial sums are added in a fixed order (group 0 + group 1), so every
//     output's summation order depends on the per-sample shape only (batch
//     invariance, as split-K).
// LDS rows are 32 f16 (64 B); the 16-B chunk c of row r sits in slot
// c ^ ((r >> 2) & 3): every 16-lane group of a 32x32x16 fragment read
// (ds_read_b128, lanes 0-31 rows 0-31 chunk 2s, lanes 32-63 chunk 2s+1) then
// covers the 64 banks once; the 8-B staging writes stay conflict-free.
#include <algorithm>
#include <type_traits>

#include "unet_kernels.hpp"

namespace cfd {

typedef float f16v __attribute__((ext_vector_type(16)));
typedef float f2 __attribute__((ext_vector_type(2)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef unsigned u4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int xswz(int row, int chunk) { return row * 64 + ((chunk ^ ((row >> 2) & 3)) << 4); }

// hi = f16(x) (RNE, packed convert), lo = f16(x - hi) by v_fma_mix, 4 values
__device__ __forceinline__ void split4_mix_x(const f4& x, uint2& hi, uint2& lo) {
    hi.x = __builtin_bit_cast(unsigned, __builtin_convertvector((f2){x[0], x[1]}, h2));
    hi.y = __builtin_bit_cast(unsigned, __builtin_convertvector((f2){x[2], x[3]}, h2));
    asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=&v"(lo.x) : "v"(x[0]), "v"(hi.x));
    asm("v_fma_mixhi_f16 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "+v"(lo.x) : "v"(x[1]), "v"(hi.x));
    asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=&v"(lo.y) : "v"(x[2]), "v"(hi.y));
    asm("v_fma_mixhi_f16 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "+v"(lo.y) : "v"(x[3]), "v"(hi.y));
}

// PF: tiles in flight through registers (1: the next tile; 2: two ahead, two
// register sets -- for short per-workgroup K ranges where one tile of compute
// does not cover a load's latency).
// XF: a fused 1x1 skip convolution (ConvArgs::xsrc1): K tiles past the 3x3 taps'
// (the "tap" ks * ks) take the raw block input at the output pixel and the skip
// weights -- [taps | x] as one GEMM, in the same split-K ranges
// BF (config E): bf16 operands (the activations rounded RNE as they are staged,
// weights from the bf16 arena), one v_mfma_f32_32x32x16_bf16 per product, one
// plane per operand -- the 3x3 convolutions K1hb's halo tiles do not cover (8^2)
template <int BM, int BN, int WGM, int WGN, int KG, int PF = 1, bool XF = false, bool BF = false>
__global__ __launch_bounds__(64 * WGM * WGN * KG, 1) void conv_x_kernel(ConvArgs a) {
    static_assert(!(XF && BF), "fused skip convolution: split compute");
    constexpr int NW = WGM * WGN * KG, NT = 64 * NW;
    constexpr int WTM = BM / WGM, WTN = BN / WGN;   // wave tile
    constexpr int TM = WTM / 32, TN = WTN / 32;     // 32x32 blocks per wave
    constexpr int RPP = NT / 8;                     // row-slices staged per pass (8 threads x 4 k)
    constexpr int AIT = BM * KG / RPP, BIT = BN * KG / RPP;
    static_assert(TM >= 1 && TN >= 1 && AIT >= 1 && BIT >= 1, "tile");
    static_assert((BM * KG) % RPP == 0 && (BN * KG) % RPP == 0, "staging");
    constexpr int ABYTES = BM * KG * 64, BBYTES = BN * KG * 64;    // one f16 plane
    constexpr int PLN = BF ? 1 : 2;                                // planes per operand
    constexpr int STAGE = PLN * ABYTES + PLN * BBYTES;             // A hi, A lo, B hi, B lo (BF: A, B)
    __shared__ __attribute__((aligned(16))) char lds[2 * STAGE];

    CFD_STAMP(a.stamps, 2, a.seq, 0);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int kg = wave / (WGM * WGN), wrem = wave % (WGM * WGN);
    const int wm = wrem / WGN, wn = wrem % WGN;

    int bx, by, bz;
    xcd_tile(a.xcd, bx, by, bz);
    const int m0 = bx * BM, n0 = by * BN;
    const int HWo = a.Hout * a.Wout;
    const int kq = tid & 7, rsub = tid >> 3;
    __shared__ int pixtab[9 * BM];   // source pixel of (tap, tile row), -1: padding

    // buffer resources (32-bit offsets; launch_conv_x checks they fit)
    const int srows = __builtin_amdgcn_readfirstlane(a.Hin * a.Win * (a.M / HWo));   // SGPR: a VGPR descriptor field costs a readfirstlane loop per load
    const __amdgpu_buffer_rsrc_t rs1 = __builtin_amdgcn_make_buffer_rsrc((void*)a.src1, 0, srows * a.C1 * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t rs2 = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(a.src2 ? (const void*)a.src2 : (const void*)a.src1), 0, a.src2 ? srows * a.C2 * 4 : 0, 0x00020000);
    const int ntap = a.ks * a.ks, KM = ntap * a.Ctot;   // the taps' K (XF: the skip part follows)
    const __amdgpu_buffer_rsrc_t rwh = __builtin_amdgcn_make_buffer_rsrc((void*)a.wbf, 0, a.Cout * KM * 2, 0x00020000);
    const __amdgpu_buffer_rsrc_t rwl = __builtin_amdgcn_make_buffer_rsrc((void*)a.wlo, 0, a.Cout * KM * 2, 0x00020000);
    __amdgpu_buffer_rsrc_t rx1 = rs1, rx2 = rs1, rxh = rwh, rxl = rwl;
    // the skip part's fields as locals: a select between two fields of `a` would
    // take the kernel argument's address and copy it to scratch
    const int XC1 = a.XC1, XC2 = a.XC2;
    const float xscale = a.x_scale, mscale = a.main_scale;
    if constexpr (XF) {
        const int XC = XC1 + XC2, mrows = __builtin_amdgcn_readfirstlane(a.M);
        rx1 = __builtin_amdgcn_make_buffer_rsrc((void*)a.xsrc1, 0, mrows * a.XC1 * 4, 0x00020000);
        rx2 = __builtin_amdgcn_make_buffer_rsrc((void*)(a.xsrc2 ? (const void*)a.xsrc2 : (const void*)a.xsrc1), 0,
                                                a.xsrc2 ? mrows * a.XC2 * 4 : 0, 0x00020000);
        rxh = __builtin_amdgcn_make_buffer_rsrc((void*)a.xwbf, 0, a.Cout * XC * 2, 0x00020000);
        rxl = __builtin_amdgcn_make_buffer_rsrc((void*)a.xwlo, 0, a.Cout * XC * 2, 0x00020000);
    }
    {
        const float rhw = 1.0f / (float)HWo, rw = 1.0f / (float)a.Wout;   // fdiv24 (M < 2^24: launch_conv_x)
        for (int e = tid; e < ntap * BM; e += NT) {
            const int tap = e / BM, r = e - tap * BM;
            const int ty = tap_row(tap, a.ks), tx = tap - ty * a.ks;
            const int m = m0 + r;
            int pix = -1;
            if (m < a.M) {
                const int b = fdiv24(m, HWo, rhw), rem = m - b * HWo;
                const int oy = fdiv24(rem, a.Wout, rw), ox = rem - oy * a.Wout;
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
                if (ok) pix = (b * a.Hin + iy) * a.Win + ix;
            }
            CFD_DASSERT(pix < srows);
            pixtab[e] = pix;
        }
    }

    // staged row-slices: A (tile row, group g), B (output channel, group g)
    int a_g[AIT], a_row[AIT], a_m[AIT];
#pragma unroll
    for (int it = 0; it < AIT; ++it) {
        const int rs = rsub + it * RPP;
        a_g[it] = rs / BM;
        a_row[it] = rs;
        a_m[it] = rs % BM;
    }
    int b_g[BIT], b_row[BIT];
    unsigned b_voff[BIT], bx_voff[BIT];
#pragma unroll
    for (int it = 0; it < BIT; ++it) {
        const int rs = rsub + it * RPP;
        b_g[it] = rs / BN;
        b_row[it] = rs;
        const int n = n0 + rs % BN;
        b_voff[it] = n < a.Cout ? (unsigned)((n * KM + 4 * kq) * 2) : 0x80000000u;
        bx_voff[it] = XF && n < a.Cout ? (unsigned)((n * (a.XC1 + a.XC2) + 4 * kq) * 2) : 0x80000000u;
    }

    const int nkt = a.K / 32;
    const int per = (nkt + gridDim.z - 1) / gridDim.z;
    const int kt0 = bz * per;
    const int kt1 = min(nkt, kt0 + per);
    // per-group K position (tap, channel base) of tile kt0 + g, advanced by KG tiles
    int cbg[KG], tpg[KG];
#pragma unroll
    for (int g = 0; g < KG; ++g) {
        const int kb = (kt0 + g) * 32;
        // tap ntap (XF): the skip part, channel kb - KM of the block input
        const int tp = XF && kb >= KM ? ntap : kb / a.Ctot;
        tpg[g] = __builtin_amdgcn_readfirstlane(tp);   // SGPRs: scalar descriptor choice
        cbg[g] = __builtin_amdgcn_readfirstlane(kb - tp * a.Ctot);
    }
    __syncthreads();   // pixtab

    f4 ra[PF][AIT];
    uint2 rbh[PF][BIT], rbl[PF][BIT];
    float lsc[PF][KG];   // XF: the staging scale of each group's tile (main_scale / x_scale)
    auto load_tile = [&](int kt, int set) __attribute__((always_inline)) {   // tiles kt + g, g < KG, into register set `set`
#pragma unroll
        for (int it = 0; it < AIT; ++it) {
            const int g = KG == 1 ? 0 : a_g[it];   // KG = 1: a constant (a runtime index puts tpg / cbg in scratch)
            const int cb = cbg[g];
            bool xt = false;
            if constexpr (XF) xt = tpg[g] == ntap;
            if (xt) {   // the skip part (XF): the block input at the output pixel itself
                const bool second = cb >= XC1;
                const unsigned csrc4 = 4u * (second ? XC2 : XC1);
                const unsigned cofs4 = 4u * ((second ? cb - XC1 : cb) + 4 * kq);
                const int m = m0 + a_m[it];
                const unsigned off = kt + g < kt1 && m < a.M ? __umul24((unsigned)m, csrc4) + cofs4 : 0x80000000u;
                ra[set][it] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(second ? rx2 : rx1, off, 0, 0));
            } else {
            const bool second = cb >= a.C1;
            const unsigned csrc4 = 4u * (second ? a.C2 : a.C1);
            const unsigned cofs4 = 4u * ((second ? cb - a.C1 : cb) + 4 * kq);
            const int pix = kt + g < kt1 ? pixtab[tpg[g] * BM + a_m[it]] : -1;
            const unsigned off = pix >= 0 ? __umul24((unsigned)pix, csrc4) + cofs4 : 0x80000000u;
            ra[set][it] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(second ? rs2 : rs1, off, 0, 0));
            }
        }
#pragma unroll
        for (int it = 0; it < BIT; ++it) {
            const int g = KG == 1 ? 0 : b_g[it];
            bool xt = false;
            if constexpr (XF) xt = tpg[g] == ntap;
            if (xt) {
                const unsigned voff = kt + g < kt1 ? bx_voff[it] : 0x80000000u;
                rbh[set][it] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rxh, voff, cbg[g] * 2, 0));
                rbl[set][it] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rxl, voff, cbg[g] * 2, 0));
            } else {
                const unsigned voff = kt + g < kt1 ? b_voff[it] : 0x80000000u;
                const int soff = (tpg[g] * a.Ctot + cbg[g]) * 2;
                rbh[set][it] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rwh, voff, soff, 0));
                if constexpr (!BF)
                    rbl[set][it] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rwl, voff, soff, 0));
            }
        }
#pragma unroll
        for (int g = 0; g < KG; ++g) {
            if constexpr (XF) lsc[set][g] = tpg[g] == ntap ? xscale : mscale;
            cbg[g] += 32 * KG;
            while (cbg[g] >= a.Ctot && tpg[g] < ntap) {   // past the last tap: the skip part (XF)
                cbg[g] -= a.Ctot;
                ++tpg[g];
            }
        }
    };
    auto store_tile = [&](int buf, int set) __attribute__((always_inline)) {
        char* base = lds + buf * STAGE;
#pragma unroll
        for (int it = 0; it < AIT; ++it) {
            const int off = xswz(a_row[it], kq >> 1) + (kq & 1) * 8;
            if constexpr (BF) {   // bf16 RNE (v_cvt_pk_bf16_f32), as the K1s bf16 tiles
                *(bf16x4*)(base + off) = __builtin_convertvector(ra[set][it], bf16x4);
                continue;
            }
            uint2 hv, lv;
            if constexpr (XF)
                split4_mix_x(ra[set][it] * lsc[set][KG == 1 ? 0 : a_g[it]], hv, lv);   // the common scale (exact)
            else
                split4_mix_x(ra[set][it], hv, lv);
            *(uint2*)(base + off) = hv;
            *(uint2*)(base + ABYTES + off) = lv;
        }
#pragma unroll
        for (int it = 0; it < BIT; ++it) {
            const int off = xswz(b_row[it], kq >> 1) + (kq & 1) * 8;
            *(uint2*)(base + PLN * ABYTES + off) = rbh[set][it];
            if constexpr (!BF) *(uint2*)(base + 2 * ABYTES + BBYTES + off) = rbl[set][it];
        }
    };

    f16v acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    const int l32 = lane & 31, hsel = lane >> 5;
    const int arow0 = kg * BM + wm * WTM + l32, brow0 = kg * BN + wn * WTN + l32;
    // one K step (tiles kt + g): prefetch the tiles PF steps ahead into register
    // set `lset`, MFMAs on LDS stage `cur`, then stage the next step's tiles
    // (register set `sset`, loaded PF - 1 steps ago) into the other LDS stage
    auto kstep = [&](int kt, int cur, int lset, int sset) __attribute__((always_inline)) {
            const bool more = kt + KG < kt1;
            if (kt + PF * KG < kt1) load_tile(kt + PF * KG, lset);
            const char* base = lds + cur * STAGE;
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const int ch = 2 * s + hsel;
                if constexpr (BF) {
                    bf16x8 fa[TM], fb[TN];
#pragma unroll
                    for (int i = 0; i < TM; ++i) fa[i] = *(const bf16x8*)(base + xswz(arow0 + 32 * i, ch));
#pragma unroll
                    for (int j = 0; j < TN; ++j) fb[j] = *(const bf16x8*)(base + ABYTES + xswz(brow0 + 32 * j, ch));
#pragma unroll
                    for (int i = 0; i < TM; ++i)
#pragma unroll
                        for (int j = 0; j < TN; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
                    continue;
                }
                h8v fah[TM], fal[TM], fbh[TN], fbl[TN];
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    const int off = xswz(arow0 + 32 * i, ch);
                    fah[i] = *(const h8v*)(base + off);
                    fal[i] = *(const h8v*)(base + ABYTES + off);
                }
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int off = xswz(brow0 + 32 * j, ch);
                    fbh[j] = *(const h8v*)(base + 2 * ABYTES + off);
                    fbl[j] = *(const h8v*)(base + 2 * ABYTES + BBYTES + off);
                }
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j) {
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fal[i], fbh[j], acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fah[i], fbl[j], acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fah[i], fbh[j], acc[i][j], 0, 0, 0);
                    }
            }
            if (more) store_tile(cur ^ 1, sset);
            __syncthreads();
    };
    if (kt0 < kt1) {
        load_tile(kt0, 0);
        if constexpr (PF == 2) {
            if (kt0 + KG < kt1) load_tile(kt0 + KG, 1);
        }
        store_tile(0, 0);
        __syncthreads();
        CFD_STAMP(a.stamps, 2, a.seq, 2);
        if constexpr (PF == 1) {
            int cur = 0;
            for (int kt = kt0; kt < kt1; kt += KG) {
                kstep(kt, cur, 0, 0);
                cur ^= 1;
            }
        } else {
            for (int kt = kt0; kt < kt1; kt += 2 * KG) {
                kstep(kt, 0, 0, 1);
                if (kt + KG < kt1) kstep(kt + KG, 1, 1, 0);
            }
        }
    }

    CFD_STAMP(a.stamps, 2, a.seq, 3);
    // combine the K groups through LDS: groups 1.. park their sums, group 0 adds
    // them in group order (fixed summation order)
    if constexpr (KG > 1) {
        float* red = (float*)lds;   // (KG-1) x WGM*WGN waves x TM*TN*16 floats x 64 lanes
        constexpr int PER_WAVE = TM * TN * 16 * 64;
        static_assert((size_t)(KG - 1) * WGM * WGN * PER_WAVE * 4 <= 2 * STAGE, "reduction fits in the stages");
        if (kg > 0) {
            float* dst = red + ((kg - 1) * WGM * WGN + wrem) * PER_WAVE;
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
#pragma unroll
                    for (int e = 0; e < 16; e += 4)
                        *(f4*)(dst + ((i * TN + j) * 16 + e) * 64 + 4 * lane) =
                            f4{acc[i][j][e], acc[i][j][e + 1], acc[i][j][e + 2], acc[i][j][e + 3]};
        }
        __syncthreads();
        if (kg > 0) return;
#pragma unroll
        for (int g = 1; g < KG; ++g) {
            const float* src = red + ((g - 1) * WGM * WGN + wrem) * PER_WAVE;
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
#pragma unroll
                    for (int e = 0; e < 16; e += 4) {
                        const f4 v = *(const f4*)(src + ((i * TN + j) * 16 + e) * 64 + 4 * lane);
                        acc[i][j][e] += v[0];
                        acc[i][j][e + 1] += v[1];
                        acc[i][j][e + 2] += v[2];
                        acc[i][j][e + 3] += v[3];
                    }
        }
    }

    // undo the power-of-two weight scale (exact); epilogue as conv_gemm_kernel
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] *= a.acc_scale;
    const int n_base = n0 + wn * WTN + l32;
    const int m_base = m0 + wm * WTM + 4 * hsel;
    if (gridDim.z > 1) {
        float* part = a.part + (int64_t)bz * a.M * a.Cout;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int m = m_base + 32 * i + 8 * (e >> 2) + (e & 3);
                if (m >= a.M) continue;
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int n = n_base + 32 * j;
                    if (n < a.Cout) part[(int64_t)m * a.Cout + n] = acc[i][j][e];
                }
            }
#ifdef CFD_STAMPS
        __builtin_amdgcn_s_waitcnt(0);
#endif
        CFD_STAMP(a.stamps, 2, a.seq, 4);
        return;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int m = m_base + 32 * i + 8 * (e >> 2) + (e & 3);
            if (m >= a.M) continue;
            const int bb = m / HWo;
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int n = n_base + 32 * j;
                if (n >= a.Cout) continue;
                float v = a.bias ? acc[i][j][e] + a.bias[n] : acc[i][j][e];
                if (XF && a.bias2) v = v + a.bias2[n];
                if (a.emb) v = v + a.emb[(int64_t)bb * a.emb_stride + n];
                if (a.res) v = a.res[(int64_t)m * a.Cout + n] + v;
                a.out[(int64_t)m * a.Cout + n] = v;
            }
        }
}

// ---------------------------------------------------------------------------
// K1h: halo-tiled 3x3 stride-1 convolution (optionally on a nearest-2x
// upsampled input).  A workgroup's BM output pixels are a TR x TW block
// (TR = BM / TW rows of TW columns, TW dividing the image width) of one sample;
// per 32-channel chunk a wave group stages the (TR + 2) x (TW + 2) input halo
// once (split to hi/lo f16 on the way into LDS) and runs the 9 taps as shifted
// views of it, so an activation is fetched once per chunk instead of once per
// tap (K1x/K1s gather the 9 im2col rows separately: 4.4x / 5.8x the activation
// bytes at BM = 128 / 256 on a 64-wide image).  Weights stream per (chunk, tap)
// through a 2-stage LDS ring, fetched two steps ahead (two register sets).  The
// next chunk's halo is loaded into registers at tap 0 and written after tap 8
// (one extra barrier per chunk), so the halo needs one LDS stage.
//
// KG wave groups (BM/32 waves each, own halo and weight ring) take the
// chunks of the workgroup's range round-robin and meet once through LDS at the
// end, group 0 adding the others' sums in group order: an in-workgroup K split
// with no partial slab in HBM (split-K over workgroups, gridDim.z, still
// composes with it).  K order is (chunk, tap) per group -- every output's
// summation order is a function of the per-sample shape only, as K1x's.  The
// planner ships BM = 256, KG = 1: 128-pixel blocks in 2 groups measured
// 0.83-1.07x of it on the config-B shapes, their weight slices serving half the
// pixels, so the split-K slab they avoid does not pay for itself (that variant
// and K1y, an LDS-DMA ring, 0.75-0.84x, were removed in round 3).
//
// Measured and not kept (tools/convbench): fragment reads software-
// pipelined across steps (3-stage ring, 2 halo stages): no change; the timing
// experiments (no global loads / no per-step LDS reads / no barriers / no LDS
// stores, wrong results) reach 1.0-1.1 / 1.1 / 1.05 / 1.2 / all four 1.3x --
// the MFMA chain alone runs at ~430 TF fp32-equivalent on random data at the
// clock the chip holds under it, ~0.52 of the 2.4 GHz split-f16 peak.
// BF (config E, K1hb): bf16 operands -- the halo rounded to bf16 (RNE) as it is
// staged, weights from the bf16 arena (a.wbf, a.wlo null) -- one
// v_mfma_f32_32x32x16_bf16 per product, one halo plane and one weight plane.
// SB (with BF; a.src_bf16): the source already holds those bf16 values (a
// GroupNorm's out_bf16 output, rounded by the same conversion): 8-byte halo
// pieces (4 channels of 2 bytes, byte offset 2 * (pixel * C + channel)) are
// copied to LDS as they are -- half the activation bytes, the same bits.
// BN: output channels per workgroup, 128 (two wave columns) or 64 (one: at small
// batch twice the workgroups, one wave per SIMD -- the same tiles' sums)
// OCC: waves per SIMD the register allocation must allow (launch bound) -- 4 lets
// two 8-wave K1hb workgroups share a CU where the grid has more than one per CU
// XF: a fused 1x1 skip convolution (ConvArgs::xsrc1, split compute, KG = 1): after
// the halo rounds the workgroup runs one step per 32-channel chunk of the raw
// block input, read at the tile's own pixels (no halo) into a double buffer of
// its own, two chunks ahead in registers, against the skip weights in the same
// ring -- the ResBlock's skip(x) + h as one GEMM over [h taps | x], no skip tensor
// written or re-read and no launch of its own.  The split-K range of the X chunks
// follows the halo chunks' (same split count); each output's summation order is
// a function of the per-sample shape only.
template <int BM, int TW, int KG = 1, bool BF = false, bool SB = false, int BN = 128, int OCC = 1, bool XF = false>
__global__ __launch_bounds__(BM * (BN / 64) * KG, OCC) void conv_h_kernel(ConvArgs a) {
    static_assert(!SB || BF, "a bf16 source needs the bf16 kernel");
    static_assert(!XF || (KG == 1 && !BF), "fused skip convolution: split compute, one K group");
    constexpr unsigned SES = SB ? 2u : 4u;   // source element bytes
    constexpr int WGN = BN / 64, WGM = BM / 64, NTG = 64 * WGM * WGN;   // threads per K group (the workgroup: NTG * KG)
    static_assert(BN == 64 || BN == 128, "K1h: 64 or 128 output channels per workgroup");
    constexpr int PL = BF ? 1 : 2;                                 // operand planes: bf16, or f16 hi + lo
    // halo row stride HW2: TW + 2 columns, padded to a multiple of 4 where a
    // 32-pixel fragment block spans two tile rows (TW = 16), so the second row's
    // lanes keep the swizzle's bank pattern (PMC: 0.25 LDS bank-conflict rate
    // unpadded); the pad columns load as zeros and are never read
    constexpr int HW2 = TW < 32 ? (TW + 2 + 3) / 4 * 4 : TW + 2;
    constexpr int TR = BM / TW, NPX = (TR + 2) * HW2;
    // halo LDS offset of 16-B chunk `chunk` of halo pixel px in halo row hr: the
    // xswz swizzle, and at TW = 16 (a 32-pixel fragment block spans two halo rows
    // 20 pixels apart) the chunk rotation also takes the row, (px/4 + 3 hr) mod 4, so
    // that the two rows' pixels of one ds_read_b128 lane group fall in different
    // bank slots (PMC: 0.24 LDS bank-conflict rate with xswz alone)
    auto hswz = [](int px, int hr, int chunk) __attribute__((always_inline)) {
        if constexpr (TW == 16) return px * 64 + ((chunk ^ (((px >> 2) + 3 * hr) & 3)) << 4);
        else return xswz(px, chunk);
    };
    constexpr int HPLANE = NPX * 64;                  // one f16 plane of the halo (64 B per pixel)
    constexpr int HIT = (NPX * 8 + NTG - 1) / NTG;    // 16-B halo pieces per thread
    // TG taps per step: the bf16 form (one MFMA per product) takes a kernel row of 3
    // taps per step and ring slot, so each barrier is amortised over as many MFMAs as
    // a split-f16 step's (3 per product, one tap); the split form keeps one tap
    constexpr int TG = BF ? 3 : 1, SPR = 9 / TG;   // taps per step, steps per chunk
    constexpr int BPLANE = BN * 64, BSTAGE = PL * BPLANE * TG;
    constexpr int BIT = BN * 4 / NTG;                 // 16-B weight pieces per thread and plane
    constexpr int GBYTES = PL * HPLANE + 2 * BSTAGE;  // one group's halo + weight ring
    static_assert(BM % TW == 0 && BIT >= 1, "tile");
    constexpr int RED = (KG - 1) * WGM * WGN * 4 * 16 * 64 * 4;   // parked sums of groups 1..
    constexpr int LMAIN = KG * GBYTES > RED ? KG * GBYTES : RED;
    constexpr int XBYTES = BM * 64 * 2;                            // one X chunk: hi + lo planes
    __shared__ __attribute__((aligned(16))) char lds[LMAIN + (XF ? 2 * XBYTES : 0)];

    CFD_STAMP(a.stamps, 3, a.seq, 0);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int kg = wave / (WGM * WGN), wrem = wave % (WGM * WGN);
    const int wm = wrem / WGN, wn = wrem % WGN;
    const int gt = tid - kg * NTG;   // thread index within the group
    char* const halo = lds + kg * GBYTES;
    char* const ring = halo + PL * HPLANE;
    int bx, by, bz;
    xcd_tile(a.xcd, bx, by, bz);
    const int n0 = by * BN;
    const int W = a.Wout, HWo = a.Hout * W;
    // tile bx -> sample, block row, block column (row-major blocks in a sample)
    const int tps = HWo / BM, tpr = W / TW;
    const int bimg = bx / tps, tl = bx - bimg * tps;
    const int y0 = (tl / tpr) * TR, x0 = (tl - (tl / tpr) * tpr) * TW;
    const int64_t mrow0 = (int64_t)bimg * HWo + (int64_t)y0 * W + x0;   // output pixel of tile position (0, 0)
    CFD_DASSERT(mrow0 + (int64_t)(TR - 1) * W + TW <= a.M && HWo % BM == 0 && W % TW == 0);

    // SGPR descriptor fields: a VGPR one costs a readfirstlane loop around every load
    const int srows = __builtin_amdgcn_readfirstlane(a.Hin * a.Win * (a.M / HWo));
    const __amdgpu_buffer_rsrc_t rs1 = __builtin_amdgcn_make_buffer_rsrc((void*)a.src1, 0, srows * a.C1 * SES, 0x00020000);
    const __amdgpu_buffer_rsrc_t rs2 = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(a.src2 ? (const void*)a.src2 : (const void*)a.src1), 0, a.src2 ? srows * a.C2 * SES : 0, 0x00020000);
    const __amdgpu_buffer_rsrc_t rwh = __builtin_amdgcn_make_buffer_rsrc((void*)a.wbf, 0, a.Cout * 9 * a.Ctot * 2, 0x00020000);
    const __amdgpu_buffer_rsrc_t rwl = __builtin_amdgcn_make_buffer_rsrc((void*)a.wlo, 0, a.Cout * 9 * a.Ctot * 2, 0x00020000);

    // halo pieces of this thread: halo pixel (gt + it*NTG) >> 3, channel quad gt & 7
    const int kq = gt & 7;
    int hpix[HIT];
#pragma unroll
    for (int it = 0; it < HIT; ++it) {
        const int hp = (gt + it * NTG) >> 3;
        int pix = -1;
        if (hp < NPX) {
            const int hr = hp / HW2, hc = hp - hr * HW2;
            const int iy = y0 - 1 + hr, ix = x0 - 1 + hc;
            if (hc < TW + 2 && iy >= 0 && iy < a.Hout && ix >= 0 && ix < W)
                pix = a.up ? (bimg * a.Hin + (iy >> 1)) * a.Win + (ix >> 1) : (bimg * a.Hin + iy) * a.Win + ix;
        }
        CFD_DASSERT(pix < srows);
        hpix[it] = pix;
    }
    // weight pieces: output channel row gt >> 2 (+ NTG/4 per it), 16-B chunk gt & 3
    const int bq = gt & 3;
    unsigned bvoff[BIT];
#pragma unroll
    for (int it = 0; it < BIT; ++it) {
        const int n = n0 + (gt >> 2) + it * (NTG / 4);
        bvoff[it] = n < a.Cout ? (unsigned)((n * 9 * a.Ctot + 8 * bq) * 2) : 0x80000000u;
    }

    // fused skip convolution: this workgroup's X chunks [xc0, xc0 + nx) (the same
    // split of the X channels as of the halo chunks), the tile pixels' offsets,
    // the sources' and the skip weights' descriptors
    constexpr int XIT = XF ? BM * 8 / NTG : 1;   // 16-B X pieces per thread and chunk
    int nx = 0, xc0 = 0;
    int xpix[XIT];
    unsigned bxoff[BIT];
    __amdgpu_buffer_rsrc_t rx1 = rs1, rx2 = rs1, rxh = rwh, rxl = rwl;
    char* const xreg = lds + LMAIN;
    // fields as locals (a select between two fields of `a` takes its address: a scratch copy)
    const int XC1 = a.XC1, XC2 = a.XC2;
    const float xscale = a.x_scale, mscale = a.main_scale;
    if constexpr (XF) {
        const int XC = a.XC1 + a.XC2, nxc = XC / 32;
        const int xper = (nxc + gridDim.z - 1) / gridDim.z;
        xc0 = bz * xper;
        nx = max(0, min(nxc, xc0 + xper) - xc0);
#pragma unroll
        for (int it = 0; it < XIT; ++it) {
            const int px = (gt + it * NTG) >> 3;
            xpix[it] = (int)(mrow0 + (px / TW) * W + (px % TW));
        }
        const int mrows = __builtin_amdgcn_readfirstlane(a.M);
        rx1 = __builtin_amdgcn_make_buffer_rsrc((void*)a.xsrc1, 0, mrows * a.XC1 * 4, 0x00020000);
        rx2 = __builtin_amdgcn_make_buffer_rsrc((void*)(a.xsrc2 ? (const void*)a.xsrc2 : (const void*)a.xsrc1), 0,
                                                a.xsrc2 ? mrows * a.XC2 * 4 : 0, 0x00020000);
        rxh = __builtin_amdgcn_make_buffer_rsrc((void*)a.xwbf, 0, a.Cout * XC * 2, 0x00020000);
        rxl = __builtin_amdgcn_make_buffer_rsrc((void*)a.xwlo, 0, a.Cout * XC * 2, 0x00020000);
#pragma unroll
        for (int it = 0; it < BIT; ++it) {
            const int n = n0 + (gt >> 2) + it * (NTG / 4);
            bxoff[it] = n < a.Cout ? (unsigned)((n * XC + 8 * bq) * 2) : 0x80000000u;
        }
    }

    // this workgroup's chunks [c0, c1); group kg takes the contiguous sub-range
    // [c0 + kg * gper, cend), one chunk per round -- the ranges a split-K of
    // gridDim.z * KG workgroups would give its splits, so with gridDim.z == 1 the
    // group sums combined in group order are splitk_reduce's sums over the slabs
    const int nch = a.Ctot / 32;
    const int per = (nch + gridDim.z - 1) / gridDim.z;
    const int c0 = bz * per, c1 = min(nch, c0 + per);
    const int gper = (max(c1 - c0, 0) + KG - 1) / KG;
    const int cend = min(c1, c0 + (kg + 1) * gper);
    const int nrounds = gper;
    auto chunk_of = [&](int r) __attribute__((always_inline)) { return c0 + kg * gper + r; };

    typedef typename std::conditional<SB, uint2, f4>::type HT;   // one halo piece in registers
    HT rh[HIT];
    constexpr int BW = BIT * TG;   // 16-B weight pieces per thread, plane and step
    u4 wx_h[BW], wx_l[BW], wy_h[BW], wy_l[BW];   // weight slices two steps deep
    auto load_halo = [&](int c) __attribute__((always_inline)) {
        const int cb = 32 * c;
        const bool second = cb >= a.C1;
        const unsigned csrc = SES * (unsigned)(second ? a.C2 + 0 : a.C1 + 0);   // bytes per source pixel (a select
        const unsigned cofs = SES * ((second ? cb - a.C1 : cb) + 4 * kq);      // of values: no argument copy)
        // one descriptor per branch (a selected descriptor would land in VGPRs)
        if (second) {
#pragma unroll
            for (int it = 0; it < HIT; ++it) {
                const unsigned off = hpix[it] >= 0 ? __umul24((unsigned)hpix[it], csrc) + cofs : 0x80000000u;
                if constexpr (SB)
                    rh[it] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rs2, off, 0, 0));
                else
                    rh[it] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs2, off, 0, 0));
            }
        } else {
#pragma unroll
            for (int it = 0; it < HIT; ++it) {
                const unsigned off = hpix[it] >= 0 ? __umul24((unsigned)hpix[it], csrc) + cofs : 0x80000000u;
                if constexpr (SB)
                    rh[it] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rs1, off, 0, 0));
                else
                    rh[it] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs1, off, 0, 0));
            }
        }
    };
    auto store_halo = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int it = 0; it < HIT; ++it) {
            const int e = gt + it * NTG;
            if (e < NPX * 8) {
                const int off = hswz(e >> 3, (e >> 3) / HW2, kq >> 1) + (kq & 1) * 8;
                if constexpr (SB) {   // already bf16: the 8 loaded bytes as they are
                    *(uint2*)(halo + off) = rh[it];
                } else if constexpr (BF) {
                    *(bf16x4*)(halo + off) = __builtin_convertvector(rh[it], bf16x4);
                } else {
                    uint2 hv, lv;
                    if constexpr (XF)
                        split4_mix_x(rh[it] * mscale, hv, lv);   // the common scale (exact)
                    else
                        split4_mix_x(rh[it], hv, lv);
                    *(uint2*)(halo + off) = hv;
                    *(uint2*)(halo + HPLANE + off) = lv;
                }
            }
        }
    };
    const int NH = nrounds * SPR;   // halo steps; the X steps follow
    // X chunk j of this workgroup into a register set / from it into X buffer j & 1.
    // Chunk j lives in the set of its step's parity ((NH + j) & 1: xr0 even, xr1 odd),
    // picked by a uniform branch -- a runtime index into one array would put it in
    // scratch
    f4 xr0[XIT], xr1[XIT];
    auto load_x = [&](int j, f4 (&dst)[XIT]) __attribute__((always_inline)) {
        if constexpr (XF) {
            const int cb = 32 * (xc0 + j);
            const bool second = cb >= XC1;
            const unsigned csrc = 4u * (unsigned)(second ? XC2 + 0 : XC1 + 0);   // prvalues: a select of values
            const unsigned cofs = 4u * ((second ? cb - XC1 : cb) + 4 * kq);
            if (second) {
#pragma unroll
                for (int it = 0; it < XIT; ++it)
                    dst[it] = __builtin_bit_cast(
                        f4, __builtin_amdgcn_raw_buffer_load_b128(rx2, __umul24((unsigned)xpix[it], csrc) + cofs, 0, 0));
            } else {
#pragma unroll
                for (int it = 0; it < XIT; ++it)
                    dst[it] = __builtin_bit_cast(
                        f4, __builtin_amdgcn_raw_buffer_load_b128(rx1, __umul24((unsigned)xpix[it], csrc) + cofs, 0, 0));
            }
        }
    };
    auto store_x = [&](int j, const f4 (&src)[XIT]) __attribute__((always_inline)) {
        if constexpr (XF) {
            char* xb = xreg + (j & 1) * XBYTES;
#pragma unroll
            for (int it = 0; it < XIT; ++it) {
                const int px = (gt + it * NTG) >> 3;
                const int off = xswz(px, kq >> 1) + (kq & 1) * 8;
                uint2 hv, lv;
                split4_mix_x(src[it] * xscale, hv, lv);
                *(uint2*)(xb + off) = hv;
                *(uint2*)(xb + BM * 64 + off) = lv;
            }
        }
    };
    // step s = (round s / SPR, taps TG (s % SPR) ..); s >= NH: X chunk s - NH
    auto load_w = [&](int s, u4 (&rbh)[BW], u4 (&rbl)[BW]) __attribute__((always_inline)) {
        if constexpr (XF) {
            if (s >= NH) {
                const int soff = 64 * (xc0 + s - NH);
#pragma unroll
                for (int it = 0; it < BIT; ++it) {
                    rbh[it] = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(rxh, bxoff[it], soff, 0));
                    rbl[it] = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(rxl, bxoff[it], soff, 0));
                }
                return;
            }
        }
        const int r = s / SPR, c = chunk_of(r);
        if (c >= cend) return;
#pragma unroll
        for (int u = 0; u < TG; ++u) {
            const int soff = (((s - SPR * r) * TG + u) * a.Ctot + 32 * c) * 2;
#pragma unroll
            for (int it = 0; it < BIT; ++it) {
                rbh[u * BIT + it] = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(rwh, bvoff[it], soff, 0));
                if constexpr (!BF)
                    rbl[u * BIT + it] = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(rwl, bvoff[it], soff, 0));
            }
        }
    };
    auto store_w = [&](int stage, const u4 (&rbh)[BW], const u4 (&rbl)[BW]) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < TG; ++u) {
            char* base = ring + stage * BSTAGE + u * PL * BPLANE;
#pragma unroll
            for (int it = 0; it < BIT; ++it) {
                const int off = xswz((gt >> 2) + it * (NTG / 4), bq);
                *(u4*)(base + off) = rbh[u * BIT + it];
                if constexpr (!BF) *(u4*)(base + BPLANE + off) = rbl[u * BIT + it];
            }
        }
    };

    f16v acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    const int l32 = lane & 31, hsel = lane >> 5;
    int hb[2], hrb[2];   // halo pixel and halo row of tap (0, 0) for this lane's output pixel, per 32-row block
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int p = wm * 64 + 32 * i + l32;
        hb[i] = (p / TW) * HW2 + (p % TW);
        hrb[i] = p / TW;
    }
    const int brow0 = wn * 64 + l32;
    const int nsteps = NH + nx;

    // one step: prefetch the weights of step s + 2, MFMAs of step s on ring stage
    // s & 1, then park step s + 1's weights (loaded a step ago) in the other
    // stage.  Every thread runs every step (the barriers are workgroup-wide); a
    // group whose chunk of the round is past the range only skips its work.
    // XF: steps s >= NH are X chunk j = s - NH (buffer j & 1, the ring's skip
    // weights).  Chunk j lives in the register set of its step's parity: at this
    // call site ldx is the set of s's parity (chunk j + 2 goes there), stx the other
    // (chunk j + 1, parked into the other buffer at the end of the step) -- fixed
    // per call site, so no runtime-selected register array (scratch)
    auto step = [&](int s, u4 (&ldh)[BW], u4 (&ldl)[BW], const u4 (&sth)[BW], const u4 (&stl)[BW],
                    f4 (&ldx)[XIT], f4 (&stx)[XIT]) __attribute__((always_inline)) {
        const bool xs = XF && s >= NH;
        const int r = s / SPR, t = s - SPR * r, j = s - NH;   // t: the step in the round (a tap, or TG taps)
        const int c = chunk_of(r);
        if (s + 2 < nsteps) load_w(s + 2, ldh, ldl);
        if (!xs && t == 0 && chunk_of(r + 1) < cend) load_halo(chunk_of(r + 1));   // in registers until this chunk's taps are done
        if constexpr (XF) {
            if (!xs && t == 0 && r + 1 == nrounds && nx > 0) {   // the last halo round: the first X chunks
                load_x(0, stx);               // step NH has the parity opposite to s = NH - 9 (XF: TG = 1)
                if (nx > 1) load_x(1, ldx);
            }
            if (xs && j + 2 < nx) load_x(j + 2, ldx);
        }
        if (xs || c < cend) {
            const char* wb = ring + (s & 1) * BSTAGE;
            if constexpr (BF) {   // TG = 3: kernel row t, its taps (t, u) against ring piece u
                const int ty = t;
#pragma unroll
                for (int u = 0; u < TG; ++u) {
                    const int tofs = ty * HW2 + u;
                    const char* wbu = wb + u * BPLANE;
#pragma unroll
                    for (int s2 = 0; s2 < 2; ++s2) {
                        const int ch = 2 * s2 + hsel;
                        bf16x8 fa[2], fb[2];
#pragma unroll
                        for (int i = 0; i < 2; ++i) fa[i] = *(const bf16x8*)(halo + hswz(hb[i] + tofs, hrb[i] + ty, ch));
#pragma unroll
                        for (int jj = 0; jj < 2; ++jj) fb[jj] = *(const bf16x8*)(wbu + xswz(brow0 + 32 * jj, ch));
#pragma unroll
                        for (int i = 0; i < 2; ++i)
#pragma unroll
                            for (int jj = 0; jj < 2; ++jj)
                                acc[i][jj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[jj], acc[i][jj], 0, 0, 0);
                    }
                }
            } else {
            // A fragments: the halo at this tap, or the X buffer at the tile pixel
            const int ty = t / 3;
            const int tofs = ty * HW2 + (t - 3 * ty);
            const char* ab = xs ? xreg + (j & 1) * XBYTES : halo;
            const int aplane = xs ? BM * 64 : HPLANE;
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                const int ch = 2 * s2 + hsel;
                h8v fah[2], fal[2], fbh[2], fbl[2];
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    CFD_DASSERT(xs || hb[i] + tofs < NPX);
                    const int off = xs ? xswz(wm * 64 + 32 * i + l32, ch) : hswz(hb[i] + tofs, hrb[i] + ty, ch);
                    fah[i] = *(const h8v*)(ab + off);
                    fal[i] = *(const h8v*)(ab + aplane + off);
                }
#pragma unroll
                for (int jj = 0; jj < 2; ++jj) {
                    const int off = xswz(brow0 + 32 * jj, ch);
                    fbh[jj] = *(const h8v*)(wb + off);
                    fbl[jj] = *(const h8v*)(wb + BPLANE + off);
                }
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int jj = 0; jj < 2; ++jj) {
                        acc[i][jj] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fal[i], fbh[jj], acc[i][jj], 0, 0, 0);
                        acc[i][jj] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fah[i], fbl[jj], acc[i][jj], 0, 0, 0);
                        acc[i][jj] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fah[i], fbh[jj], acc[i][jj], 0, 0, 0);
                    }
            }
            }
        }
        if (s + 1 < nsteps && (s + 1 >= NH || chunk_of((s + 1) / SPR) < cend)) store_w((s + 1) & 1, sth, stl);
        if constexpr (XF) {
            if (xs && j + 1 < nx) store_x(j + 1, stx);
        }
        __syncthreads();
        if (!xs && t == SPR - 1 && s + 1 < nsteps) {   // every wave is past the last tap of round r
            if (chunk_of(r + 1) < cend) store_halo();
            if constexpr (XF) {
                if (r + 1 == nrounds && nx > 0) store_x(0, stx);   // step NH: the parity opposite to s = NH - 1
            }
            __syncthreads();
        }
    };

    if (nsteps > 0) {
        load_w(0, wx_h, wx_l);
        if (nsteps > 1) load_w(1, wy_h, wy_l);
        if (NH > 0 && chunk_of(0) < cend) {
            load_halo(chunk_of(0));
            store_w(0, wx_h, wx_l);
            store_halo();
        } else if (XF && NH == 0 && nx > 0) {   // no halo chunk in this split: X steps only
            load_x(0, xr0);                 // step 0 (even): set xr0, step 1: xr1
            if (nx > 1) load_x(1, xr1);
            store_w(0, wx_h, wx_l);
            store_x(0, xr0);
        }
        __syncthreads();
        CFD_STAMP(a.stamps, 3, a.seq, 2);
        for (int s = 0; s < nsteps; s += 2) {
            step(s, wx_h, wx_l, wy_h, wy_l, xr0, xr1);
            if (s + 1 < nsteps) step(s + 1, wy_h, wy_l, wx_h, wx_l, xr1, xr0);
        }
    }

    CFD_STAMP(a.stamps, 3, a.seq, 3);
    // undo the split weights' power-of-two scale (exact), per group before they
    // are combined -- as the split-K slabs hold scaled sums
    if constexpr (!BF) {   // undo the split weights' power-of-two scale (exact)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[i][j] *= a.acc_scale;
    }
    // combine the K groups through LDS: groups 1.. park their sums, group 0 adds
    // them in group order (fixed summation order)
    if constexpr (KG > 1) {
        float* red = (float*)lds;   // (KG-1) x (WGM*2) waves x 64 floats x 64 lanes
        constexpr int PER_WAVE = 4 * 16 * 64;
        __syncthreads();            // the stages are free
        if (kg > 0) {
            float* dst = red + ((kg - 1) * WGM * WGN + wrem) * PER_WAVE;
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int e = 0; e < 16; e += 4)
                        *(f4*)(dst + ((i * 2 + j) * 16 + e) * 64 + 4 * lane) =
                            f4{acc[i][j][e], acc[i][j][e + 1], acc[i][j][e + 2], acc[i][j][e + 3]};
        }
        __syncthreads();
        if (kg > 0) return;
#pragma unroll
        for (int g = 1; g < KG; ++g) {
            const float* src = red + ((g - 1) * WGM * WGN + wrem) * PER_WAVE;
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int e = 0; e < 16; e += 4) {
                        const f4 v = *(const f4*)(src + ((i * 2 + j) * 16 + e) * 64 + 4 * lane);
                        acc[i][j][e] += v[0];
                        acc[i][j][e + 1] += v[1];
                        acc[i][j][e + 2] += v[2];
                        acc[i][j][e + 3] += v[3];
                    }
        }
    }

    const int n_base = n0 + wn * 64 + l32;
    const int p_base = wm * 64 + 4 * hsel;   // tile position of acc element 0 of block 0
    auto pix_of = [&](int p) __attribute__((always_inline)) { return mrow0 + (int64_t)(p / TW) * W + (p % TW); };
    if constexpr (KG == 1) {
        // epilogue through LDS (launch_conv's ldsepi: Cout % 4 == 0, 16-B rows): one
        // 64-pixel wave row of the tile at a time is parked in LDS and leaves as
        // float4 row pieces, bias / emb / residual read the same way -- instead of
        // 4-byte accesses two 128-B pieces per instruction (measured at config E's
        // 128^2 level: the epilogue was 19-39 us of a 60-80 us workgroup).  The
        // same adds in the same order: the same bits.
        if (a.ldsepi) {
            static_assert(64 * BN * 4 <= (int)sizeof(lds), "epilogue stage fits the LDS");
            float* stg = (float*)lds;
            const bool split = gridDim.z > 1;
            float* dstb = split ? a.part + (int64_t)bz * a.M * a.Cout : a.out;
            constexpr int Q = BN / 4;   // float4 pieces per staged pixel row
            __syncthreads();            // every wave is past its last halo / ring read
            for (int r = 0; r < WGM; ++r) {
                if (wm == r) {
#pragma unroll
                    for (int i = 0; i < 2; ++i)
#pragma unroll
                        for (int e = 0; e < 16; ++e)
#pragma unroll
                            for (int j = 0; j < 2; ++j)
                                stg[(32 * i + 8 * (e >> 2) + (e & 3) + 4 * hsel) * BN + wn * 64 + 32 * j + l32] =
                                    acc[i][j][e];
                }
                __syncthreads();
                for (int q = tid; q < 64 * Q; q += NTG) {
                    const int p = q / Q, c = (q - p * Q) * 4;
                    const int n = n0 + c;
                    if (n < a.Cout) {
                        const int64_t m = pix_of(r * 64 + p);
                        f4 v = *(const f4*)(stg + p * BN + c);
                        if (!split) {
                            if (a.bias) v = v + *(const f4*)(a.bias + n);
                            if (XF && a.bias2) v = v + *(const f4*)(a.bias2 + n);
                            if (a.emb) v = v + *(const f4*)(a.emb + (int64_t)bimg * a.emb_stride + n);
                            if (a.res) v = *(const f4*)(a.res + m * a.Cout + n) + v;
                        }
                        *(f4*)(dstb + m * a.Cout + n) = v;
                    }
                }
                __syncthreads();
            }
#ifdef CFD_STAMPS
            __builtin_amdgcn_s_waitcnt(0);
#endif
            CFD_STAMP(a.stamps, 3, a.seq, 4);
            return;
        }
    }
    if (gridDim.z > 1) {
        float* part = a.part + (int64_t)bz * a.M * a.Cout;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int64_t m = pix_of(p_base + 32 * i + 8 * (e >> 2) + (e & 3));
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int n = n_base + 32 * j;
                    if (n < a.Cout) part[(int64_t)m * a.Cout + n] = acc[i][j][e];
                }
            }
#ifdef CFD_STAMPS
        __builtin_amdgcn_s_waitcnt(0);
#endif
        CFD_STAMP(a.stamps, 3, a.seq, 4);
        return;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int64_t m = pix_of(p_base + 32 * i + 8 * (e >> 2) + (e & 3));
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int n = n_base + 32 * j;
                if (n >= a.Cout) continue;
                float v = a.bias ? acc[i][j][e] + a.bias[n] : acc[i][j][e];
                if (XF && a.bias2) v = v + a.bias2[n];
                if (a.emb) v = v + a.emb[(int64_t)bimg * a.emb_stride + n];
                if (a.res) v = a.res[(int64_t)m * a.Cout + n] + v;
                a.out[(int64_t)m * a.Cout + n] = v;
            }
        }
#ifdef CFD_STAMPS
    __builtin_amdgcn_s_waitcnt(0);
#endif
    CFD_STAMP(a.stamps, 3, a.seq, 4);
}

// K1h tile width for this shape (0: K1h does not apply): the widest of 64, 32,
// 16 dividing the image width whose 256-pixel block rows divide the height
int conv_h_tw(const ConvArgs& a) {
    const bool geo = !a.tmode && a.ks == 3 && a.stride == 1 && a.pad == 1 && a.C1 % 32 == 0 && a.C2 % 32 == 0 &&
                     (a.up ? a.Hout == 2 * a.Hin && a.Wout == 2 * a.Win : a.Hout == a.Hin && a.Wout == a.Win) &&
                     a.M % (a.Hout * a.Wout) == 0;
    if (!geo) return 0;
    for (int tw = 64; tw >= 16; tw >>= 1)
        if (a.Wout % tw == 0 && a.Hout % (256 / tw) == 0) return tw;
    return 0;
}

int launch_conv_x(const ConvArgs& a, int variant, int splits, hipStream_t st) {
    CFD_REQUIRE(a.wbf && !a.tmode, CFD_ESTATE, "conv_x: split-f16 or bf16 forward only");
    CFD_REQUIRE(a.Ctot % 32 == 0 && a.C1 % 4 == 0 && a.C2 % 4 == 0, CFD_ESHAPE, "conv_x needs channels % 32 == 0");
    CFD_REQUIRE(splits == 1 || a.part, CFD_ESTATE, "split-K needs a partial buffer");
    {   // K1x / K1h: 32-bit buffer offsets, 24-bit pixel indices
        const int64_t srows = (int64_t)a.Hin * a.Win * (a.M / (a.Hout * a.Wout));
        CFD_REQUIRE(srows < (1 << 24) && srows * std::max(a.C1, a.C2) * 4 < (1ll << 31) &&
                        (int64_t)a.Cout * a.K * 2 < (1ll << 31) && a.ks * a.ks <= 9,
                    CFD_ESHAPE, "conv_x: operands beyond 2 GiB");
    }
    auto grid = [&](int bm, int bn) __attribute__((always_inline)) {
        return dim3((unsigned)ceil_div(a.M, bm), (unsigned)ceil_div(a.Cout, bn), splits);
    };
    CFD_REQUIRE(!a.xsrc1 || variant == 1 || variant == 2 || variant == 20, CFD_ESTATE,
                "internal: a fused skip convolution runs on K1h / K1x only");
    if (variant == 22) {   // K1hb: bf16 operands, 256-pixel blocks
        const int tw = conv_h_tw(a);
        CFD_REQUIRE(tw > 0 && !a.wlo, CFD_ESHAPE, "conv_h bf16: 3x3 stride-1 with a 16/32/64-divisible width");
        const dim3 g = grid(256, 128);
        // CFD_CONV_KHB_OCC=1: where the grid has more than one workgroup per CU (the
        // 128^2 level of config E), the build whose registers allow 4 waves per SIMD,
        // two workgroups per CU (round 4, one tap per step: 128^2 launches 70-88 -> 47
        // us).  Off since round 5: with three taps per step it spills 49-73 values and
        // the one-workgroup build runs config E at 4.68 vs 4.99 ms per step (same box).
        // Same arithmetic, same bits either way.
        static const int occ = getenv("CFD_CONV_KHB_OCC") ? atoi(getenv("CFD_CONV_KHB_OCC")) : 0;
        if (occ && tw == 64 && (int64_t)g.x * g.y * g.z > 256) {
            if (a.src_bf16)
                hipLaunchKernelGGL((conv_h_kernel<256, 64, 1, true, true, 128, 4>), g, dim3(512), 0, st, a);
            else
                hipLaunchKernelGGL((conv_h_kernel<256, 64, 1, true, false, 128, 4>), g, dim3(512), 0, st, a);
            check_launch("conv_h_kernel");
            return splits;
        }
        if (a.src_bf16) {
            if (tw == 64) hipLaunchKernelGGL((conv_h_kernel<256, 64, 1, true, true>), g, dim3(512), 0, st, a);
            else if (tw == 32) hipLaunchKernelGGL((conv_h_kernel<256, 32, 1, true, true>), g, dim3(512), 0, st, a);
            else hipLaunchKernelGGL((conv_h_kernel<256, 16, 1, true, true>), g, dim3(512), 0, st, a);
        } else {
            if (tw == 64) hipLaunchKernelGGL((conv_h_kernel<256, 64, 1, true>), g, dim3(512), 0, st, a);
            else if (tw == 32) hipLaunchKernelGGL((conv_h_kernel<256, 32, 1, true>), g, dim3(512), 0, st, a);
            else hipLaunchKernelGGL((conv_h_kernel<256, 16, 1, true>), g, dim3(512), 0, st, a);
        }
        check_launch("conv_h_kernel");
        return splits;
    }
    if (variant == 26) {   // K1hb with two in-workgroup K groups (the two splits of a split-K 2)
        const int tw = conv_h_tw(a);
        CFD_REQUIRE(tw > 0 && !a.wlo && splits == 1, CFD_ESHAPE, "conv_h bf16 K groups: 3x3 stride-1, no split-K");
        const dim3 g = grid(256, 128);
        if (a.src_bf16) {
            if (tw == 64) hipLaunchKernelGGL((conv_h_kernel<256, 64, 2, true, true>), g, dim3(1024), 0, st, a);
            else if (tw == 32) hipLaunchKernelGGL((conv_h_kernel<256, 32, 2, true, true>), g, dim3(1024), 0, st, a);
            else hipLaunchKernelGGL((conv_h_kernel<256, 16, 2, true, true>), g, dim3(1024), 0, st, a);
        } else {
            if (tw == 64) hipLaunchKernelGGL((conv_h_kernel<256, 64, 2, true>), g, dim3(1024), 0, st, a);
            else if (tw == 32) hipLaunchKernelGGL((conv_h_kernel<256, 32, 2, true>), g, dim3(1024), 0, st, a);
            else hipLaunchKernelGGL((conv_h_kernel<256, 16, 2, true>), g, dim3(1024), 0, st, a);
        }
        check_launch("conv_h_kernel");
        return 1;
    }
    CFD_REQUIRE(!a.src_bf16, CFD_ESTATE, "internal: a bf16 convolution source needs the K1hb kernel");
    if (variant == 24) {   // K1h with two in-workgroup K groups, 64 output channels (LDS: 2 x 67 KB at TW 64)
        const int tw = conv_h_tw(a);
        CFD_REQUIRE(tw > 0 && splits == 1 && a.Cout % 64 == 0, CFD_ESHAPE, "conv_h K groups: 3x3 stride-1, no split-K");
        const dim3 g = grid(256, 64);
        if (tw == 64) hipLaunchKernelGGL((conv_h_kernel<256, 64, 2, false, false, 64>), g, dim3(512), 0, st, a);
        else if (tw == 32) hipLaunchKernelGGL((conv_h_kernel<256, 32, 2, false, false, 64>), g, dim3(512), 0, st, a);
        else hipLaunchKernelGGL((conv_h_kernel<256, 16, 2, false, false, 64>), g, dim3(512), 0, st, a);
        check_launch("conv_h_kernel");
        return 1;
    }
    if (variant == 20) {   // K1h: 256-pixel blocks
        const int tw = conv_h_tw(a);
        CFD_REQUIRE(tw > 0, CFD_ESHAPE, "conv_h: 3x3 stride-1 with a 16/32/64-divisible width");
        // small batch: where the 128-channel grid leaves most CUs idle (< 128
        // workgroups of 8 waves, two per SIMD), 64-channel workgroups of 4 waves --
        // twice the workgroups, one wave per SIMD, the same tiles' sums
        // (CFD_CONV_SMALLN=0 keeps 128)
        static const int smalln = smalln_below();
        const dim3 g = grid(256, 128);
        const bool xf = a.xsrc1 != nullptr;   // fused skip convolution (the XF instances)
        if ((int64_t)g.x * g.y * g.z < smalln && a.Cout % 64 == 0) {
            const dim3 g64 = grid(256, 64);
            if (xf) {
                if (tw == 64) hipLaunchKernelGGL((conv_h_kernel<256, 64, 1, false, false, 64, 1, true>), g64, dim3(256), 0, st, a);
                else if (tw == 32) hipLaunchKernelGGL((conv_h_kernel<256, 32, 1, false, false, 64, 1, true>), g64, dim3(256), 0, st, a);
                else hipLaunchKernelGGL((conv_h_kernel<256, 16, 1, false, false, 64, 1, true>), g64, dim3(256), 0, st, a);
            } else {
                if (tw == 64) hipLaunchKernelGGL((conv_h_kernel<256, 64, 1, false, false, 64>), g64, dim3(256), 0, st, a);
                else if (tw == 32) hipLaunchKernelGGL((conv_h_kernel<256, 32, 1, false, false, 64>), g64, dim3(256), 0, st, a);
                else hipLaunchKernelGGL((conv_h_kernel<256, 16, 1, false, false, 64>), g64, dim3(256), 0, st, a);
            }
            check_launch("conv_h_kernel");
            return splits;
        }
        if (xf) {
            if (tw == 64) hipLaunchKernelGGL((conv_h_kernel<256, 64, 1, false, false, 128, 1, true>), g, dim3(512), 0, st, a);
            else if (tw == 32) hipLaunchKernelGGL((conv_h_kernel<256, 32, 1, false, false, 128, 1, true>), g, dim3(512), 0, st, a);
            else hipLaunchKernelGGL((conv_h_kernel<256, 16, 1, false, false, 128, 1, true>), g, dim3(512), 0, st, a);
        } else {
            if (tw == 64) hipLaunchKernelGGL((conv_h_kernel<256, 64>), g, dim3(512), 0, st, a);
            else if (tw == 32) hipLaunchKernelGGL((conv_h_kernel<256, 32>), g, dim3(512), 0, st, a);
            else hipLaunchKernelGGL((conv_h_kernel<256, 16>), g, dim3(512), 0, st, a);
        }
        check_launch("conv_h_kernel");
        return splits;
    }
    if (!a.wlo) {   // bf16 operands (config E): the 3x3 convolutions K1hb does not tile
        CFD_REQUIRE(!a.xsrc1, CFD_ESTATE, "internal: a fused skip convolution needs split compute");
        switch (variant) {
            case 1: hipLaunchKernelGGL((conv_x_kernel<128, 128, 2, 2, 1, 1, false, true>), grid(128, 128), dim3(256), 0, st, a); break;
            case 2: hipLaunchKernelGGL((conv_x_kernel<256, 128, 4, 2, 1, 1, false, true>), grid(256, 128), dim3(512), 0, st, a); break;
            default: CFD_REQUIRE(false, CFD_EARG, "conv_x variant");
        }
        check_launch("conv_x_kernel");
        return splits;
    }
    if (a.xsrc1) {   // fused skip convolution
        switch (variant) {
            case 1: hipLaunchKernelGGL((conv_x_kernel<128, 128, 2, 2, 1, 1, true>), grid(128, 128), dim3(256), 0, st, a); break;
            case 2: hipLaunchKernelGGL((conv_x_kernel<256, 128, 4, 2, 1, 1, true>), grid(256, 128), dim3(512), 0, st, a); break;
            default: CFD_REQUIRE(false, CFD_EARG, "conv_x variant");
        }
        check_launch("conv_x_kernel");
        return splits;
    }
    switch (variant) {
        case 1: hipLaunchKernelGGL((conv_x_kernel<128, 128, 2, 2, 1>), grid(128, 128), dim3(256), 0, st, a); break;
        case 2: hipLaunchKernelGGL((conv_x_kernel<256, 128, 4, 2, 1>), grid(256, 128), dim3(512), 0, st, a); break;
        default: CFD_REQUIRE(false, CFD_EARG, "conv_x variant");
    }
    check_launch("conv_x_kernel");
    return splits;
}

}  // namespace cfd
