// K1x: split-f16 implicit-GEMM convolution on v_mfma_f32_32x32x16_f16 with
// 64x64 wave tiles (gfx950).
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
template <int BM, int BN, int WGM, int WGN, int PF = 1>
__global__ __launch_bounds__(64 * WGM * WGN, 1) void conv_x_kernel(ConvArgs a) {
    constexpr int NW = WGM * WGN, NT = 64 * NW;
    constexpr int WTM = BM / WGM, WTN = BN / WGN;   // wave tile
    constexpr int TM = WTM / 32, TN = WTN / 32;     // 32x32 blocks per wave
    constexpr int RPP = NT / 8;                     // row-slices staged per pass (8 threads x 4 k)
    constexpr int AIT = BM / RPP, BIT = BN / RPP;
    static_assert(TM >= 1 && TN >= 1 && AIT >= 1 && BIT >= 1, "tile");
    static_assert(BM % RPP == 0 && BN % RPP == 0, "staging");
    constexpr int ABYTES = BM * 64, BBYTES = BN * 64;    // one f16 plane
    constexpr int STAGE = 2 * ABYTES + 2 * BBYTES;      // A hi, A lo, B hi, B lo
    __shared__ __attribute__((aligned(16))) char lds[2 * STAGE];

    CFD_STAMP(a.stamps, 2, a.seq, 0);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WGN, wn = wave % WGN;

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
    const int ntap = a.ks * a.ks, KM = ntap * a.Ctot;
    const __amdgpu_buffer_rsrc_t rwh = __builtin_amdgcn_make_buffer_rsrc((void*)a.wbf, 0, a.Cout * KM * 2, 0x00020000);
    const __amdgpu_buffer_rsrc_t rwl = __builtin_amdgcn_make_buffer_rsrc((void*)a.wlo, 0, a.Cout * KM * 2, 0x00020000);
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

    // staged row-slices: A (tile row), B (output channel)
    int a_row[AIT];
#pragma unroll
    for (int it = 0; it < AIT; ++it) a_row[it] = rsub + it * RPP;
    int b_row[BIT];
    unsigned b_voff[BIT];
#pragma unroll
    for (int it = 0; it < BIT; ++it) {
        b_row[it] = rsub + it * RPP;
        const int n = n0 + b_row[it];
        b_voff[it] = n < a.Cout ? (unsigned)((n * KM + 4 * kq) * 2) : 0x80000000u;
    }

    const int nkt = a.K / 32;
    const int per = (nkt + gridDim.z - 1) / gridDim.z;
    const int kt0 = bz * per;
    const int kt1 = min(nkt, kt0 + per);
    // K position (tap, channel base) of tile kt0, advanced one tile per load
    int cbg, tpg;
    {
        const int kb = kt0 * 32;
        const int tp = kb / a.Ctot;
        tpg = __builtin_amdgcn_readfirstlane(tp);   // SGPRs: scalar descriptor choice
        cbg = __builtin_amdgcn_readfirstlane(kb - tp * a.Ctot);
    }
    __syncthreads();   // pixtab

    f4 ra[PF][AIT];
    uint2 rbh[PF][BIT], rbl[PF][BIT];
    auto load_tile = [&](int kt, int set) __attribute__((always_inline)) {   // tile kt into register set `set`
#pragma unroll
        for (int it = 0; it < AIT; ++it) {
            const bool second = cbg >= a.C1;
            const unsigned csrc4 = 4u * (second ? a.C2 : a.C1);
            const unsigned cofs4 = 4u * ((second ? cbg - a.C1 : cbg) + 4 * kq);
            const int pix = kt < kt1 ? pixtab[tpg * BM + a_row[it]] : -1;
            const unsigned off = pix >= 0 ? __umul24((unsigned)pix, csrc4) + cofs4 : 0x80000000u;
            ra[set][it] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(second ? rs2 : rs1, off, 0, 0));
        }
#pragma unroll
        for (int it = 0; it < BIT; ++it) {
            const unsigned voff = kt < kt1 ? b_voff[it] : 0x80000000u;
            const int soff = (tpg * a.Ctot + cbg) * 2;
            rbh[set][it] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rwh, voff, soff, 0));
            rbl[set][it] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rwl, voff, soff, 0));
        }
        cbg += 32;
        while (cbg >= a.Ctot && tpg < ntap) {
            cbg -= a.Ctot;
            ++tpg;
        }
    };
    auto store_tile = [&](int buf, int set) __attribute__((always_inline)) {
        char* base = lds + buf * STAGE;
#pragma unroll
        for (int it = 0; it < AIT; ++it) {
            const int off = xswz(a_row[it], kq >> 1) + (kq & 1) * 8;
            uint2 hv, lv;
            split4_mix_x(ra[set][it], hv, lv);
            *(uint2*)(base + off) = hv;
            *(uint2*)(base + ABYTES + off) = lv;
        }
#pragma unroll
        for (int it = 0; it < BIT; ++it) {
            const int off = xswz(b_row[it], kq >> 1) + (kq & 1) * 8;
            *(uint2*)(base + 2 * ABYTES + off) = rbh[set][it];
            *(uint2*)(base + 2 * ABYTES + BBYTES + off) = rbl[set][it];
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
    const int arow0 = wm * WTM + l32, brow0 = wn * WTN + l32;
    // one K step (tile kt): prefetch the tiles PF steps ahead into register
    // set `lset`, MFMAs on LDS stage `cur`, then stage the next step's tiles
    // (register set `sset`, loaded PF - 1 steps ago) into the other LDS stage
    auto kstep = [&](int kt, int cur, int lset, int sset) __attribute__((always_inline)) {
            const bool more = kt + 1 < kt1;
            if (kt + PF < kt1) load_tile(kt + PF, lset);
            const char* base = lds + cur * STAGE;
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const int ch = 2 * s + hsel;
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
            if (kt0 + 1 < kt1) load_tile(kt0 + 1, 1);
        }
        store_tile(0, 0);
        __syncthreads();
        CFD_STAMP(a.stamps, 2, a.seq, 2);
        if constexpr (PF == 1) {
            int cur = 0;
            for (int kt = kt0; kt < kt1; ++kt) {
                kstep(kt, cur, 0, 0);
                cur ^= 1;
            }
        } else {
            for (int kt = kt0; kt < kt1; kt += 2) {
                kstep(kt, 0, 0, 1);
                if (kt + 1 < kt1) kstep(kt + 1, 1, 1, 0);
            }
        }
    }

    CFD_STAMP(a.stamps, 2, a.seq, 3);
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
//
// Measured and not kept (tools/convbench): 128-pixel blocks in two
// in-workgroup K groups (0.83-1.07x); K1y, an LDS-DMA ring (0.75-0.84x); two K
// groups as a split-K 2 without the partial slab (3 % slower); a ResBlock's skip
// 1x1 fused in as extra K (flat); a 4-waves-per-SIMD K1hb build (spills with three
// taps per step); fragment reads software-
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
template <int BM, int TW, bool BF = false, bool SB = false, int BN = 128>
__global__ __launch_bounds__(BM * (BN / 64), 1) void conv_h_kernel(ConvArgs a) {
    static_assert(!SB || BF, "a bf16 source needs the bf16 kernel");
    constexpr unsigned SES = SB ? 2u : 4u;   // source element bytes
    constexpr int WGN = BN / 64, WGM = BM / 64, NTG = 64 * WGM * WGN;   // threads per workgroup
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
    constexpr int GBYTES = PL * HPLANE + 2 * BSTAGE;  // the halo + the weight ring
    static_assert(BM % TW == 0 && BIT >= 1, "tile");
    __shared__ __attribute__((aligned(16))) char lds[GBYTES];

    CFD_STAMP(a.stamps, 3, a.seq, 0);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WGN, wn = wave % WGN;
    const int gt = tid;
    char* const halo = lds;
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

    // this workgroup's chunks [c0, cend) (its split-K range), one chunk per round
    const int nch = a.Ctot / 32;
    const int per = (nch + gridDim.z - 1) / gridDim.z;
    const int c0 = bz * per, cend = min(nch, c0 + per);
    const int nrounds = max(cend - c0, 0);
    auto chunk_of = [&](int r) __attribute__((always_inline)) { return c0 + r; };

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
                    split4_mix_x(rh[it], hv, lv);
                    *(uint2*)(halo + off) = hv;
                    *(uint2*)(halo + HPLANE + off) = lv;
                }
            }
        }
    };
    // step s = (round s / SPR, taps TG (s % SPR) ..)
    auto load_w = [&](int s, u4 (&rbh)[BW], u4 (&rbl)[BW]) __attribute__((always_inline)) {
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
    const int nsteps = nrounds * SPR;

    // one step: prefetch the weights of step s + 2, MFMAs of step s on ring stage
    // s & 1, then park step s + 1's weights (loaded a step ago) in the other
    // stage.  Every thread runs every step (the barriers are workgroup-wide).
    auto step = [&](int s, u4 (&ldh)[BW], u4 (&ldl)[BW], const u4 (&sth)[BW], const u4 (&stl)[BW])
        __attribute__((always_inline)) {
        const int r = s / SPR, t = s - SPR * r;   // t: the step in the round (a tap, or TG taps)
        const int c = chunk_of(r);
        if (s + 2 < nsteps) load_w(s + 2, ldh, ldl);
        if (t == 0 && chunk_of(r + 1) < cend) load_halo(chunk_of(r + 1));   // in registers until this chunk's taps are done
        if (c < cend) {
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
            // A fragments: the halo at this tap
            const int ty = t / 3;
            const int tofs = ty * HW2 + (t - 3 * ty);
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                const int ch = 2 * s2 + hsel;
                h8v fah[2], fal[2], fbh[2], fbl[2];
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    CFD_DASSERT(hb[i] + tofs < NPX);
                    const int off = hswz(hb[i] + tofs, hrb[i] + ty, ch);
                    fah[i] = *(const h8v*)(halo + off);
                    fal[i] = *(const h8v*)(halo + HPLANE + off);
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
        if (s + 1 < nsteps && chunk_of((s + 1) / SPR) < cend) store_w((s + 1) & 1, sth, stl);
        __syncthreads();
        if (t == SPR - 1 && s + 1 < nsteps) {   // every wave is past the last tap of round r
            if (chunk_of(r + 1) < cend) store_halo();
            __syncthreads();
        }
    };

    if (nsteps > 0) {
        load_w(0, wx_h, wx_l);
        if (nsteps > 1) load_w(1, wy_h, wy_l);
        load_halo(chunk_of(0));
        store_w(0, wx_h, wx_l);
        store_halo();
        __syncthreads();
        CFD_STAMP(a.stamps, 3, a.seq, 2);
        for (int s = 0; s < nsteps; s += 2) {
            step(s, wx_h, wx_l, wy_h, wy_l);
            if (s + 1 < nsteps) step(s + 1, wy_h, wy_l, wx_h, wx_l);
        }
    }

    CFD_STAMP(a.stamps, 3, a.seq, 3);
    if constexpr (!BF) {   // undo the split weights' power-of-two scale (exact)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[i][j] *= a.acc_scale;
    }
    const int n_base = n0 + wn * 64 + l32;
    const int p_base = wm * 64 + 4 * hsel;   // tile position of acc element 0 of block 0
    auto pix_of = [&](int p) __attribute__((always_inline)) { return mrow0 + (int64_t)(p / TW) * W + (p % TW); };
    {
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
    if (variant == 22) {   // K1hb: bf16 operands, 256-pixel blocks
        const int tw = conv_h_tw(a);
        CFD_REQUIRE(tw > 0 && !a.wlo, CFD_ESHAPE, "conv_h bf16: 3x3 stride-1 with a 16/32/64-divisible width");
        const dim3 g = grid(256, 128);
        if (a.src_bf16) {
            if (tw == 64) hipLaunchKernelGGL((conv_h_kernel<256, 64, true, true>), g, dim3(512), 0, st, a);
            else if (tw == 32) hipLaunchKernelGGL((conv_h_kernel<256, 32, true, true>), g, dim3(512), 0, st, a);
            else hipLaunchKernelGGL((conv_h_kernel<256, 16, true, true>), g, dim3(512), 0, st, a);
        } else {
            if (tw == 64) hipLaunchKernelGGL((conv_h_kernel<256, 64, true>), g, dim3(512), 0, st, a);
            else if (tw == 32) hipLaunchKernelGGL((conv_h_kernel<256, 32, true>), g, dim3(512), 0, st, a);
            else hipLaunchKernelGGL((conv_h_kernel<256, 16, true>), g, dim3(512), 0, st, a);
        }
        check_launch("conv_h_kernel");
        return splits;
    }
    CFD_REQUIRE(!a.src_bf16, CFD_ESTATE, "internal: a bf16 convolution source needs the K1hb kernel");
    if (variant == 20) {   // K1h: 256-pixel blocks
        const int tw = conv_h_tw(a);
        CFD_REQUIRE(tw > 0, CFD_ESHAPE, "conv_h: 3x3 stride-1 with a 16/32/64-divisible width");
        // small batch: where the 128-channel grid leaves most CUs idle (< 128
        // workgroups of 8 waves, two per SIMD), 64-channel workgroups of 4 waves --
        // twice the workgroups, one wave per SIMD, the same tiles' sums
        // (CFD_CONV_SMALLN=0 keeps 128)
        static const int smalln = smalln_below();
        const dim3 g = grid(256, 128);
        if ((int64_t)g.x * g.y * g.z < smalln && a.Cout % 64 == 0) {
            const dim3 g64 = grid(256, 64);
            if (tw == 64) hipLaunchKernelGGL((conv_h_kernel<256, 64, false, false, 64>), g64, dim3(256), 0, st, a);
            else if (tw == 32) hipLaunchKernelGGL((conv_h_kernel<256, 32, false, false, 64>), g64, dim3(256), 0, st, a);
            else hipLaunchKernelGGL((conv_h_kernel<256, 16, false, false, 64>), g64, dim3(256), 0, st, a);
            check_launch("conv_h_kernel");
            return splits;
        }
        if (tw == 64) hipLaunchKernelGGL((conv_h_kernel<256, 64>), g, dim3(512), 0, st, a);
        else if (tw == 32) hipLaunchKernelGGL((conv_h_kernel<256, 32>), g, dim3(512), 0, st, a);
        else hipLaunchKernelGGL((conv_h_kernel<256, 16>), g, dim3(512), 0, st, a);
        check_launch("conv_h_kernel");
        return splits;
    }
    CFD_REQUIRE(a.wlo, CFD_ESTATE, "internal: K1x runs split-f16 operands only");
    switch (variant) {
        case 1: hipLaunchKernelGGL((conv_x_kernel<128, 128, 2, 2>), grid(128, 128), dim3(256), 0, st, a); break;
        case 2: hipLaunchKernelGGL((conv_x_kernel<256, 128, 4, 2>), grid(256, 128), dim3(512), 0, st, a); break;
        default: CFD_REQUIRE(false, CFD_EARG, "conv_x variant");
    }
    check_launch("conv_x_kernel");
    return splits;
}

}  // namespace cfd
