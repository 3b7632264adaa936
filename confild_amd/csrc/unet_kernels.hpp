// Launch interface of the U-Net kernels (unet_kernels.hip).
#pragma once
#include "common.hpp"

namespace cfd {

struct GnArgs {
    const float* src1;
    const float* src2;  // second (concatenated) source or null
    const float* gamma;
    const float* beta;
    double* part;       // (B, nchunks, 32, 2) partial sums
    float* ss;          // (B, Ctot, 2) scale / shift
    float* out;         // (B, HW, Ctot) normalised (+ SiLU) activation
    float* stats;       // optional (B, 32, 2) group mean / rstd (kept for the backward)
    int C1, C2, Ctot, HW;
    float eps;
    int silu;
    int nchunks;
    int B;
    // Optional: src1 is the still-unreduced output of a split-K convolution
    // (launch_conv with defer).  This kernel then forms x = sum_s kpart[s]
    // (+ kbias) (+ kemb[b]), then kres + x -- splitk_reduce's order, so x is
    // bit-identical -- writes it to kx (= the convolution's output) and
    // normalises it: one launch and one pass over x fewer.
    const float* kpart;  // (ksplits, B*HW, C1) partial slab, or null
    const float* kbias;
    const float* kemb;
    const float* kres;
    float* kx;           // where the reduced sum is stored (null: nowhere, nobody reads it)
    int ksplits, kemb_stride;
    unsigned long long* stamps;   // development (CFD_STAMPS builds): timestamp buffer, else null
    int seq;                      // launch sequence number (timestamps)
    // out holds bf16 (RNE of the fp32 result, (B, HW, Ctot) of 2-byte elements):
    // config E, where the consumer is a K1hb convolution that rounds its operand
    // to bf16 anyway -- the same bits, half the bytes written and re-read
    int out_bf16;
    // optional (training tape): max |stored out| reduced into this zeroed slot, one
    // atomicMax of the float bits per workgroup -- the operand range the split
    // weight gradients of the next convolution need
    unsigned* amax_out;
    // the model's planned batch (ConvArgs::plan_b; 0: 8): gn2's chunk count and
    // reach, a function of the per-sample shape and this setting only
    int plan_b;
};

struct ConvArgs {
    const float* src1;
    const float* src2;   // concat-free second source (channels C1..C1+C2) or null
    const float* w;      // packed (Cout, ks*ks, Ctot)
    const void* wbf;     // the same packing in bf16 (config E compute) / f16 hi part (split), or null
    const void* wlo;     // split compute: f16 lo part of the scaled weights, or null
    float acc_scale;     // split compute: 1 / (power-of-two weight scale)
    const float* bias;   // (Cout) or null
    const float* emb;    // (B, emb_stride) slice, or null
    const float* res;    // (M, Cout) residual, or null
    float* out;          // (M, Cout)
    float* part;         // split-K partial slab (splits, M, Cout), or null
    int C1, C2, Ctot;
    int Hin, Win, Hout, Wout;
    int stride, ks, pad, up;
    int tmode;           // transposed addressing (input-gradient of a stride-s conv)
    int Cout;
    int emb_stride;
    int M, K;
    int xcd;             // XCD-contiguous workgroup order (set by launch_conv; CFD_CONV_XCD=0: off)
    int bufaddr;         // 32-bit buffer addressing of the operands (set by launch_conv where it fits)
    int ldsepi;          // K1s: epilogue through LDS, float4 rows (set by launch_conv; CFD_CONV_LDSEPI=0: off)
    int* nonfinite;      // conv_out only: set to 1 when an output is not finite (range guard), or null
    int src_bf16;        // src1 / src2 hold bf16 (a GroupNorm's out_bf16 output): K1hb only
    // qkv convolution on K1s in split compute (conv_kv_pack_ok): the LDS epilogue also
    // writes the split attention's packed K / V fragments (attn_kv_split_kernel's
    // layout and arithmetic) from the staged tile, so no pack launch follows
    void* kvf;           // K fragments (h8v), V fragments at kvf + kv_voff h8v; null: no pack
    int64_t kv_voff;
    int kv_ch, kv_heads, kv_T;
    float kv_scale;      // the attention's q / k scale (K carries scale * log2 e)
    unsigned long long* stamps;   // development (CFD_STAMPS builds): timestamp buffer, else null
    int seq;                      // launch sequence number (timestamps)
    // the batch plan_conv tiles for (0: 8): a per-model setting
    // (cfd_unet_set_plan_batch), never the real batch, so a sample's sums do not
    // depend on the batch it runs in
    int plan_b;
};
// development: the timestamp buffer the CFD_STAMPS build's kernels write (null: off)
void stamps_set(unsigned long long* buf);
unsigned long long* stamps_buf();

struct AttnArgs {
    const float* qkv;  // (B, T, 3C)
    float* out;        // (B, T, C)
    int T, C;
    float scale;       // 1/sqrt(sqrt(ch)), applied to q and k separately
    float* lse;        // optional (B, heads, T) log-sum-exp of each softmax row
    // K4d: workgroups of one (sample, head) on one XCD (set by the launcher where
    // heads * B % 8 == 0), so its K/V fragments are fetched into one L2
    int xcdmap;
    // key-chunked launches (attention_kv_chunks > 1): chunk count, and the per-chunk
    // partials (O unnormalised, then (max, sum) pairs) the combine pass reduces
    int kc;
    float* part;
};

// GroupNorm(32)(+SiLU) backward: dx = rstd * (g - mean(g) - xhat * mean(g * xhat)),
// g = gamma * dz (* SiLU'(z)), per (sample, group).  dx is split over the two
// forward sources: channels [0, C1) -> out1 (stride C1), [C1, Ctot) -> out2.
struct GnbArgs {
    const float* x1;
    const float* x2;      // forward input sources
    const float* dz;      // (B, HW, Ctot) gradient w.r.t. the GN(+SiLU) output
    const float* ss;      // (B, Ctot, 2) forward scale / shift
    const float* stats;   // (B, 32, 2) forward mean / rstd
    const float* gamma;
    const float* addsrc;  // optional (B, HW, Ctot) added to dx (residual branch)
    float* out1;
    float* out2;
    int acc1, acc2;       // accumulate into out1 / out2 instead of overwriting
    double* part;         // scratch (B, nchunks, 32, 2)
    float* fin;           // scratch (B, 32, 2)
    // optional (training): the GroupNorm parameter-gradient partials from the same
    // pass, (B, nchunks, Ctot, 2) floats = (sum dz_eff xhat, sum dz_eff) per chunk
    float* ppart;
    // optional (training, split weight gradients): max |stored out1| reduced here
    // with one atomicMax of the float bits per workgroup (a zeroed slot)
    unsigned* amax_out;
    int C1, C2, Ctot, HW, silu, nchunks, B;
    int plan_b;   // the model's planned batch (0: 8), as GnArgs::plan_b
};

// QKVAttentionLegacy backward (flash-style, recomputes P from the saved LSE).
struct AttnBwdArgs {
    const float* qkv;   // (B, T, 3C) forward input
    const float* o;     // (B, T, C) forward output (before proj_out)
    const float* dout;  // (B, T, C) gradient w.r.t. o
    const float* lse;   // (B, heads, T)
    float* dd;          // scratch (B, heads, T): rowsum(dO * O)
    float* dqkv;        // (B, T, 3C)
    int T, C;
    float scale;
    // split compute (K9s): the packed fragments (attention_bwd_split_floats per
    // sample) and the per (sample, head, 32-token block) maxima of |dO| and |V|
    // that fix each (sample, head)'s power-of-two gradient scale; xcdmap as AttnArgs
    h8v* packs;
    float* amax;
    int heads, xcdmap;
};

struct ConvPlan {
    int bm = 128, bn = 128, splits = 1;
    int nw = 4;  // waves per workgroup (8: BM = BN = 128 only)
    int kx = -1; // >= 0: run the K1x kernel variant (conv_x.hip) instead of conv_gemm_kernel
    int pf = 1;  // K1s: K tiles in flight through registers (set by launch_conv)
};

constexpr int kGnMaxChunks = 512;
int gn_chunks(int HW);
// gn2 (the two-launch full-row GroupNorm) and the DPS GroupNorm backward: pixel
// chunks of a sample, 1024-thread workgroups beyond kGn2BigHW pixels
constexpr int kGn2BigHW = 16384, kGn2BigChunks = 256;
static_assert(kGn2BigChunks <= kGnMaxChunks, "gn2 partials live in the kGnMaxChunks slab");
int gn2_chunks(int HW, int plan_b);
// gn2's workgroup size for nchunks chunks: 1024 threads beyond 64 (the apply pass
// then reduces the chunk partials with 32 lanes per group, nchunks / 32 loads each)
inline int gn2_threads(int nchunks) { return nchunks > 64 ? 1024 : 256; }
// GroupNorm statistics + normalise (+SiLU) into a.out
void launch_gn(const GnArgs& a, int B, hipStream_t st);
// whether launch_gn runs the register-resident kernel for this shape (the only
// one that accepts a split-K source, GnArgs::kpart)
bool gn_takes_splitk(const GnArgs& a, int B);
// whether launch_gn runs the two-launch full-row form (gn2_*) for this shape: it
// then needs GnArgs::kx for a split-K source (the apply pass re-reads the sum)
bool gn2_applies(const GnArgs& a);
// part_cap_floats: split-K slab available per planned batch (ConvArgs::plan_b) (plans depend on the
// per-sample shape only, never on the batch)
ConvPlan plan_conv(const ConvArgs& a, size_t part_cap_floats);
// Returns the split count.  With defer and splits > 1 the reduction is not
// launched: the caller runs launch_splitk_reduce or hands the slab to launch_gn.
int launch_conv(const ConvArgs& a, const ConvPlan& p, hipStream_t st, bool defer = false);
void launch_splitk_reduce(const ConvArgs& a, int splits, hipStream_t st);
// Workgroup -> (m tile, n tile, split) in XCD-contiguous order (the hardware
// deals workgroups round-robin over the 8 XCDs): XCD x gets the x-th contiguous
// run of tiles.  order 1: splits fastest, then n, then m (the workgroups of an
// XCD share activation rows: every split of one pixel tile); order 2: m fastest,
// then splits, then n (they share weight slices: the small-M levels, where a
// weight slice is read by every m tile).
__device__ __forceinline__ void xcd_tile(int order, int& bx, int& by, int& bz) {
    bx = blockIdx.x;
    by = blockIdx.y;
    bz = blockIdx.z;
    if (!order) return;
    const unsigned gx = gridDim.x, gy = gridDim.y, gz = gridDim.z;
    const unsigned T = gx * gy * gz, L = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
    const unsigned q = T >> 3, r = T & 7, x = L & 7, sl = L >> 3;
    const unsigned Lp = x < r ? x * (q + 1) + sl : r * (q + 1) + (x - r) * q + sl;
    if (order == 2) {
        bx = Lp % gx;
        bz = (Lp / gx) % gz;
        by = Lp / (gx * gz);
    } else {
        bz = Lp % gz;
        by = (Lp / gz) % gy;
        bx = Lp / (gz * gy);
    }
}
// K1x / K1h (conv_x.hip): split-f16 forward convolutions on 32x32x16 MFMAs with
// 64x64 wave tiles; variant selects the kernel and tile shape
int launch_conv_x(const ConvArgs& a, int variant, int splits, hipStream_t st);
int conv_h_tw(const ConvArgs& a);   // K1h tile width for a shape, 0: not applicable
// whether launch_conv runs this plan on K1hb (the bf16 halo kernel, variant 22):
// the only convolution that reads a bf16 source (ConvArgs::src_bf16)
int smalln_below();
bool conv_runs_k1hb(const ConvArgs& a, const ConvPlan& p);
void launch_conv_in(const ConvArgs& a, hipStream_t st);
void launch_conv_out(const ConvArgs& a, hipStream_t st);
void launch_attention(const AttnArgs& a, int CH, int heads, int B, hipStream_t st);
// split-f16 attention (K4s); kvws holds attention_split_floats(T, C) floats per sample
size_t attention_split_floats(int T, int C);
// packed: the qkv convolution already wrote the K / V fragments (ConvArgs::kvf)
// key chunks of the split attention at this shape and planned batch (a function of
// neither the real batch nor the data: batch invariance), and their partials' floats
// per sample
int attention_kv_chunks(int T, int heads, int plan_b);
size_t attention_part_floats(int T, int C, int CH, int plan_b);
void launch_attention_split(const AttnArgs& a, int CH, int heads, int B, int plan_b, float* kvws, hipStream_t st,
                            bool packed);
// the K / V fragment pointers of kvws (launch_attention_split's layout): K at
// kvws, V at kvws + voff h8v
int64_t attention_split_voff(int T, int CH, int heads, int B);
// whether launch_conv runs this qkv plan through a K1s LDS epilogue that can pack
// the K / V fragments (split compute, no split-K, T % 32 == 0)
bool conv_kv_pack_ok(const ConvArgs& a, const ConvPlan& p, int T);
// backward (unet_vjp.hip)
int launch_gn_bwd(const GnbArgs& a, int B, hipStream_t st);   // returns the pixel chunks used
void launch_attention_bwd(const AttnBwdArgs& a, int CH, int heads, int B, hipStream_t st);
// K9s, the split-f16 attention backward: workspace floats per sample (packs and
// scales), whether it takes this shape, and the launcher (sets a.packs / a.amax)
size_t attention_bwd_split_floats(int T, int C);
bool attention_bwd_split_ok(int T, int CH);
void launch_attention_bwd_split(const AttnBwdArgs& a, int CH, int heads, int B, float* ws, hipStream_t st);
void launch_add(float* y, const float* x, int64_t n, hipStream_t st);
void launch_temb(const int64_t* t, const float* freqs, float* out, int dim, int B, hipStream_t st);
void launch_linear(const float* x, const float* W, const float* bias, float* y, int B, int K, int N, int act,
                   hipStream_t st);


// device helpers shared by the split attention forward (unet_kernels.hip) and
// its backward (unet_vjp.hip)
// the K scale of the split attention: q.k scale times log2 e (S in base-2 units)
__device__ __forceinline__ float kln2(float scale) { return scale * 1.44269504088896340736f; }
// hi / lo f16 halves of 8 fp32 values (the split attention's fragment operands)
// (contraction off: v - hi must not fuse with a multiply that formed v in the
// caller, so the qkv epilogue's K pack and attn_kv_split round identically)
__device__ __forceinline__ void split8_f16(const float (&v)[8], h8v& hi, h8v& lo) {
#pragma clang fp contract(off)
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        hi[t] = (_Float16)v[t];
        lo[t] = (_Float16)(v[t] - (float)hi[t]);
    }
}
// s_waitcnt immediate waiting for vmcnt <= n only (expcnt, lgkmcnt at their maxima)
constexpr int vmcnt_wait(int n) { return (n & 15) | (7 << 4) | (15 << 8) | (((n >> 4) & 3) << 14); }
}  // namespace cfd
