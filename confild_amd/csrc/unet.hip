// U-Net handle: topology (UNetModel.__init__, U/src/unet.py:427-616), parameter
// registry under the reference state_dict keys, weight packing, and the forward
// orchestration (UNetModel.forward, unet.py:634-663) over the HIP kernels of
// unet_kernels.hip.  All activations are NHWC fp32 in one caller-provided
// workspace; the forward issues only kernel launches on the given stream.
#include <algorithm>
#include <cstring>
#include <cmath>
#include <functional>
#include <map>
#include <string>
#include <vector>

#include "sampler.hpp"
#include "unet_kernels.hpp"
#include "unet_train.hpp"

namespace cfd {

enum class Pack { Raw, Conv3, Conv1, EmbW, EmbB };

struct UParam {
    std::string key;
    std::vector<int64_t> shape;
    Pack pack = Pack::Raw;
    size_t offset = 0;   // floats into the parameter arena
    size_t count = 0;
    int emb_row = 0;     // EmbW/EmbB: first row in the concatenated emb matrix
    bool set = false;
    int tpack = 0;       // input-gradient pack: 0 none, 1 transposed (Cin, taps, Cout), 2 upsample 4x4 (Cin, 16, Cout),
                         // 3 transposed with mirrored taps (a stride-1 3x3 input-gradient as a plain convolution)
    size_t toffset = 0;  // floats into the transposed arena
    float split_inv = 1.f;  // split compute: 1 / s, s = power-of-two scale of this conv weight
    float tsplit_inv = 1.f; // the same for the input-gradient pack
};

struct ResSpec {
    std::string pre;
    int cin, cout, emb_off;
};
struct AttnSpec {
    std::string pre;
    int C, heads, ch;
};

// One step of the walk (UNetModel module order).
struct Step {
    enum Kind { In, Res, Attn, Down, Up, Push, Cat, Out } kind;
    int idx = 0;    // index into res/attn specs, or conv key
    std::string conv;  // conv prefix for In/Down/Up/Out
    int cin = 0, cout = 0;
};

}  // namespace cfd

struct cfd_unet {
    cfd_unet_cfg cfg{};
    int device = 0;
    int tdim = 0;
    std::vector<cfd::UParam> params;
    std::map<std::string, int> index;
    std::vector<cfd::ResSpec> res;
    std::vector<cfd::AttnSpec> attn;
    std::vector<cfd::Step> steps;
    int emb_total = 0;      // sum of ResBlock out channels (rows of the emb matrix)
    float* arena = nullptr; // all parameters
    size_t arena_floats = 0;
    float* emb_w = nullptr; // (emb_total, tdim)
    float* emb_b = nullptr; // (emb_total)
    float* freqs = nullptr; // (mc/2) timestep-embedding frequencies
    float* arena_t = nullptr; // transposed conv weights (input-gradient path)
    size_t arena_t_floats = 0;
    uint16_t* arena_bf = nullptr;  // bf16 copy of the conv weights, same offsets as arena
    uint16_t* arena_hi = nullptr;  // split compute: f16 hi / lo parts of the scaled conv weights
    uint16_t* arena_lo = nullptr;
    uint16_t* arena_thi = nullptr;  // split compute: f16 hi / lo parts of the scaled input-gradient packs
    uint16_t* arena_tlo = nullptr;
    int compute = CFD_COMPUTE_SPLIT_F16;
    int plan_b = 0;   // the batch the convolution planner tiles for (0: 8); cfd_unet_set_plan_batch
    int tape_mode = CFD_TAPE_INPUT_VJP;   // what the next forward_tape records
    // every live tape's recording: its layout (mode), batch and planned batch, so a
    // replay (input_vjp / param_grad) walks the layout of the forward that wrote
    // THAT tape, whatever was recorded since on other tapes (host-side: no sync)
    struct TapeRec { int mode, B, plan; uint64_t seq; };
    std::map<const void*, TapeRec> tapes;
    uint64_t tape_seq = 0;
    int* nonfinite = nullptr;  // range guard flag: set by the last convolution on a non-finite eps
    mutable std::map<int, size_t> ws_cache;  // workspace bytes per B (the dry walk is host work)
    uint64_t version = 0;   // bumped by every set_param / set_compute: launch arguments (weight
                            // scales, kernel choice) captured into a graph are stale after it
    // device repack (cfd_unet_load_flat): descriptor table, block -> parameter map, amax scratch
    void* rp_desc = nullptr;
    int64_t* rp_first = nullptr;   // (nparams + 1) first block of each parameter
    float* rp_part = nullptr;      // (nblocks, 2) per-block |max| (forward pack, input-gradient pack)
    float* rp_amax = nullptr;      // (nparams, 2)
    int64_t rp_blocks = 0;
    int64_t* rp_tfirst = nullptr;  // (nparams + 1) first transposing tile of each parameter
    int64_t rp_tiles = 0;
};

namespace {

using cfd::Pack;

void add_param(cfd_unet* h, const std::string& key, std::vector<int64_t> shape, Pack pack, int emb_row = 0) {
    cfd::UParam p;
    p.key = key;
    p.shape = shape;
    p.pack = pack;
    p.emb_row = emb_row;
    p.count = 1;
    for (auto s : shape) p.count *= (size_t)s;
    h->index[key] = (int)h->params.size();
    h->params.push_back(p);
}

void add_conv(cfd_unet* h, const std::string& pre, int cin, int cout, int k, bool conv1d = false, bool up = false,
              bool mirror = false) {
    if (conv1d)
        add_param(h, pre + ".weight", {cout, cin, 1}, Pack::Conv1);
    else
        add_param(h, pre + ".weight", {cout, cin, k, k}, k == 3 ? Pack::Conv3 : Pack::Conv1);
    h->params.back().tpack = up ? 2 : mirror ? 3 : 1;
    add_param(h, pre + ".bias", {cout}, Pack::Raw);
}

void add_norm(cfd_unet* h, const std::string& pre, int c) {
    add_param(h, pre + ".weight", {c}, Pack::Raw);
    add_param(h, pre + ".bias", {c}, Pack::Raw);
}

int add_res(cfd_unet* h, const std::string& pre, int cin, int cout) {
    add_norm(h, pre + ".in_layers.0", cin);
    add_conv(h, pre + ".in_layers.2", cin, cout, 3, false, false, /*mirror=*/true);
    add_param(h, pre + ".emb_layers.1.weight", {cout, h->tdim}, Pack::EmbW, h->emb_total);
    add_param(h, pre + ".emb_layers.1.bias", {cout}, Pack::EmbB, h->emb_total);
    add_norm(h, pre + ".out_layers.0", cout);
    add_conv(h, pre + ".out_layers.3", cout, cout, 3, false, false, /*mirror=*/true);
    if (cin != cout) add_conv(h, pre + ".skip_connection", cin, cout, 1);
    h->res.push_back({pre, cin, cout, h->emb_total});
    h->emb_total += cout;
    return (int)h->res.size() - 1;
}

int add_attn(cfd_unet* h, const std::string& pre, int C) {
    const int heads = h->cfg.num_head_channels == -1 ? h->cfg.num_heads : C / h->cfg.num_head_channels;
    CFD_REQUIRE(heads > 0 && C % heads == 0, CFD_EARG, "channels not divisible into heads at " + pre);
    add_norm(h, pre + ".norm", C);
    add_conv(h, pre + ".qkv", C, 3 * C, 1, true);
    add_conv(h, pre + ".proj_out", C, C, 1, true);
    h->attn.push_back({pre, C, heads, C / heads});
    return (int)h->attn.size() - 1;
}

bool has_attn(const cfd_unet* h, int ds) {
    for (int i = 0; i < h->cfg.n_attn; ++i)
        if (h->cfg.attention_ds[i] == ds) return true;
    return false;
}

// UNetModel.__init__ walk (unet.py:469-616) producing params and steps.
void build(cfd_unet* h) {
    const auto& c = h->cfg;
    const int mc = c.model_channels;
    h->tdim = 4 * mc;
    add_param(h, "time_embed.0.weight", {h->tdim, mc}, Pack::Raw);
    add_param(h, "time_embed.0.bias", {h->tdim}, Pack::Raw);
    add_param(h, "time_embed.2.weight", {h->tdim, h->tdim}, Pack::Raw);
    add_param(h, "time_embed.2.bias", {h->tdim}, Pack::Raw);
    int ch = c.channel_mult[0] * mc;
    add_conv(h, "input_blocks.0.0", c.in_channels, ch, 3);
    h->steps.push_back({cfd::Step::In, 0, "input_blocks.0.0", c.in_channels, ch});
    h->steps.push_back({cfd::Step::Push});
    std::vector<int> chans{ch};
    int ds = 1, idx = 1;
    for (int level = 0; level < c.n_mult; ++level) {
        for (int r = 0; r < c.num_res_blocks; ++r) {
            const int cout = c.channel_mult[level] * mc;
            const std::string pre = "input_blocks." + std::to_string(idx);
            int ri = add_res(h, pre + ".0", ch, cout);
            h->steps.push_back({cfd::Step::Res, ri});
            ch = cout;
            if (has_attn(h, ds)) h->steps.push_back({cfd::Step::Attn, add_attn(h, pre + ".1", ch)});
            h->steps.push_back({cfd::Step::Push});
            chans.push_back(ch);
            ++idx;
        }
        if (level != c.n_mult - 1) {
            const std::string pre = "input_blocks." + std::to_string(idx) + ".0.op";
            add_conv(h, pre, ch, ch, 3);
            h->steps.push_back({cfd::Step::Down, 0, pre, ch, ch});
            h->steps.push_back({cfd::Step::Push});
            chans.push_back(ch);
            ds *= 2;
            ++idx;
        }
    }
    h->steps.push_back({cfd::Step::Res, add_res(h, "middle_block.0", ch, ch)});
    h->steps.push_back({cfd::Step::Attn, add_attn(h, "middle_block.1", ch)});
    h->steps.push_back({cfd::Step::Res, add_res(h, "middle_block.2", ch, ch)});
    idx = 0;
    for (int level = c.n_mult - 1; level >= 0; --level) {
        for (int i = 0; i < c.num_res_blocks + 1; ++i) {
            const int ich = chans.back();
            chans.pop_back();
            const int cout = mc * c.channel_mult[level];
            const std::string pre = "output_blocks." + std::to_string(idx);
            h->steps.push_back({cfd::Step::Cat});
            h->steps.push_back({cfd::Step::Res, add_res(h, pre + ".0", ch + ich, cout)});
            ch = cout;
            int j = 1;
            if (has_attn(h, ds)) {
                h->steps.push_back({cfd::Step::Attn, add_attn(h, pre + ".1", ch)});
                j = 2;
            }
            if (level && i == c.num_res_blocks) {
                const std::string up = pre + "." + std::to_string(j) + ".conv";
                add_conv(h, up, ch, ch, 3, false, true);
                h->steps.push_back({cfd::Step::Up, 0, up, ch, ch});
                ds /= 2;
            }
            ++idx;
        }
    }
    add_norm(h, "out.0", ch);
    add_conv(h, "out.2", c.channel_mult[0] * mc, c.out_channels, 3);
    h->steps.push_back({cfd::Step::Out, 0, "out", ch, c.out_channels});
    // arena layout (emb_layers live in the concatenated emb matrix instead)
    size_t off = 0;
    for (auto& p : h->params) {
        if (p.pack == Pack::EmbW || p.pack == Pack::EmbB) continue;
        p.offset = off;
        off += (p.count + 3) & ~size_t(3);  // keep 16-B alignment
    }
    h->arena_floats = off;
    size_t toff = 0;
    for (auto& p : h->params) {
        if (!p.tpack) continue;
        p.toffset = toff;
        toff += ((p.tpack == 2 ? p.count / 9 * 16 : p.count) + 3) & ~size_t(3);
    }
    h->arena_t_floats = toff;
}

// bf16 copy (bf16 compute) / f16 hi part (split compute) of a packed conv weight,
// or null in fp32 compute
const void* PB(const cfd_unet* h, const std::string& key) {
    if (h->compute == CFD_COMPUTE_F32) return nullptr;
    auto it = h->index.find(key);
    CFD_REQUIRE(it != h->index.end(), CFD_EKEY, "internal: missing param " + key);
    return (h->compute == CFD_COMPUTE_BF16 ? h->arena_bf : h->arena_hi) + h->params[it->second].offset;
}

// split compute: f16 lo part and 1/s of a packed conv weight (null / 1 otherwise)
const void* PL(const cfd_unet* h, const std::string& key, float* inv) {
    *inv = 1.f;
    if (h->compute != CFD_COMPUTE_SPLIT_F16) return nullptr;
    auto it = h->index.find(key);
    CFD_REQUIRE(it != h->index.end(), CFD_EKEY, "internal: missing param " + key);
    *inv = h->params[it->second].split_inv;
    return h->arena_lo + h->params[it->second].offset;
}

// fp32 -> bf16, round to nearest even (what v_cvt_pk_bf16_f32 does on the device)
uint16_t to_bf16(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);
    return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

// split compute: f16 hi / lo parts and 1/s of an input-gradient pack into a
// (nothing in the other modes: their transposed convolutions run in fp32)
void PTS(const cfd_unet* h, const std::string& key, cfd::ConvArgs* a) {
    if (h->compute != CFD_COMPUTE_SPLIT_F16) return;
    auto it = h->index.find(key);
    CFD_REQUIRE(it != h->index.end() && h->params[it->second].tpack, CFD_EKEY, "internal: missing conv " + key);
    const auto& p = h->params[it->second];
    a->wbf = h->arena_thi + p.toffset;
    a->wlo = h->arena_tlo + p.toffset;
    a->acc_scale = p.tsplit_inv;
}

const float* PT(const cfd_unet* h, const std::string& key) {
    auto it = h->index.find(key);
    CFD_REQUIRE(it != h->index.end() && h->params[it->second].tpack, CFD_EKEY, "internal: missing conv " + key);
    return h->arena_t + h->params[it->second].toffset;
}

const float* P(const cfd_unet* h, const std::string& key) {
    auto it = h->index.find(key);
    CFD_REQUIRE(it != h->index.end(), CFD_EKEY, "internal: missing param " + key);
    return h->arena + h->params[it->second].offset;
}

// A (possibly two-source) activation view, NHWC with batch B.
struct Act {
    const float* a = nullptr;
    int Ca = 0;
    const float* b = nullptr;
    int Cb = 0;
    int H = 0, W = 0;
    int C() const { return Ca + Cb; }
    bool bf16 = false;   // a holds bf16 (a GroupNorm's out_bf16 output; read by K1hb only)
};

struct Workspace {
    char* base;
    size_t off = 0;
    bool dry;
    float* take(size_t nfloats) {
        off = (off + 255) & ~size_t(255);
        float* p = dry ? nullptr : (float*)(base + off);
        off += nfloats * sizeof(float);
        return p;
    }
};

// What the input-gradient walk needs from one forward step.
struct Rec {
    Act in;                         // step input
    const float* h1 = nullptr;      // Res: in_layers output (conv1 + bias + emb)
    float *ss1 = nullptr, *st1 = nullptr;  // first GroupNorm: scale/shift, mean/rstd
    float *ss2 = nullptr, *st2 = nullptr;  // Res: out_layers GroupNorm
    float *qkv = nullptr, *o = nullptr, *lse = nullptr;  // Attn
    // with a tape: the GroupNorm(+SiLU) outputs the next convolutions read, kept,
    // and a slot with max |.| of each (the split weight gradients' X ranges)
    const float *act1 = nullptr, *act2 = nullptr;
    unsigned *amx1 = nullptr, *amx2 = nullptr;
    int skip_hs = -1;               // Res on a concat: skip-stack index of the second source
    int push_hs = -1;               // Push: skip-stack index
};

// Forward tape: every activation the input-gradient needs lives in its own
// region of the tape (nothing is recycled); recs describes where.
struct Tape {
    Workspace* tws;
    std::vector<Rec>* recs;
    // CFD_TAPE_PARAM_GRAD: also keep the GroupNorm(+SiLU) outputs and their ranges
    bool keep_gnout = false;
    // the timestep-embedding MLP's activations (kept for the parameter gradients):
    // timestep_embedding (B, mc), time_embed.0 output (B, tdim), emb (B, tdim)
    float* temb = nullptr;
    float* th1 = nullptr;
    float* emb = nullptr;
};

struct Sizes {
    size_t max_act = 0, max_qkv = 0, max_cat = 0, max_att = 0;  // floats per sample
    size_t max_kvf = 0;  // split attention's packed K/V fragments (any level)
    size_t max_abw = 0;  // split attention backward's packs and scales (attention levels)
    size_t max_apart = 0;  // key-chunked attention's partials (attention_kv_chunks > 1)
    std::vector<size_t> hs;                                     // skip-stack tensors, floats per sample
};

int plan_batch(const cfd_unet* h);

Sizes sizes(const cfd_unet* h) {
    const auto& c = h->cfg;
    const int mc = c.model_channels, S = c.image_size;
    Sizes z;
    int ch = c.channel_mult[0] * mc, hw = S, cmax = 0;
    z.max_act = (size_t)hw * hw * ch;
    z.hs.push_back((size_t)hw * hw * ch);
    for (int l = 0; l < c.n_mult; ++l) cmax = std::max(cmax, c.channel_mult[l] * mc);
    for (int l = 0; l < c.n_mult; ++l) {
        const int co = c.channel_mult[l] * mc;
        z.max_act = std::max(z.max_act, (size_t)hw * hw * std::max(co, ch));
        z.max_qkv = std::max(z.max_qkv, (size_t)hw * hw * 3 * co);
        // normalised concat input of an output block: hw^2 * (C_level + C_max)
        z.max_cat = std::max(z.max_cat, (size_t)hw * hw * (co + cmax));
        z.max_att = std::max(z.max_att, (size_t)hw * hw * co);  // heads * T <= C * T
        z.max_kvf = std::max(z.max_kvf, cfd::attention_split_floats(hw * hw, co));
        if (has_attn(h, 1 << l) || l == c.n_mult - 1) {   // (the middle block attends at the last level)
            z.max_abw = std::max(z.max_abw, cfd::attention_bwd_split_floats(hw * hw, co));
            const int heads = c.num_head_channels == -1 ? c.num_heads : co / c.num_head_channels;
            z.max_apart = std::max(z.max_apart, cfd::attention_part_floats(hw * hw, co, co / heads, plan_batch(h)));
        }
        for (int r = 0; r < c.num_res_blocks; ++r) z.hs.push_back((size_t)hw * hw * co);
        ch = co;
        if (l != c.n_mult - 1) {
            hw /= 2;
            z.hs.push_back((size_t)hw * hw * ch);
        }
    }
    z.max_cat = std::max(z.max_cat, z.max_act);
    return z;
}

// split-K partial slab
constexpr size_t kSplitPer8 = size_t(16) << 20;
// the batch the convolution planner and gn2 tile for: the model's setting
// (cfd_unet_set_plan_batch), else 8
int plan_batch(const cfd_unet* h) { return h->plan_b > 0 ? h->plan_b : 8; }
// (kSplitPer8 per planned batch: plan_conv keeps splits * (plan_b samples' M x N)
// within it, so ceil(B / plan_b) of those cover any real batch)
size_t split_cap(const cfd_unet* h, int B) {
    const int pb = plan_batch(h);
    return kSplitPer8 * (size_t)std::max(1, (B + pb - 1) / pb);
}

cfd::ConvPlan plan_checked(const cfd_unet* h, const cfd::ConvArgs& a0, size_t slab_floats) {
    cfd::ConvArgs a = a0;
    a.plan_b = plan_batch(h);
    const cfd::ConvPlan p = cfd::plan_conv(a, kSplitPer8);
    CFD_REQUIRE(p.splits == 1 || (size_t)p.splits * a.M * a.Cout <= slab_floats, CFD_ESTATE,
                "internal: split-K slab too small");
    return p;
}

// Executes (or, with ws.dry, sizes) one forward.  With a tape, the activations
// the input-gradient needs are kept in the tape and described in tape->recs;
// launch == false replays the walk to recover those pointers without running.
void run(const cfd_unet* h, const float* x, const int64_t* t, float* eps, int B, Workspace& ws, hipStream_t st,
         Tape* tape = nullptr, bool launch_req = true) {
    const auto& c = h->cfg;
    const int mc = c.model_channels, S = c.image_size;
    const Sizes z = sizes(h);
    const bool launch = launch_req && !ws.dry && !(tape && tape->tws->dry);
    const size_t kSplitCap = split_cap(h, B);
    float* temb = tape ? tape->tws->take((size_t)B * mc) : ws.take((size_t)B * mc);
    float* h1 = tape ? tape->tws->take((size_t)B * h->tdim) : ws.take((size_t)B * h->tdim);
    float* emb = tape ? tape->tws->take((size_t)B * h->tdim) : ws.take((size_t)B * h->tdim);
    if (tape) {
        tape->temb = temb;
        tape->th1 = h1;
        tape->emb = emb;
    }
    float* embo = ws.take((size_t)B * h->emb_total);
    double* gnpart = (double*)ws.take((size_t)B * cfd::kGnMaxChunks * 32 * 2 * 2);
    float* gnss = ws.take((size_t)B * 1024 * 2);
    // normalised (+SiLU) input of the next conv (widest: an output block's concat)
    float* nbuf = ws.take((size_t)B * z.max_cat);
    float* splitk = ws.take(kSplitCap);
    float* kvws = ws.take((size_t)B * z.max_kvf);
    float* apart = z.max_apart ? ws.take((size_t)B * z.max_apart) : nullptr;
    float* pool[3];
    for (auto& p : pool) p = ws.take((size_t)B * z.max_act);
    float* tmp = ws.take((size_t)B * z.max_act);
    float* skipb = ws.take((size_t)B * z.max_act);
    float* qkv = tape ? nullptr : ws.take((size_t)B * z.max_qkv);
    float* abuf = tape ? nullptr : ws.take((size_t)B * z.max_act);
    // skip stack buffers (one per Push); in the tape when recording
    std::vector<float*> hsbuf;
    for (size_t n : z.hs) hsbuf.push_back(tape ? tape->tws->take((size_t)B * n) : ws.take((size_t)B * n));
    constexpr int kGnSlots = 256;   // the kept GroupNorm outputs' range slots (tape)
    unsigned* gslots = tape ? (unsigned*)tape->tws->take(kGnSlots) : nullptr;
    int ngs = 0;
    if (ws.dry && !tape) return;
    auto keep = [&](size_t nfloats) -> float* { return tape->tws->take(nfloats); };
    if (tape && tape->keep_gnout && launch) CFD_HIP(hipMemsetAsync(gslots, 0, sizeof(unsigned) * kGnSlots, st));
    std::vector<Rec>* recs = tape ? tape->recs : nullptr;
    if (recs) recs->assign(h->steps.size(), Rec{});

    auto pick = [&](const float* busy1, const float* busy2) -> float* {
        if (!launch && (ws.dry || !busy1)) return pool[0];
        for (auto p : pool)
            if (p != busy1 && p != busy2) return p;
        throw cfd::Error{CFD_ESTATE, "internal: buffer pool exhausted"};
    };

    // timestep embedding + time_embed MLP + every ResBlock's emb_layers (nn.py:118-136, unet.py:648,199-205)
    if (launch) {
        cfd::launch_temb(t, h->freqs, temb, mc, B, st);
        cfd::launch_linear(temb, P(h, "time_embed.0.weight"), P(h, "time_embed.0.bias"), h1, B, mc, h->tdim, 0, st);
        cfd::launch_linear(h1, P(h, "time_embed.2.weight"), P(h, "time_embed.2.bias"), emb, B, h->tdim, h->tdim, 1,
                           st);
        cfd::launch_linear(emb, h->emb_w, h->emb_b, embo, B, h->tdim, h->emb_total, 1, st);
    }

    // A split-K convolution's reduction is deferred to its consumer: the
    // GroupNorm that reads it (GnArgs::kpart) or, before any other launch,
    // splitk_reduce (flush).  The partial slab is shared, so a convolution
    // also flushes first.
    struct Pending {
        cfd::ConvArgs a{};
        int splits = 0;
    } pend;
    auto flush = [&]() {
        if (pend.splits > 1 && launch) cfd::launch_splitk_reduce(pend.a, pend.splits, st);
        pend.splits = 0;
    };

    // GroupNorm(+SiLU) of `in` materialised once into nbuf (contiguous Ctot channels);
    // with a tape the scale/shift and group statistics are kept in *ss / *stats
    // keep_raw == false: a deferred split-K sum this GroupNorm reduces is read by
    // nothing else, so it is not stored (the GroupNorm of in_layers' output
    // without a tape)
    auto gn = [&](const Act& in, const std::string& pre, int silu, float** ss, float** stats,
                  bool keep_raw = true, bool bf16_out = false, const float** actp = nullptr,
                  unsigned** amxp = nullptr) -> Act {
        cfd::GnArgs g{};
        g.src1 = in.a;
        g.src2 = in.b;
        g.gamma = P(h, pre + ".weight");
        g.beta = P(h, pre + ".bias");
        g.part = gnpart;
        g.ss = gnss;
        if (tape) {
            *ss = g.ss = keep((size_t)B * in.C() * 2);
            *stats = g.stats = keep((size_t)B * 64);
        }
        g.out = nbuf;
        // CFD_TAPE_PARAM_GRAD tapes keep it (the input-VJP tapes do not: the weight
        // gradients then recompute the activated input)
        if (tape && actp && tape->keep_gnout) {   // kept for the weight gradients, with its range
            CFD_REQUIRE(!bf16_out && ngs < kGnSlots, CFD_ESTATE, "internal: kept GroupNorm output");
            g.out = keep((size_t)B * in.H * in.W * in.C());
            g.amax_out = gslots + ngs++;
            *actp = g.out;
            *amxp = g.amax_out;
        }
        g.C1 = in.Ca;
        g.C2 = in.Cb;
        g.Ctot = in.C();
        g.HW = in.H * in.W;
        g.eps = 1e-5f;
        g.plan_b = plan_batch(h);
        g.silu = silu;
        if (pend.splits > 1 && pend.a.out == in.a && pend.a.Cout == in.Ca && cfd::gn_takes_splitk(g, B)) {
            g.kpart = pend.a.part;
            g.ksplits = pend.splits;
            g.kbias = pend.a.bias;
            g.kemb = pend.a.emb;
            g.kemb_stride = pend.a.emb_stride;
            g.kres = pend.a.res;
            g.kx = keep_raw || cfd::gn2_applies(g) ? pend.a.out : nullptr;
            pend.splits = 0;
        } else {
            flush();
        }
        static const int gn_log = getenv("CFD_CONV_LOG") ? atoi(getenv("CFD_CONV_LOG")) : 0;
        if (gn_log && launch)   // development: one line per GroupNorm, in launch order
            fprintf(stderr, "GN %s %dx%d C=%d+%d ksplits=%d kres=%d kx=%d silu=%d\n", pre.c_str(), in.H, in.W, g.C1,
                    g.C2, g.kpart ? g.ksplits : 0, g.kres ? 1 : 0, g.kx ? 1 : 0, silu);
        g.out_bf16 = bf16_out ? 1 : 0;
        if (launch) cfd::launch_gn(g, B, st);
        Act r{g.out, in.C(), nullptr, 0, in.H, in.W};
        r.bf16 = bf16_out;
        return r;
    };
    auto conv_args = [&](const Act& in, const std::string& pre, int cout, int ks, int stride, int up,
                         const float* embp, const float* resp, float* out) {
        cfd::ConvArgs a{};
        a.src1 = in.a;
        a.src2 = in.b;
        a.C1 = in.Ca;
        a.C2 = in.Cb;
        a.Ctot = in.C();
        a.w = P(h, pre + ".weight");
        a.wbf = PB(h, pre + ".weight");
        a.wlo = PL(h, pre + ".weight", &a.acc_scale);
        a.bias = P(h, pre + ".bias");
        a.emb = embp;
        a.emb_stride = h->emb_total;
        a.res = resp;
        a.out = out;
        a.part = splitk;
        a.Hin = in.H;
        a.Win = in.W;
        a.Hout = up ? in.H * 2 : (stride == 2 ? (in.H + 1) / 2 : in.H);
        a.Wout = up ? in.W * 2 : (stride == 2 ? (in.W + 1) / 2 : in.W);
        a.stride = stride;
        a.ks = ks;
        a.pad = ks == 3 ? 1 : 0;
        a.up = up;
        a.Cout = cout;
        a.M = B * a.Hout * a.Wout;
        a.K = ks * ks * a.Ctot;
        a.src_bf16 = in.bf16 ? 1 : 0;
        return a;
    };
    // config E: a ResBlock GroupNorm writes bf16 where its consumer convolution runs
    // on K1hb, which rounds the operand to bf16 as it stages it -- the same bits
    // (CFD_GN_BF16OUT=0 keeps fp32 outputs)
    static const int gn_bf16out = getenv("CFD_GN_BF16OUT") ? atoi(getenv("CFD_GN_BF16OUT")) : 1;
    auto feeds_k1hb = [&](const Act& in, const std::string& pre, int cout) -> bool {
        if (!gn_bf16out || h->compute != CFD_COMPUTE_BF16) return false;
        Act n{nbuf, in.C(), nullptr, 0, in.H, in.W};
        const cfd::ConvArgs a = conv_args(n, pre, cout, 3, 1, 0, nullptr, nullptr, nullptr);
        return a.wbf && !a.wlo && cfd::conv_runs_k1hb(a, plan_checked(h, a, kSplitCap));
    };
    // tweak: adjusts the launch arguments once the plan is known (the qkv K / V pack)
    using Tweak = std::function<void(cfd::ConvArgs&, const cfd::ConvPlan&)>;
    auto conv = [&](const Act& in, const std::string& pre, int cout, int ks, int stride, int up,
                    const float* embp, const float* resp, float* out, const Tweak& tweak = {}) {
        cfd::ConvArgs a = conv_args(in, pre, cout, ks, stride, up, embp, resp, out);
        flush();
        const cfd::ConvPlan plan = plan_checked(h, a, kSplitCap);
        if (tweak) tweak(a, plan);
        CFD_REQUIRE(!a.src_bf16 || cfd::conv_runs_k1hb(a, plan), CFD_ESTATE,
                    "internal: bf16 GroupNorm output feeds a convolution other than K1hb at " + pre);
        static const int conv_log = getenv("CFD_CONV_LOG") ? atoi(getenv("CFD_CONV_LOG")) : 0;
        if (conv_log && launch)   // development: one line per convolution, in launch order
            fprintf(stderr, "CONV %s %dx%d C=%d+%d->%d ks=%d s=%d up=%d M=%d kx=%d bm=%d bn=%d nw=%d splits=%d\n",
                    pre.c_str(), a.Hin, a.Win, a.C1, a.C2, a.Cout, a.ks, a.stride, a.up, a.M, plan.kx, plan.bm,
                    plan.bn, plan.nw, plan.splits);
        if (launch) {
            const int sp = cfd::launch_conv(a, plan, st, /*defer=*/true);   // the splits it left to reduce
            if (sp > 1) {
                pend.a = a;
                pend.splits = sp;
            }
        }
    };

    std::vector<std::pair<Act, int>> stack;  // (tensor, skip index)
    Act cur;
    size_t hs_i = 0;
    int pending_skip = -1;
    for (size_t si = 0; si < h->steps.size(); ++si) {
        const auto& s = h->steps[si];
        Rec rec;
        rec.in = cur;
        // a block output that is pushed onto the skip stack is written straight
        // into its skip buffer (no copy); with a tape every output is kept
        const bool to_skip = si + 1 < h->steps.size() && h->steps[si + 1].kind == cfd::Step::Push;
        auto dest = [&](const float* busy1, const float* busy2, size_t nfl) -> float* {
            if (to_skip) return hsbuf[hs_i];
            return tape ? keep(nfl) : pick(busy1, busy2);
        };
        switch (s.kind) {
            case cfd::Step::In: {
                cfd::ConvArgs a{};
                a.src1 = x;
                a.C1 = c.in_channels;
                a.Ctot = c.in_channels;
                a.w = P(h, s.conv + ".weight");
                a.bias = P(h, s.conv + ".bias");
                a.out = hsbuf[0];
                a.Hin = a.Hout = S;
                a.Win = a.Wout = S;
                a.Cout = s.cout;
                a.M = B * S * S;
                if (launch) cfd::launch_conv_in(a, st);
                cur = Act{hsbuf[0], s.cout, nullptr, 0, S, S};
                break;
            }
            case cfd::Step::Push: {
                // the current activation must live in its own skip buffer
                float* dst = hsbuf[hs_i];
                if (cur.a != dst) {
                    flush();
                    if (launch)
                        CFD_HIP(hipMemcpyAsync(dst, cur.a, sizeof(float) * (size_t)B * cur.H * cur.W * cur.Ca,
                                               hipMemcpyDeviceToDevice, st));
                    cur.a = dst;
                }
                rec.push_hs = (int)hs_i;
                stack.push_back({cur, (int)hs_i});
                ++hs_i;
                break;
            }
            case cfd::Step::Cat: {
                const auto skip = stack.back();
                stack.pop_back();
                CFD_REQUIRE(cur.b == nullptr && skip.first.H == cur.H, CFD_ESTATE, "internal: concat shape");
                cur.b = skip.first.a;
                cur.Cb = skip.first.Ca;
                pending_skip = skip.second;
                break;
            }
            case cfd::Step::Res: {
                const auto& r = h->res[s.idx];
                CFD_REQUIRE(cur.C() == r.cin, CFD_ESTATE, "internal: ResBlock input channels at " + r.pre);
                rec.skip_hs = pending_skip;
                pending_skip = -1;
                const size_t nout = (size_t)B * cur.H * cur.W * r.cout;
                // h = in_layers(x) + emb_layers(emb)   (unet.py:236-254)
                const Act xin = gn(cur, r.pre + ".in_layers.0", 1, &rec.ss1, &rec.st1, true,
                                   feeds_k1hb(cur, r.pre + ".in_layers.2", r.cout), &rec.act1, &rec.amx1);
                // skip(x) (unet.py:255-256): its own convolution just before the
                // out_layers one (in_layers' deferred reduction still meets the
                // out_layers GroupNorm), read back as that convolution's residual
                const float* resp = nullptr;
                if (r.cin != r.cout) {
                    resp = skipb;
                } else {
                    CFD_REQUIRE(cur.b == nullptr, CFD_ESTATE, "identity skip on a concatenated input");
                    resp = cur.a;
                }
                float* hb = tape ? keep(nout) : tmp;
                conv(xin, r.pre + ".in_layers.2", r.cout, 3, 1, 0, embo + r.emb_off, nullptr, hb);
                rec.h1 = hb;
                const Act th{hb, r.cout, nullptr, 0, cur.H, cur.W};
                const Act hn = gn(th, r.pre + ".out_layers.0", 1, &rec.ss2, &rec.st2, /*keep_raw=*/tape != nullptr,
                                  feeds_k1hb(th, r.pre + ".out_layers.3", r.cout), &rec.act2, &rec.amx2);
                float* out = dest(cur.a, cur.b, nout);
                if (r.cin != r.cout)   // reads the block input, still intact: out is another buffer
                    conv(cur, r.pre + ".skip_connection", r.cout, 1, 1, 0, nullptr, nullptr, skipb);
                conv(hn, r.pre + ".out_layers.3", r.cout, 3, 1, 0, nullptr, resp, out);
                cur = Act{out, r.cout, nullptr, 0, cur.H, cur.W};
                break;
            }
            case cfd::Step::Attn: {
                const auto& at = h->attn[s.idx];
                const int T = cur.H * cur.W;
                const Act xn = gn(cur, at.pre + ".norm", 0, &rec.ss1, &rec.st1, true, false, &rec.act1, &rec.amx1);
                float* qb = tape ? keep((size_t)B * T * 3 * at.C) : qkv;
                float* ob = tape ? keep((size_t)B * T * at.C) : abuf;
                const float attn_scale = (float)(1.0 / std::sqrt(std::sqrt((double)at.ch)));
                const bool split_attn = h->compute != CFD_COMPUTE_F32 && (at.ch == 32 || at.ch == 64 || at.ch == 128);
                bool kv_packed = false;
                // the qkv convolution; in split compute its epilogue also packs K / V
                conv(xn, at.pre + ".qkv", 3 * at.C, 1, 1, 0, nullptr, nullptr, qb,
                     [&](cfd::ConvArgs& a, const cfd::ConvPlan& plan) {
                         if (!split_attn || h->compute == CFD_COMPUTE_F32 || !cfd::conv_kv_pack_ok(a, plan, T))
                             return;
                         a.kvf = kvws;
                         a.kv_voff = cfd::attention_split_voff(T, at.ch, at.heads, B);
                         a.kv_ch = at.ch;
                         a.kv_heads = at.heads;
                         a.kv_T = T;
                         a.kv_scale = attn_scale;
                         kv_packed = true;
                     });
                cfd::AttnArgs aa{qb, ob, T, at.C, attn_scale, nullptr};
                aa.part = apart;
                if (tape) aa.lse = keep((size_t)B * at.heads * T);
                rec.qkv = qb;
                rec.o = ob;
                rec.lse = aa.lse;
                flush();
                if (launch) {
                    // split-f16 attention (fp32-accurate, K4d) in the split and the bf16 modes: the
                    // reference's fp16 contract runs q.k and a.v in the low precision with an fp32
                    // softmax (unet.py:349-353), so fp32-level attention is within it; the exact
                    // fp32-MFMA kernel K4 stays for CFD_COMPUTE_F32
                    if (split_attn)
                        cfd::launch_attention_split(aa, at.ch, at.heads, B, plan_batch(h), kvws, st, kv_packed);
                    else
                        cfd::launch_attention(aa, at.ch, at.heads, B, st);
                }
                float* out = dest(cur.a, nullptr, (size_t)B * T * at.C);
                conv(Act{ob, at.C, nullptr, 0, cur.H, cur.W}, at.pre + ".proj_out", at.C, 1, 1, 0, nullptr, cur.a,
                     out);
                cur = Act{out, at.C, nullptr, 0, cur.H, cur.W};
                break;
            }
            case cfd::Step::Down: {
                const int Ho = (cur.H + 1) / 2, Wo = (cur.W + 1) / 2;
                float* out = dest(cur.a, nullptr, (size_t)B * Ho * Wo * s.cout);
                conv(cur, s.conv, s.cout, 3, 2, 0, nullptr, nullptr, out);
                cur = Act{out, s.cout, nullptr, 0, Ho, Wo};
                break;
            }
            case cfd::Step::Up: {
                float* out = tape ? keep((size_t)B * 4 * cur.H * cur.W * s.cout) : pick(cur.a, nullptr);
                conv(cur, s.conv, s.cout, 3, 1, 1, nullptr, nullptr, out);
                cur = Act{out, s.cout, nullptr, 0, cur.H * 2, cur.W * 2};
                break;
            }
            case cfd::Step::Out: {
                const Act on = gn(cur, "out.0", 1, &rec.ss1, &rec.st1, true, false, &rec.act1, &rec.amx1);
                cfd::ConvArgs a{};
                a.src1 = on.a;
                a.C1 = on.Ca;
                a.Ctot = on.Ca;
                a.w = P(h, "out.2.weight");
                a.bias = P(h, "out.2.bias");
                a.out = eps;
                a.Hin = a.Hout = cur.H;
                a.Win = a.Wout = cur.W;
                a.Cout = c.out_channels;
                a.M = B * cur.H * cur.W;
                a.K = 9 * cur.Ca;
                a.nonfinite = h->nonfinite;
                flush();
                if (launch) cfd::launch_conv_out(a, st);
                break;
            }
        }
        if (recs) (*recs)[si] = rec;
    }
    flush();
}


// Input-gradient d_x = (d eps / d x)^T d_eps of the forward recorded in the tape
// (DPS adjoint: the autograd.grad of grad_and_value through the U-Net,
// condition_methods.py:31-47; weights are constants, so only data gradients).
// Walks the steps in reverse; convolution input-gradients run on conv_gemm with
// the transposed weight packs (stride-1/2 via TMODE, Upsample+conv as one 4x4
// stride-2 convolution), GroupNorm(+SiLU) and attention backward in unet_vjp.hip.
// Parameter gradients (K11, the TrainLoop's backward) ride on the same walk: with
// pg != null every convolution's weight / bias gradient, every GroupNorm's gamma /
// beta gradient, the emb_layers and time_embed gradients are accumulated (+=)
// into pg->grad (cfd_unet_param_info order, reference shapes).
struct ParamGrad {
    float* grad = nullptr;
    const float* x = nullptr;                                     // the forward's input (B, in_ch, S, S)
    const float *temb = nullptr, *th1 = nullptr, *emb = nullptr;  // Tape's embedding activations
};

constexpr int kRangeSlots = 1024;   // zeroed once per parameter-gradient backward

void run_vjp(const cfd_unet* h, const float* d_eps, float* d_x, int B, const std::vector<Rec>& recs, Workspace& ws,
             hipStream_t st, const ParamGrad* pg = nullptr, bool pg_ws = false) {
    const auto& c = h->cfg;
    const int S = c.image_size;
    const Sizes z = sizes(h);
    const size_t kSplitCap = split_cap(h, B);
    float* splitk = ws.take(kSplitCap);
    double* gnpart = (double*)ws.take((size_t)B * cfd::kGnMaxChunks * 32 * 2 * 2);
    float* gnfin = ws.take((size_t)B * 64);
    float* gpool[4];
    for (auto& p : gpool) p = ws.take((size_t)B * z.max_cat);
    float* dqkv = ws.take((size_t)B * z.max_qkv);
    float* dd = ws.take((size_t)B * z.max_att);
    float* abws = ws.take((size_t)B * z.max_abw);
    std::vector<float*> dhs;
    for (size_t n : z.hs) dhs.push_back(ws.take((size_t)B * n));
    // parameter-gradient scratch (pg_ws: sized in the dry walk of cfd_unet_param_grad_workspace_bytes)
    float *wpart = nullptr, *cpart = nullptr, *crow = nullptr, *demb = nullptr, *dth1 = nullptr, *gpp = nullptr;
    float* wact = nullptr;
    unsigned* wamax = nullptr;
    float* wbpart = nullptr;
    size_t wcap = 0, ccap = 0, bcap = 0;
    if (pg_ws) {
        int cmax = 0;
        for (int l = 0; l < c.n_mult; ++l) cmax = std::max(cmax, c.channel_mult[l] * c.model_channels);
        wcap = (size_t)16 * 3 * cmax * 2 * cmax * 9;    // <= 16 pixel slices of Cout x Ctot x 9 (qkv: 3C x C)
        ccap = (size_t)(256 + B) * std::max(3 * cmax, h->tdim);
        wpart = ws.take(wcap);
        cpart = ws.take(ccap);    // colsum_part_floats: <= 256 + B (slice, row) pairs of F columns
        wact = ws.take((size_t)B * z.max_cat);   // the activated input of a weight-gradient product
        crow = ws.take((size_t)B * std::max(3 * cmax, h->tdim));
        demb = ws.take((size_t)B * h->tdim);
        dth1 = ws.take((size_t)B * h->tdim);
        gpp = ws.take((size_t)B * cfd::kGnMaxChunks * 2 * cmax * 2);
        wamax = (unsigned*)ws.take(kRangeSlots);   // the split weight gradients' operand ranges, a slot each
        bcap = (size_t)64 * 3 * cmax;
        wbpart = ws.take(bcap);   // bias-gradient slices of the split product kernel
    }
    if (ws.dry) return;
    std::vector<size_t> goff;
    {
        size_t o = 0;
        for (const auto& p : h->params) {
            goff.push_back(o);
            o += p.count;
        }
    }
    auto GP = [&](const std::string& key) -> float* {
        auto it = h->index.find(key);
        CFD_REQUIRE(it != h->index.end(), CFD_EKEY, "internal: no parameter " + key);
        return pg->grad + goff[it->second];
    };
    // split weight gradients: one zeroed range slot per operand range (max |dY|,
    // max |X|); the GroupNorm backward's output carries its max |.| in a slot too
    // (GnbArgs::amax_out), which a later weight gradient of that tensor reuses
    int nslot = 0;
    const bool split_w = pg && h->compute == CFD_COMPUTE_SPLIT_F16;
    auto slot = [&]() -> unsigned* {
        if (!split_w) return nullptr;
        CFD_REQUIRE(nslot < kRangeSlots, CFD_ESTATE, "internal: range slots exhausted");
        return wamax + nslot++;
    };
    // weight / bias gradient of one convolution: dY (B, Hout, Wout, cout) against its
    // forward input; ymax: a slot already holding max |dY| (or null).  Returns the
    // slot that holds max |dY| afterwards (for a later product of the same dY)
    auto wgrad = [&](const float* dy, int cout, const Act& X, const float* ss, int silu, int Hout, int Wout, int ks,
                     int stride, int pad, int up, const std::string& pre, unsigned* ymax = nullptr,
                     unsigned* xmax = nullptr) -> unsigned* {
        CFD_REQUIRE(pg_ws && cfd::colsum_part_floats((int64_t)B * Hout * Wout, cout, 1) <= ccap &&
                        (size_t)cout * X.C() * ks * ks <= wcap && (size_t)X.H * X.W * X.C() <= z.max_cat,
                    CFD_ESTATE, "internal: weight-gradient scratch");
        cfd::WgradArgs a{};
        a.part_cap = (int64_t)wcap;
        a.act = wact;
        a.dy = dy;
        a.src1 = X.a;
        a.src2 = X.b;
        a.C1 = X.Ca;
        a.C2 = X.Cb;
        a.Ctot = X.C();
        a.ss = ss;
        a.silu = silu;
        a.part = wpart;
        // split-f16 weight-gradient products in split compute (the exact fp32-MFMA
        // kernel in the fp32 / bf16 modes)
        if (split_w) {
            a.xmax_known = xmax ? 1 : 0;
            a.amax_x = xmax ? xmax : slot();
            a.ymax_known = ymax ? 1 : 0;
            a.amax_y = ymax ? ymax : slot();
        }
        a.P = (int64_t)B * Hout * Wout;
        a.Cout = cout;
        a.Hin = X.H;
        a.Win = X.W;
        a.Hout = Hout;
        a.Wout = Wout;
        a.ks = ks;
        a.stride = stride;
        a.pad = pad;
        a.up = up;
        a.bpart = wbpart;
        a.bpart_cap = (int64_t)bcap;
        a.Gb = GP(pre + ".bias");
        if (!cfd::launch_conv_wgrad(a, GP(pre + ".weight"), st)) {   // the bias gradient not fused: sum dY
            cfd::launch_colsum(dy, a.P, cout, 1, cpart, crow, st);
            cfd::launch_rows_accum(crow, 1, cout, GP(pre + ".bias"), st);
        }
        return a.amax_y;
    };
    if (pg) CFD_HIP(hipMemsetAsync(demb, 0, sizeof(float) * B * h->tdim, st));
    if (split_w) CFD_HIP(hipMemsetAsync(wamax, 0, sizeof(unsigned) * kRangeSlots, st));

    auto gfree = [&](const float* b1, const float* b2 = nullptr, const float* b3 = nullptr) -> float* {
        for (auto p : gpool)
            if (p != b1 && p != b2 && p != b3) return p;
        throw cfd::Error{CFD_ESTATE, "internal: gradient pool exhausted"};
    };
    // input-gradient of a convolution: dY (Hin x Win, Cin_bwd channels) -> dX (Hout x Wout, cout)
    auto dconv = [&](const float* dy, int cin, int Hin, int Win, const std::string& key, int cout, int Hout, int Wout,
                     int ks, int stride, int pad, int tmode, float* out) {
        {   // a pack kind runs only in its addressing mode: mirrored taps (3) as a plain
            // convolution, the transposed pack (1) through TMODE, upsample (2) plain
            auto it = h->index.find(key);
            CFD_REQUIRE(it != h->index.end(), CFD_EKEY, "internal: missing conv " + key);
            const int tp = h->params[it->second].tpack;
            CFD_REQUIRE((tp == 3 && tmode == 0) || (tp == 1 && tmode == 1) || (tp == 2 && tmode == 0) ||
                            (tp == 1 && ks == 1),
                        CFD_ESTATE, "internal: input-gradient pack kind / addressing mismatch at " + key);
        }
        cfd::ConvArgs a{};
        a.src1 = dy;
        a.C1 = cin;
        a.Ctot = cin;
        a.w = PT(h, key);
        PTS(h, key, &a);
        a.out = out;
        a.part = splitk;
        a.Hin = Hin;
        a.Win = Win;
        a.Hout = Hout;
        a.Wout = Wout;
        a.stride = stride;
        a.ks = ks;
        a.pad = pad;
        a.tmode = tmode;
        a.Cout = cout;
        a.M = B * Hout * Wout;
        a.K = ks * ks * cin;
        cfd::launch_conv(a, plan_checked(h, a, kSplitCap), st);
    };
    // with_param (training): the GroupNorm's parameter-gradient partials come out of
    // the same statistics pass (GnbArgs::ppart) and are accumulated into dgamma / dbeta
    auto gnb = [&](const Act& in, const float* ss, const float* stats, const std::string& pre, int silu,
                   const float* dz, const float* addsrc, float* out1, float* out2, bool with_param = false,
                   unsigned* amax_out = nullptr) {
        cfd::GnbArgs g{};
        g.x1 = in.a;
        g.x2 = in.b;
        g.dz = dz;
        g.ss = ss;
        g.stats = stats;
        g.gamma = P(h, pre + ".weight");
        g.addsrc = addsrc;
        g.out1 = out1;
        g.out2 = out2;
        g.part = gnpart;
        g.fin = gnfin;
        g.C1 = in.Ca;
        g.C2 = in.Cb;
        g.Ctot = in.C();
        g.HW = in.H * in.W;
        g.silu = silu;
        g.plan_b = plan_batch(h);
        if (with_param && pg) g.ppart = gpp;
        g.amax_out = amax_out;
        const int nch = cfd::launch_gn_bwd(g, B, st);
        if (g.ppart)
            cfd::launch_gn_param_accum(gpp, B * nch, g.Ctot, GP(pre + ".weight"), GP(pre + ".bias"), st);
    };

    Act dcur;  // gradient w.r.t. the current activation (single contiguous tensor)
    unsigned* dmax = nullptr;   // a range slot holding max |dcur| (split weight gradients), or null
    for (size_t si = h->steps.size(); si-- > 0;) {
        const auto& s = h->steps[si];
        const Rec& r = recs[si];
        const Act& in = r.in;
        switch (s.kind) {
            case cfd::Step::Out: {
                // out.2 input-gradient (Cout <= 4 -> C): VALU gather with mirrored taps
                float* G = gpool[0];
                cfd::ConvArgs a{};
                a.src1 = d_eps;
                a.C1 = c.out_channels;
                a.Ctot = c.out_channels;
                a.w = PT(h, "out.2.weight");
                a.out = G;
                a.Hin = a.Hout = in.H;
                a.Win = a.Wout = in.W;
                a.Cout = in.Ca;
                a.M = B * in.H * in.W;
                a.tmode = 1;
                cfd::launch_conv_in(a, st);
                float* dh = gpool[1];
                unsigned* hm = slot();
                gnb(in, r.ss1, r.st1, "out.0", 1, G, nullptr, dh, nullptr, true, hm);
                if (pg) {
                    if (r.act1)   // the kept GroupNorm(+SiLU) output and its range
                        wgrad(d_eps, c.out_channels, Act{r.act1, in.C(), nullptr, 0, in.H, in.W}, nullptr, 0, in.H,
                              in.W, 3, 1, 1, 0, "out.2", nullptr, r.amx1);
                    else
                        wgrad(d_eps, c.out_channels, in, r.ss1, 1, in.H, in.W, 3, 1, 1, 0, "out.2");
                }
                dcur = Act{dh, in.Ca, nullptr, 0, in.H, in.W};
                dmax = hm;
                break;
            }
            case cfd::Step::Up: {
                // nearest-2x + conv3x3 == one 4x4 stride-2 pad-1 convolution of dY (packed at set_param)
                float* out = gfree(dcur.a);
                if (pg) wgrad(dcur.a, dcur.Ca, in, nullptr, 0, dcur.H, dcur.W, 3, 1, 1, 1, s.conv, dmax);
                dconv(dcur.a, dcur.Ca, dcur.H, dcur.W, s.conv + ".weight", s.cin, in.H, in.W, 4, 2, 1, 0, out);
                dcur = Act{out, s.cin, nullptr, 0, in.H, in.W};
                dmax = nullptr;
                break;
            }
            case cfd::Step::Down: {
                float* out = gfree(dcur.a);
                if (pg) wgrad(dcur.a, dcur.Ca, in, nullptr, 0, dcur.H, dcur.W, 3, 2, 1, 0, s.conv, dmax);
                dconv(dcur.a, dcur.Ca, dcur.H, dcur.W, s.conv + ".weight", s.cin, in.H, in.W, 3, 2, 1, 1, out);
                dcur = Act{out, s.cin, nullptr, 0, in.H, in.W};
                dmax = nullptr;
                break;
            }
            case cfd::Step::Push:
                // the pushed tensor's gradient also arrives through its skip concat
                dmax = nullptr;   // dcur changes
                cfd::launch_add(const_cast<float*>(dcur.a), dhs[r.push_hs], (int64_t)B * dcur.H * dcur.W * dcur.Ca,
                                st);
                break;
            case cfd::Step::Cat:
                break;  // the concat's gradient split happens in the ResBlock that consumed it
            case cfd::Step::Res: {
                const auto& rs = h->res[s.idx];
                const float* dout = dcur.a;
                float* G = gfree(dout);
                // stride-1 3x3: plain convolutions with the mirrored packs (tpack 3)
                const Act h1{r.h1, rs.cout, nullptr, 0, in.H, in.W};
                unsigned* omax = dmax;   // max |dout| once known: shared by out_layers.3 and skip_connection
                if (pg)
                    omax = r.act2 ? wgrad(dout, rs.cout, Act{r.act2, rs.cout, nullptr, 0, in.H, in.W}, nullptr, 0, in.H,
                                          in.W, 3, 1, 1, 0, rs.pre + ".out_layers.3", omax, r.amx2)
                                  : wgrad(dout, rs.cout, h1, r.ss2, 1, in.H, in.W, 3, 1, 1, 0, rs.pre + ".out_layers.3",
                                          omax);
                dconv(dout, rs.cout, in.H, in.W, rs.pre + ".out_layers.3.weight", rs.cout, in.H, in.W, 3, 1, 1, 0, G);
                float* dh1 = gfree(dout, G);
                unsigned* h1max = slot();
                gnb(h1, r.ss2, r.st2, rs.pre + ".out_layers.0", 1, G, nullptr, dh1, nullptr, true, h1max);
                if (pg) {
                    if (r.act1)
                        wgrad(dh1, rs.cout, Act{r.act1, in.C(), nullptr, 0, in.H, in.W}, nullptr, 0, in.H, in.W, 3, 1, 1,
                              0, rs.pre + ".in_layers.2", h1max, r.amx1);
                    else
                        wgrad(dh1, rs.cout, in, r.ss1, 1, in.H, in.W, 3, 1, 1, 0, rs.pre + ".in_layers.2", h1max);
                    // emb_layers: d emb_out[b, c] = sum over pixels of dh1; its Linear(SiLU(emb))
                    // backward, and the gradient w.r.t. emb accumulated over the ResBlocks
                    cfd::launch_colsum(dh1, (int64_t)in.H * in.W, rs.cout, B, cpart, crow, st);
                    const std::string ek = rs.pre + ".emb_layers.1";
                    cfd::launch_linear_wgrad(crow, pg->emb, B, h->tdim, rs.cout, 1, GP(ek + ".weight"),
                                             GP(ek + ".bias"), st);
                    const float* W_emb = h->emb_w + (size_t)h->params[h->index.at(ek + ".weight")].emb_row * h->tdim;
                    cfd::launch_linear_dgrad(crow, W_emb, pg->emb, B, h->tdim, rs.cout, 1, 1, demb, st);
                }
                // G <- in_layers conv input-gradient (Ctot channels)
                dconv(dh1, rs.cout, in.H, in.W, rs.pre + ".in_layers.2.weight", in.C(), in.H, in.W, 3, 1, 1, 0, G);
                const float* addsrc = dout;
                if (rs.cin != rs.cout) {
                    if (pg) wgrad(dout, rs.cout, in, nullptr, 0, in.H, in.W, 1, 1, 0, 0, rs.pre + ".skip_connection", omax);
                    float* sk = gfree(dout, G, dh1);
                    dconv(dout, rs.cout, in.H, in.W, rs.pre + ".skip_connection.weight", in.C(), in.H, in.W, 1, 1, 0,
                          0, sk);
                    addsrc = sk;
                }
                float* dx = dh1;  // dh1 is consumed: reuse for the first source's gradient
                unsigned* xm = slot();
                gnb(in, r.ss1, r.st1, rs.pre + ".in_layers.0", 1, G, addsrc, dx,
                    in.b ? dhs[r.skip_hs] : nullptr, true, xm);
                dcur = Act{dx, in.Ca, nullptr, 0, in.H, in.W};
                dmax = xm;
                break;
            }
            case cfd::Step::Attn: {
                const auto& at = h->attn[s.idx];
                const int T = in.H * in.W;
                const float* dout = dcur.a;
                float* dA = gfree(dout);
                if (pg)
                    wgrad(dout, at.C, Act{r.o, at.C, nullptr, 0, in.H, in.W}, nullptr, 0, in.H, in.W, 1, 1, 0, 0,
                          at.pre + ".proj_out", dmax);
                dconv(dout, at.C, in.H, in.W, at.pre + ".proj_out.weight", at.C, in.H, in.W, 1, 1, 0, 0, dA);
                cfd::AttnBwdArgs ab{r.qkv, r.o, dA, r.lse, dd, dqkv, T, at.C,
                                    (float)(1.0 / std::sqrt(std::sqrt((double)at.ch)))};
                // split compute: K9s (three f16 MFMAs per product); the fp32 mode keeps
                // the fp32-MFMA kernels
                if (h->compute == CFD_COMPUTE_SPLIT_F16 && cfd::attention_bwd_split_ok(T, at.ch)) {
                    CFD_REQUIRE(cfd::attention_bwd_split_floats(T, at.C) <= z.max_abw, CFD_ESTATE,
                                "internal: attention backward workspace");
                    cfd::launch_attention_bwd_split(ab, at.ch, at.heads, B, abws, st);
                } else {
                    cfd::launch_attention_bwd(ab, at.ch, at.heads, B, st);
                }
                if (pg) {
                    if (r.act1)
                        wgrad(dqkv, 3 * at.C, Act{r.act1, at.C, nullptr, 0, in.H, in.W}, nullptr, 0, in.H, in.W, 1, 1, 0,
                              0, at.pre + ".qkv", nullptr, r.amx1);
                    else
                        wgrad(dqkv, 3 * at.C, in, r.ss1, 0, in.H, in.W, 1, 1, 0, 0, at.pre + ".qkv");
                }
                float* dxn = gfree(dout, dA);
                dconv(dqkv, 3 * at.C, in.H, in.W, at.pre + ".qkv.weight", at.C, in.H, in.W, 1, 1, 0, 0, dxn);
                unsigned* am = slot();
                gnb(in, r.ss1, r.st1, at.pre + ".norm", 0, dxn, dout, dA, nullptr, true, am);
                dcur = Act{dA, at.C, nullptr, 0, in.H, in.W};
                dmax = am;
                break;
            }
            case cfd::Step::In: {
                if (pg) {
                    wgrad(dcur.a, dcur.Ca, Act{pg->x, c.in_channels, nullptr, 0, S, S}, nullptr, 0, S, S, 3, 1, 1, 0,
                          s.conv, dmax);
                    // time_embed: emb = L2(SiLU(L1(timestep_embedding(t)))) (unet.py:470-475,648)
                    cfd::launch_linear_wgrad(demb, pg->th1, B, h->tdim, h->tdim, 1, GP("time_embed.2.weight"),
                                             GP("time_embed.2.bias"), st);
                    cfd::launch_linear_dgrad(demb, P(h, "time_embed.2.weight"), pg->th1, B, h->tdim, h->tdim, 1, 0,
                                             dth1, st);
                    cfd::launch_linear_wgrad(dth1, pg->temb, B, c.model_channels, h->tdim, 0,
                                             GP("time_embed.0.weight"), GP("time_embed.0.bias"), st);
                }
                if (!d_x) break;
                cfd::ConvArgs a{};
                a.src1 = dcur.a;
                a.C1 = dcur.Ca;
                a.Ctot = dcur.Ca;
                a.w = PT(h, s.conv + ".weight");
                a.out = d_x;
                a.Hin = a.Hout = S;
                a.Win = a.Wout = S;
                a.Cout = c.in_channels;
                a.M = B * S * S;
                a.K = 9 * dcur.Ca;
                a.tmode = 1;
                cfd::launch_conv_out(a, st);
                break;
            }
        }
    }
}

}  // namespace

extern "C" int cfd_unet_create(const cfd_unet_cfg* cfg, int device, cfd_unet** out) {
    return cfd::guard([&] {
        CFD_REQUIRE(cfg && out, CFD_EARG, "null argument");
        CFD_REQUIRE(cfg->n_mult >= 1 && cfg->n_mult <= 8 && cfg->n_attn >= 0 && cfg->n_attn <= 8, CFD_EARG,
                    "bad channel_mult / attention list");
        CFD_REQUIRE(cfg->model_channels > 0 && cfg->model_channels % 32 == 0, CFD_EARG,
                    "model_channels must be a positive multiple of 32");
        CFD_REQUIRE(cfg->in_channels >= 1 && cfg->in_channels <= 4 && cfg->out_channels >= 1 &&
                        cfg->out_channels <= 4,
                    CFD_EARG, "in/out channels must be 1..4");
        const int levels_down = cfg->n_mult - 1;
        CFD_REQUIRE(cfg->image_size > 0 && (cfg->image_size >> levels_down) << levels_down == cfg->image_size,
                    CFD_EARG, "image_size must be divisible by 2^(len(channel_mult)-1)");
        cfd::DeviceGuard dg(device);
        auto* h = new cfd_unet();
        h->cfg = *cfg;
        h->device = device;
        try {
            build(h);
            CFD_HIP(hipMalloc(&h->arena, sizeof(float) * h->arena_floats));
            CFD_HIP(hipMalloc(&h->emb_w, sizeof(float) * (size_t)h->emb_total * h->tdim));
            CFD_HIP(hipMalloc(&h->emb_b, sizeof(float) * (size_t)h->emb_total));
            CFD_HIP(hipMalloc(&h->arena_t, sizeof(float) * std::max<size_t>(h->arena_t_floats, 4)));
            CFD_HIP(hipMalloc(&h->arena_bf, sizeof(uint16_t) * std::max<size_t>(h->arena_floats, 4)));
            CFD_HIP(hipMalloc(&h->arena_hi, sizeof(uint16_t) * std::max<size_t>(h->arena_floats, 4)));
            CFD_HIP(hipMalloc(&h->arena_lo, sizeof(uint16_t) * std::max<size_t>(h->arena_floats, 4)));
            CFD_HIP(hipMalloc(&h->arena_thi, sizeof(uint16_t) * std::max<size_t>(h->arena_t_floats, 4)));
            CFD_HIP(hipMalloc(&h->arena_tlo, sizeof(uint16_t) * std::max<size_t>(h->arena_t_floats, 4)));
            const int half = cfg->model_channels / 2;
            // freqs = exp(-ln(10000) * arange(half, fp32) / half) in fp32 (nn.py:129-131)
            std::vector<float> fr(half);
            const float nl = (float)(-std::log(10000.0));
            for (int i = 0; i < half; ++i) fr[i] = std::exp((nl * (float)i) / (float)half);
            CFD_HIP(hipMalloc(&h->freqs, sizeof(float) * std::max(half, 1)));
            CFD_HIP(hipMalloc(&h->nonfinite, sizeof(int)));
            CFD_HIP(hipMemset(h->nonfinite, 0, sizeof(int)));
            CFD_HIP(hipMemcpy(h->freqs, fr.data(), sizeof(float) * half, hipMemcpyHostToDevice));
        } catch (...) {
            cfd_unet_destroy(h);
            throw;
        }
        *out = h;
    });
}

extern "C" void cfd_unet_destroy(cfd_unet* h) {
    if (!h) return;
    (void)hipFree(h->arena);
    (void)hipFree(h->emb_w);
    (void)hipFree(h->emb_b);
    (void)hipFree(h->freqs);
    (void)hipFree(h->arena_t);
    (void)hipFree(h->arena_bf);
    (void)hipFree(h->arena_hi);
    (void)hipFree(h->arena_lo);
    (void)hipFree(h->arena_thi);
    (void)hipFree(h->arena_tlo);
    (void)hipFree(h->nonfinite);
    (void)hipFree(h->rp_desc);
    (void)hipFree(h->rp_first);
    (void)hipFree(h->rp_part);
    (void)hipFree(h->rp_amax);
    (void)hipFree(h->rp_tfirst);
    delete h;
}

extern "C" int cfd_unet_num_params(const cfd_unet* h, int* n) {
    return cfd::guard([&] {
        CFD_REQUIRE(h && n, CFD_EARG, "null argument");
        *n = (int)h->params.size();
    });
}

extern "C" int cfd_unet_param_info(const cfd_unet* h, int idx, const char** key, int* ndim, int64_t shape[4]) {
    return cfd::guard([&] {
        CFD_REQUIRE(h && idx >= 0 && idx < (int)h->params.size(), CFD_EARG, "bad index");
        const auto& p = h->params[idx];
        if (key) *key = p.key.c_str();
        if (ndim) *ndim = (int)p.shape.size();
        if (shape)
            for (size_t i = 0; i < p.shape.size(); ++i) shape[i] = p.shape[i];
    });
}

extern "C" int cfd_unet_set_param(cfd_unet* h, const char* key, const float* host, size_t n) {
    return cfd::guard([&] {
        CFD_REQUIRE(h && key && host, CFD_EARG, "null argument");
        auto it = h->index.find(key);
        CFD_REQUIRE(it != h->index.end(), CFD_EKEY, std::string("unknown U-Net parameter key: ") + key);
        auto& p = h->params[it->second];
        CFD_REQUIRE(n == p.count, CFD_ESHAPE, std::string("size mismatch for ") + key);
        cfd::DeviceGuard dg(h->device);
        switch (p.pack) {
            case Pack::Raw:
                CFD_HIP(hipMemcpy(h->arena + p.offset, host, n * 4, hipMemcpyHostToDevice));
                break;
            case Pack::Conv1:
            case Pack::Conv3: {
                // 3x3: (Cout, Cin, 3, 3) -> (Cout, tap, Cin): GEMM K ordered (tap, channel)
                std::vector<float> pk(host, host + n);
                if (p.pack == Pack::Conv3) {
                    const int64_t co = p.shape[0], ci = p.shape[1];
                    for (int64_t o = 0; o < co; ++o)
                        for (int64_t i = 0; i < ci; ++i)
                            for (int tap = 0; tap < 9; ++tap)
                                pk[(o * 9 + tap) * ci + i] = host[(o * ci + i) * 9 + tap];
                }
                CFD_HIP(hipMemcpy(h->arena + p.offset, pk.data(), n * 4, hipMemcpyHostToDevice));
                std::vector<uint16_t> bf(n);
                for (size_t e = 0; e < n; ++e) bf[e] = to_bf16(pk[e]);
                CFD_HIP(hipMemcpy(h->arena_bf + p.offset, bf.data(), n * 2, hipMemcpyHostToDevice));
                // split compute: s w = wh + wl, s = 2^-e with e the frexp exponent of max|w|
                float amax = 0.f;
                for (size_t e = 0; e < n; ++e) amax = std::max(amax, std::fabs(pk[e]));
                int ex = 0;
                if (amax > 0.f) std::frexp(amax, &ex);
                const float s = std::ldexp(1.0f, -ex);
                p.split_inv = std::ldexp(1.0f, ex);
                std::vector<_Float16> hi(n), lo(n);
                for (size_t e = 0; e < n; ++e) {
                    const float v = pk[e] * s;
                    hi[e] = (_Float16)v;
                    lo[e] = (_Float16)(v - (float)hi[e]);
                }
                CFD_HIP(hipMemcpy(h->arena_hi + p.offset, hi.data(), n * 2, hipMemcpyHostToDevice));
                CFD_HIP(hipMemcpy(h->arena_lo + p.offset, lo.data(), n * 2, hipMemcpyHostToDevice));
                break;
            }
            case Pack::EmbW:
                CFD_HIP(hipMemcpy(h->emb_w + (size_t)p.emb_row * h->tdim, host, n * 4, hipMemcpyHostToDevice));
                break;
            case Pack::EmbB:
                CFD_HIP(hipMemcpy(h->emb_b + p.emb_row, host, n * 4, hipMemcpyHostToDevice));
                break;
        }
        if (p.tpack) {
            // input-gradient packs.  1: W^T as (Cin, tap, Cout) (taps not mirrored:
            // conv_gemm's TMODE gathers dY[(o + pad - tap) / stride]).  3: the same
            // with tap t stored at taps-1-t: for a stride-1 3x3 pad-1 convolution
            // dX[o] = sum_t W_t^T dY[o + 1 - t] is a plain convolution of dY with the
            // mirrored taps, so it runs on the forward kernels (K1h).  2: Upsample +
            // conv3x3 as a 4x4 stride-2 pad-1 convolution of dY: per axis, tap e of
            // the 4 sums the 3x3 taps d with a - d + 2 == e over the two nearest
            // neighbours a in {0, 1}:  e0 = w2, e1 = w1 + w2, e2 = w0 + w1, e3 = w0.
            const int64_t co = p.shape[0], ci = p.shape[1];
            const int taps = (int)(p.count / (size_t)(co * ci));
            std::vector<float> pk(p.tpack == 2 ? (size_t)ci * 16 * co : n);
            if (p.tpack == 1 || p.tpack == 3) {
                for (int64_t o = 0; o < co; ++o)
                    for (int64_t i = 0; i < ci; ++i)
                        for (int tap = 0; tap < taps; ++tap)
                            pk[((size_t)i * taps + (p.tpack == 3 ? taps - 1 - tap : tap)) * co + o] =
                                host[((size_t)o * ci + i) * taps + tap];
            } else {
                static const int dlo[4] = {2, 1, 0, 0}, dhi[4] = {2, 2, 1, 0};
                for (int64_t o = 0; o < co; ++o)
                    for (int64_t i = 0; i < ci; ++i)
                        for (int ey = 0; ey < 4; ++ey)
                            for (int ex = 0; ex < 4; ++ex) {
                                float v = 0.f;
                                for (int dy = dlo[ey]; dy <= dhi[ey]; ++dy)
                                    for (int dx = dlo[ex]; dx <= dhi[ex]; ++dx)
                                        v += host[((size_t)o * ci + i) * 9 + dy * 3 + dx];
                                pk[((size_t)i * 16 + ey * 4 + ex) * co + o] = v;
                            }
            }
            CFD_HIP(hipMemcpy(h->arena_t + p.toffset, pk.data(), pk.size() * 4, hipMemcpyHostToDevice));
            // split compute: the same power-of-two scaled hi / lo split as the forward pack
            float amax = 0.f;
            for (float v : pk) amax = std::max(amax, std::fabs(v));
            int ex = 0;
            if (amax > 0.f) std::frexp(amax, &ex);
            const float sc = std::ldexp(1.0f, -ex);
            p.tsplit_inv = std::ldexp(1.0f, ex);
            std::vector<_Float16> thi(pk.size()), tlo(pk.size());
            for (size_t e = 0; e < pk.size(); ++e) {
                const float v = pk[e] * sc;
                thi[e] = (_Float16)v;
                tlo[e] = (_Float16)(v - (float)thi[e]);
            }
            CFD_HIP(hipMemcpy(h->arena_thi + p.toffset, thi.data(), pk.size() * 2, hipMemcpyHostToDevice));
            CFD_HIP(hipMemcpy(h->arena_tlo + p.toffset, tlo.data(), pk.size() * 2, hipMemcpyHostToDevice));
        }
        p.set = true;
        ++h->version;
    });
}

// ---------------------------------------------------------------------------
// Device repack of every parameter (cfd_unet_load_flat): the packing of
// cfd_unet_set_param above, element for element, in three launches -- per-block
// |max| of each pack, per-parameter reduction, then the pack writes.  Each
// parameter spans ceil(max(count, tcount) / RP_CHUNK) blocks (tcount: the
// input-gradient pack's element count, 16 Cin Cout for the upsample pack).
namespace cfd {
constexpr int RP_CHUNK = 4096;

struct RepackDesc {
    int64_t src, count, off, toff, tcount;
    int pack, tpack, co, ci, taps, emb_row;
};

__device__ __forceinline__ int rp_param(const int64_t* __restrict__ first, int np, int64_t blk) {
    int lo = 0, hi = np;   // largest p with first[p] <= blk
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (first[mid] <= blk) lo = mid; else hi = mid;
    }
    return lo;
}

// the upsample pack's value at its element e (the 4x4 stride-2 kernel of
// nearest-2x + conv3x3: per axis e0 = w2, e1 = w1 + w2, e2 = w0 + w1, e3 = w0),
// summed in cfd_unet_set_param's order
__device__ __forceinline__ float rp_up_value(const float* __restrict__ w, const RepackDesc& d, int64_t e) {
    const int64_t o = e % d.co, r = e / d.co;
    const int q = (int)(r % 16);
    const int64_t i = r / 16;
    const int ey = q >> 2, ex = q & 3;
    const int dlo_y = ey == 0 ? 2 : ey == 1 ? 1 : 0, dhi_y = ey == 0 ? 2 : ey == 1 ? 2 : ey == 2 ? 1 : 0;
    const int dlo_x = ex == 0 ? 2 : ex == 1 ? 1 : 0, dhi_x = ex == 0 ? 2 : ex == 1 ? 2 : ex == 2 ? 1 : 0;
    const float* base = w + (o * d.ci + i) * 9;
    float v = 0.f;
    for (int dy = dlo_y; dy <= dhi_y; ++dy)
        for (int dx = dlo_x; dx <= dhi_x; ++dx) v += base[dy * 3 + dx];
    return v;
}

__global__ __launch_bounds__(256) void rp_amax_kernel(const float* __restrict__ flat,
                                                      const RepackDesc* __restrict__ desc,
                                                      const int64_t* __restrict__ first, int np,
                                                      float* __restrict__ part) {
    const int64_t blk = blockIdx.x;
    const int p = rp_param(first, np, blk);
    const RepackDesc d = desc[p];
    const float* w = flat + d.src;
    const int64_t e0 = (blk - first[p]) * RP_CHUNK;
    float m0 = 0.f, m1 = 0.f;
    for (int64_t e = e0 + threadIdx.x; e < e0 + RP_CHUNK; e += 256) {
        if (e < d.count) m0 = fmaxf(m0, fabsf(w[e]));
        if (d.tpack == 2 && e < d.tcount) m1 = fmaxf(m1, fabsf(rp_up_value(w, d, e)));
    }
    __shared__ float r0[256], r1[256];
    r0[threadIdx.x] = m0;
    r1[threadIdx.x] = m1;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s) {
            r0[threadIdx.x] = fmaxf(r0[threadIdx.x], r0[threadIdx.x + s]);
            r1[threadIdx.x] = fmaxf(r1[threadIdx.x], r1[threadIdx.x + s]);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        part[blk * 2] = r0[0];
        part[blk * 2 + 1] = d.tpack == 2 ? r1[0] : r0[0];   // the other packs permute the weights
    }
}

__global__ __launch_bounds__(256) void rp_reduce_kernel(const float* __restrict__ part,
                                                        const int64_t* __restrict__ first, float* __restrict__ amax) {
    const int p = blockIdx.x;
    float m0 = 0.f, m1 = 0.f;
    for (int64_t b = first[p] + threadIdx.x; b < first[p + 1]; b += 256) {
        m0 = fmaxf(m0, part[b * 2]);
        m1 = fmaxf(m1, part[b * 2 + 1]);
    }
    __shared__ float r0[256], r1[256];
    r0[threadIdx.x] = m0;
    r1[threadIdx.x] = m1;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s) {
            r0[threadIdx.x] = fmaxf(r0[threadIdx.x], r0[threadIdx.x + s]);
            r1[threadIdx.x] = fmaxf(r1[threadIdx.x], r1[threadIdx.x + s]);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        amax[p * 2] = r0[0];
        amax[p * 2 + 1] = r1[0];
    }
}

__device__ __forceinline__ uint16_t rp_bf16(float f) {   // to_bf16 (host) bit for bit
    const uint32_t u = __float_as_uint(f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);
    return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

__device__ __forceinline__ float rp_scale(float amax) {   // 2^-e, e the frexp exponent of amax (1 for 0)
    if (!(amax > 0.f)) return 1.f;
    int ex;
    frexpf(amax, &ex);
    return ldexpf(1.f, -ex);
}

__device__ __forceinline__ void rp_split(float v, float s, _Float16* hi, _Float16* lo, int64_t i) {
#pragma clang fp contract(off)
    const float x = v * s;
    const _Float16 h = (_Float16)x;
    hi[i] = h;
    lo[i] = (_Float16)(x - (float)h);
}

__global__ __launch_bounds__(256) void rp_pack_kernel(const float* __restrict__ flat,
                                                      const RepackDesc* __restrict__ desc,
                                                      const int64_t* __restrict__ first, int np,
                                                      const float* __restrict__ amax, float* __restrict__ arena,
                                                      uint16_t* __restrict__ arena_bf, _Float16* __restrict__ arena_hi,
                                                      _Float16* __restrict__ arena_lo, float* __restrict__ arena_t,
                                                      _Float16* __restrict__ arena_thi,
                                                      _Float16* __restrict__ arena_tlo, float* __restrict__ emb_w,
                                                      float* __restrict__ emb_b, int tdim) {
    const int64_t blk = blockIdx.x;
    const int p = rp_param(first, np, blk);
    const RepackDesc d = desc[p];
    const float* w = flat + d.src;
    const int64_t e0 = (blk - first[p]) * RP_CHUNK;
    const float s = rp_scale(amax[p * 2]), ts = rp_scale(amax[p * 2 + 1]);
    const bool conv = d.pack == (int)Pack::Conv1 || d.pack == (int)Pack::Conv3;
    // e walks the DESTINATION layouts (coalesced writes; the reads gather)
    for (int64_t e = e0 + threadIdx.x; e < e0 + RP_CHUNK; e += 256) {
        if (e < d.count) {
            if (d.pack == (int)Pack::Raw) {
                arena[d.off + e] = w[e];
            } else if (d.pack == (int)Pack::EmbW) {
                emb_w[(int64_t)d.emb_row * tdim + e] = w[e];
            } else if (d.pack == (int)Pack::EmbB) {
                emb_b[d.emb_row + e] = w[e];
            } else {
                int64_t src = e;
                if (d.pack == (int)Pack::Conv3) {   // dst (o, tap, i) <- src (o, i, tap)
                    const int64_t i = e % d.ci, ot = e / d.ci, tap = ot % 9, o = ot / 9;
                    src = (o * d.ci + i) * 9 + tap;
                }
                const float v = w[src];
                arena[d.off + e] = v;
                arena_bf[d.off + e] = rp_bf16(v);
                rp_split(v, s, arena_hi, arena_lo, d.off + e);
            }
        }
        (void)conv;
        (void)ts;   // the input-gradient packs: rp_tpack_kernel
    }
}

// The input-gradient packs of the convolution weights, src (o, i, tap) ->
// dst (i, tap', o) (tap' = tap, or taps - 1 - tap: tpack 1 / 3) or the 4x4 upsample
// pack dst (i, q, o) (tpack 2, rp_up_value): o is fastest in the destination and
// slowest in the source, so a workgroup stages a 64 (o) x RP_TI (i) x taps block of
// the source in LDS (rows of contiguous (i, tap) runs, coalesced) and writes the
// destination rows 64 o at a time (coalesced) -- the same values, the same sums
constexpr int RP_TI = 8;
__global__ __launch_bounds__(256) void rp_tpack_kernel(const float* __restrict__ flat,
                                                       const RepackDesc* __restrict__ desc,
                                                       const int64_t* __restrict__ tfirst, int np,
                                                       const float* __restrict__ amax, float* __restrict__ arena_t,
                                                       _Float16* __restrict__ arena_thi,
                                                       _Float16* __restrict__ arena_tlo) {
    const int64_t blk = blockIdx.x;
    const int p = rp_param(tfirst, np, blk);
    const RepackDesc d = desc[p];
    const float* w = flat + d.src;
    const int64_t tile = blk - tfirst[p];
    const int nti = (d.ci + RP_TI - 1) / RP_TI;
    const int o0 = (int)(tile / nti) * 64, i0 = (int)(tile % nti) * RP_TI;
    const int taps = d.taps, run = RP_TI * taps, ld = run + 1;
    __shared__ float tl[64 * (RP_TI * 9 + 1)];
    for (int e = threadIdx.x; e < 64 * run; e += 256) {
        const int ol = e / run, c = e - ol * run;
        const int o = o0 + ol, i = i0 + c / taps;
        tl[ol * ld + c] = o < d.co && i < d.ci ? w[((int64_t)o * d.ci + i0) * taps + c] : 0.f;
    }
    __syncthreads();
    const float ts = rp_scale(amax[p * 2 + 1]);
    const int ol = threadIdx.x & 63, o = o0 + ol;
    const int nq = d.tpack == 2 ? 16 : taps;   // destination rows per i
    if (o < d.co) {
        for (int r = threadIdx.x >> 6; r < RP_TI * nq; r += 4) {
            const int il = r / nq, q = r - il * nq, i = i0 + il;
            if (i >= d.ci) break;
            const float* src = tl + ol * ld + il * taps;
            float v;
            if (d.tpack == 2) {   // rp_up_value's taps in its order
                const int ey = q >> 2, ex = q & 3;
                const int dlo_y = ey == 0 ? 2 : ey == 1 ? 1 : 0, dhi_y = ey == 0 ? 2 : ey == 1 ? 2 : ey == 2 ? 1 : 0;
                const int dlo_x = ex == 0 ? 2 : ex == 1 ? 1 : 0, dhi_x = ex == 0 ? 2 : ex == 1 ? 2 : ex == 2 ? 1 : 0;
                v = 0.f;
                for (int dy = dlo_y; dy <= dhi_y; ++dy)
                    for (int dx = dlo_x; dx <= dhi_x; ++dx) v += src[dy * 3 + dx];
            } else {
                v = src[d.tpack == 3 ? taps - 1 - q : q];
            }
            const int64_t e = ((int64_t)i * nq + q) * d.co + o;
            arena_t[d.toff + e] = v;
            rp_split(v, ts, arena_thi, arena_tlo, d.toff + e);
        }
    }
}
}  // namespace cfd

extern "C" int cfd_unet_load_flat(cfd_unet* h, const float* flat, size_t n, void* stream) {
    return cfd::guard([&] {
        CFD_REQUIRE(h && flat, CFD_EARG, "null argument");
        const int np = (int)h->params.size();
        size_t total = 0;
        for (const auto& p : h->params) total += p.count;
        CFD_REQUIRE(n == total, CFD_ESHAPE, "flat buffer size differs from the parameter count");
        cfd::DeviceGuard dg(h->device);
        hipStream_t st = (hipStream_t)stream;
        if (!h->rp_desc) {
            std::vector<cfd::RepackDesc> desc(np);
            std::vector<int64_t> first(np + 1);
            int64_t src = 0, blocks = 0;
            for (int k = 0; k < np; ++k) {
                const auto& p = h->params[k];
                cfd::RepackDesc d{};
                d.src = src;
                d.count = (int64_t)p.count;
                d.off = (int64_t)p.offset;
                d.toff = (int64_t)p.toffset;
                d.pack = (int)p.pack;
                d.tpack = p.tpack;
                d.emb_row = p.emb_row;
                d.co = p.shape.size() > 1 ? (int)p.shape[0] : 1;
                d.ci = p.shape.size() > 1 ? (int)p.shape[1] : 1;
                d.taps = (int)(d.count / std::max<int64_t>(1, (int64_t)d.co * d.ci));
                d.tcount = p.tpack == 2 ? (int64_t)d.ci * 16 * d.co : d.count;
                if (p.tpack == 2) CFD_REQUIRE(d.taps == 9, CFD_ESTATE, "internal: upsample pack needs 3x3");
                desc[k] = d;
                first[k] = blocks;
                blocks += std::max<int64_t>(1, cfd::ceil_div(std::max(d.count, d.tcount), cfd::RP_CHUNK));
                src += d.count;
            }
            first[np] = blocks;
            std::vector<int64_t> tfirst(np + 1);
            int64_t tiles = 0;
            for (int k = 0; k < np; ++k) {
                const auto& d = desc[k];
                const bool conv = d.pack == (int)Pack::Conv1 || d.pack == (int)Pack::Conv3;
                tfirst[k] = tiles;
                if (conv && d.tpack) {
                    CFD_REQUIRE(d.taps <= 9 && (int64_t)d.co * d.ci * d.taps == d.count, CFD_ESTATE,
                                "internal: input-gradient pack shape");
                    tiles += cfd::ceil_div(d.co, 64) * cfd::ceil_div(d.ci, cfd::RP_TI);
                }
            }
            tfirst[np] = tiles;
            CFD_HIP(hipMalloc(&h->rp_tfirst, sizeof(int64_t) * (np + 1)));
            CFD_HIP(hipMemcpy(h->rp_tfirst, tfirst.data(), sizeof(int64_t) * (np + 1), hipMemcpyHostToDevice));
            h->rp_tiles = tiles;
            CFD_HIP(hipMalloc(&h->rp_desc, sizeof(cfd::RepackDesc) * np));
            CFD_HIP(hipMalloc(&h->rp_first, sizeof(int64_t) * (np + 1)));
            CFD_HIP(hipMalloc(&h->rp_part, sizeof(float) * 2 * blocks));
            CFD_HIP(hipMalloc(&h->rp_amax, sizeof(float) * 2 * np));
            CFD_HIP(hipMemcpy(h->rp_desc, desc.data(), sizeof(cfd::RepackDesc) * np, hipMemcpyHostToDevice));
            CFD_HIP(hipMemcpy(h->rp_first, first.data(), sizeof(int64_t) * (np + 1), hipMemcpyHostToDevice));
            h->rp_blocks = blocks;
        }
        const auto* desc = (const cfd::RepackDesc*)h->rp_desc;
        hipLaunchKernelGGL(cfd::rp_amax_kernel, dim3((unsigned)h->rp_blocks), dim3(256), 0, st, flat, desc,
                           h->rp_first, np, h->rp_part);
        cfd::check_launch("rp_amax_kernel");
        hipLaunchKernelGGL(cfd::rp_reduce_kernel, dim3(np), dim3(256), 0, st, h->rp_part, h->rp_first, h->rp_amax);
        cfd::check_launch("rp_reduce_kernel");
        hipLaunchKernelGGL(cfd::rp_pack_kernel, dim3((unsigned)h->rp_blocks), dim3(256), 0, st, flat, desc,
                           h->rp_first, np, h->rp_amax, h->arena, h->arena_bf, (_Float16*)h->arena_hi,
                           (_Float16*)h->arena_lo, h->arena_t, (_Float16*)h->arena_thi, (_Float16*)h->arena_tlo,
                           h->emb_w, h->emb_b, h->tdim);
        cfd::check_launch("rp_pack_kernel");
        if (h->rp_tiles) {
            hipLaunchKernelGGL(cfd::rp_tpack_kernel, dim3((unsigned)h->rp_tiles), dim3(256), 0, st, flat, desc,
                               h->rp_tfirst, np, h->rp_amax, h->arena_t, (_Float16*)h->arena_thi,
                               (_Float16*)h->arena_tlo);
            cfd::check_launch("rp_tpack_kernel");
        }
        std::vector<float> amax(2 * (size_t)np);
        CFD_HIP(hipMemcpyAsync(amax.data(), h->rp_amax, sizeof(float) * 2 * np, hipMemcpyDeviceToHost, st));
        CFD_HIP(hipStreamSynchronize(st));
        for (int k = 0; k < np; ++k) {
            auto& p = h->params[k];
            if (p.pack == Pack::Conv1 || p.pack == Pack::Conv3) {
                int ex = 0;
                if (amax[2 * k] > 0.f) std::frexp(amax[2 * k], &ex);
                p.split_inv = std::ldexp(1.0f, ex);
            }
            if (p.tpack) {
                int ex = 0;
                if (amax[2 * k + 1] > 0.f) std::frexp(amax[2 * k + 1], &ex);
                p.tsplit_inv = std::ldexp(1.0f, ex);
            }
            p.set = true;
        }
        ++h->version;
    });
}

extern "C" int cfd_unet_set_compute(cfd_unet* h, int compute) {
    return cfd::guard([&] {
        CFD_REQUIRE(h, CFD_EARG, "null handle");
        CFD_REQUIRE(compute == CFD_COMPUTE_F32 || compute == CFD_COMPUTE_BF16 || compute == CFD_COMPUTE_SPLIT_F16,
                    CFD_EARG, "unknown compute mode");
        if (h->compute != compute) ++h->version;
        h->compute = compute;
    });
}

extern "C" int cfd_unet_set_plan_batch(cfd_unet* h, int nominal_batch) {
    return cfd::guard([&] {
        CFD_REQUIRE(h, CFD_EARG, "null handle");
        CFD_REQUIRE(nominal_batch >= 0 && nominal_batch <= 64, CFD_EARG, "plan batch must be 0 (default) .. 64");
        if (h->plan_b != nominal_batch) {
            ++h->version;          // captured graphs hold the old tiles
            h->ws_cache.clear();   // the split-K slab is sized per planned batch
        }
        h->plan_b = nominal_batch;
    });
}

extern "C" int cfd_unet_set_time_freqs(cfd_unet* h, const float* host, int n) {
    return cfd::guard([&] {
        CFD_REQUIRE(h && host && n == h->cfg.model_channels / 2, CFD_EARG, "freqs must have model_channels/2 entries");
        cfd::DeviceGuard dg(h->device);
        CFD_HIP(hipMemcpy(h->freqs, host, sizeof(float) * n, hipMemcpyHostToDevice));
    });
}

extern "C" int cfd_unet_ready(const cfd_unet* h) {
    return cfd::guard([&] {
        CFD_REQUIRE(h, CFD_EARG, "null handle");
        for (const auto& p : h->params) CFD_REQUIRE(p.set, CFD_ESTATE, "U-Net parameter not set: " + p.key);
    });
}

namespace cfd {
size_t unet_ws_bytes(const cfd_unet* h, int B) {
    auto it = h->ws_cache.find(B);
    if (it != h->ws_cache.end()) return it->second;
    Workspace ws{nullptr, 0, true};
    run(h, nullptr, nullptr, nullptr, B, ws, nullptr);
    h->ws_cache[B] = ws.off + 256;
    return ws.off + 256;
}
void unet_check_ready(const cfd_unet* h) {
    for (const auto& p : h->params) CFD_REQUIRE(p.set, CFD_ESTATE, "U-Net parameter not set: " + p.key);
}
int unet_compute(const cfd_unet* h) { return h->compute; }
uint64_t unet_version(const cfd_unet* h) { return h->version; }
int unet_device(const cfd_unet* h) { return h->device; }
int* unet_nonfinite(const cfd_unet* h) { return h->nonfinite; }
void unet_forward_raw(const cfd_unet* h, const float* x, const int64_t* t, float* eps, int B, void* workspace,
                      hipStream_t st) {
    Workspace ws{(char*)(((uintptr_t)workspace + 255) & ~uintptr_t(255)), 0, false};
    run(h, x, t, eps, B, ws, st);
}
}  // namespace cfd

extern "C" int cfd_unet_workspace_bytes(const cfd_unet* h, int B, size_t* bytes) {
    return cfd::guard([&] {
        CFD_REQUIRE(h && bytes && B > 0, CFD_EARG, "bad argument");
        *bytes = cfd::unet_ws_bytes(h, B);
    });
}

extern "C" int cfd_unet_forward(cfd_unet* h, const float* x, const int64_t* t, float* eps, int B, void* workspace,
                                size_t ws_bytes, void* stream) {
    return cfd::guard([&] {
        CFD_REQUIRE(h && x && t && eps && workspace, CFD_EARG, "null argument");
        CFD_REQUIRE(B > 0, CFD_EARG, "B must be positive");
        cfd::unet_check_ready(h);
        CFD_REQUIRE(ws_bytes >= cfd::unet_ws_bytes(h, B), CFD_EARG, "workspace too small");
        cfd::unet_forward_raw(h, x, t, eps, B, workspace, (hipStream_t)stream);
    });
}

namespace {
// tape bytes of a forward recorded in `mode`
size_t tape_bytes_mode(const cfd_unet* h, int B, int mode) {
    Workspace ws{nullptr, 0, true}, tws{nullptr, 0, true};
    Tape tape{&tws, nullptr};
    tape.keep_gnout = mode == CFD_TAPE_PARAM_GRAD;
    run(h, nullptr, nullptr, nullptr, B, ws, nullptr, &tape, false);
    return tws.off + 256;
}
}  // namespace

extern "C" int cfd_unet_tape_bytes(const cfd_unet* h, int B, size_t* bytes) {
    return cfd::guard([&] {
        CFD_REQUIRE(h && bytes && B > 0, CFD_EARG, "bad argument");
        *bytes = tape_bytes_mode(h, B, h->tape_mode);
    });
}

namespace {
constexpr size_t kMaxTapes = 64;   // live tapes remembered per handle (oldest forgotten first)

// the recording a replay of `tape` at batch B must follow; loud on a tape this
// handle did not record, or one recorded at another batch or plan
const cfd_unet::TapeRec& tape_rec(const cfd_unet* h, const void* tape, int B, size_t tape_bytes) {
    auto it = h->tapes.find(tape);
    CFD_REQUIRE(it != h->tapes.end(), CFD_ESTATE,
                "tape was not recorded by cfd_unet_forward_tape on this handle (or was forgotten: at most 64 live "
                "tapes per handle)");
    CFD_REQUIRE(it->second.B == B, CFD_EARG, "B differs from the batch the tape was recorded at");
    CFD_REQUIRE(it->second.plan == plan_batch(h), CFD_ESTATE,
                "the planned batch changed since the tape was recorded (cfd_unet_set_plan_batch)");
    CFD_REQUIRE(tape_bytes >= tape_bytes_mode(h, B, it->second.mode), CFD_EARG, "tape too small");
    return it->second;
}
}  // namespace

extern "C" int cfd_unet_set_tape_mode(cfd_unet* h, int mode) {
    return cfd::guard([&] {
        CFD_REQUIRE(h, CFD_EARG, "null handle");
        CFD_REQUIRE(mode == CFD_TAPE_INPUT_VJP || mode == CFD_TAPE_PARAM_GRAD, CFD_EARG, "unknown tape mode");
        h->tape_mode = mode;
    });
}

extern "C" int cfd_unet_vjp_workspace_bytes(const cfd_unet* h, int B, size_t* bytes) {
    return cfd::guard([&] {
        CFD_REQUIRE(h && bytes && B > 0, CFD_EARG, "bad argument");
        Workspace ws{nullptr, 0, true};
        std::vector<Rec> none;
        run_vjp(h, nullptr, nullptr, B, none, ws, nullptr);
        *bytes = ws.off + 256;
    });
}

namespace {
char* align256(void* p) { return (char*)(((uintptr_t)p + 255) & ~uintptr_t(255)); }

void check_ready(const cfd_unet* h) {
    for (const auto& p : h->params) CFD_REQUIRE(p.set, CFD_ESTATE, "U-Net parameter not set: " + p.key);
}
}  // namespace

extern "C" int cfd_unet_forward_tape(cfd_unet* h, const float* x, const int64_t* t, float* eps, int B,
                                     void* workspace, size_t ws_bytes, void* tape, size_t tape_bytes, void* stream) {
    return cfd::guard([&] {
        CFD_REQUIRE(h && x && t && eps && workspace && tape, CFD_EARG, "null argument");
        CFD_REQUIRE(h->compute != CFD_COMPUTE_BF16, CFD_ESTATE,
                    "the input-gradient path is fp32-accurate: call cfd_unet_set_compute(h, CFD_COMPUTE_F32) "
                    "or CFD_COMPUTE_SPLIT_F16 first");
        CFD_REQUIRE(B > 0, CFD_EARG, "B must be positive");
        check_ready(h);
        size_t need = 0;
        cfd_unet_workspace_bytes(h, B, &need);
        CFD_REQUIRE(ws_bytes >= need, CFD_EARG, "workspace too small");
        CFD_REQUIRE(tape_bytes >= tape_bytes_mode(h, B, h->tape_mode), CFD_EARG, "tape too small");
        Workspace ws{align256(workspace), 0, false}, tws{align256(tape), 0, false};
        Tape tp{&tws, nullptr};
        tp.keep_gnout = h->tape_mode == CFD_TAPE_PARAM_GRAD;
        h->tapes.erase(tape);   // a re-recording replaces the old layout before anything runs
        run(h, x, t, eps, B, ws, (hipStream_t)stream, &tp, true);
        h->tapes[tape] = {h->tape_mode, B, plan_batch(h), ++h->tape_seq};
        while (h->tapes.size() > kMaxTapes) {
            auto old = h->tapes.begin();
            for (auto i = h->tapes.begin(); i != h->tapes.end(); ++i)
                if (i->second.seq < old->second.seq) old = i;
            h->tapes.erase(old);
        }
    });
}

extern "C" int cfd_unet_input_vjp(cfd_unet* h, const float* d_eps, float* d_x, int B, const void* tape,
                                  size_t tape_bytes, void* workspace, size_t ws_bytes, void* stream) {
    return cfd::guard([&] {
        CFD_REQUIRE(h && d_eps && d_x && tape && workspace, CFD_EARG, "null argument");
        CFD_REQUIRE(B > 0, CFD_EARG, "B must be positive");
        check_ready(h);
        size_t need = 0;
        cfd_unet_vjp_workspace_bytes(h, B, &need);
        CFD_REQUIRE(ws_bytes >= need, CFD_EARG, "workspace too small");
        const int mode = tape_rec(h, tape, B, tape_bytes).mode;
        // replay the forward walk (no launches) over the same tape layout to
        // recover where every saved activation lives
        Workspace fws{nullptr, 0, true}, tws{align256(const_cast<void*>(tape)), 0, false};
        std::vector<Rec> recs;
        Tape tp{&tws, &recs};
        tp.keep_gnout = mode == CFD_TAPE_PARAM_GRAD;
        run(h, nullptr, nullptr, nullptr, B, fws, nullptr, &tp, false);
        Workspace ws{align256(workspace), 0, false};
        run_vjp(h, d_eps, d_x, B, recs, ws, (hipStream_t)stream);
    });
}

extern "C" int cfd_unet_param_grad_workspace_bytes(const cfd_unet* h, int B, size_t* bytes) {
    return cfd::guard([&] {
        CFD_REQUIRE(h && bytes && B > 0, CFD_EARG, "bad argument");
        Workspace ws{nullptr, 0, true};
        std::vector<Rec> none;
        run_vjp(h, nullptr, nullptr, B, none, ws, nullptr, nullptr, true);
        *bytes = ws.off + 256;
    });
}

extern "C" int cfd_unet_param_grad(cfd_unet* h, const float* x, const float* d_eps, int B, const void* tape,
                                   size_t tape_bytes, float* grad, void* workspace, size_t ws_bytes, void* stream) {
    return cfd::guard([&] {
        CFD_REQUIRE(h && x && d_eps && tape && grad && workspace, CFD_EARG, "null argument");
        CFD_REQUIRE(B > 0, CFD_EARG, "B must be positive");
        check_ready(h);
        size_t need = 0;
        cfd_unet_param_grad_workspace_bytes(h, B, &need);
        CFD_REQUIRE(ws_bytes >= need, CFD_EARG, "workspace too small");
        const int mode = tape_rec(h, tape, B, tape_bytes).mode;
        Workspace fws{nullptr, 0, true}, tws{align256(const_cast<void*>(tape)), 0, false};
        std::vector<Rec> recs;
        Tape tp{&tws, &recs};
        tp.keep_gnout = mode == CFD_TAPE_PARAM_GRAD;
        run(h, nullptr, nullptr, nullptr, B, fws, nullptr, &tp, false);
        ParamGrad pg;
        pg.grad = grad;
        pg.x = x;
        pg.temb = tp.temb;
        pg.th1 = tp.th1;
        pg.emb = tp.emb;
        Workspace ws{align256(workspace), 0, false};
        run_vjp(h, d_eps, nullptr, B, recs, ws, (hipStream_t)stream, &pg, true);
    });
}

extern "C" int cfd_unet_check_finite(cfd_unet* h, int* nonfinite, void* stream) {
    return cfd::guard([&] {
        CFD_REQUIRE(h && nonfinite, CFD_EARG, "null argument");
        cfd::DeviceGuard dg(h->device);
        const hipStream_t st = (hipStream_t)stream;
        int v = 0;
        CFD_HIP(hipMemcpyAsync(&v, h->nonfinite, sizeof(int), hipMemcpyDeviceToHost, st));
        CFD_HIP(hipMemsetAsync(h->nonfinite, 0, sizeof(int), st));
        CFD_HIP(hipStreamSynchronize(st));
        *nonfinite = v;
    });
}
