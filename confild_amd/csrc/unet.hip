// U-Net handle: topology (UNetModel.__init__, U/src/unet.py:427-616), parameter
// registry under the reference state_dict keys, weight packing, and the forward
// orchestration (UNetModel.forward, unet.py:634-663) over the HIP kernels of
// unet_kernels.hip.  All activations are NHWC fp32 in one caller-provided
// workspace; the forward issues only kernel launches on the given stream.
#include <algorithm>
#include <cmath>
#include <map>
#include <string>
#include <vector>

#include "unet_kernels.hpp"

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

void add_conv(cfd_unet* h, const std::string& pre, int cin, int cout, int k, bool conv1d = false) {
    if (conv1d)
        add_param(h, pre + ".weight", {cout, cin, 1}, Pack::Conv1);
    else
        add_param(h, pre + ".weight", {cout, cin, k, k}, k == 3 ? Pack::Conv3 : Pack::Conv1);
    add_param(h, pre + ".bias", {cout}, Pack::Raw);
}

void add_norm(cfd_unet* h, const std::string& pre, int c) {
    add_param(h, pre + ".weight", {c}, Pack::Raw);
    add_param(h, pre + ".bias", {c}, Pack::Raw);
}

int add_res(cfd_unet* h, const std::string& pre, int cin, int cout) {
    add_norm(h, pre + ".in_layers.0", cin);
    add_conv(h, pre + ".in_layers.2", cin, cout, 3);
    add_param(h, pre + ".emb_layers.1.weight", {cout, h->tdim}, Pack::EmbW, h->emb_total);
    add_param(h, pre + ".emb_layers.1.bias", {cout}, Pack::EmbB, h->emb_total);
    add_norm(h, pre + ".out_layers.0", cout);
    add_conv(h, pre + ".out_layers.3", cout, cout, 3);
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
                add_conv(h, up, ch, ch, 3);
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

// Executes (or, with ws.dry, sizes) one forward.
void run(const cfd_unet* h, const float* x, const int64_t* t, float* eps, int B, Workspace& ws, hipStream_t st) {
    const auto& c = h->cfg;
    const int mc = c.model_channels, S = c.image_size;
    // sizes: largest activation (any block output / ResBlock intermediate) and qkv
    size_t max_act = 0, max_qkv = 0, max_c2 = 0;
    {
        int ch = c.channel_mult[0] * mc, hw = S;
        max_act = std::max(max_act, (size_t)hw * hw * ch);
        for (int l = 0; l < c.n_mult; ++l) {
            const int co = c.channel_mult[l] * mc;
            max_act = std::max(max_act, (size_t)hw * hw * std::max(co, ch));
            max_qkv = std::max(max_qkv, (size_t)hw * hw * 3 * co);
            if (l != c.n_mult - 1) hw /= 2;
            ch = co;
        }
        max_c2 = 2 * (size_t)std::max(ch, c.channel_mult[0] * mc) * 4;  // generous for concat stats
        for (int l = 0; l < c.n_mult; ++l) max_c2 = std::max(max_c2, (size_t)4 * c.channel_mult[l] * mc * 2);
    }
    // split-K partial slab: the plan needs at most 16 x (8 samples' M x N) at the
    // low-resolution levels; scale with the batch so the memory guard never trips
    const size_t kSplitCap = (size_t(8) << 20) * (size_t)std::max(1, (B + 7) / 8);
    float* temb = ws.take((size_t)B * mc);
    float* h1 = ws.take((size_t)B * h->tdim);
    float* emb = ws.take((size_t)B * h->tdim);
    float* embo = ws.take((size_t)B * h->emb_total);
    (void)max_c2;
    double* gnpart = (double*)ws.take((size_t)B * 64 * 32 * 2 * 2);
    float* gnss = ws.take((size_t)B * 1024 * 2);
    // normalised (+SiLU) input of the next conv; the widest is an output block's
    // concat (current + skip channels) at its level: bound by hw^2 * (C_level + C_max)
    size_t max_cat = 0;
    {
        int cmax = 0, hw = S;
        for (int l = 0; l < c.n_mult; ++l) cmax = std::max(cmax, c.channel_mult[l] * mc);
        for (int l = 0; l < c.n_mult; ++l) {
            max_cat = std::max(max_cat, (size_t)hw * hw * (c.channel_mult[l] * mc + cmax));
            if (l != c.n_mult - 1) hw /= 2;
        }
        max_cat = std::max(max_cat, max_act);
    }
    float* nbuf = ws.take((size_t)B * max_cat);
    float* splitk = ws.take(kSplitCap);
    float* pool[3];
    for (auto& p : pool) p = ws.take((size_t)B * max_act);
    float* tmp = ws.take((size_t)B * max_act);
    float* skipb = ws.take((size_t)B * max_act);
    float* qkv = ws.take((size_t)B * max_qkv);
    float* abuf = ws.take((size_t)B * max_act);
    // skip stack buffers (one per Push)
    std::vector<float*> hsbuf;
    {
        int ch = c.channel_mult[0] * mc, hw = S;
        hsbuf.push_back(ws.take((size_t)B * hw * hw * ch));
        for (int l = 0; l < c.n_mult; ++l) {
            const int co = c.channel_mult[l] * mc;
            for (int r = 0; r < c.num_res_blocks; ++r) hsbuf.push_back(ws.take((size_t)B * hw * hw * co));
            ch = co;
            if (l != c.n_mult - 1) {
                hw /= 2;
                hsbuf.push_back(ws.take((size_t)B * hw * hw * ch));
            }
        }
    }
    if (ws.dry) return;

    auto pick = [&](const float* busy1, const float* busy2) -> float* {
        for (auto p : pool)
            if (p != busy1 && p != busy2) return p;
        throw cfd::Error{CFD_ESTATE, "internal: buffer pool exhausted"};
    };

    // timestep embedding + time_embed MLP + every ResBlock's emb_layers (nn.py:118-136, unet.py:648,199-205)
    cfd::launch_temb(t, h->freqs, temb, mc, B, st);
    cfd::launch_linear(temb, P(h, "time_embed.0.weight"), P(h, "time_embed.0.bias"), h1, B, mc, h->tdim, 0, st);
    cfd::launch_linear(h1, P(h, "time_embed.2.weight"), P(h, "time_embed.2.bias"), emb, B, h->tdim, h->tdim, 1, st);
    cfd::launch_linear(emb, h->emb_w, h->emb_b, embo, B, h->tdim, h->emb_total, 1, st);

    // GroupNorm(+SiLU) of `in` materialised once into nbuf (contiguous Ctot channels)
    auto gn = [&](const Act& in, const std::string& pre, int silu) -> Act {
        cfd::GnArgs g{};
        g.src1 = in.a;
        g.src2 = in.b;
        g.gamma = P(h, pre + ".weight");
        g.beta = P(h, pre + ".bias");
        g.part = gnpart;
        g.ss = gnss;
        g.out = nbuf;
        g.C1 = in.Ca;
        g.C2 = in.Cb;
        g.Ctot = in.C();
        g.HW = in.H * in.W;
        g.eps = 1e-5f;
        g.silu = silu;
        cfd::launch_gn(g, B, st);
        return Act{nbuf, in.C(), nullptr, 0, in.H, in.W};
    };
    auto conv = [&](const Act& in, const std::string& pre, int cout, int ks, int stride, int up,
                    const float* embp, const float* resp, float* out) {
        cfd::ConvArgs a{};
        a.src1 = in.a;
        a.src2 = in.b;
        a.C1 = in.Ca;
        a.C2 = in.Cb;
        a.Ctot = in.C();
        a.w = P(h, pre + ".weight");
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
        cfd::launch_conv(a, cfd::plan_conv(a, kSplitCap), st);
    };

    std::vector<Act> stack;
    Act cur;
    size_t hs_i = 0;
    for (size_t si = 0; si < h->steps.size(); ++si) {
        const auto& s = h->steps[si];
        // a block output that is pushed onto the skip stack is written straight
        // into its skip buffer (no copy)
        const bool to_skip = si + 1 < h->steps.size() && h->steps[si + 1].kind == cfd::Step::Push;
        auto dest = [&](const float* busy1, const float* busy2) -> float* {
            return to_skip ? hsbuf[hs_i] : pick(busy1, busy2);
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
                cfd::launch_conv_in(a, st);
                cur = Act{hsbuf[0], s.cout, nullptr, 0, S, S};
                break;
            }
            case cfd::Step::Push: {
                // the current activation must live in its own skip buffer
                float* dst = hsbuf[hs_i];
                if (cur.a != dst) {
                    CFD_HIP(hipMemcpyAsync(dst, cur.a, sizeof(float) * (size_t)B * cur.H * cur.W * cur.Ca,
                                           hipMemcpyDeviceToDevice, st));
                    cur.a = dst;
                }
                stack.push_back(cur);
                ++hs_i;
                break;
            }
            case cfd::Step::Cat: {
                const Act skip = stack.back();
                stack.pop_back();
                CFD_REQUIRE(cur.b == nullptr && skip.H == cur.H, CFD_ESTATE, "internal: concat shape");
                cur.b = skip.a;
                cur.Cb = skip.Ca;
                break;
            }
            case cfd::Step::Res: {
                const auto& r = h->res[s.idx];
                CFD_REQUIRE(cur.C() == r.cin, CFD_ESTATE, "internal: ResBlock input channels at " + r.pre);
                // h = in_layers(x) + emb_layers(emb)   (unet.py:236-254)
                const Act xin = gn(cur, r.pre + ".in_layers.0", 1);
                conv(xin, r.pre + ".in_layers.2", r.cout, 3, 1, 0, embo + r.emb_off, nullptr, tmp);
                const Act th{tmp, r.cout, nullptr, 0, cur.H, cur.W};
                // skip(x) + out_layers(h)   (unet.py:255-256)
                const float* resp;
                if (r.cin != r.cout) {
                    conv(cur, r.pre + ".skip_connection", r.cout, 1, 1, 0, nullptr, nullptr, skipb);
                    resp = skipb;
                } else {
                    CFD_REQUIRE(cur.b == nullptr, CFD_ESTATE, "identity skip on a concatenated input");
                    resp = cur.a;
                }
                const Act hn = gn(th, r.pre + ".out_layers.0", 1);
                float* out = dest(cur.a, cur.b);
                conv(hn, r.pre + ".out_layers.3", r.cout, 3, 1, 0, nullptr, resp, out);
                cur = Act{out, r.cout, nullptr, 0, cur.H, cur.W};
                break;
            }
            case cfd::Step::Attn: {
                const auto& at = h->attn[s.idx];
                const Act xn = gn(cur, at.pre + ".norm", 0);
                conv(xn, at.pre + ".qkv", 3 * at.C, 1, 1, 0, nullptr, nullptr, qkv);
                cfd::AttnArgs aa{qkv, abuf, cur.H * cur.W, at.C, (float)(1.0 / std::sqrt(std::sqrt((double)at.ch)))};
                cfd::launch_attention(aa, at.ch, at.heads, B, st);
                float* out = dest(cur.a, nullptr);
                conv(Act{abuf, at.C, nullptr, 0, cur.H, cur.W}, at.pre + ".proj_out", at.C, 1, 1, 0, nullptr, cur.a,
                     out);
                cur = Act{out, at.C, nullptr, 0, cur.H, cur.W};
                break;
            }
            case cfd::Step::Down: {
                float* out = dest(cur.a, nullptr);
                conv(cur, s.conv, s.cout, 3, 2, 0, nullptr, nullptr, out);
                cur = Act{out, s.cout, nullptr, 0, (cur.H + 1) / 2, (cur.W + 1) / 2};
                break;
            }
            case cfd::Step::Up: {
                float* out = pick(cur.a, nullptr);
                conv(cur, s.conv, s.cout, 3, 1, 1, nullptr, nullptr, out);
                cur = Act{out, s.cout, nullptr, 0, cur.H * 2, cur.W * 2};
                break;
            }
            case cfd::Step::Out: {
                const Act on = gn(cur, "out.0", 1);
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
        CFD_HIP(hipSetDevice(device));
        auto* h = new cfd_unet();
        h->cfg = *cfg;
        h->device = device;
        try {
            build(h);
            CFD_HIP(hipMalloc(&h->arena, sizeof(float) * h->arena_floats));
            CFD_HIP(hipMalloc(&h->emb_w, sizeof(float) * (size_t)h->emb_total * h->tdim));
            CFD_HIP(hipMalloc(&h->emb_b, sizeof(float) * (size_t)h->emb_total));
            const int half = cfg->model_channels / 2;
            // freqs = exp(-ln(10000) * arange(half, fp32) / half) in fp32 (nn.py:129-131)
            std::vector<float> fr(half);
            const float nl = (float)(-std::log(10000.0));
            for (int i = 0; i < half; ++i) fr[i] = std::exp((nl * (float)i) / (float)half);
            CFD_HIP(hipMalloc(&h->freqs, sizeof(float) * std::max(half, 1)));
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
        CFD_HIP(hipSetDevice(h->device));
        switch (p.pack) {
            case Pack::Raw:
            case Pack::Conv1:
                CFD_HIP(hipMemcpy(h->arena + p.offset, host, n * 4, hipMemcpyHostToDevice));
                break;
            case Pack::Conv3: {
                // (Cout, Cin, 3, 3) -> (Cout, tap, Cin): GEMM K ordered (tap, channel)
                const int64_t co = p.shape[0], ci = p.shape[1];
                std::vector<float> pk(n);
                for (int64_t o = 0; o < co; ++o)
                    for (int64_t i = 0; i < ci; ++i)
                        for (int tap = 0; tap < 9; ++tap) pk[(o * 9 + tap) * ci + i] = host[(o * ci + i) * 9 + tap];
                CFD_HIP(hipMemcpy(h->arena + p.offset, pk.data(), n * 4, hipMemcpyHostToDevice));
                break;
            }
            case Pack::EmbW:
                CFD_HIP(hipMemcpy(h->emb_w + (size_t)p.emb_row * h->tdim, host, n * 4, hipMemcpyHostToDevice));
                break;
            case Pack::EmbB:
                CFD_HIP(hipMemcpy(h->emb_b + p.emb_row, host, n * 4, hipMemcpyHostToDevice));
                break;
        }
        p.set = true;
    });
}

extern "C" int cfd_unet_set_time_freqs(cfd_unet* h, const float* host, int n) {
    return cfd::guard([&] {
        CFD_REQUIRE(h && host && n == h->cfg.model_channels / 2, CFD_EARG, "freqs must have model_channels/2 entries");
        CFD_HIP(hipSetDevice(h->device));
        CFD_HIP(hipMemcpy(h->freqs, host, sizeof(float) * n, hipMemcpyHostToDevice));
    });
}

extern "C" int cfd_unet_ready(const cfd_unet* h) {
    return cfd::guard([&] {
        CFD_REQUIRE(h, CFD_EARG, "null handle");
        for (const auto& p : h->params) CFD_REQUIRE(p.set, CFD_ESTATE, "U-Net parameter not set: " + p.key);
    });
}

extern "C" int cfd_unet_workspace_bytes(const cfd_unet* h, int B, size_t* bytes) {
    return cfd::guard([&] {
        CFD_REQUIRE(h && bytes && B > 0, CFD_EARG, "bad argument");
        Workspace ws{nullptr, 0, true};
        run(h, nullptr, nullptr, nullptr, B, ws, nullptr);
        *bytes = ws.off + 256;
    });
}

extern "C" int cfd_unet_forward(cfd_unet* h, const float* x, const int64_t* t, float* eps, int B, void* workspace,
                                size_t ws_bytes, void* stream) {
    return cfd::guard([&] {
        CFD_REQUIRE(h && x && t && eps && workspace, CFD_EARG, "null argument");
        CFD_REQUIRE(B > 0, CFD_EARG, "B must be positive");
        for (const auto& p : h->params) CFD_REQUIRE(p.set, CFD_ESTATE, "U-Net parameter not set: " + p.key);
        size_t need = 0;
        cfd_unet_workspace_bytes(h, B, &need);
        CFD_REQUIRE(ws_bytes >= need, CFD_EARG, "workspace too small");
        Workspace ws{(char*)(((uintptr_t)workspace + 255) & ~uintptr_t(255)), 0, false};
        run(h, x, t, eps, B, ws, (hipStream_t)stream);
    });
}
