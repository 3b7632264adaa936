"""Oracle: functional CPU restatement of the guided-diffusion U-Net forward.

Follows U/src/unet.py:396-663 (UNetModel), :143-256 (ResBlock),
:259-305 (AttentionBlock), :328-358 (QKVAttentionLegacy), :81-140
(Up/Downsample) and U/src/nn.py:17-19,108-136 (GroupNorm32,
timestep_embedding), op for op in fp32 on the CPU, reading the reference
state_dict key names.  Test-only (see oracle/__init__.py).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def default_channel_mult(image_size: int):
    """U/src/script_util.py:150-160."""
    table = {512: (0.5, 1, 1, 2, 2, 4, 4), 256: (1, 1, 2, 2, 4, 4), 128: (1, 1, 2, 3, 4), 64: (1, 2, 3, 4)}
    if image_size not in table:
        raise ValueError(f"unsupported image size: {image_size}")
    return table[image_size]


class Config:
    def __init__(self, image_size, num_channels, num_res_blocks, channel_mult=None,
                 num_heads=1, num_head_channels=-1, attention_resolutions="16", in_channels=1,
                 out_channels=1):
        self.image_size = image_size
        self.model_channels = num_channels
        self.num_res_blocks = num_res_blocks
        if channel_mult is None or channel_mult == "":
            self.channel_mult = default_channel_mult(image_size)
        elif isinstance(channel_mult, str):
            self.channel_mult = tuple(int(c) for c in channel_mult.split(","))
        else:
            self.channel_mult = tuple(channel_mult)
        self.num_heads = num_heads
        self.num_head_channels = num_head_channels
        self.attention_ds = tuple(image_size // int(r) for r in str(attention_resolutions).split(","))
        self.in_channels = in_channels
        self.out_channels = out_channels


def _atleast_f32(x):
    return x if x.dtype == torch.float64 else x.float()


def _gn(sd, pre, x):
    # GroupNorm32: 32 groups, eps 1e-5, computed in fp32 (nn.py:17-19,108-115)
    # GroupNorm32 runs in fp32 (nn.py:17-19); fp64 evaluations (tests) stay fp64
    return F.group_norm(_atleast_f32(x), 32, sd[pre + ".weight"], sd[pre + ".bias"], 1e-5).type(x.dtype)


def _conv(sd, pre, x, stride=1, pad=1):
    return F.conv2d(x, sd[pre + ".weight"], sd[pre + ".bias"], stride=stride, padding=pad)


def _conv1d(sd, pre, x):
    return F.conv1d(x, sd[pre + ".weight"], sd[pre + ".bias"])


def timestep_embedding(t, dim, max_period=10000):
    half = dim // 2
    freqs = torch.exp(-math.log(max_period) * torch.arange(0, half, dtype=torch.float32) / half)
    args = t[:, None].float() * freqs[None]
    emb = torch.cat([torch.cos(args), torch.sin(args)], dim=-1)
    if dim % 2:
        emb = torch.cat([emb, torch.zeros_like(emb[:, :1])], dim=-1)
    return emb


def resblock(sd, pre, x, emb, cin, cout):
    """ResBlock._forward, unet.py:236-256 (no up/down, no scale-shift)."""
    h = F.silu(_gn(sd, pre + ".in_layers.0", x))
    h = _conv(sd, pre + ".in_layers.2", h)
    e = F.linear(F.silu(emb), sd[pre + ".emb_layers.1.weight"], sd[pre + ".emb_layers.1.bias"])
    h = h + e[..., None, None]
    h = F.silu(_gn(sd, pre + ".out_layers.0", h))
    h = _conv(sd, pre + ".out_layers.3", h)
    if cin == cout:
        skip = x
    else:
        skip = _conv(sd, pre + ".skip_connection", x, pad=0)
    return skip + h


def attention(sd, pre, x, channels, cfg: Config):
    """AttentionBlock._forward + QKVAttentionLegacy, unet.py:296-305,337-354."""
    heads = cfg.num_heads if cfg.num_head_channels == -1 else channels // cfg.num_head_channels
    b, c, hh, ww = x.shape
    xf = x.reshape(b, c, -1)
    qkv = _conv1d(sd, pre + ".qkv", _gn(sd, pre + ".norm", xf))
    bs, width, length = qkv.shape
    ch = width // (3 * heads)
    q, k, v = qkv.reshape(bs * heads, ch * 3, length).split(ch, dim=1)
    scale = 1 / math.sqrt(math.sqrt(ch))
    w = torch.einsum("bct,bcs->bts", q * scale, k * scale)
    w = torch.softmax(_atleast_f32(w), dim=-1).type(w.dtype)
    a = torch.einsum("bts,bcs->bct", w, v).reshape(bs, -1, length)
    h = _conv1d(sd, pre + ".proj_out", a)
    return (xf + h).reshape(b, c, hh, ww)


def forward(sd: dict, cfg: Config, x: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
    """UNetModel.forward, unet.py:634-663 (topology from __init__ :427-616)."""
    mc = cfg.model_channels
    emb = timestep_embedding(t, mc).to(sd["time_embed.0.weight"].dtype)  # fp64 evaluations (tests)
    emb = F.linear(emb, sd["time_embed.0.weight"], sd["time_embed.0.bias"])
    emb = F.linear(F.silu(emb), sd["time_embed.2.weight"], sd["time_embed.2.bias"])

    hs = []
    h = _conv(sd, "input_blocks.0.0", x)
    hs.append(h)
    ch = int(cfg.channel_mult[0] * mc)
    chans = [ch]
    ds, idx = 1, 1
    for level, mult in enumerate(cfg.channel_mult):
        for _ in range(cfg.num_res_blocks):
            cout = int(mult * mc)
            h = resblock(sd, f"input_blocks.{idx}.0", h, emb, ch, cout)
            ch = cout
            if ds in cfg.attention_ds:
                h = attention(sd, f"input_blocks.{idx}.1", h, ch, cfg)
            hs.append(h)
            chans.append(ch)
            idx += 1
        if level != len(cfg.channel_mult) - 1:
            h = _conv(sd, f"input_blocks.{idx}.0.op", h, stride=2)
            hs.append(h)
            chans.append(ch)
            ds *= 2
            idx += 1
    h = resblock(sd, "middle_block.0", h, emb, ch, ch)
    h = attention(sd, "middle_block.1", h, ch, cfg)
    h = resblock(sd, "middle_block.2", h, emb, ch, ch)
    idx = 0
    for level, mult in list(enumerate(cfg.channel_mult))[::-1]:
        for i in range(cfg.num_res_blocks + 1):
            ich = chans.pop()
            h = torch.cat([h, hs.pop()], dim=1)
            cout = int(mc * mult)
            h = resblock(sd, f"output_blocks.{idx}.0", h, emb, ch + ich, cout)
            ch = cout
            j = 1
            if ds in cfg.attention_ds:
                h = attention(sd, f"output_blocks.{idx}.1", h, ch, cfg)
                j = 2
            if level and i == cfg.num_res_blocks:
                h = F.interpolate(h, scale_factor=2, mode="nearest")
                h = _conv(sd, f"output_blocks.{idx}.{j}.conv", h)
                ds //= 2
            idx += 1
    h = F.silu(_gn(sd, "out.0", h))
    return _conv(sd, "out.2", h)


def param_shapes(cfg: Config) -> dict:
    """Reference state_dict key -> shape, in the reference's registration order."""
    mc, tdim = cfg.model_channels, cfg.model_channels * 4
    s = {}

    def conv(pre, cin, cout, k=3):
        s[pre + ".weight"] = (cout, cin, k, k)
        s[pre + ".bias"] = (cout,)

    def norm(pre, c):
        s[pre + ".weight"] = (c,)
        s[pre + ".bias"] = (c,)

    def res(pre, cin, cout):
        norm(pre + ".in_layers.0", cin)
        conv(pre + ".in_layers.2", cin, cout)
        s[pre + ".emb_layers.1.weight"] = (cout, tdim)
        s[pre + ".emb_layers.1.bias"] = (cout,)
        norm(pre + ".out_layers.0", cout)
        conv(pre + ".out_layers.3", cout, cout)
        if cin != cout:
            conv(pre + ".skip_connection", cin, cout, 1)

    def attn(pre, c):
        norm(pre + ".norm", c)
        s[pre + ".qkv.weight"] = (3 * c, c, 1)
        s[pre + ".qkv.bias"] = (3 * c,)
        s[pre + ".proj_out.weight"] = (c, c, 1)
        s[pre + ".proj_out.bias"] = (c,)

    s["time_embed.0.weight"] = (tdim, mc)
    s["time_embed.0.bias"] = (tdim,)
    s["time_embed.2.weight"] = (tdim, tdim)
    s["time_embed.2.bias"] = (tdim,)
    ch = int(cfg.channel_mult[0] * mc)
    conv("input_blocks.0.0", cfg.in_channels, ch)
    chans, ds, idx = [ch], 1, 1
    for level, mult in enumerate(cfg.channel_mult):
        for _ in range(cfg.num_res_blocks):
            cout = int(mult * mc)
            res(f"input_blocks.{idx}.0", ch, cout)
            ch = cout
            if ds in cfg.attention_ds:
                attn(f"input_blocks.{idx}.1", ch)
            chans.append(ch)
            idx += 1
        if level != len(cfg.channel_mult) - 1:
            conv(f"input_blocks.{idx}.0.op", ch, ch)
            chans.append(ch)
            ds *= 2
            idx += 1
    res("middle_block.0", ch, ch)
    attn("middle_block.1", ch)
    res("middle_block.2", ch, ch)
    idx = 0
    for level, mult in list(enumerate(cfg.channel_mult))[::-1]:
        for i in range(cfg.num_res_blocks + 1):
            ich = chans.pop()
            cout = int(mc * mult)
            res(f"output_blocks.{idx}.0", ch + ich, cout)
            ch = cout
            j = 1
            if ds in cfg.attention_ds:
                attn(f"output_blocks.{idx}.1", ch)
                j = 2
            if level and i == cfg.num_res_blocks:
                conv(f"output_blocks.{idx}.{j}.conv", ch, ch)
                ds //= 2
            idx += 1
    norm("out.0", ch)
    conv("out.2", int(cfg.channel_mult[0] * mc), cfg.out_channels)
    return s
