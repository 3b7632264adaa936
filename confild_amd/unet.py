"""UNetModel drop-in (U/src/unet.py:396-663) backed by the HIP library.

The module keeps the reference's parameter tree, so ``state_dict()`` /
``load_state_dict()`` use exactly the reference keys (``time_embed.0.weight``,
``input_blocks.1.0.in_layers.2.weight``, ...; 368 tensors at 64 px) and an
``ema_*.pt`` checkpoint of the reference loads unchanged.  ``forward(x, t)``
runs the whole network as one ``cfd_unet_forward`` call (include/confild.h):
weights are packed once into kernel layouts on the device and re-packed only
when a parameter changes.  There is no CPU path: a CPU input raises.
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np
import torch
import torch.nn as nn

from . import _lib


def default_channel_mult(image_size: int):
    """U/src/script_util.py:150-160."""
    table = {512: (0.5, 1, 1, 2, 2, 4, 4), 256: (1, 1, 2, 2, 4, 4), 128: (1, 1, 2, 3, 4), 64: (1, 2, 3, 4)}
    if image_size not in table:
        raise ValueError(f"unsupported image size: {image_size}")
    return table[image_size]


def param_shapes(in_channels, model_channels, out_channels, num_res_blocks, attention_resolutions,
                 channel_mult, num_heads=1, num_head_channels=-1):
    """Reference state_dict key -> shape, in registration order (unet.py:469-616)."""
    mc, tdim = model_channels, model_channels * 4
    s = {}

    def conv(pre, cin, cout, k=3, one_d=False):
        s[pre + ".weight"] = (cout, cin, 1) if one_d else (cout, cin, k, k)
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
        heads = num_heads if num_head_channels == -1 else c // num_head_channels
        if heads <= 0 or c % heads:
            raise ValueError(f"q,k,v channels {c} is not divisible by num_head_channels {num_head_channels}")
        norm(pre + ".norm", c)
        conv(pre + ".qkv", c, 3 * c, one_d=True)
        conv(pre + ".proj_out", c, c, one_d=True)

    s["time_embed.0.weight"] = (tdim, mc)
    s["time_embed.0.bias"] = (tdim,)
    s["time_embed.2.weight"] = (tdim, tdim)
    s["time_embed.2.bias"] = (tdim,)
    ch = int(channel_mult[0] * mc)
    conv("input_blocks.0.0", in_channels, ch)
    chans, ds, idx = [ch], 1, 1
    for level, mult in enumerate(channel_mult):
        for _ in range(num_res_blocks):
            cout = int(mult * mc)
            res(f"input_blocks.{idx}.0", ch, cout)
            ch = cout
            if ds in attention_resolutions:
                attn(f"input_blocks.{idx}.1", ch)
            chans.append(ch)
            idx += 1
        if level != len(channel_mult) - 1:
            conv(f"input_blocks.{idx}.0.op", ch, ch)
            chans.append(ch)
            ds *= 2
            idx += 1
    res("middle_block.0", ch, ch)
    attn("middle_block.1", ch)
    res("middle_block.2", ch, ch)
    idx = 0
    for level, mult in list(enumerate(channel_mult))[::-1]:
        for i in range(num_res_blocks + 1):
            ich = chans.pop()
            cout = int(mc * mult)
            res(f"output_blocks.{idx}.0", ch + ich, cout)
            ch = cout
            j = 1
            if ds in attention_resolutions:
                attn(f"output_blocks.{idx}.1", ch)
                j = 2
            if level and i == num_res_blocks:
                conv(f"output_blocks.{idx}.{j}.conv", ch, ch)
                ds //= 2
            idx += 1
    norm("out.0", ch)
    conv("out.2", int(channel_mult[0] * mc), out_channels)
    return s


def forward_flops(image_size, in_channels, model_channels, out_channels, num_res_blocks, attention_resolutions,
                  channel_mult, num_heads=1, num_head_channels=-1):
    """FLOPs of one sample's forward, counted as torch's FlopCounterMode counts the
    reference (2 x MAC of every convolution, bmm / einsum and addmm; GroupNorm,
    SiLU and adds are not counted), by the walk of param_shapes / unet.py:469-663.
    Returns {"conv", "attn", "linear"}: the 2-D and 1-D convolutions, the two
    attention products (4 T^2 C per block), and time_embed + every emb_layers.
    Pinned against FlopCounterMode on the CPU oracle (tests/test_host.py)."""
    mc, tdim = model_channels, model_channels * 4
    f = {"conv": 0, "attn": 0, "linear": 2 * (mc * tdim + tdim * tdim)}
    hw = image_size * image_size

    def res(cin, cout, px):
        f["conv"] += 2 * px * cout * cin * 9 + 2 * px * cout * cout * 9 + (2 * px * cout * cin if cin != cout else 0)
        f["linear"] += 2 * tdim * cout

    def attn(c, px):
        f["conv"] += 2 * px * 3 * c * c + 2 * px * c * c
        f["attn"] += 4 * px * px * c

    ch = int(channel_mult[0] * mc)
    f["conv"] += 2 * hw * ch * in_channels * 9
    chans, ds, px = [ch], 1, hw
    for level, mult in enumerate(channel_mult):
        for _ in range(num_res_blocks):
            cout = int(mult * mc)
            res(ch, cout, px)
            ch = cout
            if ds in attention_resolutions:
                attn(ch, px)
            chans.append(ch)
        if level != len(channel_mult) - 1:
            px_out = ((image_size // ds + 1) // 2) ** 2
            f["conv"] += 2 * px_out * ch * ch * 9
            chans.append(ch)
            ds *= 2
            px = px_out
    res(ch, ch, px)
    attn(ch, px)
    res(ch, ch, px)
    for level, mult in list(enumerate(channel_mult))[::-1]:
        for i in range(num_res_blocks + 1):
            ich = chans.pop()
            cout = int(mc * mult)
            res(ch + ich, cout, px)
            ch = cout
            if ds in attention_resolutions:
                attn(ch, px)
            if level and i == num_res_blocks:
                px *= 4
                f["conv"] += 2 * px * ch * ch * 9
                ds //= 2
    f["conv"] += 2 * px * out_channels * ch * 9
    return f


def _zero_init_keys(keys):
    """Modules the reference wraps in zero_module (unet.py:210-212,294,615)."""
    out = set()
    for k in keys:
        if ".out_layers.3." in k or ".proj_out." in k or k.startswith("out.2."):
            out.add(k)
    return out


class _Node(nn.Module):
    """Parameter-only container mirroring one reference submodule path."""

    def forward(self, *a, **k):  # pragma: no cover - never called
        raise RuntimeError("parameter container")


def _build_tree(root: nn.Module, shapes: dict):
    for key, shape in shapes.items():
        parts = key.split(".")
        node = root
        for p in parts[:-1]:
            child = node._modules.get(p)
            if child is None:
                child = _Node()
                node.add_module(p, child)
            node = child
        node.register_parameter(parts[-1], nn.Parameter(torch.empty(shape)))


class UNetModel(nn.Module):
    """Same constructor as the reference UNetModel (unet.py:427-449).

    Supported: the configuration every CoNFiLD recipe uses (dims=2,
    conv_resample=True, legacy attention order, no class conditioning, no
    scale-shift norm, no resblock up/down).  Other options raise
    NotImplementedError instead of silently computing something else.
    """

    def __init__(self, image_size, in_channels, model_channels, out_channels, num_res_blocks,
                 attention_resolutions, dropout=0, channel_mult=(1, 2, 4, 8), conv_resample=True, dims=2,
                 num_classes=None, use_checkpoint=False, use_fp16=False, num_heads=1, num_head_channels=-1,
                 num_heads_upsample=-1, use_scale_shift_norm=False, resblock_updown=False,
                 use_new_attention_order=False):
        super().__init__()
        unsupported = {"num_classes": num_classes is not None, "use_scale_shift_norm": use_scale_shift_norm,
                       "resblock_updown": resblock_updown, "use_new_attention_order": use_new_attention_order,
                       "conv_resample=False": not conv_resample, "dims!=2": dims != 2,
                       "num_heads_upsample": num_heads_upsample not in (-1, num_heads),
                       "non-integer channel_mult": any(float(m) != int(m) for m in channel_mult)}
        bad = [k for k, v in unsupported.items() if v]
        if bad:
            raise NotImplementedError(f"UNetModel options not implemented on the HIP path: {bad}")
        if use_fp16:
            raise NotImplementedError("use_fp16: the HIP U-Net computes fp32 (bf16 MFMA variant is a later row)")
        self.image_size = image_size
        self.in_channels = in_channels
        self.model_channels = model_channels
        self.out_channels = out_channels
        self.num_res_blocks = num_res_blocks
        self.attention_resolutions = tuple(attention_resolutions)
        self.dropout = dropout
        self.channel_mult = tuple(int(m) for m in channel_mult)
        self.num_heads = num_heads
        self.num_head_channels = num_head_channels
        self.dtype = torch.float32
        shapes = param_shapes(in_channels, model_channels, out_channels, num_res_blocks,
                              self.attention_resolutions, self.channel_mult, num_heads, num_head_channels)
        self._shapes = shapes
        _build_tree(self, shapes)
        self._reset_parameters()
        # convolution arithmetic: "split_f16" (default; fp32-accurate on f16 MFMA, DESIGN.md
        # K1s), "fp32" (exact fp32 MFMA) or "bf16" (bf16 operands, config E)
        self.compute = "split_f16"
        self.plan_batch = 0     # the batch the convolution planner tiles for (0: 8)
        self._handles = {}      # device index -> (handle ptr, uploaded signature)
        self._workspaces = {}   # (device, B) -> uint8 tensor

    # -- initialisation (reference: PyTorch defaults + zero_module) ----------
    @torch.no_grad()
    def _reset_parameters(self):
        zero = _zero_init_keys(self._shapes)
        sd = dict(self.named_parameters())
        for k, p in sd.items():
            if k in zero:
                p.zero_()
            elif p.dim() == 1 and (k.endswith("in_layers.0.weight") or k.endswith("out_layers.0.weight")
                                   or k.endswith("norm.weight") or k == "out.0.weight"):
                p.fill_(1.0)
            elif p.dim() == 1 and (k.endswith("in_layers.0.bias") or k.endswith("out_layers.0.bias")
                                   or k.endswith("norm.bias") or k == "out.0.bias"):
                p.zero_()
            else:
                wk = k[:-4] + "weight" if k.endswith("bias") else k
                fan_in = int(np.prod(self._shapes[wk][1:]))
                b = 1.0 / math.sqrt(fan_in)
                p.uniform_(-b, b)

    # -- device handle ----------------------------------------------------------
    def _cfg_struct(self):
        cfg = _lib.UNetCfg()
        cfg.image_size = self.image_size
        cfg.in_channels = self.in_channels
        cfg.model_channels = self.model_channels
        cfg.out_channels = self.out_channels
        cfg.num_res_blocks = self.num_res_blocks
        cfg.n_mult = len(self.channel_mult)
        for i, m in enumerate(self.channel_mult):
            cfg.channel_mult[i] = m
        cfg.n_attn = len(self.attention_resolutions)
        for i, d in enumerate(self.attention_resolutions):
            cfg.attention_ds[i] = d
        cfg.num_heads = self.num_heads
        cfg.num_head_channels = self.num_head_channels
        return cfg

    COMPUTE_MODES = {"fp32": 0, "bf16": 1, "split_f16": 2}

    def set_compute(self, compute: str):
        """Convolution arithmetic: "fp32" (exact fp32 MFMA), "split_f16" (three f16 MFMAs on
        22-bit operand splits: fp32-level error) or "bf16" (bf16 operands,
        fp32 accumulation).  GroupNorm, softmax, attention and the 1-channel in/out
        convolutions stay fp32 in every mode."""
        if compute not in self.COMPUTE_MODES:
            raise ValueError(f"compute must be one of {sorted(self.COMPUTE_MODES)}, got {compute!r}")
        self.compute = compute
        return self

    def set_plan_batch(self, nominal_batch: int):
        """The batch the convolution planner tiles for (0: the default 8): a per-model
        setting, so results stay bit-identical across the batches a sample runs in.
        Set it near the chains per GPU when that is far from 8 (cfd_unet_set_plan_batch)."""
        if not 0 <= int(nominal_batch) <= 64:
            raise ValueError("plan batch must be in 0..64")
        if int(nominal_batch) != self.plan_batch:
            # the workspaces hold the split-K slab, sized per planned batch; a tape
            # recorded under the old plan cannot be replayed (the library refuses it)
            self._workspaces = {}
            self._vjp_ws, self._vjp_key = None, None
            self._pg_ws, self._pg_key = None, None
            self._taped = None
        self.plan_batch = int(nominal_batch)
        return self

    def prepare(self, device=None):
        """Upload and pack the parameters into the device handle now (the first
        forward does it otherwise): a timed region can then start with the weights
        resident in HBM.  Returns self."""
        dev = torch.device(device) if device is not None else next(self.parameters()).device
        if dev.type != "cuda":
            raise _lib.CfdError("UNetModel.prepare needs a GPU device")
        self._handle(dev)
        return self

    def _signature(self):
        return tuple((p.data_ptr(), p._version) for p in self.parameters())

    def _handle(self, device: torch.device):
        lib = _lib.lib()
        dev = device.index if device.index is not None else torch.cuda.current_device()
        entry = self._handles.get(dev)
        if entry is None:
            h = C.c_void_p()
            with torch.cuda.device(dev):
                _lib.check(lib.cfd_unet_create(C.byref(self._cfg_struct()), dev, C.byref(h)), "cfd_unet_create")
            entry = [h, None]
            self._handles[dev] = entry
            # timestep frequencies computed exactly as nn.py:129-131 (torch, fp32)
            half = self.model_channels // 2
            fr = torch.exp(-math.log(10000) * torch.arange(start=0, end=half, dtype=torch.float32) / half)
            fr = fr.contiguous()
            _lib.check(lib.cfd_unet_set_time_freqs(h, C.c_void_p(fr.data_ptr()), half), "set_time_freqs")
        sig = self._signature()
        if entry[1] != sig:
            h = entry[0]
            for k, p in self.named_parameters():
                host = p.detach().to("cpu", torch.float32).contiguous()
                _lib.check(lib.cfd_unet_set_param(h, k.encode(), C.c_void_p(host.data_ptr()), host.numel()),
                           f"set_param {k}")
            _lib.check(lib.cfd_unet_ready(h), "cfd_unet_ready")
            entry[1] = sig
        _lib.check(lib.cfd_unet_set_compute(entry[0], self.COMPUTE_MODES[self.compute]), "cfd_unet_set_compute")
        _lib.check(lib.cfd_unet_set_plan_batch(entry[0], self.plan_batch), "cfd_unet_set_plan_batch")
        return entry[0]

    def _workspace(self, h, device, B):
        key = (device, B)
        ws = self._workspaces.get(key)
        if ws is None:
            n = C.c_size_t()
            _lib.check(_lib.load().cfd_unet_workspace_bytes(h, B, C.byref(n)), "workspace_bytes")
            ws = torch.empty(n.value, dtype=torch.uint8, device=device)
            self._workspaces = {key: ws}  # keep one workspace (largest recent B)
        return ws

    def _prep(self, x, timesteps, y=None):
        if y is not None:
            raise NotImplementedError("class-conditional U-Net is not part of the CoNFiLD path")
        if x.device.type != "cuda":
            raise _lib.CfdError("UNetModel.forward: input must be on the GPU (the HIP path has no CPU fallback)")
        B, Cin, H, W = x.shape
        if Cin != self.in_channels or H != self.image_size or W != self.image_size:
            raise ValueError(f"expected (B, {self.in_channels}, {self.image_size}, {self.image_size}), got "
                             f"{tuple(x.shape)}")
        x = x.detach().to(torch.float32).contiguous()
        if timesteps.is_floating_point():
            if not torch.equal(timesteps, timesteps.round()):
                raise NotImplementedError("fractional timesteps (rescale_timesteps=True) are not supported")
        t = timesteps.to(device=x.device, dtype=torch.int64).contiguous()
        if t.shape != (B,):
            raise ValueError("timesteps must have shape (B,)")
        return x, t, B

    def forward(self, x: torch.Tensor, timesteps: torch.Tensor, y=None) -> torch.Tensor:
        """UNetModel.forward (unet.py:634-663): (B, C, H, W) fp32, (B,) timesteps -> eps."""
        if x.requires_grad and torch.is_grad_enabled():
            raise NotImplementedError("torch autograd does not run through the HIP U-Net: use forward_tape + "
                                      "input_vjp (the DPS sampler in confild_amd.guided does)")
        x, t, B = self._prep(x, timesteps, y)
        h = self._handle(x.device)
        ws = self._workspace(h, x.device, B)
        eps = torch.empty((B, self.out_channels, self.image_size, self.image_size), dtype=torch.float32,
                          device=x.device)
        _lib.check(_lib.load().cfd_unet_forward(h, _lib.ptr(x), _lib.ptr(t), _lib.ptr(eps), B, _lib.ptr(ws),
                                                ws.numel(), _lib.stream_of(x.device)), "cfd_unet_forward")
        return eps

    def check_finite(self, device=None):
        """Range guard of the split-f16 convolutions: reads and clears the device flag
        that every forward's last convolution raises on a non-finite eps (an
        activation beyond the f16 range, 65504, becomes inf in the f16 hi part).
        Raises CfdError in split_f16 compute (the fp32 / bf16 modes have no such
        range; there a non-finite eps only warns).  Synchronises the stream; the
        samplers call it once per loop."""
        import warnings
        dev = torch.device(device) if device is not None else next(self.parameters()).device
        if dev.type != "cuda":
            return True
        idx = dev.index if dev.index is not None else torch.cuda.current_device()
        entry = self._handles.get(idx)
        if entry is None:
            return True
        flag = C.c_int(0)
        _lib.check(_lib.load().cfd_unet_check_finite(entry[0], C.byref(flag), _lib.stream_of(dev)),
                   "cfd_unet_check_finite")
        if not flag.value:
            return True
        if self.compute == "split_f16":
            raise _lib.CfdError("U-Net produced a non-finite eps in split_f16 compute: an activation exceeded the f16 "
                                "range (65504) of the split convolutions; run with set_compute('fp32')")
        warnings.warn(f"U-Net produced a non-finite eps ({self.compute} compute)", RuntimeWarning, stacklevel=2)
        return False

    def clear_range_flag(self, device=None):
        """Clears the range-guard flag without acting on it (a loop starting fresh)."""
        dev = torch.device(device) if device is not None else next(self.parameters()).device
        if dev.type != "cuda":
            return
        idx = dev.index if dev.index is not None else torch.cuda.current_device()
        entry = self._handles.get(idx)
        if entry is not None:
            flag = C.c_int(0)
            _lib.check(_lib.load().cfd_unet_check_finite(entry[0], C.byref(flag), _lib.stream_of(dev)),
                       "cfd_unet_check_finite")

    # -- input-gradient (DPS adjoint) ---------------------------------------------
    def forward_tape(self, x: torch.Tensor, timesteps: torch.Tensor, for_param_grad: bool = False) -> torch.Tensor:
        """forward() that also records the activations for input_vjp (bit-identical eps).
        ``for_param_grad``: also keep the GroupNorm outputs param_grad's weight
        gradients read (CFD_TAPE_PARAM_GRAD: more tape, a faster param_grad)."""
        x, t, B = self._prep(x, timesteps)
        if self.compute == "bf16":
            raise NotImplementedError("the input-gradient (DPS) path is fp32-accurate: set_compute('fp32') or "
                                      "set_compute('split_f16')")
        h = self._handle(x.device)
        lib = _lib.load()
        ws = self._workspace(h, x.device, B)
        mode = 1 if for_param_grad else 0   # CFD_TAPE_PARAM_GRAD / CFD_TAPE_INPUT_VJP
        _lib.check(lib.cfd_unet_set_tape_mode(h, mode), "cfd_unet_set_tape_mode")
        self._tape_mode = mode
        tape = self._tape_buf(h, x.device, B)
        eps = torch.empty((B, self.out_channels, self.image_size, self.image_size), dtype=torch.float32,
                          device=x.device)
        _lib.check(lib.cfd_unet_forward_tape(h, _lib.ptr(x), _lib.ptr(t), _lib.ptr(eps), B, _lib.ptr(ws), ws.numel(),
                                             _lib.ptr(tape), tape.numel(), _lib.stream_of(x.device)),
                   "cfd_unet_forward_tape")
        self._taped = (x.device, B, self._signature())
        self._tape_x = x      # the forward's input (the first convolution's weight gradient reads it)
        return eps

    def input_vjp(self, d_eps: torch.Tensor) -> torch.Tensor:
        """(d eps / d x)^T d_eps for the inputs of the last forward_tape (weights are constants)."""
        if getattr(self, "_taped", None) is None:
            raise RuntimeError("input_vjp needs a preceding forward_tape")
        dev, B, sig = self._taped
        if sig != self._signature():
            raise RuntimeError("parameters changed since forward_tape")
        if tuple(d_eps.shape) != (B, self.out_channels, self.image_size, self.image_size) or d_eps.device != dev:
            raise ValueError("d_eps must match the eps of the last forward_tape")
        h = self._handle(dev)
        lib = _lib.load()
        d_eps = d_eps.detach().to(torch.float32).contiguous()
        tape = self._tape_buf(h, dev, B)
        key = ("vjp", dev, B)
        ws = self._vjp_ws if getattr(self, "_vjp_key", None) == key else None
        if ws is None:
            n = C.c_size_t()
            _lib.check(lib.cfd_unet_vjp_workspace_bytes(h, B, C.byref(n)), "vjp workspace")
            ws = self._vjp_ws = torch.empty(n.value, dtype=torch.uint8, device=dev)
            self._vjp_key = key
        d_x = torch.empty((B, self.in_channels, self.image_size, self.image_size), dtype=torch.float32, device=dev)
        _lib.check(lib.cfd_unet_input_vjp(h, _lib.ptr(d_eps), _lib.ptr(d_x), B, _lib.ptr(tape), tape.numel(),
                                          _lib.ptr(ws), ws.numel(), _lib.stream_of(dev)), "cfd_unet_input_vjp")
        return d_x

    def param_keys(self):
        """Parameter keys in the library's flat-gradient order (cfd_unet_param_info)."""
        if getattr(self, "_pkeys", None) is not None:
            return list(self._pkeys)
        dev = next(self.parameters()).device
        h, lib = self._handle(dev), _lib.load()
        n = C.c_int()
        _lib.check(lib.cfd_unet_num_params(h, C.byref(n)), "cfd_unet_num_params")
        keys = []
        for i in range(n.value):
            k, nd, shp = C.c_char_p(), C.c_int(), (C.c_int64 * 4)()
            _lib.check(lib.cfd_unet_param_info(h, i, C.byref(k), C.byref(nd), shp), "cfd_unet_param_info")
            keys.append(k.value.decode())
        self._pkeys = tuple(keys)      # the topology is fixed at construction
        return keys

    def flat_params(self):
        """(n,) fp32 device copy of every parameter, in param_keys() order."""
        named = dict(self.named_parameters())
        return torch.cat([named[k].detach().reshape(-1).to(torch.float32) for k in self.param_keys()]).contiguous()

    def load_flat(self, flat, alias=False):
        """Copy a flat_params()-ordered buffer back into the parameters.  On the
        handle's device the library re-packs from it on the GPU (cfd_unet_load_flat:
        one repack of every kernel layout, no host round trip); elsewhere the handle
        re-packs on its next call.  ``alias``: the parameters become views of
        ``flat`` instead of copies (the training loop's master buffer: later
        loads of the same buffer copy nothing)."""
        named = dict(self.named_parameters())
        keys = self.param_keys()
        n = sum(named[k].numel() for k in keys)
        if flat.numel() != n:
            raise ValueError(f"flat buffer has {flat.numel()} values, the parameters {n}")
        o = 0
        with torch.no_grad():
            for k in keys:
                p = named[k]
                view = flat[o:o + p.numel()].view(p.shape)
                if alias and view.device == p.device and view.dtype == p.dtype:
                    if p.data_ptr() != view.data_ptr():
                        p.data = view
                else:
                    p.copy_(view)
                o += p.numel()
        dev = flat.device
        entry = self._handles.get(dev.index) if dev.type == "cuda" else None
        if entry is not None and entry[1] is not None and flat.dtype == torch.float32 and flat.is_contiguous():
            _lib.check(_lib.load().cfd_unet_load_flat(entry[0], _lib.ptr(flat), n, _lib.stream_of(dev)),
                       "cfd_unet_load_flat")
            entry[1] = self._signature()

    def param_grad(self, d_eps: torch.Tensor, grad: torch.Tensor = None) -> torch.Tensor:
        """(d eps / d params)^T d_eps for the last forward_tape, accumulated (+=) into
        grad (flat fp32, param_keys() order; a new zero buffer when None) -- the
        U-Net half of loss.backward() in the diffusion TrainLoop."""
        if getattr(self, "_taped", None) is None:
            raise RuntimeError("param_grad needs a preceding forward_tape")
        dev, B, sig = self._taped
        if sig != self._signature():
            raise RuntimeError("parameters changed since forward_tape")
        if tuple(d_eps.shape) != (B, self.out_channels, self.image_size, self.image_size) or d_eps.device != dev:
            raise ValueError("d_eps must match the eps of the last forward_tape")
        n_total = sum(p.numel() for p in self.parameters())
        if grad is None:
            grad = torch.zeros(n_total, dtype=torch.float32, device=dev)
        if grad.numel() != n_total or grad.dtype != torch.float32 or not grad.is_contiguous() or grad.device != dev:
            raise ValueError("grad must be a contiguous fp32 buffer of every parameter on the tape's device")
        h = self._handle(dev)
        lib = _lib.load()
        d_eps = d_eps.detach().to(torch.float32).contiguous()
        tape = self._tape_buf(h, dev, B)
        key = ("pgrad", dev, B)
        ws = self._pg_ws if getattr(self, "_pg_key", None) == key else None
        if ws is None:
            n = C.c_size_t()
            _lib.check(lib.cfd_unet_param_grad_workspace_bytes(h, B, C.byref(n)), "param-grad workspace")
            ws = self._pg_ws = torch.empty(n.value, dtype=torch.uint8, device=dev)
            self._pg_key = key
        _lib.check(lib.cfd_unet_param_grad(h, _lib.ptr(self._tape_x), _lib.ptr(d_eps), B, _lib.ptr(tape),
                                           tape.numel(), _lib.ptr(grad), _lib.ptr(ws), ws.numel(),
                                           _lib.stream_of(dev)), "cfd_unet_param_grad")
        return grad

    def _tape_buf(self, h, device, B):
        # sized for the mode of the last forward_tape (input_vjp / param_grad replay it)
        key = (device, B, getattr(self, "_tape_mode", 0), self.plan_batch)
        if getattr(self, "_tape_key", None) != key:
            n = C.c_size_t()
            _lib.check(_lib.load().cfd_unet_tape_bytes(h, B, C.byref(n)), "tape bytes")
            self._tape = torch.empty(n.value, dtype=torch.uint8, device=device)
            self._tape_key = key
        return self._tape

    def __del__(self):
        try:
            lib = _lib.load()
            for h, _ in self._handles.values():
                lib.cfd_unet_destroy(h)
        except Exception:
            pass
