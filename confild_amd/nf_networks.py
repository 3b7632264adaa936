"""SIRENAutodecoder_film drop-in (N/cnf/nf_networks.py:443-495) on the fused HIP kernel.

Parameter tree and state_dict keys are the reference's (``net1.{i}.weight``,
``net1.{i}.bias``, ``net2.{i}.weight``), so ``checkpoint_*.pt["model_state_dict"]``
loads unchanged.  ``forward(coords, latents)`` keeps the reference signature and
broadcasting; ``decode(...)`` additionally fuses the coordinate normaliser and the
output de-normaliser (Normalizer_ts '-11') into the same launch.
"""
from __future__ import annotations

import ctypes as C
import math

import torch
import torch.nn as nn

from . import _lib

DEFAULT_W0 = 30.0  # N/cnf/initialization.py:5


class BatchLinear(nn.Linear):
    """Parameter holder with the reference layout (components.py:55-76).  Its
    arithmetic runs inside the fused SIREN kernel, never here."""

    def forward(self, input, params=None):
        raise _lib.CfdError("BatchLinear is evaluated inside the fused HIP SIREN kernel; call the network instead")


def _sine_init(m, w0=DEFAULT_W0):
    with torch.no_grad():
        n = m.weight.size(-1)
        m.weight.uniform_(-math.sqrt(6 / n) / w0, math.sqrt(6 / n) / w0)   # initialization.py:117-125


def _first_layer_sine_init(m):
    with torch.no_grad():
        n = m.weight.size(-1)
        m.weight.uniform_(-1 / n, 1 / n)                                     # initialization.py:127-132


def latent_grad_flops(d, L, c, nh, H, rows, points):
    """FLOPs of the DPS operator's SIREN part as FlopCounterMode counts the
    reference (measurements.py:219-226 under condition_methods.py:31-47): the
    forward at ``rows`` latent rows x ``points`` sensor coordinates -- the FiLM
    products (nh + 1) x (L -> H) per row, the first coordinate layer once per
    point (the reference broadcasts it over the rows), 2(nh H^2 + Hc) per (row,
    point) pair -- and autograd's backward to the latents only: every hidden and the
    output layer's input-gradient per pair, and the FiLM products' latent gradient
    per row.  Returns {"forward", "backward"}.  Pinned against FlopCounterMode on
    the CPU oracle (tests/test_host.py)."""
    film = 2 * (nh + 1) * H * L * rows
    fwd = 2 * d * H * points + 2 * (nh * H * H + H * c) * rows * points + film
    bwd = 2 * (nh * H * H + H * c) * rows * points + film
    return {"forward": fwd, "backward": bwd}


class SIRENAutodecoder_film(nn.Module):
    """Constructor as nf_networks.py:447-478 (sine nonlinearity, no premap)."""

    def __init__(self, in_coord_features, in_latent_features, out_features, num_hidden_layers, hidden_features,
                 outermost_linear=False, nonlinearity="sine", weight_init=None, bias_init=None, premap_mode=None,
                 **kwargs):
        super().__init__()
        if nonlinearity != "sine":
            raise NotImplementedError(f"nonlinearity {nonlinearity!r}: the fused kernel implements sine only")
        if premap_mode is not None:
            raise NotImplementedError("premap_mode (FeatureMapping) is not used by any CoNFiLD recipe")
        self.in_coord_features = in_coord_features
        self.in_latent_features = in_latent_features
        self.out_features = out_features
        self.num_hidden_layers = num_hidden_layers
        self.hidden_features = hidden_features
        self.w0 = DEFAULT_W0
        self.net1 = nn.ModuleList([BatchLinear(in_coord_features, hidden_features)]
                                  + [BatchLinear(hidden_features, hidden_features) for _ in range(num_hidden_layers)]
                                  + [BatchLinear(hidden_features, out_features)])
        self.net2 = nn.ModuleList([BatchLinear(in_latent_features, hidden_features, bias=False)
                                   for _ in range(num_hidden_layers + 1)])
        init = weight_init or _sine_init
        self.net1.apply(lambda m: init(m) if isinstance(m, BatchLinear) else None)
        self.net2.apply(lambda m: init(m) if isinstance(m, BatchLinear) else None)
        _first_layer_sine_init(self.net1[0])
        _first_layer_sine_init(self.net2[0])
        if bias_init is not None:
            self.net2.apply(bias_init)
        self._handles = {}
        self._compute = None  # None: the library default (CFD_SIREN_SPLIT_F16 where H % 32 == 0)

    COMPUTE_MODES = {"f32": 0, "split_f16": 1}

    def set_compute(self, mode: str):
        """Hidden-layer arithmetic of the fused decoder: "split_f16" (3 f16 MFMAs on
        two-term splits, fp32-level error; the default) or "f32" (exact fp32 MFMA)."""
        if mode not in self.COMPUTE_MODES:
            raise ValueError(f"compute mode {mode!r} not in {sorted(self.COMPUTE_MODES)}")
        self._compute = mode
        return self

    def compute_mode(self, device) -> str:
        """The mode a decode on `device` actually runs (split_f16 falls back to f32
        when H % 32 != 0 or there is no hidden layer)."""
        v = C.c_int()
        _lib.check(_lib.load().cfd_siren_get_compute(self._handle(device), C.byref(v)), "cfd_siren_get_compute")
        return {v_: k for k, v_ in self.COMPUTE_MODES.items()}[v.value]

    # -- device handle --------------------------------------------------------
    def prepare(self, device=None):
        """Upload and pack the parameters into the device handle now (the first
        decode does it otherwise).  Returns self."""
        dev = torch.device(device) if device is not None else next(self.parameters()).device
        if dev.type != "cuda":
            raise _lib.CfdError("SIRENAutodecoder_film.prepare needs a GPU device")
        self._handle(dev)
        return self

    def _signature(self):
        return tuple((p.data_ptr(), p._version) for p in self.parameters())

    def _handle(self, device):
        lib = _lib.lib()
        dev = device.index if device.index is not None else torch.cuda.current_device()
        entry = self._handles.get(dev)
        if entry is None:
            cfg = _lib.SirenCfg(self.in_coord_features, self.in_latent_features, self.out_features,
                                self.num_hidden_layers, self.hidden_features, self.w0)
            h = C.c_void_p()
            _lib.check(lib.cfd_siren_create(C.byref(cfg), dev, C.byref(h)), "cfd_siren_create")
            entry = [h, None]
            self._handles[dev] = entry
        sig = self._signature()
        if entry[1] != sig:
            for k, p in self.named_parameters():
                host = p.detach().to("cpu", torch.float32).contiguous()
                _lib.check(lib.cfd_siren_set_param(entry[0], k.encode(), C.c_void_p(host.data_ptr()), host.numel()),
                           f"siren set_param {k}")
            _lib.check(lib.cfd_siren_ready(entry[0]), "cfd_siren_ready")
            entry[1] = sig
        if self._compute is not None:
            _lib.check(lib.cfd_siren_set_compute(entry[0], self.COMPUTE_MODES[self._compute]), "cfd_siren_set_compute")
        return entry[0]

    # -- forward ----------------------------------------------------------------
    @staticmethod
    def _flatten(coords, latents, d, L):
        if coords.shape[-1] != d:
            raise ValueError(f"coords last dim {coords.shape[-1]} != in_coord_features {d}")
        if latents.shape[-1] != L:
            raise ValueError(f"latents last dim {latents.shape[-1]} != in_latent_features {L}")
        spatial = tuple(coords.shape[:-1])
        # reference broadcasting: coords (1, N, d) x latents (b, 1, L) -> (b, N, c);
        # coords (h, w, d) x latents (b, 1, 1, L) -> (b, h, w, c)
        if latents.dim() >= 2 and any(s != 1 for s in latents.shape[1:-1]):
            raise NotImplementedError("latents must be (b, 1, ..., 1, L): one latent per output field")
        if len(spatial) == latents.dim() - 1 and len(spatial) > 1 and spatial[0] == 1:
            spatial = spatial[1:]
        b = latents.shape[0] if latents.dim() >= 2 else 1
        return coords.reshape(-1, d), latents.reshape(b, L), spatial

    def _dev_param(self, t, dev):
        """fp32 device copy of a (usually host) normaliser parameter, cached while the
        source tensor is unchanged: a host-to-device copy from pageable memory waits for
        the stream, which in the DPS step would idle the GPU between the U-Net forward
        and the SIREN tape (4 such copies per step before the cache)."""
        if t.device == dev and t.dtype == torch.float32:
            return t
        cache = self.__dict__.setdefault("_norm_dev_cache", {})
        key = (id(t), dev)
        hit = cache.get(key)
        if hit is not None and hit[0] is t and hit[1] == t._version:
            return hit[2]
        v = t.to(device=dev, dtype=torch.float32)
        cache.pop(key, None)
        cache[key] = (t, t._version, v)
        while len(cache) > self._NORM_CACHE_MAX:   # bounded: callers may build new normalisers per call
            cache.pop(next(iter(cache)))
        return v

    _NORM_CACHE_MAX = 8   # (max, min) of the coordinate and output normalisers, two devices

    def _norm_args(self, cf, N, dev, x_normalizer, y_normalizer):
        """Fusable '-11' normaliser bounds -> (coords, xmax, xmin, ymax, ymin, ystride, post)."""
        d, c = self.in_coord_features, self.out_features
        xmax = xmin = ymax = ymin = None
        ystride = 0
        if x_normalizer is not None:
            if x_normalizer.method != "-11":
                cf = x_normalizer.normalize(cf).contiguous()
            else:
                xmax = self._dev_param(x_normalizer.params[0], dev).reshape(-1).contiguous()
                xmin = self._dev_param(x_normalizer.params[1], dev).reshape(-1).contiguous()
                if xmax.numel() != d:
                    raise ValueError("coordinate normaliser must have one (max, min) per coordinate feature")
        post = None
        if y_normalizer is not None:
            if y_normalizer.method != "-11":
                post = y_normalizer
            else:
                ymax = self._dev_param(y_normalizer.params[0], dev)
                ymin = self._dev_param(y_normalizer.params[1], dev)
                if ymax.numel() == c:
                    ystride = 0
                elif ymax.numel() == N * c:
                    ystride = c
                else:
                    raise ValueError(f"output normaliser params of {ymax.numel()} values match neither (c) nor (N, c)")
                ymax = ymax.reshape(-1).contiguous()
                ymin = ymin.reshape(-1).contiguous()
        return cf, xmax, xmin, ymax, ymin, ystride, post

    def decode(self, coords, latents, x_normalizer=None, y_normalizer=None, out=None):
        """denorm(NF(norm(coords), latents)) in one fused launch (trainer.infer,
        N/scripts/train.py:265-279; pass_through_model_batch, inference_function.py:22-48).
        ``out``: a contiguous fp32 (b, N, c) tensor the fields are written into (e.g.
        a row slice of a larger batch; fused '-11' output normalisers only)."""
        d, L, c = self.in_coord_features, self.in_latent_features, self.out_features
        dev = latents.device
        if dev.type != "cuda":
            raise _lib.CfdError("SIREN decode needs GPU tensors (the HIP path has no CPU fallback)")
        if latents.requires_grad and torch.is_grad_enabled():
            raise NotImplementedError("torch autograd does not run through the HIP SIREN: use tape_forward + "
                                      "tape_vjp (the DPS sampler in confild_amd.guided does)")
        cf, lat, spatial = self._flatten(coords, latents, d, L)
        cf = cf.to(device=dev, dtype=torch.float32).contiguous()
        lat = lat.detach().to(torch.float32).contiguous()
        N = cf.shape[0]
        cf, xmax, xmin, ymax, ymin, ystride, post = self._norm_args(cf, N, dev, x_normalizer, y_normalizer)
        h = self._handle(dev)
        b = lat.shape[0]
        nbytes = C.c_size_t()
        lib = _lib.load()
        _lib.check(lib.cfd_siren_workspace_bytes(h, b, C.byref(nbytes)), "siren workspace")
        ws = torch.empty(max(nbytes.value, 16), dtype=torch.uint8, device=dev)
        if out is None:
            out = torch.empty((b, N, c), dtype=torch.float32, device=dev)
        elif (tuple(out.shape) != (b, N, c) or out.dtype != torch.float32 or not out.is_contiguous()
              or out.device != dev or post is not None):
            raise ValueError(f"out must be a contiguous fp32 ({b}, {N}, {c}) tensor on {dev} (fused '-11' output "
                             f"normaliser only)")
        _lib.check(lib.cfd_siren_forward(h, _lib.ptr(cf), N, _lib.ptr(lat), b, _lib.ptr(xmax), _lib.ptr(xmin),
                                         _lib.ptr(ymax), _lib.ptr(ymin), ystride, _lib.ptr(out), _lib.ptr(ws),
                                         ws.numel(), _lib.stream_of(dev)), "cfd_siren_forward")
        if post is not None:
            out = post.denormalize(out)
        return out.reshape((b,) + spatial + (c,))

    # -- latent gradient at a few query points (DPS measurement operator) ---------
    def tape_forward(self, coords, latents, x_normalizer=None, y_normalizer=None):
        """decode() of R latent rows (R, L) at Ns points (Ns, d) -> (R, Ns, c), keeping the
        per-layer pre-activations for tape_vjp.  Only '-11' normalisers (fused)."""
        d, L, c = self.in_coord_features, self.in_latent_features, self.out_features
        dev = latents.device
        if dev.type != "cuda":
            raise _lib.CfdError("SIREN tape_forward needs GPU tensors (the HIP path has no CPU fallback)")
        cf = coords.reshape(-1, d).to(device=dev, dtype=torch.float32).contiguous()
        lat = latents.detach().reshape(-1, L).to(torch.float32).contiguous()
        Ns, R = cf.shape[0], lat.shape[0]
        cf, xmax, xmin, ymax, ymin, ystride, post = self._norm_args(cf, Ns, dev, x_normalizer, y_normalizer)
        if post is not None or (x_normalizer is not None and xmax is None):
            raise NotImplementedError("the SIREN latent gradient fuses '-11' normalisers only")
        h = self._handle(dev)
        lib = _lib.load()
        n = C.c_size_t()
        _lib.check(lib.cfd_siren_vjp_workspace_bytes(h, Ns, R, C.byref(n)), "siren vjp workspace")
        ws = torch.empty(max(n.value, 16), dtype=torch.uint8, device=dev)
        out = torch.empty((R, Ns, c), dtype=torch.float32, device=dev)
        _lib.check(lib.cfd_siren_tape_forward(h, _lib.ptr(cf), Ns, _lib.ptr(lat), R, _lib.ptr(xmax), _lib.ptr(xmin),
                                              _lib.ptr(ymax), _lib.ptr(ymin), ystride, _lib.ptr(out), _lib.ptr(ws),
                                              ws.numel(), _lib.stream_of(dev)), "cfd_siren_tape_forward")
        # keep every buffer the kernels read until tape_vjp
        self._vjp_tape = (ws, Ns, R, ymax, ymin, ystride, cf, lat, xmax, xmin, self._signature())
        return out

    def tape_vjp(self, g_out):
        """d<g_out, tape_forward(...)>/d latents -> (R, L), for the last tape_forward."""
        tape = getattr(self, "_vjp_tape", None)
        if tape is None:
            raise RuntimeError("tape_vjp needs a preceding tape_forward")
        ws, Ns, R, ymax, ymin, ystride, _, _, _, _, sig = tape
        if sig != self._signature():
            raise RuntimeError("parameters changed since tape_forward")
        if tuple(g_out.shape) != (R, Ns, self.out_features) or g_out.device != ws.device:
            raise ValueError("g_out must match the output of the last tape_forward")
        g = g_out.detach().to(torch.float32).contiguous()
        gz = torch.empty((R, self.in_latent_features), dtype=torch.float32, device=ws.device)
        h = self._handle(ws.device)
        _lib.check(_lib.load().cfd_siren_tape_vjp(h, _lib.ptr(g), Ns, R, _lib.ptr(ymax), _lib.ptr(ymin), ystride,
                                                  _lib.ptr(gz), _lib.ptr(ws), ws.numel(), _lib.stream_of(ws.device)),
                   "cfd_siren_tape_vjp")
        return gz

    # -- training (K10: cfd_siren_train_grad; the loop is confild_amd.cnf_train) ----
    def param_keys(self):
        """Parameter keys in the library's flat-gradient order (cfd_siren_param_info)."""
        dev = next(self.parameters()).device
        if dev.type != "cuda":
            raise _lib.CfdError("SIREN training needs the parameters on a GPU")
        h, lib = self._handle(dev), _lib.load()
        n = C.c_int()
        _lib.check(lib.cfd_siren_num_params(h, C.byref(n)), "cfd_siren_num_params")
        keys = []
        for i in range(n.value):
            k, nd, shp = C.c_char_p(), C.c_int(), (C.c_int64 * 4)()
            _lib.check(lib.cfd_siren_param_info(h, i, C.byref(k), C.byref(nd), shp), "cfd_siren_param_info")
            keys.append(k.value.decode())
        return keys

    def flat_params(self):
        """(n,) fp32 device copy of every parameter, in param_keys() order."""
        named = dict(self.named_parameters())
        return torch.cat([named[k].detach().reshape(-1).to(torch.float32) for k in self.param_keys()]).contiguous()

    def load_flat(self, flat):
        """Copy a flat_params()-ordered buffer back into the parameters (the handle
        re-packs its weight images on the next call)."""
        named = dict(self.named_parameters())
        o = 0
        with torch.no_grad():
            for k in self.param_keys():
                p = named[k]
                p.copy_(flat[o:o + p.numel()].reshape(p.shape))
                o += p.numel()
        if o != flat.numel():
            raise ValueError(f"flat buffer has {flat.numel()} values, the parameters {o}")

    def train_grad(self, coords, latents, rows, target, scale, grad, grad_latents, sse):
        """One backward of MSELoss for the latent rows `rows` of the (N_samples, L)
        table `latents` at raw coordinates (N, d) against target (R, N, c); adds
        into grad (flat, param_keys() order), grad_latents (N_samples, L) and sse (1)."""
        dev = latents.device
        if dev.type != "cuda":
            raise _lib.CfdError("SIREN training needs GPU tensors (the HIP path has no CPU fallback)")
        d, L, c = self.in_coord_features, self.in_latent_features, self.out_features
        cf = coords.reshape(-1, d).to(device=dev, dtype=torch.float32).contiguous()
        N = cf.shape[0]
        rows = rows.to(device=dev, dtype=torch.int64).contiguous()
        R = rows.numel()
        if torch.unique(rows).numel() != R:
            raise ValueError("batch latent rows must be distinct")
        tgt = target.to(device=dev, dtype=torch.float32).reshape(R, N, c).contiguous()
        for t, name in ((latents, "latents"), (grad, "grad"), (grad_latents, "grad_latents"), (sse, "sse")):
            if t.dtype != torch.float32 or not t.is_contiguous() or t.device != dev:
                raise ValueError(f"{name} must be a contiguous fp32 tensor on {dev}")
        if latents.shape[-1] != L or grad_latents.shape != latents.shape:
            raise ValueError("latents / grad_latents must be (N_samples, in_latent_features)")
        h, lib = self._handle(dev), _lib.load()
        n = C.c_size_t()
        _lib.check(lib.cfd_siren_train_workspace_bytes(h, N, R, C.byref(n)), "siren train workspace")
        ws = torch.empty(max(n.value, 16), dtype=torch.uint8, device=dev)
        _lib.check(lib.cfd_siren_train_grad(h, _lib.ptr(cf), N, _lib.ptr(latents), _lib.ptr(rows), R, _lib.ptr(tgt),
                                            float(scale), _lib.ptr(grad), _lib.ptr(grad_latents), _lib.ptr(sse),
                                            _lib.ptr(ws), ws.numel(), _lib.stream_of(dev)), "cfd_siren_train_grad")

    def forward(self, coords, latents):
        """nf_networks.py:480-495 (raw, un-normalised in and out)."""
        return self.decode(coords, latents)

    def disable_gradient(self):
        for p in self.parameters():
            p.requires_grad = False

    def __del__(self):
        try:
            lib = _lib.load()
            for h, _ in self._handles.values():
                lib.cfd_siren_destroy(h)
        except Exception:
            pass
