"""Measurement operators and noises (C/src/guided_diffusion/measurements.py).

Only the Case4 operator is on the CoNFiLD path.  Its
forward is the fused HIP SIREN decode at the sensor coordinates; the DPS
sampler additionally uses ``forward_tape`` / ``vjp`` (the latent gradient).
"""
from __future__ import annotations

from abc import ABC, abstractmethod

import numpy as np
import torch

from .. import _lib
from ..inference import latent_denorm
from ..nf_networks import SIRENAutodecoder_film
from ..normalize import Normalizer_ts

__OPERATOR__ = {}


def register_operator(name: str):
    def wrapper(cls):
        if __OPERATOR__.get(name, None):
            raise NameError(f"Name {name} is already registered!")
        __OPERATOR__[name] = cls
        return cls
    return wrapper


def get_operator(name: str, **kwargs):
    """measurements.py:30-33."""
    if __OPERATOR__.get(name, None) is None:
        raise NameError(f"Name {name} is not defined.")
    return __OPERATOR__[name](**kwargs)


class LinearOperator(ABC):
    @abstractmethod
    def forward(self, data, **kwargs):
        pass


class NonLinearOperator(ABC):
    @abstractmethod
    def forward(self, data, **kwargs):
        pass

    def project(self, data, measurement, **kwargs):
        return data + measurement - self.forward(data)


def _siren_dims(sd):
    n1 = sorted(int(k.split(".")[1]) for k in sd if k.startswith("net1.") and k.endswith(".weight"))
    first, last = sd["net1.0.weight"], sd[f"net1.{n1[-1]}.weight"]
    return first.shape[1], sd["net2.0.weight"].shape[1], last.shape[0], len(n1) - 2, first.shape[0]


@register_operator(name="case4")
class Case4Operator(NonLinearOperator):
    """measurements.py:184-226.  The reference hard-codes SIRENAutodecoder_film(3,
    384, 3, 15, 384); here the dimensions are read from the checkpoint (identical
    for the reference's checkpoint, and usable for others)."""

    def __init__(self, device, coords_path, batch_size, max_val_path, min_val_path, normalizer_params_path,
                 ckpt_path) -> None:
        self.device = device
        coords = np.load(coords_path)
        self.coords = torch.tensor(coords, dtype=torch.float32, device=device)
        params = torch.load(normalizer_params_path, weights_only=True, map_location="cpu")
        x_uub, x_llb = params["x_normalizer_params"]
        y_uub, _ = params["y_normalizer0u_params"]
        _, y_llb = params["y_normalizer0l_params"]
        cin_size, cout_size = 3, 3
        self.x_normalizer = Normalizer_ts(method="-11", dim=0, params=(x_uub, x_llb))
        self.y_normalizer = Normalizer_ts(method="-11", dim=0, params=(y_uub[:cout_size], y_llb[:cout_size]))
        ckpt = torch.load(ckpt_path, weights_only=True, map_location="cpu")
        sd = ckpt["model_state_dict"]
        d, L, c, nh, H = _siren_dims(sd)
        if d != cin_size or c != cout_size:
            raise ValueError(f"Case4 SIREN must map 3 coordinates to 3 outputs, checkpoint has {d} -> {c}")
        self.model = SIRENAutodecoder_film(d, L, c, nh, H)
        self.model.load_state_dict(sd)
        self.model.eval()
        self.model.to(device)
        self.max_val = torch.from_numpy(np.load(max_val_path)).to(device)
        self.min_val = torch.from_numpy(np.load(min_val_path)).to(device)
        self.batch_size = batch_size

    @classmethod
    def from_parts(cls, device, coords, x_normalizer, y_normalizer, model, max_val, min_val, batch_size=384):
        """An operator from in-memory pieces (what a test or a synthetic run needs)."""
        op = cls.__new__(cls)
        op.device = device
        op.coords = torch.as_tensor(coords, dtype=torch.float32).to(device)
        op.x_normalizer, op.y_normalizer, op.model = x_normalizer, y_normalizer, model.to(device)
        op.max_val = torch.as_tensor(max_val).to(device)
        op.min_val = torch.as_tensor(min_val).to(device)
        op.batch_size = batch_size
        return op

    def _unnorm(self, norm_data):
        return ((norm_data[:, 0, ...] + 1) * (self.max_val - self.min_val) / 2 + self.min_val)[:, None, ...]

    def _bounds(self):
        vmax = self.max_val.to(device=self.coords.device, dtype=torch.float32).reshape(-1).contiguous()
        vmin = self.min_val.to(device=self.coords.device, dtype=torch.float32).reshape(-1).contiguous()
        return vmax, vmin

    def _rows(self, data):
        """_unnorm + rearrange "s c t l -> (s c t) l" on the GPU (cfd_latent_denorm)."""
        if data.dim() != 4 or data.shape[1] != 1:
            raise ValueError(f"Case4 latents must be (s, 1, t, l), got {tuple(data.shape)}")
        vmax, vmin = self._bounds()
        z = latent_denorm(data.detach().to(torch.float32).contiguous(), vmax, vmin)
        return z.reshape(-1, data.shape[-1])

    def forward(self, data, **kwargs):
        """(s, 1, t, l) latents in [-1, 1] -> (s*t, Ns, 3) measurements (one fused launch;
        pass_through_model_batch's row chunking does not change values)."""
        with torch.no_grad():
            return self.model.decode(self.coords, self._rows(data)[:, None], self.x_normalizer, self.y_normalizer)

    # -- adjoint used by the DPS sampler ----------------------------------------
    def forward_tape(self, data):
        return self.model.tape_forward(self.coords, self._rows(data), self.x_normalizer, self.y_normalizer)

    def vjp(self, g_out):
        """gradient w.r.t. the un-normalised latent rows of the last forward_tape."""
        return self.model.tape_vjp(g_out)


# =============
# Noise classes
# =============
__NOISE__ = {}


def register_noise(name: str):
    def wrapper(cls):
        if __NOISE__.get(name, None):
            raise NameError(f"Name {name} is already defined!")
        __NOISE__[name] = cls
        return cls
    return wrapper


def get_noise(name: str, **kwargs):
    """measurements.py:242-247."""
    if __NOISE__.get(name, None) is None:
        raise NameError(f"Name {name} is not defined.")
    noiser = __NOISE__[name](**kwargs)
    noiser.__name__ = name
    return noiser


class Noise(ABC):
    def __call__(self, data):
        return self.forward(data)

    @abstractmethod
    def forward(self, data):
        pass


@register_noise(name="clean")
class Clean(Noise):
    def forward(self, data):
        return data


@register_noise(name="gaussian")
class GaussianNoise(Noise):
    def __init__(self, sigma):
        self.sigma = sigma

    def forward(self, data):
        return data + torch.randn_like(data, device=data.device) * self.sigma


def _require_gpu(t):
    if t.device.type != "cuda":
        raise _lib.CfdError("the DPS path runs on the GPU only")
