"""Deterministic synthetic inputs for parity tests and benchmarks.

There are no pretrained checkpoints on this box (the reference's Zenodo
artefacts, README.md:81, are not fetchable), so every weight and input used by
the tests and by ``bench.py`` comes from this counter-based generator.  The
same (seed, tensor-name) pair yields the same float32 values on any machine,
which lets the GPU box regenerate full-size weights instead of shipping them.

Stream: ``splitmix64(fnv1a64(name) ^ (seed * GOLDEN) + i)`` for element ``i``;
the top 24 bits give a uniform in [0, 1).

Scaling rules (pinned in SURVEY.md section 8d / DESIGN.md):
  * U-Net conv / linear weights and biases: U(+-1/sqrt(fan_in)) (the default
    PyTorch init bound, U/src/nn.py:22-54), including the modules the
    reference zero-initialises (U/src/unet.py:210-212,294,615) so that the
    network output is not identically zero;
  * GroupNorm affine: weight U(0.75, 1.25), bias U(-0.1, 0.1);
  * SIREN: ``sine_init`` / ``first_layer_sine_init`` ranges
    (N/cnf/initialization.py:117-132); biases U(+-1/sqrt(fan_in)) (nn.Linear
    default, N/cnf/components.py:55).
"""
from __future__ import annotations

import math

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def _fnv1a64(s: str) -> int:
    h = 0xCBF29CE484222325
    for b in s.encode("utf-8"):
        h ^= b
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def uniform01(seed: int, name: str, n: int) -> np.ndarray:
    """n float64 values in [0, 1) from the (seed, name) stream."""
    base = np.uint64(_fnv1a64(name)) ^ np.uint64((seed * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF)
    with np.errstate(over="ignore"):
        idx = base + np.arange(n, dtype=np.uint64)
    z = _splitmix64(idx)
    return (z >> np.uint64(40)).astype(np.float64) * (1.0 / (1 << 24))


def uniform(seed: int, name: str, shape, lo: float, hi: float) -> np.ndarray:
    n = int(np.prod(shape)) if len(shape) else 1
    u = uniform01(seed, name, n)
    return (lo + (hi - lo) * u).astype(np.float32).reshape(shape)


def normal(seed: int, name: str, shape) -> np.ndarray:
    """Box-Muller normals (float32) from the (seed, name) stream."""
    n = int(np.prod(shape))
    m = (n + 1) // 2
    u = uniform01(seed, name, 2 * m)
    u1 = np.maximum(u[0::2], 1.0 / (1 << 25))
    u2 = u[1::2]
    r = np.sqrt(-2.0 * np.log(u1))
    z = np.concatenate([r * np.cos(2 * math.pi * u2), r * np.sin(2 * math.pi * u2)])
    return z[:n].astype(np.float32).reshape(shape)


def unet_param(seed: int, key: str, shape) -> np.ndarray:
    """Synthetic value for one U-Net state_dict entry (reference key names)."""
    shape = tuple(int(s) for s in shape)
    leaf = key.rsplit(".", 1)[-1]
    # GroupNorm parameters: 1-D weight/bias of a normalization layer.  In the
    # reference key space those are in_layers.0, out_layers.0, norm, out.0.
    is_norm = (
        key.endswith("in_layers.0." + leaf)
        or key.endswith("out_layers.0." + leaf)
        or key.endswith(".norm." + leaf)
        or key in ("out.0.weight", "out.0.bias")
    )
    if is_norm:
        if leaf == "weight":
            return uniform(seed, key, shape, 0.75, 1.25)
        return uniform(seed, key, shape, -0.1, 0.1)
    if len(shape) >= 2:
        fan_in = int(np.prod(shape[1:]))
        b = 1.0 / math.sqrt(fan_in)
        return uniform(seed, key, shape, -b, b)
    # bias: fan_in of the matching weight is unknown here; the caller passes
    # it through unet_state_dict, so this branch is only a fallback.
    return uniform(seed, key, shape, -0.05, 0.05)


def unet_state_dict(seed: int, shapes: dict) -> dict:
    """Fill every tensor of a U-Net state_dict (name -> shape) deterministically."""
    out = {}
    for key, shape in shapes.items():
        shape = tuple(int(s) for s in shape)
        leaf = key.rsplit(".", 1)[-1]
        if leaf == "bias" and len(shape) == 1:
            wkey = key[: -len("bias")] + "weight"
            wshape = shapes.get(wkey)
            if wshape is not None and len(wshape) >= 2:
                fan_in = int(np.prod(wshape[1:]))
                b = 1.0 / math.sqrt(fan_in)
                out[key] = uniform(seed, key, shape, -b, b)
                continue
        out[key] = unet_param(seed, key, shape)
    return out


def siren_state_dict(seed: int, in_coord: int, in_latent: int, out_features: int,
                     num_hidden_layers: int, hidden: int, w0: float = 30.0) -> dict:
    """State dict for SIRENAutodecoder_film (N/cnf/nf_networks.py:443-478)."""
    sd = {}
    dims = [in_coord] + [hidden] * (num_hidden_layers + 1) + [out_features]
    for i in range(num_hidden_layers + 2):
        fin, fout = dims[i], dims[i + 1]
        if i == 0:
            b = 1.0 / fin
        else:
            b = math.sqrt(6.0 / fin) / w0
        sd[f"net1.{i}.weight"] = uniform(seed, f"net1.{i}.weight", (fout, fin), -b, b)
        bb = 1.0 / math.sqrt(fin)
        sd[f"net1.{i}.bias"] = uniform(seed, f"net1.{i}.bias", (fout,), -bb, bb)
    for i in range(num_hidden_layers + 1):
        if i == 0:
            b = 1.0 / in_latent
        else:
            b = math.sqrt(6.0 / in_latent) / w0
        sd[f"net2.{i}.weight"] = uniform(seed, f"net2.{i}.weight", (hidden, in_latent), -b, b)
    return sd
