"""Oracle: SIRENAutodecoder_film forward and Normalizer_ts ('-11'), CPU fp32.

Restates N/cnf/nf_networks.py:480-495, N/cnf/components.py:19-25,55-76 and
N/cnf/utils/normalize.py:100-114.  Test-only (see oracle/__init__.py).
"""
from __future__ import annotations

import torch

W0 = 30.0  # N/cnf/initialization.py:5 DEFAULT_W0


def normalize(x, xmax, xmin):
    return (x - xmin) / (xmax - xmin) * 2 - 1


def denormalize(y, ymax, ymin):
    return (y + 1) / 2 * (ymax - ymin) + ymin


def batch_linear(x, w, b=None):
    # BatchLinear.forward: matmul with W^T, then += bias (components.py:64-76)
    out = torch.matmul(x, w.transpose(-1, -2))
    if b is not None:
        out = out + b.unsqueeze(-2)
    return out


def forward(sd: dict, coords: torch.Tensor, latents: torch.Tensor) -> torch.Tensor:
    """coords (..., N, d), latents (b, 1, L) -> (b, N, c)."""
    n_layers = sum(1 for k in sd if k.startswith("net1.") and k.endswith(".weight"))
    x = coords
    for i in range(n_layers - 1):
        x = batch_linear(x, sd[f"net1.{i}.weight"], sd[f"net1.{i}.bias"]) + batch_linear(
            latents, sd[f"net2.{i}.weight"])
        x = torch.sin(W0 * x)
    return batch_linear(x, sd[f"net1.{n_layers - 1}.weight"], sd[f"net1.{n_layers - 1}.bias"])


def decode(sd, coords, latents, xmax, xmin, ymax, ymin, batch=None):
    """trainer.infer / pass_through_model_batch: normalise -> NF -> denormalise
    (N/scripts/train.py:265-279, N/cnf/inference_function.py:22-48)."""
    b = latents.shape[0]
    batch = batch or b
    outs = []
    cn = normalize(coords, xmax, xmin)[None]
    for s in range(0, b, batch):
        raw = forward(sd, cn, latents[s:s + batch, None])
        outs.append(denormalize(raw, ymax, ymin))
    return torch.cat(outs, 0)
