"""Decode helpers with the reference signatures (N/cnf/inference_function.py:15-76)."""
from __future__ import annotations

import numpy as np
import torch

from .nf_networks import SIRENAutodecoder_film


def ReconstructFrame(data, mask, shape, fill_value=np.nan):
    """inference_function.py:15-19: scatter masked points back into the full grid (host)."""
    temp = np.empty((*shape, data.shape[-1]))
    temp[:] = fill_value
    temp[mask] = data
    return temp


def _decode(coords, latents, model, x_normalizer, y_normalizer, batch_size, device):
    if not isinstance(model, SIRENAutodecoder_film):
        raise TypeError("model must be confild_amd.nf_networks.SIRENAutodecoder_film (the fused HIP decoder)")
    t_size, latent_size = latents.shape
    device = torch.device(device) if device is not None else latents.device
    lat = latents.to(device)
    outs = []
    # the fused kernel processes every latent of a chunk in one launch; batch_size
    # bounds the (chunk, N, c) output kept live per launch, as in the reference loop
    step = t_size if batch_size is None else max(int(batch_size), 1)
    for s in range(0, t_size, step):
        outs.append(model.decode(coords.reshape(-1, coords.shape[-1]).to(device), lat[s:s + step].reshape(-1, 1,
                                 latent_size), x_normalizer, y_normalizer))
    return outs


def pass_through_model_batch(coords, latents, model, x_normalizer, y_normalizer, batch_size, device):
    """inference_function.py:22-48 -> (t, N, c) on `device`."""
    return torch.cat(_decode(coords, latents, model, x_normalizer, y_normalizer, batch_size, device), dim=0)


def decoder(coords, latents, model, x_normalizer, y_normalizer, batch_size, device):
    """inference_function.py:51-76 -> (t, N, c) on the host."""
    with torch.no_grad():
        outs = _decode(coords, latents, model, x_normalizer, y_normalizer, batch_size, device)
        return torch.cat([o.cpu() for o in outs], dim=0)
