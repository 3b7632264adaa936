"""Oracle: the CNF autodecoder training loop, CPU fp32 with torch autograd.

Restates N/scripts/train.py:385-416 (``_single_trainer`` at world_size 1): per
epoch i, ``optim_net_dec.step(); zero_grad()`` when i != 0 (the network steps
once per epoch on the gradient accumulated over the previous epoch's batches),
then per batch ``latents(idx)`` -> model -> ``MSELoss`` -> ``optim_states``
zero_grad / backward / step (the latent table steps every batch, all of its
rows, as torch.optim.Adam does).  The model is ``oracle.siren.forward``
(nf_networks.py:480-495), the latent container LatentContainer.forward
(train.py:43-63, lumped).  Test-only (see oracle/__init__.py).
"""
from __future__ import annotations

import torch

from . import siren


def train(sd: dict, latents0: torch.Tensor, coords: torch.Tensor, fois: torch.Tensor, batches, epochs: int,
          lr_nf: float, lr_latents: float, record_first_grads: bool = True):
    """sd: state dict (fp32 CPU), latents0 (N_samples, L), coords (N, d) (the
    model's raw input), fois (N_samples, N, c), batches: list of index lists
    (one epoch's order, repeated).  Returns (sd, latents, losses, first) where
    first holds the gradients of the very first backward."""
    params = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    keys = list(sd)
    lat = latents0.clone().requires_grad_(True)
    opt_net = torch.optim.Adam([params[k] for k in keys], lr=lr_nf)
    opt_lat = torch.optim.Adam([lat], lr=lr_latents)
    crit = torch.nn.MSELoss()
    losses, first = [], None
    for i in range(epochs):
        if i != 0:
            opt_net.step()
            opt_net.zero_grad()
        for idx in batches:
            idx_t = torch.as_tensor(idx, dtype=torch.int64)
            bl = lat[idx_t][:, None]                                  # LatentContainer, lumped: (B, 1, L)
            bc = coords[None].expand(len(idx), *coords.shape)         # the DataLoader's stacked coords
            out = siren.forward(params, bc, bl)
            loss = crit(out, fois[idx_t])
            opt_lat.zero_grad()
            loss.backward()
            if record_first_grads and first is None:
                first = {"net": {k: params[k].grad.detach().clone() for k in keys},
                         "latents": lat.grad.detach().clone()}
            opt_lat.step()
            losses.append(float(loss))
    return ({k: params[k].detach().clone() for k in keys}, lat.detach().clone(), losses, first)
