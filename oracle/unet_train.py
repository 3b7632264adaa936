"""Oracle: the diffusion TrainLoop's step, CPU fp32 with torch autograd.

Restates U/src/train_util.py:178-226 at world size 1, fp32, one microbatch:
zero_grad -> GaussianDiffusion.training_losses (q_sample :188-206 with the
float64 tables cast per sample to fp32 as _extract_into_tensor :899-912, the
model's eps against the noise, mean_flat of the squared error :840-846) ->
``(loss * weights).mean().backward()`` -> torch.optim.AdamW.step()
(MixedPrecisionTrainer._optimize_normal, fp16_util.py:210-215) -> update_ema
(U/src/nn.py:71-80).  The model is ``oracle.unet.forward`` and the tables
``oracle.diffusion.Tables``.  Test-only (see oracle/__init__.py).
"""
from __future__ import annotations

import torch

from . import diffusion as od
from . import unet as ou


def train(sd: dict, cfg: ou.Config, x0: torch.Tensor, ts, noises, lr: float, weight_decay: float,
          ema_rate: float, schedule: str = "cosine", steps: int = 1000):
    """sd: state dict (fp32 CPU, in the module's parameter order); ts / noises:
    per step the (B,) timesteps and the (B, C, H, W) noise.  Returns (sd, ema,
    losses, first) with first the first backward's gradients."""
    tb = od.Tables(steps, schedule, "")
    sa = torch.from_numpy(tb.alphas_cumprod ** 0.5)
    sb = torch.from_numpy((1.0 - tb.alphas_cumprod) ** 0.5)
    keys = list(sd)
    params = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    opt = torch.optim.AdamW([params[k] for k in keys], lr=lr, weight_decay=weight_decay)
    ema = {k: v.detach().clone() for k, v in sd.items()}
    losses, first = [], None
    for t, noise in zip(ts, noises):
        t = torch.as_tensor(t, dtype=torch.int64)
        opt.zero_grad()
        shp = (-1,) + (1,) * (x0.dim() - 1)
        x_t = sa[t].float().reshape(shp) * x0 + sb[t].float().reshape(shp) * noise
        eps = ou.forward(params, cfg, x_t, t)
        mse = ((noise - eps) ** 2).mean(dim=list(range(1, eps.dim())))
        loss = (mse * torch.ones(len(t))).mean()
        loss.backward()
        if first is None:
            first = {k: params[k].grad.detach().clone() for k in keys}
        opt.step()
        with torch.no_grad():
            for k in keys:
                ema[k].mul_(ema_rate).add_(params[k], alpha=1 - ema_rate)
        losses.append(float(loss.detach()))
    return {k: params[k].detach().clone() for k in keys}, ema, losses, first
