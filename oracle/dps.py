"""Oracle: one DPS (diffusion posterior sampling) step of the Case4 conditional
notebook, CPU fp32 with torch autograd.  Test-only (see oracle/__init__.py).

Restates, for the 'ddpm' sampler with EPSILON / FIXED_LARGE processors and the
'ps' conditioning method:
  * DDPM.p_sample (C/src/guided_diffusion/gaussian_diffusion.py:362-372) over
    p_mean_variance (:209-232), EpsilonXMeanProcessor (posterior_mean_variance.py:
    97-129: x0 = c1 x - c2 eps, clamp(-1, 1), mu = k1 x0 + k2 x) and
    FixedLargeVarianceProcessor (:180-199);
  * p_sample_loop's conditioning call (gaussian_diffusion.py:169-206);
  * PosteriorSampling.conditioning + grad_and_value (condition_methods.py:81-90,
    31-47): norm = ||y - A(x0_hat)||_2 over the whole tensor, x_t -= scale *
    d norm / d x_prev;
  * Case4Operator._unnorm / forward (measurements.py:219-226) over
    pass_through_model_batch (N/cnf/inference_function.py:22-48).
"""
from __future__ import annotations

import torch

from . import siren as osn
from .diffusion import Tables, _ex


def case4_forward(sd, coords, xmax, xmin, ymax, ymin, vmax, vmin, x0, batch=None):
    """Case4Operator.forward: (s, 1, t, l) latents in [-1, 1] -> (s*t, Ns, c)."""
    z = ((x0[:, 0] + 1) * (vmax - vmin) / 2 + vmin)[:, None]      # _unnorm
    z = z.reshape(-1, z.shape[-1])                                # "s c t l -> (s c t) l"
    return osn.decode(sd, coords, z, xmax, xmin, ymax, ymin, batch=batch)


def dps_step(tb: Tables, unet, operator, x, i, y, noise, scale):
    """One reverse step at respaced index i (same for the whole batch).

    unet(x, t_mapped) -> eps; operator(x0_hat) -> A(x0_hat).  Returns
    (img, x0_hat, sample, norm) as the reference's loop sees them."""
    x = x.detach().requires_grad_()
    t = torch.full((x.shape[0],), i, dtype=torch.int64)
    eps = unet(x, torch.from_numpy(tb.timestep_map)[t])
    x0 = (_ex(tb.sqrt_recip_alphas_cumprod, t) * x - _ex(tb.sqrt_recipm1_alphas_cumprod, t) * eps).clamp(-1, 1)
    mean = _ex(tb.posterior_mean_coef1, t) * x0 + _ex(tb.posterior_mean_coef2, t) * x
    sample = mean
    if i != 0:
        sample = sample + torch.exp(0.5 * _ex(tb.fixed_large_logvar, t)) * noise
    norm = torch.linalg.norm(y - operator(x0))
    grad = torch.autograd.grad(norm, x)[0]
    return (sample - grad * scale).detach(), x0.detach(), sample.detach(), norm.detach()


def dps_loop(tb: Tables, unet, operator, x_start, y, step_noise, scale):
    x = x_start
    traj = []
    for k, i in enumerate(reversed(range(tb.num_timesteps))):
        x, x0, sample, norm = dps_step(tb, unet, operator, x, i, y, step_noise[k], scale)
        traj.append((x, x0, sample, norm))
    return x, traj
