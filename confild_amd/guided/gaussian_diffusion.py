"""Guided samplers (C/src/guided_diffusion/gaussian_diffusion.py): create_sampler,
DDPM / DDIM with the conditional p_sample_loop of the Case4 notebook.

One reverse step of the 'ps' (DPS) loop, reference (gaussian_diffusion.py:
169-206, 362-372; condition_methods.py:31-47,81-90):

    out = p_sample(x)                      # eps = U(x, t); x0 = clamp(c1 x - c2 eps); sample
    norm = ||y - A(x0)||                   # A = Case4Operator.forward
    x = out.sample - scale * d norm / d x  # torch autograd through A, clamp, U

Here, with the same arithmetic per link:

    eps     = cfd_unet_forward_tape(x)                   (activations kept)
    sample  = cfd_sched_step(x, eps)                      (bit-exact DDPM/DDIM step)
    A       = cfd_siren_tape_forward(unnorm(x0))          (sensor points only)
    g_A     = cfd_dps_residual(y, A)                      (-(y - A) / ||y - A||)
    g_z     = cfd_siren_tape_vjp(g_A)
    d_eps, g_direct = cfd_dps_latent_grad(g_z)            (unnorm, clamp', c1 / c2 links)
    g_unet  = cfd_unet_input_vjp(d_eps)
    x       = cfd_dps_update(sample, g_direct, g_unet, scale)

Batches: the reference loop only runs one sample per call (its ``if t != 0``
needs a one-element t; the notebook loops over samples).  Here a batch of B
samples is B independent DPS chains -- one residual norm per sample -- so a
batched call equals B single-sample calls, and samples shard over GPUs with no
collective.  The measurement is shared by all samples ((T, Ns, c)) or given
per sample ((B*T, Ns, c)).

RNG: as the unconditional sampler, Philox(seed, counter=step) by default, or the
reference's draws through ``step_noise`` (the p_sample ``randn_like`` of every
step; the unused q_sample draw of the noisy measurement is not needed).
"""
from __future__ import annotations

import functools

import torch

from .. import _lib
from ..gaussian_diffusion import (LossType, ModelMeanType, ModelVarType, STEP_DDIM, STEP_DDPM, check_model_range,
                                  fresh_seed, get_named_beta_schedule)
from ..respace import SpacedDiffusion, space_timesteps
from .condition_methods import Identity, PosteriorSampling

__SAMPLER__ = {}


def register_sampler(name: str):
    def wrapper(cls):
        if __SAMPLER__.get(name, None):
            raise NameError(f"Name {name} is already registered!")
        __SAMPLER__[name] = cls
        return cls
    return wrapper


def get_sampler(name: str):
    if __SAMPLER__.get(name, None) is None:
        raise NameError(f"Name {name} is not defined!")
    return __SAMPLER__[name]


_MEAN = {"epsilon": ModelMeanType.EPSILON}
_VAR = {"fixed_large": ModelVarType.FIXED_LARGE, "fixed_small": ModelVarType.FIXED_SMALL}


def create_sampler(sampler, steps, noise_schedule, model_mean_type, model_var_type, dynamic_threshold, clip_denoised,
                   rescale_timesteps, timestep_respacing=""):
    """gaussian_diffusion.py:30-52."""
    cls = get_sampler(name=sampler)
    if model_mean_type not in _MEAN:
        raise NotImplementedError(f"model_mean_type {model_mean_type!r} on the HIP path (CoNFiLD uses 'epsilon')")
    if model_var_type not in _VAR:
        raise NotImplementedError(f"model_var_type {model_var_type!r} on the HIP path")
    if dynamic_threshold:
        raise NotImplementedError("dynamic_threshold on the HIP path")
    if rescale_timesteps:
        raise NotImplementedError("rescale_timesteps=True on the HIP path")
    betas = get_named_beta_schedule(noise_schedule, steps)
    if not timestep_respacing:
        timestep_respacing = [steps]
    return cls(use_timesteps=space_timesteps(steps, timestep_respacing), betas=betas,
               model_mean_type=_MEAN[model_mean_type], model_var_type=_VAR[model_var_type],
               loss_type=LossType.MSE, rescale_timesteps=False, clip_denoised=clip_denoised)


def _method_of(measurement_cond_fn):
    fn = measurement_cond_fn
    while isinstance(fn, functools.partial):
        fn = fn.func
    owner = getattr(fn, "__self__", None)
    if isinstance(owner, (PosteriorSampling, Identity)):
        return owner
    raise NotImplementedError("measurement_cond_fn must be partial(cond_method.conditioning) of a 'ps' or "
                              "'vanilla' method from confild_amd.guided.condition_methods")


class _GuidedSampler(SpacedDiffusion):
    _kind = STEP_DDPM

    def __init__(self, use_timesteps, clip_denoised=True, **kwargs):
        super().__init__(use_timesteps, **kwargs)
        self.clip_denoised = clip_denoised
        self.distances = None   # (steps, B) residual norms of the last p_sample_loop (GPU)

    def p_sample_loop(self, model, x_start, measurement, measurement_cond_fn, record=False, save_root=None, *,
                      step_noise=None, seed=None, sample_offset=0, progress=False):
        """gaussian_diffusion.py:169-206: guided reverse loop from x_start (B, 1, T, L).
        Per-step residual norms (the reference's progress-bar 'distance') are left in
        ``self.distances`` (steps, B) on the GPU."""
        if record:
            raise NotImplementedError("record=True (progress images) is not part of the HIP path")
        method = _method_of(measurement_cond_fn)
        if x_start.device.type != "cuda":
            raise _lib.CfdError("the DPS sampler runs on the GPU only (no CPU fallback)")
        if seed is None:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        x = x_start.detach().to(torch.float32).contiguous().clone()
        self.distances = torch.zeros(self.num_timesteps, x.shape[0], dtype=torch.float32, device=x.device)
        indices = list(range(self.num_timesteps))[::-1]
        if progress:
            from tqdm.auto import tqdm
            indices = tqdm(indices)
        for k, i in enumerate(indices):
            nz = None if step_noise is None else step_noise[k]
            x = self._guided_step(model, x, i, measurement, method, nz, seed, k, sample_offset, self.distances[k])[0]
        check_model_range(model, x.device)
        return x

    def p_sample_step(self, model, x, index, measurement, measurement_cond_fn, noise=None, seed=None, counter=0,
                      sample_offset=0):
        """One guided reverse step at respaced index ``index`` (p_sample + conditioning,
        gaussian_diffusion.py:188-199).  Returns dict(sample, pred_xstart, x_t, distance):
        the conditioned image, x0_hat, the unconditioned DDPM/DDIM sample, the norms.
        Without ``noise`` and ``seed`` the step draws a fresh Philox key (fresh_seed)."""
        method = _method_of(measurement_cond_fn)
        seed = fresh_seed(noise, seed)
        x = x.detach().to(torch.float32).contiguous().clone()
        dist = torch.zeros(x.shape[0], dtype=torch.float32, device=x.device)
        img, x0, sample = self._guided_step(model, x, index, measurement, method, noise, seed, counter,
                                            sample_offset, dist)
        return {"sample": img, "pred_xstart": x0, "x_t": sample, "distance": dist}

    def _guided_step(self, model, x, i, measurement, method, noise, seed, counter, sample_offset, dist_out):
        """x (B, 1, T, L) contiguous fp32 on the GPU; updated in place for 'ps'."""
        dev = x.device
        if dev.type != "cuda":
            raise _lib.CfdError("the DPS sampler runs on the GPU only (no CPU fallback)")
        lib = _lib.lib()
        st = _lib.stream_of(dev)
        B = x.shape[0]
        n = x[0].numel()
        offset = sample_offset * n
        if offset % 4:
            raise ValueError("sharded sampling needs (elements per sample * first sample) % 4 == 0")
        sched = self._sched(dev, 0.0)
        t = torch.full((B,), i, dtype=torch.int64, device=dev)
        tm = self._map_timesteps(t)
        nz = None if noise is None else noise.to(device=dev, dtype=torch.float32).contiguous()
        dps = isinstance(method, PosteriorSampling)
        clip = 1 if self.clip_denoised else 0
        eps = (model.forward_tape(x, tm) if dps else model(x, tm)).contiguous()
        sample = torch.empty_like(x)
        x0 = torch.empty_like(x)
        _lib.check(lib.cfd_sched_step(sched.handle, self._kind, clip, _lib.ptr(x), _lib.ptr(eps), _lib.ptr(t),
                                      _lib.ptr(nz), seed, counter, offset, _lib.ptr(sample), _lib.ptr(x0), n, B, st),
                   "cfd_sched_step")
        if not dps:
            return sample, x0, sample
        op = method.operator
        y = measurement.to(device=dev, dtype=torch.float32).contiguous()
        vmax, vmin = op._bounds()
        if n % vmax.numel():
            raise ValueError("latent max/min do not tile the latent")
        A = op.forward_tape(x0)                                      # (B*T, Ns, c)
        per = A.numel() // B
        if y.numel() not in (per, A.numel()):
            raise ValueError(f"measurement of {y.numel()} values matches neither one sample ({per}) "
                             f"nor the batch ({A.numel()})")
        gA = torch.empty_like(A)
        _lib.check(lib.cfd_dps_residual(_lib.ptr(y), 0 if y.numel() == per else per, _lib.ptr(A), _lib.ptr(gA),
                                        _lib.ptr(dist_out), per, B, st), "cfd_dps_residual")
        gz = op.vjp(gA)                                              # (B*T, L)
        d_eps = torch.empty_like(x)
        g_dir = torch.empty_like(x)
        _lib.check(lib.cfd_dps_latent_grad(sched.handle, clip, _lib.ptr(x), _lib.ptr(eps), _lib.ptr(t), _lib.ptr(gz),
                                           _lib.ptr(vmax), _lib.ptr(vmin), vmax.numel(), _lib.ptr(d_eps),
                                           _lib.ptr(g_dir), n, B, st), "cfd_dps_latent_grad")
        g_unet = model.input_vjp(d_eps)
        img = torch.empty_like(x)
        _lib.check(lib.cfd_dps_update(_lib.ptr(sample), _lib.ptr(g_dir), _lib.ptr(g_unet), float(method.scale),
                                      _lib.ptr(img), x.numel(), st), "cfd_dps_update")
        return img, x0, sample


@register_sampler(name="ddpm")
class DDPM(_GuidedSampler):
    _kind = STEP_DDPM


@register_sampler(name="ddim")
class DDIM(_GuidedSampler):
    """DDIM.p_sample with eta = 0 (gaussian_diffusion.py:375-403)."""
    _kind = STEP_DDIM
