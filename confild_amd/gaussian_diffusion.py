"""Diffusion schedules and the GPU reverse loop (drop-in for U/src/gaussian_diffusion.py).

Host side: the float64 coefficient tables exactly as the reference builds them
(:18-62, :118-169), cast per timestep to fp32 with the same torch ops as
``_extract_into_tensor`` (:899-912) and uploaded once.  Device side: each
reverse step is one U-Net forward (cfd_unet_forward) plus one fused epilogue
launch (cfd_sched_step: x0 prediction, clamp, posterior mean, noise).

RNG: by default the per-step normals come from the in-kernel Philox stream keyed
by a seed drawn from torch's default CPU generator at loop start (so
``torch.manual_seed`` makes runs reproducible).  For parity with a reference run,
pass ``noise=`` (x_T) and ``step_noise=`` (one tensor per step, in the
reference's draw order: gaussian_diffusion.py:430/576).
"""
from __future__ import annotations

import ctypes as C
import enum
import math
import os

import numpy as np
import torch

from . import _lib


def get_named_beta_schedule(schedule_name, num_diffusion_timesteps):
    """gaussian_diffusion.py:18-40."""
    if schedule_name == "linear":
        scale = 1000 / num_diffusion_timesteps
        return np.linspace(scale * 0.0001, scale * 0.02, num_diffusion_timesteps, dtype=np.float64)
    if schedule_name == "cosine":
        return betas_for_alpha_bar(num_diffusion_timesteps,
                                   lambda t: math.cos((t + 0.008) / 1.008 * math.pi / 2) ** 2)
    raise NotImplementedError(f"unknown beta schedule: {schedule_name}")


def betas_for_alpha_bar(num_diffusion_timesteps, alpha_bar, max_beta=0.999):
    """gaussian_diffusion.py:43-62."""
    out = []
    for i in range(num_diffusion_timesteps):
        t1, t2 = i / num_diffusion_timesteps, (i + 1) / num_diffusion_timesteps
        out.append(min(1 - alpha_bar(t2) / alpha_bar(t1), max_beta))
    return np.array(out)


class ModelMeanType(enum.Enum):
    PREVIOUS_X = enum.auto()
    START_X = enum.auto()
    EPSILON = enum.auto()


class ModelVarType(enum.Enum):
    LEARNED = enum.auto()
    FIXED_SMALL = enum.auto()
    FIXED_LARGE = enum.auto()
    LEARNED_RANGE = enum.auto()


class LossType(enum.Enum):
    MSE = enum.auto()
    RESCALED_MSE = enum.auto()
    KL = enum.auto()
    RESCALED_KL = enum.auto()

    def is_vb(self):
        return self in (LossType.KL, LossType.RESCALED_KL)


# row layout of the fp32 coefficient table (include/confild.h CFD_COEF_*)
SRA, SRM1, M1, M2, SIGMA, SQRT_ABP, DIR, SIGMA_DDIM = range(8)
STEP_DDPM, STEP_DDIM = 0, 1


def check_model_range(model, device):
    """The split-f16 range guard of a HIP U-Net (UNetModel.check_finite), if the
    model has one; any other callable passes."""
    fn = getattr(model, "check_finite", None)
    if callable(fn):
        fn(device)


def fresh_seed(noise, seed):
    """The Philox key of a single step: the caller's, or (no explicit noise and no
    seed) a fresh draw from torch's default generator, so independent calls never
    share their normals."""
    if seed is None:
        return 0 if noise is not None else int(torch.randint(0, 2 ** 62, (1,)).item())
    return int(seed)


class _Sched:
    """Device copy of one fp32 coefficient table (owns a cfd_sched handle)."""

    def __init__(self, coefs: torch.Tensor, device: int):
        lib = _lib.lib()
        self.handle = C.c_void_p()
        host = coefs.contiguous()
        _lib.check(lib.cfd_sched_create(C.c_void_p(host.data_ptr()), host.shape[0], device, C.byref(self.handle)),
                   "cfd_sched_create")

    def __del__(self):
        try:
            _lib.load().cfd_sched_destroy(self.handle)
        except Exception:
            pass


class _NativeLoop:
    """One cfd_sampler handle: the whole reverse loop on the device, one captured
    HIP graph per `unroll` steps (csrc/sampler.hip).  Keeps the U-Net handle's
    owner and the coefficient table alive for its lifetime."""

    def __init__(self, model, sched, handle, kind, clip, B, n_per_sample, tidx, tmodel, graph, unroll):
        lib = _lib.lib()
        self.model, self.sched = model, sched
        ti = np.ascontiguousarray(tidx, dtype=np.int64)
        tm = np.ascontiguousarray(tmodel, dtype=np.int64)
        self.handle = C.c_void_p()
        _lib.check(lib.cfd_sampler_create(handle, sched.handle, kind, 1 if clip else 0, B, n_per_sample, len(ti),
                                          ti.ctypes.data_as(C.c_void_p), tm.ctypes.data_as(C.c_void_p),
                                          1 if graph else 0, unroll, C.byref(self.handle)), "cfd_sampler_create")

    def run(self, x_in, x_out, k0, k1, seed, offset, device):
        _lib.check(_lib.load().cfd_sampler_run(self.handle, _lib.ptr(x_in), _lib.ptr(x_out), k0, k1, seed, offset,
                                               _lib.stream_of(device)), "cfd_sampler_run")

    def __del__(self):
        try:
            _lib.load().cfd_sampler_destroy(self.handle)
        except Exception:
            pass


# Native loop mode (CFD_SAMPLER): 2 = captured HIP graph (default), 1 = native
# host loop without a graph, 0 = the Python per-step loop
NATIVE_MODE = int(os.environ.get("CFD_SAMPLER", "2"))
GRAPH_UNROLL = int(os.environ.get("CFD_SAMPLER_UNROLL", "4"))
# the split-f16 range guard is read every RANGE_CHECK_EVERY steps (one stream sync each)
RANGE_CHECK_EVERY = 64


class GaussianDiffusion:
    """Same constructor and sampling API as the reference GaussianDiffusion (:88-169)."""

    def __init__(self, *, betas, model_mean_type, model_var_type, loss_type, rescale_timesteps=False):
        self.model_mean_type = model_mean_type
        self.model_var_type = model_var_type
        self.loss_type = loss_type
        self.rescale_timesteps = rescale_timesteps
        betas = np.array(betas, dtype=np.float64)
        self.betas = betas
        assert len(betas.shape) == 1, "betas must be 1-D"
        assert (betas > 0).all() and (betas <= 1).all()
        self.num_timesteps = int(betas.shape[0])
        alphas = 1.0 - betas
        self.alphas_cumprod = np.cumprod(alphas, axis=0)
        self.alphas_cumprod_prev = np.append(1.0, self.alphas_cumprod[:-1])
        self.alphas_cumprod_next = np.append(self.alphas_cumprod[1:], 0.0)
        self.sqrt_alphas_cumprod = np.sqrt(self.alphas_cumprod)
        self.sqrt_one_minus_alphas_cumprod = np.sqrt(1.0 - self.alphas_cumprod)
        self.log_one_minus_alphas_cumprod = np.log(1.0 - self.alphas_cumprod)
        self.sqrt_recip_alphas_cumprod = np.sqrt(1.0 / self.alphas_cumprod)
        self.sqrt_recipm1_alphas_cumprod = np.sqrt(1.0 / self.alphas_cumprod - 1)
        self.posterior_variance = betas * (1.0 - self.alphas_cumprod_prev) / (1.0 - self.alphas_cumprod)
        self.posterior_log_variance_clipped = np.log(
            np.append(self.posterior_variance[1], self.posterior_variance[1:]))
        self.posterior_mean_coef1 = betas * np.sqrt(self.alphas_cumprod_prev) / (1.0 - self.alphas_cumprod)
        self.posterior_mean_coef2 = (1.0 - self.alphas_cumprod_prev) * np.sqrt(alphas) / (1.0 - self.alphas_cumprod)
        self._scheds = {}
        self._natives = {}

    def _model_timesteps_host(self, indices):
        """Model timesteps of table indices (identity; SpacedDiffusion: timestep_map)."""
        return list(indices)

    # -- model wrapping (identity here; SpacedDiffusion remaps) -------------------
    def _map_timesteps(self, t):
        if self.rescale_timesteps:
            raise NotImplementedError("rescale_timesteps=True")
        return t

    # -- coefficient table ----------------------------------------------------
    def _logvar_table(self):
        if self.model_var_type == ModelVarType.FIXED_LARGE:
            return np.log(np.append(self.posterior_variance[1], self.betas[1:]))   # :278-284
        if self.model_var_type == ModelVarType.FIXED_SMALL:
            return self.posterior_log_variance_clipped
        raise NotImplementedError(f"model_var_type {self.model_var_type} (learned variance) on the HIP path")

    def coef_table(self, eta: float = 0.0) -> torch.Tensor:
        """(num_timesteps, 8) fp32: the per-timestep scalars the reference extracts with
        ``th.from_numpy(arr)[t].float()`` and combines with fp32 torch ops."""
        f = lambda a: torch.from_numpy(np.asarray(a, dtype=np.float64)).float()  # noqa: E731
        n = self.num_timesteps
        tab = torch.zeros(n, 8, dtype=torch.float32)
        tab[:, SRA] = f(self.sqrt_recip_alphas_cumprod)
        tab[:, SRM1] = f(self.sqrt_recipm1_alphas_cumprod)
        tab[:, M1] = f(self.posterior_mean_coef1)
        tab[:, M2] = f(self.posterior_mean_coef2)
        tab[:, SIGMA] = torch.exp(0.5 * f(self._logvar_table()))                      # :431-438
        ab, abp = f(self.alphas_cumprod), f(self.alphas_cumprod_prev)
        sigma = eta * torch.sqrt((1 - abp) / (1 - ab)) * torch.sqrt(1 - ab / abp)     # :559-563
        tab[:, SQRT_ABP] = torch.sqrt(abp)
        tab[:, DIR] = torch.sqrt(1 - abp - sigma ** 2)
        tab[:, SIGMA_DDIM] = sigma
        return tab

    def _sched(self, device: torch.device, eta: float):
        dev = device.index if device.index is not None else torch.cuda.current_device()
        key = (dev, float(eta))
        s = self._scheds.get(key)
        if s is None:
            s = _Sched(self.coef_table(eta), dev)
            self._scheds[key] = s
        return s

    # -- single steps (public API of the reference) ----------------------------
    def _check_mean_type(self):
        if self.model_mean_type != ModelMeanType.EPSILON:
            raise NotImplementedError(f"model_mean_type {self.model_mean_type} on the HIP path (CoNFiLD uses EPSILON)")

    def _step(self, kind, model, x, t, clip_denoised, denoised_fn, cond_fn, model_kwargs, noise, seed, counter, eta,
              offset=0):
        self._check_mean_type()
        if denoised_fn is not None or cond_fn is not None:
            raise NotImplementedError("denoised_fn / cond_fn (use the DPS sampler for conditioning)")
        if x.device.type != "cuda":
            raise _lib.CfdError("the HIP sampler needs GPU tensors (no CPU fallback)")
        model_kwargs = model_kwargs or {}
        x = x.contiguous()
        eps = model(x, self._map_timesteps(t), **model_kwargs)
        if eps.shape != x.shape:
            raise NotImplementedError("learned-variance model outputs (2C channels) on the HIP path")
        eps = eps.to(torch.float32).contiguous()
        out = torch.empty_like(x)
        xs = torch.empty_like(x)
        nz = None
        if noise is not None:
            nz = noise.to(device=x.device, dtype=torch.float32).contiguous()
        sched = self._sched(x.device, eta)
        n = x[0].numel()
        _lib.check(_lib.load().cfd_sched_step(sched.handle, kind, 1 if clip_denoised else 0, _lib.ptr(x),
                                              _lib.ptr(eps), _lib.ptr(t), _lib.ptr(nz), seed, counter, offset,
                                              _lib.ptr(out), _lib.ptr(xs), n, x.shape[0],
                                              _lib.stream_of(x.device)), "cfd_sched_step")
        return {"sample": out, "pred_xstart": xs}

    def p_sample(self, model, x, t, clip_denoised=True, denoised_fn=None, cond_fn=None, model_kwargs=None,
                 noise=None, seed=None, counter=0):
        """gaussian_diffusion.py:395-439 (noise: explicit normals, else Philox(seed, counter);
        with neither, a fresh seed per call from torch's generator, like the
        reference's fresh ``randn_like`` at :430)."""
        seed = fresh_seed(noise, seed)
        t = t.to(device=x.device, dtype=torch.int64).contiguous()
        with torch.no_grad():
            return self._step(STEP_DDPM, model, x, t, clip_denoised, denoised_fn, cond_fn, model_kwargs, noise,
                              seed, counter, 0.0)

    def ddim_sample(self, model, x, t, clip_denoised=True, denoised_fn=None, cond_fn=None, model_kwargs=None,
                    eta=0.0, noise=None, seed=None, counter=0):
        """gaussian_diffusion.py:537-585 (noise / seed as p_sample)."""
        seed = fresh_seed(noise, seed)
        t = t.to(device=x.device, dtype=torch.int64).contiguous()
        with torch.no_grad():
            return self._step(STEP_DDIM, model, x, t, clip_denoised, denoised_fn, cond_fn, model_kwargs, noise,
                              seed, counter, eta)

    # -- loops ------------------------------------------------------------------
    def _loop(self, kind, model, shape, noise, clip_denoised, denoised_fn, cond_fn, model_kwargs, device,
              progress, eta, step_noise, seed, sample_offset=0):
        if device is None:
            try:
                device = next(model.parameters()).device
            except (AttributeError, StopIteration):
                device = torch.device("cuda", torch.cuda.current_device())
        device = torch.device(device)
        if device.type != "cuda":
            raise _lib.CfdError("the HIP sampler runs on the GPU only; move the model to a HIP device")
        assert isinstance(shape, (tuple, list))
        lib = _lib.lib()
        if seed is None:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        per_sample = int(np.prod(shape[1:]))
        offset = sample_offset * per_sample   # Philox position of this shard's first element
        if offset % 4:
            raise ValueError("sharded sampling needs (elements per sample * first sample) % 4 == 0")
        if noise is not None:
            img = noise.to(device=device, dtype=torch.float32).contiguous()
        else:
            img = torch.empty(*shape, dtype=torch.float32, device=device)
            _lib.check(lib.cfd_randn(_lib.ptr(img), img.numel(), seed, 1 << 40, offset, _lib.stream_of(device)),
                       "cfd_randn")
        indices = list(range(self.num_timesteps))[::-1]
        if progress:
            from tqdm.auto import tqdm
            indices = tqdm(indices)
        B = shape[0]
        ts = torch.arange(self.num_timesteps, dtype=torch.int64, device=device)
        self._clear_range_flag(model, device)
        for k, i in enumerate(indices):
            t = ts[i:i + 1].expand(B).contiguous()
            nz = None if step_noise is None else step_noise[k]
            with torch.no_grad():
                out = self._step(kind, model, img, t, clip_denoised, denoised_fn, cond_fn, model_kwargs, nz,
                                 seed, k, eta, offset)
            if (k + 1) % RANGE_CHECK_EVERY == 0 or k == len(indices) - 1:
                check_model_range(model, device)   # every RANGE_CHECK_EVERY steps: one stream sync
            yield out
            img = out["sample"]

    @staticmethod
    def _clear_range_flag(model, device):
        """Drop a range-guard flag an earlier call left set, so a loop reports only its own steps."""
        fn = getattr(model, "clear_range_flag", None)
        if callable(fn):
            fn(device)

    def _native_ok(self, model, denoised_fn, cond_fn, model_kwargs, step_noise, progress):
        from .unet import UNetModel
        return (NATIVE_MODE > 0 and isinstance(model, UNetModel) and denoised_fn is None and cond_fn is None
                and not model_kwargs and step_noise is None and not progress and not self.rescale_timesteps)

    def _native_loop(self, kind, model, shape, noise, clip_denoised, device, eta, seed, sample_offset):
        """The whole reverse loop on the device (csrc/sampler.hip): bit-identical to
        _loop with Philox noise, without per-step host work."""
        self._check_mean_type()
        if device is None:
            device = next(model.parameters()).device
        device = torch.device(device)
        if device.type != "cuda":
            raise _lib.CfdError("the HIP sampler runs on the GPU only; move the model to a HIP device")
        lib = _lib.lib()
        if seed is None:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        B = shape[0]
        per_sample = int(np.prod(shape[1:]))
        offset = sample_offset * per_sample
        if offset % 4:
            raise ValueError("sharded sampling needs (elements per sample * first sample) % 4 == 0")
        if tuple(shape[1:]) != (model.in_channels, model.image_size, model.image_size):
            raise ValueError(f"shape {tuple(shape)} does not match the model's input")
        if noise is not None:
            img = noise.to(device=device, dtype=torch.float32).contiguous()
        else:
            img = torch.empty(*shape, dtype=torch.float32, device=device)
            _lib.check(lib.cfd_randn(_lib.ptr(img), img.numel(), seed, 1 << 40, offset, _lib.stream_of(device)),
                       "cfd_randn")
        h = model._handle(device)   # uploads changed parameters, sets the compute mode
        sched = self._sched(device, eta)
        dev = device.index if device.index is not None else torch.cuda.current_device()
        key = (id(model), dev, kind, bool(clip_denoised), float(eta), B, NATIVE_MODE, GRAPH_UNROLL)
        nl = self._natives.get(key)
        if nl is None or nl.model is not model:
            tidx = list(range(self.num_timesteps))[::-1]
            with torch.cuda.device(dev):
                nl = _NativeLoop(model, sched, h, kind, clip_denoised, B, per_sample, tidx,
                                 self._model_timesteps_host(tidx), NATIVE_MODE >= 2, GRAPH_UNROLL)
            # one loop per (model, device): a new batch size / mode replaces the old one and its buffers
            self._natives = {k: v for k, v in self._natives.items() if k[:2] != key[:2]}
            self._natives[key] = nl
        out = torch.empty_like(img)
        self._clear_range_flag(model, device)
        n = self.num_timesteps
        for k0 in range(0, n, RANGE_CHECK_EVERY):
            k1 = min(n, k0 + RANGE_CHECK_EVERY)
            nl.run(img if k0 == 0 else None, out if k1 == n else None, k0, k1, seed, offset, device)
            check_model_range(model, device)
        return out

    def p_sample_loop(self, model, shape, noise=None, clip_denoised=True, denoised_fn=None, cond_fn=None,
                      model_kwargs=None, device=None, progress=False, step_noise=None, seed=None, sample_offset=0):
        """gaussian_diffusion.py:441-485.  ``sample_offset``: index of this call's first
        sample in a larger (sharded) batch, so the Philox noise equals the unsharded run's.
        With Philox noise and a HIP UNetModel the loop runs natively (one HIP graph
        per step, csrc/sampler.hip); explicit step_noise / progress use the Python loop."""
        if self._native_ok(model, denoised_fn, cond_fn, model_kwargs, step_noise, progress):
            return self._native_loop(STEP_DDPM, model, shape, noise, clip_denoised, device, 0.0, seed, sample_offset)
        final = None
        for s in self.p_sample_loop_progressive(model, shape, noise, clip_denoised, denoised_fn, cond_fn,
                                                model_kwargs, device, progress, step_noise, seed, sample_offset):
            final = s
        return final["sample"]

    def p_sample_loop_progressive(self, model, shape, noise=None, clip_denoised=True, denoised_fn=None,
                                  cond_fn=None, model_kwargs=None, device=None, progress=False, step_noise=None,
                                  seed=None, sample_offset=0):
        """gaussian_diffusion.py:487-535."""
        yield from self._loop(STEP_DDPM, model, shape, noise, clip_denoised, denoised_fn, cond_fn, model_kwargs,
                              device, progress, 0.0, step_noise, seed, sample_offset)

    def ddim_sample_loop(self, model, shape, noise=None, clip_denoised=True, denoised_fn=None, cond_fn=None,
                         model_kwargs=None, device=None, progress=False, eta=0.0, step_noise=None, seed=None,
                         sample_offset=0):
        """gaussian_diffusion.py:625-662 (native loop as p_sample_loop)."""
        if self._native_ok(model, denoised_fn, cond_fn, model_kwargs, step_noise, progress):
            return self._native_loop(STEP_DDIM, model, shape, noise, clip_denoised, device, eta, seed, sample_offset)
        final = None
        for s in self.ddim_sample_loop_progressive(model, shape, noise, clip_denoised, denoised_fn, cond_fn,
                                                   model_kwargs, device, progress, eta, step_noise, seed,
                                                   sample_offset):
            final = s
        return final["sample"]

    def ddim_sample_loop_progressive(self, model, shape, noise=None, clip_denoised=True, denoised_fn=None,
                                     cond_fn=None, model_kwargs=None, device=None, progress=False, eta=0.0,
                                     step_noise=None, seed=None, sample_offset=0):
        """gaussian_diffusion.py:664-707."""
        yield from self._loop(STEP_DDIM, model, shape, noise, clip_denoised, denoised_fn, cond_fn, model_kwargs,
                              device, progress, eta, step_noise, seed, sample_offset)

    # -- training (the diffusion TrainLoop's loss, U/src/gaussian_diffusion.py:188-206, :744-853) ---------
    def _train_coefs(self, t):
        """(sqrt(abar_t), sqrt(1 - abar_t)) gathered per sample and cast to fp32, as
        _extract_into_tensor does (:899-912): float64 table, index, .float()."""
        dev = t.device
        cache = self.__dict__.setdefault("_qtabs", {})
        tabs = cache.get(dev)
        if tabs is None:
            tabs = (torch.from_numpy(self.sqrt_alphas_cumprod).to(dev),
                    torch.from_numpy(self.sqrt_one_minus_alphas_cumprod).to(dev))
            cache[dev] = tabs
        return tabs[0][t].float().contiguous(), tabs[1][t].float().contiguous()

    def q_sample(self, x_start, t, noise=None):
        """x_t = sqrt(abar_t) x_start + sqrt(1 - abar_t) noise (:188-206), one
        cfd_q_sample launch (bit-exact against the reference's fp32 ops)."""
        if noise is None:
            noise = torch.randn_like(x_start)
        if noise.shape != x_start.shape:
            raise ValueError("noise must have the shape of x_start")
        if x_start.device.type != "cuda":
            raise _lib.CfdError("q_sample runs on the GPU (cfd_q_sample)")
        x0 = x_start.detach().to(torch.float32).contiguous()
        nz = noise.detach().to(torch.float32).contiguous()
        a, s = self._train_coefs(t.to(device=x0.device, dtype=torch.int64))
        xt = torch.empty_like(x0)
        B = x0.shape[0]
        _lib.check(_lib.load().cfd_q_sample(_lib.ptr(x0), _lib.ptr(nz), _lib.ptr(a), _lib.ptr(s), _lib.ptr(xt),
                                            x0.numel() // B, B, _lib.stream_of(x0.device)), "cfd_q_sample")
        return xt

    def training_losses(self, model, x_start, t, model_kwargs=None, noise=None, valid=False, weights=None,
                        grad=None):
        """GaussianDiffusion.training_losses (:744-853) for the MSE loss types with
        a fixed variance: returns {"mse", "loss"} (or {"valid_mse"} when ``valid``),
        one value per sample.

        The reference's caller then runs ``(terms["loss"] * weights).mean().backward()``
        (train_util.py:210-215); here that backward is this call's ``grad`` argument:
        when given (the flat fp32 gradient of ``model.param_keys()``), the gradient of
        ``(loss * weights).mean()`` (weights None = 1) is ADDED into it -- the U-Net
        forward records its tape, cfd_eps_mse forms the loss and d eps in one pass,
        cfd_unet_param_grad walks the network back."""
        if model_kwargs:
            raise NotImplementedError("class-conditional training (model_kwargs) is not on the HIP path")
        if self.loss_type not in (LossType.MSE, LossType.RESCALED_MSE):
            raise NotImplementedError(f"loss_type {self.loss_type} on the HIP path (the MSE losses are)")
        if self.model_var_type not in (ModelVarType.FIXED_SMALL, ModelVarType.FIXED_LARGE):
            raise NotImplementedError("learned variance (the vb term) is not on the HIP path")
        if self.model_mean_type not in (ModelMeanType.EPSILON, ModelMeanType.START_X):
            raise NotImplementedError(f"model_mean_type {self.model_mean_type} in training")
        if valid and grad is not None:
            raise ValueError("a validation pass has no gradient")
        if noise is None:
            noise = torch.randn_like(x_start)
        x_start = x_start.detach().to(torch.float32).contiguous()
        x_t = self.q_sample(x_start, t, noise=noise)
        tm = self._map_timesteps(t.to(device=x_t.device))
        with torch.no_grad():
            out = model.forward_tape(x_t, tm, for_param_grad=True) if grad is not None else model(x_t, tm)
        target = noise if self.model_mean_type == ModelMeanType.EPSILON else x_start
        target = target.detach().to(torch.float32).contiguous()
        if out.shape != target.shape:
            raise ValueError(f"model output {tuple(out.shape)} against target {tuple(target.shape)}")
        B = out.shape[0]
        n_per = out.numel() // B
        sse = torch.empty(B, dtype=torch.float32, device=out.device)
        d_out = torch.empty_like(out)
        w = None
        if weights is not None:
            w = weights.detach().to(device=out.device, dtype=torch.float32).contiguous()
        _lib.check(_lib.load().cfd_eps_mse(_lib.ptr(out), _lib.ptr(target), _lib.ptr(w),
                                           _lib.ptr(d_out), n_per, B, C.c_float(2.0 / (B * n_per)),
                                           _lib.ptr(sse), _lib.stream_of(out.device)), "cfd_eps_mse")
        mse = sse / n_per
        if valid:
            return {"valid_mse": mse}
        if grad is not None:
            model.param_grad(d_out, grad)
        return {"mse": mse, "loss": mse}
