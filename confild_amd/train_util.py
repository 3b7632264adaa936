"""The diffusion TrainLoop on the HIP path (drop-in for U/src/train_util.py).

Same constructor, ``run_loop`` / ``run_step`` / ``forward_backward`` /
``forward_valid`` / ``save`` and checkpoint files as the reference TrainLoop
(train_util.py:22-330) at fp32 (``use_fp16`` is refused: the master weights are
the model's fp32 parameters, MixedPrecisionTrainer._optimize_normal).  One step:

* zero the flat fp32 gradient of every parameter (``model.param_keys()`` order);
* per microbatch: ``ScheduleSampler.sample`` (numpy RNG, the reference's call),
  ``GaussianDiffusion.training_losses(..., grad=)`` -- cfd_q_sample, the U-Net
  forward with its tape, cfd_eps_mse (per-sample MSE and d eps of
  ``(loss * weights).mean()``), cfd_unet_param_grad adding the microbatch's
  parameter gradient (the reference's ``loss.backward()``);
* multi-GPU: the gradient is averaged over the ranks (one RCCL all-reduce of the
  flat buffer -- DistributedDataParallel's averaged gradients);
* AdamW (``cfd_adam_step`` with decoupled weight decay, torch.optim.AdamW) on the
  flat parameters, copied back into the module (the handle re-packs them);
* per EMA rate ``cfd_ema_update`` (src.nn.update_ema); learning-rate annealing
  as ``_anneal_lr``.

Checkpoints: ``model{step:06d}.pt``, ``ema_{rate}_{step:06d}.pt`` (the module's
state dict) and ``opt{step:06d}.pt`` (torch.optim.AdamW's state-dict layout) in
``log_dir``, loadable by the reference and resumable from the reference's files
(``torch.load(weights_only=True)``).
"""
from __future__ import annotations

import os

import torch

from . import _lib
from .cnf_train import Adam
from .resample import LossAwareSampler, UniformSampler


def _dist():
    import torch.distributed as dist
    return dist if dist.is_available() and dist.is_initialized() else None


def parse_resume_step_from_filename(filename):
    """train_util.py:298-310: path/to/modelNNNNNN.pt -> NNNNNN (0 otherwise)."""
    split = filename.split("model")
    if len(split) < 2:
        return 0
    try:
        return int(split[-1].split(".")[0])
    except ValueError:
        return 0


def find_ema_checkpoint(main_checkpoint, step, rate):
    """train_util.py:324-331."""
    if main_checkpoint is None:
        return None
    path = os.path.join(os.path.dirname(main_checkpoint), f"ema_{rate}_{step:06d}.pt")
    return path if os.path.exists(path) else None


class _KV:
    """The logger's logkv / logkv_mean / dumpkvs accumulator (U/src/logger.py)."""

    def __init__(self):
        self.vals, self.counts, self.history = {}, {}, []

    def logkv(self, k, v):
        self.vals[k], self.counts[k] = v, 1

    def logkv_mean(self, k, v):
        n = self.counts.get(k, 0)
        self.vals[k] = (self.vals.get(k, 0.0) * n + v) / (n + 1)
        self.counts[k] = n + 1

    def dumpkvs(self):
        out = dict(self.vals)
        self.history.append(out)
        self.vals, self.counts = {}, {}
        return out


class TrainLoop:
    """train_util.py:22-296 (see the module docstring).  ``log_dir`` replaces the
    reference's ``logger.get_dir()`` (None: no checkpoint files)."""

    def __init__(self, *, model, diffusion, train_data, batch_size, microbatch, lr, ema_rate, log_interval,
                 save_interval, resume_checkpoint, valid_data=None, use_fp16=False, fp16_scale_growth=1e-3,
                 schedule_sampler=None, weight_decay=0.0, lr_anneal_steps=0, final_lr=0.0, log_dir=None):
        if use_fp16:
            raise NotImplementedError("fp16 training (loss scaling) is not on the HIP path; the fp32 trainer is")
        if getattr(model, "dropout", 0):
            raise NotImplementedError("dropout > 0 in the U-Net's training forward is not on the HIP path")
        self.model, self.diffusion = model, diffusion
        self.train_data, self.valid_data = train_data, valid_data
        self.batch_size = batch_size
        self.microbatch = microbatch if microbatch > 0 else batch_size
        self.lr = lr
        self.ema_rate = [ema_rate] if isinstance(ema_rate, float) else [float(x) for x in str(ema_rate).split(",")]
        self.log_interval, self.save_interval = log_interval, save_interval
        self.resume_checkpoint = resume_checkpoint
        self.use_fp16, self.fp16_scale_growth = False, fp16_scale_growth
        self.schedule_sampler = schedule_sampler or UniformSampler(diffusion)
        self.weight_decay, self.lr_anneal_steps, self.final_lr = weight_decay, lr_anneal_steps, final_lr
        self.log_dir = log_dir
        self.step, self.resume_step = 0, 0
        d = _dist()
        self.world_size = d.get_world_size() if d else 1
        self.rank = d.get_rank() if d else 0
        self.global_batch = self.batch_size * self.world_size
        self.device = next(model.parameters()).device
        if self.device.type != "cuda":
            raise _lib.CfdError("the diffusion TrainLoop needs the model on a GPU")
        self.logger = _KV()

        self._load_and_sync_parameters()
        self.keys = model.param_keys()
        named = dict(model.named_parameters())
        offs, o = {}, 0
        for k in self.keys:
            offs[k] = o
            o += named[k].numel()
        # torch.optim's param order is model.parameters(): spans map it onto the flat buffer
        self._spans = [(offs[k], tuple(p.shape)) for k, p in model.named_parameters()]
        self.params = model.flat_params()                       # the fp32 master parameters
        self.grad = torch.zeros_like(self.params)
        self.opt = Adam(self.params, self.lr, weight_decay=self.weight_decay)
        if self.resume_step:
            self._load_optimizer_state()
            self.ema_params = [self._load_ema_parameters(r) for r in self.ema_rate]
        else:
            self.ema_params = [self.params.clone() for _ in self.ema_rate]

    # -- checkpoints ---------------------------------------------------------------
    def _load_and_sync_parameters(self):
        ck = self.resume_checkpoint
        if ck:
            self.resume_step = parse_resume_step_from_filename(ck)
            if self.rank == 0:
                sd = torch.load(ck, map_location=self.device, weights_only=True)
                self.model.load_state_dict(sd)
        d = _dist()
        if d and self.world_size > 1:
            with torch.no_grad():
                for p in self.model.parameters():
                    d.broadcast(p.data, 0)

    def _flat_of_state_dict(self, sd):
        return torch.cat([sd[k].to(device=self.device, dtype=torch.float32).reshape(-1)
                          for k in self.keys]).contiguous()

    def _load_ema_parameters(self, rate):
        ema = self.params.clone()
        path = find_ema_checkpoint(self.resume_checkpoint, self.resume_step, rate)
        if path and self.rank == 0:
            ema = self._flat_of_state_dict(torch.load(path, map_location=self.device, weights_only=True))
        d = _dist()
        if d and self.world_size > 1:
            d.broadcast(ema, 0)
        return ema

    def _load_optimizer_state(self):
        path = os.path.join(os.path.dirname(self.resume_checkpoint), f"opt{self.resume_step:06}.pt")
        if os.path.exists(path):
            self.opt.load_torch_state_dict(torch.load(path, map_location=self.device, weights_only=True),
                                           self._spans)

    def _state_dict_of_flat(self, flat):
        sd = self.model.state_dict()
        named = dict(self.model.named_parameters())
        o = 0
        for k in self.keys:
            n = named[k].numel()
            sd[k] = flat[o:o + n].reshape(named[k].shape).clone()
            o += n
        return sd

    def save(self):
        """train_util.py:272-296."""
        step = self.step + self.resume_step
        if self.rank == 0 and self.log_dir:
            os.makedirs(self.log_dir, exist_ok=True)
            torch.save(self._state_dict_of_flat(self.params), os.path.join(self.log_dir, f"model{step:06d}.pt"))
            for rate, ema in zip(self.ema_rate, self.ema_params):
                torch.save(self._state_dict_of_flat(ema), os.path.join(self.log_dir, f"ema_{rate}_{step:06d}.pt"))
            torch.save(self.opt.torch_state_dict(self._spans), os.path.join(self.log_dir, f"opt{step:06d}.pt"))
        d = _dist()
        if d and self.world_size > 1:
            d.barrier()

    # -- the loop ------------------------------------------------------------------
    def run_loop(self):
        """train_util.py:156-176 (``valid_data`` None: no validation pass)."""
        while not self.lr_anneal_steps or self.step + self.resume_step < self.lr_anneal_steps:
            train_batch, = next(self.train_data)
            valid_batch = next(self.valid_data)[0] if self.valid_data is not None else None
            self.run_step(train_batch, valid_batch, None)
            if self.step % self.log_interval == 0:
                self.logger.dumpkvs()
            if self.step % self.save_interval == 0:
                self.save()
                if os.environ.get("DIFFUSION_TRAINING_TEST", "") and self.step > 0:
                    return
            self.step += 1
        if (self.step - 1) % self.save_interval != 0:
            self.save()

    def run_step(self, train_batch, valid_batch=None, cond=None, noise=None):
        """train_util.py:178-188.  ``noise``: optional per-sample noise of the
        training batch (a replay hook; None draws torch.randn_like like the
        reference's training_losses)."""
        if cond:
            raise NotImplementedError("class-conditional training is not on the HIP path")
        self.forward_backward(train_batch, noise=noise)
        if valid_batch is not None:
            self.forward_valid(valid_batch)
        self._optimize()
        self._update_ema()
        self._anneal_lr()
        self.log_step()

    def forward_backward(self, batch, cond=None, noise=None):
        """train_util.py:190-226: the gradients of every microbatch's
        ``(loss * weights).mean()`` summed into ``self.grad``."""
        self.grad.zero_()
        for i in range(0, batch.shape[0], self.microbatch):
            micro = batch[i:i + self.microbatch].to(self.device)
            t, weights = self.schedule_sampler.sample(micro.shape[0], self.device)
            nz = noise[i:i + self.microbatch].to(self.device) if noise is not None else None
            losses = self.diffusion.training_losses(self.model, micro, t, noise=nz, weights=weights,
                                                    grad=self.grad)
            if isinstance(self.schedule_sampler, LossAwareSampler):
                self.schedule_sampler.update_with_local_losses(t, losses["loss"].detach())
            self._log_loss_dict(t, {k: v * weights for k, v in losses.items()})

    def forward_valid(self, batch, cond=None):
        """train_util.py:228-254 (no gradient)."""
        for i in range(0, batch.shape[0], self.microbatch):
            micro = batch[i:i + self.microbatch].to(self.device)
            t, weights = self.schedule_sampler.sample(micro.shape[0], self.device)
            losses = self.diffusion.training_losses(self.model, micro, t, valid=True)
            self._log_loss_dict(t, {k: v * weights for k, v in losses.items()})

    def _optimize(self):
        """MixedPrecisionTrainer._optimize_normal (fp16_util.py:210-215) after DDP's
        gradient averaging."""
        d = _dist()
        if d and self.world_size > 1:
            d.all_reduce(self.grad)
            self.grad.div_(self.world_size)
        self.logger.logkv_mean("grad_norm", float(torch.linalg.vector_norm(self.grad)))
        self.logger.logkv_mean("param_norm", float(torch.linalg.vector_norm(self.params)))
        self.opt.step(self.grad)
        self.model.load_flat(self.params, alias=True)   # the module's tensors are views of the master buffer

    def _update_ema(self):
        lib = _lib.load()
        for rate, ema in zip(self.ema_rate, self.ema_params):
            _lib.check(lib.cfd_ema_update(_lib.ptr(ema), _lib.ptr(self.params), self.params.numel(),
                                          float(rate), _lib.stream_of(self.device)), "cfd_ema_update")

    def _anneal_lr(self):
        """train_util.py:260-266."""
        if not self.lr_anneal_steps:
            return
        frac = (self.step + self.resume_step) / self.lr_anneal_steps
        self.opt.lr = self.final_lr * frac + self.lr * (1 - frac)

    def log_step(self):
        self.logger.logkv("step", self.step + self.resume_step)
        self.logger.logkv("samples", (self.step + self.resume_step + 1) * self.global_batch)

    def _log_loss_dict(self, ts, losses):
        """log_loss_dict (train_util.py:334-340): mean and per-quartile means."""
        tq = ts.cpu().numpy()
        for k, v in losses.items():
            vals = v.detach().cpu().numpy()
            self.logger.logkv_mean(k, float(vals.mean()))
            for sub_t, sub in zip(tq, vals):
                self.logger.logkv_mean(f"{k}_q{int(4 * sub_t / self.diffusion.num_timesteps)}", float(sub))

    def ema_state_dict(self, i=0):
        """The EMA parameters of rate ``self.ema_rate[i]`` as a module state dict."""
        return self._state_dict_of_flat(self.ema_params[i])


__all__ = ["TrainLoop", "parse_resume_step_from_filename", "find_ema_checkpoint"]
