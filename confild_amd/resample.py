"""Timestep schedule samplers of the diffusion TrainLoop (drop-in for
U/src/resample.py).  Host-side numpy: the draws use numpy's global RNG with the
reference's exact call (``np.random.choice(len(p), size=(B,), p=p)``, :43-56), so
a seeded run draws the reference's timesteps."""
from __future__ import annotations

from abc import ABC, abstractmethod

import numpy as np
import torch


def create_named_schedule_sampler(name, diffusion):
    """resample.py:8-20."""
    if name == "uniform":
        return UniformSampler(diffusion)
    if name == "loss-second-moment":
        return LossSecondMomentResampler(diffusion)
    raise NotImplementedError(f"unknown schedule sampler: {name}")


class ScheduleSampler(ABC):
    """resample.py:23-57: importance sampling over the diffusion steps."""

    @abstractmethod
    def weights(self):
        """Positive per-step weights (need not be normalised)."""

    def sample(self, batch_size, device):
        """(timesteps int64, importance weights fp32) on ``device``."""
        w = self.weights()
        p = w / np.sum(w)
        idx = np.random.choice(len(p), size=(batch_size,), p=p)
        wts = 1 / (len(p) * p[idx])
        return torch.from_numpy(idx).long().to(device), torch.from_numpy(wts).float().to(device)


class UniformSampler(ScheduleSampler):
    """resample.py:60-66."""

    def __init__(self, diffusion):
        self.diffusion = diffusion
        self._weights = np.ones([diffusion.num_timesteps])

    def weights(self):
        return self._weights


class LossAwareSampler(ScheduleSampler):
    """resample.py:69-117: weights updated from the ranks' losses (all-gathered)."""

    def update_with_local_losses(self, local_ts, local_losses):
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            ws = dist.get_world_size()
            sizes = [torch.zeros(1, dtype=torch.int32, device=local_ts.device) for _ in range(ws)]
            dist.all_gather(sizes, torch.tensor([len(local_ts)], dtype=torch.int32, device=local_ts.device))
            sizes = [int(x.item()) for x in sizes]
            mx = max(sizes)
            tb = [torch.zeros(mx).to(local_ts) for _ in sizes]
            lb = [torch.zeros(mx).to(local_losses) for _ in sizes]
            pad_t = torch.zeros(mx).to(local_ts)
            pad_t[:len(local_ts)] = local_ts
            pad_l = torch.zeros(mx).to(local_losses)
            pad_l[:len(local_losses)] = local_losses
            dist.all_gather(tb, pad_t)
            dist.all_gather(lb, pad_l)
            ts = [int(x.item()) for y, n in zip(tb, sizes) for x in y[:n]]
            losses = [float(x.item()) for y, n in zip(lb, sizes) for x in y[:n]]
        else:
            ts = [int(x) for x in local_ts.tolist()]
            losses = [float(x) for x in local_losses.tolist()]
        self.update_with_all_losses(ts, losses)

    @abstractmethod
    def update_with_all_losses(self, ts, losses):
        """Deterministic update from every rank's (timestep, loss) pairs."""


class LossSecondMomentResampler(LossAwareSampler):
    """resample.py:120-150: sqrt of the mean squared recent loss per step, mixed
    with ``uniform_prob`` of the uniform distribution once every step has
    ``history_per_term`` losses."""

    def __init__(self, diffusion, history_per_term=10, uniform_prob=0.001):
        self.diffusion = diffusion
        self.history_per_term = history_per_term
        self.uniform_prob = uniform_prob
        self._loss_history = np.zeros([diffusion.num_timesteps, history_per_term], dtype=np.float64)
        self._loss_counts = np.zeros([diffusion.num_timesteps], dtype=np.int64)

    def weights(self):
        if not self._warmed_up():
            return np.ones([self.diffusion.num_timesteps], dtype=np.float64)
        w = np.sqrt(np.mean(self._loss_history ** 2, axis=-1))
        w /= np.sum(w)
        w *= 1 - self.uniform_prob
        w += self.uniform_prob / len(w)
        return w

    def update_with_all_losses(self, ts, losses):
        for t, loss in zip(ts, losses):
            if self._loss_counts[t] == self.history_per_term:
                self._loss_history[t, :-1] = self._loss_history[t, 1:]
                self._loss_history[t, -1] = loss
            else:
                self._loss_history[t, self._loss_counts[t]] = loss
                self._loss_counts[t] += 1

    def _warmed_up(self):
        return bool((self._loss_counts == self.history_per_term).all())
