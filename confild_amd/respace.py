"""Timestep respacing (drop-in for U/src/respace.py)."""
from __future__ import annotations

import numpy as np
import torch

from .gaussian_diffusion import GaussianDiffusion


def space_timesteps(num_timesteps, section_counts):
    """respace.py:7-60: equal-portion striding, or "ddimN" integer striding."""
    if isinstance(section_counts, str):
        if section_counts.startswith("ddim"):
            desired = int(section_counts[len("ddim"):])
            for i in range(1, num_timesteps):
                if len(range(0, num_timesteps, i)) == desired:
                    return set(range(0, num_timesteps, i))
            raise ValueError(f"cannot create exactly {num_timesteps} steps with an integer stride")
        section_counts = [int(x) for x in section_counts.split(",")]
    size_per, extra = divmod(num_timesteps, len(section_counts))
    start_idx, all_steps = 0, []
    for i, count in enumerate(section_counts):
        size = size_per + (1 if i < extra else 0)
        if size < count:
            raise ValueError(f"cannot divide section of {size} steps into {count}")
        frac_stride = 1 if count <= 1 else (size - 1) / (count - 1)
        cur = 0.0
        for _ in range(count):
            all_steps.append(start_idx + round(cur))
            cur += frac_stride
        start_idx += size
    return set(all_steps)


class SpacedDiffusion(GaussianDiffusion):
    """respace.py:63-113: re-derives betas on the kept timesteps and remaps the
    model's timesteps through ``timestep_map`` (the _WrappedModel of :116-128)."""

    def __init__(self, use_timesteps, **kwargs):
        self.use_timesteps = set(use_timesteps)
        self.timestep_map = []
        self.original_num_steps = len(kwargs["betas"])
        base = GaussianDiffusion(**kwargs)
        last, new_betas = 1.0, []
        for i, a in enumerate(base.alphas_cumprod):
            if i in self.use_timesteps:
                new_betas.append(1 - a / last)
                last = a
                self.timestep_map.append(i)
        kwargs["betas"] = np.array(new_betas)
        super().__init__(**kwargs)
        self._maps = {}

    def _model_timesteps_host(self, indices):
        return [self.timestep_map[i] for i in indices]

    def _map_timesteps(self, t):
        dev = t.device
        m = self._maps.get(dev)
        if m is None:
            m = torch.tensor(self.timestep_map, dtype=torch.int64, device=dev)
            self._maps[dev] = m
        new_t = m[t]
        if self.rescale_timesteps:
            raise NotImplementedError("rescale_timesteps=True")
        return new_t
