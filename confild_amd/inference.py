"""Drop-in for UnconditionalDiffusionTraining_and_Generation/scripts/inference.py.

    python -m confild_amd.inference case.yml                      # 1 GPU
    torchrun --nproc-per-node 8 -m confild_amd.inference case.yml # 8 GPUs

Same YAML keys as the reference (training_recipes/*.yml).  Optional keys, with
reference-preserving defaults:
  timestep_respacing: ""      (reference: full `steps`)
  sampler: ddpm | ddim        (reference: ddpm, p_sample_loop)
  coords_path: null           (reference: the CNF trainer's training points)
  seed: 42                    (reference: torch.manual_seed(42), inference.py:17)
  precision: fp32 | bf16      (reference: fp32.  fp32 runs the U-Net convolutions as
                               split-f16, fp32-level error; bf16 = config E, bf16
                               operands with fp32 accumulation, GroupNorm/softmax fp32)
  compute: split_f16 | fp32 | bf16   (explicit U-Net compute mode; overrides precision)
Known deviation (fixed on purpose): ``channel_mult`` from the YAML IS passed to
create_model (the reference reads but drops it, inference.py:38-44, so its own
case4.yml raises ValueError).

Flow (inference.py:20-81): sample (B, 1, T, L) latents on the GPU(s) ->
de-normalise with max_val/min_val -> CNF decode of every latent row over the
query points (one fused launch per chunk) -> np.save((B*T, N, c)) on rank 0.
Multi-GPU: samples are sharded over ranks (dist.sharded_samples) with the
unsharded Philox stream, weights are broadcast from rank 0 once, decoded
fields are gathered to rank 0.
"""
from __future__ import annotations

import sys

import numpy as np
import torch

from . import _lib, dist
from .read_input import basic_input
from .script_util import create_gaussian_diffusion, create_model
from .trainer import trainer


def latent_denorm(gen: torch.Tensor, vmax: torch.Tensor, vmin: torch.Tensor) -> torch.Tensor:
    """(gen + 1) * (max - min) / 2 + min on the GPU (cfd_latent_denorm); max/min are
    scalars or broadcast over gen's trailing dimensions."""
    period = vmax.numel()
    if vmin.numel() != period or gen.numel() % period or (period > 1 and
                                                          tuple(gen.shape[-vmax.dim():]) != tuple(vmax.shape)):
        raise ValueError(f"max/min of shape {tuple(vmax.shape)} do not broadcast over the latents' trailing dims")
    out = torch.empty_like(gen)
    _lib.check(_lib.lib().cfd_latent_denorm(_lib.ptr(gen), _lib.ptr(out), gen.numel(), _lib.ptr(vmax),
                                            _lib.ptr(vmin), period, _lib.stream_of(gen.device)), "latent_denorm")
    return out


PRECISIONS = {"fp32": "split_f16", "float32": "split_f16", "bf16": "bf16", "bfloat16": "bf16"}


def unet_compute(inp) -> str:
    """U-Net compute mode from the optional ``compute`` / ``precision`` YAML keys."""
    explicit = getattr(inp, "compute", None)
    if explicit is not None:
        return str(explicit)
    prec = str(getattr(inp, "precision", "fp32")).lower()
    if prec not in PRECISIONS:
        raise ValueError(f"precision must be one of {sorted(PRECISIONS)}, got {prec!r}")
    return PRECISIONS[prec]


def run(yaml_path: str):
    rank, world, device = dist.init_from_env()
    if device.type != "cuda":
        raise _lib.CfdError("confild_amd.inference needs a GPU")
    inp = basic_input(yaml_path)
    seed = int(getattr(inp, "seed", 42))
    torch.manual_seed(seed)
    np.random.seed(seed)
    # Philox key of the reverse loop, drawn first so it depends only on `seed`
    # (identical on every rank)
    loop_seed = int(torch.randint(0, 2 ** 62, (1,)).item())

    model = create_model(image_size=inp.image_size, num_channels=inp.num_channels,
                         num_res_blocks=inp.num_res_blocks, num_heads=inp.num_heads,
                         num_head_channels=inp.num_head_channels,
                         attention_resolutions=inp.attention_resolutions,
                         channel_mult=getattr(inp, "channel_mult", None))
    model.set_compute(unet_compute(inp))
    if rank == 0:
        model.load_state_dict(torch.load(inp.ema_path, weights_only=True, map_location="cpu"))
    model.to(device)
    dist.broadcast_module(model)
    diff = create_gaussian_diffusion(steps=inp.steps, noise_schedule=inp.noise_schedule,
                                     timestep_respacing=getattr(inp, "timestep_respacing", ""))
    sampler = getattr(inp, "sampler", "ddpm")
    B, T, L = inp.test_batch_size, inp.time_length, inp.latent_length

    def sample(start, count):
        fn = diff.p_sample_loop if sampler == "ddpm" else diff.ddim_sample_loop
        return fn(model, (count, 1, T, L), seed=loop_seed, sample_offset=start)[:, 0]

    gen = dist.sharded_samples(sample, B)                    # (B, T, L) on every rank

    max_val = torch.as_tensor(np.load(inp.max_val), dtype=torch.float32).to(device).contiguous()
    min_val = torch.as_tensor(np.load(inp.min_val), dtype=torch.float32).to(device).contiguous()
    gen = latent_denorm(gen.contiguous(), max_val, min_val)   # inference.py:59-61

    cnf = trainer(basic_input(inp.cnf_case_file_path), infer_mode=getattr(inp, "coords_path", None) is not None)
    cnf.load(-1, siren_only=True)
    cnf.nf.to(device)
    coord = cnf.train_coord
    if getattr(inp, "coords_path", None):
        coord = torch.as_tensor(np.load(inp.coords_path), dtype=torch.float32)
    # lumped (N, d) points, or an (h, w, d) grid: the reference keeps the grid
    # shape and saves (B*T, h, w, c) (train.py:274-277, inference.py:75-81)
    coord = coord.to(device)
    spatial = tuple(coord.shape[:-1])
    npts = int(np.prod(spatial))
    lat = gen.reshape(B * T, L)
    # rows per launch bounded by ~2 GiB of output
    rows = max(1, (2 << 30) // (npts * cnf.nf.out_features * 4))
    fields = []
    s, e = dist.shard_range(B * T, rank, world)
    for a in range(s, e, rows):
        fields.append(cnf.infer(coord, lat[a:min(e, a + rows)]))
    local = torch.cat(fields) if fields else torch.empty((0,) + spatial + (cnf.nf.out_features,), device=device)
    if world > 1:   # gather the decoded fields to rank 0 over RCCL
        sizes = [dist.shard_range(B * T, r, world)[1] - dist.shard_range(B * T, r, world)[0] for r in range(world)]
        local = dist.gather_cat(local, 0, sizes, dst=0)
    if rank == 0:
        out = local.cpu().numpy()
        np.save(inp.save_path, out)                          # (B*T, N, c) or (B*T, h, w, c), inference.py:79-81
        return out
    return None


if __name__ == "__main__":
    run(sys.argv[1])
