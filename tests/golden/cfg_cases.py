"""Shared definitions of the config-shape golden cases (make_golden_cfg.py writes
them by running the reference; tests/test_gpu_cfg.py replays them on the HIP
path).  Nothing here imports the reference: every weight, input, noise draw and
on-disk file is regenerated from ``confild_amd.synth`` seeds, so only outputs are
stored in the fixtures."""
from __future__ import annotations

import os

import numpy as np
import torch

from confild_amd import synth

# config B (BASELINE.json configs[1]): Case4 uncond U-Net 64^2, DDPM respaced "256"
TRAJ_B = dict(tag="trajB", seed=1234, B=1, image_size=64, respacing="256",
              unet=dict(image_size=64, num_channels=128, num_res_blocks=2, channel_mult=None, num_heads=4,
                        num_head_channels=64, attention_resolutions="32,16,8"),
              checkpoints=(0, 1, 2, 4, 8, 16, 32, 64, 128, 192, 240, 250, 254, 255))

# config E (configs[4]): Case3 uncond U-Net 128^2 (default mult 1,1,2,3,4), the full
# 1000-step DDPM schedule: two 20-step segments of the reference's own p_sample,
# (start index, steps) -- the loop's first steps and its last
TRAJ_E = dict(tag="trajE", seed=1234, image_size=128, segments=((999, 20), (19, 20)), keep=(0, 1, 2, 4, 9, 14, 19),
              unet=dict(image_size=128, num_channels=128, num_res_blocks=2, channel_mult=None, num_heads=4,
                        num_head_channels=64, attention_resolutions="32,16,8"))

# config E, a longer stretch (round 4): 100 consecutive steps of the same loop
# (indices 599..500), so the bf16 operands' drift is stated over 100 steps
TRAJ_E100 = dict(tag="trajE100", start=599, n=100, keep=tuple(range(0, 100, 10)) + (99,))

# config E, the whole loop (round 6): all 1000 steps (999..0) of the same loop from
# a seeded x_T, so the bf16 operands' drift is stated over the line's full sampling
TRAJ_E1000 = dict(tag="trajE1000", keep=tuple(range(0, 1000, 100)) + (999,))

# config A (configs[0]): Case1 uncond 32^2 mult (1,2,3,4), DDIM-50, 1k-coord decode
CFG_A = dict(tag="cfgA", seed=1234, image_size=32, respacing="ddim50", vmax=1.5, vmin=-1.5,
             unet=dict(image_size=32, num_channels=128, num_res_blocks=2, channel_mult="1,2,3,4", num_heads=4,
                       num_head_channels=64, attention_resolutions="32,16,8"),
             siren=(2, 32, 3, 10, 128), siren_seed=1234, N=1000)

# config D (configs[3]) widths: DPS with the config-B U-Net and SIREN(3, 64, 3, 15, 384), 10 sensors
DPS_D = dict(tag="dpsD", seed=1234, respacing="256", scale=1.0, Ns=10, indices=(200, 37, 0),
             unet=dict(image_size=64, num_channels=128, num_res_blocks=2, channel_mult="", num_heads=4,
                       num_head_channels=64, attention_resolutions="32,16,8"),
             siren=(3, 64, 3, 15, 384), siren_seed=4321)

# the real Case4 notebook (inference_phy_random_sensor.ipynb cells 11-20): 384^2 latent,
# channel_mult "1, 1, 2, 2, 4, 4", the Case4 operator's SIREN(3, 384, 3, 15, 384), 10 sensors
CASE4_OP = dict(seed=77, T=384, L=384, Ns=10, batch_size=384, siren_seed=4242, unet_seed=1234, dps_index=500,
                unet=dict(image_size=384, num_channels=128, num_res_blocks=2, channel_mult="1, 1, 2, 2, 4, 4",
                          num_heads=4, num_head_channels=64, attention_resolutions="32,16,8"))


# the real Case4 loop: 10 consecutive DDPM + 'ps' steps at 384^2 (indices 500 .. 491)
CASE4_STEPS = dict(start=500, n=10)


def noise_for(tag: str, k: int, shape) -> np.ndarray:
    """The k-th normal tensor a reference run draws (torch.randn_like, in order)."""
    return synth.normal(7, f"{tag}/noise{k}", tuple(shape))


def unet_weights(state_dict_or_shapes, seed: int) -> dict:
    shapes = {k: tuple(v.shape) if hasattr(v, "shape") else tuple(v) for k, v in state_dict_or_shapes.items()}
    return synth.unet_state_dict(seed, shapes)


def case4_files(tmp: str) -> dict:
    """The on-disk inputs of Case4Operator.__init__ (measurements.py:184-217), from
    synth seeds: coords.npy, data_max/min.npy, a normaliser file with the
    x_normalizer_params / y_normalizer0u_params / y_normalizer0l_params keys (the
    y bounds carry more channels than the 3 the operator keeps), and
    checkpoint_20000.pt with the hard-coded SIREN(3, 384, 3, 15, 384)."""
    c = CASE4_OP
    s = c["siren_seed"]
    paths = {k: os.path.join(tmp, v) for k, v in dict(coords="coords.npy", max="data_max.npy", min="data_min.npy",
                                                       normalizer="normalizer_params.pt",
                                                       ckpt="checkpoint_20000.pt").items()}
    np.save(paths["coords"], synth.uniform(s, "case4/sensors", (c["Ns"], 3), -0.5, 2.0))
    np.save(paths["max"], synth.uniform(s, "case4/vmax", (c["L"],), 1.0, 2.0))
    np.save(paths["min"], -synth.uniform(s, "case4/vmin", (c["L"],), 1.0, 2.0))
    T = torch.from_numpy
    xhi, xlo = synth.uniform(s, "case4/xhi", (1, 3), 2.0, 2.5), synth.uniform(s, "case4/xlo", (1, 3), -1.0, -0.5)
    y0u = (T(synth.uniform(s, "case4/y0u_hi", (5,), 0.5, 2.0)), T(synth.uniform(s, "case4/y0u_lo", (5,), -9., -8.)))
    y0l = (T(synth.uniform(s, "case4/y0l_hi", (5,), 8.0, 9.0)), T(-synth.uniform(s, "case4/y0l_lo", (5,), 0.5, 2.)))
    torch.save({"x_normalizer_params": (T(xhi), T(xlo)), "y_normalizer0u_params": y0u,
                "y_normalizer0l_params": y0l}, paths["normalizer"])
    sd = synth.siren_state_dict(s, 3, 384, 3, 15, 384)
    torch.save({"epoch": 20000, "model_state_dict": {k: T(v) for k, v in sd.items()}}, paths["ckpt"])
    return paths


# CNF_inference (N/cnf/inference_function.py:79-304) on a trained-checkpoint
# directory: (name, dims, lumped, is_pub, SIREN (d, L, c, nh, H), data shape,
# latent count, predict indices)
CNF_INF = {
    "grid2d": dict(dims=2, lumped=False, is_pub=False, siren=(2, 16, 3, 2, 32), data_shape=(7, 12, 10, 3),
                   n_lat=7, idx=[0, 3, 5, 6], seed=31),
    "lumped3d_pub": dict(dims=3, lumped=True, is_pub=True, siren=(3, 24, 3, 3, 64), data_shape=(9, 300, 3),
                         n_lat=9, idx=[8, 1, 4], seed=32),
}

# the Case4 notebook's post-processing (cells 26-32): decoder over the masked
# points, rearrange, ReconstructFrame into the infos.npz Mask grid
POST = dict(siren=(3, 16, 3, 2, 32), grid=(8, 6, 5), s=2, t=3, seed=41)


def cnf_inference_files(tmp: str, name: str) -> dict:
    """checkpoint dir (checkpoint_*.pt + normalizer_params.pt), config YAML and a
    data .npy for CNF_inference, from synth seeds."""
    import yaml
    c = CNF_INF[name]
    d, L, co, nh, H = c["siren"]
    s = c["seed"]
    T = torch.from_numpy
    ck = os.path.join(tmp, "ckpt")
    os.makedirs(ck, exist_ok=True)
    sd = {k: T(v) for k, v in synth.siren_state_dict(s, d, L, co, nh, H).items()}
    lat = T(synth.normal(s, "cnfinf/latents", (c["n_lat"], L)) * np.float32(0.5))
    hidden = lat if c["is_pub"] else {"latents": lat}
    torch.save({"epoch": 5, "model_state_dict": sd, "hidden_states": hidden}, os.path.join(ck, "checkpoint_5.pt"))
    npts = int(np.prod(c["data_shape"][1:-1]))
    yshape = (1, npts, co) if c["lumped"] else (1, co)
    torch.save({"x_normalizer_params": (T(synth.uniform(s, "cnfinf/xhi", (1, d), 1.0, 1.5)),
                                        T(synth.uniform(s, "cnfinf/xlo", (1, d), -0.5, 0.0))),
                "y_normalizer_params": (T(synth.uniform(s, "cnfinf/yhi", yshape, 0.5, 2.0)),
                                        T(-synth.uniform(s, "cnfinf/ylo", yshape, 0.5, 2.0)))},
               os.path.join(ck, "normalizer_params.pt"))
    cfg = {"dims": c["dims"], "lumped_latent": c["lumped"], "hidden_size": L,
           "NF": {"name": "SIRENAutodecoder_film", "in_coord_features": d, "out_features": co,
                  "num_hidden_layers": nh, "hidden_features": H}}
    with open(os.path.join(tmp, "cnf.yml"), "w") as f:
        yaml.safe_dump(cfg, f)
    np.save(os.path.join(tmp, "data.npy"), synth.uniform(s, "cnfinf/data", c["data_shape"], -1.0, 1.0))
    return dict(checkpoint=os.path.join(ck, "checkpoint_5.pt"), config=os.path.join(tmp, "cnf.yml"),
                data=os.path.join(tmp, "data.npy"))


def cnf_inference_coords(name: str) -> np.ndarray:
    c = CNF_INF[name]
    d = c["siren"][0]
    return synth.uniform(c["seed"], "cnfinf/coords", tuple(c["data_shape"][1:-1]) + (d,), 0.0, 1.0)


def post_inputs():
    """Mask grid, masked coordinates, (s*t, L) latents and normaliser bounds."""
    c = POST
    d, L, co, nh, H = c["siren"]
    s = c["seed"]
    mask = synth.uniform(s, "post/mask", c["grid"], 0.0, 1.0) < 0.55
    n = int(mask.sum())
    coords = synth.uniform(s, "post/coords", (n, d), 0.0, 1.0)
    lat = synth.normal(s, "post/lat", (c["s"] * c["t"], L)) * np.float32(0.5)
    xhi, xlo = np.ones((1, d), np.float32), np.zeros((1, d), np.float32)
    yhi = synth.uniform(s, "post/yhi", (co,), 0.5, 2.0)
    ylo = -synth.uniform(s, "post/ylo", (co,), 0.5, 2.0)
    return mask, coords, lat, xhi, xlo, yhi, ylo
