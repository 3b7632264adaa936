"""Generate the DPS (Case4 conditional) golden fixture by running the REFERENCE.

Run in the build container only (the reference tree does not exist on the GPU
box):

    python tests/golden/make_golden_dps.py

Drives the reference's own guided sampler exactly as the Case4 notebook does
(ConditionalDiffusionGeneration/inference_scripts/Case4/random_sensor/
inference_phy_random_sensor.ipynb, cells 11-23): ``create_model`` (C/src/
guided_diffusion/unet.py:25-92), ``create_sampler('ddpm', ...)``
(gaussian_diffusion.py:30-52), ``get_noise('gaussian', sigma=0)``,
``get_conditioning_method('ps', scale)`` (condition_methods.py:81-90) and
``DDPM.p_sample_loop`` (gaussian_diffusion.py:169-206) with the Case4 operator
(measurements.py:184-226) -- at fixture scale:

  * the U-Net is small (16x16 latent) with synthetic weights from
    ``confild_amd.synth``;
  * ``Case4Operator.__init__`` hard-codes a (3, 384, 3, 15, 384) SIREN and reads
    checkpoint files, so the operator is built with ``__new__`` and its
    attributes (coords, normalisers, SIREN, latent bounds, batch size) are set
    to small synthetic ones; its ``_unnorm`` / ``forward`` are the reference's.

Every ``torch.randn_like`` draw of the loop is recorded (the p_sample noise and
the q_sample noise of the unused noisy measurement, interleaved) so the HIP
sampler can replay the same noise.  The only shim is the tensorboard stand-in
also used by make_golden.py.  Recorded per step: x0_hat, the DDPM sample,
the conditioned image, and the residual norm.
"""
from __future__ import annotations

import os
import sys

sys.dont_write_bytecode = True
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, REF, os.path.join(REF, "ConditionalNeuralField")]

import types  # noqa: E402

# in-process stand-in for torch.utils.tensorboard (not installed; imported at
# ConditionalNeuralField/scripts/train.py:13, never used on this path)
_tb = types.ModuleType("torch.utils.tensorboard")
_tb.SummaryWriter = object
sys.modules["torch.utils.tensorboard"] = _tb

import numpy as np  # noqa: E402
import torch  # noqa: E402

from confild_amd import synth  # noqa: E402

torch.set_num_threads(8)

CASES = {
    # name: (unet kwargs, siren dims (d, L, c, nh, H), sensors, steps respacing, scale, seed)
    "dps_tiny16": (dict(image_size=16, num_channels=32, num_res_blocks=1, channel_mult="1,2",
                        num_heads=1, num_head_channels=16, attention_resolutions="8"),
                   (3, 16, 3, 2, 32), 5, "8", 1.0, 21),
    "dps_tiny16_s3": (dict(image_size=16, num_channels=32, num_res_blocks=1, channel_mult="1,2",
                           num_heads=1, num_head_channels=16, attention_resolutions="8"),
                      (3, 16, 3, 2, 32), 12, "6", 3.0, 22),
}


def build(case):
    from ConditionalDiffusionGeneration.src.guided_diffusion.unet import create_model
    from ConditionalDiffusionGeneration.src.guided_diffusion import measurements as ms
    from cnf.nf_networks import SIRENAutodecoder_film
    from cnf.utils.normalize import Normalizer_ts

    kw, (d, L, c, nh, H), Ns, resp, scale, seed = CASES[case]
    S = kw["image_size"]
    torch.manual_seed(0)
    model = create_model(**kw, model_path="")           # prints "Randomly initialize"
    sd = synth.unet_state_dict(seed, {k: tuple(v.shape) for k, v in model.state_dict().items()})
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    model.eval()

    nf = SIRENAutodecoder_film(d, L, c, nh, H)
    ssd = synth.siren_state_dict(seed + 100, d, L, c, nh, H)
    nf.load_state_dict({k: torch.from_numpy(v) for k, v in ssd.items()})
    nf.eval()

    op = ms.Case4Operator.__new__(ms.Case4Operator)
    op.device = torch.device("cpu")
    coords = synth.uniform(seed, "sensors", (Ns, d), -0.5, 2.0)
    op.coords = torch.tensor(coords, dtype=torch.float32)
    xhi = synth.uniform(seed, "xhi", (1, d), 2.0, 2.5)
    xlo = synth.uniform(seed, "xlo", (1, d), -1.0, -0.5)
    yhi = synth.uniform(seed, "yhi", (c,), 0.5, 2.0)
    ylo = synth.uniform(seed, "ylo", (c,), -2.0, -0.5)
    op.x_normalizer = Normalizer_ts(method="-11", dim=0, params=(torch.from_numpy(xhi), torch.from_numpy(xlo)))
    op.y_normalizer = Normalizer_ts(method="-11", dim=0, params=(torch.from_numpy(yhi), torch.from_numpy(ylo)))
    op.model = nf
    vmax = synth.uniform(seed, "vmax", (L,), 1.0, 2.0)
    vmin = synth.uniform(seed, "vmin", (L,), -2.0, -1.0)
    op.max_val = torch.from_numpy(vmax)
    op.min_val = torch.from_numpy(vmin)
    op.batch_size = 6                                   # exercises pass_through_model_batch chunking
    arrays = dict(kwargs=np.array(repr(kw)), seed=np.int64(seed), siren_seed=np.int64(seed + 100),
                  siren_dims=np.array([d, L, c, nh, H], dtype=np.int64), coords=coords, xhi=xhi, xlo=xlo,
                  yhi=yhi, ylo=ylo, vmax=vmax, vmin=vmin, respacing=np.array(resp), scale=np.float64(scale),
                  op_batch=np.int64(op.batch_size))
    return model, op, arrays, S, L, Ns, resp, scale, seed


def gen(case):
    from ConditionalDiffusionGeneration.src.guided_diffusion.condition_methods import get_conditioning_method
    from ConditionalDiffusionGeneration.src.guided_diffusion.gaussian_diffusion import create_sampler
    from ConditionalDiffusionGeneration.src.guided_diffusion.measurements import get_noise

    model, op, arrays, S, L, Ns, resp, scale, seed = build(case)
    T = S
    # a measurement of a "true" latent through the same operator
    x_true = torch.from_numpy(synth.uniform(seed, "xtrue", (1, 1, T, L), -0.9, 0.9))
    with torch.no_grad():
        y = op.forward(x_true)                          # (T, Ns, 3)
    mask = torch.ones_like(y)
    noiser = get_noise(sigma=0.0, name="gaussian")
    cond = get_conditioning_method(operator=op, noiser=noiser, name="ps", scale=scale)
    sampler = create_sampler(sampler="ddpm", steps=1000, noise_schedule="cosine", model_mean_type="epsilon",
                             model_var_type="fixed_large", dynamic_threshold=False, clip_denoised=True,
                             rescale_timesteps=False, timestep_respacing=resp)
    rec = {"x0": [], "sample": [], "img": [], "dist": []}

    def cond_fn(x_t, measurement, noisy_measurement, x_prev, x_0_hat):
        rec["x0"].append(x_0_hat.detach().clone())
        rec["sample"].append(x_t.detach().clone())
        img, dist = cond.conditioning(x_t=x_t, measurement=measurement, noisy_measurement=noisy_measurement,
                                      x_prev=x_prev, x_0_hat=x_0_hat)
        rec["img"].append(img.detach().clone())
        rec["dist"].append(float(dist.detach()))
        return img, dist

    draws = []
    real = torch.randn_like

    def recording_randn_like(t, *a, **k):
        out = real(t, *a, **k)
        draws.append(out.detach().clone())
        return out

    torch.manual_seed(seed)
    x_start = torch.randn(1, 1, T, L)
    torch.randn_like = recording_randn_like
    try:
        out = sampler.p_sample_loop(model=model, x_start=x_start, measurement=mask * y, measurement_cond_fn=cond_fn,
                                    record=False, save_root=None)
    finally:
        torch.randn_like = real
    n = len(rec["img"])
    assert len(draws) == 2 * n, (len(draws), n)
    arrays.update(x_start=x_start.detach().numpy(), x_true=x_true.numpy(), measurement=y.numpy(),
                  step_noise=torch.stack(draws[0::2]).numpy(), x0=torch.stack(rec["x0"]).numpy(),
                  sample=torch.stack(rec["sample"]).numpy(), img=torch.stack(rec["img"]).numpy(),
                  dist=np.array(rec["dist"]), out=out.detach().numpy(),
                  timestep_map=np.array(sampler.timestep_map, dtype=np.int64))
    path = os.path.join(HERE, f"{case}.npz")
    np.savez_compressed(path, **arrays)
    print(f"wrote {path} ({os.path.getsize(path) / 1024:.1f} KiB), steps {n}, dist {rec['dist'][0]:.4f} -> "
          f"{rec['dist'][-1]:.4f}")


if __name__ == "__main__":
    for case in CASES:
        gen(case)
