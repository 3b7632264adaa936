"""Generate the golden fixtures by running the REFERENCE implementation.

Run in the build container only (the reference tree does not exist on the GPU
box):

    python tests/golden/make_golden.py

It imports semihkacmaz/CoNFiLD from /root/reference (read-only; bytecode
writing is disabled), feeds it deterministic synthetic weights from
``confild_amd.synth`` and records inputs and outputs as small ``.npz`` files
next to this script.  The reference's own test suite pins nothing for this
path, so these fixtures are what pins the oracle.

The only shim is an in-process stand-in module for ``torch.utils.tensorboard``
(not installed here; imported at ConditionalNeuralField/scripts/train.py:13 and
never used on the inference path).
"""
from __future__ import annotations

import os
import sys
import tempfile
import types

sys.dont_write_bytecode = True
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, REF, os.path.join(REF, "UnconditionalDiffusionTraining_and_Generation"),
                os.path.join(REF, "ConditionalNeuralField")]

_tb = types.ModuleType("torch.utils.tensorboard")
_tb.SummaryWriter = object
sys.modules["torch.utils.tensorboard"] = _tb

import numpy as np  # noqa: E402
import torch  # noqa: E402
import yaml  # noqa: E402

from confild_amd import synth  # noqa: E402

torch.set_num_threads(8)


def _save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    print(f"wrote {path} ({os.path.getsize(path)/1024:.1f} KiB)")


# ---------------------------------------------------------------------------
# 1. schedules + respacing (U/src/gaussian_diffusion.py:18-169, respace.py)
# ---------------------------------------------------------------------------
def gen_schedules():
    from src import gaussian_diffusion as gd
    from src.respace import space_timesteps
    from src.script_util import create_gaussian_diffusion

    out = {}
    for sched in ("cosine", "linear"):
        out[f"{sched}_1000_betas"] = gd.get_named_beta_schedule(sched, 1000)
    cases = {"id": "", "s256": "256", "ddim50": "ddim50", "ddim5": "ddim5", "s8": "8",
             "s10_20_30": "10,20,30", "s250": "250", "s100": "100"}
    for tag, resp in cases.items():
        d = create_gaussian_diffusion(steps=1000, noise_schedule="cosine", timestep_respacing=resp)
        out[f"{tag}_timestep_map"] = np.array(d.timestep_map, dtype=np.int64)
        for attr in ("betas", "alphas_cumprod", "alphas_cumprod_prev", "sqrt_recip_alphas_cumprod",
                     "sqrt_recipm1_alphas_cumprod", "posterior_variance",
                     "posterior_log_variance_clipped", "posterior_mean_coef1", "posterior_mean_coef2"):
            out[f"{tag}_{attr}"] = getattr(d, attr)
    # linear schedule with respacing too
    d = create_gaussian_diffusion(steps=1000, noise_schedule="linear", timestep_respacing="50")
    out["lin50_timestep_map"] = np.array(d.timestep_map, dtype=np.int64)
    out["lin50_betas"] = d.betas
    # space_timesteps error behaviour: ddim256 @ 1000 is impossible (respace.py:30-37)
    errs = []
    for args in ((1000, "ddim256"), (10, "20"), (100, "ddim7")):
        try:
            space_timesteps(*args)
            errs.append("ok")
        except ValueError as e:
            errs.append("ValueError:" + str(e))
    out["space_errors"] = np.array(errs)
    out["space_300_10_15_20"] = np.array(sorted(space_timesteps(300, [10, 15, 20])), dtype=np.int64)
    _save("schedules.npz", **out)


# ---------------------------------------------------------------------------
# 2. U-Net forward (U/src/unet.py:396-663 via script_util.create_model)
# ---------------------------------------------------------------------------
UNET_CASES = {
    # name: (create_model kwargs, batch, seed)
    "tiny16": (dict(image_size=16, num_channels=32, num_res_blocks=1, channel_mult="1,2",
                    num_heads=4, num_head_channels=16, attention_resolutions="8"), 2, 11),
    "small32": (dict(image_size=32, num_channels=32, num_res_blocks=2, channel_mult="1,2,3",
                     num_heads=4, num_head_channels=32, attention_resolutions="16,8"), 2, 12),
    "heads16": (dict(image_size=16, num_channels=64, num_res_blocks=1, channel_mult="1,1",
                     num_heads=2, num_head_channels=-1, attention_resolutions="16,8"), 1, 13),
    # BASELINE.json configs at full width (weights regenerated from the seed on
    # the GPU box; only inputs/outputs are stored)
    "cfgA32": (dict(image_size=32, num_channels=128, num_res_blocks=2, channel_mult="1,2,3,4",
                    num_heads=4, num_head_channels=64, attention_resolutions="32,16,8"), 1, 1234),
    "cfgB64": (dict(image_size=64, num_channels=128, num_res_blocks=2, channel_mult=None,
                    num_heads=4, num_head_channels=64, attention_resolutions="32,16,8"), 1, 1234),
    "cfgE128": (dict(image_size=128, num_channels=128, num_res_blocks=2, channel_mult=None,
                     num_heads=4, num_head_channels=64, attention_resolutions="32,16,8"), 1, 1234),
}


def unet_inputs(case, B, image_size, seed):
    x = synth.normal(seed, f"{case}/x", (B, 1, image_size, image_size))
    t = (np.arange(B, dtype=np.int64) * 337 + 41) % 1000
    return x, t


def gen_unet():
    from src.script_util import create_model
    for case, (kw, B, seed) in UNET_CASES.items():
        torch.manual_seed(0)
        m = create_model(**kw)
        shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
        sd = synth.unet_state_dict(seed, shapes)
        m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
        m.eval()
        x, t = unet_inputs(case, B, kw["image_size"], seed)
        with torch.no_grad():
            eps = m(torch.from_numpy(x), torch.from_numpy(t)).numpy()
        _save(f"unet_{case}.npz", x=x, t=t, eps=eps, seed=np.int64(seed),
              keys=np.array(list(shapes.keys())), kwargs=np.array(repr(kw)),
              nparams=np.int64(sum(int(np.prod(s)) for s in shapes.values())))


# ---------------------------------------------------------------------------
# 3. sampler trajectories with the noise recorded (gaussian_diffusion.py:426-628)
# ---------------------------------------------------------------------------
def _record_noise(shape, nsteps, seed=42):
    g = torch.Generator().manual_seed(seed)
    n0 = torch.randn(*shape, generator=g)
    steps = [torch.randn(*shape, generator=g) for _ in range(nsteps)]
    return n0, torch.stack(steps)


def gen_trajectories():
    from src.script_util import create_model, create_gaussian_diffusion
    kw, B, seed = UNET_CASES["tiny16"]
    torch.manual_seed(0)
    m = create_model(**kw)
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    sd = synth.unet_state_dict(seed, shapes)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m.eval()
    shape = (B, 1, 16, 16)
    for tag, resp, loop in (("ddpm8", "8", "p_sample_loop_progressive"),
                            ("ddim5", "ddim5", "ddim_sample_loop_progressive")):
        diff = create_gaussian_diffusion(steps=1000, noise_schedule="cosine", timestep_respacing=resp)
        n = diff.num_timesteps
        n0, steps = _record_noise(shape, n)
        # the reference draws from the global generator: seed it identically
        torch.manual_seed(42)
        samples, xstarts = [], []
        for out in getattr(diff, loop)(m, shape):
            samples.append(out["sample"].numpy())
            xstarts.append(out["pred_xstart"].numpy())
        _save(f"traj_{tag}.npz", noise0=n0.numpy(), noise=steps.numpy(),
              samples=np.stack(samples), pred_xstart=np.stack(xstarts),
              timestep_map=np.array(diff.timestep_map, dtype=np.int64))


# ---------------------------------------------------------------------------
# 4. SIREN / FiLM CNF (N/cnf/nf_networks.py:443-495) + normalizers
# ---------------------------------------------------------------------------
SIREN_CASES = {
    # name: (d, L, c, nh, H, N coords, b latents, seed)
    "s2d": (2, 16, 3, 3, 32, 100, 4, 21),
    "s3d": (3, 24, 3, 4, 48, 77, 3, 22),
    "caseA": (2, 32, 3, 10, 128, 64, 5, 23),
    "case4w": (3, 64, 3, 15, 384, 40, 2, 24),
}


def gen_siren():
    from ConditionalNeuralField.cnf.nf_networks import SIRENAutodecoder_film
    from ConditionalNeuralField.cnf.utils.normalize import Normalizer_ts
    for case, (d, L, c, nh, H, N, b, seed) in SIREN_CASES.items():
        net = SIRENAutodecoder_film(d, L, c, nh, H)
        sd = synth.siren_state_dict(seed, d, L, c, nh, H)
        net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
        coords = synth.uniform(seed, f"{case}/coords", (N, d), 0.0, 1.0)
        lat = synth.normal(seed, f"{case}/lat", (b, L)) * np.float32(0.5)
        xmin = np.zeros((1, d), np.float32)
        xmax = np.ones((1, d), np.float32)
        yhi = synth.uniform(seed, f"{case}/yhi", (1, N, c), 0.5, 2.0)
        ylo = -synth.uniform(seed, f"{case}/ylo", (1, N, c), 0.5, 2.0)
        xn = Normalizer_ts(params=(torch.from_numpy(xmax), torch.from_numpy(xmin)), method="-11", dim=0)
        yn = Normalizer_ts(params=(torch.from_numpy(yhi), torch.from_numpy(ylo)), method="-11", dim=0)
        with torch.no_grad():
            raw = net(xn.normalize(torch.from_numpy(coords))[None], torch.from_numpy(lat)[:, None])
            out = yn.denormalize(raw)
        _save(f"siren_{case}.npz", coords=coords, latents=lat, xmin=xmin, xmax=xmax,
              ymax=yhi, ymin=ylo, raw=raw.numpy(), out=out.numpy(), seed=np.int64(seed),
              dims=np.array([d, L, c, nh, H], dtype=np.int64))


# ---------------------------------------------------------------------------
# 5. trainer.infer + decoder/pass_through_model_batch surfaces
#    (N/scripts/train.py:74-279,481-528; N/cnf/inference_function.py:22-76)
# ---------------------------------------------------------------------------
def gen_trainer():
    from ConditionalNeuralField.scripts.train import trainer
    from basicutility import ReadInput as ri
    from ConditionalNeuralField.cnf.inference_function import decoder, pass_through_model_batch
    d, L, c, nh, H, N, b, seed = SIREN_CASES["s3d"]
    with tempfile.TemporaryDirectory() as tmp:
        sd = synth.siren_state_dict(seed, d, L, c, nh, H)
        xmax = torch.ones(1, d)
        xmin = torch.zeros(1, d)
        yhi = torch.from_numpy(synth.uniform(seed, "tr/yhi", (1, N, c), 0.5, 2.0))
        ylo = torch.from_numpy(-synth.uniform(seed, "tr/ylo", (1, N, c), 0.5, 2.0))
        torch.save({"x_normalizer_params": (xmax, xmin), "y_normalizer_params": (yhi, ylo)},
                   os.path.join(tmp, "normalizer_params.pt"))
        for ep in (3, 17):
            torch.save({"epoch": ep, "model_state_dict": {k: torch.from_numpy(v) * (1.0 if ep == 17 else 0.5)
                                                          for k, v in sd.items()},
                        "optim_net_dec_dict": {}, "optim_states_dict": {}, "hidden_states": {}},
                       os.path.join(tmp, f"checkpoint_{ep}.pt"))
        cfg = {"save_path": tmp, "lumped_latent": True, "normalizer": {"method": "-11", "dim": 0},
               "multiGPU": 1, "hidden_size": L, "dims": d,
               "NF": {"name": "SIRENAutodecoder_film", "out_features": c,
                      "num_hidden_layers": nh, "hidden_features": H}}
        ypath = os.path.join(tmp, "cnf.yml")
        with open(ypath, "w") as f:
            yaml.safe_dump(cfg, f)
        tr = trainer(ri.basic_input(ypath), infer_mode=True)
        tr.load(-1, siren_only=True)
        coords = torch.from_numpy(synth.uniform(seed, "tr/coords", (N, d), 0.0, 1.0))
        lat = torch.from_numpy(synth.normal(seed, "tr/lat", (b, L)))
        out = tr.infer(coords, lat)
        dec = decoder(coords, lat, tr.nf, tr.in_normalizer, tr.out_normalizer, 2, "cpu")
        with torch.no_grad():
            ptm = pass_through_model_batch(coords, lat, tr.nf, tr.in_normalizer, tr.out_normalizer, 2, "cpu")
        _save("trainer_infer.npz", coords=coords.numpy(), latents=lat.numpy(), out=out.numpy(),
              decoder=dec.numpy(), pass_through=ptm.numpy(), yhi=yhi.numpy(), ylo=ylo.numpy(),
              seed=np.int64(seed), dims=np.array([d, L, c, nh, H], dtype=np.int64))


if __name__ == "__main__":
    print("torch", torch.__version__)
    gen_schedules()
    gen_unet()
    gen_trajectories()
    gen_siren()
    gen_trainer()
    _save("meta.npz", torch_version=np.array(torch.__version__), numpy_version=np.array(np.__version__))
