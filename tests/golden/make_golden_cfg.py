"""Golden fixtures at the BASELINE.json configuration shapes, made by running the
REFERENCE (round 2: parity at config widths, not just fixture scale).

Run in the build container only (the reference tree does not exist on the GPU
box):

    python tests/golden/make_golden_cfg.py [trajB] [trajE] [cfgA] [dpsD] [case4op] [case4dps] [case4steps]

Same conventions as make_golden.py / make_golden_dps.py: the reference is
imported read-only from /root/reference with bytecode writing off, weights are
``confild_amd.synth`` (regenerated from the seed on the GPU box, never stored),
and the only shim is the in-process ``torch.utils.tensorboard`` stand-in.  Every
normal the reference draws (``th.randn_like`` per step) is replaced, for the
duration of the run, by ``noise_for(tag, k, shape)`` -- a counter-based stream
the GPU tests regenerate -- so no noise tensor is stored.

Fixtures
  * golden_trajB.npz  -- config B: the full 256-step DDPM reverse loop
    (U/src/gaussian_diffusion.py:441-535, respacing "256") of the 64x64 U-Net
    at B = 1, samples at checkpoint steps + the final latent;
  * golden_trajE.npz  -- config E: two 20-step segments (indices 999..980 and
    19..0) of the 1000-step DDPM loop of the 128x128 default-mult U-Net at
    B = 1 through the reference's p_sample, sample and x0_hat per step;
  * golden_trajE100.npz -- config E: 100 consecutive steps (indices 599..500)
    of the same loop, sample and x0_hat every 10 steps and at the end;
  * golden_case4steps.npz -- the real Case4 loop: 10 consecutive DDPM + 'ps'
    steps (indices 500..491) at 384^2: per step the residual norm, image and
    x0_hat on a 4x-strided subgrid and whole-image checksums; the final image;
  * golden_cfgA.npz   -- config A end to end: the DDIM-50 loop
    (gaussian_diffusion.py:625-707) of the 32x32 mult-(1,2,3,4) U-Net, the
    latent de-normalisation of scripts/inference.py:59-61 and the CNF decode of
    all 32 latent rows on 1000 coordinates with SIRENAutodecoder_film(2, 32, 3,
    10, 128) (nf_networks.py:480-495, normalize.py:100-114);
  * golden_dpsD.npz   -- config D widths: DPS steps (C/gaussian_diffusion.py:
    181-199, condition_methods.py:31-47,81-90) with the 64x64 U-Net and a
    SIREN(3, 64, 3, 15, 384) Case4 operator at 10 sensors;
  * golden_case4op.npz -- the Case4 operator built by its FILE constructor
    (measurements.py:184-217: coords.npy, max/min .npy, a normaliser file with
    x_normalizer_params / y_normalizer0u_params / y_normalizer0l_params, a
    checkpoint_*.pt of the hard-coded SIREN(3, 384, 3, 15, 384)) and its
    forward on a (1, 1, 384, 384) latent;
  * golden_case4dps.npz -- the real Case4 notebook shapes
    (inference_phy_random_sensor.ipynb cells 11-23): the 384x384 U-Net with
    channel_mult "1, 1, 2, 2, 4, 4" (108.4 M parameters) and that operator, one
    DDPM+'ps' step at index 500 of 1000.
"""
from __future__ import annotations

import os
import sys
import tempfile
import time
import types

sys.dont_write_bytecode = True
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [HERE, REPO, REF, os.path.join(REF, "UnconditionalDiffusionTraining_and_Generation"),
                os.path.join(REF, "ConditionalNeuralField")]

_tb = types.ModuleType("torch.utils.tensorboard")
_tb.SummaryWriter = object
sys.modules["torch.utils.tensorboard"] = _tb

import numpy as np  # noqa: E402
import torch  # noqa: E402

from confild_amd import synth  # noqa: E402
from cfg_cases import (CASE4_OP, CASE4_STEPS, CFG_A, CNF_INF, DPS_D, POST, TRAJ_B, TRAJ_E, TRAJ_E100, TRAJ_E1000,  # noqa: E402
                       case4_files,
                       cnf_inference_coords, cnf_inference_files, noise_for, post_inputs, unet_weights)

torch.set_num_threads(8)


def _save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    print(f"wrote {path} ({os.path.getsize(path) / 1024:.1f} KiB)", flush=True)


class _Noise:
    """Replaces torch.randn_like for the duration of a reference run with the
    counter-based stream noise_for(tag, k, shape), in draw order."""

    def __init__(self, tag):
        self.tag, self.k, self.real = tag, 0, torch.randn_like

    def __call__(self, x, *a, **kw):
        out = torch.from_numpy(noise_for(self.tag, self.k, tuple(x.shape))).to(x.dtype)
        self.k += 1
        return out

    def __enter__(self):
        torch.randn_like = self
        return self

    def __exit__(self, *exc):
        torch.randn_like = self.real


def _ref_unet(kw, seed):
    from src.script_util import create_model
    torch.manual_seed(0)
    m = create_model(**kw)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in unet_weights(m.state_dict(), seed).items()})
    return m.eval()


# ---------------------------------------------------------------------------
def gen_trajB():
    from src.script_util import create_gaussian_diffusion
    c = TRAJ_B
    m = _ref_unet(c["unet"], c["seed"])
    diff = create_gaussian_diffusion(steps=1000, noise_schedule="cosine", timestep_respacing=c["respacing"])
    shape = (c["B"], 1, c["image_size"], c["image_size"])
    x_T = torch.from_numpy(noise_for(c["tag"] + "/xT", 0, shape))
    samples, x0s = {}, {}
    t0 = time.time()
    with _Noise(c["tag"]), torch.no_grad():
        for k, out in enumerate(diff.p_sample_loop_progressive(m, shape, noise=x_T)):
            if k in c["checkpoints"]:
                samples[k] = out["sample"].numpy()
                x0s[k] = out["pred_xstart"].numpy()
            final = out["sample"]
    print(f"trajB: {diff.num_timesteps} steps in {time.time() - t0:.1f} s")
    ks = sorted(samples)
    _save("golden_trajB.npz", checkpoints=np.array(ks, dtype=np.int64), samples=np.stack([samples[k] for k in ks]),
          pred_xstart=np.stack([x0s[k] for k in ks]), final=final.numpy(),
          timestep_map=np.array(diff.timestep_map, dtype=np.int64))


# ---------------------------------------------------------------------------
def gen_trajE():
    """config E: two 20-step segments of the 1000-step DDPM loop of the 128^2
    U-Net (the reference's p_sample, gaussian_diffusion.py:395-439), B = 1."""
    from src.script_util import create_gaussian_diffusion
    c = TRAJ_E
    m = _ref_unet(c["unet"], c["seed"])
    diff = create_gaussian_diffusion(steps=1000, noise_schedule="cosine", timestep_respacing="")
    S = c["image_size"]
    shape = (1, 1, S, S)
    out_arrays = {}
    t0 = time.time()
    for start, n in c["segments"]:
        x = torch.from_numpy(noise_for(f"{c['tag']}/x{start}", 0, shape))
        samples, x0s = [], []
        with _Noise(f"{c['tag']}/{start}"), torch.no_grad():
            for i in range(start, start - n, -1):
                out = diff.p_sample(m, x, torch.tensor([i]), clip_denoised=True)
                x = out["sample"]
                samples.append(x.numpy())
                x0s.append(out["pred_xstart"].numpy())
        keep = list(c["keep"])
        out_arrays[f"samples{start}"] = np.stack([samples[k] for k in keep])
        out_arrays[f"pred_xstart{start}"] = np.stack([x0s[k] for k in keep])
    print(f"trajE: {sum(n for _, n in c['segments'])} steps in {time.time() - t0:.1f} s")
    _save("golden_trajE.npz", keep=np.array(c["keep"], dtype=np.int64), **out_arrays)


def gen_trajE100():
    """config E: 100 consecutive steps (599..500) of the 1000-step DDPM loop of the
    128^2 U-Net through the reference's p_sample, B = 1, from a seeded x."""
    from src.script_util import create_gaussian_diffusion
    c = TRAJ_E100
    m = _ref_unet(TRAJ_E["unet"], TRAJ_E["seed"])
    diff = create_gaussian_diffusion(steps=1000, noise_schedule="cosine", timestep_respacing="")
    S = TRAJ_E["image_size"]
    shape = (1, 1, S, S)
    x = torch.from_numpy(noise_for(f"{c['tag']}/x", 0, shape))
    samples, x0s = [], []
    t0 = time.time()
    with _Noise(f"{c['tag']}/steps"), torch.no_grad():
        for i in range(c["start"], c["start"] - c["n"], -1):
            out = diff.p_sample(m, x, torch.tensor([i]), clip_denoised=True)
            x = out["sample"]
            samples.append(x.numpy())
            x0s.append(out["pred_xstart"].numpy())
    print(f"trajE100: {c['n']} steps in {time.time() - t0:.1f} s")
    keep = list(c["keep"])
    _save("golden_trajE100.npz", keep=np.array(keep, dtype=np.int64), samples=np.stack([samples[k] for k in keep]),
          pred_xstart=np.stack([x0s[k] for k in keep]))


def gen_trajE1000():
    """config E: the whole 1000-step DDPM loop (999..0) of the 128^2 U-Net through
    the reference's p_sample, B = 1, from a seeded x_T; sample and x0_hat every
    100 steps and at the end."""
    from src.script_util import create_gaussian_diffusion
    c = TRAJ_E1000
    m = _ref_unet(TRAJ_E["unet"], TRAJ_E["seed"])
    diff = create_gaussian_diffusion(steps=1000, noise_schedule="cosine", timestep_respacing="")
    S = TRAJ_E["image_size"]
    shape = (1, 1, S, S)
    x = torch.from_numpy(noise_for(f"{c['tag']}/x", 0, shape))
    keep = list(c["keep"])
    samples, x0s = [], []
    t0 = time.time()
    with _Noise(f"{c['tag']}/steps"), torch.no_grad():
        for k, i in enumerate(range(999, -1, -1)):
            out = diff.p_sample(m, x, torch.tensor([i]), clip_denoised=True)
            x = out["sample"]
            if k in keep:
                samples.append(x.numpy())
                x0s.append(out["pred_xstart"].numpy())
    print(f"trajE1000: 1000 steps in {time.time() - t0:.1f} s")
    _save("golden_trajE1000.npz", keep=np.array(keep, dtype=np.int64), samples=np.stack(samples),
          pred_xstart=np.stack(x0s))


# ---------------------------------------------------------------------------
def gen_cfgA():
    from ConditionalNeuralField.cnf.nf_networks import SIRENAutodecoder_film
    from ConditionalNeuralField.cnf.utils.normalize import Normalizer_ts
    from src.script_util import create_gaussian_diffusion
    c = CFG_A
    m = _ref_unet(c["unet"], c["seed"])
    diff = create_gaussian_diffusion(steps=1000, noise_schedule="cosine", timestep_respacing=c["respacing"])
    S = c["image_size"]
    shape = (1, 1, S, S)
    x_T = torch.from_numpy(noise_for(c["tag"] + "/xT", 0, shape))
    with _Noise(c["tag"]), torch.no_grad():
        gen = diff.ddim_sample_loop(m, shape, noise=x_T, eta=0.0)[:, 0]           # (1, T, L)
    vmax, vmin = torch.tensor(c["vmax"]), torch.tensor(c["vmin"])
    lat = (gen + 1) * (vmax - vmin) / 2. + vmin                                     # inference.py:61
    d, L, co, nh, H = c["siren"]
    nf = SIRENAutodecoder_film(d, L, co, nh, H)
    nf.load_state_dict({k: torch.from_numpy(v) for k, v in synth.siren_state_dict(c["siren_seed"], d, L, co, nh,
                                                                                   H).items()})
    N = c["N"]
    coords = synth.uniform(c["siren_seed"], "cfgA/coords", (N, d), 0.0, 1.0)
    yhi = synth.uniform(c["siren_seed"], "cfgA/yhi", (1, N, co), 0.5, 2.0)
    ylo = -synth.uniform(c["siren_seed"], "cfgA/ylo", (1, N, co), 0.5, 2.0)
    xn = Normalizer_ts(params=(torch.ones(1, d), torch.zeros(1, d)), method="-11", dim=0)
    yn = Normalizer_ts(params=(torch.from_numpy(yhi), torch.from_numpy(ylo)), method="-11", dim=0)
    rows = lat.reshape(-1, L)
    with torch.no_grad():   # trainer.infer per latent row (train.py:265-279, inference.py:75-77)
        fields = torch.cat([yn.denormalize(nf(xn.normalize(torch.from_numpy(coords)), rows[i:i + 1][:, None]))
                            for i in range(rows.shape[0])])
    _save("golden_cfgA.npz", latent=gen.numpy(), latent_denorm=lat.numpy(), coords=coords, ymax=yhi, ymin=ylo,
          fields=fields.numpy(), timestep_map=np.array(diff.timestep_map, dtype=np.int64))


# ---------------------------------------------------------------------------
def _ref_dps_step(model, op, sampler, x, idx, measurement, scale, tag):
    """One iteration of C/gaussian_diffusion.py:181-199 through the reference's
    own p_sample, q_sample and PosteriorSampling.conditioning."""
    from ConditionalDiffusionGeneration.src.guided_diffusion.condition_methods import get_conditioning_method
    from ConditionalDiffusionGeneration.src.guided_diffusion.measurements import get_noise
    cond = get_conditioning_method(operator=op, noiser=get_noise(sigma=0.0, name="gaussian"), name="ps",
                                   scale=scale)
    img = x.clone()
    time_ = torch.tensor([idx] * img.shape[0])
    with _Noise(tag):
        img = img.requires_grad_()
        out = sampler.p_sample(x=img, t=time_, model=model)
        noisy = sampler.q_sample(measurement, t=time_)
        sample = out["sample"].detach().clone()   # conditioning updates x_t in place (condition_methods.py:88)
        img2, dist = cond.conditioning(x_t=out["sample"], measurement=measurement, noisy_measurement=noisy,
                                       x_prev=img, x_0_hat=out["pred_xstart"])
    return img2.detach(), out["pred_xstart"].detach(), sample, float(dist.detach())


def _sampler(respacing):
    from ConditionalDiffusionGeneration.src.guided_diffusion.gaussian_diffusion import create_sampler
    return create_sampler(sampler="ddpm", steps=1000, noise_schedule="cosine", model_mean_type="epsilon",
                          model_var_type="fixed_large", dynamic_threshold=False, clip_denoised=True,
                          rescale_timesteps=False, timestep_respacing=respacing)


def _guided_unet(kw, seed, path=None):
    from ConditionalDiffusionGeneration.src.guided_diffusion.unet import create_model
    torch.manual_seed(0)
    if path is not None:   # the notebook's way: create_model(..., model_path=ema file)
        return create_model(**kw, model_path=path).eval()
    m = create_model(**kw, model_path="")
    m.load_state_dict({k: torch.from_numpy(v) for k, v in unet_weights(m.state_dict(), seed).items()})
    return m.eval()


def gen_dpsD():
    from ConditionalDiffusionGeneration.src.guided_diffusion import measurements as ms
    from cnf.nf_networks import SIRENAutodecoder_film
    from cnf.utils.normalize import Normalizer_ts
    c = DPS_D
    model = _guided_unet(c["unet"], c["seed"])
    d, L, co, nh, H = c["siren"]
    nf = SIRENAutodecoder_film(d, L, co, nh, H)
    nf.load_state_dict({k: torch.from_numpy(v) for k, v in synth.siren_state_dict(c["siren_seed"], d, L, co, nh,
                                                                                   H).items()})
    nf.eval()
    s = c["siren_seed"]
    op = ms.Case4Operator.__new__(ms.Case4Operator)
    op.device = torch.device("cpu")
    coords = synth.uniform(s, "dpsD/sensors", (c["Ns"], d), 0.0, 1.0)
    op.coords = torch.from_numpy(coords)
    xhi, xlo = np.ones((1, d), np.float32), np.zeros((1, d), np.float32)
    yhi = synth.uniform(s, "dpsD/yhi", (co,), 0.5, 2.0)
    ylo = -synth.uniform(s, "dpsD/ylo", (co,), 0.5, 2.0)
    op.x_normalizer = Normalizer_ts(method="-11", dim=0, params=(torch.from_numpy(xhi), torch.from_numpy(xlo)))
    op.y_normalizer = Normalizer_ts(method="-11", dim=0, params=(torch.from_numpy(yhi), torch.from_numpy(ylo)))
    op.model = nf
    vmax = synth.uniform(s, "dpsD/vmax", (L,), 1.0, 2.0)
    vmin = -synth.uniform(s, "dpsD/vmin", (L,), 1.0, 2.0)
    op.max_val, op.min_val = torch.from_numpy(vmax), torch.from_numpy(vmin)
    op.batch_size = 16
    S = c["unet"]["image_size"]
    x_true = torch.from_numpy(synth.uniform(s, "dpsD/xtrue", (1, 1, S, L), -0.9, 0.9))
    with torch.no_grad():
        y = op.forward(x_true)
    sampler = _sampler(c["respacing"])
    out = dict(coords=coords, xhi=xhi, xlo=xlo, yhi=yhi, ylo=ylo, vmax=vmax, vmin=vmin, measurement=y.numpy(),
               indices=np.array(c["indices"], dtype=np.int64))
    for j, idx in enumerate(c["indices"]):
        x = torch.from_numpy(synth.normal(s, f"dpsD/x{idx}", (1, 1, S, L)))
        t0 = time.time()
        img, x0, sample, dist = _ref_dps_step(model, op, sampler, x, idx, y, c["scale"], f"{c['tag']}/{idx}")
        print(f"dpsD step {idx}: {time.time() - t0:.1f} s, dist {dist:.5f}")
        out.update({f"img{j}": img.numpy(), f"x0{j}": x0.numpy(), f"sample{j}": sample.numpy(),
                    f"dist{j}": np.float64(dist)})
    _save("golden_dpsD.npz", **out)


# ---------------------------------------------------------------------------
def _case4_operator(tmp):
    from ConditionalDiffusionGeneration.src.guided_diffusion.measurements import get_operator
    paths = case4_files(tmp)
    return get_operator(device=torch.device("cpu"), name="case4", coords_path=paths["coords"],
                        max_val_path=paths["max"], min_val_path=paths["min"],
                        normalizer_params_path=paths["normalizer"], ckpt_path=paths["ckpt"],
                        batch_size=CASE4_OP["batch_size"])


def gen_case4op():
    c = CASE4_OP
    with tempfile.TemporaryDirectory() as tmp:
        op = _case4_operator(tmp)
        x = torch.from_numpy(synth.uniform(c["seed"], "case4op/x", (1, 1, c["T"], c["L"]), -0.95, 0.95))
        t0 = time.time()
        with torch.no_grad():
            A = op.forward(x)
        print(f"case4op forward {tuple(A.shape)} in {time.time() - t0:.1f} s")
    _save("golden_case4op.npz", A=A.numpy())


def gen_case4dps():
    c = CASE4_OP
    with tempfile.TemporaryDirectory() as tmp:
        op = _case4_operator(tmp)
        kw = c["unet"]
        from ConditionalDiffusionGeneration.src.guided_diffusion.unet import create_model
        torch.manual_seed(0)
        shapes = {k: tuple(v.shape) for k, v in create_model(**kw, model_path="").state_dict().items()}
        ema = os.path.join(tmp, "ema_0.9999_400000.pt")
        torch.save({k: torch.from_numpy(v) for k, v in synth.unet_state_dict(c["unet_seed"], shapes).items()}, ema)
        model = _guided_unet(kw, c["unet_seed"], path=ema)      # the notebook's create_model(model_path=...)
        x_true = torch.from_numpy(synth.uniform(c["seed"], "case4op/x", (1, 1, c["T"], c["L"]), -0.95, 0.95))
        with torch.no_grad():
            y = op.forward(x_true)                               # the measurement: (384, 10, 3)
        sampler = _sampler("")
        idx = c["dps_index"]
        x = torch.from_numpy(synth.normal(c["seed"], f"case4dps/x{idx}", (1, 1, c["T"], c["L"])))
        t0 = time.time()
        img, x0, sample, dist = _ref_dps_step(model, op, sampler, x, idx, y, 1.0, f"case4dps/{idx}")
        print(f"case4dps step {idx}: {time.time() - t0:.1f} s, dist {dist:.5f}")
        # eps is recovered exactly enough from the stored inputs: keep x0 (pre-clamp info lost) and img
    _save("golden_case4dps.npz", img=img.numpy(), x0=x0.numpy(), dist=np.float64(dist), index=np.int64(idx),
          nparams=np.int64(sum(int(np.prod(s)) for s in shapes.values())))


def gen_case4steps():
    """The real Case4 loop over CASE4_STEPS["n"] consecutive DDPM + 'ps' steps (the
    notebook's p_sample_loop body, C/gaussian_diffusion.py:181-199), each with its
    own recorded noise, from a synth state at index CASE4_STEPS["start"]."""
    c, cs = CASE4_OP, CASE4_STEPS
    with tempfile.TemporaryDirectory() as tmp:
        op = _case4_operator(tmp)
        kw = c["unet"]
        from ConditionalDiffusionGeneration.src.guided_diffusion.unet import create_model
        torch.manual_seed(0)
        shapes = {k: tuple(v.shape) for k, v in create_model(**kw, model_path="").state_dict().items()}
        ema = os.path.join(tmp, "ema_0.9999_400000.pt")
        torch.save({k: torch.from_numpy(v) for k, v in synth.unet_state_dict(c["unet_seed"], shapes).items()}, ema)
        model = _guided_unet(kw, c["unet_seed"], path=ema)
        x_true = torch.from_numpy(synth.uniform(c["seed"], "case4op/x", (1, 1, c["T"], c["L"]), -0.95, 0.95))
        with torch.no_grad():
            y = op.forward(x_true)
        sampler = _sampler("")
        x = torch.from_numpy(synth.normal(c["seed"], f"case4steps/x{cs['start']}", (1, 1, c["T"], c["L"])))
        imgs, x0s, dists = [], [], []
        t0 = time.time()
        for idx in range(cs["start"], cs["start"] - cs["n"], -1):
            x, x0, _, dist = _ref_dps_step(model, op, sampler, x, idx, y, 1.0, f"case4steps/{idx}")
            imgs.append(x.numpy())
            x0s.append(x0.numpy())
            dists.append(dist)
            print(f"case4 step {idx}: dist {dist:.5f} ({time.time() - t0:.0f} s)", flush=True)
    imgs, x0s = np.stack(imgs), np.stack(x0s)
    # compact: every step on a 4x-strided 96x96 subgrid, whole-image checksums, the final image in full
    _save("golden_case4steps.npz", dists=np.array(dists), img_sub=imgs[..., ::4, ::4].copy(),
          x0_sub=x0s[..., ::4, ::4].copy(), img_sum=imgs.astype(np.float64).sum(axis=(1, 2, 3, 4)),
          img_absmax=np.abs(imgs).max(axis=(1, 2, 3, 4)), img_final=imgs[-1])


# ---------------------------------------------------------------------------
def gen_cnfinf():
    """CNF_inference (inference_function.py:79-304): normal and is_pub checkpoints,
    predict on given indices, create_coordinates_grid from the data shape."""
    from ConditionalNeuralField.cnf.inference_function import CNF_inference
    out = {}
    for name in CNF_INF:
        with tempfile.TemporaryDirectory() as tmp:
            f = cnf_inference_files(tmp, name)
            inf = CNF_inference(checkpoint_path=f["checkpoint"], config_path=f["config"], data_path=f["data"],
                                device="cpu", is_pub=CNF_INF[name]["is_pub"])
            coords = torch.from_numpy(cnf_inference_coords(name))
            pred = inf.predict(coords, CNF_INF[name]["idx"], batch_size=2)
            out[f"{name}_pred"] = pred.numpy()
            out[f"{name}_grid"] = inf.create_coordinates_grid().numpy()
            out[f"{name}_grid_shape"] = inf.create_coordinates_grid(
                tuple(CNF_INF[name]["data_shape"][1:-1])[:3] if len(CNF_INF[name]["data_shape"]) > 3
                else (5, 4)).numpy()
            lat_one = inf.latents(torch.LongTensor([1, 2]))
            out[f"{name}_latent_shape"] = np.array(lat_one.shape, dtype=np.int64)
    _save("golden_cnfinf.npz", **out)


def gen_post():
    """The Case4 notebook's decode + ReconstructFrame (cells 26-32) at small scale."""
    from cnf.inference_function import ReconstructFrame, decoder
    from cnf.nf_networks import SIRENAutodecoder_film
    from cnf.utils.normalize import Normalizer_ts
    from einops import rearrange
    c = POST
    d, L, co, nh, H = c["siren"]
    mask, coords, lat, xhi, xlo, yhi, ylo = post_inputs()
    nf = SIRENAutodecoder_film(d, L, co, nh, H)
    nf.load_state_dict({k: torch.from_numpy(v) for k, v in synth.siren_state_dict(c["seed"], d, L, co, nh,
                                                                                   H).items()})
    xn = Normalizer_ts(method="-11", dim=0, params=(torch.from_numpy(xhi), torch.from_numpy(xlo)))
    yn = Normalizer_ts(method="-11", dim=0, params=(torch.from_numpy(yhi), torch.from_numpy(ylo)))
    fields = decoder(torch.from_numpy(coords), torch.from_numpy(lat), nf, xn, yn, batch_size=4, device="cpu")
    fields = rearrange(fields, "(s t) co c -> s t co c", t=c["t"])
    frames = [ReconstructFrame(fields[ss, kk].numpy(), mask=mask, shape=c["grid"], fill_value=0.)
              for ss in range(c["s"]) for kk in range(c["t"])]
    frames = rearrange(np.stack(frames), "(s t) x y z c -> s t x y z c", t=c["t"])
    nanf = ReconstructFrame(fields[0, 0].numpy(), mask=mask, shape=c["grid"])   # default fill: NaN
    _save("golden_post.npz", frames=frames.astype(np.float32), nan_frame=nanf.astype(np.float32))


GEN = {"trajB": gen_trajB, "trajE": gen_trajE, "trajE100": gen_trajE100, "trajE1000": gen_trajE1000, "case4steps": gen_case4steps, "cfgA": gen_cfgA, "dpsD": gen_dpsD, "case4op": gen_case4op, "case4dps": gen_case4dps,
       "cnfinf": gen_cnfinf, "post": gen_post}

if __name__ == "__main__":
    print("torch", torch.__version__)
    for name in (sys.argv[1:] or list(GEN)):
        GEN[name]()
