"""GPU parity: the HIP path (through the C ABI) against the reference's golden
fixtures and the CPU oracle on identical inputs.

Tolerances (fp32 everywhere; the HIP kernels sum in a different order than
MKL/oneDNN on the CPU):
  * U-Net forward: max|d| / max|ref| <= 1e-5 (measured values are
    printed and recorded in DESIGN.md section 5);
  * one sampler step given the same eps and noise: bit-exact;
  * short trajectories (8 DDPM / 5 DDIM steps): max|d| <= 1e-4;
  * SIREN/FiLM decode: max|d| <= 2e-5 * max(1, max|ref|) (sin(30 x) amplifies
    argument rounding by 30).
"""
import ast

import numpy as np
import pytest
import torch

from conftest import golden
from confild_amd import _lib, synth
from confild_amd.nf_networks import SIRENAutodecoder_film
from confild_amd.normalize import Normalizer_ts
from confild_amd.script_util import create_gaussian_diffusion, create_model
from oracle import diffusion as od
from oracle import siren as osn
from oracle import unet as ou

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _unet(name):
    g = golden(f"unet_{name}.npz")
    kw = ast.literal_eval(str(g["kwargs"]))
    m = create_model(**kw)
    sd = synth.unet_state_dict(int(g["seed"]), {k: tuple(v.shape) for k, v in m.state_dict().items()})
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    return g, kw, m.to(DEV), {k: torch.from_numpy(v) for k, v in sd.items()}


@pytest.mark.parametrize("name", ["tiny16", "small32", "heads16", "cfgA32", "cfgB64", "cfgE128"])
def test_unet_forward_vs_reference_golden(hip, name):
    g, kw, m, _ = _unet(name)
    eps = m(torch.from_numpy(g["x"]).to(DEV), torch.from_numpy(g["t"]).to(DEV)).cpu().numpy()
    ref = g["eps"]
    err = np.abs(eps - ref).max() / np.abs(ref).max()
    print(f"U-Net {name} vs reference: {err:.2e}")
    assert err <= 1e-5, err


def test_unet_batch_vs_oracle_cfgB(hip):
    g, kw, m, sd = _unet("cfgB64")
    B = 3
    x = torch.from_numpy(synth.normal(5, "bx", (B, 1, 64, 64)))
    t = torch.tensor([999, 500, 0], dtype=torch.int64)
    eps = m(x.to(DEV), t.to(DEV)).cpu()
    with torch.no_grad():
        ref = ou.forward(sd, ou.Config(**kw), x, t)
    err = (eps - ref).abs().max().item() / ref.abs().max().item()
    print(f"U-Net cfgB64 B=3 vs oracle: {err:.2e}")
    assert err <= 1e-5, err
    # batch independence: sample 1 alone equals sample 1 in the batch
    e1 = m(x[1:2].to(DEV), t[1:2].to(DEV)).cpu()
    assert (e1 - eps[1:2]).abs().max().item() <= 1e-5 * ref.abs().max().item()


def test_ddpm_step_bitexact(hip):
    d = create_gaussian_diffusion(steps=1000, noise_schedule="cosine", timestep_respacing="256")
    tb = od.Tables(1000, "cosine", "256")
    B, S = 4, 64
    x = torch.from_numpy(synth.normal(1, "x", (B, 1, S, S)))
    eps = torch.from_numpy(synth.normal(2, "e", (B, 1, S, S)))
    z = torch.from_numpy(synth.normal(3, "z", (B, 1, S, S)))
    t = torch.tensor([255, 100, 1, 0], dtype=torch.int64)
    model = lambda xx, tt: eps.to(DEV)  # noqa: E731
    for kind in ("ddpm", "ddim"):
        if kind == "ddpm":
            out = d.p_sample(model, x.to(DEV), t.to(DEV), noise=z.to(DEV))
            ref, xs = od.ddpm_step(tb, x, t, eps, z)
        else:
            out = d.ddim_sample(model, x.to(DEV), t.to(DEV), noise=z.to(DEV))
            ref, xs = od.ddim_step(tb, x, t, eps, z)
        assert torch.equal(out["sample"].cpu(), ref), kind
        assert torch.equal(out["pred_xstart"].cpu(), xs), kind


@pytest.mark.parametrize("tag,resp,loop", [("ddpm8", "8", "p_sample_loop_progressive"),
                                           ("ddim5", "ddim5", "ddim_sample_loop_progressive")])
def test_trajectory_vs_reference_golden(hip, tag, resp, loop):
    tr = golden(f"traj_{tag}.npz")
    _, _, m, _ = _unet("tiny16")
    d = create_gaussian_diffusion(steps=1000, noise_schedule="cosine", timestep_respacing=resp)
    steps = list(getattr(d, loop)(m, (2, 1, 16, 16), noise=torch.from_numpy(tr["noise0"]).to(DEV),
                                  step_noise=[torch.from_numpy(n).to(DEV) for n in tr["noise"]]))
    for k, out in enumerate(steps):
        assert np.abs(out["sample"].cpu().numpy() - tr["samples"][k]).max() <= 1e-4, k
        assert np.abs(out["pred_xstart"].cpu().numpy() - tr["pred_xstart"][k]).max() <= 1e-4, k


def test_device_rng_is_normal_and_deterministic(hip):
    lib = _lib.lib()
    a = torch.empty(1 << 20, device=DEV)
    b = torch.empty(1 << 20, device=DEV)
    for buf in (a, b):
        _lib.check(lib.cfd_randn(_lib.ptr(buf), buf.numel(), 1234, 7, 0, None), "randn")
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    assert abs(a.mean().item()) < 5e-3 and abs(a.std().item() - 1) < 5e-3
    _lib.check(lib.cfd_randn(_lib.ptr(b), b.numel(), 1234, 8, 0, None), "randn")
    torch.cuda.synchronize()
    assert not torch.equal(a, b)
    # offset addressing: the second half drawn alone equals the second half of the whole
    half = torch.empty(1 << 19, device=DEV)
    _lib.check(lib.cfd_randn(_lib.ptr(half), half.numel(), 1234, 7, 1 << 19, None), "randn")
    torch.cuda.synchronize()
    assert torch.equal(half, a[1 << 19:])


def test_latent_denorm_bitexact(hip):
    x = torch.from_numpy(synth.normal(4, "lat", (8, 64, 64)))
    vmax = torch.from_numpy(synth.uniform(4, "mx", (64,), 1.0, 2.0))
    vmin = torch.from_numpy(synth.uniform(4, "mn", (64,), -2.0, -1.0))
    y = torch.empty(x.shape, device=DEV)
    xd, mxd, mnd = x.to(DEV), vmax.to(DEV), vmin.to(DEV)
    _lib.check(_lib.lib().cfd_latent_denorm(_lib.ptr(xd), _lib.ptr(y), x.numel(), _lib.ptr(mxd), _lib.ptr(mnd), 64,
                                            None), "denorm")
    ref = (x + 1) * (vmax - vmin) / 2. + vmin   # scripts/inference.py:61
    assert torch.equal(y.cpu(), ref)


def _siren(case):
    g = golden(f"siren_{case}.npz")
    d, L, c, nh, H = (int(v) for v in g["dims"])
    net = SIRENAutodecoder_film(d, L, c, nh, H)
    sd = {k: torch.from_numpy(v) for k, v in synth.siren_state_dict(int(g["seed"]), d, L, c, nh, H).items()}
    net.load_state_dict(sd)
    return g, net.to(DEV), sd


@pytest.mark.parametrize("case", ["s2d", "s3d", "caseA", "case4w"])
def test_siren_vs_reference_golden(hip, case):
    g, net, _ = _siren(case)
    xn = Normalizer_ts(params=(torch.from_numpy(g["xmax"]), torch.from_numpy(g["xmin"])), method="-11", dim=0)
    yn = Normalizer_ts(params=(torch.from_numpy(g["ymax"]), torch.from_numpy(g["ymin"])), method="-11", dim=0)
    out = net.decode(torch.from_numpy(g["coords"]).to(DEV), torch.from_numpy(g["latents"]).to(DEV)[:, None], xn, yn)
    ref = g["out"]
    assert np.abs(out.cpu().numpy() - ref).max() <= 2e-5 * max(1.0, np.abs(ref).max())
    # raw forward keeps the reference signature (coords (1, N, d), latents (b, 1, L))
    raw = net(xn.normalize(torch.from_numpy(g["coords"]))[None].to(DEV),
              torch.from_numpy(g["latents"]).to(DEV)[:, None])
    assert raw.shape == g["raw"].shape
    assert np.abs(raw.cpu().numpy() - g["raw"]).max() <= 2e-5


@pytest.mark.parametrize("dims,N,b", [((3, 64, 3, 15, 384), 4099, 3), ((3, 384, 3, 15, 384), 1000, 2),
                                      ((2, 128, 2, 17, 256), 777, 4), ((2, 32, 3, 10, 128), 1000, 2)])
def test_siren_config_widths_vs_oracle(hip, dims, N, b):
    d, L, c, nh, H = dims
    sd = {k: torch.from_numpy(v) for k, v in synth.siren_state_dict(1234, d, L, c, nh, H).items()}
    net = SIRENAutodecoder_film(d, L, c, nh, H)
    net.load_state_dict(sd)
    net.to(DEV)
    coords = torch.from_numpy(synth.uniform(7, "co", (N, d), 0.0, 1.0))
    lat = torch.from_numpy(synth.normal(11, "la", (b, L))) * 0.5
    ymax = torch.from_numpy(synth.uniform(9, "yx", (1, N, c), 0.5, 2.0))
    ymin = -torch.from_numpy(synth.uniform(9, "yn", (1, N, c), 0.5, 2.0))
    xn = Normalizer_ts(params=(torch.ones(1, d), torch.zeros(1, d)), method="-11", dim=0)
    yn = Normalizer_ts(params=(ymax, ymin), method="-11", dim=0)
    out = net.decode(coords.to(DEV), lat.to(DEV)[:, None], xn, yn).cpu()
    ref = osn.decode(sd, coords, lat, torch.ones(1, d), torch.zeros(1, d), ymax, ymin)
    assert out.shape == ref.shape
    assert (out - ref).abs().max().item() <= 2e-5 * max(1.0, ref.abs().max().item())


def test_trainer_infer_vs_reference_golden(hip, tmp_path):
    import yaml
    from confild_amd.read_input import basic_input
    from confild_amd.trainer import trainer
    from confild_amd.inference_function import decoder, pass_through_model_batch
    g = golden("trainer_infer.npz")
    d, L, c, nh, H = (int(v) for v in g["dims"])
    sd = synth.siren_state_dict(int(g["seed"]), d, L, c, nh, H)
    torch.save({"x_normalizer_params": (torch.ones(1, d), torch.zeros(1, d)),
                "y_normalizer_params": (torch.from_numpy(g["yhi"]), torch.from_numpy(g["ylo"]))},
               tmp_path / "normalizer_params.pt")
    torch.save({"epoch": 17, "model_state_dict": {k: torch.from_numpy(v) for k, v in sd.items()}},
               tmp_path / "checkpoint_17.pt")
    cfg = {"save_path": str(tmp_path), "lumped_latent": True, "normalizer": {"method": "-11", "dim": 0},
           "multiGPU": 1, "hidden_size": L, "dims": d,
           "NF": {"name": "SIRENAutodecoder_film", "out_features": c, "num_hidden_layers": nh, "hidden_features": H}}
    (tmp_path / "cnf.yml").write_text(yaml.safe_dump(cfg))
    tr = trainer(basic_input(str(tmp_path / "cnf.yml")), infer_mode=True)
    tr.load(-1, siren_only=True)
    tr.nf.to(DEV)
    coords = torch.from_numpy(g["coords"]).to(DEV)
    lat = torch.from_numpy(g["latents"]).to(DEV)
    out = tr.infer(coords, lat).cpu().numpy()
    tol = 2e-5 * max(1.0, np.abs(g["out"]).max())
    assert np.abs(out - g["out"]).max() <= tol
    dec = decoder(coords, lat, tr.nf, tr.in_normalizer, tr.out_normalizer, 2, DEV).numpy()
    assert np.abs(dec - g["decoder"]).max() <= tol
    ptm = pass_through_model_batch(coords, lat, tr.nf, tr.in_normalizer, tr.out_normalizer, 2, DEV).cpu().numpy()
    assert np.abs(ptm - g["pass_through"]).max() <= tol


def test_gpu_path_fails_loudly_on_bad_input(hip):
    _, _, m, _ = _unet("tiny16")
    with pytest.raises(ValueError):
        m(torch.zeros(1, 1, 8, 8, device=DEV), torch.zeros(1, dtype=torch.int64, device=DEV))
    x = torch.zeros(1, 1, 16, 16, device=DEV, requires_grad=True)
    with pytest.raises(NotImplementedError):
        m(x, torch.zeros(1, dtype=torch.int64, device=DEV))
