"""GPU parity of the DPS adjoint path.

* U-Net input-gradient (cfd_unet_forward_tape + cfd_unet_input_vjp) against
  torch autograd through the CPU oracle U-Net, on the reference-pinned fixtures;
* SIREN latent gradient at sensor points (cfd_siren_tape_forward / _vjp)
  against autograd through the CPU oracle SIREN;
* the whole guided loop (create_sampler / get_operator / 'ps' conditioning)
  against the reference's own run (tests/golden/dps_*.npz, make_golden_dps.py),
  replaying its recorded noise;
* a batch of DPS chains equals the chains run one by one (bit-exact), which is
  what makes the path shard over GPUs without a collective.

Tolerances (fp32; the adjoint sums in a different order than autograd): the
input-gradients within 2e-4 of their max magnitude; the guided trajectory
within 1e-4 of the latent scale per step.
"""
import ast
import functools

import numpy as np
import pytest
import torch

from conftest import golden
from confild_amd import synth
from confild_amd.nf_networks import SIRENAutodecoder_film
from confild_amd.normalize import Normalizer_ts
from confild_amd.script_util import create_model
from oracle import siren as osn
from oracle import unet as ou

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _unet(name):
    g = golden(f"unet_{name}.npz")
    kw = ast.literal_eval(str(g["kwargs"]))
    cfg = ou.Config(**kw)
    sd_np = synth.unet_state_dict(int(g["seed"]), ou.param_shapes(cfg))
    m = create_model(**kw)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd_np.items()})
    return g, cfg, {k: torch.from_numpy(v) for k, v in sd_np.items()}, m.to(DEV)


@pytest.mark.parametrize("name", ["tiny16", "small32", "heads16", "cfgA32", "cfgB64"])
def test_unet_input_vjp_matches_autograd(hip, name):
    g, cfg, sd, m = _unet(name)
    x = torch.from_numpy(g["x"])
    t = torch.from_numpy(g["t"])
    d_eps = torch.from_numpy(synth.normal(5, f"{name}/deps", tuple(x.shape)))
    # reference: autograd through the oracle forward (CPU fp32)
    xr = x.clone().requires_grad_()
    eps_ref = ou.forward(sd, cfg, xr, t)
    (gx_ref,) = torch.autograd.grad(eps_ref, xr, d_eps)
    # HIP: forward with a tape (bit-identical to the plain forward), then the VJP
    eps_plain = m(x.to(DEV), t.to(DEV))
    eps_tape = m.forward_tape(x.to(DEV), t.to(DEV))
    assert torch.equal(eps_plain, eps_tape)
    gx = m.input_vjp(d_eps.to(DEV)).cpu()
    scale = float(gx_ref.abs().max())
    err = float((gx - gx_ref).abs().max()) / scale
    assert err < 2e-4, err


def test_unet_input_vjp_is_linear_and_batch_invariant(hip):
    g, cfg, sd, m = _unet("tiny16")
    x = torch.from_numpy(synth.normal(7, "lin/x", (3, 1, 16, 16))).to(DEV)
    t = torch.tensor([5, 500, 999], device=DEV)
    a = torch.from_numpy(synth.normal(7, "lin/a", (3, 1, 16, 16))).to(DEV)
    b = torch.from_numpy(synth.normal(7, "lin/b", (3, 1, 16, 16))).to(DEV)
    m.forward_tape(x, t)
    ga, gb, gab = m.input_vjp(a), m.input_vjp(b), m.input_vjp(2 * a + b)
    assert float((gab - (2 * ga + gb)).abs().max()) < 1e-5 * float(gab.abs().max())
    # one sample at a time gives the same gradient bits
    for s in range(3):
        m.forward_tape(x[s:s + 1], t[s:s + 1])
        assert torch.equal(m.input_vjp(a[s:s + 1]), ga[s:s + 1])


@pytest.mark.parametrize("dims,Ns,R", [((3, 16, 3, 2, 32), 5, 7), ((3, 64, 3, 15, 384), 10, 24),
                                        ((2, 32, 2, 4, 128), 17, 3)])
def test_siren_latent_vjp_matches_autograd(hip, dims, Ns, R):
    d, L, c, nh, H = dims
    sd_np = synth.siren_state_dict(31, d, L, c, nh, H)
    sd = {k: torch.from_numpy(v) for k, v in sd_np.items()}
    nf = SIRENAutodecoder_film(d, L, c, nh, H)
    nf.load_state_dict(sd)
    nf.to(DEV)
    coords = torch.from_numpy(synth.uniform(31, "c", (Ns, d), -0.5, 2.0))
    xhi, xlo = torch.full((1, d), 2.2), torch.full((1, d), -0.7)
    yhi = torch.from_numpy(synth.uniform(31, "yhi", (c,), 0.5, 2.0))
    ylo = -yhi
    z = torch.from_numpy(synth.normal(31, "z", (R, L))) * 0.5
    gout = torch.from_numpy(synth.normal(31, "g", (R, Ns, c)))
    zr = z.clone().requires_grad_()
    ref = osn.decode(sd, coords, zr, xhi, xlo, yhi, ylo)
    (gz_ref,) = torch.autograd.grad(ref, zr, gout)
    xn = Normalizer_ts(params=(xhi, xlo), method="-11", dim=0)
    yn = Normalizer_ts(params=(yhi, ylo), method="-11", dim=0)
    out = nf.tape_forward(coords.to(DEV), z.to(DEV), xn, yn)
    ref = ref.detach()
    assert float((out.cpu() - ref).abs().max()) < 2e-5 * max(1.0, float(ref.abs().max()))
    gz = nf.tape_vjp(gout.to(DEV)).cpu()
    err = float((gz - gz_ref).abs().max()) / float(gz_ref.abs().max())
    assert err < 1e-3, err


def _tape_case(seed, dims, Ns, R):
    d, L, c, nh, H = dims
    sd_np = synth.siren_state_dict(seed, d, L, c, nh, H)
    coords = torch.from_numpy(synth.uniform(seed, "c", (Ns, d), -0.5, 2.0))
    xhi, xlo = torch.full((1, d), 2.2), torch.full((1, d), -0.7)
    yhi = torch.from_numpy(synth.uniform(seed, "yhi", (c,), 0.5, 2.0))
    z = torch.from_numpy(synth.normal(seed, "z", (R, L))) * 0.5
    gout = torch.from_numpy(synth.normal(seed, "g", (R, Ns, c)))
    return sd_np, coords, (xhi, xlo, yhi, -yhi), z, gout


@pytest.mark.parametrize("dims", [(3, 64, 3, 15, 384), (2, 32, 2, 4, 128)], ids=["h384", "h128"])
def test_split_tape_is_fp32_level_and_scale_exact(hip, dims):
    """K9t (the split-f16 tape, the default at H = 128 / 256 / 384) against an fp64
    autograd evaluation of the oracle: output and latent gradient within 2x the
    exact-fp32 tape's own error (+1e-7 of the max); the backward's per-pair
    power-of-two operand scaling makes the gradient exactly homogeneous under
    power-of-two gradient scales (2^-40 .. 2^40, far outside f16's range); rows
    taped alone equal the same rows taped in a larger batch, bit for bit (Ns = 10:
    16-pair tiles straddle rows)."""
    d, L, c, nh, H = dims
    Ns, R = 10, 24
    sd_np, coords, (xhi, xlo, yhi, ylo), z, gout = _tape_case(41, dims, Ns, R)
    sd64 = {k: torch.from_numpy(v).double() for k, v in sd_np.items()}
    z64 = z.double().requires_grad_()
    ref = osn.decode(sd64, coords.double(), z64, xhi.double(), xlo.double(), yhi.double(), ylo.double())
    (gz_ref,) = torch.autograd.grad(ref, z64, gout.double())
    ref, gz_ref = ref.detach(), gz_ref.detach()
    xn = Normalizer_ts(params=(xhi, xlo), method="-11", dim=0)
    yn = Normalizer_ts(params=(yhi, ylo), method="-11", dim=0)
    res = {}
    for mode in ("f32", "split_f16"):
        nf = SIRENAutodecoder_film(d, L, c, nh, H)
        nf.load_state_dict({k: torch.from_numpy(v) for k, v in sd_np.items()})
        nf.to(DEV).set_compute(mode)
        out = nf.tape_forward(coords.to(DEV), z.to(DEV), xn, yn)
        gz = nf.tape_vjp(gout.to(DEV))
        res[mode] = (nf, out, gz)
    eo = {m: float((res[m][1].cpu().double() - ref).abs().max()) for m in res}
    eg = {m: float((res[m][2].cpu().double() - gz_ref).abs().max()) for m in res}
    assert eo["split_f16"] <= 2 * eo["f32"] + 1e-7 * float(ref.abs().max()), eo
    assert eg["split_f16"] <= 2 * eg["f32"] + 1e-7 * float(gz_ref.abs().max()), eg
    nf, out, gz = res["split_f16"]
    g = gout.to(DEV)
    for k in (-40, -12, 12, 40):
        nf.tape_forward(coords.to(DEV), z.to(DEV), xn, yn)
        assert torch.equal(nf.tape_vjp(g * 2.0 ** k), gz * 2.0 ** k), k
    # rows 5..8 alone: the same output and gradient bits
    o2 = nf.tape_forward(coords.to(DEV), z[5:9].to(DEV), xn, yn)
    g2 = nf.tape_vjp(g[5:9])
    assert torch.equal(o2, out[5:9]) and torch.equal(g2, gz[5:9])


# ---------------------------------------------------------------------------
# the guided loop of the Case4 notebook vs the reference's recorded run
# ---------------------------------------------------------------------------
def _dps_setup(name):
    from confild_amd.guided.condition_methods import get_conditioning_method
    from confild_amd.guided.gaussian_diffusion import create_sampler
    from confild_amd.guided.measurements import Case4Operator, get_noise
    from confild_amd.guided.unet import create_model as guided_model
    g = golden(f"{name}.npz")
    kw = ast.literal_eval(str(g["kwargs"]))
    model = guided_model(**kw)                         # no model_path: random init (weights set below)
    sd = synth.unet_state_dict(int(g["seed"]), {k: tuple(v.shape) for k, v in model.state_dict().items()})
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    model.to(DEV)
    d, L, c, nh, H = (int(v) for v in g["siren_dims"])
    nf = SIRENAutodecoder_film(d, L, c, nh, H)
    nf.load_state_dict({k: torch.from_numpy(v) for k, v in synth.siren_state_dict(int(g["siren_seed"]), d, L, c, nh,
                                                                                   H).items()})
    T = lambda k: torch.from_numpy(g[k])  # noqa: E731
    op = Case4Operator.from_parts(DEV, T("coords"), Normalizer_ts(params=(T("xhi"), T("xlo")), method="-11", dim=0),
                                  Normalizer_ts(params=(T("yhi"), T("ylo")), method="-11", dim=0), nf, T("vmax"),
                                  T("vmin"), batch_size=int(g["op_batch"]))
    cond = get_conditioning_method(operator=op, noiser=get_noise(sigma=0.0, name="gaussian"), name="ps",
                                   scale=float(g["scale"]))
    sampler = create_sampler(sampler="ddpm", steps=1000, noise_schedule="cosine", model_mean_type="epsilon",
                             model_var_type="fixed_large", dynamic_threshold=False, clip_denoised=True,
                             rescale_timesteps=False, timestep_respacing=str(g["respacing"]))
    return g, model, op, cond, sampler


@pytest.mark.parametrize("name", ["dps_tiny16", "dps_tiny16_s3"])
def test_dps_loop_matches_reference(hip, name):
    g, model, op, cond, sampler = _dps_setup(name)
    y = torch.from_numpy(g["measurement"]).to(DEV)
    # the operator itself
    A = op.forward(torch.from_numpy(g["x_true"]).to(DEV)).cpu().numpy()
    assert np.abs(A - g["measurement"]).max() < 2e-5 * max(1.0, np.abs(g["measurement"]).max())
    steps = len(g["img"])
    fn = functools.partial(cond.conditioning)
    # per step, from the reference's own state (isolates each step's arithmetic)
    for k in range(steps):
        xin = torch.from_numpy(g["x_start"] if k == 0 else g["img"][k - 1]).to(DEV)
        out = sampler.p_sample_step(model, xin, steps - 1 - k, y, fn, noise=torch.from_numpy(g["step_noise"][k]))
        lat = max(1.0, float(np.abs(g["img"][k]).max()))
        for key, ref in (("pred_xstart", g["x0"][k]), ("x_t", g["sample"][k]), ("sample", g["img"][k])):
            err = float(np.abs(out[key].cpu().numpy() - ref).max()) / lat
            assert err < 1e-4, (k, key, err)
        assert abs(float(out["distance"][0]) - g["dist"][k]) < 1e-4 * max(1.0, g["dist"][k])
    # and the whole loop from x_start
    x = torch.from_numpy(g["x_start"]).to(DEV)
    out = sampler.p_sample_loop(model=model, x_start=x, measurement=y, measurement_cond_fn=fn, record=False,
                                save_root=None, step_noise=torch.from_numpy(g["step_noise"]))
    err = float(np.abs(out.cpu().numpy() - g["out"]).max()) / max(1.0, float(np.abs(g["out"]).max()))
    assert err < 5e-4, err
    dist = sampler.distances[:, 0].cpu().numpy()
    assert np.abs(dist - g["dist"]).max() < 1e-3 * max(1.0, g["dist"].max())


def test_dps_batch_equals_single_chains(hip):
    g, model, op, cond, sampler = _dps_setup("dps_tiny16")
    y = torch.from_numpy(g["measurement"]).to(DEV)
    fn = functools.partial(cond.conditioning)
    xs = torch.from_numpy(synth.normal(3, "dps/xs", (3, 1, 16, 16))).to(DEV)
    full = sampler.p_sample_loop(model=model, x_start=xs, measurement=y, measurement_cond_fn=fn, seed=99)
    dfull = sampler.distances.clone()
    for s in range(3):
        one = sampler.p_sample_loop(model=model, x_start=xs[s:s + 1], measurement=y, measurement_cond_fn=fn,
                                    seed=99, sample_offset=s)
        assert torch.equal(one, full[s:s + 1]), s
        assert torch.equal(sampler.distances[:, 0], dfull[:, s]), s
    assert torch.isfinite(full).all()


@pytest.mark.parametrize("name", ["tiny16", "cfgB64"])
def test_unet_input_vjp_split_is_fp32_level(hip, name):
    """Split-f16 transposed convolutions (default compute): the input-gradient's
    error against float64 autograd stays within 2x the fp32 kernels' error
    (+1e-7 of the gradient scale), as for the forward (test_gpu_unet_split.py)."""
    g, cfg, sd, m = _unet(name)
    x = torch.from_numpy(g["x"])
    t = torch.from_numpy(g["t"])
    d_eps = torch.from_numpy(synth.normal(5, f"{name}/deps", tuple(x.shape)))
    xr = x.double().requires_grad_()
    eps_ref = ou.forward({k: v.double() for k, v in sd.items()}, cfg, xr, t)
    (gx64,) = torch.autograd.grad(eps_ref, xr, d_eps.double())
    err = {}
    for mode in ("fp32", "split_f16"):
        m.set_compute(mode)
        m.forward_tape(x.to(DEV), t.to(DEV))
        err[mode] = float((m.input_vjp(d_eps.to(DEV)).cpu().double() - gx64).abs().max())
    m.set_compute("split_f16")
    scale = float(gx64.abs().max())
    assert err["split_f16"] <= 2 * err["fp32"] + 1e-7 * scale, (err, scale)
