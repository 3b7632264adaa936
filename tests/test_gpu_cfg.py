"""GPU parity at the BASELINE.json configuration shapes, against fixtures made by
running the reference (tests/golden/make_golden_cfg.py).  Weights, inputs,
noise and the Case4 operator's files are regenerated from synth seeds
(tests/golden/cfg_cases.py); only the reference's outputs are stored.

Stated tolerances, all relative to max(1, max|ref|); the values measured on
MI355X (round 2) are in brackets and in DESIGN.md section 5:
  * config B, the full 256-step DDPM loop at B = 1 with the reference's noise:
    every checkpoint sample and the final latent <= 1e-5 [max 1.3e-6, final
    1.3e-6]; x0_hat <= 5e-4 [1.5e-4 at step 1, where sqrt(1/abar - 1) ~ 1e2
    multiplies the eps rounding; 1.3e-6 at the end].  The loop re-injects noise
    and clamps x0, so the drift does not grow chaotically over the 256 steps;
  * config A, DDIM-50 + de-normalisation + 1000-coordinate decode of the 32
    rows: latent <= 1e-4 [1.9e-5: DDIM has no noise to wash out rounding],
    fields <= 5e-5 [4.8e-6], the decoder alone on the reference's latents
    <= 2e-5 [6.4e-7];
  * config D widths, DPS steps at indices 200, 37, 0 from the same state:
    x0_hat, the DDPM sample and the conditioned image <= 2e-5 [4.2e-6], the
    residual norm <= 1e-5 relative [1.2e-7];
  * real Case4 (384^2 U-Net, 108 M parameters, operator from files): operator
    forward <= 2e-5 [6.0e-7], one DPS step at index 500 <= 2e-5 [x0 2.5e-6,
    image 3.6e-7, norm 1.6e-7].
"""
import os
import sys

import numpy as np
import pytest
import torch

from conftest import GOLDEN, golden
from confild_amd import synth
from confild_amd.nf_networks import SIRENAutodecoder_film
from confild_amd.normalize import Normalizer_ts
from confild_amd.script_util import create_gaussian_diffusion, create_model

sys.path.insert(0, GOLDEN)
from cfg_cases import (CASE4_OP, CASE4_STEPS, CFG_A, DPS_D, TRAJ_B, TRAJ_E, TRAJ_E100, TRAJ_E1000,  # noqa: E402
                       case4_files,
                       noise_for, unet_weights)

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _rel(a, ref):
    a = a.detach().cpu().numpy() if torch.is_tensor(a) else np.asarray(a)
    return float(np.abs(a - ref).max()) / max(1.0, float(np.abs(ref).max()))


def _unet(case, factory=create_model):
    m = factory(**case["unet"])
    m.load_state_dict({k: torch.from_numpy(v) for k, v in unet_weights(m.state_dict(), case["seed"]).items()})
    return m.to(DEV)


def _noise_list(tag, n, shape):
    return [torch.from_numpy(noise_for(tag, k, shape)).to(DEV) for k in range(n)]


@pytest.mark.parametrize("plan", [0, 1, 2], ids=["plan8", "plan1", "plan2"])
def test_configB_full_256_step_trajectory(hip, plan):
    """The 256-step config-B loop against the reference, at the default planned
    batch (8, the weak-scaling line) and at the plans the timed small-batch points
    use (1: bench.py's strong-scaling shard at 8 GPUs and --per-gpu-batch 1;
    2: its 4-GPU shard): the same 1e-5 bound at every plan."""
    c = TRAJ_B
    g = golden("golden_trajB.npz")
    m = _unet(c)
    m.set_plan_batch(plan)
    d = create_gaussian_diffusion(steps=1000, noise_schedule="cosine", timestep_respacing=c["respacing"])
    assert np.array_equal(np.asarray(d.timestep_map), g["timestep_map"])
    shape = (c["B"], 1, c["image_size"], c["image_size"])
    x_T = torch.from_numpy(noise_for(c["tag"] + "/xT", 0, shape)).to(DEV)
    errs = {}
    cks = [int(k) for k in g["checkpoints"]]
    for k, out in enumerate(d.p_sample_loop_progressive(m, shape, noise=x_T,
                                                        step_noise=_noise_list(c["tag"], d.num_timesteps, shape))):
        if k in cks:
            j = cks.index(k)
            errs[k] = (_rel(out["sample"], g["samples"][j]), _rel(out["pred_xstart"], g["pred_xstart"][j]))
        final = out["sample"]
    errs["final"] = _rel(final, g["final"])
    print(f"config-B trajectory drift at plan {plan or 8} (sample, x0) per checkpoint:", errs)
    assert errs["final"] <= 1e-5, errs
    assert max(v[0] for k, v in errs.items() if k != "final") <= 1e-5, errs
    assert max(v[1] for k, v in errs.items() if k != "final") <= 5e-4, errs


@pytest.mark.parametrize("compute", ["split_f16", "fp32", "bf16"])
def test_configE_1000_step_segments(hip, compute):
    """Config E: the 128^2 default-mult U-Net in the 1000-step DDPM loop, two
    20-step segments (indices 999..980 and 19..0) of the reference's own p_sample
    with its noise.  x0_hat = sqrt(1/abar) x - sqrt(1/abar - 1) eps amplifies an
    eps error by a = sqrt(1/abar_t - 1) (~1.6e4 at t = 999 of 1000), so x0_hat is
    bounded through the eps error it implies, err(x0_hat) / max(1, a).
    fp32-accurate modes: every kept sample <= 1e-5 of max(1, |ref|), implied eps
    error <= 1e-5.  bf16 operands (the config-E line): the drift against the
    reference's fp32 run, measured and bounded: sample
    <= BF16_SAMPLE, implied eps error <= BF16_EPS."""
    c = TRAJ_E
    g = golden("golden_trajE.npz")
    m = _unet(c)
    m.set_compute(compute)
    d = create_gaussian_diffusion(steps=1000, noise_schedule="cosine", timestep_respacing="")
    S = c["image_size"]
    shape = (1, 1, S, S)
    keep = [int(k) for k in g["keep"]]
    worst = {}
    for start, n in c["segments"]:
        x = torch.from_numpy(noise_for(f"{c['tag']}/x{start}", 0, shape)).to(DEV)
        es, ee = [], []
        for k, i in enumerate(range(start, start - n, -1)):
            nz = torch.from_numpy(noise_for(f"{c['tag']}/{start}", k, shape)).to(DEV)
            out = d.p_sample(m, x, torch.tensor([i], device=DEV), noise=nz)
            x = out["sample"]
            if k in keep:
                j = keep.index(k)
                es.append(_rel(x, g[f"samples{start}"][j]))
                ee.append(_rel(out["pred_xstart"], g[f"pred_xstart{start}"][j]) /
                          max(1.0, float(d.sqrt_recipm1_alphas_cumprod[i])))
        worst[start] = (max(es), max(ee), es[-1])
    print(f"config E {compute}: per segment (max sample err, max implied eps err, final sample err): {worst}")
    if compute == "bf16":
        assert max(v[0] for v in worst.values()) <= BF16_SAMPLE, worst
        assert max(v[1] for v in worst.values()) <= BF16_EPS, worst
    else:
        assert max(v[0] for v in worst.values()) <= 1e-5, worst
        assert max(v[1] for v in worst.values()) <= 1e-5, worst


# measured (MI355X, round 3): sample 1.1e-3, implied eps 7.5e-3 (first segment); 4.7e-4 in the last
BF16_SAMPLE, BF16_EPS = 3e-3, 2e-2


@pytest.mark.parametrize("compute", ["split_f16", "bf16"])
def test_configE_100_consecutive_steps(hip, compute):
    """Config E over a longer stretch: 100 consecutive steps (indices 599..500) of
    the 1000-step DDPM loop of the 128^2 U-Net against the reference's own fp32
    run with its noise (golden_trajE100.npz), sample and x0_hat every 10 steps.
    The bf16-operand drift is the number the config-E line carries, stated over
    100 steps: sample <= BF16_SAMPLE_100 of max(1, |ref|) (measured in brackets
    below), x0_hat <= BF16_X0_100; the fp32-accurate split-f16 mode <= 1e-5."""
    c = TRAJ_E100
    g = golden("golden_trajE100.npz")
    m = _unet(TRAJ_E)
    m.set_compute(compute)
    d = create_gaussian_diffusion(steps=1000, noise_schedule="cosine", timestep_respacing="")
    S = TRAJ_E["image_size"]
    shape = (1, 1, S, S)
    keep = [int(k) for k in g["keep"]]
    x = torch.from_numpy(noise_for(f"{c['tag']}/x", 0, shape)).to(DEV)
    es, ex = [], []
    for k, i in enumerate(range(c["start"], c["start"] - c["n"], -1)):
        nz = torch.from_numpy(noise_for(f"{c['tag']}/steps", k, shape)).to(DEV)
        out = d.p_sample(m, x, torch.tensor([i], device=DEV), noise=nz)
        x = out["sample"]
        if k in keep:
            j = keep.index(k)
            es.append(_rel(x, g["samples"][j]))
            ex.append(_rel(out["pred_xstart"], g["pred_xstart"][j]))
    print(f"config E {compute}, 100 steps 599..500: sample err every 10 steps {['%.2e' % e for e in es]}, "
          f"x0_hat {['%.2e' % e for e in ex]}")
    if compute == "bf16":
        assert max(es) <= BF16_SAMPLE_100 and max(ex) <= BF16_X0_100, (es, ex)
    else:
        assert max(es) <= 1e-5 and max(ex) <= 1e-4, (es, ex)


@pytest.mark.parametrize("compute", ["split_f16", "bf16"])
def test_configE_full_1000_step_loop(hip, compute):
    """Config E's whole sampling: all 1000 steps (999..0) of the DDPM loop of the
    128^2 U-Net against the reference's own fp32 run with its noise
    (golden_trajE1000.npz), sample and x0_hat every 100 steps and at the end.
    split-f16: the fp32 contract (sample <= 1e-5 of max(1, |ref|) at every kept
    step, x0_hat <= 5e-4 -- x0_hat amplifies an eps error by sqrt(1/abar - 1) at
    the high-noise steps); bf16 operands (the config-E line): the drift over the
    line's full sampling, bounded at ~1.5x the measured (BF16_*_1000 below)."""
    c = TRAJ_E1000
    g = golden("golden_trajE1000.npz")
    m = _unet(TRAJ_E)
    m.set_compute(compute)
    d = create_gaussian_diffusion(steps=1000, noise_schedule="cosine", timestep_respacing="")
    S = TRAJ_E["image_size"]
    shape = (1, 1, S, S)
    keep = [int(k) for k in g["keep"]]
    x = torch.from_numpy(noise_for(f"{c['tag']}/x", 0, shape)).to(DEV)
    es, ee = [], []
    for k, i in enumerate(range(999, -1, -1)):
        nz = torch.from_numpy(noise_for(f"{c['tag']}/steps", k, shape)).to(DEV)
        out = d.p_sample(m, x, torch.tensor([i], device=DEV), noise=nz)
        x = out["sample"]
        if k in keep:
            j = keep.index(k)
            es.append(_rel(x, g["samples"][j]))
            # x0_hat through the eps error it implies (as the segment test): an eps
            # error is amplified by sqrt(1/abar_t - 1), ~1.6e4 at t = 999
            ee.append(_rel(out["pred_xstart"], g["pred_xstart"][j]) /
                      max(1.0, float(d.sqrt_recipm1_alphas_cumprod[i])))
    print(f"config E {compute}, 1000 steps: sample err every 100 steps {['%.2e' % e for e in es]}, "
          f"implied eps err {['%.2e' % e for e in ee]}")
    if compute == "bf16":
        assert max(es) <= BF16_SAMPLE_1000 and max(ee) <= BF16_EPS_1000, (es, ee)
    else:
        assert max(es) <= 1e-5 and max(ee) <= 5e-4, (es, ee)


# bf16 drift over the whole 1000-step loop, ~1.5x the measured (MI355X, round 6:
# sample 7.4e-4 after 1 step, 9.4e-4 after 300, 2.3e-3 after 500, 1.6e-2 at the end;
# implied eps error 4.9e-2 at step 100, 1.6e-2 at the end)
BF16_SAMPLE_1000, BF16_EPS_1000 = 2.4e-2, 7.5e-2


# bf16 drift over the 100 steps, ~1.5x the measured worst (MI355X, round 4: sample
# 7.2e-4 after 100 steps growing ~linearly from 9e-6 after 1; x0_hat 1.26e-2, flat)
BF16_SAMPLE_100, BF16_X0_100 = 1.1e-3, 2e-2


@pytest.mark.parametrize("plan", [0, 1], ids=["plan8", "plan1"])
def test_configA_ddim50_and_decode_end_to_end(hip, plan):
    """Config A end to end at the default planned batch and at 1 (the plan the
    config-A line is timed at: one sample per GPU; key-chunked attention at 32^2)."""
    from confild_amd.inference import latent_denorm
    c = CFG_A
    g = golden("golden_cfgA.npz")
    m = _unet(c)
    m.set_plan_batch(plan)
    d = create_gaussian_diffusion(steps=1000, noise_schedule="cosine", timestep_respacing=c["respacing"])
    assert np.array_equal(np.asarray(d.timestep_map), g["timestep_map"])
    S = c["image_size"]
    shape = (1, 1, S, S)
    x_T = torch.from_numpy(noise_for(c["tag"] + "/xT", 0, shape)).to(DEV)
    gen = d.ddim_sample_loop(m, shape, noise=x_T, eta=0.0,
                             step_noise=_noise_list(c["tag"], d.num_timesteps, shape))[:, 0]
    e_lat = _rel(gen, g["latent"])
    lat = latent_denorm(gen.contiguous(), torch.full((1,), c["vmax"], device=DEV),
                        torch.full((1,), c["vmin"], device=DEV))
    e_den = _rel(lat, g["latent_denorm"])
    dd, L, co, nh, H = c["siren"]
    nf = SIRENAutodecoder_film(dd, L, co, nh, H)
    nf.load_state_dict({k: torch.from_numpy(v) for k, v in synth.siren_state_dict(c["siren_seed"], dd, L, co, nh,
                                                                                   H).items()})
    nf.to(DEV)
    xn = Normalizer_ts(params=(torch.ones(1, dd), torch.zeros(1, dd)), method="-11", dim=0)
    yn = Normalizer_ts(params=(torch.from_numpy(g["ymax"]), torch.from_numpy(g["ymin"])), method="-11", dim=0)
    fields = nf.decode(torch.from_numpy(g["coords"]).to(DEV), lat.reshape(-1, L)[:, None], xn, yn)
    e_f = _rel(fields, g["fields"])
    # the decoder alone, on the reference's own latents (isolates the CNF error)
    f_ref_lat = nf.decode(torch.from_numpy(g["coords"]).to(DEV),
                          torch.from_numpy(g["latent_denorm"]).reshape(-1, L)[:, None].to(DEV), xn, yn)
    e_dec = _rel(f_ref_lat, g["fields"])
    print(f"config A: latent {e_lat:.2e}, denorm {e_den:.2e}, fields {e_f:.2e}, decoder alone {e_dec:.2e}")
    assert e_lat <= 1e-4 and e_den <= 1e-4
    assert e_dec <= 2e-5
    assert e_f <= 5e-5


def _operator_D(g):
    from confild_amd.guided.measurements import Case4Operator
    c = DPS_D
    dd, L, co, nh, H = c["siren"]
    nf = SIRENAutodecoder_film(dd, L, co, nh, H)
    nf.load_state_dict({k: torch.from_numpy(v) for k, v in synth.siren_state_dict(c["siren_seed"], dd, L, co, nh,
                                                                                   H).items()})
    T = lambda k: torch.from_numpy(g[k])  # noqa: E731
    return Case4Operator.from_parts(DEV, T("coords"), Normalizer_ts(params=(T("xhi"), T("xlo")), method="-11", dim=0),
                                    Normalizer_ts(params=(T("yhi"), T("ylo")), method="-11", dim=0), nf, T("vmax"),
                                    T("vmin"), batch_size=16)


def _guided(respacing, op, scale):
    from confild_amd.guided.condition_methods import get_conditioning_method
    from confild_amd.guided.gaussian_diffusion import create_sampler
    from confild_amd.guided.measurements import get_noise
    cond = get_conditioning_method(operator=op, noiser=get_noise(sigma=0.0, name="gaussian"), name="ps", scale=scale)
    sampler = create_sampler(sampler="ddpm", steps=1000, noise_schedule="cosine", model_mean_type="epsilon",
                             model_var_type="fixed_large", dynamic_threshold=False, clip_denoised=True,
                             rescale_timesteps=False, timestep_respacing=respacing)
    return cond, sampler


def test_configD_dps_steps_at_config_widths(hip):
    from confild_amd.guided.unet import create_model as guided_model
    c = DPS_D
    g = golden("golden_dpsD.npz")
    model = _unet(c, guided_model)
    op = _operator_D(g)
    cond, sampler = _guided(c["respacing"], op, c["scale"])
    y = torch.from_numpy(g["measurement"]).to(DEV)
    S, L = c["unet"]["image_size"], c["siren"][1]
    for j, idx in enumerate(c["indices"]):
        x = torch.from_numpy(synth.normal(c["siren_seed"], f"dpsD/x{idx}", (1, 1, S, L))).to(DEV)
        nz = torch.from_numpy(noise_for(f"{c['tag']}/{idx}", 0, (1, 1, S, L)))   # p_sample's randn_like
        out = sampler.p_sample_step(model, x, idx, y, cond.conditioning, noise=nz)
        e = {k: _rel(out[k], g[f"{r}{j}"]) for k, r in (("pred_xstart", "x0"), ("x_t", "sample"), ("sample", "img"))}
        ed = abs(float(out["distance"][0]) - float(g[f"dist{j}"])) / float(g[f"dist{j}"])
        print(f"config D step {idx}: {e}, norm rel {ed:.2e}")
        assert max(e.values()) <= 2e-5 and ed <= 1e-5, (idx, e, ed)


def test_configD_batched_chains_equal_single_chains(hip):
    """Config D as the bench runs it -- 8 chains per GPU of the 64^2 guided U-Net
    with SIREN(3, 64, 3, 15, 384) at 10 sensors, the whole 256-step 'ps' loop --
    equals the 8 chains run one by one, bit for bit (sample and per-step residual
    norm): a chain's arithmetic does not depend on the batch it runs in, so the
    chains shard over GPUs with no collective (tiny16 version: test_gpu_dps.py)."""
    from confild_amd.guided.unet import create_model as guided_model
    c = DPS_D
    g = golden("golden_dpsD.npz")
    model = _unet(c, guided_model)
    op = _operator_D(g)
    cond, sampler = _guided(c["respacing"], op, c["scale"])
    y = torch.from_numpy(g["measurement"]).to(DEV)
    S, L = c["unet"]["image_size"], c["siren"][1]
    xs = torch.from_numpy(synth.normal(c["siren_seed"], "dpsD/batched_xs", (8, 1, S, L))).to(DEV)
    full = sampler.p_sample_loop(model=model, x_start=xs, measurement=y, measurement_cond_fn=cond.conditioning,
                                 seed=2024)
    dfull = sampler.distances.clone()
    assert torch.isfinite(full).all() and dfull.shape[1] == 8
    for s in range(8):
        one = sampler.p_sample_loop(model=model, x_start=xs[s:s + 1], measurement=y,
                                    measurement_cond_fn=cond.conditioning, seed=2024, sample_offset=s)
        assert torch.equal(one, full[s:s + 1]), s
        assert torch.equal(sampler.distances[:, 0], dfull[:, s]), s


def test_configD_dps_chain_vs_oracle(hip):
    """Config D widths, 12 consecutive guided steps (indices 30 .. 19 of the 256-step
    loop), each from the HIP path's own previous image, against the CPU oracle's
    autograd chain from the same start and noise (oracle/dps.py, itself pinned to
    the reference's steps at these widths by test_oracle_configD_dps_steps).  Per
    step image <= 2e-5 of the latent scale and residual norm <= 1e-5 relative
    [MI355X, round 5: the image error grows ~linearly, 7.9e-7 -> 4.5e-6 over the 12
    steps; norms <= 9.4e-7]."""
    from confild_amd.guided.unet import create_model as guided_model
    from oracle import diffusion as od
    from oracle import dps as odps
    from oracle import unet as ou
    c = DPS_D
    g = golden("golden_dpsD.npz")
    model = _unet(c, guided_model)
    op = _operator_D(g)
    cond, sampler = _guided(c["respacing"], op, c["scale"])
    y = torch.from_numpy(g["measurement"])
    S, L = c["unet"]["image_size"], c["siren"][1]
    cfg = ou.Config(**c["unet"])
    sd = {k: torch.from_numpy(v) for k, v in unet_weights(ou.param_shapes(cfg), c["seed"]).items()}
    dd, _, co, nh, H = c["siren"]
    ssd = {k: torch.from_numpy(v) for k, v in synth.siren_state_dict(c["siren_seed"], dd, L, co, nh, H).items()}
    T = lambda k: torch.from_numpy(g[k])  # noqa: E731
    operator = lambda x0: odps.case4_forward(ssd, T("coords"), T("xhi"), T("xlo"), T("yhi"), T("ylo"),  # noqa: E731
                                             T("vmax"), T("vmin"), x0, batch=16)
    unet = lambda x, t: ou.forward(sd, cfg, x, t)  # noqa: E731
    tb = od.Tables(1000, "cosine", c["respacing"])
    x_ref = torch.from_numpy(synth.normal(c["siren_seed"], "dpsD/chain_x", (1, 1, S, L)))
    x_hip = x_ref.to(DEV)
    worst = 0.0
    for k, idx in enumerate(range(30, 18, -1)):
        nz = torch.from_numpy(noise_for(f"{c['tag']}/chain", k, (1, 1, S, L)))
        x_ref, _, _, norm_ref = odps.dps_step(tb, unet, operator, x_ref, idx, y, nz, c["scale"])
        out = sampler.p_sample_step(model, x_hip, idx, y.to(DEV), cond.conditioning, noise=nz.to(DEV))
        x_hip = out["sample"]
        lat = max(1.0, float(x_ref.abs().max()))
        err = float((x_hip.cpu() - x_ref).abs().max()) / lat
        en = abs(float(out["distance"][0]) - float(norm_ref)) / float(norm_ref)
        worst = max(worst, err)
        print(f"config D chain step {idx}: image {err:.2e}, norm rel {en:.2e}")
        assert err <= 2e-5 and en <= 1e-5, (idx, err, en)
    assert worst <= 2e-5


def _case4_operator(tmp):
    from confild_amd.guided.measurements import get_operator
    paths = case4_files(str(tmp))
    return get_operator(device=DEV, name="case4", coords_path=paths["coords"], max_val_path=paths["max"],
                        min_val_path=paths["min"], normalizer_params_path=paths["normalizer"],
                        ckpt_path=paths["ckpt"], batch_size=CASE4_OP["batch_size"])


def test_case4_operator_from_files(hip, tmp_path):
    c = CASE4_OP
    g = golden("golden_case4op.npz")
    op = _case4_operator(tmp_path)
    x = torch.from_numpy(synth.uniform(c["seed"], "case4op/x", (1, 1, c["T"], c["L"]), -0.95, 0.95)).to(DEV)
    A = op.forward(x)
    err = _rel(A, g["A"])
    print(f"Case4 operator (files, SIREN(3,384,3,15,384), 10 sensors): {err:.2e}")
    assert A.shape == g["A"].shape and err <= 2e-5


def test_case4_real_shape_dps_step(hip, tmp_path):
    """The notebook's 384^2 U-Net (channel_mult 1,1,2,2,4,4) loaded from an ema
    file by create_model(model_path=...), the file-built operator, one DDPM+'ps'
    step at index 500 of 1000, against the reference's own step."""
    from confild_amd.guided.unet import create_model as guided_model
    c = CASE4_OP
    g = golden("golden_case4dps.npz")
    op = _case4_operator(tmp_path)
    kw = c["unet"]
    shapes = {k: tuple(v.shape) for k, v in guided_model(**kw).state_dict().items()}
    assert sum(int(np.prod(s)) for s in shapes.values()) == int(g["nparams"])
    ema = tmp_path / "ema_0.9999_400000.pt"
    torch.save({k: torch.from_numpy(v) for k, v in synth.unet_state_dict(c["unet_seed"], shapes).items()}, ema)
    model = guided_model(**kw, model_path=str(ema)).to(DEV)
    y = torch.from_numpy(golden("golden_case4op.npz")["A"]).to(DEV)   # the reference's measurement of x_true
    cond, sampler = _guided("", op, 1.0)
    idx = int(g["index"])
    x = torch.from_numpy(synth.normal(c["seed"], f"case4dps/x{idx}", (1, 1, c["T"], c["L"]))).to(DEV)
    nz = torch.from_numpy(noise_for(f"case4dps/{idx}", 0, (1, 1, c["T"], c["L"])))
    out = sampler.p_sample_step(model, x, idx, y, cond.conditioning, noise=nz)
    e_x0 = _rel(out["pred_xstart"], g["x0"])
    e_img = _rel(out["sample"], g["img"])
    ed = abs(float(out["distance"][0]) - float(g["dist"])) / float(g["dist"])
    print(f"Case4 384^2 DPS step {idx}: x0 {e_x0:.2e}, img {e_img:.2e}, norm {ed:.2e}")
    assert e_x0 <= 2e-5 and e_img <= 2e-5 and ed <= 1e-5
    os.remove(ema)


@pytest.mark.parametrize("plan", [0, 2], ids=["plan8", "plan2"])
def test_case4_real_shape_10_consecutive_dps_steps(hip, tmp_path, plan):
    """Run at the default planned batch (8) and at the plan bench.py times real
    Case4 with (DPS_CFG["Case4"]["plan_batch"] = 2: gn2's 1024-thread chunks at
    384^2 and the plan-2 split-K counts).  The notebook's loop body over 10 consecutive steps (indices 500..491) at
    384^2, each step fed the previous step's output and the reference's noise:
    the drift of a chain, not one step.  Per step: image <= 5e-5 and x0_hat
    <= 3e-4 of max(1, |ref|) on the fixture's 4x-strided subgrid, residual norm
    <= 1e-5 relative, whole-image sum within 1e-5 relative of its L1 scale; the
    final image in full: <= 2e-3, and at most 0.1% of its elements beyond 5e-5.
    Measured (MI355X, round 3): the image error is
    3.8e-7 after the first step and 1.2e-5 from the second on, flat to the tenth
    (a few elements whose x0_hat sits at the clamp boundary switch the clamp's
    derivative mask in the 'ps' gradient: a step, not a growing drift); x0_hat
    follows the state at ~1.4x (sqrt(1/abar) ~ 1.4 at t ~ 500): <= 9.2e-5;
    norms <= 2.2e-6; sums <= 1.5e-8; the final image 5.2e-4 at its worst element
    (the clamp-mask elements, off the subgrid)."""
    from confild_amd.guided.unet import create_model as guided_model
    c, cs = CASE4_OP, CASE4_STEPS
    g = golden("golden_case4steps.npz")
    op = _case4_operator(tmp_path)
    kw = c["unet"]
    shapes = {k: tuple(v.shape) for k, v in guided_model(**kw).state_dict().items()}
    ema = tmp_path / "ema_0.9999_400000.pt"
    torch.save({k: torch.from_numpy(v) for k, v in synth.unet_state_dict(c["unet_seed"], shapes).items()}, ema)
    model = guided_model(**kw, model_path=str(ema)).to(DEV)
    model.set_plan_batch(plan)
    os.remove(ema)
    y = torch.from_numpy(golden("golden_case4op.npz")["A"]).to(DEV)
    cond, sampler = _guided("", op, 1.0)
    shape = (1, 1, c["T"], c["L"])
    x = torch.from_numpy(synth.normal(c["seed"], f"case4steps/x{cs['start']}", shape)).to(DEV)
    errs = []
    for k, idx in enumerate(range(cs["start"], cs["start"] - cs["n"], -1)):
        nz = torch.from_numpy(noise_for(f"case4steps/{idx}", 0, shape))
        out = sampler.p_sample_step(model, x, idx, y, cond.conditioning, noise=nz)
        x = out["sample"]
        e_img = _rel(x[..., ::4, ::4], g["img_sub"][k])
        e_x0 = _rel(out["pred_xstart"][..., ::4, ::4], g["x0_sub"][k])
        e_d = abs(float(out["distance"][0]) - float(g["dists"][k])) / float(g["dists"][k])
        s = float(x.double().sum())
        e_sum = abs(s - float(g["img_sum"][k])) / (float(x.abs().double().sum()))
        errs.append((idx, e_img, e_x0, e_d, e_sum))
    e_fin = _rel(x, g["img_final"])
    dfin = np.abs(x.cpu().numpy() - g["img_final"]) / max(1.0, float(np.abs(g["img_final"]).max()))
    n_off = int((dfin > 5e-5).sum())
    print(f"Case4 final image: {n_off} of {dfin.size} elements beyond 5e-5, 99.9th percentile "
          f"{np.percentile(dfin, 99.9):.2e}")
    print(f"Case4 384^2 10-step chain at plan {plan or 8} (idx, img, x0, norm, sum):", [tuple(round(v, 9) if isinstance(v, float) else v
                                                                     for v in e) for e in errs], f"final {e_fin:.2e}")
    assert max(e[1] for e in errs) <= 5e-5 and max(e[2] for e in errs) <= 3e-4, errs
    assert max(e[3] for e in errs) <= 1e-5 and max(e[4] for e in errs) <= 1e-5, errs
    assert e_fin <= 2e-3 and n_off <= dfin.size // 1000, (e_fin, n_off)


@pytest.mark.parametrize("name", ["grid2d", "lumped3d_pub"])
def test_cnf_inference_predict_vs_reference(hip, tmp_path, name):
    """CNF_inference.predict on the fused decoder against the reference's predict
    of the same checkpoint directory (2-D grid latents; lumped is_pub latents)."""
    from cfg_cases import CNF_INF, cnf_inference_coords, cnf_inference_files
    from confild_amd.inference_function import CNF_inference
    c = CNF_INF[name]
    g = golden("golden_cnfinf.npz")
    f = cnf_inference_files(str(tmp_path), name)
    inf = CNF_inference(f["checkpoint"], f["config"], f["data"], device="cuda", is_pub=c["is_pub"])
    pred = inf.predict(torch.from_numpy(cnf_inference_coords(name)), c["idx"], batch_size=2)
    err = _rel(pred, g[f"{name}_pred"])
    print(f"CNF_inference {name}: {err:.2e}")
    assert pred.shape == g[f"{name}_pred"].shape and err <= 2e-5
    allp = inf.get_all_predictions(torch.from_numpy(cnf_inference_coords(name)))
    assert torch.equal(allp[c["idx"]], pred)


def test_case4_postprocessing_chain_vs_reference(hip):
    """The notebook's cells 26-32: decoder over the masked points, rearrange
    "(s t) co c -> s t co c", ReconstructFrame of every frame into the Mask grid."""
    from cfg_cases import POST, post_inputs
    from einops import rearrange
    from confild_amd.inference_function import ReconstructFrame, decoder
    g = golden("golden_post.npz")
    d, L, co, nh, H = POST["siren"]
    mask, coords, lat, xhi, xlo, yhi, ylo = post_inputs()
    nf = SIRENAutodecoder_film(d, L, co, nh, H)
    nf.load_state_dict({k: torch.from_numpy(v) for k, v in synth.siren_state_dict(POST["seed"], d, L, co, nh,
                                                                                   H).items()})
    nf.to(DEV)
    T = torch.from_numpy
    xn = Normalizer_ts(method="-11", dim=0, params=(T(xhi), T(xlo)))
    yn = Normalizer_ts(method="-11", dim=0, params=(T(yhi), T(ylo)))
    fields = decoder(T(coords).to(DEV), T(lat).to(DEV), nf, xn, yn, batch_size=4, device=DEV)
    fields = rearrange(fields, "(s t) co c -> s t co c", t=POST["t"])
    frames = np.stack([ReconstructFrame(fields[s, t].numpy(), mask=mask, shape=POST["grid"], fill_value=0.)
                       for s in range(POST["s"]) for t in range(POST["t"])])
    frames = rearrange(frames, "(s t) x y z c -> s t x y z c", t=POST["t"])
    err = _rel(frames, g["frames"])
    assert frames.shape == g["frames"].shape and err <= 2e-5, err
    assert np.array_equal(frames[..., 0][:, :, ~mask], np.zeros_like(frames[..., 0][:, :, ~mask]))
