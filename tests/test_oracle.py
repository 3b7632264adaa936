"""Pin the CPU oracle against the golden fixtures produced by the reference itself
(tests/golden/make_golden.py).  CPU only."""
import ast

import numpy as np
import pytest
import torch

from conftest import golden
from confild_amd import synth
from oracle import diffusion as od
from oracle import siren as osn
from oracle import unet as ou
from oracle import dps as odps

SCHED = golden("schedules.npz")
RESP = {"id": "", "s256": "256", "ddim50": "ddim50", "ddim5": "ddim5", "s8": "8",
        "s10_20_30": "10,20,30", "s250": "250", "s100": "100"}
ATTRS = ("betas", "alphas_cumprod", "alphas_cumprod_prev", "sqrt_recip_alphas_cumprod",
         "sqrt_recipm1_alphas_cumprod", "posterior_variance", "posterior_log_variance_clipped",
         "posterior_mean_coef1", "posterior_mean_coef2")


@pytest.mark.parametrize("sched", ["cosine", "linear"])
def test_beta_schedule_bitexact(sched):
    assert np.array_equal(od.beta_schedule(sched, 1000), SCHED[f"{sched}_1000_betas"])


@pytest.mark.parametrize("tag", list(RESP))
def test_respaced_tables_bitexact(tag):
    tb = od.Tables(1000, "cosine", RESP[tag])
    assert np.array_equal(tb.timestep_map, SCHED[f"{tag}_timestep_map"])
    for a in ATTRS:
        assert np.array_equal(getattr(tb, a), SCHED[f"{tag}_{a}"]), a


def test_space_timesteps_errors_and_sections():
    errs = list(SCHED["space_errors"])
    for args, want in zip(((1000, "ddim256"), (10, "20"), (100, "ddim7")), errs):
        try:
            od.space_timesteps(*args)
            got = "ok"
        except ValueError as e:
            got = "ValueError:" + str(e)
        assert got == want
    assert sorted(od.space_timesteps(300, [10, 15, 20])) == list(SCHED["space_300_10_15_20"])


def _unet_case(name):
    g = golden(f"unet_{name}.npz")
    kw = ast.literal_eval(str(g["kwargs"]))
    cfg = ou.Config(**kw)
    shapes = ou.param_shapes(cfg)
    assert list(shapes) == list(g["keys"])  # same keys, same registration order
    sd = {k: torch.from_numpy(v) for k, v in synth.unet_state_dict(int(g["seed"]), shapes).items()}
    return g, cfg, sd


@pytest.mark.parametrize("name", ["tiny16", "small32", "heads16", "cfgA32", "cfgB64"])
def test_unet_forward_matches_reference(name):
    g, cfg, sd = _unet_case(name)
    with torch.no_grad():
        eps = ou.forward(sd, cfg, torch.from_numpy(g["x"]), torch.from_numpy(g["t"])).numpy()
    ref = g["eps"]
    err = np.abs(eps - ref).max() / np.abs(ref).max()
    assert err < 1e-5, err


def _tiny_model():
    g, cfg, sd = _unet_case("tiny16")
    return lambda x, t: ou.forward(sd, cfg, x, t)


@pytest.mark.parametrize("tag,resp,kind", [("ddpm8", "8", "ddpm"), ("ddim5", "ddim5", "ddim")])
def test_sampler_trajectory_matches_reference(tag, resp, kind):
    tr = golden(f"traj_{tag}.npz")
    tb = od.Tables(1000, "cosine", resp)
    assert np.array_equal(tb.timestep_map, tr["timestep_map"])
    x, traj = od.sample_loop(tb, _tiny_model(), torch.from_numpy(tr["noise0"]),
                             torch.from_numpy(tr["noise"]), kind)
    for k, (xk, xs) in enumerate(traj):
        assert np.abs(xk.numpy() - tr["samples"][k]).max() < 1e-5, k
        assert np.abs(xs.numpy() - tr["pred_xstart"][k]).max() < 1e-5, k


def test_single_ddpm_step_bitexact():
    """Given the reference's own eps, one oracle step reproduces the reference sample bit for bit."""
    tr = golden("traj_ddpm8.npz")
    tb = od.Tables(1000, "cosine", "8")
    model = _tiny_model()
    x = torch.from_numpy(tr["noise0"])
    t = torch.full((2,), tb.num_timesteps - 1, dtype=torch.int64)
    with torch.no_grad():
        eps = model(x, torch.from_numpy(tb.timestep_map)[t])
    x1, _ = od.ddpm_step(tb, x, t, eps, torch.from_numpy(tr["noise"][0]))
    assert np.abs(x1.numpy() - tr["samples"][0]).max() < 1e-6


@pytest.mark.parametrize("case", ["s2d", "s3d", "caseA", "case4w"])
def test_siren_matches_reference(case):
    g = golden(f"siren_{case}.npz")
    d, L, c, nh, H = (int(v) for v in g["dims"])
    sd = {k: torch.from_numpy(v) for k, v in synth.siren_state_dict(int(g["seed"]), d, L, c, nh, H).items()}
    out = osn.decode(sd, torch.from_numpy(g["coords"]), torch.from_numpy(g["latents"]),
                     torch.from_numpy(g["xmax"]), torch.from_numpy(g["xmin"]),
                     torch.from_numpy(g["ymax"]), torch.from_numpy(g["ymin"]))
    assert np.abs(out.numpy() - g["out"]).max() < 1e-5


def test_synth_generator_is_stable():
    # golden values of the counter-based generator (guards the weight recipe)
    u = synth.uniform(1234, "input_blocks.0.0.weight", (4,), -1.0, 1.0)
    assert u.dtype == np.float32
    v = synth.uniform(1234, "input_blocks.0.0.weight", (4,), -1.0, 1.0)
    assert np.array_equal(u, v)
    assert not np.array_equal(u, synth.uniform(1235, "input_blocks.0.0.weight", (4,), -1.0, 1.0))
    n = synth.normal(7, "x", (10001,))
    assert abs(float(n.mean())) < 0.05 and abs(float(n.std()) - 1) < 0.05


# ---------------------------------------------------------------------------
# DPS (Case4 conditional): the oracle's autograd DPS
# loop replays the reference's own guided sampler run (make_golden_dps.py)
# ---------------------------------------------------------------------------
def dps_case(name):
    """(golden, Tables, unet, operator, siren sd) of a DPS fixture, CPU oracle."""
    from oracle import diffusion as od
    g = golden(f"{name}.npz")
    kw = ast.literal_eval(str(g["kwargs"]))
    cfg = ou.Config(**kw)
    sd = {k: torch.from_numpy(v) for k, v in synth.unet_state_dict(int(g["seed"]), ou.param_shapes(cfg)).items()}
    d, L, c, nh, H = (int(v) for v in g["siren_dims"])
    ssd = {k: torch.from_numpy(v) for k, v in synth.siren_state_dict(int(g["siren_seed"]), d, L, c, nh, H).items()}
    tb = od.Tables(1000, "cosine", str(g["respacing"]))
    T = lambda k: torch.from_numpy(g[k])  # noqa: E731
    operator = lambda x0: odps.case4_forward(ssd, T("coords"), T("xhi"), T("xlo"), T("yhi"), T("ylo"),  # noqa: E731
                                             T("vmax"), T("vmin"), x0, batch=int(g["op_batch"]))
    unet = lambda x, t: ou.forward(sd, cfg, x, t)  # noqa: E731
    return g, tb, unet, operator, ssd


@pytest.mark.parametrize("name", ["dps_tiny16", "dps_tiny16_s3"])
def test_dps_loop_matches_reference(name):
    g, tb, unet, operator, _ = dps_case(name)
    assert np.array_equal(tb.timestep_map, g["timestep_map"])
    with torch.no_grad():
        assert np.abs(operator(torch.from_numpy(g["x_true"])).numpy() - g["measurement"]).max() < 1e-6
    _, traj = odps.dps_loop(tb, unet, operator, torch.from_numpy(g["x_start"]), torch.from_numpy(g["measurement"]),
                            torch.from_numpy(g["step_noise"]), float(g["scale"]))
    for k, (img, x0, sample, norm) in enumerate(traj):
        scale = max(1.0, float(np.abs(g["img"][k]).max()))
        assert np.abs(x0.numpy() - g["x0"][k]).max() < 2e-5 * scale, k
        assert np.abs(sample.numpy() - g["sample"][k]).max() < 2e-5 * scale, k
        assert np.abs(img.numpy() - g["img"][k]).max() < 2e-5 * scale, k
        assert abs(float(norm) - g["dist"][k]) < 1e-5 * max(1.0, g["dist"][k]), k
    assert np.abs(traj[-1][0].numpy() - g["out"]).max() < 2e-5 * max(1.0, float(np.abs(g["out"]).max()))


# ---------------------------------------------------------------------------
# config-shape fixtures (tests/golden/make_golden_cfg.py): the oracle against
# the reference at the BASELINE.json widths, at CPU-affordable lengths
# ---------------------------------------------------------------------------
def _cfg_cases():
    import sys
    from conftest import GOLDEN
    if GOLDEN not in sys.path:
        sys.path.insert(0, GOLDEN)
    import cfg_cases
    return cfg_cases


def test_oracle_configB_trajectory_prefix():
    """First 8 of the 256 DDPM steps of config B (the full loop is the GPU test)."""
    cc = _cfg_cases()
    c = cc.TRAJ_B
    g = golden("golden_trajB.npz")
    cfg = ou.Config(**c["unet"])
    sd = {k: torch.from_numpy(v) for k, v in cc.unet_weights(ou.param_shapes(cfg), c["seed"]).items()}
    tb = od.Tables(1000, "cosine", c["respacing"])
    shape = (c["B"], 1, c["image_size"], c["image_size"])
    x = torch.from_numpy(cc.noise_for(c["tag"] + "/xT", 0, shape))
    cks = [int(k) for k in g["checkpoints"]]
    with torch.no_grad():
        for k, i in enumerate(reversed(range(tb.num_timesteps))):
            if k > 8:
                break
            t = torch.full((c["B"],), i, dtype=torch.int64)
            eps = ou.forward(sd, cfg, x, torch.from_numpy(tb.timestep_map)[t])
            x, x0 = od.ddpm_step(tb, x, t, eps, torch.from_numpy(cc.noise_for(c["tag"], k, shape)))
            if k in cks:
                j = cks.index(k)
                assert np.abs(x.numpy() - g["samples"][j]).max() < 2e-5, k
                assert np.abs(x0.numpy() - g["pred_xstart"][j]).max() < 2e-5, k


def test_oracle_configA_end_to_end():
    cc = _cfg_cases()
    c = cc.CFG_A
    g = golden("golden_cfgA.npz")
    cfg = ou.Config(**c["unet"])
    sd = {k: torch.from_numpy(v) for k, v in cc.unet_weights(ou.param_shapes(cfg), c["seed"]).items()}
    tb = od.Tables(1000, "cosine", c["respacing"])
    assert np.array_equal(tb.timestep_map, g["timestep_map"])
    S = c["image_size"]
    x = torch.from_numpy(cc.noise_for(c["tag"] + "/xT", 0, (1, 1, S, S)))
    with torch.no_grad():
        for k, i in enumerate(reversed(range(tb.num_timesteps))):
            t = torch.full((1,), i, dtype=torch.int64)
            eps = ou.forward(sd, cfg, x, torch.from_numpy(tb.timestep_map)[t])
            x, _ = od.ddim_step(tb, x, t, eps, torch.from_numpy(cc.noise_for(c["tag"], k, (1, 1, S, S))))
    assert np.abs(x[:, 0].numpy() - g["latent"]).max() < 1e-4
    d, L, co, nh, H = c["siren"]
    ssd = {k: torch.from_numpy(v) for k, v in synth.siren_state_dict(c["siren_seed"], d, L, co, nh, H).items()}
    T = torch.from_numpy
    with torch.no_grad():
        f = osn.decode(ssd, T(g["coords"]), T(g["latent_denorm"]).reshape(-1, L), torch.ones(1, d),
                       torch.zeros(1, d), T(g["ymax"]), T(g["ymin"]))
    assert np.abs(f.numpy() - g["fields"]).max() < 2e-5 * max(1.0, float(np.abs(g["fields"]).max()))


def test_oracle_configD_dps_steps():
    cc = _cfg_cases()
    c = cc.DPS_D
    g = golden("golden_dpsD.npz")
    cfg = ou.Config(**c["unet"])
    sd = {k: torch.from_numpy(v) for k, v in cc.unet_weights(ou.param_shapes(cfg), c["seed"]).items()}
    d, L, co, nh, H = c["siren"]
    ssd = {k: torch.from_numpy(v) for k, v in synth.siren_state_dict(c["siren_seed"], d, L, co, nh, H).items()}
    T = lambda k: torch.from_numpy(g[k])  # noqa: E731
    operator = lambda x0: odps.case4_forward(ssd, T("coords"), T("xhi"), T("xlo"), T("yhi"), T("ylo"),  # noqa: E731
                                             T("vmax"), T("vmin"), x0, batch=16)
    unet = lambda x, t: ou.forward(sd, cfg, x, t)  # noqa: E731
    tb = od.Tables(1000, "cosine", c["respacing"])
    S = c["unet"]["image_size"]
    for j, idx in enumerate(c["indices"]):
        x = torch.from_numpy(synth.normal(c["siren_seed"], f"dpsD/x{idx}", (1, 1, S, L)))
        nz = torch.from_numpy(cc.noise_for(f"{c['tag']}/{idx}", 0, (1, 1, S, L)))
        img, x0, sample, norm = odps.dps_step(tb, unet, operator, x, idx, T("measurement"), nz, c["scale"])
        sc = max(1.0, float(np.abs(g[f"img{j}"]).max()))
        assert np.abs(x0.numpy() - g[f"x0{j}"]).max() < 2e-5 * sc, idx
        assert np.abs(sample.numpy() - g[f"sample{j}"]).max() < 2e-5 * sc, idx
        assert np.abs(img.numpy() - g[f"img{j}"]).max() < 2e-5 * sc, idx
        assert abs(float(norm) - float(g[f"dist{j}"])) < 1e-5 * float(g[f"dist{j}"]), idx


def test_oracle_case4_operator_from_files(tmp_path):
    """The operator's file formats (measurements.py:184-217) read by the oracle
    side: y bounds from y_normalizer0u (upper) / y_normalizer0l (lower), first 3."""
    cc = _cfg_cases()
    c = cc.CASE4_OP
    g = golden("golden_case4op.npz")
    p = cc.case4_files(str(tmp_path))
    prm = torch.load(p["normalizer"], weights_only=True)
    ssd = torch.load(p["ckpt"], weights_only=True)["model_state_dict"]
    xh, xl = prm["x_normalizer_params"]
    yh, yl = prm["y_normalizer0u_params"][0][:3], prm["y_normalizer0l_params"][1][:3]
    x = torch.from_numpy(synth.uniform(c["seed"], "case4op/x", (1, 1, c["T"], c["L"]), -0.95, 0.95))
    with torch.no_grad():
        A = odps.case4_forward(ssd, torch.from_numpy(np.load(p["coords"])).float(), xh, xl, yh, yl,
                               torch.from_numpy(np.load(p["max"])), torch.from_numpy(np.load(p["min"])), x,
                               batch=c["batch_size"])
    assert np.abs(A.numpy() - g["A"]).max() < 2e-5 * max(1.0, float(np.abs(g["A"]).max()))


def test_oracle_configE_segment_prefix():
    """First 4 steps of each config-E segment (128^2 U-Net, 1000-step DDPM)."""
    cc = _cfg_cases()
    c = cc.TRAJ_E
    g = golden("golden_trajE.npz")
    cfg = ou.Config(**c["unet"])
    sd = {k: torch.from_numpy(v) for k, v in cc.unet_weights(ou.param_shapes(cfg), c["seed"]).items()}
    tb = od.Tables(1000, "cosine", "")
    S = c["image_size"]
    shape = (1, 1, S, S)
    keep = [int(k) for k in g["keep"]]
    with torch.no_grad():
        for start, _ in c["segments"]:
            x = torch.from_numpy(cc.noise_for(f"{c['tag']}/x{start}", 0, shape))
            for k, i in enumerate(range(start, start - 4, -1)):
                t = torch.full((1,), i, dtype=torch.int64)
                eps = ou.forward(sd, cfg, x, t)
                x, x0 = od.ddpm_step(tb, x, t, eps, torch.from_numpy(cc.noise_for(f"{c['tag']}/{start}", k, shape)))
                if k in keep:
                    j = keep.index(k)
                    assert np.abs(x.numpy() - g[f"samples{start}"][j]).max() < 2e-5, (start, k)
                    amp = max(1.0, float(tb.sqrt_recipm1_alphas_cumprod[i]))
                    assert np.abs(x0.numpy() - g[f"pred_xstart{start}"][j]).max() < 2e-5 * amp, (start, k)


def test_oracle_configE_100_step_fixture_prefix():
    """The first 11 steps (keep indices 0 and 10) of the 100-step config-E
    fixture (indices 599..500) through the oracle: bit-level agreement with the
    reference's own run pins the fixture the GPU drift test reads."""
    cc = _cfg_cases()
    c, ce = cc.TRAJ_E100, cc.TRAJ_E
    g = golden("golden_trajE100.npz")
    cfg = ou.Config(**ce["unet"])
    sd = {k: torch.from_numpy(v) for k, v in cc.unet_weights(ou.param_shapes(cfg), ce["seed"]).items()}
    tb = od.Tables(1000, "cosine", "")
    S = ce["image_size"]
    shape = (1, 1, S, S)
    keep = [int(k) for k in g["keep"]]
    with torch.no_grad():
        x = torch.from_numpy(cc.noise_for(f"{c['tag']}/x", 0, shape))
        for k, i in enumerate(range(c["start"], c["start"] - 11, -1)):
            t = torch.full((1,), i, dtype=torch.int64)
            eps = ou.forward(sd, cfg, x, t)
            x, x0 = od.ddpm_step(tb, x, t, eps, torch.from_numpy(cc.noise_for(f"{c['tag']}/steps", k, shape)))
            if k in keep:
                j = keep.index(k)
                assert np.abs(x.numpy() - g["samples"][j]).max() < 2e-5, k
                amp = max(1.0, float(tb.sqrt_recipm1_alphas_cumprod[i]))
                assert np.abs(x0.numpy() - g["pred_xstart"][j]).max() < 2e-5 * amp, k


def test_oracle_case4_chain_first_step(tmp_path):
    """The first step of the real-Case4 10-step chain fixture (384^2 U-Net, the
    file-built operator) through the oracle's autograd DPS step."""
    cc = _cfg_cases()
    c, cs = cc.CASE4_OP, cc.CASE4_STEPS
    g = golden("golden_case4steps.npz")
    p = cc.case4_files(str(tmp_path))
    prm = torch.load(p["normalizer"], weights_only=True)
    ssd = torch.load(p["ckpt"], weights_only=True)["model_state_dict"]
    xh, xl = prm["x_normalizer_params"]
    yh, yl = prm["y_normalizer0u_params"][0][:3], prm["y_normalizer0l_params"][1][:3]
    coords = torch.from_numpy(np.load(p["coords"])).float()
    vmax, vmin = torch.from_numpy(np.load(p["max"])), torch.from_numpy(np.load(p["min"]))
    operator = lambda x0: odps.case4_forward(ssd, coords, xh, xl, yh, yl, vmax, vmin, x0,  # noqa: E731
                                             batch=c["batch_size"])
    cfg = ou.Config(**{**c["unet"], "channel_mult": c["unet"]["channel_mult"].replace(" ", "")})
    sd = {k: torch.from_numpy(v) for k, v in synth.unet_state_dict(c["unet_seed"], ou.param_shapes(cfg)).items()}
    unet = lambda x, t: ou.forward(sd, cfg, x, t)  # noqa: E731
    shape = (1, 1, c["T"], c["L"])
    y = torch.from_numpy(golden("golden_case4op.npz")["A"])
    x = torch.from_numpy(synth.normal(c["seed"], f"case4steps/x{cs['start']}", shape))
    idx = cs["start"]
    nz = torch.from_numpy(cc.noise_for(f"case4steps/{idx}", 0, shape))
    img, x0, _, norm = odps.dps_step(od.Tables(1000, "cosine", ""), unet, operator, x, idx, y, nz, 1.0)
    sc = max(1.0, float(np.abs(g["img_sub"][0]).max()))
    assert np.abs(img[..., ::4, ::4].numpy() - g["img_sub"][0]).max() < 2e-5 * sc
    assert np.abs(x0[..., ::4, ::4].numpy() - g["x0_sub"][0]).max() < 2e-5
    assert abs(float(norm) - float(g["dists"][0])) < 1e-5 * float(g["dists"][0])


def _cnftrain_case():
    g = golden("golden_cnftrain.npz")
    c = ast.literal_eval(str(g["case"]))
    sd = {k: torch.from_numpy(v) for k, v in
          synth.siren_state_dict(c["seed"], c["d"], c["L"], c["c"], c["nh"], c["H"]).items()}
    sizes = [int(s) for s in g["batch_sizes"]]
    order = [int(i) for i in g["batch_order"]]
    batches, o = [], 0
    for s in sizes:
        batches.append(order[o:o + s])
        o += s
    return g, c, sd, batches


def test_oracle_cnf_training_loop_matches_reference():
    """oracle/cnf_train.py (the restated _single_trainer loop, train.py:385-416)
    against the reference's own run (make_golden_train.py): first-backward
    gradients, per-batch losses, final parameters and latents."""
    from oracle import cnf_train as oct
    g, c, sd, batches = _cnftrain_case()
    sd_f, lat_f, losses, first = oct.train(sd, torch.from_numpy(g["latents0"]), torch.from_numpy(g["coords"]),
                                           torch.from_numpy(g["fois"]), batches, c["epochs"], c["lr_nf"],
                                           c["lr_latents"])
    for k, v in first["net"].items():
        ref = g["g_" + k]
        assert np.abs(v.numpy() - ref).max() <= 1e-6 * max(1.0, np.abs(ref).max()), k
    assert np.abs(first["latents"].numpy() - g["g_latents"]).max() <= 1e-6 * np.abs(g["g_latents"]).max()
    assert np.allclose(losses, g["losses"], rtol=1e-6, atol=0)
    for k, v in sd_f.items():
        assert np.abs(v.numpy() - g["p_" + k]).max() <= 1e-6, k
    assert np.abs(lat_f.numpy() - g["latents_final"]).max() <= 1e-6


def test_oracle_unet_trainloop_matches_reference():
    """oracle/unet_train.py (the restated TrainLoop step: q_sample, eps MSE,
    backward, AdamW, EMA; train_util.py:178-226) against the reference's own run
    (make_golden_unet_train.py): losses, first-step gradients, parameters and
    EMA after two steps (tolerances: tests/unettrain_check.py)."""
    from oracle import unet_train as out
    from unettrain_check import check
    g = golden("golden_unettrain.npz")
    c = ast.literal_eval(str(g["case"]))
    kw = ast.literal_eval(str(g["kwargs"]))
    cfg = ou.Config(**kw)
    shapes = ou.param_shapes(cfg)
    sd = {k: torch.from_numpy(v) for k, v in synth.unet_state_dict(int(g["weight_seed"]), shapes).items()}
    names = [str(n) for n in g["names"]]
    assert sorted(names) == sorted(sd)
    sd_f, ema, losses, first = out.train(sd, cfg, torch.from_numpy(g["x0"]), c["t"],
                                         [torch.from_numpy(n) for n in g["noise"]], c["lr"], c["weight_decay"],
                                         c["ema_rate"], c["schedule"])
    rep = check(g, c, names, losses, {k: v.numpy() for k, v in first.items()},
                {k: v.numpy() for k, v in sd_f.items()}, {k: v.numpy() for k, v in ema.items()},
                rtol_loss0=1e-6, rtol_loss1=1e-5, tol_grad=1e-5, atol_grad=1e-7, tol_param=1e-6,
                frac_loose=1e-3)
    print(rep)
