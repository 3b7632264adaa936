"""CPU tests of the host side: library exports, reference key layout, schedule
tables, factories and failure behaviour.  No GPU calls."""
import ast
import ctypes as C
import os
import re

import numpy as np
import pytest
import torch

from conftest import ROOT, golden
from confild_amd import _lib
from confild_amd import gaussian_diffusion as gd
from confild_amd.respace import space_timesteps
from confild_amd.script_util import create_gaussian_diffusion, create_model
from oracle import diffusion as od


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    hdr = open(os.path.join(ROOT, "include", "confild.h")).read()
    declared = set(re.findall(r"\b(cfd_[a-z_0-9]+)\s*\(", hdr))
    assert declared, "no declarations parsed"
    for name in declared:
        assert hasattr(lib, name), name
    assert declared == set(_lib.EXPORTS)
    assert b"gfx950" in lib.cfd_version()


def test_so_contains_gfx950_code_object():
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_no_cpu_fallback():
    m = create_model(image_size=16, num_channels=32, num_res_blocks=1, channel_mult="1,2", num_heads=4,
                     num_head_channels=16, attention_resolutions="8")
    with pytest.raises(_lib.CfdError):
        m(torch.zeros(1, 1, 16, 16), torch.zeros(1, dtype=torch.int64))


@pytest.mark.parametrize("name", ["tiny16", "small32", "heads16", "cfgA32", "cfgB64", "cfgE128"])
def test_unet_state_dict_keys_match_reference(name):
    g = golden(f"unet_{name}.npz")
    kw = ast.literal_eval(str(g["kwargs"]))
    m = create_model(**kw)
    sd = m.state_dict()
    assert list(sd.keys()) == list(g["keys"])
    assert sum(v.numel() for v in sd.values()) == int(g["nparams"])


def test_create_model_errors_like_reference():
    with pytest.raises(ValueError):
        create_model(image_size=384, num_channels=128, num_res_blocks=2)  # no default mult (script_util.py:160)
    with pytest.raises(NotImplementedError):
        create_model(image_size=64, num_channels=128, num_res_blocks=2, use_scale_shift_norm=True)


RESP = {"id": "", "s256": "256", "ddim50": "ddim50", "ddim5": "ddim5", "s8": "8", "s10_20_30": "10,20,30"}


@pytest.mark.parametrize("tag", list(RESP))
def test_product_tables_bitexact_vs_reference(tag):
    S = golden("schedules.npz")
    d = create_gaussian_diffusion(steps=1000, noise_schedule="cosine", timestep_respacing=RESP[tag])
    assert np.array_equal(np.array(d.timestep_map), S[f"{tag}_timestep_map"])
    for a in ("betas", "alphas_cumprod", "alphas_cumprod_prev", "sqrt_recip_alphas_cumprod",
              "sqrt_recipm1_alphas_cumprod", "posterior_variance", "posterior_log_variance_clipped",
              "posterior_mean_coef1", "posterior_mean_coef2"):
        assert np.array_equal(getattr(d, a), S[f"{tag}_{a}"]), a


def test_space_timesteps_matches_reference_errors():
    S = golden("schedules.npz")
    for args, want in zip(((1000, "ddim256"), (10, "20"), (100, "ddim7")), list(S["space_errors"])):
        try:
            space_timesteps(*args)
            got = "ok"
        except ValueError as e:
            got = "ValueError:" + str(e)
        assert got == want


def test_coef_table_matches_oracle_step_scalars():
    """The fp32 per-step scalars the kernel uses are exactly the reference's
    extracted-and-cast values (checked through the oracle's formulas)."""
    d = create_gaussian_diffusion(steps=1000, noise_schedule="cosine", timestep_respacing="256")
    tab = d.coef_table()
    tb = od.Tables(1000, "cosine", "256")
    f = lambda a: torch.from_numpy(a).float()  # noqa: E731
    assert torch.equal(tab[:, gd.SRA], f(tb.sqrt_recip_alphas_cumprod))
    assert torch.equal(tab[:, gd.SRM1], f(tb.sqrt_recipm1_alphas_cumprod))
    assert torch.equal(tab[:, gd.M1], f(tb.posterior_mean_coef1))
    assert torch.equal(tab[:, gd.M2], f(tb.posterior_mean_coef2))
    assert torch.equal(tab[:, gd.SIGMA], torch.exp(0.5 * f(tb.fixed_large_logvar)))


def test_step_arithmetic_emulation_bitexact():
    """Emulate the kernel's fp32 operation order on the CPU (no FMA) and compare
    with the oracle step bit for bit: documents why the GPU step is bit-exact."""
    tr = golden("traj_ddpm8.npz")
    d = create_gaussian_diffusion(steps=1000, noise_schedule="cosine", timestep_respacing="8")
    tab = d.coef_table().numpy()
    tb = od.Tables(1000, "cosine", "8")
    x = tr["noise0"]
    eps = np.random.default_rng(0).standard_normal(x.shape).astype(np.float32)
    z = tr["noise"][0]
    t = 7
    c = tab[t]
    xs = np.clip(c[gd.SRA] * x - c[gd.SRM1] * eps, -1, 1).astype(np.float32)
    mean = c[gd.M1] * xs + c[gd.M2] * x
    out = mean + np.float32(1.0) * c[gd.SIGMA] * z
    ref, _ = od.ddpm_step(tb, torch.from_numpy(x), torch.full((2,), t), torch.from_numpy(eps), torch.from_numpy(z))
    assert np.array_equal(out, ref.numpy())


def test_siren_state_dict_keys_match_reference_layout():
    from confild_amd.nf_networks import SIRENAutodecoder_film
    net = SIRENAutodecoder_film(3, 384, 3, 15, 384)
    keys = list(net.state_dict().keys())
    assert keys[0] == "net1.0.weight" and keys[-1] == "net2.15.weight"
    assert net.state_dict()["net1.16.weight"].shape == (3, 384)
    assert sum(v.numel() for v in net.state_dict().values()) == 4579587  # reference SIRENAutodecoder_film(3,384,3,15,384)


def test_trainer_loads_reference_files(tmp_path):
    import yaml
    from confild_amd import synth
    from confild_amd.read_input import basic_input
    from confild_amd.trainer import trainer
    sd = synth.siren_state_dict(5, 3, 8, 3, 2, 32)
    torch.save({"x_normalizer_params": (torch.ones(1, 3), torch.zeros(1, 3)),
                "y_normalizer_params": (torch.ones(1, 5, 3), -torch.ones(1, 5, 3))},
               tmp_path / "normalizer_params.pt")
    for ep in (2, 11):
        torch.save({"epoch": ep, "model_state_dict": {k: torch.from_numpy(v) for k, v in sd.items()},
                    "optim_net_dec_dict": {}, "optim_states_dict": {}, "hidden_states": {}},
                   tmp_path / f"checkpoint_{ep}.pt")
    cfg = {"save_path": str(tmp_path), "lumped_latent": True, "normalizer": {"method": "-11", "dim": 0},
           "multiGPU": 1, "hidden_size": 8, "dims": 3,
           "NF": {"name": "SIRENAutodecoder_film", "out_features": 3, "num_hidden_layers": 2, "hidden_features": 32}}
    (tmp_path / "c.yml").write_text(yaml.safe_dump(cfg))
    tr = trainer(basic_input(str(tmp_path / "c.yml")), infer_mode=True)
    tr.load(-1, siren_only=True)
    assert tr.start_epoch == 11
    assert torch.equal(tr.nf.state_dict()["net1.1.weight"], torch.from_numpy(sd["net1.1.weight"]))
    with pytest.raises(FileNotFoundError):
        cfg["save_path"] = str(tmp_path / "missing")
        (tmp_path / "d.yml").write_text(yaml.safe_dump(cfg))
        trainer(basic_input(str(tmp_path / "d.yml")), infer_mode=True)


def test_inference_precision_key():
    """inference.py's optional precision / compute YAML keys (config E reachable
    through the drop-in driver)."""
    from types import SimpleNamespace as NS
    from confild_amd.inference import unet_compute
    assert unet_compute(NS()) == "split_f16"
    assert unet_compute(NS(precision="fp32")) == "split_f16"
    assert unet_compute(NS(precision="bf16")) == "bf16"
    assert unet_compute(NS(precision="bf16", compute="fp32")) == "fp32"
    with pytest.raises(ValueError):
        unet_compute(NS(precision="fp16"))


def test_guided_create_model_fails_loudly(tmp_path):
    """a bad checkpoint raises (the reference silently random-inits,
    C/unet.py:86-90; random_init_on_error=True keeps that behaviour)."""
    from confild_amd.guided.unet import create_model as gcm
    kw = dict(image_size=16, num_channels=32, num_res_blocks=1, channel_mult="1,2", num_heads=4,
              num_head_channels=16, attention_resolutions="8")
    with pytest.raises(RuntimeError):
        gcm(**kw, model_path=str(tmp_path / "missing.pt"))
    torch.save({"bogus": torch.zeros(1)}, tmp_path / "bad.pt")
    with pytest.raises(RuntimeError):
        gcm(**kw, model_path=str(tmp_path / "bad.pt"))
    m = gcm(**kw, model_path=str(tmp_path / "bad.pt"), random_init_on_error=True)
    good = {k: v.clone() + 1 for k, v in m.state_dict().items()}
    torch.save(good, tmp_path / "good.pt")
    m2 = gcm(**kw, model_path=str(tmp_path / "good.pt"))
    assert all(torch.equal(m2.state_dict()[k], v) for k, v in good.items())
    with pytest.warns(UserWarning):
        gcm(**kw)


def test_single_step_default_noise_is_fresh():
    """p_sample / ddim_sample without noise or seed draw a fresh Philox key per call
    (the reference draws a fresh randn_like per call, gaussian_diffusion.py:430)."""
    torch.manual_seed(0)
    a = gd.fresh_seed(None, None)
    b = gd.fresh_seed(None, None)
    assert a != b
    assert gd.fresh_seed(torch.zeros(1), None) == 0
    assert gd.fresh_seed(None, 7) == 7


def _cfg_cases():
    import sys
    from conftest import GOLDEN
    if GOLDEN not in sys.path:
        sys.path.insert(0, GOLDEN)
    import cfg_cases
    return cfg_cases


@pytest.mark.parametrize("name", ["grid2d", "lumped3d_pub"])
def test_cnf_inference_host_side_matches_reference(tmp_path, name):
    """CNF_inference (inference_function.py:79-304) on CPU: checkpoint / normaliser /
    YAML loading, the is_pub remap of a bare latent tensor, LatentContainer's
    expand dims and create_coordinates_grid, against the reference's own run."""
    from confild_amd.inference_function import CNF_inference
    cc = _cfg_cases()
    c = cc.CNF_INF[name]
    g = golden("golden_cnfinf.npz")
    f = cc.cnf_inference_files(str(tmp_path), name)
    inf = CNF_inference(f["checkpoint"], f["config"], f["data"], device="cpu", is_pub=c["is_pub"])
    assert np.array_equal(inf.create_coordinates_grid().numpy(), g[f"{name}_grid"])
    shape = tuple(c["data_shape"][1:-1])[:3] if len(c["data_shape"]) > 3 else (5, 4)
    assert np.array_equal(inf.create_coordinates_grid(shape).numpy(), g[f"{name}_grid_shape"])
    assert tuple(inf.latents(torch.LongTensor([1, 2])).shape) == tuple(g[f"{name}_latent_shape"])
    ck = torch.load(f["checkpoint"], weights_only=True)
    lat = ck["hidden_states"] if c["is_pub"] else ck["hidden_states"]["latents"]
    assert torch.equal(inf.latents.latents.detach(), lat)
    with pytest.raises(_lib.CfdError):      # no CPU fallback for the decode itself
        inf.predict(torch.from_numpy(cc.cnf_inference_coords(name)), [0])
    with pytest.raises(FileNotFoundError):
        CNF_inference(f["checkpoint"] + ".missing", f["config"], f["data"], device="cpu")
    if not c["is_pub"]:   # no latent codes in hidden_states (inference_function.py:185-187)
        torch.save({**ck, "hidden_states": {}}, f["checkpoint"])
        with pytest.raises(ValueError):
            CNF_inference(f["checkpoint"], f["config"], f["data"], device="cpu")


def test_reconstruct_frame_matches_reference():
    """ReconstructFrame (inference_function.py:15-19): scatter of masked points
    into the infos.npz Mask grid, zero and default-NaN fill, as the reference
    produced them in the Case4 notebook's post-processing chain (golden_post)."""
    from confild_amd.inference_function import ReconstructFrame
    cc = _cfg_cases()
    g = golden("golden_post.npz")
    mask = cc.post_inputs()[0]
    fr = g["frames"]
    for s in range(fr.shape[0]):
        for t in range(fr.shape[1]):
            out = ReconstructFrame(fr[s, t][mask], mask=mask, shape=cc.POST["grid"], fill_value=0.)
            assert np.array_equal(out.astype(np.float32), fr[s, t])
    nanf = ReconstructFrame(g["nan_frame"][mask], mask=mask, shape=cc.POST["grid"])
    assert np.array_equal(np.isnan(nanf), np.isnan(g["nan_frame"]))
    assert np.array_equal(nanf[mask].astype(np.float32), g["nan_frame"][mask])


@pytest.mark.parametrize("shuffle", [False, True])
def test_cnf_train_batch_order_is_the_dataloaders(shuffle):
    """confild_amd.cnf_train draws the reference DataLoader's batch order
    (train.py:375-380): the same sampler classes and the same global-RNG draws."""
    from torch.utils.data import DataLoader, Dataset
    from confild_amd.cnf_train import _batches

    class _Idx(Dataset):
        def __len__(self):
            return 11

        def __getitem__(self, i):
            return i

    for epoch in range(2):
        torch.manual_seed(7 + epoch)
        want = [b.tolist() for b in DataLoader(_Idx(), batch_size=4, shuffle=shuffle)]
        torch.manual_seed(7 + epoch)
        assert _batches(11, 4, shuffle, 1, 0, epoch) == want


def test_cnf_train_distributed_batches_are_the_reference_loaders():
    """world_size > 1: the reference's ``DataLoader(dataset, shuffle=False,
    sampler=DistributedSampler(dataset))`` (train.py:360-365) -- the sampler's
    default shuffle=True, seed 0 -- with ``set_epoch(i)`` each epoch (train.py:398):
    a different random shard per rank and epoch, together a partition."""
    from torch.utils.data import DataLoader, Dataset, DistributedSampler
    from confild_amd.cnf_train import _batches

    class _Idx(Dataset):
        def __len__(self):
            return 10

        def __getitem__(self, i):
            return i

    seen = []
    for epoch in range(3):
        got_all = []
        for r in range(2):
            sampler = DistributedSampler(_Idx(), num_replicas=2, rank=r)
            sampler.set_epoch(epoch)
            torch.manual_seed(11 + epoch)
            want = [b.tolist() for b in DataLoader(_Idx(), batch_size=3, shuffle=False, sampler=sampler)]
            torch.manual_seed(11 + epoch)
            got = _batches(10, 3, False, 2, r, epoch)
            assert got == want
            got_all += [i for b in got for i in b]
        assert sorted(got_all) == list(range(10))
        seen.append(got_all)
    assert seen[0] != seen[1], "set_epoch must reshuffle the shards"


def test_schedule_samplers_match_reference_draws():
    """confild_amd.resample (U/src/resample.py): UniformSampler draws with the
    reference's numpy call (np.random.choice over p = w / sum(w), weights
    1 / (T p[t]) -- exactly 1 for the uniform case); LossSecondMomentResampler
    stays uniform until every step has history_per_term losses, then weights by
    the RMS of the recent losses mixed with uniform_prob."""
    from confild_amd.resample import LossSecondMomentResampler, create_named_schedule_sampler
    diff = create_gaussian_diffusion(steps=50, noise_schedule="cosine")
    s = create_named_schedule_sampler("uniform", diff)
    np.random.seed(3)
    t, w = s.sample(7, "cpu")
    np.random.seed(3)
    assert t.tolist() == np.random.choice(50, size=(7,), p=np.ones(50) / 50).tolist()
    assert t.dtype == torch.int64 and torch.equal(w, torch.ones(7))
    ls = LossSecondMomentResampler(diff, history_per_term=2, uniform_prob=0.1)
    ts = list(range(50))
    ls.update_with_all_losses(ts, [1.0] * 50)
    assert np.array_equal(ls.weights(), np.ones(50))
    ls.update_with_local_losses(torch.arange(50), torch.arange(50, dtype=torch.float32))
    w = ls.weights()
    rms = np.sqrt((1.0 + np.arange(50.0) ** 2) / 2)
    assert np.allclose(w, rms / rms.sum() * 0.9 + 0.1 / 50)
    with pytest.raises(NotImplementedError):
        create_named_schedule_sampler("nope", diff)


def test_trainloop_host_side():
    """TrainLoop helpers (train_util.py:298-331) and its loud refusals."""
    from confild_amd.train_util import TrainLoop, find_ema_checkpoint, parse_resume_step_from_filename
    assert parse_resume_step_from_filename("/a/b/model012345.pt") == 12345
    assert parse_resume_step_from_filename("/a/b/ema.pt") == 0
    assert find_ema_checkpoint(None, 3, 0.9) is None
    m = create_model(image_size=16, num_channels=32, num_res_blocks=1, attention_resolutions="8",
                     channel_mult="1,2")
    diff = create_gaussian_diffusion(steps=100, noise_schedule="cosine")
    kw = dict(model=m, diffusion=diff, train_data=None, batch_size=2, microbatch=-1, lr=1e-4, ema_rate="0.9999",
              log_interval=1, save_interval=1, resume_checkpoint="")
    with pytest.raises(NotImplementedError):
        TrainLoop(**kw, use_fp16=True)
    with pytest.raises(_lib.CfdError):
        TrainLoop(**kw)                      # a CPU model: the loop runs on the GPU only


@pytest.mark.parametrize("case", ["tiny", "cfgA32", "cfgB64"])
def test_flop_counts_match_flopcounter_on_the_oracle(case):
    """confild_amd.unet.forward_flops (the bench's roofline numerator) equals
    torch's FlopCounterMode over the oracle forward, and forward conv + 2 x
    attention equals its count of the input-gradient (autograd.grad to x: the
    DPS adjoint); nf_networks.latent_grad_flops equals FlopCounterMode over the
    oracle SIREN forward and its gradient to the latents."""
    from torch.utils.flop_counter import FlopCounterMode

    from confild_amd import synth
    from confild_amd.nf_networks import latent_grad_flops
    from confild_amd.unet import forward_flops
    from oracle import siren as osn
    from oracle import unet as ou
    kw = {"tiny": dict(image_size=16, num_channels=32, num_res_blocks=1, channel_mult="1,2", num_heads=2,
                       num_head_channels=16, attention_resolutions="8"),
          "cfgA32": dict(image_size=32, num_channels=128, num_res_blocks=2, channel_mult="1,2,3,4", num_heads=4,
                         num_head_channels=64, attention_resolutions="32,16,8"),
          "cfgB64": dict(image_size=64, num_channels=128, num_res_blocks=2, channel_mult="", num_heads=4,
                         num_head_channels=64, attention_resolutions="32,16,8")}[case]
    cfg = ou.Config(**kw)
    sd = {k: torch.from_numpy(v) for k, v in synth.unet_state_dict(1, ou.param_shapes(cfg)).items()}
    S = kw["image_size"]
    x = torch.randn(1, 1, S, S, requires_grad=True)
    with FlopCounterMode(display=False) as fc:
        eps = ou.forward(sd, cfg, x, torch.tensor([10]))
    with FlopCounterMode(display=False) as fc2:
        torch.autograd.grad(eps, x, torch.randn_like(eps))
    f = forward_flops(S, 1, cfg.model_channels, 1, cfg.num_res_blocks, set(cfg.attention_ds), cfg.channel_mult,
                      cfg.num_heads, cfg.num_head_channels)
    assert sum(f.values()) == fc.get_total_flops()
    assert f["conv"] + 2 * f["attn"] == fc2.get_total_flops()
    if case == "cfgB64":
        assert sum(f.values()) == 68_614_488_064     # 68.61 GF per sample
    d, L, c, nh, H = 3, 64, 3, 15, 384
    ssd = {k: torch.from_numpy(v) for k, v in synth.siren_state_dict(1, d, L, c, nh, H).items()}
    z = torch.randn(5, 1, L, requires_grad=True)
    with FlopCounterMode(display=False) as fs:
        y = osn.forward(ssd, torch.rand(1, 10, d), z)
    with FlopCounterMode(display=False) as fs2:
        torch.autograd.grad(y, z, torch.randn_like(y))
    assert latent_grad_flops(d, L, c, nh, H, 5, 10) == {"forward": fs.get_total_flops(),
                                                         "backward": fs2.get_total_flops()}
