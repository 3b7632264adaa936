"""GPU end-to-end: shard invariance of the sampler and the inference.py drop-in
driver (tiny shapes).  The driver's output is checked against the product path
composed by hand and its decode against the CPU oracle on the same latents."""
import ast

import numpy as np
import pytest
import torch
import yaml

from conftest import golden
from confild_amd import synth
from confild_amd.script_util import create_gaussian_diffusion, create_model
from oracle import siren as osn
from oracle import unet as ou

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _tiny():
    g = golden("unet_tiny16.npz")
    kw = ast.literal_eval(str(g["kwargs"]))
    m = create_model(**kw)
    sd = synth.unet_state_dict(int(g["seed"]), {k: tuple(v.shape) for k, v in m.state_dict().items()})
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    return kw, m.to(DEV), sd


def test_unet_output_is_batch_invariant(hip):
    """A sample's eps does not depend on the batch it is computed in (fixed
    summation order), so sharding samples over ranks cannot change results."""
    g = golden("unet_cfgB64.npz")
    kw = ast.literal_eval(str(g["kwargs"]))
    m = create_model(**kw)
    sd = synth.unet_state_dict(int(g["seed"]), {k: tuple(v.shape) for k, v in m.state_dict().items()})
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m.to(DEV)
    x = torch.from_numpy(synth.normal(8, "bi", (8, 1, 64, 64))).to(DEV)
    t = torch.arange(8, dtype=torch.int64, device=DEV) * 111
    full = m(x, t)
    for s, e in ((0, 1), (3, 5), (5, 8)):
        assert torch.equal(m(x[s:e], t[s:e]), full[s:e]), (s, e)


def test_sharded_sampling_equals_unsharded(hip):
    _, m, _ = _tiny()
    d = create_gaussian_diffusion(steps=1000, noise_schedule="cosine", timestep_respacing="8")
    full = d.p_sample_loop(m, (4, 1, 16, 16), seed=77)
    a = d.p_sample_loop(m, (1, 1, 16, 16), seed=77, sample_offset=0)
    b = d.p_sample_loop(m, (3, 1, 16, 16), seed=77, sample_offset=1)
    assert torch.equal(torch.cat([a, b]), full)
    # and the run is a real sample: finite, not the initial noise
    assert torch.isfinite(full).all()


@pytest.mark.parametrize("layout", ["lumped", "grid"])
def test_inference_driver_end_to_end(hip, tmp_path, layout):
    """lumped: (N, d) points and a per-point output normaliser, saved (B*T, N, c).
    grid: an (h, w, 2) coordinate grid (the case2 family's train_coord) and a
    per-channel normaliser; the reference keeps the grid and saves (B*T, h, w, c)."""
    from confild_amd import inference
    kw, m, sd = _tiny()
    torch.save({k: torch.from_numpy(v) for k, v in sd.items()}, tmp_path / "ema.pt")
    if layout == "lumped":
        d, L, c, nh, H = 3, 16, 3, 2, 32
        spatial = (300,)
        yhi = torch.from_numpy(synth.uniform(5, "yhi", (1, 300, c), 0.5, 2.0))
    else:
        d, L, c, nh, H = 2, 16, 3, 2, 32
        spatial = (12, 10)
        yhi = torch.from_numpy(synth.uniform(5, "yhi", (1, c), 0.5, 2.0))
    N = int(np.prod(spatial))
    ssd = synth.siren_state_dict(5, d, L, c, nh, H)
    cnf_dir = tmp_path / "cnf"
    cnf_dir.mkdir()
    torch.save({"x_normalizer_params": (torch.ones(1, d), torch.zeros(1, d)),
                "y_normalizer_params": (yhi, -yhi)}, cnf_dir / "normalizer_params.pt")
    torch.save({"epoch": 1, "model_state_dict": {k: torch.from_numpy(v) for k, v in ssd.items()}},
               cnf_dir / "checkpoint_1.pt")
    coords = synth.uniform(5, "coords", spatial + (d,), 0.0, 1.0)
    np.save(tmp_path / "coords.npy", coords)
    cnf_cfg = {"save_path": str(cnf_dir), "coor_path": str(tmp_path / "coords.npy"),
               "lumped_latent": layout == "lumped",
               "normalizer": {"method": "-11", "dim": 0}, "multiGPU": 1, "hidden_size": L, "dims": d,
               "NF": {"name": "SIRENAutodecoder_film", "out_features": c, "num_hidden_layers": nh,
                      "hidden_features": H}}
    (tmp_path / "cnf.yml").write_text(yaml.safe_dump(cnf_cfg))
    np.save(tmp_path / "max.npy", np.float32(1.5))
    np.save(tmp_path / "min.npy", np.float32(-1.5))
    cfg = {"test_batch_size": 2, "time_length": 16, "latent_length": 16, "image_size": 16,
           "num_channels": kw["num_channels"], "num_res_blocks": kw["num_res_blocks"],
           "channel_mult": kw["channel_mult"], "num_heads": kw["num_heads"],
           "num_head_channels": kw["num_head_channels"], "attention_resolutions": kw["attention_resolutions"],
           "ema_path": str(tmp_path / "ema.pt"), "steps": 1000, "noise_schedule": "cosine",
           "timestep_respacing": "8", "max_val": str(tmp_path / "max.npy"), "min_val": str(tmp_path / "min.npy"),
           "cnf_case_file_path": str(tmp_path / "cnf.yml"), "save_path": str(tmp_path / "out.npy")}
    (tmp_path / "case.yml").write_text(yaml.safe_dump(cfg))
    out = inference.run(str(tmp_path / "case.yml"))
    saved = np.load(tmp_path / "out.npy")
    assert saved.shape == (2 * 16,) + spatial + (c,) and np.array_equal(saved, out)

    # same latents through the product path by hand, then the CPU oracle decode
    torch.manual_seed(42)
    seed = int(torch.randint(0, 2 ** 62, (1,)).item())
    diff = create_gaussian_diffusion(steps=1000, noise_schedule="cosine", timestep_respacing="8")
    lat = diff.p_sample_loop(m, (2, 1, 16, 16), seed=seed)[:, 0]
    lat = ((lat + 1) * (1.5 + 1.5) / 2. - 1.5).reshape(32, 16).cpu()
    ref = osn.decode({k: torch.from_numpy(v) for k, v in ssd.items()}, torch.from_numpy(coords).reshape(N, d), lat,
                     torch.ones(1, d), torch.zeros(1, d), yhi, -yhi)
    ref = ref.reshape((32,) + spatial + (c,))
    assert np.abs(saved - ref.numpy()).max() <= 2e-5 * max(1.0, float(ref.abs().max()))
