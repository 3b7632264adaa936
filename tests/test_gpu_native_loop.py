"""GPU: the native reverse loop (csrc/sampler.hip, cfd_sampler_*) against the
Python per-step loop it replaces (cfd_unet_forward + cfd_sched_step per step,
gaussian_diffusion.py:441-535 / 625-707).  Same kernels, same arguments, Philox
counter = step number: the results must be bit-identical, captured into a HIP
graph (1 or several steps per graph) or launched from the native host loop, for
DDPM and DDIM, respaced and not, and for a sharded batch (sample_offset)."""
import ast

import pytest
import torch

from conftest import golden
from confild_amd import gaussian_diffusion as gd
from confild_amd import synth
from confild_amd.script_util import create_gaussian_diffusion, create_model

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _model(name):
    g = golden(f"unet_{name}.npz")
    kw = ast.literal_eval(str(g["kwargs"]))
    m = create_model(**kw)
    sd = synth.unet_state_dict(int(g["seed"]), {k: tuple(v.shape) for k, v in m.state_dict().items()})
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    return m.to(DEV), kw


def _run(monkeypatch, mode, unroll, fn, *a, **k):
    monkeypatch.setattr(gd, "NATIVE_MODE", mode)
    monkeypatch.setattr(gd, "GRAPH_UNROLL", unroll)
    return fn(*a, **k)


@pytest.mark.parametrize("respacing,ddim,B", [("8", False, 2), ("ddim5", True, 1), ("10,20,30", False, 3)])
def test_native_loop_bit_identical_to_python_loop(hip, monkeypatch, respacing, ddim, B):
    m, kw = _model("tiny16")
    S = kw["image_size"]
    d = create_gaussian_diffusion(steps=1000, noise_schedule="cosine", timestep_respacing=respacing)
    loop = d.ddim_sample_loop if ddim else d.p_sample_loop
    ref = _run(monkeypatch, 0, 1, loop, m, (B, 1, S, S), seed=1234)
    for mode, unroll in ((1, 1), (2, 1), (2, 4), (2, 7)):
        got = _run(monkeypatch, mode, unroll, loop, m, (B, 1, S, S), seed=1234)
        assert torch.equal(got, ref), (respacing, mode, unroll, (got - ref).abs().max().item())
    # the graph replays again with another seed and explicit initial noise
    x0 = torch.from_numpy(synth.normal(3, "x0", (B, 1, S, S))).to(DEV)
    a = _run(monkeypatch, 0, 1, loop, m, (B, 1, S, S), noise=x0, seed=99)
    b = _run(monkeypatch, 2, 4, loop, m, (B, 1, S, S), noise=x0, seed=99)
    assert torch.equal(a, b)
    assert torch.isfinite(b).all() and not torch.equal(b, x0)


def test_native_loop_sharded_and_64px(hip, monkeypatch):
    """config-B widths (64^2 U-Net), 3 steps of the "256" schedule's pattern on a
    short respacing; a sharded batch equals the unsharded one."""
    m, kw = _model("cfgB64")
    d = create_gaussian_diffusion(steps=1000, noise_schedule="cosine", timestep_respacing="6")
    full = _run(monkeypatch, 0, 1, d.p_sample_loop, m, (3, 1, 64, 64), seed=5)
    nat = _run(monkeypatch, 2, 4, d.p_sample_loop, m, (3, 1, 64, 64), seed=5)
    assert torch.equal(full, nat)
    a = _run(monkeypatch, 2, 4, d.p_sample_loop, m, (1, 1, 64, 64), seed=5, sample_offset=0)
    b = _run(monkeypatch, 2, 4, d.p_sample_loop, m, (2, 1, 64, 64), seed=5, sample_offset=1)
    assert torch.equal(torch.cat([a, b]), full)


def test_native_loop_sees_new_weights_and_compute(hip, monkeypatch):
    """A captured graph keeps the weight arena's pointers: weights loaded later are
    used; a compute-mode change re-captures."""
    m, kw = _model("tiny16")
    S = kw["image_size"]
    d = create_gaussian_diffusion(steps=1000, noise_schedule="cosine", timestep_respacing="5")
    first = _run(monkeypatch, 2, 4, d.p_sample_loop, m, (1, 1, S, S), seed=3)
    with torch.no_grad():
        for p in m.parameters():
            p.mul_(0.5)
    ref = _run(monkeypatch, 0, 1, d.p_sample_loop, m, (1, 1, S, S), seed=3)
    got = _run(monkeypatch, 2, 4, d.p_sample_loop, m, (1, 1, S, S), seed=3)
    assert torch.equal(got, ref) and not torch.equal(got, first)
    m.set_compute("fp32")
    ref32 = _run(monkeypatch, 0, 1, d.p_sample_loop, m, (1, 1, S, S), seed=3)
    got32 = _run(monkeypatch, 2, 4, d.p_sample_loop, m, (1, 1, S, S), seed=3)
    assert torch.equal(got32, ref32)
    m.set_compute("split_f16")


def test_native_loop_range_guard(hip, monkeypatch):
    """The split-f16 range guard fires in the native loop too (first conv weights x 1e5)."""
    from confild_amd import _lib
    m, kw = _model("tiny16")
    S = kw["image_size"]
    big = {k: v.clone() for k, v in m.state_dict().items()}
    big["input_blocks.0.0.weight"] *= 1e5
    m.load_state_dict(big)
    d = create_gaussian_diffusion(steps=1000, noise_schedule="cosine", timestep_respacing="4")
    with pytest.raises(_lib.CfdError):
        _run(monkeypatch, 2, 4, d.p_sample_loop, m, (1, 1, S, S), seed=3)
