"""The planner's nominal batch (cfd_unet_set_plan_batch / UNetModel.set_plan_batch):
a per-model setting that changes the convolution tiles, split-K counts and kernel
family, never with the real batch -- so with any setting a sample's eps and its
DPS input-gradient are bit-identical whatever batch it runs in (the property the
chain sharding rests on), and each setting stays within fp32-level rounding of
the default plan."""
import pytest
import torch

from confild_amd import synth
from confild_amd.script_util import create_model

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _model(S, mult, seed=21):
    m = create_model(image_size=S, num_channels=128, num_res_blocks=2, channel_mult=mult, num_heads=4,
                     num_head_channels=64, attention_resolutions="32,16,8")
    m.load_state_dict({k: torch.from_numpy(v) for k, v in
                       synth.unet_state_dict(seed, {k: tuple(v.shape) for k, v in m.state_dict().items()}).items()})
    return m.to(DEV)


@pytest.mark.parametrize("pb", [1, 2, 4])
def test_plan_batch_forward_is_batch_invariant(hip, pb):
    m = _model(64, "")
    x = torch.from_numpy(synth.normal(8, "pb/x", (3, 1, 64, 64))).to(DEV)
    t = torch.tensor([999, 250, 7], device=DEV)
    ref = m(x, t)                       # the default plan (8)
    m.set_plan_batch(pb)
    full = m(x, t)
    for s in range(3):
        assert torch.equal(m(x[s:s + 1], t[s:s + 1]), full[s:s + 1]), (pb, s)
    err = float((full - ref).abs().max()) / float(ref.abs().max())
    assert err < 1e-5, (pb, err)
    m.set_plan_batch(0)
    assert torch.equal(m(x, t), ref)


def test_plan_batch_input_vjp_is_batch_invariant(hip):
    m = _model(32, "1,2,3,4").set_plan_batch(2)
    x = torch.from_numpy(synth.normal(9, "pb/xv", (2, 1, 32, 32))).to(DEV)
    t = torch.tensor([600, 20], device=DEV)
    d = torch.from_numpy(synth.normal(9, "pb/dv", (2, 1, 32, 32))).to(DEV)
    m.forward_tape(x, t)
    g = m.input_vjp(d)
    for s in range(2):
        m.forward_tape(x[s:s + 1], t[s:s + 1])
        assert torch.equal(m.input_vjp(d[s:s + 1]), g[s:s + 1]), s


def test_plan_batch_rejects_out_of_range(hip):
    m = _model(32, "1,2,3,4")
    with pytest.raises(ValueError):
        m.set_plan_batch(65)


def test_plan_batch_change_resizes_native_loop(hip):
    """A native sampling loop created at one planned batch keeps working after the
    model's planned batch changes (the split-K slab in its workspace grows; its
    graphs are recaptured), and the chains still shard bit-exactly."""
    from confild_amd.script_util import create_gaussian_diffusion
    m = _model(64, "")
    d = create_gaussian_diffusion(steps=1000, noise_schedule="cosine", timestep_respacing="6")
    shape = (2, 1, 64, 64)
    a = d.p_sample_loop(m, shape, seed=5)
    m.set_plan_batch(2)
    b = d.p_sample_loop(m, shape, seed=5)
    one = d.p_sample_loop(m, (1, 1, 64, 64), seed=5, sample_offset=1)
    assert torch.equal(one, b[1:2])
    assert torch.isfinite(b).all()
    assert float((a - b).abs().max()) < 1e-3 * max(1.0, float(a.abs().max()))
