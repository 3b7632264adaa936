"""GPU parity of the U-Net parameter gradients (K11, cfd_unet_param_grad: the
backward of the diffusion TrainLoop, U/src/train_util.py:196-240) against torch
autograd through the CPU oracle U-Net (pinned to the reference by the golden
fixtures), on the reference-pinned topologies: every convolution weight / bias,
GroupNorm gamma / beta, emb_layers and time_embed parameter.

Tolerance (fp32 weight-gradient products over the pixels, summed in a different
order than autograd, on top of the split-f16 forward): each gradient tensor
within 2e-4 of its max magnitude (the input-gradient test's bound), floored at
1e-3 of the largest gradient of the model (gradients that vanish analytically
are rounding noise on both sides; measured 5e-6 where none vanish, heads16).
"""
import ast

import numpy as np
import pytest
import torch

from conftest import golden
from confild_amd import synth
from confild_amd.script_util import create_model
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


@pytest.mark.parametrize("name", ["tiny16", "small32", "heads16"])
def test_unet_param_grad_matches_autograd(hip, name):
    g, cfg, sd, m = _unet(name)
    x = torch.from_numpy(g["x"])
    t = torch.from_numpy(g["t"])
    d_eps = torch.from_numpy(synth.normal(5, f"{name}/deps", tuple(x.shape)))
    params = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    eps_ref = ou.forward(params, cfg, x, t)
    grads = torch.autograd.grad(eps_ref, list(params.values()), d_eps)
    ref = dict(zip(params.keys(), grads))
    m.forward_tape(x.to(DEV), t.to(DEV))
    flat = m.param_grad(d_eps.to(DEV)).cpu()
    named = dict(m.named_parameters())
    gmax = max(float(r.abs().max()) for r in ref.values())
    o, errs = 0, []
    for k in m.param_keys():
        n = named[k].numel()
        got = flat[o:o + n].reshape(named[k].shape)
        o += n
        r = ref[k]
        # floor: gradients that vanish analytically (the biases in front of a one-channel-
        # per-group GroupNorm, at 32 channels: its output ignores per-channel shifts) are
        # sums of O(1-100) pixel terms cancelling to rounding noise on both sides (~1e-5)
        scale = max(float(r.abs().max()), 1e-3 * gmax)
        errs.append((float((got - r).abs().max()) / scale, k, float(r.abs().max())))
    assert o == flat.numel()
    errs.sort(reverse=True)
    print(f"{name}: {len(ref)} parameter gradients (max |grad| {gmax:.3e}); worst: {errs[:4]}")
    assert errs[0][0] < 2e-4, errs[:8]


def test_unet_param_grad_accumulates_and_is_deterministic(hip):
    g, cfg, sd, m = _unet("tiny16")
    x = torch.from_numpy(g["x"]).to(DEV)
    t = torch.from_numpy(g["t"]).to(DEV)
    d = torch.from_numpy(synth.normal(6, "acc/d", tuple(x.shape))).to(DEV)
    m.forward_tape(x, t)
    g1 = m.param_grad(d)
    g2 = m.param_grad(d)
    assert torch.equal(g1, g2)
    acc = m.param_grad(d, g1.clone())
    assert float((acc - 2 * g1).abs().max()) <= 1e-6 * float(g1.abs().max())
