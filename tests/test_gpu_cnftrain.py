"""GPU parity of the CNF autodecoder training step (K10, SURVEY.md section 8 f4:
N/scripts/train.py:334-416) against the reference's own run
(tests/golden/golden_cnftrain.npz, make_golden_train.py):

* one backward (cfd_siren_train_grad): every net1 / net2 parameter gradient and
  the latent-table gradient;
* the whole loop (confild_amd.cnf_train.train_autodecoder, Adam by
  cfd_adam_step): per-batch losses, final parameters and latents;
* coordinate chunking adds up to the unchunked gradient; two runs are
  bit-identical (no atomics, fixed reduction orders).

Tolerances (fp32; the library sums the pair products in a different order than
autograd): gradients within 1e-5 of each tensor's max magnitude, losses 1e-5
relative; after the Adam steps (whose first update is lr * sign(g), so a
gradient element within rounding of zero may move the other way) parameters
within 1e-5 absolute on all but at most 0.1 % of elements, every element within
2 lr x its step count.
"""
import ast

import numpy as np
import pytest
import torch

from conftest import golden
from confild_amd import synth
from confild_amd.cnf_train import train_autodecoder
from confild_amd.nf_networks import SIRENAutodecoder_film

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _setup():
    g = golden("golden_cnftrain.npz")
    c = ast.literal_eval(str(g["case"]))
    nf = SIRENAutodecoder_film(c["d"], c["L"], c["c"], c["nh"], c["H"])
    nf.load_state_dict({k: torch.from_numpy(v) for k, v in
                        synth.siren_state_dict(c["seed"], c["d"], c["L"], c["c"], c["nh"], c["H"]).items()})
    nf.to(DEV)
    Z = torch.from_numpy(g["latents0"]).to(DEV).contiguous()
    return g, c, nf, Z


def _first_batch(g):
    return [int(i) for i in g["batch_order"][:int(g["batch_sizes"][0])]]


def _grads(nf, Z, g, c, coords, fois, chunk=None):
    rows = torch.tensor(_first_batch(g), dtype=torch.int64, device=DEV)
    grad = torch.zeros_like(nf.flat_params())
    gz = torch.zeros_like(Z)
    sse = torch.zeros(1, device=DEV)
    N = coords.shape[0]
    scale = 2.0 / (len(rows) * N * c["c"])
    per = chunk or N
    for c0 in range(0, N, per):
        nf.train_grad(coords[c0:c0 + per], Z, rows, fois[rows, c0:c0 + per], scale, grad, gz, sse)
    torch.cuda.synchronize()
    return grad, gz, sse


def test_train_grad_matches_reference_backward():
    g, c, nf, Z = _setup()
    coords = torch.from_numpy(g["coords"]).to(DEV)
    fois = torch.from_numpy(g["fois"]).to(DEV)
    grad, gz, sse = _grads(nf, Z, g, c, coords, fois)
    o = 0
    named = dict(nf.named_parameters())
    for k in nf.param_keys():
        n = named[k].numel()
        got = grad[o:o + n].cpu().numpy().reshape(named[k].shape)
        ref = g["g_" + k]
        err = np.abs(got - ref).max() / max(np.abs(ref).max(), 1e-30)
        print(f"{k}: rel err {err:.2e}")
        assert err <= 1e-5, k
        o += n
    err = np.abs(gz.cpu().numpy() - g["g_latents"]).max() / np.abs(g["g_latents"]).max()
    print(f"latents: rel err {err:.2e}")
    assert err <= 1e-5
    R = int(g["batch_sizes"][0])
    loss = float(sse) / (R * coords.shape[0] * c["c"])
    assert abs(loss - g["losses"][0]) <= 1e-5 * g["losses"][0]


def test_train_grad_chunked_equals_whole_and_is_deterministic():
    g, c, nf, Z = _setup()
    coords = torch.from_numpy(g["coords"]).to(DEV)
    fois = torch.from_numpy(g["fois"]).to(DEV)
    g1, z1, s1 = _grads(nf, Z, g, c, coords, fois)
    g2, z2, s2 = _grads(nf, Z, g, c, coords, fois)
    assert torch.equal(g1, g2) and torch.equal(z1, z2) and torch.equal(s1, s2)
    g3, z3, _ = _grads(nf, Z, g, c, coords, fois, chunk=64)
    assert (g3 - g1).abs().max() <= 1e-5 * g1.abs().max()
    assert (z3 - z1).abs().max() <= 1e-5 * z1.abs().max()


def test_training_loop_matches_reference_run():
    g, c, nf, Z = _setup()
    losses = []
    train_autodecoder(nf, Z, torch.from_numpy(g["coords"]), torch.from_numpy(g["fois"]), c["epochs"], c["batch"],
                      {"nf": c["lr_nf"], "latents": c["lr_latents"]}, shuffle=False,
                      on_batch=lambda i, idx, loss: losses.append(loss))
    torch.cuda.synchronize()
    print("losses", losses, "ref", list(g["losses"]))
    assert np.allclose(losses, g["losses"], rtol=1e-5, atol=0)
    n_net_steps = c["epochs"] - 1
    n_lat_steps = len(losses)
    for k, p in nf.named_parameters():
        d = np.abs(p.detach().cpu().numpy() - g["p_" + k])
        print(f"{k}: max {d.max():.2e}, > 1e-5: {(d > 1e-5).mean():.4f}")
        assert (d > 1e-5).mean() <= 1e-3 and d.max() <= 2 * c["lr_nf"] * n_net_steps, k
    d = np.abs(Z.cpu().numpy() - g["latents_final"])
    print(f"latents: max {d.max():.2e}, > 1e-5: {(d > 1e-5).mean():.4f}")
    assert (d > 1e-5).mean() <= 1e-3 and d.max() <= 2 * c["lr_latents"] * n_lat_steps
