"""The optimiser and EMA kernels in isolation, on identical gradients:

* ``cfd_adam_step`` (through ``confild_amd.cnf_train.Adam``) against
  ``torch.optim.AdamW`` / ``torch.optim.Adam`` stepping the same tensor on the
  same GPU -- the reference's TrainLoop (U/src/train_util.py:78-80, 214-226) and
  CNF loop (N/scripts/train.py:385-416) step on their GPU with torch's default,
  the multi-tensor (foreach) path: **bit-exact** (parameters, exp_avg,
  exp_avg_sq) over several steps, both lerp branches, weight decay on and off;
* against torch's single-tensor path and its CPU kernels, one step from the same
  state: the moments exact (GPU single-tensor) / within 2 ulp (CPU), the parameter within 2^-22 of (its magnitude
  plus the step's) -- i.e. within an ulp of the larger -- the reason, pinned by
  tools/dev/optim_probe.py: the single-tensor GPU path
  divides by the bias-correction scalar as a multiplication by its reciprocal,
  and the CPU kernels run addcmul as fma(value * g, g, v), addcdiv as
  p + (value * m) / denom and a vectorised sqrt that is not always correctly
  rounded;
* ``cfd_ema_update`` against update_ema (U/src/nn.py:71-80,
  ``targ.mul_(rate).add_(src, alpha=1 - rate)``): bit-exact on the GPU and on
  the CPU;
* an AdamW state saved by ``Adam.torch_state_dict`` (the reference's opt*.pt
  layout) loads into ``torch.optim.AdamW``, whose next step equals
  ``cfd_adam_step``'s bit for bit (decoupled decay survives the round trip).
"""
import ctypes as C

import numpy as np
import pytest
import torch

from confild_amd import _lib
from confild_amd.cnf_train import Adam

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _grads(n, steps, seed):
    g = torch.Generator().manual_seed(seed)
    out = []
    for k in range(steps):
        x = torch.randn(n, generator=g) * 10.0 ** (-1 - k % 4)
        x[::97] = 0.0                                    # exact zeros
        x[1::89] *= 1e-20                                # tiny values (v underflows toward 0)
        out.append(x)
    return out


def _ulp(a, b):
    ia = a.cpu().view(torch.int32).to(torch.int64)
    ib = b.cpu().view(torch.int32).to(torch.int64)
    ia = torch.where(ia < 0, -(ia & 0x7FFFFFFF), ia)
    ib = torch.where(ib < 0, -(ib & 0x7FFFFFFF), ib)
    return int((ia - ib).abs().max())


@pytest.mark.parametrize("wd,betas,n", [(0.01, (0.9, 0.999), 1 << 20), (0.0, (0.9, 0.999), 1000003),
                                        (0.05, (0.3, 0.99), 65537)])
def test_adam_step_matches_torch_foreach_on_gpu(hip, wd, betas, n):
    lr, eps, steps = 3e-4, 1e-8, 6
    p0 = torch.randn(n, generator=torch.Generator().manual_seed(1)) * 0.05
    ours = p0.to(DEV)
    opt = Adam(ours, lr, betas=betas, eps=eps, weight_decay=wd)
    ref = p0.clone().to(DEV).requires_grad_(True)
    cls = torch.optim.AdamW if wd > 0 else torch.optim.Adam
    topt = cls([ref], lr=lr, betas=betas, eps=eps, weight_decay=wd)   # foreach: torch's default on the GPU
    for g in _grads(n, steps, 2):
        gd = g.to(DEV)
        opt.step(gd)
        ref.grad = gd.clone()
        topt.step()
        st = topt.state[ref]
        assert torch.equal(opt.exp_avg, st["exp_avg"])
        assert torch.equal(opt.exp_avg_sq, st["exp_avg_sq"])
        assert torch.equal(ours, ref.detach())


def test_adam_step_within_an_ulp_of_torch_single_tensor_and_cpu(hip):
    n, lr, wd, eps = 1 << 18, 1e-4, 0.01, 1e-8
    p = (torch.randn(n, generator=torch.Generator().manual_seed(3)) * 0.05).to(DEV)
    opt = Adam(p, lr, eps=eps, weight_decay=wd)
    worst = {}
    for k, g in enumerate(_grads(n, 4, 5)):
        # from the same state (parameters, moments, step k), one step each
        for dev in (DEV, torch.device("cpu")):
            r = p.detach().clone().to(dev).requires_grad_(True)
            o = torch.optim.AdamW([r], lr=lr, eps=eps, weight_decay=wd, foreach=False)
            if k:
                o.state[r] = {"step": torch.tensor(float(k)), "exp_avg": opt.exp_avg.clone().to(dev),
                              "exp_avg_sq": opt.exp_avg_sq.clone().to(dev)}
            r.grad = g.to(dev)
            o.step()
            q = p.clone()
            qo = Adam(q, lr, eps=eps, weight_decay=wd)
            qo.exp_avg.copy_(opt.exp_avg)
            qo.exp_avg_sq.copy_(opt.exp_avg_sq)
            qo.steps = k
            qo.step(g.to(DEV))
            for name, a_, b_ in (("exp_avg", qo.exp_avg, o.state[r]["exp_avg"]),
                                 ("exp_avg_sq", qo.exp_avg_sq, o.state[r]["exp_avg_sq"])):
                key = (dev.type, name)
                worst[key] = max(worst.get(key, 0), _ulp(a_, b_))
            want, before = r.detach().cpu(), p.cpu()
            rel = float(((q.cpu() - want).abs() / (want.abs() + (want - before).abs())).max())
            worst[(dev.type, "param_rel")] = max(worst.get((dev.type, "param_rel"), 0.0), rel)
        opt.step(g.to(DEV))
    print("single-tensor GPU / CPU AdamW, worst moment difference in ulp, parameter relative:", worst)
    # moments: exact on the GPU; on the CPU within 2 ulp (the gradient products
    # of the 1e-20-scaled elements are subnormal, where an ulp is absolute)
    assert all(v <= 2 for k, v in worst.items() if k[1] != "param_rel"), worst
    assert all(v <= 2.0 ** -22 for k, v in worst.items() if k[1] == "param_rel"), worst
    assert worst[("cuda", "exp_avg")] == 0 and worst[("cuda", "exp_avg_sq")] == 0


@pytest.mark.parametrize("rate", [0.9999, 0.99, 0.5])
def test_ema_update_matches_update_ema(hip, rate):
    n = 1 << 20
    gen = torch.Generator().manual_seed(6)
    t0 = torch.randn(n, generator=gen) * 0.05
    src = torch.randn(n, generator=gen) * 0.05
    lib = _lib.load()
    for dev in (DEV, torch.device("cpu")):
        targ = t0.to(DEV)
        _lib.check(lib.cfd_ema_update(_lib.ptr(targ), _lib.ptr(src.to(DEV)), n, C.c_double(rate),
                                      _lib.stream_of(DEV)), "cfd_ema_update")
        want = t0.clone().to(dev)
        want.mul_(rate).add_(src.to(dev), alpha=1 - rate)   # update_ema, nn.py:71-80
        assert torch.equal(targ.cpu(), want.cpu()), dev


def test_adamw_state_dict_round_trip_through_torch(hip):
    """opt*.pt written by Adam.torch_state_dict loads into torch.optim.AdamW
    (decoupled_weight_decay kept); the next step of both is the same bits."""
    shapes = [(64, 33), (17,), (8, 4, 3, 3)]
    spans, o = [], 0
    for s in shapes:
        spans.append((o, s))
        o += int(np.prod(s))
    flat = (torch.randn(o, generator=torch.Generator().manual_seed(8)) * 0.05).to(DEV)
    opt = Adam(flat, 2e-4, weight_decay=0.01)
    grads = _grads(o, 3, 9)
    for g in grads[:2]:
        opt.step(g.to(DEV))
    sd = opt.torch_state_dict(spans)
    assert sd["param_groups"][0]["decoupled_weight_decay"] is True
    params = [flat[a:a + int(np.prod(s))].clone().reshape(s).requires_grad_(True) for a, s in spans]
    topt = torch.optim.AdamW(params, lr=1.0)
    topt.load_state_dict(sd)
    assert topt.param_groups[0]["decoupled_weight_decay"] and topt.param_groups[0]["weight_decay"] == 0.01
    for (a, s), p in zip(spans, params):
        p.grad = grads[2].to(DEV)[a:a + int(np.prod(s))].reshape(s).clone()
    topt.step()
    opt.step(grads[2].to(DEV))
    for (a, s), p in zip(spans, params):
        assert torch.equal(flat[a:a + int(np.prod(s))].reshape(s), p.detach())
    # and back: torch's state resumes here
    opt2 = Adam(flat.clone(), 2e-4, weight_decay=0.01)
    opt2.load_torch_state_dict(topt.state_dict(), spans)
    assert opt2.steps == 3 and torch.equal(opt2.exp_avg, opt.exp_avg) and torch.equal(opt2.exp_avg_sq, opt.exp_avg_sq)
    bad = topt.state_dict()
    bad["state"][0]["exp_avg"] = bad["state"][0]["exp_avg"].reshape(-1)[:10]
    with pytest.raises(ValueError):
        opt2.load_torch_state_dict(bad, spans)
