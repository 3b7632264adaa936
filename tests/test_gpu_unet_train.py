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
import os

import numpy as np
import pytest
import torch

from conftest import golden
from confild_amd import synth
from confild_amd.script_util import create_model
from oracle import unet as ou

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
HERE = os.path.dirname(os.path.abspath(__file__))


# 128 / 256 / 384 / 512 channels: every convolution of the weight-gradient walk on
# the 128-tile kernel (the golden topologies' 16-64 channels run the 64-tile one)
WIDE = {"image_size": 16, "num_channels": 128, "num_res_blocks": 1, "channel_mult": "1,2", "num_heads": 4,
        "num_head_channels": 64, "attention_resolutions": "8"}


def _unet(name):
    if name == "wide128":
        g = {"kwargs": repr(WIDE), "seed": 31, "x": synth.normal(32, "wide/x", (2, 1, 16, 16)),
             "t": np.array([17, 903], dtype=np.int64)}
    else:
        g = golden(f"unet_{name}.npz")
    kw = ast.literal_eval(str(g["kwargs"]))
    cfg = ou.Config(**kw)
    sd_np = synth.unet_state_dict(int(g["seed"]), ou.param_shapes(cfg))
    m = create_model(**kw)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd_np.items()})
    return g, cfg, {k: torch.from_numpy(v) for k, v in sd_np.items()}, m.to(DEV)


@pytest.mark.parametrize("name", ["tiny16", "small32", "heads16", "wide128"])
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


@pytest.mark.parametrize("tail", ["normal", "outliers"])
@pytest.mark.parametrize("kept", [False, True])
def test_unet_param_grad_split_is_fp32_level(hip, tail, kept):
    """Split-f16 weight-gradient products (split compute, the default; every
    convolution of wide128 runs them): each gradient tensor's error against a
    float64 autograd evaluation stays within 2x the fp32 mode's (exact fp32-MFMA
    products) + 1e-7 of the model's largest gradient -- the criterion the split
    forward and input-gradient meet (test_gpu_unet_split.py, test_gpu_dps.py).
    ``kept``: the CFD_TAPE_PARAM_GRAD tape (GroupNorm outputs and their ranges
    kept by the forward) or the input-VJP tape (the operands recomputed).
    ``outliers``: a heavy-tailed d_eps (eight pixels 1e4x the rest), so every
    backward tensor's bulk sits far below its maximum -- the operand scaling must
    keep the bulk's hi / lo halves in the f16 normal range."""
    g, cfg, sd, m = _unet("wide128")
    x = torch.from_numpy(g["x"])
    t = torch.from_numpy(g["t"])
    d_eps = torch.from_numpy(synth.normal(5, "wide128/deps", tuple(x.shape)))
    if tail == "outliers":
        flat_idx = torch.from_numpy(synth.normal(6, "wide128/outl", (8,))).abs().mul(997).long() % d_eps.numel()
        d_eps.view(-1)[flat_idx] *= 1e4
    params = {k: v.double().requires_grad_(True) for k, v in sd.items()}
    eps_ref = ou.forward(params, cfg, x.double(), t)
    ref = dict(zip(params.keys(), torch.autograd.grad(eps_ref, list(params.values()), d_eps.double())))
    gmax = max(float(r.abs().max()) for r in ref.values())
    named = dict(m.named_parameters())
    err = {}
    for mode in ("fp32", "split_f16"):
        m.set_compute(mode)
        m.forward_tape(x.to(DEV), t.to(DEV), for_param_grad=kept)
        flat = m.param_grad(d_eps.to(DEV)).cpu().double()
        o, e = 0, {}
        for k in m.param_keys():
            n = named[k].numel()
            e[k] = float((flat[o:o + n].reshape(named[k].shape) - ref[k]).abs().max())
            o += n
        err[mode] = e
    worst = sorted(((err["split_f16"][k] - 2 * err["fp32"][k]) / gmax, k) for k in err["fp32"])[-4:]
    print(f"wide128 split vs fp32 gradient error (excess over 2x fp32, / max grad {gmax:.3e}): {worst}")
    for k in err["fp32"]:
        assert err["split_f16"][k] <= 2 * err["fp32"][k] + 1e-7 * gmax, (k, err["split_f16"][k], err["fp32"][k])


def test_unet_param_grad_split_large_groupnorm(hip):
    """The GroupNorms of a 128^2 x 256-channel level run the three-kernel path
    (gn_partial / gn_finalize / gn_apply) and gn_apply's bounded grid-stride loop
    covers > 4096 x 256 float4 quads per workgroup grid (B = 4: 4.2 M), so each
    thread handles several quads.  The range slot each kept output carries (the
    split weight gradients' operand scale) must be the max over all of them: split
    and fp32 parameter gradients agree to fp32 level, with the kept-output tape
    and with the recomputed operands alike (an underestimated range overflows the
    f16 halves)."""
    kw = {"image_size": 128, "num_channels": 128, "num_res_blocks": 1, "channel_mult": "2,2", "num_heads": 4,
          "num_head_channels": 64, "attention_resolutions": "16"}
    m = create_model(**kw)
    sd = synth.unet_state_dict(41, {k: tuple(v.shape) for k, v in m.state_dict().items()})
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m.to(DEV)
    x = torch.from_numpy(synth.normal(42, "gnbig/x", (4, 1, 128, 128))).to(DEV)
    t = torch.tensor([3, 250, 600, 990], dtype=torch.int64, device=DEV)
    d = torch.from_numpy(synth.normal(43, "gnbig/d", (4, 1, 128, 128))).to(DEV)
    grads = {}
    for mode, kept in (("fp32", True), ("split_f16", True), ("split_f16", False)):
        m.set_compute(mode)
        m.forward_tape(x, t, for_param_grad=kept)
        grads[(mode, kept)] = m.param_grad(d).cpu()
    named = dict(m.named_parameters())
    ref = grads[("fp32", True)]
    gmax = float(ref.abs().max())
    for key in (("split_f16", True), ("split_f16", False)):
        got, o, worst = grads[key], 0, (0.0, "")
        assert torch.isfinite(got).all(), key
        for k in m.param_keys():
            n = named[k].numel()
            r, gk = ref[o:o + n], got[o:o + n]
            o += n
            e = float((gk - r).abs().max()) / max(float(r.abs().max()), 1e-3 * gmax)
            worst = max(worst, (e, k))
        print(f"128^2 x 256ch B=4, split vs fp32 parameter gradients, {key}: worst {worst}")
        assert worst[0] < 2e-4, (key, worst)


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


class _FixedSampler:
    """A schedule sampler replaying given timesteps (uniform weights 1)."""

    def __init__(self, ts):
        self.ts = [list(t) for t in ts]

    def sample(self, batch_size, device):
        t, self.ts[0] = self.ts[0][:batch_size], self.ts[0][batch_size:]
        if not self.ts[0]:
            self.ts.pop(0)
        return torch.tensor(t, dtype=torch.int64, device=device), torch.ones(batch_size, device=device)


def _trainloop(c, m, ts, microbatch=-1, **kw):
    from confild_amd.script_util import create_gaussian_diffusion
    from confild_amd.train_util import TrainLoop
    diff = create_gaussian_diffusion(steps=1000, noise_schedule=c["schedule"], timestep_respacing="")
    return TrainLoop(model=m, diffusion=diff, train_data=None, batch_size=c["B"], microbatch=microbatch,
                     lr=c["lr"], ema_rate=c["ema_rate"], log_interval=1, save_interval=1000,
                     resume_checkpoint=kw.pop("resume_checkpoint", ""), weight_decay=c["weight_decay"],
                     schedule_sampler=_FixedSampler(ts), **kw)


def _unpack(loop, flat):
    named = dict(loop.model.named_parameters())
    out, o = {}, 0
    for k in loop.keys:
        n = named[k].numel()
        out[k] = flat[o:o + n].reshape(named[k].shape).cpu().numpy()
        o += n
    return out


def test_trainloop_matches_reference_run(hip, tmp_path):
    """confild_amd.train_util.TrainLoop (q_sample, eps MSE, U-Net param grads,
    AdamW, EMA all in the library) against the reference TrainLoop's own run
    (golden_unettrain.npz, make_golden_unet_train.py): per-step losses, the first
    step's gradients, parameters and EMA after 2 steps (tolerances in
    tests/unettrain_check.py); then save -> resume restores the state."""
    from unettrain_check import check
    g = golden("golden_unettrain.npz")
    c = ast.literal_eval(str(g["case"]))
    _, cfg, sd, m = _unet(c["net"])
    loop = _trainloop(c, m, c["t"], log_dir=str(tmp_path))
    x0 = torch.from_numpy(g["x0"]).to(DEV)
    losses, first, grads = [], None, []
    p_start = loop.params.clone()
    for k in range(c["steps"]):
        loop.run_step(x0, None, None, noise=torch.from_numpy(g["noise"][k]).to(DEV))
        grads.append(loop.grad.clone())
        if first is None:
            first = _unpack(loop, loop.grad)
        losses.append(loop.logger.dumpkvs()["loss"])
    # the optimiser and EMA on our own gradients are the reference's bit for bit:
    # torch.optim.AdamW (its GPU default, foreach) over the per-parameter tensors and
    # update_ema (nn.py:71-80) replayed from the same start -- so what the parameter
    # bound below still allows is the propagation of the gradients' rounding alone
    named = dict(m.named_parameters())
    views, o = [], 0
    rp = p_start.clone()
    for k in loop.keys:
        n = named[k].numel()
        views.append(rp[o:o + n].view(named[k].shape))
        o += n
    tparams = [v.clone().requires_grad_(True) for v in views]
    topt = torch.optim.AdamW(tparams, lr=c["lr"], weight_decay=c["weight_decay"])
    tema = [t.detach().clone() for t in tparams]
    for gk in grads:
        o = 0
        for t in tparams:
            t.grad = gk[o:o + t.numel()].view(t.shape).clone()
            o += t.numel()
        topt.step()
        for targ, src in zip(tema, tparams):
            targ.mul_(c["ema_rate"]).add_(src.detach(), alpha=1 - c["ema_rate"])
    assert torch.equal(torch.cat([t.detach().reshape(-1) for t in tparams]), loop.params)
    assert torch.equal(torch.cat([t.reshape(-1) for t in tema]), loop.ema_params[0])
    names = [str(n) for n in g["names"]]
    rep = check(g, c, names, losses, first, _unpack(loop, loop.params), _unpack(loop, loop.ema_params[0]),
                rtol_loss0=2e-5, rtol_loss1=1e-4, tol_grad=2e-4, atol_grad=5e-6, tol_param=1e-4,
                frac_loose=1e-2)
    print(rep)
    # the module holds the stepped parameters
    named = dict(m.named_parameters())
    fin = _unpack(loop, loop.params)
    assert all(np.array_equal(named[k].detach().cpu().numpy(), fin[k]) for k in loop.keys)
    # checkpoints in the reference's names and layouts; resume restores params / EMA / Adam state
    loop.step = c["steps"]
    loop.save()
    st = c["steps"]
    for f in (f"model{st:06d}.pt", f"ema_{c['ema_rate']}_{st:06d}.pt", f"opt{st:06d}.pt"):
        assert (tmp_path / f).exists(), f
    osd = torch.load(tmp_path / f"opt{st:06d}.pt", weights_only=True)
    assert len(osd["state"]) == len(list(m.parameters())) and float(osd["state"][0]["step"]) == c["steps"]
    _, _, _, m2 = _unet(c["net"])
    loop2 = _trainloop(c, m2, [], resume_checkpoint=str(tmp_path / f"model{st:06d}.pt"))
    assert loop2.resume_step == st
    assert torch.equal(loop2.params, loop.params)
    assert torch.equal(loop2.ema_params[0], loop.ema_params[0])
    assert torch.equal(loop2.opt.exp_avg, loop.opt.exp_avg) and loop2.opt.steps == loop.opt.steps


def test_trainloop_microbatches_sum_their_means(hip):
    """forward_backward's microbatch loop (train_util.py:192-226): each
    microbatch's (loss * weights).mean() is backpropagated and the gradients add,
    so microbatch 1 over B = 2 gives the sum of the two one-sample gradients =
    twice the full batch's mean gradient (within the parameter-gradient
    tolerance, 2e-4 of the largest: B = 1 and B = 2 pick different split-K
    kernels, measured 5.6e-5)."""
    g = golden("golden_unettrain.npz")
    c = ast.literal_eval(str(g["case"]))
    x0 = torch.from_numpy(g["x0"]).to(DEV)
    nz = torch.from_numpy(g["noise"][0]).to(DEV)
    grads = []
    for mb in (-1, 1):
        _, _, _, m = _unet(c["net"])
        loop = _trainloop(c, m, [c["t"][0]], microbatch=mb)
        loop.forward_backward(x0, noise=nz)
        grads.append(loop.grad.clone())
    full, micro = grads
    scale = float(full.abs().max())
    assert float((micro - 2 * full).abs().max()) <= 2e-4 * scale


@pytest.mark.parametrize("name", ["tiny16", "small32", "wide128"])
def test_load_flat_device_repack_is_bitexact(hip, name):
    """cfd_unet_load_flat (the TrainLoop's parameter update, packed on the GPU)
    against the host packing of cfd_unet_set_param: after loading perturbed
    parameters both ways, eps (split-f16 and bf16 compute), the input VJP and the
    parameter gradients are bit-identical."""
    g, cfg, sd, m = _unet(name)
    x = torch.from_numpy(g["x"]).to(DEV)
    t = torch.from_numpy(g["t"]).to(DEV)
    m(x, t)                                     # the handle exists and holds the initial pack
    flat = m.flat_params()
    flat = (flat * (1 + 0.01 * torch.randn_like(flat)) + 1e-3 * torch.randn_like(flat)).contiguous()
    m.load_flat(flat)                           # device repack
    _, _, _, ref = _unet(name)
    ref.load_flat(flat.clone())                 # no handle yet: the host pack on first use
    d = torch.from_numpy(synth.normal(9, "lf/d", tuple(x.shape))).to(DEV)
    for mode in ("bf16", "split_f16"):
        m.set_compute(mode)
        ref.set_compute(mode)
        assert torch.equal(m(x, t), ref(x, t)), mode
    assert torch.equal(m.forward_tape(x, t), ref.forward_tape(x, t))
    assert torch.equal(m.input_vjp(d), ref.input_vjp(d))
    m.forward_tape(x, t)
    ref.forward_tape(x, t)
    assert torch.equal(m.param_grad(d), ref.param_grad(d))


def test_trainloop_ddp_two_ranks(hip, tmp_path):
    """Two TrainLoop ranks (one sample each, gloo over device tensors on the same
    GPU): the flat gradient is averaged across the ranks (DistributedDataParallel),
    so both ranks hold the same gradient, parameters and EMA bit for bit, and that
    gradient is the single-process gradient of the two-sample batch (within the
    parameter-gradient tolerance: B = 1 and B = 2 choose different split-K plans)."""
    import socket
    import subprocess
    import sys
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = str(tmp_path / "ddp")
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(HERE, "ddp_trainloop_worker.py"),
           out]
    res = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert res.returncode == 0, res.stderr[-3000:]
    r0 = torch.load(out + ".rank0.pt", weights_only=True)
    r1 = torch.load(out + ".rank1.pt", weights_only=True)
    for k in ("grad", "params", "ema"):
        assert torch.equal(r0[k], r1[k]), k
    g = golden("golden_unettrain.npz")
    c = ast.literal_eval(str(g["case"]))
    _, _, _, m = _unet(c["net"])
    loop = _trainloop(c, m, [c["t"][0]])
    loop.forward_backward(torch.from_numpy(g["x0"]).to(DEV), noise=torch.from_numpy(g["noise"][0]).to(DEV))
    full = loop.grad.cpu()
    assert float((r0["grad"] - full).abs().max()) <= 2e-4 * float(full.abs().max())


def test_tape_layout_is_per_tape_through_the_c_abi(hip):
    """Two live tapes of different modes on one handle (C ABI directly): tape A
    recorded for param_grad (CFD_TAPE_PARAM_GRAD), then tape B for the input-VJP
    (the smaller layout).  param_grad on A afterwards replays A's own layout -- the
    same gradients, bit for bit, as right after A was recorded -- and input_vjp on
    B equals the Python API's.  A pointer the handle never recorded, and a replay
    at another batch, are refused (no silent wrong layout)."""
    import ctypes as C
    from confild_amd import _lib
    g, cfg, sd, m = _unet("wide128")
    x = torch.from_numpy(g["x"]).to(DEV)
    t = torch.from_numpy(g["t"]).to(DEV)
    d = torch.from_numpy(synth.normal(5, "tapes/d", tuple(x.shape))).to(DEV)
    B = x.shape[0]
    lib = _lib.load()
    h = m._handle(DEV)
    ws = m._workspace(h, DEV, B)
    st = _lib.stream_of(DEV)
    P = _lib.ptr

    def nbytes(fn):
        n = C.c_size_t()
        _lib.check(fn(h, B, C.byref(n)), "bytes")
        return n.value

    def record(mode, xx):
        _lib.check(lib.cfd_unet_set_tape_mode(h, mode), "mode")
        tape = torch.empty(nbytes(lib.cfd_unet_tape_bytes), dtype=torch.uint8, device=DEV)
        eps = torch.empty_like(xx)
        _lib.check(lib.cfd_unet_forward_tape(h, P(xx), P(t), P(eps), B, P(ws), ws.numel(), P(tape), tape.numel(), st),
                   "forward_tape")
        return tape

    pws = torch.empty(nbytes(lib.cfd_unet_param_grad_workspace_bytes), dtype=torch.uint8, device=DEV)
    vws = torch.empty(nbytes(lib.cfd_unet_vjp_workspace_bytes), dtype=torch.uint8, device=DEV)
    n_total = sum(p.numel() for p in m.parameters())

    def pgrad(tape):
        gr = torch.zeros(n_total, device=DEV)
        _lib.check(lib.cfd_unet_param_grad(h, P(x), P(d), B, P(tape), tape.numel(), P(gr), P(pws), pws.numel(), st),
                   "param_grad")
        return gr

    tape_a = record(1, x)
    g_a = pgrad(tape_a)
    x2 = (x * 0.5 + 0.1).contiguous()
    tape_b = record(0, x2)
    assert tape_b.numel() < tape_a.numel()
    assert torch.equal(pgrad(tape_a), g_a)
    dx = torch.empty_like(x)
    _lib.check(lib.cfd_unet_input_vjp(h, P(d), P(dx), B, P(tape_b), tape_b.numel(), P(vws), vws.numel(), st), "vjp")
    m.forward_tape(x2, t)
    assert torch.equal(m.input_vjp(d), dx)
    stray = torch.empty_like(tape_a)
    with pytest.raises(_lib.CfdError, match="not recorded"):
        _lib.check(lib.cfd_unet_input_vjp(h, P(d), P(dx), B, P(stray), stray.numel(), P(vws), vws.numel(), st), "vjp")
    with pytest.raises(_lib.CfdError, match="batch"):
        _lib.check(lib.cfd_unet_input_vjp(h, P(d), P(dx), 1, P(tape_b), tape_b.numel(), P(vws), vws.numel(), st),
                   "vjp")


def test_param_grad_after_plan_batch_change(hip):
    """param_grad, then set_plan_batch(2), then forward_tape + param_grad: the
    param-grad workspace (it holds the split-K slab, sized per planned batch) is
    re-sized, and the gradients stay within fp32 rounding of the default plan's."""
    g, cfg, sd, m = _unet("wide128")
    x = torch.from_numpy(g["x"]).to(DEV)
    t = torch.from_numpy(g["t"]).to(DEV)
    d = torch.from_numpy(synth.normal(5, "pgplan/d", tuple(x.shape))).to(DEV)
    m.forward_tape(x, t)
    ref = m.param_grad(d)
    for pb in (2, 1):
        m.set_plan_batch(pb)
        with pytest.raises(RuntimeError):
            m.param_grad(d)          # the tape of the old plan is not replayed
        m.forward_tape(x, t)
        got = m.param_grad(d)
        err = float((got - ref).abs().max()) / float(ref.abs().max())
        assert torch.isfinite(got).all() and err < 1e-4, (pb, err)
