"""Kernel-level timing of the HIP path with HIP events (development tool).

    python tools/kbench.py siren [--latents 64]      # config-B CNF decode
    python tools/kbench.py unet  [--batch 8]         # one U-Net forward
    python tools/kbench.py sweep                      # both, short
    python tools/kbench.py dps   [--batch 8]         # one DPS step (config D) and its parts
    python tools/kbench.py train                      # one CNF training step (Case4 recipe widths)
    python tools/kbench.py utrain --batch 16 --size 128   # one diffusion TrainLoop step (Case1 recipe)
Prints one JSON line per measurement.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from confild_amd import synth  # noqa: E402

DEV = torch.device("cuda", 0)


def timeit(fn, iters=5, warm=1):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2], ts[0]


def bench_siren(latents=64, npts=64 ** 3, dims=(3, 64, 3, 15, 384), iters=3, compute=None):
    from confild_amd.nf_networks import SIRENAutodecoder_film
    d, L, c, nh, H = dims
    net = SIRENAutodecoder_film(d, L, c, nh, H)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in synth.siren_state_dict(1234, d, L, c, nh, H).items()})
    net.to(DEV)
    if compute:
        net.set_compute(compute)
    coords = torch.rand(npts, d, device=DEV)
    lat = torch.randn(latents, 1, L, device=DEV) * 0.5
    med, best = timeit(lambda: net(coords, lat), iters=iters)
    flops = latents * npts * 2 * (d * H + nh * H * H + H * c)
    print(json.dumps({"kernel": "siren", "compute": net.compute_mode(DEV),
                      "variant": os.environ.get("CFD_SIREN_VARIANT", "0"), "dims": dims,
                      "latents": latents, "npts": npts, "ms": med, "best_ms": best,
                      "tflops": flops / (best / 1e3) / 1e12}), flush=True)


def bench_unet(batch=8, size=64, iters=10, bf16=False, compute=None, mult="", plan=0):
    from confild_amd.script_util import create_model
    m = create_model(image_size=size, num_channels=128, num_res_blocks=2, num_heads=4, num_head_channels=64,
                     attention_resolutions="32,16,8", use_bf16=bf16, channel_mult=mult)
    sd = synth.unet_state_dict(1234, {k: tuple(v.shape) for k, v in m.state_dict().items()})
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m.to(DEV)
    if compute:
        m.set_compute(compute)
    m.set_plan_batch(plan)
    x = torch.randn(batch, 1, size, size, device=DEV)
    t = torch.full((batch,), 500, dtype=torch.int64, device=DEV)
    med, best = timeit(lambda: m(x, t), iters=iters, warm=2)
    gf = {32: 19.23, 64: 68.61, 128: 140.75}.get(size, float("nan"))
    print(json.dumps({"kernel": "unet_forward", "compute": m.compute, "batch": batch, "size": size, "plan": plan, "ms": med,
                      "best_ms": best,
                      "tflops": batch * gf * 1e9 / (best / 1e3) / 1e12}), flush=True)


def bench_dps(batch=8, size=64, ns=10, dims=(3, 64, 3, 15, 384), iters=5):
    """Config D: one guided (DPS) reverse step of B chains and its components."""
    import functools
    from confild_amd.guided.condition_methods import get_conditioning_method
    from confild_amd.guided.gaussian_diffusion import create_sampler
    from confild_amd.guided.measurements import Case4Operator, get_noise
    from confild_amd.nf_networks import SIRENAutodecoder_film
    from confild_amd.normalize import Normalizer_ts
    from confild_amd.script_util import create_model
    m = create_model(image_size=size, num_channels=128, num_res_blocks=2, num_heads=4, num_head_channels=64,
                     attention_resolutions="32,16,8")
    sd = synth.unet_state_dict(1234, {k: tuple(v.shape) for k, v in m.state_dict().items()})
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m.to(DEV)
    d, L, c, nh, H = dims
    nf = SIRENAutodecoder_film(d, L, c, nh, H)
    nf.load_state_dict({k: torch.from_numpy(v) for k, v in synth.siren_state_dict(1234, d, L, c, nh, H).items()})
    coords = torch.rand(ns, d)
    xn = Normalizer_ts(params=(torch.ones(1, d), torch.zeros(1, d)), method="-11", dim=0)
    yn = Normalizer_ts(params=(torch.ones(c), -torch.ones(c)), method="-11", dim=0)
    op = Case4Operator.from_parts(DEV, coords, xn, yn, nf, torch.full((L,), 1.5), torch.full((L,), -1.5))
    cond = get_conditioning_method(operator=op, noiser=get_noise(sigma=0.0, name="gaussian"), name="ps", scale=1.0)
    smp = create_sampler(sampler="ddpm", steps=1000, noise_schedule="cosine", model_mean_type="epsilon",
                         model_var_type="fixed_large", dynamic_threshold=False, clip_denoised=True,
                         rescale_timesteps=False, timestep_respacing="256")
    fn = functools.partial(cond.conditioning)
    x = torch.randn(batch, 1, size, size, device=DEV)
    y = torch.randn(size, ns, c, device=DEV)
    t = torch.full((batch,), 500, dtype=torch.int64, device=DEV)
    res = {"kernel": "dps_step", "batch": batch, "size": size, "sensors": ns}
    res["step_ms"], _ = timeit(lambda: smp.p_sample_step(m, x, 128, y, fn, seed=1, counter=0), iters=iters, warm=2)
    res["unet_fwd_ms"], _ = timeit(lambda: m(x, t), iters=iters)
    res["unet_fwd_tape_ms"], _ = timeit(lambda: m.forward_tape(x, t), iters=iters)
    de = torch.randn_like(x)
    res["unet_vjp_ms"], _ = timeit(lambda: m.input_vjp(de), iters=iters)
    x0 = x.clamp(-1, 1)
    res["siren_tape_fwd_ms"], _ = timeit(lambda: op.forward_tape(x0), iters=iters)
    g = torch.randn(batch * size, ns, c, device=DEV)
    res["siren_vjp_ms"], _ = timeit(lambda: op.vjp(g), iters=iters)
    print(json.dumps(res), flush=True)


def bench_train(rows=4, npts=65536, dims=(3, 384, 3, 15, 384), iters=3):
    """One CNF training backward (cfd_siren_train_grad) at the Case4 recipe widths
    (N/training_recipes/case4.yml: SIREN(3, 384, 3, 15, 384), batch 4) plus the
    latent Adam step, on `npts` coordinates."""
    from confild_amd.cnf_train import Adam
    from confild_amd.nf_networks import SIRENAutodecoder_film
    d, L, c, nh, H = dims
    net = SIRENAutodecoder_film(d, L, c, nh, H)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in synth.siren_state_dict(1234, d, L, c, nh, H).items()})
    net.to(DEV)
    coords = torch.rand(npts, d, device=DEV) * 2 - 1
    Z = (torch.randn(64, L, device=DEV) * 0.5).contiguous()
    fois = torch.rand(rows, npts, c, device=DEV) * 2 - 1
    r = torch.arange(rows, device=DEV)
    grad = torch.zeros_like(net.flat_params())
    gz = torch.zeros_like(Z)
    sse = torch.zeros(1, device=DEV)
    opt = Adam(Z, 1e-5)

    def step():
        net.train_grad(coords, Z, r, fois, 2.0 / fois.numel(), grad, gz, sse)
        opt.step(gz)
    med, best = timeit(step, iters=iters)
    pairs = rows * npts
    flops = pairs * 2 * (3 * nh * H * H + 3 * (d * H + H * c))   # forward + delta chain + weight gradients
    print(json.dumps({"kernel": "cnf_train_step", "dims": dims, "rows": rows, "npts": npts, "ms": med,
                      "best_ms": best, "pairs_per_s": pairs / (best / 1e3), "tflops": flops / (best / 1e3) / 1e12}),
          flush=True)


def bench_unet_train(batch=16, size=128, mult="", iters=5):
    """One diffusion TrainLoop.run_step (U/src/train_util.py:178-226: q_sample,
    U-Net forward with tape, eps MSE, parameter gradients, AdamW, EMA) at the
    recipe widths (U/training_recipes/case1.yml: 128^2, batch 16, 128 channels,
    lr 5e-5, EMA 0.9999), and its parts."""
    from confild_amd.script_util import create_gaussian_diffusion, create_model
    from confild_amd.train_util import TrainLoop
    m = create_model(image_size=size, num_channels=128, num_res_blocks=2, num_heads=4, num_head_channels=64,
                     attention_resolutions="32,16,8", channel_mult=mult)
    sd = synth.unet_state_dict(1234, {k: tuple(v.shape) for k, v in m.state_dict().items()})
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m.to(DEV)
    diff = create_gaussian_diffusion(steps=1000, noise_schedule="cosine")
    loop = TrainLoop(model=m, diffusion=diff, train_data=None, batch_size=batch, microbatch=-1, lr=5e-5,
                     ema_rate="0.9999", log_interval=1000, save_interval=10000, resume_checkpoint="")
    x0 = torch.rand(batch, 1, size, size, device=DEV) * 2 - 1
    res = {"kernel": "unet_train_step", "batch": batch, "size": size, "mult": mult,
           "n_params": loop.params.numel()}
    res["step_ms"], best = timeit(lambda: loop.run_step(x0), iters=iters, warm=2)
    res["samples_per_s"] = batch / (best / 1e3)
    t = torch.randint(0, 1000, (batch,), device=DEV)
    x = torch.randn_like(x0)
    res["fwd_tape_ms"], _ = timeit(lambda: m.forward_tape(x, t), iters=iters)
    d = torch.randn_like(x0)
    res["param_grad_ms"], _ = timeit(lambda: m.param_grad(d, loop.grad), iters=iters)
    res["adamw_ms"], _ = timeit(lambda: loop.opt.step(loop.grad), iters=iters)
    res["ema_ms"], _ = timeit(loop._update_ema, iters=iters)
    res["load_flat_ms"], _ = timeit(lambda: m.load_flat(loop.params), iters=iters)
    gf = {64: 68.61, 128: 140.75}.get(size)
    if gf and not mult:
        res["tflops_3x_fwd"] = 3 * batch * gf * 1e9 / (best / 1e3) / 1e12
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("what", choices=["siren", "unet", "sweep", "dps", "train", "utrain"])
    ap.add_argument("--latents", type=int, default=64)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--bf16", action="store_true")
    ap.add_argument("--mult", default="", help="U-Net channel_mult (32^2 needs one: 1,2,3,4)")
    ap.add_argument("--compute", choices=["f32", "split_f16"], default=None)
    ap.add_argument("--unet-compute", choices=["fp32", "split_f16", "bf16"], default=None)
    ap.add_argument("--dims", default="3,64,3,15,384", help="SIREN d,L,c,nh,H")
    ap.add_argument("--plan", type=int, default=0, help="U-Net planned batch (0: 8)")
    a = ap.parse_args()
    if a.what in ("siren", "sweep"):
        bench_siren(a.latents, dims=tuple(int(v) for v in a.dims.split(",")), compute=a.compute)
    if a.what in ("unet", "sweep"):
        bench_unet(a.batch, a.size, bf16=a.bf16, compute=a.unet_compute, mult=a.mult, plan=a.plan)
    if a.what == "dps":
        bench_dps(a.batch, a.size)
    if a.what == "train":
        bench_train()
    if a.what == "utrain":
        bench_unet_train(a.batch, a.size, a.mult)
