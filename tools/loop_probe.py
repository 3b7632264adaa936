"""Timing probe of the reverse loop per step: Python loop vs native loop vs
captured HIP graphs (CFD_SAMPLER modes 0/1/2, unroll), at the config-A (32^2,
mult 1,2,3,4, DDIM-50, B = 1) and config-B (64^2, B = 1 / 8) shapes.

  python tools/loop_probe.py            # prints one JSON line per (config, B, mode)
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from confild_amd import gaussian_diffusion as gd  # noqa: E402
from confild_amd import synth  # noqa: E402
from confild_amd.script_util import create_gaussian_diffusion, create_model  # noqa: E402

DEV = torch.device("cuda", 0)


def model(size, mult, compute="split_f16"):
    m = create_model(image_size=size, num_channels=128, num_res_blocks=2, num_heads=4, num_head_channels=64,
                     attention_resolutions="32,16,8", channel_mult=mult)
    sd = synth.unet_state_dict(1234, {k: tuple(v.shape) for k, v in m.state_dict().items()})
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m = m.to(DEV).set_compute(compute)
    return m.set_plan_batch(int(os.environ.get("LOOP_PLAN", "0")))   # LOOP_PLAN: the planned batch


def forward_ms(m, B, size, iters=20):
    x = torch.randn(B, 1, size, size, device=DEV)
    t = torch.full((B,), 500, dtype=torch.int64, device=DEV)
    m(x, t)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        m(x, t)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


def main():
    cases = [("A", 32, "1,2,3,4", "ddim50", True, 1, "split_f16"), ("B1", 64, "", "256", False, 1, "split_f16"),
             ("B8", 64, "", "256", False, 8, "split_f16"), ("E100", 128, "", "100", False, 8, "bf16"),
             ("E1000", 128, "", "", False, 8, "bf16")]
    only = sys.argv[1:]
    modes = ((0, 1), (1, 1), (2, 1), (2, 4), (2, 16))
    if os.environ.get("LOOP_MODES"):
        modes = tuple(tuple(int(v) for v in x.split(":")) for x in os.environ["LOOP_MODES"].split(","))
    for name, size, mult, resp, ddim, B, compute in cases:
        if only and name not in only:
            continue
        m = model(size, mult, compute)
        print(json.dumps({"case": name, "forward_ms": forward_ms(m, B, size)}), flush=True)
        d = create_gaussian_diffusion(steps=1000, noise_schedule="cosine", timestep_respacing=resp)
        loop = d.ddim_sample_loop if ddim else d.p_sample_loop
        for mode, unroll in modes:
            gd.NATIVE_MODE, gd.GRAPH_UNROLL = mode, unroll
            loop(m, (B, 1, size, size), seed=1)   # warm (capture)
            torch.cuda.synchronize()
            reps = 1 if d.num_timesteps >= 1000 else 3
            t0 = time.perf_counter()
            for r in range(reps):
                out = loop(m, (B, 1, size, size), seed=2 + r)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / reps
            print(json.dumps({"case": name, "B": B, "mode": mode, "unroll": unroll, "steps": d.num_timesteps,
                              "loop_s": dt, "ms_per_step": dt / d.num_timesteps * 1e3,
                              "finite": bool(torch.isfinite(out).all())}), flush=True)


if __name__ == "__main__":
    main()
