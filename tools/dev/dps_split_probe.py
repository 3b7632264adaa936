"""Development probe: config D's 8 chains as one DPS step on the whole chip vs two
groups of 4 chains stepping side by side on CU halves (separate model handles)."""
import functools
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from confild_amd import synth  # noqa: E402
from confild_amd.guided.condition_methods import get_conditioning_method  # noqa: E402
from confild_amd.guided.gaussian_diffusion import create_sampler  # noqa: E402
from confild_amd.guided.measurements import Case4Operator, get_noise  # noqa: E402
from confild_amd.nf_networks import SIRENAutodecoder_film  # noqa: E402
from confild_amd.normalize import Normalizer_ts  # noqa: E402
from confild_amd.script_util import create_model  # noqa: E402
from confild_amd.streams import CuRangeStream, cu_count  # noqa: E402

DEV = torch.device("cuda", 0)
size, ns = 64, 10
d, L, c, nh, H = 3, 64, 3, 15, 384
coords = torch.rand(ns, d)


def setup():
    m = create_model(image_size=size, num_channels=128, num_res_blocks=2, num_heads=4, num_head_channels=64,
                     attention_resolutions="32,16,8")
    m.load_state_dict({k: torch.from_numpy(v) for k, v in
                       synth.unet_state_dict(1234, {k: tuple(v.shape) for k, v in m.state_dict().items()}).items()})
    m.to(DEV)
    nf = SIRENAutodecoder_film(d, L, c, nh, H)
    nf.load_state_dict({k: torch.from_numpy(v) for k, v in synth.siren_state_dict(1234, d, L, c, nh, H).items()})
    xn = Normalizer_ts(params=(torch.ones(1, d), torch.zeros(1, d)), method="-11", dim=0)
    yn = Normalizer_ts(params=(torch.ones(c), -torch.ones(c)), method="-11", dim=0)
    op = Case4Operator.from_parts(DEV, coords, xn, yn, nf, torch.full((L,), 1.5), torch.full((L,), -1.5))
    cond = get_conditioning_method(operator=op, noiser=get_noise(sigma=0.0, name="gaussian"), name="ps", scale=1.0)
    smp = create_sampler(sampler="ddpm", steps=1000, noise_schedule="cosine", model_mean_type="epsilon",
                         model_var_type="fixed_large", dynamic_threshold=False, clip_denoised=True,
                         rescale_timesteps=False, timestep_respacing="256")
    return m, smp, functools.partial(cond.conditioning)


a, b = setup(), setup()
y = torch.randn(size, ns, c, device=DEV)
x8 = torch.randn(8, 1, size, size, device=DEV)
x4a, x4b = x8[:4].clone(), x8[4:].clone()
n = cu_count(DEV)
sa, sb = CuRangeStream(DEV, 0, n // 2), CuRangeStream(DEV, n // 2, n - n // 2)


def step(s, x, k):
    m, smp, fn = s
    return smp.p_sample_step(m, x, 128 - k % 100, y, fn, seed=1, counter=k)["sample"]


def timed(fn, it=6):
    for _ in range(2):
        fn(0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(it):
        fn(k)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / it


print("8 chains, whole chip: %.2f ms per step" % timed(lambda k: step(a, x8, k)), flush=True)
print("4 chains, whole chip: %.2f ms per step" % timed(lambda k: step(a, x4a, k)), flush=True)


def halves(k):
    sa.stream.wait_stream(torch.cuda.current_stream())
    sb.stream.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(sa.stream):
        step(a, x4a, k)
    with torch.cuda.stream(sb.stream):
        step(b, x4b, k)


print("2 x 4 chains on CU halves: %.2f ms per step (8 chains)" % timed(halves), flush=True)
