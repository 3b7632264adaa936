"""Where a fresh process's first reverse loop spends its extra time (development
tool): config E's U-Net (128^2, B = 8, bf16) and config B's (64^2, B = 8,
split-f16), each timed as first forward, second forward, first 8-step native
loop (graph capture + first replays), second 8-step loop, then a 200-step loop,
all wall-clock with a device sync around each.

    python tools/dev/first_call.py E
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from confild_amd import synth  # noqa: E402
from confild_amd.script_util import create_gaussian_diffusion, create_model  # noqa: E402

DEV = torch.device("cuda", 0)


def timed(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t0) * 1e3, 2)


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "E"
    size, compute = (128, "bf16") if which == "E" else (64, "split_f16")
    out = {"case": which}
    t0 = time.perf_counter()
    m = create_model(image_size=size, num_channels=128, num_res_blocks=2, num_heads=4, num_head_channels=64,
                     attention_resolutions="32,16,8", channel_mult="")
    sd = synth.unet_state_dict(1234, {k: tuple(v.shape) for k, v in m.state_dict().items()})
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m.to(DEV).set_compute(compute)
    out["build_ms"] = round((time.perf_counter() - t0) * 1e3, 1)
    x = torch.randn(8, 1, size, size, device=DEV)
    t = torch.full((8,), 500, dtype=torch.int64, device=DEV)
    out["fwd1_ms"] = timed(lambda: m(x, t))
    out["fwd2_ms"] = timed(lambda: m(x, t))
    for name, resp in (("loop8", "8"), ("loop200", "200")):
        d = create_gaussian_diffusion(steps=1000, noise_schedule="cosine", timestep_respacing=resp)
        out[name + "_first_ms"] = timed(lambda: d.p_sample_loop(m, (8, 1, size, size), seed=1))
        out[name + "_second_ms"] = timed(lambda: d.p_sample_loop(m, (8, 1, size, size), seed=2))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
