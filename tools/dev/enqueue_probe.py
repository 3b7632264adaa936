"""Development probe: host enqueue time vs GPU time of the U-Net calls the DPS
step makes (config D widths, B = 8)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from confild_amd import synth  # noqa: E402
from confild_amd.script_util import create_model  # noqa: E402

DEV = torch.device("cuda", 0)
m = create_model(image_size=64, num_channels=128, num_res_blocks=2, num_heads=4, num_head_channels=64,
                 attention_resolutions="32,16,8")
m.load_state_dict({k: torch.from_numpy(v) for k, v in
                   synth.unet_state_dict(1234, {k: tuple(v.shape) for k, v in m.state_dict().items()}).items()})
m.to(DEV)
x = torch.randn(8, 1, 64, 64, device=DEV)
t = torch.full((8,), 500, dtype=torch.int64, device=DEV)
d = torch.randn_like(x)
for name, fn in (("forward", lambda: m(x, t)), ("forward_tape", lambda: m.forward_tape(x, t)),
                 ("input_vjp", lambda: m.input_vjp(d))):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    enq, tot = [], []
    for _ in range(10):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        enq.append((t1 - t0) * 1e3)
        tot.append((t2 - t0) * 1e3)
    enq.sort()
    tot.sort()
    print(f"{name}: enqueue {enq[5]:.3f} ms, enqueue+run {tot[5]:.3f} ms", flush=True)
