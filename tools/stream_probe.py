"""Development probe: one U-Net forward at B = 8 on one stream against the same
8 samples as K concurrent forwards of B = 8/K on K streams (batch-invariant: the
outputs must be bit-identical).  Prints ms per forward for each K."""
import ctypes as C
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from confild_amd import _lib, synth  # noqa: E402
from confild_amd.script_util import create_model  # noqa: E402

dev = torch.device("cuda", 0)
m = create_model(image_size=64, num_channels=128, num_res_blocks=2, num_heads=4, num_head_channels=64,
                 attention_resolutions="32,16,8")
m.load_state_dict({k: torch.from_numpy(v) for k, v in
                   synth.unet_state_dict(1234, {k: tuple(v.shape) for k, v in m.state_dict().items()}).items()})
m.to(dev)
lib = _lib.load()
h = m._handle(dev)
B = 8
x = torch.randn(B, 1, 64, 64, device=dev)
t = torch.full((B,), 500, dtype=torch.int64, device=dev)


def ws_for(b):
    n = C.c_size_t()
    _lib.check(lib.cfd_unet_workspace_bytes(h, b, C.byref(n)), "ws")
    return torch.empty(n.value, dtype=torch.uint8, device=dev)


ref = m(x, t)
torch.cuda.synchronize()
for K in (1, 2, 4):
    b = B // K
    streams = [torch.cuda.Stream(device=dev) for _ in range(K)]
    wss = [ws_for(b) for _ in range(K)]
    eps = torch.empty_like(ref)
    xs = [x[i * b:(i + 1) * b].contiguous() for i in range(K)]
    ts = [t[i * b:(i + 1) * b].contiguous() for i in range(K)]
    outs = [torch.empty(b, 1, 64, 64, device=dev) for _ in range(K)]

    def run():
        ev = torch.cuda.current_stream().record_event()
        done = []
        for i in range(K):
            s = streams[i]
            s.wait_event(ev)
            _lib.check(lib.cfd_unet_forward(h, _lib.ptr(xs[i]), _lib.ptr(ts[i]), _lib.ptr(outs[i]), b,
                                            _lib.ptr(wss[i]), wss[i].numel(), C.c_void_p(s.cuda_stream)), "fwd")
            done.append(s.record_event())
        for e in done:
            torch.cuda.current_stream().wait_event(e)

    for _ in range(3):
        run()
    torch.cuda.synchronize()
    a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 30
    a.record()
    for _ in range(n):
        run()
    z.record()
    z.synchronize()
    same = all(torch.equal(outs[i], ref[i * b:(i + 1) * b]) for i in range(K))
    print(f"K={K} streams x B={b}: {a.elapsed_time(z) / n:.3f} ms per 8-sample forward, bit-identical {same}",
          flush=True)
