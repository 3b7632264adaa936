"""Development probe: config B's sampling loop and CNF decode on disjoint CU sets
(hipExtStreamCreateWithCUMask), alone and concurrently -- does overlapping the
decode of batch k with the sampling of batch k+1 pay?"""
import ctypes
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from confild_amd import _lib  # noqa: E402

DEV = torch.device("cuda", 0)
hip = ctypes.CDLL("libamdhip64.so")
NCU = torch.cuda.get_device_properties(0).multi_processor_count


def masked_stream(cus):
    words = (NCU + 31) // 32
    mask = (ctypes.c_uint32 * words)()
    for c in cus:
        mask[c // 32] |= 1 << (c % 32)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(words), mask)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(s.value, device=DEV)


o = bench.setup_B(DEV, 0, 1, "split_f16", "split_f16")
S = bench.S


def sample(seed):
    lat = o["diff"].p_sample_loop(o["model"], (8, 1, S, S), seed=seed)[:, 0]
    den = torch.empty_like(lat)
    _lib.check(_lib.load().cfd_latent_denorm(_lib.ptr(lat), _lib.ptr(den), lat.numel(), _lib.ptr(o["vmax"]),
                                             _lib.ptr(o["vmin"]), 1, _lib.stream_of(DEV)), "denorm")
    return den


def decode(den):
    return o["nf"].decode(o["coords"], den.reshape(8 * S, 1, S), o["xn"], o["yn"])


den0 = sample(1)
decode(den0)
torch.cuda.synchronize()


def timed(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3, r


print("full chip: sample %.1f ms, decode %.1f ms" % (timed(lambda: sample(2))[0], timed(lambda: decode(den0))[0]),
      flush=True)
for ku in (128, 112, 96):
    su = masked_stream(range(ku))
    sd = masked_stream(range(ku, NCU))

    def on(s, fn):
        with torch.cuda.stream(s):
            return fn()

    ts = timed(lambda: on(su, lambda: sample(3)))[0]
    td = timed(lambda: on(sd, lambda: decode(den0)))[0]

    def both():   # the decode first: the sampling loop synchronises its stream on the host
        with torch.cuda.stream(sd):
            b = decode(den0)
        with torch.cuda.stream(su):
            a = sample(4)
        return a, b

    tb = timed(both)[0]
    print(f"U-Net on {ku} CUs: sample {ts:.1f} ms | decode on {NCU - ku}: {td:.1f} ms | both together {tb:.1f} ms",
          flush=True)
