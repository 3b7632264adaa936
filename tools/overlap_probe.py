"""Probe: serial vs stream-overlapped generation (development tool).
U-Net sampling of batch k+1 on one stream while batch k decodes on another."""
import os, sys, time, json
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench
from confild_amd import _lib

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
objs = bench.setup(dev)
model, diff, nf, coords, xn, yn, vmax, vmin = objs
B, S = bench.B, bench.S

def sample(seed):
    lat = diff.p_sample_loop(model, (B, 1, S, S), seed=seed)[:, 0]
    den = torch.empty_like(lat)
    _lib.check(_lib.load().cfd_latent_denorm(_lib.ptr(lat), _lib.ptr(den), lat.numel(), _lib.ptr(vmax),
                                             _lib.ptr(vmin), 1, _lib.stream_of(dev)), "denorm")
    return den

def decode(den):
    return nf.decode(coords, den.reshape(B * S, 1, S), xn, yn)

K = int(os.environ.get("K", "3"))
# warm
decode(sample(1)); torch.cuda.synchronize()
t0 = time.perf_counter()
for k in range(K):
    f = decode(sample(100 + k))
torch.cuda.synchronize()
ser = (time.perf_counter() - t0) / K
res = {"serial_s": ser}
for prio in (0, -1):
    su = torch.cuda.Stream(device=dev, priority=prio)
    sd = torch.cuda.Stream(device=dev, priority=0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(su):
        den = sample(200)
    outs = []
    for k in range(K):
        ev = torch.cuda.Event()
        ev.record(su)
        sd.wait_event(ev)
        with torch.cuda.stream(sd):
            den.record_stream(sd)
            outs.append(decode(den))
        if k + 1 < K:
            with torch.cuda.stream(su):
                den = sample(201 + k)
    torch.cuda.synchronize()
    res[f"overlap_prio{prio}_s"] = (time.perf_counter() - t0) / K
    del outs
print(json.dumps(res), flush=True)
