"""Config B batches serial vs overlapped on CU-masked streams: seconds per batch,
and each phase alone on its CU share.  Batch k's CNF decode runs on one CU set
while batch k+1 is sampled on the other (hipExtStreamCreateWithCUMask).
Measured (profiles/r03k_overlap_cu_probe.log): not a gain -- DESIGN.md section 4."""
import ctypes as C
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from confild_amd import _lib  # noqa: E402

# --- CU-masked streams straight from the HIP runtime (development probe only) ---
_hip = C.CDLL("libamdhip64.so")


def cu_streams(device, stride):
    """(sampling stream, decode stream): CU i samples when i % stride == 0."""
    idx = torch.device(device).index or 0
    n_cu = torch.cuda.get_device_properties(idx).multi_processor_count
    words = (n_cu + 31) // 32
    smp, dec = (C.c_uint32 * words)(), (C.c_uint32 * words)()
    for i in range(n_cu):
        m = smp if i % stride == 0 else dec
        m[i // 32] |= 1 << (i % 32)
    out = []
    for m in (smp, dec):
        h = C.c_void_p()
        rc = _hip.hipExtStreamCreateWithCUMask(C.byref(h), C.c_uint32(words), m)
        assert rc == 0, f"hipExtStreamCreateWithCUMask: {rc}"
        out.append(torch.cuda.ExternalStream(h.value, device=torch.device("cuda", idx)))
    return out[0], out[1], n_cu


def release(stream):
    _hip.hipStreamDestroy(C.c_void_p(stream.cuda_stream))


def run_overlapped(n_batches, sample, decode, s_smp, s_dec, ev=None):
    """sample(k) -> latents (on the current stream), decode(latents) -> fields.
    Batch k's decode is queued on s_dec behind an event on s_smp and batch k+1's
    sampling is queued right after it, so the two overlap.  The caller's stream
    waits for both at the end.  ev: optional per-batch [start, sampled, decoded]
    event triples (recorded on the streams that did the work).  Returns the last
    batch's fields."""
    cur = torch.cuda.current_stream()
    s_smp.wait_stream(cur)
    s_dec.wait_stream(cur)
    out = None
    for k in range(n_batches):
        with torch.cuda.stream(s_smp):
            if ev is not None:
                ev[k][0].record(s_smp)
            lat = sample(k)
            done = torch.cuda.Event()
            done.record(s_smp)
            if ev is not None:
                ev[k][1].record(s_smp)
        s_dec.wait_event(done)
        with torch.cuda.stream(s_dec):
            lat.record_stream(s_dec)
            out = decode(lat)
            if ev is not None:
                ev[k][2].record(s_dec)
    cur.wait_stream(s_smp)
    cur.wait_stream(s_dec)
    if out is not None:
        out.record_stream(cur)
    return out


dev = torch.device("cuda", 0)
o = bench.setup_B(dev, 0, 1, "split_f16", "split_f16")
S = bench.S


def sample(k):
    lat = o["diff"].p_sample_loop(o["model"], (8, 1, S, S), seed=10 ** 6 + k, sample_offset=0)[:, 0]
    den = torch.empty_like(lat)
    _lib.check(_lib.load().cfd_latent_denorm(_lib.ptr(lat), _lib.ptr(den), lat.numel(), _lib.ptr(o["vmax"]),
                                             _lib.ptr(o["vmin"]), 1, _lib.stream_of(dev)), "denorm")
    return den


def decode(den):
    return o["nf"].decode(o["coords"], den.reshape(8 * S, 1, S), o["xn"], o["yn"])


def timed(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = fn()
    torch.cuda.synchronize()
    return time.perf_counter() - t0, r


NB = int(os.environ.get("NB", "4"))
decode(sample(-1))
t, ref = timed(lambda: [decode(sample(k)) for k in range(NB)][-1])
print(json.dumps({"mode": "serial", "s_per_batch": t / NB}), flush=True)
for stride in [int(x) for x in os.environ.get("STRIDES", "4,3,6").split(",")]:
    s_smp, s_dec, n_cu = cu_streams(dev, stride)
    with torch.cuda.stream(s_smp):
        ts, lat = timed(lambda: sample(0))
    with torch.cuda.stream(s_dec):
        td, _ = timed(lambda: decode(lat))
    t, out = timed(lambda: run_overlapped(NB, sample, decode, s_smp, s_dec))
    same = bool(torch.equal(out, ref))
    print(json.dumps({"mode": "overlap", "stride": stride, "sample_cus": (n_cu + stride - 1) // stride,
                      "sample_alone_s": ts, "decode_alone_s": td, "s_per_batch": t / NB,
                      "last_batch_bit_identical": same}), flush=True)
    torch.cuda.synchronize()
    release(s_smp)
    release(s_dec)
