"""Development: the clock the config-B decoder (siren_split32, K7t) actually runs
at, measured inside the kernel -- replacing the GRBM_GUI_ACTIVE / 8 / duration
estimate (MI355X_MICROARCH.md "DVFS give-back" item 6).

The CFD_STAMPS build (make -C confild_amd/csrc STAMPS=1) has wave 0 of every
61st tile column record s_memrealtime (100 MHz) and s_memtime (shader cycles)
at kernel entry and exit (kind 5).  Per stamped workgroup the clock is
d(memtime) / d(realtime) x 100 MHz; the median over workgroups is reported for:
  whole   the decode on all CUs, after >= 2 s of back-to-back decodes
  half    the decode alone on CUs [n/2, n) (bench.py PipelineB's decode half)
  piped   the same half while the 256-step config-B sampler runs on CUs [0, n/2)
          (the headline's pipelined condition; the stamped workgroups that ran
          while the sampler ran are reported separately)

    CFD_LIB=libconfild_hip_stamps.so python tools/dev/siren_clock.py --json out.json
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
os.environ.setdefault("CFD_LIB", "libconfild_hip_stamps.so")

import bench  # noqa: E402
from confild_amd import _lib  # noqa: E402
from confild_amd.streams import CuRangeStream, cu_count  # noqa: E402

DEV = torch.device("cuda", 0)
NREC = 1 << 20


def collect(buf):
    b = buf.cpu().numpy().view(np.uint64)
    n = int(min(b[0], NREC))
    r = b[8:8 + 8 * n].reshape(n, 8)
    kind = (r[:, 1] >> np.uint64(56)).astype(np.int64)
    slot = (r[:, 1] & np.uint64(0xFFFFFF)).astype(np.int64)
    key = (r[:, 2].astype(np.int64) << 20) ^ ((r[:, 1] >> np.uint64(24)) & np.uint64(0xFFFFFFFF)).astype(np.int64)
    sel = kind == 5
    ent = {k: (rt, mt) for k, rt, mt, s in zip(key[sel], r[sel, 0], r[sel, 3], slot[sel]) if s == 0}
    out = []
    for k, rt, mt, s in zip(key[sel], r[sel, 0], r[sel, 3], slot[sel]):
        if s == 4 and k in ent:
            rt0, mt0 = ent[k]
            drt = int(rt) - int(rt0)
            if drt > 0:
                out.append((int(rt0), int(rt), (int(mt) - int(mt0)) / drt * 0.1))   # GHz
    return out


def summary(rows, t_lo=None, t_hi=None):
    if t_lo is not None:
        rows = [r for r in rows if r[0] >= t_lo and r[1] <= t_hi]
    if not rows:
        return None
    g = np.array([r[2] for r in rows])
    span = (max(r[1] for r in rows) - min(r[0] for r in rows)) / 1e8
    return {"workgroups": len(rows), "clock_ghz_median": float(np.median(g)), "p10": float(np.percentile(g, 10)),
            "p90": float(np.percentile(g, 90)), "wg_us_median": float(np.median([(r[1] - r[0]) / 100 for r in rows])),
            "span_s": span}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default="")
    args = ap.parse_args()
    lib = _lib.load()
    lib.cfd_stamps_set.argtypes = [ctypes.c_void_p]
    o = bench.setup_B(DEV, 0, 1, "split_f16", "split_f16")
    nf, coords = o["nf"], o["coords"]
    lat = torch.randn(8 * bench.S, 1, bench.S, device=DEV) * 0.5
    flops = lat.shape[0] * coords.shape[0] * bench.siren_flops_per_pair(**bench.CNF_B)
    buf = torch.zeros(8 + 8 * NREC, dtype=torch.int64, device=DEV)
    res = {"kernel": "siren_split32<12,0,4> (K7t)", "flops_per_launch": flops}

    def stamped(fn, stream):
        buf.zero_()
        torch.cuda.synchronize()
        _lib.check(lib.cfd_stamps_set(ctypes.c_void_p(buf.data_ptr())), "cfd_stamps_set")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(stream):
            e0.record()
            fn()
            e1.record()
        torch.cuda.synchronize()
        _lib.check(lib.cfd_stamps_set(None), "cfd_stamps_set")
        return collect(buf), e0.elapsed_time(e1)

    dec = lambda: nf.decode(coords, lat, o["xn"], o["yn"])  # noqa: E731
    main_s = torch.cuda.current_stream()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 2.5:      # >= 2 s of back-to-back decodes
        dec()
        torch.cuda.synchronize()
    rows, ms = stamped(dec, main_s)
    res["whole"] = dict(summary(rows), launch_ms=ms, tflops=flops / ms / 1e9, cus=cu_count(DEV))
    n = cu_count(DEV)
    with CuRangeStream(DEV, 0, n // 2) as su, CuRangeStream(DEV, n // 2, n - n // 2) as sd:
        for _ in range(2):
            with torch.cuda.stream(sd.stream):
                dec()
        torch.cuda.synchronize()
        rows, ms = stamped(dec, sd.stream)
        res["half"] = dict(summary(rows), launch_ms=ms, tflops=flops / ms / 1e9, cus=n - n // 2)
        # the pipelined condition: the sampler on the other half for the whole decode.
        # One sampling pass first, outside the stamped window: it captures the
        # sampler's HIP graphs with no stamp buffer set (the U-Net kernels of the
        # stamps build would otherwise fill the buffer)
        with torch.cuda.stream(su.stream):
            bench.sample_B(o, DEV, 10 ** 6 - 1, 0, 8)
        torch.cuda.synchronize()
        buf.zero_()
        torch.cuda.synchronize()
        _lib.check(lib.cfd_stamps_set(ctypes.c_void_p(buf.data_ptr())), "cfd_stamps_set")
        u0, u1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        d0, d1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        # the decode is enqueued first: the sampler's host loop synchronises its
        # stream every 64 steps, so enqueueing it first would hold the decode back
        with torch.cuda.stream(sd.stream):
            d0.record()
            dec()
            d1.record()
        with torch.cuda.stream(su.stream):
            u0.record()
            for k in range(2):
                bench.sample_B(o, DEV, 10 ** 6 + k, 0, 8)
            u1.record()
        torch.cuda.synchronize()
        _lib.check(lib.cfd_stamps_set(None), "cfd_stamps_set")
        rows = collect(buf)
        ms = d0.elapsed_time(d1)
        res["piped"] = dict(summary(rows), launch_ms=ms, tflops=flops / ms / 1e9, cus=n - n // 2,
                            sampler_ms=u0.elapsed_time(u1),
                            decode_within_sampling=d0.elapsed_time(u0) <= 50 and d0.elapsed_time(d1) <= d0.elapsed_time(u1))
    res["method"] = ("d(s_memtime) / d(s_memrealtime) x 100 MHz per stamped workgroup (entry -> exit), median; "
                     "MI355X_MICROARCH.md DVFS give-back item 6")
    print(json.dumps(res, indent=1))
    if args.json:
        json.dump(res, open(args.json, "w"), indent=1)


if __name__ == "__main__":
    main()
