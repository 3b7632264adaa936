"""Development: where a small-batch U-Net forward spends its time INSIDE its
kernels.  Runs one forward on the CFD_STAMPS build (make -C confild_amd/csrc
STAMPS=1 -> lib/libconfild_hip_stamps.so), whose convolution (K1s kind 1, K1x 2,
K1h 3) and register-resident GroupNorm (4) kernels have wave 0 of every
workgroup record s_memrealtime (100 MHz) at named points:
  slot 0  kernel entry            slot 1  prologue done (pixel table / loads in)
  slot 2  first tile staged       slot 3  K loop done       slot 4  stores done
and prints, per launch and summed per kind: the workgroup count, the span from
the first workgroup's entry to the last one's end, the dispatch skew, and the
median per-workgroup phase durations; plus the gaps between launches.

    CFD_LIB=libconfild_hip_stamps.so python tools/dev/stamps.py --size 64 --batch 1
"""
import argparse
import collections
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ.setdefault("CFD_LIB", "libconfild_hip_stamps.so")

from confild_amd import _lib, synth  # noqa: E402
from confild_amd.script_util import create_model  # noqa: E402

KIND = {1: "K1s", 2: "K1x", 3: "K1h", 4: "GN"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--mult", default="")
    ap.add_argument("--detail", type=int, default=40, help="launches printed in detail")
    ap.add_argument("--json", default="")
    ap.add_argument("--bf16", action="store_true", help="bf16-operand U-Net (config E arithmetic)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    m = create_model(image_size=args.size, num_channels=128, num_res_blocks=2, num_heads=4, num_head_channels=64,
                     attention_resolutions="32,16,8", channel_mult=args.mult, use_bf16=args.bf16)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in
                       synth.unet_state_dict(1234, {k: tuple(v.shape) for k, v in m.state_dict().items()}).items()})
    m.to(dev)
    x = torch.randn(args.batch, 1, args.size, args.size, device=dev)
    t = torch.full((args.batch,), 500, dtype=torch.int64, device=dev)
    for _ in range(3):
        m(x, t)
    torch.cuda.synchronize()
    lib = _lib.load()
    lib.cfd_stamps_set.argtypes = [ctypes.c_void_p]
    buf = torch.zeros(8 + 8 * (1 << 20), dtype=torch.int64, device=dev)
    _lib.check(lib.cfd_stamps_set(ctypes.c_void_p(buf.data_ptr())), "cfd_stamps_set")
    m(x, t)
    torch.cuda.synchronize()
    _lib.check(lib.cfd_stamps_set(None), "cfd_stamps_set")
    b = buf.cpu().numpy().view(np.uint64)
    n = int(b[0])
    rec = b[8:8 + 8 * n].reshape(n, 8)
    tt = rec[:, 0].astype(np.int64)
    code = rec[:, 1]
    kind = (code >> np.uint64(56)).astype(np.int64)
    seq = ((code >> np.uint64(24)) & np.uint64(0xFFFFFFFF)).astype(np.int64)
    slot = (code & np.uint64(0xFFFFFF)).astype(np.int64)
    blk = rec[:, 2]
    hwid = rec[:, 4]
    # compute unit of a stamp: XCC, SE, SH, CU fields of HW_ID / XCC_ID
    cu_of = ((hwid >> np.uint64(32)) & np.uint64(0xF)) * np.uint64(1 << 8) + ((hwid >> np.uint64(13)) & np.uint64(7)) * \
        np.uint64(32) + ((hwid >> np.uint64(12)) & np.uint64(1)) * np.uint64(16) + ((hwid >> np.uint64(8)) & np.uint64(0xF))
    launches = []
    for s in sorted(set(seq.tolist())):
        sel = seq == s
        k = int(kind[sel][0])
        ph = collections.defaultdict(dict)
        for ti, sl, bl in zip(tt[sel], slot[sel], blk[sel]):
            ph[int(bl)][int(sl)] = int(ti)
        wgs = list(ph.values())
        # residency: per compute unit, the most workgroups of this launch running at once
        cus = {}
        for ti, sl, bl, cu in zip(tt[sel], slot[sel], blk[sel], cu_of[sel]):
            if sl == 0:
                cus.setdefault(int(cu), []).append(int(bl))
        conc = 0
        for cu, bls in cus.items():
            ev = []
            for bl in bls:
                w = ph[bl]
                if 0 in w and (4 in w or 3 in w):
                    ev += [(w[0], 1), (w.get(4, w.get(3)), -1)]
            ev.sort(key=lambda e: (e[0], e[1]))
            c = m = 0
            for _, d in ev:
                c += d
                m = max(m, c)
            conc = max(conc, m)
        t0 = [w[0] for w in wgs if 0 in w]
        t4 = [w.get(4, w.get(3)) for w in wgs if (4 in w or 3 in w)]
        if not t0 or not t4:
            continue

        def med(a, bb):
            v = [w[bb] - w[a] for w in wgs if a in w and bb in w]
            return float(np.median(v)) * 10 if v else None   # 10 ns ticks -> ns

        launches.append(dict(seq=s, kind=KIND.get(k, str(k)), wgs=len(wgs), cus=len(cus), per_cu=conc,
                             start=min(t0) * 10, end=max(t4) * 10,
                             skew=(max(t0) - min(t0)) * 10, p01=med(0, 1), p02=med(0, 2), p12=med(1, 2),
                             p23=med(2, 3), p34=med(3, 4), p04=med(0, 4) or med(0, 3)))
    launches.sort(key=lambda d: d["start"])
    t_first = launches[0]["start"]
    print(f"{len(launches)} instrumented launches, {n} stamps; forward span (first entry -> last end) "
          f"{(launches[-1]['end'] - t_first) / 1e3:.1f} us")
    fmt = lambda v: "   -  " if v is None else f"{v / 1e3:6.2f}"  # noqa: E731
    print("  seq kind   WGs  CUs /cu   start    span  skew | 0->1  0->2  2->3  3->4  wg-total   gap-before")
    prev_end = None
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for i, d in enumerate(launches):
        gap = None if prev_end is None else d["start"] - prev_end
        prev_end = d["end"]
        span = d["end"] - d["start"]
        pk = per[d["kind"]]
        pk["n"] += 1
        pk["span"] += span
        for key in ("p02", "p23", "p34", "p04"):
            pk[key] += d[key] or 0.0
        pk["gap"] += gap or 0.0
        if i < args.detail:
            print(f"  {d['seq']:4d} {d['kind']:4s} {d['wgs']:5d} {d['cus']:4d} {d['per_cu']:3d} "
                  f"{(d['start'] - t_first) / 1e3:7.1f} {span / 1e3:7.2f} "
                  f"{d['skew'] / 1e3:5.2f} | {fmt(d['p01'])}{fmt(d['p02'])}{fmt(d['p23'])}{fmt(d['p34'])} "
                  f"{fmt(d['p04'])}   {fmt(gap)}")
    print("per kind (us, summed over launches): n, span, median WG first-stage (0->2), K loop (2->3), "
          "epilogue (3->4), WG total, gaps before")
    out = {}
    for k, v in per.items():
        out[k] = {kk: (vv / 1e3 if kk != "n" else vv) for kk, vv in v.items()}
        print(f"  {k:4s} n={int(v['n']):3d} span {v['span'] / 1e3:8.1f}  first {v['p02'] / 1e3:7.1f}  "
              f"loop {v['p23'] / 1e3:7.1f}  epi {v['p34'] / 1e3:7.1f}  wg {v['p04'] / 1e3:7.1f}  gaps {v['gap'] / 1e3:7.1f}")
    if args.json:
        with open(args.json, "w") as f:
            json.dump({"launches": launches, "per_kind": out}, f)


if __name__ == "__main__":
    main()
