"""Bit-identity check of two in-tree builds of the library (development tool):
runs a fixed set of HIP-path computations in a child process per build
(CFD_LIB selects the build) and compares the outputs' hashes.

    python tools/libdiff.py libconfild_hip_pre.so libconfild_hip.so
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import hashlib, json, sys, torch
sys.path.insert(0, sys.argv[1])
from confild_amd import synth
from confild_amd.script_util import create_model
from confild_amd.nf_networks import SIRENAutodecoder_film
out = {}
def h(t):
    return hashlib.sha256(t.detach().cpu().contiguous().numpy().tobytes()).hexdigest()[:16]
cases = [(32, "1,2,3,4", "split_f16", (1, 3)), (64, "", "split_f16", (1, 2, 8)), (128, "", "bf16", (2,)),
         (64, "", "fp32", (2,)), (128, "", "split_f16", (1,)), (384, "1,1,2,2,4,4", "split_f16", (1,))]
for S, mult, comp, Bs in cases:
    m = create_model(image_size=S, num_channels=128, num_res_blocks=2, channel_mult=mult, num_heads=4,
                     num_head_channels=64, attention_resolutions="32,16,8")
    m.load_state_dict({k: torch.from_numpy(v) for k, v in
                       synth.unet_state_dict(7, {k: tuple(v.shape) for k, v in m.state_dict().items()}).items()})
    m.to("cuda").set_compute(comp)
    for pb in ((0, 1, 2) if S == 64 else (0,)):
        m.set_plan_batch(pb)
        for B in Bs:
            x = torch.from_numpy(synth.normal(3, f"ld/x{S}", (B, 1, S, S))).cuda()
            t = torch.tensor([999, 500, 3, 250, 700, 10, 900, 60][:B], dtype=torch.int64).cuda()
            out[f"fwd/{S}/{comp}/pb{pb}/B{B}"] = h(m(x, t))
            if comp != "bf16" and S <= 128:
                m.forward_tape(x, t)
                d = torch.from_numpy(synth.normal(4, f"ld/d{S}", (B, 1, S, S))).cuda()
                out[f"vjp/{S}/{comp}/pb{pb}/B{B}"] = h(m.input_vjp(d))
                if S <= 64 and B <= 2:
                    m.forward_tape(x, t, for_param_grad=True)
                    out[f"pgrad/{S}/{comp}/pb{pb}/B{B}"] = h(m.param_grad(d))
    m.set_plan_batch(0)
for dims in ((3, 64, 3, 15, 384), (2, 32, 3, 10, 128), (2, 128, 2, 17, 256), (3, 48, 3, 5, 96)):
    nf = SIRENAutodecoder_film(*dims)
    nf.load_state_dict({k: torch.from_numpy(v) for k, v in synth.siren_state_dict(5, *dims).items()})
    nf.to("cuda")
    g = torch.Generator().manual_seed(1)
    coords = torch.rand(20000, dims[0], generator=g).cuda()
    lat = (torch.randn(6, 1, dims[1], generator=g) * 0.5).cuda()
    out[f"siren/{dims}"] = h(nf(coords, lat))
print(json.dumps(out))
"""


def run(lib):
    env = dict(os.environ, CFD_LIB=lib)
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], capture_output=True, text=True, env=env, timeout=600)
    if r.returncode != 0:
        print(r.stderr[-3000:])
        raise SystemExit(1)
    return json.loads(r.stdout.strip().splitlines()[-1])


if __name__ == "__main__":
    a, b = sys.argv[1], sys.argv[2]
    ra, rb = run(a), run(b)
    diff = [k for k in ra if ra[k] != rb.get(k)]
    print(json.dumps({"a": a, "b": b, "cases": len(ra), "differ": diff}))
    sys.exit(1 if diff else 0)
