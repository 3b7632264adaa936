"""SIREN tape kernels (DPS adjoint) timed alone, per in-tree library build
(development tool): one child process per build (CFD_LIB selects it), HIP events
around tape_forward and tape_vjp at the config-D (8 chains x 64 rows x 10 sensors)
and real-Case4 (384 rows x 10 sensors) pair counts, median of 20, plus a hash of
the outputs so builds that should agree can be compared.

    python tools/dev/tape_bench.py libconfild_hip_k9t0.so libconfild_hip.so
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CHILD = r"""
import hashlib, json, sys, torch
sys.path.insert(0, sys.argv[1])
from confild_amd import synth
from confild_amd.nf_networks import SIRENAutodecoder_film
from confild_amd.normalize import Normalizer_ts
dev = torch.device("cuda", 0)
d, L, c, nh, H = 3, 64, 3, 15, 384
nf = SIRENAutodecoder_film(d, L, c, nh, H)
nf.load_state_dict({k: torch.from_numpy(v) for k, v in synth.siren_state_dict(5, d, L, c, nh, H).items()})
nf.to(dev)
xn = Normalizer_ts(params=(torch.full((1, d), 1.0), torch.full((1, d), -1.0)), method="-11", dim=0)
yn = Normalizer_ts(params=(torch.full((c,), 2.0), torch.full((c,), -2.0)), method="-11", dim=0)
res = {}
for name, R in (("D", 512), ("Case4", 384)):
    coords = torch.from_numpy(synth.uniform(5, "c", (10, d), -1.0, 1.0)).to(dev)
    z = (torch.from_numpy(synth.normal(5, "z", (R, L))) * 0.5).to(dev)
    g = torch.from_numpy(synth.normal(5, "g", (R, 10, c))).to(dev)
    tf, tb = [], []
    for it in range(25):
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record(); out = nf.tape_forward(coords, z, xn, yn); e1.record(); gz = nf.tape_vjp(g); e2.record()
        e2.synchronize()
        if it >= 5:
            tf.append(e0.elapsed_time(e1)); tb.append(e1.elapsed_time(e2))
    tf.sort(); tb.sort()
    hh = lambda t: hashlib.sha256(t.detach().cpu().numpy().tobytes()).hexdigest()[:12]
    res[name] = {"fwd_ms": tf[len(tf) // 2], "vjp_ms": tb[len(tb) // 2], "out": hh(out), "gz": hh(gz)}
print(json.dumps(res))
"""


def main():
    libs = sys.argv[1:] or ["libconfild_hip.so"]
    rows = {}
    for rnd in range(2):
        for lib in libs:
            env = dict(os.environ, CFD_LIB=lib)
            p = subprocess.run([sys.executable, "-c", CHILD, ROOT], env=env, capture_output=True, text=True,
                               timeout=300)
            if p.returncode != 0:
                print(p.stderr[-3000:], file=sys.stderr)
                sys.exit(p.returncode)
            rows.setdefault(lib, []).append(json.loads(p.stdout.strip().splitlines()[-1]))
    print(json.dumps(rows, indent=1))


if __name__ == "__main__":
    main()
