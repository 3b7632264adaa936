"""Development: eps of split-f16 U-Nets (config-A / config-B widths, B = 1 / 3) under
environment settings, each in a child process, compared bit for bit with the
first setting (and max |diff|).  python tools/dev/env_bits.py "" "CFD_ATTN_KVFUSE=0" ..."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CHILD = r"""
import json, sys, torch, numpy as np
sys.path.insert(0, sys.argv[1])
from confild_amd import synth
from confild_amd.script_util import create_model
out = {}
for S, mult in ((32, "1,2,3,4"), (64, "")):
    m = create_model(image_size=S, num_channels=128, num_res_blocks=2, channel_mult=mult, num_heads=4,
                     num_head_channels=64, attention_resolutions="32,16,8")
    m.load_state_dict({k: torch.from_numpy(v) for k, v in
                       synth.unet_state_dict(11, {k: tuple(v.shape) for k, v in m.state_dict().items()}).items()})
    m.to("cuda")
    for B in (1, 3):
        x = torch.from_numpy(synth.normal(4, f"knob/x{S}", (B, 1, S, S))).cuda()
        t = torch.tensor([999, 400, 3][:B], dtype=torch.int64).cuda()
        e = m(x, t).cpu().numpy()
        np.save(f"{sys.argv[2]}_{S}_{B}.npy", e)
        out[f"{S}/{B}"] = 1
print(json.dumps(out))
"""
base = None
os.makedirs("gpurun_out/envbits", exist_ok=True)
for i, setting in enumerate(sys.argv[1:]):
    env = dict(os.environ)
    for kv in setting.split():
        k, v = kv.split("=")
        env[k] = v
    tag = f"gpurun_out/envbits/s{i}"
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT, tag], capture_output=True, text=True, env=env, timeout=300)
    if r.returncode:
        print(setting, "FAILED", r.stderr[-2000:])
        sys.exit(1)
    res = {}
    for S in (32, 64):
        for B in (1, 3):
            e = np.load(f"{tag}_{S}_{B}.npy")
            if i == 0:
                res[f"{S}/{B}"] = "base"
            else:
                b = np.load(f"gpurun_out/envbits/s0_{S}_{B}.npy")
                res[f"{S}/{B}"] = "same" if np.array_equal(e, b) else f"maxdiff {float(np.abs(e - b).max()):.3e}"
    print(json.dumps({"setting": setting or "(default)", **res}), flush=True)
