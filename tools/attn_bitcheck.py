"""Development check: the U-Net forward under two environments (child processes)
must be bit-identical (e.g. CFD_ATTN_DMA=0 vs 1).  Usage: attn_bitcheck.py ENV_A ENV_B"""
import os
import subprocess
import sys

CHILD = r"""
import sys, torch, numpy as np
sys.path.insert(0, sys.argv[1])
from confild_amd import synth
from confild_amd.script_util import create_model
dev = torch.device("cuda", 0)
m = create_model(image_size=64, num_channels=128, num_res_blocks=2, num_heads=4, num_head_channels=64,
                 attention_resolutions="32,16,8")
m.load_state_dict({k: torch.from_numpy(v) for k, v in synth.unet_state_dict(1234, {k: tuple(v.shape) for k, v in m.state_dict().items()}).items()})
m.to(dev)
x = torch.from_numpy(synth.normal(3, "bit/x", (3, 1, 64, 64))).to(dev)
t = torch.tensor([5, 400, 999], device=dev)
np.save(sys.argv[2], m(x, t).cpu().numpy())
"""
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
outs = []
for i, e in enumerate(sys.argv[1:3]):
    env = dict(os.environ)
    k, v = e.split("=", 1)
    env[k] = v
    f = f"/tmp/bitcheck_{i}.npy"
    subprocess.run([sys.executable, "-c", CHILD, root, f], env=env, check=True)
    import numpy as np
    outs.append(np.load(f))
import numpy as np
d = np.abs(outs[0] - outs[1]).max()
print("max |diff| =", d, "bit-identical" if (outs[0] == outs[1]).all() else "DIFFERENT")
