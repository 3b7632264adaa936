"""Dev: dump bf16 U-Net outputs of the tiny16 fixture for CPU-side analysis."""
import ast, sys, os
sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"]
import numpy as np, torch
from conftest import golden
from confild_amd import synth
from confild_amd.script_util import create_model
g = golden("unet_tiny16.npz"); kw = ast.literal_eval(str(g["kwargs"]))
m = create_model(**kw, use_bf16=True)
sd = synth.unet_state_dict(int(g["seed"]), {k: tuple(v.shape) for k, v in m.state_dict().items()})
m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}); m.to("cuda")
eps = m(torch.from_numpy(g["x"]).cuda(), torch.from_numpy(g["t"]).cuda()).cpu().numpy()
np.save("gpurun_out/bf16_tiny16.npy", eps)
print("saved", eps.shape)
