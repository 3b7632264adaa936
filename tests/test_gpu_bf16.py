"""GPU parity of the bf16-operand U-Net (config E, BASELINE.json configs[4]).

Two references, on the reference-pinned fixtures:
  * an emulation: the CPU oracle with every convolution that runs on
    conv_gemm fed bf16-rounded (RNE) operands and accumulating in fp32 -- the
    same arithmetic up to summation order, so a tight bound;
  * the fp32 oracle itself: the precision cost of bf16 operands, stated.
Tolerances (max|diff| / max|ref|) per topology, about 1.5x the largest value
measured over rounds 1-2 (emulation / fp32): tiny16 <= 8e-3 / 1e-2 (measured
4.8e-3 / 6.5e-3), small32 <= 1.5e-2 / 1.7e-2 (1.0e-2 / 1.13e-2), the config-E
width cfgE128 <= 8e-3 / 1e-2 (5.5e-3 / 6.9e-3).  The emulation cannot be
matched more tightly: bf16 rounding of fp32 values that differ by an ulp
(torch's vs this GroupNorm, say) flips roundings near the boundaries, and the
network amplifies that -- jittering the emulation's pre-rounding values by
1e-7 relative moves its own output by 3.8e-3.  A wrong operand layout would
be off by O(1).
"""
import ast

import pytest
import torch

from conftest import golden
from confild_amd import synth
from confild_amd.script_util import create_model
from oracle import unet as ou

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _bf(t):
    return t.to(torch.bfloat16).to(torch.float32)


class _Bf16Convs:
    """Round conv operands to bf16 where the HIP path does (every conv except the
    1-channel first/last ones, which run fp32 on the VALU)."""

    def __enter__(self):
        self.c2, self.c1 = c2, c1 = ou.F.conv2d, ou.F.conv1d

        def conv2d(x, w, b=None, stride=1, padding=0, *a, **k):
            if w.shape[0] > 4 and w.shape[1] > 4:
                x, w = _bf(x), _bf(w)
            return c2(x, w, b, stride, padding, *a, **k)

        def conv1d(x, w, b=None, *a, **k):
            return c1(_bf(x), _bf(w), b, *a, **k)

        ou.F.conv2d, ou.F.conv1d = conv2d, conv1d
        return self

    def __exit__(self, *exc):
        ou.F.conv2d, ou.F.conv1d = self.c2, self.c1


BOUNDS = {"tiny16": (8e-3, 1e-2), "small32": (1.5e-2, 1.7e-2), "cfgE128": (8e-3, 1e-2)}


@pytest.mark.parametrize("name", ["tiny16", "small32", "cfgE128"])
def test_bf16_unet_matches_emulation_and_fp32(hip, name):
    g = golden(f"unet_{name}.npz")
    kw = ast.literal_eval(str(g["kwargs"]))
    cfg = ou.Config(**kw)
    sd_np = synth.unet_state_dict(int(g["seed"]), ou.param_shapes(cfg))
    sd = {k: torch.from_numpy(v) for k, v in sd_np.items()}
    m = create_model(**kw, use_bf16=True)
    m.load_state_dict(sd)
    m.to(DEV)
    x, t = torch.from_numpy(g["x"]), torch.from_numpy(g["t"])
    eps = m(x.to(DEV), t.to(DEV)).cpu()
    with torch.no_grad(), _Bf16Convs():
        emu = ou.forward(sd, cfg, x, t)
    ref32 = torch.from_numpy(g["eps"])
    e_emu = float((eps - emu).abs().max() / emu.abs().max())
    e_32 = float((eps - ref32).abs().max() / ref32.abs().max())
    print(f"{name}: bf16 vs emulation {e_emu:.2e}, vs fp32 reference {e_32:.2e}")
    b_emu, b_32 = BOUNDS[name]
    assert e_emu < b_emu, e_emu
    assert e_32 < b_32, e_32
    # fp32 mode on the same module is the fp32 path again
    m.set_compute("fp32")
    e_back = float((m(x.to(DEV), t.to(DEV)).cpu() - ref32).abs().max() / ref32.abs().max())
    assert e_back < 1e-4, e_back


def test_bf16_unet_batch_invariant(hip):
    g = golden("unet_tiny16.npz")
    kw = ast.literal_eval(str(g["kwargs"]))
    m = create_model(**kw, use_bf16=True)
    sd = synth.unet_state_dict(int(g["seed"]), {k: tuple(v.shape) for k, v in m.state_dict().items()})
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m.to(DEV)
    x = torch.from_numpy(synth.normal(4, "bf", (5, 1, 16, 16))).to(DEV)
    t = torch.tensor([3, 77, 500, 901, 999], device=DEV)
    full = m(x, t)
    assert torch.equal(m(x[1:3], t[1:3]), full[1:3])
    with pytest.raises(NotImplementedError):
        m.forward_tape(x, t)


_GN_BF16_CHILD = r"""
import json, sys, torch
sys.path.insert(0, sys.argv[1])
from confild_amd import synth
from confild_amd.script_util import create_model
out = {}
for S, mult, B in ((16, "1,2", 3), (32, "1,2,2", 2), (64, "", 2), (128, "", 1)):
    kw = dict(image_size=S, num_channels=128 if S >= 64 else 64, num_res_blocks=2, channel_mult=mult, num_heads=4,
              num_head_channels=32, attention_resolutions="32,16,8" if S >= 64 else "8,4", use_bf16=True)
    m = create_model(**kw)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in
                       synth.unet_state_dict(9, {k: tuple(v.shape) for k, v in m.state_dict().items()}).items()})
    m.to("cuda")
    x = torch.from_numpy(synth.normal(3, f"gnbf/x{S}", (B, 1, S, S))).cuda()
    t = torch.tensor([999, 400, 3][:B], dtype=torch.int64).cuda()
    eps = m(x, t).cpu()
    out[S] = eps.numpy().tobytes().hex()
print(json.dumps(out))
"""


def test_gn_bf16_output_is_bit_identical(hip):
    """Config E's ResBlock GroupNorms write bf16 where their consumer runs K1hb
    (CFD_GN_BF16OUT, default on): the consumer would round the fp32 output to bf16
    (RNE) as it stages it, so eps must be bit-identical to the fp32-output path at
    every K1hb tile width (16^2 / 32^2 / 64^2 halo tiles) and batch, with the two
    concatenated skip sources included (the output blocks)."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = {}
    for flag in ("0", "1"):
        env = dict(os.environ, CFD_GN_BF16OUT=flag)
        r = subprocess.run([sys.executable, "-c", _GN_BF16_CHILD, root], capture_output=True, text=True, env=env,
                           timeout=240)
        assert r.returncode == 0, r.stderr[-3000:]
        res[flag] = json.loads(r.stdout.strip().splitlines()[-1])
    for S in res["0"]:
        assert res["0"][S] == res["1"][S], f"{S}^2: bf16 GroupNorm output changed eps"
