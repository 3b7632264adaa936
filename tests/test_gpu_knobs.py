"""Launch-shape switches that must not change a single bit: they pick how the
work is scheduled -- the register-ring depth of the K1s convolution tiles
(CFD_CONV_PF, default 2), the convolution tiles' workgroup order over the XCDs
(CFD_CONV_XCD: 3 the round-5 per-level order, 0 dispatch order; default 4), the 64-channel small-batch workgroups of K1h / K1s (default,
CFD_CONV_SMALLN=0 restores 128), the K1h / K1hb split-K 2 run as two
in-workgroup K groups instead of two workgroups and a partial slab
(CFD_CONV_KHG: 1 wherever it applies; default 0, never), the K1hb register
build for two workgroups per CU (CFD_CONV_KHB_OCC, off by default since round 5; on above 256
workgroups: the 128^2 batch-5 case), the K1s / K1h epilogues through LDS
(CFD_CONV_LDSEPI, default on), the attention workgroups of one (sample, head)
on one XCD (CFD_ATTN_XCD, default on) -- never the tiles' K order or the split-K boundaries, so every
output's summation order, and hence eps, is unchanged.  Each setting runs in a
child process (the switches are read once per process) over split-f16 U-Nets at
the config-A and config-B widths, at batch 1 and 3 (the small-batch shapes these
are for), and bf16 (config-E arithmetic) U-Nets with bf16 GroupNorm outputs,
compared bit for bit with the default."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, sys, torch
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
        out[f"{S}/{B}"] = m(x, t).cpu().numpy().tobytes().hex()
for S, mult, B in ((32, "1,2,2", 2), (64, "", 2), (128, "1,1", 5)):
    m = create_model(image_size=S, num_channels=128, num_res_blocks=2, channel_mult=mult, num_heads=4,
                     num_head_channels=64, attention_resolutions="32,16,8", use_bf16=True)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in
                       synth.unet_state_dict(12, {k: tuple(v.shape) for k, v in m.state_dict().items()}).items()})
    m.to("cuda")
    x = torch.from_numpy(synth.normal(5, f"knob/xb{S}", (B, 1, S, S))).cuda()
    t = torch.tensor([999, 3, 500, 40, 700][:B], dtype=torch.int64).cuda()
    out[f"bf16/{S}"] = m(x, t).cpu().numpy().tobytes().hex()
print(json.dumps(out))
"""


def _run(env_extra):
    env = dict(os.environ, **env_extra)
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], capture_output=True, text=True, env=env, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("knob", ["CFD_CONV_PF=1", "CFD_CONV_PF=3", "CFD_CONV_SMALLN=0", "CFD_CONV_KHG=1",
                                  "CFD_CONV_KHB_OCC=1", "CFD_CONV_LDSEPI=0", "CFD_ATTN_XCD=0", "CFD_CONV_XCD=3",
                                  "CFD_CONV_XCD=0"])
def test_schedule_switch_is_bit_identical(hip, knob):
    # K1h's in-workgroup K groups take no fused skip convolution (conv_takes_skip):
    # that switch is compared with the skip convolutions unfused on both sides
    extra = {"CFD_CONV_SKIPFUSE": "0"} if knob.startswith("CFD_CONV_KHG") else {}
    base = _run(extra)
    k, v = knob.split("=")
    got = _run(dict(extra, **{k: v}))
    for key in base:
        assert got[key] == base[key], f"{knob} changed eps at {key}"


FUSED = r"""
import ast, json, sys, numpy as np, torch
sys.path.insert(0, sys.argv[1])
from confild_amd import synth
from confild_amd.script_util import create_model
out = {}
for name in ("small32", "cfgA32", "cfgB64"):
    g = np.load(f"{sys.argv[1]}/tests/golden/unet_{name}.npz", allow_pickle=False)
    kw = ast.literal_eval(str(g["kwargs"]))
    m = create_model(**kw)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in
                       synth.unet_state_dict(int(g["seed"]), {k: tuple(v.shape) for k, v in m.state_dict().items()}).items()})
    m.to("cuda")
    eps = m(torch.from_numpy(g["x"]).cuda(), torch.from_numpy(g["t"]).cuda()).cpu().numpy()
    out[name] = float(np.abs(eps - g["eps"]).max() / np.abs(g["eps"]).max())
print(json.dumps(out))
"""


@pytest.mark.parametrize("mode", ["1", "2"])
def test_fused_skip_convolution_vs_reference(hip, mode):
    """The ResBlock skip 1x1 convolution fused into out_layers (CFD_CONV_SKIPFUSE:
    1 on K1h, 2 on K1x too; off by default, measured slower): the U-Nets with
    concatenated skips against the reference goldens at the forward's 1e-5."""
    env = dict(os.environ, CFD_CONV_SKIPFUSE=mode)
    r = subprocess.run([sys.executable, "-c", FUSED, ROOT], capture_output=True, text=True, env=env, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    errs = json.loads(r.stdout.strip().splitlines()[-1])
    print(f"fused skip ({mode}) vs reference: {errs}")
    assert max(errs.values()) <= 1e-5, errs


BF16_EPS = r"""
import json, sys, numpy as np, torch
sys.path.insert(0, sys.argv[1])
from confild_amd import synth
from confild_amd.script_util import create_model
out = {}
for S, mult, B in ((32, "1,2,2", 2), (64, "", 2)):
    m = create_model(image_size=S, num_channels=128, num_res_blocks=2, channel_mult=mult, num_heads=4,
                     num_head_channels=64, attention_resolutions="32,16,8", use_bf16=True)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in
                       synth.unet_state_dict(12, {k: tuple(v.shape) for k, v in m.state_dict().items()}).items()})
    m.to("cuda")
    x = torch.from_numpy(synth.normal(5, f"knob/xb{S}", (B, 1, S, S))).cuda()
    t = torch.tensor([999, 3][:B], dtype=torch.int64).cuda()
    out[str(S)] = m(x, t).cpu().numpy().ravel().tolist()
print(json.dumps(out))
"""


def test_bf16_k1x_option_matches_k1s_tiles(hip):
    """CFD_CONV_KXB=1 (off by default, measured 0.4% slower): config E's 8^2 3x3
    convolutions on K1x with bf16 operands instead of the K1s bf16 tiles -- the
    same operand rounding, another accumulation order: eps within bf16 rounding
    of the default (the bf16 suite's 1.5e-2 of max |eps|)."""
    def run(extra):
        r = subprocess.run([sys.executable, "-c", BF16_EPS, ROOT], capture_output=True, text=True,
                           env=dict(os.environ, **extra), timeout=240)
        assert r.returncode == 0, r.stderr[-3000:]
        return json.loads(r.stdout.strip().splitlines()[-1])
    import numpy as np
    base, got = run({}), run({"CFD_CONV_KXB": "1"})
    for k in base:
        b, g = np.array(base[k]), np.array(got[k])
        err = np.abs(g - b).max() / np.abs(b).max()
        print(f"bf16 {k}^2: K1x vs K1s tiles {err:.2e}")
        assert err <= 1.5e-2, (k, err)
