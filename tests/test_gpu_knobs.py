"""Every process-wide switch the HIP library reads (CFD_* environment
variables, read once per process), each exercised here; round 6 removed the
rest (their defaults are now code, the measured-slower variants deleted).

Schedule switches that must not change a single bit -- they pick how the work
is scheduled, never the tiles' K order or the split-K boundaries, so every
output's summation order, and hence eps, is unchanged:
  CFD_CONV_PF      the register-ring depth of the K1s convolution tiles (1-3; default 2)
  CFD_CONV_XCD     the convolution tiles' workgroup order over the XCDs (0 dispatch
                   order, 3 the round-5 per-level order; default 4)
  CFD_CONV_SMALLN  the 64-channel small-batch workgroups of K1h / K1s (0 keeps 128)
  CFD_CONV_LDSEPI  the K1s / K1h epilogues through LDS (default on)
  CFD_ATTN_XCD     the attention workgroups of one (sample, head) on one XCD (default on)
  CFD_GN_BF16OUT   config E's bf16 GroupNorm outputs feeding K1hb (default on)
  CFD_CONV_LOG     one stderr line per convolution / GroupNorm plan (diagnostic)
Each runs in a child process over split-f16 U-Nets at the config-A and config-B
widths, at batch 1 and 3 (the small-batch shapes these are for), and bf16
(config-E arithmetic) U-Nets with bf16 GroupNorm outputs, compared bit for bit
with the default.
And one that changes the kernel (so the summation order), pinned to fp32
rounding: CFD_CONV_FORCE_K1S, the K1s fallback of the K1x / K1h plans.
"""
import json
import os
import subprocess
import sys

import pytest

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


# every CFD_* switch read by confild_amd/csrc, and the test below that covers it
SWITCHES = {"CFD_CONV_PF": "schedule", "CFD_CONV_XCD": "schedule", "CFD_CONV_SMALLN": "schedule",
            "CFD_CONV_LDSEPI": "schedule", "CFD_ATTN_XCD": "schedule", "CFD_CONV_LOG": "schedule",
            "CFD_GN_BF16OUT": "gn_bf16", "CFD_CONV_FORCE_K1S": "forced_k1s"}


def test_every_library_switch_is_tested():
    """The library's switch surface is exactly SWITCHES (source scan, no GPU)."""
    import glob
    import re
    found = set()
    for f in glob.glob(os.path.join(ROOT, "confild_amd", "csrc", "*.*")):
        found |= set(re.findall(r'(?:getenv|env_int)\("(CFD_[A-Z0-9_]+)"', open(f).read()))
    assert found == set(SWITCHES), (sorted(found - set(SWITCHES)), sorted(set(SWITCHES) - found))
    assert len(found) <= 12


@pytest.mark.gpu
@pytest.mark.parametrize("knob", ["CFD_CONV_PF=1", "CFD_CONV_PF=3", "CFD_CONV_SMALLN=0", "CFD_CONV_LDSEPI=0",
                                  "CFD_ATTN_XCD=0", "CFD_CONV_XCD=3", "CFD_CONV_XCD=0", "CFD_GN_BF16OUT=0",
                                  "CFD_CONV_LOG=1"])
def test_schedule_switch_is_bit_identical(hip, knob):
    base = _run({})
    k, v = knob.split("=")
    got = _run({k: v})
    for key in base:
        assert got[key] == base[key], f"{knob} changed eps at {key}"


@pytest.mark.gpu
def test_forced_k1s_fallback_matches(hip, tmp_path):
    """The planner's K1x / K1h plans fall back to K1s 128x128 8-wave tiles with the
    same split count when their 32-bit operand offsets would overflow (sources
    beyond 2^24 pixels or 2 GiB).  CFD_CONV_FORCE_K1S=1 forces that fallback; in
    a fresh process (the switch is read once) the split-f16 and bf16 forwards of
    the config-B width U-Net must agree with the shipped kernels: split-f16 within
    fp32 rounding (1e-5 of max|eps|), bf16 within its own tolerance (1e-2)."""
    import numpy as np
    code = (
        "import ast, sys, torch, numpy as np\n"
        "sys.path.insert(0, 'tests'); sys.path.insert(0, '.')\n"
        "from conftest import golden\n"
        "from confild_amd import synth\n"
        "from confild_amd.script_util import create_model\n"
        "g = golden('unet_cfgB64.npz'); kw = ast.literal_eval(str(g['kwargs']))\n"
        "m = create_model(**kw)\n"
        "sd = synth.unet_state_dict(int(g['seed']), {k: tuple(v.shape) for k, v in m.state_dict().items()})\n"
        "m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}); m.to('cuda')\n"
        "x = torch.from_numpy(synth.normal(8, 'fb', (2, 1, 64, 64))).cuda()\n"
        "t = torch.tensor([999, 300], device='cuda')\n"
        "out = {c: m.set_compute(c)(x, t).cpu().numpy() for c in ('split_f16', 'bf16')}\n"
        "np.savez(sys.argv[1], **out)\n")
    res = {}
    for force in ("0", "1"):
        path = str(tmp_path / f"k1s_fallback_{force}.npz")
        env = dict(os.environ, CFD_CONV_FORCE_K1S=force)
        r = subprocess.run([sys.executable, "-c", code, path], cwd=ROOT, env=env, capture_output=True, text=True,
                           timeout=240)
        assert r.returncode == 0, r.stderr[-3000:]
        res[force] = np.load(path)
    for c, tol in (("split_f16", 1e-5), ("bf16", 1e-2)):
        a, b = res["0"][c], res["1"][c]
        err = float(np.abs(a - b).max() / np.abs(a).max())
        print(f"forced K1s fallback, {c}: {err:.2e}")
        assert err <= tol, (c, err)
