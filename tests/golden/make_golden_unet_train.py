"""Golden fixture of the diffusion TrainLoop's step, made by running the
REFERENCE's own objects (build container only; the reference tree does not exist
on the GPU box):

    python tests/golden/make_golden_unet_train.py

``src.train_util.TrainLoop`` itself does not import here (mpi4py and blobfile are
absent), so its ``run_step`` at world size 1, fp32, no
microbatching and the uniform schedule sampler is replayed with the reference's
pieces in its order (U/src/train_util.py:173-240, fp16_util.py
MixedPrecisionTrainer._optimize_normal): ``zero_grad`` ->
``GaussianDiffusion.training_losses`` (U/src/gaussian_diffusion.py:744-853, the
MSE-on-eps term) -> ``(losses["loss"] * weights).mean().backward()`` ->
``torch.optim.AdamW.step()`` -> ``src.nn.update_ema``.  The timesteps and the
noise are recorded (the TrainLoop draws them from numpy's and torch's global
RNGs), the model is the tiny16 fixture U-Net with ``confild_amd.synth`` weights
(regenerated on the GPU box), the batch is stored.

Fixture golden_unettrain.npz: the case, x_start, per-step t and noise, per-step
losses, the first step's gradients, the parameters and the EMA parameters after
the run (each tensor as its float64 sum, its first 256 values and every 29th
value after them).
"""
from __future__ import annotations

import ast
import os
import sys
import types

sys.dont_write_bytecode = True
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [HERE, REPO, REF, os.path.join(REF, "UnconditionalDiffusionTraining_and_Generation")]

_tb = types.ModuleType("torch.utils.tensorboard")
_tb.SummaryWriter = object
sys.modules["torch.utils.tensorboard"] = _tb

import numpy as np  # noqa: E402
import torch  # noqa: E402

from confild_amd import synth  # noqa: E402

CASE = dict(net="tiny16", B=2, steps=2, lr=1e-3, weight_decay=0.01, ema_rate=0.9, schedule="cosine",
            t=[[17, 903], [512, 3]], seed=777)


def main():
    from src.nn import update_ema
    from src.script_util import create_gaussian_diffusion, create_model
    c = CASE
    g = np.load(os.path.join(HERE, f"unet_{c['net']}.npz"))
    kw = ast.literal_eval(str(g["kwargs"]))
    torch.manual_seed(0)
    model = create_model(**kw)
    sd = synth.unet_state_dict(int(g["seed"]), {k: tuple(v.shape) for k, v in model.state_dict().items()})
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    diffusion = create_gaussian_diffusion(steps=1000, noise_schedule=c["schedule"], timestep_respacing="")
    S = kw["image_size"]
    x0 = synth.normal(c["seed"], "utrain/x0", (c["B"], 1, S, S)).astype(np.float32)
    noises = [synth.normal(c["seed"], f"utrain/noise{k}", (c["B"], 1, S, S)).astype(np.float32)
              for k in range(c["steps"])]
    params = list(model.parameters())
    names = [k for k, _ in model.named_parameters()]
    opt = torch.optim.AdamW(params, lr=c["lr"], weight_decay=c["weight_decay"])
    ema = [p.detach().clone() for p in params]
    losses, first = [], None
    model.train()
    for k in range(c["steps"]):
        opt.zero_grad()
        t = torch.tensor(c["t"][k], dtype=torch.int64)
        weights = torch.ones(c["B"])                      # UniformSampler: 1 / (len(p) p[t]) = 1
        terms = diffusion.training_losses(model, torch.from_numpy(x0), t, noise=torch.from_numpy(noises[k]))
        loss = (terms["loss"] * weights).mean()
        loss.backward()
        if first is None:
            first = {"g_" + n: p.grad.detach().numpy().copy() for n, p in zip(names, params)}
        opt.step()
        update_ema(ema, params, rate=c["ema_rate"])
        losses.append(float(loss.detach()))
    final = {"p_" + n: p.detach().numpy().copy() for n, p in zip(names, params)}
    final.update({"e_" + n: e.numpy().copy() for n, e in zip(names, ema)})
    # keep the fixture small: every tensor's sum in float64, its first 256 values and
    # every 29th value after them (the tests compare exactly these)
    def cut(d):
        out = {}
        for k, v in d.items():
            f = v.reshape(-1)
            out[k] = np.concatenate([f[:256], f[256::29]])
            out[k + "__sum"] = np.array(f.astype(np.float64).sum())
        return out
    first, final = cut(first), cut(final)
    path = os.path.join(HERE, "golden_unettrain.npz")
    np.savez_compressed(path, case=np.array(repr(c)), kwargs=g["kwargs"], weight_seed=g["seed"], x0=x0,
                        noise=np.stack(noises), losses=np.array(losses), names=np.array(names),
                        torch_version=np.array(torch.__version__), **first, **final)
    print(f"wrote {path} ({os.path.getsize(path) / 1024:.1f} KiB); losses {losses}")


if __name__ == "__main__":
    main()
