"""Comparison of a diffusion TrainLoop replay against golden_unettrain.npz (the
reference's own run, tests/golden/make_golden_unet_train.py); shared by the CPU
oracle pin (test_oracle.py) and the GPU parity test (test_gpu_unet_train.py).

The fixture holds every tensor's float64 sum plus its first 256 values and every
29th value after them; ``cut`` takes the same subset of ours.

Tolerances (stated per call):
* losses: step 1 is a forward only (``rtol_loss0``); step 2 runs on the updated
  parameters (``rtol_loss1``);
* first-step gradients: each tensor within ``tol_grad`` of its max |grad| plus
  ``atol_grad`` of the model's largest gradient -- small gradients that are long
  pixel sums with heavy cancellation (the attention GroupNorm gammas, ~3e-3 of
  the largest) carry the absolute rounding level of the fp32-accurate forward
  (measured 1.8e-6 of the largest on the GPU), and gradients that vanish
  analytically are rounding noise on both sides;
* parameters and EMA after the run: the optimiser and the EMA are pinned
  separately and exactly -- cfd_adam_step / cfd_ema_update equal torch.optim.AdamW
  and update_ema bit for bit on the same gradients (tests/test_gpu_optim.py), and
  the GPU TrainLoop test replays them on its own gradients bit for bit -- so what
  this bound covers is only how the first-step gradients' rounding (pinned above
  at ``tol_grad``) propagates through Adam: its first steps move every element
  by about lr * sign(grad), so an element whose gradient is rounding noise can
  move the other way, and the second step's m / sqrt(v) amplifies the relative
  error of small gradients.  Every element within 2 lr steps (1 + wd) of the
  reference, and all but ``frac_loose`` of them within ``tol_param`` (GPU,
  measured: 11.8% of the elements differ by more than 1e-3 lr, 1.7% by 1e-2 lr,
  0.29% by 0.1 lr, 0.05% by 0.5 lr; the CPU oracle is bit-exact).
"""
import numpy as np


def cut(v):
    f = np.asarray(v, dtype=np.float32).reshape(-1)
    return np.concatenate([f[:256], f[256::29]]), float(f.astype(np.float64).sum())


def check(g, case, names, losses, first, final, ema, rtol_loss0, rtol_loss1, tol_grad, atol_grad, tol_param,
          frac_loose):
    report = {}
    assert abs(losses[0] - g["losses"][0]) <= rtol_loss0 * abs(g["losses"][0]), (losses, g["losses"])
    assert abs(losses[1] - g["losses"][1]) <= rtol_loss1 * abs(g["losses"][1]), (losses, g["losses"])
    report["loss_rel"] = [abs(a - b) / abs(b) for a, b in zip(losses, g["losses"])]
    gmax = max(float(np.abs(g["g_" + k]).max()) for k in names)
    errs = []
    for k in names:
        sub, s = cut(first[k])
        ref = g["g_" + k]
        bound = tol_grad * float(np.abs(ref).max()) + atol_grad * gmax
        e = float(np.abs(sub - ref).max()) / bound * tol_grad
        n = np.asarray(first[k]).size
        assert abs(s - float(g["g_" + k + "__sum"])) <= bound * n, (k, s, float(g["g_" + k + "__sum"]))
        errs.append((e, k, float(np.abs(ref).max()) / gmax))
    errs.sort(reverse=True)
    report["grad_worst"] = errs[:4]
    assert errs[0][0] <= tol_grad, (errs[:6], gmax)
    bound = 2 * case["lr"] * case["steps"] * (1 + case["weight_decay"]) + 1e-6
    loose, total, dmax = 0, 0, 0.0
    hist = np.zeros(4, dtype=np.int64)
    for pre, tens in (("p_", final), ("e_", ema)):
        for k in names:
            sub, s = cut(tens[k])
            d = np.abs(sub - g[pre + k])
            dmax = max(dmax, float(d.max()))
            assert d.max() <= bound, (pre + k, float(d.max()), bound)
            loose += int((d > tol_param).sum())
            hist += [(d > th).sum() for th in (1e-6, 1e-5, 1e-4, 5e-4)]
            total += d.size
            n = np.asarray(tens[k]).size
            assert abs(s - float(g[pre + k + "__sum"])) <= bound * n, (pre + k, s)
    report["param_loose_frac"] = loose / total
    report["param_frac_above_1e-6_1e-5_1e-4_5e-4"] = (hist / total).round(5).tolist()
    report["param_dmax"] = dmax
    assert loose <= frac_loose * total, report
    return report
