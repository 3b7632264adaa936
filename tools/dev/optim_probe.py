"""Development probe: which float32 operation order torch's AdamW (single-tensor
and foreach) and update_ema (targ.mul_(rate).add_(src, alpha=1-rate)) run on a
device, against emulations (fma emulated in float64, one rounding).  Used to pin
cfd_adam_step / cfd_ema_update to the reference's arithmetic."""
import sys

import numpy as np
import torch

f, d64 = np.float32, np.float64


def fma(a, b, c):
    return (np.asarray(a, d64) * np.asarray(b, d64) + np.asarray(c, d64)).astype(f)


def probe(dev):
    torch.manual_seed(0)
    n = 1 << 20
    lr, b1, b2, eps, wd = 1e-4, 0.9, 0.999, 1e-8, 0.01
    p0 = torch.randn(n) * 0.05
    for foreach in (False, True):
        p = p0.clone().to(dev).requires_grad_(True)
        opt = torch.optim.AdamW([p], lr=lr, betas=(b1, b2), eps=eps, weight_decay=wd, foreach=foreach)
        P = p0.numpy().copy()
        M = np.zeros(n, f)
        V = np.zeros(n, f)
        for step in range(1, 4):
            g = torch.randn(n) * 1e-2 * step
            p.grad = g.to(dev)
            opt.step()
            G = g.numpy()
            em = opt.state[p]["exp_avg"].cpu().numpy().copy()
            ev = opt.state[p]["exp_avg_sq"].cpu().numpy().copy()
            pp = p.detach().cpu().numpy().copy()
            w1 = f(1 - b1)
            mc = {"fma(w,g-m,m)": fma(w1, (G - M).astype(f), M), "m+w*(g-m)": (M + (w1 * (G - M).astype(f)).astype(f)).astype(f)}
            V1 = (V * f(b2)).astype(f)
            vc = {"fma(val*g,g,V1)": fma((f(1 - b2) * G).astype(f), G, V1),
                  "V1+(val*g)*g": (V1 + ((f(1 - b2) * G).astype(f) * G).astype(f)).astype(f),
                  "fma(val,g*g,V1)": fma(f(1 - b2), (G * G).astype(f), V1)}
            bc1, bc2 = 1 - b1 ** step, 1 - b2 ** step
            sq = np.sqrt(ev.astype(d64)).astype(f)        # correctly rounded
            den = ((sq / f(bc2 ** 0.5)).astype(f) + f(eps)).astype(f)
            Pd = (P * f(1 - lr * wd)).astype(f)
            s = f(-lr / bc1)
            pc = {"Pd+(s*m)/d": (Pd + ((s * em).astype(f) / den).astype(f)).astype(f),
                  "Pd+s*(m/d)": (Pd + (s * (em / den).astype(f)).astype(f)).astype(f),
                  "fma(s,m/d,Pd)": fma(s, (em / den).astype(f), Pd)}
            print(dev, "foreach" if foreach else "single", step,
                  {k: float(np.mean(v == em)) for k, v in mc.items()},
                  {k: float(np.mean(v == ev)) for k, v in vc.items()},
                  {k: float(np.mean(v == pp)) for k, v in pc.items()})
            P, M, V = pp, em, ev
    t = torch.randn(n) * 0.05
    src = torch.randn(n) * 0.05
    rate = 0.9999
    got = t.clone().to(dev).mul_(rate).add_(src.to(dev), alpha=1 - rate).cpu().numpy()
    T, S = t.numpy(), src.numpy()
    tr = (T * f(rate)).astype(f)
    ec = {"fma(src,omr,t*r)": fma(S, f(1 - rate), tr), "t*r+src*omr": (tr + (S * f(1 - rate)).astype(f)).astype(f)}
    print(dev, "ema", {k: float(np.mean(v == got)) for k, v in ec.items()})


if __name__ == "__main__":
    for d in sys.argv[1:] or ["cpu"]:
        probe(torch.device(d))
