"""Golden fixture of the CNF autodecoder training loop, made by running the
REFERENCE's own objects (build container only; the reference tree does not
exist on the GPU box):

    python tests/golden/make_golden_train.py

The reference pieces: ``cnf.nf_networks.SIRENAutodecoder_film``,
``scripts.train.LatentContainer`` and ``scripts.train.basic_set`` through a
``torch.utils.data.DataLoader`` (shuffle=False, so the batch order is fixed),
``torch.nn.MSELoss`` and the two ``torch.optim.Adam`` optimisers stepped as
``_single_trainer`` steps them (N/scripts/train.py:385-416: the network once per
epoch from epoch 1 on, on the gradient accumulated over the previous epoch; the
latent table every batch).  Weights come from ``confild_amd.synth`` (regenerated
on the GPU box from the seed), the initial latents, coordinates and targets are
stored.  Same import conventions as make_golden.py (read-only reference,
bytecode writing off, the ``torch.utils.tensorboard`` stand-in).

Fixture golden_cnftrain.npz: inputs, the first backward's gradients (every
parameter and the latent table), the per-batch losses and the parameters and
latents after the run.
"""
from __future__ import annotations

import os
import sys
import types

sys.dont_write_bytecode = True
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [HERE, REPO, REF, os.path.join(REF, "ConditionalNeuralField")]

_tb = types.ModuleType("torch.utils.tensorboard")
_tb.SummaryWriter = object
sys.modules["torch.utils.tensorboard"] = _tb

import numpy as np  # noqa: E402
import torch  # noqa: E402

from confild_amd import synth  # noqa: E402

# the case: SIREN(d, L, c, nh, H), samples x coordinates, batch, epochs, learning rates
CASE = dict(d=3, L=16, c=3, nh=3, H=64, samples=6, N=300, batch=4, epochs=3, lr_nf=1e-3, lr_latents=1e-2,
            seed=4321)


def main():
    from cnf.nf_networks import SIRENAutodecoder_film
    from scripts.train import LatentContainer, basic_set
    from torch.utils.data import DataLoader
    c = CASE
    torch.manual_seed(0)
    model = SIRENAutodecoder_film(c["d"], c["L"], c["c"], c["nh"], c["H"])
    sd = synth.siren_state_dict(c["seed"], c["d"], c["L"], c["c"], c["nh"], c["H"])
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    keys = list(model.state_dict())
    lat0 = synth.normal(c["seed"], "train/latents", (c["samples"], c["L"])).astype(np.float32) * np.float32(0.5)
    coords = synth.uniform(c["seed"], "train/coords", (c["N"], c["d"]), -1.0, 1.0)
    fois = synth.uniform(c["seed"], "train/fois", (c["samples"], c["N"], c["c"]), -1.0, 1.0)
    latents = LatentContainer(c["samples"], c["L"], c["d"], lumped=True)
    latents.latents.data = torch.from_numpy(lat0.copy())
    loader = DataLoader(basic_set(torch.from_numpy(fois), torch.from_numpy(coords)), batch_size=c["batch"],
                        shuffle=False)
    opt_net = torch.optim.Adam(model.parameters(), lr=c["lr_nf"])
    opt_lat = torch.optim.Adam(latents.parameters(), lr=c["lr_latents"])
    crit = torch.nn.MSELoss()
    losses, first, batches = [], None, []
    for i in range(c["epochs"]):                        # train.py:395-416 at world_size 1
        if i != 0:
            opt_net.step()
            opt_net.zero_grad()
        for batch_coords, batch_fois, idx in loader:
            if i == 0:
                batches.append(idx.numpy())
            out = model(batch_coords, latents(idx))
            loss = crit(out, batch_fois)
            opt_lat.zero_grad()
            loss.backward()
            if first is None:
                first = {"g_" + k: p.grad.detach().numpy().copy() for k, p in model.named_parameters()}
                first["g_latents"] = latents.latents.grad.detach().numpy().copy()
            opt_lat.step()
            losses.append(float(loss))
    final = {"p_" + k: v.detach().numpy().copy() for k, v in model.state_dict().items()}
    path = os.path.join(HERE, "golden_cnftrain.npz")
    np.savez_compressed(path, case=np.array(repr(c)), keys=np.array(keys), latents0=lat0, coords=coords, fois=fois,
                        batch_order=np.concatenate(batches), batch_sizes=np.array([len(b) for b in batches]),
                        losses=np.array(losses), latents_final=latents.latents.detach().numpy().copy(),
                        torch_version=np.array(torch.__version__), **first, **final)
    print(f"wrote {path} ({os.path.getsize(path) / 1024:.1f} KiB); losses {losses}")


if __name__ == "__main__":
    main()
