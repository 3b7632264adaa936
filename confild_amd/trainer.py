"""Inference subset of the CNF ``trainer`` (N/scripts/train.py:74-279, 481-528).

Same constructor, ``load`` and ``infer`` as the reference; the training half
(train / _single_trainer / save, :281-479) is out of scope.
``infer`` runs normalise -> SIREN -> de-normalise as ONE fused HIP launch.
"""
from __future__ import annotations

import glob
import os

import numpy as np
import torch

from . import nf_networks
from .normalize import Normalizer_ts


class LatentContainer(torch.nn.Module):
    """train.py:43-63 (holds the stored training latents)."""

    def __init__(self, N_samples, N_features, dims, lumped=False):
        super().__init__()
        self.lumped = lumped
        self.dims = dims
        self.latents = torch.nn.Parameter(torch.zeros((N_samples, N_features), dtype=torch.float32))

    def forward(self, batch_ids):
        z = self.latents[batch_ids]
        extra = 1 if self.lumped else self.dims
        return z.reshape(z.shape[0], *([1] * extra), z.shape[-1])


class trainer:
    def __init__(self, hyper_para, infer_mode=False, infer_dps=False) -> None:
        self.world_size = getattr(hyper_para, "multiGPU", 1)
        self.hyper_para = hyper_para
        self.train_coord = None
        if not infer_mode:
            # default query points (train.py:147-159): coor_path, else a linspace
            # lattice inferred from the data's spatial shape
            if hasattr(hyper_para, "coor_path") and os.path.exists(str(hyper_para.coor_path)):
                coord = np.load(hyper_para.coor_path, allow_pickle=False)
            elif hasattr(hyper_para, "data_path") and os.path.exists(str(hyper_para.data_path)):
                fois = np.load(hyper_para.data_path, mmap_mode="r", allow_pickle=False)
                spatial = fois.shape[1:-1]
                grids = [np.linspace(0, 1, i) for i in spatial]
                coord = np.stack(np.meshgrid(*grids, indexing="ij"), axis=-1)
            else:
                raise FileNotFoundError("infer_mode=False needs coor_path or data_path for the default query points "
                                        "(train.py:147-159)")
            self.train_coord = torch.tensor(coord, dtype=torch.float32)

        self.in_normalizer = Normalizer_ts(**hyper_para.normalizer)
        self.out_normalizer = Normalizer_ts(**hyper_para.normalizer)
        path = f"{hyper_para.save_path}/normalizer_params.pt"
        if os.path.exists(path):
            params = torch.load(path, weights_only=True, map_location="cpu")
            self.in_normalizer.params = params["x_normalizer_params"]
            self.out_normalizer.params = params["y_normalizer_params"]
        else:
            raise FileNotFoundError(f"{path} does not exist")

        nf = hyper_para.NF
        if "kwargs" in nf:
            raise NotImplementedError("NF kwargs form")
        if nf["name"] != "SIRENAutodecoder_film":
            raise NotImplementedError(f"NF {nf['name']!r}: only SIRENAutodecoder_film (every CoNFiLD recipe) "
                                      "is on the HIP path")
        self.nf = nf_networks.SIRENAutodecoder_film(
            in_coord_features=hyper_para.dims, in_latent_features=hyper_para.hidden_size,
            out_features=nf["out_features"], num_hidden_layers=nf["num_hidden_layers"],
            hidden_features=nf["hidden_features"])

    def infer(self, coord, latents):
        """train.py:265-279 -> (b, N, c) (or (b, h, w, c) for grid coordinates)."""
        coord = coord if coord is not None else self.train_coord
        if coord is None:
            raise ValueError("no query coordinates: pass coord (infer_mode=True has no training points)")
        with torch.no_grad():
            return self.nf.decode(coord, latents.reshape(latents.shape[0], -1)[:, None],
                                  self.in_normalizer, self.out_normalizer)

    def load(self, checkpoint_id: int, siren_only=False):
        """train.py:481-528: newest checkpoint_*.pt when checkpoint_id == -1."""
        save = self.hyper_para.save_path
        if checkpoint_id == -1:
            ids = [int(p.split("_")[-1].split(".")[0]) for p in glob.glob(f"{save}/checkpoint_*.pt")]
            if not ids:
                raise FileNotFoundError(f"no checkpoint_*.pt in {save}")
            checkpoint_id = max(ids)
        ckpt = torch.load(f"{save}/checkpoint_{checkpoint_id}.pt", weights_only=True, map_location="cpu")
        self.nf.load_state_dict(ckpt["model_state_dict"])
        self.start_epoch = ckpt["epoch"]
        if not siren_only:
            lat = ckpt["hidden_states"]["latents"]
            self.N_samples = lat.shape[0]
            self.latents = LatentContainer(self.N_samples, self.hyper_para.hidden_size, self.hyper_para.dims,
                                           self.hyper_para.lumped_latent)
            self.latents.load_state_dict(ckpt["hidden_states"])
            self.optim_dict = {k: ckpt[k] for k in ("optim_net_dec_dict", "optim_states_dict") if k in ckpt}
            return self.nf, self.latents, self.optim_dict, ckpt["epoch"]
        self.optim_dict = {"optim_net_dec_dict": ckpt.get("optim_net_dec_dict")}
