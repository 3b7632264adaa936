"""Decode helpers with the reference signatures (N/cnf/inference_function.py:15-76)."""
from __future__ import annotations

import numpy as np
import torch

from .nf_networks import SIRENAutodecoder_film


def ReconstructFrame(data, mask, shape, fill_value=np.nan):
    """inference_function.py:15-19: scatter masked points back into the full grid (host)."""
    temp = np.empty((*shape, data.shape[-1]))
    temp[:] = fill_value
    temp[mask] = data
    return temp


def _decode(coords, latents, model, x_normalizer, y_normalizer, batch_size, device):
    if not isinstance(model, SIRENAutodecoder_film):
        raise TypeError("model must be confild_amd.nf_networks.SIRENAutodecoder_film (the fused HIP decoder)")
    t_size, latent_size = latents.shape
    device = torch.device(device) if device is not None else latents.device
    lat = latents.to(device)
    outs = []
    # the fused kernel processes every latent of a chunk in one launch; batch_size
    # bounds the (chunk, N, c) output kept live per launch, as in the reference loop
    step = t_size if batch_size is None else max(int(batch_size), 1)
    for s in range(0, t_size, step):
        outs.append(model.decode(coords.reshape(-1, coords.shape[-1]).to(device), lat[s:s + step].reshape(-1, 1,
                                 latent_size), x_normalizer, y_normalizer))
    return outs


def pass_through_model_batch(coords, latents, model, x_normalizer, y_normalizer, batch_size, device):
    """inference_function.py:22-48 -> (t, N, c) on `device`."""
    return torch.cat(_decode(coords, latents, model, x_normalizer, y_normalizer, batch_size, device), dim=0)


def decoder(coords, latents, model, x_normalizer, y_normalizer, batch_size, device):
    """inference_function.py:51-76 -> (t, N, c) on the host."""
    with torch.no_grad():
        outs = _decode(coords, latents, model, x_normalizer, y_normalizer, batch_size, device)
        return torch.cat([o.cpu() for o in outs], dim=0)


class CNF_inference:
    """inference_function.py:79-304: decode the stored training latents of a CNF
    checkpoint (Analysis entry point) on the fused HIP decoder.

    Same constructor, attributes and methods as the reference: the checkpoint,
    its directory's ``normalizer_params.pt``, the YAML's ``NF`` block (with the
    latent width taken from the checkpoint), the ``is_pub`` remap of the
    authors' checkpoints whose ``hidden_states`` is the bare latent tensor
    (:183-205), ``predict`` (:219-259), ``get_all_predictions`` and
    ``create_coordinates_grid``.  Files load with ``weights_only=True``; the data
    file is memory-mapped (only its shape is used).  There is no CPU path:
    ``predict`` on a CPU device raises (the reference silently falls back)."""

    def __init__(self, checkpoint_path, config_path, data_path, device="cuda", is_pub=False):
        import os

        import yaml

        from .normalize import Normalizer_ts
        for path, name in ((checkpoint_path, "checkpoint"), (config_path, "config"), (data_path, "data")):
            if not os.path.exists(path):
                raise FileNotFoundError(f"{name.capitalize()} file not found at {path}")
        self.is_pub = is_pub
        self.device = torch.device(device if torch.cuda.is_available() and device == "cuda" else "cpu")
        self.checkpoint = torch.load(checkpoint_path, map_location="cpu", weights_only=True)
        self.checkpoint_path = checkpoint_path
        with open(config_path, "r") as f:
            self.config = yaml.safe_load(f)
        self.data = np.load(data_path, mmap_mode="r", allow_pickle=False)
        print(f"Data loaded from {data_path}, shape: {self.data.shape}")
        norm_path = f"{os.path.dirname(checkpoint_path)}/normalizer_params.pt"
        if not os.path.exists(norm_path):
            raise FileNotFoundError(f"Normalizer parameters not found at {norm_path}. Cannot proceed with inference.")
        self.norm_params = torch.load(norm_path, map_location="cpu", weights_only=True)
        self.x_normalizer = Normalizer_ts()
        self.y_normalizer = Normalizer_ts()
        self.x_normalizer.params = self.norm_params["x_normalizer_params"]
        self.y_normalizer.params = self.norm_params["y_normalizer_params"]
        self._load_model()

    def _load_model(self):
        """inference_function.py:160-205."""
        from .trainer import LatentContainer
        nf_config = self.config.get("NF", {})
        model_type = nf_config.get("name", "SIRENAutodecoder_film")
        model_params = {k: v for k, v in nf_config.items() if k != "name"}
        if "kwargs" in nf_config:
            model_params = dict(nf_config["kwargs"])
        if model_type != "SIRENAutodecoder_film":
            raise NotImplementedError(f"NF {model_type!r}: only SIRENAutodecoder_film (every CoNFiLD recipe) is on "
                                      "the HIP path")
        hidden = self.checkpoint["hidden_states"]
        latent_params = hidden if self.is_pub else hidden.get("latents")
        if latent_params is None:
            raise ValueError("Could not find latent codes in checkpoint")
        N_samples, N_features = latent_params.shape
        model_params.setdefault("in_latent_features", N_features)
        self.model = SIRENAutodecoder_film(**model_params)
        self.latents = LatentContainer(N_samples=N_samples, N_features=N_features, dims=self.config.get("dims", 2),
                                       lumped=self.config.get("lumped_latent", False))
        self.model.load_state_dict(self.checkpoint["model_state_dict"])
        if self.is_pub:   # the authors' checkpoints store the bare latent tensor
            param_name = list(self.latents.state_dict().keys())[0]
            self.latents.load_state_dict({param_name: hidden})
        else:
            self.latents.load_state_dict(hidden)
        self.model.to(self.device).eval()
        self.latents.to(self.device).eval()

    def predict(self, coords, latent_indices, batch_size=16, normalize=True):
        """inference_function.py:219-259 -> predictions on the host, (n, *coords.shape[:-1], c)."""
        if isinstance(latent_indices, int):
            latent_indices = [latent_indices]
        coords = torch.tensor(coords, dtype=torch.float32) if not isinstance(coords, torch.Tensor) else coords
        coords = coords.to(self.device)
        latent_indices = torch.as_tensor(latent_indices, dtype=torch.long)
        out = []
        with torch.no_grad():
            for i in range(0, len(latent_indices), batch_size):
                z = self.latents(latent_indices[i:i + batch_size].to(self.device))
                if normalize and self.x_normalizer is not None:
                    pred = self.model.decode(coords, z, self.x_normalizer, self.y_normalizer)
                else:
                    pred = self.model(coords, z)
                out.append(pred.cpu())
        return torch.cat(out, dim=0)

    def get_all_predictions(self, coords, batch_size=16, normalize=True):
        return self.predict(coords, torch.arange(self.latents.latents.shape[0]), batch_size, normalize)

    def create_coordinates_grid(self, shape=None):
        """inference_function.py:265-304 (linspace(0, 1) 'ij' grid)."""
        if shape is None:
            spatial = self.data.shape[1:-1] if len(self.data.shape) > 3 else self.data.shape[1:]
            axes = [np.linspace(0, 1, i) for i in spatial]
            return torch.tensor(np.stack(np.meshgrid(*axes, indexing="ij"), axis=-1), dtype=torch.float32)
        if len(shape) not in (2, 3):
            raise ValueError(f"Unsupported shape dimensionality: {shape}")
        axes = [torch.linspace(0, 1, n) for n in shape]
        return torch.stack(torch.meshgrid(*axes, indexing="ij"), dim=-1)
