"""CNF autodecoder training on the HIP path: the loop of ``trainer._single_trainer``
(N/scripts/train.py:334-416) with every arithmetic step in the library.

Per epoch ``i``: when ``i != 0`` (and the network is not fixed) the network takes
one Adam step on the gradient it accumulated over the previous epoch's batches
and that gradient is cleared (``optim_net_dec.step(); zero_grad()``); then per
batch of sample indices the latent gradient is cleared, one backward of
``MSELoss(model(coords, latents(idx)), fois[idx])`` runs as
``cfd_siren_train_grad`` (forward with tape, loss gradient, backward through the
SIREN chain, every weight-gradient product, added into the accumulated network
gradient), and the whole latent table takes one Adam step (``optim_states``).
Adam is ``cfd_adam_step`` (torch.optim.Adam's single-tensor update, defaults
betas (0.9, 0.999), eps 1e-8).

Multi-GPU (``world_size > 1``, DistributedDataParallel semantics): every
backward's network and latent gradients are averaged over the ranks (RCCL
all-reduce, ``torch.distributed``) before they are accumulated / stepped, and the
batches come from ``DistributedSampler`` as in the reference.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib


class Adam:
    """torch.optim.Adam (amsgrad off; weight_decay > 0: torch.optim.AdamW) over one
    contiguous fp32 device tensor, stepped by cfd_adam_step."""

    def __init__(self, param, lr, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        if param.dtype != torch.float32 or not param.is_contiguous() or param.device.type != "cuda":
            raise ValueError("Adam needs a contiguous fp32 GPU tensor")
        self.param, self.lr, self.betas, self.eps = param, float(lr), tuple(float(b) for b in betas), float(eps)
        self.weight_decay = float(weight_decay)   # > 0: AdamW's decoupled decay (torch.optim.AdamW)
        self.exp_avg = torch.zeros_like(param)
        self.exp_avg_sq = torch.zeros_like(param)
        self.steps = 0

    def step(self, grad):
        if grad.shape != self.param.shape or grad.dtype != torch.float32 or not grad.is_contiguous():
            raise ValueError("gradient must match the parameter (contiguous fp32)")
        self.steps += 1
        _lib.check(_lib.load().cfd_adam_step(_lib.ptr(self.param), _lib.ptr(grad), _lib.ptr(self.exp_avg),
                                             _lib.ptr(self.exp_avg_sq), self.param.numel(), C.c_double(self.lr),
                                             C.c_double(self.betas[0]), C.c_double(self.betas[1]),
                                             C.c_double(self.eps), C.c_double(self.weight_decay), self.steps,
                                             _lib.stream_of(self.param.device)),
                   "cfd_adam_step")

    def torch_state_dict(self, spans):
        """torch.optim.Adam(W)'s state_dict for the parameters laid out in this flat
        tensor at ``spans`` ((offset, shape) per parameter, in the optimizer's param
        order) -- the file format of the reference's opt checkpoints."""
        state = {}
        if self.steps:
            for i, (o, shp) in enumerate(spans):
                n = 1
                for d in shp:
                    n *= d
                state[i] = {"step": torch.tensor(float(self.steps)),
                            "exp_avg": self.exp_avg[o:o + n].reshape(shp).clone(),
                            "exp_avg_sq": self.exp_avg_sq[o:o + n].reshape(shp).clone()}
        # decoupled_weight_decay: torch >= 2.9 defines AdamW as Adam with it set, and
        # Adam.__setstate__ defaults a missing key to False (L2-coupled decay) -- so
        # the key is written, True for the decoupled update this optimizer runs
        group = {"lr": self.lr, "betas": self.betas, "eps": self.eps, "weight_decay": self.weight_decay,
                 "amsgrad": False, "maximize": False, "foreach": None, "capturable": False,
                 "differentiable": False, "fused": None, "decoupled_weight_decay": self.weight_decay > 0,
                 "params": list(range(len(spans)))}
        return {"state": state, "param_groups": [group]}

    def load_torch_state_dict(self, sd, spans):
        """Inverse of torch_state_dict (a reference opt checkpoint resumes here)."""
        groups = sd["param_groups"]
        if len(groups) != 1 or len(groups[0]["params"]) != len(spans):
            raise ValueError("optimizer state has a different parameter layout")
        g = groups[0]
        wd = float(g.get("weight_decay", 0.0))
        if wd > 0 and not g.get("decoupled_weight_decay", True):
            raise ValueError("optimizer state is L2-coupled Adam (decoupled_weight_decay False); "
                             "cfd_adam_step runs the decoupled (AdamW) update")
        self.lr, self.betas, self.eps = float(g["lr"]), tuple(float(b) for b in g["betas"]), float(g["eps"])
        self.weight_decay = wd
        steps = set()
        for i, (o, shp) in enumerate(spans):
            st = sd["state"].get(i, sd["state"].get(str(i)))
            if st is None:
                steps.add(0)
                continue
            n = 1
            for d in shp:
                n *= d
            for key in ("exp_avg", "exp_avg_sq"):
                if tuple(st[key].shape) != tuple(shp):
                    raise ValueError(f"optimizer state {key} of parameter {i} has shape {tuple(st[key].shape)}, "
                                     f"the parameter {tuple(shp)}")
            self.exp_avg[o:o + n].copy_(st["exp_avg"].reshape(-1))
            self.exp_avg_sq[o:o + n].copy_(st["exp_avg_sq"].reshape(-1))
            steps.add(int(float(st["step"])))
        if len(steps) != 1:
            raise ValueError("per-parameter step counts differ; the flat optimizer keeps one")
        self.steps = steps.pop()


def _batches(n, batch_size, shuffle, world_size, rank, epoch, generator=None):
    """The reference's DataLoader index order: RandomSampler / SequentialSampler
    (world_size 1) or ``DistributedSampler(dataset)`` -- its defaults, shuffle=True
    and seed 0, reshuffled per epoch by ``set_epoch`` (train.py:360-365,398)."""
    from torch.utils.data import BatchSampler, DistributedSampler, RandomSampler, SequentialSampler
    # a DataLoader iterator draws its worker base seed from the RNG first
    # (torch.utils.data.dataloader._BaseDataLoaderIter), then the sampler its own
    torch.empty((), dtype=torch.int64).random_(generator=generator)
    idx = range(n)
    if world_size > 1:
        s = DistributedSampler(idx, num_replicas=world_size, rank=rank)
        s.set_epoch(epoch)
    else:
        s = RandomSampler(idx, generator=generator) if shuffle else SequentialSampler(idx)
    return [list(b) for b in BatchSampler(s, batch_size, drop_last=False)]


def train_autodecoder(model, latents, coords, fois, epochs, batch_size, lr, start_epoch=0, shuffle=True,
                      fix_nf=False, world_size=1, rank=0, coord_chunk=1 << 18, on_batch=None, generator=None):
    """Train ``model`` (confild_amd.nf_networks.SIRENAutodecoder_film, on the GPU)
    and ``latents`` (a trainer.LatentContainer, or its (N_samples, L) table) on
    raw coordinates ``coords`` (N, d) and targets ``fois`` (N_samples, N, c) as
    ``_single_trainer`` does (lr: {"nf": ..., "latents": ...}).  Returns the
    per-epoch mean losses; the parameters and the latent table are updated in
    place.  ``coord_chunk`` bounds the (row, coordinate) pairs of one library call
    (the tape holds (nh+1) x H x 2 floats per pair); the gradients of the chunks
    add up to the batch's."""
    table = latents.latents if hasattr(latents, "latents") else latents
    dev = table.device
    if dev.type != "cuda":
        raise _lib.CfdError("CNF training needs the latents on a GPU")
    Z = table.data
    if Z.dtype != torch.float32 or not Z.is_contiguous():
        raise ValueError("the latent table must be contiguous fp32")
    coords = coords.reshape(-1, model.in_coord_features).to(device=dev, dtype=torch.float32).contiguous()
    fois = fois.to(device=dev, dtype=torch.float32)
    n_samples, N = fois.shape[0], coords.shape[0]
    if fois.shape[1] != N or fois.shape[-1] != model.out_features or Z.shape[0] != n_samples:
        raise ValueError("fois must be (N_samples, N, out_features) against coords (N, d) and the latent table")
    flat = model.flat_params()
    g_net = torch.zeros_like(flat)
    g_step = torch.zeros_like(flat) if world_size > 1 else g_net
    g_lat = torch.zeros_like(Z)
    opt_net = Adam(flat, lr["nf"])
    opt_lat = Adam(Z, lr["latents"])
    sse = torch.zeros(1, dtype=torch.float32, device=dev)
    dist = None
    if world_size > 1:
        import torch.distributed as dist
    epoch_losses = []
    for i in range(start_epoch, start_epoch + epochs):
        if i != 0 and not fix_nf:
            opt_net.step(g_net)                  # optim_net_dec.step(); zero_grad()
            g_net.zero_()
            model.load_flat(flat)
        losses = []
        for idx in _batches(n_samples, batch_size, shuffle, world_size, rank, i, generator):
            rows = torch.as_tensor(idx, dtype=torch.int64, device=dev)
            g_lat.zero_()                        # optim_states.zero_grad()
            if g_step is not g_net:
                g_step.zero_()
            sse.zero_()
            R = len(idx)
            scale = 2.0 / (R * N * model.out_features)
            per = max(1, coord_chunk // R)
            for c0 in range(0, N, per):
                c1 = min(N, c0 + per)
                model.train_grad(coords[c0:c1], Z, rows, fois[rows, c0:c1], scale, g_step, g_lat, sse)
            if dist is not None:                 # DDP: each backward's gradients averaged over the ranks
                dist.all_reduce(g_step)
                g_step.div_(world_size)
                g_net.add_(g_step)
                dist.all_reduce(g_lat)
                g_lat.div_(world_size)
            opt_lat.step(g_lat)
            loss = float(sse) / (R * N * model.out_features)
            losses.append(loss)
            if on_batch is not None:
                on_batch(i, idx, loss)
        epoch_losses.append(sum(losses) / len(losses))
    if not fix_nf:
        model.load_flat(flat)
    model._train_state = {"net_grad": g_net, "net_adam": opt_net, "latent_adam": opt_lat}
    return epoch_losses
