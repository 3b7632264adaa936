"""One process per GPU over RCCL ("nccl" backend on ROCm): sharding of the
generation path.

The path shards embarrassingly, so the only collectives are
  * a one-off broadcast of the weights from rank 0 (bucketed: one collective per
    256 MiB of parameters rather than one per tensor), and
  * a gather of the finished results (latents / decoded fields) to rank 0.
There is no per-step collective.

Sharding units
  * diffusion: samples.  Rank r owns samples [B*r/G, B*(r+1)/G) and draws the
    Philox noise of exactly those samples (sample_offset), so the sharded batch
    is bit-identical to the unsharded one;
  * CNF decode: query coordinates.  Rank r owns coordinates [N*r/G, N*(r+1)/G)
    and the matching rows of a per-point output normaliser; every rank decodes
    all latents over its coordinates, the (b, N_r, c) slabs are all-gathered and
    concatenated along N.

Every helper takes the compute as a callable, so the CPU tests (gloo,
world_size 2) exercise the same sharding and collective code with the oracle as
the compute.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

BUCKET_BYTES = 256 << 20


def world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def init_from_env(backend=None):
    """torchrun-style init.  Returns (rank, world_size, device)."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    if ws > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = backend or ("nccl" if device.type == "cuda" else "gloo")
        kw = {"device_id": device} if backend == "nccl" else {}
        dist.init_process_group(backend, rank=rank, world_size=ws, **kw)
    return rank, ws, device


def shard_range(n: int, rank: int, world_size: int):
    """Contiguous, near-even [start, end) of n units for `rank`."""
    return n * rank // world_size, n * (rank + 1) // world_size


@torch.no_grad()
def broadcast_module(module: torch.nn.Module, src: int = 0, group=None):
    """Broadcast every parameter/buffer of `module` from `src`, flattened into
    dtype-homogeneous buckets (one collective per bucket)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return
    tensors = [t for t in list(module.parameters()) + list(module.buffers())]
    bucket, size = [], 0

    def flush():
        nonlocal bucket, size
        if not bucket:
            return
        flat = torch.cat([t.detach().reshape(-1) for t in bucket])
        dist.broadcast(flat, src=src, group=group)
        off = 0
        for t in bucket:
            n = t.numel()
            t.copy_(flat[off:off + n].view_as(t))   # bumps _version: device weight caches re-upload
            off += n
        bucket, size = [], 0

    for t in tensors:
        if bucket and (t.dtype != bucket[0].dtype or size + t.numel() * t.element_size() > BUCKET_BYTES):
            flush()
        bucket.append(t)
        size += t.numel() * t.element_size()
    flush()


def all_gather_cat(x: torch.Tensor, dim: int, sizes, group=None) -> torch.Tensor:
    """Concatenate per-rank tensors of (possibly) different extent along `dim`.
    `sizes[r]` is rank r's extent; slabs are padded to the max for the collective."""
    r, g = dist.get_rank(group), dist.get_world_size(group)
    mx = max(sizes)
    pad = list(x.shape)
    pad[dim] = mx
    buf = torch.zeros(pad, dtype=x.dtype, device=x.device)
    buf.narrow(dim, 0, x.shape[dim]).copy_(x)
    outs = [torch.empty_like(buf) for _ in range(g)]
    dist.all_gather(outs, buf, group=group)
    return torch.cat([o.narrow(dim, 0, sizes[i]) for i, o in enumerate(outs)], dim=dim)


def gather_cat(x: torch.Tensor, dim: int, sizes, dst: int = 0, group=None):
    """Like all_gather_cat but only `dst` receives (and returns) the result.
    Along dim 0 the ranks' slabs land directly in their rows of the result (no
    padding, no concatenation copy); other dims pad to the largest slab."""
    r, g = dist.get_rank(group), dist.get_world_size(group)
    if dim == 0:
        x = x.contiguous()
        if r != dst:
            if x.shape[0]:
                dist.gather(x if x.shape[0] == max(sizes) else _pad0(x, max(sizes)), None, dst=dst, group=group)
            else:
                dist.gather(x.new_zeros((max(sizes),) + tuple(x.shape[1:])), None, dst=dst, group=group)
            return None
        mx = max(sizes)
        if all(sz == mx for sz in sizes):
            out = torch.empty((sum(sizes),) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
            dist.gather(x, list(out.split(sizes)), dst=dst, group=group)
            return out
        outs = [torch.empty((mx,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device) for _ in range(g)]
        dist.gather(_pad0(x, mx), outs, dst=dst, group=group)
        return torch.cat([o[:sizes[i]] for i, o in enumerate(outs)], 0)
    mx = max(sizes)
    pad = list(x.shape)
    pad[dim] = mx
    buf = torch.zeros(pad, dtype=x.dtype, device=x.device)
    buf.narrow(dim, 0, x.shape[dim]).copy_(x)
    outs = [torch.empty_like(buf) for _ in range(g)] if r == dst else None
    dist.gather(buf, outs, dst=dst, group=group)
    if r != dst:
        return None
    return torch.cat([o.narrow(dim, 0, sizes[i]) for i, o in enumerate(outs)], dim=dim)


def _pad0(x, n):
    if x.shape[0] == n:
        return x
    buf = x.new_zeros((n,) + tuple(x.shape[1:]))
    buf[:x.shape[0]].copy_(x)
    return buf


def sharded_decode(decode_fn, coords: torch.Tensor, latents: torch.Tensor, ymax=None, ymin=None, group=None):
    """Coordinate-sharded CNF decode: decode_fn(coords_r, latents, ymax_r, ymin_r)
    -> (b, N_r, c) on each rank; returns the full (b, N, c) on every rank.
    Per-point normaliser tables (1, N, c) are sliced with the coordinates."""
    rank, g = (dist.get_rank(group), dist.get_world_size(group)) if dist.is_initialized() else (0, 1)
    N = coords.shape[0]
    s, e = shard_range(N, rank, g)
    per_point = ymax is not None and ymax.numel() != ymax.shape[-1]
    ym = ymax[..., s:e, :] if per_point else ymax
    yn = ymin[..., s:e, :] if per_point else ymin
    out = decode_fn(coords[s:e], latents, ym, yn)
    if g == 1:
        return out
    sizes = [shard_range(N, r, g)[1] - shard_range(N, r, g)[0] for r in range(g)]
    return all_gather_cat(out, 1, sizes, group)


def sharded_samples(sample_fn, B: int, group=None):
    """Sample-sharded generation: sample_fn(start, count) -> (count, ...) on each
    rank; returns the full (B, ...) batch on every rank (all-gather)."""
    rank, g = (dist.get_rank(group), dist.get_world_size(group)) if dist.is_initialized() else (0, 1)
    if B < g:
        raise ValueError(f"batch of {B} samples cannot be sharded over {g} ranks (every rank needs >= 1 sample)")
    s, e = shard_range(B, rank, g)
    out = sample_fn(s, e - s)
    if g == 1:
        return out
    sizes = [shard_range(B, r, g)[1] - shard_range(B, r, g)[0] for r in range(g)]
    return all_gather_cat(out, 0, sizes, group)
