"""Benchmark: CoNFiLD generation on MI355X (BASELINE.json metric: generated
fields/sec, 256-step sample + CNF decode, Case4 latent, 1/2/4/8 GPU).

Default (``--config B``): one step = one pass of BASELINE.json configs[1]:
  * the 256-step DDPM reverse loop (cosine-1000 respaced "256", FIXED_LARGE,
    clip) of the 64x64 latent U-Net (create_model(64, 128 ch, 2 res blocks,
    attention 32,16,8, 64-ch heads): 89.5 M parameters);
  * latent de-normalisation (scripts/inference.py:59-61);
  * CNF decode of every latent row with SIRENAutodecoder_film(3, 64, 3, 15, 384)
    on the 64^3 = 262,144-point lattice (normaliser + per-point de-normaliser
    fused) -> fields of shape (64, 262144, 3) resident in HBM.

Multi-GPU (one process per GPU, torchrun, RCCL = the "nccl" backend), the
north-star design: rank 0 builds the weights and
broadcasts them once (dist.broadcast_module); samples are sharded with the
world-size-invariant Philox stream (sample_offset); every rank decodes the rows
of its own samples; the decoded fields are gathered to rank 0 over xGMI inside
the timed region (``--no-gather`` keeps them on their ranks).
  * ``--scaling weak`` (default): 8 samples per GPU (global batch 8 N);
  * ``--scaling strong``: config B's global batch of 8 split over the ranks
    (1 sample per GPU at N = 8).

``--config C`` (BASELINE.json configs[2]): CNF-only decode of 256 latents x 2^22
uniform coordinates with the Case4 CNF SIREN(3, 384, 3, 15, 384), coordinates
sharded over the ranks (dist.sharded_decode's layout), slabs gathered to rank 0.

Weights and inputs are synthetic and seeded (confild_amd.synth); there is no
network access for checkpoints.  Rank 0 prints ONE JSON line with the driver
contract, a ``roofline`` object for the dominant kernel (the CNF decoder, HIP
events on its stream), a ``roofline_unet`` object for the U-Net forward, and a
``cpu_baseline`` (the oracle on this host's cores, rank 0, N = 1).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

B = 8            # config B samples per batch
S = 64           # latent image (T = L = 64)
STEPS = "256"    # timestep respacing
GRID = 64        # 64^3 lattice
CNF_B = dict(d=3, L=64, c=3, nh=15, H=384)
CNF_C = dict(d=3, L=384, c=3, nh=15, H=384)
C_COORDS = 1 << 22
C_LATENTS = 256
FMA_PEAK_TFLOPS = 157.3    # MI355X fp32 matrix peak (MI355X_MICROARCH.md chip table)
F16_PEAK_TFLOPS = 2500.0   # MI355X dense f16/bf16 matrix peak (same table; no sparsity)
# measured: every SIMD issuing v_mfma_f32_32x32x16_f16 back to back on random
# operands: 1693.5 TFLOP/s f16 at two waves per SIMD (tools/mfma_peak.cpp,
# profiles/r02_mfma_peak.json; zero operands: 2477 at 2.36 GHz) and up to 1809.9
# at one wave per SIMD, one dependent chain or several (tools/mfma_chain.cpp,
# profiles/r02_mfma_chain.json) -- the higher, the decoder's configuration, is
# the ceiling used.  /3 = what a split-f16 kernel can reach on real data at the
# clock the chip holds
F16_SUSTAINED_TFLOPS = 1809.9
UNET_FLOPS_PER_SAMPLE = 68.61e9   # config-B U-Net forward, 2*MAC of conv/bmm/addmm (FlopCounter)
METRIC = "generated fields/sec (256-step sample + CNF decode), Case4 latent, 1/2/4/8 GPU"

# dominant-kernel roofline per decoder compute mode:
#   (kernel name, peak in algorithmic fp32 TFLOP/s, basis, committed PMC record)
ROOFLINE = {
    "split_f16": ("siren_split32", F16_PEAK_TFLOPS / 3,
                  "f16 dense MFMA peak / 3 (three f16 MFMAs per fp32 product)", "r06c_pipe_pmc.json"),
    "f32": ("siren_fused", FMA_PEAK_TFLOPS, "fp32 MFMA peak", "r01_siren_pmc.json"),
}
PIPE_PMC_PAIRS = 8 * S * GRID ** 3     # the r06c record's decodes: config B's 512 latent rows x 64^3
CLOCK_RECORD = "r06d_siren_clock.json"  # tools/dev/siren_clock.py: the decoder's in-kernel clock


def _profile(fname):
    try:
        return json.load(open(os.path.join(ROOT, "profiles", fname)))
    except (OSError, ValueError):
        return None


def measured_traffic(mode, latents, npts, cus=None):
    """Per-launch fabric bytes of the decoder kernel from the committed rocprofv3
    PMC record, scaled from its launch geometry to this one (same SIREN widths).
    split_f16: the HEAD record of the pipelined config-B bench (tools/pipe_pmc.py),
    the dispatches on `cus` CUs (the side-by-side half, or the whole chip)."""
    kname, _, _, fname = ROOFLINE[mode]
    rec = _profile(fname)
    if rec is None:
        return None
    if "decoder_dispatches" in rec:
        ds = [d for d in rec["decoder_dispatches"] if cus is None or d["cus"] == cus] or rec["decoder_dispatches"]
        return sum(d["traffic_bytes"] for d in ds) / len(ds) * (latents * npts) / PIPE_PMC_PAIRS
    launch = rec.get("launch", {})
    ref_pairs = launch.get("latents", 0) * launch.get("coords", 0)
    if not ref_pairs or f"{kname}<" not in rec.get("kernel", ""):
        return None
    return rec["traffic_bytes_per_launch"] * (latents * npts) / ref_pairs


def measured_mfma_util(mode, cus=None):
    """Matrix-pipe busy fraction of the decoder from the committed HEAD PMC record
    (the dispatches on `cus` CUs), and its clock measured inside the kernel
    (s_memtime / s_memrealtime, tools/dev/siren_clock.py) under the same condition."""
    kname, _, _, fname = ROOFLINE[mode]
    rec = _profile(fname)
    if rec is None or "decoder_dispatches" not in rec:
        return None
    ds = [d for d in rec["decoder_dispatches"] if cus is None or d["cus"] == cus] or rec["decoder_dispatches"]
    out = {"mfma_busy_frac": sum(d["mfma_busy_frac"] for d in ds) / len(ds),
           "valu_per_mfma": sum(d["valu_per_mfma"] for d in ds) / len(ds),
           "clock_ghz_grbm": sum(d["clock_ghz_grbm"] for d in ds) / len(ds),
           "source": f"profiles/{fname} (rocprofv3 --pmc passes of bench.py --steps 4, serialised dispatches)"}
    clk = _profile(CLOCK_RECORD)
    if clk:
        cond = "whole" if cus == 256 or cus is None else "piped"
        if cond in clk and clk[cond]:
            out["clock_ghz_in_kernel"] = clk[cond]["clock_ghz_median"]
            out["clock_condition"] = cond
            out["clock_source"] = f"profiles/{CLOCK_RECORD}"
    return out


def siren_flops_per_pair(d, L, c, nh, H):
    return 2 * (d * H + nh * H * H + H * c)


# ---------------------------------------------------------------------------
# distributed plumbing
# ---------------------------------------------------------------------------
def rank_env(n, rank, port):
    """Environment of rank `rank` of an n-rank single-node job (what torchrun sets)."""
    return {"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n),
            "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
            "HSA_ENABLE_IPC_MODE_LEGACY": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0")}


def launch_ranks(n, argv):
    """``bench.py --gpus N`` without a launcher: start N rank processes of this
    script (one per GPU, the torchrun environment) and return the job's exit
    code.  Runs before anything touches HIP in this process (no exec: the ranks
    are children); rank 0's JSON line reaches stdout through the inherited pipe."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    import time
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update(rank_env(n, r, port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    return wait_ranks(procs, time.sleep)


def wait_ranks(procs, sleep):
    """Poll every rank (as torchrun's agent does): the first one to exit non-zero
    ends the job -- the others, which would otherwise sit in a rendezvous or a
    collective until the backend timeout, are terminated (then killed) -- and its
    code is returned; 0 once all have exited cleanly."""
    while True:
        rcs = [p.poll() for p in procs]
        bad = next((rc for rc in rcs if rc not in (None, 0)), None)
        if bad is not None:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=10)
                except Exception:
                    p.kill()
                    p.wait()
            return bad
        if all(rc == 0 for rc in rcs):
            return 0
        sleep(0.2)


def init_dist():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    return rank, world, dev


def barrier(dev, world):
    torch.cuda.synchronize(dev)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        torch.cuda.synchronize(dev)


def max_over_ranks(v, dev, world):
    if world == 1:
        return v
    import torch.distributed as dist
    t = torch.tensor([v], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.item()


def gather_to_root(x, dim, sizes, world):
    """Rank 0 receives every rank's slab concatenated along `dim` (RCCL gather).
    A one-rank job without a process group returns x; with one (the world-size-1
    RCCL test of the pipelined path) the collective runs."""
    import torch.distributed as tdist
    if world == 1 and not (tdist.is_available() and tdist.is_initialized()):
        return x
    from confild_amd import dist as cdist
    return cdist.gather_cat(x, dim, sizes, dst=0)


# ---------------------------------------------------------------------------
# config B: sample -> de-normalise -> decode
# ---------------------------------------------------------------------------
def setup_B(dev, rank, world, siren_compute, unet_compute, plan_batch=0):
    from confild_amd import dist as cdist
    from confild_amd import synth
    from confild_amd.nf_networks import SIRENAutodecoder_film
    from confild_amd.normalize import Normalizer_ts
    from confild_amd.script_util import create_gaussian_diffusion, create_model
    model = create_model(image_size=S, num_channels=128, num_res_blocks=2, num_heads=4, num_head_channels=64,
                         attention_resolutions="32,16,8")
    c = CNF_B
    nf = SIRENAutodecoder_film(c["d"], c["L"], c["c"], c["nh"], c["H"])
    if rank == 0:   # rank 0 owns the "checkpoint"; the others receive it over RCCL
        sd = synth.unet_state_dict(1234, {k: tuple(v.shape) for k, v in model.state_dict().items()})
        model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
        nf.load_state_dict({k: torch.from_numpy(v) for k, v in
                            synth.siren_state_dict(1234, c["d"], c["L"], c["c"], c["nh"], c["H"]).items()})
    model.to(dev)
    nf.to(dev)
    cdist.broadcast_module(model)
    cdist.broadcast_module(nf)
    model.set_compute(unet_compute)
    # the planned batch (cfd_unet_set_plan_batch): 0 = 8, config B's batch per GPU.
    # main() re-plans for the per-GPU sample count when that is below 8 (the same
    # count on every rank, so all ranks tile alike); the strong-scaling point plans
    # for its largest shard -- a stated choice: its samples then differ from the
    # 8-per-GPU plan's by fp32 rounding only (pinned over the whole 256-step loop by
    # tests/test_gpu_cfg.py::test_configB_full_256_step_trajectory[plan1])
    model.set_plan_batch(max(plan_batch, 0))
    nf.set_compute(siren_compute)
    model.prepare(dev)   # weights packed and resident before any timed step
    nf.prepare(dev)
    diff = create_gaussian_diffusion(steps=1000, noise_schedule="cosine", timestep_respacing=STEPS)
    ax = torch.linspace(0, 1, GRID)
    coords = torch.stack(torch.meshgrid(ax, ax, ax, indexing="ij"), -1).reshape(-1, 3).to(dev)
    N = coords.shape[0]
    xn = Normalizer_ts(params=(torch.ones(1, 3, device=dev), torch.zeros(1, 3, device=dev)), method="-11", dim=0)
    ymax = torch.from_numpy(synth.uniform(9, "ymax", (1, N, 3), 0.5, 2.0)).to(dev)
    ymin = -torch.from_numpy(synth.uniform(9, "ymin", (1, N, 3), 0.5, 2.0)).to(dev)
    yn = Normalizer_ts(params=(ymax, ymin), method="-11", dim=0)
    vmax = torch.full((1,), 1.5, device=dev)
    vmin = torch.full((1,), -1.5, device=dev)
    return dict(model=model, diff=diff, nf=nf, coords=coords, xn=xn, yn=yn, vmax=vmax, vmin=vmin)


def sample_B(o, dev, seed, start, count):
    """This rank's samples of one batch: the 256-step loop, then de-normalised."""
    from confild_amd import _lib
    lat = o["diff"].p_sample_loop(o["model"], (count, 1, S, S), seed=seed, sample_offset=start)[:, 0]
    den = torch.empty_like(lat)
    _lib.check(_lib.load().cfd_latent_denorm(_lib.ptr(lat), _lib.ptr(den), lat.numel(), _lib.ptr(o["vmax"]),
                                             _lib.ptr(o["vmin"]), 1, _lib.stream_of(dev)), "denorm")
    return den


class PipelineB:
    """Config B as a two-stage pipeline over the chip's two CU halves
    (cfd_stream_create_cu_range): the decode of batch k-1 runs on one half while
    batch k is sampled on the other; the first batch samples on the whole chip.
    Every batch is sampled and decoded exactly once inside the timed region (no
    work moves out of it); only the order of independent batches overlaps.

    The sampler finishes its batch first (round 5: 1.6 s against the decode's
    2.2 s per batch on 128 + 128 CUs), so the decode of batch k-1 is split by
    latent rows: rows [0, n1) on the decode half beside the sampling, rows
    [n1, R) on the sampling half right after it, written into one (R, N, c)
    tensor.  n1 is re-balanced from the measured rates of the batch before last
    so that both halves finish together.  A row's fields are the same bits
    whichever launch decodes it (one workgroup = one latent row x 128 coordinates;
    tests/test_gpu_pipeline.py)."""

    def __init__(self, o, dev, start, count, sizes, world, gather, sample_cus=None, split=True):
        from confild_amd.streams import CuRangeStream, cu_count
        n = cu_count(dev)
        # CUs of the sampling stream: half the chip, three quarters where the decode is
        # small (<= 2 samples per batch: the 8-GPU strong share; 128 / 160 / 192 / 224
        # CUs measured 709 / 697 / 692 / 745 ms per one-sample batch, profiles/r06u_*)
        if sample_cus is None:
            h = n * 3 // 4 if count * S <= 128 else n // 2
        else:
            h = int(sample_cus)
        self.su = CuRangeStream(dev, 0, h)
        self.sd = CuRangeStream(dev, h, n - h)
        self.cus = (h, n - h)
        self.cu_share = (n - h) / n
        self.o, self.dev, self.start, self.count = o, dev, start, count
        self.sizes, self.world, self.gather = sizes, world, gather
        self.R = count * S
        self.split = split
        self.n1 = self.R if not split else self._rows(0.86 * self.R)
        self.hist = []        # per side-by-side batch: (sampling events, part-B events, n1, part-A events)
        # the gather of a finished batch waits for both halves' parts on a stream of
        # its own (an unmasked, non-default stream), so neither half waits for the other
        self.sg = torch.cuda.Stream(dev) if gather else None

    def _rows(self, x):
        return int(max(self.R // 2, min(self.R, round(x / 8) * 8)))

    def _rebalance(self):
        """n1 for the next batch from a finished one: the rows the decode half
        covers in the time the sampling half takes to sample and decode the rest."""
        if len(self.hist) < 2:
            return
        (u0, u1), (d0, d1), n1, pa = self.hist[-2]
        if pa is None or not all(e.query() for e in (u1, d1, pa[1])):
            return
        ts, tb, ta = u0.elapsed_time(u1), d0.elapsed_time(d1), pa[0].elapsed_time(pa[1])
        n2 = self.R - n1
        if tb <= 0 or ta <= 0 or n2 <= 0:
            return
        rb, ra = n1 / tb, n2 / ta
        self.n1 = self._rows((ts + self.R / ra) / (1 / rb + 1 / ra))

    def _decode_rows(self, den, full, r0, r1, stream):
        with torch.cuda.stream(stream):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            self.o["nf"].decode(self.o["coords"], den.reshape(self.R, 1, S)[r0:r1], self.o["xn"], self.o["yn"],
                                out=full[r0:r1])
            e1.record()
        den.record_stream(stream)
        return e0, e1

    def _finish(self, full, events):
        """The gather of a batch once every part of it is written (multi-GPU)."""
        if not self.gather:
            return full
        for e in events:
            self.sg.wait_event(e)
        with torch.cuda.stream(self.sg):
            f = gather_to_root(full, 0, self.sizes, self.world)   # RCCL on the gather stream
        return f

    def run(self, seeds, keep=None):
        """Samples and decodes one batch per seed; returns (sampling events,
        the side-by-side decode-half parts' events, the last batch's fields).
        `keep` (a list, tests): every batch's fields are appended to it in seed
        order.  self.rows_b: the rows of each side-by-side decode-half part."""
        # nothing is enqueued on the default stream between the first sample and the
        # end: it is the legacy NULL stream, and any operation on it orders every
        # blocking stream behind it (a wait there serialised the two halves)
        main = torch.cuda.current_stream(self.dev)
        nf, coords = self.o["nf"], self.o["coords"]
        evu, evd, pend, out = [], [], None, None
        self.rows_b = []
        # every batch's field tensor stays referenced until the run has ended (the
        # two halves write its parts; main waits for both before returning), so
        # no block is re-used while a part is still being written -- and none is
        # tied to the CU-masked streams, which close() destroys
        self._live = []
        for i, seed in enumerate(seeds):
            if pend is not None:
                den, ready = pend
                full = torch.empty((self.R, coords.shape[0], nf.out_features), dtype=torch.float32, device=self.dev)
                self._live.append(full)
                n1 = self.n1
                self.sd.stream.wait_event(ready)
                eb = self._decode_rows(den, full, 0, n1, self.sd.stream)
                evd.append(eb)
                self.rows_b.append(n1)
                self.su.stream.wait_event(ready)   # the sampler's buffers: one batch at a time
            with torch.cuda.stream(main if i == 0 else self.su.stream):
                u0, u1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                u0.record()
                den_next = sample_B(self.o, self.dev, seed, self.start, self.count)
                u1.record()
            evu.append((u0, u1))
            if pend is not None:
                ea = self._decode_rows(den, full, n1, self.R, self.su.stream) if n1 < self.R else None
                self.hist.append(((u0, u1), eb, n1, ea))
                out = self._finish(full, [eb[1]] + ([ea[1]] if ea else []))
                if keep is not None:
                    keep.append(out)
                if self.split:
                    self._rebalance()
            pend = (den_next, u1)
        # the last batch: its decode on the whole chip once both halves are done
        main.wait_stream(self.su.stream)
        main.wait_stream(self.sd.stream)
        if self.sg is not None:
            main.wait_stream(self.sg)
        den, ready = pend
        full = torch.empty((self.R, coords.shape[0], nf.out_features), dtype=torch.float32, device=self.dev)
        with torch.cuda.stream(main):
            nf.decode(coords, den.reshape(self.R, 1, S), self.o["xn"], self.o["yn"], out=full)
            out = gather_to_root(full, 0, self.sizes, self.world) if self.gather else full
        if keep is not None:
            keep.append(out)
        self._live = [] if keep is None else self._live   # main has waited for both halves
        return evu, evd, out

    def close(self):
        self.su.close()
        self.sd.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False


def step_B(o, dev, seed, start, count, ev=None):
    """This rank's samples [start, start+count) of one batch: sample -> de-normalise
    -> decode.  Returns fields (count*T, N, c).  ev: 3 events (U-Net start,
    decode start, decode end)."""
    from confild_amd import _lib
    if ev is not None:
        ev[0].record()
    lat = o["diff"].p_sample_loop(o["model"], (count, 1, S, S), seed=seed, sample_offset=start)[:, 0]
    den = torch.empty_like(lat)
    _lib.check(_lib.load().cfd_latent_denorm(_lib.ptr(lat), _lib.ptr(den), lat.numel(), _lib.ptr(o["vmax"]),
                                             _lib.ptr(o["vmin"]), 1, _lib.stream_of(dev)), "denorm")
    if ev is not None:
        ev[1].record()
    fields = o["nf"].decode(o["coords"], den.reshape(count * S, 1, S), o["xn"], o["yn"])
    if ev is not None:
        ev[2].record()
    return fields


# ---------------------------------------------------------------------------
# configs A and E (BASELINE.json configs[0] / configs[4]): the same sample ->
# de-normalise -> decode chain at their own shapes, samples sharded like B (weak)
#   A: Case1 uncond, U-Net 32^2 (channel_mult 1,2,3,4), DDIM-50, SIREN(2,32,3,10,128)
#      on 1000 coordinates, B = 1 per GPU (the reference's CPU-runnable case)
#   E: Case3, U-Net 128^2 with bf16 convolution operands (fp32 accumulate), DDPM
#      1000 steps, SIREN(2,128,2,17,256) on a 256^2 lattice, B = 8 per GPU (64 on 8)
# ---------------------------------------------------------------------------
UNCOND_CFG = {
    "A": dict(size=32, channel_mult="1,2,3,4", respacing="ddim50", ddim=True, batch=1,
              siren=dict(d=2, L=32, c=3, nh=10, H=128), coords=1000, unet="split_f16",
              gflops=19.23, plan_batch=1),   # one sample per GPU: planned for 1 (pinned by test_gpu_cfg.py)
    "E": dict(size=128, channel_mult="", respacing="", ddim=False, batch=8,
              siren=dict(d=2, L=128, c=2, nh=17, H=256), coords=256 * 256, unet="bf16",
              gflops=140.75, plan_batch=0),
}


def main_uncond(args, rank, world, dev):
    from confild_amd import _lib
    from confild_amd import dist as cdist
    from confild_amd import synth
    from confild_amd.nf_networks import SIRENAutodecoder_film
    from confild_amd.normalize import Normalizer_ts
    from confild_amd.script_util import create_gaussian_diffusion, create_model
    c = UNCOND_CFG[args.config]
    Sz, sc = c["size"], c["siren"]
    model = create_model(image_size=Sz, num_channels=128, num_res_blocks=2, num_heads=4, num_head_channels=64,
                         attention_resolutions="32,16,8", channel_mult=c["channel_mult"])
    nf = SIRENAutodecoder_film(sc["d"], sc["L"], sc["c"], sc["nh"], sc["H"])
    if rank == 0:
        sd = synth.unet_state_dict(1234, {k: tuple(v.shape) for k, v in model.state_dict().items()})
        model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
        nf.load_state_dict({k: torch.from_numpy(v) for k, v in
                            synth.siren_state_dict(1234, sc["d"], sc["L"], sc["c"], sc["nh"], sc["H"]).items()})
    model.to(dev)
    nf.to(dev)
    cdist.broadcast_module(model)
    cdist.broadcast_module(nf)
    model.set_compute(c["unet"] if args.unet_compute == "split_f16" else args.unet_compute)
    model.set_plan_batch(c["plan_batch"] if args.plan_batch < 0 else args.plan_batch)
    nf.set_compute(args.siren_compute)
    # weights packed and resident before any timed step (with --warmup 0 the first
    # timed forward would otherwise pay the host-side packing)
    model.prepare(dev)
    nf.prepare(dev)
    diff = create_gaussian_diffusion(steps=1000, noise_schedule="cosine", timestep_respacing=c["respacing"])
    nsteps = diff.num_timesteps
    if args.config == "E":
        ax = torch.linspace(0, 1, 256)
        coords = torch.stack(torch.meshgrid(ax, ax, indexing="ij"), -1).reshape(-1, 2).to(dev)
    else:
        coords = torch.from_numpy(synth.uniform(7, "A/coords", (c["coords"], 2), 0.0, 1.0)).to(dev)
    N = coords.shape[0]
    xn = Normalizer_ts(params=(torch.ones(1, 2, device=dev), torch.zeros(1, 2, device=dev)), method="-11", dim=0)
    ymax = torch.from_numpy(synth.uniform(9, "ymax", (1, N, sc["c"]), 0.5, 2.0)).to(dev)
    ymin = -torch.from_numpy(synth.uniform(9, "ymin", (1, N, sc["c"]), 0.5, 2.0)).to(dev)
    yn = Normalizer_ts(params=(ymax, ymin), method="-11", dim=0)
    vmax, vmin = torch.full((1,), 1.5, device=dev), torch.full((1,), -1.5, device=dev)
    batch = args.batch or c["batch"]
    glob = batch * world
    start = rank * batch
    sizes = [batch * Sz] * world

    def one(k, ev=None):
        if ev is not None:
            ev[0].record()
        loop = diff.ddim_sample_loop if c["ddim"] else diff.p_sample_loop
        lat = loop(model, (batch, 1, Sz, Sz), seed=10 ** 6 + k, sample_offset=start)[:, 0]
        den = torch.empty_like(lat)
        _lib.check(_lib.load().cfd_latent_denorm(_lib.ptr(lat), _lib.ptr(den), lat.numel(), _lib.ptr(vmax),
                                                 _lib.ptr(vmin), 1, _lib.stream_of(dev)), "denorm")
        if ev is not None:
            ev[1].record()
        f = nf.decode(coords, den.reshape(batch * Sz, 1, Sz), xn, yn)
        if ev is not None:
            ev[2].record()
        return gather_to_root(f, 0, sizes, world) if world > 1 and not args.no_gather else f

    for w in range(args.warmup):
        one(-1 - w)
    barrier(dev, world)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        out = one(k, evs[k])
    barrier(dev, world)
    elapsed = max_over_ranks(time.perf_counter() - t0, dev, world)
    unet_ms = float(np.mean([ev[0].elapsed_time(ev[1]) for ev in evs]))
    dec_ms = float(np.mean([ev[1].elapsed_time(ev[2]) for ev in evs]))
    model.check_finite(dev)
    if rank == 0:
        assert torch.isfinite(out).all().item(), "non-finite output"
        mode = nf.compute_mode(dev)
        kname, peak, peak_basis, _ = ROOFLINE[mode]
        flops = batch * Sz * N * siren_flops_per_pair(**sc)
        uf = batch * c["gflops"] * 1e9 * nsteps
        ua = uf / (unet_ms / 1e3) / 1e12
        upeak = F16_PEAK_TFLOPS if model.compute == "bf16" else F16_PEAK_TFLOPS / 3
        rec = {"metric": METRIC.replace("256-step", f"{nsteps}-step").replace("Case4", "Case1" if args.config == "A"
                                                                               else "Case3"),
               "value": glob * args.steps / elapsed, "unit": "fields/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": "bf16" if model.compute == "bf16" else "f32",
               "data": "synthetic (seeded weights and inputs; no checkpoints)",
               "compute": {"unet": model.compute, "cnf_decoder": mode},
               "config": {"workload": (f"config {args.config}: U-Net {Sz}x{Sz} (channel_mult "
                                       f"{c['channel_mult'] or 'default'}), {'DDIM-50' if c['ddim'] else 'DDPM'} "
                                       f"{nsteps} steps, {batch}/GPU, CNF SIREN({sc['d']},{sc['L']},{sc['c']},"
                                       f"{sc['nh']},{sc['H']}) decode of {Sz} latent rows per sample on {N} coords"),
                          "global_batch": glob, "seq_len": Sz, "parallelism": f"dp{world} ({batch} samples per GPU)",
                          "plan_batch": model.plan_batch or 8},
               "roofline": {"bound": "mfma", "kernel": f"{kname} (+siren_film)",
                            "achieved": flops / (dec_ms / 1e3) / 1e12, "peak": peak, "peak_basis": peak_basis,
                            "unit": "TFLOP/s", "frac": flops / (dec_ms / 1e3) / 1e12 / peak, "traffic": None,
                            "flops_per_launch": flops, "launch_ms": dec_ms},
               "roofline_unet": {"bound": "mfma", "kernel": f"U-Net forward x {nsteps} steps (all kernels + step)",
                                 "achieved": ua, "peak": upeak,
                                 "peak_basis": "bf16 dense MFMA peak" if model.compute == "bf16" else
                                 "f16 dense MFMA peak / 3 (split-f16 convolutions)",
                                 "unit": "TFLOP/s", "frac": ua / upeak, "flops": uf, "ms": unet_ms,
                                 "ms_per_forward": unet_ms / nsteps},
               "cpu_baseline": None if args.no_cpu_baseline or world > 1 else cpu_baseline(args.config),
               "rccl_ranks": world}
        print(json.dumps(rec), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


# ---------------------------------------------------------------------------
# config C: coordinate-sharded CNF-only decode
# ---------------------------------------------------------------------------
def setup_C(dev, rank, world, siren_compute):
    from confild_amd import dist as cdist
    from confild_amd import synth
    from confild_amd.nf_networks import SIRENAutodecoder_film
    from confild_amd.normalize import Normalizer_ts
    c = CNF_C
    nf = SIRENAutodecoder_film(c["d"], c["L"], c["c"], c["nh"], c["H"])
    if rank == 0:
        nf.load_state_dict({k: torch.from_numpy(v) for k, v in
                            synth.siren_state_dict(1234, c["d"], c["L"], c["c"], c["nh"], c["H"]).items()})
    nf.to(dev)
    cdist.broadcast_module(nf)
    nf.set_compute(siren_compute)
    nf.prepare(dev)
    coords, lat, ymax, ymin, (s, e) = c_inputs(rank, world, C_COORDS, C_LATENTS, c["L"])
    lat = lat.to(dev)
    if world > 1:   # latents travel from rank 0 (the sampler's output in a full pipeline)
        import torch.distributed as dist
        dist.broadcast(lat, src=0)
    xn = Normalizer_ts(params=(torch.ones(1, 3, device=dev), torch.zeros(1, 3, device=dev)), method="-11", dim=0)
    yn = Normalizer_ts(params=(ymax.to(dev), ymin.to(dev)), method="-11", dim=0)
    return dict(nf=nf, coords=coords.to(dev), lat=lat[:, None], xn=xn, yn=yn, shard=(s, e))


def c_inputs(rank, world, n_coords, n_latents, L):
    """Config C inputs of one rank: its contiguous coordinate shard with the
    matching rows of the per-point output normaliser, and all latents.  The
    counter-based stream makes every shard independent of the rank count."""
    from confild_amd import dist as cdist
    from confild_amd import synth
    s, e = cdist.shard_range(n_coords, rank, world)
    coords = torch.from_numpy(synth.uniform(7, "C/coords", (n_coords, 3), 0.0, 1.0)[s:e])
    lat = torch.from_numpy(synth.normal(11, "C/latents", (n_latents, L)) * np.float32(0.5))
    ymax = torch.from_numpy(synth.uniform(9, "C/ymax", (1, n_coords, 3), 0.5, 2.0)[:, s:e])
    ymin = -torch.from_numpy(synth.uniform(9, "C/ymin", (1, n_coords, 3), 0.5, 2.0)[:, s:e])
    return coords, lat, ymax, ymin, (s, e)


def b_shards(scaling, world, per_gpu=B):
    """Config B sample shards [(start, count)] per rank: `per_gpu` (default 8) per
    GPU (weak) or the global batch of 8 split (strong)."""
    from confild_amd import dist as cdist
    glob = per_gpu * world if scaling == "weak" else B
    if glob < world:
        raise ValueError(f"strong scaling needs a global batch >= world size ({glob} < {world})")
    return [(cdist.shard_range(glob, r, world)[0],
             cdist.shard_range(glob, r, world)[1] - cdist.shard_range(glob, r, world)[0]) for r in range(world)]


# ---------------------------------------------------------------------------
# config D (guided DPS loop at the config-B widths) and the real Case4 notebook
# shapes (384^2 latent, channel_mult 1,1,2,2,4,4, SIREN(3,384,3,15,384), 1000 steps)
# ---------------------------------------------------------------------------
DPS_CFG = {
    "D": dict(size=64, channel_mult="", siren=(3, 64, 3, 15, 384), respacing="256", batch=8, plan_batch=0),
    # plan_batch: the batch the convolution planner tiles for (cfd_unet_set_plan_batch;
    # 0 = 8).  One chain per GPU at 384^2: 2 (measured r05o, 30 steps, same box:
    # 8 -> 50.2, 1 -> 53.5, 2 -> 54.9, 4 -> 54.7 it/s)
    "Case4": dict(size=384, channel_mult="1, 1, 2, 2, 4, 4", siren=(3, 384, 3, 15, 384), respacing="",
                  batch=1, plan_batch=2),
}


def setup_dps(dev, rank, world, which, batch, plan_batch=-1):
    """The notebook's objects (inference_phy_random_sensor.ipynb cells 11-20) with
    synthetic weights: guided create_model, a Case4 operator with 10 sensors, 'ps'
    conditioning (scale 1, sigma 0), the 'ddpm' sampler."""
    import functools
    from confild_amd import dist as cdist
    from confild_amd import synth
    from confild_amd.guided.condition_methods import get_conditioning_method
    from confild_amd.guided.gaussian_diffusion import create_sampler
    from confild_amd.guided.measurements import Case4Operator, get_noise
    from confild_amd.guided.unet import create_model as guided_model
    from confild_amd.nf_networks import SIRENAutodecoder_film
    from confild_amd.normalize import Normalizer_ts
    c = DPS_CFG[which]
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")   # no model_path: weights are set (or broadcast) below
        m = guided_model(image_size=c["size"], num_channels=128, num_res_blocks=2, channel_mult=c["channel_mult"],
                         num_heads=4, num_head_channels=64, attention_resolutions="32,16,8")
    d, L, co, nh, H = c["siren"]
    nf = SIRENAutodecoder_film(d, L, co, nh, H)
    if rank == 0:
        m.load_state_dict({k: torch.from_numpy(v) for k, v in
                           synth.unet_state_dict(1234, {k: tuple(v.shape) for k, v in m.state_dict().items()}).items()})
        nf.load_state_dict({k: torch.from_numpy(v) for k, v in synth.siren_state_dict(1234, d, L, co, nh, H).items()})
    m.set_plan_batch(c["plan_batch"] if plan_batch < 0 else plan_batch)
    m.to(dev)
    nf.to(dev)
    cdist.broadcast_module(m)
    cdist.broadcast_module(nf)
    m.prepare(dev)
    nf.prepare(dev)
    ns = 10
    coords = torch.from_numpy(synth.uniform(5, "dps/sensors", (ns, d), 0.0, 1.0))
    xn = Normalizer_ts(params=(torch.ones(1, d), torch.zeros(1, d)), method="-11", dim=0)
    yn = Normalizer_ts(params=(torch.full((co,), 2.0), torch.full((co,), -2.0)), method="-11", dim=0)
    op = Case4Operator.from_parts(dev, coords, xn, yn, nf, torch.full((L,), 1.5), torch.full((L,), -1.5),
                                  batch_size=384)
    cond = get_conditioning_method(operator=op, noiser=get_noise(sigma=0.0, name="gaussian"), name="ps", scale=1.0)
    smp = create_sampler(sampler="ddpm", steps=1000, noise_schedule="cosine", model_mean_type="epsilon",
                         model_var_type="fixed_large", dynamic_threshold=False, clip_denoised=True,
                         rescale_timesteps=False, timestep_respacing=c["respacing"])
    # the measurement: the operator applied to a fixed latent
    S = c["size"]
    x_true = torch.from_numpy(synth.uniform(6, "dps/xtrue", (1, 1, S, L), -0.9, 0.9)).to(dev)
    y = op.forward(x_true)
    return dict(model=m, op=op, cond=cond, sampler=smp, fn=functools.partial(cond.conditioning), y=y, S=S, L=L)


# ---------------------------------------------------------------------------
# CPU baseline (oracle on this host's cores)
# ---------------------------------------------------------------------------
def _cpu_info():
    model = platform.processor() or "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    try:   # cgroup v2 CPU share of this process
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = max(1, int(int(q) / int(p)))
    except (OSError, ValueError):
        pass
    tpc = 1
    try:
        sib = open("/sys/devices/system/cpu/cpu0/topology/thread_siblings_list").read().strip()
        tpc = len([x for part in sib.split(",") for x in
                   (range(int(part.split("-")[0]), int(part.split("-")[1]) + 1) if "-" in part else [part])])
    except (OSError, ValueError):
        pass
    physical = max(1, aff // tpc)
    threads = min(physical, quota) if quota else physical
    return dict(cpu_model=model, affinity_cpus=aff, threads_per_core=tpc, cgroup_cpu_quota=quota), threads


def _time_loop(fn, n_min, budget_s):
    fn()  # warm
    t0 = time.perf_counter()
    n = 0
    while n < n_min or (time.perf_counter() - t0 < budget_s and n < 2 * n_min):
        fn()
        n += 1
    return (time.perf_counter() - t0) / n, n


def _unet_oracle(size, mult):
    from confild_amd import synth
    from oracle import unet as ou
    cfg = ou.Config(image_size=size, num_channels=128, num_res_blocks=2, num_heads=4, num_head_channels=64,
                    attention_resolutions="32,16,8", channel_mult=mult)
    sd = {k: torch.from_numpy(v) for k, v in synth.unet_state_dict(1234, ou.param_shapes(cfg)).items()}
    return cfg, sd


def _siren_oracle(c):
    from confild_amd import synth
    return {k: torch.from_numpy(v) for k, v in synth.siren_state_dict(1234, c["d"], c["L"], c["c"], c["nh"],
                                                                      c["H"]).items()}


def _decode_rate(c, npts, nl):
    """Seconds per (coordinate, latent) pair of the oracle decode, one chunk."""
    from oracle import siren as osn
    ssd = _siren_oracle(c)
    d = c["d"]
    coords = torch.rand(npts, d)
    lat = torch.randn(nl, c["L"])
    one, mone = torch.ones(1, d), -torch.ones(1, c["c"])
    with torch.no_grad():
        osn.decode(ssd, coords[:1024], lat[:1], one, torch.zeros(1, d), torch.ones(1, c["c"]), mone)
        t0 = time.perf_counter()
        osn.decode(ssd, coords, lat, one, torch.zeros(1, d), torch.ones(1, c["c"]), mone)
        dec_s = time.perf_counter() - t0
    return dec_s / (npts * nl), dec_s, npts * nl


def cpu_baseline(config):
    """The oracle (torch CPU restatement of the reference path, the same aten ops
    in the same order) on all physical cores this process may use (SURVEY 8d,
    BASELINE.md section 3), on a bounded sample of the line's workload:
      A      the whole DDIM-50 loop + de-normalisation + decode, end to end, best of 3;
      B / E  8 (B) / 2 (E) U-Net forwards at B = 8 and one decode chunk, extrapolated
             linearly (the per-step and per-pair costs are constant);
      C      one decode chunk of 2^20 pairs, extrapolated;
      D / Case4  k guided steps of one chain (U-Net forward + autograd through the
             Case4 operator and the U-Net), extrapolated to it/s.
    The measured parts and the extrapolation are separate fields."""
    from confild_amd import synth
    from oracle import diffusion as od
    from oracle import unet as ou
    info, threads = _cpu_info()
    torch.set_num_threads(threads)
    out = {"unit": "fields/s", "cores": threads, "kind": "port", "torch": torch.__version__, **info}
    if config == "A":
        c = UNCOND_CFG["A"]
        cfg, sd = _unet_oracle(c["size"], c["channel_mult"])
        ssd = _siren_oracle(c["siren"])
        from oracle import siren as osn
        tb = od.Tables(1000, "cosine", c["respacing"])
        Sz, sc = c["size"], c["siren"]
        coords = torch.from_numpy(synth.uniform(7, "A/coords", (c["coords"], 2), 0.0, 1.0))
        ymax = torch.from_numpy(synth.uniform(9, "ymax", (1, c["coords"], sc["c"]), 0.5, 2.0))
        ymin = -torch.from_numpy(synth.uniform(9, "ymin", (1, c["coords"], sc["c"]), 0.5, 2.0))

        def run():
            g = torch.Generator().manual_seed(42)
            x0 = torch.randn(1, 1, Sz, Sz, generator=g)
            noise = [torch.randn(1, 1, Sz, Sz, generator=g) for _ in range(tb.num_timesteps)]
            with torch.no_grad():
                lat, _ = od.sample_loop(tb, lambda x, t: ou.forward(sd, cfg, x, t), x0, noise, kind="ddim")
                den = (lat[:, 0] + 1) * (1.5 - -1.5) / 2 + -1.5
                return osn.decode(ssd, coords, den.reshape(Sz, Sz), torch.ones(1, 2), torch.zeros(1, 2), ymax, ymin)
        times = []
        for _ in range(3):
            t0 = time.perf_counter()
            f = run()
            times.append(time.perf_counter() - t0)
        assert torch.isfinite(f).all()
        out["measured"] = {"end_to_end_s": times, "best_s": min(times)}
        out["value"] = 1.0 / min(times)
        out["sample"] = (f"oracle on {threads} threads: the whole config-A pipeline (DDIM-50 at 32^2 B=1, "
                         f"de-normalisation, decode of 32 rows x 1000 coords), best of 3, no extrapolation")
        return out
    if config in ("D", "Case4"):
        from confild_amd.normalize import Normalizer_ts  # noqa: F401  (shapes only)
        from oracle import dps as odps
        c = DPS_CFG[config]
        mult = c["channel_mult"].replace(" ", "")
        cfg, sd = _unet_oracle(c["size"], mult)
        d, L, co, nh, H = c["siren"]
        ssd = _siren_oracle(dict(d=d, L=L, c=co, nh=nh, H=H))
        tb = od.Tables(1000, "cosine", c["respacing"])
        Sz = c["size"]
        coords = torch.from_numpy(synth.uniform(5, "dps/sensors", (10, d), 0.0, 1.0))
        one_d, zero_d = torch.ones(1, d), torch.zeros(1, d)
        yx, yn = torch.full((co,), 2.0), torch.full((co,), -2.0)
        vx, vn = torch.full((L,), 1.5), torch.full((L,), -1.5)
        op = lambda x0: odps.case4_forward(ssd, coords, one_d, zero_d, yx, yn, vx, vn, x0)  # noqa: E731
        unet = lambda x, t: ou.forward(sd, cfg, x, t)  # noqa: E731
        x = torch.from_numpy(synth.normal(1000, "dps/xT", (1, 1, Sz, L)))
        with torch.no_grad():
            y = op(torch.from_numpy(synth.uniform(6, "dps/xtrue", (1, 1, Sz, L), -0.9, 0.9)))
        k = 4 if config == "D" else 2
        odps.dps_step(tb, unet, op, x, tb.num_timesteps - 1, y, torch.randn_like(x), 1.0)   # warm
        t0 = time.perf_counter()
        for j in range(k):
            x = odps.dps_step(tb, unet, op, x, tb.num_timesteps - 1 - j, y, torch.randn_like(x), 1.0)[0]
        dt = (time.perf_counter() - t0) / k
        out.update(unit="it/s", value=1.0 / dt, measured={"guided_steps": k, "s_per_step": dt, "chains": 1},
                   sample=(f"oracle on {threads} threads: {k} guided DPS steps of one chain ({Sz}^2 U-Net forward "
                           f"+ autograd through the Case4 operator at 10 sensors and the U-Net), it/s = 1 / s per "
                           f"step (independent chains: the rate per chain)"))
        return out
    if config in ("B", "E"):
        if config == "B":
            cfg, sd = _unet_oracle(S, "")
            nf_c, size, nb, steps, rows, npts_field = CNF_B, S, 8, 256, S, GRID ** 3
        else:
            e = UNCOND_CFG["E"]
            cfg, sd = _unet_oracle(e["size"], "")
            nf_c, size, nb, steps, rows, npts_field = e["siren"], e["size"], 2, 1000, e["size"], e["coords"]
        x = torch.randn(B, 1, size, size)
        t = torch.full((B,), 500, dtype=torch.int64)
        with torch.no_grad():
            unet_step, nstep = _time_loop(lambda: ou.forward(sd, cfg, x, t), nb, 0.0)
        pair_s, dec_s, pairs = _decode_rate(nf_c, 65536, 16)
        per_field = steps * unet_step / B + rows * npts_field * pair_s
        out["measured"] = {"unet_forward_b8_s": unet_step, "unet_forwards": nstep,
                           "decode_pairs": pairs, "decode_s": dec_s, "ns_per_pair": pair_s * 1e9}
        out["extrapolated"] = {"unet_s_per_field": steps * unet_step / B,
                               "decode_s_per_field": rows * npts_field * pair_s, "s_per_field": per_field}
        out["sample"] = (f"oracle on {threads} threads (fp32; the reference has no bf16 path): {nstep} U-Net forwards "
                         f"at B={B} ({unet_step:.3f} s each) + one decode of {pairs} pairs ({dec_s:.1f} s); "
                         f"extrapolated to {steps} steps per {B} samples + {rows} x {npts_field} pairs per field")
        out["value"] = 1.0 / per_field
        return out
    pair_s, dec_s, pairs = _decode_rate(CNF_C, 65536, 16)
    per_field = C_COORDS * pair_s
    out["measured"] = {"decode_pairs": pairs, "decode_s": dec_s, "ns_per_pair": pair_s * 1e9}
    out["extrapolated"] = {"s_per_field": per_field}
    out["sample"] = (f"oracle on {threads} threads: one decode of {pairs} pairs ({dec_s:.1f} s); extrapolated to "
                     f"{C_COORDS} coords per field")
    out["value"] = 1.0 / per_field
    return out


# ---------------------------------------------------------------------------
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", choices=["A", "B", "C", "D", "E", "Case4"], default="B")
    ap.add_argument("--dps-steps", type=int, default=0,
                    help="D / Case4: time this many reverse steps of the loop (0: the whole loop)")
    ap.add_argument("--batch", type=int, default=0,
                    help="A / E: samples per GPU; D / Case4: chains per GPU (0: the config's)")
    ap.add_argument("--plan-batch", type=int, default=-1,
                    help="A / B / D / E / Case4: the U-Net planner's nominal batch (-1: the config's; 0: 8)")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="weak")
    ap.add_argument("--no-gather", action="store_true", help="keep decoded fields on their ranks")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="B: sample and decode each batch in sequence on the whole chip (the default pipelines "
                         "from 4 timed steps)")
    ap.add_argument("--siren-compute", choices=["split_f16", "f32"], default="split_f16")
    ap.add_argument("--unet-compute", choices=["split_f16", "fp32"], default="split_f16")
    ap.add_argument("--per-gpu-batch", type=int, default=0,
                    help="B: samples per GPU in weak scaling (0: config B's 8); 1 = the per-rank share of the "
                         "8-GPU strong point")
    ap.add_argument("--launch-check", action="store_true",
                    help="print each rank's launch environment and exit before any GPU call (tests)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        if args.launch_check:   # the parent has not initialised HIP when it starts the ranks
            print(json.dumps({"parent_hip_initialized": bool(torch.cuda.is_initialized())}), flush=True)
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) != args.gpus and "--gpus" in sys.argv:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}")
    if args.launch_check:
        print(json.dumps({k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR")}),
              flush=True)
        return

    rank, world, dev = init_dist()
    from confild_amd import dist as cdist
    gather = world > 1 and not args.no_gather

    if args.config in ("D", "Case4"):
        return main_dps(args, rank, world, dev)
    if args.config in ("A", "E"):
        return main_uncond(args, rank, world, dev)
    if args.config == "B":
        o = setup_B(dev, rank, world, args.siren_compute, args.unet_compute, args.plan_batch)
        nf = o["nf"]
        shards = b_shards(args.scaling, world, args.per_gpu_batch or B)
        glob = sum(cnt for _, cnt in shards)
        start, count = shards[rank]
        sizes = [cnt * S for _, cnt in shards]
        big = max(cnt for _, cnt in shards)
        if args.plan_batch < 0 and big < B:
            # fewer samples per GPU than 8 (--per-gpu-batch): every rank plans the
            # convolutions for the largest shard (one plan for the whole job)
            o["model"].set_plan_batch(big)

        def one(k, ev=None):
            f = step_B(o, dev, seed=10 ** 6 + k, start=start, count=count, ev=ev)
            return gather_to_root(f, 0, sizes, world) if gather else f

        def strong_point():
            """Config B's global batch of 8 split over the ranks (the strong-scaling
            point), timed like the main line, for the nested "strong" object: the
            model planned for the per-GPU share (so its sums differ in rounding from
            the 8-per-GPU plan) and pipelined like the main line."""
            sh = b_shards("strong", world)
            st_, cn = sh[rank]
            sz = [c_ * S for _, c_ in sh]
            big_s = max(c_ for _, c_ in sh)
            prev = o["model"].plan_batch
            try:
                if args.plan_batch < 0:
                    o["model"].set_plan_batch(big_s if big_s < B else 0)
                piped = not args.no_pipeline and args.steps >= 4
                if piped:
                    with PipelineB(o, dev, st_, cn, sz, world, gather) as pp:
                        if args.warmup:
                            pp.run([2 * 10 ** 6 - 1 - w for w in range(args.warmup)])
                        barrier(dev, world)
                        t0 = time.perf_counter()
                        pp.run([2 * 10 ** 6 + k for k in range(args.steps)])
                        barrier(dev, world)
                        el = max_over_ranks(time.perf_counter() - t0, dev, world)
                else:
                    def f(k):
                        r = step_B(o, dev, seed=2 * 10 ** 6 + k, start=st_, count=cn)
                        return gather_to_root(r, 0, sz, world) if gather else r
                    for w in range(args.warmup):
                        f(-1 - w)
                    barrier(dev, world)
                    t0 = time.perf_counter()
                    for k in range(args.steps):
                        f(k)
                    barrier(dev, world)
                    el = max_over_ranks(time.perf_counter() - t0, dev, world)
                return {"value": B * args.steps / el, "unit": "fields/s", "ms_per_step": el / args.steps * 1e3,
                        "global_batch": B, "per_gpu": [c_ for _, c_ in sh], "scaling": "strong",
                        "plan_batch": o["model"].plan_batch or B,
                        "plan_note": "planned for the largest shard (a stated choice, DESIGN.md section 7): "
                                     "samples equal the 8-per-GPU plan's within fp32 rounding, not bit for bit",
                        "pipelined": piped}
            finally:
                o["model"].set_plan_batch(prev)
        c = CNF_B
        npts = GRID ** 3
        rows_local = count * S
        fields_per_step = glob
    else:
        o = setup_C(dev, rank, world, args.siren_compute)
        nf = o["nf"]
        s, e = o["shard"]
        sizes = [cdist.shard_range(C_COORDS, r, world)[1] - cdist.shard_range(C_COORDS, r, world)[0]
                 for r in range(world)]

        def one(k, ev=None):
            if ev is not None:
                ev[0].record()
                ev[1].record()
            f = nf.decode(o["coords"], o["lat"], o["xn"], o["yn"])                # (256, N_r, 3)
            if ev is not None:
                ev[2].record()
            return gather_to_root(f, 1, sizes, world) if gather else f
        c = CNF_C
        npts = e - s
        rows_local = C_LATENTS
        fields_per_step = C_LATENTS
    mode = nf.compute_mode(dev)
    kname, peak, peak_basis, _ = ROOFLINE[mode]

    # config B with >= 4 timed steps: the two-stage pipeline (PipelineB); the
    # decoder's roofline is then against the MFMA peak of its CU half
    pipe = PipelineB(o, dev, start, count, sizes, world, gather) if (
        args.config == "B" and not args.no_pipeline and args.steps >= 4) else None
    if pipe is not None:
        if args.warmup:
            pipe.run([10 ** 6 - 1 - w for w in range(args.warmup)])
        barrier(dev, world)
        t0 = time.perf_counter()
        evu, evd, out = pipe.run([10 ** 6 + k for k in range(args.steps)])
        barrier(dev, world)
        elapsed = max_over_ranks(time.perf_counter() - t0, dev, world)
        unet_ms = float(np.mean([a.elapsed_time(b) for a, b in evu]))
        # the decode half's side-by-side parts (rows [0, n1) of each batch)
        dec_ms = float(np.mean([a.elapsed_time(b) for a, b in evd]))
        dec_rows = float(np.mean(pipe.rows_b))
        peak, peak_basis = peak * pipe.cu_share, f"{peak_basis} x the decode stream's CU share {pipe.cu_share:g}"
    else:
        for w in range(args.warmup):
            one(-1 - w)
        barrier(dev, world)
        evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
        t0 = time.perf_counter()
        for k in range(args.steps):
            out = one(k, evs[k])
        barrier(dev, world)
        elapsed = max_over_ranks(time.perf_counter() - t0, dev, world)
        unet_ms = float(np.mean([ev[0].elapsed_time(ev[1]) for ev in evs]))
        dec_ms = float(np.mean([ev[1].elapsed_time(ev[2]) for ev in evs]))
    value = fields_per_step * args.steps / elapsed
    # FLOP of one timed decoder launch: a whole batch's rows, or (pipelined) the
    # decode half's part of a batch
    launch_rows = rows_local if pipe is None else dec_rows
    flops = launch_rows * npts * siren_flops_per_pair(**c)
    achieved = flops / (dec_ms / 1e3) / 1e12
    if rank == 0 and out is not None:
        assert torch.isfinite(out).all().item(), "non-finite output"
    strong = strong_point() if args.config == "B" and world > 1 and args.scaling == "weak" else None
    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(args.config)
        par = (f"dp{world} ({f'{count} samples per GPU' if args.scaling == 'weak' else 'global batch 8 split'}"
               f"{', fields gathered to rank 0' if gather else ''})") if args.config == "B" else \
            f"coord-sharded over {world} GPU(s){', slabs gathered to rank 0' if gather else ''}"
        if args.config == "B":
            workload = (f"config B (Case4 uncond), {args.scaling} scaling: U-Net 64x64, global batch "
                        f"{fields_per_step} ({count}/GPU), DDPM 256 steps (cosine, respaced), CNF SIREN(3,64,3,15,384) "
                        f"decode of {S} latent rows per sample on the 64^3 lattice")
        else:
            workload = (f"config C (Case4 CNF-only): SIREN(3,384,3,15,384) decode of {C_LATENTS} latents x 2^22 "
                        f"uniform coords, coordinate-sharded")
        dshare = 1.0 if pipe is None else pipe.cu_share
        dcus = None if pipe is None else pipe.cus[1]
        rec = {
            "metric": METRIC if args.config == "B" else
            "decoded fields/sec (CNF-only, 2^22 coords per field), Case4 CNF, 1/2/4/8 GPU",
            "value": value, "unit": "fields/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": args.scaling if args.config == "B" else "strong",
            "vs_baseline": None, "dtype": "f32", "data": "synthetic (seeded weights and inputs; no checkpoints)",
            "compute": {"unet": ("fp32 via split-f16 convolutions (3x v_mfma_f32_32x32x16/16x16x32_f16 on 22-bit "
                                 "operand splits; error vs fp64 = fp32's, DESIGN.md K1h/K1x/K1s); "
                                 "GroupNorm/softmax fp32, attention split-f16 (K4s)"
                                 if args.config == "B" and o["model"].compute == "split_f16" else
                                 "fp32 (v_mfma_f32_16x16x4_f32)" if args.config == "B" else None),
                        "cnf_decoder": ("fp32 via split-f16 (3x v_mfma_f32_32x32x16_f16 on 22-bit operand "
                                        "splits; error vs fp64 = fp32's, DESIGN.md K7t)" if mode == "split_f16"
                                        else "fp32 (v_mfma_f32_16x16x4_f32)")},
            "config": {"workload": workload, "global_batch": fields_per_step, "seq_len": S if args.config == "B"
                       else C_COORDS, "parallelism": par},
            "roofline": {"bound": "mfma", "kernel": f"{kname} (+siren_film)", "achieved": achieved,
                         "peak": peak, "peak_basis": peak_basis, "unit": "TFLOP/s", "frac": achieved / peak,
                         "traffic": measured_traffic(mode, launch_rows, npts, dcus) if args.config == "B" else None,
                         "traffic_source": f"profiles/{ROOFLINE[mode][3]}" if args.config == "B" else None,
                         # fields written + coordinates and per-point bounds read + the split weight image
                         "algorithmic_bytes": launch_rows * npts * c["c"] * 4 + npts * (c["d"] + 2 * c["c"]) * 4
                         + c["nh"] * c["H"] * c["H"] * 4,
                         "flops_per_launch": flops, "launch_ms": dec_ms, "launch_rows": launch_rows,
                         "pmc": measured_mfma_util(mode, dcus) if args.config == "B" else None,
                         **({"peak_sustained": F16_SUSTAINED_TFLOPS / 3 * dshare,
                             "frac_sustained": achieved / (F16_SUSTAINED_TFLOPS / 3 * dshare),
                             "sustained_basis": "measured back-to-back f16 MFMA on random operands / 3 "
                                                "(tools/mfma_chain.cpp, profiles/r02_mfma_chain.json)"}
                            if mode == "split_f16" else {})},
            "cpu_baseline": cpu,
            "rccl_ranks": world,
        }
        if args.config == "B":
            rec["plan_batch"] = o["model"].plan_batch or B
        if pipe is not None:
            rec["pipeline"] = {"sample_cus": pipe.cus[0], "decode_cus": pipe.cus[1],
                               "sample_ms_per_batch": unet_ms, "decode_half_ms_per_batch": dec_ms,
                               "rows_per_batch": pipe.R, "decode_half_rows": pipe.rows_b,
                               "note": "batch k-1 decoded while batch k samples: rows [0, n1) on the decode CU "
                                       "half beside the sampling, rows [n1, R) on the sampling half after it "
                                       "(n1 re-balanced per batch); the first batch samples and the last decodes "
                                       "on the whole chip (bench.py PipelineB); roofline.launch_ms and "
                                       "flops_per_launch = the decode half's parts"}
        if strong is not None:
            rec["strong"] = strong
        if args.config == "B":
            # the whole chip's rate: every algorithmic FLOP of a step (256 U-Net
            # forwards + the decode of its samples) / (ms_per_step x the chip peak)
            step_flops = count * UNET_FLOPS_PER_SAMPLE * 256 + rows_local * npts * siren_flops_per_pair(**c)
            chip = step_flops / (elapsed / args.steps) / 1e12
            rec["roofline"]["frac_chip"] = chip / (F16_PEAK_TFLOPS / 3)
            rec["roofline_chip"] = {"bound": "mfma", "flops_per_step": step_flops, "achieved": chip,
                                    "peak": F16_PEAK_TFLOPS / 3, "unit": "TFLOP/s", "frac": chip / (F16_PEAK_TFLOPS / 3),
                                    "basis": "all algorithmic FLOP of a step (U-Net x 256 + decode) / ms_per_step, "
                                             "against the whole chip's split-f16 peak (f16 dense / 3)"}
            uf = count * UNET_FLOPS_PER_SAMPLE * 256
            ua = uf / (unet_ms / 1e3) / 1e12
            # pipelined: all but the first batch sample on the other CU half
            ush = 1.0 if pipe is None else (1 + (args.steps - 1) * pipe.cus[0] / sum(pipe.cus)) / args.steps
            rec["roofline_unet"] = {"bound": "mfma", "kernel": "U-Net forward x 256 steps (all kernels + step)",
                                    "achieved": ua, "peak": F16_PEAK_TFLOPS / 3 * ush,
                                    "peak_basis": "f16 dense MFMA peak / 3 (split-f16 convolutions)" +
                                    ("" if pipe is None else f" x the sampling stream's mean CU share {ush:.3f}"),
                                    "unit": "TFLOP/s", "frac": ua / (F16_PEAK_TFLOPS / 3 * ush), "flops": uf,
                                    "ms": unet_ms, "ms_per_forward": unet_ms / 256,
                                    "peak_sustained": F16_SUSTAINED_TFLOPS / 3 * ush,
                                    "frac_sustained": ua / (F16_SUSTAINED_TFLOPS / 3 * ush)}
        print(json.dumps(rec), flush=True)
    if pipe is not None:
        pipe.close()
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def main_dps(args, rank, world, dev):
    """Guided DPS loop (C/gaussian_diffusion.py:169-206 with 'ps' conditioning):
    config D = the 256-step loop at config-B widths, B chains per GPU; Case4 = the
    notebook's 384^2 1000-step loop (its published 9.26-9.35 it/s at one sample,
    inference_phy_random_sensor.ipynb:321-330).  A step = one chain-batch reverse
    step (U-Net forward with tape, DDPM step, SIREN at the sensors, latent
    gradient, U-Net input-VJP, update); it/s = steps x chains / s.  With
    --dps-steps the loop is timed over its first K steps (every step costs the
    same)."""
    from confild_amd import synth
    c = DPS_CFG[args.config]
    batch = args.batch or c["batch"]
    o = setup_dps(dev, rank, world, args.config, batch, args.plan_batch)
    smp = o["sampler"]
    nsteps = smp.num_timesteps
    timed = min(args.dps_steps, nsteps) if args.dps_steps else nsteps
    x0 = torch.from_numpy(synth.normal(1000 + rank, "dps/xT", (batch, 1, o["S"], o["L"]))).to(dev)

    def run(k_steps, seed):
        x = x0.clone()
        dist_buf = torch.zeros(batch, device=dev)
        for k, i in enumerate(range(nsteps - 1, nsteps - 1 - k_steps, -1)):
            x = smp._guided_step(o["model"], x, i, o["y"], o["cond"], None, seed, k, rank * batch, dist_buf)[0]
        return x

    for w in range(args.warmup):
        run(min(3, timed), 7 + w)
    barrier(dev, world)
    t0 = time.perf_counter()
    for k in range(args.steps):
        out = run(timed, 100 + k)
    barrier(dev, world)
    elapsed = max_over_ranks(time.perf_counter() - t0, dev, world)
    assert torch.isfinite(out).all().item(), "non-finite output"
    o["model"].check_finite(dev)
    steps_total = timed * args.steps
    its = steps_total * batch * world / elapsed
    # counted FLOPs per chain-step (FlopCounterMode's convention, pinned in
    # tests/test_host.py): U-Net forward with tape + its input-VJP (convolutions
    # once more, both attention products twice) + the SIREN at the sensors,
    # forward and backward to the latents
    from confild_amd.nf_networks import latent_grad_flops
    from confild_amd.unet import forward_flops
    m = o["model"]
    uf = forward_flops(m.image_size, m.in_channels, m.model_channels, m.out_channels, m.num_res_blocks,
                       set(m.attention_resolutions), m.channel_mult, m.num_heads, m.num_head_channels)
    d, L, co, nh, H = c["siren"]
    sf = latent_grad_flops(d, L, co, nh, H, o["S"], 10)
    per_chain = sum(uf.values()) + uf["conv"] + 2 * uf["attn"] + sf["forward"] + sf["backward"]
    achieved = per_chain * steps_total * batch / (elapsed * 1e12)   # per GPU
    if rank == 0:
        rec = {"metric": "guided DPS reverse steps/sec (it/s summed over chains), Case4 conditional",
               "value": its, "unit": "it/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": elapsed / steps_total * 1e3, "higher_is_better": True, "scaling": "weak",
               "vs_baseline": None, "dtype": "f32", "data": "synthetic (seeded weights and inputs; no checkpoints)",
               "config": {"workload": (f"config {args.config}: guided 'ps' DDPM loop, U-Net {o['S']}^2 "
                                       f"(channel_mult {c['channel_mult'] or 'default'}), SIREN{c['siren']} at 10 "
                                       f"sensors, {nsteps}-step schedule, {timed} steps timed, {batch} chain(s)/GPU"),
                          "global_batch": batch * world, "seq_len": o["S"],
                          "parallelism": f"dp{world} (independent chains)"},
               "reference_published": ("9.26-9.35 it/s at one chain, unstated NVIDIA GPU "
                                       "(inference_phy_random_sensor.ipynb:321-330)") if args.config == "Case4" else None,
               "per_chain_it_s": its / (batch * world),
               "roofline": {"bound": "mfma", "kernel": "whole guided step (U-Net forward with tape + input-VJP on "
                                                       "split-f16 MFMA, SIREN tape on fp32 MFMA, step kernels)",
                            "achieved": achieved, "peak": F16_PEAK_TFLOPS / 3,
                            "peak_basis": "f16 dense MFMA peak / 3 (split-f16 convolutions)", "unit": "TFLOP/s",
                            "frac": achieved / (F16_PEAK_TFLOPS / 3),
                            "peak_sustained": F16_SUSTAINED_TFLOPS / 3,
                            "frac_sustained": achieved / (F16_SUSTAINED_TFLOPS / 3), "traffic": None,
                            "flops_per_chain_step": per_chain,
                            "flops_split": {"unet_forward": sum(uf.values()), "unet_input_vjp": uf["conv"] + 2 * uf["attn"],
                                            "siren_forward": sf["forward"], "siren_backward": sf["backward"]}},
               "cpu_baseline": None if args.no_cpu_baseline or world > 1 else cpu_baseline(args.config),
               "rccl_ranks": world}
        print(json.dumps(rec), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
