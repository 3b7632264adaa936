"""Benchmark: CoNFiLD Case4 unconditional generation on MI355X.

One step = one batch of the BASELINE.json configs[1] workload on each GPU:
  * 256-step DDPM reverse loop (cosine-1000 respaced "256", FIXED_LARGE, clip) of
    the 64x64 latent U-Net (create_model(64, 128 ch, 2 res blocks, attention
    32,16,8, 64-ch heads): 89.5 M parameters) at batch 8;
  * latent de-normalisation (scripts/inference.py:59-61);
  * CNF decode of all 8 x 64 latent rows with SIRENAutodecoder_film(3, 64, 3, 15,
    384) on the 64^3 = 262,144-point lattice (normaliser + per-point
    de-normaliser fused) -> 8 fields of shape (64, 262144, 3) resident in HBM.
Weights and inputs are synthetic (confild_amd.synth, seed 1234); there is no
network access for checkpoints.  Multi-GPU: one process per GPU (torchrun), each
rank generates its own batch of 8 (weak scaling, no data-path collective).

Prints ONE JSON line (rank 0) with the driver contract plus a ``roofline`` object
for the dominant kernel (the CNF decoder, timed with HIP events on its stream) and
a ``cpu_baseline`` measured on this host's cores with the oracle (rank 0, N=1).

The U-Net convolutions (split_f16 conv_gemm) and the decoder's hidden layers run by
default as split-f16 (siren_fused_split: three
f16 MFMAs per fp32 product on 22-bit operand splits, fp32-level error against an
fp64 evaluation -- tests/test_gpu_siren_split.py); its roofline is the f16 dense
MFMA peak / 3.  ``--siren-compute f32`` runs the exact fp32 MFMA chain
(siren_fused) against the fp32 MFMA peak instead.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

B = 8            # samples per GPU
S = 64           # latent image (T = L = 64)
STEPS = "256"    # timestep respacing
GRID = 64        # 64^3 lattice
CNF = dict(d=3, L=64, c=3, nh=15, H=384)
FMA_PEAK_TFLOPS = 157.3    # MI355X fp32 matrix peak (MI355X_MICROARCH.md chip table)
F16_PEAK_TFLOPS = 2500.0   # MI355X dense f16/bf16 matrix peak (same table; no sparsity)
HBM_PEAK_GBS = 8000.0

# dominant-kernel roofline per decoder compute mode:
#   (kernel name, peak in algorithmic fp32 TFLOP/s, basis, committed PMC record)
ROOFLINE = {
    "split_f16": ("siren_split32", F16_PEAK_TFLOPS / 3,
                  "f16 dense MFMA peak / 3 (three f16 MFMAs per fp32 product)", "r01_siren_split32_pmc.json"),
    "f32": ("siren_fused", FMA_PEAK_TFLOPS, "fp32 MFMA peak", "r01_siren_pmc.json"),
}


def measured_traffic(mode, latents, npts):
    """Per-launch fabric bytes of the decoder kernel from the committed rocprofv3
    PMC record (tools/pmc_traffic.py), scaled from its launch geometry to this one."""
    kname, _, _, fname = ROOFLINE[mode]
    try:
        rec = json.load(open(os.path.join(ROOT, "profiles", fname)))
    except (OSError, ValueError):
        return None
    launch = rec.get("launch", {})
    ref_pairs = launch.get("latents", 0) * launch.get("coords", 0)
    if not ref_pairs or f"{kname}<" not in rec.get("kernel", ""):
        return None
    return rec["traffic_bytes_per_launch"] * (latents * npts) / ref_pairs


def measured_mfma_util(kname):
    """Matrix-pipe busy fraction and held clock of the decoder kernel from the
    committed rocprofv3 record (tools/gpujob_mfma_util.sh, tools/mfma_util.py)."""
    try:
        rec = json.load(open(os.path.join(ROOT, "profiles", "r01_mfma_util.json")))
    except (OSError, ValueError):
        return None
    for k, v in rec.items():
        if k.startswith(f"cfd::{kname}<") and isinstance(v, dict):
            return {"mfma_busy_frac": v["mfma_busy_frac"], "held_clock_ghz": v["held_clock_ghz"],
                    "source": "profiles/r01_mfma_util.json"}
    return None


def siren_flops_per_pair(d, L, c, nh, H):
    return 2 * (d * H + nh * H * H + H * c)


def unet_flops_per_sample():
    # conv/bmm/addmm MAC*2 for the config-B U-Net forward (FlopCounter, torch 2.10)
    return 68.61e9


def setup(dev, siren_compute="split_f16", unet_compute="split_f16"):
    from confild_amd import synth
    from confild_amd.nf_networks import SIRENAutodecoder_film
    from confild_amd.normalize import Normalizer_ts
    from confild_amd.script_util import create_gaussian_diffusion, create_model
    model = create_model(image_size=S, num_channels=128, num_res_blocks=2, num_heads=4, num_head_channels=64,
                         attention_resolutions="32,16,8")
    sd = synth.unet_state_dict(1234, {k: tuple(v.shape) for k, v in model.state_dict().items()})
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    model.to(dev)
    model.set_compute(unet_compute)
    diff = create_gaussian_diffusion(steps=1000, noise_schedule="cosine", timestep_respacing=STEPS)
    c = CNF
    nf = SIRENAutodecoder_film(c["d"], c["L"], c["c"], c["nh"], c["H"])
    nf.load_state_dict({k: torch.from_numpy(v) for k, v in
                        synth.siren_state_dict(1234, c["d"], c["L"], c["c"], c["nh"], c["H"]).items()})
    nf.to(dev)
    nf.set_compute(siren_compute)
    ax = torch.linspace(0, 1, GRID)
    coords = torch.stack(torch.meshgrid(ax, ax, ax, indexing="ij"), -1).reshape(-1, 3).to(dev)
    N = coords.shape[0]
    xn = Normalizer_ts(params=(torch.ones(1, 3, device=dev), torch.zeros(1, 3, device=dev)), method="-11", dim=0)
    ymax = torch.from_numpy(synth.uniform(9, "ymax", (1, N, 3), 0.5, 2.0)).to(dev)
    ymin = -torch.from_numpy(synth.uniform(9, "ymin", (1, N, 3), 0.5, 2.0)).to(dev)
    yn = Normalizer_ts(params=(ymax, ymin), method="-11", dim=0)
    vmax = torch.full((1,), 1.5, device=dev)
    vmin = torch.full((1,), -1.5, device=dev)
    return model, diff, nf, coords, xn, yn, vmax, vmin


def generate(objs, dev, seed, ev=None):
    """One batch: sample -> de-normalise -> decode.  Returns fields (B*T, N, c)."""
    from confild_amd import _lib
    model, diff, nf, coords, xn, yn, vmax, vmin = objs
    lat = diff.p_sample_loop(model, (B, 1, S, S), seed=seed)[:, 0]          # (B, T, L)
    den = torch.empty_like(lat)
    _lib.check(_lib.load().cfd_latent_denorm(_lib.ptr(lat), _lib.ptr(den), lat.numel(), _lib.ptr(vmax),
                                             _lib.ptr(vmin), 1, _lib.stream_of(dev)), "denorm")
    if ev is not None:
        ev[0].record()
    fields = nf.decode(coords, den.reshape(B * S, 1, S), xn, yn)              # (B*T, N, c)
    if ev is not None:
        ev[1].record()
    return fields


def cpu_baseline(budget_s=20.0):
    """Oracle (torch CPU restatement of the reference path) on this host's cores,
    on a bounded sample; extrapolated to fields/s.  The reference itself never
    runs on the GPU box."""
    from confild_amd import synth
    from oracle import siren as osn
    from oracle import unet as ou
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    threads = max(1, min(threads, 16))
    torch.set_num_threads(threads)
    cfg = ou.Config(image_size=S, num_channels=128, num_res_blocks=2, num_heads=4, num_head_channels=64,
                    attention_resolutions="32,16,8")
    sd = {k: torch.from_numpy(v) for k, v in synth.unet_state_dict(1234, ou.param_shapes(cfg)).items()}
    x = torch.randn(B, 1, S, S)
    t = torch.full((B,), 500, dtype=torch.int64)
    with torch.no_grad():
        ou.forward(sd, cfg, x[:1], t[:1])  # warm
        t0 = time.perf_counter()
        nstep = 0
        while True:
            ou.forward(sd, cfg, x, t)
            nstep += 1
            if time.perf_counter() - t0 > budget_s / 2 or nstep >= 3:
                break
        unet_step = (time.perf_counter() - t0) / nstep
    c = CNF
    ssd = {k: torch.from_numpy(v) for k, v in synth.siren_state_dict(1234, c["d"], c["L"], c["c"], c["nh"],
                                                                      c["H"]).items()}
    npts = 16384
    coords = torch.rand(npts, 3)
    lat = torch.randn(2, c["L"])
    with torch.no_grad():
        osn.decode(ssd, coords[:1024], lat[:1], torch.ones(1, 3), torch.zeros(1, 3), torch.ones(1, 3),
                   -torch.ones(1, 3))
        t0 = time.perf_counter()
        nd = 0
        while True:
            osn.decode(ssd, coords, lat, torch.ones(1, 3), torch.zeros(1, 3), torch.ones(1, 3), -torch.ones(1, 3))
            nd += 1
            if time.perf_counter() - t0 > budget_s / 2 or nd >= 4:
                break
        pair_s = (time.perf_counter() - t0) / (nd * npts * lat.shape[0])
    N = GRID ** 3
    per_field = 256 * unet_step / B + S * N * pair_s
    return {"value": 1.0 / per_field, "unit": "fields/s", "cores": threads, "kind": "port",
            "sample": (f"oracle (torch CPU restatement): {nstep} U-Net forwards at B={B} "
                       f"({unet_step:.3f} s each) + {nd} decodes of {lat.shape[0]} latents x {npts} coords "
                       f"({pair_s * 1e9:.1f} ns/pair); extrapolated to 256 steps/{B} samples + {S}x{N} pairs "
                       f"per field")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--siren-compute", choices=["split_f16", "f32"], default="split_f16")
    ap.add_argument("--unet-compute", choices=["split_f16", "fp32"], default="split_f16")
    args = ap.parse_args()

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
    objs = setup(dev, args.siren_compute, args.unet_compute)
    mode = objs[2].compute_mode(dev)
    kname, peak, peak_basis, _ = ROOFLINE[mode]

    def barrier():
        torch.cuda.synchronize(dev)
        if world > 1:
            import torch.distributed as dist
            dist.barrier()
            torch.cuda.synchronize(dev)

    for w in range(args.warmup):
        generate(objs, dev, seed=1000 * rank + w)
    barrier()
    ev = [torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)]
    dec_ms = []
    t0 = time.perf_counter()
    for k in range(args.steps):
        fields = generate(objs, dev, seed=10 ** 6 + 1000 * rank + k, ev=ev)
        ev[1].synchronize()
        dec_ms.append(ev[0].elapsed_time(ev[1]))
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        import torch.distributed as dist
        tt = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = tt.item()
    fields_total = B * world * args.steps
    value = fields_total / elapsed
    c = CNF
    pairs = B * S * GRID ** 3
    flops = pairs * siren_flops_per_pair(**c)
    dec_s = float(np.mean(dec_ms)) / 1e3
    achieved = flops / dec_s / 1e12
    assert torch.isfinite(fields).all().item(), "non-finite output"
    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline()
        rec = {
            "metric": "generated fields/sec (256-step sample + CNF decode), Case4 latent, 1/2/4/8 GPU",
            "value": value, "unit": "fields/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32", "data": "synthetic (seeded weights and inputs; no checkpoints)",
            "compute": {"unet": ("fp32 via split-f16 convolutions (3x v_mfma_f32_16x16x32_f16 on 22-bit operand "
                                 "splits; error vs fp64 = fp32's, DESIGN.md K1s); GroupNorm/softmax/attention fp32"
                                 if objs[0].compute == "split_f16" else "fp32 (v_mfma_f32_16x16x4_f32)"),
                        "cnf_decoder": ("fp32 via split-f16 (3x v_mfma_f32_32x32x16_f16 on 22-bit operand "
                                        "splits; error vs fp64 = fp32's, DESIGN.md K7t)" if mode == "split_f16"
                                        else "fp32 (v_mfma_f32_16x16x4_f32)")},
            "config": {"workload": "Case4 uncond: U-Net 64x64 B=8/GPU, DDPM 256 steps (cosine, respaced), "
                                   "CNF SIREN(3,64,3,15,384) decode of 8x64 latents on a 64^3 lattice",
                       "global_batch": B * world, "seq_len": S, "parallelism": f"dp{world} (independent batches)"},
            "roofline": {"bound": "mfma", "kernel": f"{kname} (+siren_film)", "achieved": achieved,
                         "peak": peak, "peak_basis": peak_basis, "unit": "TFLOP/s", "frac": achieved / peak,
                         "traffic": measured_traffic(mode, B * S, GRID ** 3), "flops_per_launch": flops,
                         "launch_ms": dec_s * 1e3, "pmc": measured_mfma_util(kname),
                         "unet_share_ms": (elapsed / args.steps - dec_s) * 1e3},
            "cpu_baseline": cpu,
        }
        print(json.dumps(rec), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
