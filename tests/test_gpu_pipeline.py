"""The timed configuration of the headline line: bench.py's PipelineB (config B
as a two-stage pipeline over the chip's CU halves: the decode of batch k-1 on
one half while batch k samples on the other, cross-stream events between them)
must give, for every batch, the same bits as step_B -- the same seed sampled
and decoded in sequence on the whole chip.  Each side-by-side decode is split by
latent rows between the decode half (beside the sampling) and the sampling half
(after it), re-balanced per batch; the rows' fields must not depend on the
split.  An ordering bug between the two streams (a decode reading a latent the
sampler is still writing, a sampler overwriting the buffers of a pending
decode) would show here as a mismatch.

The second test runs the pipelined decode's RCCL gather (dist.gather on the
CU-masked decode stream, bench.py gather_to_root) under a one-rank "nccl"
process group on the one GPU, so the path the 8-GPU line takes has executed:
rank 0's gathered fields are its own, bit for bit.

Both run at 2 samples per batch (a sample's bits do not depend on the batch it
runs in: test_gpu_plan_batch.py, test_gpu_cfg.py) to keep the test short; the
model keeps the bench's plan (8)."""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
COUNT = 2


@pytest.fixture(scope="module")
def cfgB(hip):
    import bench
    return bench, bench.setup_B(DEV, 0, 1, "split_f16", "split_f16")


def test_pipeline_fields_equal_sequential_step(cfgB):
    bench, o = cfgB
    seeds = [10 ** 6 + k for k in range(5)]
    kept = []
    with bench.PipelineB(o, DEV, 0, COUNT, [COUNT * bench.S], 1, False) as pp:
        evu, evd, last = pp.run(seeds, keep=kept)
    torch.cuda.synchronize()
    assert len(kept) == len(seeds) and kept[-1] is last
    assert len(evu) == len(seeds) and len(evd) == len(seeds) - 1
    # the side-by-side decodes were split by rows between the two CU halves
    assert len(pp.rows_b) == len(seeds) - 1 and pp.rows_b[0] < COUNT * bench.S
    assert all(COUNT * bench.S // 2 <= r <= COUNT * bench.S for r in pp.rows_b)
    for seed, f in zip(seeds, kept):
        ref = bench.step_B(o, DEV, seed, 0, COUNT)
        torch.cuda.synchronize()
        assert f.shape == (COUNT * bench.S, bench.GRID ** 3, 3)
        assert torch.isfinite(ref).all()
        assert torch.equal(f, ref), (seed, float((f - ref).abs().max()))
    # different seeds give different fields (the comparison is not vacuous)
    assert not torch.equal(kept[0], kept[1])


def test_pipeline_rccl_gather_on_cu_masked_stream(cfgB):
    import torch.distributed as dist
    bench, o = cfgB
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=DEV)
    try:
        seeds = [10 ** 6 + 7, 10 ** 6 + 8, 10 ** 6 + 9]
        kept = []
        with bench.PipelineB(o, DEV, 0, COUNT, [COUNT * bench.S], 1, True) as pp:
            pp.run(seeds, keep=kept)
        torch.cuda.synchronize()
        for seed, f in zip(seeds, kept):
            ref = bench.step_B(o, DEV, seed, 0, COUNT)
            torch.cuda.synchronize()
            assert f.data_ptr() != ref.data_ptr()
            assert torch.equal(f, ref), seed
        # the gather itself, on the CU-masked stream, into a fresh buffer
        with bench.PipelineB(o, DEV, 0, COUNT, [COUNT * bench.S], 1, True) as pp:
            x = torch.randn(COUNT * bench.S, 1000, 3, device=DEV)
            pp.sd.stream.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(pp.sd.stream):
                g = bench.gather_to_root(x, 0, [x.shape[0]], 1)
            torch.cuda.synchronize()
            assert g.data_ptr() != x.data_ptr() and torch.equal(g, x)
    finally:
        dist.destroy_process_group()
