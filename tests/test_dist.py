"""Multi-process (gloo, world_size 2, CPU) tests of the sharding and collective
code in confild_amd.dist.  The compute is the CPU oracle, plugged in through the
same callables the GPU path uses; the GPU path itself is the HIP decode."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from confild_amd import dist as cdist
from confild_amd import synth


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, fn, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, fn(rank, world)))
    except Exception as e:  # surface the failure to the parent
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def _run(fn, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
    return out


def _siren_decode_fn():
    from oracle import siren as osn
    d, L, c, nh, H = 3, 16, 3, 2, 32
    sd = {k: torch.from_numpy(v) for k, v in synth.siren_state_dict(3, d, L, c, nh, H).items()}

    def fn(coords, latents, ymax, ymin):
        return osn.decode(sd, coords, latents, torch.ones(1, d), torch.zeros(1, d), ymax, ymin)
    return fn


def _case_sharded_decode(rank, world):
    N, b = 1001, 5
    coords = torch.from_numpy(synth.uniform(1, "c", (N, 3), 0.0, 1.0))
    lat = torch.from_numpy(synth.normal(2, "z", (b, 16)))
    ymax = torch.from_numpy(synth.uniform(3, "ymax", (1, N, 3), 0.5, 2.0))
    ymin = -ymax
    fn = _siren_decode_fn()
    full = cdist.sharded_decode(fn, coords, lat, ymax, ymin)
    ref = fn(coords, lat, ymax, ymin)
    return bool(torch.equal(full, ref)), tuple(full.shape)


def _case_sharded_samples(rank, world):
    B = 7

    def sample_fn(start, count):  # deterministic per global sample index
        return torch.stack([torch.full((4, 4), float(start + i)) for i in range(count)])
    full = cdist.sharded_samples(sample_fn, B)
    return [float(v) for v in full[:, 0, 0]]


def _case_broadcast(rank, world):
    torch.manual_seed(100 + rank)  # different init per rank
    m = torch.nn.Sequential(torch.nn.Linear(8, 8), torch.nn.Linear(8, 3))
    cdist.broadcast_module(m, src=0)
    return [float(p.sum()) for p in m.parameters()]


def _case_gather(rank, world):
    N = 9
    s, e = cdist.shard_range(N, rank, world)
    x = torch.arange(s, e, dtype=torch.float32)[None].repeat(2, 1)
    sizes = [cdist.shard_range(N, r, world)[1] - cdist.shard_range(N, r, world)[0] for r in range(world)]
    out = cdist.gather_cat(x, 1, sizes, dst=0)
    return None if out is None else out[0].tolist()


def test_shard_range_covers_exactly():
    for n in (1, 7, 64, 1000):
        for g in (1, 2, 3, 8):
            spans = [cdist.shard_range(n, r, g) for r in range(g)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(g - 1))


def test_coordinate_sharded_decode_equals_unsharded():
    out = _run(_case_sharded_decode)
    assert out[0] == (True, (5, 1001, 3)) and out[1] == (True, (5, 1001, 3)), out


def test_sample_sharding_preserves_global_order():
    out = _run(_case_sharded_samples)
    assert out[0] == out[1] == [float(i) for i in range(7)]


def test_bucketed_weight_broadcast():
    out = _run(_case_broadcast)
    assert out[0] == out[1]


def test_gather_to_root_uneven():
    out = _run(_case_gather)
    assert out[0] == [float(i) for i in range(9)] and out[1] is None


def _case_broadcast_bumps_version(rank, world):
    """Cached device weights are keyed on (data_ptr, _version): the broadcast must
    bump _version so a handle uploaded before it re-uploads."""
    torch.manual_seed(200 + rank)
    m = torch.nn.Linear(4, 4)
    before = [p._version for p in m.parameters()]
    cdist.broadcast_module(m, src=0)
    after = [p._version for p in m.parameters()]
    return all(a > b for a, b in zip(after, before))


def _case_too_few_samples(rank, world):
    try:
        cdist.sharded_samples(lambda s, c: torch.zeros(c, 2), world - 1)
    except ValueError:
        return "ValueError"
    return "no error"


def test_broadcast_bumps_parameter_version():
    assert _run(_case_broadcast_bumps_version) == {0: True, 1: True}


def test_sharded_samples_rejects_batch_below_world():
    assert _run(_case_too_few_samples) == {0: "ValueError", 1: "ValueError"}


def _case_gather_dim0(rank, world):
    """gather_cat along dim 0: equal slabs land in place, uneven ones are padded."""
    out = {}
    for n in (2 * world, 2 * world + 1):
        s, e = cdist.shard_range(n, rank, world)
        x = torch.arange(s, e, dtype=torch.float32)[:, None].repeat(1, 3)
        sizes = [cdist.shard_range(n, r, world)[1] - cdist.shard_range(n, r, world)[0] for r in range(world)]
        g = cdist.gather_cat(x, 0, sizes, dst=0)
        out[n] = None if g is None else g[:, 0].tolist()
    return out


def _case_bench_config_C(rank, world):
    """bench.py config C's sharding: per-rank coordinate shards + per-point
    normaliser rows, latents broadcast, slabs gathered to rank 0 along N --
    equal to the unsharded decode (oracle compute, small sizes)."""
    import bench
    from oracle import siren as osn
    d, L, c, nh, H = 3, 16, 3, 2, 32
    sd = {k: torch.from_numpy(v) for k, v in synth.siren_state_dict(3, d, L, c, nh, H).items()}
    n_coords, n_lat = 1003, 4
    coords, lat, ymax, ymin, (s, e) = bench.c_inputs(rank, world, n_coords, n_lat, L)
    dist.broadcast(lat, src=0)
    part = osn.decode(sd, coords, lat, torch.ones(1, 3), torch.zeros(1, 3), ymax, ymin)
    sizes = [cdist.shard_range(n_coords, r, world)[1] - cdist.shard_range(n_coords, r, world)[0]
             for r in range(world)]
    full = bench.gather_to_root(part, 1, sizes, world)
    if rank != 0:
        return full is None
    ac, al, ax, an, _ = bench.c_inputs(0, 1, n_coords, n_lat, L)
    ref = osn.decode(sd, ac, al, torch.ones(1, 3), torch.zeros(1, 3), ax, an)
    return bool(torch.equal(full, ref))


def _case_bench_config_B(rank, world):
    """bench.py config B's sample shards (weak and strong) gathered to rank 0 in
    global sample order (stand-in compute: rows tagged by global sample index)."""
    import bench
    res = {}
    for scaling in ("weak", "strong"):
        shards = bench.b_shards(scaling, world)
        start, count = shards[rank]
        rows = torch.cat([torch.full((2, 3), float(start + i)) for i in range(count)])   # 2 rows per sample
        g = bench.gather_to_root(rows, 0, [2 * cnt for _, cnt in shards], world)
        res[scaling] = None if g is None else g[::2, 0].tolist()
    return res


def test_gather_cat_dim0_in_place_and_padded():
    out = _run(_case_gather_dim0)
    assert out[0] == {4: [0.0, 1.0, 2.0, 3.0], 5: [0.0, 1.0, 2.0, 3.0, 4.0]}, out
    assert out[1] == {4: None, 5: None}


def test_bench_config_C_sharding_equals_unsharded():
    assert _run(_case_bench_config_C) == {0: True, 1: True}


def test_bench_config_B_shards_weak_and_strong():
    out = _run(_case_bench_config_B)
    assert out[0] == {"weak": [float(i) for i in range(16)], "strong": [float(i) for i in range(8)]}, out
    assert out[1] == {"weak": None, "strong": None}
