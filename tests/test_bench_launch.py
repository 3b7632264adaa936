"""bench.py --gpus N without a launcher starts N rank processes itself (the
driver's `python bench.py --gpus N` must yield N RCCL ranks): each child gets the
torchrun environment (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR), and the
parent has not initialised HIP when it starts them (CPU test, --launch-check
stops every rank before any GPU call)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_self_launch_sets_rank_env():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--launch-check"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert lines[0] == {"parent_hip_initialized": False}
    ranks = sorted(lines[1:], key=lambda d: int(d["RANK"]))
    assert [(d["RANK"], d["LOCAL_RANK"], d["WORLD_SIZE"], d["MASTER_ADDR"]) for d in ranks] == \
        [(str(i), str(i), "3", "127.0.0.1") for i in range(3)]


def test_bench_rejects_gpus_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--launch-check"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


def test_wait_ranks_fails_fast_and_stops_the_others():
    """A rank that exits non-zero ends the job: the ranks still running (here a
    sleeping child standing in for one blocked in a rendezvous) are terminated and
    the failing code is returned, instead of waiting for the backend timeout."""
    import time
    sys.path.insert(0, ROOT)
    import bench
    hang = subprocess.Popen([sys.executable, "-c", "import time; time.sleep(600)"])
    fail = subprocess.Popen([sys.executable, "-c", "import sys; sys.exit(7)"])
    t0 = time.time()
    assert bench.wait_ranks([hang, fail], time.sleep) == 7
    assert time.time() - t0 < 60 and hang.poll() is not None
    ok = [subprocess.Popen([sys.executable, "-c", "pass"]) for _ in range(2)]
    assert bench.wait_ranks(ok, time.sleep) == 0
