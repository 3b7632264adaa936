"""Config B's pipelined step (bench.py PipelineB) at several CU splits between
the sampling and the decode streams (development tool): fields/s over K timed
batches after W warmup batches, per split, in one process.

    python tools/dev/pipe_split.py 96 112 128 144 160
    PIPE_COUNT=1 PIPE_PLAN=1 python tools/dev/pipe_split.py 128 160 192 224   # the strong share
"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

DEV = torch.device("cuda", 0)


def main():
    splits = [int(v) for v in sys.argv[1:]] or [128]
    W, K = 3, 8
    count = int(os.environ.get("PIPE_COUNT", "8"))
    o = bench.setup_B(DEV, 0, 1, "split_f16", "split_f16", plan_batch=int(os.environ.get("PIPE_PLAN", "0")))
    R = count * bench.S
    out = []
    for rnd in range(2):
        for h in splits:
            with bench.PipelineB(o, DEV, 0, count, [R], 1, False, sample_cus=h) as pp:
                pp.run([10 ** 6 + k for k in range(W)])
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                pp.run([2 * 10 ** 6 + k for k in range(K)])
                torch.cuda.synchronize()
                el = time.perf_counter() - t0
            rec = {"round": rnd, "count": count, "sample_cus": h, "fields_per_s": count * K / el, "ms_per_batch": el / K * 1e3,
                   "rows_b": pp.rows_b[-3:]}
            out.append(rec)
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
