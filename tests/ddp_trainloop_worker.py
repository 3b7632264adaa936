"""Worker of tests/test_gpu_unet_train.py::test_trainloop_ddp_two_ranks: one rank
of a 2-process TrainLoop step on the same GPU (gloo over device tensors; the flat
gradient is averaged across the ranks as DistributedDataParallel does).

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port P tests/ddp_trainloop_worker.py OUT_PREFIX

Rank r trains on sample r of the golden TrainLoop case and writes its averaged
gradient, parameters and EMA after one step to OUT_PREFIX.rank{r}.pt.
"""
import ast
import os
import sys

import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.dirname(HERE)]

from conftest import golden  # noqa: E402
from confild_amd import synth  # noqa: E402
from confild_amd.script_util import create_gaussian_diffusion, create_model  # noqa: E402
from confild_amd.train_util import TrainLoop  # noqa: E402


class _Fixed:
    def __init__(self, t):
        self.t = t

    def sample(self, batch_size, device):
        return (torch.tensor(self.t[:batch_size], dtype=torch.int64, device=device),
                torch.ones(batch_size, device=device))


def main(out):
    dist.init_process_group("gloo")
    r = dist.get_rank()
    dev = torch.device("cuda", 0)
    g = golden("golden_unettrain.npz")
    c = ast.literal_eval(str(g["case"]))
    gu = golden(f"unet_{c['net']}.npz")
    kw = ast.literal_eval(str(gu["kwargs"]))
    m = create_model(**kw)
    sd = synth.unet_state_dict(int(gu["seed"]), {k: tuple(v.shape) for k, v in m.state_dict().items()})
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m.to(dev)
    diff = create_gaussian_diffusion(steps=1000, noise_schedule=c["schedule"], timestep_respacing="")
    loop = TrainLoop(model=m, diffusion=diff, train_data=None, batch_size=1, microbatch=-1, lr=c["lr"],
                     ema_rate=c["ema_rate"], log_interval=1, save_interval=1000, resume_checkpoint="",
                     weight_decay=c["weight_decay"], schedule_sampler=_Fixed([c["t"][0][r]]))
    assert loop.world_size == 2
    x0 = torch.from_numpy(g["x0"][r:r + 1]).to(dev)
    nz = torch.from_numpy(g["noise"][0][r:r + 1]).to(dev)
    loop.run_step(x0, None, None, noise=nz)
    torch.cuda.synchronize()
    torch.save({"grad": loop.grad.cpu(), "params": loop.params.cpu(), "ema": loop.ema_params[0].cpu()},
               f"{out}.rank{r}.pt")
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
