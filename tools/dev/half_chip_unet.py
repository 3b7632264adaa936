"""Config B's U-Net forward (64^2, B = 8, split-f16) on one CU half (development
tool, for a kernel trace): the graph-loop sampler on a CuRangeStream of CUs
[0, n) as the pipelined bench runs it, with nothing on the other half.

    rocprofv3 --kernel-trace --stats -d out -o run -- python3 tools/dev/half_chip_unet.py 128
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from confild_amd import synth  # noqa: E402
from confild_amd.script_util import create_gaussian_diffusion, create_model  # noqa: E402
from confild_amd.streams import CuRangeStream  # noqa: E402

DEV = torch.device("cuda", 0)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    m = create_model(image_size=64, num_channels=128, num_res_blocks=2, num_heads=4, num_head_channels=64,
                     attention_resolutions="32,16,8")
    sd = synth.unet_state_dict(1234, {k: tuple(v.shape) for k, v in m.state_dict().items()})
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m.to(DEV).prepare(DEV)
    d = create_gaussian_diffusion(steps=1000, noise_schedule="cosine", timestep_respacing="16")
    with CuRangeStream(DEV, 0, n) as su:
        with torch.cuda.stream(su.stream):
            d.p_sample_loop(m, (8, 1, 64, 64), seed=1)   # capture + warm
            d.p_sample_loop(m, (8, 1, 64, 64), seed=2)
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
