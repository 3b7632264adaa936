"""GPU parity of config C at its full size (BASELINE.json configs[2]): the Case4
CNF SIREN(3, 384, 3, 15, 384) decoding 256 latents x 2^22 uniform coordinates
in one cfd_siren_forward call -- bench.py's workload (c_inputs, one rank).

The output (256, 2^22, 3) has 3.2e9 elements: past 2^31, so the kernel's store
offsets must be 64-bit.  A seeded subset of 16 latent rows x 256 coordinates
(4096 pairs) is compared with the CPU oracle (oracle.siren.decode, the
reference's nf_networks.py:480-495 + normalize.py:100-114); 8 of the rows are
>= 171, whose elements all lie beyond 2^31.  Tolerance as the other decode
tests: max|d| <= 2e-5 * max(1, max|ref|)."""
import numpy as np
import pytest
import torch

from confild_amd import synth
from confild_amd.nf_networks import SIRENAutodecoder_film
from confild_amd.normalize import Normalizer_ts
from oracle import siren as osn

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def test_configC_full_size_decode_subset_vs_oracle(hip):
    import bench
    c = bench.CNF_C
    sd = {k: torch.from_numpy(v) for k, v in synth.siren_state_dict(1234, c["d"], c["L"], c["c"], c["nh"],
                                                                     c["H"]).items()}
    nf = SIRENAutodecoder_film(c["d"], c["L"], c["c"], c["nh"], c["H"])
    nf.load_state_dict(sd)
    nf.to(DEV)
    coords, lat, ymax, ymin, _ = bench.c_inputs(0, 1, bench.C_COORDS, bench.C_LATENTS, c["L"])
    xn = Normalizer_ts(params=(torch.ones(1, 3), torch.zeros(1, 3)), method="-11", dim=0)
    yn = Normalizer_ts(params=(ymax.to(DEV), ymin.to(DEV)), method="-11", dim=0)
    out = nf.decode(coords.to(DEV), lat.to(DEV)[:, None], xn, yn)
    N = bench.C_COORDS
    assert out.shape == (bench.C_LATENTS, N, 3) and out.numel() > 2 ** 31
    rng = np.random.default_rng(2024)
    rows = np.concatenate([rng.choice(171, 8, replace=False), 171 + rng.choice(bench.C_LATENTS - 171, 8,
                                                                                replace=False)])
    cols = np.sort(np.concatenate([rng.choice(N, 252, replace=False), [0, 1, N - 2, N - 1]]))
    got = out[torch.from_numpy(rows).to(DEV)][:, torch.from_numpy(cols).to(DEV)].cpu()
    assert torch.isfinite(out[-1]).all() and torch.isfinite(out[171]).all()
    del out
    ci = torch.from_numpy(cols)
    with torch.no_grad():
        ref = osn.decode(sd, coords[ci], lat[torch.from_numpy(rows)], torch.ones(1, 3), torch.zeros(1, 3),
                         ymax[:, ci], ymin[:, ci])
    err = float((got - ref).abs().max()) / max(1.0, float(ref.abs().max()))
    print(f"config C full-size decode, 4096-pair subset vs oracle: {err:.2e} (rows {sorted(rows.tolist())})")
    assert err <= 2e-5, err
