"""CU-partitioned streams (cfd_stream_create_cu_range, confild_amd.streams): the
kernels run on a subset of the compute units and compute the same bits as on the
whole chip -- the property bench.py's config-B pipeline (the decode of one batch
beside the sampling of the next) rests on."""
import pytest
import torch

from confild_amd import synth
from confild_amd.nf_networks import SIRENAutodecoder_film
from confild_amd.script_util import create_model
from confild_amd.streams import CuRangeStream, cu_count

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def test_cu_range_streams_give_identical_bits(hip):
    m = create_model(image_size=32, num_channels=128, num_res_blocks=2, channel_mult="1,2,3,4", num_heads=4,
                     num_head_channels=64, attention_resolutions="32,16,8")
    m.load_state_dict({k: torch.from_numpy(v) for k, v in
                       synth.unet_state_dict(3, {k: tuple(v.shape) for k, v in m.state_dict().items()}).items()})
    m.to(DEV)
    nf = SIRENAutodecoder_film(3, 64, 3, 15, 384)
    nf.load_state_dict({k: torch.from_numpy(v) for k, v in synth.siren_state_dict(3, 3, 64, 3, 15, 384).items()})
    nf.to(DEV)
    x = torch.from_numpy(synth.normal(3, "cu/x", (2, 1, 32, 32))).to(DEV)
    t = torch.tensor([900, 12], device=DEV)
    coords = torch.rand(4096, 3, device=DEV)
    lat = torch.randn(8, 1, 64, device=DEV) * 0.5
    ref_e, ref_f = m(x, t), nf.decode(coords, lat)
    n = cu_count(DEV)
    assert n >= 2
    a, b = CuRangeStream(DEV, 0, n // 2), CuRangeStream(DEV, n // 2, n - n // 2)
    try:
        a.stream.wait_stream(torch.cuda.current_stream())
        b.stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(a.stream):
            e = m(x, t)
        with torch.cuda.stream(b.stream):
            f = nf.decode(coords, lat)
        torch.cuda.synchronize()
        assert torch.equal(e, ref_e)
        assert torch.equal(f, ref_f)
    finally:
        a.close()
        b.close()


def test_cu_range_rejects_bad_ranges(hip):
    from confild_amd import _lib
    n = cu_count(DEV)
    with pytest.raises(_lib.CfdError):
        CuRangeStream(DEV, n - 1, 2)
