"""CPU oracle for the CoNFiLD generation hot path -- TEST INFRASTRUCTURE ONLY.

This package restates, on the CPU with PyTorch fp32 / numpy float64, the
reference algorithms the HIP path replaces:

  * ``oracle.diffusion`` -- beta schedules, respacing, DDPM/DDIM step maths
    (U/src/gaussian_diffusion.py, U/src/respace.py);
  * ``oracle.unet``      -- the guided-diffusion U-Net forward
    (U/src/unet.py, U/src/nn.py);
  * ``oracle.siren``     -- SIRENAutodecoder_film + Normalizer_ts
    (N/cnf/nf_networks.py, N/cnf/components.py, N/cnf/utils/normalize.py).

It is pinned against golden fixtures produced by running the reference itself
in the build container (tests/golden/make_golden.py; see tests/test_oracle.py).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg
may import this package, and only as the checker / the timed CPU baseline.
The product package ``confild_amd`` never imports it and has no CPU fallback.
"""
