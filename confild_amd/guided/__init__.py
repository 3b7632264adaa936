"""Drop-in for ConditionalDiffusionGeneration/src/guided_diffusion (the Case4
conditional / DPS path).

    from confild_amd.guided.unet import create_model
    from confild_amd.guided.condition_methods import get_conditioning_method
    from confild_amd.guided.measurements import get_noise, get_operator
    from confild_amd.guided.gaussian_diffusion import create_sampler

The notebook code (inference_phy_random_sensor.ipynb cells 11-23) runs
unchanged on these imports.  The reference differentiates the measurement norm
through the U-Net and the SIREN with torch autograd; here the sampler recognises
the 'ps' conditioning method and runs the fused adjoint instead: U-Net forward
with a tape, SIREN tape forward at the sensors, residual norm, SIREN latent
VJP, clamp / un-normalisation links, U-Net input VJP, update -- all HIP kernels
(cfd_unet_forward_tape / cfd_unet_input_vjp, cfd_siren_tape_forward /
cfd_siren_tape_vjp, cfd_dps_*).
"""
