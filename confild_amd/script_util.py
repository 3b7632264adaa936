"""Factories with the reference signatures (U/src/script_util.py:130-187, 388-426)."""
from __future__ import annotations

from . import gaussian_diffusion as gd
from .respace import SpacedDiffusion, space_timesteps
from .unet import UNetModel


def create_model(image_size, num_channels, num_res_blocks, dims=2, out_channels=1, channel_mult=None,
                 learn_sigma=False, class_cond=False, use_checkpoint=False, attention_resolutions="16",
                 num_heads=1, num_head_channels=-1, num_heads_upsample=-1, use_scale_shift_norm=False, dropout=0,
                 resblock_updown=False, use_fp16=False, use_new_attention_order=False, use_bf16=False):
    """script_util.py:130-187 (channel_mult defaults by image size; attention ds = image_size // res).
    ``use_bf16`` (not in the reference): bf16 convolution operands with fp32
    accumulation, the config-E arithmetic (BASELINE.json configs[4])."""
    if channel_mult is None or channel_mult == "":
        if image_size == 512:
            channel_mult = (0.5, 1, 1, 2, 2, 4, 4)
        elif image_size == 256:
            channel_mult = (1, 1, 2, 2, 4, 4)
        elif image_size == 128:
            channel_mult = (1, 1, 2, 3, 4)
        elif image_size == 64:
            channel_mult = (1, 2, 3, 4)
        else:
            raise ValueError(f"unsupported image size: {image_size}")
    elif isinstance(channel_mult, str):
        channel_mult = tuple(int(c) for c in channel_mult.split(","))
    else:
        channel_mult = tuple(channel_mult)
    if isinstance(attention_resolutions, int):
        attention_ds = [image_size // attention_resolutions]
    else:
        attention_ds = [image_size // int(r) for r in str(attention_resolutions).split(",")]
    if learn_sigma:
        raise NotImplementedError("learn_sigma=True (learned variance) is not part of the CoNFiLD path")
    model = UNetModel(image_size=image_size, in_channels=out_channels, model_channels=num_channels,
                      out_channels=out_channels, num_res_blocks=num_res_blocks,
                      attention_resolutions=tuple(attention_ds), dropout=dropout, channel_mult=channel_mult,
                      num_classes=(1000 if class_cond else None), use_checkpoint=use_checkpoint, use_fp16=use_fp16,
                      num_heads=num_heads, num_head_channels=num_head_channels,
                      num_heads_upsample=num_heads_upsample, use_scale_shift_norm=use_scale_shift_norm,
                      resblock_updown=resblock_updown, use_new_attention_order=use_new_attention_order, dims=dims)
    return model.set_compute("bf16") if use_bf16 else model


def create_gaussian_diffusion(*, steps=1000, learn_sigma=False, sigma_small=False, noise_schedule="linear",
                              use_kl=False, predict_xstart=False, rescale_timesteps=False,
                              rescale_learned_sigmas=False, timestep_respacing=""):
    """script_util.py:388-426: SpacedDiffusion with EPSILON + FIXED_LARGE (+ MSE)."""
    betas = gd.get_named_beta_schedule(noise_schedule, steps)
    if use_kl:
        loss_type = gd.LossType.RESCALED_KL
    elif rescale_learned_sigmas:
        loss_type = gd.LossType.RESCALED_MSE
    else:
        loss_type = gd.LossType.MSE
    if not timestep_respacing:
        timestep_respacing = [steps]
    return SpacedDiffusion(
        use_timesteps=space_timesteps(steps, timestep_respacing),
        betas=betas,
        model_mean_type=gd.ModelMeanType.EPSILON if not predict_xstart else gd.ModelMeanType.START_X,
        model_var_type=((gd.ModelVarType.FIXED_LARGE if not sigma_small else gd.ModelVarType.FIXED_SMALL)
                        if not learn_sigma else gd.ModelVarType.LEARNED_RANGE),
        loss_type=loss_type,
        rescale_timesteps=rescale_timesteps,
    )
