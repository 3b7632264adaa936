"""create_model of the conditional notebook (C/src/guided_diffusion/unet.py:25-92)."""
from __future__ import annotations

import warnings

import torch

from ..unet import UNetModel

NUM_CLASSES = 1000


def create_model(image_size, num_channels, num_res_blocks, out_channels=1, channel_mult="", learn_sigma=False,
                 class_cond=False, use_checkpoint=False, attention_resolutions="16", num_heads=1, num_head_channels=-1,
                 num_heads_upsample=-1, use_scale_shift_norm=False, dropout=0, resblock_updown=False, use_fp16=False,
                 use_new_attention_order=False, model_path="", random_init_on_error=False):
    """Same arguments as the reference (C/unet.py:25-92).  Checkpoints load with
    weights_only=True.

    Loading fails loudly: a missing, unreadable or
    mismatched ``model_path`` raises instead of silently keeping random weights,
    which is what the reference does (C/unet.py:86-90: print + random init).
    ``random_init_on_error=True`` restores the reference's behaviour.  An empty
    ``model_path`` asks for no checkpoint at all: the model keeps its
    initialisation and a warning says so."""
    if channel_mult == "":
        table = {512: (0.5, 1, 1, 2, 2, 4, 4), 256: (1, 1, 2, 2, 4, 4), 128: (1, 1, 2, 3, 4), 64: (1, 2, 3, 4)}
        if image_size not in table:
            raise ValueError(f"unsupported image size: {image_size}")
        channel_mult = table[image_size]
    else:
        channel_mult = tuple(int(ch_mult) for ch_mult in channel_mult.split(","))
    if isinstance(attention_resolutions, int):
        attention_ds = [image_size // attention_resolutions]
    elif isinstance(attention_resolutions, str):
        attention_ds = [image_size // int(res) for res in attention_resolutions.split(",")]
    else:
        raise NotImplementedError
    model = UNetModel(image_size=image_size, in_channels=out_channels, model_channels=num_channels,
                      out_channels=(out_channels if not learn_sigma else 2 * out_channels),
                      num_res_blocks=num_res_blocks, attention_resolutions=tuple(attention_ds), dropout=dropout,
                      channel_mult=channel_mult, num_classes=(NUM_CLASSES if class_cond else None),
                      use_checkpoint=use_checkpoint, use_fp16=use_fp16, num_heads=num_heads,
                      num_head_channels=num_head_channels, num_heads_upsample=num_heads_upsample,
                      use_scale_shift_norm=use_scale_shift_norm, resblock_updown=resblock_updown,
                      use_new_attention_order=use_new_attention_order)
    if not model_path:
        warnings.warn("guided create_model without model_path: randomly initialised U-Net", stacklevel=2)
        return model
    try:
        model.load_state_dict(torch.load(model_path, map_location="cpu", weights_only=True))
    except Exception as e:
        if not random_init_on_error:
            raise RuntimeError(f"could not load U-Net weights from {model_path!r}: {e} (pass "
                               "random_init_on_error=True for the reference's silent random init)") from e
        print(f"Got exception: {e} / Randomly initialize")   # the reference's behaviour (unet.py:86-90)
    return model
