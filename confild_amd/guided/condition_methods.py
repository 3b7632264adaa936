"""Conditioning methods (C/src/guided_diffusion/condition_methods.py).

'ps' (PosteriorSampling, :81-90) and 'vanilla' (Identity, :52-56) are on the
CoNFiLD path.  Their gradient step is executed by the DPS sampler
(confild_amd.guided.gaussian_diffusion), which recognises the method object
behind ``partial(cond_method.conditioning)`` and runs the fused HIP adjoint;
torch autograd does not run through the HIP U-Net / SIREN.
"""
from __future__ import annotations

from abc import ABC

__CONDITIONING_METHOD__ = {}


def register_conditioning_method(name: str):
    def wrapper(cls):
        if __CONDITIONING_METHOD__.get(name, None):
            raise NameError(f"Name {name} is already registered!")
        __CONDITIONING_METHOD__[name] = cls
        return cls
    return wrapper


_NOT_BUILT = {"projection", "mcg", "ps_linear_decay", "ps+"}


def get_conditioning_method(name: str, operator, noiser, **kwargs):
    """condition_methods.py:17-20."""
    if name in _NOT_BUILT:
        raise NotImplementedError(f"conditioning method {name!r} is not on the CoNFiLD path (use 'ps')")
    if __CONDITIONING_METHOD__.get(name, None) is None:
        raise NameError(f"Name {name} is not defined!")
    return __CONDITIONING_METHOD__[name](operator=operator, noiser=noiser, **kwargs)


class ConditioningMethod(ABC):
    def __init__(self, operator, noiser, **kwargs):
        self.operator = operator
        self.noiser = noiser


@register_conditioning_method(name="vanilla")
class Identity(ConditioningMethod):
    def conditioning(self, x_t, **kwargs):
        return x_t, None


@register_conditioning_method(name="ps")
class PosteriorSampling(ConditioningMethod):
    def __init__(self, operator, noiser, **kwargs):
        super().__init__(operator, noiser)
        self.scale = kwargs.get("scale", 1.0)
        if getattr(noiser, "__name__", "gaussian") != "gaussian":
            raise NotImplementedError("PosteriorSampling on the HIP path: gaussian noiser only (as the Case4 notebook)")

    def conditioning(self, x_prev, x_t, x_0_hat, measurement, **kwargs):
        raise NotImplementedError(
            "PosteriorSampling.conditioning differentiates through the U-Net with autograd in the reference; "
            "here the DPS sampler (create_sampler(...).p_sample_loop) runs the fused adjoint -- pass "
            "partial(cond_method.conditioning) to it as measurement_cond_fn")
