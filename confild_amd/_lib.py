"""ctypes binding of the C ABI in include/confild.h (libconfild_hip.so).

The product path has no CPU fallback: if the in-tree library is missing or no
GPU is visible, every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libconfild_hip.so")
# development A/B runs only: CFD_LIB names another in-tree build of the same library
if os.environ.get("CFD_LIB"):
    LIB_PATH = os.path.join(_HERE, "lib", os.path.basename(os.environ["CFD_LIB"]))

_lock = threading.Lock()
_lib = None

c_f32p = C.POINTER(C.c_float)
c_i64p = C.POINTER(C.c_int64)


class CfdError(RuntimeError):
    pass


class UNetCfg(C.Structure):
    _fields_ = [("image_size", C.c_int), ("in_channels", C.c_int), ("model_channels", C.c_int),
                ("out_channels", C.c_int), ("num_res_blocks", C.c_int), ("n_mult", C.c_int),
                ("channel_mult", C.c_int * 8), ("n_attn", C.c_int), ("attention_ds", C.c_int * 8),
                ("num_heads", C.c_int), ("num_head_channels", C.c_int)]


class SirenCfg(C.Structure):
    _fields_ = [("in_coord_features", C.c_int), ("in_latent_features", C.c_int), ("out_features", C.c_int),
                ("num_hidden_layers", C.c_int), ("hidden_features", C.c_int), ("w0", C.c_float)]


# name -> (restype, argtypes)
_SIGS = {
    "cfd_last_error": (C.c_char_p, []),
    "cfd_version": (C.c_char_p, []),
    "cfd_unet_create": (C.c_int, [C.POINTER(UNetCfg), C.c_int, C.POINTER(C.c_void_p)]),
    "cfd_unet_destroy": (None, [C.c_void_p]),
    "cfd_unet_num_params": (C.c_int, [C.c_void_p, C.POINTER(C.c_int)]),
    "cfd_unet_param_info": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_int),
                                      C.c_int64 * 4]),
    "cfd_unet_set_param": (C.c_int, [C.c_void_p, C.c_char_p, C.c_void_p, C.c_size_t]),
    "cfd_unet_set_time_freqs": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int]),
    "cfd_unet_ready": (C.c_int, [C.c_void_p]),
    "cfd_unet_load_flat": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]),
    "cfd_unet_set_compute": (C.c_int, [C.c_void_p, C.c_int]),
    "cfd_unet_set_plan_batch": (C.c_int, [C.c_void_p, C.c_int]),
    "cfd_device_cu_count": (C.c_int, [C.c_int, C.POINTER(C.c_int)]),
    "cfd_stream_create_cu_range": (C.c_int, [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p)]),
    "cfd_stream_destroy": (C.c_int, [C.c_void_p]),
    "cfd_unet_check_finite": (C.c_int, [C.c_void_p, C.POINTER(C.c_int), C.c_void_p]),
    "cfd_unet_workspace_bytes": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_size_t)]),
    "cfd_unet_forward": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p,
                                   C.c_size_t, C.c_void_p]),
    "cfd_unet_tape_bytes": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_size_t)]),
    "cfd_unet_vjp_workspace_bytes": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_size_t)]),
    "cfd_unet_forward_tape": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p,
                                        C.c_size_t, C.c_void_p, C.c_size_t, C.c_void_p]),
    "cfd_unet_input_vjp": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_size_t,
                                     C.c_void_p, C.c_size_t, C.c_void_p]),
    "cfd_unet_set_tape_mode": (C.c_int, [C.c_void_p, C.c_int]),
    "cfd_sched_create": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_void_p)]),
    "cfd_sched_destroy": (None, [C.c_void_p]),
    "cfd_sched_step": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                 C.c_uint64, C.c_uint64, C.c_uint64, C.c_void_p, C.c_void_p, C.c_int64, C.c_int,
                                 C.c_void_p]),
    "cfd_sampler_create": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int64, C.c_int,
                                     C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_void_p)]),
    "cfd_sampler_destroy": (None, [C.c_void_p]),
    "cfd_sampler_run": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_uint64, C.c_uint64,
                                  C.c_void_p]),
    "cfd_randn": (C.c_int, [C.c_void_p, C.c_int64, C.c_uint64, C.c_uint64, C.c_uint64, C.c_void_p]),
    "cfd_sine_probe": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_int, C.c_void_p]),
    "cfd_latent_denorm": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_int64,
                                    C.c_void_p]),
    "cfd_dps_residual": (C.c_int, [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_int,
                                   C.c_void_p]),
    "cfd_dps_latent_grad": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                      C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_int64, C.c_int,
                                      C.c_void_p]),
    "cfd_dps_update": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_float, C.c_void_p, C.c_int64,
                                 C.c_void_p]),
    "cfd_siren_create": (C.c_int, [C.POINTER(SirenCfg), C.c_int, C.POINTER(C.c_void_p)]),
    "cfd_siren_destroy": (None, [C.c_void_p]),
    "cfd_siren_num_params": (C.c_int, [C.c_void_p, C.POINTER(C.c_int)]),
    "cfd_siren_param_info": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_int),
                                       C.c_int64 * 4]),
    "cfd_siren_set_param": (C.c_int, [C.c_void_p, C.c_char_p, C.c_void_p, C.c_size_t]),
    "cfd_siren_ready": (C.c_int, [C.c_void_p]),
    "cfd_siren_workspace_bytes": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_size_t)]),
    "cfd_siren_set_compute": (C.c_int, [C.c_void_p, C.c_int]),
    "cfd_siren_get_compute": (C.c_int, [C.c_void_p, C.POINTER(C.c_int)]),
    "cfd_siren_forward": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_int, C.c_void_p,
                                    C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p,
                                    C.c_size_t, C.c_void_p]),
    "cfd_siren_vjp_workspace_bytes": (C.c_int, [C.c_void_p, C.c_int64, C.c_int, C.POINTER(C.c_size_t)]),
    "cfd_siren_tape_forward": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_int, C.c_void_p,
                                         C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p,
                                         C.c_size_t, C.c_void_p]),
    "cfd_siren_tape_vjp": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_int, C.c_void_p, C.c_void_p,
                                     C.c_int64, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]),
    "cfd_siren_train_workspace_bytes": (C.c_int, [C.c_void_p, C.c_int64, C.c_int, C.POINTER(C.c_size_t)]),
    "cfd_siren_train_grad": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_int,
                                       C.c_void_p, C.c_float, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_size_t, C.c_void_p]),
    "cfd_unet_param_grad_workspace_bytes": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_size_t)]),
    "cfd_unet_param_grad": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_size_t,
                                      C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]),
    "cfd_eps_mse": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_int, C.c_float,
                              C.c_void_p, C.c_void_p]),
    "cfd_ema_update": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_double, C.c_void_p]),
    "cfd_q_sample": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_int,
                               C.c_void_p]),
    "cfd_adam_step": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_double, C.c_double,
                                C.c_double, C.c_double, C.c_double, C.c_int64, C.c_void_p]),
}

EXPORTS = tuple(_SIGS)


def load(path: str = LIB_PATH):
    """Load (once) and type the library.  Raises if it is not built."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise CfdError(f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                           "(or `make -C confild_amd/csrc`)")
        lib = C.CDLL(path)
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def lib():
    """The library, for GPU use: also requires a visible HIP device."""
    import torch
    if not torch.cuda.is_available():
        raise CfdError("confild_amd needs an AMD GPU (MI355X); no HIP device is visible and there is no CPU path")
    return load()


def check(rc: int, what: str = ""):
    if rc != 0:
        msg = load().cfd_last_error().decode()
        kind = {1: "bad argument", 2: "HIP error", 3: "unknown key", 4: "shape error", 5: "state error"}.get(rc, rc)
        raise CfdError(f"{what}: {kind}: {msg}")


def ptr(t) -> C.c_void_p:
    """Device (or host) data pointer of a torch tensor / None."""
    if t is None:
        return None
    return C.c_void_p(t.data_ptr())


def stream_of(device) -> C.c_void_p:
    import torch
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)
