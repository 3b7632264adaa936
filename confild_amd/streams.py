"""CU-partitioned HIP streams (cfd_stream_create_cu_range): kernels launched on
such a stream run on a fixed subset of the device's compute units only, so two
independent pipelines (config B's sampling loop and the CNF decode of the
previous batch) can share the chip side by side."""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib


def cu_count(device) -> int:
    device = torch.device(device)
    idx = device.index if device.index is not None else torch.cuda.current_device()
    n = C.c_int(0)
    _lib.check(_lib.load().cfd_device_cu_count(idx, C.byref(n)), "cfd_device_cu_count")
    return n.value


class CuRangeStream:
    """A torch-usable stream bound to CUs [first, first + count) of `device`.

    The HIP stream is destroyed by close() (also on leaving a ``with`` block, or
    when the object is collected) after a device synchronise, so no queued work
    and no caching-allocator block recorded on it outlives the stream."""

    def __init__(self, device, first: int, count: int):
        device = torch.device(device)
        self.device_index = device.index if device.index is not None else torch.cuda.current_device()
        self._handle = None
        h = C.c_void_p()
        _lib.check(_lib.load().cfd_stream_create_cu_range(self.device_index, int(first), int(count), C.byref(h)),
                   "cfd_stream_create_cu_range")
        self._handle = h
        self.first, self.count = int(first), int(count)
        self.stream = torch.cuda.ExternalStream(h.value, device=torch.device("cuda", self.device_index))

    def close(self):
        if self._handle is not None and self._handle.value:
            torch.cuda.synchronize(self.device_index)
            _lib.check(_lib.load().cfd_stream_destroy(self._handle), "cfd_stream_destroy")
        self._handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    def __del__(self):
        import sys
        if sys.is_finalizing():   # the HIP runtime may already be gone
            return
        try:
            self.close()
        except Exception:
            pass
