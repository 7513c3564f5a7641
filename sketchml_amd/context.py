"""Per-device codec contexts bound to torch's current HIP stream.

PyTorch is plumbing here: it provides device memory and the stream; all codec work runs in
libskml.so's kernels.
"""
from __future__ import annotations

import ctypes as C
import threading

import torch

from . import _lib
from .exceptions import check

_local = threading.local()


class Context:
    def __init__(self, device: int):
        self.device = device
        self._h = C.c_void_p()
        with torch.cuda.device(device):
            stream = torch.cuda.current_stream(device).cuda_stream
        check(_lib.lib.skml_ctx_create(device, C.c_void_p(stream), C.byref(self._h)), "ctx_create")
        self._stream = stream

    @property
    def handle(self):
        st = torch.cuda.current_stream(self.device).cuda_stream
        if st != self._stream:
            check(_lib.lib.skml_ctx_set_stream(self._h, C.c_void_p(st)), "set_stream")
            self._stream = st
        return self._h

    def sync(self):
        check(_lib.lib.skml_ctx_sync(self.handle), "sync")

    def __del__(self):
        try:
            if self._h:
                _lib.lib.skml_ctx_destroy(self._h)
        except Exception:
            pass


def get_context(device=None) -> Context:
    if device is None:
        device = torch.cuda.current_device()
    if isinstance(device, torch.device):
        device = device.index if device.index is not None else torch.cuda.current_device()
    ctxs = getattr(_local, "ctxs", None)
    if ctxs is None:
        ctxs = _local.ctxs = {}
    if device not in ctxs:
        ctxs[device] = Context(device)
    return ctxs[device]


def alloc_aligned(nbytes: int, device, align: int = 256) -> torch.Tensor:
    """A uint8 device tensor whose data pointer is `align`-byte aligned."""
    buf = torch.empty(nbytes + align, dtype=torch.uint8, device=device)
    off = (-buf.data_ptr()) % align
    return buf[off: off + nbytes]


def as_device_values(values, device=None) -> torch.Tensor:
    """Device-resident contiguous, 16-byte aligned view of a gradient: float64 input (a torch
    float64 tensor or a numpy float64 array, the reference's double[]) stays fp64; everything
    else becomes fp32."""
    if isinstance(values, torch.Tensor):
        wide = values.dtype == torch.float64
    else:
        import numpy as np
        wide = np.asarray(values).dtype == np.float64
    if not wide:
        return as_device_f32(values, device)
    if isinstance(values, torch.Tensor):
        t = values if values.is_cuda else values.to(device or torch.cuda.current_device())
    else:
        import numpy as np
        t = torch.from_numpy(np.ascontiguousarray(values, dtype=np.float64)).to(
            device or torch.cuda.current_device())
    t = t.contiguous().view(-1)
    if t.data_ptr() % 16:
        t = t.clone()
    return t


def as_device_f32(values, device=None) -> torch.Tensor:
    """Device-resident contiguous, 16-byte aligned fp32 view (copies host arrays to the GPU)."""
    if isinstance(values, torch.Tensor):
        t = values
        if not t.is_cuda:
            t = t.to(device or torch.cuda.current_device())
    else:
        import numpy as np
        t = torch.from_numpy(np.ascontiguousarray(values, dtype=np.float32)).to(
            device or torch.cuda.current_device())
    if t.dtype != torch.float32:
        t = t.to(torch.float32)
    t = t.contiguous().view(-1)
    if t.data_ptr() % 16:
        t = t.clone()
    return t
