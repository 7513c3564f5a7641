"""Multi-GPU exchange of compressed gradient buckets.

Each rank (one process per GPU) encodes its own bucket: buckets are independent, so there is no
collective in the data path (weak scaling, config C4; contiguous shards of one big gradient for
C5).  The one real exchange step -- every worker receiving every other worker's compressed
gradient, done through Spark in the reference (GeneralizedLinearModel.scala:145-150) -- is an
RCCL all-gather of the fixed-size payloads over xGMI (skml_allgather), followed on each rank by
the fused decode + sum + scale (skml_dense_decode_sum_f32).

The control plane (unique-id broadcast, size agreement) rides on torch.distributed, so it runs
on gloo in CPU tests and on the RCCL process group on the GPU box.
"""
from __future__ import annotations

import ctypes as C
from typing import Callable, Optional

import torch
import torch.distributed as dist

from . import _lib
from .exceptions import check


def shard_range(n_total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous bucket of rank r: [r*floor(n/P), ...), the last rank takes the remainder
    (the slicing of parallelQuantizeToBins, Quantizer.java:105-107)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    per = n_total // world
    lo = rank * per
    hi = n_total if rank == world - 1 else lo + per
    return lo, hi


def agree_sizes(nbytes: int, group=None) -> list[int]:
    """All ranks' payload sizes (variable-size sparse payloads are padded to the max)."""
    world = dist.get_world_size(group)
    t = torch.tensor([int(nbytes)], dtype=torch.int64)
    if dist.get_backend(group) == "nccl":
        t = t.cuda()
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t, group=group)
    return [int(v.item()) for v in out]


def broadcast_unique_id(make_id: Callable[[], bytes], group=None, src: int = 0) -> bytes:
    """Rank `src` creates the RCCL unique id; every rank receives the same bytes."""
    obj = [make_id() if dist.get_rank(group) == src else None]
    dist.broadcast_object_list(obj, src=src, group=group)
    uid = obj[0]
    if not isinstance(uid, (bytes, bytearray)) or len(uid) != _lib.UNIQUE_ID_BYTES:
        raise RuntimeError("bad unique id from rank %d" % src)
    return bytes(uid)


def _rccl_unique_id() -> bytes:
    uid = (C.c_uint8 * _lib.UNIQUE_ID_BYTES)()
    check(_lib.lib.skml_comm_unique_id(uid), "comm_unique_id")
    return bytes(uid)


class PayloadExchange:
    """RCCL communicator over the ranks of `group` for all-gathering compressed payloads."""

    def __init__(self, ctx_handle, group=None, make_id: Optional[Callable[[], bytes]] = None):
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self._ctx = ctx_handle
        uid = broadcast_unique_id(make_id or _rccl_unique_id, group)
        buf = (C.c_uint8 * _lib.UNIQUE_ID_BYTES).from_buffer_copy(uid)
        self._comm = C.c_void_p()
        check(_lib.lib.skml_comm_init_rank(ctx_handle, buf, self.world, self.rank, C.byref(self._comm)),
              "comm_init_rank")

    def allgather(self, payload: torch.Tensor, nbytes: int, out: torch.Tensor) -> None:
        """out[r*nbytes:(r+1)*nbytes] = rank r's payload (asynchronous on the context stream)."""
        if out.numel() * out.element_size() < nbytes * self.world:
            raise ValueError("all-gather output too small")
        check(_lib.lib.skml_allgather(self._ctx, self._comm, C.c_void_p(payload.data_ptr()), nbytes,
                                      C.c_void_p(out.data_ptr())), "allgather")

    def close(self) -> None:
        if self._comm:
            _lib.lib.skml_comm_destroy(self._comm)
            self._comm = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def decode_sum(ctx_handle, payloads: torch.Tensor, nranks: int, stride: int, n: int, scale: float,
               out: torch.Tensor) -> None:
    """Fused decode of `nranks` gathered payloads + double-precision sum + scale
    (Gradient.sum then timesBy(1/P), ml/gradient/Gradient.scala:44-49)."""
    check(_lib.lib.skml_dense_decode_sum_f32(ctx_handle, C.c_void_p(payloads.data_ptr()), nranks, stride,
                                             C.c_void_p(out.data_ptr()), n, float(scale)), "decode_sum")
