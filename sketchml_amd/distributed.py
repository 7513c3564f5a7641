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

import numpy as np

from . import _lib
from .context import as_device_values, get_context
from .exceptions import SketchMLException, check


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


def blob_stride(sizes: list[int]) -> int:
    """Slot size of the padded all-gather: the largest payload, rounded up to 256 bytes (every
    slot, and so every blob, stays 256-byte aligned)."""
    return max(256, (max(sizes) + 255) // 256 * 256)


def gather_blobs(local: torch.Tensor, stride: int, group=None, exchange: Optional[PayloadExchange] = None):
    """All-gather of one `stride`-byte slot per rank (a blob padded to the agreed stride): rank r's
    slot lands at r * stride.  RCCL through `exchange` (or the nccl process group); a host-memory
    group (gloo) goes through host copies."""
    world = dist.get_world_size(group)
    if local.numel() * local.element_size() != stride:
        raise ValueError("the local slot must be exactly `stride` bytes")
    allb = torch.empty(stride * world, dtype=torch.uint8, device=local.device)
    if exchange is not None:
        # the communicator's context may run on its own stream: the slot is complete before the
        # all-gather reads it, and the gathered blobs before the caller's stream uses them
        torch.cuda.current_stream(local.device).synchronize()
        exchange.allgather(local, stride, allb)
        check(_lib.lib.skml_ctx_sync(exchange._ctx), "ctx_sync")
    elif dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(allb, local.view(torch.uint8), group=group)
    else:
        parts = [torch.empty(stride, dtype=torch.uint8) for _ in range(world)]
        dist.all_gather(parts, local.view(torch.uint8).cpu(), group=group)
        allb.copy_(torch.cat(parts).to(local.device))
    return allb


def exchange_sparse(payload, dim: int, group=None, exchange: Optional[PayloadExchange] = None,
                    scale: float | None = None):
    """One DP step of the ml path on P GPUs (GeneralizedLinearModel.scala:145-156): the sizes are
    all-gathered, every rank exports its compressed sparse gradient straight into a slot of the
    largest size, the slots are all-gathered (RCCL over xGMI), and every rank computes Gradient.sum
    of all P payloads (rank order) and the 1/P average, in double, on its own GPU.
    Returns (the dense double average, the gathered blobs, stride)."""
    from .sparse import decode_sum as _sparse_decode_sum
    world = dist.get_world_size(group)
    stride = blob_stride(agree_sizes(payload.export_bytes(), group))
    local = torch.empty(stride, dtype=torch.uint8, device=torch.device("cuda", payload.device))
    payload.export(local)
    allb = gather_blobs(local, stride, group, exchange)
    avg = _sparse_decode_sum(allb, world, stride, dim, 1.0 / world if scale is None else scale)
    return avg, allb, stride


def decode_sum(ctx_handle, payloads: torch.Tensor, nranks: int, stride: int, n: int, scale: float,
               out: torch.Tensor) -> None:
    """Fused decode of `nranks` gathered payloads + double-precision sum + scale
    (Gradient.sum then timesBy(1/P), ml/gradient/Gradient.scala:44-49)."""
    check(_lib.lib.skml_dense_decode_sum_f32(ctx_handle, C.c_void_p(payloads.data_ptr()), nranks, stride,
                                             C.c_void_p(out.data_ptr()), n, float(scale)), "decode_sum")


# ---- one split table across ranks (SURVEY §8e single-split-table mode) ----------------------
def parallel_slices(n_total: int, parts: int) -> list[int]:
    """Slice sizes of QuantileQuantizer.parallelQuantize (QuantileQuantizer.java:66-68): n/T
    each, the last slice takes the remainder."""
    if parts < 1:
        raise SketchMLException(f"Invalid parallelism: {parts}")
    per = n_total // parts
    return [per] * (parts - 1) + [n_total - per * (parts - 1)]


def record_bytes(fp64: bool = False) -> int:
    return int(_lib.lib.skml_sketch_record_bytes(1 if fp64 else 0))


def sketch_shard(values, shard_sizes, shard: int, seed: int = 0) -> torch.Tensor:
    """This rank's slice sketch as a fixed-size device record (skml_dense_sketch_shard_f32 / _f64:
    fp64 values, the reference's double[], stay fp64)."""
    x = as_device_values(values)
    wide = x.dtype == torch.float64
    sizes = np.ascontiguousarray(shard_sizes, dtype=np.int64)
    rec = torch.empty(record_bytes(wide), dtype=torch.uint8, device=x.device)
    ctx = get_context(x.device)
    fn = _lib.lib.skml_dense_sketch_shard_f64 if wide else _lib.lib.skml_dense_sketch_shard_f32
    check(fn(ctx.handle, C.c_void_p(x.data_ptr()), x.numel(), sizes.ctypes.data_as(_lib.i64p), len(sizes),
             int(shard), int(seed), C.c_void_p(rec.data_ptr())), "sketch_shard")
    return rec


def quantize_sharded(values, shard_sizes, shard: int, records: torch.Tensor, binNum: int = 256, seed: int = 0,
                     dedup: bool = False):
    """QuantileQuantizer of shard `shard` against the merged sketch of all shards' records."""
    from .quantization import QuantileQuantizer
    q = QuantileQuantizer(binNum, seed)
    q._encode_sharded(values, shard_sizes, shard, records, dedup)
    return q


def parallel_quantize_across_ranks(values, n_total: int, binNum: int = 256, seed: int = 0, group=None,
                                   exchange: Optional[PayloadExchange] = None):
    """parallelQuantize with T = world size over one logical gradient of n_total values whose
    rank-r slice (parallel_slices) is `values` on this rank's GPU: sketch, all-gather the
    records in rank order (RCCL, via `exchange` or the torch process group), merge, quantise."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    sizes = parallel_slices(n_total, world)
    rec = sketch_shard(values, sizes, rank, seed)
    nb = rec.numel()
    allrec = torch.empty(nb * world, dtype=torch.uint8, device=rec.device)
    if exchange is not None:
        exchange.allgather(rec, nb, allrec)
    elif dist.get_backend(group) == "nccl":  # RCCL; its stream waits on the codec's (current) stream
        dist.all_gather_into_tensor(allrec, rec, group=group)
    else:  # a host-memory process group (gloo): the records (~13 KB each) go through the host
        parts = [torch.empty(nb, dtype=torch.uint8) for _ in range(world)]
        dist.all_gather(parts, rec.cpu(), group=group)
        allrec.copy_(torch.cat(parts))
    return quantize_sharded(values, sizes, rank, allrec, binNum, seed)
