"""Probe: a world-2 RCCL communicator with both ranks on one GPU (the N > 1 exchange of bench.py's
multi-GPU step, rehearsed on a one-GPU box).  Each rank encodes its own 2^22-float bucket (seed
10 + rank), the payloads are all-gathered over RCCL and every rank decodes the sum; the result is
compared with the sum of both payloads decoded locally.  Prints one JSON line per rank.
usage: python tools/rccl_two_rank_probe.py
"""
import ctypes as C
import json
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sketchml_amd as sk
    from sketchml_amd import _lib, distributed as D
    lib = _lib.lib
    ctx = sk.get_context(0).handle
    n = 1 << 22
    nb = lib.skml_dense_payload_bytes(n, 256)
    stride = (nb + 255) // 256 * 256
    p = _lib.Params()
    lib.skml_params_default(C.byref(p))
    p.bin_num = 256
    pls = []
    for r in range(world):
        g = torch.Generator(device="cuda").manual_seed(10 + r)
        x = torch.randn(n, device="cuda", generator=g)
        pl = sk.alloc_aligned(stride, "cuda")
        p.seed = 10 + r
        assert lib.skml_dense_encode_f32(ctx, C.c_void_p(x.data_ptr()), n, C.byref(p), C.c_void_p(pl.data_ptr()),
                                         stride) == 0, _lib.last_error()
        pls.append(pl)
    ex = D.PayloadExchange(ctx)
    allp = sk.alloc_aligned(stride * world, "cuda")
    ex.allgather(pls[rank], stride, allp)
    out = torch.empty(n, dtype=torch.float32, device="cuda")
    D.decode_sum(ctx, allp, world, stride, n, 1.0 / world, out)
    want = torch.empty(world * stride, dtype=torch.uint8, device="cuda")
    for r in range(world):
        want[r * stride:(r + 1) * stride].copy_(pls[r][:stride])
    ref = torch.empty(n, dtype=torch.float32, device="cuda")
    D.decode_sum(ctx, want, world, stride, n, 1.0 / world, ref)
    torch.cuda.synchronize()
    ex.close()
    print(json.dumps({"rank": rank, "world": world, "gathered_equal": bool(torch.equal(allp[:world * stride], want)),
                      "sum_equal": bool(torch.equal(out, ref))}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    mp.spawn(run, args=(2, 29613), nprocs=2)
