"""World-size-2 gloo tests of the multi-GPU control plane (sketchml_amd/distributed.py) on CPU:
unique-id broadcast, payload-size agreement, bucket sharding.  The RCCL data path itself
(skml_comm_init_rank + skml_allgather) runs on the GPU box with a world-size-1 communicator in
tests/test_gpu_configs.py (byte-identical copy, PayloadExchange + decode_sum, and the C4
eight-bucket all-gather layout), and with N ranks in bench.py --gpus N."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from sketchml_amd import distributed as D
        uid = D.broadcast_unique_id(lambda: bytes(range(128)))
        lo, hi = D.shard_range(2**30, world, rank)
        sizes = D.agree_sizes(1000 + 17 * rank)
        q.put((rank, uid, lo, hi, sizes))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_control_plane():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    uids = {r[1] for r in res}
    assert uids == {bytes(range(128))}                       # every rank got rank 0's id
    assert res[0][2] == 0 and res[0][3] == res[1][2] and res[1][3] == 2**30  # contiguous shards
    assert res[0][4] == res[1][4] == [1000, 1017]            # same size table everywhere


@pytest.mark.parametrize("n,world", [(10, 3), (2**26, 8), (2**30, 8), (7, 8)])
def test_shard_range_partitions(n, world):
    from sketchml_amd.distributed import shard_range
    spans = [shard_range(n, world, r) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == n
    assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))


@pytest.mark.parametrize("n,world", [(10, 3), (2**26 + 5, 8), (7, 8), (0, 2)])
def test_parallel_slices_are_the_parallelquantize_slicing(n, world):
    """QuantileQuantizer.java:66-68: n/T per slice, the last takes the remainder; the same
    split as the bucket sharding."""
    from sketchml_amd.distributed import parallel_slices, shard_range
    sizes = parallel_slices(n, world)
    assert sum(sizes) == n and all(s == n // world for s in sizes[:-1])
    assert sizes == [hi - lo for lo, hi in (shard_range(n, world, r) for r in range(world))]


def _blob_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from sketchml_amd import distributed as D
        nbytes = 1000 + 700 * rank                      # variable-size payloads
        stride = D.blob_stride(D.agree_sizes(nbytes))
        local = torch.zeros(stride, dtype=torch.uint8)
        local[:nbytes] = (rank + 1) % 256
        allb = D.gather_blobs(local, stride)
        q.put((rank, stride, allb.numpy().copy()))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_padded_blob_gather():
    """Sparse payloads differ in size: sizes are agreed first, each rank's blob goes in a slot of
    the largest size rounded to 256 bytes, and slot r holds rank r's bytes on every rank."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_blob_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    stride = (1700 + 255) // 256 * 256
    for rank, st, allb in res:
        assert st == stride and len(allb) == world * stride
        for r in range(world):
            n = 1000 + 700 * r
            assert (allb[r * stride: r * stride + n] == r + 1).all()
            assert (allb[r * stride + n: (r + 1) * stride] == 0).all()
