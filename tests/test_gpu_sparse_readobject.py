"""GPU parity of the sparse read side: GroupedMinMaxSketch.readObject (GroupedMinMaxSketch.java:
161-172) with MinMaxSketch / HuffmanEncoder / DeltaAdaptiveEncoder readObject (MinMaxSketch.java:
99-108, HuffmanEncoder.java:127-166,193-207, DeltaAdaptiveEncoder.java:172-188).

Bar: a stream written by skml_sparse_serialize (whose bytes equal the oracle's field stream,
tests/test_gpu_sparse.py::test_sparse_serialize_matches_oracle) reads back into a device payload
whose restore() keys and bins equal the oracle's restore() exactly, and which serialises to the
same bytes again.  The Huffman tables are decoded on the device by the speculative parallel
decoder; the large cases span hundreds of 2048-bit segments, so resynchronisation is exercised.
The oracle is only the checker.
"""
import struct

import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _data(dim, density, seed, kind="normal"):
    rng = np.random.default_rng(seed)
    keys = np.nonzero(rng.random(dim) < density)[0].astype(np.int32)
    if kind == "normal":
        vals = rng.standard_normal(len(keys)).astype(np.float32)
    elif kind == "dups":
        vals = rng.integers(-3, 4, len(keys)).astype(np.float32)
    elif kind == "const":
        vals = np.full(len(keys), 0.5, dtype=np.float32)
    else:
        raise ValueError(kind)
    return keys, vals


@pytest.mark.parametrize("dim,density,bins,groups,rows,kind", [
    (50000, 0.2, 256, 8, 2, "normal"),
    (2**20 + 77, 0.1, 256, 8, 2, "normal"),      # ~0.3 M cells per table: many segments
    (300000, 0.3, 1024, 4, 3, "normal"),         # long codes (> 12 bits) go through the tree walk
    (80000, 0.15, 16, 2, 1, "dups"),
    (20000, 0.1, 64, 16, 8, "normal"),
    (40000, 0.05, 256, 2, 2, "const"),           # bin_num 2: one- or two-symbol tables
])
def test_read_object_round_trip(gpu, dim, density, bins, groups, rows, kind):
    keys, vals = _data(dim, density, dim % 1000 + bins, kind)
    pl = gpu.encode_sparse(torch.from_numpy(keys).cuda(), torch.from_numpy(vals).cuda(), bins, groups, rows,
                           0.3, 3, 4)
    osp = O.sparse_compress(keys, vals.astype(np.float64), bins, groups, rows, 0.3, 3, 4)
    data = pl.serialize()
    # keys + bins (GroupedMinMaxSketch.restore) from the stream alone
    sk = gpu.GroupedMinMaxSketch.readObject(data)
    rk, rb = sk.restore()
    ok, ob = osp.restore()
    assert np.array_equal(rk.cpu().numpy(), ok)
    assert np.array_equal(rb.cpu().numpy(), ob)
    assert (sk.groupNum, sk.rowNum, sk.binNum, sk.zeroValue) == (groups, rows, osp.q.bin_num, osp.q.zero_idx)
    # with quantValues: the full SparseVectorCompressor.decompressSparse
    back = gpu.SparsePayload.deserialize(data, osp.q.values())
    k2, v2 = back.restore()
    assert np.array_equal(k2.cpu().numpy(), ok)
    assert np.array_equal(v2.cpu().numpy(), osp.q.values()[ob].astype(np.float32))
    # the decoded MinMax tables re-serialise to the same bytes
    assert back.serialize() == data
    for g in range(groups):
        if osp.tables[g] is not None:
            assert np.array_equal(back.group(g)["table"], osp.tables[g]), g


def test_read_object_rejects_malformed(gpu):
    keys, vals = _data(30000, 0.2, 1)
    pl = gpu.encode_sparse(torch.from_numpy(keys).cuda(), torch.from_numpy(vals).cuda(), 256, 8, 2, 0.3, 1, 1)
    data = pl.serialize()
    with pytest.raises(gpu.SketchMLException):
        gpu.SparsePayload.deserialize(data[: len(data) // 2])
    bad = bytearray(data)
    bad[0:4] = struct.pack(">i", 1000)  # groupNum beyond the supported 64
    with pytest.raises(gpu.SketchMLException):
        gpu.SparsePayload.deserialize(bytes(bad))


def test_decode_without_values_is_refused(gpu):
    keys, vals = _data(30000, 0.2, 2)
    pl = gpu.encode_sparse(torch.from_numpy(keys).cuda(), torch.from_numpy(vals).cuda(), 256, 8, 2, 0.3, 1, 1)
    back = gpu.SparsePayload.deserialize(pl.serialize())
    with pytest.raises(gpu.SketchMLException):
        back.restore()
