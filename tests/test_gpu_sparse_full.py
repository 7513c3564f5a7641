"""Sparse codec parity at BASELINE C3's full size and on the reference's own double values.

C3: a 2^28-dim dense fp32 gradient with 10 % nnz (seed 3), 256 bins, 8 groups, 2 rows,
colRatio 0.3.  At this size a group holds ~3.4 M keys, its MinMax table ~1 M columns, and the hash
`% size` runs through the multiply-based modulus (skml_sparse.hip java_hash_fm / DivU32), so the
device path is compared element for element with the C restatement (oracle/skml_oracle.c):
quantizer header and splits, per group size / colNum / hash ids / MinMax table / DeltaAdaptive
choice, bit lengths and BitSet words, restore() keys and bins, and the serialised HuffmanEncoder
items and words of every table.

fp64 values (SketchGradient.fromSparse, SparseVectorCompressor.compressSparse on double[]): values
that are not fp32-representable must give the oracle's double split samples and bins, which an
fp32-narrowed path does not.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests.test_gpu_sparse import _check_sparse, _parse_sparse_stream

pytestmark = pytest.mark.gpu


def _compare_groups(pl, osp, groups):
    for g in range(groups):
        gg = pl.group(g)
        assert gg["size"] == osp.group_size[g], g
        if osp.tables[g] is None:
            assert gg["size"] == 0
            continue
        assert gg["col_num"] == osp.col_num[g]
        assert gg["hash_ids"] == list(osp.hash_ids[g])
        assert np.array_equal(gg["table"], osp.tables[g]), g
        d = osp.deltas[g]
        assert (gg["num_intervals"], gg["flag_kind"]) == (d["num_intervals"], d["flag_kind"]), g
        assert (gg["n_flag_bits"], gg["n_delta_bits"]) == (d["n_flag_bits"], d["n_delta_bits"]), g
        assert np.array_equal(gg["flag_words"], d["flag_words"]), g
        assert np.array_equal(gg["delta_words"], d["delta_words"]), g


def test_c3_full_size_matches_oracle(gpu):
    """Both C3 entry points at full size against one oracle result: to_sparse + encode_sparse, and
    encode_dense_as_sparse (the call bench.py times: compaction into the context's scratch, then
    encode_kv), whose keys the oracle's own toSparse (DenseDoubleGradient.scala:64-89) produces."""
    dim = 2**28
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(dim, device="cuda", generator=g)
    x[torch.rand(dim, device="cuda", generator=g) >= 0.1] = 0.0
    pl_dense = gpu.encode_dense_as_sparse(x, 256, 8, 2, 0.3, 3, 3)
    keys, vals = gpu.to_sparse(x)
    xh = x.cpu().numpy()
    del x
    pl = gpu.encode_sparse(keys, vals, 256, 8, 2, 0.3, 3, 3)
    kh, vh = keys.cpu().numpy(), vals.cpu().numpy()
    assert len(kh) > 26_000_000
    ok_keys, ok_vals = O.to_sparse(xh.astype(np.float64))
    del xh
    assert np.array_equal(kh, ok_keys) and np.array_equal(vh.astype(np.float64), ok_vals)
    osp = O.sparse_compress(ok_keys, ok_vals, 256, 8, 2, 0.3, 3, 3)
    del ok_keys, ok_vals
    # the timed entry point first: header, every group, restore
    hdr, splits = pl_dense.quant_header()
    assert (hdr.bin_num, hdr.zero_idx, hdr.min, hdr.max) == (osp.q.bin_num, osp.q.zero_idx, osp.q.min, osp.q.max)
    assert np.array_equal(splits, osp.q.splits)
    _compare_groups(pl_dense, osp, 8)
    rk, rb = pl_dense.restore_bins()
    ok, ob = osp.restore()
    assert np.array_equal(rk.cpu().numpy(), ok)
    assert np.array_equal(rb.cpu().numpy(), ob)
    del rk, rb, pl_dense
    hdr, splits = pl.quant_header()
    assert (hdr.bin_num, hdr.zero_idx, hdr.min, hdr.max) == (osp.q.bin_num, osp.q.zero_idx, osp.q.min, osp.q.max)
    assert np.array_equal(splits, osp.q.splits)
    assert int(osp.col_num.max()) > 900_000       # the large-modulus regime of the hash
    _compare_groups(pl, osp, 8)
    rk, rb = pl.restore_bins()
    assert np.array_equal(rk.cpu().numpy(), ok)
    assert np.array_equal(rb.cpu().numpy(), ob)
    del rk, rb
    _, rv = pl.restore()
    want = osp.q.values()[ob].astype(np.float32)
    assert np.array_equal(rv.cpu().numpy().view(np.uint32), want.view(np.uint32))
    # the writeObject stream: every table's HuffmanEncoder items and BitSet words
    head, sketches, encoders = _parse_sparse_stream(pl.serialize())
    assert (head["G"], head["B"], head["zero"]) == (8, osp.q.bin_num, osp.q.zero_idx)
    for gi in range(8):
        if osp.tables[gi] is None:
            assert sketches[gi] is None
            continue
        want_h = O.huffman_encode(osp.tables[gi])
        assert sketches[gi]["items"] == [tuple(int(v) for v in it) for it in want_h["items"]], gi
        assert np.array_equal(sketches[gi]["longs"], want_h["words"]), gi
        d = osp.deltas[gi]
        assert np.array_equal(encoders[gi]["flags"], d["flag_words"]) and \
            np.array_equal(encoders[gi]["deltas"], d["delta_words"]), gi


def _f64_data(dim, density, seed):
    rng = np.random.default_rng(seed)
    keys = np.nonzero(rng.random(dim) < density)[0].astype(np.int32)
    vals = rng.standard_normal(len(keys))              # doubles, almost none fp32-representable
    return keys, vals


@pytest.mark.parametrize("dim,density,bins,groups,rows", [(60000, 0.3, 256, 8, 2), (2**20 + 77, 0.1, 256, 8, 2),
                                                          (200000, 0.2, 16, 4, 3)])
def test_sparse_f64_values_match_oracle(gpu, dim, density, bins, groups, rows):
    keys, vals = _f64_data(dim, density, dim + bins)
    assert np.mean(vals.astype(np.float32).astype(np.float64) != vals) > 0.99
    pl = gpu.encode_sparse(torch.from_numpy(keys).cuda(), torch.from_numpy(vals).cuda(), bins, groups, rows, 0.3,
                           dim, 7)
    osp = O.sparse_compress(keys, vals, bins, groups, rows, 0.3, dim, 7)
    hdr, splits = pl.quant_header()
    assert (hdr.bin_num, hdr.zero_idx, hdr.min, hdr.max) == (osp.q.bin_num, osp.q.zero_idx, osp.q.min, osp.q.max)
    assert np.array_equal(splits, osp.q.splits)        # the double samples themselves
    # an fp32-narrowed encode of the same values picks different samples: the f64 path matters
    o32 = O.sparse_compress(keys, vals.astype(np.float32).astype(np.float64), bins, groups, rows, 0.3, dim, 7)
    assert not np.array_equal(o32.q.splits, osp.q.splits)
    _compare_groups(pl, osp, groups)
    rk, rb = pl.restore_bins()
    ok, ob = osp.restore()
    assert np.array_equal(rk.cpu().numpy(), ok)
    assert np.array_equal(rb.cpu().numpy(), ob)
    k64, v64 = pl.restore(torch.float64)
    assert np.array_equal(k64.cpu().numpy(), ok)
    assert np.array_equal(v64.cpu().numpy(), osp.q.values()[ob])  # quantValues[bin] in double, exact


def test_sparse_f64_dense_gradient_path(gpu):
    """DenseDoubleGradient.toAuto -> SketchGradient.fromSparse on a double[] gradient: |v| > 1e-8
    tested in double (values around EPS that an fp32 image would move across it), the doubles binned."""
    rng = np.random.default_rng(31)
    dim = 3 * 8192 * 7 + 5
    x = np.where(rng.random(dim) < 0.15, rng.standard_normal(dim), 0.0)
    r = rng.random(dim)
    x[r < 0.01] = 1e-8                                  # not > EPS
    x[(r >= 0.01) & (r < 0.02)] = 1.0000000000000002e-8  # > EPS in double; its fp32 image is below EPS
    x[(r >= 0.02) & (r < 0.025)] = -np.nextafter(1e-8, 1.0)
    x[(r >= 0.025) & (r < 0.03)] = np.nan                # |NaN| > EPS is false
    xd = torch.from_numpy(x).cuda()
    k, v = gpu.to_sparse(xd)
    want = np.nonzero(np.abs(x) > 1e-8)[0]
    assert v.dtype == torch.float64
    assert np.array_equal(k.cpu().numpy(), want)
    assert np.array_equal(v.cpu().numpy(), x[want])
    pl = gpu.encode_dense_as_sparse(xd, 256, 8, 2, 0.3, 5, 6)
    osp = O.sparse_compress(want.astype(np.int32), x[want], 256, 8, 2, 0.3, 5, 6)
    _, splits = pl.quant_header()
    assert np.array_equal(splits, osp.q.splits)
    rk, rb = pl.restore_bins()
    ok, ob = osp.restore()
    assert np.array_equal(rk.cpu().numpy(), ok) and np.array_equal(rb.cpu().numpy(), ob)


@pytest.mark.parametrize("dim", [1, 8191, 8192, 8193, 5 * 8192 + 3, 2**21 + 17])
def test_compaction_f64_exact(gpu, dim):
    rng = np.random.default_rng(dim)
    x = rng.standard_normal(dim)
    x[rng.random(dim) < 0.6] = 0.0
    k, v = gpu.to_sparse(torch.from_numpy(x).cuda())
    want = np.nonzero(np.abs(x) > 1e-8)[0]
    assert np.array_equal(k.cpu().numpy(), want)
    assert np.array_equal(v.cpu().numpy(), x[want])


def test_sparse_f64_host_entry_points(gpu):
    """skml_sparse_encode_kv_host_f64 / skml_sparse_decode_host_f64 (the JNI path of
    HipSparseVectorCompressor: int[] keys, double[] values in, double quantValues[bin] out)."""
    import ctypes as C
    from sketchml_amd import _lib
    from sketchml_amd.context import get_context
    from sketchml_amd.sparse import _params
    keys, vals = _f64_data(90000, 0.25, 4)
    p = _params(256, 8, 2, 0.3, 9, 10)
    h = C.c_void_p()
    ctx = get_context(0).handle
    assert _lib.lib.skml_sparse_encode_kv_host_f64(ctx, keys.ctypes.data_as(C.c_void_p), vals.ctypes.data_as(C.c_void_p),
                                                   len(keys), C.byref(p), C.byref(h)) == 0, _lib.last_error()
    try:
        ko = np.zeros(len(keys), np.int32)
        vo = np.zeros(len(keys), np.float64)
        assert _lib.lib.skml_sparse_decode_host_f64(ctx, h, ko.ctypes.data_as(C.c_void_p),
                                                    vo.ctypes.data_as(C.c_void_p)) == 0, _lib.last_error()
    finally:
        _lib.lib.skml_sparse_free(h)
    osp = O.sparse_compress(keys, vals, 256, 8, 2, 0.3, 9, 10)
    ok, ob = osp.restore()
    assert np.array_equal(ko, ok)
    assert np.array_equal(vo, osp.q.values()[ob])


def test_sparse_f32_still_matches(gpu):
    """fp32 values keep the fp32 kernels (encode_sparse dispatches on the value dtype)."""
    rng = np.random.default_rng(2)
    keys = np.nonzero(rng.random(50000) < 0.2)[0].astype(np.int32)
    vals = rng.standard_normal(len(keys)).astype(np.float32)
    _check_sparse(gpu, keys, vals, seed=3, hash_seed=4)


def _cal_group_edges(zero, bins, groups):
    """FSketchUtils.calGroupEdges (frequency/FSketchUtils.java:9-28)."""
    if groups == 2:
        return [zero, bins]
    bpg = bins // groups
    e = zero if zero < bpg else (bpg + zero % bpg if zero % bpg < bpg // 2 else zero % bpg)
    return [e + i * bpg for i in range(groups - 1)] + [bins]


def _has_mixed_group(zero, bins, groups):
    """A group with bins on both sides of zeroIdx: there the MinMax insert needs the key order for
    ties (the 8-byte pair path); everywhere else the device inserts 4-byte (distance, sign) pairs."""
    lo = 0
    for hi in _cal_group_edges(zero, bins, groups):
        if lo < zero < hi - 1:
            return True
        lo = max(lo, hi)
    return False


@pytest.mark.parametrize("pos_frac,mixed,dim", [(0.02, True, 200000), (0.05, True, 200000), (0.5, False, 200000),
                                                  (0.03, True, 2000003), (0.5, False, 2000003)])
def test_minmax_pair_width_paths(gpu, pos_frac, mixed, dim):
    """Mostly negative values put zeroIdx in the last group, which then holds bins on both sides of
    it (8-byte pairs, the first insert wins a distance tie); balanced values keep every group
    one-sided (4-byte pairs).  Both give the oracle's tables, bit for bit.  The larger dim spans
    several 32768-cell buckets (the 8-byte path takes each in four 8192-cell sub-ranges)."""
    rng = np.random.default_rng(5)
    keys = np.nonzero(rng.random(dim) < 0.3)[0].astype(np.int32)
    vals = -np.abs(rng.standard_normal(len(keys)))
    vals[rng.random(len(keys)) < pos_frac] *= -1
    osp = O.sparse_compress(keys, vals, 256, 8, 2, 0.3, 1, 2)
    assert _has_mixed_group(osp.q.zero_idx, osp.q.bin_num, 8) == mixed
    pl = gpu.encode_sparse(torch.from_numpy(keys).cuda(), torch.from_numpy(vals).cuda(), 256, 8, 2, 0.3, 1, 2)
    _compare_groups(pl, osp, 8)
    rk, rb = pl.restore_bins()
    ok, ob = osp.restore()
    assert np.array_equal(rk.cpu().numpy(), ok) and np.array_equal(rb.cpu().numpy(), ob)


@pytest.mark.parametrize("pos_frac,mixed", [(0.5, False), (0.03, True)])
def test_minmax_without_staging_scratch(gpu, pos_frac, mixed):
    """When the MinMax staging scratch (hashed cells, per-(tile, bucket) reservations) cannot be
    allocated, the encode falls back to key-carrying pairs and the rehashing scatter instead of
    failing (skml_debug_sparse_scratch_fail simulates the failed allocations); the tables still
    equal the oracle's."""
    from sketchml_amd import _lib
    rng = np.random.default_rng(17)
    dim = 2000003
    keys = np.nonzero(rng.random(dim) < 0.3)[0].astype(np.int32)
    vals = -np.abs(rng.standard_normal(len(keys)))
    vals[rng.random(len(keys)) < pos_frac] *= -1
    osp = O.sparse_compress(keys, vals, 256, 8, 2, 0.3, 1, 2)
    assert _has_mixed_group(osp.q.zero_idx, osp.q.bin_num, 8) == mixed
    _lib.lib.skml_debug_sparse_scratch_fail(1)
    try:
        pl = gpu.encode_sparse(torch.from_numpy(keys).cuda(), torch.from_numpy(vals).cuda(), 256, 8, 2, 0.3, 1, 2)
    finally:
        _lib.lib.skml_debug_sparse_scratch_fail(0)
    _compare_groups(pl, osp, 8)
    rk, rb = pl.restore_bins()
    ok, ob = osp.restore()
    assert np.array_equal(rk.cpu().numpy(), ok) and np.array_equal(rb.cpu().numpy(), ob)
