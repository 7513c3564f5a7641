"""GPU parity of the sparse codec (SketchGradient.fromSparse / SparseVectorCompressor path) against
the CPU restatement.

Bar (SURVEY.md §8c "Sparse"): compaction keys/values exact; quantizer header and splits equal;
per group: size, colNum, hash ids, MinMaxSketch table, DeltaAdaptive choice, bit lengths and
BitSet words bit-exact; restore() keys and bins exact; decoded values = (float) quantValues[bin].
All device work goes through libskml.so; the oracle is only the checker.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _sparse_data(dim, density, seed, kind="normal"):
    rng = np.random.default_rng(seed)
    mask = rng.random(dim) < density
    keys = np.nonzero(mask)[0].astype(np.int32)
    if kind == "normal":
        vals = rng.standard_normal(len(keys)).astype(np.float32)
    elif kind == "positive":
        vals = (np.abs(rng.standard_normal(len(keys))) + 0.1).astype(np.float32)
    elif kind == "negative":
        vals = (-np.abs(rng.standard_normal(len(keys))) - 0.1).astype(np.float32)
    elif kind == "dups":
        vals = rng.integers(-4, 5, len(keys)).astype(np.float32)
    else:
        raise ValueError(kind)
    return keys, vals


def _check_sparse(gpu, keys, vals, bins=256, groups=8, rows=2, ratio=0.3, seed=0, hash_seed=0):
    pl = gpu.encode_sparse(torch.from_numpy(keys).cuda(), torch.from_numpy(vals).cuda(), bins, groups, rows,
                           ratio, seed, hash_seed)
    osp = O.sparse_compress(keys, vals.astype(np.float64), bins, groups, rows, ratio, seed, hash_seed)
    hdr, splits = pl.quant_header()
    assert hdr.bin_num == osp.q.bin_num and hdr.zero_idx == osp.q.zero_idx
    assert hdr.min == osp.q.min and hdr.max == osp.q.max
    assert np.array_equal(splits, osp.q.splits)
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
        assert gg["num_intervals"] == d["num_intervals"] and gg["flag_kind"] == d["flag_kind"]
        assert gg["n_flag_bits"] == d["n_flag_bits"] and gg["n_delta_bits"] == d["n_delta_bits"]
        assert np.array_equal(gg["flag_words"], d["flag_words"]), g
        assert np.array_equal(gg["delta_words"], d["delta_words"]), g
    rk, rv = pl.restore()
    ok, ob = osp.restore()
    assert np.array_equal(rk.cpu().numpy(), ok)
    want = osp.q.values()[ob].astype(np.float32)
    assert np.array_equal(rv.cpu().numpy().view(np.uint32), want.view(np.uint32))
    return pl, osp


@pytest.mark.parametrize("dim,density", [(1000, 0.5), (50000, 0.1), (300000, 0.02), (2**20 + 77, 0.1)])
def test_sparse_matches_oracle(gpu, dim, density):
    keys, vals = _sparse_data(dim, density, dim)
    _check_sparse(gpu, keys, vals, seed=dim, hash_seed=3)


@pytest.mark.parametrize("kind", ["positive", "negative", "dups"])
def test_sparse_edge_values(gpu, kind):
    """positive: zeroIdx 0 -> group 0 empty (null sketch); negative: zeroIdx B-1; dups: dedup'd
    bins and many equal distances (MinMax tie rule)."""
    keys, vals = _sparse_data(40000, 0.3, 11, kind)
    _check_sparse(gpu, keys, vals, seed=5, hash_seed=1)


@pytest.fixture(params=["one_pass", pytest.param("one_pass_plain", marks=pytest.mark.ab),
                        pytest.param("persistent_query", marks=pytest.mark.ab),
                        pytest.param("bounds_pass", marks=pytest.mark.ab),
                        pytest.param("dec_lookback", marks=pytest.mark.ab),
                        pytest.param("dec_lookback_scan", marks=pytest.mark.ab), "rounds"])
def merge_form(request):
    """restore in every form (the A/B-build-only ones marked `ab`).  one_pass (the default): tiles of one group through the compile-time-hash
    query (k_dec_keys MODE 1) and the edge tiles through the generic one, Sort.merge as the
    one-pass key-range merge with the next range's loads in flight.  one_pass_plain: the same merge
    without that prefetch.  persistent_query: the compile-time-hash query in persistent workgroups
    (A/B form, slower at 2^28).  bounds_pass: the key ranges' bounds from k_rs_bounds instead of the
    key query.  dec_lookback: the bit lengths and deltas in one pass with decoupled look-backs (A/B
    form, slower); dec_lookback_scan: the same with the deltas' tile prefixes from a scan after it.
    rounds: the round-3 forms forced through skml_debug_form (one generic
    query per row for every tile, the pairwise merge rounds, which are also the fallback for
    irregular input)."""
    from sketchml_amd import _lib
    forms = {"rs_rounds": 1, "dec_rows_serial": 1} if request.param == "rounds" else \
        {"rs_rounds": 2} if request.param == "one_pass_plain" else \
        {"dec_rows_serial": 2} if request.param == "persistent_query" else \
        {"run_bounds": 1} if request.param == "bounds_pass" else \
        {"dec_lookback": 1} if request.param == "dec_lookback" else \
        {"dec_lookback": 2} if request.param == "dec_lookback_scan" else {}
    with _lib.forced_forms(**forms):
        yield request.param


def _merge_path():
    from sketchml_amd import _lib
    return _lib.lib.skml_debug_sparse_merge_path()


@pytest.mark.parametrize("form", ["runs", "ballot"])
def test_partition_scatter_forms(gpu, form):
    """The partition scatter's few-groups forms: per-thread runs of 8 elements ranked from packed
    per-group counts (default) and the ballot-ranked form (SKML_FORM_PART_BALLOT); ragged last
    tile, 2 to 8 groups, 8- and 16-bit codes."""
    from sketchml_amd import _lib
    with _lib.forced_forms(part_ballot=1 if form == "ballot" else 0):
        for groups, bins, dim in ((8, 256, 200003), (2, 16, 70001), (5, 512, 99991)):
            keys, vals = _sparse_data(dim, 0.2, groups + dim, "normal")
            _check_sparse(gpu, keys, vals, bins, groups, 2, 0.3, seed=groups, hash_seed=bins)


@pytest.mark.parametrize("groups,rows,ratio,bins", [(2, 1, 0.3, 256), (4, 3, 0.5, 64), (16, 8, 0.1, 1024),
                                                    (64, 2, 0.3, 4096), (8, 2, 1.7, 16), (3, 1, 0.3, 128),
                                                    (5, 2, 0.3, 256), (7, 3, 0.2, 512)])
def test_sparse_shapes(gpu, groups, rows, ratio, bins, merge_form):
    """Odd group counts leave an unpaired run in restore's Sort.merge rounds."""
    keys, vals = _sparse_data(120000, 0.15, groups * 100 + rows, "normal")
    _check_sparse(gpu, keys, vals, bins, groups, rows, ratio, seed=7, hash_seed=groups)
    assert _merge_path() == (2 if merge_form == "rounds" else 1)


@pytest.mark.parametrize("groups", [7, 8])
def test_sparse_restore_many_merge_tiles(gpu, groups, merge_form):
    """~630 K keys: every Sort.merge round spans ~150 merge tiles of 4,096 outputs, with tile
    boundaries inside and at the ends of the merged pairs (k_merge_splits); the one-pass merge
    covers 257 key ranges of 8,192 keys, ~2.5 K keys each."""
    keys, vals = _sparse_data(2**21 + 3, 0.3, 40 + groups, "normal")
    _check_sparse(gpu, keys, vals, 256, groups, 2, 0.3, seed=11, hash_seed=groups)
    assert _merge_path() == (2 if merge_form == "rounds" else 1)


@pytest.mark.parametrize("layout", ["range_edges", "full_ranges", "far_apart", "int_max"])
def test_sparse_restore_key_ranges(gpu, layout, merge_form):
    """Keys placed against the one-pass merge's 8,192-key ranges: on and next to range edges
    (0, 8191, 8192, ...), whole ranges filled (every bitmap bit set, ranges of 8,192
    elements), keys ranges apart up to 2^31 - 2 (empty ranges between, a run's bounds filled over
    a gap), and a key of INT32_MAX, which Sort.merge never selects (its `< Integer.MAX_VALUE`
    test): the one-pass form hands that input to the rounds (path 3), whose result the oracle
    states."""
    rng = np.random.default_rng(len(layout))
    if layout == "range_edges":
        e = np.arange(1, 40, dtype=np.int64) * 8192
        keys = np.unique(np.concatenate([[0, 1, 8190, 8191], e - 1, e, e + 1, 2**31 - 8192 + np.arange(-2, 3)]))
    elif layout == "full_ranges":
        keys = np.arange(3 * 65536 + 100, dtype=np.int64) + 65536
    elif layout == "far_apart":
        keys = np.unique(np.concatenate([rng.integers(0, 2**31 - 1, 3000), [2**31 - 2, 0, 8192 * 262143]]))
    else:
        keys = np.unique(np.concatenate([rng.integers(0, 2**20, 5000), [2**31 - 2, 2**31 - 1]]))
    keys = keys.astype(np.int32)
    vals = rng.standard_normal(len(keys)).astype(np.float32)
    pl, osp = _check_sparse(gpu, keys, vals, 256, 8, 2, 0.3, seed=3, hash_seed=4)
    rk, rb = pl.restore_bins()
    ok, ob = osp.restore()
    assert np.array_equal(rk.cpu().numpy(), ok) and np.array_equal(rb.cpu().numpy(), ob)
    if merge_form == "rounds":
        assert _merge_path() == 2
    else:
        assert _merge_path() == (3 if layout == "int_max" else 1)


def test_sparse_key_gaps_choose_each_interval_kind(gpu):
    """Wide and mixed key gaps so groups pick different (numIntervals, flagKind) and the first key
    is 0 (delta 0 needs 1 bit)."""
    rng = np.random.default_rng(5)
    gaps = np.concatenate([rng.integers(1, 3, 3000), rng.integers(1, 1 << 20, 3000), rng.integers(1, 40, 3000)])
    keys = np.concatenate([[0], np.cumsum(gaps)]).astype(np.int32)
    vals = rng.standard_normal(len(keys)).astype(np.float32)
    pl, osp = _check_sparse(gpu, keys, vals, 256, 8, 2, 0.3, 1, 2)
    kinds = {(d["num_intervals"], d["flag_kind"]) for d in osp.deltas if d is not None}
    assert len(kinds) >= 2


def test_sparse_empty(gpu):
    keys = np.zeros(0, np.int32)
    vals = np.zeros(0, np.float32)
    pl = gpu.encode_sparse(torch.from_numpy(keys).cuda(), torch.from_numpy(vals).cuda())
    assert pl.nnz() == 0
    k, v = pl.restore()
    assert k.numel() == 0 and v.numel() == 0


def test_sparse_rejects_non_increasing_keys(gpu):
    """DeltaAdaptiveEncoder.encode throws "Log for" only when a group's own keys do not ascend
    (Maths.log2nlz); all-positive values put every key in group 1 (edges {zeroIdx=0, B})."""
    keys = np.array([5, 9, 9, 12, 40, 41], dtype=np.int32)
    vals = np.array([0.5, 1, 2, 0.25, 0.75, 1], dtype=np.float32)
    with pytest.raises(O.OracleError):
        O.sparse_compress(keys, vals.astype(np.float64), 4, 2)
    with pytest.raises(gpu.SketchMLException, match="Log for"):
        gpu.encode_sparse(torch.from_numpy(keys).cuda(), torch.from_numpy(vals).cuda(), 4, 2)


def test_sparse_duplicate_keys_across_groups_are_kept(gpu, merge_form):
    """A key repeated in two different groups is legal for the reference (each group ascends);
    Sort.merge then emits the lower group's copy first.  The one-pass merge sees the repeated bit
    and hands the payload to the merge rounds (path 3)."""
    keys = np.array([5, 9, 9, 12, 40, 41], dtype=np.int32)
    vals = np.array([0.5, -1, 2, 0.25, -0.5, 1], dtype=np.float32)
    pl, osp = _check_sparse(gpu, keys, vals, 4, 2, 1, 0.5, 1, 1)
    assert _merge_path() == (2 if merge_form == "rounds" else 3)
    rk, rb = pl.restore_bins()
    ok, ob = osp.restore()
    assert np.array_equal(rk.cpu().numpy(), ok) and np.array_equal(rb.cpu().numpy(), ob)
    assert _merge_path() == (2 if merge_form == "rounds" else 3)


def test_sparse_length_mismatch(gpu):
    with pytest.raises(gpu.SketchMLException, match="do not match"):
        gpu.SparseVectorCompressor().compressSparse(torch.arange(5, dtype=torch.int32).cuda(),
                                                    torch.ones(4, device="cuda"))


def test_compaction_exact(gpu):
    rng = np.random.default_rng(3)
    for dim in (1, 4095, 4096, 4097, 16383, 16384, 16385, 3 * 16384 + 5, 2**18 + 3, 2**22 + 1234):
        x = rng.standard_normal(dim).astype(np.float32)
        r = rng.random(dim)
        x[r < 0.5] = 0.0
        x[(r >= 0.5) & (r < 0.55)] = np.float32(1e-8)              # not > 1e-8 (double compare)
        x[(r >= 0.55) & (r < 0.6)] = np.nextafter(np.float32(1e-8), np.float32(1))
        x[(r >= 0.6) & (r < 0.62)] = -np.float32(2e-9)
        x[(r >= 0.62) & (r < 0.63)] = np.nan                        # |NaN| > EPS is false
        k, v = gpu.to_sparse(torch.from_numpy(x).cuda())
        want = np.nonzero(np.abs(x.astype(np.float64)) > 1e-8)[0]
        assert np.array_equal(k.cpu().numpy(), want)
        assert np.array_equal(v.cpu().numpy().view(np.uint32), x[want].view(np.uint32))


@pytest.mark.parametrize("dim,density", [(65535, 0.1), (65536, 0.1), (65537, 0.05), (5 * 65536 + 77, 0.1),
                                         (2**21 + 9, 0.124), (2**21 + 9, 0.13), (3 * 65536, 0.0),
                                         (2**26 + 9, 0.1), (2**26 + 9, 0.125), (2**26 + 9, 0.13)])
def test_compaction_big_tiles(gpu, dim, density):
    """The 65,536-value tiles of k_compact_big: kept values staged in LDS up to 8,192 per tile (a
    tile above that re-reads its input), partial last tiles, all-zero input.  At 2^26 + 9 there
    are more tiles (1,025) than resident workgroups (3 per CU), so each persistent workgroup takes
    a second tile (prefetched during its first tile's stores) and looks back across tiles held by
    other workgroups; at densities around and above 1/8 some or all tiles take the re-read path."""
    rng = np.random.default_rng(dim)
    x = np.where(rng.random(dim) < density, rng.standard_normal(dim), 0.0).astype(np.float32)
    x[rng.random(dim) < 0.001] = np.float32(1e-8)
    k, v = gpu.to_sparse(torch.from_numpy(x).cuda())
    want = np.nonzero(np.abs(x.astype(np.float64)) > 1e-8)[0]
    assert np.array_equal(k.cpu().numpy(), want)
    assert np.array_equal(v.cpu().numpy().view(np.uint32), x[want].view(np.uint32))


def test_dense_as_sparse_matches_oracle(gpu):
    rng = np.random.default_rng(8)
    dim = 400000
    x = np.where(rng.random(dim) < 0.1, rng.standard_normal(dim), 0.0).astype(np.float32)
    pl = gpu.encode_dense_as_sparse(torch.from_numpy(x).cuda(), 256, 8, 2, 0.3, 4, 9)
    keys, vals = O.to_sparse(x.astype(np.float64))
    osp = O.sparse_compress(keys, vals, 256, 8, 2, 0.3, 4, 9)
    rk, rv = pl.restore()
    ok, ob = osp.restore()
    assert np.array_equal(rk.cpu().numpy(), ok)
    assert np.array_equal(rv.cpu().numpy(), osp.q.values()[ob].astype(np.float32))


def test_sparse_vector_compressor_surface(gpu):
    keys, vals = _sparse_data(30000, 0.2, 21)
    c = gpu.SparseVectorCompressor(quantBinNum=128, seed=2, hashSeed=4)
    c.compressSparse(keys, vals)
    assert c.size() == len(keys)
    k, v = c.decompressSparse()
    osp = O.sparse_compress(keys, vals.astype(np.float64), 128, 8, 2, 0.3, 2, 4)
    ok, ob = osp.restore()
    assert np.array_equal(k.cpu().numpy(), ok)
    dense = c.decompressDense()
    assert dense.numel() == int(keys.max()) + 1
    assert np.array_equal(dense.cpu().numpy()[ok], osp.q.values()[ob].astype(np.float32))
    c.timesBy(0.5)
    c.timesBy(3.0)
    _, v2 = c.decompressSparse()
    qv = osp.q.values() * 0.5 * 3.0   # quantValues[i] *= x, twice (SparseVectorCompressor.java:128-134)
    assert np.array_equal(v2.cpu().numpy(), qv[ob].astype(np.float32))


@pytest.mark.parametrize("case", ["dense", "wide", "mixed", "single", "zero_first"])
def test_delta_adaptive_matches_oracle(gpu, case):
    rng = np.random.default_rng(len(case))
    if case == "dense":
        keys = np.cumsum(rng.integers(1, 3, 100000))
    elif case == "wide":
        keys = np.cumsum(rng.integers(1, 1 << 24, 5000))
    elif case == "mixed":
        keys = np.cumsum(np.where(rng.random(70000) < 0.9, rng.integers(1, 8, 70000), rng.integers(1, 1 << 16, 70000)))
    elif case == "single":
        keys = np.array([123456])
    else:
        keys = np.concatenate([[0], np.cumsum(rng.integers(1, 100, 3000))])
    keys = keys.astype(np.int32)
    enc = gpu.DeltaAdaptiveEncoder()
    enc.encode(torch.from_numpy(keys).cuda())
    want = O.delta_encode(keys)
    assert enc.numIntervals == want["num_intervals"] and enc.flagKind == want["flag_kind"]
    assert enc.nFlagBits == want["n_flag_bits"] and enc.nDeltaBits == want["n_delta_bits"]
    assert np.array_equal(enc.flagWords.cpu().numpy().view(np.uint64), want["flag_words"])
    assert np.array_equal(enc.deltaWords.cpu().numpy().view(np.uint64), want["delta_words"])
    assert np.array_equal(enc.decode().cpu().numpy(), keys)


def test_c3_size_properties(gpu):
    """BASELINE C3 (2^28-dim dense, 10 % nnz): P5 keys round-trip exactly, P6 the MinMax bin is
    never farther from zeroIdx than the element's own bin, decoded values come from the LUT."""
    dim = 2**28
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(dim, device="cuda", generator=g)
    x[torch.rand(dim, device="cuda", generator=g) >= 0.1] = 0.0
    keys, vals = gpu.to_sparse(x)
    pl = gpu.encode_sparse(keys, vals, 256, 8, 2, 0.3, 3, 3)
    rk, rv = pl.restore()
    assert torch.equal(rk, keys)                                        # P5
    hdr, splits = pl.quant_header()
    sp = torch.from_numpy(splits).cuda().float()
    true_bins = torch.searchsorted(sp, vals, right=True)
    lut = torch.from_numpy(pl.values()).cuda()
    got_bins = torch.searchsorted(lut.float(), rv)  # rv is a LUT entry; recover its bin
    assert torch.equal(lut.float()[got_bins], rv)
    z = hdr.zero_idx
    assert torch.all((got_bins - z).abs() <= (true_bins - z).abs())     # P6
    del x


def _parse_sparse_stream(b):
    """Reader of skml_sparse_serialize's field stream (GroupedMinMaxSketch.writeObject order)."""
    import struct
    off = 0

    def take(fmt):
        nonlocal off
        v = struct.unpack_from(fmt, b, off)[0]
        off += struct.calcsize(fmt)
        return v

    head = dict(G=take(">i"), rows=take(">i"), ratio=take(">d"), B=take(">i"), zero=take(">i"))
    sketches, encoders = [], []
    for _ in range(head["G"]):
        if not take(">B"):
            sketches.append(None)
            continue
        sk = dict(rows=take(">i"), cols=take(">i"), zero=take(">i"))
        sk["hashes"] = [(take(">i"), take(">i"), take(">i")) for _ in range(sk["rows"])]
        sk["items"] = [(take(">i"), take(">i"), take(">i")) for _ in range(take(">i"))]
        sk["longs"] = np.array([take(">Q") for _ in range(take(">i"))], dtype=np.uint64)
        sk["size"] = take(">i")
        sketches.append(sk)
    for _ in range(head["G"]):
        if not take(">B"):
            encoders.append(None)
            continue
        e = dict(size=take(">i"), m=take(">i"), kind=bool(take(">B")))
        e["flags"] = np.array([take(">Q") for _ in range(take(">i"))], dtype=np.uint64)
        e["deltas"] = np.array([take(">Q") for _ in range(take(">i"))], dtype=np.uint64)
        encoders.append(e)
    assert off == len(b)
    return head, sketches, encoders


@pytest.mark.parametrize("bins,groups,rows", [(256, 8, 2), (16, 4, 3), (1024, 2, 1)])
def test_sparse_serialize_matches_oracle(gpu, bins, groups, rows):
    """A14: the field stream carries each group's MinMaxSketch (hash ids, HuffmanEncoder of the
    table: items + BitSet words + size) and DeltaAdaptiveEncoder, equal to the oracle's."""
    keys, vals = _sparse_data(80000, 0.15, bins + groups, "normal")
    pl, osp = _check_sparse(gpu, keys, vals, bins, groups, rows, 0.3, 2, 5)
    head, sketches, encoders = _parse_sparse_stream(pl.serialize())
    assert (head["G"], head["rows"], head["ratio"], head["B"], head["zero"]) == \
        (groups, rows, 0.3, osp.q.bin_num, osp.q.zero_idx)
    bkdr = {3: 31, 4: 131, 5: 267, 6: 1313, 7: 13131}
    for g in range(groups):
        if osp.tables[g] is None:
            assert sketches[g] is None and encoders[g] is None
            continue
        sk = sketches[g]
        assert (sk["rows"], sk["cols"], sk["zero"], sk["size"]) == (rows, osp.col_num[g], osp.q.zero_idx,
                                                                   rows * osp.col_num[g])
        assert sk["hashes"] == [(int(h), int(osp.col_num[g]), bkdr.get(int(h), 0)) for h in osp.hash_ids[g]]
        want = O.huffman_encode(osp.tables[g])
        assert sk["items"] == [tuple(int(v) for v in it) for it in want["items"]]
        assert np.array_equal(sk["longs"], want["words"])
        assert np.array_equal(want["decoded"], osp.tables[g])        # the oracle's own round trip
        d = osp.deltas[g]
        e = encoders[g]
        assert (e["size"], e["m"], e["kind"]) == (d["size"], d["num_intervals"], d["flag_kind"])
        assert np.array_equal(e["flags"], d["flag_words"]) and np.array_equal(e["deltas"], d["delta_words"])


@pytest.mark.parametrize("kind", ["normal", "positive", "dups"])
def test_sparse_uniform_quantizer_matches_oracle(gpu, kind):
    """SparseVectorCompressor with QuantizationType.UNIFORM (SparseVectorCompressor.java:60-62):
    uniform splits, then the same grouped MinMax sketch and DeltaAdaptive keys."""
    keys, vals = _sparse_data(120000, 0.1, 77, kind)
    c = gpu.SparseVectorCompressor(gpu.QuantizationType.UNIFORM, 128, seed=1, hashSeed=2)
    c.compressSparse(torch.from_numpy(keys).cuda(), torch.from_numpy(vals).cuda())
    osp = O.sparse_compress(keys, vals.astype(np.float64), 128, 8, 2, 0.3, 1, 2, uniform=True)
    hdr, splits = c.mmSketches.payload.quant_header()
    assert hdr.bin_num == osp.q.bin_num == 128 and hdr.zero_idx == osp.q.zero_idx
    assert np.array_equal(splits, osp.q.splits)
    for g in range(8):
        gg = c.mmSketches.payload.group(g)
        assert gg["size"] == osp.group_size[g]
        if osp.tables[g] is not None:
            assert np.array_equal(gg["table"], osp.tables[g]), g
    k, v = c.decompressSparse()
    ok, ob = osp.restore()
    assert np.array_equal(k.cpu().numpy(), ok)
    assert np.array_equal(v.cpu().numpy(), osp.q.values()[ob].astype(np.float32))
