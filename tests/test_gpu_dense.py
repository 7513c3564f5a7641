"""GPU parity of the dense codec (QuantileQuantizer.quantize path) against the CPU restatement.

Bar: same seed -> bin_num, zero_idx, min, max and every split equal, bins
bit-exact, decoded fp32 equal to (float) of the oracle's double midpoint (so the decode L2
difference to the oracle is 0, well inside the stated tolerance of 2^-24 * ||oracle||_2).
All device work goes through libskml.so (C ABI); the oracle is only the checker.
"""
import ctypes as C

import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _data(n, seed, kind="normal"):
    rng = np.random.default_rng(seed)
    if kind == "normal":
        x = rng.standard_normal(n).astype(np.float32)
    elif kind == "app":  # sample/App.java:33-40: N(0,1) w.p. 0.9 else exactly 0
        x = np.where(rng.random(n) < 0.9, rng.standard_normal(n), 0.0).astype(np.float32)
    elif kind == "signed_zero":
        x = rng.standard_normal(n).astype(np.float32)
        r = rng.random(n)
        x[r < 0.2] = 0.0
        x[(r >= 0.2) & (r < 0.4)] = -0.0
    elif kind == "dups":
        x = rng.integers(-5, 6, n).astype(np.float32)
    elif kind == "special":
        x = rng.standard_normal(n).astype(np.float32)
        x[rng.random(n) < 0.05] = np.float32(1e-42)   # denormal
        x[rng.random(n) < 0.05] = np.float32(-1e-42)
        x[rng.random(n) < 0.01] = np.inf
        x[rng.random(n) < 0.01] = -np.inf
    elif kind == "negative":
        x = -np.abs(rng.standard_normal(n)).astype(np.float32) - 0.5
    elif kind == "positive":
        x = np.abs(rng.standard_normal(n)).astype(np.float32) + 0.5
    elif kind == "const":
        x = np.full(n, 3.25, dtype=np.float32)
    else:
        raise ValueError(kind)
    return x


def _check(gq, oq, x, check_bins=True):
    assert gq.getBinNum() == oq.bin_num
    assert gq.getZeroIdx() == oq.zero_idx
    assert gq.getMin() == oq.min and gq.getMax() == oq.max
    gs = gq.getSplits()
    assert gs.shape == oq.splits.shape
    assert np.array_equal(gs.view(np.uint64), oq.splits.view(np.uint64)) or np.array_equal(gs, oq.splits)
    if check_bins:
        gb = gq.getBins().cpu().numpy()
        assert np.array_equal(gb, oq.bins)
        dec = gq.decode().cpu().numpy()
        want = oq.values()[oq.bins].astype(np.float32)
        assert np.array_equal(dec.view(np.uint32), want.view(np.uint32))


SIZES = [1, 2, 100, 255, 256, 257, 511, 1000, 4096, 16384, 16384 + 300, 65536, 65536 * 2 + 777,
         2**20 + 12345]


@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("kind", ["normal", "app"])
def test_quantize_matches_oracle(gpu, n, kind):
    x = _data(n, n, kind)
    seed = 1000 + n
    gq = gpu.QuantileQuantizer(256, seed=seed)
    gq.quantize(torch.from_numpy(x).cuda())
    oq = O.quantize(x.astype(np.float64), 256, seed)
    _check(gq, oq, x)


@pytest.mark.parametrize("kind", ["signed_zero", "dups", "special", "negative", "positive", "const"])
@pytest.mark.parametrize("n", [300, 4096 * 3 + 11, 2**18 + 5])
def test_quantize_edge_data(gpu, kind, n):
    x = _data(n, 7 * n, kind)
    gq = gpu.QuantileQuantizer(256, seed=77)
    gq.quantize(torch.from_numpy(x).cuda())
    oq = O.quantize(x.astype(np.float64), 256, 77)
    _check(gq, oq, x)


@pytest.mark.parametrize("forms", [(0, 2), pytest.param((1, 3, 4, 5), marks=pytest.mark.ab)], ids=["shipped", "ab"])
@pytest.mark.parametrize("kind", ["normal", "signed_zero"])
def test_leaf_forms_match_oracle(gpu, kind, forms):
    """The sketch leaf's forms give the oracle's sketch, on 4,096 full tiles plus a partial one:
    the split leaf (four waves per 64-chunk tile; the default at every size, 0 and 2), and in the
    A/B build one wave per tile (1) and the hybrids that end a large bucket with split tiles (the
    last 12.5 / 25 / 50 % split).  signed_zero sends rounds through the exact (count-based) merge
    path in every form."""
    from sketchml_amd import _lib
    n = 4096 * 64 * 256 + 12345
    x = _data(n, 91, kind)
    oq = O.quantize(x.astype(np.float64), 256, 91)
    xt = torch.from_numpy(x).cuda()
    for form in forms:
        with _lib.forced_forms(leaf_split=form):
            gq = gpu.QuantileQuantizer(256, seed=91)
            gq.quantize(xt)
            _check(gq, oq, x)


def test_deferred_quantize(gpu):
    """deferred=True queues the encode without a host synchronisation and reuses the payload;
    results equal the eager path, and NaN surfaces at the first getter."""
    q = gpu.QuantileQuantizer(256, seed=3, deferred=True)
    for n, s in [(2**20 + 5, 1), (2**20 + 5, 2), (70000, 3)]:
        x = _data(n, s, "normal")
        req = q.binNum  # Quantizer.binNum becomes the effective count after each quantize (Java too)
        q.quantize(torch.from_numpy(x).cuda())
        _check(q, O.quantize(x.astype(np.float64), req, 3), x)
    x[5] = np.nan
    q.quantize(torch.from_numpy(x).cuda())  # queued: no exception yet
    with pytest.raises(gpu.QuantileSketchException):
        q.getBinNum()


def test_deferred_back_to_back_matches_eager(gpu):
    """Two deferred quantizes with no getter between them: the second runs with the binNum that
    Maths.unique reduced in the first (QuantileQuantizer.java:42), as the eager path does, and the
    first payload keeps its bytes (each encode owns its buffer)."""
    rng = np.random.default_rng(9)
    xs = [np.round(rng.standard_normal(200_003), 1).astype(np.float32) for _ in range(2)]  # ~80 distinct values
    eager = gpu.QuantileQuantizer(256, seed=4)
    lazy = gpu.QuantileQuantizer(256, seed=4, deferred=True)
    kept = []
    for x in xs:
        eager.quantize(torch.from_numpy(x).cuda())
        lazy.quantize(torch.from_numpy(x).cuda())
        kept.append((lazy.payload, eager.getBinNum(), eager.getBins().clone()))
    assert kept[0][1] < 256  # unique shrank the first encode's binNum
    assert lazy.getBinNum() == eager.getBinNum()
    assert torch.equal(lazy.getBins(), eager.getBins())
    first = gpu.QuantileQuantizer(256, seed=4)
    first.quantize(torch.from_numpy(xs[0]).cuda())
    h = first._load_header()
    used = h.codes_offset + (len(xs[0]) * h.code_bits + 7) // 8  # header, splits and codes (not the tail pad)
    assert torch.equal(kept[0][0][:used].cpu(), first.payload[:used].cpu())
    bad = torch.from_numpy(np.array([1.0, np.nan, 2.0] * 100, np.float32)).cuda()
    with pytest.raises(gpu.QuantileSketchException):
        eager.quantize(bad)
    lazy.quantize(bad)
    with pytest.raises(gpu.QuantileSketchException):
        lazy.quantize(torch.from_numpy(xs[0]).cuda())  # the queued NaN encode surfaces here
    eager.quantize(torch.from_numpy(xs[0]).cuda())
    lazy.quantize(torch.from_numpy(xs[0]).cuda())  # reported once; this one runs
    assert lazy.getBinNum() == eager.getBinNum()
    assert torch.equal(lazy.getBins(), eager.getBins())


def test_leaf_exact_path_handover(gpu):
    """The 64-keys-per-lane leaf runs a wave's rounds on a fast loop until the wave has seen both
    -0.0 and +0.0, then redoes that round and the rest on the exact-merge loop.  Zeros placed so
    that the switch happens in rounds 0..3 of different waves (16 chunks per round, 64 per wave),
    with the carry stack already holding nodes from the fast loop."""
    n = 2**20 + 4097  # 64 full 64-chunk tiles plus a partial one
    x = _data(n, 11, "normal")
    chunk = lambda tile, c: (tile * 64 + c) * 256
    for tile, c_neg, c_pos in [(1, 0, 0), (3, 20, 50), (5, 33, 34), (8, 5, 63), (9, 63, 2), (20, 47, 48)]:
        x[chunk(tile, c_neg) + 7] = -0.0
        x[chunk(tile, c_pos) + 100] = 0.0
    x[chunk(30, 12) + 1] = -0.0  # only one sign: stays on the fast loop
    for seed in (5, 6):
        gq = gpu.QuantileQuantizer(256, seed=seed)
        gq.quantize(torch.from_numpy(x).cuda())
        _check(gq, O.quantize(x.astype(np.float64), 256, seed), x)


@pytest.mark.parametrize("bins", [2, 3, 4, 16, 17, 255, 256, 1000, 4096])
def test_bin_counts_and_code_widths(gpu, bins):
    n = 3 * 2**16 + 999
    x = _data(n, bins, "normal")
    gq = gpu.QuantileQuantizer(bins, seed=bins)
    gq.quantize(torch.from_numpy(x).cuda())
    oq = O.quantize(x.astype(np.float64), bins, bins)
    _check(gq, oq, x)


def test_large_pow2_exact(gpu):
    n = 2**24  # multi-pass upper merges (tree level 16)
    x = _data(n, 5, "normal")
    gq = gpu.QuantileQuantizer(256, seed=42)
    gq.quantize(torch.from_numpy(x).cuda())
    oq = O.quantize(x.astype(np.float64), 256, 42)
    assert oq.bin_num == 129
    _check(gq, oq, x)


def test_large_ragged_exact(gpu):
    n = 2**23 + 2**21 + 2**13 + 12345  # several trees of different levels + tail
    x = _data(n, 6, "app")
    gq = gpu.QuantileQuantizer(256, seed=4242)
    gq.quantize(torch.from_numpy(x).cuda())
    oq = O.quantize(x.astype(np.float64), 256, 4242)
    _check(gq, oq, x)


def test_full_size_properties(gpu):
    """BASELINE config 2 size (2^26): size-independent properties instead of the oracle."""
    n = 2**26
    g = torch.Generator(device="cuda").manual_seed(2)
    x = torch.randn(n, device="cuda", generator=g)
    gq = gpu.QuantileQuantizer(256, seed=2)
    gq.quantize(x)
    assert gq.getBinNum() == 129                      # K2: 128 retained samples
    sp = torch.from_numpy(gq.getSplits()).to(torch.float32).cuda()
    bins = gq.getBins()
    want = torch.searchsorted(sp, x, right=True).to(torch.int32)  # P1 upper_bound
    assert torch.equal(bins, want)
    dec = gq.decode()
    vals = torch.from_numpy(gq.getValues()).cuda()
    edges = torch.cat([torch.tensor([gq.getMin()], device="cuda", dtype=torch.float64),
                       sp.double(), torch.tensor([gq.getMax()], device="cuda", dtype=torch.float64)])
    half = (edges[1:] - edges[:-1]) / 2
    err = (dec.double() - x.double()).abs()
    assert torch.all(err <= half[bins.long()] * (1 + 1e-6) + 1e-6 * dec.double().abs())  # P2 (+ fp32 rounding)
    assert torch.equal(dec, vals[bins.long()].float())
    # determinism (P4): same seed, same payload
    gq2 = gpu.QuantileQuantizer(256, seed=2)
    gq2.quantize(x)
    used = [(0, 64 + 8 * (gq.getBinNum() - 1)), (gq._load_header().codes_offset, n)]
    for off, ln in used:  # header + live splits, and the n code bytes
        assert torch.equal(gq.payload[off:off + ln], gq2.payload[off:off + ln])


def test_parallel_quantize_keeps_duplicate_splits(gpu):
    n = 70000
    x = _data(n, 9, "dups")
    gq = gpu.QuantileQuantizer(64, seed=5)
    gpu.Parallel.setParallelism(1)
    gq.parallelQuantize(torch.from_numpy(x).cuda())
    oq = O.parallel_quantize(x.astype(np.float64), 64, threads=1, seed=5)
    assert gq.getBinNum() == 64
    _check(gq, oq, x)


def test_nan_raises(gpu):
    x = _data(5000, 1, "normal")
    x[1234] = np.nan
    gq = gpu.QuantileQuantizer(256)
    with pytest.raises(gpu.QuantileSketchException, match="NaN"):
        gq.quantize(torch.from_numpy(x).cuda())


def test_invalid_partition_number(gpu):
    with pytest.raises(gpu.QuantileSketchException, match="partition"):
        gpu.QuantileQuantizer(1).quantize(torch.ones(10, device="cuda"))


def test_empty_input(gpu):
    gq = gpu.QuantileQuantizer(8, seed=1)
    gq.quantize(torch.empty(0, device="cuda"))
    oq = O.quantize(np.zeros(0), 8, 1)
    assert gq.getBinNum() == oq.bin_num == 8
    assert np.all(np.isnan(gq.getSplits()))
    assert gq.getMin() == oq.min and gq.getMax() == oq.max and gq.getZeroIdx() == oq.zero_idx


def test_write_object_bytes_match_oracle(gpu):
    for n, bins in ((3, 4), (1000, 256), (70001, 300)):
        x = _data(n, n, "normal")
        gq = gpu.QuantileQuantizer(bins, seed=3)
        gq.quantize(torch.from_numpy(x).cuda())
        oq = O.quantize(x.astype(np.float64), bins, 3)
        data = gq.writeObject()
        assert data == oq.write_ref()
        back = gpu.Quantizer.readObject(data)
        assert torch.equal(back.getBins(), gq.getBins())
        assert np.array_equal(back.getSplits(), gq.getSplits())


def test_times_by_matches_oracle(gpu):
    x = _data(20000, 3, "normal")
    gq = gpu.QuantileQuantizer(256, seed=8)
    gq.quantize(torch.from_numpy(x).cuda())
    oq = O.quantize(x.astype(np.float64), 256, 8)
    gq.timesBy(0.25)
    O.lib().orc_times_by(C.byref(oq.hdr), 0.25)
    oq2 = O.OracleQuant(oq.hdr, oq.bins)
    want = oq2.values()[oq.bins].astype(np.float32)
    assert np.array_equal(gq.decode().cpu().numpy(), want)


def test_split_injected_mode(gpu):
    from sketchml_amd import _lib
    n = 50001
    x = torch.from_numpy(_data(n, 11, "normal")).cuda()
    splits = np.array([-1.5, -0.5, -0.5, 0.0, 0.25, 1.0, 2.0], dtype=np.float64)
    nb = _lib.lib.skml_dense_payload_bytes(n, len(splits) + 1)
    pl = gpu.alloc_aligned(nb, "cuda")
    ctx = gpu.get_context()
    st = _lib.lib.skml_dense_encode_with_splits_f32(ctx.handle, C.c_void_p(x.data_ptr()), n,
                                                    splits.ctypes.data_as(_lib.dblp), len(splits),
                                                    -5.0, 5.0, C.c_void_p(pl.data_ptr()), nb)
    assert st == 0
    bins = torch.empty(n, dtype=torch.int32, device="cuda")
    assert _lib.lib.skml_dense_bins_i32(ctx.handle, C.c_void_p(pl.data_ptr()), C.c_void_p(bins.data_ptr()), n) == 0
    torch.cuda.synchronize()
    want = np.searchsorted(splits, x.cpu().numpy().astype(np.float64), side="right")
    assert np.array_equal(bins.cpu().numpy(), want)


def _encode_with_splits(gpu, x, splits, mn, mx):
    from sketchml_amd import _lib
    n = x.numel()
    nb = _lib.lib.skml_dense_payload_bytes(n, len(splits) + 1)
    pl = gpu.alloc_aligned(nb, "cuda")
    ctx = gpu.get_context()
    sp = np.ascontiguousarray(splits, dtype=np.float64)
    st = _lib.lib.skml_dense_encode_with_splits_f32(ctx.handle, C.c_void_p(x.data_ptr()), n,
                                                    sp.ctypes.data_as(_lib.dblp), len(sp), mn, mx,
                                                    C.c_void_p(pl.data_ptr()), nb)
    assert st == 0
    bins = torch.empty(n, dtype=torch.int32, device="cuda")
    assert _lib.lib.skml_dense_bins_i32(ctx.handle, C.c_void_p(pl.data_ptr()), C.c_void_p(bins.data_ptr()), n) == 0
    torch.cuda.synchronize()
    return bins.cpu().numpy()


def _oracle_index_of(splits, mn, mx, xs):
    """Quantizer.indexOf per value (oracle restatement, Quantizer.java:49-72)."""
    h = O.QuantHeader()
    h.bin_num = len(splits) + 1
    h.min, h.max = mn, mx
    for i, s in enumerate(splits):
        h.splits[i] = float(s)
    if mn > 0.0:
        h.zero_idx = 0
    elif mx < 0.0:
        h.zero_idx = h.bin_num - 1
    else:
        h.zero_idx = int(np.sum(np.asarray(splits) < 0.0))
    f = O.lib().orc_index_of
    return np.array([f(C.byref(h), float(v)) for v in xs], dtype=np.int32)


@pytest.mark.parametrize("case", ["irrational", "dense_bucket", "two_bins", "wide", "zeros"])
def test_split_injected_exact_compare(gpu, case):
    """Double splits that fp32 cannot represent: the LUT / Eytzinger tables hold RU(split) and
    must still give indexOf's answer for every float, including values adjacent to a split,
    +-0, +-inf, denormals and NaN (indexOf's NaN bin)."""
    rng = np.random.default_rng(len(case) * 7919)
    if case == "irrational":
        splits = np.sort(rng.standard_normal(255)) * np.pi
    elif case == "dense_bucket":  # > 15 splits inside one LUT bucket -> Eytzinger fallback
        splits = 1.0 + np.arange(300) * 3e-7 + 1e-9
    elif case == "two_bins":
        splits = np.array([0.1])
    elif case == "wide":
        splits = np.sort(np.concatenate([-np.logspace(-40, 38, 60), np.logspace(-40, 38, 60),
                                         [-1e300, 1e300, -1e-300, 1e-300]]))
    else:
        splits = np.array([-1e-45, -0.0, 0.0, 0.0, 1e-45, 1.0])
    s32 = splits.astype(np.float32)
    near = np.concatenate([s32, np.nextafter(s32, np.float32(np.inf)), np.nextafter(s32, np.float32(-np.inf))])
    special = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, -np.nan, 1e-45, -1e-45, 3.4e38, -3.4e38],
                       dtype=np.float32)
    body = (rng.standard_normal(40000) * (np.abs(splits).max() if case != "wide" else 1.0)).astype(np.float32)
    x = np.concatenate([near, special, body, near]).astype(np.float32)
    mn, mx = -10.0, 10.0
    got = _encode_with_splits(gpu, torch.from_numpy(x).cuda(), splits, mn, mx)
    want = _oracle_index_of(splits, mn, mx, x.astype(np.float64))
    assert np.array_equal(got, want)


def test_decode_sum(gpu):
    from sketchml_amd import _lib
    n, P = 100003, 3
    ctx = gpu.get_context()
    nb = _lib.lib.skml_dense_payload_bytes(n, 256)
    allp = gpu.alloc_aligned(nb * P, "cuda")
    want = np.zeros(n, dtype=np.float64)
    for p in range(P):
        x = _data(n, 100 + p, "normal")
        xt = torch.from_numpy(x).cuda()
        pr = _lib.Params()
        _lib.lib.skml_params_default(C.byref(pr))
        pr.seed = p
        st = _lib.lib.skml_dense_encode_f32(ctx.handle, C.c_void_p(xt.data_ptr()), n, C.byref(pr),
                                            C.c_void_p(allp.data_ptr() + p * nb), nb)
        assert st == 0
        torch.cuda.synchronize()
        oq = O.quantize(x.astype(np.float64), 256, p)
        want += oq.values()[oq.bins]
    out = torch.empty(n, dtype=torch.float32, device="cuda")
    assert _lib.lib.skml_dense_decode_sum_f32(ctx.handle, C.c_void_p(allp.data_ptr()), P, nb,
                                              C.c_void_p(out.data_ptr()), n, 1.0 / P) == 0
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), (want * (1.0 / P)).astype(np.float32))


# (P, requested bins per payload, n), with the oracle's effective bin counts: 8-bit codes (8 x 136,
# 8 x up to 221, and 16 x up to 235, which takes the per-payload kernel); 4-, 2- and 1-bit codes;
# a mixed-width set (the per-payload kernel); n = 15 (tail only).
@pytest.mark.parametrize("P,bins,n", [(8, [256] * 8, 2**20 + 13), (8, [256] * 8, 40005),
                                      (8, [512] * 8, 2**18 + 3), (4, [1024] * 4, 50001),
                                      (16, [512] * 16, 40000 + 5), (5, [16] * 5, 2**18 + 7), (4, [4] * 4, 99999),
                                      (3, [2] * 3, 4097), (6, [256, 16, 4, 2, 256, 16], 50001), (1, [256], 15)])
@pytest.mark.parametrize("kernel", ["occ", pytest.param("occ_nopf", marks=pytest.mark.ab), "plain"])
def test_decode_sum_forms(gpu, P, bins, n, kernel):
    """k_decode_sum_occ (8 elements per lane, P <= 8 tables of the largest bin count in LDS; with
    and without the next step's code prefetch) and the per-payload kernel (P > 8, mixed widths,
    > 256 bins): bit-exact against the oracle's decodes summed in double
    in payload order, then x 1/P (Gradient.sum + timesBy, ml/gradient/Gradient.scala:44-49).
    Requested bins 512 with Maths.unique give effective counts up to 256 (8-bit codes).
    kernel "plain": SKML_FORM_DECODE_SUM = 1 selects the one-table-per-payload kernel (its
    software-pipelined form when the width is common and P <= 8)."""
    from sketchml_amd import _lib
    with _lib.forced_forms(decode_sum={"occ": 0, "plain": 1, "occ_nopf": 2}[kernel]):
        _decode_sum_case(gpu, P, bins, n)


def _decode_sum_case(gpu, P, bins, n):
    from sketchml_amd import _lib
    ctx = gpu.get_context()
    nb = max(_lib.lib.skml_dense_payload_bytes(n, b) for b in bins)
    nb = (nb + 255) // 256 * 256
    allp = gpu.alloc_aligned(nb * P, "cuda")
    want = np.zeros(n, dtype=np.float64)
    for p in range(P):
        x = _data(n, 300 + p, "normal")
        xt = torch.from_numpy(x).cuda()
        pr = _lib.Params()
        _lib.lib.skml_params_default(C.byref(pr))
        pr.seed, pr.bin_num = p, bins[p]
        assert _lib.lib.skml_dense_encode_f32(ctx.handle, C.c_void_p(xt.data_ptr()), n, C.byref(pr),
                                              C.c_void_p(allp.data_ptr() + p * nb), nb) == 0
        torch.cuda.synchronize()
        oq = O.quantize(x.astype(np.float64), bins[p], p)
        want += oq.values()[oq.bins]
    out = torch.empty(n, dtype=torch.float32, device="cuda")
    assert _lib.lib.skml_dense_decode_sum_f32(ctx.handle, C.c_void_p(allp.data_ptr()), P, nb,
                                              C.c_void_p(out.data_ptr()), n, 1.0 / P) == 0, _lib.last_error()
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), (want * (1.0 / P)).astype(np.float32))


@pytest.mark.parametrize("P,bins", [(8, 1024), (8, 1023), (7, 1024), (2, 4096)])
def test_decode_sum_lds_boundary(gpu, P, bins):
    """16-bit codes at the edge of the occupancy form's LDS: P tables of `bins` doubles plus the
    kernel's static code-pointer array must fit 64 KB, so 8 x 1,024 bins (exactly 64 KB of tables)
    take the per-payload kernel and 8 x 1,023 / 7 x 1,024 the occupancy form.  A sketch cannot
    keep 1,024 distinct splits, so the payloads come from the split-injected encode; the expected
    sum is every payload's Quantizer.getValues()[indexOf(x)] (Quantizer.java:39-72) in double in
    payload order, x 1/P."""
    from sketchml_amd import _lib
    ctx = gpu.get_context()
    n = 70001
    nb = (_lib.lib.skml_dense_payload_bytes(n, bins) + 255) // 256 * 256
    allp = gpu.alloc_aligned(nb * P, "cuda")
    want = np.zeros(n, dtype=np.float64)
    rng = np.random.default_rng(P * 10007 + bins)
    for p in range(P):
        splits = np.sort(rng.choice(np.arange(-4 * bins, 4 * bins), bins - 1, replace=False)) / 1024.0
        mn, mx = -8.0, 8.0
        x = np.clip(rng.standard_normal(n) * 2.0, mn, mx).astype(np.float32)
        sp = np.ascontiguousarray(splits, dtype=np.float64)
        xt = torch.from_numpy(x).cuda()
        assert _lib.lib.skml_dense_encode_with_splits_f32(ctx.handle, C.c_void_p(xt.data_ptr()), n,
                                                          sp.ctypes.data_as(_lib.dblp), len(sp), mn, mx,
                                                          C.c_void_p(allp.data_ptr() + p * nb), nb) == 0
        torch.cuda.synchronize()
        h = O.QuantHeader()
        h.bin_num, h.n, h.min, h.max = bins, n, mn, mx
        for i, s in enumerate(sp):
            h.splits[i] = float(s)
        h.zero_idx = int(np.sum(sp < 0.0))
        vals = np.zeros(bins, dtype=np.float64)
        O.lib().orc_get_values(C.byref(h), vals.ctypes.data_as(O.dblp))
        want += vals[np.searchsorted(sp, x.astype(np.float64), side="right")]
    out = torch.empty(n, dtype=torch.float32, device="cuda")
    assert _lib.lib.skml_dense_decode_sum_f32(ctx.handle, C.c_void_p(allp.data_ptr()), P, nb,
                                              C.c_void_p(out.data_ptr()), n, 1.0 / P) == 0, _lib.last_error()
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), (want * (1.0 / P)).astype(np.float32))


def test_dense_vector_compressor_surface(gpu):
    x = torch.from_numpy(_data(12345, 1, "app")).cuda()
    comp = gpu.DenseVectorCompressor(gpu.QuantizationType.QUANTILE, 256, seed=9)
    comp.compressDense(x)
    oq = O.quantize(x.cpu().numpy().astype(np.float64), 256, 9)
    dec = comp.decompressDense().cpu().numpy()
    assert np.array_equal(dec, oq.values()[oq.bins].astype(np.float32))
    keys, vals = comp.decompressSparse()
    assert keys.numel() == 12345 and torch.equal(vals.cpu(), torch.from_numpy(dec))
    assert comp.size() == 12345.0
    assert comp.memoryBytes() == 12 + len(oq.write_ref())


@pytest.mark.parametrize("sizes", [[2**20, 2**20 + 77, 3, 300000, 2**21], [2**22, 2**22]])
def test_quantize_buckets_matches_single_encodes(gpu, sizes):
    """skml_dense_encode_batch_f32 (two internal streams) == skml_dense_encode_f32 per bucket."""
    xs = [torch.from_numpy(_data(n, 40 + i, "normal")).cuda() for i, n in enumerate(sizes)]
    qs = gpu.QuantileQuantizer.quantizeBuckets(xs, 256, seed=3)
    for x, q in zip(xs, qs):
        one = gpu.QuantileQuantizer(256, seed=3)
        one.quantize(x)
        h = one._load_header()
        assert np.array_equal(q.getSplits(), one.getSplits())
        assert q._load_header().zero_idx == h.zero_idx
        nbytes = (x.numel() * h.code_bits + 7) // 8
        assert torch.equal(q.payload[h.codes_offset:h.codes_offset + nbytes],
                           one.payload[h.codes_offset:h.codes_offset + nbytes])
        oq = O.quantize(x.cpu().numpy().astype(np.float64), 256, seed=3) if x.numel() < 400000 else None
        if oq is not None:
            assert np.array_equal(q.getBins().cpu().numpy(), oq.bins)


def test_quantize_buckets_nan_raises(gpu):
    xs = [torch.randn(5000, device="cuda") for _ in range(3)]
    xs[1][17] = float("nan")
    with pytest.raises(gpu.QuantileSketchException):
        gpu.QuantileQuantizer.quantizeBuckets(xs, 256)


def test_sketch_gradient_dense_and_sparse(gpu):
    """SketchGradient (ml/gradient/SketchGradient.scala): fromDense / fromSparse, timesBy on the
    bucket values in double, toDense / toSparse / toAuto, against the oracle's values and bins."""
    from sketchml_amd import gradient as G
    rng = np.random.default_rng(12)
    dim = 200003
    dense = np.where(rng.random(dim) < 0.2, rng.standard_normal(dim), 0.0).astype(np.float32)
    sg = G.SketchGradient(G.DenseDoubleGradient(dim, torch.from_numpy(dense).cuda()), 256, seed=1)
    oq = O.quantize(dense.astype(np.float64), 256, seed=1)
    assert sg.countNNZ() == dim
    sg.timesBy(0.25)
    assert np.array_equal(sg.toDense().values.cpu().numpy(), (oq.values() * 0.25)[oq.bins])
    auto = sg.toAuto()  # ~20 % nnz after decode? the zeros decode to the zero bin's midpoint
    assert auto.kind() in (G.Kind.DenseDouble, G.Kind.SparseDouble)
    # sparse side: DenseDoubleGradient.toSparse -> SketchGradient.fromSparse -> toSparse
    sp = G.DenseDoubleGradient(dim, torch.from_numpy(dense).cuda()).toAuto()
    assert sp.kind() == G.Kind.SparseDouble
    keys = np.nonzero(np.abs(dense) > 1e-8)[0]
    assert np.array_equal(sp.indices.cpu().numpy(), keys)
    sk2 = G.SketchGradient(sp, 256, 8, 2, 0.3, seed=1, hashSeed=2)
    osp = O.sparse_compress(keys.astype(np.int32), dense[keys].astype(np.float64), 256, 8, 2, 0.3, 1, 2)
    ok, ob = osp.restore()
    sk2.timesBy(2.0)
    back = sk2.toSparse()
    assert np.array_equal(back.indices.cpu().numpy(), ok)
    assert np.array_equal(back.values.cpu().numpy(), (osp.q.values() * 2.0)[ob])
