"""The ml path's DP exchange of sparse gradients on one GPU.

- export / import: one contiguous device blob per payload (skml_sparse_export / _import) that
  round-trips to the same restore() and the same writeObject stream; corrupt blobs are refused.
- Gradient.sum (ml/gradient/Gradient.scala:44-49) of P payloads, skml_sparse_decode_sum_f64:
  bit-exact against the oracle's restore() of each payload summed in double, payload by payload,
  with SparseDoubleGradient.toAuto's dense/sparse rule (DenseDoubleGradient.plusBy).
- the RCCL path with a world-1 communicator: sizes agreed, blob exported into its padded slot,
  all-gathered, summed.
"""
import ctypes as C

import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu

EPS = 1e-8


def oracle_sum(osps, dim, scale=1.0):
    """Gradient.sum over the oracle's payloads (oracle.gradient_sum: DenseDoubleGradient(dim), then
    plusBy(p.toAuto) in order); returns (sum, forms)."""
    return O.gradient_sum(((k, osp.q.values()[b]) for osp in osps for k, b in [osp.restore()]), dim, scale)


def _payload(gpu, dim, density, seed, bins=256, tiny=0.0, groups=8):
    rng = np.random.default_rng(seed)
    keys = np.nonzero(rng.random(dim) < density)[0].astype(np.int32)
    vals = rng.standard_normal(len(keys))
    if tiny:
        t = rng.random(len(keys)) < tiny
        vals[t] = rng.uniform(-3e-9, 3e-9, int(t.sum()))
    pl = gpu.encode_sparse(torch.from_numpy(keys).cuda(), torch.from_numpy(vals).cuda(), bins, groups, 2, 0.3, seed,
                           seed + 100)
    osp = O.sparse_compress(keys, vals, bins, groups, 2, 0.3, seed, seed + 100)
    return pl, osp


def _gather_local(payloads):
    """The all-gather's output layout on one GPU: slot p = payload p's blob, stride = the largest."""
    from sketchml_amd.distributed import blob_stride
    sizes = [p.export_bytes() for p in payloads]
    stride = blob_stride(sizes)
    allb = torch.zeros(stride * len(payloads), dtype=torch.uint8, device="cuda")
    for i, p in enumerate(payloads):
        p.export(allb[i * stride:(i + 1) * stride])
    return allb, stride


def test_export_import_round_trip(gpu):
    pl, osp = _payload(gpu, 300000, 0.15, 1)
    blob = pl.export()
    assert blob.numel() == pl.export_bytes() and blob.numel() % 256 == 0
    back = gpu.SparsePayload.from_blob(blob)
    blob.fill_(0)                                 # the import owns its copy
    k0, b0 = pl.restore_bins()
    k1, b1 = back.restore_bins()
    assert torch.equal(k0, k1) and torch.equal(b0, b1)
    _, v1 = back.restore(torch.float64)
    ok, ob = osp.restore()
    assert np.array_equal(v1.cpu().numpy(), osp.q.values()[ob])
    assert back.serialize() == pl.serialize()     # writeObject of the imported payload is the same stream
    h0, s0 = pl.quant_header()
    h1, s1 = back.quant_header()
    assert (h0.bin_num, h0.zero_idx, h0.min, h0.max) == (h1.bin_num, h1.zero_idx, h1.min, h1.max)
    assert np.array_equal(s0, s1)
    pl.times_by(0.5)                              # quantValues travel timesBy'd
    back2 = gpu.SparsePayload.from_blob(pl.export())
    _, v2 = back2.restore(torch.float64)
    assert np.array_equal(v2.cpu().numpy(), (osp.q.values() * 0.5)[ob])


def _blob_header(blob):
    from sketchml_amd import _lib
    return _lib.SparseBlobHeader.from_buffer_copy(blob[:256].cpu().numpy().tobytes())


def _blob_cells(blob):
    """The MinMax cells of a blob as int32: the exact narrow image widened (top code -> the fill)."""
    h = _blob_header(blob)
    raw = blob[h.off_tables:h.off_tables + h.ncells * h.table_width // 8].cpu().numpy()
    if h.table_width == 32:
        return raw.view(np.int32)
    cells = raw.view(np.uint8 if h.table_width == 8 else np.uint16).astype(np.int64)
    fill = int(blob[256 + 16:256 + 20].cpu().numpy().view(np.int32)[0])  # SpGroups.fill
    cells[cells == (1 << h.table_width) - 1] = fill
    return cells.astype(np.int32)


@pytest.mark.parametrize("bins,width", [(256, 8), (3000, 16)])
def test_blob_carries_exact_narrow_tables(gpu, bins, width):
    """The exchange blob carries the MinMax tables as the encoder's exact narrow image: 8 bits a
    cell for at most 255 effective bins, 16 bits up to 65,535, the fill as the top code.  Widened,
    the cells equal the int32 table the payload serialises (MinMaxSketch.writeObject's table,
    MinMaxSketch.java:88-97) -- the same payload read back by readObject has no narrow image and
    exports int32 cells -- and a Gradient.sum over blobs of all three widths is exact."""
    dim = 120011
    pl, osp = _payload(gpu, dim, 0.3, 55, bins=bins)
    assert (osp.q.bin_num <= 255) == (width == 8)
    blob = pl.export()
    h = _blob_header(blob)
    assert (h.version, h.table_width) == (2, width)
    wide = gpu.SparsePayload.deserialize(pl.serialize(), quant_values=pl.values())
    blob32 = wide.export()
    assert _blob_header(blob32).table_width == 32
    assert blob.numel() < blob32.numel()
    assert np.array_equal(_blob_cells(blob), _blob_cells(blob32))
    tables = np.concatenate([pl.group(g)["table"] for g in range(8) if pl.group(g)["size"] > 0])
    assert np.array_equal(np.sort(_blob_cells(blob)), np.sort(tables))
    back = gpu.SparsePayload.from_blob(blob)          # the imported payload: cells widened again
    assert back.serialize() == pl.serialize()
    k0, b0 = pl.restore_bins()
    k1, b1 = back.restore_bins()
    assert torch.equal(k0, k1) and torch.equal(b0, b1)
    p8, o8 = _payload(gpu, dim, 0.2, 56, bins=256)
    allb, stride = _gather_local([pl, wide, p8, back])
    got = gpu.decode_sum(allb, 4, stride, dim, 0.25).cpu().numpy()
    want, _ = oracle_sum([osp, osp, o8, osp], dim, 0.25)
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))


def test_corrupt_blobs_are_refused(gpu):
    pl, _ = _payload(gpu, 50000, 0.2, 2)
    blob = pl.export()
    bad = blob.clone()
    bad[0] ^= 0xFF                                # magic
    with pytest.raises(gpu.SketchMLException):
        gpu.SparsePayload.from_blob(bad)
    bad = blob.clone()
    G = 8
    off = 256 + 280 + 8 * G                       # SpGroups.gstart[G] (the total) inside the blob
    bad[off:off + 8] = torch.tensor(np.array([123456789], dtype=np.int64).view(np.uint8), device="cuda")
    with pytest.raises(gpu.SketchMLException, match="inconsistent"):
        gpu.SparsePayload.from_blob(bad)
    with pytest.raises(gpu.SketchMLException):    # shorter than the blob says
        gpu.SparsePayload.from_blob(blob, 1024)
    from sketchml_amd import _lib
    woff = _lib.SparseBlobHeader.table_width.offset
    for w in (12, 16):                            # not a cell width; not this bin count's narrow width
        bad = blob.clone()
        bad[woff:woff + 4] = torch.from_numpy(np.array([w], dtype=np.int32).view(np.uint8)).cuda()
        with pytest.raises(gpu.SketchMLException):
            gpu.SparsePayload.from_blob(bad)
    # a key beyond the sum's dimension (SparseDoubleGradient's bound check)
    with pytest.raises(gpu.SketchMLException, match="outside"):
        gpu.decode_sum(blob, 1, blob.numel(), 1000)



def test_decode_sum_refuses_a_corrupt_payload_among_several(gpu):
    """Gradient.sum reads every payload's header and meta in two strided copies: a payload with a
    bad magic, one whose sections run past the stride and one with inconsistent offsets are each
    refused by index, and the intact set still sums exactly."""
    dim = 40009
    pls, osps = zip(*[_payload(gpu, dim, 0.2, 30 + p) for p in range(3)])
    allb, stride = _gather_local(pls)
    bad = allb.clone()
    bad[stride] ^= 0xFF                           # payload 1's magic
    with pytest.raises(gpu.SketchMLException, match="payload 1"):
        gpu.decode_sum(bad, 3, stride, dim)
    bad = allb.clone()
    total = np.array([stride + 256], dtype=np.int64).view(np.uint8)
    bad[2 * stride + 8:2 * stride + 16] = torch.from_numpy(total).cuda()  # payload 2 claims more than its slot
    with pytest.raises(gpu.SketchMLException, match="payload 2"):
        gpu.decode_sum(bad, 3, stride, dim)
    got = gpu.decode_sum(allb, 3, stride, dim).cpu().numpy()
    want, _ = oracle_sum(osps, dim)
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))


def test_decode_sum_payload_meta_past_the_first_read(gpu):
    """A payload of 3,000 bins carries ~48 KB of splits and values, past the 16 KB that the first
    strided read-back takes of every blob: the metas are read again whole, and the sum is exact."""
    dim = 50021
    pls, osps = zip(*[_payload(gpu, dim, 0.3, 40, bins=256), _payload(gpu, dim, 0.3, 41, bins=3000)])
    allb, stride = _gather_local(pls)
    got = gpu.decode_sum(allb, 2, stride, dim).cpu().numpy()
    want, _ = oracle_sum(osps, dim)
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))


@pytest.mark.parametrize("bins,forms", [(256, {}), (1000, {}), (256, {"rs_rounds": 1}),
                                        pytest.param(256, {"rs_rounds": 2}, marks=pytest.mark.ab)])
def test_restore_values_refuse_bins_outside_quant_values(gpu, bins, forms):
    """quantValues[bin] with a bin past the values (SparseVectorCompressor.java:118-126 throws
    ArrayIndexOutOfBoundsException): every MinMax cell of an imported blob overwritten with binNum
    + 5.  restore() of the values refuses it through the pipelined one-pass merge (256 and 1,000
    values), the plain one-pass kernel and the merge rounds alike; restore_bins() returns the raw
    cells as MinMaxSketch.query does."""
    from sketchml_amd import _lib
    pl, osp = _payload(gpu, 60000, 0.2, 4, bins=bins)
    blob = pl.export().clone()
    h = _lib.SparseBlobHeader.from_buffer_copy(blob[:256].cpu().numpy().tobytes())
    beff = osp.q.bin_num
    # the cells in the blob's width (the exact narrow image: the top code is the fill)
    dt = {8: np.uint8, 16: np.uint16, 32: np.int32}[h.table_width]
    assert h.table_width == (8 if beff <= 255 else 16)
    value = min(beff + 5, (1 << h.table_width) - 2)  # outside quantValues, below the top code
    assert value >= beff
    cells = torch.from_numpy(np.full(h.ncells, value, dtype=dt).view(np.uint8)).cuda()
    blob[h.off_tables:h.off_tables + cells.numel()] = cells
    bad = gpu.SparsePayload.from_blob(blob)
    with _lib.forced_forms(**forms):
        _, b = bad.restore_bins()
        assert int(b.min()) == value and int(b.max()) == value
        for dt in (torch.float32, torch.float64):
            with pytest.raises(gpu.SketchMLException, match="outside"):
                bad.restore(dt)
        _, v = pl.restore(torch.float64)             # the context recovers for a good payload
        assert torch.isfinite(v).all()


# Gradient.sum's tile kernels: vtile_rmw (the default for payloads of <= 8 groups and <= 256
# quantValues: a 512-key sum tile in LDS per wave, each element added into it row by row,
# payload by payload, with the next tile's element loads in flight, dense-form payloads swept at
# their end; the run bounds come from the key query,
# vtile_rmw_bounds_pass: from their own k_agg_bounds pass),
# vtile_pf (vtile with the next tile's element loads in flight), vtile (
# one wave per 512-key tile stages every payload's bins with presence bits and sums each key in
# registers, payload after payload, 8 payloads per launch; restores on two streams), wave
# (SKML_FORM_AGG_TILES: one wave per payload adding into a 4,096-key LDS tile, the form for any
# other shape) and wave_serial (the wave tiles with the generic per-row MinMax query and one
# stream); vtile2 / vtile4 take two / four staged tiles per wave round (one round of element
# loads); vtile_pf loads the next tile's elements while a tile is summed.  Every form is exact, and every form refuses a key repeated across a payload's groups.
KERNELS = {"vtile_rmw": {}, "vtile_rmw_bounds_pass": {"run_bounds": 1},
           "vtile_pf": {"agg_tiles": 4},
           "vtile": {"agg_tiles": 5}, "vtile2": {"agg_tiles": 3}, "vtile4": {"agg_tiles": 2},
           "wave": {"agg_tiles": 1},
           "wave_serial": {"agg_tiles": 1, "dec_rows_serial": 1, "agg_one_lane": 1}}


AB_KERNELS = {"vtile_rmw_bounds_pass", "vtile_pf", "vtile", "vtile2", "vtile4"}  # only in the A/B build


@pytest.fixture(params=[pytest.param(k, marks=pytest.mark.ab) if k in AB_KERNELS else k for k in sorted(KERNELS)])
def agg_kernel(request):
    from sketchml_amd import _lib
    with _lib.forced_forms(**KERNELS[request.param]):
        yield request.param


def test_decode_sum_eight_payloads_matches_oracle(gpu, agg_kernel):
    dim = 2**20 + 5
    pls, osps = zip(*[_payload(gpu, dim, 0.1 + 0.02 * p, 10 + p) for p in range(8)])
    allb, stride = _gather_local(pls)
    got = gpu.decode_sum(allb, 8, stride, dim).cpu().numpy()
    want, forms = oracle_sum(osps, dim)
    assert set(forms) == {"sparse"}
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))
    got_avg = gpu.decode_sum(allb, 8, stride, dim, 1.0 / 8).cpu().numpy()
    assert np.array_equal(got_avg.view(np.uint64), (want * (1.0 / 8)).view(np.uint64))


def test_decode_sum_dense_form_payloads(gpu, agg_kernel):
    """Payloads with more than dim * 2 / 3 live values reach plusBy in dense form: bucket values with
    |v| <= 1e-8 (the tiny cluster's midpoints) are not added."""
    dim = 30011
    p0, o0 = _payload(gpu, dim, 0.97, 21, tiny=0.15)    # dense form
    p1, o1 = _payload(gpu, dim, 0.3, 22, tiny=0.5)      # sparse form: its tiny values are added
    p2, o2 = _payload(gpu, dim, 0.95, 23, tiny=0.12)    # dense again
    allb, stride = _gather_local([p0, p1, p2])
    got = gpu.decode_sum(allb, 3, stride, dim).cpu().numpy()
    want, forms = oracle_sum([o0, o1, o2], dim)
    assert forms == ["dense", "sparse", "dense"]
    assert np.any(np.abs(o1.q.values()) <= EPS)          # the tiny values really exist
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))


def test_decode_sum_many_payloads_and_groups(gpu, agg_kernel):
    """Shapes past the wave-tile form's 8 payloads x 8 groups: nine payloads in one launch, and
    payloads of 12 groups, take the 4,096-key tiles; a dense-enough payload runs past the
    per-lane registers of a tile."""
    dim = 200003
    pls, osps = zip(*[_payload(gpu, dim, 0.05 + 0.01 * p, 50 + p) for p in range(9)])
    allb, stride = _gather_local(pls)
    got = gpu.decode_sum(allb, 9, stride, dim).cpu().numpy()
    want, _ = oracle_sum(osps, dim)
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))
    pls, osps = zip(*[_payload(gpu, dim, 0.4, 60 + p, groups=12) for p in range(3)])
    allb, stride = _gather_local(pls)
    got = gpu.decode_sum(allb, 3, stride, dim).cpu().numpy()
    want, _ = oracle_sum(osps, dim)
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))


def _dup_payload(gpu, dim, seed, groups=4, bins=256):
    """A payload whose keys repeat across groups (legal for the sketch module's restore, see
    test_sparse_duplicate_keys_across_groups_are_kept): each repeated key carries one value far
    below and one far above the rest, so its copies land in the first and the last group."""
    rng = np.random.default_rng(seed)
    keys = np.nonzero(rng.random(dim) < 0.2)[0].astype(np.int32)
    vals = rng.standard_normal(len(keys)).clip(-4, 4)
    rep = np.sort(rng.choice(len(keys), 300, replace=False))
    ins = np.zeros(len(keys), dtype=bool)
    ins[rep] = True
    keys2 = np.repeat(keys, np.where(ins, 2, 1))
    vals2 = np.empty(len(keys2))
    pos = np.cumsum(np.where(ins, 2, 1)) - np.where(ins, 2, 1)
    vals2[pos] = np.where(ins, -6.0 - rng.random(len(keys)), vals)
    vals2[pos[ins] + 1] = 6.0 + rng.random(int(ins.sum()))
    pl = gpu.encode_sparse(torch.from_numpy(keys2).cuda(), torch.from_numpy(vals2).cuda(), bins, groups, 2, 0.3, seed,
                           seed + 100)
    osp = O.sparse_compress(keys2, vals2, bins, groups, 2, 0.3, seed, seed + 100)
    return pl, osp


@pytest.mark.parametrize("shape", ["two", "nine_payloads", "twelve_groups", "bins_512"])
def test_decode_sum_keys_repeated_across_groups(gpu, agg_kernel, shape):
    """SketchGradient.toSparse builds a SparseDoubleGradient from the restored keys, whose
    constructor requires them strictly increasing (SparseDoubleGradient.scala:12): a key repeated
    across a payload's groups fails Gradient.sum.  Every tile form sees the repeat (presence
    bits) and the call raises; shapes past the wave-tile form (9 payloads, 12 groups, 512 bins)
    take the 4,096-key tiles."""
    dim = 100003
    groups = 12 if shape == "twelve_groups" else 4
    bins = 512 if shape == "bins_512" else 256
    npay = 9 if shape == "nine_payloads" else 2
    good = [_payload(gpu, dim, 0.2, 71 + p, groups=groups, bins=bins) for p in range(npay - 1)]
    p1, o1 = _dup_payload(gpu, dim, 72, groups=groups, bins=bins)
    k1, _ = o1.restore()
    assert len(np.unique(k1)) < len(k1)                   # the repeats survive the codec
    pls = [g[0] for g in good] + [p1]
    osps = [g[1] for g in good] + [o1]
    with pytest.raises(O.GradientSumError, match="strictly increasing"):
        oracle_sum(osps, dim)
    allb, stride = _gather_local(pls)
    with pytest.raises(gpu.SketchMLException, match="strictly increasing"):
        gpu.decode_sum(allb, npay, stride, dim)
    # the payloads without the repeat still sum exactly (the error left no state behind)
    allb, stride = _gather_local(pls[:-1])
    got = gpu.decode_sum(allb, npay - 1, stride, dim).cpu().numpy()
    want, _ = oracle_sum(osps[:-1], dim)
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))


@pytest.mark.parametrize("order", ["wide_first", "narrow_first", "all_wide"])
def test_decode_sum_mixed_bin_widths(gpu, agg_kernel, order):
    """Payloads whose quantValues need 2-byte bins (bin_num > 256, requested 512) and 1-byte ones
    (256) in one sum: each restore writes its bins at its own byte offset (a 2-byte
    payload before a 1-byte one used to overlap it)."""
    dim = 150001
    spec = {"wide_first": [512, 256, 512, 256], "narrow_first": [256, 512, 256], "all_wide": [512, 1024, 512]}[order]
    pls, osps = zip(*[_payload(gpu, dim, 0.12 + 0.03 * p, 90 + p, bins=b) for p, b in enumerate(spec)])
    assert any(len(o.q.values()) > 256 for o in osps)
    allb, stride = _gather_local(pls)
    got = gpu.decode_sum(allb, len(spec), stride, dim, 0.25).cpu().numpy()
    want, forms = oracle_sum(osps, dim, 0.25)
    assert set(forms) == {"sparse"}
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))


def test_decode_sum_refuses_empty_payloads(gpu, agg_kernel):
    """An empty restore cannot reach Gradient.sum in the reference: SketchGradient.toSparse builds
    SparseDoubleGradient(dim, [], []), whose constructor reads indices.head and throws
    (SparseDoubleGradient.scala:11).  The oracle raises there, and so does the library, whichever
    position the empty payload holds."""
    dim = 4096
    empty = gpu.encode_sparse(torch.zeros(0, dtype=torch.int32).cuda(), torch.zeros(0, dtype=torch.float64).cuda())
    p1, o1 = _payload(gpu, dim, 0.2, 31)
    with pytest.raises(O.GradientSumError):
        O.gradient_sum([(np.zeros(0, np.int32), np.zeros(0)), (o1.restore()[0], o1.q.values()[o1.restore()[1]])], dim)
    for order in ([empty, p1], [p1, empty]):
        allb, stride = _gather_local(order)
        with pytest.raises(gpu.SketchMLException, match="head of empty list"):
            gpu.decode_sum(allb, 2, stride, dim)
    allb, stride = _gather_local([p1])  # the context stays usable
    got = gpu.decode_sum(allb, 1, stride, dim).cpu().numpy()
    want, _ = oracle_sum([o1], dim)
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))


def test_sparse_exchange_world1_rccl(gpu):
    """distributed.exchange_sparse over a world-1 group with the RCCL communicator
    (PayloadExchange): sizes, the padded slot, the all-gather, the sum and 1/P."""
    import torch.distributed as dist
    from sketchml_amd import distributed as D
    store = dist.HashStore()
    dist.init_process_group("gloo", store=store, rank=0, world_size=1)
    try:
        dim = 700001
        pl, osp = _payload(gpu, dim, 0.1, 41)
        ex = D.PayloadExchange(gpu.get_context().handle)
        try:
            avg, allb, stride = D.exchange_sparse(pl, dim, exchange=ex)
            torch.cuda.synchronize()
        finally:
            ex.close()
        assert stride % 256 == 0 and stride >= pl.export_bytes()
        assert torch.equal(allb[: pl.export_bytes()], pl.export())
        want, _ = oracle_sum([osp], dim)
        assert np.array_equal(avg.cpu().numpy().view(np.uint64), want.view(np.uint64))
    finally:
        dist.destroy_process_group()


def _c3_dense(seed, dim=2**28):
    """A C3-shaped dense gradient as bench.py builds rank r's (seed 3 + r): N(0, 1), 10 % kept."""
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.randn(dim, device="cuda", generator=g)
    x[torch.rand(dim, device="cuda", generator=g) >= 0.1] = 0.0
    return x


def test_decode_sum_eight_distinct_c3_payloads_full_size(gpu):
    """The sum bench.py times (extras.other_configs.sparse_aggregate) at its own size: 8 distinct
    C3 payloads (2^28 dims, 10 % nnz, dense seeds 3 .. 10, the DP step's per-rank gradients) through
    Gradient.sum x 1/8, bit-exact against the oracle's Gradient.sum of the oracle's own encodes
    (toSparse, SparseVectorCompressor.compressSparse, restore).  The union of keys covers ~57 % of
    the dims, so the 524,288 wave tiles see run pieces that do not line up across payloads.  Both
    tile forms are checked against the one oracle sum."""
    from concurrent.futures import ThreadPoolExecutor
    from sketchml_amd import _lib
    from sketchml_amd.distributed import blob_stride
    dim, P = 2**28, 8
    blobs, host = [], []
    for p in range(P):
        x = _c3_dense(3 + p, dim)
        pl = gpu.encode_dense_as_sparse(x, 256, 8, 2, 0.3, 3 + p, 3 + p)
        blobs.append(pl.export())
        host.append(O.to_sparse(x.cpu().numpy().astype(np.float64)))
        del x, pl
    stride = blob_stride([b.numel() for b in blobs])
    allb = torch.zeros(stride * P, dtype=torch.uint8, device="cuda")
    for p, b in enumerate(blobs):
        allb[p * stride:p * stride + b.numel()].copy_(b)
    del blobs

    def oracle_restore(p):  # the C oracle releases the GIL: the 8 encodes run side by side
        k, v = host[p]
        osp = O.sparse_compress(k, v, 256, 8, 2, 0.3, 3 + p, 3 + p)
        rk, rb = osp.restore()
        return rk, osp.q.values()[rb]

    with ThreadPoolExecutor(8) as ex:
        restored = list(ex.map(oracle_restore, range(P)))
    del host
    union = np.zeros(dim, dtype=bool)
    for k, _ in restored:
        union[k] = True
    assert 0.5 < union.mean() < 0.6                     # distinct key sets, not copies
    del union
    want, forms = O.gradient_sum(restored, dim, 1.0 / P)
    del restored
    assert forms == ["sparse"] * P
    # sum tile in LDS, 4,096-key tiles; the A/B build: staged tiles (prefetching, 1, 2, 4 per round)
    for form in (0, 1) + ((4, 5, 3, 2) if _lib.AB_BUILD else ()):
        with _lib.forced_forms(agg_tiles=form):
            got = gpu.decode_sum(allb, P, stride, dim, 1.0 / P)
            torch.cuda.synchronize()
            assert np.array_equal(got.cpu().numpy().view(np.uint64), want.view(np.uint64)), form
            del got
