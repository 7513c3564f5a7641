"""GPU path against the committed golden vectors (tests/golden/*.npz): no oracle call at all, the
expected outputs are the fixtures themselves."""
import glob
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _names(prefix):
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLD, prefix + "*.npz")))


def _load(name):
    return np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)


@pytest.mark.parametrize("name", _names("dense_"))
def test_dense_golden(gpu, name):
    g = _load(name)
    q = gpu.QuantileQuantizer(int(g["bin_num_req"]), seed=int(g["seed"]))
    q.quantize(torch.from_numpy(g["x"]).cuda())
    assert q.getBinNum() == int(g["bin_num"]) and q.getZeroIdx() == int(g["zero_idx"])
    assert q.getMin() == float(g["min"]) and q.getMax() == float(g["max"])
    assert np.array_equal(q.getSplits(), g["splits"])
    assert np.array_equal(q.getBins().cpu().numpy(), g["bins"])
    assert np.array_equal(q.getValues(), g["values"])
    assert np.array_equal(q.decode().cpu().numpy(), g["values"][g["bins"]].astype(np.float32))
    assert q.writeObject() == g["write_ref"].tobytes()


def _check_quant(q, g):
    assert q.getBinNum() == int(g["bin_num"]) and q.getZeroIdx() == int(g["zero_idx"])
    assert np.float64(q.getMin()).tobytes() == np.float64(g["min"]).tobytes()
    assert np.float64(q.getMax()).tobytes() == np.float64(g["max"]).tobytes()
    assert np.array_equal(q.getSplits(), g["splits"], equal_nan=True)
    assert np.array_equal(q.getBins().cpu().numpy(), g["bins"])
    assert np.array_equal(q.decode(dtype=torch.float64).cpu().numpy(), g["values"][g["bins"]], equal_nan=True)
    assert q.writeObject() == g["write_ref"].tobytes()


@pytest.mark.parametrize("name", _names("f64_"))
def test_f64_golden(gpu, name):
    g = _load(name)
    q = gpu.QuantileQuantizer(int(g["bin_num_req"]), seed=int(g["seed"]))
    q.quantize(torch.from_numpy(g["x"]).cuda())  # float64 tensor: the fp64 path
    _check_quant(q, g)


@pytest.mark.parametrize("name", _names("uniform_"))
def test_uniform_golden(gpu, name):
    g = _load(name)
    q = gpu.UniformQuantizer(int(g["bin_num_req"]))
    q.quantize(torch.from_numpy(g["x"]).cuda())
    _check_quant(q, g)


@pytest.mark.parametrize("name", _names("sparse_"))
def test_sparse_golden(gpu, name):
    g = _load(name)
    bins, groups, rows, seed, hseed = (int(v) for v in g["params"])
    pl = gpu.encode_sparse(torch.from_numpy(g["keys"]).cuda(), torch.from_numpy(g["vals"]).cuda(), bins, groups,
                           rows, float(g["col_ratio"]), seed, hseed)
    hdr, splits = pl.quant_header()
    assert hdr.bin_num == int(g["bin_num"]) and hdr.zero_idx == int(g["zero_idx"])
    assert np.array_equal(splits, g["splits"])
    for gi in range(groups):
        d = pl.group(gi)
        assert d["size"] == int(g["group_size"][gi])
        if f"table_{gi}" not in g.files:
            continue
        assert d["col_num"] == int(g["col_num"][gi]) and d["hash_ids"] == list(g["hash_ids"][gi])
        assert np.array_equal(d["table"], g[f"table_{gi}"])
        assert [d["num_intervals"], int(d["flag_kind"]), d["n_flag_bits"], d["n_delta_bits"]] == \
            list(g[f"delta_meta_{gi}"])
        assert np.array_equal(d["flag_words"], g[f"flag_words_{gi}"])
        assert np.array_equal(d["delta_words"], g[f"delta_words_{gi}"])
    k, v = pl.restore()
    assert np.array_equal(k.cpu().numpy(), g["restored_keys"])
    vals = pl.values()
    assert np.array_equal(v.cpu().numpy(), vals[g["restored_bins"]].astype(np.float32))


@pytest.mark.parametrize("name", _names("delta_"))
def test_delta_golden(gpu, name):
    g = _load(name)
    enc = gpu.DeltaAdaptiveEncoder()
    enc.encode(torch.from_numpy(g["keys"]).cuda())
    assert [enc.numIntervals, int(enc.flagKind), enc.nFlagBits, enc.nDeltaBits] == list(g["meta"])
    assert np.array_equal(enc.flagWords.cpu().numpy().view(np.uint64), g["flag_words"])
    assert np.array_equal(enc.deltaWords.cpu().numpy().view(np.uint64), g["delta_words"])
    assert np.array_equal(enc.decode().cpu().numpy(), g["keys"])
