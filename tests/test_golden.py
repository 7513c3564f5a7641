"""CPU tests: the oracle against the committed golden vectors (tests/golden/, written by
tests/golden/make_golden.py), and the C-ABI library's exported surface (no compute calls)."""
import ctypes as C
import glob
import os
import re

import numpy as np
import pytest

from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def _load(name):
    return np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)


DENSE = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLD, "dense_*.npz")))
SPARSE = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLD, "sparse_*.npz")))
DELTA = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLD, "delta_*.npz")))
WIDE = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLD, "f64_*.npz")))
UNIFORM = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLD, "uniform_*.npz")))


def test_fixtures_present():
    assert len(DENSE) >= 7 and len(SPARSE) >= 2 and len(DELTA) >= 3
    assert len(WIDE) >= 3 and len(UNIFORM) >= 4


def _check_quant(q, g):
    assert q.bin_num == int(g["bin_num"]) and q.zero_idx == int(g["zero_idx"])
    assert np.float64(q.min).tobytes() == np.float64(g["min"]).tobytes()
    assert np.float64(q.max).tobytes() == np.float64(g["max"]).tobytes()
    assert np.array_equal(q.splits, g["splits"], equal_nan=True)
    assert np.array_equal(q.bins, g["bins"])
    assert np.array_equal(q.values(), g["values"], equal_nan=True)
    assert q.write_ref() == g["write_ref"].tobytes()


@pytest.mark.parametrize("name", WIDE)
def test_oracle_f64_golden(name):
    g = _load(name)
    assert g["x"].dtype == np.float64
    _check_quant(O.quantize(g["x"], int(g["bin_num_req"]), int(g["seed"])), g)


@pytest.mark.parametrize("name", UNIFORM)
def test_oracle_uniform_golden(name):
    g = _load(name)
    _check_quant(O.uniform_quantize(g["x"].astype(np.float64), int(g["bin_num_req"])), g)


@pytest.mark.parametrize("name", DENSE)
def test_oracle_dense_golden(name):
    g = _load(name)
    q = O.quantize(g["x"].astype(np.float64), int(g["bin_num_req"]), int(g["seed"]))
    assert q.bin_num == int(g["bin_num"]) and q.zero_idx == int(g["zero_idx"])
    assert q.min == float(g["min"]) and q.max == float(g["max"])
    assert np.array_equal(q.splits, g["splits"])
    assert np.array_equal(q.bins, g["bins"])
    assert np.array_equal(q.values(), g["values"])
    assert q.write_ref() == g["write_ref"].tobytes()


@pytest.mark.parametrize("name", SPARSE)
def test_oracle_sparse_golden(name):
    g = _load(name)
    bins, groups, rows, seed, hseed = (int(v) for v in g["params"])
    s = O.sparse_compress(g["keys"], g["vals"].astype(np.float64), bins, groups, rows, float(g["col_ratio"]),
                          seed, hseed)
    assert s.q.bin_num == int(g["bin_num"]) and s.q.zero_idx == int(g["zero_idx"])
    assert np.array_equal(s.q.splits, g["splits"])
    assert np.array_equal(s.group_size, g["group_size"])
    assert np.array_equal(s.col_num, g["col_num"]) and np.array_equal(s.hash_ids, g["hash_ids"])
    for gi in range(groups):
        if f"table_{gi}" not in g.files:
            assert s.tables[gi] is None
            continue
        assert np.array_equal(s.tables[gi], g[f"table_{gi}"])
        d = s.deltas[gi]
        assert [d["num_intervals"], int(d["flag_kind"]), d["n_flag_bits"], d["n_delta_bits"]] == \
            list(g[f"delta_meta_{gi}"])
        assert np.array_equal(d["flag_words"], g[f"flag_words_{gi}"])
        assert np.array_equal(d["delta_words"], g[f"delta_words_{gi}"])
    rk, rb = s.restore()
    assert np.array_equal(rk, g["restored_keys"]) and np.array_equal(rb, g["restored_bins"])


@pytest.mark.parametrize("name", DELTA)
def test_oracle_delta_golden(name):
    g = _load(name)
    d = O.delta_encode(g["keys"])
    assert [d["num_intervals"], int(d["flag_kind"]), d["n_flag_bits"], d["n_delta_bits"]] == list(g["meta"])
    assert np.array_equal(d["flag_words"], g["flag_words"])
    assert np.array_equal(d["delta_words"], g["delta_words"])
    assert np.array_equal(d["decoded"], g["keys"])


def test_oracle_random_hash_golden():
    g = _load("misc_random_hash")
    r = O.JavaRandom(42)
    assert [r.next_int() for _ in range(16)] == list(g["ints"])
    r = O.JavaRandom(-7)
    assert [r.next_int(b) for b in (1, 2, 3, 7, 8, 100, 1000, 1 << 20, 2**31 - 1)] == list(g["bounded"])
    for h in range(8):
        assert [O.java_hash(h, int(k), 1009) for k in g["keys"]] == list(g["hashes"][h])
    for s in range(6):
        assert list(O.pick_hashes(s, 8)) == list(g["picks"][s])
    for i, z in enumerate((0, 10, 31, 32, 47, 48, 128, 200, 255)):
        assert list(O.group_edges(z, 256, 8)) == list(g["edges"][i])


# ---- the C ABI: every function declared in include/skml.h is exported by libskml.so ----
def _declared_functions():
    with open(os.path.join(ROOT, "include", "skml.h")) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[A-Za-z_][A-Za-z0-9_]*\s*\**\s*(skml_[a-z0-9_]+)\s*\(", text, flags=re.M)
    return sorted(set(names))


def test_abi_exports_every_declared_symbol():
    import sketchml_amd
    from sketchml_amd import _lib
    declared = _declared_functions()
    assert len(declared) >= 38
    lib = C.CDLL(sketchml_amd.LIB_PATH)
    missing = [n for n in declared if not hasattr(lib, n)]
    assert not missing, missing
    # the Python binding covers the whole declared surface, and nothing undeclared
    assert sorted(_lib.EXPORTED) == declared


def test_form_ids_match_header():
    """sketchml_amd._lib.FORMS mirrors the SKML_FORM_* ids of include/skml.h; skml_debug_form
    returns the previous value and -1 for an unknown id (host-only)."""
    from sketchml_amd import _lib
    with open(os.path.join(ROOT, "include", "skml.h")) as f:
        ids = {m.group(1).lower(): int(m.group(2)) for m in re.finditer(r"#define SKML_FORM_([A-Z_]+) (\d+)", f.read())}
    count = ids.pop("count")
    assert ids == _lib.FORMS and count == len(ids)
    assert _lib.lib.skml_debug_form(count, 1) == -1
    with _lib.forced_forms(rs_rounds=1):
        assert _lib.lib.skml_debug_form(_lib.FORMS["rs_rounds"], 1) == 1
    assert _lib.lib.skml_debug_form(_lib.FORMS["rs_rounds"], 0) == 0
    # the product library refuses the forms only the A/B build carries, and changes nothing
    ab_only = [("leaf_split", 1), ("leaf_split", 4), ("decode_sum", 2), ("rs_rounds", 2), ("dec_rows_serial", 2),
               ("agg_tiles", 2), ("agg_tiles", 5), ("run_bounds", 1), ("dec_lookback", 1), ("dec_lookback", 2)]
    for name, v in ab_only:
        if _lib.AB_BUILD:
            assert _lib.lib.skml_debug_form(_lib.FORMS[name], v) == 0
            assert _lib.lib.skml_debug_form(_lib.FORMS[name], 0) == v
        else:
            assert _lib.lib.skml_debug_form(_lib.FORMS[name], v) == -2
            assert _lib.lib.skml_debug_form(_lib.FORMS[name], 0) == 0
            other = "part_ballot" if name == "rs_rounds" else "rs_rounds"
            with pytest.raises(_lib.FormNotBuilt):
                with _lib.forced_forms(**{other: 1, name: v}):
                    pass
            assert _lib.lib.skml_debug_form(_lib.FORMS[other], 0) == 0  # restored on the way out


def test_abi_host_only_calls():
    """Calls that touch no device: defaults, version, payload sizing, error reporting."""
    from sketchml_amd import _lib
    p = _lib.Params()
    _lib.lib.skml_params_default(C.byref(p))
    assert (p.bin_num, p.group_num, p.row_num, p.dedup) == (256, 8, 2, 1) and p.col_ratio == 0.3
    assert _lib.lib.skml_version()
    # header 64 B + 255 splits padded to 256 B, then codes for n rounded up to 1024 elements
    assert _lib.lib.skml_dense_payload_bytes(1000, 256) == 2304 + 1024
    assert _lib.lib.skml_dense_payload_bytes(1000, 4) == 256 + 256
    assert _lib.lib.skml_dense_payload_bytes(2**26, 256) == 2304 + 2**26
    assert _lib.lib.skml_dense_payload_bytes(10, 1) == 0      # bin_num < 2: invalid
    assert _lib.lib.skml_sparse_free(None) == 0
    assert _lib.lib.skml_ctx_sync(None) == _lib.SKML_E_ARG
    assert "NULL" in _lib.last_error()
