#!/usr/bin/env python3
"""Generate the committed golden vectors in tests/golden/ from the CPU restatement (oracle/).

The reference (Java 8) cannot be built or run in this image (no JDK), so these fixtures are
produced by the C restatement after it passed the hand-derived known-answer tests
(tests/test_oracle.py K1-K8) and the independent numpy cross-check.  They pin the oracle across
rounds (any change to it that alters an output fails tests/test_golden.py) and give the GPU
tests fixed expected outputs.  Inputs are small and seeded; outputs are stored exactly
(float64 / int32 / uint64) in one .npz per case with allow_pickle=False.

usage: python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import oracle as O  # noqa: E402


def dense_cases():
    rng = np.random.default_rng(20261015)
    cases = {
        "dense_app_1000": (np.where(rng.random(1000) < 0.9, rng.standard_normal(1000), 0.0), 256, 1),
        "dense_normal_4096": (rng.standard_normal(4096), 256, 2),          # B_eff = 129
        "dense_ragged_70001": (rng.standard_normal(70001), 256, 3),
        "dense_signed_zero_5000": (np.where(rng.random(5000) < 0.4, np.where(rng.random(5000) < 0.5, 0.0, -0.0),
                                            rng.standard_normal(5000)), 64, 4),
        "dense_negative_3000": (-np.abs(rng.standard_normal(3000)) - 0.5, 16, 5),  # max = Double.MIN_VALUE
        "dense_dups_20000": (rng.integers(-5, 6, 20000).astype(np.float64), 256, 6),
        "dense_bins4_100000": (rng.standard_normal(100000), 4, 7),
    }
    for name, (x, bins, seed) in cases.items():
        x = x.astype(np.float32).astype(np.float64)  # the device path takes fp32 input
        q = O.quantize(x, bins, seed)
        np.savez(os.path.join(HERE, name + ".npz"), x=x.astype(np.float32), bin_num_req=bins, seed=seed,
                 bin_num=q.bin_num, zero_idx=q.zero_idx, min=q.min, max=q.max, splits=q.splits,
                 bins=q.bins.astype(np.int32), values=q.values(), write_ref=np.frombuffer(q.write_ref(), np.uint8))


def sparse_cases():
    rng = np.random.default_rng(7)
    for name, dim, dens, bins, groups, rows, ratio, seed, hseed in (
            ("sparse_20000_g8", 20000, 0.2, 256, 8, 2, 0.3, 1, 2),
            ("sparse_50000_g4", 50000, 0.05, 64, 4, 3, 0.5, 3, 4)):
        mask = rng.random(dim) < dens
        keys = np.nonzero(mask)[0].astype(np.int32)
        vals = rng.standard_normal(len(keys)).astype(np.float32)
        s = O.sparse_compress(keys, vals.astype(np.float64), bins, groups, rows, ratio, seed, hseed)
        rk, rb = s.restore()
        out = dict(keys=keys, vals=vals, params=np.array([bins, groups, rows, seed, hseed], np.int64),
                   col_ratio=ratio, bin_num=s.q.bin_num, zero_idx=s.q.zero_idx, splits=s.q.splits,
                   group_size=s.group_size, col_num=s.col_num, hash_ids=s.hash_ids,
                   restored_keys=rk, restored_bins=rb)
        for g in range(groups):
            if s.tables[g] is None:
                continue
            d = s.deltas[g]
            out[f"table_{g}"] = s.tables[g]
            out[f"delta_meta_{g}"] = np.array([d["num_intervals"], int(d["flag_kind"]), d["n_flag_bits"],
                                               d["n_delta_bits"]], np.int64)
            out[f"flag_words_{g}"] = d["flag_words"]
            out[f"delta_words_{g}"] = d["delta_words"]
        np.savez(os.path.join(HERE, name + ".npz"), **out)


def misc_cases():
    # java.util.Random draws and the 8 Int2IntHash functions on fixed keys
    r = O.JavaRandom(42)
    ints = np.array([r.next_int() for _ in range(16)], np.int64)
    r = O.JavaRandom(-7)
    bounded = np.array([r.next_int(b) for b in (1, 2, 3, 7, 8, 100, 1000, 1 << 20, 2**31 - 1)], np.int64)
    keys = np.array([0, 1, 2, 9, 10, 99, 12345, 2**31 - 1, -1, -12345], np.int64)
    hashes = np.array([[O.java_hash(h, int(k), 1009) for k in keys] for h in range(8)], np.int64)
    picks = np.array([O.pick_hashes(s, 8) for s in range(6)], np.int64)
    edges = np.array([O.group_edges(z, 256, 8) for z in (0, 10, 31, 32, 47, 48, 128, 200, 255)], np.int64)
    np.savez(os.path.join(HERE, "misc_random_hash.npz"), ints=ints, bounded=bounded, keys=keys, hashes=hashes,
             picks=picks, edges=edges)
    rng = np.random.default_rng(11)
    for name, keys in (("delta_dense", np.cumsum(rng.integers(1, 3, 5000))),
                       ("delta_wide", np.cumsum(rng.integers(1, 1 << 22, 2000))),
                       ("delta_zero_first", np.concatenate([[0], np.cumsum(rng.integers(1, 50, 3000))]))):
        d = O.delta_encode(keys.astype(np.int32))
        np.savez(os.path.join(HERE, name + ".npz"), keys=keys.astype(np.int32),
                 meta=np.array([d["num_intervals"], int(d["flag_kind"]), d["n_flag_bits"], d["n_delta_bits"]], np.int64),
                 flag_words=d["flag_words"], delta_words=d["delta_words"])


def wide_and_uniform_cases():
    """fp64-input quantile cases (x stored as float64: values below fp32 precision) and uniform
    quantizer cases (UniformQuantizer.java:21-45) on fp32 and fp64 input."""
    rng = np.random.default_rng(20261016)
    wide = {
        "f64_normal_70001": (rng.standard_normal(70001), 256, 21),
        "f64_close_40000": (1.0 + rng.integers(0, 5000, 40000) * 2.0**-40, 64, 22),
        "f64_signed_zero_9000": (np.where(rng.random(9000) < 0.4, np.where(rng.random(9000) < 0.5, 0.0, -0.0),
                                          rng.standard_normal(9000)), 256, 23),
    }
    for name, (x, bins, seed) in wide.items():
        q = O.quantize(x, bins, seed)
        np.savez(os.path.join(HERE, name + ".npz"), x=x, bin_num_req=bins, seed=seed,
                 bin_num=q.bin_num, zero_idx=q.zero_idx, min=q.min, max=q.max, splits=q.splits,
                 bins=q.bins.astype(np.int32), values=q.values(), write_ref=np.frombuffer(q.write_ref(), np.uint8))
    x_nan = rng.standard_normal(20000)
    x_nan[rng.random(20000) < 0.03] = np.nan
    x_zero = np.abs(rng.standard_normal(5000)) + 1.0
    x_zero[10] = -0.0
    x_zero[20::7] = 0.0
    uni = {
        "uniform_f32_app_30000": (np.where(rng.random(30000) < 0.9, rng.standard_normal(30000), 0.0)
                                  .astype(np.float32), 256),
        "uniform_f64_nan_20000": (x_nan, 100),
        "uniform_f64_zero_first_5000": (x_zero, 16),
        "uniform_f32_negative_3000": ((-np.abs(rng.standard_normal(3000)) - 0.5).astype(np.float32), 8),
    }
    for name, (x, bins) in uni.items():
        q = O.uniform_quantize(x.astype(np.float64), bins)
        np.savez(os.path.join(HERE, name + ".npz"), x=x, bin_num_req=bins,
                 bin_num=q.bin_num, zero_idx=q.zero_idx, min=q.min, max=q.max, splits=q.splits,
                 bins=q.bins.astype(np.int32), values=q.values(), write_ref=np.frombuffer(q.write_ref(), np.uint8))


if __name__ == "__main__":
    # `make_golden.py wide` regenerates only the fp64 / uniform fixtures
    if sys.argv[1:] != ["wide"]:
        dense_cases()
        sparse_cases()
        misc_cases()
    wide_and_uniform_cases()
    print("written:", sorted(f for f in os.listdir(HERE) if f.endswith(".npz")))
