"""CPU model of the sign-alternating network that k_leaf64's fast loop runs (skml_sketch.hip,
sgn_flip / sgn_stage_rev / sgn_stages_eq / sgn_level_compact / sgn_run_pos).

One round of one wave: 64 lanes x 64 registers, 16 chunks of 256 values (4 lanes per chunk).  The
model applies exactly the device stages (odd lanes hold -x; fused flip max(y, -partner); same-sign
med3 stages with the selector ((lane & D) == 0) ^ bit J; in-lane bitonic clean + compaction keeping
stored parity odd ^ (lane & 1)) and checks the level-4 node against the reference's sort-and-compact
tree (HeapQuantileSketch.java:107-124 / QSketchUtils.java:45-82: sort each 256-value base buffer,
keep alternate ranks by the RNG bit, merge pairs and compact again) on random, tied, denormal and
one-signed data.  The GPU parity tests check the kernel itself against the oracle.
"""
import numpy as np
import pytest

LANES = np.arange(64)
SIGN = np.where(LANES & 1, -1.0, 1.0).astype(np.float32)


def _xor_read(y, mask):
    return y[LANES ^ mask]


def _halfclean(y):
    y = y.copy()
    d = y.shape[1] // 2
    while d >= 1:
        for i in range(y.shape[1]):
            j = i ^ d
            if j > i:
                lo, hi = np.minimum(y[:, i], y[:, j]), np.maximum(y[:, i], y[:, j])
                y[:, i], y[:, j] = lo, hi
        d //= 2
    return y


def _sel_max(mask, level):
    return (((LANES & mask) == 0) ^ (((LANES >> level) & 1) == 1))[:, None]


def _level(y, level, odd=None):
    y = np.maximum(y, -_xor_read(y, (1 << level) - 1))          # sgn_flip
    if level >= 2:
        p = _xor_read(y, 1 << (level - 1))[:, ::-1]              # sgn_stage_rev
        y = np.where(_sel_max(1 << (level - 1), level), np.maximum(y, p), np.minimum(y, p))
        d = 1 << (level - 2)
        while d >= 2:                                            # sgn_stages_eq
            p = _xor_read(y, d)
            y = np.where(_sel_max(d, level), np.maximum(y, p), np.minimum(y, p))
            d //= 2
    y = _halfclean(y)
    if odd is not None:                                          # halfclean_regs_compact
        keep_odd = (odd.astype(bool) ^ (SIGN < 0))[:, None]
        y = np.where(keep_odd, y[:, 1::2], y[:, 0::2])
    return y


def _device_round(x, bits):
    y = np.stack([x[l >> 2][(l & 3)::4] for l in range(64)]).astype(np.float32) * SIGN[:, None]
    y = np.sort(y, axis=1)                                       # sort_regs_oddeven<64>
    y = _level(y, 1)
    y = _level(y, 2, bits[0][LANES >> 2])
    for level, tree in zip(range(3, 7), range(1, 5)):
        y = _level(y, level, bits[tree][LANES >> level])
    real = y * SIGN[:, None]
    pos = np.where(LANES & 1, LANES >> 1, 63 - (LANES >> 1))     # sgn_run_pos
    out = np.empty(128, np.float32)
    for l in range(64):
        out[2 * pos[l]:2 * pos[l] + 2] = real[l] if SIGN[l] > 0 else real[l][::-1]
    return out


def _reference_round(x, bits):
    nodes = [np.sort(x[c])[bits[0][c]::2] for c in range(16)]
    for lv in range(1, 5):
        nodes = [np.sort(np.concatenate([nodes[2 * i], nodes[2 * i + 1]]))[bits[lv][i]::2]
                 for i in range(len(nodes) // 2)]
    return nodes[0]


@pytest.mark.parametrize("kind", ["normal", "ties", "denormal", "positive", "negative"])
def test_sign_alternating_network_equals_sort_and_compact(kind):
    rng = np.random.default_rng({"normal": 1, "ties": 2, "denormal": 3, "positive": 4, "negative": 5}[kind])
    for _ in range(12):
        if kind == "normal":
            x = rng.standard_normal((16, 256))
        elif kind == "ties":
            x = rng.integers(-4, 4, (16, 256)).astype(np.float64)
        elif kind == "denormal":
            x = rng.standard_normal((16, 256)) * 1e-39
        elif kind == "positive":
            x = np.abs(rng.standard_normal((16, 256)))
        else:
            x = -np.abs(rng.standard_normal((16, 256))) - 1.0
        x = x.astype(np.float32)
        bits = [rng.integers(0, 2, 16 >> lv) for lv in range(5)]
        np.testing.assert_array_equal(_device_round(x, bits), _reference_round(x, bits))
