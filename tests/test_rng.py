"""The counter RNG (csrc/pt_rng.h) restated in numpy, pinned against the oracle."""
import numpy as np

M = 0xFFFFFFFF


def lowbias32(x):
    x = int(x) & M
    x ^= x >> 16
    x = (x * 0x7feb352d) & M
    x ^= x >> 15
    x = (x * 0x846ca68b) & M
    x ^= x >> 16
    return x


def draw(seed, pixel, sample, k):
    h = lowbias32(((seed * 0x9E3779B9) & M) ^ pixel)
    base = lowbias32(h ^ ((sample * 0x85EBCA6B) & M))
    v = lowbias32(base ^ ((k * 0xC2B2AE35 + 0x27D4EB2F) & M))
    return (v >> 8) / 16777216.0


def test_counter_rng_matches_oracle(restate):
    rng = np.random.default_rng(0)
    for _ in range(200):
        seed, pix, spl = (int(v) for v in rng.integers(0, 2**32, 3, dtype=np.uint64))
        k = int(rng.integers(0, 40))
        assert restate.rng_draw(seed, pix, spl, k) == draw(seed, pix, spl, k)


def test_counter_rng_uniformity(restate):
    v = np.array([draw(7, p, 0, 0) for p in range(20000)])
    assert abs(v.mean() - 0.5) < 0.01 and 0.0 <= v.min() and v.max() < 1.0
    hist, _ = np.histogram(v, bins=20, range=(0, 1))
    assert hist.min() > 850 and hist.max() < 1150
