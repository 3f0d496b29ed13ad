"""The counter-based dropout scheme (csrc/common.h, include/mmseq.h `mmseq_dropout`) restated in
numpy and checked for the statistics a Bernoulli(p) mask must have (CPU; the GPU tests check that
every kernel applies exactly this mask: tests/test_dropout_gpu.py). One lowbias32 hash per element
quad, its second 32 bits by one multiply: per-field rate, independence of the four fields of a
quad and across nearby elements, flat field histograms."""
import numpy as np
import pytest

M32 = np.uint64(0xFFFFFFFF)


def _splitmix(z):
    z = (z + 0x9E3779B97F4A7C15) & ((1 << 64) - 1)
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & ((1 << 64) - 1)
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & ((1 << 64) - 1)
    return z ^ (z >> 31)


def _keys(seed, stream):  # make_drop
    key = _splitmix(seed ^ _splitmix(0x5BD1E995 + stream))
    return np.uint64(key & 0xFFFFFFFF), np.uint64((key >> 32) | 1)


def _lowbias32(x):
    x = x ^ (x >> np.uint64(16))
    x = (x * np.uint64(0x7FEB352D)) & M32
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & M32
    return x ^ (x >> np.uint64(16))


def fields(seed, stream, nquads):
    """The four 16-bit fields of quads 0 .. nquads - 1 (drop_hash / drop_hash2)."""
    k0, k1 = _keys(seed, stream)
    q = np.arange(nquads, dtype=np.uint64)
    h = _lowbias32(((q ^ k0) + k1) & M32)
    m = (h * np.uint64(0x9E3779B1)) & M32
    h2 = m ^ (m >> np.uint64(16))
    sh, lo = np.uint64(16), np.uint64(0xFFFF)
    return np.stack([h & lo, h >> sh, h2 & lo, h2 >> sh], 1)


@pytest.mark.parametrize("seed,stream", [(12345, 7), (2024, 5), (1, 99)])
def test_quad_dropout_statistics(seed, stream):
    p = 0.1
    thr = round(p * 65536)
    f = fields(seed, stream, 1 << 20)
    d = f < thr
    n = d.shape[0]
    sd = np.sqrt(p * (1 - p) / n)
    assert np.all(np.abs(d.mean(0) - p) < 5 * sd), d.mean(0)
    for a in range(4):
        for b in range(a + 1, 4):
            both = (d[:, a] & d[:, b]).mean()
            assert abs(both - p * p) < 5 * np.sqrt(p * p / n), (a, b, both)
    flat = d.reshape(-1)
    for lag in (1, 2, 3, 4, 5, 8, 64, 2052):
        both = (flat[:-lag] & flat[lag:]).mean()
        assert abs(both - p * p) < 5 * np.sqrt(p * p / flat.size), (lag, both)
    for j in range(4):
        hist = np.bincount((f[:, j] >> np.uint64(12)).astype(np.int64), minlength=16) / n
        assert np.abs(hist - 1 / 16).max() < 5 * np.sqrt(1 / 16 / n) + 1e-4, j
