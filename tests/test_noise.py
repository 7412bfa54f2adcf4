"""CPU checks of the training-noise generator's restatement (oracle/philox.py):
the published Random123 Philox4x32-10 known-answer vectors, and the
statistics of the U[0,1) stream built on it (the quantizers' replacement for
torch.rand_like, modelling/blocks/entropy_model.py:230,333)."""
import numpy as np
from scipy import stats

from oracle import philox


def test_philox_known_answers():
    for ctr, key, out in philox.KAT:
        got = philox.philox4x32_10(np.array([ctr], np.uint32), np.array([key], np.uint32))[0]
        assert [int(v) for v in got] == list(out), (ctr, key)


def test_stream_uses_all_four_words():
    # elements 4j .. 4j+3 are the four words of block j
    w = philox.philox4x32_10(np.array([[5, 0, 0, 0]], np.uint32), np.array([[7, 0]], np.uint32))[0]
    u = philox.uniform(4, seed=7, offset=20)
    assert np.array_equal(u, (w >> 8).astype(np.float32) / np.float32(2 ** 24))


def test_stream_statistics():
    n = 1 << 20
    u = philox.uniform(n, seed=0x1234_5678_9abc, offset=1 << 33).astype(np.float64)
    assert u.min() >= 0.0 and u.max() < 1.0
    assert abs(u.mean() - 0.5) < 4 * np.sqrt(1 / 12 / n)
    assert abs(u.var() - 1 / 12) < 4 * np.sqrt((1 / 80 - 1 / 144) / n)
    assert stats.kstest(u, "uniform").pvalue > 1e-3
