"""The in-kernel training noise (row a12: the reference's torch.rand_like(x) - 0.5,
modelling/blocks/entropy_model.py:230 for z and :333 for y) on the HIP path:
Philox4x32-10 against the published Random123 known-answer vectors, the
U[0,1) stream bit-exact against the CPU restatement (oracle/philox.py), its
statistics, and the counter bookkeeping of a training step (z and y draws
disjoint, no counter reused across steps)."""
import numpy as np
import pytest
import torch
from scipy import stats

from oracle import philox

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _uniform(n, seed, offset):
    from image_compression_amd import _lib
    u = torch.empty(n, device=DEV)
    _lib.check(_lib.load().ic_uniform(_lib.ptr(u), n, _lib.c_ull(seed), _lib.c_ull(offset),
                                      _lib.stream_of(u)), "uniform")
    return u.cpu().numpy()


def test_philox_kat_on_device():
    from image_compression_amd import _lib
    inp = torch.from_numpy(np.array([list(c) + list(k) for c, k, _ in philox.KAT], np.uint32).view(np.int32)).to(DEV)
    out = torch.empty(len(philox.KAT) * 4, dtype=torch.int32, device=DEV)
    _lib.check(_lib.load().ic_philox_kat(_lib.ptr(inp), _lib.ptr(out), len(philox.KAT), _lib.stream_of(out)),
               "philox_kat")
    got = out.cpu().numpy().view(np.uint32).reshape(-1, 4)
    for g, (_, _, ref) in zip(got, philox.KAT):
        assert [int(v) for v in g] == list(ref)


@pytest.mark.parametrize("seed,offset,n", [(0, 0, 4096), (0x1234_5678_9abc, 4 * 0xFFFFFFF0, 1000),
                                           (2 ** 63 + 5, 1 << 40, 333)])
def test_uniform_matches_restatement(seed, offset, n):
    # the last case crosses no boundary; the second crosses the 2^32 block carry into counter word 1
    assert np.array_equal(_uniform(n, seed, offset), philox.uniform(n, seed, offset))


def test_uniform_rejects_unaligned_offset():
    from image_compression_amd import _lib
    u = torch.empty(8, device=DEV)
    assert _lib.load().ic_uniform(_lib.ptr(u), 8, _lib.c_ull(1), _lib.c_ull(2), _lib.stream_of(u)) == 1001


def test_uniform_statistics():
    n = 1 << 22
    u = _uniform(n, 0xC0FFEE, 0).astype(np.float64)
    assert u.min() >= 0.0 and u.max() < 1.0
    assert abs(u.mean() - 0.5) < 4 * np.sqrt(1 / 12 / n)
    assert abs(u.var() - 1 / 12) < 4 * np.sqrt((1 / 80 - 1 / 144) / n)
    assert stats.kstest(u[: 1 << 20], "uniform").pvalue > 1e-3
    # consecutive draws uncorrelated (lag 1 and lag 4, the block stride)
    for lag in (1, 4):
        r = np.corrcoef(u[:-lag], u[lag:])[0, 1]
        assert abs(r) < 4 / np.sqrt(n), (lag, r)


def test_training_step_counters():
    """Quantizers on zero inputs return u - 0.5 exactly: the z draw takes the first
    counters of a step, the y draw the next ones (4-aligned, disjoint), and
    begin_step moves the base past everything the previous step drew."""
    from image_compression_amd import functional as IF, noise
    from image_compression_amd.modelling.blocks.entropy_model import EntropyModel
    from image_compression_amd import get_cfg_defaults
    noise.reseed(987654321)
    cfg = get_cfg_defaults()
    em = EntropyModel(192, cfg).to(DEV).train()
    N = 3
    z = torch.zeros(N, 192, 2, 2, device=DEV)
    y = torch.zeros(N, 192, 5, 3, device=DEV)    # 8640 elements
    scale = torch.ones_like(y)
    nz, ny = z.numel(), y.numel()
    seen = []
    for step in range(2):
        noise.begin_step(z.device)
        base = int(noise.device_state(z.device)[1])
        qz, _, _ = em(z)
        qy, _ = IF.conditional(y, scale, None, 0, True)
        uz = (IF._to_last(qz.detach()) + 0.5).reshape(-1).cpu().numpy()
        uy = (qy.detach() + 0.5).reshape(-1).cpu().numpy()
        assert np.array_equal(uz, philox.uniform(nz, 987654321, base))
        oy = base + (nz + 3) // 4 * 4
        assert np.array_equal(uy, philox.uniform(ny, 987654321, oy))
        seen.append((base, oy + ny))
    (b0, e0), (b1, _) = seen
    assert b1 >= e0          # step 2's counters start past everything step 1 drew
