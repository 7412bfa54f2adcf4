"""ORACLE — test infrastructure only, never the product path.

CPU restatement (numpy, uint32 arithmetic) of the training-noise generator the
HIP quantizers use in place of the reference's `torch.rand_like(x) - 0.5`
(modelling/blocks/entropy_model.py:230 for z, :333 for y).  The generator is
Philox4x32-10 (Salmon, Moraes, Dror, Shaw, "Parallel random numbers: as easy as
1, 2, 3", SC'11; the Random123 library's philox4x32_R with R = 10).  The
reference itself does not define this stream (it uses torch's CPU generator),
so it is pinned to the published Random123 known-answer vectors
(`KAT` below, checked by tests/test_noise.py) instead of to reference output.

Stream definition (include/imgcomp.h, ic_uniform): element i of stream `seed`
is word (i & 3) of philox4x32_10(counter = {i >> 2 as 64 bits, 0, 0},
key = {seed & 0xffffffff, seed >> 32}), mapped to U[0,1) as (word >> 8) / 2^24.
"""
import numpy as np

M0, M1 = np.uint32(0xD2511F53), np.uint32(0xCD9E8D57)
W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)

# Random123 kat_vectors, philox4x32 with 10 rounds: (counter[4], key[2]) -> output[4]
KAT = [
    ((0x00000000, 0x00000000, 0x00000000, 0x00000000), (0x00000000, 0x00000000),
     (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff, 0xffffffff, 0xffffffff, 0xffffffff), (0xffffffff, 0xffffffff),
     (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
]


def _mulhilo(a, b):
    p = a.astype(np.uint64) * np.uint64(b)
    return (p >> np.uint64(32)).astype(np.uint32), (p & np.uint64(0xFFFFFFFF)).astype(np.uint32)


def philox4x32_10(ctr, key):
    """ctr: uint32 array [..., 4]; key: uint32 array [..., 2] -> uint32 [..., 4]."""
    c = np.array(ctr, dtype=np.uint32, copy=True)
    k = np.array(key, dtype=np.uint32, copy=True)
    c0, c1, c2, c3 = c[..., 0], c[..., 1], c[..., 2], c[..., 3]
    k0, k1 = k[..., 0], k[..., 1]
    with np.errstate(over="ignore"):
        for _ in range(10):
            hi0, lo0 = _mulhilo(c0, M0)
            hi1, lo1 = _mulhilo(c2, M1)
            c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
            k0 = (k0 + W0).astype(np.uint32)
            k1 = (k1 + W1).astype(np.uint32)
    return np.stack([c0, c1, c2, c3], axis=-1)


def uniform(n, seed, offset=0):
    """Elements offset .. offset + n - 1 of stream `seed` as float32 in [0, 1)."""
    idx = np.arange(offset, offset + n, dtype=np.uint64)
    blk = idx >> np.uint64(2)
    ctr = np.zeros(idx.shape + (4,), dtype=np.uint32)
    ctr[:, 0] = (blk & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    ctr[:, 1] = (blk >> np.uint64(32)).astype(np.uint32)
    key = np.zeros(idx.shape + (2,), dtype=np.uint32)
    key[:, 0] = np.uint32(seed & 0xFFFFFFFF)
    key[:, 1] = np.uint32((seed >> 32) & 0xFFFFFFFF)
    w = philox4x32_10(ctr, key)[np.arange(n), (idx & np.uint64(3)).astype(np.int64)]
    return ((w >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)).astype(np.float32)
