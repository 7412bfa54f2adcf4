"""Training-noise source for the entropy bottleneck.

The reference draws `torch.rand_like(x) - 0.5` inside forward
(modelling/blocks/entropy_model.py:230 for z, :333 for y; call order
meta_arch/bmshl2018.py:73,76).  Here the uniforms are generated inside the
quantize kernels by a counter-based Philox4x32-10 stream, so no noise tensor is
materialised in HBM.

The stream state lives on the device: a 2-word tensor {seed, base} per device.
Each draw in a step uses counters base + offset + i, where `offset` is a host
counter of the elements drawn so far in the step; `begin_step()` (called at the
top of every training forward) advances the device base by the previous
step's total with a kernel (ic_philox_advance).  Because the advance is a
kernel rather than a changed launch argument, a training step captured into a
hipGraph (image_compression_amd.step) replays with fresh noise every time.
The seed is drawn once from torch's default CPU generator (so
`torch.manual_seed` makes runs reproducible).  Under data parallelism every
rank seeds its CPU generator alike, so the rank is folded into the Philox key
(`rank_key`): rank r > 0 draws from key splitmix64(seed, r), independent of
every other rank's stream, and rank 0 keeps the single-process key.  The
reference draws `torch.rand_like` over the batch it holds (one process), so
every image there gets its own noise; without the fold, image i of every rank
would share one noise tensor.

For bit-level parity with the reference, exact uniform draws can be injected:

    with injected_noise([u_z, u_y]):
        model(x)

consumes u_z at the factorized (z) model and u_y at the conditional (y) model,
the reference's call order.
"""
import contextlib
import threading

import torch

from . import _lib

_state = threading.local()


def _st():
    if not hasattr(_state, "dev"):
        _state.seed = None
        _state.dev = {}       # device -> int64[2] {seed, base} tensor
        _state.offset = {}    # device -> counters drawn so far this step
        _state.rank = {}      # device -> the data-parallel rank its key was made for
        _state.queue = []
    return _state


def _key(device):
    d = torch.device(device)
    if d.index is None:
        return (d.type, torch.cuda.current_device() if d.type == "cuda" else 0)
    return (d.type, d.index)


_MASK62 = (1 << 62) - 1


def _splitmix64(x):
    x = (x + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return x ^ (x >> 31)


def rank_key(seed, rank):
    """The Philox key of data-parallel rank `rank` for the shared seed `seed`: the seed
    itself on rank 0, a splitmix64 hash of (seed, rank) elsewhere (62 bits, like the seed)."""
    if rank == 0:
        return int(seed)
    return _splitmix64(_splitmix64(int(seed)) ^ int(rank)) & _MASK62


def _dist_rank():
    import torch.distributed as dist
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def process_key(seed):
    """This process's Philox key for the shared seed (rank_key of its data-parallel rank)."""
    return rank_key(seed, _dist_rank())


def device_state(device):
    """The {seed, base} tensor of `device` (created on first use; the key folds in this
    process's data-parallel rank, see rank_key).  A state created before the process group
    was initialised carries rank 0's key; if the rank has changed since, the key word is
    rewritten in place (the base, i.e. the counters already drawn, is kept), so no two ranks
    ever share a stream because of when the first draw happened."""
    s = _st()
    k = _key(device)
    rank = _dist_rank()
    if k not in s.dev:
        if s.seed is None:
            s.seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        s.dev[k] = torch.tensor([rank_key(s.seed, rank), 0], dtype=torch.int64, device=torch.device(*k))
        s.offset[k] = 0
        s.rank[k] = rank
    elif s.rank.get(k) != rank:
        s.dev[k][0].fill_(rank_key(s.seed, rank))
        s.rank[k] = rank
    return s.dev[k]


def philox_stream(n, device):
    """Reserve n elements of this step's stream; returns (state tensor, offset).
    Reservations are whole Philox blocks (4 elements), so every draw starts at a
    4-aligned offset and the z and y draws of a step never share a block."""
    s = _st()
    st = device_state(device)
    k = _key(device)
    off = s.offset[k]
    s.offset[k] = off + (int(n) + 3) // 4 * 4
    return st, off


def begin_step(device):
    """Advance the device base past the counters the previous step drew."""
    s = _st()
    k = _key(device)
    n = s.offset.get(k, 0)
    if n:
        _lib.ops().philox_advance(s.dev[k], int(n))
        s.offset[k] = 0


def reseed(seed=None):
    s = _st()
    s.seed = None if seed is None else int(seed)
    s.dev = {}
    s.offset = {}
    s.rank = {}


def pop_injected():
    s = _st()
    if s.queue:
        return s.queue.pop(0)
    return None


@contextlib.contextmanager
def injected_noise(draws):
    """Inject U[0,1) draws (tensors shaped like z then y) consumed in call order."""
    s = _st()
    old = s.queue
    s.queue = list(draws)
    try:
        yield
    finally:
        left = s.queue
        s.queue = old
        if left:
            raise RuntimeError(f"injected_noise: {len(left)} draw(s) were not consumed")
