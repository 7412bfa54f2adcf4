"""Training-noise source for the entropy bottleneck.

The reference draws `torch.rand_like(x) - 0.5` inside forward
(modelling/blocks/entropy_model.py:230 for z, :333 for y; call order
meta_arch/bmshl2018.py:73,76).  Here the uniforms are generated inside the
quantize kernels by a counter-based Philox4x32-10 stream, so no noise tensor is
materialised in HBM.  The stream seed is drawn once from torch's default CPU
generator (so `torch.manual_seed` makes runs reproducible) and the counter
advances by the number of elements each call consumes.

For bit-level parity with the reference, exact uniform draws can be injected:

    with injected_noise([u_z, u_y]):
        model(x)

consumes u_z at the factorized (z) model and u_y at the conditional (y) model,
the reference's call order.
"""
import contextlib
import threading

import torch

_state = threading.local()


def _st():
    if not hasattr(_state, "seed"):
        _state.seed = None
        _state.offset = 0
        _state.queue = []
    return _state


def philox_stream(n):
    """Reserve n counters; returns (seed, offset)."""
    s = _st()
    if s.seed is None:
        s.seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        s.offset = 0
    off = s.offset
    s.offset += int(n)
    return s.seed, off


def reseed(seed=None):
    s = _st()
    s.seed = None if seed is None else int(seed)
    s.offset = 0


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
