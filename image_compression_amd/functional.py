"""Autograd functions over the HIP kernels of libimgcomp.so.

Every forward/backward here launches hand-written gfx950 kernels through the
C ABI (include/imgcomp.h) on torch's current stream.  PyTorch provides only
allocation (caching allocator), stream handles and the autograd graph.
There is deliberately no CPU / eager fallback: CPU tensors raise.

Layout convention: activations with >= 32 channels live in NHWC
(torch.channels_last) so every GEMM operand row is channel-contiguous; the
3-channel image tensors stay NCHW and take the generic gather path.
"""
import ctypes
import os
import weakref

import torch
from torch.autograd import Function

from . import _lib
from . import noise as _noise

CL = torch.channels_last


def _L():
    return _lib.load()


def _cl(t):
    """Channels-last (NHWC) dense view/copy for GEMM operands with many channels."""
    if t.shape[1] >= 32 and t.stride(1) != 1:
        return t.contiguous(memory_format=CL)
    if not (t.is_contiguous() or t.is_contiguous(memory_format=CL)):
        return t.contiguous()
    return t


def _new_act(N, C, H, W, device):
    if C >= 32:
        return torch.empty((N, C, H, W), device=device, dtype=torch.float32, memory_format=CL)
    return torch.empty((N, C, H, W), device=device, dtype=torch.float32)


def _is_dense(t):
    """Non-overlapping and dense storage in some dimension order."""
    if t.numel() <= 1:
        return True
    expect = 1
    for s, n in sorted((s, n) for s, n in zip(t.stride(), t.shape) if n != 1):
        if s != expect:
            return False
        expect *= n
    return True


def _dense(t):
    if t.is_contiguous() or _is_dense(t):
        return t
    return t.contiguous()


def _match(g, ref):
    """Return g with exactly ref's strides (elementwise kernels index storage)."""
    if g.shape == ref.shape and g.stride() == ref.stride() and _is_dense(g):
        return g
    out = torch.empty_like(ref)
    out.copy_(g)
    return out


def _ws(nbytes, device):
    return _lib.workspace(nbytes, device)


def _n(t):
    return ctypes.c_longlong(t.numel())


# launch-plan log (tests): while a list is installed by `record_plans`, every conv / GDN op
# appends the plan (ic_conv_plan) of each launch it makes, so a test can show which kernel
# instances a whole training step ran
_PLAN_LOG = None


class record_plans:
    def __enter__(self):
        global _PLAN_LOG
        self.log, _PLAN_LOG = [], []
        return _PLAN_LOG

    def __exit__(self, *exc):
        global _PLAN_LOG
        _PLAN_LOG = None
        return False


def _log_plan(op, a, b, k=1, stride=1, pad=0, math=0):
    if _PLAN_LOG is not None:
        _PLAN_LOG.append(dict(_lib.plan(op, a, b, k, stride, pad, math), op=op))


# ============================================================== convolutions
# Column sums of a gradient computed by the op that produced it (GDN backward: sum over pixels
# of dx), handed to the conv whose output received that gradient, which then skips its own
# bias-gradient pass over the same tensor.  Keyed by the gradient tensor itself (weakref +
# version counter): a gradient changed in between (or any other tensor) falls back to the pass.
_COLSUMS = {}
_HANDOFF = os.environ.get("IMGCOMP_COLSUM_HANDOFF", "1") != "0"  # 0: every conv takes its own pass (A/B)


def _put_colsum(t, s):
    if not _HANDOFF:
        return
    for k in [k for k, (r, _, _) in _COLSUMS.items() if r() is None]:
        del _COLSUMS[k]
    _COLSUMS[t.data_ptr()] = (weakref.ref(t), t._version, s)


def _take_colsum(t):
    e = _COLSUMS.pop(t.data_ptr(), None)
    if e is None:
        return None
    r, ver, s = e
    return s if (r() is t and t._version == ver) else None


class Conv2dFn(Function):
    """torch.nn.Conv2d forward/backward (analysis.py:55, prior_analysis.py:54-56), each
    launch one torch.ops.imgcomp op (csrc/torch_ops.cpp -> C ABI)."""

    @staticmethod
    def forward(ctx, x, weight, bias, stride, padding, act, math=0):
        _lib.require_device(x, weight, bias)
        x = _cl(x)
        w = weight.contiguous()
        b = None if bias is None else bias.contiguous()
        if w.shape[1] != x.shape[1] or w.shape[2] != w.shape[3]:
            raise RuntimeError(f"conv2d: weight {tuple(w.shape)} does not match input {tuple(x.shape)}")
        y = _lib.ops().conv2d_fwd(x, w, b, stride, padding, int(act), int(math))
        _log_plan("conv2d_fwd", x, y, w.shape[2], stride, padding, math)
        ctx.conf = (stride, padding, act, b is not None, int(math))
        ctx.save_for_backward(x, w, y if act else None)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w, y = ctx.saved_tensors
        stride, padding, act, has_b, math = ctx.conf
        pre = _take_colsum(gy) if (has_b and not act) else None  # bias gradient formed by gy's producer
        if act:
            gy = relu_bwd(y, gy)
        gy = _cl(gy)
        dx = dw = db = None
        ops, k = _lib.ops(), w.shape[2]
        if ctx.needs_input_grad[0]:
            dx = ops.conv2d_dgrad(gy, w, x, stride, padding, math)
            _log_plan("conv2d_dgrad", gy, dx, k, stride, padding, math)
        if ctx.needs_input_grad[1] or (has_b and ctx.needs_input_grad[2]):
            dw, db = ops.conv2d_wgrad(x, gy, w, stride, padding, has_b and pre is None, math)
            _log_plan("conv2d_wgrad", x, gy, k, stride, padding, math)
            db = (db if pre is None else pre) if has_b else None
        return dx, dw, db, None, None, None, None


class ConvTranspose2dFn(Function):
    """torch.nn.ConvTranspose2d forward/backward (synthesis.py:55-57, prior_synthesis.py:54-56)."""

    @staticmethod
    def forward(ctx, x, weight, bias, stride, padding, output_padding, act, math=0):
        _lib.require_device(x, weight, bias)
        x = _cl(x)
        w = weight.contiguous()
        b = None if bias is None else bias.contiguous()
        if w.shape[0] != x.shape[1] or w.shape[2] != w.shape[3]:
            raise RuntimeError(f"conv_transpose2d: weight {tuple(w.shape)} does not match input {tuple(x.shape)}")
        y = _lib.ops().conv_transpose2d_fwd(x, w, b, stride, padding, output_padding, int(act), int(math))
        _log_plan("conv_transpose2d_fwd", x, y, w.shape[2], stride, padding, math)
        ctx.conf = (stride, padding, act, b is not None, int(math))
        ctx.save_for_backward(x, w, y if act else None)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w, y = ctx.saved_tensors
        stride, padding, act, has_b, math = ctx.conf
        pre = _take_colsum(gy) if (has_b and not act) else None  # bias gradient formed by gy's producer
        if act:
            gy = relu_bwd(y, gy)
        gy = _cl(gy)
        dx = dw = db = None
        ops, k = _lib.ops(), w.shape[2]
        if ctx.needs_input_grad[0]:
            dx = ops.conv_transpose2d_dgrad(gy, w, x, stride, padding, math)
            _log_plan("conv_transpose2d_dgrad", gy, dx, k, stride, padding, math)
        if ctx.needs_input_grad[1] or (has_b and ctx.needs_input_grad[2]):
            dw, db = ops.conv_transpose2d_wgrad(x, gy, w, stride, padding, has_b and pre is None, math)
            _log_plan("conv_transpose2d_wgrad", x, gy, k, stride, padding, math)
            db = (db if pre is None else pre) if has_b else None
        return dx, dw, db, None, None, None, None, None


# include/imgcomp.h IC_MATH_*: "fp32" exact fp32 MFMA; "bf16" bf16 operands, fp32 accumulation
# (reduced precision, config C3); "fp32_split" fp32 arithmetic on the bf16 MFMA through an exact
# three-term bf16 split of both operands (six products, error of an fp32 fma chain)
MATH = {"fp32": 0, "bf16": 1, "fp32_split": 2}


def conv2d(x, weight, bias=None, stride=1, padding=0, act=0, math=0):
    """`math` (forward and input gradient): 0 fp32 (default), 1 bf16 operands with fp32
    accumulation, 2 fp32 by exact bf16 split (see MATH)."""
    return Conv2dFn.apply(x, weight, bias, int(stride), int(padding), int(act), int(math))


def conv_transpose2d(x, weight, bias=None, stride=1, padding=0, output_padding=0, act=0, math=0):
    return ConvTranspose2dFn.apply(x, weight, bias, int(stride), int(padding), int(output_padding), int(act),
                                   int(math))


# ============================================================== GDN
class GDNFn(Function):
    """modelling/layers/gdn.py:84-86 given re-parameterised gamma (C,C,1,1), beta (C,)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, inverse, math=0, math_fwd=0):
        _lib.require_device(x, gamma, beta)
        x = _cl(x)
        g = gamma.contiguous()
        b = beta.contiguous()
        y, norm = _lib.ops().gdn_fwd(x, g, b, bool(inverse), int(math_fwd))
        _log_plan("gdn_fwd", x, None, math=math_fwd)
        ctx.inverse = bool(inverse)
        ctx.math = int(math)
        ctx.save_for_backward(x, norm, g)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, norm, g = ctx.saved_tensors
        gy = _match(gy, x)
        # dx's column sums come with it (the fused backward forms them from its dx tiles): the
        # bias gradient of the conv that produced x, taken by that conv's backward (_take_colsum)
        dx, dg, dbeta, dxsum = _lib.ops().gdn_bwd_sum(x, norm, gy, g, ctx.inverse, ctx.math)
        _put_colsum(dx, dxsum)
        _log_plan("gdn_bwd", x, None, math=ctx.math)
        return dx, dg, dbeta, None, None, None


def gdn(x, gamma, beta, inverse=False, math=0, math_fwd=0):
    """`math` 2: the backward's dgamma GEMM in split arithmetic (C = 192); `math_fwd` 2: the
    forward on the split implicit GEMM instead of the fused fp32 kernel."""
    return GDNFn.apply(x, gamma, beta, bool(inverse), int(math), int(math_fwd))


class NonNegFn(Function):
    """NonNegativeParam.forward (gdn.py:59-62): max(p, bound)^2 - pedestal."""

    @staticmethod
    def forward(ctx, p, bound, pedestal):
        _lib.require_device(p)
        p = p.contiguous()
        out = torch.empty_like(p)
        _lib.check(_L().ic_nonneg_fwd(_lib.ptr(p), _n(p), float(bound), float(pedestal), _lib.ptr(out),
                                      _lib.stream_of(p)), "nonneg_fwd")
        ctx.bound = float(bound)
        ctx.save_for_backward(p)
        return out

    @staticmethod
    def backward(ctx, g):
        (p,) = ctx.saved_tensors
        g = _match(g, p)
        gi = torch.empty_like(p)
        _lib.check(_L().ic_nonneg_bwd(_lib.ptr(p), _lib.ptr(g), _n(p), ctx.bound, _lib.ptr(gi),
                                      _lib.stream_of(p)), "nonneg_bwd")
        return gi, None, None


# ============================================================== elementwise
class BoundFn(Function):
    @staticmethod
    def forward(ctx, x, bound, upper):
        _lib.require_device(x)
        x = _dense(x)
        y = torch.empty_like(x)
        _lib.check(_L().ic_bound_fwd(_lib.ptr(x), _n(x), float(bound), int(upper), _lib.ptr(y),
                                     _lib.stream_of(x)), "bound_fwd")
        ctx.conf = (float(bound), int(upper))
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        bound, upper = ctx.conf
        g = _match(g, x)
        gx = torch.empty_like(x)
        _lib.check(_L().ic_bound_bwd(_lib.ptr(x), _lib.ptr(g), _n(x), bound, upper, _lib.ptr(gx),
                                     _lib.stream_of(x)), "bound_bwd")
        return gx, None, None


class ReLUFn(Function):
    @staticmethod
    def forward(ctx, x):
        _lib.require_device(x)
        x = _dense(x)
        y = torch.empty_like(x)
        _lib.check(_L().ic_relu_fwd(_lib.ptr(x), _n(x), _lib.ptr(y), _lib.stream_of(x)), "relu_fwd")
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, g):
        (y,) = ctx.saved_tensors
        return relu_bwd(y, g)


def relu_bwd(y, g):
    g = _match(g, y)
    gx = torch.empty_like(y)
    _lib.check(_L().ic_relu_bwd(_lib.ptr(y), _lib.ptr(g), _n(y), _lib.ptr(gx), _lib.stream_of(y)), "relu_bwd")
    return gx


class AbsFn(Function):
    @staticmethod
    def forward(ctx, x):
        _lib.require_device(x)
        x = _dense(x)
        y = torch.empty_like(x)
        _lib.check(_L().ic_abs_fwd(_lib.ptr(x), _n(x), _lib.ptr(y), _lib.stream_of(x)), "abs_fwd")
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        g = _match(g, x)
        gx = torch.empty_like(x)
        _lib.check(_L().ic_abs_bwd(_lib.ptr(x), _lib.ptr(g), _n(x), _lib.ptr(gx), _lib.stream_of(x)), "abs_bwd")
        return gx


class ExpClampFn(Function):
    """torch.clamp(v.exp(), lo, hi) of prior_synthesis.py:72."""

    @staticmethod
    def forward(ctx, v, lo, hi):
        _lib.require_device(v)
        v = _dense(v)
        s = torch.empty_like(v)
        e = torch.empty_like(v)
        _lib.check(_L().ic_exp_clamp_fwd(_lib.ptr(v), _n(v), float(lo), float(hi), _lib.ptr(s), _lib.ptr(e),
                                         _lib.stream_of(v)), "exp_clamp_fwd")
        ctx.conf = (float(lo), float(hi))
        ctx.save_for_backward(e)
        return s

    @staticmethod
    def backward(ctx, g):
        (e,) = ctx.saved_tensors
        lo, hi = ctx.conf
        g = _match(g, e)
        gv = torch.empty_like(e)
        _lib.check(_L().ic_exp_clamp_bwd(_lib.ptr(e), _lib.ptr(g), _n(e), lo, hi, _lib.ptr(gv),
                                         _lib.stream_of(e)), "exp_clamp_bwd")
        return gv, None, None


# ============================================================== losses
class CELossFn(Function):
    """_ce_loss (entropy_model.py:185): sum clamp(-ln(p+1e-10)/ln 2, 0, 50)."""

    @staticmethod
    def forward(ctx, p):
        _lib.require_device(p)
        p = _dense(p)
        out = torch.empty((), device=p.device, dtype=torch.float32)
        L = _L()
        nb = L.ic_reduce_ws(p.numel())
        buf = _ws(nb, p.device)
        _lib.check(L.ic_ce_loss_fwd(_lib.ptr(p), _n(p), _lib.ptr(out), _lib.ptr(buf), nb, _lib.stream_of(p)),
                   "ce_loss_fwd")
        ctx.save_for_backward(p)
        return out

    @staticmethod
    def backward(ctx, g):
        (p,) = ctx.saved_tensors
        g = g.contiguous()
        gp = torch.empty_like(p)
        _lib.check(_L().ic_ce_loss_bwd(_lib.ptr(p), _lib.ptr(g), _n(p), _lib.ptr(gp), _lib.stream_of(p)),
                   "ce_loss_bwd")
        return gp


class MSEFn(Function):
    """nn.MSELoss(reduction='mean')(input, target)."""

    @staticmethod
    def forward(ctx, a, b):
        _lib.require_device(a, b)
        a = _dense(a)
        b = _match(b, a)
        out = torch.empty((), device=a.device, dtype=torch.float32)
        L = _L()
        nb = L.ic_reduce_ws(a.numel())
        buf = _ws(nb, a.device)
        _lib.check(L.ic_mse_fwd(_lib.ptr(a), _lib.ptr(b), _n(a), _lib.ptr(out), _lib.ptr(buf), nb,
                                _lib.stream_of(a)), "mse_fwd")
        ctx.save_for_backward(a, b)
        return out

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        g = g.contiguous()
        ga = torch.empty_like(a) if ctx.needs_input_grad[0] else None
        gb = torch.empty_like(b) if ctx.needs_input_grad[1] else None
        _lib.check(_L().ic_mse_bwd(_lib.ptr(a), _lib.ptr(b), _lib.ptr(g), _n(a), _lib.ptr(ga), _lib.ptr(gb),
                                   _lib.stream_of(a)), "mse_bwd")
        return ga, gb


# ============================================================== entropy models
def _to_last(t):
    """(N, C, *) -> dense (N, *, C) so that channel = flat index % C."""
    return t.movedim(1, -1).contiguous()


def _from_last(t):
    return t.movedim(-1, 1)


class FactorizedFn(Function):
    """EntropyModel._quantize + _prob_mass (entropy_model.py:216-269).
    Returns (q, p) in the input's logical (N, C, *) shape."""

    @staticmethod
    def forward(ctx, z, mode, u, seed, offset, *params):
        _lib.require_device(z, None if mode == 3 else u, *params)
        L = _L()
        C = z.shape[1]
        zl = _to_last(z)
        # mode 3: `u` is the device {seed, base} state of the Philox stream
        ul = u if (u is None or mode == 3) else _to_last(u.to(z.dtype))
        q = torch.empty_like(zl)
        p = torch.empty_like(zl)
        prm = [t.contiguous() for t in params]
        cp = _lib.ICFactParams(*[ctypes.c_void_p(t.data_ptr()) for t in prm])
        _lib.check(L.ic_factorized_fwd(_lib.ptr(zl), _n(zl), C, ctypes.byref(cp), int(mode), _lib.ptr(ul),
                                       ctypes.c_ulonglong(seed), ctypes.c_ulonglong(offset), _lib.ptr(q),
                                       _lib.ptr(p), _lib.stream_of(z)), "factorized_fwd")
        ctx.mode = int(mode)
        ctx.C = C
        ctx.save_for_backward(q, *prm)
        return _from_last(q), _from_last(p)

    @staticmethod
    def backward(ctx, gq, gp):
        q, *prm = ctx.saved_tensors
        L = _L()
        gql = None if gq is None else _to_last(gq)
        gpl = None if gp is None else _to_last(gp)
        dz = torch.empty_like(q)
        grads = [torch.empty_like(t) for t in prm]
        cp = _lib.ICFactParams(*[ctypes.c_void_p(t.data_ptr()) for t in prm])
        cg = _lib.ICFactGrads(*[ctypes.c_void_p(t.data_ptr()) for t in grads])
        _lib.check(L.ic_factorized_bwd(_lib.ptr(q), _n(q), ctx.C, ctypes.byref(cp),
                                       None if ctx.mode == 1 else _lib.ptr(gql), _lib.ptr(gpl), _lib.ptr(dz),
                                       ctypes.byref(cg), _lib.stream_of(q)), "factorized_bwd")
        if ctx.mode == 1:  # torch.round has zero gradient
            dz.zero_()
        return (_from_last(dz), None, None, None, None, *grads)


def _fact_net(dims, params):
    """ic_fact_net for CDF layers of widths `dims` (1, DIMS..., 1) and their flat params
    [w0, b0, f0, w1, b1, f1, ..., w_last, b_last] (CDFEstimator.flat_params order)."""
    net = _lib.ICFactNet()
    L = len(dims) - 1
    net.nlayers = L
    for i, d in enumerate(dims):
        net.dims[i] = int(d)
    k = 0
    for layer in range(L):
        net.w[layer] = params[k].data_ptr()
        net.b[layer] = params[k + 1].data_ptr()
        k += 2
        if layer < L - 1:
            net.f[layer] = params[k].data_ptr()
            k += 1
    return net


class FactorizedNetFn(Function):
    """EntropyModel with any CDF MLP widths (cfg DIMS) and any BIN (entropy_model.py:88-99,
    :198, :229-232, :259-269) on the generic kernels (ic_factorized_*_net)."""

    @staticmethod
    def forward(ctx, z, mode, u, seed, offset, dims, bin_, *params):
        _lib.require_device(z, None if mode == 3 else u, *params)
        if len(dims) - 1 > _lib.FACT_MAXL or max(dims[1:-1] or [1]) > _lib.FACT_MAXW:
            raise NotImplementedError(f"CDF MLP dims {list(dims)}: the generic kernel takes <= {_lib.FACT_MAXL} "
                                      f"layers of width <= {_lib.FACT_MAXW}")
        C = z.shape[1]
        zl = _to_last(z)
        ul = u if (u is None or mode == 3) else _to_last(u.to(z.dtype))
        q = torch.empty_like(zl)
        p = torch.empty_like(zl)
        prm = [t.contiguous() for t in params]
        net = _fact_net(dims, prm)
        _lib.check(_L().ic_factorized_fwd_net(_lib.ptr(zl), _n(zl), C, ctypes.byref(net), float(bin_), int(mode),
                                              _lib.ptr(ul), ctypes.c_ulonglong(seed), ctypes.c_ulonglong(offset),
                                              _lib.ptr(q), _lib.ptr(p), _lib.stream_of(z)), "factorized_fwd_net")
        ctx.conf = (int(mode), C, tuple(dims), float(bin_))
        ctx.save_for_backward(q, *prm)
        return _from_last(q), _from_last(p)

    @staticmethod
    def backward(ctx, gq, gp):
        q, *prm = ctx.saved_tensors
        mode, C, dims, bin_ = ctx.conf
        gql = None if gq is None else _to_last(gq)
        gpl = None if gp is None else _to_last(gp)
        dz = torch.empty_like(q)
        grads = [torch.empty_like(t) for t in prm]
        net = _fact_net(dims, prm)
        g = _lib.ICFactNetGrads()
        k = 0
        for layer in range(len(dims) - 1):
            g.w[layer] = grads[k].data_ptr()
            g.b[layer] = grads[k + 1].data_ptr()
            k += 2
            if layer < len(dims) - 2:
                g.f[layer] = grads[k].data_ptr()
                k += 1
        _lib.check(_L().ic_factorized_bwd_net(_lib.ptr(q), _n(q), C, ctypes.byref(net), bin_,
                                              None if mode == 1 else _lib.ptr(gql), _lib.ptr(gpl), _lib.ptr(dz),
                                              ctypes.byref(g), _lib.stream_of(q)), "factorized_bwd_net")
        if mode == 1:  # torch.round has zero gradient
            dz.zero_()
        return (_from_last(dz), None, None, None, None, None, None, *grads)


class ConditionalFn(Function):
    """SymmetricConditionalModel._quantize + _prob_mass (entropy_model.py:319-352)."""

    @staticmethod
    def forward(ctx, y, scale, mean, kind, mode, u, seed, offset, bin_=1.0):
        _lib.require_device(y, scale, mean, None if mode == 3 else u)
        L = _L()
        y = _dense(y)
        scale = _match(scale, y)
        if mean is not None:
            mean = _match(mean, y)
        if u is not None and mode != 3:  # mode 3: `u` is the Philox device state
            u = _match(u.to(y.dtype), y)
        q = torch.empty_like(y)
        p = torch.empty_like(y)
        _lib.check(L.ic_conditional_fwd_bin(_lib.ptr(y), _lib.ptr(scale), _lib.ptr(mean), _n(y), int(kind),
                                            int(mode), _lib.ptr(u), ctypes.c_ulonglong(seed),
                                            ctypes.c_ulonglong(offset), float(bin_), _lib.ptr(q), _lib.ptr(p),
                                            _lib.stream_of(y)), "conditional_fwd")
        ctx.conf = (int(kind), int(mode), mean is not None, float(bin_))
        ctx.save_for_backward(q, scale, mean)
        return q, p

    @staticmethod
    def backward(ctx, gq, gp):
        q, scale, mean = ctx.saved_tensors
        kind, mode, has_mean, bin_ = ctx.conf
        L = _L()
        gq = None if gq is None else _match(gq, q)
        gp = None if gp is None else _match(gp, q)
        dy = torch.empty_like(q) if ctx.needs_input_grad[0] else None
        ds = torch.empty_like(q) if ctx.needs_input_grad[1] else None
        dm = torch.empty_like(q) if (has_mean and ctx.needs_input_grad[2]) else None
        _lib.check(L.ic_conditional_bwd_bin(_lib.ptr(q), _lib.ptr(scale), _lib.ptr(mean), _n(q), kind, bin_,
                                            _lib.ptr(gq), _lib.ptr(gp), _lib.ptr(dy), _lib.ptr(ds), _lib.ptr(dm),
                                            _lib.stream_of(q)), "conditional_bwd")
        if mode == 1 and dy is not None:  # round: zero gradient through q
            if gp is None:
                dy.zero_()
            else:
                dy.zero_()
        return dy, ds, dm, None, None, None, None, None, None


class QuantizeFn(Function):
    """SymmetricConditionalModel._quantize alone (entropy_model.py:319-336): y + (u - bin/2) in
    training (straight-through: dq/dy = 1), round(y) in evaluation (zero gradient).  The same
    draws, element for element, as ConditionalFn's quantization (ic_quantize)."""

    @staticmethod
    def forward(ctx, y, mode, u, seed, offset, bin_):
        _lib.require_device(y, None if mode == 3 else u)
        y = _dense(y)
        if u is not None and mode != 3:
            u = _match(u.to(y.dtype), y)
        q = torch.empty_like(y)
        _lib.check(_L().ic_quantize(_lib.ptr(y), _n(y), int(mode), _lib.ptr(u), ctypes.c_ulonglong(seed),
                                    ctypes.c_ulonglong(offset), float(bin_), _lib.ptr(q), _lib.stream_of(y)),
                   "quantize")
        ctx.mode = int(mode)
        return q

    @staticmethod
    def backward(ctx, gq):
        if ctx.mode == 1:  # torch.round has zero gradient
            return torch.zeros_like(gq), None, None, None, None, None
        return gq, None, None, None, None, None


def quantize(y, train, u=None, bin_=1.0):
    """The conditional model's quantization on its own (see conditional_likelihood)."""
    if not train:
        mode, seed, off = 1, 0, 0
    elif u is not None:
        mode, seed, off = 0, 0, 0
    else:
        mode, seed = 3, 0
        u, off = _noise.philox_stream(y.numel(), y.device)
    return QuantizeFn.apply(y, mode, u, seed, off, float(bin_))


def conditional_likelihood(q, scale, mean, kind, bin_=1.0):
    """The conditional model's likelihood of already-quantized symbols q (ConditionalFn mode 4:
    q passes through unchanged, gradients reach q and scale as in the fused op)."""
    return ConditionalFn.apply(q, scale, mean, kind, 4, None, 0, 0, float(bin_))[1]


def factorized(z, params, train, u=None, dims=(1, 3, 3, 3, 1), bin_=1.0):
    """Returns (q, p) for EntropyModel; `u` optional injected U[0,1) draws.  The default CDF MLP
    (DIMS [3, 3, 3]) with BIN 1 runs the fused fixed-width kernels, anything else the generic ones."""
    if not train:
        mode, seed, off = 1, 0, 0
    elif u is not None:
        mode, seed, off = 0, 0, 0
    else:
        mode, seed = 3, 0
        u, off = _noise.philox_stream(z.numel(), z.device)
    if list(dims) == [1, 3, 3, 3, 1] and float(bin_) == 1.0:
        return FactorizedFn.apply(z, mode, u, seed, off, *params)
    return FactorizedNetFn.apply(z, mode, u, seed, off, tuple(int(d) for d in dims), float(bin_), *params)


def conditional(y, scale, mean, kind, train, u=None, bin_=1.0):
    if not train:
        mode, seed, off = 1, 0, 0
    elif u is not None:
        mode, seed, off = 0, 0, 0
    else:
        mode, seed = 3, 0
        u, off = _noise.philox_stream(y.numel(), y.device)
    return ConditionalFn.apply(y, scale, mean, kind, mode, u, seed, off, float(bin_))


class SqDiffFn(Function):
    """(a - b)^2 elementwise: nn.MSELoss(reduction='none')."""

    @staticmethod
    def forward(ctx, a, b):
        _lib.require_device(a, b)
        a = _dense(a)
        b = _match(b, a)
        out = torch.empty_like(a)
        _lib.check(_L().ic_sqdiff_fwd(_lib.ptr(a), _lib.ptr(b), _n(a), _lib.ptr(out), _lib.stream_of(a)),
                   "sqdiff_fwd")
        ctx.save_for_backward(a, b)
        return out

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        g = _match(g, a)
        ga = torch.empty_like(a) if ctx.needs_input_grad[0] else None
        gb = torch.empty_like(b) if ctx.needs_input_grad[1] else None
        _lib.check(_L().ic_sqdiff_bwd(_lib.ptr(a), _lib.ptr(b), _lib.ptr(g), _n(a), _lib.ptr(ga), _lib.ptr(gb),
                                      _lib.stream_of(a)), "sqdiff_bwd")
        return ga, gb


class MSSSIMFn(Function):
    """SSIM / MS-SSIM loss (modelling/loss.py:48-188)."""

    @staticmethod
    def forward(ctx, a, b, conf):
        _lib.require_device(a, b)
        L = _L()
        a = a.contiguous()
        b = b.contiguous()
        N, C, H, W = a.shape
        (nlev, fs, sigma, max_val, log_scale, single, k1, k2, eps, weights) = conf
        sb = L.ic_msssim_state_bytes(N, C, H, W, nlev, fs)
        if sb == 0:
            raise RuntimeError(f"ms-ssim: image {H}x{W} too small for {nlev} levels of a {fs}x{fs} window")
        state = torch.empty(sb // 4, device=a.device, dtype=torch.float32)
        nb = L.ic_msssim_ws(N, C, H, W, nlev, fs)
        buf = _ws(nb, a.device)
        wts = (ctypes.c_float * nlev)(*weights)
        out = torch.empty((N,) if (single and log_scale) else (), device=a.device, dtype=torch.float32)
        _lib.check(L.ic_msssim_fwd(_lib.ptr(a), _lib.ptr(b), N, C, H, W, nlev, fs, sigma, max_val, int(log_scale),
                                   int(single), k1, k2, eps, ctypes.cast(wts, ctypes.c_void_p), _lib.ptr(out),
                                   _lib.ptr(state), _lib.ptr(buf), nb, _lib.stream_of(a)), "msssim_fwd")
        ctx.conf = conf
        ctx.shape = (N, C, H, W)
        ctx.save_for_backward(state)
        return out

    @staticmethod
    def backward(ctx, g):
        (state,) = ctx.saved_tensors
        L = _L()
        N, C, H, W = ctx.shape
        (nlev, fs, sigma, max_val, log_scale, single, k1, k2, eps, weights) = ctx.conf
        g = g.contiguous()
        ga = torch.empty((N, C, H, W), device=g.device, dtype=torch.float32) if ctx.needs_input_grad[0] else None
        gb = torch.empty((N, C, H, W), device=g.device, dtype=torch.float32) if ctx.needs_input_grad[1] else None
        nb = L.ic_msssim_ws(N, C, H, W, nlev, fs)
        buf = _ws(nb, g.device)
        wts = (ctypes.c_float * nlev)(*weights)
        _lib.check(L.ic_msssim_bwd(N, C, H, W, nlev, fs, sigma, max_val, int(log_scale), int(single), k1, k2, eps,
                                   ctypes.cast(wts, ctypes.c_void_p), _lib.ptr(g), _lib.ptr(state), _lib.ptr(ga),
                                   _lib.ptr(gb), _lib.ptr(buf), nb, _lib.stream_of(g)), "msssim_bwd")
        return ga, gb, None


def msssim(img1, img2, mod, weights, single_scale):
    conf = (len(weights), int(mod.filter_size), float(mod.filter_sigma), float(mod.max_val), bool(mod.log_scale),
            bool(single_scale), float(mod.k1), float(mod.k2), float(mod.eps), [float(w) for w in weights])
    return MSSSIMFn.apply(img1, img2, conf)
