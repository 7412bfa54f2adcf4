"""Autograd functions over the HIP kernels of libimgcomp.so.

Every forward/backward here launches hand-written gfx950 kernels through the
C ABI (include/imgcomp.h) on torch's current stream.  PyTorch provides only
allocation (caching allocator), stream handles and the autograd graph.
There is deliberately no CPU / eager fallback: CPU tensors raise.

Layout convention: activations with >= 32 channels live in NHWC
(torch.channels_last) so every GEMM operand row is channel-contiguous; the
3-channel image tensors stay NCHW and take the generic gather path.
"""
import os
import threading
import weakref

import torch
from torch.autograd import Function

from . import _lib
from . import noise as _noise

CL = torch.channels_last


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
# bias-gradient pass over the same tensor.  Keyed by the gradient tensor itself (device +
# storage pointer, checked against a weakref and the version counter): a gradient changed in
# between (or any other tensor) falls back to the pass.  Backward passes of several devices may
# run concurrently (one autograd thread per device; nn.DataParallel replicas), so the table is
# locked.
_COLSUMS = {}
_COLSUMS_LOCK = threading.Lock()


def _colsum_key(t):
    return (t.device.index, t.data_ptr())


def _put_colsum(t, s):
    with _COLSUMS_LOCK:
        for k in [k for k, (r, _, _) in _COLSUMS.items() if r() is None]:
            del _COLSUMS[k]
        _COLSUMS[_colsum_key(t)] = (weakref.ref(t), t._version, s)


def _take_colsum(t):
    with _COLSUMS_LOCK:
        e = _COLSUMS.pop(_colsum_key(t), None)
    if e is None:
        return None
    r, ver, s = e
    return s if (r() is t and t._version == ver) else None


# ---------------------------------------------------------- bf16 activation copies (config C3)
# A GDN whose output feeds a conv forward on the bf16 DMA tiles (GDN.xb & 1), or whose input
# gradient feeds a transposed conv's input gradient there (GDN.xb & 2), writes that tensor's compact
# NHWC bf16 copy in the same kernel (torch.ops.imgcomp.gdn_fwd_xb / gdn_bwd_sum_xb) and leaves it
# here, keyed like the column sums above; the consuming conv takes it (conv2d_fwd_xb /
# conv_transpose2d_dgrad_xb) and reads 2 B per element instead of converting the fp32 tensor.
_BF16 = {}
_BF16_LOCK = threading.Lock()
BF16_COPY_STATS = {"put": 0, "hit": 0}


def _put_bf16(t, tb):
    with _BF16_LOCK:
        for k in [k for k, (r, _, _) in _BF16.items() if r() is None]:
            del _BF16[k]
        _BF16[_colsum_key(t)] = (weakref.ref(t), t._version, tb)
        BF16_COPY_STATS["put"] += 1


def _take_bf16(t):
    with _BF16_LOCK:
        e = _BF16.pop(_colsum_key(t), None)
    if e is None:
        return None
    r, ver, tb = e
    if r() is t and t._version == ver and tb.shape == t.shape and tb.stride() == t.stride():
        BF16_COPY_STATS["hit"] += 1
        return tb
    return None


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
        xb = _take_bf16(x) if int(math) & MATH["bf16"] else None
        if xb is not None:
            y = _lib.ops().conv2d_fwd_xb(x, xb, w, b, stride, padding, int(act), int(math))
        else:
            y = _lib.ops().conv2d_fwd(x, w, b, stride, padding, int(act), int(math))
        _log_plan("conv2d_fwd", x, y, w.shape[2], stride, padding, math)
        # x's bf16 copy, for the weight gradient with dy's (conv2d_wgrad_xb); held to the backward
        # (2 B per element of x) only when that weight gradient will run
        ctx.xb = xb if ctx.needs_input_grad[1] else None
        ctx.conf = (stride, padding, act, b is not None, int(math))
        ctx.save_for_backward(x, w, y if act else None)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w, y = ctx.saved_tensors
        stride, padding, act, has_b, math = ctx.conf
        # the bias gradient formed by gy's producer (taken only where this node owns the bias gradient)
        pre = _take_colsum(gy) if (has_b and not act and ctx.needs_input_grad[2]) else None
        gyb = _take_bf16(gy) if (math & MATH["bf16"]) and not act else None
        if act:
            gy = relu_bwd(y, gy)
        gy = _cl(gy)
        dx = dw = db = None
        ops, k = _lib.ops(), w.shape[2]
        if ctx.needs_input_grad[0]:
            if gyb is not None and gyb.stride() == gy.stride():
                dx = ops.conv2d_dgrad_xb(gy, gyb, w, x, stride, padding, math)
            else:
                dx = ops.conv2d_dgrad(gy, w, x, stride, padding, math)
            _log_plan("conv2d_dgrad", gy, dx, k, stride, padding, math)
        if ctx.needs_input_grad[1] or (has_b and ctx.needs_input_grad[2]):
            xb, ctx.xb = ctx.xb, None
            if xb is not None and gyb is not None and gyb.stride() == gy.stride():
                dw, db = ops.conv2d_wgrad_xb(x, xb, gy, gyb, w, stride, padding, has_b and pre is None, math)
            else:
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
        xb = _take_bf16(x) if int(math) & MATH["bf16"] else None
        if xb is not None:
            y = _lib.ops().conv_transpose2d_fwd_xb(x, xb, w, b, stride, padding, output_padding, int(act), int(math))
        else:
            y = _lib.ops().conv_transpose2d_fwd(x, w, b, stride, padding, output_padding, int(act), int(math))
        _log_plan("conv_transpose2d_fwd", x, y, w.shape[2], stride, padding, math)
        # x's bf16 copy, for the weight gradient with dy's (conv_transpose2d_wgrad_xb); held to the backward
        # (2 B per element of x) only when that weight gradient will run
        ctx.xb = xb if ctx.needs_input_grad[1] else None
        ctx.conf = (stride, padding, act, b is not None, int(math))
        ctx.save_for_backward(x, w, y if act else None)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w, y = ctx.saved_tensors
        stride, padding, act, has_b, math = ctx.conf
        # the bias gradient formed by gy's producer (taken only where this node owns the bias gradient)
        pre = _take_colsum(gy) if (has_b and not act and ctx.needs_input_grad[2]) else None
        gyb = _take_bf16(gy) if (math & MATH["bf16"]) and not act else None
        if act:
            gy = relu_bwd(y, gy)
        gy = _cl(gy)
        dx = dw = db = None
        ops, k = _lib.ops(), w.shape[2]
        if ctx.needs_input_grad[0]:
            if gyb is not None and gyb.stride() == gy.stride():
                dx = ops.conv_transpose2d_dgrad_xb(gy, gyb, w, x, stride, padding, math)
            else:
                dx = ops.conv_transpose2d_dgrad(gy, w, x, stride, padding, math)
            _log_plan("conv_transpose2d_dgrad", gy, dx, k, stride, padding, math)
        if ctx.needs_input_grad[1] or (has_b and ctx.needs_input_grad[2]):
            xb, ctx.xb = ctx.xb, None
            if xb is not None and gyb is not None and gyb.stride() == gy.stride():
                dw, db = ops.conv_transpose2d_wgrad_xb(x, xb, gy, gyb, w, stride, padding, has_b and pre is None, math)
            else:
                dw, db = ops.conv_transpose2d_wgrad(x, gy, w, stride, padding, has_b and pre is None, math)
            _log_plan("conv_transpose2d_wgrad", x, gy, k, stride, padding, math)
            db = (db if pre is None else pre) if has_b else None
        return dx, dw, db, None, None, None, None, None


# include/imgcomp.h IC_MATH_*: "fp32" exact fp32 MFMA; "bf16" bf16 operands, fp32 accumulation
# (reduced precision, config C3); "fp32_split" fp32 arithmetic on the bf16 MFMA through an exact
# three-term bf16 split of both operands (six products, error of an fp32 fma chain)
MATH = {"fp32": 0, "bf16": 1, "fp32_split": 2}


# ---------------------------------------------------------- eval-mode weight caching
# Inside `weight_cache()` (Evaluator.run_eval's eager path; GraphForward does not enter it: a
# captured graph already holds its pack launches), forwards without autograd keep each
# conv weight's MFMA pack in a workspace of its own and skip the pack launch while the weight is
# unchanged (include/imgcomp.h IC_MATH_WPACKED), and NonNegativeParam keeps its re-parameterised
# value: the eval forward then launches only the layer kernels.  An entry is valid for the same
# tensor object (weakref) at the same version counter (every in-place update bumps it: torch ops,
# load_state_dict's copy_, and solver.AdamW, which bumps it after its kernel) on the same stream
# (the pack workspace also holds the split-K partials) and, for packs, the same operand geometry.
# The stream is keyed by its raw handle: a stream destroyed inside one scope whose handle is reused
# by a new stream would find the old entry, but the weakref and version checks still decide a hit,
# and every entry is dropped when the outermost scope exits.
IC_MATH_WPACKED = 4
_WCACHE = {}
_WCACHE_LOCK = threading.Lock()
_WCACHE_DEPTH = [0]


class weight_cache:
    """Scope in which no-grad forwards reuse weight packs and re-parameterisations.  Entries are
    dropped when the outermost scope exits."""

    def __enter__(self):
        with _WCACHE_LOCK:
            _WCACHE_DEPTH[0] += 1
        return self

    def __exit__(self, *exc):
        with _WCACHE_LOCK:
            _WCACHE_DEPTH[0] -= 1
            if _WCACHE_DEPTH[0] == 0:
                _WCACHE.clear()
        return False


def _wcache_on(t):
    return _WCACHE_DEPTH[0] > 0 and not torch.is_grad_enabled() and t.is_cuda


def _wcache_get(kind, t, geom):
    """(entry dict, hit) for tensor t; the entry is reset unless t, its version and geom match."""
    stream = torch.cuda.current_stream(t.device).cuda_stream
    key = (kind, t.device.index, t.data_ptr(), stream, geom)  # one entry per geometry (portrait / landscape)
    with _WCACHE_LOCK:
        for k in [k for k, e in _WCACHE.items() if e["ref"]() is None]:
            del _WCACHE[k]
        e = _WCACHE.get(key)
        hit = e is not None and e["ref"]() is t and e["ver"] == t._version
        if not hit:
            ws = e.get("ws") if e is not None else None  # keep the (grown) workspace
            e = {"ref": weakref.ref(t), "ver": t._version}
            if ws is not None:
                e["ws"] = ws
            _WCACHE[key] = e
        return e, hit


def _cached_conv(op, x, weight, bias, args, math):
    _lib.require_device(x, weight, bias)
    x = _cl(x)
    w = weight.contiguous()
    b = None if bias is None else bias.contiguous()
    geom = (op, tuple(x.shape), tuple(x.stride()), tuple(w.shape), args, int(math))
    e, hit = _wcache_get("pack", weight, geom)
    if "ws" not in e:
        e["ws"] = torch.empty(16, dtype=torch.uint8, device=x.device)
    m = int(math) | (IC_MATH_WPACKED if hit else 0)
    fn = getattr(_lib.ops(), op)
    y = fn(x, w, b, *args, m, e["ws"])
    _log_plan(op.replace("_ws", ""), x, y, w.shape[2], args[0], args[1], math)
    return y


def nonneg_cached(p, bound, pedestal):
    """NonNegFn.apply(p, ...) kept per (tensor, version) inside `weight_cache()`."""
    if not _wcache_on(p):
        return NonNegFn.apply(p, bound, pedestal)
    e, hit = _wcache_get("nonneg", p, (float(bound), float(pedestal)))
    if not hit or "val" not in e:
        e["val"] = NonNegFn.apply(p, bound, pedestal)
    return e["val"]


# ---------------------------------------------------------- weight gradients on a stream of their own
# A conv whose forward runs on a stream registered here (the hyperprior side stream, see
# Compressor2018) gets its weight / bias gradient as a separate autograd node whose forward, and so
# whose backward, runs on the registered weight-gradient stream:
#     y = Join(ConvData(x, w.detach(), b.detach()), WGrad(x, w, b))
# WGrad is created first, so its sequence number is lower than ConvData's: when Join's gradient
# arrives, the engine runs ConvData's backward (the input gradient, on the side stream) before
# WGrad's (the weight gradient, on its own stream).  The hyperprior's backward chain -- the input
# gradients that g_a's backward waits for -- then no longer queues behind its weight gradients,
# which run beside the rest of the step.  The parameters' AccumulateGrad nodes are made on the
# weight-gradient stream (the parameters enter the graph through WGrad), the end of backward joins
# every leaf stream, and the arithmetic is the unsplit conv's (the same kernels on the same operands).
_WG_STREAMS = {}   # producing stream handle -> the stream its convs' weight gradients run on
_ZERO = {}         # device index -> a zero scalar (WGrad's output is an expanded view of it)


def route_weight_gradients(stream, wstream):
    """Convs run on `stream` compute their weight gradients on `wstream` (see above)."""
    _WG_STREAMS[stream.cuda_stream] = wstream


def _wgrad_stream(x, weight):
    if not _WG_STREAMS or not x.is_cuda or not torch.is_grad_enabled() or not weight.requires_grad:
        return None
    return _WG_STREAMS.get(torch.cuda.current_stream(x.device).cuda_stream)


class _ConvWGradFn(Function):
    """The weight and bias gradient of a conv (WGrad above).  Forward: nothing (an expanded zero of
    the conv output's shape); backward, on the stream the forward ran on: the wgrad kernels."""

    @staticmethod
    def forward(ctx, x, weight, bias, holder, conf, shape):
        dev = x.device.index
        if dev not in _ZERO:
            _ZERO[dev] = torch.zeros((), device=x.device, dtype=torch.float32)
        ctx.holder = holder
        ctx.conf = conf
        ctx.has_b = bias is not None
        ctx.save_for_backward(x, weight)
        return _ZERO[dev].expand(shape)

    @staticmethod
    def backward(ctx, gz):
        x, w = ctx.saved_tensors
        transposed, stride, padding, act, math = ctx.conf
        cur = torch.cuda.current_stream(x.device)
        x.record_stream(cur)   # x and the incoming gradient were allocated on the producing stream
        gz.record_stream(cur)
        pre = _take_colsum(gz) if (ctx.has_b and not act) else None  # bias gradient formed by gz's producer
        if pre is not None:
            pre.record_stream(cur)
        if act:
            # the fused-ReLU output was allocated on the producing (side) stream and is read here
            ctx.holder["y"].record_stream(cur)
        gy = relu_bwd(ctx.holder["y"], gz) if act else gz
        gy = _cl(gy)
        ops, k = _lib.ops(), w.shape[2]
        fb = ctx.has_b and pre is None
        if transposed:
            dw, db = ops.conv_transpose2d_wgrad(x, gy, w, stride, padding, fb, math)
            _log_plan("conv_transpose2d_wgrad", x, gy, k, stride, padding, math)
        else:
            dw, db = ops.conv2d_wgrad(x, gy, w, stride, padding, fb, math)
            _log_plan("conv2d_wgrad", x, gy, k, stride, padding, math)
        return None, dw, ((db if pre is None else pre) if ctx.has_b else None), None, None, None


class _JoinFn(Function):
    """y, passing its gradient to both the input-gradient and the weight-gradient node."""

    @staticmethod
    def forward(ctx, y, z):
        return y.view_as(y)

    @staticmethod
    def backward(ctx, g):
        return g, g


def _deferred_wgrad(ws, data_fn, x, weight, bias, args, conf, shape):
    ws.wait_stream(torch.cuda.current_stream(x.device))
    holder = {}
    with torch.cuda.stream(ws):
        z = _ConvWGradFn.apply(x, weight, bias, holder, conf, shape)
    y = data_fn.apply(x, weight.detach(), None if bias is None else bias.detach(), *args)
    if conf[3]:
        holder["y"] = y
    return _JoinFn.apply(y, z)


def conv2d(x, weight, bias=None, stride=1, padding=0, act=0, math=0):
    """`math` (forward and input gradient): 0 fp32 (default), 1 bf16 operands with fp32
    accumulation, 2 fp32 by exact bf16 split (see MATH)."""
    if _wcache_on(x):
        return _cached_conv("conv2d_fwd_ws", x, weight, bias, (int(stride), int(padding), int(act)), math)
    ws = _wgrad_stream(x, weight)
    if ws is not None:
        k = weight.shape[2]
        N, _, H, W = x.shape
        shape = (N, weight.shape[0], (H + 2 * padding - k) // stride + 1, (W + 2 * padding - k) // stride + 1)
        return _deferred_wgrad(ws, Conv2dFn, x, weight, bias, (int(stride), int(padding), int(act), int(math)),
                               (False, int(stride), int(padding), int(act), int(math)), shape)
    return Conv2dFn.apply(x, weight, bias, int(stride), int(padding), int(act), int(math))


def conv_transpose2d(x, weight, bias=None, stride=1, padding=0, output_padding=0, act=0, math=0):
    if _wcache_on(x):
        return _cached_conv("conv_transpose2d_fwd_ws", x, weight, bias,
                            (int(stride), int(padding), int(output_padding), int(act)), math)
    ws = _wgrad_stream(x, weight)
    if ws is not None:
        k = weight.shape[2]
        N, _, H, W = x.shape
        shape = (N, weight.shape[1], (H - 1) * stride - 2 * padding + k + output_padding,
                 (W - 1) * stride - 2 * padding + k + output_padding)
        return _deferred_wgrad(ws, ConvTranspose2dFn, x, weight, bias,
                               (int(stride), int(padding), int(output_padding), int(act), int(math)),
                               (True, int(stride), int(padding), int(act), int(math)), shape)
    return ConvTranspose2dFn.apply(x, weight, bias, int(stride), int(padding), int(output_padding), int(act),
                                   int(math))


# ============================================================== GDN
_NORM_RECOMPUTE = os.environ.get("IMGCOMP_GDN_NORM_RECOMPUTE", "1") != "0"  # A/B knob (diagnostic)


def _norm_recompute(x, math, math_fwd):
    """Whether GDN leaves norm out of its forward and recomputes it in the backward: bf16 operands in
    both directions at C = 192 (the fused bf16 kernels, config C3)."""
    return bool(_NORM_RECOMPUTE and (int(math) & MATH["bf16"]) and (int(math_fwd) & MATH["bf16"]) and x.dim() == 4
                and x.shape[1] == 192)


class GDNFn(Function):
    """modelling/layers/gdn.py:84-86 given re-parameterised gamma (C,C,1,1), beta (C,)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, inverse, math=0, math_fwd=0, xb=0):
        _lib.require_device(x, gamma, beta)
        x = _cl(x)
        g = gamma.contiguous()
        b = beta.contiguous()
        # xb & 1: y's bf16 copy for the next conv's forward; xb & 2: dx's for the previous
        # transposed conv's input gradient (bf16 operands only; see _put_bf16)
        # (not under the eval weight cache: its convs (_cached_conv) never take the copy)
        copy = bool((xb & 1) and (int(math_fwd) & MATH["bf16"]) and not _wcache_on(x))
        # bf16 operands at C = 192 (config C3): norm is not stored; the backward forms it again from
        # x, gamma and beta, bitwise as the forward did (include/imgcomp.h ic_gdn_fwd_rn, round 6)
        ctx.rn = _norm_recompute(x, math, math_fwd)
        if ctx.rn:
            y, yb = _lib.ops().gdn_fwd_rn(x, g, b, bool(inverse), int(math_fwd), copy)
            norm = b  # saved in norm's place: the backward's beta
        elif copy:
            y, norm, yb = _lib.ops().gdn_fwd_xb(x, g, b, bool(inverse), int(math_fwd))
        else:
            y, norm = _lib.ops().gdn_fwd(x, g, b, bool(inverse), int(math_fwd))
        if copy:
            _put_bf16(y, yb)
        _log_plan("gdn_fwd", x, None, math=math_fwd)
        ctx.inverse = bool(inverse)
        ctx.math = int(math)
        ctx.xb = int(xb)
        ctx.save_for_backward(x, norm, g)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, norm, g = ctx.saved_tensors
        gy = _match(gy, x)
        # dx's column sums come with it (the fused backward forms them from its dx tiles): the
        # bias gradient of the conv that produced x, taken by that conv's backward (_take_colsum)
        copy = bool((ctx.xb & 2) and (ctx.math & MATH["bf16"]))
        if ctx.rn:  # `norm` holds beta here
            dx, dg, dbeta, dxsum, dxb = _lib.ops().gdn_bwd_sum_rn(x, norm, gy, g, ctx.inverse, ctx.math, copy)
            if copy:
                _put_bf16(dx, dxb)
        elif copy:
            dx, dg, dbeta, dxsum, dxb = _lib.ops().gdn_bwd_sum_xb(x, norm, gy, g, ctx.inverse, ctx.math)
            _put_bf16(dx, dxb)
        else:
            dx, dg, dbeta, dxsum = _lib.ops().gdn_bwd_sum(x, norm, gy, g, ctx.inverse, ctx.math)
        _put_colsum(dx, dxsum)
        _log_plan("gdn_bwd", x, None, math=ctx.math)
        return dx, dg, dbeta, None, None, None, None


def gdn(x, gamma, beta, inverse=False, math=0, math_fwd=0, xb=0):
    """`math` 2: the backward's dgamma GEMM in split arithmetic (C = 192); `math_fwd` 2: the
    forward on the split implicit GEMM instead of the fused fp32 kernel; `xb`: bf16 copies of the
    output (1) / input gradient (2) for the neighbouring conv (bf16 operands, see _put_bf16)."""
    return GDNFn.apply(x, gamma, beta, bool(inverse), int(math), int(math_fwd), int(xb))


class NonNegFn(Function):
    """NonNegativeParam.forward (gdn.py:59-62): max(p, bound)^2 - pedestal."""

    @staticmethod
    def forward(ctx, p, bound, pedestal):
        _lib.require_device(p)
        p = p.contiguous()
        out = _lib.ops().nonneg_fwd(p, float(bound), float(pedestal))
        ctx.bound = float(bound)
        ctx.save_for_backward(p)
        return out

    @staticmethod
    def backward(ctx, g):
        (p,) = ctx.saved_tensors
        return _lib.ops().nonneg_bwd(p, _match(g, p), ctx.bound), None, None


class NonNegMultiFn(Function):
    """NonNegativeParam.forward (gdn.py:59-62) of several parameters in one launch, and their
    gradients in one launch (torch.ops.imgcomp.nonneg_multi_*; bitwise NonNegFn per tensor).
    Compressor2018 applies it to each transform's GDN gamma / beta once per forward: 2 launches per
    transform per step instead of 12 (6 GDN layers x 2 parameters, forward and backward)."""

    @staticmethod
    def forward(ctx, bounds, peds, *params):
        _lib.require_device(*params)
        ps = [p.contiguous() for p in params]
        outs = _lib.ops().nonneg_multi_fwd(ps, [float(b) for b in bounds], [float(q) for q in peds])
        ctx.bounds = [float(b) for b in bounds]
        ctx.save_for_backward(*ps)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gs):
        ps = ctx.saved_tensors
        out = [None] * len(ps)
        idx = [i for i, g in enumerate(gs) if g is not None]
        if idx:
            gi = _lib.ops().nonneg_multi_bwd([ps[i] for i in idx], [_match(gs[i], ps[i]) for i in idx],
                                             [ctx.bounds[i] for i in idx])
            for i, g in zip(idx, gi):
                out[i] = g
        return (None, None, *out)


# ============================================================== elementwise
class BoundFn(Function):
    """LowerBound (upper=False) / UpperBound (upper=True), layers/bound.py:28-59."""

    @staticmethod
    def forward(ctx, x, bound, upper):
        _lib.require_device(x)
        x = _dense(x)
        y = _lib.ops().bound_fwd(x, float(bound), bool(upper))
        ctx.conf = (float(bound), bool(upper))
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        bound, upper = ctx.conf
        return _lib.ops().bound_bwd(x, _match(g, x), bound, upper), None, None


class ReLUFn(Function):
    @staticmethod
    def forward(ctx, x):
        _lib.require_device(x)
        y = _lib.ops().relu_fwd(_dense(x))
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, g):
        (y,) = ctx.saved_tensors
        return relu_bwd(y, g)


def relu_bwd(y, g):
    return _lib.ops().relu_bwd(y, _match(g, y))


class AbsFn(Function):
    @staticmethod
    def forward(ctx, x):
        _lib.require_device(x)
        x = _dense(x)
        ctx.save_for_backward(x)
        return _lib.ops().abs_fwd(x)

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        return _lib.ops().abs_bwd(x, _match(g, x))


class ExpClampFn(Function):
    """torch.clamp(v.exp(), lo, hi) of prior_synthesis.py:72."""

    @staticmethod
    def forward(ctx, v, lo, hi):
        _lib.require_device(v)
        s, e = _lib.ops().exp_clamp_fwd(_dense(v), float(lo), float(hi))
        ctx.conf = (float(lo), float(hi))
        ctx.save_for_backward(e)
        return s

    @staticmethod
    def backward(ctx, g):
        (e,) = ctx.saved_tensors
        lo, hi = ctx.conf
        return _lib.ops().exp_clamp_bwd(e, _match(g, e), lo, hi), None, None


# ============================================================== losses
class CELossFn(Function):
    """_ce_loss (entropy_model.py:185): sum clamp(-ln(p+1e-10)/ln 2, 0, 50)."""

    @staticmethod
    def forward(ctx, p):
        _lib.require_device(p)
        p = _dense(p)
        ctx.save_for_backward(p)
        return _lib.ops().ce_loss_fwd(p)

    @staticmethod
    def backward(ctx, g):
        (p,) = ctx.saved_tensors
        return _lib.ops().ce_loss_bwd(p, g)


class MSEFn(Function):
    """nn.MSELoss(reduction='mean')(input, target)."""

    @staticmethod
    def forward(ctx, a, b):
        _lib.require_device(a, b)
        a = _dense(a)
        b = _match(b, a)
        ctx.save_for_backward(a, b)
        return _lib.ops().mse_fwd(a, b)

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        ga, gb = _lib.ops().mse_bwd(a, b, g, ctx.needs_input_grad[0], ctx.needs_input_grad[1])
        return (ga if ctx.needs_input_grad[0] else None), (gb if ctx.needs_input_grad[1] else None)


# ============================================================== entropy models
def _to_last(t):
    """(N, C, *) -> dense (N, *, C) so that channel = flat index % C."""
    return t.movedim(1, -1).contiguous()


def _from_last(t):
    return t.movedim(-1, 1)


def _noise_arg(z, mode, u, last=False):
    """The `u` operand of the quantizers: injected U[0,1) draws (mode 0, laid out like the
    operand), the device Philox state (mode 3) or nothing."""
    if u is None or mode == 3:
        return u
    u = u.to(z.dtype)
    return _to_last(u) if last else _match(u, z)


class FactorizedFn(Function):
    """EntropyModel._quantize + _prob_mass (entropy_model.py:216-269).
    Returns (q, p) in the input's logical (N, C, *) shape."""

    @staticmethod
    def forward(ctx, z, mode, u, seed, offset, *params):
        _lib.require_device(z, None if mode == 3 else u, *params)
        C = z.shape[1]
        zl = _to_last(z)
        prm = [t.contiguous() for t in params]
        q, p = _lib.ops().factorized_fwd(zl, C, prm, int(mode), _noise_arg(zl, mode, u, last=True), int(seed),
                                         int(offset))
        ctx.mode = int(mode)
        ctx.C = C
        ctx.save_for_backward(q, *prm)
        return _from_last(q), _from_last(p)

    @staticmethod
    def backward(ctx, gq, gp):
        q, *prm = ctx.saved_tensors
        gql = None if (gq is None or ctx.mode == 1) else _to_last(gq)
        gpl = None if gp is None else _to_last(gp)
        dz, grads = _lib.ops().factorized_bwd(q, ctx.C, prm, gql, gpl)
        if ctx.mode == 1:  # torch.round has zero gradient
            dz.zero_()
        return (_from_last(dz), None, None, None, None, *grads)


class FactorizedNetFn(Function):
    """EntropyModel with any CDF MLP widths (cfg DIMS) and any BIN (entropy_model.py:88-99,
    :198, :229-232, :259-269) on the generic kernels (torch.ops.imgcomp.factorized_net_*): the
    register kernels up to 5 hidden layers of width <= 8, the wide kernels beyond (up to 31 hidden
    layers of width <= 256)."""

    @staticmethod
    def forward(ctx, z, mode, u, seed, offset, dims, bin_, *params):
        _lib.require_device(z, None if mode == 3 else u, *params)
        if len(dims) - 1 > _lib.FACT_NET_MAXL or max(dims[1:-1] or [1]) > _lib.FACT_WIDE_MAXW:
            raise NotImplementedError(f"CDF MLP dims {list(dims)}: the kernels take <= {_lib.FACT_NET_MAXL} "
                                      f"layers of width <= {_lib.FACT_WIDE_MAXW}")
        C = z.shape[1]
        zl = _to_last(z)
        prm = [t.contiguous() for t in params]
        q, p = _lib.ops().factorized_net_fwd(zl, C, list(dims), float(bin_), prm, int(mode),
                                             _noise_arg(zl, mode, u, last=True), int(seed), int(offset))
        ctx.conf = (int(mode), C, tuple(dims), float(bin_))
        ctx.save_for_backward(q, *prm)
        return _from_last(q), _from_last(p)

    @staticmethod
    def backward(ctx, gq, gp):
        q, *prm = ctx.saved_tensors
        mode, C, dims, bin_ = ctx.conf
        gql = None if (gq is None or mode == 1) else _to_last(gq)
        gpl = None if gp is None else _to_last(gp)
        dz, grads = _lib.ops().factorized_net_bwd(q, C, list(dims), bin_, prm, gql, gpl)
        if mode == 1:  # torch.round has zero gradient
            dz.zero_()
        return (_from_last(dz), None, None, None, None, None, None, *grads)


class ConditionalFn(Function):
    """SymmetricConditionalModel._quantize + _prob_mass (entropy_model.py:319-352)."""

    @staticmethod
    def forward(ctx, y, scale, mean, kind, mode, u, seed, offset, bin_=1.0):
        _lib.require_device(y, scale, mean, None if mode == 3 else u)
        y = _dense(y)
        scale = _match(scale, y)
        if mean is not None:
            mean = _match(mean, y)
        q, p = _lib.ops().conditional_fwd(y, scale, mean, int(kind), int(mode), _noise_arg(y, mode, u), int(seed),
                                          int(offset), float(bin_))
        ctx.conf = (int(kind), int(mode), mean is not None, float(bin_))
        ctx.save_for_backward(q, scale, mean)
        return q, p

    @staticmethod
    def backward(ctx, gq, gp):
        q, scale, mean = ctx.saved_tensors
        kind, mode, has_mean, bin_ = ctx.conf
        gq = None if gq is None else _match(gq, q)
        gp = None if gp is None else _match(gp, q)
        need = ctx.needs_input_grad
        dy, ds, dm = _lib.ops().conditional_bwd(q, scale, mean, kind, bin_, gq, gp, need[0], need[1],
                                                has_mean and need[2])
        dy = dy if need[0] else None
        if mode == 1 and dy is not None:  # round: zero gradient through q
            dy.zero_()
        return (dy, ds if need[1] else None, dm if (has_mean and need[2]) else None,
                None, None, None, None, None, None)


class QuantizeFn(Function):
    """SymmetricConditionalModel._quantize alone (entropy_model.py:319-336): y + (u - bin/2) in
    training (straight-through: dq/dy = 1), round(y) in evaluation (zero gradient).  The same
    draws, element for element, as ConditionalFn's quantization (torch.ops.imgcomp.quantize)."""

    @staticmethod
    def forward(ctx, y, mode, u, seed, offset, bin_):
        _lib.require_device(y, None if mode == 3 else u)
        y = _dense(y)
        q = _lib.ops().quantize(y, int(mode), _noise_arg(y, mode, u), int(seed), int(offset), float(bin_))
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
        ctx.save_for_backward(a, b)
        return _lib.ops().sqdiff_fwd(a, b)

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        ga, gb = _lib.ops().sqdiff_bwd(a, b, _match(g, a), ctx.needs_input_grad[0], ctx.needs_input_grad[1])
        return (ga if ctx.needs_input_grad[0] else None), (gb if ctx.needs_input_grad[1] else None)


class MSSSIMFn(Function):
    """SSIM / MS-SSIM loss (modelling/loss.py:48-188)."""

    @staticmethod
    def forward(ctx, a, b, conf):
        _lib.require_device(a, b)
        (nlev, fs, sigma, max_val, log_scale, single, k1, k2, eps, weights) = conf
        out, state = _lib.ops().msssim_fwd(a, b, nlev, fs, sigma, max_val, bool(log_scale), int(single), k1, k2, eps,
                                           list(weights))
        ctx.conf = conf
        ctx.shape = tuple(a.shape)
        ctx.save_for_backward(state)
        return out

    @staticmethod
    def backward(ctx, g):
        (state,) = ctx.saved_tensors
        (nlev, fs, sigma, max_val, log_scale, single, k1, k2, eps, weights) = ctx.conf
        need = ctx.needs_input_grad
        ga, gb = _lib.ops().msssim_bwd(g, state, list(ctx.shape), nlev, fs, sigma, max_val, bool(log_scale),
                                       int(single), k1, k2, eps, list(weights), need[0], need[1])
        return (ga if need[0] else None), (gb if need[1] else None), None


def msssim(img1, img2, mod, weights, single_scale):
    conf = (len(weights), int(mod.filter_size), float(mod.filter_sigma), float(mod.max_val), bool(mod.log_scale),
            bool(single_scale), float(mod.k1), float(mod.k2), float(mod.eps), [float(w) for w in weights])
    return MSSSIMFn.apply(img1, img2, conf)
