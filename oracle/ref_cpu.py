"""ORACLE — test infrastructure only, never the product path.

A CPU restatement (PyTorch ops on the CPU, fp32 or fp64) of the reference's
hot path: the Balle-2018 scale-hyperprior forward pass and RD loss of
`modelling/meta_arch/bmshl2018.py:68-98`, written functionally over a flat
parameter dict whose keys equal the reference's `state_dict()` keys.
Backward comes from autograd on these CPU ops (plus the reference's custom
bound gradients, restated below).

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg
may import this module, and only as the checker / the timed CPU baseline.
It is pinned against the golden fixtures generated from the real reference
(`tools/gen_golden.py` -> `tests/golden/*.npz`, checked by
`tests/test_oracle_golden.py`).

Every function cites the reference file:line it restates (paths relative to
the reference repository root).
"""
import math

import torch
import torch.nn.functional as F

LN2 = math.log(2.0)


# ---------------------------------------------------------------- bounds
class _LowerBoundFn(torch.autograd.Function):
    """modelling/layers/bound.py:28-42: forward max(x, b); backward passes the
    gradient where x >= b or where the incoming gradient is negative."""

    @staticmethod
    def forward(ctx, x, bound):
        ctx.save_for_backward(x)
        ctx.bound = bound
        return torch.clamp(x, min=bound)

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        keep = (x >= ctx.bound) | (g < 0)
        return g * keep.to(g.dtype), None


class _UpperBoundFn(torch.autograd.Function):
    """modelling/layers/bound.py:45-59: forward min(x, b); backward passes the
    gradient where x <= b or where the incoming gradient is positive."""

    @staticmethod
    def forward(ctx, x, bound):
        ctx.save_for_backward(x)
        ctx.bound = bound
        return torch.clamp(x, max=bound)

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        keep = (x <= ctx.bound) | (g > 0)
        return g * keep.to(g.dtype), None


def lower_bound(x, b):
    return _LowerBoundFn.apply(x, float(b))


def upper_bound(x, b):
    return _UpperBoundFn.apply(x, float(b))


# ---------------------------------------------------------------- GDN
def nonneg(param, minimum=0.0, offset=2.0 ** -18):
    """modelling/layers/gdn.py:42-62 NonNegativeParam.forward:
    ped = offset^2, bound = (minimum + ped^2)^0.5, val = max(p, bound)^2 - ped."""
    ped32 = torch.tensor(float(offset) ** 2, dtype=torch.float32)
    bound = float((float(minimum) + ped32 ** 2) ** 0.5)  # fp32, as gdn.py:53
    v = lower_bound(param, bound)
    return v * v - ped32.to(param.dtype)


def gdn(x, gamma_param, beta_param, inverse=False, relu=False,
        beta_min=1e-6, offset=2.0 ** -18, bf16_bwd=False, bf16_fwd=False):
    """modelling/layers/gdn.py:79-88: y = x / sqrt(conv1x1(x^2, gamma) + beta)
    (x * sqrt(...) when inverse).  bf16_bwd: the backward's two contractions take
    bf16-rounded operands (_GDNBwdRounded; config C3 emulation, forward GDN only);
    bf16_fwd: the forward's gamma x^2 takes bf16-rounded gamma and x^2 (C3 emulation)."""
    if relu:
        x = F.relu(x)
    gamma = nonneg(gamma_param, 0.0, offset)
    beta = nonneg(beta_param, beta_min, offset)
    if (bf16_bwd or bf16_fwd) and not inverse:
        return _GDNBwdRounded.apply(x, gamma, beta, bool(bf16_fwd), bool(bf16_bwd))
    norm = torch.sqrt(F.conv2d(x * x, gamma, beta))
    return x * norm if inverse else x / norm


class _GDNBwdRounded(torch.autograd.Function):
    """y = x * v^-1/2, v = beta + gamma x^2, with the contractions on bf16-rounded operands where
    flagged: forward (rf) v = beta + rnd(gamma) rnd(x^2); backward (rb), with q = dL/dv =
    -1/2 dy x v^-3/2, dx = dy v^-1/2 + 2 x (rnd(q) rnd(gamma)), dgamma = rnd(q)^T rnd(x^2),
    dbeta = sum q (exact operands where not flagged).  Not the reference's arithmetic: the emulation
    of config C3's bf16-operand GDN (csrc/gdn_fused.hip, gdn_fwd_x3s_kernel<192, 1> and BF)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, rf=False, rb=True):
        v = F.conv2d(_rnd(x * x), _rnd(gamma), beta) if rf else F.conv2d(x * x, gamma, beta)
        ctx.rb = rb
        ctx.save_for_backward(x, gamma, v)
        return x / torch.sqrt(v)

    @staticmethod
    def backward(ctx, dy):
        x, gamma, v = ctx.saved_tensors
        rs = v.rsqrt()
        q = -0.5 * dy * x * rs * rs * rs
        r = _rnd if ctx.rb else (lambda t: t)
        g2 = r(gamma.reshape(gamma.shape[0], gamma.shape[1]))
        qr = r(q)
        dxg = torch.einsum("bnhw,nk->bkhw", qr, g2)
        dx = dy * rs + 2.0 * x * dxg
        dgamma = torch.einsum("bnhw,bkhw->nk", qr, r(x * x)).reshape(gamma.shape)
        dbeta = q.sum((0, 2, 3))
        return dx, dgamma, dbeta, None, None


def gdn_init(C, gamma_init=0.1, offset=2.0 ** -18):
    """Initial raw parameters of gdn.py:69-74 / :51-56."""
    ped = torch.tensor(float(offset) ** 2)
    g0 = torch.eye(C).view(C, C, 1, 1) * gamma_init
    b0 = torch.ones(C)
    gp = torch.sqrt(torch.max(g0 + ped, ped))
    bp = torch.sqrt(torch.max(b0 + ped, ped))
    return gp, bp


# ---------------------------------------------------------------- ReLU ties
def _relu(x, ctl):
    """F.relu, or (with a control dict) a ReLU whose gradient mask is given.

    ReLU's derivative jumps at 0, so a pre-activation that lies within
    rounding error of 0 can take either side in two correct fp32
    implementations, and the two gradients then differ by that element's
    whole contribution.  Tests compare the HIP path with this oracle under
    the HIP path's masks (ctl["masks"], consumed in call order) and check
    separately that every mask the two disagree on sits on such a tie
    (ctl["pre"] receives this oracle's pre-activations in call order)."""
    if ctl is None:
        return F.relu(x)
    ctl.setdefault("pre", []).append(x.detach())
    masks = ctl.get("masks")
    if masks:
        return x * masks[len(ctl["pre"]) - 1].to(x.dtype)
    return F.relu(x)


# ---------------------------------------------------------------- bf16 operand emulation
def _rnd(t):
    """round to bf16 (nearest even) and back: what a bf16-operand GEMM sees of t"""
    return t.to(torch.bfloat16).to(t.dtype)


class _ConvRounded(torch.autograd.Function):
    """A convolution (or transposed convolution) whose forward, input-gradient and
    weight-gradient GEMMs each take bf16-rounded operands when flagged (rf, rd, rw),
    accumulated exactly in the working dtype.  Not the reference's arithmetic: the
    emulation of BASELINE config C3's bf16-operand kernels, so a test can separate the
    rounding of the operands (a property of the config) from the kernels' own error.
    With no flag set it equals the plain op."""

    @staticmethod
    def forward(ctx, x, w, b, stride, pad, opad, transposed, rf, rd, rw):
        ctx.save_for_backward(x, w)
        ctx.cfg = (stride, pad, transposed, rd, rw)
        xi, wi = (_rnd(x), _rnd(w)) if rf else (x, w)
        if transposed:
            y = F.conv_transpose2d(xi, wi, b, stride=stride, padding=pad, output_padding=opad)
        else:
            y = F.conv2d(xi, wi, b, stride=stride, padding=pad)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        stride, pad, transposed, rd, rw = ctx.cfg
        dx = dw = None
        if ctx.needs_input_grad[0]:
            g, wd = (_rnd(gy), _rnd(w)) if rd else (gy, w)
            dx = (F.conv2d(g, wd, None, stride=stride, padding=pad) if transposed
                  else torch.nn.grad.conv2d_input(x.shape, wd, g, stride=stride, padding=pad))
        if ctx.needs_input_grad[1]:
            g, xw = (_rnd(gy), _rnd(x)) if rw else (gy, x)
            dw = (torch.nn.grad.conv2d_weight(g, w.shape, xw, stride=stride, padding=pad) if transposed
                  else torch.nn.grad.conv2d_weight(xw, w.shape, g, stride=stride, padding=pad))
        db = gy.sum((0, 2, 3)) if ctx.needs_input_grad[2] else None
        return dx, dw, db, None, None, None, None, None, None, None


def _conv(x, w, b, stride, pad, name, bf16, transposed=False, opad=0):
    """F.conv2d / F.conv_transpose2d; with `bf16` (a dict: weight name -> (fwd, dgrad, wgrad)
    flags, and GDN gamma-parameter name -> (forward, backward) flags) the GEMMs flagged for this
    layer take bf16-rounded operands (_ConvRounded)."""
    flags = bf16.get(name) if bf16 else None
    if flags and any(flags):
        return _ConvRounded.apply(x, w, b, stride, pad, opad, transposed, *flags)
    if transposed:
        return F.conv_transpose2d(x, w, b, stride=stride, padding=pad, output_padding=opad)
    return F.conv2d(x, w, b, stride=stride, padding=pad)


# ---------------------------------------------------------------- transforms
def analysis(P, x, strides=(2, 2, 2, 2), k=5, prefix="analysis_transform.layers.", bf16=None):
    """modelling/blocks/analysis.py:44-71: conv(k, s, pad k//2) with GDN after
    all but the last conv.  bf16: see _conv."""
    n = len(strides)
    for i, s in enumerate(strides):
        name = f"{prefix}{2*i}.weight"
        x = _conv(x, P[name], P[f"{prefix}{2*i}.bias"], s, k // 2, name, bf16)
        if i < n - 1:
            gf = bf16.get(f"{prefix}{2*i+1}.gamma.param") if bf16 else None
            x = gdn(x, P[f"{prefix}{2*i+1}.gamma.param"], P[f"{prefix}{2*i+1}.beta.param"],
                    bf16_bwd=bool(gf and gf[1]), bf16_fwd=bool(gf and gf[0]))
    return x


def synthesis(P, x, strides=(2, 2, 2, 2), k=5, prefix="synthesis_transform.layers.", bf16=None):
    """modelling/blocks/synthesis.py:44-71: conv_transpose(k, s, pad k//2,
    output_padding s-1) with forward GDN (not IGDN, synthesis.py:65) after all
    but the last layer.  bf16: see _conv."""
    n = len(strides)
    for i, s in enumerate(strides):
        name = f"{prefix}{2*i}.weight"
        x = _conv(x, P[name], P[f"{prefix}{2*i}.bias"], s, k // 2, name, bf16, transposed=True, opad=s - 1)
        if i < n - 1:
            gf = bf16.get(f"{prefix}{2*i+1}.gamma.param") if bf16 else None
            x = gdn(x, P[f"{prefix}{2*i+1}.gamma.param"], P[f"{prefix}{2*i+1}.beta.param"],
                    bf16_bwd=bool(gf and gf[1]), bf16_fwd=bool(gf and gf[0]))
    return x


def hyper_analysis(P, x, strides=(1, 2, 2), kernels=(3, 5, 5), prefix="prior_analysis._layers.", relu_ctl=None,
                   bf16=None):
    """modelling/blocks/prior_analysis.py:43-71: conv, ReLU, conv, ReLU, conv
    (no bias on the last conv).  bf16: see _conv."""
    n = len(strides)
    for i, (s, k) in enumerate(zip(strides, kernels)):
        b = P.get(f"{prefix}{2*i}.bias") if i < n - 1 else None
        name = f"{prefix}{2*i}.weight"
        x = _conv(x, P[name], b, s, k // 2, name, bf16)
        if i < n - 1:
            x = _relu(x, relu_ctl)
    return x


def hyper_synthesis(P, x, strides=(1, 2, 2), kernels=(3, 5, 5), prefix="prior_synthesis._layers.", relu_ctl=None,
                    bf16=None):
    """modelling/blocks/prior_synthesis.py:44-72: reversed kernels/strides,
    conv_transpose + ReLU, last layer then clamp(exp(.), 1e-10, 1e10).  bf16: see _conv."""
    n = len(strides)
    for i, (s, k) in enumerate(zip(reversed(strides), reversed(kernels))):
        name = f"{prefix}{2*i}.weight"
        x = _conv(x, P[name], P[f"{prefix}{2*i}.bias"], s, k // 2, name, bf16, transposed=True, opad=s - 1)
        if i < n - 1:
            x = _relu(x, relu_ctl)
    return torch.clamp(x.exp(), 1e-10, 1e10)


# ---------------------------------------------------------------- entropy models
def ce_loss(p):
    """modelling/blocks/entropy_model.py:171-185: sum clamp(-ln(p+1e-10)/ln2, 0, 50)."""
    return torch.clamp(-1.0 * torch.log(p + 1e-10) / LN2, 0, 50).sum()


def cdf_logits(P, x, n_layers=None, prefix="entropy_model._cdf_estimator.layers."):
    """entropy_model.py:67-78 (CDFLayer) and :101-114 (CDFEstimator): per
    channel c, h <- softplus(W_c) h + b_c, then h <- h + tanh(h) tanh(f_c) on all
    but the last layer. x: (N, C, *).

    Reference quirk, reproduced on purpose: the output is re-permuted with the
    SAME permutation used on the way in (entropy_model.py:108-113), not its
    inverse, so for a 4-D input (N, C, H, W) the result has shape
    (N, W, C, H) with out[n, w, c, h] = cdf(x)[n, c, h, w].  Only the returned
    probability tensor's layout is affected (the CE sum is permutation
    invariant)."""
    if n_layers is None:  # len(DIMS) + 1 layers (entropy_model.py:90), as many as P holds
        n_layers = 0
        while f"{prefix}{n_layers}.weight" in P:
            n_layers += 1
    N, C = x.shape[:2]
    sp = x.shape[2:]
    order = [0] + list(range(2, x.dim())) + [1]
    h = x.permute(*order).reshape(-1, C, 1, 1)
    for i in range(n_layers):
        h = torch.matmul(F.softplus(P[f"{prefix}{i}.weight"]), h) + P[f"{prefix}{i}.bias"]
        if i < n_layers - 1:
            h = h + torch.tanh(h) * torch.tanh(P[f"{prefix}{i}.factor"])
    return h.view(N, *sp, C).permute(*order)


def factorized(P, z, u=None, train=True, bin_=1.0, sym=None):
    """entropy_model.py:204-269 EntropyModel.forward: noise (u - bin/2, :230) or
    round (:234); likelihood via the detached sign trick (:259-269).  `sym` (eval only, test
    infrastructure): the symbols to use in place of round(z) — another implementation's
    rounding, so that a symbol sitting within float error of a .5 boundary (a tie, checked by
    the caller) does not decide the comparison of everything downstream."""
    half = bin_ / 2
    if train:
        q = z + (u - half).detach()
    elif sym is not None:
        q = z * 0 + torch.as_tensor(sym).to(z.dtype)  # zero gradient, like torch.round
    else:
        q = torch.round(z)
    lower = cdf_logits(P, q - half)
    upper = cdf_logits(P, q + half)
    sign = -torch.sign(lower + upper).detach()
    p = sign * (torch.sigmoid(upper * sign) - torch.sigmoid(lower * sign))
    return q, p, ce_loss(p)


def laplace_cdf(v):
    """torch.distributions.Laplace(0,1).cdf as called by entropy_model.py:374-375."""
    return 0.5 - 0.5 * v.sign() * torch.expm1(-v.abs())


def normal_cdf(v):
    """torch.distributions.Normal(0,1).cdf as called by entropy_model.py:361-362."""
    return 0.5 * (1 + torch.erf(v * 1.0 / math.sqrt(2)))


def conditional(y, scale, u=None, train=True, kind="laplace", mean=0, bin_=1.0, sym=None):
    """entropy_model.py:280-352: noise/round then
    p = F((half - |y~ - mean|)/scale) - F((-half - |y~ - mean|)/scale).  `sym`: as factorized."""
    half = bin_ / 2
    if train:
        q = y + (u - half).detach()
    elif sym is not None:
        q = y * 0 + torch.as_tensor(sym).to(y.dtype)
    else:
        q = torch.round(y)
    a = torch.abs(q - mean)
    cdf = laplace_cdf if kind == "laplace" else normal_cdf
    p = cdf((half - a) / scale) - cdf((-half - a) / scale)
    return q, p


# ---------------------------------------------------------------- losses
def mse(a, b):
    """nn.MSELoss(reduction='mean') as configured by modelling/loss.py:25."""
    return ((a - b) ** 2).mean()


def _gauss_filter2d(size=11, sigma=1.5, dtype=torch.float32):
    """modelling/loss.py:113-121: softmax(-(x^2+y^2)/(2 sigma^2)) over a
    size x size grid with coordinates arange(size)+0.5-size/2."""
    r = torch.arange(size, dtype=dtype) + 0.5 - size / 2
    g = -(r[:, None] ** 2 + r[None, :] ** 2) / (2.0 * sigma * sigma)
    return F.softmax(g.reshape(-1), dim=0).reshape(1, 1, size, size)


def _ssim_terms(a, b, filt, c1, c2, eps, log_scale):
    """modelling/loss.py:75-101 (_ssim): valid 11x11 filtering per channel,
    spatial+channel mean, LowerBound(eps) then log (log scale)."""
    N, C, H, W = a.shape

    def filt2(t):
        t = F.conv2d(t.reshape(-1, 1, t.shape[2], t.shape[3]), filt.to(t.dtype))
        return t.reshape(N, C, t.shape[2], t.shape[3])

    mu1, mu2 = filt2(a), filt2(b)
    mu1_sq, mu2_sq, mu12 = mu1 * mu1, mu2 * mu2, mu1 * mu2
    s1 = filt2(a * a) - mu1_sq
    s2 = filt2(b * b) - mu2_sq
    s12 = filt2(a * b) - mu12
    cs = (2.0 * s12 + c2) / (s1 + s2 + c2)
    ssim = cs * (2.0 * mu12 + c1) / (mu1_sq + mu2_sq + c1)
    ssim, cs = ssim.mean((1, 2, 3)), cs.mean((1, 2, 3))
    e = eps if log_scale else 0.0
    ssim, cs = lower_bound(ssim, e), lower_bound(cs, e)
    if log_scale:
        return ssim.log(), cs.log()
    return ssim, cs


def _downsample(t):
    """modelling/loss.py:176-188: reflect-pad odd sizes then avg_pool 2."""
    h, w = t.shape[2], t.shape[3]
    if (w % 2) + (h % 2):
        t = F.pad(t, (0, w % 2, 0, h % 2), mode="reflect")
    return F.avg_pool2d(t, kernel_size=2)


def ms_ssim_loss(a, b, max_val=255.0, size=11, sigma=1.5, k1=0.01, k2=0.03,
                 log_scale=True, eps=1e-5,
                 weights=(0.0448, 0.2856, 0.3001, 0.2363, 0.1333)):
    """modelling/loss.py:124-174 MS_SSIMLoss (log form :141-156, product form
    :158-174)."""
    a = a * max_val
    b = b * max_val
    filt = _gauss_filter2d(size, sigma, a.dtype)
    c1, c2 = (k1 * max_val) ** 2, (k2 * max_val) ** 2
    n = len(weights)
    if log_scale:
        res = 0.0
        for i, w in enumerate(weights, 1):
            ssim, cs = _ssim_terms(a, b, filt, c1, c2, eps, True)
            if i < n:
                res = res + cs * w
                a, b = _downsample(a), _downsample(b)
            else:
                res = res + ssim * w
        return -res.mean()
    res = torch.ones((a.shape[0],), dtype=a.dtype)
    for i, w in enumerate(weights, 1):
        ssim, cs = _ssim_terms(a, b, filt, c1, c2, eps, False)
        if i < n:
            res = res * cs ** w
            a, b = _downsample(a), _downsample(b)
        else:
            res = res * ssim ** w
    return 1.0 - res.mean()


def ssim_loss(a, b, max_val=255.0, size=11, sigma=1.5, k1=0.01, k2=0.03,
              log_scale=False, eps=1e-5):
    """modelling/loss.py:48-73 SSIMLoss."""
    a = a * max_val
    b = b * max_val
    filt = _gauss_filter2d(size, sigma, a.dtype)
    ssim, _ = _ssim_terms(a, b, filt, (k1 * max_val) ** 2, (k2 * max_val) ** 2, eps, log_scale)
    if log_scale:
        return -ssim
    return 1.0 - ssim.mean()


# ---------------------------------------------------------------- eval metrics
def psnr_metric(a, b, max_val=255.0):
    """utils/metric.py:26-36 on images already scaled by 255 (the Monitor
    multiplies x, x~ by 255 first, engine/monitor.py:118-121): per-image
    10 * (2 log10(max) - log(mse)/ln 10), mse over (C, H, W)."""
    m = F.mse_loss(a, b, reduction="none").mean((1, 2, 3))
    return 10.0 * (2 * math.log10(max_val) - m.log() / math.log(10))


def ms_ssim_metric_db(a, b, max_val=255.0, size=11, sigma=1.5, k1=0.01, k2=0.03,
                      weights=(0.0448, 0.2856, 0.3001, 0.2363, 0.1333)):
    """utils/metric.py:100-138 MS_SSIM(in_dB=True) on images already scaled by
    255: per-image prod_l max(cs_l, 0)^w_l * max(ssim_L, 0)^w_L (SSIM with
    non_negative=True, metric.py:39-72), then -10 log10(1 - result)."""
    filt = _gauss_filter2d(size, sigma, a.dtype)
    c1, c2 = (k1 * max_val) ** 2, (k2 * max_val) ** 2
    res = torch.ones((a.shape[0],), dtype=a.dtype)
    n = len(weights)
    for i, w in enumerate(weights, 1):
        ssim, cs = _ssim_terms(a, b, filt, c1, c2, 0.0, False)
        ssim, cs = torch.clamp_min(ssim, 0.0), torch.clamp_min(cs, 0.0)
        if i < n:
            res = res * cs ** w
            a, b = _downsample(a), _downsample(b)
        else:
            res = res * ssim ** w
    return -10.0 * (1.0 - res).log() / math.log(10)


# ---------------------------------------------------------------- full model
def forward(P, x, u_z=None, u_y=None, train=True, cond="laplace",
            loss_names=("MSE",), lam=256.0, ssim_log=True,
            strides=(2, 2, 2, 2), hp_strides=(1, 2, 2), hp_kernels=(3, 5, 5), relu_ctl=None, bin_=1.0,
            bf16=None, sym_z=None, sym_y=None):
    """modelling/meta_arch/bmshl2018.py:68-98 Compressor2018.forward.
    Returns dict of intermediates and the loss dict.  bf16: per-layer bf16 operand
    emulation of the convolutions' GEMMs (_conv; None = exact).  sym_z / sym_y (eval):
    symbols fed in place of round(z) / round(y) (see factorized)."""
    N, C, H, W = x.shape
    num_pixels = N * H * W
    y = analysis(P, x, strides, bf16=bf16)
    z = hyper_analysis(P, torch.abs(y), hp_strides, hp_kernels, relu_ctl=relu_ctl, bf16=bf16)
    z_tilde, p_z, ce_z = factorized(P, z, u_z, train, bin_, sym=sym_z)
    sigma = hyper_synthesis(P, z_tilde, hp_strides, hp_kernels, relu_ctl=relu_ctl, bf16=bf16)
    y_tilde, p_y = conditional(y, sigma, u_y, train, cond, bin_=bin_, sym=sym_y)
    ce_y = ce_loss(p_y)
    x_raw = synthesis(P, y_tilde, strides, bf16=bf16)
    x_tilde = lower_bound(upper_bound(x_raw, 1.0), 0.0)
    dist = {}
    for name in loss_names:
        if name == "MSE":
            dist[name] = mse(x, x_tilde)
        elif name == "MS_SSIMLoss":
            dist[name] = ms_ssim_loss(x, x_tilde, log_scale=ssim_log)
        elif name == "SSIMLoss":
            dist[name] = ssim_loss(x, x_tilde, log_scale=ssim_log)
        else:
            raise KeyError(name)
    total_dist = sum(dist.values())
    entropy = (ce_z + ce_y) / num_pixels
    total = lam * total_dist + entropy
    losses = {"z_entropy": ce_z.detach() / num_pixels,
              "y_entropy": ce_y.detach() / num_pixels,
              "bpp": entropy.detach(), "total_loss": total}
    losses.update({k: v.detach() for k, v in dist.items()})
    out = dict(y=y, z=z, z_tilde=z_tilde, p_z=p_z, ce_z=ce_z, sigma=sigma,
               y_tilde=y_tilde, p_y=p_y, ce_y=ce_y, x_tilde_raw=x_raw,
               x_tilde=x_tilde)
    return out, losses


def run(params, x, u_z=None, u_y=None, train=True, dtype=torch.float64, **kw):
    """Convenience: forward + backward of total_loss. `params`: dict of
    numpy/tensors keyed like the reference state_dict. Returns
    (out, losses, grads) as CPU tensors of `dtype`."""
    P = {k: torch.as_tensor(v).to(dtype).clone().requires_grad_(True)
         for k, v in params.items()}
    xt = torch.as_tensor(x).to(dtype)
    uz = None if u_z is None else torch.as_tensor(u_z).to(dtype)
    uy = None if u_y is None else torch.as_tensor(u_y).to(dtype)
    out, losses = forward(P, xt, uz, uy, train, **kw)
    losses["total_loss"].backward()
    grads = {k: p.grad for k, p in P.items()}
    return out, losses, grads
