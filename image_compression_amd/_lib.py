"""ctypes binding of libimgcomp.so (the C ABI declared in include/imgcomp.h).

The shared library is built in-tree by `make -C image_compression_amd/csrc`
(or `__graft_entry__.build()`).  There is no fallback: if the library or a
ROCm device is missing, every op raises RuntimeError.
"""
import ctypes
import os

import torch  # noqa: F401  (must be imported first: shares its HIP runtime)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libimgcomp.so")
# kernel-development override (A/B variants of the in-tree library)
LIB_PATH = os.environ.get("IMGCOMP_LIB") or LIB_PATH

c_int, c_ll, c_ull, c_size, c_float, c_void = (ctypes.c_int, ctypes.c_longlong, ctypes.c_ulonglong,
                                              ctypes.c_size_t, ctypes.c_float, ctypes.c_void_p)


class ICAct(ctypes.Structure):
    _fields_ = [("data", c_void), ("n", c_int), ("c", c_int), ("h", c_int), ("w", c_int),
                ("sn", c_ll), ("sc", c_ll), ("sh", c_ll), ("sw", c_ll)]


_FACT_FIELDS = ["w0", "b0", "f0", "w1", "b1", "f1", "w2", "b2", "f2", "w3", "b3"]


class ICFactParams(ctypes.Structure):
    _fields_ = [(f, c_void) for f in _FACT_FIELDS]


class ICFactGrads(ctypes.Structure):
    _fields_ = [(f, c_void) for f in _FACT_FIELDS]


FACT_MAXL, FACT_MAXW = 6, 8  # IC_FACT_MAXL / IC_FACT_MAXW: the register kernels
FACT_NET_MAXL, FACT_WIDE_MAXW = 32, 256  # IC_FACT_NET_MAXL / IC_FACT_WIDE_MAXW: the wide kernels (any geometry)


class ICFactNet(ctypes.Structure):
    _fields_ = [("nlayers", c_int), ("dims", c_int * (FACT_NET_MAXL + 1)), ("w", c_void * FACT_NET_MAXL),
                ("b", c_void * FACT_NET_MAXL), ("f", c_void * FACT_NET_MAXL)]


class ICFactNetGrads(ctypes.Structure):
    _fields_ = [("w", c_void * FACT_NET_MAXL), ("b", c_void * FACT_NET_MAXL), ("f", c_void * FACT_NET_MAXL)]


class ICAdamWTensor(ctypes.Structure):
    _fields_ = [("param", c_void), ("grad", c_void), ("exp_avg", c_void), ("exp_avg_sq", c_void),
                ("n", c_ll), ("lr", c_float), ("weight_decay", c_float)]


class ICNonNegTensor(ctypes.Structure):
    _fields_ = [("p", ctypes.c_void_p), ("out", ctypes.c_void_p), ("gout", ctypes.c_void_p), ("gin", ctypes.c_void_p),
                ("n", ctypes.c_longlong), ("bound", ctypes.c_float), ("pedestal", ctypes.c_float)]


class ICPlan(ctypes.Structure):
    _fields_ = [("kernel", c_int), ("bm", c_int), ("bn", c_int), ("ksplit", c_int), ("nsplit", c_int),
                ("im2col", c_int), ("variant", c_int), ("blocks", c_ll)]


P = ctypes.POINTER
_ACT = P(ICAct)

# name -> (restype, argtypes); mirrors include/imgcomp.h one to one
SIGNATURES = {
    "ic_version": (c_int, []),
    "ic_conv_plan": (c_int, [c_int, _ACT, _ACT, c_int, c_int, c_int, c_int, P(ICPlan)]),
    "ic_device_sync_check": (c_int, [c_void]),
    "ic_conv2d_fwd_ws_ex": (c_size, [_ACT, c_int, c_int, c_int, _ACT, c_int]),
    "ic_conv2d_fwd_ex": (c_int, [_ACT, c_void, c_void, c_int, c_int, c_int, _ACT, c_int, c_int, c_void, c_size,
                                 c_void]),
    "ic_conv2d_dgrad_ws_ex": (c_size, [_ACT, c_int, c_int, c_int, _ACT, c_int]),
    "ic_conv2d_dgrad_ex": (c_int, [_ACT, c_void, c_int, c_int, c_int, _ACT, c_int, c_void, c_size, c_void]),
    "ic_conv_transpose2d_fwd_ws_ex": (c_size, [_ACT, c_int, c_int, c_int, _ACT, c_int]),
    "ic_conv_transpose2d_fwd_ex": (c_int, [_ACT, c_void, c_void, c_int, c_int, c_int, _ACT, c_int, c_int, c_void,
                                           c_size, c_void]),
    "ic_conv_transpose2d_dgrad_ws_ex": (c_size, [_ACT, c_int, c_int, c_int, _ACT, c_int]),
    "ic_conv_transpose2d_dgrad_ex": (c_int, [_ACT, c_void, c_int, c_int, c_int, _ACT, c_int, c_void, c_size,
                                             c_void]),
    "ic_conv2d_fwd_ws": (c_size, [_ACT, c_int, c_int, c_int, _ACT]),
    "ic_conv2d_fwd": (c_int, [_ACT, c_void, c_void, c_int, c_int, c_int, _ACT, c_int, c_void, c_size, c_void]),
    "ic_conv2d_dgrad_ws": (c_size, [_ACT, c_int, c_int, c_int, _ACT]),
    "ic_conv2d_dgrad": (c_int, [_ACT, c_void, c_int, c_int, c_int, _ACT, c_void, c_size, c_void]),
    "ic_conv2d_wgrad_ws": (c_size, [_ACT, _ACT, c_int, c_int, c_int]),
    "ic_conv2d_wgrad": (c_int, [_ACT, _ACT, c_int, c_int, c_int, c_void, c_void, c_void, c_size, c_void]),
    "ic_conv_transpose2d_fwd_ws": (c_size, [_ACT, c_int, c_int, c_int, _ACT]),
    "ic_conv_transpose2d_fwd": (c_int, [_ACT, c_void, c_void, c_int, c_int, c_int, _ACT, c_int, c_void, c_size, c_void]),
    "ic_conv_transpose2d_dgrad_ws": (c_size, [_ACT, c_int, c_int, c_int, _ACT]),
    "ic_conv_transpose2d_dgrad": (c_int, [_ACT, c_void, c_int, c_int, c_int, _ACT, c_void, c_size, c_void]),
    "ic_conv_transpose2d_wgrad_ws": (c_size, [_ACT, _ACT, c_int, c_int, c_int]),
    "ic_conv_transpose2d_wgrad": (c_int, [_ACT, _ACT, c_int, c_int, c_int, c_void, c_void, c_void, c_size, c_void]),
    "ic_conv2d_wgrad_ws_ex": (c_size, [_ACT, _ACT, c_int, c_int, c_int, c_int]),
    "ic_conv2d_wgrad_ex": (c_int, [_ACT, _ACT, c_int, c_int, c_int, c_void, c_void, c_int, c_void, c_size, c_void]),
    "ic_conv_transpose2d_wgrad_ws_ex": (c_size, [_ACT, _ACT, c_int, c_int, c_int, c_int]),
    "ic_conv_transpose2d_wgrad_ex": (c_int, [_ACT, _ACT, c_int, c_int, c_int, c_void, c_void, c_int, c_void, c_size,
                                             c_void]),
    "ic_gdn_fwd_ws": (c_size, [_ACT]),
    "ic_gdn_fwd": (c_int, [_ACT, c_void, c_void, c_int, _ACT, c_void, c_void, c_size, c_void]),
    "ic_gdn_bwd_ws": (c_size, [_ACT]),
    "ic_gdn_bwd": (c_int, [_ACT, c_void, c_void, c_void, c_int, _ACT, c_void, c_void, c_void, c_size, c_void]),
    "ic_gdn_fwd_ws_ex": (c_size, [_ACT, c_int]),
    "ic_gdn_fwd_ex": (c_int, [_ACT, c_void, c_void, c_int, _ACT, c_void, c_int, c_void, c_size, c_void]),
    "ic_gdn_bwd_ex": (c_int, [_ACT, c_void, c_void, c_void, c_int, _ACT, c_void, c_void, c_int, c_void, c_size,
                              c_void]),
    "ic_gdn_bwd_sum_ex": (c_int, [_ACT, c_void, c_void, c_void, c_int, _ACT, c_void, c_void, c_void, c_int, c_void, c_size,
                                  c_void]),
    # bf16 activation copies (config C3): include/imgcomp.h ic_gdn_fwd_xb ... ic_conv_transpose2d_dgrad_xb
    "ic_gdn_fwd_xb": (c_int, [_ACT, c_void, c_void, c_int, _ACT, c_void, c_void, c_int, c_void, c_size, c_void]),
    "ic_gdn_bwd_sum_xb": (c_int, [_ACT, c_void, c_void, c_void, c_int, _ACT, c_void, c_void, c_void, c_void, c_int,
                                  c_void, c_size, c_void]),
    # norm recomputed by the C3 backward (round 6): include/imgcomp.h ic_gdn_fwd_rn, ic_gdn_bwd_sum_rn
    "ic_gdn_fwd_rn": (c_int, [_ACT, c_void, c_void, c_int, _ACT, c_void, c_int, c_void, c_size, c_void]),
    "ic_gdn_bwd_sum_rn": (c_int, [_ACT, c_void, c_void, c_void, c_int, _ACT, c_void, c_void, c_void, c_void, c_int,
                                  c_void, c_size, c_void]),
    "ic_conv2d_fwd_xb": (c_int, [_ACT, c_void, c_void, c_void, c_int, c_int, c_int, _ACT, c_int, c_int, c_void, c_size,
                                 c_void]),
    "ic_conv_transpose2d_dgrad_xb": (c_int, [_ACT, c_void, c_void, c_int, c_int, c_int, _ACT, c_int, c_void, c_size,
                                             c_void]),
    "ic_conv2d_dgrad_xb": (c_int, [_ACT, c_void, c_void, c_int, c_int, c_int, _ACT, c_int, c_void, c_size, c_void]),
    "ic_conv2d_wgrad_xb": (c_int, [_ACT, c_void, _ACT, c_void, c_int, c_int, c_int, c_void, c_void, c_int, c_void,
                                   c_size, c_void]),
    "ic_conv_transpose2d_wgrad_xb": (c_int, [_ACT, c_void, _ACT, c_void, c_int, c_int, c_int, c_void, c_void, c_int,
                                             c_void, c_size, c_void]),
    "ic_conv_transpose2d_fwd_xb": (c_int, [_ACT, c_void, c_void, c_void, c_int, c_int, c_int, _ACT, c_int, c_int,
                                           c_void, c_size, c_void]),
    "ic_nonneg_fwd": (c_int, [c_void, c_ll, c_float, c_float, c_void, c_void]),
    "ic_nonneg_bwd": (c_int, [c_void, c_void, c_ll, c_float, c_void, c_void]),
    "ic_bound_fwd": (c_int, [c_void, c_ll, c_float, c_int, c_void, c_void]),
    "ic_bound_bwd": (c_int, [c_void, c_void, c_ll, c_float, c_int, c_void, c_void]),
    "ic_relu_fwd": (c_int, [c_void, c_ll, c_void, c_void]),
    "ic_relu_bwd": (c_int, [c_void, c_void, c_ll, c_void, c_void]),
    "ic_abs_fwd": (c_int, [c_void, c_ll, c_void, c_void]),
    "ic_abs_bwd": (c_int, [c_void, c_void, c_ll, c_void, c_void]),
    "ic_exp_clamp_fwd": (c_int, [c_void, c_ll, c_float, c_float, c_void, c_void, c_void]),
    "ic_exp_clamp_bwd": (c_int, [c_void, c_void, c_ll, c_float, c_float, c_void, c_void]),
    "ic_reduce_ws": (c_size, [c_ll]),
    "ic_ce_loss_fwd": (c_int, [c_void, c_ll, c_void, c_void, c_size, c_void]),
    "ic_ce_loss_bwd": (c_int, [c_void, c_void, c_ll, c_void, c_void]),
    "ic_mse_fwd": (c_int, [c_void, c_void, c_ll, c_void, c_void, c_size, c_void]),
    "ic_mse_bwd": (c_int, [c_void, c_void, c_void, c_ll, c_void, c_void, c_void]),
    "ic_uniform": (c_int, [c_void, c_ll, c_ull, c_ull, c_void]),
    "ic_philox_advance": (c_int, [c_void, c_ull, c_void]),
    "ic_philox_kat": (c_int, [c_void, c_void, c_int, c_void]),
    "ic_psnr": (c_int, [c_void, c_void, c_int, c_ll, c_float, c_void, c_void]),
    "ic_psnr_ws": (c_size, [c_int, c_ll]),
    "ic_psnr_ex": (c_int, [c_void, c_void, c_int, c_ll, c_float, c_void, c_void, c_size, c_void]),
    "ic_images_u8_to_input": (c_int, [c_void, c_ll, c_ll, c_ll, c_int, c_int, c_int, c_int, c_void, c_void, c_void,
                                      c_void]),
    "ic_nonneg_multi": (c_int, [P(ICNonNegTensor), c_int, c_int, c_void]),
    "ic_adamw_step": (c_int, [P(ICAdamWTensor), c_int, ctypes.c_double, ctypes.c_double, c_float, c_float, c_ll,
                              c_void]),
    "ic_factorized_fwd": (c_int, [c_void, c_ll, c_int, P(ICFactParams), c_int, c_void, c_ull, c_ull, c_void, c_void, c_void]),
    "ic_factorized_bwd": (c_int, [c_void, c_ll, c_int, P(ICFactParams), c_void, c_void, c_void, P(ICFactGrads), c_void]),
    "ic_conditional_fwd": (c_int, [c_void, c_void, c_void, c_ll, c_int, c_int, c_void, c_ull, c_ull, c_void, c_void, c_void]),
    "ic_conditional_bwd": (c_int, [c_void, c_void, c_void, c_ll, c_int, c_void, c_void, c_void, c_void, c_void, c_void]),
    "ic_conditional_fwd_bin": (c_int, [c_void, c_void, c_void, c_ll, c_int, c_int, c_void, c_ull, c_ull, c_float,
                                       c_void, c_void, c_void]),
    "ic_conditional_bwd_bin": (c_int, [c_void, c_void, c_void, c_ll, c_int, c_float, c_void, c_void, c_void, c_void,
                                       c_void, c_void]),
    "ic_quantize": (c_int, [c_void, c_ll, c_int, c_void, c_ull, c_ull, c_float, c_void, c_void]),
    "ic_factorized_fwd_net": (c_int, [c_void, c_ll, c_int, P(ICFactNet), c_float, c_int, c_void, c_ull, c_ull, c_void,
                                      c_void, c_void]),
    "ic_factorized_bwd_net": (c_int, [c_void, c_ll, c_int, P(ICFactNet), c_float, c_void, c_void, c_void,
                                      P(ICFactNetGrads), c_void]),
    "ic_factorized_net_ws": (c_size, [c_ll, c_int, P(ICFactNet), c_int]),
    "ic_factorized_fwd_net_ex": (c_int, [c_void, c_ll, c_int, P(ICFactNet), c_float, c_int, c_void, c_ull, c_ull,
                                         c_void, c_void, c_void, c_size, c_void]),
    "ic_factorized_bwd_net_ex": (c_int, [c_void, c_ll, c_int, P(ICFactNet), c_float, c_void, c_void, c_void,
                                         P(ICFactNetGrads), c_void, c_size, c_void]),
    "ic_msssim_state_bytes": (c_size, [c_int, c_int, c_int, c_int, c_int, c_int]),
    "ic_msssim_ws": (c_size, [c_int, c_int, c_int, c_int, c_int, c_int]),
    "ic_msssim_fwd": (c_int, [c_void, c_void, c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_float, c_int,
                              c_int, c_float, c_float, c_float, c_void, c_void, c_void, c_void, c_size, c_void]),
    "ic_msssim_bwd": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_float, c_int, c_int, c_float,
                              c_float, c_float, c_void, c_void, c_void, c_void, c_void, c_void, c_size, c_void]),
    "ic_sqdiff_fwd": (c_int, [c_void, c_void, c_ll, c_void, c_void]),
    "ic_sqdiff_bwd": (c_int, [c_void, c_void, c_void, c_ll, c_void, c_void, c_void]),
}

_lib = None
_load_error = None
TORCH_OPS_PATH = os.path.join(os.path.dirname(LIB_PATH), "libimgcomp_torch.so")
_ops = None


def ops():
    """torch.ops.imgcomp (the TORCH_LIBRARY registration of the conv / GDN launchers,
    csrc/torch_ops.cpp); loads libimgcomp_torch.so once, raises RuntimeError if absent."""
    global _ops
    if _ops is None:
        load()
        if not os.path.exists(TORCH_OPS_PATH):
            raise RuntimeError(f"imgcomp: torch op library not built ({TORCH_OPS_PATH} missing); run "
                               "`make -C image_compression_amd/csrc` or __graft_entry__.build()")
        torch.ops.load_library(TORCH_OPS_PATH)
        _ops = torch.ops.imgcomp
    return _ops


def load():
    """Load libimgcomp.so once; raise RuntimeError (never fall back) on failure."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"imgcomp: HIP library not built ({LIB_PATH} missing); run "
            "`make -C image_compression_amd/csrc` or __graft_entry__.build()")
    try:
        lib = ctypes.CDLL(LIB_PATH)
    except OSError as e:  # pragma: no cover
        raise RuntimeError(f"imgcomp: cannot load {LIB_PATH}: {e}") from e
    for name, (res, args) in SIGNATURES.items():
        if not hasattr(lib, name):
            continue  # reported by exported_symbols()/tests
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def exported_symbols():
    lib = load()
    return {n for n in SIGNATURES if hasattr(lib, n)}


def check(rc, what):
    if rc != 0:
        kind = {1001: "unsupported/inconsistent arguments", 1002: "workspace too small"}.get(rc, "HIP error")
        raise RuntimeError(f"imgcomp: {what} failed with status {rc} ({kind})")


def act(t):
    """ic_act for a 4-D tensor (logical N,C,H,W, any strides)."""
    if t.dim() != 4:
        raise RuntimeError(f"imgcomp: expected a 4-D tensor, got shape {tuple(t.shape)}")
    s = t.stride()
    return ICAct(c_void(t.data_ptr()), t.shape[0], t.shape[1], t.shape[2], t.shape[3], s[0], s[1], s[2], s[3])


# ic_conv_plan op codes and kernel ids (include/imgcomp.h)
OPS = {"conv2d_fwd": 0, "conv2d_dgrad": 1, "conv2d_wgrad": 2, "conv_transpose2d_fwd": 3,
       "conv_transpose2d_dgrad": 4, "conv_transpose2d_wgrad": 5, "gdn_fwd": 6, "gdn_bwd": 7}
KERNELS = {1: "ig_fp32", 2: "ig_fp32_gather", 3: "ig_bf16", 4: "ig_split", 5: "ig_split_bf16", 6: "edge_conv",
           7: "im2col_gemm", 8: "tconv_few", 9: "tconv_few_rows", 10: "gemm_col2im", 11: "wg_fp32",
           12: "wg_fp32_gather", 13: "wg_ldsdma", 14: "wg_split", 15: "edge_wgrad", 16: "gdn_fused",
           17: "gdn_fused_split", 18: "gdn_gemm", 20: "wg_bf16",
           21: "gdn_fused_bf16", 22: "ig_split_dma", 23: "edge_conv_bf16", 24: "tconv_few_rows_bf16",
           25: "edge_wgrad_bf16", 26: "ig_bf16_dma"}


def plan(op, a, b=None, k=1, stride=1, pad=0, math=0):
    """The launch plan (kernel, tile, K / pixel splits) that `op` takes for these operands
    (ic_conv_plan; no launch).  a / b: tensors or ICAct, in the order of the op's
    workspace query (fwd: x, y; dgrad: dy, dx; wgrad: x, dy; gdn: x)."""
    L = load()
    aa = a if isinstance(a, ICAct) else act(a)
    bb = aa if b is None else (b if isinstance(b, ICAct) else act(b))
    out = ICPlan()
    rc = L.ic_conv_plan(OPS[op], aa, bb, k, stride, pad, int(math), ctypes.byref(out))
    check(rc, f"plan({op})")
    return {"kernel": KERNELS.get(out.kernel, out.kernel), "bm": out.bm, "bn": out.bn, "ksplit": out.ksplit,
            "nsplit": out.nsplit, "im2col": out.im2col, "variant": out.variant, "blocks": out.blocks}


def ptr(t):
    return None if t is None else c_void(t.data_ptr())


def stream_of(t):
    return c_void(torch.cuda.current_stream(t.device).cuda_stream)


def require_device(*ts):
    for t in ts:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError("imgcomp: HIP kernels need tensors on a ROCm (cuda) device; "
                               f"got a tensor on {t.device}")
        if t.dtype != torch.float32:
            raise RuntimeError(f"imgcomp: fp32 tensors expected, got {t.dtype}")


def workspace(nbytes, device):
    n = max(int(nbytes), 16)
    return torch.empty(n, dtype=torch.uint8, device=device)
