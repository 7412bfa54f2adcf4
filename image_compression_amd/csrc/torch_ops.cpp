// torch.ops.imgcomp.* — the conv / transposed-conv / GDN launchers of libimgcomp.so
// registered as PyTorch operators (TORCH_LIBRARY), so the autograd Functions in
// image_compression_amd/functional.py dispatch through the PyTorch op registry
// instead of ctypes, and FX / fake-tensor tracing sees real operators with
// shape (Meta) kernels.  Each op is one C-ABI call of include/imgcomp.h on the
// current HIP stream of the input's device, with its workspace from PyTorch's
// caching allocator; the C ABI stays the non-torch binding.
//
// Reference interfaces these replace: torch.nn.Conv2d in modelling/blocks/analysis.py:55 and
// prior_analysis.py:54-56; torch.nn.ConvTranspose2d in modelling/blocks/synthesis.py:55-57 and
// prior_synthesis.py:54-56; GDN.forward in modelling/layers/gdn.py:79-88 (backward by autograd there).
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/library.h>

#include <tuple>

#include "../../include/imgcomp.h"

namespace {

using at::Tensor;

void check_operand(const Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda(), "imgcomp: ", what, " must be on a ROCm device, got ", t.device());
  TORCH_CHECK(t.scalar_type() == at::kFloat, "imgcomp: ", what, " must be float32, got ", t.scalar_type());
}

ic_act act_of(const Tensor& t) {
  TORCH_CHECK(t.dim() == 4, "imgcomp: expected a 4-D tensor, got ", t.sizes());
  ic_act a;
  a.data = t.data_ptr<float>();
  a.n = (int)t.size(0); a.c = (int)t.size(1); a.h = (int)t.size(2); a.w = (int)t.size(3);
  a.sn = t.stride(0); a.sc = t.stride(1); a.sh = t.stride(2); a.sw = t.stride(3);
  return a;
}

// activations with >= 32 channels live channels-last (NHWC): GEMM operand rows are channel-contiguous
at::MemoryFormat act_format(int64_t c) { return c >= 32 ? at::MemoryFormat::ChannelsLast : at::MemoryFormat::Contiguous; }

Tensor new_act(const Tensor& like, int64_t n, int64_t c, int64_t h, int64_t w) {
  return at::empty({n, c, h, w}, like.options().memory_format(act_format(c)));
}

// PyTorch-ROCm exposes HIP devices under the "cuda" device type; these are its HIP stream / guard APIs for them
void* stream_of(const Tensor& t) {
  return (void*)c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index()).stream();
}

Tensor workspace(const Tensor& like, size_t nbytes) {
  return at::empty({(int64_t)std::max<size_t>(nbytes, 16)}, like.options().dtype(at::kByte));
}

void check_rc(int rc, const char* what) {
  TORCH_CHECK(rc == 0, "imgcomp: ", what, " failed with status ", rc,
              rc == IC_ERR_ARG ? " (unsupported/inconsistent arguments)"
                               : rc == IC_ERR_WORKSPACE ? " (workspace too small)" : " (HIP error)");
}

float* opt_ptr(const c10::optional<Tensor>& t) { return t.has_value() && t->defined() ? t->data_ptr<float>() : nullptr; }

// ---------------------------------------------------------------- conv2d
Tensor conv2d_fwd(const Tensor& x, const Tensor& w, const c10::optional<Tensor>& b, int64_t stride, int64_t pad,
                  int64_t act, int64_t math) {
  check_operand(x, "x");
  check_operand(w, "weight");
  if (b.has_value()) check_operand(*b, "bias");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  TORCH_CHECK(w.dim() == 4 && w.size(1) == x.size(1) && w.size(2) == w.size(3), "conv2d: weight ", w.sizes(),
              " does not match input ", x.sizes());
  const int64_t k = w.size(2);
  const int64_t ho = (x.size(2) + 2 * pad - k) / stride + 1, wo = (x.size(3) + 2 * pad - k) / stride + 1;
  Tensor y = new_act(x, x.size(0), w.size(0), ho, wo);
  const ic_act ax = act_of(x), ay = act_of(y);
  const size_t nb = ic_conv2d_fwd_ws_ex(&ax, (int)k, (int)stride, (int)pad, &ay, (int)math);
  Tensor ws = workspace(x, nb);
  check_rc(ic_conv2d_fwd_ex(&ax, w.data_ptr<float>(), opt_ptr(b), (int)k, (int)stride, (int)pad, &ay, (int)act,
                            (int)math, ws.data_ptr(), nb, stream_of(x)),
           "conv2d_fwd");
  return y;
}

// The forward with a caller-owned workspace that persists across calls (eval-mode weight caching,
// functional._cached_fwd): grown here when too small (only on a packing call — with IC_MATH_WPACKED the
// pack must already be in it, so a short workspace is an error).
void ensure_ws(Tensor& ws, size_t nb, int64_t math, const char* what) {
  if ((size_t)ws.numel() >= nb) return;
  TORCH_CHECK(!(math & IC_MATH_WPACKED), "imgcomp: ", what, ": IC_MATH_WPACKED with a workspace of ", ws.numel(),
              " bytes, the op needs ", nb);
  ws.resize_({(int64_t)nb});
}
Tensor conv2d_fwd_ws(const Tensor& x, const Tensor& w, const c10::optional<Tensor>& b, int64_t stride, int64_t pad,
                     int64_t act, int64_t math, Tensor& ws) {
  check_operand(x, "x");
  check_operand(w, "weight");
  if (b.has_value()) check_operand(*b, "bias");
  TORCH_CHECK(ws.device() == x.device() && ws.scalar_type() == at::kByte && ws.dim() == 1 && ws.is_contiguous(),
              "conv2d_fwd_ws: the workspace must be a contiguous uint8 vector on the input's device");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  TORCH_CHECK(w.dim() == 4 && w.size(1) == x.size(1) && w.size(2) == w.size(3), "conv2d: weight ", w.sizes(),
              " does not match input ", x.sizes());
  const int64_t k = w.size(2);
  const int64_t ho = (x.size(2) + 2 * pad - k) / stride + 1, wo = (x.size(3) + 2 * pad - k) / stride + 1;
  Tensor y = new_act(x, x.size(0), w.size(0), ho, wo);
  const ic_act ax = act_of(x), ay = act_of(y);
  const size_t nb = ic_conv2d_fwd_ws_ex(&ax, (int)k, (int)stride, (int)pad, &ay, (int)(math & ~IC_MATH_WPACKED));
  ensure_ws(ws, nb, math, "conv2d_fwd_ws");
  check_rc(ic_conv2d_fwd_ex(&ax, w.data_ptr<float>(), opt_ptr(b), (int)k, (int)stride, (int)pad, &ay, (int)act,
                            (int)math, ws.data_ptr(), (size_t)ws.numel(), stream_of(x)),
           "conv2d_fwd_ws");
  return y;
}
Tensor conv_transpose2d_fwd_ws(const Tensor& x, const Tensor& w, const c10::optional<Tensor>& b, int64_t stride,
                               int64_t pad, int64_t output_padding, int64_t act, int64_t math, Tensor& ws) {
  check_operand(x, "x");
  check_operand(w, "weight");
  if (b.has_value()) check_operand(*b, "bias");
  TORCH_CHECK(ws.device() == x.device() && ws.scalar_type() == at::kByte && ws.dim() == 1 && ws.is_contiguous(),
              "conv_transpose2d_fwd_ws: the workspace must be a contiguous uint8 vector on the input's device");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  TORCH_CHECK(w.dim() == 4 && w.size(0) == x.size(1) && w.size(2) == w.size(3), "conv_transpose2d: weight ",
              w.sizes(), " does not match input ", x.sizes());
  const int64_t k = w.size(2);
  const int64_t ho = (x.size(2) - 1) * stride - 2 * pad + k + output_padding;
  const int64_t wo = (x.size(3) - 1) * stride - 2 * pad + k + output_padding;
  Tensor y = new_act(x, x.size(0), w.size(1), ho, wo);
  const ic_act ax = act_of(x), ay = act_of(y);
  const size_t nb =
      ic_conv_transpose2d_fwd_ws_ex(&ax, (int)k, (int)stride, (int)pad, &ay, (int)(math & ~IC_MATH_WPACKED));
  ensure_ws(ws, nb, math, "conv_transpose2d_fwd_ws");
  check_rc(ic_conv_transpose2d_fwd_ex(&ax, w.data_ptr<float>(), opt_ptr(b), (int)k, (int)stride, (int)pad, &ay,
                                      (int)act, (int)math, ws.data_ptr(), (size_t)ws.numel(), stream_of(x)),
           "conv_transpose2d_fwd_ws");
  return y;
}

// dx has the shape and memory format of x
Tensor conv2d_dgrad(const Tensor& dy, const Tensor& w, const Tensor& x, int64_t stride, int64_t pad, int64_t math) {
  check_operand(dy, "dy");
  check_operand(w, "weight");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(dy.device());
  Tensor dx = at::empty(x.sizes(), dy.options().memory_format(x.suggest_memory_format()));
  const ic_act ag = act_of(dy), adx = act_of(dx);
  const int k = (int)w.size(2);
  const size_t nb = ic_conv2d_dgrad_ws_ex(&ag, k, (int)stride, (int)pad, &adx, (int)math);
  Tensor ws = workspace(dy, nb);
  check_rc(ic_conv2d_dgrad_ex(&ag, w.data_ptr<float>(), k, (int)stride, (int)pad, &adx, (int)math, ws.data_ptr(), nb,
                              stream_of(dy)),
           "conv2d_dgrad");
  return dx;
}

// (dw, db); db is empty when bias is false
std::tuple<Tensor, Tensor> conv2d_wgrad(const Tensor& x, const Tensor& dy, const Tensor& w, int64_t stride, int64_t pad,
                                        bool bias, int64_t math) {
  check_operand(x, "x");
  check_operand(dy, "dy");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(dy.device());
  Tensor dw = at::empty_like(w, at::MemoryFormat::Contiguous);
  Tensor db = at::empty({bias ? w.size(0) : 0}, w.options());
  const ic_act ax = act_of(x), ag = act_of(dy);
  const int k = (int)w.size(2);
  const size_t nb = ic_conv2d_wgrad_ws_ex(&ax, &ag, k, (int)stride, (int)pad, (int)math);
  Tensor ws = workspace(dy, nb);
  check_rc(ic_conv2d_wgrad_ex(&ax, &ag, k, (int)stride, (int)pad, dw.data_ptr<float>(),
                              bias ? db.data_ptr<float>() : nullptr, (int)math, ws.data_ptr(), nb, stream_of(dy)),
           "conv2d_wgrad");
  return {dw, db};
}

// ---------------------------------------------------------------- conv_transpose2d
Tensor conv_transpose2d_fwd(const Tensor& x, const Tensor& w, const c10::optional<Tensor>& b, int64_t stride,
                            int64_t pad, int64_t output_padding, int64_t act, int64_t math) {
  check_operand(x, "x");
  check_operand(w, "weight");
  if (b.has_value()) check_operand(*b, "bias");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  TORCH_CHECK(w.dim() == 4 && w.size(0) == x.size(1) && w.size(2) == w.size(3), "conv_transpose2d: weight ",
              w.sizes(), " does not match input ", x.sizes());
  const int64_t k = w.size(2);
  const int64_t ho = (x.size(2) - 1) * stride - 2 * pad + k + output_padding;
  const int64_t wo = (x.size(3) - 1) * stride - 2 * pad + k + output_padding;
  Tensor y = new_act(x, x.size(0), w.size(1), ho, wo);
  const ic_act ax = act_of(x), ay = act_of(y);
  const size_t nb = ic_conv_transpose2d_fwd_ws_ex(&ax, (int)k, (int)stride, (int)pad, &ay, (int)math);
  Tensor ws = workspace(x, nb);
  check_rc(ic_conv_transpose2d_fwd_ex(&ax, w.data_ptr<float>(), opt_ptr(b), (int)k, (int)stride, (int)pad, &ay,
                                      (int)act, (int)math, ws.data_ptr(), nb, stream_of(x)),
           "conv_transpose2d_fwd");
  return y;
}

Tensor conv_transpose2d_dgrad(const Tensor& dy, const Tensor& w, const Tensor& x, int64_t stride, int64_t pad,
                              int64_t math) {
  check_operand(dy, "dy");
  check_operand(w, "weight");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(dy.device());
  Tensor dx = new_act(dy, x.size(0), x.size(1), x.size(2), x.size(3));
  const ic_act ag = act_of(dy), adx = act_of(dx);
  const int k = (int)w.size(2);
  const size_t nb = ic_conv_transpose2d_dgrad_ws_ex(&ag, k, (int)stride, (int)pad, &adx, (int)math);
  Tensor ws = workspace(dy, nb);
  check_rc(ic_conv_transpose2d_dgrad_ex(&ag, w.data_ptr<float>(), k, (int)stride, (int)pad, &adx, (int)math,
                                        ws.data_ptr(), nb, stream_of(dy)),
           "conv_transpose2d_dgrad");
  return dx;
}

std::tuple<Tensor, Tensor> conv_transpose2d_wgrad(const Tensor& x, const Tensor& dy, const Tensor& w, int64_t stride,
                                                  int64_t pad, bool bias, int64_t math) {
  check_operand(x, "x");
  check_operand(dy, "dy");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(dy.device());
  Tensor dw = at::empty_like(w, at::MemoryFormat::Contiguous);
  Tensor db = at::empty({bias ? w.size(1) : 0}, w.options());
  const ic_act ax = act_of(x), ag = act_of(dy);
  const int k = (int)w.size(2);
  const size_t nb = ic_conv_transpose2d_wgrad_ws_ex(&ax, &ag, k, (int)stride, (int)pad, (int)math);
  Tensor ws = workspace(dy, nb);
  check_rc(ic_conv_transpose2d_wgrad_ex(&ax, &ag, k, (int)stride, (int)pad, dw.data_ptr<float>(),
                                        bias ? db.data_ptr<float>() : nullptr, (int)math, ws.data_ptr(), nb,
                                        stream_of(dy)),
           "conv_transpose2d_wgrad");
  return {dw, db};
}

// ---------------------------------------------------------------- GDN
// gamma [C][C] (or [C][C][1][1]), beta [C], already re-parameterised (NonNegativeParam)
std::tuple<Tensor, Tensor> gdn_fwd(const Tensor& x, const Tensor& gamma, const Tensor& beta, bool inverse,
                                   int64_t math) {
  check_operand(x, "x");
  check_operand(gamma, "gamma");
  check_operand(beta, "beta");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  TORCH_CHECK(gamma.numel() == x.size(1) * x.size(1) && beta.numel() == x.size(1), "gdn: parameters do not match ",
              x.sizes());
  Tensor y = at::empty_like(x);
  Tensor norm = at::empty_like(x);
  const ic_act ax = act_of(x), ay = act_of(y);
  const size_t nb = ic_gdn_fwd_ws_ex(&ax, (int)math);
  Tensor ws = workspace(x, nb);
  check_rc(ic_gdn_fwd_ex(&ax, gamma.data_ptr<float>(), beta.data_ptr<float>(), inverse ? 1 : 0, &ay,
                         norm.data_ptr<float>(), (int)math, ws.data_ptr(), nb, stream_of(x)),
           "gdn_fwd");
  return {y, norm};
}

// dy must have x's strides (the caller matches them)
std::tuple<Tensor, Tensor, Tensor> gdn_bwd(const Tensor& x, const Tensor& norm, const Tensor& dy, const Tensor& gamma,
                                           bool inverse, int64_t math) {
  check_operand(x, "x");
  check_operand(dy, "dy");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  TORCH_CHECK(dy.sizes() == x.sizes() && dy.strides() == x.strides(), "gdn_bwd: dy must have x's shape and strides");
  Tensor dx = at::empty_like(x);
  Tensor dg = at::empty_like(gamma, at::MemoryFormat::Contiguous);
  Tensor dbeta = at::empty({x.size(1)}, gamma.options());
  const ic_act ax = act_of(x), adx = act_of(dx);
  const size_t nb = ic_gdn_bwd_ws(&ax);
  Tensor ws = workspace(x, nb);
  check_rc(ic_gdn_bwd_ex(&ax, norm.data_ptr<float>(), dy.data_ptr<float>(), gamma.data_ptr<float>(), inverse ? 1 : 0,
                         &adx, dg.data_ptr<float>(), dbeta.data_ptr<float>(), (int)math, ws.data_ptr(), nb,
                         stream_of(x)),
           "gdn_bwd");
  return {dx, dg, dbeta};
}

// gdn_bwd plus the column sums of dx over all pixels (the producing conv's bias gradient)
std::tuple<Tensor, Tensor, Tensor, Tensor> gdn_bwd_sum(const Tensor& x, const Tensor& norm, const Tensor& dy,
                                                       const Tensor& gamma, bool inverse, int64_t math) {
  check_operand(x, "x");
  check_operand(dy, "dy");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  TORCH_CHECK(dy.sizes() == x.sizes() && dy.strides() == x.strides(), "gdn_bwd_sum: dy must have x's shape and strides");
  Tensor dx = at::empty_like(x);
  Tensor dg = at::empty_like(gamma, at::MemoryFormat::Contiguous);
  Tensor dbeta = at::empty({x.size(1)}, gamma.options());
  Tensor dxsum = at::empty({x.size(1)}, gamma.options());
  const ic_act ax = act_of(x), adx = act_of(dx);
  const size_t nb = ic_gdn_bwd_ws(&ax);
  Tensor ws = workspace(x, nb);
  check_rc(ic_gdn_bwd_sum_ex(&ax, norm.data_ptr<float>(), dy.data_ptr<float>(), gamma.data_ptr<float>(),
                             inverse ? 1 : 0, &adx, dg.data_ptr<float>(), dbeta.data_ptr<float>(),
                             dxsum.data_ptr<float>(), (int)math, ws.data_ptr(), nb, stream_of(x)),
           "gdn_bwd_sum");
  return {dx, dg, dbeta, dxsum};
}


// ---------------------------------------------------------------- bf16 activation copies (C3)
// The GDN output / input gradient also as a bf16 tensor of the same shape and strides (compact NHWC),
// and the conv forward / transposed-conv input gradient that reads such a copy (include/imgcomp.h
// ic_gdn_fwd_xb, ic_gdn_bwd_sum_xb, ic_conv2d_fwd_xb, ic_conv_transpose2d_dgrad_xb).
void check_copy(const Tensor& b, const Tensor& like, const char* what) {
  TORCH_CHECK(b.is_cuda() && b.scalar_type() == at::kBFloat16 && b.sizes() == like.sizes() &&
                  b.strides() == like.strides(),
              "imgcomp: ", what, " must be a bf16 tensor with the shape and strides of its fp32 tensor");
}
std::tuple<Tensor, Tensor, Tensor> gdn_fwd_xb(const Tensor& x, const Tensor& gamma, const Tensor& beta, bool inverse,
                                              int64_t math) {
  check_operand(x, "x");
  check_operand(gamma, "gamma");
  check_operand(beta, "beta");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  TORCH_CHECK(gamma.numel() == x.size(1) * x.size(1) && beta.numel() == x.size(1), "gdn: parameters do not match ",
              x.sizes());
  Tensor y = at::empty_like(x);
  Tensor norm = at::empty_like(x);
  Tensor yb = at::empty_like(x, x.options().dtype(at::kBFloat16));
  const ic_act ax = act_of(x), ay = act_of(y);
  const size_t nb = ic_gdn_fwd_ws_ex(&ax, (int)math);
  Tensor ws = workspace(x, nb);
  check_rc(ic_gdn_fwd_xb(&ax, gamma.data_ptr<float>(), beta.data_ptr<float>(), inverse ? 1 : 0, &ay,
                         norm.data_ptr<float>(), yb.data_ptr(), (int)math, ws.data_ptr(), nb, stream_of(x)),
           "gdn_fwd_xb");
  return {y, norm, yb};
}
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor> gdn_bwd_sum_xb(const Tensor& x, const Tensor& norm, const Tensor& dy,
                                                                  const Tensor& gamma, bool inverse, int64_t math) {
  check_operand(x, "x");
  check_operand(dy, "dy");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  TORCH_CHECK(dy.sizes() == x.sizes() && dy.strides() == x.strides(), "gdn_bwd_sum_xb: dy must have x's shape and strides");
  Tensor dx = at::empty_like(x);
  Tensor dg = at::empty_like(gamma, at::MemoryFormat::Contiguous);
  Tensor dbeta = at::empty({x.size(1)}, gamma.options());
  Tensor dxsum = at::empty({x.size(1)}, gamma.options());
  Tensor dxb = at::empty_like(x, x.options().dtype(at::kBFloat16));
  const ic_act ax = act_of(x), adx = act_of(dx);
  const size_t nb = ic_gdn_bwd_ws(&ax);
  Tensor ws = workspace(x, nb);
  check_rc(ic_gdn_bwd_sum_xb(&ax, norm.data_ptr<float>(), dy.data_ptr<float>(), gamma.data_ptr<float>(),
                             inverse ? 1 : 0, &adx, dg.data_ptr<float>(), dbeta.data_ptr<float>(),
                             dxsum.data_ptr<float>(), dxb.data_ptr(), (int)math, ws.data_ptr(), nb, stream_of(x)),
           "gdn_bwd_sum_xb");
  return {dx, dg, dbeta, dxsum, dxb};
}
// norm recomputed (C3, round 6; include/imgcomp.h ic_gdn_fwd_rn / ic_gdn_bwd_sum_rn): the forward leaves norm
// out, the backward forms it again from x, gamma and beta.  xb: also the bf16 copy of y / dx (else an empty
// bf16 tensor is returned in its place).
std::tuple<Tensor, Tensor> gdn_fwd_rn(const Tensor& x, const Tensor& gamma, const Tensor& beta, bool inverse,
                                      int64_t math, bool xb) {
  check_operand(x, "x");
  check_operand(gamma, "gamma");
  check_operand(beta, "beta");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  TORCH_CHECK(gamma.numel() == x.size(1) * x.size(1) && beta.numel() == x.size(1), "gdn: parameters do not match ",
              x.sizes());
  Tensor y = at::empty_like(x);
  Tensor yb = xb ? at::empty_like(x, x.options().dtype(at::kBFloat16)) : at::empty({0}, x.options().dtype(at::kBFloat16));
  const ic_act ax = act_of(x), ay = act_of(y);
  const size_t nb = ic_gdn_fwd_ws_ex(&ax, (int)math);
  Tensor ws = workspace(x, nb);
  check_rc(ic_gdn_fwd_rn(&ax, gamma.data_ptr<float>(), beta.data_ptr<float>(), inverse ? 1 : 0, &ay,
                         xb ? yb.data_ptr() : nullptr, (int)math, ws.data_ptr(), nb, stream_of(x)),
           "gdn_fwd_rn");
  return {y, yb};
}
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor> gdn_bwd_sum_rn(const Tensor& x, const Tensor& beta, const Tensor& dy,
                                                                  const Tensor& gamma, bool inverse, int64_t math,
                                                                  bool xb) {
  check_operand(x, "x");
  check_operand(dy, "dy");
  check_operand(beta, "beta");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  TORCH_CHECK(dy.sizes() == x.sizes() && dy.strides() == x.strides(), "gdn_bwd_sum_rn: dy must have x's shape and strides");
  TORCH_CHECK(beta.numel() == x.size(1), "gdn_bwd_sum_rn: beta does not match ", x.sizes());
  Tensor dx = at::empty_like(x);
  Tensor dg = at::empty_like(gamma, at::MemoryFormat::Contiguous);
  Tensor dbeta = at::empty({x.size(1)}, gamma.options());
  Tensor dxsum = at::empty({x.size(1)}, gamma.options());
  Tensor dxb = xb ? at::empty_like(x, x.options().dtype(at::kBFloat16)) : at::empty({0}, x.options().dtype(at::kBFloat16));
  const ic_act ax = act_of(x), adx = act_of(dx);
  const size_t nb = ic_gdn_bwd_ws(&ax);
  Tensor ws = workspace(x, nb);
  check_rc(ic_gdn_bwd_sum_rn(&ax, beta.data_ptr<float>(), dy.data_ptr<float>(), gamma.data_ptr<float>(),
                             inverse ? 1 : 0, &adx, dg.data_ptr<float>(), dbeta.data_ptr<float>(),
                             dxsum.data_ptr<float>(), xb ? dxb.data_ptr() : nullptr, (int)math, ws.data_ptr(), nb,
                             stream_of(x)),
           "gdn_bwd_sum_rn");
  return {dx, dg, dbeta, dxsum, dxb};
}
Tensor conv2d_fwd_xb(const Tensor& x, const Tensor& xb, const Tensor& w, const c10::optional<Tensor>& b, int64_t stride,
                     int64_t pad, int64_t act, int64_t math) {
  check_operand(x, "x");
  check_operand(w, "weight");
  check_copy(xb, x, "xb");
  if (b.has_value()) check_operand(*b, "bias");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  TORCH_CHECK(w.dim() == 4 && w.size(1) == x.size(1) && w.size(2) == w.size(3), "conv2d: weight ", w.sizes(),
              " does not match input ", x.sizes());
  const int64_t k = w.size(2);
  const int64_t ho = (x.size(2) + 2 * pad - k) / stride + 1, wo = (x.size(3) + 2 * pad - k) / stride + 1;
  Tensor y = new_act(x, x.size(0), w.size(0), ho, wo);
  const ic_act ax = act_of(x), ay = act_of(y);
  const size_t nb = ic_conv2d_fwd_ws_ex(&ax, (int)k, (int)stride, (int)pad, &ay, (int)math | IC_MATH_XB);
  Tensor ws = workspace(x, nb);
  check_rc(ic_conv2d_fwd_xb(&ax, xb.data_ptr(), w.data_ptr<float>(), opt_ptr(b), (int)k, (int)stride, (int)pad, &ay,
                            (int)act, (int)math, ws.data_ptr(), nb, stream_of(x)),
           "conv2d_fwd_xb");
  return y;
}
Tensor conv_transpose2d_dgrad_xb(const Tensor& dy, const Tensor& dyb, const Tensor& w, const Tensor& x, int64_t stride,
                                 int64_t pad, int64_t math) {
  check_operand(dy, "dy");
  check_operand(w, "weight");
  check_copy(dyb, dy, "dyb");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(dy.device());
  Tensor dx = new_act(dy, x.size(0), x.size(1), x.size(2), x.size(3));
  const ic_act ag = act_of(dy), adx = act_of(dx);
  const int k = (int)w.size(2);
  const size_t nb = ic_conv_transpose2d_dgrad_ws_ex(&ag, k, (int)stride, (int)pad, &adx, (int)math | IC_MATH_XB);
  Tensor ws = workspace(dy, nb);
  check_rc(ic_conv_transpose2d_dgrad_xb(&ag, dyb.data_ptr(), w.data_ptr<float>(), k, (int)stride, (int)pad, &adx,
                                        (int)math, ws.data_ptr(), nb, stream_of(dy)),
           "conv_transpose2d_dgrad_xb");
  return dx;
}

Tensor conv2d_dgrad_xb(const Tensor& dy, const Tensor& dyb, const Tensor& w, const Tensor& x, int64_t stride,
                       int64_t pad, int64_t math) {
  check_operand(dy, "dy");
  check_operand(w, "weight");
  check_copy(dyb, dy, "dyb");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(dy.device());
  Tensor dx = new_act(dy, x.size(0), x.size(1), x.size(2), x.size(3));
  const ic_act ag = act_of(dy), adx = act_of(dx);
  const int k = (int)w.size(2);
  const size_t nb = ic_conv2d_dgrad_ws_ex(&ag, k, (int)stride, (int)pad, &adx, (int)math | IC_MATH_XB);
  Tensor ws = workspace(dy, nb);
  check_rc(ic_conv2d_dgrad_xb(&ag, dyb.data_ptr(), w.data_ptr<float>(), k, (int)stride, (int)pad, &adx, (int)math,
                              ws.data_ptr(), nb, stream_of(dy)),
           "conv2d_dgrad_xb");
  return dx;
}
Tensor conv_transpose2d_fwd_xb(const Tensor& x, const Tensor& xb, const Tensor& w, const c10::optional<Tensor>& b,
                               int64_t stride, int64_t pad, int64_t opad, int64_t act, int64_t math) {
  check_operand(x, "x");
  check_operand(w, "weight");
  check_copy(xb, x, "xb");
  if (b.has_value()) check_operand(*b, "bias");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  TORCH_CHECK(w.dim() == 4 && w.size(0) == x.size(1) && w.size(2) == w.size(3), "conv_transpose2d: weight ", w.sizes(),
              " does not match input ", x.sizes());
  const int64_t k = w.size(2);
  const int64_t ho = (x.size(2) - 1) * stride - 2 * pad + k + opad, wo = (x.size(3) - 1) * stride - 2 * pad + k + opad;
  Tensor y = new_act(x, x.size(0), w.size(1), ho, wo);
  const ic_act ax = act_of(x), ay = act_of(y);
  const size_t nb = ic_conv_transpose2d_fwd_ws_ex(&ax, (int)k, (int)stride, (int)pad, &ay, (int)math | IC_MATH_XB);
  Tensor ws = workspace(x, nb);
  check_rc(ic_conv_transpose2d_fwd_xb(&ax, xb.data_ptr(), w.data_ptr<float>(), opt_ptr(b), (int)k, (int)stride,
                                      (int)pad, &ay, (int)act, (int)math, ws.data_ptr(), nb, stream_of(x)),
           "conv_transpose2d_fwd_xb");
  return y;
}

template <bool TR>
std::tuple<Tensor, Tensor> wgrad_xb(const Tensor& x, const Tensor& xb, const Tensor& dy, const Tensor& dyb,
                                    const Tensor& w, int64_t stride, int64_t pad, bool bias, int64_t math) {
  check_operand(x, "x");
  check_operand(dy, "dy");
  check_copy(xb, x, "xb");
  check_copy(dyb, dy, "dyb");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(dy.device());
  Tensor dw = at::empty_like(w, at::MemoryFormat::Contiguous);
  Tensor db = at::empty({bias ? (TR ? w.size(1) : w.size(0)) : 0}, w.options());
  const ic_act ax = act_of(x), ag = act_of(dy);
  const int k = (int)w.size(2);
  const size_t nb = TR ? ic_conv_transpose2d_wgrad_ws_ex(&ax, &ag, k, (int)stride, (int)pad, (int)math)
                       : ic_conv2d_wgrad_ws_ex(&ax, &ag, k, (int)stride, (int)pad, (int)math);
  Tensor ws = workspace(dy, nb);
  float* dbp = bias ? db.data_ptr<float>() : nullptr;
  const int rc = TR ? ic_conv_transpose2d_wgrad_xb(&ax, xb.data_ptr(), &ag, dyb.data_ptr(), k, (int)stride, (int)pad,
                                                   dw.data_ptr<float>(), dbp, (int)math, ws.data_ptr(), nb,
                                                   stream_of(dy))
                    : ic_conv2d_wgrad_xb(&ax, xb.data_ptr(), &ag, dyb.data_ptr(), k, (int)stride, (int)pad,
                                         dw.data_ptr<float>(), dbp, (int)math, ws.data_ptr(), nb, stream_of(dy));
  check_rc(rc, TR ? "conv_transpose2d_wgrad_xb" : "conv2d_wgrad_xb");
  return {dw, db};
}
std::tuple<Tensor, Tensor> conv2d_wgrad_xb(const Tensor& x, const Tensor& xb, const Tensor& dy, const Tensor& dyb,
                                           const Tensor& w, int64_t stride, int64_t pad, bool bias, int64_t math) {
  return wgrad_xb<false>(x, xb, dy, dyb, w, stride, pad, bias, math);
}
std::tuple<Tensor, Tensor> conv_transpose2d_wgrad_xb(const Tensor& x, const Tensor& xb, const Tensor& dy,
                                                     const Tensor& dyb, const Tensor& w, int64_t stride, int64_t pad,
                                                     bool bias, int64_t math) {
  return wgrad_xb<true>(x, xb, dy, dyb, w, stride, pad, bias, math);
}

// ---------------------------------------------------------------- elementwise, losses, entropy models
// Reference interfaces: NonNegativeParam.forward (layers/gdn.py:59-62), Lower/UpperBound
// (layers/bound.py:28-59), ReLU / torch.abs (prior_analysis.py:65, bmshl2018.py:72), the exp-clamp of
// prior_synthesis.py:72, _ce_loss (blocks/entropy_model.py:171-185), nn.MSELoss (loss.py:25),
// EntropyModel / CDFEstimator (entropy_model.py:47-269), SymmetricConditionalModel and its Laplacian /
// Gaussian kinds (entropy_model.py:272-378), SSIMLoss / MS_SSIMLoss (loss.py:48-188).
// The elementwise launchers index dense storage: every operand of one call has the same strides.
void check_dense(const Tensor& t, const char* what) {
  check_operand(t, what);
  TORCH_CHECK(t.is_non_overlapping_and_dense(), "imgcomp: ", what, " must be dense (non-overlapping) storage");
}

// same shape and the same strides on every dimension of extent > 1 (a size-1 dimension's
// stride addresses nothing): element i of the dense storage is the same logical element in both
bool same_layout(const Tensor& a, const Tensor& b) {
  if (a.sizes() != b.sizes()) return false;
  for (int64_t i = 0; i < a.dim(); ++i)
    if (a.size(i) > 1 && a.stride(i) != b.stride(i)) return false;
  return true;
}

void check_same_layout(const Tensor& a, const Tensor& b, const char* what) {
  check_dense(b, what);
  TORCH_CHECK(same_layout(a, b), "imgcomp: ", what, " must have the shape and strides of its partner operand");
}

Tensor like(const Tensor& t) { return at::empty_like(t, at::MemoryFormat::Preserve); }
Tensor none_like(const Tensor& t) { return at::empty({0}, t.options()); }

Tensor nonneg_fwd(const Tensor& p, double bound, double ped) {
  check_dense(p, "param");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(p.device());
  Tensor out = like(p);
  check_rc(ic_nonneg_fwd(p.data_ptr<float>(), p.numel(), (float)bound, (float)ped, out.data_ptr<float>(), stream_of(p)),
           "nonneg_fwd");
  return out;
}
Tensor nonneg_bwd(const Tensor& p, const Tensor& g, double bound) {
  check_dense(p, "param");
  check_same_layout(p, g, "gradient");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(p.device());
  Tensor gi = like(p);
  check_rc(ic_nonneg_bwd(p.data_ptr<float>(), g.data_ptr<float>(), p.numel(), (float)bound, gi.data_ptr<float>(),
                         stream_of(p)),
           "nonneg_bwd");
  return gi;
}
// NonNegativeParam of several tensors, one launch (ic_nonneg_multi)
std::vector<Tensor> nonneg_multi_run(at::TensorList p, at::TensorList g, at::ArrayRef<double> bound,
                                     at::ArrayRef<double> ped, bool bwd) {
  TORCH_CHECK(p.size() == bound.size() && (bwd ? g.size() == p.size() : ped.size() == p.size()),
              "nonneg_multi: one bound (and pedestal / gradient) per tensor");
  std::vector<Tensor> outs;
  std::vector<ic_nonneg_tensor> ts(p.size());
  for (size_t i = 0; i < p.size(); ++i) {
    check_dense(p[i], "param");
    TORCH_CHECK(p[i].device() == p[0].device(), "nonneg_multi: tensors on one device");
    if (bwd) check_same_layout(p[i], g[i], "gradient");
    outs.push_back(like(p[i]));
    ts[i] = ic_nonneg_tensor{p[i].data_ptr<float>(), bwd ? nullptr : outs[i].data_ptr<float>(),
                             bwd ? g[i].data_ptr<float>() : nullptr, bwd ? outs[i].data_ptr<float>() : nullptr,
                             (long long)p[i].numel(), (float)bound[i], bwd ? 0.f : (float)ped[i]};
  }
  if (p.empty()) return outs;
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(p[0].device());
  check_rc(ic_nonneg_multi(ts.data(), (int)ts.size(), bwd ? 1 : 0, stream_of(p[0])), "nonneg_multi");
  return outs;
}
std::vector<Tensor> nonneg_multi_fwd(at::TensorList p, at::ArrayRef<double> bound, at::ArrayRef<double> ped) {
  return nonneg_multi_run(p, {}, bound, ped, false);
}
std::vector<Tensor> nonneg_multi_bwd(at::TensorList p, at::TensorList g, at::ArrayRef<double> bound) {
  return nonneg_multi_run(p, g, bound, {}, true);
}
Tensor bound_fwd(const Tensor& x, double bound, bool upper) {
  check_dense(x, "x");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  Tensor y = like(x);
  check_rc(ic_bound_fwd(x.data_ptr<float>(), x.numel(), (float)bound, upper ? 1 : 0, y.data_ptr<float>(), stream_of(x)),
           "bound_fwd");
  return y;
}
Tensor bound_bwd(const Tensor& x, const Tensor& g, double bound, bool upper) {
  check_dense(x, "x");
  check_same_layout(x, g, "gradient");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  Tensor gx = like(x);
  check_rc(ic_bound_bwd(x.data_ptr<float>(), g.data_ptr<float>(), x.numel(), (float)bound, upper ? 1 : 0,
                        gx.data_ptr<float>(), stream_of(x)),
           "bound_bwd");
  return gx;
}
Tensor relu_fwd(const Tensor& x) {
  check_dense(x, "x");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  Tensor y = like(x);
  check_rc(ic_relu_fwd(x.data_ptr<float>(), x.numel(), y.data_ptr<float>(), stream_of(x)), "relu_fwd");
  return y;
}
Tensor relu_bwd(const Tensor& y, const Tensor& g) {
  check_dense(y, "y");
  check_same_layout(y, g, "gradient");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(y.device());
  Tensor gx = like(y);
  check_rc(ic_relu_bwd(y.data_ptr<float>(), g.data_ptr<float>(), y.numel(), gx.data_ptr<float>(), stream_of(y)),
           "relu_bwd");
  return gx;
}
Tensor abs_fwd(const Tensor& x) {
  check_dense(x, "x");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  Tensor y = like(x);
  check_rc(ic_abs_fwd(x.data_ptr<float>(), x.numel(), y.data_ptr<float>(), stream_of(x)), "abs_fwd");
  return y;
}
Tensor abs_bwd(const Tensor& x, const Tensor& g) {
  check_dense(x, "x");
  check_same_layout(x, g, "gradient");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  Tensor gx = like(x);
  check_rc(ic_abs_bwd(x.data_ptr<float>(), g.data_ptr<float>(), x.numel(), gx.data_ptr<float>(), stream_of(x)),
           "abs_bwd");
  return gx;
}
// (sigma, e = exp(v)); e is what the backward reads
std::tuple<Tensor, Tensor> exp_clamp_fwd(const Tensor& v, double lo, double hi) {
  check_dense(v, "v");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(v.device());
  Tensor s = like(v), e = like(v);
  check_rc(ic_exp_clamp_fwd(v.data_ptr<float>(), v.numel(), (float)lo, (float)hi, s.data_ptr<float>(),
                            e.data_ptr<float>(), stream_of(v)),
           "exp_clamp_fwd");
  return {s, e};
}
Tensor exp_clamp_bwd(const Tensor& e, const Tensor& g, double lo, double hi) {
  check_dense(e, "e");
  check_same_layout(e, g, "gradient");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(e.device());
  Tensor gv = like(e);
  check_rc(ic_exp_clamp_bwd(e.data_ptr<float>(), g.data_ptr<float>(), e.numel(), (float)lo, (float)hi,
                            gv.data_ptr<float>(), stream_of(e)),
           "exp_clamp_bwd");
  return gv;
}
Tensor ce_loss_fwd(const Tensor& p) {
  check_dense(p, "p");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(p.device());
  Tensor out = at::empty({}, p.options());
  const size_t nb = ic_reduce_ws(p.numel());
  Tensor ws = workspace(p, nb);
  check_rc(ic_ce_loss_fwd(p.data_ptr<float>(), p.numel(), out.data_ptr<float>(), ws.data_ptr(), nb, stream_of(p)),
           "ce_loss_fwd");
  return out;
}
Tensor ce_loss_bwd(const Tensor& p, const Tensor& g) {
  check_dense(p, "p");
  check_operand(g, "gradient");
  TORCH_CHECK(g.numel() == 1, "ce_loss_bwd: the gradient of a scalar loss is one value");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(p.device());
  Tensor gc = g.contiguous();
  Tensor gp = like(p);
  check_rc(ic_ce_loss_bwd(p.data_ptr<float>(), gc.data_ptr<float>(), p.numel(), gp.data_ptr<float>(), stream_of(p)),
           "ce_loss_bwd");
  return gp;
}
Tensor mse_fwd(const Tensor& a, const Tensor& b) {
  check_dense(a, "input");
  check_same_layout(a, b, "target");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(a.device());
  Tensor out = at::empty({}, a.options());
  const size_t nb = ic_reduce_ws(a.numel());
  Tensor ws = workspace(a, nb);
  check_rc(ic_mse_fwd(a.data_ptr<float>(), b.data_ptr<float>(), a.numel(), out.data_ptr<float>(), ws.data_ptr(), nb,
                      stream_of(a)),
           "mse_fwd");
  return out;
}
// (ga, gb); a gradient that is not wanted comes back empty (0 elements)
std::tuple<Tensor, Tensor> mse_bwd(const Tensor& a, const Tensor& b, const Tensor& g, bool need_a, bool need_b) {
  check_dense(a, "input");
  check_same_layout(a, b, "target");
  check_operand(g, "gradient");
  TORCH_CHECK(g.numel() == 1, "mse_bwd: the gradient of a scalar loss is one value");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(a.device());
  Tensor gc = g.contiguous();
  Tensor ga = need_a ? like(a) : none_like(a), gb = need_b ? like(b) : none_like(b);
  check_rc(ic_mse_bwd(a.data_ptr<float>(), b.data_ptr<float>(), gc.data_ptr<float>(), a.numel(),
                      need_a ? ga.data_ptr<float>() : nullptr, need_b ? gb.data_ptr<float>() : nullptr, stream_of(a)),
           "mse_bwd");
  return {ga, gb};
}
Tensor sqdiff_fwd(const Tensor& a, const Tensor& b) {
  check_dense(a, "input");
  check_same_layout(a, b, "target");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(a.device());
  Tensor out = like(a);
  check_rc(ic_sqdiff_fwd(a.data_ptr<float>(), b.data_ptr<float>(), a.numel(), out.data_ptr<float>(), stream_of(a)),
           "sqdiff_fwd");
  return out;
}
std::tuple<Tensor, Tensor> sqdiff_bwd(const Tensor& a, const Tensor& b, const Tensor& g, bool need_a, bool need_b) {
  check_dense(a, "input");
  check_same_layout(a, b, "target");
  check_same_layout(a, g, "gradient");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(a.device());
  Tensor ga = need_a ? like(a) : none_like(a), gb = need_b ? like(b) : none_like(b);
  check_rc(ic_sqdiff_bwd(a.data_ptr<float>(), b.data_ptr<float>(), g.data_ptr<float>(), a.numel(),
                         need_a ? ga.data_ptr<float>() : nullptr, need_b ? gb.data_ptr<float>() : nullptr, stream_of(a)),
           "sqdiff_bwd");
  return {ga, gb};
}

// ---- training noise: mode 3 takes the device Philox state {seed, base} (int64[2]) as `u`
const void* noise_ptr(const std::optional<Tensor>& u, int64_t mode, const Tensor& like_t) {
  if (mode == 0) {
    TORCH_CHECK(u.has_value() && u->defined(), "imgcomp: mode 0 needs the uniform draws u");
    check_same_layout(like_t, *u, "u");
    return u->data_ptr<float>();
  }
  if (mode == 3) {
    TORCH_CHECK(u.has_value() && u->defined() && u->is_cuda() && u->scalar_type() == at::kLong && u->numel() == 2 &&
                    u->is_contiguous(),
                "imgcomp: mode 3 needs the device Philox state (int64[2] {seed, base})");
    return u->data_ptr();
  }
  return nullptr;
}

// the factorized model's 11 fixed-width parameter tensors (DIMS [3, 3, 3]) in CDFEstimator order
ic_fact_params fact_params(at::TensorList prm) {
  TORCH_CHECK(prm.size() == 11, "factorized: expected the 11 CDF parameter tensors, got ", prm.size());
  for (const Tensor& t : prm) check_operand(t, "CDF parameter");
  const float* v[11];
  for (int i = 0; i < 11; ++i) {
    TORCH_CHECK(prm[i].is_contiguous(), "factorized: CDF parameters must be contiguous");
    v[i] = prm[i].data_ptr<float>();
  }
  return ic_fact_params{v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], v[8], v[9], v[10]};
}

// z is the channels-last dense (N, ..., C) view: channel = flat index % C
std::tuple<Tensor, Tensor> factorized_fwd(const Tensor& z, int64_t C, at::TensorList prm, int64_t mode,
                                          const std::optional<Tensor>& u, int64_t seed, int64_t offset) {
  check_operand(z, "z");
  TORCH_CHECK(z.is_contiguous(), "factorized_fwd: z must be the contiguous channels-last view");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(z.device());
  const ic_fact_params cp = fact_params(prm);
  Tensor q = like(z), p = like(z);
  check_rc(ic_factorized_fwd(z.data_ptr<float>(), z.numel(), (int)C, &cp, (int)mode, (const float*)noise_ptr(u, mode, z),
                             (unsigned long long)seed, (unsigned long long)offset, q.data_ptr<float>(),
                             p.data_ptr<float>(), stream_of(z)),
           "factorized_fwd");
  return {q, p};
}

const float* opt_grad(const std::optional<Tensor>& g, const Tensor& like_t, const char* what) {
  if (!g.has_value() || !g->defined()) return nullptr;
  check_same_layout(like_t, *g, what);
  return g->data_ptr<float>();
}

std::tuple<Tensor, std::vector<Tensor>> factorized_bwd(const Tensor& q, int64_t C, at::TensorList prm,
                                                       const std::optional<Tensor>& dq, const std::optional<Tensor>& dp) {
  check_operand(q, "q");
  TORCH_CHECK(q.is_contiguous(), "factorized_bwd: q must be contiguous");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(q.device());
  const ic_fact_params cp = fact_params(prm);
  std::vector<Tensor> grads;
  for (const Tensor& t : prm) grads.push_back(at::empty_like(t));
  float* g[11];
  for (int i = 0; i < 11; ++i) g[i] = grads[i].data_ptr<float>();
  const ic_fact_grads cg{g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], g[8], g[9], g[10]};
  Tensor dz = like(q);
  check_rc(ic_factorized_bwd(q.data_ptr<float>(), q.numel(), (int)C, &cp, opt_grad(dq, q, "dq"), opt_grad(dp, q, "dp"),
                             dz.data_ptr<float>(), &cg, stream_of(q)),
           "factorized_bwd");
  return {dz, grads};
}

// any CDF MLP: dims = {1, DIMS..., 1}; params [w0, b0, f0, w1, b1, f1, ..., w_last, b_last]
ic_fact_net fact_net(at::IntArrayRef dims, at::TensorList prm) {
  const int L = (int)dims.size() - 1;
  TORCH_CHECK(L >= 1 && L <= IC_FACT_NET_MAXL, "factorized: CDF MLP of ", L, " layers (at most ", IC_FACT_NET_MAXL,
              ")");
  TORCH_CHECK((int64_t)prm.size() == 3 * L - 1, "factorized: expected ", 3 * L - 1, " CDF parameter tensors");
  ic_fact_net net{};
  net.nlayers = L;
  for (int i = 0; i <= L; ++i) net.dims[i] = (int)dims[i];
  int k = 0;
  for (int l = 0; l < L; ++l) {
    for (int j = 0; j < (l < L - 1 ? 3 : 2); ++j) {
      check_operand(prm[k + j], "CDF parameter");
      TORCH_CHECK(prm[k + j].is_contiguous(), "factorized: CDF parameters must be contiguous");
    }
    net.w[l] = prm[k].data_ptr<float>();
    net.b[l] = prm[k + 1].data_ptr<float>();
    net.f[l] = l < L - 1 ? prm[k + 2].data_ptr<float>() : nullptr;
    k += l < L - 1 ? 3 : 2;
  }
  return net;
}

std::tuple<Tensor, Tensor> factorized_net_fwd(const Tensor& z, int64_t C, at::IntArrayRef dims, double bin,
                                              at::TensorList prm, int64_t mode, const std::optional<Tensor>& u,
                                              int64_t seed, int64_t offset) {
  check_operand(z, "z");
  TORCH_CHECK(z.is_contiguous(), "factorized_net_fwd: z must be the contiguous channels-last view");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(z.device());
  const ic_fact_net net = fact_net(dims, prm);
  Tensor q = like(z), p = like(z);
  const size_t nb = ic_factorized_net_ws(z.numel(), (int)C, &net, 0);  // 0: the register kernels
  Tensor ws = workspace(z, nb);
  check_rc(ic_factorized_fwd_net_ex(z.data_ptr<float>(), z.numel(), (int)C, &net, (float)bin, (int)mode,
                                    (const float*)noise_ptr(u, mode, z), (unsigned long long)seed,
                                    (unsigned long long)offset, q.data_ptr<float>(), p.data_ptr<float>(),
                                    ws.data_ptr(), nb, stream_of(z)),
           "factorized_net_fwd");
  return {q, p};
}

std::tuple<Tensor, std::vector<Tensor>> factorized_net_bwd(const Tensor& q, int64_t C, at::IntArrayRef dims, double bin,
                                                           at::TensorList prm, const std::optional<Tensor>& dq,
                                                           const std::optional<Tensor>& dp) {
  check_operand(q, "q");
  TORCH_CHECK(q.is_contiguous(), "factorized_net_bwd: q must be contiguous");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(q.device());
  const ic_fact_net net = fact_net(dims, prm);
  std::vector<Tensor> grads;
  for (const Tensor& t : prm) grads.push_back(at::empty_like(t));
  ic_fact_net_grads g{};
  const int L = net.nlayers;
  int k = 0;
  for (int l = 0; l < L; ++l) {
    g.w[l] = grads[k].data_ptr<float>();
    g.b[l] = grads[k + 1].data_ptr<float>();
    g.f[l] = l < L - 1 ? grads[k + 2].data_ptr<float>() : nullptr;
    k += l < L - 1 ? 3 : 2;
  }
  Tensor dz = like(q);
  const size_t nb = ic_factorized_net_ws(q.numel(), (int)C, &net, 1);
  Tensor ws = workspace(q, nb);
  check_rc(ic_factorized_bwd_net_ex(q.data_ptr<float>(), q.numel(), (int)C, &net, (float)bin, opt_grad(dq, q, "dq"),
                                    opt_grad(dp, q, "dp"), dz.data_ptr<float>(), &g, ws.data_ptr(), nb, stream_of(q)),
           "factorized_net_bwd");
  return {dz, grads};
}

Tensor quantize(const Tensor& y, int64_t mode, const std::optional<Tensor>& u, int64_t seed, int64_t offset,
                double bin) {
  check_dense(y, "y");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(y.device());
  Tensor q = like(y);
  check_rc(ic_quantize(y.data_ptr<float>(), y.numel(), (int)mode, (const float*)noise_ptr(u, mode, y),
                       (unsigned long long)seed, (unsigned long long)offset, (float)bin, q.data_ptr<float>(),
                       stream_of(y)),
           "quantize");
  return q;
}

std::tuple<Tensor, Tensor> conditional_fwd(const Tensor& y, const Tensor& scale, const std::optional<Tensor>& mean,
                                           int64_t kind, int64_t mode, const std::optional<Tensor>& u, int64_t seed,
                                           int64_t offset, double bin) {
  check_dense(y, "y");
  check_same_layout(y, scale, "scale");
  const float* mp = opt_grad(mean, y, "mean");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(y.device());
  Tensor q = like(y), p = like(y);
  check_rc(ic_conditional_fwd_bin(y.data_ptr<float>(), scale.data_ptr<float>(), mp, y.numel(), (int)kind, (int)mode,
                                  (const float*)noise_ptr(u, mode, y), (unsigned long long)seed,
                                  (unsigned long long)offset, (float)bin, q.data_ptr<float>(), p.data_ptr<float>(),
                                  stream_of(y)),
           "conditional_fwd");
  return {q, p};
}

// (dy, dscale, dmean); an unwanted gradient comes back empty
std::tuple<Tensor, Tensor, Tensor> conditional_bwd(const Tensor& q, const Tensor& scale,
                                                   const std::optional<Tensor>& mean, int64_t kind, double bin,
                                                   const std::optional<Tensor>& dq, const std::optional<Tensor>& dp,
                                                   bool need_y, bool need_scale, bool need_mean) {
  check_dense(q, "q");
  check_same_layout(q, scale, "scale");
  const float* mp = opt_grad(mean, q, "mean");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(q.device());
  need_mean = need_mean && mp != nullptr;
  Tensor dy = need_y ? like(q) : none_like(q), ds = need_scale ? like(q) : none_like(q),
         dm = need_mean ? like(q) : none_like(q);
  check_rc(ic_conditional_bwd_bin(q.data_ptr<float>(), scale.data_ptr<float>(), mp, q.numel(), (int)kind, (float)bin,
                                  opt_grad(dq, q, "dq"), opt_grad(dp, q, "dp"), need_y ? dy.data_ptr<float>() : nullptr,
                                  need_scale ? ds.data_ptr<float>() : nullptr, need_mean ? dm.data_ptr<float>() : nullptr,
                                  stream_of(q)),
           "conditional_bwd");
  return {dy, ds, dm};
}

// advance the device Philox base past the n draws of the previous step (in place)
void philox_advance(const Tensor& state, int64_t n) {
  TORCH_CHECK(state.is_cuda() && state.scalar_type() == at::kLong && state.numel() == 2 && state.is_contiguous(),
              "philox_advance: expected the device state int64[2] {seed, base}");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(state.device());
  check_rc(ic_philox_advance((unsigned long long*)state.data_ptr(), (unsigned long long)n, stream_of(state)),
           "philox_advance");
}

// ---- SSIM / MS-SSIM: (loss, state); state (written here, read by the backward) sized by ic_msssim_state_bytes
std::tuple<Tensor, Tensor> msssim_fwd(const Tensor& a_, const Tensor& b_, int64_t nlev, int64_t fs, double sigma,
                                      double max_val, bool log_scale, int64_t single, double k1, double k2, double eps,
                                      at::ArrayRef<double> weights) {
  check_operand(a_, "img1");
  check_operand(b_, "img2");
  TORCH_CHECK(a_.dim() == 4 && a_.sizes() == b_.sizes(), "msssim: two images of one 4-D shape expected");
  TORCH_CHECK((int64_t)weights.size() == nlev, "msssim: one weight per level");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(a_.device());
  const Tensor a = a_.contiguous(), b = b_.contiguous();
  const int N = (int)a.size(0), C = (int)a.size(1), H = (int)a.size(2), W = (int)a.size(3);
  const size_t sb = ic_msssim_state_bytes(N, C, H, W, (int)nlev, (int)fs);
  TORCH_CHECK(sb > 0, "ms-ssim: image ", H, "x", W, " too small for ", nlev, " levels of a ", fs, "x", fs, " window");
  Tensor state = at::empty({(int64_t)(sb / 4)}, a.options());
  const size_t nb = ic_msssim_ws(N, C, H, W, (int)nlev, (int)fs);
  Tensor ws = workspace(a, nb);
  std::vector<float> w(weights.begin(), weights.end());
  Tensor out = (single && log_scale) ? at::empty({N}, a.options()) : at::empty({}, a.options());
  check_rc(ic_msssim_fwd(a.data_ptr<float>(), b.data_ptr<float>(), N, C, H, W, (int)nlev, (int)fs, (float)sigma,
                         (float)max_val, log_scale ? 1 : 0, (int)single, (float)k1, (float)k2, (float)eps, w.data(),
                         out.data_ptr<float>(), state.data_ptr<float>(), ws.data_ptr(), nb, stream_of(a)),
           "msssim_fwd");
  return {out, state};
}

std::tuple<Tensor, Tensor> msssim_bwd(const Tensor& g_, const Tensor& state, at::IntArrayRef shape, int64_t nlev,
                                      int64_t fs, double sigma, double max_val, bool log_scale, int64_t single,
                                      double k1, double k2, double eps, at::ArrayRef<double> weights, bool need_a,
                                      bool need_b) {
  check_operand(g_, "gradient");
  check_operand(state, "state");
  TORCH_CHECK(shape.size() == 4 && (int64_t)weights.size() == nlev, "msssim_bwd: 4-D shape and one weight per level");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(g_.device());
  const Tensor g = g_.contiguous();
  const int N = (int)shape[0], C = (int)shape[1], H = (int)shape[2], W = (int)shape[3];
  TORCH_CHECK((size_t)state.numel() * 4 >= ic_msssim_state_bytes(N, C, H, W, (int)nlev, (int)fs),
              "msssim_bwd: state too small for this shape");
  const size_t nb = ic_msssim_ws(N, C, H, W, (int)nlev, (int)fs);
  Tensor ws = workspace(g, nb);
  std::vector<float> w(weights.begin(), weights.end());
  Tensor ga = need_a ? at::empty(shape, g.options()) : none_like(g);
  Tensor gb = need_b ? at::empty(shape, g.options()) : none_like(g);
  check_rc(ic_msssim_bwd(N, C, H, W, (int)nlev, (int)fs, (float)sigma, (float)max_val, log_scale ? 1 : 0, (int)single,
                         (float)k1, (float)k2, (float)eps, w.data(), g.data_ptr<float>(), state.data_ptr<float>(),
                         need_a ? ga.data_ptr<float>() : nullptr, need_b ? gb.data_ptr<float>() : nullptr,
                         ws.data_ptr(), nb, stream_of(g)),
           "msssim_bwd");
  return {ga, gb};
}

// ---------------------------------------------------------------- shape (Meta) kernels
Tensor conv2d_fwd_meta(const Tensor& x, const Tensor& w, const c10::optional<Tensor>&, int64_t stride, int64_t pad,
                       int64_t, int64_t) {
  const int64_t k = w.size(2);
  return at::empty({x.size(0), w.size(0), (x.size(2) + 2 * pad - k) / stride + 1, (x.size(3) + 2 * pad - k) / stride + 1},
                   x.options().memory_format(act_format(w.size(0))));
}
Tensor conv2d_fwd_ws_meta(const Tensor& x, const Tensor& w, const c10::optional<Tensor>& b, int64_t stride,
                          int64_t pad, int64_t act, int64_t math, Tensor&) {
  return conv2d_fwd_meta(x, w, b, stride, pad, act, math);
}
Tensor conv2d_dgrad_meta(const Tensor& dy, const Tensor&, const Tensor& x, int64_t, int64_t, int64_t) {
  return at::empty(x.sizes(), dy.options().memory_format(x.suggest_memory_format()));
}
std::tuple<Tensor, Tensor> conv2d_wgrad_meta(const Tensor&, const Tensor&, const Tensor& w, int64_t, int64_t, bool bias,
                                             int64_t) {
  return {at::empty_like(w, at::MemoryFormat::Contiguous), at::empty({bias ? w.size(0) : 0}, w.options())};
}
Tensor conv_transpose2d_fwd_meta(const Tensor& x, const Tensor& w, const c10::optional<Tensor>&, int64_t stride,
                                 int64_t pad, int64_t op, int64_t, int64_t) {
  const int64_t k = w.size(2);
  return at::empty({x.size(0), w.size(1), (x.size(2) - 1) * stride - 2 * pad + k + op,
                    (x.size(3) - 1) * stride - 2 * pad + k + op},
                   x.options().memory_format(act_format(w.size(1))));
}
Tensor conv_transpose2d_fwd_ws_meta(const Tensor& x, const Tensor& w, const c10::optional<Tensor>& b,
                                    int64_t stride, int64_t pad, int64_t op, int64_t act, int64_t math, Tensor&) {
  return conv_transpose2d_fwd_meta(x, w, b, stride, pad, op, act, math);
}
Tensor conv_transpose2d_dgrad_meta(const Tensor& dy, const Tensor&, const Tensor& x, int64_t, int64_t, int64_t) {
  return at::empty(x.sizes(), dy.options().memory_format(act_format(x.size(1))));
}
std::tuple<Tensor, Tensor> conv_transpose2d_wgrad_meta(const Tensor&, const Tensor&, const Tensor& w, int64_t, int64_t,
                                                       bool bias, int64_t) {
  return {at::empty_like(w, at::MemoryFormat::Contiguous), at::empty({bias ? w.size(1) : 0}, w.options())};
}
std::tuple<Tensor, Tensor> gdn_fwd_meta(const Tensor& x, const Tensor&, const Tensor&, bool, int64_t) {
  return {at::empty_like(x), at::empty_like(x)};
}
std::tuple<Tensor, Tensor, Tensor> gdn_bwd_meta(const Tensor& x, const Tensor&, const Tensor&, const Tensor& gamma, bool,
                                                int64_t) {
  return {at::empty_like(x), at::empty_like(gamma, at::MemoryFormat::Contiguous), at::empty({x.size(1)}, gamma.options())};
}

std::tuple<Tensor, Tensor, Tensor, Tensor> gdn_bwd_sum_meta(const Tensor& x, const Tensor&, const Tensor&,
                                                            const Tensor& gamma, bool, int64_t) {
  return {at::empty_like(x), at::empty_like(gamma, at::MemoryFormat::Contiguous), at::empty({x.size(1)}, gamma.options()),
          at::empty({x.size(1)}, gamma.options())};
}


std::tuple<Tensor, Tensor, Tensor> gdn_fwd_xb_meta(const Tensor& x, const Tensor&, const Tensor&, bool, int64_t) {
  return {at::empty_like(x), at::empty_like(x), at::empty_like(x, x.options().dtype(at::kBFloat16))};
}
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor> gdn_bwd_sum_xb_meta(const Tensor& x, const Tensor&, const Tensor&,
                                                                       const Tensor& gamma, bool, int64_t) {
  return {at::empty_like(x), at::empty_like(gamma, at::MemoryFormat::Contiguous), at::empty({x.size(1)}, gamma.options()),
          at::empty({x.size(1)}, gamma.options()), at::empty_like(x, x.options().dtype(at::kBFloat16))};
}
std::tuple<Tensor, Tensor> gdn_fwd_rn_meta(const Tensor& x, const Tensor&, const Tensor&, bool, int64_t, bool xb) {
  return {at::empty_like(x), xb ? at::empty_like(x, x.options().dtype(at::kBFloat16))
                                : at::empty({0}, x.options().dtype(at::kBFloat16))};
}
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor> gdn_bwd_sum_rn_meta(const Tensor& x, const Tensor&, const Tensor&,
                                                                       const Tensor& gamma, bool, int64_t, bool xb) {
  return {at::empty_like(x), at::empty_like(gamma, at::MemoryFormat::Contiguous), at::empty({x.size(1)}, gamma.options()),
          at::empty({x.size(1)}, gamma.options()),
          xb ? at::empty_like(x, x.options().dtype(at::kBFloat16)) : at::empty({0}, x.options().dtype(at::kBFloat16))};
}
Tensor conv2d_fwd_xb_meta(const Tensor& x, const Tensor&, const Tensor& w, const c10::optional<Tensor>& b,
                          int64_t stride, int64_t pad, int64_t act, int64_t math) {
  return conv2d_fwd_meta(x, w, b, stride, pad, act, math);
}
Tensor conv_transpose2d_dgrad_xb_meta(const Tensor& dy, const Tensor&, const Tensor& w, const Tensor& x, int64_t s,
                                      int64_t p, int64_t m) {
  return conv_transpose2d_dgrad_meta(dy, w, x, s, p, m);
}

Tensor conv2d_dgrad_xb_meta(const Tensor& dy, const Tensor&, const Tensor& w, const Tensor& x, int64_t s, int64_t p,
                            int64_t m) {
  return conv2d_dgrad_meta(dy, w, x, s, p, m);
}
Tensor conv_transpose2d_fwd_xb_meta(const Tensor& x, const Tensor&, const Tensor& w, const c10::optional<Tensor>& b,
                                    int64_t stride, int64_t pad, int64_t op, int64_t act, int64_t math) {
  return conv_transpose2d_fwd_meta(x, w, b, stride, pad, op, act, math);
}

std::tuple<Tensor, Tensor> conv2d_wgrad_xb_meta(const Tensor& x, const Tensor&, const Tensor& dy, const Tensor&,
                                                const Tensor& w, int64_t s, int64_t p, bool bias, int64_t m) {
  return conv2d_wgrad_meta(x, dy, w, s, p, bias, m);
}
std::tuple<Tensor, Tensor> conv_transpose2d_wgrad_xb_meta(const Tensor& x, const Tensor&, const Tensor& dy,
                                                          const Tensor&, const Tensor& w, int64_t s, int64_t p,
                                                          bool bias, int64_t m) {
  return conv_transpose2d_wgrad_meta(x, dy, w, s, p, bias, m);
}

// elementwise / loss / entropy shape kernels
Tensor like_meta1(const Tensor& x) { return at::empty_like(x, at::MemoryFormat::Preserve); }
Tensor nonneg_fwd_meta(const Tensor& p, double, double) { return like_meta1(p); }
Tensor nonneg_bwd_meta(const Tensor& p, const Tensor&, double) { return like_meta1(p); }
std::vector<Tensor> nonneg_multi_fwd_meta(at::TensorList p, at::ArrayRef<double>, at::ArrayRef<double>) {
  std::vector<Tensor> o;
  for (const auto& t : p) o.push_back(like_meta1(t));
  return o;
}
std::vector<Tensor> nonneg_multi_bwd_meta(at::TensorList p, at::TensorList, at::ArrayRef<double>) {
  std::vector<Tensor> o;
  for (const auto& t : p) o.push_back(like_meta1(t));
  return o;
}
Tensor bound_fwd_meta(const Tensor& x, double, bool) { return like_meta1(x); }
Tensor bound_bwd_meta(const Tensor& x, const Tensor&, double, bool) { return like_meta1(x); }
Tensor unary_meta(const Tensor& x) { return like_meta1(x); }
Tensor binary_meta(const Tensor& x, const Tensor&) { return like_meta1(x); }
std::tuple<Tensor, Tensor> exp_clamp_fwd_meta(const Tensor& v, double, double) { return {like_meta1(v), like_meta1(v)}; }
Tensor exp_clamp_bwd_meta(const Tensor& e, const Tensor&, double, double) { return like_meta1(e); }
Tensor scalar_loss_meta1(const Tensor& p) { return at::empty({}, p.options()); }
Tensor scalar_loss_meta2(const Tensor& a, const Tensor&) { return at::empty({}, a.options()); }
Tensor ce_loss_bwd_meta(const Tensor& p, const Tensor&) { return like_meta1(p); }
std::tuple<Tensor, Tensor> pair_grad_meta(const Tensor& a, const Tensor& b, const Tensor&, bool need_a, bool need_b) {
  return {need_a ? like_meta1(a) : at::empty({0}, a.options()), need_b ? like_meta1(b) : at::empty({0}, b.options())};
}
std::tuple<Tensor, Tensor> factorized_fwd_meta(const Tensor& z, int64_t, at::TensorList, int64_t,
                                               const std::optional<Tensor>&, int64_t, int64_t) {
  return {like_meta1(z), like_meta1(z)};
}
std::tuple<Tensor, std::vector<Tensor>> factorized_bwd_meta(const Tensor& q, int64_t, at::TensorList prm,
                                                            const std::optional<Tensor>&, const std::optional<Tensor>&) {
  std::vector<Tensor> g;
  for (const Tensor& t : prm) g.push_back(at::empty_like(t));
  return {like_meta1(q), g};
}
std::tuple<Tensor, Tensor> factorized_net_fwd_meta(const Tensor& z, int64_t, at::IntArrayRef, double, at::TensorList,
                                                   int64_t, const std::optional<Tensor>&, int64_t, int64_t) {
  return {like_meta1(z), like_meta1(z)};
}
std::tuple<Tensor, std::vector<Tensor>> factorized_net_bwd_meta(const Tensor& q, int64_t, at::IntArrayRef, double,
                                                                at::TensorList prm, const std::optional<Tensor>&,
                                                                const std::optional<Tensor>&) {
  std::vector<Tensor> g;
  for (const Tensor& t : prm) g.push_back(at::empty_like(t));
  return {like_meta1(q), g};
}
Tensor quantize_meta(const Tensor& y, int64_t, const std::optional<Tensor>&, int64_t, int64_t, double) {
  return like_meta1(y);
}
std::tuple<Tensor, Tensor> conditional_fwd_meta(const Tensor& y, const Tensor&, const std::optional<Tensor>&, int64_t,
                                                int64_t, const std::optional<Tensor>&, int64_t, int64_t, double) {
  return {like_meta1(y), like_meta1(y)};
}
std::tuple<Tensor, Tensor, Tensor> conditional_bwd_meta(const Tensor& q, const Tensor&, const std::optional<Tensor>& mean,
                                                        int64_t, double, const std::optional<Tensor>&,
                                                        const std::optional<Tensor>&, bool need_y, bool need_scale,
                                                        bool need_mean) {
  const Tensor e = at::empty({0}, q.options());
  need_mean = need_mean && mean.has_value() && mean->defined();
  return {need_y ? like_meta1(q) : e, need_scale ? like_meta1(q) : e, need_mean ? like_meta1(q) : e};
}
void philox_advance_meta(const Tensor&, int64_t) {}
std::tuple<Tensor, Tensor> msssim_fwd_meta(const Tensor& a, const Tensor&, int64_t nlev, int64_t fs, double, double,
                                           bool log_scale, int64_t single, double, double, double, at::ArrayRef<double>) {
  const size_t sb = ic_msssim_state_bytes((int)a.size(0), (int)a.size(1), (int)a.size(2), (int)a.size(3), (int)nlev,
                                          (int)fs);
  TORCH_CHECK(sb > 0, "ms-ssim: image too small for the levels and window");
  return {(single && log_scale) ? at::empty({a.size(0)}, a.options()) : at::empty({}, a.options()),
          at::empty({(int64_t)(sb / 4)}, a.options())};
}
std::tuple<Tensor, Tensor> msssim_bwd_meta(const Tensor& g, const Tensor&, at::IntArrayRef shape, int64_t, int64_t,
                                           double, double, bool, int64_t, double, double, double, at::ArrayRef<double>,
                                           bool need_a, bool need_b) {
  return {need_a ? at::empty(shape, g.options()) : at::empty({0}, g.options()),
          need_b ? at::empty(shape, g.options()) : at::empty({0}, g.options())};
}

}  // namespace

TORCH_LIBRARY(imgcomp, m) {
  m.def("conv2d_fwd(Tensor x, Tensor weight, Tensor? bias, int stride, int padding, int act, int math) -> Tensor");
  m.def("conv2d_fwd_ws(Tensor x, Tensor weight, Tensor? bias, int stride, int padding, int act, int math, "
        "Tensor(a!) ws) -> Tensor");
  m.def("conv2d_dgrad(Tensor dy, Tensor weight, Tensor x, int stride, int padding, int math) -> Tensor");
  m.def("conv2d_wgrad(Tensor x, Tensor dy, Tensor weight, int stride, int padding, bool bias, int math) -> "
        "(Tensor, Tensor)");
  m.def("conv_transpose2d_fwd(Tensor x, Tensor weight, Tensor? bias, int stride, int padding, int output_padding, "
        "int act, int math) -> Tensor");
  m.def("conv_transpose2d_fwd_ws(Tensor x, Tensor weight, Tensor? bias, int stride, int padding, "
        "int output_padding, int act, int math, Tensor(a!) ws) -> Tensor");
  m.def("conv_transpose2d_dgrad(Tensor dy, Tensor weight, Tensor x, int stride, int padding, int math) -> Tensor");
  m.def("conv_transpose2d_wgrad(Tensor x, Tensor dy, Tensor weight, int stride, int padding, bool bias, int math) -> "
        "(Tensor, Tensor)");
  m.def("gdn_fwd(Tensor x, Tensor gamma, Tensor beta, bool inverse, int math) -> (Tensor, Tensor)");
  m.def("gdn_bwd(Tensor x, Tensor norm, Tensor dy, Tensor gamma, bool inverse, int math) -> (Tensor, Tensor, Tensor)");
  m.def("gdn_bwd_sum(Tensor x, Tensor norm, Tensor dy, Tensor gamma, bool inverse, int math) -> "
        "(Tensor, Tensor, Tensor, Tensor)");
  m.def("gdn_fwd_xb(Tensor x, Tensor gamma, Tensor beta, bool inverse, int math) -> (Tensor, Tensor, Tensor)");
  m.def("gdn_bwd_sum_xb(Tensor x, Tensor norm, Tensor dy, Tensor gamma, bool inverse, int math) -> "
        "(Tensor, Tensor, Tensor, Tensor, Tensor)");
  m.def("gdn_fwd_rn(Tensor x, Tensor gamma, Tensor beta, bool inverse, int math, bool xb) -> (Tensor, Tensor)");
  m.def("gdn_bwd_sum_rn(Tensor x, Tensor beta, Tensor dy, Tensor gamma, bool inverse, int math, bool xb) -> "
        "(Tensor, Tensor, Tensor, Tensor, Tensor)");
  m.def("conv2d_fwd_xb(Tensor x, Tensor xb, Tensor weight, Tensor? bias, int stride, int padding, int act, "
        "int math) -> Tensor");
  m.def("conv_transpose2d_dgrad_xb(Tensor dy, Tensor dyb, Tensor weight, Tensor x, int stride, int padding, "
        "int math) -> Tensor");
  m.def("conv2d_dgrad_xb(Tensor dy, Tensor dyb, Tensor weight, Tensor x, int stride, int padding, int math) -> Tensor");
  m.def("conv2d_wgrad_xb(Tensor x, Tensor xb, Tensor dy, Tensor dyb, Tensor weight, int stride, int padding, "
        "bool bias, int math) -> (Tensor, Tensor)");
  m.def("conv_transpose2d_wgrad_xb(Tensor x, Tensor xb, Tensor dy, Tensor dyb, Tensor weight, int stride, "
        "int padding, bool bias, int math) -> (Tensor, Tensor)");
  m.def("conv_transpose2d_fwd_xb(Tensor x, Tensor xb, Tensor weight, Tensor? bias, int stride, int padding, "
        "int output_padding, int act, int math) -> Tensor");
  m.def("nonneg_fwd(Tensor p, float bound, float pedestal) -> Tensor");
  m.def("nonneg_bwd(Tensor p, Tensor grad, float bound) -> Tensor");
  m.def("nonneg_multi_fwd(Tensor[] p, float[] bound, float[] pedestal) -> Tensor[]");
  m.def("nonneg_multi_bwd(Tensor[] p, Tensor[] grad, float[] bound) -> Tensor[]");
  m.def("bound_fwd(Tensor x, float bound, bool upper) -> Tensor");
  m.def("bound_bwd(Tensor x, Tensor grad, float bound, bool upper) -> Tensor");
  m.def("relu_fwd(Tensor x) -> Tensor");
  m.def("relu_bwd(Tensor y, Tensor grad) -> Tensor");
  m.def("abs_fwd(Tensor x) -> Tensor");
  m.def("abs_bwd(Tensor x, Tensor grad) -> Tensor");
  m.def("exp_clamp_fwd(Tensor v, float lo, float hi) -> (Tensor, Tensor)");
  m.def("exp_clamp_bwd(Tensor e, Tensor grad, float lo, float hi) -> Tensor");
  m.def("ce_loss_fwd(Tensor p) -> Tensor");
  m.def("ce_loss_bwd(Tensor p, Tensor grad) -> Tensor");
  m.def("mse_fwd(Tensor input, Tensor target) -> Tensor");
  m.def("mse_bwd(Tensor input, Tensor target, Tensor grad, bool need_input, bool need_target) -> (Tensor, Tensor)");
  m.def("sqdiff_fwd(Tensor input, Tensor target) -> Tensor");
  m.def("sqdiff_bwd(Tensor input, Tensor target, Tensor grad, bool need_input, bool need_target) -> (Tensor, Tensor)");
  m.def("factorized_fwd(Tensor z, int channels, Tensor[] params, int mode, Tensor? u, int seed, int offset) -> "
        "(Tensor, Tensor)");
  m.def("factorized_bwd(Tensor q, int channels, Tensor[] params, Tensor? dq, Tensor? dp) -> (Tensor, Tensor[])");
  m.def("factorized_net_fwd(Tensor z, int channels, int[] dims, float bin, Tensor[] params, int mode, Tensor? u, "
        "int seed, int offset) -> (Tensor, Tensor)");
  m.def("factorized_net_bwd(Tensor q, int channels, int[] dims, float bin, Tensor[] params, Tensor? dq, Tensor? dp) -> "
        "(Tensor, Tensor[])");
  m.def("quantize(Tensor y, int mode, Tensor? u, int seed, int offset, float bin) -> Tensor");
  m.def("conditional_fwd(Tensor y, Tensor scale, Tensor? mean, int kind, int mode, Tensor? u, int seed, int offset, "
        "float bin) -> (Tensor, Tensor)");
  m.def("conditional_bwd(Tensor q, Tensor scale, Tensor? mean, int kind, float bin, Tensor? dq, Tensor? dp, "
        "bool need_y, bool need_scale, bool need_mean) -> (Tensor, Tensor, Tensor)");
  m.def("philox_advance(Tensor(a!) state, int n) -> ()");
  m.def("msssim_fwd(Tensor img1, Tensor img2, int levels, int filter_size, float filter_sigma, float max_val, "
        "bool log_scale, int single, float k1, float k2, float eps, float[] weights) -> (Tensor, Tensor)");
  m.def("msssim_bwd(Tensor grad, Tensor state, int[] shape, int levels, int filter_size, float filter_sigma, "
        "float max_val, bool log_scale, int single, float k1, float k2, float eps, float[] weights, bool need_img1, "
        "bool need_img2) -> (Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(imgcomp, CUDA, m) {  // the CUDA dispatch key is PyTorch-ROCm's HIP device key
  m.impl("conv2d_fwd", conv2d_fwd);
  m.impl("conv2d_fwd_ws", conv2d_fwd_ws);
  m.impl("conv_transpose2d_fwd_ws", conv_transpose2d_fwd_ws);
  m.impl("conv2d_dgrad", conv2d_dgrad);
  m.impl("conv2d_wgrad", conv2d_wgrad);
  m.impl("conv_transpose2d_fwd", conv_transpose2d_fwd);
  m.impl("conv_transpose2d_dgrad", conv_transpose2d_dgrad);
  m.impl("conv_transpose2d_wgrad", conv_transpose2d_wgrad);
  m.impl("gdn_fwd", gdn_fwd);
  m.impl("gdn_bwd", gdn_bwd);
  m.impl("gdn_bwd_sum", gdn_bwd_sum);
  m.impl("gdn_fwd_xb", gdn_fwd_xb);
  m.impl("gdn_bwd_sum_xb", gdn_bwd_sum_xb);
  m.impl("gdn_fwd_rn", gdn_fwd_rn);
  m.impl("gdn_bwd_sum_rn", gdn_bwd_sum_rn);
  m.impl("conv2d_fwd_xb", conv2d_fwd_xb);
  m.impl("conv_transpose2d_dgrad_xb", conv_transpose2d_dgrad_xb);
  m.impl("conv2d_dgrad_xb", conv2d_dgrad_xb);
  m.impl("conv2d_wgrad_xb", conv2d_wgrad_xb);
  m.impl("conv_transpose2d_wgrad_xb", conv_transpose2d_wgrad_xb);
  m.impl("conv_transpose2d_fwd_xb", conv_transpose2d_fwd_xb);
  m.impl("nonneg_fwd", nonneg_fwd);
  m.impl("nonneg_bwd", nonneg_bwd);
  m.impl("nonneg_multi_fwd", nonneg_multi_fwd);
  m.impl("nonneg_multi_bwd", nonneg_multi_bwd);
  m.impl("bound_fwd", bound_fwd);
  m.impl("bound_bwd", bound_bwd);
  m.impl("relu_fwd", relu_fwd);
  m.impl("relu_bwd", relu_bwd);
  m.impl("abs_fwd", abs_fwd);
  m.impl("abs_bwd", abs_bwd);
  m.impl("exp_clamp_fwd", exp_clamp_fwd);
  m.impl("exp_clamp_bwd", exp_clamp_bwd);
  m.impl("ce_loss_fwd", ce_loss_fwd);
  m.impl("ce_loss_bwd", ce_loss_bwd);
  m.impl("mse_fwd", mse_fwd);
  m.impl("mse_bwd", mse_bwd);
  m.impl("sqdiff_fwd", sqdiff_fwd);
  m.impl("sqdiff_bwd", sqdiff_bwd);
  m.impl("factorized_fwd", factorized_fwd);
  m.impl("factorized_bwd", factorized_bwd);
  m.impl("factorized_net_fwd", factorized_net_fwd);
  m.impl("factorized_net_bwd", factorized_net_bwd);
  m.impl("quantize", quantize);
  m.impl("conditional_fwd", conditional_fwd);
  m.impl("conditional_bwd", conditional_bwd);
  m.impl("philox_advance", philox_advance);
  m.impl("msssim_fwd", msssim_fwd);
  m.impl("msssim_bwd", msssim_bwd);
}

TORCH_LIBRARY_IMPL(imgcomp, Meta, m) {
  m.impl("conv2d_fwd", conv2d_fwd_meta);
  m.impl("conv2d_fwd_ws", conv2d_fwd_ws_meta);
  m.impl("conv_transpose2d_fwd_ws", conv_transpose2d_fwd_ws_meta);
  m.impl("conv2d_dgrad", conv2d_dgrad_meta);
  m.impl("conv2d_wgrad", conv2d_wgrad_meta);
  m.impl("conv_transpose2d_fwd", conv_transpose2d_fwd_meta);
  m.impl("conv_transpose2d_dgrad", conv_transpose2d_dgrad_meta);
  m.impl("conv_transpose2d_wgrad", conv_transpose2d_wgrad_meta);
  m.impl("gdn_fwd", gdn_fwd_meta);
  m.impl("gdn_bwd", gdn_bwd_meta);
  m.impl("gdn_bwd_sum", gdn_bwd_sum_meta);
  m.impl("gdn_fwd_xb", gdn_fwd_xb_meta);
  m.impl("gdn_bwd_sum_xb", gdn_bwd_sum_xb_meta);
  m.impl("gdn_fwd_rn", gdn_fwd_rn_meta);
  m.impl("gdn_bwd_sum_rn", gdn_bwd_sum_rn_meta);
  m.impl("conv2d_fwd_xb", conv2d_fwd_xb_meta);
  m.impl("conv_transpose2d_dgrad_xb", conv_transpose2d_dgrad_xb_meta);
  m.impl("conv2d_dgrad_xb", conv2d_dgrad_xb_meta);
  m.impl("conv2d_wgrad_xb", conv2d_wgrad_xb_meta);
  m.impl("conv_transpose2d_wgrad_xb", conv_transpose2d_wgrad_xb_meta);
  m.impl("conv_transpose2d_fwd_xb", conv_transpose2d_fwd_xb_meta);
  m.impl("nonneg_fwd", nonneg_fwd_meta);
  m.impl("nonneg_bwd", nonneg_bwd_meta);
  m.impl("nonneg_multi_fwd", nonneg_multi_fwd_meta);
  m.impl("nonneg_multi_bwd", nonneg_multi_bwd_meta);
  m.impl("bound_fwd", bound_fwd_meta);
  m.impl("bound_bwd", bound_bwd_meta);
  m.impl("relu_fwd", unary_meta);
  m.impl("relu_bwd", binary_meta);
  m.impl("abs_fwd", unary_meta);
  m.impl("abs_bwd", binary_meta);
  m.impl("exp_clamp_fwd", exp_clamp_fwd_meta);
  m.impl("exp_clamp_bwd", exp_clamp_bwd_meta);
  m.impl("ce_loss_fwd", scalar_loss_meta1);
  m.impl("ce_loss_bwd", ce_loss_bwd_meta);
  m.impl("mse_fwd", scalar_loss_meta2);
  m.impl("mse_bwd", pair_grad_meta);
  m.impl("sqdiff_fwd", binary_meta);
  m.impl("sqdiff_bwd", pair_grad_meta);
  m.impl("factorized_fwd", factorized_fwd_meta);
  m.impl("factorized_bwd", factorized_bwd_meta);
  m.impl("factorized_net_fwd", factorized_net_fwd_meta);
  m.impl("factorized_net_bwd", factorized_net_bwd_meta);
  m.impl("quantize", quantize_meta);
  m.impl("conditional_fwd", conditional_fwd_meta);
  m.impl("conditional_bwd", conditional_bwd_meta);
  m.impl("philox_advance", philox_advance_meta);
  m.impl("msssim_fwd", msssim_fwd_meta);
  m.impl("msssim_bwd", msssim_bwd_meta);
}
