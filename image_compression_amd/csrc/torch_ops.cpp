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

// ---------------------------------------------------------------- shape (Meta) kernels
Tensor conv2d_fwd_meta(const Tensor& x, const Tensor& w, const c10::optional<Tensor>&, int64_t stride, int64_t pad,
                       int64_t, int64_t) {
  const int64_t k = w.size(2);
  return at::empty({x.size(0), w.size(0), (x.size(2) + 2 * pad - k) / stride + 1, (x.size(3) + 2 * pad - k) / stride + 1},
                   x.options().memory_format(act_format(w.size(0))));
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

}  // namespace

TORCH_LIBRARY(imgcomp, m) {
  m.def("conv2d_fwd(Tensor x, Tensor weight, Tensor? bias, int stride, int padding, int act, int math) -> Tensor");
  m.def("conv2d_dgrad(Tensor dy, Tensor weight, Tensor x, int stride, int padding, int math) -> Tensor");
  m.def("conv2d_wgrad(Tensor x, Tensor dy, Tensor weight, int stride, int padding, bool bias, int math) -> "
        "(Tensor, Tensor)");
  m.def("conv_transpose2d_fwd(Tensor x, Tensor weight, Tensor? bias, int stride, int padding, int output_padding, "
        "int act, int math) -> Tensor");
  m.def("conv_transpose2d_dgrad(Tensor dy, Tensor weight, Tensor x, int stride, int padding, int math) -> Tensor");
  m.def("conv_transpose2d_wgrad(Tensor x, Tensor dy, Tensor weight, int stride, int padding, bool bias, int math) -> "
        "(Tensor, Tensor)");
  m.def("gdn_fwd(Tensor x, Tensor gamma, Tensor beta, bool inverse, int math) -> (Tensor, Tensor)");
  m.def("gdn_bwd(Tensor x, Tensor norm, Tensor dy, Tensor gamma, bool inverse, int math) -> (Tensor, Tensor, Tensor)");
  m.def("gdn_bwd_sum(Tensor x, Tensor norm, Tensor dy, Tensor gamma, bool inverse, int math) -> "
        "(Tensor, Tensor, Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(imgcomp, CUDA, m) {  // the CUDA dispatch key is PyTorch-ROCm's HIP device key
  m.impl("conv2d_fwd", conv2d_fwd);
  m.impl("conv2d_dgrad", conv2d_dgrad);
  m.impl("conv2d_wgrad", conv2d_wgrad);
  m.impl("conv_transpose2d_fwd", conv_transpose2d_fwd);
  m.impl("conv_transpose2d_dgrad", conv_transpose2d_dgrad);
  m.impl("conv_transpose2d_wgrad", conv_transpose2d_wgrad);
  m.impl("gdn_fwd", gdn_fwd);
  m.impl("gdn_bwd", gdn_bwd);
  m.impl("gdn_bwd_sum", gdn_bwd_sum);
}

TORCH_LIBRARY_IMPL(imgcomp, Meta, m) {
  m.impl("conv2d_fwd", conv2d_fwd_meta);
  m.impl("conv2d_dgrad", conv2d_dgrad_meta);
  m.impl("conv2d_wgrad", conv2d_wgrad_meta);
  m.impl("conv_transpose2d_fwd", conv_transpose2d_fwd_meta);
  m.impl("conv_transpose2d_dgrad", conv_transpose2d_dgrad_meta);
  m.impl("conv_transpose2d_wgrad", conv_transpose2d_wgrad_meta);
  m.impl("gdn_fwd", gdn_fwd_meta);
  m.impl("gdn_bwd", gdn_bwd_meta);
  m.impl("gdn_bwd_sum", gdn_bwd_sum_meta);
}
