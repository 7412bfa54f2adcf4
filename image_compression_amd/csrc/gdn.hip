// GDN / IGDN (modelling/layers/gdn.py:79-88) on the implicit-GEMM kernel.
//
// forward : norm = beta + Gamma * x^2     (1x1 GEMM, x^2 formed in the A-load)
//           y = x / sqrt(norm)            (fused epilogue, norm saved)
// backward: q   = dL/dnorm = -0.5 dy x norm^-3/2   (IGDN: +0.5 dy x norm^-1/2)
//           dx  = dy / sqrt(norm) + 2 x (q Gamma)  (1x1 GEMM with Gamma^T, fused epilogue)
//           dGamma = q^T x^2  (wgrad kernel, x^2 in the load), dbeta = colsum(q)
#include "../../include/imgcomp.h"
#include "gemm.h"

namespace {

__global__ void gdn_q_kernel(const float* x, const float* nrm, const float* dy, long long n,
                             int inverse, float* q) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const float s = sqrtf(nrm[i]);
    q[i] = inverse ? 0.5f * dy[i] * x[i] / s : -0.5f * dy[i] * x[i] / (nrm[i] * s);
  }
}

long long act_numel(const ic_act* a) { return (long long)a->n * a->c * a->h * a->w; }

bool dense_like(const ic_act* a) {
  // storage must be non-overlapping and dense (any dim order)
  long long st[4] = {a->sn, a->sc, a->sh, a->sw};
  long long sz[4] = {a->n, a->c, a->h, a->w};
  // simple check: max offset + 1 == numel and all strides positive
  long long mx = 0;
  for (int i = 0; i < 4; ++i) {
    if (st[i] <= 0 && sz[i] > 1) return false;
    mx += (sz[i] - 1) * st[i];
  }
  return mx + 1 == act_numel(a);
}

struct Carve {
  char* base;
  size_t off;
  float* take(size_t bytes) {
    float* p = (float*)(base + off);
    off += ic_align(bytes, 256);
    return p;
  }
};

void gemm1x1(IgDesc& d, const ic_act* x, const ic_act* y) {
  d.x = x->data; d.xs_n = x->sn; d.xs_h = x->sh; d.xs_w = x->sw; d.xs_c = x->sc;
  d.Hx = x->h; d.Wx = x->w; d.Cin = x->c; d.N = x->n; d.stride = 1;
  d.y = y->data; d.ys_n = y->sn; d.ys_h = y->sh; d.ys_w = y->sw; d.ys_c = y->sc; d.Cout = y->c;
  d.generic = (x->c % 32 != 0) || (x->sc != 1);
  d.nphase = 1;
  IgPhase& P = d.ph[0];
  P.T = 1; P.dy[0] = 0; P.dx[0] = 0;
  P.Hg = y->h; P.Wg = y->w; P.oys = 1; P.oxs = 1; P.oy0 = 0; P.ox0 = 0;
  d.Kc = d.generic ? (int)ic_align((size_t)x->c, 32) : x->c;
}

// y (and x) compact NHWC: the layout of the bf16 copies (ic_gdn_fwd_xb / ic_gdn_bwd_sum_xb)
static bool compact_nhwc(const ic_act* a) {
  return a->sc == 1 && a->sw == a->c && a->sh == (long long)a->w * a->c && a->sn == (long long)a->h * a->w * a->c &&
         a->c % 8 == 0;
}

// yb (non-null): y's compact NHWC bf16 copy as well -- written by the fused bf16 kernel's epilogue, or
// converted after any other path
int gdn_fwd_impl(const ic_act* x, const float* gamma, const float* beta, int inverse,
                 const ic_act* y, float* norm, void* ws, size_t wsb, hipStream_t s, size_t* need, int math = 0,
                 void* yb = nullptr) {
  const long long P = (long long)x->n * x->h * x->w;
  if (yb && !need && !compact_nhwc(y)) return IC_ERR_ARG;
  // split arithmetic: the fused split kernel (C = 192), else the implicit GEMM
  // (1x1, x^2 squared in the staging, GDN epilogue)
  const bool split = (math & IC_MATH_SPLIT) && x->c % 32 == 0 && x->sc == 1 && x->c >= 64;
  // the workspace query answers for the general path (the fused one needs none)
  if (!need && (!split || x->c == 192) && gdn_fused_ok(x->data, y->data, norm, x->c, x->sc, x->sw, x->sh, x->sn, x->h, x->w, P) &&
      x->sn == y->sn && x->sc == y->sc && x->sh == y->sh && x->sw == y->sw &&
      ((uintptr_t)gamma & 15) == 0) {
    const int mode = (math & IC_MATH_BF16) && split && x->c == 192 ? 2 : split ? 1 : 0;
    if (!norm && mode != 2) return IC_ERR_ARG;  // norm left out: the bf16 kernel only (ic_gdn_fwd_rn)
    int rc = gdn_fwd_fused(x->data, gamma, beta, inverse, y->data, norm, x->c, P, s, mode, mode == 2 ? yb : nullptr);
    if (rc || !yb || mode == 2) return rc;
    return ig_cvt_bf16(y->data, yb, act_numel(y), s);
  }
  if (!need && !norm) return IC_ERR_ARG;
  IgDesc d = {};
  gemm1x1(d, x, y);
  d.bias = beta;
  d.epi = inverse ? EPI_IGDN : EPI_GDN;
  d.a_op = AOP_SQUARE;
  d.aux0 = x->data;
  d.aux_out = norm;
  d.x3 = split ? 1 : 0;
  const size_t part = ig_plan(d);
  const size_t wpb = (size_t)d.Npad * d.Kc * (d.x3 ? 6 : 4);
  d.wplane = (long long)d.Npad * d.Kc;
  const size_t tot = ic_align(wpb, 256) + ic_align(part, 256);
  if (need) { *need = tot; return IC_OK; }
  if (x->sn != y->sn || x->sc != y->sc || x->sh != y->sh || x->sw != y->sw) return IC_ERR_ARG;
  if (wsb < tot) return IC_ERR_WORKSPACE;
  Carve cv{(char*)ws, 0};
  float* wp = cv.take(wpb);
  d.partial = part ? cv.take(part) : nullptr;
  d.ph[0].wp = wp;
  const int z = 0;
  int rc = pack_weights(gamma, x->c, x->c, 1, 0, d.generic, 1, &z, &z, d.Npad, d.Kc, wp, s, d.x3 ? 2 : 0);
  if (rc) return rc;
  rc = ig_run(d, s);
  if (rc || !yb) return rc;
  return ig_cvt_bf16(y->data, yb, act_numel(y), s);
}

int gdn_bwd_impl(const ic_act* x, const float* norm, const float* dy, const float* gamma, int inverse,
                 const ic_act* dx, float* dgamma, float* dbeta, void* ws, size_t wsb, hipStream_t s,
                 size_t* need, int math = 0, float* dxsum = nullptr, void* dxb = nullptr, const float* beta = nullptr);

// dxb: dx's compact NHWC bf16 copy as well (the fused bf16 kernel writes it; any other path converts)
int gdn_bwd_impl_xb(const ic_act* x, const float* norm, const float* dy, const float* gamma, int inverse,
                    const ic_act* dx, float* dgamma, float* dbeta, void* ws, size_t wsb, hipStream_t s, int math,
                    float* dxsum, void* dxb) {
  if (!compact_nhwc(dx)) return IC_ERR_ARG;
  return gdn_bwd_impl(x, norm, dy, gamma, inverse, dx, dgamma, dbeta, ws, wsb, s, nullptr, math, dxsum, dxb);
}

int gdn_bwd_impl(const ic_act* x, const float* norm, const float* dy, const float* gamma, int inverse,
                 const ic_act* dx, float* dgamma, float* dbeta, void* ws, size_t wsb, hipStream_t s,
                 size_t* need, int math, float* dxsum, void* dxb, const float* beta) {
  const long long n = act_numel(x);
  const long long P = (long long)x->n * x->h * x->w;
  // fused path: x, dx, norm, dy all NHWC-dense with x's strides; its workspace
  // (per-block dgamma partials) is also reserved by the query below
  const size_t fused_ws = gdn_bwd_fused_ws(x->c, P);
  if (!need && gdn_fused_ok(x->data, dx->data, norm, x->c, x->sc, x->sw, x->sh, x->sn, x->h, x->w, P) &&
      ((uintptr_t)dy & 15) == 0 && x->sn == dx->sn && x->sc == dx->sc && x->sh == dx->sh && x->sw == dx->sw &&
      wsb >= fused_ws) {
    const int mode = (math & IC_MATH_BF16) && x->c == 192 ? 2 : (math & IC_MATH_SPLIT) ? 1 : 0;
    if (!norm && mode != 2) return IC_ERR_ARG;  // norm recomputed: the bf16 kernel only (ic_gdn_bwd_sum_rn)
    int rc = gdn_bwd_fused(x->data, norm, dy, gamma, inverse, dx->data, dgamma, dbeta, x->c, P, ws, s, mode, dxsum,
                           mode == 2 ? dxb : nullptr, beta);
    if (rc || !dxb || mode == 2) return rc;
    return ig_cvt_bf16(dx->data, dxb, act_numel(dx), s);
  }
  if (!need && !norm) return IC_ERR_ARG;  // norm recomputed: the fused bf16 kernel only
  if (dxb && !need) {  // the general path, then the copy
    int rc = gdn_bwd_impl(x, norm, dy, gamma, inverse, dx, dgamma, dbeta, ws, wsb, s, nullptr, math, dxsum, nullptr);
    if (rc) return rc;
    return ig_cvt_bf16(dx->data, dxb, act_numel(dx), s);
  }
  // q has x's layout
  ic_act qa = *x;
  IgDesc d = {};
  gemm1x1(d, &qa, dx);
  d.epi = inverse ? EPI_IGDN_BWD : EPI_GDN_BWD;
  d.aux0 = x->data; d.aux1 = norm; d.aux2 = dy;
  const size_t part = ig_plan(d);
  const size_t wpb = (size_t)d.Npad * d.Kc * 4;
  WgDesc w = {};
  w.g = nullptr; w.gs_n = x->sn; w.gs_h = x->sh; w.gs_w = x->sw; w.gs_c = x->sc;
  w.Hg = x->h; w.Wg = x->w; w.Cg = x->c;
  w.x = x->data; w.xs_n = x->sn; w.xs_h = x->sh; w.xs_w = x->sw; w.xs_c = x->sc;
  w.Hx = x->h; w.Wx = x->w; w.Cx = x->c;
  w.N = x->n; w.stride = 1; w.T = 1; w.dy[0] = 0; w.dx[0] = 0; w.x_op = AOP_SQUARE;
  w.generic = (x->c % 4 != 0) || (x->sc != 1);
  const size_t wpart = wg_plan(w);
  const size_t cs = colsum_ws((long long)x->n * x->h * x->w, x->c);
  const size_t tot = ic_align((size_t)n * 4, 256) + ic_align(wpb, 256) + ic_align(part, 256) +
                     ic_align(wpart, 256) + ic_align(cs, 256);
  if (need) { *need = tot > fused_ws ? tot : fused_ws; return IC_OK; }
  if (!dense_like(x)) return IC_ERR_ARG;
  if (x->sn != dx->sn || x->sc != dx->sc || x->sh != dx->sh || x->sw != dx->sw) return IC_ERR_ARG;
  if (wsb < tot) return IC_ERR_WORKSPACE;
  Carve cv{(char*)ws, 0};
  float* q = cv.take((size_t)n * 4);
  float* wp = cv.take(wpb);
  d.partial = part ? cv.take(part) : nullptr;
  w.partial = cv.take(wpart);
  float* csw = cv.take(cs);
  long long blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(gdn_q_kernel, dim3((unsigned)blocks), dim3(256), 0, s, x->data, norm, dy, n,
                     inverse, q);
  IC_CHECK_LAUNCH();
  // dx = f(dy, x, norm) + 2 x * (q Gamma): B^T[n=ci][k=co] = Gamma[co][ci] -> transposed pack
  d.x = q;
  d.ph[0].wp = wp;
  const int z = 0;
  int rc = pack_weights(gamma, x->c, x->c, 1, 1, d.generic, 1, &z, &z, d.Npad, d.Kc, wp, s);
  if (rc) return rc;
  rc = ig_run(d, s);
  if (rc) return rc;
  if (dgamma) {
    w.g = q;
    rc = wg_run(w, s);
    if (rc) return rc;
    const int kk0 = 0;
    rc = wg_reduce(w, dgamma, &kk0, 1, s);
    if (rc) return rc;
  }
  if (dbeta) {
    rc = colsum(q, x->sn, x->sc, x->sh, x->sw, x->n, x->c, x->h, x->w, dbeta, 1.f, csw, s);
    if (rc) return rc;
  }
  if (dxsum) {
    rc = colsum(dx->data, dx->sn, dx->sc, dx->sh, dx->sw, dx->n, dx->c, dx->h, dx->w, dxsum, 1.f, csw, s);
    if (rc) return rc;
  }
  return IC_OK;
}

}  // namespace

// ic_conv_plan(IC_OP_GDN_*): the dispatch conditions of gdn_fwd_impl / gdn_bwd_impl
int gdn_plan(int bwd, const ic_act* x, int math) {
  if (!act_fits32(x)) return IC_ERR_ARG;
  const long long P = (long long)x->n * x->h * x->w;
  const bool fused = gdn_fused_ok(x->data, x->data, x->data, x->c, x->sc, x->sw, x->sh, x->sn, x->h, x->w, P);
  const bool split = (math & IC_MATH_SPLIT) != 0;
  if (!bwd) {
    const bool fsplit = split && x->c % 32 == 0 && x->sc == 1 && x->c >= 64;
    if ((!fsplit || x->c == 192) && fused) {
      plan_report(fsplit && (math & IC_MATH_BF16) ? IC_KERNEL_GDN_FUSED_BF16
                  : fsplit                         ? IC_KERNEL_GDN_FUSED_SPLIT
                                                   : IC_KERNEL_GDN_FUSED,
                  fsplit ? 32 : 16, x->c, 1, 0, 0, -1);
      return IC_OK;
    }
  } else if (fused) {
    plan_report((math & IC_MATH_BF16) && x->c == 192 ? IC_KERNEL_GDN_FUSED_BF16
                : split && x->c == 192                  ? IC_KERNEL_GDN_FUSED_SPLIT
                                                        : IC_KERNEL_GDN_FUSED,
                16, x->c, 1, 0, 0, -1);
    return IC_OK;
  }
  size_t n = 0;
  ic_plan* sink = g_plan_sink;
  g_plan_sink = nullptr;
  const int rc = bwd ? gdn_bwd_impl(x, nullptr, nullptr, nullptr, 0, x, nullptr, nullptr, nullptr, 0, 0, &n, math)
                     : gdn_fwd_impl(x, nullptr, nullptr, 0, x, nullptr, nullptr, 0, 0, &n, math);
  g_plan_sink = sink;
  if (rc) return rc;
  plan_report(IC_KERNEL_GDN_GEMM, 0, x->c, 1, 0, 0, -1);
  return IC_OK;
}

extern "C" {

size_t ic_gdn_fwd_ws(const ic_act* x) {
  size_t n = 0;
  gdn_fwd_impl(x, nullptr, nullptr, 0, x, nullptr, nullptr, 0, 0, &n);
  return n;
}
int ic_gdn_fwd(const ic_act* x, const float* gamma, const float* beta, int inverse, const ic_act* y,
               float* norm, void* ws, size_t ws_bytes, void* stream) {
  return gdn_fwd_impl(x, gamma, beta, inverse, y, norm, ws, ws_bytes, (hipStream_t)stream, nullptr);
}
size_t ic_gdn_bwd_ws(const ic_act* x) {
  size_t n = 0;
  gdn_bwd_impl(x, nullptr, nullptr, nullptr, 0, x, nullptr, nullptr, nullptr, 0, 0, &n);
  return n;
}
int ic_gdn_bwd(const ic_act* x, const float* norm, const float* dy, const float* gamma, int inverse,
               const ic_act* dx, float* dgamma, float* dbeta, void* ws, size_t ws_bytes,
               void* stream) {
  return gdn_bwd_impl(x, norm, dy, gamma, inverse, dx, dgamma, dbeta, ws, ws_bytes,
                      (hipStream_t)stream, nullptr);
}

int ic_gdn_fwd_ex(const ic_act* x, const float* gamma, const float* beta, int inverse, const ic_act* y, float* norm,
                  int math, void* ws, size_t ws_bytes, void* stream) {
  return gdn_fwd_impl(x, gamma, beta, inverse, y, norm, ws, ws_bytes, (hipStream_t)stream, nullptr, math);
}
size_t ic_gdn_fwd_ws_ex(const ic_act* x, int math) {
  size_t n = 0;
  gdn_fwd_impl(x, nullptr, nullptr, 0, x, nullptr, nullptr, 0, 0, &n, math);
  return n;
}
int ic_gdn_bwd_ex(const ic_act* x, const float* norm, const float* dy, const float* gamma, int inverse,
                  const ic_act* dx, float* dgamma, float* dbeta, int math, void* ws, size_t ws_bytes, void* stream) {
  return gdn_bwd_impl(x, norm, dy, gamma, inverse, dx, dgamma, dbeta, ws, ws_bytes, (hipStream_t)stream, nullptr,
                      math);
}
int ic_gdn_bwd_sum_ex(const ic_act* x, const float* norm, const float* dy, const float* gamma, int inverse,
                      const ic_act* dx, float* dgamma, float* dbeta, float* dxsum, int math, void* ws,
                      size_t ws_bytes, void* stream) {
  return gdn_bwd_impl(x, norm, dy, gamma, inverse, dx, dgamma, dbeta, ws, ws_bytes, (hipStream_t)stream, nullptr,
                      math, dxsum);
}
int ic_gdn_fwd_xb(const ic_act* x, const float* gamma, const float* beta, int inverse, const ic_act* y, float* norm,
                  void* yb, int math, void* ws, size_t ws_bytes, void* stream) {
  if (!yb) return IC_ERR_ARG;
  return gdn_fwd_impl(x, gamma, beta, inverse, y, norm, ws, ws_bytes, (hipStream_t)stream, nullptr, math, yb);
}
int ic_gdn_bwd_sum_xb(const ic_act* x, const float* norm, const float* dy, const float* gamma, int inverse,
                      const ic_act* dx, float* dgamma, float* dbeta, float* dxsum, void* dxb, int math, void* ws,
                      size_t ws_bytes, void* stream) {
  if (!dxb) return IC_ERR_ARG;
  return gdn_bwd_impl_xb(x, norm, dy, gamma, inverse, dx, dgamma, dbeta, ws, ws_bytes, (hipStream_t)stream, math,
                         dxsum, dxb);
}

int ic_gdn_fwd_rn(const ic_act* x, const float* gamma, const float* beta, int inverse, const ic_act* y, void* yb,
                  int math, void* ws, size_t ws_bytes, void* stream) {
  if (yb && !compact_nhwc(y)) return IC_ERR_ARG;
  return gdn_fwd_impl(x, gamma, beta, inverse, y, nullptr, ws, ws_bytes, (hipStream_t)stream, nullptr, math, yb);
}
int ic_gdn_bwd_sum_rn(const ic_act* x, const float* beta, const float* dy, const float* gamma, int inverse,
                      const ic_act* dx, float* dgamma, float* dbeta, float* dxsum, void* dxb, int math, void* ws,
                      size_t ws_bytes, void* stream) {
  if (!beta || (dxb && !compact_nhwc(dx))) return IC_ERR_ARG;
  return gdn_bwd_impl(x, nullptr, dy, gamma, inverse, dx, dgamma, dbeta, ws, ws_bytes, (hipStream_t)stream, nullptr,
                      math, dxsum, dxb, beta);
}

}  // extern "C"
