// C-ABI convolution entry points (conv2d / conv_transpose2d: fwd, dgrad, wgrad)
// built on the two gather-GEMM kernel families of igemm.hip / wgrad.hip.
//
//   conv fwd       = "direct"     gather (stride s, taps dy = ky - pad)
//   conv dgrad     = "transposed" gather (s*s sub-pixel phases)
//   tconv fwd      = "transposed" gather (+bias, +act)
//   tconv dgrad    = "direct"     gather
//   conv wgrad     = wgrad(G = dy, X = x)
//   tconv wgrad    = wgrad(G = x,  X = dy)   (same index relation)
#include "../../include/imgcomp.h"
#include "gemm.h"

#ifndef EDGE_BF16
#define EDGE_BF16 1  // C3 (IC_MATH_BF16): the 3-channel image edges on bf16 operands too; 0: split arithmetic
#endif
#ifndef TAP_PARITY_ORDER
#define TAP_PARITY_ORDER 1  // stride-2 direct convs walk even kernel rows first, then odd (conv_impl); 0: row order
#endif

thread_local ic_plan* g_plan_sink = nullptr;

namespace {

struct Carve {
  char* base;
  size_t off;
  float* take(size_t bytes) {
    float* p = (float*)(base + off);
    off += ic_align(bytes, 256);
    return p;
  }
};

void set_x(IgDesc& d, const ic_act* x) {
  d.x = x->data; d.xs_n = x->sn; d.xs_h = x->sh; d.xs_w = x->sw; d.xs_c = x->sc;
  d.Hx = x->h; d.Wx = x->w; d.Cin = x->c; d.N = x->n;
}
void set_y(IgDesc& d, const ic_act* y) {
  d.y = y->data; d.ys_n = y->sn; d.ys_h = y->sh; d.ys_w = y->sw; d.ys_c = y->sc; d.Cout = y->c;
}


constexpr int FEW_CH = 8;  // image-edge layers (3 channels) go through im2col / col2im

// few input channels: xcol = im2col(x) (K = k*k*C padded to 32), then one 1x1 GEMM
int direct_im2col(const ic_act* x, const float* W, const float* bias, int k, int stride, int pad,
                  const ic_act* y, int epi, void* ws, size_t wsb, hipStream_t s, size_t* need, int math = 0) {
  const int T = k * k;
  const int Kp = (int)ic_align((size_t)T * x->c, 32);
  if ((epi == EPI_NONE || epi == EPI_RELU) && edge_conv_ok(x->c, k, stride, x->sw, y->sc, y->c, y->sw, y->sh, y->sn)) {
    // patch-gather kernel (edge.hip): no im2col columns in HBM
    const int Npad = ig_npad(y->c);
    const size_t wpb = (size_t)Npad * Kp * 4;
    // 2: bf16 operands (C3), 1: split arithmetic, 0: fp32 MFMA
    const int split = (EDGE_BF16 && (math & IC_MATH_BF16)) ? 2 : (math & IC_MATH_SPLIT) ? 1 : 0;
    if (need) {
      // edge_conv_x3_kernel (variant 1) in split arithmetic or with bf16 operands
      const bool x3 = edge_conv_split(split, T * x->c, y->c);
      plan_report(x3 && split == 2 ? IC_KERNEL_EDGE_CONV_BF16 : IC_KERNEL_EDGE_CONV, 64, y->c, 1, 0, 0, -1, x3 ? 1 : 0);
      *need = ic_align(wpb, 256);
      return IC_OK;
    }
    if (wsb < wpb) return IC_ERR_WORKSPACE;
    float* wp = (float*)ws;
    int ky[IC_MAXT], kx[IC_MAXT];
    for (int t = 0; t < T; ++t) { ky[t] = t / k; kx[t] = t % k; }
    if (!(math & IC_MATH_WPACKED)) {
      int rc = pack_weights(W, y->c, x->c, k, 0, 1, T, ky, kx, Npad, Kp, wp, s);
      if (rc) return rc;
    }
    return edge_conv_run(x->data, x->sn, x->sc, x->sh, x->sw, x->n, x->c, x->h, x->w, wp, Kp, bias, k, stride, pad,
                         y->data, y->sn, y->sc, y->sh, y->sw, y->c, y->h, y->w, epi == EPI_RELU, s, split);
  }
  const long long rows = (long long)x->n * y->h * y->w;
  ic_act xc;
  xc.data = nullptr; xc.n = x->n; xc.c = Kp; xc.h = y->h; xc.w = y->w;
  xc.sn = (long long)y->h * y->w * Kp; xc.sc = 1; xc.sh = (long long)y->w * Kp; xc.sw = Kp;
  IgDesc d = {};
  set_x(d, &xc);
  set_y(d, y);
  d.stride = 1; d.generic = 0; d.bias = bias; d.epi = epi; d.a_op = AOP_NONE;
  d.nphase = 1;
  IgPhase& P = d.ph[0];
  P.T = 1; P.dy[0] = 0; P.dx[0] = 0;
  P.Hg = y->h; P.Wg = y->w; P.oys = 1; P.oxs = 1; P.oy0 = 0; P.ox0 = 0;
  d.Kc = Kp;
  const size_t part = ig_plan(d);
  const size_t xcb = (size_t)rows * Kp * 4;
  const size_t wpb = (size_t)d.Npad * Kp * 4;
  const size_t tot = ic_align(xcb, 256) + ic_align(wpb, 256) + ic_align(part, 256);
  if (need) {
    plan_report(IC_KERNEL_IM2COL_GEMM, d.bm, d.bn, d.ksplit, 0, 1, ig_grid_blocks(d));
    *need = tot;
    return IC_OK;
  }
  if (wsb < tot) return IC_ERR_WORKSPACE;
  Carve cv{(char*)ws, 0};
  float* xcol = cv.take(xcb);
  float* wp = cv.take(wpb);
  d.partial = part ? cv.take(part) : nullptr;
  d.x = xcol;
  P.wp = wp;
  int ky[IC_MAXT], kx[IC_MAXT];
  for (int t = 0; t < T; ++t) { ky[t] = t / k; kx[t] = t % k; }
  int rc = im2col_run(x->data, x->sn, x->sc, x->sh, x->sw, x->n, x->c, x->h, x->w, y->h, y->w, stride, k, pad,
                      Kp, xcol, s);
  if (rc) return rc;
  rc = pack_weights(W, y->c, x->c, k, 0, 1, T, ky, kx, d.Npad, Kp, wp, s);
  if (rc) return rc;
  return ig_run(d, s);
}

// few output channels of a transposed conv: ycol[p][(t,b)] = x[p] . W[:, b, t] (one 1x1 GEMM
// with N = k*k*B) then the deterministic sub-pixel gather col2im (+bias, act)
int transposed_col2im(const ic_act* x, const float* W, const float* bias, int k, int stride, int pad,
                      const ic_act* y, int epi, void* ws, size_t wsb, hipStream_t s, size_t* need) {
  if (epi != EPI_NONE && epi != EPI_RELU) return IC_ERR_ARG;
  const int T = k * k;
  const int ncol = T * y->c;
  const long long rows = (long long)x->n * x->h * x->w;
  ic_act yc;
  yc.data = nullptr; yc.n = x->n; yc.c = ncol; yc.h = x->h; yc.w = x->w;
  yc.sn = (long long)x->h * x->w * ncol; yc.sc = 1; yc.sh = (long long)x->w * ncol; yc.sw = ncol;
  IgDesc d = {};
  set_x(d, x);
  set_y(d, &yc);
  d.stride = 1;
  d.generic = (x->c % 32 != 0) || (x->sc != 1);
  d.bias = nullptr; d.epi = EPI_NONE; d.a_op = AOP_NONE;
  d.nphase = 1;
  IgPhase& P = d.ph[0];
  P.T = 1; P.dy[0] = 0; P.dx[0] = 0;
  P.Hg = x->h; P.Wg = x->w; P.oys = 1; P.oxs = 1; P.oy0 = 0; P.ox0 = 0;
  d.Kc = d.generic ? (int)ic_align((size_t)x->c, 32) : x->c;
  const size_t part = ig_plan(d);
  const size_t ycb = (size_t)rows * ncol * 4;
  const size_t wpb = (size_t)d.Npad * d.Kc * 4;
  const size_t tot = ic_align(ycb, 256) + ic_align(wpb, 256) + ic_align(part, 256);
  if (need) {
    plan_report(IC_KERNEL_GEMM_COL2IM, d.bm, d.bn, d.ksplit, 0, 1, ig_grid_blocks(d));
    *need = tot;
    return IC_OK;
  }
  if (wsb < tot) return IC_ERR_WORKSPACE;
  Carve cv{(char*)ws, 0};
  float* ycol = cv.take(ycb);
  float* wp = cv.take(wpb);
  d.partial = part ? cv.take(part) : nullptr;
  d.y = ycol;
  P.wp = wp;
  int ky[IC_MAXT], kx[IC_MAXT];
  for (int t = 0; t < T; ++t) { ky[t] = t / k; kx[t] = t % k; }
  if (d.generic) return IC_ERR_ARG;  // A (input channels) is wide on every caller
  int rc = pack_weights(W, x->c, y->c, k, 2, 0, T, ky, kx, d.Npad, d.Kc, wp, s);
  if (rc) return rc;
  rc = ig_run(d, s);
  if (rc) return rc;
  return col2im_run(ycol, ncol, x->n, x->h, x->w, bias, y->data, y->sn, y->sc, y->sh, y->sw, y->c, y->h, y->w, k,
                    stride, pad, epi == EPI_RELU, s);
}

// y[a] = sum_{t,b} x[b] @ (gy*s + ky - pad) * W[a][b][ky][kx]   (W: [A=y->c][B=x->c][k][k])
// xb (IC_MATH_XB in math): x's compact NHWC bf16 copy, made by its producer (ic_gdn_fwd_xb /
// ic_gdn_bwd_sum_xb): the bf16 DMA tiles read it instead of converting x into the workspace (and the
// workspace query leaves that space out)
int direct_impl(const ic_act* x, const float* W, const float* bias, int k, int stride, int pad,
                const ic_act* y, int epi, int aop, const float* aux0, const float* aux1,
                const float* aux2, float* aux_out, void* ws, size_t wsb, hipStream_t s, size_t* need,
                int math = 0, const void* xb = nullptr) {
  const bool have_xb = (math & IC_MATH_XB) != 0;
  math &= ~IC_MATH_XB;
  if (have_xb && !need && !xb) return IC_ERR_ARG;
  if (k < 1 || k * k > IC_MAXT || stride < 1) return IC_ERR_ARG;
  if (x->n != y->n) return IC_ERR_ARG;
  if (!act_fits32(x) || !act_fits32(y)) return IC_ERR_ARG;  // 32-bit element offsets in the kernels
  if ((x->h + 2 * pad - k) / stride + 1 != y->h || (x->w + 2 * pad - k) / stride + 1 != y->w)
    return IC_ERR_ARG;
  if (x->c <= FEW_CH && aop == AOP_NONE)
    return direct_im2col(x, W, bias, k, stride, pad, y, epi, ws, wsb, s, need, math);
  IgDesc d = {};
  set_x(d, x);
  set_y(d, y);
  d.stride = stride;
  d.generic = (x->c % 32 != 0) || (x->sc != 1);
  d.bias = bias; d.epi = epi; d.a_op = aop;
  d.aux0 = aux0; d.aux1 = aux1; d.aux2 = aux2; d.aux_out = aux_out;
  d.nphase = 1;
  IgPhase& P = d.ph[0];
  P.T = k * k;
  int ky[IC_MAXT], kx[IC_MAXT];
  for (int t = 0; t < P.T; ++t) {
    // TAP_PARITY_ORDER: kernel rows 0, 2, 4, 1, 3 (k = 5).  Tap row ky reads input rows 2y + ky - pad,
    // so even and odd kernel rows read disjoint rows: taken parity by parity, the input rows a
    // channel chunk's taps read stay in the XCD's L2 across those taps.  r05e, PMC FETCH per g_a.2
    // fwd launch: ig_kernel_x3d 0.86 -> 0.58 GB, ig_kernel_bf16 1.65 -> 1.09 GB; time equal / -2.5 %
    const int r = t / k, ne = (k + 1) / 2;
    ky[t] = (stride == 2 && TAP_PARITY_ORDER) ? (r < ne ? 2 * r : 2 * (r - ne) + 1) : r;
    kx[t] = t % k;
    P.dy[t] = ky[t] - pad; P.dx[t] = kx[t] - pad;
  }
  P.Hg = y->h; P.Wg = y->w; P.oys = 1; P.oxs = 1; P.oy0 = 0; P.ox0 = 0;
  d.Kc = d.generic ? (int)ic_align((size_t)P.T * x->c, 32) : x->c;
  d.bf16 = (math & IC_MATH_BF16) && !d.generic && x->c % 64 == 0 && aop == AOP_NONE;
  d.x3 = (math & IC_MATH_SPLIT) && !d.bf16 && !d.generic && aop == AOP_NONE;
  d.b16d_ok = 1;
  const size_t part = ig_plan(d);
  const size_t esz = d.bf16 ? 2 : (d.x3 ? 6 : 4);
  const size_t wpb = d.generic ? (size_t)d.Npad * d.Kc * 4 : (size_t)P.T * d.Npad * x->c * esz;
  d.wplane = (long long)P.T * d.Npad * x->c;
  // bf16 DMA tiles: the input as a compact NHWC bf16 copy in the workspace (after the pack, which
  // IC_MATH_WPACKED keeps at the workspace's start)
  const long long xel = (long long)x->n * x->h * x->w * x->c;
  const size_t xbb = (d.dma && d.bf16 && !have_xb) ? (size_t)xel * 2 : 0;
  const size_t tot = ic_align(wpb, 256) + ic_align(part, 256) + ic_align(xbb, 256);
  if (need) {
    plan_report(ig_kernel_kind(d), d.bm, d.bn, d.ksplit, 0, 0, ig_grid_blocks(d));
    *need = tot;
    return IC_OK;
  }
  if (wsb < tot) return IC_ERR_WORKSPACE;
  Carve cv{(char*)ws, 0};
  float* wp = cv.take(wpb);
  d.partial = part ? cv.take(part) : nullptr;
  P.wp = wp;
  if (!(math & IC_MATH_WPACKED)) {
    int rc = pack_weights(W, y->c, x->c, k, 0, d.generic, P.T, ky, kx, d.Npad, d.Kc, wp, s, d.x3 ? 2 : d.bf16);
    if (rc) return rc;
  }
  if (d.dma && d.bf16) {
    if (have_xb) {
      d.xb = xb;
    } else {
      void* xc = cv.take(xbb);
      int rc = ig_cvt_bf16(x->data, xc, xel, s);
      if (rc) return rc;
      d.xb = xc;
    }
  }
  return ig_run(d, s);
}

// y[b] at (s*iy - pad + ky) += x[a] @ iy * W[a][b][ky][kx]    (W: [A=x->c][B=y->c][k][k])
// xb (IC_MATH_XB): as direct_impl -- x's bf16 copy for the bf16 DMA tiles of the phases
int transposed_impl(const ic_act* x, const float* W, const float* bias, int k, int stride, int pad,
                    const ic_act* y, int epi, void* ws, size_t wsb, hipStream_t s, size_t* need, int math = 0,
                    const void* xb = nullptr) {
  const bool have_xb = (math & IC_MATH_XB) != 0;
  math &= ~IC_MATH_XB;
  if (have_xb && !need && !xb) return IC_ERR_ARG;
  if (k < 1 || k * k > IC_MAXT || stride < 1 || stride > 2) return IC_ERR_ARG;
  if (x->n != y->n) return IC_ERR_ARG;
  if (!act_fits32(x) || !act_fits32(y)) return IC_ERR_ARG;  // 32-bit element offsets in the kernels
  if ((y->h + 2 * pad - k) / stride + 1 != x->h || (y->w + 2 * pad - k) / stride + 1 != x->w)
    return IC_ERR_ARG;
  if ((epi == EPI_NONE || epi == EPI_RELU) &&
      tconv_few_ok(x->c, y->c, k, stride, pad, x->sc, x->sw, x->sh, x->sn, x->h, x->w)) {
    // output-row-stationary kernel (edge.hip): no column buffer in HBM
    const int split = (EDGE_BF16 && (math & IC_MATH_BF16)) ? 2 : (math & IC_MATH_SPLIT) ? 1 : 0;
    if (need) {
      const int kind = tconv_few_kind(x->h, x->w, k, pad, y->h);
      // variant 1: the input-row kernel in split arithmetic or with bf16 operands
      const bool x3 = kind == IC_KERNEL_TCONV_FEW_ROWS && split && x->c % 32 == 0;
      plan_report(x3 && split == 2 ? IC_KERNEL_TCONV_FEW_ROWS_BF16 : kind, 0, y->c, 1, 0, 0, -1, x3 ? 1 : 0);
      *need = 0;
      return IC_OK;
    }
    return tconv_few_run(x->data, x->n, x->h, x->w, x->c, W, y->c, k, pad, bias, epi == EPI_RELU, y->data, y->sn,
                         y->sc, y->sh, y->sw, y->h, y->w, s, split);
  }
  if (y->c <= FEW_CH && x->c % 32 == 0 && x->sc == 1)
    return transposed_col2im(x, W, bias, k, stride, pad, y, epi, ws, wsb, s, need);
  IgDesc d = {};
  set_x(d, x);
  set_y(d, y);
  d.stride = 1;
  d.generic = (x->c % 32 != 0) || (x->sc != 1);
  d.bias = bias; d.epi = epi; d.a_op = AOP_NONE;
  int pky[IC_MAXPH][IC_MAXT], pkx[IC_MAXPH][IC_MAXT];
  int np = 0, tmax = 0;
  for (int py = 0; py < stride; ++py)
    for (int px = 0; px < stride; ++px) {
      IgPhase& P = d.ph[np];
      const int Hg = (y->h - py + stride - 1) / stride, Wg = (y->w - px + stride - 1) / stride;
      if (Hg <= 0 || Wg <= 0) continue;
      int T = 0;
      for (int a = 0; a < k; ++a) {
        const int ny = py + pad - a;
        if (((ny % stride) + stride) % stride) continue;
        for (int b = 0; b < k; ++b) {
          const int nx = px + pad - b;
          if (((nx % stride) + stride) % stride) continue;
          pky[np][T] = a; pkx[np][T] = b;
          P.dy[T] = ny / stride;  // exact division (ny multiple of stride)
          P.dx[T] = nx / stride;
          ++T;
        }
      }
      if (T == 0) return IC_ERR_ARG;
      P.T = T; P.Hg = Hg; P.Wg = Wg;
      P.oys = stride; P.oxs = stride; P.oy0 = py; P.ox0 = px;
      tmax = T > tmax ? T : tmax;
      ++np;
    }
  d.nphase = np;
  d.Kc = d.generic ? (int)ic_align((size_t)tmax * x->c, 32) : x->c;
  d.bf16 = (math & IC_MATH_BF16) && !d.generic && x->c % 64 == 0;
  int ttot = 0;
  for (int p = 0; p < np; ++p) ttot += d.ph[p].T;
  d.x3 = (math & IC_MATH_SPLIT) && !d.bf16 && !d.generic && ttot <= IC_MAXT;
  d.b16d_ok = ttot <= IC_MAXT;  // the bf16 DMA tiles need the one-launch pack of every phase (below)
  const size_t part = ig_plan(d);
  if (d.x3) {
    // one pack of three bf16 planes [part][t over all phases][Npad][Cin]
    d.wplane = (long long)ttot * d.Npad * x->c;
    const size_t wb = (size_t)d.wplane * 6;
    const size_t tot = ic_align(part, 256) + ic_align(wb, 256);
    if (need) {
      plan_report(ig_kernel_kind(d), d.bm, d.bn, d.ksplit, 0, 0, ig_grid_blocks(d));
      *need = tot;
      return IC_OK;
    }
    if (wsb < tot) return IC_ERR_WORKSPACE;
    Carve cv{(char*)ws, 0};
    d.partial = part ? cv.take(part) : nullptr;
    __bf16* base = (__bf16*)cv.take(wb);
    int aky[IC_MAXT], akx[IC_MAXT], t0 = 0;
    for (int p = 0; p < np; ++p) {
      d.ph[p].wp = (const float*)(base + (size_t)t0 * d.Npad * x->c);
      for (int t = 0; t < d.ph[p].T; ++t) { aky[t0 + t] = pky[p][t]; akx[t0 + t] = pkx[p][t]; }
      t0 += d.ph[p].T;
    }
    if (!(math & IC_MATH_WPACKED)) {
      int rc = pack_weights(W, x->c, y->c, k, 1, 0, ttot, aky, akx, d.Npad, d.Kc, (float*)base, s, 2);
      if (rc) return rc;
    }
    return ig_run(d, s);
  }
  size_t wpb[IC_MAXPH];
  size_t tot = ic_align(part, 256);
  for (int p = 0; p < np; ++p) {
    wpb[p] = d.generic ? (size_t)d.Npad * d.Kc * 4 : (size_t)d.ph[p].T * d.Npad * x->c * (d.bf16 ? 2 : 4);
    tot += ic_align(wpb[p], 256);
  }
  const long long xel = (long long)x->n * x->h * x->w * x->c;
  const size_t xbb = (d.dma && d.bf16 && !have_xb) ? (size_t)xel * 2 : 0;
  tot += ic_align(xbb, 256);
  if (need) {
    plan_report(ig_kernel_kind(d), d.bm, d.bn, d.ksplit, 0, 0, ig_grid_blocks(d));
    *need = tot;
    return IC_OK;
  }
  if (wsb < tot) return IC_ERR_WORKSPACE;
  Carve cv{(char*)ws, 0};
  d.partial = part ? cv.take(part) : nullptr;
  if (d.dma && d.bf16) {  // the bf16 DMA tiles' A operand: the caller's copy, or x converted here
    if (have_xb) {
      d.xb = xb;
    } else {
      void* xc = cv.take(xbb);
      int rc = ig_cvt_bf16(x->data, xc, xel, s);
      if (rc) return rc;
      d.xb = xc;
    }
  }
  // fast layout: the phases' [t][n][r] packs are back to back in the
  // workspace (each a multiple of 256 B), so one launch packs every phase
  bool contiguous = !d.generic;
  for (int p = 0; p < np; ++p) contiguous = contiguous && wpb[p] % 256 == 0;
  if (d.dma && !(contiguous && ttot <= IC_MAXT)) return IC_ERR_ARG;
  if (contiguous && ttot <= IC_MAXT) {
    int aky[IC_MAXT], akx[IC_MAXT], t0 = 0;
    for (int p = 0; p < np; ++p) {
      float* wp = cv.take(wpb[p]);
      d.ph[p].wp = wp;
      for (int t = 0; t < d.ph[p].T; ++t) { aky[t0 + t] = pky[p][t]; akx[t0 + t] = pkx[p][t]; }
      t0 += d.ph[p].T;
    }
    if (!(math & IC_MATH_WPACKED)) {
      int rc = pack_weights(W, x->c, y->c, k, 1, 0, ttot, aky, akx, d.Npad, d.Kc, (float*)d.ph[0].wp, s, d.bf16);
      if (rc) return rc;
    }
    return ig_run(d, s);
  }
  for (int p = 0; p < np; ++p) {
    float* wp = cv.take(wpb[p]);
    d.ph[p].wp = wp;
    if (math & IC_MATH_WPACKED) continue;
    int rc = pack_weights(W, x->c, y->c, k, 1, d.generic, d.ph[p].T, pky[p], pkx[p], d.Npad, d.Kc, wp, s, d.bf16);
    if (rc) return rc;
  }
  return ig_run(d, s);
}

// dW[g][c][ky][kx] = sum_p G[p][g] * X[p*s + ky - pad][c]; db = colsum(bias_src)
// g16 / x16: G's and X's bf16 copies (ic_conv*_wgrad_xb; used by the bf16 tap-group kernel, else ignored)
int wgrad_impl(const ic_act* G, const ic_act* X, int k, int stride, int pad, float* dw,
               const ic_act* bias_src, float* db, void* ws, size_t wsb, hipStream_t s, size_t* need, int math = 0,
               const void* g16 = nullptr, const void* x16 = nullptr) {
  if (k < 1 || k * k > IC_MAXT || stride < 1) return IC_ERR_ARG;
  if (G->n != X->n) return IC_ERR_ARG;
  if (!act_fits32(G) || !act_fits32(X)) return IC_ERR_ARG;  // 32-bit element offsets in the kernels
  if ((X->h + 2 * pad - k) / stride + 1 != G->h || (X->w + 2 * pad - k) / stride + 1 != G->w)
    return IC_ERR_ARG;
  WgDesc d = {};
  d.g = G->data; d.gs_n = G->sn; d.gs_h = G->sh; d.gs_w = G->sw; d.gs_c = G->sc;
  d.Hg = G->h; d.Wg = G->w; d.Cg = G->c;
  d.x = X->data; d.xs_n = X->sn; d.xs_h = X->sh; d.xs_w = X->sw; d.xs_c = X->sc;
  d.Hx = X->h; d.Wx = X->w; d.Cx = X->c;
  d.N = G->n; d.stride = stride; d.T = k * k; d.x_op = AOP_NONE;
  d.generic = (X->c % 4 != 0) || (X->sc != 1);
  d.split_ok = (math & IC_MATH_SPLIT) ? 1 : 0;
  d.bf16 = (math & IC_MATH_BF16) ? 1 : 0;
  d.x3 = (d.split_ok || d.bf16) ? 1 : 0;  // the bf16 form runs on the split kernel family
  if (d.bf16) { d.g16 = g16; d.x16 = x16; }
  int kk_of_t[IC_MAXT];
  for (int t = 0; t < d.T; ++t) {
    d.dy[t] = t / k - pad; d.dx[t] = t % k - pad; kk_of_t[t] = t;
  }
  // few X channels, wide NHWC G: patch-gather wgrad (edge.hip); the bias
  // gradient comes from its all-ones column when the bias belongs to G
  if (X->c <= FEW_CH && edge_wgrad_ok(X->c, k, stride, X->sw, G->data, G->c, G->sc, G->sw, G->sh, G->sn, G->h, G->w)) {
    const int split = (EDGE_BF16 && (math & IC_MATH_BF16)) ? 2 : (math & IC_MATH_SPLIT) ? 1 : 0;
    // the bias gradient from G's all-ones column, except with bf16 operands (it would sum rounded G)
    const bool db_from_g = db && bias_src->data == G->data && split != 2;
    const int Kc = k * k * X->c + (db_from_g ? 1 : 0);
    const size_t slab = edge_wgrad_ws(G->c, Kc, edge_units(G->n, G->h, G->w));
    const size_t cs = (db && !db_from_g) ? colsum_ws((long long)bias_src->n * bias_src->h * bias_src->w, bias_src->c) : 0;
    if (need) {
      plan_report(split == 2 ? IC_KERNEL_EDGE_WGRAD_BF16 : IC_KERNEL_EDGE_WGRAD, G->c, Kc, 1, 0, 0, -1,
                  split ? 1 : 0);  // 1: split arithmetic or bf16 operands
      *need = ic_align(slab, 256) + ic_align(cs, 256);
      return IC_OK;
    }
    if (wsb < ic_align(slab, 256) + ic_align(cs, 256)) return IC_ERR_WORKSPACE;
    int rc = edge_wgrad_run(G->data, G->c, X->data, X->sn, X->sc, X->sh, X->sw, X->n, X->c, X->h, X->w, G->h, G->w,
                            k, stride, pad, dw, db_from_g ? db : nullptr, ws, s, split);
    if (rc) return rc;
    if (db && !db_from_g)
      rc = colsum(bias_src->data, bias_src->sn, bias_src->sc, bias_src->sh, bias_src->sw, bias_src->n, bias_src->c,
                  bias_src->h, bias_src->w, db, 1.f, (char*)ws + ic_align(slab, 256), s);
    return rc;
  }
  // few X channels: wgrad against xcol = im2col(X) on G's grid (1 tap, K = Kp)
  const bool few = X->c <= FEW_CH;
  const int Kp = (int)ic_align((size_t)d.T * X->c, 32);
  size_t xcb = 0;
  if (few) {
    xcb = (size_t)G->n * G->h * G->w * Kp * 4;
    d.Hx = G->h; d.Wx = G->w; d.Cx = Kp; d.stride = 1; d.T = 1; d.dy[0] = 0; d.dx[0] = 0;
    d.xs_c = 1; d.xs_w = Kp; d.xs_h = (long long)G->w * Kp; d.xs_n = (long long)G->h * G->w * Kp;
    d.generic = 0;
    d.x3 = 0;
    d.bf16 = 0;
  }
  const size_t part = wg_plan(d);
  const size_t cs = db ? colsum_ws((long long)bias_src->n * bias_src->h * bias_src->w, bias_src->c) : 0;
  const size_t tot = ic_align(part, 256) + ic_align(cs, 256) + ic_align(xcb, 256);
  if (need) {
    if (g_plan_sink) {
      WgDesc q = d;
      wg_prepare(q);
      plan_report(wg_kernel_kind(q), q.bm, q.bn, 1, q.nsplit, few ? 1 : 0, wg_grid_blocks(q), q.rowfast);
    }
    *need = tot;
    return IC_OK;
  }
  if (wsb < tot) return IC_ERR_WORKSPACE;
  Carve cv{(char*)ws, 0};
  d.partial = cv.take(part);
  float* csw = cs ? cv.take(cs) : nullptr;
  int rc;
  if (few) {
    float* xcol = cv.take(xcb);
    d.x = xcol;
    rc = im2col_run(X->data, X->sn, X->sc, X->sh, X->sw, X->n, X->c, X->h, X->w, G->h, G->w, stride, k, pad, Kp,
                    xcol, s);
    if (rc) return rc;
  }
  rc = wg_run(d, s);
  if (rc) return rc;
  if (few) {
    // reduce the (t, c)-flattened columns straight into [g][c][ky][kx]
    WgDesc r = d;
    r.generic = 1; r.T = k * k; r.Cx = X->c;
    rc = wg_reduce(r, dw, kk_of_t, k * k, s);
  } else {
    rc = wg_reduce(d, dw, kk_of_t, k * k, s);
  }
  if (rc) return rc;
  if (db) {
    rc = colsum(bias_src->data, bias_src->sn, bias_src->sc, bias_src->sh, bias_src->sw, bias_src->n,
                bias_src->c, bias_src->h, bias_src->w, db, 1.f, csw, s);
    if (rc) return rc;
  }
  return IC_OK;
}

size_t need_or_zero(int rc, size_t n) { return rc ? 0 : n; }

}  // namespace

extern "C" {

int ic_version(void) { return 3; }  // 3: ic_fact_net / ic_fact_net_grads hold IC_FACT_NET_MAXL layers (round 6)

int ic_conv_plan(int op, const ic_act* a, const ic_act* b, int k, int stride, int pad, int math, ic_plan* out) {
  if (!out || !a || (!b && op != IC_OP_GDN_FWD && op != IC_OP_GDN_BWD)) return IC_ERR_ARG;
  ic_plan p = {0, 0, 0, 1, 0, 0, 0, -1};
  g_plan_sink = &p;
  size_t n = 0;
  int rc;
  switch (op) {
    case IC_OP_CONV2D_FWD:
    case IC_OP_TCONV_DGRAD:
      rc = direct_impl(a, nullptr, nullptr, k, stride, pad, b, EPI_NONE, AOP_NONE, nullptr, nullptr, nullptr,
                       nullptr, nullptr, 0, 0, &n, math);
      break;
    case IC_OP_CONV2D_DGRAD:
    case IC_OP_TCONV_FWD:
      rc = transposed_impl(a, nullptr, nullptr, k, stride, pad, b, EPI_NONE, nullptr, 0, 0, &n, math);
      break;
    case IC_OP_CONV2D_WGRAD:  // G = dy, X = x, bias from dy
      rc = wgrad_impl(b, a, k, stride, pad, nullptr, b, (float*)1, nullptr, 0, 0, &n, math);
      break;
    case IC_OP_TCONV_WGRAD:   // G = x, X = dy, bias from dy
      rc = wgrad_impl(a, b, k, stride, pad, nullptr, b, (float*)1, nullptr, 0, 0, &n, math);
      break;
    case IC_OP_GDN_FWD:
    case IC_OP_GDN_BWD:
      rc = gdn_plan(op == IC_OP_GDN_BWD, a, math);
      break;
    default:
      rc = IC_ERR_ARG;
  }
  g_plan_sink = nullptr;
  if (rc == IC_OK && p.kernel == 0) rc = IC_ERR_ARG;
  if (rc == IC_OK) *out = p;
  return rc;
}

size_t ic_conv2d_fwd_ws_ex(const ic_act* x, int k, int stride, int pad, const ic_act* y, int math) {
  size_t n = 0;
  int rc = direct_impl(x, nullptr, nullptr, k, stride, pad, y, EPI_NONE, AOP_NONE, nullptr, nullptr,
                       nullptr, nullptr, nullptr, 0, 0, &n, math);
  return need_or_zero(rc, n);
}
int ic_conv2d_fwd_ex(const ic_act* x, const float* w, const float* b, int k, int stride, int pad,
                     const ic_act* y, int act, int math, void* ws, size_t ws_bytes, void* stream) {
  return direct_impl(x, w, b, k, stride, pad, y, act ? EPI_RELU : EPI_NONE, AOP_NONE, nullptr,
                     nullptr, nullptr, nullptr, ws, ws_bytes, (hipStream_t)stream, nullptr, math);
}
size_t ic_conv2d_fwd_ws(const ic_act* x, int k, int stride, int pad, const ic_act* y) {
  return ic_conv2d_fwd_ws_ex(x, k, stride, pad, y, 0);
}
int ic_conv2d_fwd_xb(const ic_act* x, const void* xb, const float* w, const float* b, int k, int stride, int pad,
                     const ic_act* y, int act, int math, void* ws, size_t ws_bytes, void* stream) {
  return direct_impl(x, w, b, k, stride, pad, y, act ? EPI_RELU : EPI_NONE, AOP_NONE, nullptr,
                     nullptr, nullptr, nullptr, ws, ws_bytes, (hipStream_t)stream, nullptr, math | IC_MATH_XB, xb);
}
int ic_conv2d_fwd(const ic_act* x, const float* w, const float* b, int k, int stride, int pad,
                  const ic_act* y, int act, void* ws, size_t ws_bytes, void* stream) {
  return ic_conv2d_fwd_ex(x, w, b, k, stride, pad, y, act, 0, ws, ws_bytes, stream);
}

size_t ic_conv2d_dgrad_ws_ex(const ic_act* dy, int k, int stride, int pad, const ic_act* dx, int math) {
  size_t n = 0;
  int rc = transposed_impl(dy, nullptr, nullptr, k, stride, pad, dx, EPI_NONE, nullptr, 0, 0, &n, math);
  return need_or_zero(rc, n);
}
int ic_conv2d_dgrad_ex(const ic_act* dy, const float* w, int k, int stride, int pad, const ic_act* dx, int math,
                       void* ws, size_t ws_bytes, void* stream) {
  // conv weight [Cout][Cin] is the transposed-gather weight [A=Cout (dy ch)][B=Cin (dx ch)]
  return transposed_impl(dy, w, nullptr, k, stride, pad, dx, EPI_NONE, ws, ws_bytes,
                         (hipStream_t)stream, nullptr, math);
}
int ic_conv2d_dgrad_xb(const ic_act* dy, const void* dyb, const float* w, int k, int stride, int pad,
                       const ic_act* dx, int math, void* ws, size_t ws_bytes, void* stream) {
  return transposed_impl(dy, w, nullptr, k, stride, pad, dx, EPI_NONE, ws, ws_bytes, (hipStream_t)stream, nullptr,
                         math | IC_MATH_XB, dyb);
}
size_t ic_conv2d_dgrad_ws(const ic_act* dy, int k, int stride, int pad, const ic_act* dx) {
  return ic_conv2d_dgrad_ws_ex(dy, k, stride, pad, dx, 0);
}
int ic_conv2d_dgrad(const ic_act* dy, const float* w, int k, int stride, int pad, const ic_act* dx,
                    void* ws, size_t ws_bytes, void* stream) {
  return ic_conv2d_dgrad_ex(dy, w, k, stride, pad, dx, 0, ws, ws_bytes, stream);
}

size_t ic_conv2d_wgrad_ws(const ic_act* x, const ic_act* dy, int k, int stride, int pad) {
  size_t n = 0;
  int rc = wgrad_impl(dy, x, k, stride, pad, nullptr, dy, (float*)1, nullptr, 0, 0, &n);
  return need_or_zero(rc, n);
}
int ic_conv2d_wgrad(const ic_act* x, const ic_act* dy, int k, int stride, int pad, float* dw,
                    float* db, void* ws, size_t ws_bytes, void* stream) {
  return wgrad_impl(dy, x, k, stride, pad, dw, dy, db, ws, ws_bytes, (hipStream_t)stream, nullptr);
}

size_t ic_conv_transpose2d_fwd_ws_ex(const ic_act* x, int k, int stride, int pad, const ic_act* y, int math) {
  size_t n = 0;
  int rc = transposed_impl(x, nullptr, nullptr, k, stride, pad, y, EPI_NONE, nullptr, 0, 0, &n, math);
  return need_or_zero(rc, n);
}
int ic_conv_transpose2d_fwd_ex(const ic_act* x, const float* w, const float* b, int k, int stride, int pad,
                               const ic_act* y, int act, int math, void* ws, size_t ws_bytes, void* stream) {
  return transposed_impl(x, w, b, k, stride, pad, y, act ? EPI_RELU : EPI_NONE, ws, ws_bytes,
                         (hipStream_t)stream, nullptr, math);
}
int ic_conv_transpose2d_fwd_xb(const ic_act* x, const void* xb, const float* w, const float* b, int k, int stride,
                               int pad, const ic_act* y, int act, int math, void* ws, size_t ws_bytes, void* stream) {
  return transposed_impl(x, w, b, k, stride, pad, y, act ? EPI_RELU : EPI_NONE, ws, ws_bytes, (hipStream_t)stream,
                         nullptr, math | IC_MATH_XB, xb);
}
size_t ic_conv_transpose2d_fwd_ws(const ic_act* x, int k, int stride, int pad, const ic_act* y) {
  return ic_conv_transpose2d_fwd_ws_ex(x, k, stride, pad, y, 0);
}
int ic_conv_transpose2d_fwd(const ic_act* x, const float* w, const float* b, int k, int stride,
                            int pad, const ic_act* y, int act, void* ws, size_t ws_bytes,
                            void* stream) {
  return ic_conv_transpose2d_fwd_ex(x, w, b, k, stride, pad, y, act, 0, ws, ws_bytes, stream);
}

size_t ic_conv_transpose2d_dgrad_ws_ex(const ic_act* dy, int k, int stride, int pad, const ic_act* dx, int math) {
  size_t n = 0;
  int rc = direct_impl(dy, nullptr, nullptr, k, stride, pad, dx, EPI_NONE, AOP_NONE, nullptr, nullptr,
                       nullptr, nullptr, nullptr, 0, 0, &n, math);
  return need_or_zero(rc, n);
}
int ic_conv_transpose2d_dgrad_ex(const ic_act* dy, const float* w, int k, int stride, int pad, const ic_act* dx,
                                 int math, void* ws, size_t ws_bytes, void* stream) {
  // tconv weight [Cin][Cout] is the direct-gather weight [A=Cin (dx ch)][B=Cout (dy ch)]
  return direct_impl(dy, w, nullptr, k, stride, pad, dx, EPI_NONE, AOP_NONE, nullptr, nullptr,
                     nullptr, nullptr, ws, ws_bytes, (hipStream_t)stream, nullptr, math);
}
size_t ic_conv_transpose2d_dgrad_ws(const ic_act* dy, int k, int stride, int pad, const ic_act* dx) {
  return ic_conv_transpose2d_dgrad_ws_ex(dy, k, stride, pad, dx, 0);
}
int ic_conv_transpose2d_dgrad_xb(const ic_act* dy, const void* dyb, const float* w, int k, int stride, int pad,
                                 const ic_act* dx, int math, void* ws, size_t ws_bytes, void* stream) {
  return direct_impl(dy, w, nullptr, k, stride, pad, dx, EPI_NONE, AOP_NONE, nullptr, nullptr,
                     nullptr, nullptr, ws, ws_bytes, (hipStream_t)stream, nullptr, math | IC_MATH_XB, dyb);
}
int ic_conv_transpose2d_dgrad(const ic_act* dy, const float* w, int k, int stride, int pad,
                              const ic_act* dx, void* ws, size_t ws_bytes, void* stream) {
  return ic_conv_transpose2d_dgrad_ex(dy, w, k, stride, pad, dx, 0, ws, ws_bytes, stream);
}

size_t ic_conv2d_wgrad_ws_ex(const ic_act* x, const ic_act* dy, int k, int stride, int pad, int math) {
  size_t n = 0;
  int rc = wgrad_impl(dy, x, k, stride, pad, nullptr, dy, (float*)1, nullptr, 0, 0, &n, math);
  return need_or_zero(rc, n);
}
int ic_conv2d_wgrad_ex(const ic_act* x, const ic_act* dy, int k, int stride, int pad, float* dw, float* db, int math,
                       void* ws, size_t ws_bytes, void* stream) {
  return wgrad_impl(dy, x, k, stride, pad, dw, dy, db, ws, ws_bytes, (hipStream_t)stream, nullptr, math);
}
int ic_conv2d_wgrad_xb(const ic_act* x, const void* xb, const ic_act* dy, const void* dyb, int k, int stride, int pad,
                       float* dw, float* db, int math, void* ws, size_t ws_bytes, void* stream) {
  return wgrad_impl(dy, x, k, stride, pad, dw, dy, db, ws, ws_bytes, (hipStream_t)stream, nullptr, math, dyb, xb);
}

size_t ic_conv_transpose2d_wgrad_ws(const ic_act* x, const ic_act* dy, int k, int stride, int pad) {
  size_t n = 0;
  int rc = wgrad_impl(x, dy, k, stride, pad, nullptr, dy, (float*)1, nullptr, 0, 0, &n);
  return need_or_zero(rc, n);
}
int ic_conv_transpose2d_wgrad(const ic_act* x, const ic_act* dy, int k, int stride, int pad,
                              float* dw, float* db, void* ws, size_t ws_bytes, void* stream) {
  return wgrad_impl(x, dy, k, stride, pad, dw, dy, db, ws, ws_bytes, (hipStream_t)stream, nullptr);
}

size_t ic_conv_transpose2d_wgrad_ws_ex(const ic_act* x, const ic_act* dy, int k, int stride, int pad, int math) {
  size_t n = 0;
  int rc = wgrad_impl(x, dy, k, stride, pad, nullptr, dy, (float*)1, nullptr, 0, 0, &n, math);
  return need_or_zero(rc, n);
}
int ic_conv_transpose2d_wgrad_ex(const ic_act* x, const ic_act* dy, int k, int stride, int pad, float* dw, float* db,
                                 int math, void* ws, size_t ws_bytes, void* stream) {
  return wgrad_impl(x, dy, k, stride, pad, dw, dy, db, ws, ws_bytes, (hipStream_t)stream, nullptr, math);
}
int ic_conv_transpose2d_wgrad_xb(const ic_act* x, const void* xb, const ic_act* dy, const void* dyb, int k,
                                 int stride, int pad, float* dw, float* db, int math, void* ws, size_t ws_bytes,
                                 void* stream) {
  return wgrad_impl(x, dy, k, stride, pad, dw, dy, db, ws, ws_bytes, (hipStream_t)stream, nullptr, math, xb, dyb);
}

}  // extern "C"
