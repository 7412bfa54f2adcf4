/*
 * imgcomp.h — C ABI of libimgcomp.so, the MI355X (gfx950) kernels behind the
 * Balle-2018 scale-hyperprior hot path of hieu1999210/image_compression.
 *
 * Every entry point:
 *   - takes raw device pointers (fp32), plain sizes and a hipStream_t
 *     (passed as void* so this header needs no HIP include);
 *   - launches asynchronously on that stream; never allocates, frees or
 *     synchronises (graph-capturable); keeps no pointer after it returns;
 *   - returns 0 on success, a hipError_t value on a launch failure, or
 *     IC_ERR_ARG (1001) / IC_ERR_WORKSPACE (1002).  The Python host layer
 *     turns any non-zero status into RuntimeError (reference error
 *     behaviour: torch raises RuntimeError on bad shapes).
 *   - Ops that need scratch take (ws, ws_bytes); the matching *_ws() query
 *     returns the byte count for the same arguments.
 *
 * Activations are described by ic_act: logical [n][c][h][w] with arbitrary
 * element strides.  The GEMM fast paths want channel stride 1 (NHWC,
 * torch.channels_last); other layouts take the generic gather path.
 *
 * Reference interfaces replaced (paths relative to the reference repo):
 *   conv2d_*            torch.nn.Conv2d in modelling/blocks/analysis.py:55,
 *                       modelling/blocks/prior_analysis.py:54-56
 *   conv_transpose2d_*  torch.nn.ConvTranspose2d in modelling/blocks/synthesis.py:55-57,
 *                       modelling/blocks/prior_synthesis.py:54-56
 *   gdn_*               modelling/layers/gdn.py:79-88 (GDN.forward)
 *   nonneg_*            modelling/layers/gdn.py:59-62 (NonNegativeParam.forward)
 *   bound_*             modelling/layers/bound.py:28-59 (LowerBound / UpperBound)
 *   relu_*, abs_*       nn.ReLU (prior_*.py), torch.abs (meta_arch/bmshl2018.py:72)
 *   exp_clamp_*         modelling/blocks/prior_synthesis.py:72
 *   factorized_*        modelling/blocks/entropy_model.py:204-269 (EntropyModel)
 *   conditional_*       modelling/blocks/entropy_model.py:280-378 (Laplacian/Gaussian)
 *   ce_loss_*           modelling/blocks/entropy_model.py:171-185 (_ce_loss)
 *   mse_*, sqdiff_*     nn.MSELoss(reduction="mean"/"none") in modelling/loss.py:25
 *   msssim_*            modelling/loss.py:48-188 (SSIMLoss, MS_SSIMLoss)
 *   adamw_step          torch.optim.AdamW of solver/optim.py:20-45 + clip_grad_value_ of
 *                       engine/trainer.py:189-190 (the training step around the path)
 */
#ifndef IMGCOMP_H
#define IMGCOMP_H
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define IC_ERR_ARG 1001
#define IC_ERR_WORKSPACE 1002

typedef struct ic_act {
  float* data;
  int n, c, h, w;
  long long sn, sc, sh, sw; /* element strides */
} ic_act;

/* ---- library ---- */
int ic_version(void);                 /* ABI version (monotonic; 3: ic_fact_net with IC_FACT_NET_MAXL layers) */
int ic_device_sync_check(void* stream); /* hipStreamQuery-free no-op launch test */

/* ---- Conv2d (k x k, stride, zero pad): y = conv(x, w) + b, act 0=none 1=relu
 *      w: [Cout][Cin][k][k]; b: [Cout] or NULL; y->c = Cout, y->h = (x->h+2pad-k)/stride+1 */
size_t ic_conv2d_fwd_ws(const ic_act* x, int k, int stride, int pad, const ic_act* y);
int ic_conv2d_fwd(const ic_act* x, const float* w, const float* b, int k, int stride, int pad,
                  const ic_act* y, int act, void* ws, size_t ws_bytes, void* stream);
/* dx = conv2d input-gradient of dy (no bias); dx->c = Cin */
size_t ic_conv2d_dgrad_ws(const ic_act* dy, int k, int stride, int pad, const ic_act* dx);
int ic_conv2d_dgrad(const ic_act* dy, const float* w, int k, int stride, int pad, const ic_act* dx,
                    void* ws, size_t ws_bytes, void* stream);
/* dw [Cout][Cin][k][k] = weight gradient; db [Cout] (optional, NULL to skip) */
size_t ic_conv2d_wgrad_ws(const ic_act* x, const ic_act* dy, int k, int stride, int pad);
int ic_conv2d_wgrad(const ic_act* x, const ic_act* dy, int k, int stride, int pad, float* dw,
                    float* db, void* ws, size_t ws_bytes, void* stream);

/* ---- ConvTranspose2d: w [Cin][Cout][k][k]; y->h = (x->h-1)*stride - 2pad + k + output_padding */
size_t ic_conv_transpose2d_fwd_ws(const ic_act* x, int k, int stride, int pad, const ic_act* y);
int ic_conv_transpose2d_fwd(const ic_act* x, const float* w, const float* b, int k, int stride,
                            int pad, const ic_act* y, int act, void* ws, size_t ws_bytes,
                            void* stream);
size_t ic_conv_transpose2d_dgrad_ws(const ic_act* dy, int k, int stride, int pad, const ic_act* dx);
int ic_conv_transpose2d_dgrad(const ic_act* dy, const float* w, int k, int stride, int pad,
                              const ic_act* dx, void* ws, size_t ws_bytes, void* stream);
size_t ic_conv_transpose2d_wgrad_ws(const ic_act* x, const ic_act* dy, int k, int stride, int pad);
int ic_conv_transpose2d_wgrad(const ic_act* x, const ic_act* dy, int k, int stride, int pad,
                              float* dw, float* db, void* ws, size_t ws_bytes, void* stream);

/* ---- math modes of the conv fwd / dgrad "_ex" variants (the plain entry points are math 0).
 *      IC_MATH_BF16: operands rounded to bf16 (round-to-nearest-even), fp32 accumulation on
 *      v_mfma_f32_32x32x16_bf16 — the bf16 configuration of BASELINE config C3 — for layers
 *      whose reduction channel count is a multiple of 64; others (the 3-channel image edges)
 *      and all weight gradients / GDN stay fp32. */
#define IC_MATH_FP32 0
#define IC_MATH_BF16 1
/*      IC_MATH_SPLIT: fp32 arithmetic on the bf16 MFMA — each fp32 operand split exactly into
 *      three bf16 terms, six cross products accumulated in fp32 (error of an fp32 fma chain,
 *      3/8 of the native fp32 MFMA's cycles per MAC); layers with reduction channels % 32 == 0
 *      and >= 64 output channels, others run the native fp32 kernel. */
#define IC_MATH_SPLIT 2
/*      IC_MATH_WPACKED (conv / transposed-conv forward only, or-ed into a math mode): the workspace
 *      already holds this weight's pack, written by an earlier forward with the same weight
 *      values, activation shapes / strides, math mode and workspace; the pack launch is skipped
 *      (eval-mode weight caching, functional.py).  Paths whose pack is not kept in the workspace
 *      (the im2col fallback, the row-stationary transposed edge) ignore it.  The caller owns the invalidation: any change of
 *      the weight needs a forward without the flag first. */
#define IC_MATH_WPACKED 4
/*      IC_MATH_XB (or-ed into IC_MATH_BF16, in the workspace query of a conv / transposed conv forward or
 *      input gradient whose caller passes the input's bf16 copy to the matching *_xb entry point): the
 *      workspace leaves out the space the conversion of x would take. */
#define IC_MATH_XB 8
size_t ic_conv2d_fwd_ws_ex(const ic_act* x, int k, int stride, int pad, const ic_act* y, int math);
int ic_conv2d_fwd_ex(const ic_act* x, const float* w, const float* b, int k, int stride, int pad,
                     const ic_act* y, int act, int math, void* ws, size_t ws_bytes, void* stream);
size_t ic_conv2d_dgrad_ws_ex(const ic_act* dy, int k, int stride, int pad, const ic_act* dx, int math);
int ic_conv2d_dgrad_ex(const ic_act* dy, const float* w, int k, int stride, int pad, const ic_act* dx,
                       int math, void* ws, size_t ws_bytes, void* stream);
size_t ic_conv_transpose2d_fwd_ws_ex(const ic_act* x, int k, int stride, int pad, const ic_act* y, int math);
int ic_conv_transpose2d_fwd_ex(const ic_act* x, const float* w, const float* b, int k, int stride, int pad,
                               const ic_act* y, int act, int math, void* ws, size_t ws_bytes, void* stream);
size_t ic_conv_transpose2d_dgrad_ws_ex(const ic_act* dy, int k, int stride, int pad, const ic_act* dx,
                                       int math);
int ic_conv_transpose2d_dgrad_ex(const ic_act* dy, const float* w, int k, int stride, int pad,
                                 const ic_act* dx, int math, void* ws, size_t ws_bytes, void* stream);

/* weight gradients with a math mode: IC_MATH_SPLIT runs the split kernel on 192-channel-tile NHWC
 * operands (>= 128 channels each side), the fp32 kernel otherwise; IC_MATH_BF16 runs bf16 operands with
 * fp32 accumulation on the same operands where the two-wave kernel applies (output maps >= 16 wide,
 * row-aligned 32-pixel steps) and falls back to split arithmetic (when IC_MATH_SPLIT is also set) or
 * fp32 elsewhere. */
size_t ic_conv2d_wgrad_ws_ex(const ic_act* x, const ic_act* dy, int k, int stride, int pad, int math);
int ic_conv2d_wgrad_ex(const ic_act* x, const ic_act* dy, int k, int stride, int pad, float* dw, float* db,
                       int math, void* ws, size_t ws_bytes, void* stream);
size_t ic_conv_transpose2d_wgrad_ws_ex(const ic_act* x, const ic_act* dy, int k, int stride, int pad, int math);
int ic_conv_transpose2d_wgrad_ex(const ic_act* x, const ic_act* dy, int k, int stride, int pad, float* dw,
                                 float* db, int math, void* ws, size_t ws_bytes, void* stream);

/* ---- GDN: norm = beta + conv1x1(x^2, gamma); y = x / sqrt(norm) (inverse: x * sqrt(norm)).
 *      gamma [C][C], beta [C] (already re-parameterised); x, y, norm share one layout. */
size_t ic_gdn_fwd_ws(const ic_act* x);
int ic_gdn_fwd(const ic_act* x, const float* gamma, const float* beta, int inverse,
               const ic_act* y, float* norm, void* ws, size_t ws_bytes, void* stream);
size_t ic_gdn_bwd_ws(const ic_act* x);
int ic_gdn_bwd(const ic_act* x, const float* norm, const float* dy, const float* gamma, int inverse,
               const ic_act* dx, float* dgamma, float* dbeta, void* ws, size_t ws_bytes,
               void* stream);
/* math = IC_MATH_SPLIT (C % 32 == 0, C >= 64, channel-contiguous): the forward runs in split arithmetic —
 * the fused kernel for NHWC-dense C = 192, otherwise the split implicit GEMM (x^2 squared in its staging,
 * the divide in its epilogue). */
size_t ic_gdn_fwd_ws_ex(const ic_act* x, int math);
int ic_gdn_fwd_ex(const ic_act* x, const float* gamma, const float* beta, int inverse, const ic_act* y, float* norm,
                  int math, void* ws, size_t ws_bytes, void* stream);
/* math = IC_MATH_SPLIT: the fused backward (C = 192) forms dgamma in split arithmetic (fp32 via three bf16
 * terms on the bf16 MFMA), dx on the fp32 MFMA.  math = IC_MATH_BF16 (C = 192, config C3): both of its
 * GEMMs (dx's q.gamma and dgamma's q^T x^2) on bf16 operands with fp32 accumulation.  Other shapes stay
 * on the fp32 MFMA. */
int ic_gdn_bwd_ex(const ic_act* x, const float* norm, const float* dy, const float* gamma, int inverse,
                  const ic_act* dx, float* dgamma, float* dbeta, int math, void* ws, size_t ws_bytes, void* stream);
/* ic_gdn_bwd_ex plus dxsum[c] = sum over all pixels of dx[.,c,.,.] (C floats): the bias gradient of
 * the convolution that produced the GDN input (reference analysis.py / synthesis.py: conv -> GDN),
 * formed by the fused backward from its dx tiles instead of a separate pass over dx.  Same workspace
 * as ic_gdn_bwd_ws. */
int ic_gdn_bwd_sum_ex(const ic_act* x, const float* norm, const float* dy, const float* gamma, int inverse,
                      const ic_act* dx, float* dgamma, float* dbeta, float* dxsum, int math, void* ws,
                      size_t ws_bytes, void* stream);

/* ---- bf16 activation copies (config C3, round 5): a GDN forward / backward whose output feeds a
 *      192 -> 192 conv forward / transposed-conv input gradient on the bf16 DMA tiles also writes that
 *      output as a compact NHWC bf16 copy (round to nearest even: the operand the conv would form);
 *      the conv reads the copy (2 B per element, nothing converted).  y / dx must be compact NHWC
 *      (channel stride 1), C % 8 == 0.  Replace (reference modelling/layers/gdn.py:79-88 feeding
 *      modelling/blocks/analysis.py:55, synthesis.py:55-57) the plain forms above. */
int ic_gdn_fwd_xb(const ic_act* x, const float* gamma, const float* beta, int inverse, const ic_act* y, float* norm,
                  void* yb, int math, void* ws, size_t ws_bytes, void* stream);
int ic_gdn_bwd_sum_xb(const ic_act* x, const float* norm, const float* dy, const float* gamma, int inverse,
                      const ic_act* dx, float* dgamma, float* dbeta, float* dxsum, void* dxb, int math, void* ws,
                      size_t ws_bytes, void* stream);
/* ---- norm recomputed (config C3, round 6): the GDN forward with bf16 operands (IC_MATH_BF16 | IC_MATH_SPLIT,
 *      C = 192, NHWC-dense) can leave norm = beta + Gamma x^2 out, and the backward forms it again per tile
 *      from x, Gamma and beta -- the forward's operands, products and order, so bitwise the same norm.  Both
 *      kernels are HBM-bound there; together they move 24 instead of 32 bytes per element.  yb / dxb: the
 *      optional bf16 copies of ic_gdn_fwd_xb / ic_gdn_bwd_sum_xb (NULL: none).  Any other math mode, C or
 *      layout is IC_ERR_ARG.  Workspaces: ic_gdn_fwd_ws_ex / ic_gdn_bwd_ws.  Replace (reference
 *      modelling/layers/gdn.py:79-88) ic_gdn_fwd_xb / ic_gdn_bwd_sum_xb in C3's training step. */
int ic_gdn_fwd_rn(const ic_act* x, const float* gamma, const float* beta, int inverse, const ic_act* y, void* yb,
                  int math, void* ws, size_t ws_bytes, void* stream);
int ic_gdn_bwd_sum_rn(const ic_act* x, const float* beta, const float* dy, const float* gamma, int inverse,
                      const ic_act* dx, float* dgamma, float* dbeta, float* dxsum, void* dxb, int math, void* ws,
                      size_t ws_bytes, void* stream);
/* xb / dyb: the input's bf16 copy (NULL is an error; the workspace from *_ws_ex with math | IC_MATH_XB) */
int ic_conv2d_fwd_xb(const ic_act* x, const void* xb, const float* w, const float* b, int k, int stride, int pad,
                     const ic_act* y, int act, int math, void* ws, size_t ws_bytes, void* stream);
int ic_conv_transpose2d_dgrad_xb(const ic_act* dy, const void* dyb, const float* w, int k, int stride, int pad,
                                 const ic_act* dx, int math, void* ws, size_t ws_bytes, void* stream);
/* the same for the phases of a transposed conv forward / conv input gradient (stride-2 sub-pixel phases on
 * the DMA tiles where every phase has >= 256 tiles of 256 rows) */
int ic_conv_transpose2d_fwd_xb(const ic_act* x, const void* xb, const float* w, const float* b, int k, int stride,
                               int pad, const ic_act* y, int act, int math, void* ws, size_t ws_bytes, void* stream);
int ic_conv2d_dgrad_xb(const ic_act* dy, const void* dyb, const float* w, int k, int stride, int pad,
                       const ic_act* dx, int math, void* ws, size_t ws_bytes, void* stream);
/* weight gradients reading both operands' bf16 copies (x's from its producer's forward, dy's from its
 * producer's backward); workspace from *_wgrad_ws_ex */
int ic_conv2d_wgrad_xb(const ic_act* x, const void* xb, const ic_act* dy, const void* dyb, int k, int stride, int pad,
                       float* dw, float* db, int math, void* ws, size_t ws_bytes, void* stream);
int ic_conv_transpose2d_wgrad_xb(const ic_act* x, const void* xb, const ic_act* dy, const void* dyb, int k,
                                 int stride, int pad, float* dw, float* db, int math, void* ws, size_t ws_bytes,
                                 void* stream);

/* ---- launch-plan query: which kernel instance, tile and K / pixel split a conv or GDN op would launch
 *      for these shapes (no launch, no device access; the same decision code as the launching entry
 *      points).  op selects the entry point and the meaning of (a, b):
 *        IC_OP_CONV2D_FWD   a = x,  b = y     IC_OP_TCONV_FWD    a = x,  b = y
 *        IC_OP_CONV2D_DGRAD a = dy, b = dx    IC_OP_TCONV_DGRAD  a = dy, b = dx
 *        IC_OP_CONV2D_WGRAD a = x,  b = dy    IC_OP_TCONV_WGRAD  a = x,  b = dy
 *        IC_OP_GDN_FWD      a = x (b unused; k, stride, pad ignored)    IC_OP_GDN_BWD  likewise
 *      Returns 0 and fills *out, or IC_ERR_ARG for shapes the launch would reject (including tensors
 *      whose element offsets exceed the kernels' 32-bit indexing).  Used by the parity tests to prove
 *      they reach the kernel instances the benchmark runs. */
#define IC_OP_CONV2D_FWD 0
#define IC_OP_CONV2D_DGRAD 1
#define IC_OP_CONV2D_WGRAD 2
#define IC_OP_TCONV_FWD 3
#define IC_OP_TCONV_DGRAD 4
#define IC_OP_TCONV_WGRAD 5
#define IC_OP_GDN_FWD 6
#define IC_OP_GDN_BWD 7
/* kernel ids */
#define IC_KERNEL_IG_FP32 1         /* ig_kernel: implicit GEMM on the fp32 MFMA */
#define IC_KERNEL_IG_FP32_GATHER 2  /* ig_kernel, flattened (tap, channel) gather */
#define IC_KERNEL_IG_BF16 3         /* ig_kernel_bf16: bf16 operands, 64-channel chunks */
#define IC_KERNEL_IG_SPLIT 4        /* ig_kernel_x3s: fp32 by the exact three-term bf16 split */
#define IC_KERNEL_IG_SPLIT_BF16 5   /* ig_kernel_x3s with one bf16 product (bf16 operands) */
#define IC_KERNEL_EDGE_CONV 6       /* edge_conv_kernel: few-channel image -> wide map */
#define IC_KERNEL_IM2COL_GEMM 7     /* im2col columns + ig_kernel */
#define IC_KERNEL_TCONV_FEW 8       /* tconv_few_kernel: wide map -> few-channel image, output-row stationary */
#define IC_KERNEL_TCONV_FEW_ROWS 9  /* tconv_few2_kernel: the same, input-row stationary */
#define IC_KERNEL_GEMM_COL2IM 10    /* ig_kernel + col2im gather */
#define IC_KERNEL_WG_FP32 11        /* wg_kernel: weight gradient on the fp32 MFMA */
#define IC_KERNEL_WG_FP32_GATHER 12 /* wg_kernel, flattened (tap, channel) columns */
#define IC_KERNEL_WG_LDSDMA 13      /* wg_glds_kernel: fp32 MFMA, LDS-DMA staged */
#define IC_KERNEL_WG_SPLIT 14       /* wg_x3d_kernel (two waves per SIMD, maps >= 32 wide) / wg_x3_kernel:
                                       weight gradient in split arithmetic */
#define IC_KERNEL_EDGE_WGRAD 15     /* edge_wgrad_kernel */
#define IC_KERNEL_GDN_FUSED 16      /* gdn_fwd_fused_kernel / gdn_bwd_fused_kernel (fp32 dx) */
#define IC_KERNEL_GDN_FUSED_SPLIT 17 /* gdn_fwd_x3s_kernel / gdn_bwd_fused_kernel with split dgamma */
#define IC_KERNEL_GDN_GEMM 18       /* GDN on the implicit GEMM (+ wgrad kernel for dgamma) */
/* 19: retired (a halo-reusing split kernel, measured slower) */
#define IC_KERNEL_WG_BF16 20        /* wg_x3d_kernel with bf16 operands (one product), fp32 accumulation */
#define IC_KERNEL_GDN_FUSED_BF16 21 /* gdn_bwd_fused_kernel with bf16 operands in both GEMMs */
#define IC_KERNEL_IG_SPLIT_DMA 22   /* ig_kernel_x3d: split arithmetic, 256-row tiles, operands by LDS-DMA */
#define IC_KERNEL_EDGE_CONV_BF16 23 /* edge_conv_x3_kernel with bf16 operands (one product), fp32 accumulation */
#define IC_KERNEL_TCONV_FEW_ROWS_BF16 24 /* tconv_few2_kernel with bf16 operands (one product) */
#define IC_KERNEL_EDGE_WGRAD_BF16 25 /* edge_wgrad_kernel with bf16 operands (one product) */
#define IC_KERNEL_IG_BF16_DMA 26    /* ig_kernel_b16d: bf16 operands, 256-row tiles, operands by LDS-DMA (C3) */
typedef struct ic_plan {
  int kernel;        /* IC_KERNEL_* of the main launch */
  int bm, bn;        /* block tile: output rows (pixels; weight-gradient: G channels) x columns */
  int ksplit;        /* implicit GEMM K splits (1 = none; > 1 adds a deterministic partial-sum pass) */
  int nsplit;        /* weight gradient pixel splits (0 for other ops) */
  int im2col;        /* 1 when a column buffer is materialised in HBM */
  int variant;       /* kernel-specific template variant (weight gradient: 1 = row-fast addressing;
                        edge conv, edge weight gradient, input-row transposed conv: 1 = split arithmetic) */
  long long blocks;  /* workgroups of the main launch (-1 when not reported) */
} ic_plan;
int ic_conv_plan(int op, const ic_act* a, const ic_act* b, int k, int stride, int pad, int math, ic_plan* out);

/* ---- elementwise on dense storage of n elements ---- */
/* NonNegativeParam: v = max(p, bound); out = v*v - ped */
int ic_nonneg_fwd(const float* p, long long n, float bound, float ped, float* out, void* stream);
int ic_nonneg_bwd(const float* p, const float* gout, long long n, float bound, float* gin, void* stream);
/* NonNegativeParam of several tensors in one launch (a training step's GDN gamma / beta:
 * reference gdn.py:59-62, called once per GDN layer): per tensor, backward = 0 -> out = max(p,
 * bound)^2 - pedestal; backward = 1 -> gin = the gradient of ic_nonneg_bwd given gout.  Bitwise the
 * per-tensor entry points. */
typedef struct ic_nonneg_tensor {
  const float* p;
  float* out;          /* forward output (unused in the backward) */
  const float* gout;   /* backward: dL/dout */
  float* gin;          /* backward: dL/dp */
  long long n;
  float bound;
  float pedestal;
} ic_nonneg_tensor;
int ic_nonneg_multi(const ic_nonneg_tensor* tensors, int ntensors, int backward, void* stream);
/* LowerBound (upper=0): max(x,b); UpperBound (upper=1): min(x,b) — with the reference's
 * pass-through gradients */
int ic_bound_fwd(const float* x, long long n, float bound, int upper, float* y, void* stream);
int ic_bound_bwd(const float* x, const float* g, long long n, float bound, int upper, float* gx,
                 void* stream);
int ic_relu_fwd(const float* x, long long n, float* y, void* stream);
int ic_relu_bwd(const float* y, const float* g, long long n, float* gx, void* stream);
int ic_abs_fwd(const float* x, long long n, float* y, void* stream);
int ic_abs_bwd(const float* x, const float* g, long long n, float* gx, void* stream);
/* sigma = clamp(exp(v), lo, hi); saves e = exp(v) for the backward */
int ic_exp_clamp_fwd(const float* v, long long n, float lo, float hi, float* sigma, float* e,
                     void* stream);
int ic_exp_clamp_bwd(const float* e, const float* g, long long n, float lo, float hi, float* gv,
                     void* stream);

/* ---- reductions (deterministic, two-level) ---- */
size_t ic_reduce_ws(long long n);
/* out[0] = sum clamp(-ln(p+1e-10)/ln2, 0, 50) */
int ic_ce_loss_fwd(const float* p, long long n, float* out, void* ws, size_t ws_bytes, void* stream);
/* gp = gout[0] * d/dp (gout: device scalar) */
int ic_ce_loss_bwd(const float* p, const float* gout, long long n, float* gp, void* stream);
/* out[0] = mean((a-b)^2) */
int ic_mse_fwd(const float* a, const float* b, long long n, float* out, void* ws, size_t ws_bytes,
               void* stream);
/* ga = gout*2(a-b)/n (NULL to skip), gb = -ga (NULL to skip) */
int ic_mse_bwd(const float* a, const float* b, const float* gout, long long n, float* ga, float* gb,
               void* stream);

/* ---- noise: the training-noise stream (replaces torch.rand_like of entropy_model.py:230,333).
 *      Element i of stream `seed` is word (i & 3) of Philox4x32-10(counter {i >> 2 as 64 bits, 0, 0},
 *      key {seed lo, seed hi}), mapped to U[0,1) by its top 24 bits: u[i] = element offset + i.
 *      offset must be a multiple of 4 (whole Philox blocks; IC_ERR_ARG otherwise). */
int ic_uniform(float* u, long long n, unsigned long long seed, unsigned long long offset,
               void* stream);
/* raw Philox4x32-10 for known-answer tests: in (device) holds n items {c0, c1, c2, c3, k0, k1},
 * out (device) receives n items {r0, r1, r2, r3} */
int ic_philox_kat(const unsigned* in, unsigned* out, int n, void* stream);
/* graph-safe noise stream: a device-resident state {seed, base}; quantizers in
 * mode 3 draw elements base + offset + i of stream seed.  Advancing the base by the
 * elements one training step consumed is itself a kernel, so a captured
 * hipGraph replays with fresh noise every time.  state[1] += n rounded up to a multiple of 4 */
int ic_philox_advance(unsigned long long* state, unsigned long long n, void* stream);

/* ---- factorized entropy model (z): C channels, elements e with channel c = idx % C
 *      (channels-last storage). params (device, fp32, reference shapes flattened):
 *      w0[C*3] b0[C*3] f0[C*3] w1[C*9] b1[C*3] f1[C*3] w2[C*9] b2[C*3] f2[C*3] w3[C*3] b3[C]
 *      mode: 0 = noise with given u (u in [0,1), y = z + (u - 0.5)), 1 = round,
 *            2 = noise from Philox(seed, offset),
 *            3 = noise from Philox(state[0], state[1] + offset) with `u` pointing to the
 *                device state {seed, base} of ic_philox_advance (`seed` ignored).
 *      Modes 2 and 3 take a 4-aligned offset only (IC_ERR_ARG otherwise) and mode 3 a
 *      4-aligned state[1] (ic_philox_advance keeps it so; a caller writing the state
 *      itself must too): every draw is then whole Philox blocks and every quantizer
 *      kernel maps element i to the same counter */
typedef struct ic_fact_params {
  const float *w0, *b0, *f0, *w1, *b1, *f1, *w2, *b2, *f2, *w3, *b3;
} ic_fact_params;
int ic_factorized_fwd(const float* z, long long n, int C, const ic_fact_params* prm, int mode,
                      const float* u, unsigned long long seed, unsigned long long offset,
                      float* q, float* p, void* stream);
/* given dq (NULL = 0) and dp (NULL = 0): dz (= dq + through p) and per-channel
 * parameter gradients (same layout as params; written, not accumulated) */
typedef struct ic_fact_grads {
  float *w0, *b0, *f0, *w1, *b1, *f1, *w2, *b2, *f2, *w3, *b3;
} ic_fact_grads;
int ic_factorized_bwd(const float* q, long long n, int C, const ic_fact_params* prm,
                      const float* dq, const float* dp, float* dz, const ic_fact_grads* grd,
                      void* stream);

/* ---- factorized entropy model, any CDF MLP (cfg.MODEL.ENTROPY_MODEL.DIMS) and BIN
 *      (modelling/blocks/entropy_model.py:88-99 CDFEstimator, :198 / :229-232 / :259-269 BIN):
 *      layer l maps dims[l] -> dims[l+1] channels-wise, dims = {1, DIMS..., 1}; per layer
 *      w[l] [C][dims[l+1]][dims[l]], b[l] [C][dims[l+1]], f[l] [C][dims[l+1]] (NULL on the last
 *      layer: no gate).  Noise u - bin/2, mass between q -+ bin/2.  Modes as ic_factorized_fwd. */
#define IC_FACT_MAXL 6   /* layers (len(DIMS) + 1) the register kernels take */
#define IC_FACT_MAXW 8   /* hidden width the register kernels take */
#define IC_FACT_NET_MAXL 32   /* layers of ic_fact_net: the wide kernels' limit */
#define IC_FACT_WIDE_MAXW 256 /* hidden width of the wide kernels */
typedef struct ic_fact_net {
  int nlayers;
  int dims[IC_FACT_NET_MAXL + 1];
  const float* w[IC_FACT_NET_MAXL];
  const float* b[IC_FACT_NET_MAXL];
  const float* f[IC_FACT_NET_MAXL];
} ic_fact_net;
typedef struct ic_fact_net_grads {
  float* w[IC_FACT_NET_MAXL];
  float* b[IC_FACT_NET_MAXL];
  float* f[IC_FACT_NET_MAXL];
} ic_fact_net_grads;
/* Geometries within IC_FACT_MAXL layers of width <= IC_FACT_MAXW run the register kernels and need no
 * workspace; larger ones (up to IC_FACT_NET_MAXL layers of width <= IC_FACT_WIDE_MAXW) run the wide
 * kernels, whose workspace ic_factorized_net_ws gives (bwd: 0 forward, 1 backward).  The plain entry
 * points are the _ex ones without a workspace (IC_ERR_WORKSPACE on a wide geometry). */
size_t ic_factorized_net_ws(long long n, int C, const ic_fact_net* net, int bwd);
int ic_factorized_fwd_net(const float* z, long long n, int C, const ic_fact_net* net, float bin, int mode,
                          const float* u, unsigned long long seed, unsigned long long offset, float* q, float* p,
                          void* stream);
int ic_factorized_bwd_net(const float* q, long long n, int C, const ic_fact_net* net, float bin, const float* dq,
                          const float* dp, float* dz, const ic_fact_net_grads* grd, void* stream);
int ic_factorized_fwd_net_ex(const float* z, long long n, int C, const ic_fact_net* net, float bin, int mode,
                             const float* u, unsigned long long seed, unsigned long long offset, float* q, float* p,
                             void* ws, size_t ws_bytes, void* stream);
int ic_factorized_bwd_net_ex(const float* q, long long n, int C, const ic_fact_net* net, float bin, const float* dq,
                             const float* dp, float* dz, const ic_fact_net_grads* grd, void* ws, size_t ws_bytes,
                             void* stream);

/* ---- quantization of the conditional model alone (entropy_model.py:331-336): q = y + (u - bin/2)
 *      (modes 0 / 2 / 3 as ic_conditional_fwd, the same draws element for element) or round(y) (mode 1) */
int ic_quantize(const float* y, long long n, int mode, const float* u, unsigned long long seed,
                unsigned long long offset, float bin, float* q, void* stream);

/* ---- conditional (Laplacian kind=0 / Gaussian kind=1), mean = 0 or tensor ----
 *      q = y + (u - 0.5) (mode 0), round(y) (mode 1), Philox (mode 2), Philox on the
 *      device state `u` (mode 3, as for ic_factorized_fwd)
 *      p = F((0.5-|q-mean|)/scale) - F((-0.5-|q-mean|)/scale) */
int ic_conditional_fwd(const float* y, const float* scale, const float* mean, long long n, int kind,
                       int mode, const float* u, unsigned long long seed,
                       unsigned long long offset, float* q, float* p, void* stream);
int ic_conditional_bwd(const float* q, const float* scale, const float* mean, long long n, int kind,
                       const float* dq, const float* dp, float* dy, float* dscale, float* dmean,
                       void* stream);
/* the same with the quantization bin of cfg.MODEL.ENTROPY_MODEL.BIN (the plain entry points: 1):
 * noise u - bin/2, p = F((bin/2-|q-mean|)/scale) - F((-bin/2-|q-mean|)/scale)
 * (entropy_model.py:278, :331-334, :343-350) */
/* mode 4 (the _bin entry points): y is already quantized, q = y -- the likelihood half of the model
 * after ic_quantize (the model runs the hyperprior on a second stream meanwhile) */
int ic_conditional_fwd_bin(const float* y, const float* scale, const float* mean, long long n, int kind, int mode,
                           const float* u, unsigned long long seed, unsigned long long offset, float bin, float* q,
                           float* p, void* stream);
int ic_conditional_bwd_bin(const float* q, const float* scale, const float* mean, long long n, int kind, float bin,
                           const float* dq, const float* dp, float* dy, float* dscale, float* dmean, void* stream);

/* ---- optimizer: multi-tensor AdamW with fused clip_grad_value_ ----
 * torch.optim.AdamW (solver/optim.py:20-45: per-parameter lr / weight_decay
 * groups) preceded by clip_grad_value_(clip) (engine/trainer.py:189-190; clip
 * <= 0 disables it; clipped gradients are written back).  `step` is the
 * 1-based step count used for the bias corrections (betas in double, like the
 * reference's Python floats).  All pointers device fp32. */
typedef struct ic_adamw_tensor {
  float* param;
  float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  long long n;
  float lr;
  float weight_decay;
} ic_adamw_tensor;
int ic_adamw_step(const ic_adamw_tensor* tensors, int ntensors, double beta1, double beta2, float eps,
                  float clip, long long step, void* stream);

/* ---- SSIM / MS-SSIM (modelling/loss.py:48-188) on [N][C][H][W] contiguous images in [0,1].
 *      nlev levels (MS-SSIM: 5, weights[nlev] host array; single=1 for SSIMLoss, nlev=1).
 *      out: log_scale && single -> out[N] = -log(max(ssim_n, eps)); else out[0] = loss.
 *      single = 2 (with log_scale = 0, eps = 0): the evaluation metric of
 *      utils/metric.py:100-124 — out[N] = -10 log10(1 - prod_l max(cs_l,0)^w_l * max(ssim,0)^w_L)
 *      per image (MS_SSIM(in_dB=True), images scaled by max_val); forward only.
 *      `state` (ic_msssim_state_bytes) is written by fwd and read by bwd. */
size_t ic_msssim_state_bytes(int N, int C, int H, int W, int nlev, int filter_size);
size_t ic_msssim_ws(int N, int C, int H, int W, int nlev, int filter_size);
int ic_msssim_fwd(const float* a, const float* b, int N, int C, int H, int W, int nlev, int filter_size,
                  float filter_sigma, float max_val, int log_scale, int single, float k1, float k2,
                  float eps, const float* weights, float* out, float* state, void* ws, size_t ws_bytes,
                  void* stream);
int ic_msssim_bwd(int N, int C, int H, int W, int nlev, int filter_size, float filter_sigma,
                  float max_val, int log_scale, int single, float k1, float k2, float eps,
                  const float* weights, const float* gout, const float* state, float* ga, float* gb,
                  void* ws, size_t ws_bytes, void* stream);

/* ---- evaluation metric: per-image PSNR in dB (utils/metric.py:26-36) of images scaled by
 *      max_val: out[n] = 10 (2 log10(max_val) - log(mse_n) / ln 10), a, b [N][per_image] ---- */
int ic_psnr(const float* a, const float* b, int N, long long per_image, float max_val, float* out, void* stream);
/* the same over 128 blocks per image: partials in ws (ic_psnr_ws bytes), summed in fixed order
 * (deterministic); N <= 65535 */
size_t ic_psnr_ws(int N, long long per_image);
int ic_psnr_ex(const float* a, const float* b, int N, long long per_image, float max_val, float* out, void* ws,
               size_t ws_bytes, void* stream);

/* ---- host data path: uint8 HWC images (byte strides sn, sh, sw; channel stride 1) -> fp32
 *      NCHW model input (x/255 - mean[c]) / std[c] (transforms.py ToTensor, ChannelFirst,
 *      Normalize; mean/std host arrays of C <= 3 values or NULL for 0 / 1) ---- */
int ic_images_u8_to_input(const unsigned char* x, long long sn, long long sh, long long sw, int N, int C, int H,
                          int W, const float* mean, const float* std, float* y, void* stream);

/* ---- elementwise squared difference (MSE with reduction="none") ---- */
int ic_sqdiff_fwd(const float* a, const float* b, long long n, float* out, void* stream);
int ic_sqdiff_bwd(const float* a, const float* b, const float* g, long long n, float* ga, float* gb,
                  void* stream);

#ifdef __cplusplus
}
#endif
#endif
