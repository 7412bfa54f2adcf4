// Internal descriptors of the two gather-GEMM kernel families.
//
//  (1) ig_*  "implicit GEMM" output-stationary convolution:
//        out[m][n] = sum_k A[m][k] * Bt[n][k]
//      m = output grid pixel (img, gy, gx) of one sub-pixel phase,
//      k = (tap t, input channel c); A[m][(t,c)] = x[img, gy*s+dy_t, gx*s+dx_t, c]
//      (zero outside the image), Bt = packed weights [T][Npad][Cin].
//      A stride-s transposed conv (= conv dgrad) is up to s*s phases, each a
//      dense stride-1 gather conv with 2..3 x 2..3 taps (no zero stuffing).
//  (2) wg_*  weight gradient (split-K over pixels):
//        dW[g][(t,c)] = sum_p G[p][g] * X[p*s + d_t][c]
#pragma once
#include "common.h"
#include "../../include/imgcomp.h"

enum IgEpilogue {
  EPI_NONE = 0,
  EPI_RELU = 1,
  EPI_GDN = 2,        // y = aux0 / sqrt(v),  aux_out = v (norm)
  EPI_IGDN = 3,       // y = aux0 * sqrt(v),  aux_out = v
  EPI_GDN_BWD = 4,    // y = aux2 / sqrt(aux1) + 2*aux0*v
  EPI_IGDN_BWD = 5    // y = aux2 * sqrt(aux1) + 2*aux0*v
};
enum IgAOp { AOP_NONE = 0, AOP_SQUARE = 1, AOP_ABS = 2 };

struct IgPhase {
  const float* wp;  // fast: [T][Npad][Cin]; generic: [Npad][Kpad]
  int T;
  int Hg, Wg;       // output grid of this phase
  int oys, oxs, oy0, ox0;  // output pixel = (gy*oys+oy0, gx*oxs+ox0)
  int mtiles;
  long long m_off;  // row offset of this phase inside the split-K partial buffer
  FastDiv fd_hw, fd_w;  // divide by Hg*Wg and by Wg
  int dy[IC_MAXT], dx[IC_MAXT];
};

struct IgDesc {
  const float* x;
  long long xs_n, xs_h, xs_w, xs_c;
  int Hx, Wx, Cin;
  int N, stride;
  int Cout, Npad, Kc;  // Kc: fast = Cin, generic = Kpad (T*Cin rounded up to 32)
  int generic;
  float* y;
  long long ys_n, ys_h, ys_w, ys_c;
  const float* bias;
  int epi, a_op;
  const float* aux0;
  const float* aux1;
  const float* aux2;
  float* aux_out;
  int nphase;
  int ksplit, kcps;  // K splits and K-chunks (of 32) per split
  float* partial;    // [ksplit][Mtot][Cout]
  long long Mtot;
  int bm, bn;        // chosen tile (set by ig_plan)
  int bf16;          // bf16 operands, fp32 accumulation (fast path, Cin % 64 == 0); wp holds bf16
  int dma;           // split tiles of 256 rows on ig_kernel_x3d (set by ig_plan)
  int x3;            // fp32 by exact three-term bf16 split (fast path, Cin % 32 == 0); wp holds three
                     // bf16 planes [part][t][Npad][Cin], part p at wp + p * wplane (bf16 elements)
  long long wplane;
  const void* xb;    // with bf16 && dma: x as compact NHWC bf16 (ig_kernel_b16d's A operand), same element offsets
  int b16d_ok;       // the caller provides xb when ig_plan picks the bf16 DMA tiles (direct_impl)
  IgPhase ph[IC_MAXPH];
};

// Fill tile choice, mtiles, split-K; returns partial-buffer bytes needed.
size_t ig_plan(IgDesc& d);
int ig_run(IgDesc& d, hipStream_t s);
// x (compact NHWC fp32, n elements, n % 8 == 0) -> xb (bf16, round to nearest even)
int ig_cvt_bf16(const float* x, void* xb, long long n, hipStream_t s);
// IC_KERNEL_* that ig_run launches for a planned descriptor, and its grid size
int ig_kernel_kind(const IgDesc& d);
long long ig_grid_blocks(const IgDesc& d);
// N padding the packed-weight layout must use for `Cout`
int ig_npad(int Cout);

struct WgDesc {
  const float* g;
  long long gs_n, gs_h, gs_w, gs_c;
  int Hg, Wg, Cg;
  const float* x;
  long long xs_n, xs_h, xs_w, xs_c;
  int Hx, Wx, Cx;
  int N, stride, T;
  int x_op;        // AOP_SQUARE -> x^2
  int g_vec;       // G rows channel-contiguous (float4 loads)
  int generic;     // columns = (t, c) flattened
  int ncols;       // fast: Cx ; generic: T*Cx
  int bm, bn;
  int mtiles, ntiles;
  long long P;     // N*Hg*Wg
  int pps, nsplit; // pixels per split, number of splits
  FastDiv fd_hw, fd_w;  // divide a pixel index by Hg*Wg and by Wg (set by wg_run)
  int rowfast;     // Wg and pixels-per-split multiples of the 16-pixel K step (set by wg_run)
  float* partial;  // [nsplit][Tp][Cg][ncols]
  int x3;          // fp32 by exact three-term bf16 split (wg_x3_kernel); cleared by wg_plan when unsupported
  int bf16;        // with x3: bf16 operands on the two-wave kernel (wg_x3d_kernel<..., 1>); cleared by wg_plan
                   // where that kernel does not run
  int split_ok;    // split arithmetic allowed (IC_MATH_SPLIT): wg_plan's fallback when bf16 is cleared
  const void* g16; // with bf16: G and X as bf16 copies (compact NHWC, the fp32 tensors' element offsets),
  const void* x16; //   read by the producer waves of wg_x3p_kernel instead of converting (C3, round 5)
  int dy[IC_MAXT], dx[IC_MAXT];
};

size_t wg_plan(WgDesc& d);
int wg_run(WgDesc& d, hipStream_t s);
// launch-time fields (fast divisors, row-fast mode); then the IC_KERNEL_* wg_run launches and its grid
void wg_prepare(WgDesc& d);
int wg_kernel_kind(const WgDesc& d);
long long wg_grid_blocks(const WgDesc& d);

// launch-plan reporting (ic_conv_plan): set for the calling thread by the query entry point; the
// ops' workspace-query paths fill it when it is non-null
extern thread_local ic_plan* g_plan_sink;
static inline void plan_report(int kernel, int bm, int bn, int ksplit, int nsplit, int im2col, long long blocks,
                               int variant = 0) {
  if (!g_plan_sink) return;
  g_plan_sink->kernel = kernel; g_plan_sink->bm = bm; g_plan_sink->bn = bn; g_plan_sink->ksplit = ksplit;
  g_plan_sink->nsplit = nsplit; g_plan_sink->im2col = im2col; g_plan_sink->blocks = blocks;
  g_plan_sink->variant = variant;
}
// element offsets the kernels index with 32-bit arithmetic: every addressed element of `a` below 2^31
static inline bool act_fits32(const ic_act* a) {
  if (a->n < 0 || a->c < 0 || a->h < 0 || a->w < 0) return false;
  long long mx = 0;
  const long long ext[4] = {a->n, a->c, a->h, a->w}, st[4] = {a->sn, a->sc, a->sh, a->sw};
  for (int i = 0; i < 4; ++i) {
    if (ext[i] > 1) mx += (ext[i] - 1) * (st[i] < 0 ? -st[i] : st[i]);
  }
  return mx < (1LL << 31) && (long long)a->n * a->h * a->w < (1LL << 31);
}
// out[g][c][kk(t)] (+)= sum over splits; kk_of_t maps tap -> ky*k+kx, kk = k*k
int wg_reduce(const WgDesc& d, float* out, const int* kk_of_t, int kk, hipStream_t s);

// column sums: out[c] = scale * sum over pixels of t[n,c,h,w]
size_t colsum_ws(long long rows, int C);
int colsum(const float* t, long long s_n, long long s_c, long long s_h, long long s_w,
           int N, int C, int H, int W, float* out, float scale, void* ws, hipStream_t s);

// weight packing
//  mode 0 (direct):     wp[t][a][b]   = W[a][b][ky_t][kx_t]   (out ch a, reduce b)
//  mode 1 (transposed): wp[t][b][a]   = W[a][b][ky_t][kx_t]   (out ch b, reduce a)
//  generic: the (t, reduce-ch) pair is flattened into a Kpad-long row.
//  mode 2 (scatter):    wp[0][t*B + b][a] = W[a][b][ky_t][kx_t]   (rows n >= T*B zero)
int pack_weights(const float* W, int A, int B, int k, int mode, int generic,
                 int T, const int* ky, const int* kx, int Npad, int Kpad,
                 float* wp, hipStream_t s, int out_bf16 = 0);
// out_bf16: 1 -> wp is __bf16[] (rounded); 2 -> wp is three __bf16 planes (exact split
// w = w0 + w1 + w2, plane stride = the pack's element count)

// few-channel edges (im2col.hip)
int im2col_run(const float* x, long long sn, long long sc, long long sh, long long sw, int N, int C, int H,
               int W, int Hg, int Wg, int stride, int k, int pad, int Kp, float* out, hipStream_t s);
int col2im_run(const float* ycol, int ncol, int N, int Hi, int Wi, const float* bias, float* y, long long sn,
               long long sc, long long sh, long long sw, int B, int Ho, int Wo, int k, int stride, int pad,
               int act, hipStream_t s);

// fused GDN (gdn_fused.hip): NHWC-dense, C in {64,128,192}
bool gdn_fused_ok(const float* x, const float* y, const float* norm, int C, long long sc, long long sw, long long sh,
                  long long sn, int H, int W, long long P);
int gdn_fwd_fused(const float* x, const float* gamma, const float* beta, int inverse, float* y, float* norm, int C,
                  long long P, hipStream_t s, int split = 0,  // split: C = 192 in split arithmetic
                  void* yb = nullptr);                         // with split 2 (bf16): y's bf16 copy too;
                                                               // split 2 with norm == nullptr: no norm
size_t gdn_bwd_fused_ws(int C, long long P);
int gdn_bwd_fused(const float* x, const float* norm, const float* dy, const float* gamma, int inverse, float* dx,
                  float* dgamma, float* dbeta, int C, long long P, void* ws, hipStream_t s, int split = 0,
                  float* dxsum = nullptr,   // split: 1 split dgamma, 2 bf16 operands in both GEMMs (C = 192);
                  void* dxb = nullptr,      // dxsum: column sums of dx over all pixels (C), when non-null;
                                            // dxb (split 2): dx's bf16 copy too
                  const float* beta = nullptr);  // split 2 with norm == nullptr: norm recomputed from
                                                 // x, gamma and beta (C = 192)

// image-edge convolutions (edge.hip): few-channel NCHW image <-> wide NHWC maps
bool edge_conv_ok(int C, int k, int stride, long long sw, long long ys_c, int Cout, long long ys_w, long long ys_h,
                  long long ys_n);
// the split edge conv runs for these (IC_MATH_SPLIT, T*C <= 96)
bool edge_conv_split(int split, int TC, int Cout);
int edge_conv_run(const float* x, long long sn, long long sc, long long sh, long long sw, int N, int C, int H, int W,
                  const float* wp, int Kp, const float* bias, int k, int stride, int pad, float* y, long long ys_n,
                  long long ys_c, long long ys_h, long long ys_w, int Cout, int Ho, int Wo, int relu, hipStream_t s,
                  int split = 0);  // split: IC_MATH_SPLIT
bool edge_wgrad_ok(int C, int k, int stride, long long sw, const float* G, int CG, long long gs_c, long long gs_w,
                   long long gs_h, long long gs_n, int Ho, int Wo);
long long edge_units(int N, int Ho, int Wo);
bool tconv_few_ok(int Cin, int Cout, int k, int stride, int pad, long long xsc, long long xsw, long long xsh,
                  long long xsn, int Hin, int Win);
int tconv_few_run(const float* x, int N, int Hin, int Win, int Cin, const float* W, int Cout, int k, int pad,
                  const float* bias, int relu, float* y, long long ysn, long long ysc, long long ysh, long long ysw,
                  int Hout, int Wout, hipStream_t s, int split = 0);  // split: IC_MATH_SPLIT (input-row kernel)
// IC_KERNEL_TCONV_FEW_ROWS or IC_KERNEL_TCONV_FEW: which one tconv_few_run launches
int tconv_few_kind(int Hin, int Win, int k, int pad, int Hout);
// ic_conv_plan for GDN (gdn.hip): reports through g_plan_sink
int gdn_plan(int bwd, const ic_act* x, int math);
size_t edge_wgrad_ws(int CG, int Kc, long long units);
int edge_wgrad_run(const float* G, int CG, const float* x, long long sn, long long sc, long long sh, long long sw,
                   int N, int C, int H, int W, int Ho, int Wo, int k, int stride, int pad, float* dw, float* db,
                   void* ws, hipStream_t s, int split = 0);  // split: IC_MATH_SPLIT
