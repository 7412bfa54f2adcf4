// Few-channel convolution edges (the 3-channel image at both ends of the
// codec) mapped onto the fast implicit-GEMM / wgrad kernels:
//   im2col : x[n][c][iy][ix] -> xcol[n][gy][gx][(t,c) padded to Kp]  (NHWC, 1x1-conv input)
//   col2im : y[n][b][oy][ox] = bias[b] + sum_t ycol[n][iy][ix][(t,b)]  (sub-pixel gather,
//            deterministic, each ycol element read once)
// so a 3->192 5x5 conv becomes one K=96 GEMM, and a 192->3 transposed conv one
// N=75(->128) GEMM plus this gather, instead of 10x-padded MFMA tiles.
#include "gemm.h"

namespace {

struct Im2colArgs {
  const float* x;
  long long sn, sc, sh, sw;
  int N, C, H, W;
  int Hg, Wg, stride, Kp, T;
  float* out;
  int dy[IC_MAXT], dx[IC_MAXT];
};

__global__ void im2col_k(const Im2colArgs a) {
  const long long total = (long long)a.N * a.Hg * a.Wg * a.Kp;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int k = (int)(i % a.Kp);
    const long long pix = i / a.Kp;
    const int gx = (int)(pix % a.Wg);
    const long long t2 = pix / a.Wg;
    const int gy = (int)(t2 % a.Hg);
    const int n = (int)(t2 / a.Hg);
    const int t = k / a.C, c = k - (k / a.C) * a.C;
    float v = 0.f;
    if (t < a.T) {
      const int iy = gy * a.stride + a.dy[t], ix = gx * a.stride + a.dx[t];
      if ((unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W)
        v = a.x[n * a.sn + c * a.sc + (long long)iy * a.sh + (long long)ix * a.sw];
    }
    a.out[i] = v;
  }
}

struct Col2imArgs {
  const float* ycol;  // [N][Hi][Wi][ncol], column = t*B + b
  const float* bias;
  float* y;
  long long sn, sc, sh, sw;
  int N, B, Ho, Wo, Hi, Wi, ncol, k, stride, pad, act;
};

__global__ void col2im_k(const Col2imArgs a) {
  const long long total = (long long)a.N * a.B * a.Ho * a.Wo;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(i % a.B);
    const long long r = i / a.B;
    const int ox = (int)(r % a.Wo);
    const long long r2 = r / a.Wo;
    const int oy = (int)(r2 % a.Ho);
    const int n = (int)(r2 / a.Ho);
    float v = 0.f;
    for (int ky = 0; ky < a.k; ++ky) {
      const int ny = oy + a.pad - ky;
      if (ny < 0 || ny % a.stride) continue;
      const int iy = ny / a.stride;
      if (iy >= a.Hi) continue;
      for (int kx = 0; kx < a.k; ++kx) {
        const int nx = ox + a.pad - kx;
        if (nx < 0 || nx % a.stride) continue;
        const int ix = nx / a.stride;
        if (ix >= a.Wi) continue;
        v += a.ycol[(((long long)n * a.Hi + iy) * a.Wi + ix) * a.ncol + (ky * a.k + kx) * a.B + b];
      }
    }
    if (a.bias) v += a.bias[b];
    if (a.act) v = v > 0.f ? v : 0.f;
    a.y[n * a.sn + b * a.sc + (long long)oy * a.sh + (long long)ox * a.sw] = v;
  }
}

inline unsigned grid_for(long long n) {
  long long b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  return (unsigned)b;
}

}  // namespace

int im2col_run(const float* x, long long sn, long long sc, long long sh, long long sw, int N, int C, int H,
               int W, int Hg, int Wg, int stride, int k, int pad, int Kp, float* out, hipStream_t s) {
  Im2colArgs a;
  a.x = x; a.sn = sn; a.sc = sc; a.sh = sh; a.sw = sw; a.N = N; a.C = C; a.H = H; a.W = W;
  a.Hg = Hg; a.Wg = Wg; a.stride = stride; a.Kp = Kp; a.T = k * k; a.out = out;
  if (a.T > IC_MAXT) return IC_ERR_ARG;
  for (int t = 0; t < a.T; ++t) { a.dy[t] = t / k - pad; a.dx[t] = t % k - pad; }
  hipLaunchKernelGGL(im2col_k, dim3(grid_for((long long)N * Hg * Wg * Kp)), dim3(256), 0, s, a);
  IC_CHECK_LAUNCH();
  return IC_OK;
}

int col2im_run(const float* ycol, int ncol, int N, int Hi, int Wi, const float* bias, float* y, long long sn,
               long long sc, long long sh, long long sw, int B, int Ho, int Wo, int k, int stride, int pad,
               int act, hipStream_t s) {
  Col2imArgs a;
  a.ycol = ycol; a.bias = bias; a.y = y; a.sn = sn; a.sc = sc; a.sh = sh; a.sw = sw;
  a.N = N; a.B = B; a.Ho = Ho; a.Wo = Wo; a.Hi = Hi; a.Wi = Wi; a.ncol = ncol; a.k = k; a.stride = stride;
  a.pad = pad; a.act = act;
  hipLaunchKernelGGL(col2im_k, dim3(grid_for((long long)N * B * Ho * Wo)), dim3(256), 0, s, a);
  IC_CHECK_LAUNCH();
  return IC_OK;
}
