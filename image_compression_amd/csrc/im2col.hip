// Few-channel convolution edges (the 3-channel image at both ends of the
// codec) mapped onto the fast implicit-GEMM / wgrad kernels:
//   im2col : x[n][c][iy][ix] -> xcol[n][gy][gx][(t,c) padded to Kp]  (NHWC, 1x1-conv input)
//   col2im : y[n][b][oy][ox] = bias[b] + sum_t ycol[n][iy][ix][(t,b)]  (sub-pixel gather,
//            deterministic, each ycol element read once)
// so a 3->192 5x5 conv becomes one K=96 GEMM, and a 192->3 transposed conv one
// N=75(->128) GEMM plus this gather, instead of 10x-padded MFMA tiles.
#include "gemm.h"

namespace {

constexpr int MAXKP = 128;  // padded (tap, channel) columns handled by im2col

struct Im2colArgs {
  const float* x;
  int N, C, H, W;
  int Hg, Wg, stride, Kp;
  FastDiv fd_k4, fd_hw, fd_w;
  float* out;
  int koff[MAXKP];           // element offset of column k relative to the pixel's tap-(0,0) origin
                             // kdy == -128 marks a zero (padding) column
  signed char kdy[MAXKP], kdx[MAXKP];
};

// thread = 4 consecutive columns of one output pixel (one float4 store):
// consecutive lanes write consecutive 16 B of the [pixel][Kp] rows.
__global__ void __launch_bounds__(256) im2col_k(const Im2colArgs a, long long sn, long long sh, long long sw) {
  const uint32_t K4 = (uint32_t)a.Kp >> 2;
  const uint32_t total = (uint32_t)a.N * a.Hg * a.Wg * K4;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const uint32_t pix = fdiv(i, a.fd_k4);
    const int k0 = (int)(i - pix * K4) * 4;
    const uint32_t n = fdiv(pix, a.fd_hw);
    const uint32_t rem = pix - n * a.fd_hw.d;
    const uint32_t gy = fdiv(rem, a.fd_w);
    const uint32_t gx = rem - gy * a.fd_w.d;
    const int iy0 = (int)gy * a.stride, ix0 = (int)gx * a.stride;
    const float* xb = a.x + (long long)n * sn + (long long)iy0 * sh + (long long)ix0 * sw;
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = k0 + e;
      const int off = a.koff[k];
      const int iy = iy0 + a.kdy[k], ix = ix0 + a.kdx[k];
      v[e] = (a.kdy[k] != -128 && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W) ? xb[off] : 0.f;
    }
    *(floatx4v*)(a.out + (size_t)pix * a.Kp + k0) = floatx4v{v[0], v[1], v[2], v[3]};
  }
}

struct Col2imArgs {
  const float* ycol;  // [N][Hi][Wi][ncol], column = t*B + b
  const float* bias;
  float* y;
  long long sn, sc, sh, sw;
  int N, B, Ho, Wo, Hi, Wi, ncol, k, stride, pad, act;
  FastDiv fd_b, fd_wo, fd_ho;
};

__global__ void __launch_bounds__(256) col2im_k(const Col2imArgs a) {
  const uint32_t total = (uint32_t)a.N * a.B * a.Ho * a.Wo;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    // i enumerates (n, oy, ox, b) with b fastest: neighbouring lanes read
    // neighbouring columns of the same ycol rows
    const uint32_t r = fdiv(i, a.fd_b);
    const int b = (int)(i - r * a.fd_b.d);
    const uint32_t r2 = fdiv(r, a.fd_wo);
    const int ox = (int)(r - r2 * a.fd_wo.d);
    const uint32_t n = fdiv(r2, a.fd_ho);
    const int oy = (int)(r2 - n * a.fd_ho.d);
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
        v += a.ycol[(((size_t)n * a.Hi + iy) * a.Wi + ix) * a.ncol + (ky * a.k + kx) * a.B + b];
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
  a.x = x; a.N = N; a.C = C; a.H = H; a.W = W;
  a.Hg = Hg; a.Wg = Wg; a.stride = stride; a.Kp = Kp; a.out = out;
  const int T = k * k;
  if (T > IC_MAXT || Kp > MAXKP || Kp % 4 != 0 || T * C > Kp) return IC_ERR_ARG;
  if ((long long)N * Hg * Wg * (Kp / 4) >= (1LL << 31)) return IC_ERR_ARG;  // fdiv range
  for (int kk = 0; kk < Kp; ++kk) {
    const int t = kk / C, c = kk % C;
    if (t < T) {
      const int dy = t / k - pad, dx = t % k - pad;
      a.kdy[kk] = (signed char)dy; a.kdx[kk] = (signed char)dx;
      // relative to the tap-(0,0) pixel; may be negative (bounds are tested on iy/ix)
      const long long off = c * sc + dy * sh + dx * sw;
      if (off < -(1LL << 30) || off > (1LL << 30)) return IC_ERR_ARG;
      a.koff[kk] = (int)off;
    } else {
      a.kdy[kk] = -128; a.kdx[kk] = 0; a.koff[kk] = 0;  // zero column
    }
  }
  a.fd_k4 = make_fastdiv((uint32_t)(Kp / 4));
  a.fd_hw = make_fastdiv((uint32_t)(Hg * Wg));
  a.fd_w = make_fastdiv((uint32_t)Wg);
  hipLaunchKernelGGL(im2col_k, dim3(grid_for((long long)N * Hg * Wg * (Kp / 4))), dim3(256), 0, s, a, sn, sh, sw);
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
  if ((long long)N * B * Ho * Wo >= (1LL << 31)) return IC_ERR_ARG;  // fdiv range
  a.fd_b = make_fastdiv((uint32_t)B);
  a.fd_wo = make_fastdiv((uint32_t)Wo);
  a.fd_ho = make_fastdiv((uint32_t)Ho);
  hipLaunchKernelGGL(col2im_k, dim3(grid_for((long long)N * B * Ho * Wo)), dim3(256), 0, s, a);
  IC_CHECK_LAUNCH();
  return IC_OK;
}
