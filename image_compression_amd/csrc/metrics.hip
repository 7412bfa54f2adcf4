// Evaluation metrics and the host data path's device half.
//
//   ic_psnr        per-image PSNR in dB of two [N][...] fp32 images in [0,1]
//                  scaled by max_val: utils/metric.py:26-36
//                  10 * (2 log10(max) - log(mean((max a - max b)^2)) / ln 10)
//   ic_psnr_ex     the same over PSNR_NB blocks per image (partials in a workspace, summed in
//                  fixed order by a second launch: deterministic); ic_psnr's one block per
//                  image took 1.6 ms on a 512x768 Kodak image (r03zr)
//   ic_images_u8_to_input
//                  uint8 HWC crops -> fp32 NCHW model input:
//                  data_utils/transforms/transforms.py ToTensor + ChannelFirst +
//                  Normalize (x / 255 - mean) / std, so a loader ships 1 byte per
//                  channel over PCIe and the device expands it (4x less H2D).
#include "../../include/imgcomp.h"
#include "common.h"

namespace {

// one block per image, fixed-order reduction (deterministic)
__global__ void __launch_bounds__(256) psnr_kernel(const float* a, const float* b, long long per, float max_val,
                                                   float* out) {
  __shared__ float lds[16];
  const float* pa = a + (long long)blockIdx.x * per;
  const float* pb = b + (long long)blockIdx.x * per;
  float acc[1] = {0.f};
  for (long long i = threadIdx.x; i < per; i += 256) {
    const float d = max_val * pa[i] - max_val * pb[i];
    acc[0] += d * d;
  }
  block_sum<1>(acc, lds);
  if (threadIdx.x == 0) {
    const float mse = acc[0] / (float)per;
    out[blockIdx.x] = 10.f * (2.f * log10f(max_val) - logf(mse) / 2.302585092994046f);
  }
}

// partial sums of squared scaled differences: block (b, n) takes elements [b*chunk, (b+1)*chunk)
// of image n, float4 loads when `vec`
constexpr int PSNR_NB = 128;
__global__ void __launch_bounds__(256) psnr_partial_kernel(const float* a, const float* b, long long per,
                                                           long long chunk, int vec, float max_val, float* part) {
  __shared__ float lds[16];
  const int n = blockIdx.y;
  const long long lo = (long long)blockIdx.x * chunk, hi = min(per, lo + chunk);
  const float* pa = a + (long long)n * per;
  const float* pb = b + (long long)n * per;
  float acc[1] = {0.f};
  if (vec) {
    for (long long i = lo + 4 * threadIdx.x; i < hi; i += 1024) {
      const floatx4v va = *(const floatx4v*)(pa + i), vb = *(const floatx4v*)(pb + i);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float d = max_val * va[r] - max_val * vb[r];
        acc[0] += d * d;
      }
    }
  } else {
    for (long long i = lo + threadIdx.x; i < hi; i += 256) {
      const float d = max_val * pa[i] - max_val * pb[i];
      acc[0] += d * d;
    }
  }
  block_sum<1>(acc, lds);
  if (threadIdx.x == 0) part[n * PSNR_NB + blockIdx.x] = acc[0];
}

__global__ void __launch_bounds__(64) psnr_final_kernel(const float* part, long long per, float max_val, float* out) {
  if (threadIdx.x != 0) return;
  double s = 0.0;
  for (int i = 0; i < PSNR_NB; ++i) s += part[blockIdx.x * PSNR_NB + i];
  const float mse = (float)(s / (double)per);
  out[blockIdx.x] = 10.f * (2.f * log10f(max_val) - logf(mse) / 2.302585092994046f);
}

// x[n][h][w][c] uint8 (any pixel/row/image strides in bytes) -> y[n][c][h][w] fp32
__global__ void u8_to_input_kernel(const uint8_t* x, long long sn, long long sh, long long sw, int N, int C, int H,
                                   int W, float m0, float m1, float m2, float s0, float s1, float s2, float* y) {
  const long long total = (long long)N * C * H * W;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int w = (int)(i % W);
    long long r = i / W;
    const int h = (int)(r % H);
    r /= H;
    const int c = (int)(r % C);
    const int n = (int)(r / C);
    const float v = (float)x[n * sn + h * sh + w * sw + c] / 255.f;
    const float m = c == 0 ? m0 : (c == 1 ? m1 : m2);
    const float sd = c == 0 ? s0 : (c == 1 ? s1 : s2);
    y[i] = (v - m) / sd;
  }
}

}  // namespace

extern "C" {

size_t ic_psnr_ws(int N, long long per_image) {
  (void)per_image;
  return N < 1 ? 0 : (size_t)N * PSNR_NB * sizeof(float);
}

int ic_psnr_ex(const float* a, const float* b, int N, long long per_image, float max_val, float* out, void* ws,
               size_t ws_bytes, void* stream) {
  if (N < 1 || per_image < 1 || N > 65535) return IC_ERR_ARG;
  if (!ws || ws_bytes < ic_psnr_ws(N, per_image)) return IC_ERR_WORKSPACE;
  long long chunk = (per_image + PSNR_NB - 1) / PSNR_NB;
  chunk = (chunk + 3) & ~3LL;  // float4 chunks stay 16-B aligned
  const int vec = (per_image % 4 == 0) && ((uintptr_t)a % 16 == 0) && ((uintptr_t)b % 16 == 0);
  hipLaunchKernelGGL(psnr_partial_kernel, dim3(PSNR_NB, N), dim3(256), 0, (hipStream_t)stream, a, b, per_image,
                     chunk, vec, max_val, (float*)ws);
  IC_CHECK_LAUNCH();
  hipLaunchKernelGGL(psnr_final_kernel, dim3(N), dim3(64), 0, (hipStream_t)stream, (const float*)ws, per_image,
                     max_val, out);
  IC_CHECK_LAUNCH();
  return IC_OK;
}

int ic_psnr(const float* a, const float* b, int N, long long per_image, float max_val, float* out, void* stream) {
  if (N < 1 || per_image < 1) return IC_ERR_ARG;
  hipLaunchKernelGGL(psnr_kernel, dim3(N), dim3(256), 0, (hipStream_t)stream, a, b, per_image, max_val, out);
  IC_CHECK_LAUNCH();
  return IC_OK;
}

int ic_images_u8_to_input(const unsigned char* x, long long sn, long long sh, long long sw, int N, int C, int H, int W,
                          const float* mean, const float* std, float* y, void* stream) {
  if (C < 1 || C > 3) return IC_ERR_ARG;
  float m[3] = {0.f, 0.f, 0.f}, sd[3] = {1.f, 1.f, 1.f};
  for (int c = 0; c < C; ++c) {
    m[c] = mean ? mean[c] : 0.f;
    sd[c] = std ? std[c] : 1.f;
  }
  const long long total = (long long)N * C * H * W;
  long long blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) return IC_OK;
  hipLaunchKernelGGL(u8_to_input_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, x, sn, sh, sw,
                     N, C, H, W, m[0], m[1], m[2], sd[0], sd[1], sd[2], y);
  IC_CHECK_LAUNCH();
  return IC_OK;
}

}  // extern "C"
