// Evaluation metrics and the host data path's device half.
//
//   ic_psnr        per-image PSNR in dB of two [N][...] fp32 images in [0,1]
//                  scaled by max_val: utils/metric.py:26-36
//                  10 * (2 log10(max) - log(mean((max a - max b)^2)) / ln 10)
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
