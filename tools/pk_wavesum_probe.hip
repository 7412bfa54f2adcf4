// fact_bwd_k's reduction pattern in isolation (round-3 verdict item 1): every thread of a 256-thread
// block holds 43 fp32 accumulators, updates them with outer-product FMAs (what the compiler packs
// into v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32 in fact_bwd_k's mlp_bwd), and reduces them with
// the same block_sum as entropy.hip (wave_sum through ds_bpermute, then LDS); the block's 43 sums are
// written per iteration.  The same launch on an idle GPU and beside a hog on another stream (MFMA
// loop, or nothing) must give bitwise equal outputs.  Built twice by tools/_abl/run scripts: with
// packed fp32 (compiler default) and with -packed-fp32-ops disabled.
//   hipcc --offload-arch=gfx950 -O3 tools/pk_wavesum_probe.hip -o tools/_abl/pk_wavesum_pk
//   hipcc --offload-arch=gfx950 -O3 -Xclang -target-feature -Xclang -packed-fp32-ops tools/pk_wavesum_probe.hip \
//         -o tools/_abl/pk_wavesum_nopk
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../image_compression_amd/csrc/common.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

constexpr int NG = 43;

__device__ __forceinline__ float hashf(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return (float)(x >> 8) * (1.0f / 16777216.0f) - 0.5f;
}

// per iteration: every thread forms h0[3], da1[3], h1[3], da2[3] and accumulates the 3x3 outer
// products into G[9..17] / G[24..32] (as mlp_bwd), the rest into the other slots; block_sum; thread 0
// writes the 43 sums of this (block, iteration)
__global__ void __launch_bounds__(256) probe(float* out, int iters) {
  __shared__ float lds[16 * NG];
  const unsigned t = blockIdx.x * 256 + threadIdx.x;
  for (int it = 0; it < iters; ++it) {
    float G[NG];
#pragma unroll
    for (int j = 0; j < NG; ++j) G[j] = 0.f;
    for (int e = 0; e < 2; ++e) {
      const unsigned s = (t * 977u + it * 131u + e * 7u) * 16u;
      float h0[3], da1[3], h1[3], da2[3];
#pragma unroll
      for (int o = 0; o < 3; ++o) {
        h0[o] = hashf(s + o);
        da1[o] = hashf(s + 3 + o) * 1e-3f;
        h1[o] = h0[o] + tanhf(h0[o]) * 0.3f;
        da2[o] = da1[o] * (1.f + (1.f - h1[o] * h1[o]) * 0.2f);
      }
#pragma unroll
      for (int o = 0; o < 3; ++o)
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          G[9 + o * 3 + i] += da1[o] * h0[i];
          G[24 + o * 3 + i] += da2[o] * h1[i];
        }
#pragma unroll
      for (int o = 0; o < 3; ++o) {
        G[o] += da1[o] * h0[o];
        G[3 + o] += da1[o];
        G[6 + o] += da2[o] * h1[o];
        G[18 + o] += da2[o];
        G[21 + o] += da1[o] * h1[o];
        G[33 + o] += da2[o] * h0[o];
        G[36 + o] += h1[o] * 1e-3f;
        G[39 + o] += h0[o] * da2[o];
      }
      G[42] += da1[0] + da2[2];
    }
    block_sum<NG>(G, lds);
    if (threadIdx.x == 0) {
#pragma unroll
      for (int j = 0; j < NG; ++j) out[((size_t)blockIdx.x * iters + it) * NG + j] = G[j];
    }
  }
}

__global__ void __launch_bounds__(256) hog_mfma(float* out, int iters) {
  bf16x8 a, b;
  for (int e = 0; e < 8; ++e) {
    a[e] = (__bf16)hashf(threadIdx.x * 8 + e);
    b[e] = (__bf16)hashf(threadIdx.x * 8 + e + 4096);
  }
  floatx4v c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  for (int i = 0; i < iters; ++i) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c0) : "v"(a), "v"(b));
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c1) : "v"(a), "v"(b));
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c2) : "v"(a), "v"(b));
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c3) : "v"(a), "v"(b));
  }
  const floatx4v s = (c0 + c1) + (c2 + c3);
  out[blockIdx.x * blockDim.x + threadIdx.x] = s[0] + s[1] + s[2] + s[3];
}

int main(int argc, char** argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 192;  // one block per C2 channel, as fact_bwd_k
  const int iters = argc > 2 ? atoi(argv[2]) : 64;
  const int reps = argc > 3 ? atoi(argv[3]) : 50;
  const int hog_iters = argc > 4 ? atoi(argv[4]) : 100000;
  const size_t n = (size_t)blocks * iters * NG;
  float *ref, *got, *hout;
  CK(hipMalloc(&ref, n * 4));
  CK(hipMalloc(&got, n * 4));
  CK(hipMalloc(&hout, 256 * 256 * 4));
  hipStream_t sh, sp;
  CK(hipStreamCreateWithFlags(&sh, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sp, hipStreamNonBlocking));
  hipLaunchKernelGGL(probe, dim3(blocks), dim3(256), 0, sp, ref, iters);
  CK(hipDeviceSynchronize());
  std::vector<float> hr(n), hg(n);
  CK(hipMemcpy(hr.data(), ref, n * 4, hipMemcpyDeviceToHost));
  const char* hogs[2] = {"none", "mfma"};
  for (int hog = 0; hog < 2; ++hog) {
    long long bad_launch = 0, bad_elem = 0;
    for (int r = 0; r < reps; ++r) {
      if (hog) hipLaunchKernelGGL(hog_mfma, dim3(256), dim3(256), 0, sh, hout, hog_iters);
      for (int k = 0; k < 4; ++k) {
        hipLaunchKernelGGL(probe, dim3(blocks), dim3(256), 0, sp, got, iters);
        CK(hipStreamSynchronize(sp));
        CK(hipMemcpy(hg.data(), got, n * 4, hipMemcpyDeviceToHost));
        long long b = 0;
        for (size_t i = 0; i < n; ++i) b += memcmp(&hr[i], &hg[i], 4) != 0;
        bad_elem += b;
        bad_launch += b != 0;
      }
      CK(hipDeviceSynchronize());
    }
    printf("{\"probe\": \"wavesum\", \"hog\": \"%s\", \"launches\": %d, \"mismatching_launches\": %lld, "
           "\"mismatching_sums\": %lld, \"sums_per_launch\": %zu}\n",
           hogs[hog], reps * 4, bad_launch, bad_elem, n);
    fflush(stdout);
  }
  return 0;
}
