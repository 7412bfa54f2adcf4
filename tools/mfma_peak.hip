// MFMA peak microbenchmark for this box ("re-measure with
// an MFMA microbench on the box; report both").  Every SIMD runs waves that
// issue v_mfma_f32_32x32x2_f32 (fp32) or v_mfma_f32_16x16x32_bf16 (the
// instruction fp32_split runs on) back to back on independent accumulators,
// with RANDOM operands (the chip holds a lower clock on random bf16 data than on
// zeros: MI355X_MICROARCH.md, DVFS give-back), and s_memtime brackets each
// wave's loop, so the run also yields the shader clock the MFMAs ran at.
// One JSON line per (instruction, waves per SIMD).
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_peak.hip -o tools/_abl/mfma_peak && tools/_abl/mfma_peak
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float floatx16 __attribute__((ext_vector_type(16)));


__global__ void __launch_bounds__(256) mfma_loop(float* out, unsigned long long* ticks, int ITERS) {
  floatx16 acc[4];
  for (int i = 0; i < 4; ++i)
    for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
  float a = 1.0f + threadIdx.x * 1e-7f, b = 1.0f - threadIdx.x * 1e-7f;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[i], 0, 0, 0);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int i = 0; i < 4; ++i)
    for (int e = 0; e < 16; ++e) s += acc[i][e];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) ticks[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

typedef float floatx4v __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ unsigned hash32(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

__global__ void __launch_bounds__(256) mfma_loop_bf16(float* out, unsigned long long* ticks, int ITERS) {
  // random bf16 operands in [-1, 1), distinct per lane and per register
  bf16x8 a[4], b[4];
  const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
  for (int i = 0; i < 4; ++i)
    for (int e = 0; e < 8; ++e) {
      a[i][e] = (__bf16)((float)(hash32(t * 64 + i * 8 + e) >> 8) * (2.0f / 16777216.0f) - 1.0f);
      b[i][e] = (__bf16)((float)(hash32(t * 64 + 32 + i * 8 + e) >> 8) * (2.0f / 16777216.0f) - 1.0f);
    }
  const floatx4v z = {0.f, 0.f, 0.f, 0.f};
  floatx4v c0 = z, c1 = z, c2 = z, c3 = z, c4 = z, c5 = z, c6 = z, c7 = z;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  // inline asm keeps each accumulator in one AGPR quad (the compiler's own
  // allocation rotated them through copies); 8 independent chains
#define MF(c, x, y) asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(x), "v"(y))
  for (int it = 0; it < ITERS; ++it) {
    MF(c0, a[0], b[0]); MF(c1, a[1], b[0]); MF(c2, a[2], b[1]); MF(c3, a[3], b[1]);
    MF(c4, a[0], b[2]); MF(c5, a[1], b[2]); MF(c6, a[2], b[3]); MF(c7, a[3], b[3]);
  }
#undef MF
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const floatx4v sv = ((c0 + c1) + (c2 + c3)) + ((c4 + c5) + (c6 + c7));
  const float s = sv[0] + sv[1] + sv[2] + sv[3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) ticks[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

#define CK(x) (void)(x)

int main(int argc, char** argv) {
  const int ITERS = argc > 1 ? atoi(argv[1]) : 20000;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  for (int kind = 0; kind < 2; ++kind)
  for (int wps : {1, 2}) {  // waves per SIMD
    const int blocks = cus * wps;  // 4 waves (one per SIMD) per block
    float* out;
    unsigned long long* ticks;
    CK(hipMalloc(&out, (size_t)blocks * 256 * 4));
    CK(hipMalloc(&ticks, (size_t)blocks * 4 * 8));
    const int iters = kind ? ITERS * 4 : ITERS;
    auto launch = [&]() {
      if (kind) hipLaunchKernelGGL(mfma_loop_bf16, dim3(blocks), dim3(256), 0, 0, out, ticks, iters);
      else hipLaunchKernelGGL(mfma_loop, dim3(blocks), dim3(256), 0, 0, out, ticks, iters);
    };
    // >= 2 s of back-to-back launches at full size first: let the clock settle under load
    const auto w0 = std::chrono::steady_clock::now();
    while (std::chrono::duration<double>(std::chrono::steady_clock::now() - w0).count() < 2.0) {
      for (int w = 0; w < 20; ++w) launch();
      CK(hipDeviceSynchronize());
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> t((size_t)blocks * 4);
    CK(hipMemcpy(t.data(), ticks, t.size() * 8, hipMemcpyDeviceToHost));
    double mean = 0;
    for (auto v : t) mean += (double)v;
    mean /= t.size();
    const double nmfma = (double)iters * (kind ? 8 : 4);  // per wave
    const double flop = (double)blocks * 4 * nmfma * (kind ? 16.0 * 16 * 32 * 2 : 32.0 * 32 * 2 * 2);
    const double tf = flop / (ms * 1e-3) / 1e12;
    // cycles per MFMA per SIMD from the wave's own clock
    const double cyc_per_mfma = mean / (nmfma * wps);
    printf("{\"instr\": \"%s\", \"operands\": \"%s\", \"waves_per_simd\": %d, \"cus\": %d, \"ms\": %.3f, \"tflops\": %.1f, \"memtime_ticks_per_wave\": %.0f, "
           "\"clock_ghz_from_memtime\": %.3f, \"cycles_per_mfma_per_simd\": %.1f}\n",
           kind ? "v_mfma_f32_16x16x32_bf16" : "v_mfma_f32_32x32x2_f32", kind ? "random" : "near-constant", wps,
           cus, ms, tf, mean, mean / (ms * 1e-3) / 1e9, cyc_per_mfma);
    CK(hipFree(out));
    CK(hipFree(ticks));
  }
  return 0;
}
