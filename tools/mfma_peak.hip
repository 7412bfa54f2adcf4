// fp32 MFMA peak microbenchmark for this box ("re-measure with
// an MFMA microbench on the box; report both").  Every SIMD runs waves that
// issue v_mfma_f32_32x32x2_f32 back to back on independent accumulators, and
// s_memtime brackets each wave's loop, so the run also yields the shader clock
// the MFMAs actually ran at.
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_peak.hip -o tools/_abl/mfma_peak && tools/_abl/mfma_peak
#include <hip/hip_runtime.h>
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

#define CK(x) (void)(x)

int main(int argc, char** argv) {
  const int ITERS = argc > 1 ? atoi(argv[1]) : 20000;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  for (int wps : {1, 2}) {  // waves per SIMD
    const int blocks = cus * wps;  // 4 waves (one per SIMD) per block
    float* out;
    unsigned long long* ticks;
    CK(hipMalloc(&out, (size_t)blocks * 256 * 4));
    CK(hipMalloc(&ticks, (size_t)blocks * 4 * 8));
    hipLaunchKernelGGL(mfma_loop, dim3(blocks), dim3(256), 0, 0, out, ticks, ITERS);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(mfma_loop, dim3(blocks), dim3(256), 0, 0, out, ticks, ITERS);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> t((size_t)blocks * 4);
    CK(hipMemcpy(t.data(), ticks, t.size() * 8, hipMemcpyDeviceToHost));
    double mean = 0;
    for (auto v : t) mean += (double)v;
    mean /= t.size();
    const double flop = (double)blocks * 4 * ITERS * 4 * 32 * 32 * 2 * 2;
    const double tf = flop / (ms * 1e-3) / 1e12;
    // cycles per MFMA per SIMD from the wave's own clock
    const double cyc_per_mfma = mean / (ITERS * 4.0 * wps);
    printf("{\"waves_per_simd\": %d, \"cus\": %d, \"ms\": %.3f, \"tflops\": %.1f, \"memtime_ticks_per_wave\": %.0f, "
           "\"clock_ghz_from_memtime\": %.3f, \"cycles_per_mfma_per_simd\": %.1f}\n",
           wps, cus, ms, tf, mean, mean / (ms * 1e-3) / 1e9, cyc_per_mfma);
    CK(hipFree(out));
    CK(hipFree(ticks));
  }
  return 0;
}
