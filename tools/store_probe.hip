// Store-pattern probe (diagnostic; round 6): 403 MB of fp32 written by 256 blocks x 512 threads, one
// 16-B dwordx4 store per lane and instruction, in two address patterns:
//   seg : the edge conv's epilogue -- lane (li = lane & 15, lq = lane >> 4) writes pixel li's channels
//         nbase + 16 j + 4 lq .. + 3 (a wave instruction = 16 segments of 64 B at a 768-B pixel stride);
//         a unit = 64 pixels x 192 channels (48 KB), waves w & 3 own channel slices, w >> 2 pixel halves
//   row : the same 48 KB per unit written as contiguous 1 KB per wave instruction
// Both with the 6 stores per wave and unit issued in one burst, units grid-strided like the kernel.
//   hipcc --offload-arch=gfx950 -O3 -o tools/_abl/store_probe tools/store_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));

template <bool ROW>
__global__ void __launch_bounds__(512, 1) store_k(float* __restrict__ y, int units, float v) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int li = lane & 15, lq = lane >> 4;
  const int nbase = (w & 3) * 48, mt0 = 2 * (w >> 2);
  const f4 val = {v, v + 1.f, v + 2.f, v + 3.f};
  for (int u = blockIdx.x; u < units; u += gridDim.x) {
    float* base = y + (size_t)u * 64 * 192;
    if (ROW) {
      // wave w: 1 KB contiguous per instruction, 6 instructions = its 6 KB of the unit's 48 KB
#pragma unroll
      for (int k = 0; k < 6; ++k) *(f4*)(base + (size_t)(w * 6 + k) * 256 + lane * 4) = val;
    } else {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const int px = 16 * (mt0 + t) + li;
          *(f4*)(base + (size_t)px * 192 + nbase + 16 * j + 4 * lq) = val;
        }
    }
  }
}

int main() {
  const int units = 32 * 128 * 2;  // 32 images x 128 rows x 2 segments of 64 pixels (g_a.0's output)
  const size_t n = (size_t)units * 64 * 192;
  float* y;
  if (hipMalloc(&y, n * 4) != hipSuccess) return 1;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int pass = 0; pass < 2; ++pass)
    for (int row = 0; row < 2; ++row) {
      for (int r = 0; r < 3; ++r) {
        if (row) hipLaunchKernelGGL(store_k<true>, dim3(256), dim3(512), 0, 0, y, units, 1.f);
        else hipLaunchKernelGGL(store_k<false>, dim3(256), dim3(512), 0, 0, y, units, 1.f);
      }
      hipEventRecord(a);
      const int reps = 20;
      for (int r = 0; r < reps; ++r) {
        if (row) hipLaunchKernelGGL(store_k<true>, dim3(256), dim3(512), 0, 0, y, units, 1.f);
        else hipLaunchKernelGGL(store_k<false>, dim3(256), dim3(512), 0, 0, y, units, 1.f);
      }
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0.f;
      hipEventElapsedTime(&ms, a, b);
      ms /= reps;
      printf("%s: %.4f ms per launch, %.2f TB/s (%zu MB)\n", row ? "row (1 KB contiguous per instruction)"
                                                            : "seg (16 x 64 B per instruction, edge conv)",
             ms, n * 4 / (ms * 1e-3) / 1e12, n * 4 >> 20);
    }
  hipFree(y);
  return 0;
}
