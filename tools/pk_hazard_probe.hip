// Packed-fp32 hazard probe (round-3 verdict item 1): does a v_pk_*_f32 result read by the very next
// instruction come out stale when other waves on the same SIMD run MFMAs?
//
// The round-3 fault: fact_bwd_k (entropy.hip), built with packed fp32, returned wrong w1 / w2 gradient
// elements in concurrent steps only.  Its ISA reduces the 43 per-thread accumulators with
//     v_pk_add_f32 v[32:33], v[32:33], v[34:35]
//     ds_bpermute_b32 v34, v121, v32       <- reads the packed result the next cycle
//     ds_bpermute_b32 v35, v121, v33
// This probe runs exactly such sequences from inline asm (so no compiler padding) in one-wave blocks,
// each lane checking the value the consumer saw against the register's settled value, while a hog
// kernel on another stream keeps every SIMD busy with MFMAs (or with plain VALU FMAs, or nothing).
// Variants (V):
//   0 pk_add -> ds_bpermute lo, hi            (the compiler's sequence)
//   1 pk_add -> s_nop 4 -> ds_bpermute lo, hi
//   2 two v_add_f32 -> ds_bpermute lo, hi     (scalar control)
//   3 pk_add -> ds_write_b64 -> ds_read_b64   (the LDS-only reduction's pattern)
//   4 pk_fma -> ds_bpermute lo, hi
//   5 pk_mul -> ds_bpermute lo, hi
//   6 pk_add -> v_mov_b32 x2 (VALU consumer)
//   7 pk_add -> global_store_dwordx2 -> load back
// Output: one line per (hog, variant): mismatching lane-iterations out of the total.
//   hipcc --offload-arch=gfx950 -O3 tools/pk_hazard_probe.hip -o tools/_abl/pk_hazard_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float floatx4v __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

__device__ __forceinline__ unsigned hash32(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

// MFMA hog: every wave issues v_mfma_f32_16x16x32_bf16 back to back on random operands.
__global__ void __launch_bounds__(256) hog_mfma(float* out, int iters) {
  bf16x8 a[2], b[2];
  const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
  for (int i = 0; i < 2; ++i)
    for (int e = 0; e < 8; ++e) {
      a[i][e] = (__bf16)((float)(hash32(t * 64 + i * 8 + e) >> 8) * (2.0f / 16777216.0f) - 1.0f);
      b[i][e] = (__bf16)((float)(hash32(t * 64 + 32 + i * 8 + e) >> 8) * (2.0f / 16777216.0f) - 1.0f);
    }
  floatx4v c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
#define MF(c, x, y) asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(x), "v"(y))
  for (int it = 0; it < iters; ++it) {
    MF(c0, a[0], b[0]); MF(c1, a[1], b[0]); MF(c2, a[0], b[1]); MF(c3, a[1], b[1]);
  }
#undef MF
  const floatx4v s = (c0 + c1) + (c2 + c3);
  out[t] = s[0] + s[1] + s[2] + s[3];
}

// VALU hog: independent fma chains, no MFMA.
__global__ void __launch_bounds__(256) hog_valu(float* out, int iters) {
  float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3;
  for (int it = 0; it < iters * 4; ++it) {
    asm volatile("v_fma_f32 %0, %0, %4, 1.0\n v_fma_f32 %1, %1, %4, 1.0\n v_fma_f32 %2, %2, %4, 1.0\n"
                 " v_fma_f32 %3, %3, %4, 1.0"
                 : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3)
                 : "v"(0.5f));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3;
}

// Probe: one wave per block.  x (two lanes of values) advances by c each iteration; the consumer's view
// of the producer's result is compared bitwise with the register's settled value.
template <int V>
__global__ void __launch_bounds__(64) probe(unsigned* errs, float* dump, float* gbuf, int iters) {
  __shared__ float lds[128];  // the only LDS of the kernel: offset 0
  const unsigned lane = threadIdx.x;
  const unsigned gid = blockIdx.x * 64 + lane;
  float x0 = (float)(lane & 7), x1 = (float)(lane >> 3);
  const float c0 = 1.0f, c1 = 2.0f;
  const unsigned paddr = lane * 4u, laddr = lane * 8u;
  float* gp = gbuf + 2 * gid;
  unsigned nerr = 0;
  lds[lane] = 0.f;
  __syncthreads();
  for (int it = 0; it < iters; ++it) {
    float g0, g1, n0, n1;
#define PRE "v_mov_b32 v40, %[x0]\n v_mov_b32 v41, %[x1]\n v_mov_b32 v42, %[c0]\n v_mov_b32 v43, %[c1]\n" \
            " v_mov_b32 v46, 1.0\n v_mov_b32 v47, 1.0\n s_nop 4\n"
#define POST "s_waitcnt lgkmcnt(0) vmcnt(0)\n s_nop 4\n v_mov_b32 %[g0], v44\n v_mov_b32 %[g1], v45\n" \
             " v_mov_b32 %[n0], v40\n v_mov_b32 %[n1], v41\n"
#define OPS : [g0] "=v"(g0), [g1] "=v"(g1), [n0] "=v"(n0), [n1] "=v"(n1) \
            : [x0] "v"(x0), [x1] "v"(x1), [c0] "v"(c0), [c1] "v"(c1), [pa] "v"(paddr), [la] "v"(laddr), \
              [gp] "v"(gp) \
            : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "memory"
    if constexpr (V == 0) {
      asm volatile(PRE "v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n"
                   " ds_bpermute_b32 v44, %[pa], v40\n ds_bpermute_b32 v45, %[pa], v41\n" POST OPS);
    } else if constexpr (V == 1) {
      asm volatile(PRE "v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n s_nop 4\n"
                   " ds_bpermute_b32 v44, %[pa], v40\n ds_bpermute_b32 v45, %[pa], v41\n" POST OPS);
    } else if constexpr (V == 2) {
      asm volatile(PRE "v_add_f32 v40, v40, v42\n v_add_f32 v41, v41, v43\n"
                   " ds_bpermute_b32 v44, %[pa], v40\n ds_bpermute_b32 v45, %[pa], v41\n" POST OPS);
    } else if constexpr (V == 3) {
      asm volatile(PRE "v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n"
                   " ds_write_b64 %[la], v[40:41]\n s_waitcnt lgkmcnt(0)\n ds_read_b64 v[44:45], %[la]\n" POST OPS);
    } else if constexpr (V == 4) {
      asm volatile(PRE "v_pk_fma_f32 v[40:41], v[40:41], v[46:47], v[42:43]\n"
                   " ds_bpermute_b32 v44, %[pa], v40\n ds_bpermute_b32 v45, %[pa], v41\n" POST OPS);
    } else if constexpr (V == 5) {
      asm volatile(PRE "v_pk_mul_f32 v[40:41], v[40:41], v[46:47]\n v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n"
                   " v_pk_mul_f32 v[40:41], v[40:41], v[46:47]\n"
                   " ds_bpermute_b32 v44, %[pa], v40\n ds_bpermute_b32 v45, %[pa], v41\n" POST OPS);
    } else if constexpr (V == 6) {
      asm volatile(PRE "v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n v_mov_b32 v44, v40\n v_mov_b32 v45, v41\n" POST OPS);
    } else {
      asm volatile(PRE "v_pk_add_f32 v[40:41], v[40:41], v[42:43]\n global_store_dwordx2 %[gp], v[40:41], off\n"
                   " s_waitcnt vmcnt(0)\n global_load_dwordx2 v[44:45], %[gp], off\n" POST OPS);
    }
#undef PRE
#undef POST
#undef OPS
    const bool bad = __float_as_uint(g0) != __float_as_uint(n0) || __float_as_uint(g1) != __float_as_uint(n1);
    if (bad) {
      if (nerr == 0) {
        dump[4 * gid + 0] = g0; dump[4 * gid + 1] = n0; dump[4 * gid + 2] = g1; dump[4 * gid + 3] = n1;
      }
      ++nerr;
    }
    x0 = n0; x1 = n1;
  }
  errs[gid] = nerr;
}

typedef void (*probe_fn)(unsigned*, float*, float*, int);

int main(int argc, char** argv) {
  const int probe_iters = argc > 1 ? atoi(argv[1]) : 4096;
  const int reps = argc > 2 ? atoi(argv[2]) : 16;
  const int hog_iters = argc > 3 ? atoi(argv[3]) : 400000;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const int pblocks = cus * 8;  // 8 one-wave blocks per CU: 2 per SIMD
  const int hblocks = cus;      // one 4-wave block per CU: 1 wave per SIMD
  unsigned* errs; float *dump, *gbuf, *hout;
  CK(hipMalloc(&errs, sizeof(unsigned) * pblocks * 64));
  CK(hipMalloc(&dump, sizeof(float) * pblocks * 64 * 4));
  CK(hipMalloc(&gbuf, sizeof(float) * pblocks * 64 * 2));
  CK(hipMalloc(&hout, sizeof(float) * hblocks * 256 * 2));
  hipStream_t sh, sp;
  CK(hipStreamCreateWithFlags(&sh, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sp, hipStreamNonBlocking));
  hipEvent_t h0, h1, p0, p1;
  CK(hipEventCreate(&h0)); CK(hipEventCreate(&h1)); CK(hipEventCreate(&p0)); CK(hipEventCreate(&p1));
  probe_fn fns[8] = {probe<0>, probe<1>, probe<2>, probe<3>, probe<4>, probe<5>, probe<6>, probe<7>};
  const char* names[8] = {"pk_add>bpermute", "pk_add>nop4>bpermute", "2xadd>bpermute", "pk_add>ds_write_b64",
                          "pk_fma>bpermute", "pk_mul,add,mul>bpermute", "pk_add>v_mov", "pk_add>global_store"};
  const char* hogs[3] = {"none", "valu", "mfma"};
  std::vector<unsigned> he(pblocks * 64);
  std::vector<float> hd(pblocks * 64 * 4);
  for (int hog = 0; hog < 3; ++hog) {
    for (int v = 0; v < 8; ++v) {
      CK(hipMemset(errs, 0, sizeof(unsigned) * pblocks * 64));
      CK(hipMemset(dump, 0, sizeof(float) * pblocks * 64 * 4));
      CK(hipDeviceSynchronize());
      unsigned long long tot_err = 0, tot = 0;
      int lanes_bad = 0;
      float hog_ms = 0.f, probe_ms = 0.f;
      for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(h0, sh));
        if (hog == 1) hipLaunchKernelGGL(hog_valu, dim3(hblocks), dim3(256), 0, sh, hout, hog_iters);
        if (hog == 2) hipLaunchKernelGGL(hog_mfma, dim3(hblocks), dim3(256), 0, sh, hout, hog_iters);
        CK(hipEventRecord(h1, sh));
        CK(hipEventRecord(p0, sp));
        hipLaunchKernelGGL(fns[v], dim3(pblocks), dim3(64), 0, sp, errs, dump, gbuf, probe_iters);
        CK(hipEventRecord(p1, sp));
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        float a, b;
        CK(hipEventElapsedTime(&a, h0, h1));
        CK(hipEventElapsedTime(&b, p0, p1));
        hog_ms += a; probe_ms += b;
        CK(hipMemcpy(he.data(), errs, sizeof(unsigned) * pblocks * 64, hipMemcpyDeviceToHost));
        for (unsigned e : he) { tot_err += e; lanes_bad += e != 0; }
        tot += (unsigned long long)pblocks * 64 * probe_iters;
      }
      CK(hipMemcpy(hd.data(), dump, sizeof(float) * hd.size(), hipMemcpyDeviceToHost));
      int shown = 0;
      char ex[256] = "";
      for (size_t i = 0; i < he.size() && !shown; ++i)
        if (he[i]) {
          snprintf(ex, sizeof ex, " first: lane %zu got (%g,%g) want (%g,%g)", i, hd[4 * i], hd[4 * i + 2],
                   hd[4 * i + 1], hd[4 * i + 3]);
          shown = 1;
        }
      printf("{\"hog\": \"%s\", \"variant\": %d, \"seq\": \"%s\", \"mismatch\": %llu, \"checked\": %llu, "
             "\"hog_ms\": %.2f, \"probe_ms\": %.2f}%s\n",
             hogs[hog], v, names[v], tot_err, tot, hog_ms / reps, probe_ms / reps, ex);
      fflush(stdout);
    }
  }
  return 0;
}
