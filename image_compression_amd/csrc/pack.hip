// Weight re-packing for the implicit-GEMM kernels (per call; weights change
// every optimizer step).  PyTorch layout W[a][b][ky][kx] ->
//   direct     : out channel a, reduce channel b
//   transposed : out channel b, reduce channel a
//   fast       : wp[t][n][r]          (n < Npad, zero rows for n >= Nout)
//   generic    : wp[n][t*R + r]       (row padded with zeros to Kpad)
#include "gemm.h"

namespace {
struct PackArgs {
  const float* W;
  float* wp;
  int out_bf16;
  int A, B, k, mode, generic, T, Npad, Kpad;
  int ky[IC_MAXT], kx[IC_MAXT];
};

__device__ __forceinline__ void store_packed(const PackArgs& p, long long i, long long total, float v) {
  if (p.out_bf16 == 2) {  // three planes of the exact split, plane stride = total
    __bf16 h, m, l;
    split3_bf16(v, h, m, l);
    __bf16* o = (__bf16*)p.wp;
    o[i] = h;
    o[i + total] = m;
    o[i + 2 * total] = l;
  } else if (p.out_bf16) {
    ((__bf16*)p.wp)[i] = (__bf16)v;  // round to nearest even
  } else {
    p.wp[i] = v;
  }
}

__global__ void pack_kernel(const PackArgs p) {
  const int Nout = p.mode == 0 ? p.A : p.B;
  const int R = p.mode == 0 ? p.B : p.A;
  const long long total = p.mode == 2 ? (long long)p.Npad * p.A
                        : (p.generic ? (long long)p.Npad * p.Kpad : (long long)p.T * p.Npad * R);
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    int t, n, r;
    if (p.generic) {
      n = (int)(i / p.Kpad);
      const int kf = (int)(i - (long long)n * p.Kpad);
      t = kf / R;
      r = kf - t * R;
    } else {
      r = (int)(i % R);
      const long long tn = i / R;
      n = (int)(tn % p.Npad);
      t = (int)(tn / p.Npad);
    }
    float v = 0.f;
    if (p.mode == 2) {
      // i = n * A + a with n = tt * B + b
      const int a = (int)(i % p.A);
      const int nn = (int)(i / p.A);
      const int tt = nn / p.B, b = nn - (nn / p.B) * p.B;
      if (tt < p.T) v = p.W[(((long long)a * p.B + b) * p.k + p.ky[tt]) * p.k + p.kx[tt]];
      store_packed(p, i, total, v);
      continue;
    }
    if (n < Nout && t < p.T) {
      const int a = p.mode == 0 ? n : r;
      const int b = p.mode == 0 ? r : n;
      v = p.W[(((long long)a * p.B + b) * p.k + p.ky[t]) * p.k + p.kx[t]];
    }
    store_packed(p, i, total, v);
  }
}
// fast layouts (mode 0 / 1, not generic): tap t = blockIdx.y, one thread per
// (n, r) of it; 32-bit index arithmetic (the generic kernel's 64-bit divisions
// dominated its time)
__global__ void pack_fast_kernel(const PackArgs p) {
  const int Nout = p.mode == 0 ? p.A : p.B;
  const uint32_t R = (uint32_t)(p.mode == 0 ? p.B : p.A);
  const uint32_t nr = (uint32_t)p.Npad * R;
  const uint32_t total = (uint32_t)p.T * nr;
  const int t = blockIdx.y;
  const int toff = p.ky[t] * p.k + p.kx[t], kk = p.k * p.k;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nr; i += gridDim.x * blockDim.x) {
    const uint32_t n = i / R, r = i - n * R;
    float v = 0.f;
    if ((int)n < Nout) v = p.W[(p.mode == 0 ? n * (uint32_t)p.B + r : r * (uint32_t)p.B + n) * (uint32_t)kk + toff];
    store_packed(p, (long long)((uint32_t)t * nr + i), (long long)total, v);
  }
}
}  // namespace

int pack_weights(const float* W, int A, int B, int k, int mode, int generic, int T, const int* ky,
                 const int* kx, int Npad, int Kpad, float* wp, hipStream_t s, int out_bf16) {
  if (T > IC_MAXT || T < 1) return IC_ERR_ARG;
  PackArgs p;
  p.W = W; p.wp = wp; p.out_bf16 = out_bf16; p.A = A; p.B = B; p.k = k; p.mode = mode; p.generic = generic; p.T = T;
  p.Npad = Npad; p.Kpad = Kpad;
  for (int t = 0; t < T; ++t) { p.ky[t] = ky[t]; p.kx[t] = kx[t]; }
  const int R = mode == 0 ? B : A;
  const long long total = mode == 2 ? (long long)Npad * A : (generic ? (long long)Npad * Kpad : (long long)T * Npad * R);
  if (!generic && mode < 2 && total < (1ll << 31)) {
    const long long nr = (long long)Npad * R;
    long long blocks = (nr + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    hipLaunchKernelGGL(pack_fast_kernel, dim3((unsigned)blocks, T), dim3(256), 0, s, p);
    IC_CHECK_LAUNCH();
    return IC_OK;
  }
  long long blocks = (total + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(pack_kernel, dim3((unsigned)blocks), dim3(256), 0, s, p);
  IC_CHECK_LAUNCH();
  return IC_OK;
}
