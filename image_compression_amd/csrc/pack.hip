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

// tiled fast layouts (mode 0 / 1, k <= 5, R even, B % 4 == 0): one block per PK_TN x PK_TR tile of
// (n, r), all taps.  The tile's source is PK_TN (mode 0) or PK_TR (mode 1) runs of contiguous floats
// (a row of W[a][b][ky][kx] over (b, tap) or over (a-fixed) (n, tap)): staged through LDS with 16-B
// loads, about three per thread and all in flight together, then written with four tap groups of 64
// threads, two consecutive r per thread (one 4-B store per plane).  The per-element kernel
// (pack_fast_kernel) reads W with a stride of k*k floats (mode 0) or B*k*k floats (mode 1) per lane,
// a cache line per lane: 30-40 us per 192 x 192 5x5 weight on the main queue, 12 per C2 step.
typedef __bf16 pk_bf16x2 __attribute__((ext_vector_type(2)));
constexpr int PK_TN = 4, PK_TR = 32, PK_NT = 256;
__global__ void __launch_bounds__(PK_NT) pack_tile_kernel(const PackArgs p) {
  __shared__ __attribute__((aligned(16))) float ws[PK_TN * PK_TR * 25];
  const int Nout = p.mode == 0 ? p.A : p.B;
  const int R = p.mode == 0 ? p.B : p.A;
  const int kk = p.k * p.k;
  const int r0 = blockIdx.x * PK_TR, n0 = blockIdx.y * PK_TN;
  const int tid = threadIdx.x;
  // rows of the tile's source: mode 0 rows n (PK_TR * kk floats each), mode 1 rows r (PK_TN * kk)
  const int nrows = p.mode == 0 ? PK_TN : PK_TR;
  const int len = (p.mode == 0 ? PK_TR : PK_TN) * kk;  // a multiple of 4
  const int row0 = p.mode == 0 ? n0 : r0, rowmax = p.mode == 0 ? Nout : R;
  const int valid = p.mode == 0 ? min(PK_TR, R - r0) * kk : max(0, min(PK_TN, Nout - n0)) * kk;
  const int col0 = p.mode == 0 ? r0 : n0;
  const int nv = nrows * (len >> 2);
  // every load unconditional, at an index clamped into W, the zero fill by select: loads under a
  // per-element condition became branches with a vmcnt(0) wait each (49 in series per thread)
  constexpr int NIT = (PK_TN * PK_TR * 25 / 4 + PK_NT - 1) / PK_NT;  // float4 groups per thread (k <= 5)
  const long long wlast = (long long)p.A * p.B * kk - 1;
  float v[NIT][4];
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int j = min(tid + PK_NT * it, nv - 1);
    const int row = j / (len >> 2), q = 4 * (j - row * (len >> 2));
    const long long base = ((long long)min(row0 + row, rowmax - 1) * p.B + col0) * kk + q;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[it][e] = p.W[min(base + e, wlast)];
  }
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int j = tid + PK_NT * it;
    if (j >= nv) continue;
    const int row = j / (len >> 2), q = 4 * (j - row * (len >> 2));
    const bool rok = row0 + row < rowmax;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int qq = q + e;
      const float x = (rok && qq < valid) ? v[it][e] : 0.f;
      if (p.mode == 0) {
        ws[row * len + qq] = x;  // [nl][rl][tap]
      } else {
        const int nl = qq / kk, tap = qq - nl * kk;
        ws[(nl * PK_TR + row) * kk + tap] = x;
      }
    }
  }
  __syncthreads();
  const long long nrow = (long long)p.Npad * R, total = (long long)p.T * nrow;
  const int tg = tid >> 6, l = tid & 63;
  const int nl = l >> 4, rl = 2 * (l & 15);
  const int n = n0 + nl, r = r0 + rl;
  if (n >= p.Npad || r >= R) return;
  for (int t = tg; t < p.T; t += PK_NT / 64) {
    const int toff = p.ky[t] * p.k + p.kx[t];
    const float v0 = ws[(nl * PK_TR + rl) * kk + toff], v1 = ws[(nl * PK_TR + rl + 1) * kk + toff];
    const long long i = t * nrow + (long long)n * R + r;
    if (p.out_bf16 == 2) {
      __bf16 h0, m0, l0, h1, m1, l1;
      split3_bf16(v0, h0, m0, l0);
      split3_bf16(v1, h1, m1, l1);
      __bf16* o = (__bf16*)p.wp;
      *(pk_bf16x2*)(o + i) = pk_bf16x2{h0, h1};
      *(pk_bf16x2*)(o + i + total) = pk_bf16x2{m0, m1};
      *(pk_bf16x2*)(o + i + 2 * total) = pk_bf16x2{l0, l1};
    } else if (p.out_bf16) {
      *(pk_bf16x2*)((__bf16*)p.wp + i) = pk_bf16x2{(__bf16)v0, (__bf16)v1};
    } else {
      *(float2*)(p.wp + i) = make_float2(v0, v1);
    }
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
  if (!generic && mode < 2 && k <= 5 && R % 2 == 0 && B % 4 == 0 && ((uintptr_t)W & 15) == 0 && total < (1ll << 31)) {
    hipLaunchKernelGGL(pack_tile_kernel, dim3((R + PK_TR - 1) / PK_TR, (Npad + PK_TN - 1) / PK_TN), dim3(PK_NT), 0, s, p);
    IC_CHECK_LAUNCH();
    return IC_OK;
  }
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
