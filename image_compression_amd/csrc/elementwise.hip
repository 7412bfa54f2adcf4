// Elementwise ops and deterministic reductions of the hot path (HBM-bound).
// All operate on dense storage of n fp32 elements; float4 vectorised where the
// pointer alignment allows (Guideline 13), grid-stride otherwise.
#include "../../include/imgcomp.h"
#include "common.h"

namespace {

constexpr float LN2F = 0.693147180559945309f;

inline unsigned grid_for(long long n, int per_thread = 1) {
  long long b = (n / per_thread + 255) / 256;
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  return (unsigned)b;
}

#define GRID_STRIDE(i, n) \
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < (n); i += (long long)gridDim.x * blockDim.x)

__global__ void nonneg_fwd_k(const float* p, long long n, float bound, float ped, float* out) {
  GRID_STRIDE(i, n) {
    const float v = fmaxf(p[i], bound);
    out[i] = v * v - ped;
  }
}
// LowerBound backward (bound.py:36-42) on g_v = 2 v g_out
__global__ void nonneg_bwd_k(const float* p, const float* go, long long n, float bound, float* gi) {
  GRID_STRIDE(i, n) {
    const float x = p[i];
    const float v = fmaxf(x, bound);
    const float g = go[i] * v * 2.f;  // d(v*v)/dv = 2v (autograd: g*v + g*v)
    gi[i] = (x >= bound || g < 0.f) ? g : 0.f;
  }
}

// NonNegativeParam over up to NN_MAXT tensors in one launch (block c handles chunk c of the
// concatenation; the per-element expressions are nonneg_fwd_k's / nonneg_bwd_k's, bitwise)
constexpr int NN_MAXT = 16, NN_CHUNK = 2048;
struct NonNegMulti {
  const float* p[NN_MAXT];
  float* out[NN_MAXT];
  const float* go[NN_MAXT];
  float* gi[NN_MAXT];
  long long n[NN_MAXT];
  float bound[NN_MAXT], ped[NN_MAXT];
  int chunk_begin[NN_MAXT + 1];
  int nt;
};
template <bool BWD>
__global__ void __launch_bounds__(256) nonneg_multi_k(const NonNegMulti a) {
  const int c = blockIdx.x;
  int k = 0;
  while (k + 1 < a.nt && c >= a.chunk_begin[k + 1]) ++k;
  const long long base = (long long)(c - a.chunk_begin[k]) * NN_CHUNK;
  const long long end = base + NN_CHUNK < a.n[k] ? base + NN_CHUNK : a.n[k];
  for (long long i = base + threadIdx.x; i < end; i += blockDim.x) {
    const float x = a.p[k][i];
    const float v = fmaxf(x, a.bound[k]);
    if (BWD) {
      const float g = a.go[k][i] * v * 2.f;
      a.gi[k][i] = (x >= a.bound[k] || g < 0.f) ? g : 0.f;
    } else {
      a.out[k][i] = v * v - a.ped[k];
    }
  }
}

__global__ void bound_fwd_k(const float* x, long long n, float b, int upper, float* y) {
  GRID_STRIDE(i, n) {
    const float v = x[i];
    y[i] = upper ? (v < b ? v : b) : (v > b ? v : b);
  }
}
__global__ void bound_bwd_k(const float* x, const float* g, long long n, float b, int upper, float* gx) {
  GRID_STRIDE(i, n) {
    const float v = x[i], gg = g[i];
    const bool pass = upper ? (v <= b || gg > 0.f) : (v >= b || gg < 0.f);
    gx[i] = pass ? gg : 0.f;
  }
}

__global__ void relu_fwd_k(const float* x, long long n, float* y) {
  GRID_STRIDE(i, n) {
    const float v = x[i];
    y[i] = v > 0.f ? v : (v != v ? v : 0.f);
  }
}
// torch threshold_backward: grad where result > 0
__global__ void relu_bwd_k(const float* y, const float* g, long long n, float* gx) {
  GRID_STRIDE(i, n) gx[i] = y[i] > 0.f ? g[i] : 0.f;
}
__global__ void abs_fwd_k(const float* x, long long n, float* y) {
  GRID_STRIDE(i, n) y[i] = fabsf(x[i]);
}
// d|x|/dx = sign(x) (0 at 0)
__global__ void abs_bwd_k(const float* x, const float* g, long long n, float* gx) {
  GRID_STRIDE(i, n) {
    const float v = x[i];
    const float sg = v > 0.f ? 1.f : (v < 0.f ? -1.f : 0.f);
    gx[i] = g[i] * sg;
  }
}
__global__ void exp_clamp_fwd_k(const float* v, long long n, float lo, float hi, float* s, float* e) {
  GRID_STRIDE(i, n) {
    const float ev = expf(v[i]);
    if (e) e[i] = ev;
    s[i] = fminf(fmaxf(ev, lo), hi);
  }
}
// clamp backward: pass where lo <= e <= hi; exp backward: * e
__global__ void exp_clamp_bwd_k(const float* e, const float* g, long long n, float lo, float hi, float* gv) {
  GRID_STRIDE(i, n) {
    const float ev = e[i];
    gv[i] = (ev >= lo && ev <= hi) ? g[i] * ev : 0.f;
  }
}

// ---- reductions: partial[block] then one final block (fixed order) ----
constexpr int RED_BLOCKS = 1024;

template <int OP>
__device__ __forceinline__ float red_term(const float* a, const float* b, long long i) {
  if (OP == 0) {  // ce: clamp(-ln(p + 1e-10)/ln2, 0, 50)
    const float t = -logf(a[i] + 1e-10f) / LN2F;
    return fminf(fmaxf(t, 0.f), 50.f);
  } else {  // squared error
    const float d = a[i] - b[i];
    return d * d;
  }
}

template <int OP>
__global__ void reduce_partial_k(const float* a, const float* b, long long n, float* part) {
  __shared__ float lds[64];
  float v[1] = {0.f};
  GRID_STRIDE(i, n) v[0] += red_term<OP>(a, b, i);
  block_sum<1>(v, lds);
  if (threadIdx.x == 0) part[blockIdx.x] = v[0];
}

__global__ void reduce_final_k(const float* part, int nb, float scale, float* out) {
  __shared__ float lds[64];
  float v[1] = {0.f};
  for (int i = threadIdx.x; i < nb; i += blockDim.x) v[0] += part[i];
  block_sum<1>(v, lds);
  if (threadIdx.x == 0) out[0] = v[0] * scale;
}

int reduce_run(int op, const float* a, const float* b, long long n, float scale, float* out, void* ws,
               size_t wsb, hipStream_t s) {
  if (wsb < RED_BLOCKS * sizeof(float)) return IC_ERR_WORKSPACE;
  float* part = (float*)ws;
  long long nb = (n + 255) / 256;
  if (nb > RED_BLOCKS) nb = RED_BLOCKS;
  if (nb < 1) nb = 1;
  if (op == 0)
    hipLaunchKernelGGL(reduce_partial_k<0>, dim3((unsigned)nb), dim3(256), 0, s, a, b, n, part);
  else
    hipLaunchKernelGGL(reduce_partial_k<1>, dim3((unsigned)nb), dim3(256), 0, s, a, b, n, part);
  IC_CHECK_LAUNCH();
  hipLaunchKernelGGL(reduce_final_k, dim3(1), dim3(256), 0, s, part, (int)nb, scale, out);
  IC_CHECK_LAUNCH();
  return IC_OK;
}

// torch: clamp(-1 * log(p + 1e-10) / LOG2, 0, 50): grad mask 0 <= t <= 50
__global__ void ce_bwd_k(const float* p, const float* gout, long long n, float* gp) {
  const float g = gout[0];
  GRID_STRIDE(i, n) {
    const float pe = p[i] + 1e-10f;
    const float t = -logf(pe) / LN2F;
    gp[i] = (t >= 0.f && t <= 50.f) ? g * (-1.f / (pe * LN2F)) : 0.f;
  }
}

__global__ void mse_bwd_k(const float* a, const float* b, const float* gout, long long n, float* ga, float* gb) {
  const float g = gout[0] * (2.f / (float)n);
  GRID_STRIDE(i, n) {
    const float d = (a[i] - b[i]) * g;
    if (ga) ga[i] = d;
    if (gb) gb[i] = -d;
  }
}

__global__ void sqdiff_fwd_k(const float* a, const float* b, long long n, float* o) {
  GRID_STRIDE(i, n) {
    const float d = a[i] - b[i];
    o[i] = d * d;
  }
}
__global__ void sqdiff_bwd_k(const float* a, const float* b, const float* g, long long n, float* ga, float* gb) {
  GRID_STRIDE(i, n) {
    const float d = 2.f * (a[i] - b[i]) * g[i];
    if (ga) ga[i] = d;
    if (gb) gb[i] = -d;
  }
}

// u[i] = element off + i of the stream (off % 4 == 0): one Philox block per thread and quad
__global__ void uniform_k(float* u, long long n, unsigned long long seed, unsigned long long off) {
  const long long nq = (n + 3) >> 2;
  for (long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x; j < nq; j += (long long)gridDim.x * blockDim.x) {
    const floatx4v r = philox_uniform4(seed, (off >> 2) + (unsigned long long)j);
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (4 * j + e < n) u[4 * j + e] = r[e];
  }
}

// raw Philox4x32-10 blocks for the known-answer test: in[6 i ..] = {c0, c1, c2, c3, k0, k1}
__global__ void philox_kat_k(const uint32_t* in, uint32_t* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t c[4] = {in[6 * i], in[6 * i + 1], in[6 * i + 2], in[6 * i + 3]};
  philox4x32_10(c, in[6 * i + 4], in[6 * i + 5]);
#pragma unroll
  for (int e = 0; e < 4; ++e) out[4 * i + e] = c[e];
}

}  // namespace

namespace {
// the stream base moves in whole Philox blocks (multiples of 4 elements)
__global__ void philox_advance_k(unsigned long long* state, unsigned long long n) {
  if (threadIdx.x == 0) state[1] += (n + 3) & ~3ull;
}
}  // namespace

extern "C" {

int ic_device_sync_check(void* stream) {
  hipLaunchKernelGGL(uniform_k, dim3(1), dim3(64), 0, (hipStream_t)stream, (float*)nullptr, 0LL, 0ULL, 0ULL);
  IC_CHECK_LAUNCH();
  return IC_OK;
}

int ic_nonneg_fwd(const float* p, long long n, float bound, float ped, float* out, void* stream) {
  hipLaunchKernelGGL(nonneg_fwd_k, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, p, n, bound, ped, out);
  IC_CHECK_LAUNCH();
  return IC_OK;
}
int ic_nonneg_bwd(const float* p, const float* gout, long long n, float bound, float* gin, void* stream) {
  hipLaunchKernelGGL(nonneg_bwd_k, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, p, gout, n, bound, gin);
  IC_CHECK_LAUNCH();
  return IC_OK;
}
int ic_nonneg_multi(const ic_nonneg_tensor* ts, int ntensors, int backward, void* stream) {
  if (ntensors < 0 || (ntensors > 0 && !ts)) return IC_ERR_ARG;
  int cur = 0;
  while (cur < ntensors) {
    NonNegMulti a;
    a.nt = 0;
    int chunks = 0;
    for (; cur < ntensors && a.nt < NN_MAXT; ++cur) {
      const ic_nonneg_tensor& e = ts[cur];
      if (e.n <= 0) continue;
      if (!e.p || (backward ? (!e.gout || !e.gin) : !e.out)) return IC_ERR_ARG;
      const int k = a.nt++;
      a.p[k] = e.p; a.out[k] = e.out; a.go[k] = e.gout; a.gi[k] = e.gin;
      a.n[k] = e.n; a.bound[k] = e.bound; a.ped[k] = e.pedestal;
      a.chunk_begin[k] = chunks;
      chunks += (int)((e.n + NN_CHUNK - 1) / NN_CHUNK);
    }
    if (a.nt == 0) continue;
    a.chunk_begin[a.nt] = chunks;
    if (backward)
      hipLaunchKernelGGL(nonneg_multi_k<true>, dim3(chunks), dim3(256), 0, (hipStream_t)stream, a);
    else
      hipLaunchKernelGGL(nonneg_multi_k<false>, dim3(chunks), dim3(256), 0, (hipStream_t)stream, a);
    IC_CHECK_LAUNCH();
  }
  return IC_OK;
}
int ic_bound_fwd(const float* x, long long n, float bound, int upper, float* y, void* stream) {
  hipLaunchKernelGGL(bound_fwd_k, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x, n, bound, upper, y);
  IC_CHECK_LAUNCH();
  return IC_OK;
}
int ic_bound_bwd(const float* x, const float* g, long long n, float bound, int upper, float* gx, void* stream) {
  hipLaunchKernelGGL(bound_bwd_k, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x, g, n, bound, upper, gx);
  IC_CHECK_LAUNCH();
  return IC_OK;
}
int ic_relu_fwd(const float* x, long long n, float* y, void* stream) {
  hipLaunchKernelGGL(relu_fwd_k, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x, n, y);
  IC_CHECK_LAUNCH();
  return IC_OK;
}
int ic_relu_bwd(const float* y, const float* g, long long n, float* gx, void* stream) {
  hipLaunchKernelGGL(relu_bwd_k, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, y, g, n, gx);
  IC_CHECK_LAUNCH();
  return IC_OK;
}
int ic_abs_fwd(const float* x, long long n, float* y, void* stream) {
  hipLaunchKernelGGL(abs_fwd_k, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x, n, y);
  IC_CHECK_LAUNCH();
  return IC_OK;
}
int ic_abs_bwd(const float* x, const float* g, long long n, float* gx, void* stream) {
  hipLaunchKernelGGL(abs_bwd_k, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x, g, n, gx);
  IC_CHECK_LAUNCH();
  return IC_OK;
}
int ic_exp_clamp_fwd(const float* v, long long n, float lo, float hi, float* sigma, float* e, void* stream) {
  hipLaunchKernelGGL(exp_clamp_fwd_k, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, v, n, lo, hi, sigma, e);
  IC_CHECK_LAUNCH();
  return IC_OK;
}
int ic_exp_clamp_bwd(const float* e, const float* g, long long n, float lo, float hi, float* gv, void* stream) {
  hipLaunchKernelGGL(exp_clamp_bwd_k, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, e, g, n, lo, hi, gv);
  IC_CHECK_LAUNCH();
  return IC_OK;
}

size_t ic_reduce_ws(long long n) { (void)n; return RED_BLOCKS * sizeof(float); }

int ic_ce_loss_fwd(const float* p, long long n, float* out, void* ws, size_t ws_bytes, void* stream) {
  return reduce_run(0, p, nullptr, n, 1.f, out, ws, ws_bytes, (hipStream_t)stream);
}
int ic_ce_loss_bwd(const float* p, const float* gout, long long n, float* gp, void* stream) {
  hipLaunchKernelGGL(ce_bwd_k, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, p, gout, n, gp);
  IC_CHECK_LAUNCH();
  return IC_OK;
}
int ic_mse_fwd(const float* a, const float* b, long long n, float* out, void* ws, size_t ws_bytes, void* stream) {
  return reduce_run(1, a, b, n, 1.f / (float)n, out, ws, ws_bytes, (hipStream_t)stream);
}
int ic_mse_bwd(const float* a, const float* b, const float* gout, long long n, float* ga, float* gb, void* stream) {
  hipLaunchKernelGGL(mse_bwd_k, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, a, b, gout, n, ga, gb);
  IC_CHECK_LAUNCH();
  return IC_OK;
}
int ic_sqdiff_fwd(const float* a, const float* b, long long n, float* out, void* stream) {
  hipLaunchKernelGGL(sqdiff_fwd_k, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, a, b, n, out);
  IC_CHECK_LAUNCH();
  return IC_OK;
}
int ic_sqdiff_bwd(const float* a, const float* b, const float* g, long long n, float* ga, float* gb, void* stream) {
  hipLaunchKernelGGL(sqdiff_bwd_k, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, a, b, g, n, ga, gb);
  IC_CHECK_LAUNCH();
  return IC_OK;
}
int ic_uniform(float* u, long long n, unsigned long long seed, unsigned long long offset, void* stream) {
  if (offset & 3) return IC_ERR_ARG;
  if (n <= 0) return IC_OK;
  hipLaunchKernelGGL(uniform_k, dim3(grid_for((n + 3) / 4)), dim3(256), 0, (hipStream_t)stream, u, n, seed, offset);
  IC_CHECK_LAUNCH();
  return IC_OK;
}

int ic_philox_kat(const unsigned* in, unsigned* out, int n, void* stream) {
  if (n <= 0) return IC_OK;
  hipLaunchKernelGGL(philox_kat_k, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, in, out, n);
  IC_CHECK_LAUNCH();
  return IC_OK;
}

int ic_philox_advance(unsigned long long* state, unsigned long long n, void* stream) {
  hipLaunchKernelGGL(philox_advance_k, dim3(1), dim3(64), 0, (hipStream_t)stream, state, n);
  IC_CHECK_LAUNCH();
  return IC_OK;
}

}  // extern "C"
