// Entropy bottleneck kernels (HBM/latency-bound elementwise work).
//
// factorized : modelling/blocks/entropy_model.py:47-114 (CDF MLP 1-3-3-3-1 per
//              channel) and :204-269 (noise/round, sign-trick likelihood).
//              One block per channel: the per-channel parameter gradients are
//              block reductions in a fixed order (deterministic).
// conditional: entropy_model.py:280-378, Laplacian (default) / Gaussian CDF.
#include "../../include/imgcomp.h"
#include "common.h"

namespace {

__device__ __forceinline__ float softplusf(float x) { return x > 20.f ? x : log1pf(expf(x)); }
__device__ __forceinline__ float dsoftplusf(float x) { return x > 20.f ? 1.f : 1.f / (1.f + expf(-x)); }
__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + expf(-x)); }
__device__ __forceinline__ float signf_(float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); }

struct ChanParams {
  float sw0[3], b0[3], tf0[3];
  float sw1[9], b1[3], tf1[3];
  float sw2[9], b2[3], tf2[3];
  float sw3[3], b3;
};

__device__ __forceinline__ void load_chan(const ic_fact_params& P, int c, ChanParams& q) {
#pragma unroll
  for (int o = 0; o < 3; ++o) {
    q.sw0[o] = softplusf(P.w0[c * 3 + o]);
    q.b0[o] = P.b0[c * 3 + o];
    q.tf0[o] = tanhf(P.f0[c * 3 + o]);
    q.b1[o] = P.b1[c * 3 + o];
    q.tf1[o] = tanhf(P.f1[c * 3 + o]);
    q.b2[o] = P.b2[c * 3 + o];
    q.tf2[o] = tanhf(P.f2[c * 3 + o]);
    q.sw3[o] = softplusf(P.w3[c * 3 + o]);
  }
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    q.sw1[j] = softplusf(P.w1[c * 9 + j]);
    q.sw2[j] = softplusf(P.w2[c * 9 + j]);
  }
  q.b3 = P.b3[c];
}

// activations of one MLP evaluation (pre-gate a*, post-gate h*)
struct Acts {
  float a0[3], h0[3], a1[3], h1[3], a2[3], h2[3];
  float out;
};

__device__ __forceinline__ void mlp_fwd(const ChanParams& q, float v, Acts& A) {
#pragma unroll
  for (int o = 0; o < 3; ++o) {
    A.a0[o] = q.sw0[o] * v + q.b0[o];
    A.h0[o] = A.a0[o] + tanhf(A.a0[o]) * q.tf0[o];
  }
#pragma unroll
  for (int o = 0; o < 3; ++o) {
    A.a1[o] = q.sw1[o * 3 + 0] * A.h0[0] + q.sw1[o * 3 + 1] * A.h0[1] + q.sw1[o * 3 + 2] * A.h0[2] + q.b1[o];
    A.h1[o] = A.a1[o] + tanhf(A.a1[o]) * q.tf1[o];
  }
#pragma unroll
  for (int o = 0; o < 3; ++o) {
    A.a2[o] = q.sw2[o * 3 + 0] * A.h1[0] + q.sw2[o * 3 + 1] * A.h1[1] + q.sw2[o * 3 + 2] * A.h1[2] + q.b2[o];
    A.h2[o] = A.a2[o] + tanhf(A.a2[o]) * q.tf2[o];
  }
  A.out = q.sw3[0] * A.h2[0] + q.sw3[1] * A.h2[1] + q.sw3[2] * A.h2[2] + q.b3;
}

// gradient accumulators layout (43 floats):
// [0..2] w0, [3..5] b0, [6..8] f0, [9..17] w1, [18..20] b1, [21..23] f1,
// [24..32] w2, [33..35] b2, [36..38] f2, [39..41] w3, [42] b3
constexpr int NG = 43;

// backward of one evaluation with upstream g; accumulates "raw" gradients wrt
// softplus(W) (converted to W by the caller once per channel) and returns dv.
__device__ __forceinline__ float mlp_bwd(const ChanParams& q, float v, const Acts& A, float g, float (&G)[NG]) {
  float dh2[3], da2[3], dh1[3], da1[3], dh0[3], da0[3];
  // layer 3
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    G[39 + i] += g * A.h2[i];
    dh2[i] = g * q.sw3[i];
  }
  G[42] += g;
  // layer 2 gate
#pragma unroll
  for (int o = 0; o < 3; ++o) {
    const float th = tanhf(A.a2[o]);
    da2[o] = dh2[o] * (1.f + (1.f - th * th) * q.tf2[o]);
    G[36 + o] += dh2[o] * th;  // * (1 - tf^2) applied by caller
    G[33 + o] += da2[o];
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    dh1[i] = 0.f;
#pragma unroll
    for (int o = 0; o < 3; ++o) {
      G[24 + o * 3 + i] += da2[o] * A.h1[i];
      dh1[i] += q.sw2[o * 3 + i] * da2[o];
    }
  }
#pragma unroll
  for (int o = 0; o < 3; ++o) {
    const float th = tanhf(A.a1[o]);
    da1[o] = dh1[o] * (1.f + (1.f - th * th) * q.tf1[o]);
    G[21 + o] += dh1[o] * th;
    G[18 + o] += da1[o];
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    dh0[i] = 0.f;
#pragma unroll
    for (int o = 0; o < 3; ++o) {
      G[9 + o * 3 + i] += da1[o] * A.h0[i];
      dh0[i] += q.sw1[o * 3 + i] * da1[o];
    }
  }
  float dv = 0.f;
#pragma unroll
  for (int o = 0; o < 3; ++o) {
    const float th = tanhf(A.a0[o]);
    da0[o] = dh0[o] * (1.f + (1.f - th * th) * q.tf0[o]);
    G[6 + o] += dh0[o] * th;
    G[3 + o] += da0[o];
    G[0 + o] += da0[o] * v;
    dv += q.sw0[o] * da0[o];
  }
  return dv;
}

__device__ __forceinline__ float quant(float x, int mode, const float* u, long long i,
                                       unsigned long long seed, unsigned long long off) {
  if (mode == 1) return rintf(x);
  float uu;
  if (mode == 0) {
    uu = u[i];
  } else if (mode == 3) {  // device-resident {seed, base} (graph-safe stream)
    const unsigned long long* st = (const unsigned long long*)u;
    uu = philox_uniform(st[0], st[1] + off + (unsigned long long)i);
  } else {
    uu = philox_uniform(seed, off + (unsigned long long)i);
  }
  return x + (uu - 0.5f);
}

__global__ void fact_fwd_k(const float* z, long long n, int C, const ic_fact_params P, int mode,
                           const float* u, unsigned long long seed, unsigned long long off, float* qo,
                           float* po) {
  const int c = blockIdx.x;
  ChanParams q;
  load_chan(P, c, q);
  const long long ne = n / C;
  for (long long e = threadIdx.x; e < ne; e += blockDim.x) {
    const long long i = e * C + c;
    const float qv = quant(z[i], mode, u, i, seed, off);
    qo[i] = qv;
    Acts lo, up;
    mlp_fwd(q, qv - 0.5f, lo);
    mlp_fwd(q, qv + 0.5f, up);
    const float s = -signf_(lo.out + up.out);
    po[i] = s * (sigmoidf_(up.out * s) - sigmoidf_(lo.out * s));
  }
}

__global__ void __launch_bounds__(256) fact_bwd_k(const float* qin, long long n, int C, const ic_fact_params P,
                           const float* dq, const float* dp, float* dz, const ic_fact_grads GR, int round_mode) {
  // built without packed-fp32 VALU instructions, like every source (Makefile NOPK): with them this
  // kernel sometimes returned wrong w1 / w2 gradient sums in concurrent model steps (a mitigation,
  // DESIGN.md section 10a)
  __shared__ float lds[16 * NG];
  const int c = blockIdx.x;
  ChanParams q;
  load_chan(P, c, q);
  float G[NG];
#pragma unroll
  for (int j = 0; j < NG; ++j) G[j] = 0.f;
  const long long ne = n / C;
  for (long long e = threadIdx.x; e < ne; e += blockDim.x) {
    const long long i = e * C + c;
    const float qv = qin[i];
    float dqv = 0.f;
    const float gp = dp ? dp[i] : 0.f;
    if (gp != 0.f) {
      Acts lo, up;
      mlp_fwd(q, qv - 0.5f, lo);
      mlp_fwd(q, qv + 0.5f, up);
      const float s = -signf_(lo.out + up.out);
      const float su = sigmoidf_(s * up.out), sl = sigmoidf_(s * lo.out);
      // p = s*(sig(s*up) - sig(s*lo)), s detached
      const float gup = gp * s * su * (1.f - su) * s;
      const float glo = -gp * s * sl * (1.f - sl) * s;
      dqv += mlp_bwd(q, qv + 0.5f, up, gup, G);
      dqv += mlp_bwd(q, qv - 0.5f, lo, glo, G);
    }
    if (dz) dz[i] = round_mode ? 0.f : (dq ? dq[i] : 0.f) + dqv;
  }
  block_sum<NG>(G, lds);
  if (threadIdx.x == 0) {
    // every parameter read before the first gradient store (the stores may alias the parameters as far
    // as the compiler knows, so interleaved they serialised each load behind the store before it)
    float w0[3], w3[3], f0[3], f1[3], f2[3], w1[9], w2[9];
#pragma unroll
    for (int o = 0; o < 3; ++o) {
      w0[o] = P.w0[c * 3 + o]; w3[o] = P.w3[c * 3 + o];
      f0[o] = P.f0[c * 3 + o]; f1[o] = P.f1[c * 3 + o]; f2[o] = P.f2[c * 3 + o];
    }
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      w1[j] = P.w1[c * 9 + j];
      w2[j] = P.w2[c * 9 + j];
    }
#pragma unroll
    for (int o = 0; o < 3; ++o) {
      GR.w0[c * 3 + o] = G[0 + o] * dsoftplusf(w0[o]);
      GR.b0[c * 3 + o] = G[3 + o];
      const float t0 = tanhf(f0[o]);
      GR.f0[c * 3 + o] = G[6 + o] * (1.f - t0 * t0);
      GR.b1[c * 3 + o] = G[18 + o];
      const float t1 = tanhf(f1[o]);
      GR.f1[c * 3 + o] = G[21 + o] * (1.f - t1 * t1);
      GR.b2[c * 3 + o] = G[33 + o];
      const float t2 = tanhf(f2[o]);
      GR.f2[c * 3 + o] = G[36 + o] * (1.f - t2 * t2);
      GR.w3[c * 3 + o] = G[39 + o] * dsoftplusf(w3[o]);
    }
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      GR.w1[c * 9 + j] = G[9 + j] * dsoftplusf(w1[j]);
      GR.w2[c * 9 + j] = G[24 + j] * dsoftplusf(w2[j]);
    }
    GR.b3[c] = G[42];
  }
}

// ---------------------------------------------------------------- conditional
__device__ __forceinline__ float cdf_lap(float v) {
  return 0.5f - 0.5f * signf_(v) * expm1f(-fabsf(v));
}
__device__ __forceinline__ float dcdf_lap(float v) {
  const float sg = signf_(v);
  return 0.5f * sg * sg * (expm1f(-fabsf(v)) + 1.f);
}
constexpr float RSQRT2 = 0.70710678118654752f;
constexpr float TWO_OVER_SQRTPI = 1.12837916709551257f;
__device__ __forceinline__ float cdf_gauss(float v) { return 0.5f * (1.f + erff(v * 1.0f * RSQRT2)); }
__device__ __forceinline__ float dcdf_gauss(float v) {
  const float t = v * RSQRT2;
  return 0.5f * TWO_OVER_SQRTPI * expf(-t * t) * RSQRT2;
}

__device__ __forceinline__ void cond_elem(const float* y, const float* sc, const float* mean, long long i, int kind,
                                          float uu, int mode, float half, float* qo, float* po) {
  // noise u - bin/2 (entropy_model.py:331-334), round (:336), mass over +-bin/2 (:347-350)
  const float qv = mode == 1 ? rintf(y[i]) : y[i] + (uu - half);
  qo[i] = qv;
  const float a = fabsf(qv - (mean ? mean[i] : 0.f));
  const float s = sc[i];
  const float vu = (half - a) / s, vl = (-half - a) / s;
  po[i] = kind == 0 ? cdf_lap(vu) - cdf_lap(vl) : cdf_gauss(vu) - cdf_gauss(vl);
}

// one quad of elements per thread and iteration: in the Philox modes one Philox block
// (four uniforms) serves the quad (stream offsets are 4-aligned)
__global__ void cond_fwd_k(const float* y, const float* sc, const float* mean, long long n, int kind, int mode,
                           const float* u, unsigned long long seed, unsigned long long off, float half, float* qo,
                           float* po) {
  const long long nq = (n + 3) >> 2;
  for (long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x; j < nq; j += (long long)gridDim.x * blockDim.x) {
    floatx4v r = {0.f, 0.f, 0.f, 0.f};
    if (mode == 3) {
      const unsigned long long* st = (const unsigned long long*)u;
      r = philox_uniform4(st[0], ((st[1] + off) >> 2) + (unsigned long long)j);
    } else if (mode == 2) {
      r = philox_uniform4(seed, (off >> 2) + (unsigned long long)j);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const long long i = 4 * j + e;
      // mode 4: y is already quantized (q = y + 0)
      if (i < n) cond_elem(y, sc, mean, i, kind, mode == 0 ? u[i] : (mode == 4 ? half : r[e]), mode, half, qo, po);
    }
  }
}

__global__ void cond_bwd_k(const float* q, const float* sc, const float* mean, long long n, int kind, float half,
                           const float* dq, const float* dp, float* dy, float* ds, float* dm) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float d = q[i] - (mean ? mean[i] : 0.f);
    const float a = fabsf(d);
    const float s = sc[i];
    const float vu = (half - a) / s, vl = (-half - a) / s;
    const float g = dp ? dp[i] : 0.f;
    const float fu = kind == 0 ? dcdf_lap(vu) : dcdf_gauss(vu);
    const float fl = kind == 0 ? dcdf_lap(vl) : dcdf_gauss(vl);
    const float gvu = g * fu, gvl = -g * fl;   // dL/dvu, dL/dvl
    const float ga = -(gvu + gvl) / s;         // dv/da = -1/s for both
    const float gs = -(gvu * vu + gvl * vl) / s;
    const float gd = ga * signf_(d);
    if (dy) dy[i] = (dq ? dq[i] : 0.f) + gd;
    if (ds) ds[i] = gs;
    if (dm) dm[i] = -gd;
  }
}

// ---------------------------------------------------------------- generic factorized model
// Any CDF MLP widths (cfg.MODEL.ENTROPY_MODEL.DIMS: hidden widths <= IC_FACT_MAXW,
// len(DIMS) + 1 <= IC_FACT_MAXL layers; entropy_model.py:88-99) and any BIN
// (noise u - bin/2, mass over +-bin/2: :229-232, :259-269).  One block per
// channel; the channel's transformed parameters (softplus W, b, tanh f) sit in
// LDS.  Every loop runs to the compile-time maxima under a width predicate, so
// activations stay in registers.  Backward: per round of FE elements, thread t
// backpropagates evaluation t & 1 (lower / upper) of element t >> 1 and writes
// its per-layer terms -- delta = dL/da, the gate term dL/dh * tanh(a), the
// layer input h -- to LDS row t; then each thread sums its own parameters' terms
// over the round's rows in row order (deterministic, no atomics).
constexpr int FMW = IC_FACT_MAXW, FML = IC_FACT_MAXL;
constexpr int FNT = 128;             // threads per block (FNT / 2 elements per round)
constexpr int FPJ = (FML * (FMW * FMW + 2 * FMW) + FNT - 1) / FNT;  // parameters per thread

struct FactLayout {  // offsets of layer l's softplus(W) [dout][din], b [dout], tanh(f) [dout] in LDS
  int ow[FML], ob[FML], of[FML], nprm;
  int rd[FML], rg[FML], rh[FML], nrow;  // row offsets of delta, gate term, layer input
};

__device__ __forceinline__ void fact_layout(const ic_fact_net& N, FactLayout& F) {
  int o = 0, r = 0;
#pragma unroll
  for (int l = 0; l < FML; ++l) {
    const int din = l < N.nlayers ? N.dims[l] : 0, dout = l < N.nlayers ? N.dims[l + 1] : 0;
    F.ow[l] = o; o += dout * din;
    F.ob[l] = o; o += dout;
    F.of[l] = o; o += (l < N.nlayers - 1) ? dout : 0;
    F.rd[l] = r; r += dout;
    F.rg[l] = r; r += dout;
    F.rh[l] = r; r += din;
  }
  F.nprm = o;
  F.nrow = r;
}

// the channel's parameters, transformed, into LDS (softplus W, b, tanh f)
__device__ __forceinline__ void fact_load_lds(const ic_fact_net& N, const FactLayout& F, int c, float* prm) {
  for (int l = 0; l < N.nlayers; ++l) {
    const int din = N.dims[l], dout = N.dims[l + 1];
    for (int j = threadIdx.x; j < dout * din; j += blockDim.x) prm[F.ow[l] + j] = softplusf(N.w[l][c * dout * din + j]);
    for (int j = threadIdx.x; j < dout; j += blockDim.x) {
      prm[F.ob[l] + j] = N.b[l][c * dout + j];
      if (l < N.nlayers - 1) prm[F.of[l] + j] = tanhf(N.f[l][c * dout + j]);
    }
  }
}

// logits of one evaluation at v; REC keeps the pre-gate values A and the layer inputs H
template <bool REC>
__device__ __forceinline__ float fact_eval(const ic_fact_net& N, const FactLayout& F, const float* prm, float v,
                                           float (&A)[FML][FMW], float (&H)[FML][FMW]) {
  float h[FMW];
#pragma unroll
  for (int i = 0; i < FMW; ++i) h[i] = i == 0 ? v : 0.f;
#pragma unroll
  for (int l = 0; l < FML; ++l) {
    if (l >= N.nlayers) break;
    const int din = N.dims[l], dout = N.dims[l + 1];
    const bool gate = l < N.nlayers - 1;
    float hn[FMW];
#pragma unroll
    for (int o = 0; o < FMW; ++o) {
      hn[o] = 0.f;
      if (o < dout) {
        float s = prm[F.ob[l] + o];
#pragma unroll
        for (int i = 0; i < FMW; ++i)
          if (i < din) s += prm[F.ow[l] + o * din + i] * h[i];
        if (REC) A[l][o] = s;
        hn[o] = gate ? s + tanhf(s) * prm[F.of[l] + o] : s;
      }
    }
#pragma unroll
    for (int i = 0; i < FMW; ++i) {
      if (REC) H[l][i] = h[i];
      h[i] = hn[i];
    }
  }
  return h[0];
}

__global__ void fact_fwd_net_k(const float* z, long long n, int C, const ic_fact_net N, float half, int mode,
                               const float* u, unsigned long long seed, unsigned long long off, float* qo, float* po) {
  extern __shared__ float flds[];
  const int c = blockIdx.x;
  FactLayout F;
  fact_layout(N, F);
  fact_load_lds(N, F, c, flds);
  __syncthreads();
  float A[FML][FMW], H[FML][FMW];
  const long long ne = n / C;
  for (long long e = threadIdx.x; e < ne; e += blockDim.x) {
    const long long i = e * C + c;
    float qv;
    if (mode == 1) {
      qv = rintf(z[i]);
    } else {
      float uu;
      if (mode == 0) uu = u[i];
      else if (mode == 3) {
        const unsigned long long* st = (const unsigned long long*)u;
        uu = philox_uniform(st[0], st[1] + off + (unsigned long long)i);
      } else {
        uu = philox_uniform(seed, off + (unsigned long long)i);
      }
      qv = z[i] + (uu - half);
    }
    qo[i] = qv;
    const float lo = fact_eval<false>(N, F, flds, qv - half, A, H);
    const float up = fact_eval<false>(N, F, flds, qv + half, A, H);
    const float s = -signf_(lo + up);
    po[i] = s * (sigmoidf_(up * s) - sigmoidf_(lo * s));
  }
}

__global__ void __launch_bounds__(FNT) fact_bwd_net_k(const float* qin, long long n, int C, const ic_fact_net N,
                                                      float half, const float* dq, const float* dp, float* dz,
                                                      const ic_fact_net_grads GR) {
  extern __shared__ float flds[];
  const int c = blockIdx.x, t = threadIdx.x;
  FactLayout F;
  fact_layout(N, F);
  float* prm = flds;
  float* rows = flds + F.nprm;           // [FNT][nrow]
  float* dvb = rows + FNT * F.nrow;      // [FNT] input gradients of the two evaluations
  fact_load_lds(N, F, c, prm);
  // the parameters this thread owns: index j = t + FNT k; term = row[oa] * (ob < 0 ? 1 : row[ob])
  int oa[FPJ], ob[FPJ];
  float acc[FPJ];
#pragma unroll
  for (int k = 0; k < FPJ; ++k) {
    acc[k] = 0.f;
    oa[k] = -1;
    ob[k] = -1;
    int j = t + FNT * k;
    for (int l = 0; l < N.nlayers && oa[k] < 0; ++l) {
      const int din = N.dims[l], dout = N.dims[l + 1];
      const int nl = dout * din + dout + (l < N.nlayers - 1 ? dout : 0);
      if (j >= nl) { j -= nl; continue; }
      if (j < dout * din) { oa[k] = F.rd[l] + j / din; ob[k] = F.rh[l] + j % din; }
      else if (j < dout * din + dout) { oa[k] = F.rd[l] + (j - dout * din); }
      else { oa[k] = F.rg[l] + (j - dout * din - dout); }
    }
  }
  __syncthreads();
  float A[FML][FMW], H[FML][FMW];
  const long long ne = n / C;
  const int which = t & 1;  // 0: lower (q - half), 1: upper (q + half)
  for (long long e0 = 0; e0 < ne; e0 += FNT / 2) {
    const long long e = e0 + (t >> 1);
    float* row = rows + t * F.nrow;
    float dv = 0.f;
    const bool live = e < ne;
    const long long i = e * C + c;
    const float gp = (live && dp) ? dp[i] : 0.f;
    if (live && gp != 0.f) {
      const float qv = qin[i];
      float A2[FML][FMW], H2[FML][FMW];
      const float lo = fact_eval<true>(N, F, prm, qv - half, which ? A2 : A, which ? H2 : H);
      const float up = fact_eval<true>(N, F, prm, qv + half, which ? A : A2, which ? H : H2);
      const float s = -signf_(lo + up);
      const float su = sigmoidf_(s * up), sl = sigmoidf_(s * lo);
      // p = s (sig(s up) - sig(s lo)), s detached
      float g = which ? gp * s * su * (1.f - su) * s : -gp * s * sl * (1.f - sl) * s;
      float dh[FMW];
#pragma unroll
      for (int o = 0; o < FMW; ++o) dh[o] = o == 0 ? g : 0.f;
#pragma unroll
      for (int l = FML - 1; l >= 0; --l) {
        if (l >= N.nlayers) continue;
        const int din = N.dims[l], dout = N.dims[l + 1];
        const bool gate = l < N.nlayers - 1;
        float da[FMW];
#pragma unroll
        for (int o = 0; o < FMW; ++o) {
          da[o] = 0.f;
          if (o < dout) {
            if (gate) {
              const float th = tanhf(A[l][o]);
              da[o] = dh[o] * (1.f + (1.f - th * th) * prm[F.of[l] + o]);
              row[F.rg[l] + o] = dh[o] * th;
            } else {
              da[o] = dh[o];
              row[F.rg[l] + o] = 0.f;
            }
            row[F.rd[l] + o] = da[o];
          }
        }
#pragma unroll
        for (int i2 = 0; i2 < FMW; ++i2) {
          float sacc = 0.f;
          if (i2 < din) {
            row[F.rh[l] + i2] = H[l][i2];
#pragma unroll
            for (int o = 0; o < FMW; ++o)
              if (o < dout) sacc += prm[F.ow[l] + o * din + i2] * da[o];
          }
          dh[i2] = sacc;
        }
      }
      dv = dh[0];
    } else {
      for (int r = 0; r < F.nrow; ++r) row[r] = 0.f;
    }
    dvb[t] = dv;
    __syncthreads();
    if (live && which == 0 && dz) dz[i] = (dq ? dq[i] : 0.f) + (dvb[t] + dvb[t + 1]);
#pragma unroll
    for (int k = 0; k < FPJ; ++k) {
      if (oa[k] < 0) continue;
      float sacc = 0.f;
      for (int r = 0; r < FNT; ++r) {
        const float* rr = rows + r * F.nrow;
        sacc += ob[k] < 0 ? rr[oa[k]] : rr[oa[k]] * rr[ob[k]];
      }
      acc[k] += sacc;
    }
    __syncthreads();
  }
  // raw sums -> parameter gradients (softplus' for W, 1 - tanh^2 for f)
#pragma unroll
  for (int k = 0; k < FPJ; ++k) {
    if (oa[k] < 0) continue;
    int j = t + FNT * k;
    for (int l = 0; l < N.nlayers; ++l) {
      const int din = N.dims[l], dout = N.dims[l + 1];
      const int nl = dout * din + dout + (l < N.nlayers - 1 ? dout : 0);
      if (j >= nl) { j -= nl; continue; }
      if (j < dout * din) {
        GR.w[l][c * dout * din + j] = acc[k] * dsoftplusf(N.w[l][c * dout * din + j]);
      } else if (j < dout * din + dout) {
        GR.b[l][c * dout + (j - dout * din)] = acc[k];
      } else {
        const int o = j - dout * din - dout;
        const float tf = tanhf(N.f[l][c * dout + o]);
        GR.f[l][c * dout + o] = acc[k] * (1.f - tf * tf);
      }
      break;
    }
  }
}

// the conditional model's quantization alone (entropy_model.py:331-336), element for
// element as cond_fwd_k forms it: q = y + (u - bin/2) or round(y)
__global__ void quant_k(const float* y, long long n, int mode, const float* u, unsigned long long seed,
                        unsigned long long off, float half, float* qo) {
  const long long nq = (n + 3) >> 2;
  for (long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x; j < nq; j += (long long)gridDim.x * blockDim.x) {
    floatx4v r = {0.f, 0.f, 0.f, 0.f};
    if (mode == 3) {
      const unsigned long long* st = (const unsigned long long*)u;
      r = philox_uniform4(st[0], ((st[1] + off) >> 2) + (unsigned long long)j);
    } else if (mode == 2) {
      r = philox_uniform4(seed, (off >> 2) + (unsigned long long)j);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const long long i = 4 * j + e;
      if (i < n) qo[i] = mode == 1 ? rintf(y[i]) : y[i] + ((mode == 0 ? u[i] : r[e]) - half);
    }
  }
}

// a well-formed net the wide kernels take (up to IC_FACT_NET_MAXL layers of width <= IC_FACT_WIDE_MAXW)
bool fact_net_valid(const ic_fact_net* N) {
  if (!N || N->nlayers < 1 || N->nlayers > IC_FACT_NET_MAXL || N->dims[0] != 1 || N->dims[N->nlayers] != 1)
    return false;
  for (int l = 0; l < N->nlayers; ++l) {
    if (N->dims[l + 1] < 1 || N->dims[l + 1] > IC_FACT_WIDE_MAXW || !N->w[l] || !N->b[l]) return false;
    if (l < N->nlayers - 1 && !N->f[l]) return false;
  }
  return true;
}
// ... within the register kernels' limits
bool fact_net_ok(const ic_fact_net* N) {
  if (!fact_net_valid(N) || N->nlayers > FML) return false;
  for (int l = 0; l < N->nlayers; ++l)
    if (N->dims[l + 1] > FMW) return false;
  return true;
}

size_t fact_net_lds(const ic_fact_net* N, bool bwd) {
  int prm = 0, row = 0;
  for (int l = 0; l < N->nlayers; ++l) {
    const int din = N->dims[l], dout = N->dims[l + 1];
    prm += dout * din + dout + (l < N->nlayers - 1 ? dout : 0);
    row += 2 * dout + din;
  }
  return ((size_t)prm + (bwd ? (size_t)FNT * row + FNT : 0)) * sizeof(float);
}

// ---------------------------------------------------------------- CDF MLP of any geometry (wide)
// Nets past the register kernels' limits (more than IC_FACT_MAXL layers or a hidden width above
// IC_FACT_MAXW; entropy_model.py:88-99 builds any DIMS), up to IC_FACT_NET_MAXL layers of width <=
// IC_FACT_WIDE_MAXW: the register kernels' arithmetic in the same order (a layer's products summed
// over its inputs in index order, the same gate and sigmoid formulas), with each thread's activations
// in a scratch of the workspace instead of registers and the channel's transformed parameters
// (softplus W, b, tanh f) formed once per call into the workspace.  One wave per channel.  Backward as
// fact_bwd_net_k: per round of FW / 2 elements, lane t backpropagates evaluation t & 1 of element t >> 1
// and writes its per-layer terms to row t (in the workspace); after the barrier each lane sums the
// terms of the parameters it owns over the rows in row order -- deterministic, no atomics.
constexpr int FW = 64;
struct WideLayout {
  int ow[IC_FACT_NET_MAXL], ob[IC_FACT_NET_MAXL], of[IC_FACT_NET_MAXL];  // parameter offsets per layer
  int rd[IC_FACT_NET_MAXL], rg[IC_FACT_NET_MAXL], rh[IC_FACT_NET_MAXL];  // row offsets: delta, gate term, input
  int aa[IC_FACT_NET_MAXL], ah[IC_FACT_NET_MAXL];                        // activation record: pre-gate, input
  int np, nrow, nact, wmax;
};

WideLayout wide_layout(const ic_fact_net& N) {
  WideLayout F{};
  int o = 0, r = 0, a = 0, wm = 1;
  for (int l = 0; l < N.nlayers; ++l) {
    const int din = N.dims[l], dout = N.dims[l + 1];
    F.ow[l] = o; o += dout * din;
    F.ob[l] = o; o += dout;
    F.of[l] = o; o += l < N.nlayers - 1 ? dout : 0;
    F.rd[l] = r; r += dout;
    F.rg[l] = r; r += dout;
    F.rh[l] = r; r += din;
    F.aa[l] = a; a += dout;
    F.ah[l] = a; a += din;
    wm = max(wm, dout);
  }
  F.np = o; F.nrow = r; F.nact = a; F.wmax = wm;
  return F;
}

// workspace (floats): transformed parameters [C][np]; per lane of each channel's wave: the evaluation
// scratch (2 wmax), and in the backward the activation record (nact), its row (nrow), plus [C][np]
// parameter sums
struct WideWs {
  size_t tp, scr, act, rows, acc, total;
};
WideWs wide_ws(int C, const WideLayout& F, bool bwd) {
  WideWs w{};
  size_t o = 0;
  auto take = [&](size_t floats) { const size_t at = o; o += ic_align(floats * 4, 256); return at; };
  w.tp = take((size_t)C * F.np);
  w.scr = take((size_t)C * FW * 2 * F.wmax);
  if (bwd) {
    w.act = take((size_t)C * FW * F.nact);
    w.rows = take((size_t)C * FW * F.nrow);
    w.acc = take((size_t)C * F.np);
  }
  w.total = o;
  return w;
}

__global__ void __launch_bounds__(FW) fact_wide_prep_k(const ic_fact_net N, const WideLayout F, float* __restrict__ tp) {
  const int c = blockIdx.x;
  float* t = tp + (size_t)c * F.np;
  for (int l = 0; l < N.nlayers; ++l) {
    const int din = N.dims[l], dout = N.dims[l + 1];
    for (int j = threadIdx.x; j < dout * din; j += FW) t[F.ow[l] + j] = softplusf(N.w[l][(size_t)c * dout * din + j]);
    for (int j = threadIdx.x; j < dout; j += FW) {
      t[F.ob[l] + j] = N.b[l][(size_t)c * dout + j];
      if (l < N.nlayers - 1) t[F.of[l] + j] = tanhf(N.f[l][(size_t)c * dout + j]);
    }
  }
}

// logits of one evaluation at v (as fact_eval); act != nullptr records each layer's input and pre-gate values
__device__ float wide_eval(const ic_fact_net& N, const WideLayout& F, const float* __restrict__ tp, float v,
                           float* h, float* hn, float* act) {
  h[0] = v;
  for (int l = 0; l < N.nlayers; ++l) {
    const int din = N.dims[l], dout = N.dims[l + 1];
    const bool gate = l < N.nlayers - 1;
    if (act)
      for (int i = 0; i < din; ++i) act[F.ah[l] + i] = h[i];
    for (int o = 0; o < dout; ++o) {
      float s = tp[F.ob[l] + o];
      const float* w = tp + F.ow[l] + o * din;
      for (int i = 0; i < din; ++i) s += w[i] * h[i];
      if (act) act[F.aa[l] + o] = s;
      hn[o] = gate ? s + tanhf(s) * tp[F.of[l] + o] : s;
    }
    float* t = h; h = hn; hn = t;
  }
  return h[0];
}

__global__ void __launch_bounds__(FW) fact_fwd_wide_k(const float* z, long long n, int C, const ic_fact_net N,
                                                      const WideLayout F, float half, int mode, const float* u,
                                                      unsigned long long seed, unsigned long long off, float* qo,
                                                      float* po, const float* __restrict__ tp_all, float* scr_all) {
  const int c = blockIdx.x, t = threadIdx.x;
  const float* tp = tp_all + (size_t)c * F.np;
  float* h = scr_all + ((size_t)c * FW + t) * 2 * F.wmax;
  const long long ne = n / C;
  for (long long e = t; e < ne; e += FW) {
    const long long i = e * C + c;
    float qv;
    if (mode == 1) {
      qv = rintf(z[i]);
    } else {
      float uu;
      if (mode == 0) uu = u[i];
      else if (mode == 3) {
        const unsigned long long* st = (const unsigned long long*)u;
        uu = philox_uniform(st[0], st[1] + off + (unsigned long long)i);
      } else {
        uu = philox_uniform(seed, off + (unsigned long long)i);
      }
      qv = z[i] + (uu - half);
    }
    qo[i] = qv;
    const float lo = wide_eval(N, F, tp, qv - half, h, h + F.wmax, nullptr);
    const float up = wide_eval(N, F, tp, qv + half, h, h + F.wmax, nullptr);
    const float s = -signf_(lo + up);
    po[i] = s * (sigmoidf_(up * s) - sigmoidf_(lo * s));
  }
}

// the rows term of parameter j: row[oa] * (ob < 0 ? 1 : row[ob]) (fact_bwd_net_k's ownership map)
__device__ void wide_param_rows(const ic_fact_net& N, const WideLayout& F, int j, int& oa, int& ob) {
  oa = -1; ob = -1;
  for (int l = 0; l < N.nlayers; ++l) {
    const int din = N.dims[l], dout = N.dims[l + 1];
    const int nl = dout * din + dout + (l < N.nlayers - 1 ? dout : 0);
    if (j >= nl) { j -= nl; continue; }
    if (j < dout * din) { oa = F.rd[l] + j / din; ob = F.rh[l] + j % din; }
    else if (j < dout * din + dout) { oa = F.rd[l] + (j - dout * din); }
    else { oa = F.rg[l] + (j - dout * din - dout); }
    return;
  }
}

__global__ void __launch_bounds__(FW) fact_bwd_wide_k(const float* qin, long long n, int C, const ic_fact_net N,
                                                      const WideLayout F, float half, const float* dq, const float* dp,
                                                      float* dz, const ic_fact_net_grads GR,
                                                      const float* __restrict__ tp_all, float* scr_all, float* act_all,
                                                      float* rows_all, float* acc_all) {
  __shared__ float dvb[FW];
  const int c = blockIdx.x, t = threadIdx.x;
  const float* tp = tp_all + (size_t)c * F.np;
  float* h = scr_all + ((size_t)c * FW + t) * 2 * F.wmax;  // evaluation scratch, then dh / da
  float* act = act_all + ((size_t)c * FW + t) * F.nact;
  float* rows = rows_all + (size_t)c * FW * F.nrow;
  float* row = rows + (size_t)t * F.nrow;
  float* acc = acc_all + (size_t)c * F.np;
  for (int j = t; j < F.np; j += FW) acc[j] = 0.f;
  const long long ne = n / C;
  const int which = t & 1;  // 0: lower (q - half), 1: upper (q + half)
  for (long long e0 = 0; e0 < ne; e0 += FW / 2) {
    const long long e = e0 + (t >> 1);
    float dv = 0.f;
    const bool live = e < ne;
    const long long i = e * C + c;
    const float gp = (live && dp) ? dp[i] : 0.f;
    if (live && gp != 0.f) {
      const float qv = qin[i];
      const float lo = wide_eval(N, F, tp, qv - half, h, h + F.wmax, which ? nullptr : act);
      const float up = wide_eval(N, F, tp, qv + half, h, h + F.wmax, which ? act : nullptr);
      const float s = -signf_(lo + up);
      const float su = sigmoidf_(s * up), sl = sigmoidf_(s * lo);
      // p = s (sig(s up) - sig(s lo)), s detached
      const float g = which ? gp * s * su * (1.f - su) * s : -gp * s * sl * (1.f - sl) * s;
      float* dh = h;
      float* da = h + F.wmax;
      dh[0] = g;
      for (int l = N.nlayers - 1; l >= 0; --l) {
        const int din = N.dims[l], dout = N.dims[l + 1];
        const bool gate = l < N.nlayers - 1;
        for (int o = 0; o < dout; ++o) {
          float d;
          if (gate) {
            const float th = tanhf(act[F.aa[l] + o]);
            d = dh[o] * (1.f + (1.f - th * th) * tp[F.of[l] + o]);
            row[F.rg[l] + o] = dh[o] * th;
          } else {
            d = dh[o];
            row[F.rg[l] + o] = 0.f;
          }
          row[F.rd[l] + o] = d;
          da[o] = d;
        }
        for (int i2 = 0; i2 < din; ++i2) {
          row[F.rh[l] + i2] = act[F.ah[l] + i2];
          float sacc = 0.f;
          for (int o = 0; o < dout; ++o) sacc += tp[F.ow[l] + o * din + i2] * da[o];
          dh[i2] = sacc;
        }
      }
      dv = dh[0];
    } else {
      for (int r = 0; r < F.nrow; ++r) row[r] = 0.f;
    }
    dvb[t] = dv;
    __syncthreads();  // the rows (workspace) and dvb: visible to the whole wave
    if (live && which == 0 && dz) dz[i] = (dq ? dq[i] : 0.f) + (dvb[t] + dvb[t + 1]);
    for (int j = t; j < F.np; j += FW) {
      int oa, ob;
      wide_param_rows(N, F, j, oa, ob);
      float sacc = 0.f;
      for (int r = 0; r < FW; ++r) {
        const float* rr = rows + (size_t)r * F.nrow;
        sacc += ob < 0 ? rr[oa] : rr[oa] * rr[ob];
      }
      acc[j] += sacc;
    }
    __syncthreads();
  }
  // raw sums -> parameter gradients (softplus' for W, 1 - tanh^2 for f)
  for (int j0 = t; j0 < F.np; j0 += FW) {
    int j = j0;
    for (int l = 0; l < N.nlayers; ++l) {
      const int din = N.dims[l], dout = N.dims[l + 1];
      const int nl = dout * din + dout + (l < N.nlayers - 1 ? dout : 0);
      if (j >= nl) { j -= nl; continue; }
      if (j < dout * din) {
        GR.w[l][(size_t)c * dout * din + j] = acc[j0] * dsoftplusf(N.w[l][(size_t)c * dout * din + j]);
      } else if (j < dout * din + dout) {
        GR.b[l][(size_t)c * dout + (j - dout * din)] = acc[j0];
      } else {
        const int o = j - dout * din - dout;
        const float tf = tanhf(N.f[l][(size_t)c * dout + o]);
        GR.f[l][(size_t)c * dout + o] = acc[j0] * (1.f - tf * tf);
      }
      break;
    }
  }
}

}  // namespace

extern "C" {

int ic_factorized_fwd(const float* z, long long n, int C, const ic_fact_params* prm, int mode, const float* u,
                      unsigned long long seed, unsigned long long offset, float* q, float* p, void* stream) {
  if (C <= 0 || n % C != 0 || (mode == 0 && !u)) return IC_ERR_ARG;
  if ((mode == 2 || mode == 3) && (offset & 3)) return IC_ERR_ARG;  // whole Philox blocks
  hipLaunchKernelGGL(fact_fwd_k, dim3(C), dim3(256), 0, (hipStream_t)stream, z, n, C, *prm, mode, u, seed,
                     offset, q, p);
  IC_CHECK_LAUNCH();
  return IC_OK;
}

int ic_factorized_bwd(const float* q, long long n, int C, const ic_fact_params* prm, const float* dq,
                      const float* dp, float* dz, const ic_fact_grads* grd, void* stream) {
  if (C <= 0 || n % C != 0) return IC_ERR_ARG;
  hipLaunchKernelGGL(fact_bwd_k, dim3(C), dim3(256), 0, (hipStream_t)stream, q, n, C, *prm, dq, dp, dz, *grd, 0);
  IC_CHECK_LAUNCH();
  return IC_OK;
}

int ic_quantize(const float* y, long long n, int mode, const float* u, unsigned long long seed,
                unsigned long long offset, float bin, float* q, void* stream) {
  if ((mode == 0 && !u) || mode < 0 || mode > 3 || !(bin > 0.f)) return IC_ERR_ARG;
  if ((mode == 2 || mode == 3) && (offset & 3)) return IC_ERR_ARG;  // whole Philox blocks (4 draws)
  long long b = (n + 1023) / 1024;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  hipLaunchKernelGGL(quant_k, dim3((unsigned)b), dim3(256), 0, (hipStream_t)stream, y, n, mode, u, seed, offset,
                     0.5f * bin, q);
  IC_CHECK_LAUNCH();
  return IC_OK;
}

int ic_conditional_fwd_bin(const float* y, const float* scale, const float* mean, long long n, int kind, int mode,
                           const float* u, unsigned long long seed, unsigned long long offset, float bin, float* q,
                           float* p, void* stream) {
  if ((mode == 0 && !u) || mode < 0 || mode > 4) return IC_ERR_ARG;
  if (!(bin > 0.f)) return IC_ERR_ARG;
  if ((mode == 2 || mode == 3) && (offset & 3)) return IC_ERR_ARG;  // stream offsets are whole Philox blocks
  long long b = (n + 1023) / 1024;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  hipLaunchKernelGGL(cond_fwd_k, dim3((unsigned)b), dim3(256), 0, (hipStream_t)stream, y, scale, mean, n, kind,
                     mode, u, seed, offset, 0.5f * bin, q, p);
  IC_CHECK_LAUNCH();
  return IC_OK;
}

int ic_conditional_fwd(const float* y, const float* scale, const float* mean, long long n, int kind, int mode,
                       const float* u, unsigned long long seed, unsigned long long offset, float* q, float* p,
                       void* stream) {
  return ic_conditional_fwd_bin(y, scale, mean, n, kind, mode, u, seed, offset, 1.f, q, p, stream);
}

int ic_conditional_bwd_bin(const float* q, const float* scale, const float* mean, long long n, int kind, float bin,
                           const float* dq, const float* dp, float* dy, float* dscale, float* dmean, void* stream) {
  if (!(bin > 0.f)) return IC_ERR_ARG;
  long long b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  hipLaunchKernelGGL(cond_bwd_k, dim3((unsigned)b), dim3(256), 0, (hipStream_t)stream, q, scale, mean, n, kind,
                     0.5f * bin, dq, dp, dy, dscale, dmean);
  IC_CHECK_LAUNCH();
  return IC_OK;
}

int ic_conditional_bwd(const float* q, const float* scale, const float* mean, long long n, int kind,
                       const float* dq, const float* dp, float* dy, float* dscale, float* dmean, void* stream) {
  return ic_conditional_bwd_bin(q, scale, mean, n, kind, 1.f, dq, dp, dy, dscale, dmean, stream);
}

size_t ic_factorized_net_ws(long long n, int C, const ic_fact_net* net, int bwd) {
  (void)n;
  if (C <= 0 || !fact_net_valid(net)) return 0;
  if (fact_net_ok(net) && fact_net_lds(net, bwd != 0) <= 160 * 1024) return 0;  // the register kernels
  return wide_ws(C, wide_layout(*net), bwd != 0).total;
}

int ic_factorized_fwd_net_ex(const float* z, long long n, int C, const ic_fact_net* net, float bin, int mode,
                             const float* u, unsigned long long seed, unsigned long long offset, float* q, float* p,
                             void* ws, size_t ws_bytes, void* stream) {
  if (C <= 0 || n % C != 0 || (mode == 0 && !u) || !fact_net_valid(net) || !(bin > 0.f)) return IC_ERR_ARG;
  if ((mode == 2 || mode == 3) && (offset & 3)) return IC_ERR_ARG;  // whole Philox blocks
  if (fact_net_ok(net)) {
    hipLaunchKernelGGL(fact_fwd_net_k, dim3(C), dim3(FNT), fact_net_lds(net, false), (hipStream_t)stream, z, n, C,
                       *net, 0.5f * bin, mode, u, seed, offset, q, p);
    IC_CHECK_LAUNCH();
    return IC_OK;
  }
  const WideLayout F = wide_layout(*net);
  const WideWs W = wide_ws(C, F, false);
  if (!ws || ws_bytes < W.total) return IC_ERR_WORKSPACE;
  char* b = (char*)ws;
  hipLaunchKernelGGL(fact_wide_prep_k, dim3(C), dim3(FW), 0, (hipStream_t)stream, *net, F, (float*)(b + W.tp));
  hipLaunchKernelGGL(fact_fwd_wide_k, dim3(C), dim3(FW), 0, (hipStream_t)stream, z, n, C, *net, F, 0.5f * bin, mode, u,
                     seed, offset, q, p, (const float*)(b + W.tp), (float*)(b + W.scr));
  IC_CHECK_LAUNCH();
  return IC_OK;
}

int ic_factorized_bwd_net_ex(const float* q, long long n, int C, const ic_fact_net* net, float bin, const float* dq,
                             const float* dp, float* dz, const ic_fact_net_grads* grd, void* ws, size_t ws_bytes,
                             void* stream) {
  if (C <= 0 || n % C != 0 || !fact_net_valid(net) || !grd || !(bin > 0.f)) return IC_ERR_ARG;
  for (int l = 0; l < net->nlayers; ++l)
    if (!grd->w[l] || !grd->b[l] || (l < net->nlayers - 1 && !grd->f[l])) return IC_ERR_ARG;
  const size_t lds = fact_net_lds(net, true);
  if (fact_net_ok(net) && lds <= 160 * 1024) {
    hipLaunchKernelGGL(fact_bwd_net_k, dim3(C), dim3(FNT), lds, (hipStream_t)stream, q, n, C, *net, 0.5f * bin, dq,
                       dp, dz, *grd);
    IC_CHECK_LAUNCH();
    return IC_OK;
  }
  const WideLayout F = wide_layout(*net);
  const WideWs W = wide_ws(C, F, true);
  if (!ws || ws_bytes < W.total) return IC_ERR_WORKSPACE;
  char* b = (char*)ws;
  hipLaunchKernelGGL(fact_wide_prep_k, dim3(C), dim3(FW), 0, (hipStream_t)stream, *net, F, (float*)(b + W.tp));
  hipLaunchKernelGGL(fact_bwd_wide_k, dim3(C), dim3(FW), 0, (hipStream_t)stream, q, n, C, *net, F, 0.5f * bin, dq, dp,
                     dz, *grd, (const float*)(b + W.tp), (float*)(b + W.scr), (float*)(b + W.act),
                     (float*)(b + W.rows), (float*)(b + W.acc));
  IC_CHECK_LAUNCH();
  return IC_OK;
}

int ic_factorized_fwd_net(const float* z, long long n, int C, const ic_fact_net* net, float bin, int mode,
                          const float* u, unsigned long long seed, unsigned long long offset, float* q, float* p,
                          void* stream) {
  return ic_factorized_fwd_net_ex(z, n, C, net, bin, mode, u, seed, offset, q, p, nullptr, 0, stream);
}

int ic_factorized_bwd_net(const float* q, long long n, int C, const ic_fact_net* net, float bin, const float* dq,
                          const float* dp, float* dz, const ic_fact_net_grads* grd, void* stream) {
  return ic_factorized_bwd_net_ex(q, n, C, net, bin, dq, dp, dz, grd, nullptr, 0, stream);
}

}  // extern "C"
