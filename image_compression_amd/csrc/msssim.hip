// SSIM / MS-SSIM distortion loss (reference modelling/loss.py:48-188) on HIP.
//
// The 11x11 window softmax(-(x^2+y^2)/2s^2) is the outer product of two 1-D
// normalised Gaussians, so every "valid" 2-D filtering is a horizontal 11-tap
// pass followed by a vertical one (22 instead of 121 MACs per output), over the
// five moment images {a, b, a^2, b^2, ab}.  Means are deterministic two-level
// reductions.  Backward recomputes the filtered moments, forms the five
// per-pixel map derivatives, applies the adjoint (transposed) separable
// filter, and walks the pyramid coarse -> fine through the adjoint of
// reflect-pad + 2x2 average pooling.
//
// state (kept by the caller between fwd and bwd):
//   pyramid a_l, b_l (scaled by max_val) for every level, then
//   stats[l][P][2] = (sum cs, sum ssim) per plane and level.
#include "../../include/imgcomp.h"
#include "common.h"

namespace {

constexpr int MAXLEV = 8;
constexpr int MAXF = 15;

struct Geo {
  int N, C, P, nlev, fs;
  int H[MAXLEV], W[MAXLEV];
  long long off[MAXLEV];  // float offset of level l's a-pyramid (b follows at + P*H*W)
  long long stats_off;    // float offset of stats
  long long total;        // floats in state
};

bool make_geo(int N, int C, int H, int W, int nlev, int fs, Geo& g) {
  if (nlev < 1 || nlev > MAXLEV || fs < 1 || fs > MAXF) return false;
  g.N = N; g.C = C; g.P = N * C; g.nlev = nlev; g.fs = fs;
  long long o = 0;
  int h = H, w = W;
  for (int l = 0; l < nlev; ++l) {
    if (h < fs || w < fs) return false;
    g.H[l] = h; g.W[l] = w; g.off[l] = o;
    o += 2LL * g.P * h * w;
    h = (h + 1) / 2; w = (w + 1) / 2;
  }
  g.stats_off = o;
  o += (long long)nlev * g.P * 2;
  g.total = o;
  return true;
}

struct Filt {
  float g[MAXF];
  int fs;
};

Filt make_filt(int fs, float sigma) {
  Filt f;
  f.fs = fs;
  double e[MAXF], s = 0;
  for (int i = 0; i < fs; ++i) {
    const double r = i + 0.5 - fs / 2.0;
    e[i] = exp(-(r * r) / (2.0 * sigma * sigma));
    s += e[i];
  }
  for (int i = 0; i < fs; ++i) f.g[i] = (float)(e[i] / s);
  return f;
}

#define GS(i, n) for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < (n); i += (long long)gridDim.x * blockDim.x)

inline unsigned grid_for(long long n) {
  long long b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  return (unsigned)b;
}

__global__ void scale_copy_k(const float* a, const float* b, long long n, float s, float* oa, float* ob) {
  GS(i, n) { oa[i] = a[i] * s; ob[i] = b[i] * s; }
}

// reflect-pad (0,1) on odd sizes then 2x2 average pool
__device__ __forceinline__ int refl(int i, int n) { return i < n ? i : 2 * n - 2 - i; }
__global__ void down_k(const float* in, int P2, int H, int W, float* out) {
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;
  const long long n = (long long)P2 * Ho * Wo;
  GS(i, n) {
    const int x = (int)(i % Wo);
    const long long t = i / Wo;
    const int y = (int)(t % Ho);
    const long long p = t / Ho;
    const float* src = in + p * H * W;
    const int y0 = refl(2 * y, H), y1 = refl(2 * y + 1, H), x0 = refl(2 * x, W), x1 = refl(2 * x + 1, W);
    out[i] = (src[(long long)y0 * W + x0] + src[(long long)y0 * W + x1] + src[(long long)y1 * W + x0] +
              src[(long long)y1 * W + x1]) * 0.25f;
  }
}

// adjoint of down_k, accumulated into gin (gather form)
__global__ void down_adj_k(const float* gout, int P2, int H, int W, float* gin) {
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;
  const long long n = (long long)P2 * H * W;
  GS(i, n) {
    const int x = (int)(i % W);
    const long long t = i / W;
    const int y = (int)(t % H);
    const long long p = t / H;
    const float* g = gout + p * Ho * Wo;
    int ry[2], rx[2], nry = 1, nrx = 1;
    ry[0] = y / 2; rx[0] = x / 2;
    if ((H & 1) && y == H - 2) ry[nry++] = (H - 1) / 2;
    if ((W & 1) && x == W - 2) rx[nrx++] = (W - 1) / 2;
    float s = 0.f;
    for (int a = 0; a < nry; ++a)
      for (int b = 0; b < nrx; ++b) s += g[(long long)ry[a] * Wo + rx[b]];
    gin[i] += 0.25f * s;
  }
}

// horizontal valid pass over the 5 moments: th[q][p][y][xv]
__global__ void hfilt_k(const float* a, const float* b, int P, int H, int W, const Filt f, float* th) {
  const int Wv = W - f.fs + 1;
  const long long n = (long long)P * H * Wv;
  GS(i, n) {
    const int xv = (int)(i % Wv);
    const long long t = i / Wv;  // p*H + y
    const float* ra = a + t * W + xv;
    const float* rb = b + t * W + xv;
    float s0 = 0, s1 = 0, s2 = 0, s3 = 0, s4 = 0;
    for (int k = 0; k < f.fs; ++k) {
      const float g = f.g[k], va = ra[k], vb = rb[k];
      s0 += g * va; s1 += g * vb; s2 += g * (va * va); s3 += g * (vb * vb); s4 += g * (va * vb);
    }
    th[0 * n + i] = s0; th[1 * n + i] = s1; th[2 * n + i] = s2; th[3 * n + i] = s3; th[4 * n + i] = s4;
  }
}

struct Mom {
  float ma, mb, saa, sbb, sab;
};
__device__ __forceinline__ Mom vfilt_at(const float* th, long long nh, int H, int Wv, int p, int yv, int xv,
                                        const Filt& f) {
  Mom m = {0, 0, 0, 0, 0};
  const long long base = ((long long)p * H + yv) * Wv + xv;
  for (int k = 0; k < f.fs; ++k) {
    const float g = f.g[k];
    const long long o = base + (long long)k * Wv;
    m.ma += g * th[o]; m.mb += g * th[nh + o]; m.saa += g * th[2 * nh + o];
    m.sbb += g * th[3 * nh + o]; m.sab += g * th[4 * nh + o];
  }
  return m;
}

// per-plane sums of the cs and ssim maps; grid (blocks_per_plane, P)
__global__ void vstats_k(const float* th, int P, int H, int W, const Filt f, float c1, float c2, float* part) {
  __shared__ float lds[32];
  const int Wv = W - f.fs + 1, Hv = H - f.fs + 1;
  const long long nh = (long long)P * H * Wv;
  const int p = blockIdx.y;
  const long long npix = (long long)Hv * Wv;
  float v[2] = {0.f, 0.f};
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < npix; i += (long long)gridDim.x * blockDim.x) {
    const int yv = (int)(i / Wv), xv = (int)(i % Wv);
    const Mom m = vfilt_at(th, nh, H, Wv, p, yv, xv, f);
    const float mu12 = m.ma * m.mb;
    const float s1 = m.saa - m.ma * m.ma, s2 = m.sbb - m.mb * m.mb, s12 = m.sab - mu12;
    const float cs = (2.f * s12 + c2) / (s1 + s2 + c2);
    const float ss = cs * (2.f * mu12 + c1) / (m.ma * m.ma + m.mb * m.mb + c1);
    v[0] += cs; v[1] += ss;
  }
  block_sum<2>(v, lds);
  if (threadIdx.x == 0) {
    part[((long long)p * gridDim.x + blockIdx.x) * 2 + 0] = v[0];
    part[((long long)p * gridDim.x + blockIdx.x) * 2 + 1] = v[1];
  }
}

__global__ void vstats_final_k(const float* part, int P, int nb, float* stats) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  float a = 0, b = 0;
  for (int k = 0; k < nb; ++k) { a += part[((long long)p * nb + k) * 2]; b += part[((long long)p * nb + k) * 2 + 1]; }
  stats[p * 2] = a; stats[p * 2 + 1] = b;
}

struct Comb {
  int N, C, nlev, log_scale, single;
  float eps;
  float w[MAXLEV];
  float cnt[MAXLEV];  // C * Hv * Wv per level
};

// per-image value v[n] and the loss; stats at state + stats_off laid out [l][P][2]
__device__ __forceinline__ void level_means(const float* stats, const Comb& cb, int l, int n, float& cs, float& ss) {
  float a = 0, b = 0;
  for (int c = 0; c < cb.C; ++c) {
    const long long idx = ((long long)l * cb.N * cb.C + (long long)n * cb.C + c) * 2;
    a += stats[idx]; b += stats[idx + 1];
  }
  cs = a / cb.cnt[l];
  ss = b / cb.cnt[l];
}

__global__ void combine_k(const float* stats, const Comb cb, float* out) {
  // single block
  __shared__ float vals[1024];
  for (int n = threadIdx.x; n < cb.N; n += blockDim.x) {
    float v = cb.log_scale ? 0.f : 1.f;
    for (int l = 0; l < cb.nlev; ++l) {
      float cs, ss;
      level_means(stats, cb, l, n, cs, ss);
      const float e = cb.log_scale ? cb.eps : 0.f;
      cs = fmaxf(cs, e); ss = fmaxf(ss, e);
      const float t = (l < cb.nlev - 1) ? cs : ss;
      if (cb.log_scale) v += logf(t) * cb.w[l];
      else v *= (cb.single == 1 ? t : powf(t, cb.w[l]));
    }
    if (cb.single == 2) out[n] = -10.f * logf(1.f - v) / 2.302585092994046f;  // metric, dB per image
    else if (cb.single && cb.log_scale) out[n] = -v;
    else vals[n] = v;
  }
  __syncthreads();
  if (threadIdx.x == 0 && cb.single != 2 && !(cb.single && cb.log_scale)) {
    float s = 0;
    for (int n = 0; n < cb.N; ++n) s += vals[n];
    const float m = s / (float)cb.N;
    out[0] = cb.log_scale ? -m : 1.f - m;
  }
}

// coefficients gc[l][n], gs[l][n] = dLoss / d(map value) for each pixel of plane n*C+c
__global__ void coef_k(const float* stats, const Comb cb, const float* gout, float* coef) {
  for (int n = threadIdx.x; n < cb.N; n += blockDim.x) {
    // dLoss/dv[n]
    float gv;
    if (cb.single && cb.log_scale) gv = -gout[n];
    else gv = (cb.log_scale ? -gout[0] : -gout[0]) / (float)cb.N;
    // v = sum w_l log(t_l)  or  prod t_l^w_l
    float tv[MAXLEV], traw[MAXLEV];
    float prod = 1.f;
    for (int l = 0; l < cb.nlev; ++l) {
      float cs, ss;
      level_means(stats, cb, l, n, cs, ss);
      traw[l] = (l < cb.nlev - 1) ? cs : ss;
      const float e = cb.log_scale ? cb.eps : 0.f;
      tv[l] = fmaxf(traw[l], e);
      prod *= cb.log_scale ? 1.f : (cb.single ? tv[l] : powf(tv[l], cb.w[l]));
    }
    for (int l = 0; l < cb.nlev; ++l) {
      float dt;
      if (cb.log_scale) dt = gv * cb.w[l] / tv[l];
      else if (cb.single) dt = gv;  // v = t
      else dt = gv * prod * cb.w[l] / tv[l];
      const float e = cb.log_scale ? cb.eps : 0.f;
      // LowerBound backward (bound.py:36-42)
      if (!(traw[l] >= e || dt < 0.f)) dt = 0.f;
      const float per_pix = dt / cb.cnt[l];
      const bool is_ss = !(l < cb.nlev - 1);
      coef[((long long)l * cb.N + n) * 2 + 0] = is_ss ? 0.f : per_pix;  // d/d cs-map
      coef[((long long)l * cb.N + n) * 2 + 1] = is_ss ? per_pix : 0.f;  // d/d ssim-map
    }
  }
}

// per valid pixel: derivatives wrt the five filtered moments -> D[q][p][yv][xv]
__global__ void dmaps_k(const float* th, int P, int C, int H, int W, const Filt f, float c1, float c2,
                        const float* coef_l, float* D) {
  const int Wv = W - f.fs + 1, Hv = H - f.fs + 1;
  const long long nh = (long long)P * H * Wv;
  const long long nv = (long long)P * Hv * Wv;
  GS(i, nv) {
    const int xv = (int)(i % Wv);
    const long long t = i / Wv;
    const int yv = (int)(t % Hv);
    const int p = (int)(t / Hv);
    const int n = p / C;
    const float gC = coef_l[n * 2], gS = coef_l[n * 2 + 1];
    const Mom m = vfilt_at(th, nh, H, Wv, p, yv, xv, f);
    const float A1 = 2.f * m.ma * m.mb + c1, B1 = m.ma * m.ma + m.mb * m.mb + c1;
    const float A2 = 2.f * (m.sab - m.ma * m.mb) + c2;
    const float B2 = (m.saa - m.ma * m.ma) + (m.sbb - m.mb * m.mb) + c2;
    const float cs = A2 / B2, lum = A1 / B1;
    const float ucs = gC + gS * lum, ul = gS * cs;
    const float gA2 = ucs / B2, gB2 = -ucs * A2 / (B2 * B2);
    const float gA1 = ul / B1, gB1 = -ul * A1 / (B1 * B1);
    const float dma = -2.f * m.mb * gA2 - 2.f * m.ma * gB2 + 2.f * m.mb * gA1 + 2.f * m.ma * gB1;
    const float dmb = -2.f * m.ma * gA2 - 2.f * m.mb * gB2 + 2.f * m.ma * gA1 + 2.f * m.mb * gB1;
    D[0 * nv + i] = dma; D[1 * nv + i] = dmb; D[2 * nv + i] = gB2; D[3 * nv + i] = gB2; D[4 * nv + i] = 2.f * gA2;
  }
}

// vertical adjoint: E[q][p][y][xv] = sum_k g[k] D[q][p][y-k][xv]
__global__ void vadj_k(const float* D, int P, int H, int W, const Filt f, float* E) {
  const int Wv = W - f.fs + 1, Hv = H - f.fs + 1;
  const long long nv = (long long)P * Hv * Wv, nh = (long long)P * H * Wv;
  GS(i, nh) {
    const int xv = (int)(i % Wv);
    const long long t = i / Wv;
    const int y = (int)(t % H);
    const int p = (int)(t / H);
    float s[5] = {0, 0, 0, 0, 0};
    for (int k = 0; k < f.fs; ++k) {
      const int yv = y - k;
      if (yv < 0 || yv >= Hv) continue;
      const long long o = ((long long)p * Hv + yv) * Wv + xv;
      const float g = f.g[k];
#pragma unroll
      for (int q = 0; q < 5; ++q) s[q] += g * D[q * nv + o];
    }
#pragma unroll
    for (int q = 0; q < 5; ++q) E[q * nh + i] = s[q];
  }
}

// horizontal adjoint + moment chain rule, accumulated into (ga, gb) of this level
__global__ void hadj_k(const float* E, const float* a, const float* b, int P, int H, int W, const Filt f,
                       float* ga, float* gb) {
  const int Wv = W - f.fs + 1;
  const long long nh = (long long)P * H * Wv, n = (long long)P * H * W;
  GS(i, n) {
    const int x = (int)(i % W);
    const long long t = i / W;  // p*H + y
    float s[5] = {0, 0, 0, 0, 0};
    for (int k = 0; k < f.fs; ++k) {
      const int xv = x - k;
      if (xv < 0 || xv >= Wv) continue;
      const long long o = t * Wv + xv;
      const float g = f.g[k];
#pragma unroll
      for (int q = 0; q < 5; ++q) s[q] += g * E[q * nh + o];
    }
    const float va = a[i], vb = b[i];
    ga[i] += s[0] + 2.f * va * s[2] + vb * s[4];
    gb[i] += s[1] + 2.f * vb * s[3] + va * s[4];
  }
}

__global__ void scale_out_k(const float* ga, const float* gb, long long n, float s, float* oa, float* ob) {
  GS(i, n) {
    if (oa) oa[i] = ga[i] * s;
    if (ob) ob[i] = gb[i] * s;
  }
}

// ---------------------------------------------------------------- fused tile kernels (filter size 11)
// One block per (tile, plane) does a level's whole separable filtering in LDS, so the five filtered
// moment images (and in the backward the five derivative maps and their vertical adjoint) never go
// to HBM: the forward reads a and b once per level, the backward reads a, b and the level's gradient
// once and writes the gradient once.  The naive chain (hfilt -> vstats; hfilt -> dmaps -> vadj -> hadj)
// wrote and re-read 5 moment planes two to three times per level (C4 level 0: 63 MB each).
#ifndef MSSSIM_FUSED
#define MSSSIM_FUSED 1
#endif
constexpr int FMAX = 11;                      // fused kernels: filter size 11 (every reference config)
constexpr int FTW = 64, FTH = 16;             // forward: valid outputs per tile
constexpr int FRW = FTW + FMAX - 1, FRH = FTH + FMAX - 1;
constexpr int FAP = 76;                       // forward input pitch (>= FRW, four-aligned 14-wide windows)
// backward: gradient pixels per tile.  32 x 22: the phases' work items (42 x 11 moment rows, 32 x 11
// derivative rows, 22 x 11 adjoint rows, 22 x 8 output groups) take as many 256-thread rounds as 32 x 16
// took (2, 2, 1, 1) for 1.375x the pixels; 78 KB of LDS, two blocks per CU
constexpr int BTW = 32, BTH = 22;
constexpr int BDW = BTW + FMAX - 1, BDH = BTH + FMAX - 1;          // derivative-map region
constexpr int BDP = 44;                       // its pitch: 11 groups of four columns
constexpr int BIW = BTW + 2 * (FMAX - 1), BIH = BTH + 2 * (FMAX - 1);  // input region
constexpr int BAP = 56;                       // backward input pitch (>= BDP + 12)
static_assert(FRW <= FAP && FAP >= FTW + 12 && BDW <= BDP && BIW <= BAP && BAP >= BDP + 12, "tile pitches");

// Every pass of the fused kernels works on four consecutive columns per thread: the 14 inputs a
// four-output window of the 11-tap filter needs are four 16-B LDS reads (three to five times fewer LDS
// instructions than one column per thread, which left the level-0 backward LDS-bound), and the
// division-heavy SSIM formulas use one reciprocal per denominator (v_rcp_f32, 1 ulp: relative ~1e-7,
// far inside the 1e-4 bar).
__device__ __forceinline__ void ld16(const float* p, float (&v)[16]) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const floatx4v t = *(const floatx4v*)(p + 4 * k);
    v[4 * k] = t[0]; v[4 * k + 1] = t[1]; v[4 * k + 2] = t[2]; v[4 * k + 3] = t[3];
  }
}
__device__ __forceinline__ void st4(float* p, const float (&v)[4]) { *(floatx4v*)p = floatx4v{v[0], v[1], v[2], v[3]}; }
__device__ __forceinline__ floatx4v ld4(const float* p) { return *(const floatx4v*)p; }

// horizontal pass of one row, four output columns: m[q][o] = sum_k g[k] mom_q(a[o + k], b[o + k])
template <int FS>
__device__ __forceinline__ void hmom4(const float* ar, const float* br, const Filt& f, float (&m)[5][4]) {
  float va[16], vb[16];
  ld16(ar, va);
  ld16(br, vb);
#pragma unroll
  for (int o = 0; o < 4; ++o) {
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f, s4 = 0.f;
#pragma unroll
    for (int k = 0; k < FS; ++k) {
      const float g = f.g[k], x = va[o + k], y = vb[o + k];
      s0 += g * x; s1 += g * y; s2 += g * (x * x); s3 += g * (y * y); s4 += g * (x * y);
    }
    m[0][o] = s0; m[1][o] = s1; m[2][o] = s2; m[3][o] = s3; m[4][o] = s4;
  }
}

// forward: per tile of FTW x FTH valid outputs, the per-plane partial sums of the cs and ssim maps
// (part[p][tile][2], summed per plane in a fixed order by vstats_final_k)
// FS (the filter size) is a template constant: fully unrolled taps, the weights in SGPRs
template <int FS>
__global__ void __launch_bounds__(256) ssim_fwd_tile_k(const float* __restrict__ a, const float* __restrict__ b,
                                                       int H, int W, const Filt f, float c1, float c2,
                                                       float* __restrict__ part) {
  static_assert(FS <= FMAX, "LDS regions sized for FMAX");
  __shared__ __attribute__((aligned(16))) float A[FRH][FAP], B[FRH][FAP];
  __shared__ __attribute__((aligned(16))) float HM[5][FRH][FTW];
  __shared__ float red[32];
  constexpr int fs = FS;
  const int Wv = W - fs + 1, Hv = H - fs + 1;
  const int p = blockIdx.z;
  const int x0 = blockIdx.x * FTW, y0 = blockIdx.y * FTH;
  const int tid = threadIdx.x;
  const float* pa = a + (long long)p * H * W;
  const float* pb = b + (long long)p * H * W;
  const int rw = min(FTW, Wv - x0) + fs - 1, rh = min(FTH, Hv - y0) + fs - 1;
  for (int i = tid; i < FRH * FAP; i += 256) {
    const int r = i / FAP, c = i - (i / FAP) * FAP;
    const bool in = r < rh && c < rw;
    const long long o = (long long)(y0 + r) * W + x0 + c;
    A[r][c] = in ? pa[o] : 0.f;
    B[r][c] = in ? pb[o] : 0.f;
  }
  __syncthreads();
  for (int i = tid; i < FRH * (FTW / 4); i += 256) {
    const int r = i / (FTW / 4), c = 4 * (i - (i / (FTW / 4)) * (FTW / 4));
    float m[5][4];
    hmom4<FS>(&A[r][c], &B[r][c], f, m);
#pragma unroll
    for (int q = 0; q < 5; ++q) st4(&HM[q][r][c], m[q]);
  }
  __syncthreads();
  float v0 = 0.f, v1 = 0.f;
  for (int i = tid; i < FTH * (FTW / 4); i += 256) {
    const int r = i / (FTW / 4), c = 4 * (i - (i / (FTW / 4)) * (FTW / 4));
    floatx4v mm[5];
#pragma unroll
    for (int q = 0; q < 5; ++q) mm[q] = floatx4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < FS; ++k) {
      const float g = f.g[k];
#pragma unroll
      for (int q = 0; q < 5; ++q) mm[q] += g * ld4(&HM[q][r + k][c]);
    }
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      if (y0 + r >= Hv || x0 + c + o >= Wv) continue;
      const float ma = mm[0][o], mb = mm[1][o];
      const float mu12 = ma * mb;
      const float s1 = mm[2][o] - ma * ma, s2 = mm[3][o] - mb * mb, s12 = mm[4][o] - mu12;
      const float cs = (2.f * s12 + c2) * __builtin_amdgcn_rcpf(s1 + s2 + c2);
      v0 += cs;
      v1 += cs * (2.f * mu12 + c1) * __builtin_amdgcn_rcpf(ma * ma + mb * mb + c1);
    }
  }
  float v[2] = {v0, v1};
  block_sum<2>(v, red);
  if (tid == 0) {
    const long long t = (long long)p * gridDim.x * gridDim.y + blockIdx.y * gridDim.x + blockIdx.x;
    part[t * 2] = v[0];
    part[t * 2 + 1] = v[1];
  }
}

// backward: per tile of BTW x BTH pixels of a level, the gradient contribution of that level's map
// sums (coef_l = dLoss / d(per-pixel cs, ssim) for each image), accumulated into (ga, gb).
//   D (four maps: d/d ma, mb, saa = sbb, sab) at the valid outputs whose windows reach the tile, from
//   the moments recomputed there; E = vertical adjoint of D on the tile rows; the horizontal adjoint
//   and the moments' chain rule onto the tile pixels (as dmaps_k -> vadj_k -> hadj_k)
template <int FS>
__global__ void __launch_bounds__(256) ssim_bwd_tile_k(const float* __restrict__ a, const float* __restrict__ b,
                                                       int C, int H, int W, const Filt f, float c1, float c2,
                                                       const float* __restrict__ coef_l, float* __restrict__ ga,
                                                       float* __restrict__ gb) {
  static_assert(FS <= FMAX, "LDS regions sized for FMAX");
  __shared__ __attribute__((aligned(16))) float A[BIH][BAP], B[BIH][BAP];
  __shared__ __attribute__((aligned(16))) float HM[5][BIH][BDP];  // horizontal moments; then E[4][BTH][BDP]
  __shared__ __attribute__((aligned(16))) float D[4][BDH][BDP];
  constexpr int fs = FS, h = FS - 1;
  constexpr int NC = BDP / 4;  // column groups of the moment / derivative regions
  const int Wv = W - fs + 1, Hv = H - fs + 1;
  const int p = blockIdx.z, n = p / C;
  const int x0 = blockIdx.x * BTW, y0 = blockIdx.y * BTH;
  const int ox = x0 - h, oy = y0 - h;  // origin of the input and D regions
  constexpr int ih = BTH + 2 * h, dh = BTH + h, dw = BTW + h;
  const int tid = threadIdx.x;
  const float* pa = a + (long long)p * H * W;
  const float* pb = b + (long long)p * H * W;
  const float gC = coef_l[n * 2], gS = coef_l[n * 2 + 1];
  for (int i = tid; i < ih * BAP; i += 256) {
    const int r = i / BAP, c = i - (i / BAP) * BAP;
    const int y = oy + r, x = ox + c;
    const bool in = (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W && c < BIW;
    const long long o = (long long)y * W + x;
    A[r][c] = in ? pa[o] : 0.f;
    B[r][c] = in ? pb[o] : 0.f;
  }
  __syncthreads();
  for (int i = tid; i < ih * NC; i += 256) {
    const int r = i / NC, c = 4 * (i - (i / NC) * NC);
    float m[5][4];
    hmom4<FS>(&A[r][c], &B[r][c], f, m);
#pragma unroll
    for (int q = 0; q < 5; ++q) st4(&HM[q][r][c], m[q]);
  }
  __syncthreads();
  for (int i = tid; i < dh * NC; i += 256) {
    const int r = i / NC, c = 4 * (i - (i / NC) * NC);
    floatx4v mm[5];
#pragma unroll
    for (int q = 0; q < 5; ++q) mm[q] = floatx4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < FS; ++k) {
      const float g = f.g[k];
#pragma unroll
      for (int q = 0; q < 5; ++q) mm[q] += g * ld4(&HM[q][r + k][c]);
    }
    float d[4][4];
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      const int yv = oy + r, xv = ox + c + o;
      const bool valid = (unsigned)yv < (unsigned)Hv && (unsigned)xv < (unsigned)Wv && c + o < dw;
      const float ma = mm[0][o], mb = mm[1][o];
      const float A1 = 2.f * ma * mb + c1, B1 = ma * ma + mb * mb + c1;
      const float A2 = 2.f * (mm[4][o] - ma * mb) + c2;
      const float B2 = (mm[2][o] - ma * ma) + (mm[3][o] - mb * mb) + c2;
      const float iB1 = __builtin_amdgcn_rcpf(B1), iB2 = __builtin_amdgcn_rcpf(B2);
      const float cs = A2 * iB2, lum = A1 * iB1;
      const float ucs = gC + gS * lum, ul = gS * cs;
      const float gA2 = ucs * iB2, gB2 = -gA2 * cs;   // -ucs A2 / B2^2
      const float gA1 = ul * iB1, gB1 = -gA1 * lum;   // -ul A1 / B1^2
      d[0][o] = valid ? -2.f * mb * gA2 - 2.f * ma * gB2 + 2.f * mb * gA1 + 2.f * ma * gB1 : 0.f;
      d[1][o] = valid ? -2.f * ma * gA2 - 2.f * mb * gB2 + 2.f * ma * gA1 + 2.f * mb * gB1 : 0.f;
      d[2][o] = valid ? gB2 : 0.f;
      d[3][o] = valid ? 2.f * gA2 : 0.f;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) st4(&D[q][r][c], d[q]);
  }
  __syncthreads();
  // vertical adjoint onto the tile rows: E[q][y][c] = sum_k g[k] D[q][y + h - k][c]  (E over HM)
  float (*E)[BIH][BDP] = HM;
  for (int i = tid; i < BTH * NC; i += 256) {
    const int y = i / NC, c = 4 * (i - (i / NC) * NC);
    floatx4v e[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) e[q] = floatx4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < FS; ++k) {
      const float g = f.g[k];
#pragma unroll
      for (int q = 0; q < 4; ++q) e[q] += g * ld4(&D[q][y + h - k][c]);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) *(floatx4v*)&E[q][y][c] = e[q];
  }
  __syncthreads();
  // horizontal adjoint and the moments' chain rule (hadj_k): s_q[y][x] = sum_k g[k] E[q][y][x + h - k]
  for (int i = tid; i < BTH * (BTW / 4); i += 256) {
    const int y = i / (BTW / 4), x = 4 * (i - (i / (BTW / 4)) * (BTW / 4));
    float s[4][4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float ev[16];
      ld16(&E[q][y][x], ev);  // columns x .. x + 15 hold x + h - k for k = 0..10 and the four outputs
#pragma unroll
      for (int o = 0; o < 4; ++o) {
        float t = 0.f;
#pragma unroll
        for (int k = 0; k < FS; ++k) t += f.g[k] * ev[o + h - k];
        s[q][o] = t;
      }
    }
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      if (y0 + y >= H || x0 + x + o >= W) continue;
      const float va = A[y + h][x + o + h], vb = B[y + h][x + o + h];
      const long long off = (long long)p * H * W + (long long)(y0 + y) * W + x0 + x + o;
      ga[off] += s[0][o] + 2.f * va * s[2][o] + vb * s[3][o];
      gb[off] += s[1][o] + 2.f * vb * s[2][o] + va * s[3][o];
    }
  }
}

int vstats_blocks(int Hv, int Wv) {
  long long n = (long long)Hv * Wv;
  long long b = (n + 255) / 256;
  if (b > 64) b = 64;
  if (b < 1) b = 1;
  return (int)b;
}

bool fused_ok(const Geo& g) { return MSSSIM_FUSED && g.fs == FMAX; }

// forward tiles per plane of level l (fused path)
int fwd_tiles(const Geo& g, int l, int& tx, int& ty) {
  tx = (g.W[l] - g.fs + 1 + FTW - 1) / FTW;
  ty = (g.H[l] - g.fs + 1 + FTH - 1) / FTH;
  return tx * ty;
}

size_t fwd_ws_bytes(const Geo& g) {
  // th (5 planes at the largest level; naive path only) + stats partials (per plane: <= 64 blocks of
  // vstats_k, or one per forward tile)
  const long long Wv = g.W[0] - g.fs + 1;
  size_t th = fused_ok(g) ? 0 : (size_t)5 * g.P * g.H[0] * Wv * 4;
  int nb = 64;
  if (fused_ok(g))
    for (int l = 0; l < g.nlev; ++l) {
      int tx, ty;
      nb = max(nb, fwd_tiles(g, l, tx, ty));
    }
  size_t part = (size_t)g.P * nb * 2 * 4;
  return ic_align(th, 256) + ic_align(part, 256);
}

size_t bwd_ws_bytes(const Geo& g) {
  const long long Wv = g.W[0] - g.fs + 1, Hv = g.H[0] - g.fs + 1;
  size_t th = fused_ok(g) ? 0 : (size_t)5 * g.P * g.H[0] * Wv * 4;
  size_t D = fused_ok(g) ? 0 : (size_t)5 * g.P * Hv * Wv * 4;
  size_t E = th;
  size_t grads = 0;
  for (int l = 0; l < g.nlev; ++l) grads += (size_t)2 * g.P * g.H[l] * g.W[l] * 4;
  size_t coef = (size_t)g.nlev * g.N * 2 * 4;
  return ic_align(th, 256) + ic_align(D, 256) + ic_align(E, 256) + ic_align(grads, 256) + ic_align(coef, 256);
}

Comb make_comb(const Geo& g, int log_scale, int single, float eps, const float* weights) {
  Comb cb;
  cb.N = g.N; cb.C = g.C; cb.nlev = g.nlev; cb.log_scale = log_scale; cb.single = single; cb.eps = eps;
  for (int l = 0; l < g.nlev; ++l) {
    cb.w[l] = weights ? weights[l] : 1.f;
    cb.cnt[l] = (float)((long long)g.C * (g.H[l] - g.fs + 1) * (g.W[l] - g.fs + 1));
  }
  return cb;
}

}  // namespace

extern "C" {

size_t ic_msssim_state_bytes(int N, int C, int H, int W, int nlev, int filter_size) {
  Geo g;
  if (!make_geo(N, C, H, W, nlev, filter_size, g)) return 0;
  return (size_t)g.total * 4;
}

size_t ic_msssim_ws(int N, int C, int H, int W, int nlev, int filter_size) {
  Geo g;
  if (!make_geo(N, C, H, W, nlev, filter_size, g)) return 0;
  const size_t a = fwd_ws_bytes(g), b = bwd_ws_bytes(g);
  return a > b ? a : b;
}

int ic_msssim_fwd(const float* a, const float* b, int N, int C, int H, int W, int nlev, int filter_size,
                  float filter_sigma, float max_val, int log_scale, int single, float k1, float k2, float eps,
                  const float* weights, float* out, float* state, void* ws, size_t ws_bytes, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  Geo g;
  if (!make_geo(N, C, H, W, nlev, filter_size, g) || g.N > 1024) return IC_ERR_ARG;
  if (ws_bytes < fwd_ws_bytes(g)) return IC_ERR_WORKSPACE;
  const Filt f = make_filt(filter_size, filter_sigma);
  const float c1 = (k1 * max_val) * (k1 * max_val), c2 = (k2 * max_val) * (k2 * max_val);
  char* wsb = (char*)ws;
  float* th = (float*)wsb;
  float* part = (float*)(wsb + (fused_ok(g) ? 0 : ic_align((size_t)5 * g.P * g.H[0] * (g.W[0] - g.fs + 1) * 4, 256)));
  const long long n0 = (long long)g.P * H * W;
  hipLaunchKernelGGL(scale_copy_k, dim3(grid_for(n0)), dim3(256), 0, s, a, b, n0, max_val, state + g.off[0],
                     state + g.off[0] + n0);
  IC_CHECK_LAUNCH();
  for (int l = 0; l < nlev; ++l) {
    const int Hl = g.H[l], Wl = g.W[l];
    const long long nl = (long long)g.P * Hl * Wl;
    const float* al = state + g.off[l];
    const float* bl = al + nl;
    if (l > 0) {
      const long long np = (long long)g.P * g.H[l - 1] * g.W[l - 1];
      // a and b of level l-1 are contiguous: pool both planes sets in one launch
      hipLaunchKernelGGL(down_k, dim3(grid_for(2 * nl)), dim3(256), 0, s, state + g.off[l - 1], 2 * g.P,
                         g.H[l - 1], g.W[l - 1], state + g.off[l]);
      IC_CHECK_LAUNCH();
      (void)np;
    }
    int nb;
    if (fused_ok(g)) {
      int tx, ty;
      nb = fwd_tiles(g, l, tx, ty);
      hipLaunchKernelGGL(ssim_fwd_tile_k<FMAX>, dim3(tx, ty, g.P), dim3(256), 0, s, al, bl, Hl, Wl, f, c1, c2, part);
      IC_CHECK_LAUNCH();
    } else {
      const long long nhf = (long long)g.P * Hl * (Wl - g.fs + 1);
      hipLaunchKernelGGL(hfilt_k, dim3(grid_for(nhf)), dim3(256), 0, s, al, bl, g.P, Hl, Wl, f, th);
      IC_CHECK_LAUNCH();
      nb = vstats_blocks(Hl - g.fs + 1, Wl - g.fs + 1);
      hipLaunchKernelGGL(vstats_k, dim3(nb, g.P), dim3(256), 0, s, th, g.P, Hl, Wl, f, c1, c2, part);
      IC_CHECK_LAUNCH();
    }
    hipLaunchKernelGGL(vstats_final_k, dim3((g.P + 255) / 256), dim3(256), 0, s, part, g.P, nb,
                       state + g.stats_off + (long long)l * g.P * 2);
    IC_CHECK_LAUNCH();
  }
  const Comb cb = make_comb(g, log_scale, single, eps, weights);
  hipLaunchKernelGGL(combine_k, dim3(1), dim3(256), 0, s, state + g.stats_off, cb, out);
  IC_CHECK_LAUNCH();
  return IC_OK;
}

int ic_msssim_bwd(int N, int C, int H, int W, int nlev, int filter_size, float filter_sigma, float max_val,
                  int log_scale, int single, float k1, float k2, float eps, const float* weights,
                  const float* gout, const float* state, float* ga, float* gb, void* ws, size_t ws_bytes,
                  void* stream) {
  hipStream_t s = (hipStream_t)stream;
  Geo g;
  if (!make_geo(N, C, H, W, nlev, filter_size, g) || g.N > 1024) return IC_ERR_ARG;
  if (ws_bytes < bwd_ws_bytes(g)) return IC_ERR_WORKSPACE;
  const Filt f = make_filt(filter_size, filter_sigma);
  const float c1 = (k1 * max_val) * (k1 * max_val), c2 = (k2 * max_val) * (k2 * max_val);
  const long long Wv0 = g.W[0] - g.fs + 1, Hv0 = g.H[0] - g.fs + 1;
  const bool fz = fused_ok(g);
  char* p = (char*)ws;
  float* th = (float*)p; p += fz ? 0 : ic_align((size_t)5 * g.P * g.H[0] * Wv0 * 4, 256);
  float* D = (float*)p; p += fz ? 0 : ic_align((size_t)5 * g.P * Hv0 * Wv0 * 4, 256);
  float* E = (float*)p; p += fz ? 0 : ic_align((size_t)5 * g.P * g.H[0] * Wv0 * 4, 256);
  float* grads = (float*)p;
  long long goff[MAXLEV];
  long long gt = 0;
  for (int l = 0; l < nlev; ++l) { goff[l] = gt; gt += 2LL * g.P * g.H[l] * g.W[l]; }
  p += ic_align((size_t)gt * 4, 256);
  float* coef = (float*)p;
  if (hipMemsetAsync(grads, 0, (size_t)gt * 4, s) != hipSuccess) return IC_ERR_ARG;
  const Comb cb = make_comb(g, log_scale, single, eps, weights);
  hipLaunchKernelGGL(coef_k, dim3(1), dim3(256), 0, s, state + g.stats_off, cb, gout, coef);
  IC_CHECK_LAUNCH();
  for (int l = nlev - 1; l >= 0; --l) {
    const int Hl = g.H[l], Wl = g.W[l];
    const long long nl = (long long)g.P * Hl * Wl;
    const float* al = state + g.off[l];
    const float* bl = al + nl;
    float* gal = grads + goff[l];
    float* gbl = gal + nl;
    if (l < nlev - 1) {
      // pull the coarser level's gradient back through pooling (a and b together)
      hipLaunchKernelGGL(down_adj_k, dim3(grid_for(2 * nl)), dim3(256), 0, s, grads + goff[l + 1], 2 * g.P, Hl, Wl,
                         gal);
      IC_CHECK_LAUNCH();
    }
    if (fz) {
      hipLaunchKernelGGL(ssim_bwd_tile_k<FMAX>, dim3((Wl + BTW - 1) / BTW, (Hl + BTH - 1) / BTH, g.P), dim3(256), 0, s, al,
                         bl, g.C, Hl, Wl, f, c1, c2, coef + (long long)l * g.N * 2, gal, gbl);
      IC_CHECK_LAUNCH();
      continue;
    }
    const long long Wv = Wl - g.fs + 1, Hv = Hl - g.fs + 1;
    const long long nhf = (long long)g.P * Hl * Wv, nv = (long long)g.P * Hv * Wv;
    hipLaunchKernelGGL(hfilt_k, dim3(grid_for(nhf)), dim3(256), 0, s, al, bl, g.P, Hl, Wl, f, th);
    IC_CHECK_LAUNCH();
    hipLaunchKernelGGL(dmaps_k, dim3(grid_for(nv)), dim3(256), 0, s, th, g.P, g.C, Hl, Wl, f, c1, c2,
                       coef + (long long)l * g.N * 2, D);
    IC_CHECK_LAUNCH();
    hipLaunchKernelGGL(vadj_k, dim3(grid_for(nhf)), dim3(256), 0, s, D, g.P, Hl, Wl, f, E);
    IC_CHECK_LAUNCH();
    hipLaunchKernelGGL(hadj_k, dim3(grid_for(nl)), dim3(256), 0, s, E, al, bl, g.P, Hl, Wl, f, gal, gbl);
    IC_CHECK_LAUNCH();
  }
  const long long n0 = (long long)g.P * H * W;
  hipLaunchKernelGGL(scale_out_k, dim3(grid_for(n0)), dim3(256), 0, s, grads, grads + n0, n0, max_val, ga, gb);
  IC_CHECK_LAUNCH();
  return IC_OK;
}

}  // extern "C"
