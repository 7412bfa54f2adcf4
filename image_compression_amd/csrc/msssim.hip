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

int vstats_blocks(int Hv, int Wv) {
  long long n = (long long)Hv * Wv;
  long long b = (n + 255) / 256;
  if (b > 64) b = 64;
  if (b < 1) b = 1;
  return (int)b;
}

size_t fwd_ws_bytes(const Geo& g) {
  // th (5 planes at the largest level) + stats partials
  const long long Wv = g.W[0] - g.fs + 1;
  size_t th = (size_t)5 * g.P * g.H[0] * Wv * 4;
  size_t part = (size_t)g.P * 64 * 2 * 4;
  return ic_align(th, 256) + ic_align(part, 256);
}

size_t bwd_ws_bytes(const Geo& g) {
  const long long Wv = g.W[0] - g.fs + 1, Hv = g.H[0] - g.fs + 1;
  size_t th = (size_t)5 * g.P * g.H[0] * Wv * 4;
  size_t D = (size_t)5 * g.P * Hv * Wv * 4;
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
  float* part = (float*)(wsb + ic_align((size_t)5 * g.P * g.H[0] * (g.W[0] - g.fs + 1) * 4, 256));
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
    const long long nhf = (long long)g.P * Hl * (Wl - g.fs + 1);
    hipLaunchKernelGGL(hfilt_k, dim3(grid_for(nhf)), dim3(256), 0, s, al, bl, g.P, Hl, Wl, f, th);
    IC_CHECK_LAUNCH();
    const int nb = vstats_blocks(Hl - g.fs + 1, Wl - g.fs + 1);
    hipLaunchKernelGGL(vstats_k, dim3(nb, g.P), dim3(256), 0, s, th, g.P, Hl, Wl, f, c1, c2, part);
    IC_CHECK_LAUNCH();
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
  char* p = (char*)ws;
  float* th = (float*)p; p += ic_align((size_t)5 * g.P * g.H[0] * Wv0 * 4, 256);
  float* D = (float*)p; p += ic_align((size_t)5 * g.P * Hv0 * Wv0 * 4, 256);
  float* E = (float*)p; p += ic_align((size_t)5 * g.P * g.H[0] * Wv0 * 4, 256);
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
