// Weight-gradient GEMM on fp32 MFMA (v_mfma_f32_32x32x2_f32), gfx950.
//
//   C[g][col] = sum_p G[p][g] * X[p*s + d_t][c]      (col = c on the fast path,
//                                                     col = (t,c) flattened generic)
// The reduction runs over output pixels p, split across blocks (split-K) so
// that a 25-tap 192x192 layer still launches ~1000 blocks; every block writes a
// partial slab and a second kernel sums the slabs in a fixed order
// (deterministic, no float atomics) while scattering into the PyTorch weight
// layout [g][c][ky][kx].
//
// LDS holds BK=16 pixel rows of both operands, channel-contiguous (exactly as
// they sit in NHWC memory); a half-wave reads 32 consecutive floats of one row
// per operand fragment (ds_read_b32, conflict-free).
#include "gemm.h"

namespace {

template <int BM, int BN, int WM, int WN, bool GEN>
__global__ void __launch_bounds__(256, 2) wg_kernel(const WgDesc d) {
  constexpr int BK = 16;
  constexpr int WAVES_N = BN / WN;
  constexpr int TM = WM / 32, TN = WN / 32;
  constexpr int G4 = BM / 4, X4 = BN / 4;              // float4 per row
  constexpr int GPASS = (BK * G4 + 255) / 256, XPASS = (BK * X4 + 255) / 256;
  static_assert((BM / WM) * (BN / WN) == 4, "4 waves per block");
  __shared__ __attribute__((aligned(16))) float Gs[BK * BM];
  __shared__ __attribute__((aligned(16))) float Xs[BK * BN];

  const int tiles = d.mtiles * d.ntiles;
  const int bx = blockIdx.x;
  const int t = GEN ? 0 : bx / tiles;
  const int rem = bx - t * tiles;
  const int mt = rem / d.ntiles, nt = rem - (rem / d.ntiles) * d.ntiles;
  const int g0 = mt * BM, c0 = nt * BN;
  const int split = blockIdx.y;
  const long long pb = (long long)split * d.pps;
  long long pe = pb + d.pps;
  if (pe > d.P) pe = d.P;
  const long long HW = (long long)d.Hg * d.Wg;
  const int tid = threadIdx.x;
  const int dyt = GEN ? 0 : d.dy[t], dxt = GEN ? 0 : d.dx[t];

  floatx4v rg[GPASS], rx[XPASS];

  auto gload = [&](long long p0) {
#pragma unroll
    for (int q = 0; q < GPASS; ++q) {
      const int f = tid + 256 * q;
      floatx4v v = {0.f, 0.f, 0.f, 0.f};
      if (f < BK * G4) {
        const int row = f / G4, c4 = f - (f / G4) * G4;
        const long long p = p0 + row;
        const int col = g0 + c4 * 4;
        if (p < pe && col < d.Cg) {
          const long long img = p / HW;
          const long long rr = p - img * HW;
          const int gy = (int)(rr / d.Wg), gx = (int)(rr - (long long)(rr / d.Wg) * d.Wg);
          const float* gp = d.g + img * d.gs_n + (long long)gy * d.gs_h + (long long)gx * d.gs_w;
          if (d.g_vec) {
            v = *(const floatx4v*)(gp + col);
          } else {
            float e4[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) e4[e] = (col + e < d.Cg) ? gp[(long long)(col + e) * d.gs_c] : 0.f;
            v = floatx4v{e4[0], e4[1], e4[2], e4[3]};
          }
        }
      }
      rg[q] = v;
    }
#pragma unroll
    for (int q = 0; q < XPASS; ++q) {
      const int f = tid + 256 * q;
      floatx4v v = {0.f, 0.f, 0.f, 0.f};
      if (f < BK * X4) {
        const int row = f / X4, c4 = f - (f / X4) * X4;
        const long long p = p0 + row;
        if (p < pe) {
          const long long img = p / HW;
          const long long rr = p - img * HW;
          const int gy = (int)(rr / d.Wg), gx = (int)(rr - (long long)(rr / d.Wg) * d.Wg);
          if constexpr (!GEN) {
            const int col = c0 + c4 * 4;
            const int iy = gy * d.stride + dyt, ix = gx * d.stride + dxt;
            if (col < d.Cx && (unsigned)iy < (unsigned)d.Hx && (unsigned)ix < (unsigned)d.Wx) {
              v = *(const floatx4v*)(d.x + img * d.xs_n + (long long)iy * d.xs_h + (long long)ix * d.xs_w + col);
              if (d.x_op == AOP_SQUARE) v = v * v;
            }
          } else {
            float e4[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int j = c0 + c4 * 4 + e;
              const int tt = j / d.Cx, cx = j - (j / d.Cx) * d.Cx;
              float val = 0.f;
              if (tt < d.T) {
                const int iy = gy * d.stride + d.dy[tt], ix = gx * d.stride + d.dx[tt];
                if ((unsigned)iy < (unsigned)d.Hx && (unsigned)ix < (unsigned)d.Wx) {
                  val = d.x[img * d.xs_n + (long long)iy * d.xs_h + (long long)ix * d.xs_w + (long long)cx * d.xs_c];
                  if (d.x_op == AOP_SQUARE) val *= val;
                }
              }
              e4[e] = val;
            }
            v = floatx4v{e4[0], e4[1], e4[2], e4[3]};
          }
        }
      }
      rx[q] = v;
    }
  };
  auto sstore = [&]() {
#pragma unroll
    for (int q = 0; q < GPASS; ++q) {
      const int f = tid + 256 * q;
      if (f < BK * G4) *(floatx4v*)&Gs[f * 4] = rg[q];
    }
#pragma unroll
    for (int q = 0; q < XPASS; ++q) {
      const int f = tid + 256 * q;
      if (f < BK * X4) *(floatx4v*)&Xs[f * 4] = rx[q];
    }
  };

  const int lane = tid & 63, w = tid >> 6;
  const int wm = w / WAVES_N, wn = w - (w / WAVES_N) * WAVES_N;
  const int r = lane & 31, h = lane >> 5;
  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  if (pb < pe) {
    gload(pb);
    sstore();
  }
  __syncthreads();
  for (long long p0 = pb; p0 < pe; p0 += BK) {
    if (p0 + BK < pe) gload(p0 + BK);
#pragma unroll
    for (int s = 0; s < BK / 2; ++s) {
      const int k = 2 * s + h;
      float a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = Gs[k * BM + wm * WM + i * 32 + r];
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = Xs[k * BN + wn * WN + j * 32 + r];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
    if (p0 + BK < pe) sstore();
    __syncthreads();
  }

  const int Tp = GEN ? 1 : d.T;
  float* slab = d.partial + ((long long)split * Tp + t) * (long long)d.Cg * d.ncols;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int gr = g0 + wm * WM + i * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
      if (gr >= d.Cg) continue;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = c0 + wn * WN + j * 32 + r;
        if (col < d.ncols) slab[(long long)gr * d.ncols + col] = acc[i][j][reg];
      }
    }
}

struct WgRed {
  const float* partial;
  float* out;
  int nsplit, Tp, T, Cg, Cx, ncols, kk, generic;
  int kk_of_t[IC_MAXT];
};

__global__ void wg_reduce_kernel(const WgRed r) {
  const long long total = (long long)r.Cg * r.Cx * r.T;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    // i enumerates (g, t, c) with c fastest: coalesced slab reads
    const int c = (int)(i % r.Cx);
    const long long gt = i / r.Cx;
    const int t = (int)(gt % r.T);
    const int g = (int)(gt / r.T);
    const int tp = r.generic ? 0 : t;
    const int col = r.generic ? t * r.Cx + c : c;
    const long long stride = (long long)r.Tp * r.Cg * r.ncols;
    const float* src = r.partial + ((long long)tp * r.Cg + g) * r.ncols + col;
    float v = 0.f;
    for (int s = 0; s < r.nsplit; ++s) v += src[s * stride];
    r.out[((long long)g * r.Cx + c) * r.kk + r.kk_of_t[t]] = v;
  }
}

template <int BM, int BN, int WM, int WN, bool GEN>
int wg_launch_t(const WgDesc& d, hipStream_t s) {
  const int Tp = GEN ? 1 : d.T;
  dim3 grid(d.mtiles * d.ntiles * Tp, d.nsplit);
  hipLaunchKernelGGL((wg_kernel<BM, BN, WM, WN, GEN>), grid, dim3(256), 0, s, d);
  IC_CHECK_LAUNCH();
  return IC_OK;
}

// ---------------------------------------------------------------- colsum
__global__ void colsum_partial_kernel(const float* t, long long s_n, long long s_c, long long s_h,
                                      long long s_w, int N, int C, int H, int W, long long rows,
                                      long long rpb, float* part) {
  const long long r0 = (long long)blockIdx.x * rpb;
  long long r1 = r0 + rpb;
  if (r1 > rows) r1 = rows;
  const long long HW = (long long)H * W;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float acc = 0.f;
    for (long long rr = r0; rr < r1; ++rr) {
      const long long img = rr / HW, q = rr - img * HW;
      const long long y = q / W, x = q - (q / W) * W;
      acc += t[img * s_n + y * s_h + x * s_w + (long long)c * s_c];
    }
    part[(long long)blockIdx.x * C + c] = acc;
  }
}

__global__ void colsum_final_kernel(const float* part, int nb, int C, float scale, float* out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float acc = 0.f;
  for (int b = 0; b < nb; ++b) acc += part[(long long)b * C + c];
  out[c] = acc * scale;
}

int colsum_blocks(long long rows) {
  long long nb = (rows + 127) / 128;
  if (nb > 1024) nb = 1024;
  if (nb < 1) nb = 1;
  return (int)nb;
}

}  // namespace

size_t wg_plan(WgDesc& d) {
  if (d.generic) { d.bm = 192; d.bn = 64; d.ncols = d.T * d.Cx; }
  else { d.bm = 192; d.bn = (d.Cx >= 128) ? 192 : 64; d.ncols = d.Cx; }
  d.mtiles = ic_cdiv(d.Cg, d.bm);
  d.ntiles = ic_cdiv(d.ncols, d.bn);
  d.P = (long long)d.N * d.Hg * d.Wg;
  const long long tiles = (long long)d.mtiles * d.ntiles * (d.generic ? 1 : d.T);
  long long ns = (1024 + tiles - 1) / tiles;
  long long maxs = (d.P + 63) / 64;  // at least 64 pixels per split
  if (ns > maxs) ns = maxs;
  if (ns < 1) ns = 1;
  long long pps = (d.P + ns - 1) / ns;
  pps = (pps + 15) / 16 * 16;
  d.pps = (int)pps;
  d.nsplit = (int)((d.P + pps - 1) / pps);
  if (d.nsplit < 1) d.nsplit = 1;
  const int Tp = d.generic ? 1 : d.T;
  return (size_t)d.nsplit * Tp * (size_t)d.Cg * d.ncols * sizeof(float);
}

int wg_run(WgDesc& d, hipStream_t s) {
  if (d.P == 0) return IC_OK;
  d.g_vec = (d.gs_c == 1 && d.Cg % 4 == 0);
  if (!d.generic && (d.xs_c != 1 || d.Cx % 4 != 0)) return IC_ERR_ARG;
  if (d.generic) return wg_launch_t<192, 64, 96, 32, true>(d, s);
  if (d.bn == 192) return wg_launch_t<192, 192, 96, 96, false>(d, s);
  return wg_launch_t<192, 64, 96, 32, false>(d, s);
}

int wg_reduce(const WgDesc& d, float* out, const int* kk_of_t, int kk, hipStream_t s) {
  WgRed r;
  r.partial = d.partial; r.out = out; r.nsplit = d.nsplit; r.Tp = d.generic ? 1 : d.T; r.T = d.T;
  r.Cg = d.Cg; r.Cx = d.Cx; r.ncols = d.ncols; r.kk = kk; r.generic = d.generic;
  for (int t = 0; t < d.T; ++t) r.kk_of_t[t] = kk_of_t[t];
  const long long total = (long long)d.Cg * d.Cx * d.T;
  long long blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) return IC_OK;
  hipLaunchKernelGGL(wg_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, s, r);
  IC_CHECK_LAUNCH();
  return IC_OK;
}

size_t colsum_ws(long long rows, int C) {
  return (size_t)colsum_blocks(rows) * C * sizeof(float);
}

int colsum(const float* t, long long s_n, long long s_c, long long s_h, long long s_w, int N, int C,
           int H, int W, float* out, float scale, void* ws, hipStream_t s) {
  const long long rows = (long long)N * H * W;
  const int nb = colsum_blocks(rows);
  const long long rpb = (rows + nb - 1) / nb;
  float* part = (float*)ws;
  hipLaunchKernelGGL(colsum_partial_kernel, dim3(nb), dim3(256), 0, s, t, s_n, s_c, s_h, s_w, N, C, H,
                     W, rows, rpb, part);
  IC_CHECK_LAUNCH();
  hipLaunchKernelGGL(colsum_final_kernel, dim3((C + 255) / 256), dim3(256), 0, s, part, nb, C, scale, out);
  IC_CHECK_LAUNCH();
  return IC_OK;
}
