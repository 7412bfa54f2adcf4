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
#include <type_traits>

#include "gemm.h"
#include <algorithm>

#ifndef WG_X3_TWO
#define WG_X3_TWO 0  // split wgrad: 1 = two blocks per CU (swizzled unpadded rows), 0 = one (padded rows)
#endif

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

  // XCD-aware work order: hardware places block b on XCD b % 8; consecutive
  // work items (the taps / tiles of one pixel split, which share G and X rows)
  // are given to blocks of the same XCD so those rows are reused in its L2.
  const int Tp = GEN ? 1 : d.T;
  const int tiles = d.mtiles * d.ntiles;
  const int nblk = tiles * Tp * d.nsplit;
  const int b = blockIdx.x;
  const int wid = (b & 7) * (int)(gridDim.x >> 3) + (b >> 3);  // gridDim.x % 8 == 0
  if (wid >= nblk) return;
  const int per_split = tiles * Tp;
  const int split = wid / per_split;
  const int bx = wid - split * per_split;
  const int t = GEN ? 0 : bx / tiles;
  const int rem = bx - t * tiles;
  const int mt = rem / d.ntiles, nt = rem - (rem / d.ntiles) * d.ntiles;
  const int g0 = mt * BM, c0 = nt * BN;
  const uint32_t pb = (uint32_t)split * (uint32_t)d.pps;
  uint32_t pe = pb + (uint32_t)d.pps;
  if (pe > (uint32_t)d.P) pe = (uint32_t)d.P;
  const int tid = threadIdx.x;
  const int dyt = GEN ? 0 : d.dy[t], dxt = GEN ? 0 : d.dx[t];

  floatx4v rg[GPASS], rx[XPASS];

  // pixel p -> (img, gy, gx) with 32-bit magic division (P < 2^31)
  auto pix = [&](uint32_t p, uint32_t& img, int& gy, int& gx) {
    img = fdiv(p, d.fd_hw);
    const uint32_t rr = p - img * d.fd_hw.d;
    const uint32_t y = fdiv(rr, d.fd_w);
    gy = (int)y;
    gx = (int)(rr - y * d.fd_w.d);
  };

  auto gload = [&](uint32_t p0) {
#pragma unroll
    for (int q = 0; q < GPASS; ++q) {
      const int f = tid + 256 * q;
      floatx4v v = {0.f, 0.f, 0.f, 0.f};
      if (f < BK * G4) {
        const int row = f / G4, c4 = f - (f / G4) * G4;
        const uint32_t p = p0 + row;
        const int col = g0 + c4 * 4;
        if (p < pe && col < d.Cg) {
          uint32_t img; int gy, gx;
          pix(p, img, gy, gx);
          const float* gp = d.g + (long long)img * d.gs_n + (long long)gy * d.gs_h + (long long)gx * d.gs_w;
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
        const uint32_t p = p0 + row;
        if (p < pe) {
          uint32_t img; int gy, gx;
          pix(p, img, gy, gx);
          if constexpr (!GEN) {
            const int col = c0 + c4 * 4;
            const int iy = gy * d.stride + dyt, ix = gx * d.stride + dxt;
            if (col < d.Cx && (unsigned)iy < (unsigned)d.Hx && (unsigned)ix < (unsigned)d.Wx) {
              v = *(const floatx4v*)(d.x + (long long)img * d.xs_n + (long long)iy * d.xs_h +
                                     (long long)ix * d.xs_w + col);
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
                  val = d.x[(long long)img * d.xs_n + (long long)iy * d.xs_h + (long long)ix * d.xs_w +
                            (long long)cx * d.xs_c];
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
  for (uint32_t p0 = pb; p0 < pe; p0 += BK) {
    const bool more = p0 + BK < pe;
    if (more) gload(p0 + BK);
#pragma unroll
    for (int s = 0; s < BK / 2; ++s) {
      const int k = 2 * s + h;
      float a[TM], bb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = Gs[k * BM + wm * WM + i * 32 + r];
#pragma unroll
      for (int j = 0; j < TN; ++j) bb[j] = Xs[k * BN + wn * WN + j * 32 + r];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], bb[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
    if (more) sstore();
    __syncthreads();
  }

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

// Fast path (G and X channel-contiguous, 4-channel aligned): both operand
// tiles are staged global -> LDS by LDS-DMA (global_load_lds_dwordx4, no VGPR
// round trip) into two LDS buffers, so tile i+1 streams in while the MFMAs
// consume tile i; one barrier per 16-pixel K-step.  The LDS image is exactly
// lane-linear ([k][m] rows, no padding) as LDS-DMA requires; out-of-range rows
// (past the split, outside the image = zero padding) read a zero page.
__device__ __attribute__((aligned(16))) float wg_zero_page[4];

// LDS image rows are k (pixel) major; odd rows have their 16-B chunks XOR 8
// (a 32-float shift), so the two lane halves of a fragment read (rows k, k+1
// at the same columns) hit different banks.  Applied on the DMA source.
__device__ __forceinline__ int wg_swz(int k, int col) { return ((((col >> 2) ^ ((k & 1) << 3))) << 2) | (col & 3); }

template <int BM, int BN, int WM, int WN, bool XSQ>
__global__ void __launch_bounds__(256, 2) wg_glds_kernel(const WgDesc d) {
  constexpr int BK = 16;
  constexpr int WAVES_N = BN / WN;
  constexpr int TM = WM / 32, TN = WN / 32;
  constexpr int G4 = BM / 4, X4 = BN / 4;
  constexpr int GPASS = BK * G4 / 256, XPASS = BK * X4 / 256;
  static_assert(BK * G4 % 256 == 0 && BK * X4 % 256 == 0, "whole LDS-DMA passes");
  static_assert((BM / WM) * (BN / WN) == 4, "4 waves per block");
  constexpr int STAGE = BK * (BM + BN);
  __shared__ __attribute__((aligned(16))) float lds[2 * STAGE];

  const int tiles = d.mtiles * d.ntiles;
  const int nblk = tiles * d.T * d.nsplit;
  const int b = blockIdx.x;
  const int wid = (b & 7) * (int)(gridDim.x >> 3) + (b >> 3);  // XCD-grouped; gridDim.x % 8 == 0
  if (wid >= nblk) return;
  const int per_split = tiles * d.T;
  const int split = wid / per_split;
  const int bx = wid - split * per_split;
  const int t = bx / tiles;
  const int rem = bx - t * tiles;
  const int mt = rem / d.ntiles, nt = rem - (rem / d.ntiles) * d.ntiles;
  const int g0 = mt * BM, c0 = nt * BN;
  const uint32_t pb = (uint32_t)split * (uint32_t)d.pps;
  uint32_t pe = pb + (uint32_t)d.pps;
  if (pe > (uint32_t)d.P) pe = (uint32_t)d.P;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int dyt = d.dy[t], dxt = d.dx[t];

  // Row-fast staging (d.rowfast): a 16-pixel K step never crosses an output
  // row, so image / output row / first column are uniform per step (scalar
  // unit) and each lane only adds its constant row and column offsets: a few
  // VALU per LDS-DMA instead of two divisions and three 64-bit products.
  int goff[GPASS], xoff[XPASS], xix[XPASS];
  bool gok[GPASS], xok[XPASS];
#pragma unroll
  for (int q = 0; q < GPASS; ++q) {
    const int f = tid + 256 * q;
    const int row = f / G4, c4 = (f - (f / G4) * G4) ^ ((row & 1) << 3);
    const int col = g0 + c4 * 4;
    gok[q] = col < d.Cg;
    goff[q] = row * (int)d.gs_w + col;
  }
#pragma unroll
  for (int q = 0; q < XPASS; ++q) {
    const int f = tid + 256 * q;
    const int row = f / X4, c4 = (f - (f / X4) * X4) ^ ((row & 1) << 3);
    const int col = c0 + c4 * 4;
    xok[q] = col < d.Cx;
    xix[q] = row * d.stride;
    xoff[q] = row * d.stride * (int)d.xs_w + col;
  }

  auto stage = [&](uint32_t p0, int buf) {
    float* Gs = lds + buf * STAGE;
    float* Xs = Gs + BK * BM;
    if (d.rowfast) {
      const uint32_t img = fdiv(p0, d.fd_hw);
      const uint32_t rr = p0 - img * d.fd_hw.d;
      const uint32_t gy = fdiv(rr, d.fd_w);
      const uint32_t gx0 = rr - gy * d.fd_w.d;
      const float* gb = d.g + (long long)img * d.gs_n + (long long)gy * d.gs_h + (long long)gx0 * d.gs_w;
      const int iy = (int)gy * d.stride + dyt, ix0 = (int)gx0 * d.stride + dxt;
      const bool rowok = (unsigned)iy < (unsigned)d.Hx;
      const float* xb = d.x + (long long)img * d.xs_n + (long long)iy * d.xs_h + (long long)ix0 * d.xs_w;
#pragma unroll
      for (int q = 0; q < GPASS; ++q) {
        const int f = tid + 256 * q;
        const float* src = gok[q] ? gb + goff[q] : wg_zero_page;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)(Gs + (f - lane) * 4), 16, 0, 0);
      }
#pragma unroll
      for (int q = 0; q < XPASS; ++q) {
        const int f = tid + 256 * q;
        const bool ok = rowok && xok[q] && (unsigned)(ix0 + xix[q]) < (unsigned)d.Wx;
        const float* src = ok ? xb + xoff[q] : wg_zero_page;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)(Xs + (f - lane) * 4), 16, 0, 0);
      }
      return;
    }
#pragma unroll
    for (int q = 0; q < GPASS; ++q) {
      const int f = tid + 256 * q;
      const int row = f / G4, c4 = (f - (f / G4) * G4) ^ ((row & 1) << 3);
      const uint32_t p = p0 + row;
      const int col = g0 + c4 * 4;
      const float* src = wg_zero_page;
      if (p < pe && col < d.Cg) {
        const uint32_t img = fdiv(p, d.fd_hw);
        const uint32_t rr = p - img * d.fd_hw.d;
        const uint32_t gy = fdiv(rr, d.fd_w);
        const uint32_t gx = rr - gy * d.fd_w.d;
        src = d.g + (long long)img * d.gs_n + (long long)gy * d.gs_h + (long long)gx * d.gs_w + col;
      }
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(Gs + (f - lane) * 4), 16, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < XPASS; ++q) {
      const int f = tid + 256 * q;
      const int row = f / X4, c4 = (f - (f / X4) * X4) ^ ((row & 1) << 3);
      const uint32_t p = p0 + row;
      const int col = c0 + c4 * 4;
      const float* src = wg_zero_page;
      if (p < pe && col < d.Cx) {
        const uint32_t img = fdiv(p, d.fd_hw);
        const uint32_t rr = p - img * d.fd_hw.d;
        const uint32_t gy = fdiv(rr, d.fd_w);
        const uint32_t gx = rr - gy * d.fd_w.d;
        const int iy = (int)gy * d.stride + dyt, ix = (int)gx * d.stride + dxt;
        if ((unsigned)iy < (unsigned)d.Hx && (unsigned)ix < (unsigned)d.Wx)
          src = d.x + (long long)img * d.xs_n + (long long)iy * d.xs_h + (long long)ix * d.xs_w + col;
      }
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(Xs + (f - lane) * 4), 16, 0, 0);
    }
  };

  const int wm = w / WAVES_N, wn = w - (w / WAVES_N) * WAVES_N;
  const int r = lane & 31, h = lane >> 5;
  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  if (pb < pe) stage(pb, 0);
  int buf = 0;
  for (uint32_t p0 = pb; p0 < pe; p0 += BK) {
    __syncthreads();  // tile `buf` landed (vmcnt(0) + barrier); everyone is done with buf^1
    if (p0 + BK < pe) stage(p0 + BK, buf ^ 1);
    const float* Gs = lds + buf * STAGE;
    const float* Xs = Gs + BK * BM;
#pragma unroll
    for (int s = 0; s < BK / 2; ++s) {
      const int k = 2 * s + h;
      float a[TM], bb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = Gs[k * BM + wg_swz(k, wm * WM + i * 32 + r)];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const float v = Xs[k * BN + wg_swz(k, wn * WN + j * 32 + r)];
        bb[j] = XSQ ? v * v : v;
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], bb[j], acc[i][j], 0, 0, 0);
    }
    buf ^= 1;
  }

  float* slab = d.partial + ((long long)split * d.T + t) * (long long)d.Cg * d.ncols;
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


// ------------------------------------------------------------------ fp32 by exact bf16 split
// Weight gradient with fp32 arithmetic on the bf16 MFMA (IC_MATH_SPLIT): both
// operands are split exactly into three bf16 terms (split3_bf16) and the six
// cross products are accumulated in fp32 on v_mfma_f32_32x32x16_bf16.  The
// reduction axis (pixels) is the MFMA K axis, but G and X are channel-
// contiguous (NHWC), so the 16-pixel K step is staged as [pixel][channel] bf16
// images and the fragments (8 consecutive pixels of one channel per lane) are
// read transposed with ds_read_b64_tr_b16.  Image rows are 224 bf16 (448 B):
// the four rows of one transposed read start 48 dwords apart mod 64, so a
// 32-lane half covers all 64 banks once.
//
// One block per CU (4 waves, 96x96 wave tiles, 144 accumulators each, 512
// registers per lane available): two LDS buffers, one barrier per K step;
// each step's global loads are issued a full step ahead (register staging,
// split + store after the step's MFMAs).
typedef __bf16 wg_bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 wg_bf16x8 __attribute__((ext_vector_type(8)));

// TWO: two blocks per CU — unpadded 192-bf16 rows whose 16-B chunks are
// XOR-swizzled by 4 on rows with bit 1 set (the four rows of a transposed read
// then start 0 / 32 / 16 / 48 dwords apart mod 64), 74 KB of LDS per block.
#ifndef WG_X3_SPREAD
#define WG_X3_SPREAD 1  // row-fast refill loads issued per slot right after its store, spread among the MFMAs (4.40 -> 4.33 ms over all wgrad ops)
#endif
#ifndef WG_X3_DEPTH
#define WG_X3_DEPTH 2  // steps of global loads in flight ahead of their split + store (2 or 3)
#endif
template <bool ROWFAST, bool XSQ, bool TWO>
__global__ void __launch_bounds__(256, TWO ? 2 : 1) wg_x3_kernel(const WgDesc d) {
  constexpr int BM = 192, BN = 192, WM = 96, WN = 96, BK = 16;
  constexpr int TM = WM / 32, TN = WN / 32;
  constexpr int PITCH = TWO ? 192 : 224;    // bf16 per image row
  constexpr int DEPTH = TWO ? 1 : WG_X3_DEPTH;  // register sets of staged loads in flight
  constexpr int PLANE = BK * PITCH;         // one part of one operand
  constexpr int OPER = 3 * PLANE;           // three parts
  constexpr int STAGE = 2 * OPER;           // G and X
  constexpr int C4 = BM / 4;                // float4 per staged row (BM == BN)
  constexpr int QP = BK * C4 / 256;         // float4 per thread per operand
  static_assert(BM == BN && BK * C4 % 256 == 0, "staging map");
  __shared__ __attribute__((aligned(16))) __bf16 lds[2 * STAGE];

  const int tiles = d.mtiles * d.ntiles;
  const int nblk = tiles * d.T * d.nsplit;
  const int b = blockIdx.x;
  const int wid = (b & 7) * (int)(gridDim.x >> 3) + (b >> 3);  // XCD-grouped; gridDim.x % 8 == 0
  if (wid >= nblk) return;
  const int per_split = tiles * d.T;
  const int split = wid / per_split;
  const int bx = wid - split * per_split;
  const int t = bx / tiles;
  const int rem = bx - t * tiles;
  const int mt = rem / d.ntiles, nt = rem - (rem / d.ntiles) * d.ntiles;
  const int g0 = mt * BM, c0 = nt * BN;
  const uint32_t pb = (uint32_t)split * (uint32_t)d.pps;
  uint32_t pe = pb + (uint32_t)d.pps;
  if (pe > (uint32_t)d.P) pe = (uint32_t)d.P;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int dyt = d.dy[t], dxt = d.dx[t];

  int srow[QP], scol[QP];
#pragma unroll
  for (int q = 0; q < QP; ++q) {
    const int f = tid + 256 * q;
    srow[q] = f / C4;
    scol[q] = (f - (f / C4) * C4) * 4;
  }

  // two register sets: a step's global loads are issued two steps before its split + store
  floatx4v g0r[QP], x0r[QP], g1r[QP], x1r[QP], g2r[QP], x2r[QP];  // g2r/x2r: DEPTH 3 only
  // live == false (a refill past the split) still issues every load, from the
  // zero page: with the loads unconditional the compiler's vmcnt bookkeeping
  // keeps both register sets in flight (a branch around them made it drain all
  // loads, vmcnt(0), one step after they were issued)
  // row-fast refill split per staged slot (WG_X3_SPREAD): the step's uniform
  // bases once, then slot q's two loads right after slot q has been stored
  struct RowBase {
    const float* gb;
    const float* xb;
    int ix0;
    bool rowok, live;
  };
  auto row_base = [&](uint32_t p0, bool live) {
    const uint32_t img = fdiv(p0, d.fd_hw);
    const uint32_t rr = p0 - img * d.fd_hw.d;
    const uint32_t gy = fdiv(rr, d.fd_w);
    const uint32_t gx0 = rr - gy * d.fd_w.d;
    const int iy = (int)gy * d.stride + dyt;
    return RowBase{d.g + (long long)img * d.gs_n + (long long)gy * d.gs_h + (long long)gx0 * d.gs_w,
                   d.x + (long long)img * d.xs_n + (long long)iy * d.xs_h, (int)gx0 * d.stride + dxt,
                   live && (unsigned)iy < (unsigned)d.Hx, live};
  };
  auto gload_q = [&](const RowBase& rb, int q, floatx4v (&rg)[QP], floatx4v (&rx)[QP]) {
    const int gcol = g0 + scol[q], xcol = c0 + scol[q];
    const int ix = rb.ix0 + srow[q] * d.stride;
    const float* gs = (rb.live && gcol < d.Cg) ? rb.gb + (long long)srow[q] * d.gs_w + gcol : wg_zero_page;
    const float* xs = (rb.rowok && xcol < d.Cx && (unsigned)ix < (unsigned)d.Wx)
                          ? rb.xb + (long long)ix * d.xs_w + xcol : wg_zero_page;
    rg[q] = *(const floatx4v*)gs;
    floatx4v vx = *(const floatx4v*)xs;
    if (XSQ) vx = vx * vx;
    rx[q] = vx;
  };
  auto gload = [&](uint32_t p0, floatx4v (&rg)[QP], floatx4v (&rx)[QP], bool live = true) {
    if (ROWFAST) {
      // a 16-pixel step never crosses an output row: image / row / first column are uniform
      const uint32_t img = fdiv(p0, d.fd_hw);
      const uint32_t rr = p0 - img * d.fd_hw.d;
      const uint32_t gy = fdiv(rr, d.fd_w);
      const uint32_t gx0 = rr - gy * d.fd_w.d;
      const float* gb = d.g + (long long)img * d.gs_n + (long long)gy * d.gs_h + (long long)gx0 * d.gs_w;
      const int iy = (int)gy * d.stride + dyt, ix0 = (int)gx0 * d.stride + dxt;
      const bool rowok = live && (unsigned)iy < (unsigned)d.Hx;
      const float* xb = d.x + (long long)img * d.xs_n + (long long)iy * d.xs_h;
#pragma unroll
      for (int q = 0; q < QP; ++q) {
        // branch-free: padding and out-of-range columns read a zero page
        const int gcol = g0 + scol[q], xcol = c0 + scol[q];
        const int ix = ix0 + srow[q] * d.stride;
        const float* gs = (live && gcol < d.Cg) ? gb + (long long)srow[q] * d.gs_w + gcol : wg_zero_page;
        const float* xs = (rowok && xcol < d.Cx && (unsigned)ix < (unsigned)d.Wx)
                              ? xb + (long long)ix * d.xs_w + xcol : wg_zero_page;
        rg[q] = *(const floatx4v*)gs;
        floatx4v vx = *(const floatx4v*)xs;
        if (XSQ) vx = vx * vx;
        rx[q] = vx;
      }
      return;
    }
#pragma unroll
    for (int q = 0; q < QP; ++q) {
      const uint32_t p = p0 + srow[q];
      floatx4v vg = {0.f, 0.f, 0.f, 0.f}, vx = {0.f, 0.f, 0.f, 0.f};
      if (live && p < pe) {
        const uint32_t img = fdiv(p, d.fd_hw);
        const uint32_t rr = p - img * d.fd_hw.d;
        const uint32_t gy = fdiv(rr, d.fd_w);
        const uint32_t gx = rr - gy * d.fd_w.d;
        const int gcol = g0 + scol[q], xcol = c0 + scol[q];
        if (gcol < d.Cg)
          vg = *(const floatx4v*)(d.g + (long long)img * d.gs_n + (long long)gy * d.gs_h + (long long)gx * d.gs_w +
                                  gcol);
        const int iy = (int)gy * d.stride + dyt, ix = (int)gx * d.stride + dxt;
        if (xcol < d.Cx && (unsigned)iy < (unsigned)d.Hx && (unsigned)ix < (unsigned)d.Wx) {
          vx = *(const floatx4v*)(d.x + (long long)img * d.xs_n + (long long)iy * d.xs_h + (long long)ix * d.xs_w +
                                  xcol);
          if (XSQ) vx = vx * vx;
        }
      }
      rg[q] = vg;
      rx[q] = vx;
    }
  };
  // split + store one staged float4 of each operand (q), so the store pass can
  // be spread between the MFMA groups of the previous step
  auto sstore_q = [&](int buf, int q, const floatx4v (&rg)[QP], const floatx4v (&rx)[QP]) {
    __bf16* base = lds + buf * STAGE;
#pragma unroll
    for (int op = 0; op < 2; ++op) {
      const floatx4v v = op == 0 ? rg[q] : rx[q];
      wg_bf16x4 vh, vm, vl;
      if (WG_SPLIT_PK) {
        split3_bf16x4(v, vh, vm, vl);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          __bf16 hh, mm, ll;
          split3_bf16(v[e], hh, mm, ll);
          vh[e] = hh; vm[e] = mm; vl[e] = ll;
        }
      }
      __bf16* dst = base + op * OPER + srow[q] * PITCH + (scol[q] ^ (TWO ? ((srow[q] >> 1) & 1) << 5 : 0));
      *(wg_bf16x4*)dst = vh;
      *(wg_bf16x4*)(dst + PLANE) = vm;
      *(wg_bf16x4*)(dst + 2 * PLANE) = vl;
    }
  };
  auto sstore = [&](int buf, const floatx4v (&rg)[QP], const floatx4v (&rx)[QP]) {
#pragma unroll
    for (int q = 0; q < QP; ++q) sstore_q(buf, q, rg, rx);
  };

  const int wm = w >> 1, wn = w & 1;
  const int r = lane & 31, h = lane >> 5;
  // transposed-read address of this lane inside one plane: row 8h + q, column 16*(r>=16) + 4p
  const int li = lane & 15;
  const int tr_row = (8 * h + (li >> 2)) * PITCH;
  const int tr_col = 16 * ((lane >> 4) & 1) + 4 * (li & 3);
  const int tr_sw = TWO ? ((li >> 3) & 1) << 5 : 0;  // rows 8h + (li >> 2) (+4): bit 1 = bit 3 of li
  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  // step p0 computes LDS buffer `buf`, stores the set holding step p0 + BK into
  // buf ^ 1 (interleaved with the MFMAs), then reloads that set with step p0 + 3 BK
  auto step = [&](int p0, int buf, floatx4v (&rg)[QP], floatx4v (&rx)[QP]) {
    const __bf16* sb = lds + buf * STAGE;
    auto tr8 = [&](const __bf16* src) {
      const wg_bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) wg_bf16x4*)src);
      const wg_bf16x4 hi =
          __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) wg_bf16x4*)(src + 4 * PITCH));
      return (wg_bf16x8)__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    };
    // B fragments: all three column groups held across the row groups (one
    // block per CU), or re-read per (row, column) group (TWO: register budget)
    wg_bf16x8 bb[3][TWO ? 1 : TN];
    if constexpr (!TWO) {
#pragma unroll
      for (int q = 0; q < 3; ++q)
#pragma unroll
        for (int j = 0; j < TN; ++j) bb[q][j] = tr8(sb + OPER + q * PLANE + tr_row + ((wn * WN + j * 32 + tr_col) ^ tr_sw));
    }
    static_assert(QP == TM, "one staged float4 per MFMA row group");
    constexpr bool SPREAD = ROWFAST && !TWO && WG_X3_SPREAD;
    const uint32_t pn = (uint32_t)(p0 + (DEPTH + 1) * BK);
    RowBase nb{};
    if constexpr (SPREAD) nb = row_base(pn, (int)pn < (int)pe);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      wg_bf16x8 a[3];  // one row group's A fragments at a time (register pressure)
#pragma unroll
      for (int q = 0; q < 3; ++q) a[q] = tr8(sb + q * PLANE + tr_row + ((wm * WM + i * 32 + tr_col) ^ tr_sw));
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int jb = TWO ? 0 : j;
        if constexpr (TWO) {
#pragma unroll
          for (int q = 0; q < 3; ++q) bb[q][0] = tr8(sb + OPER + q * PLANE + tr_row + ((wn * WN + j * 32 + tr_col) ^ tr_sw));
        }
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], bb[0][jb], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], bb[1][jb], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], bb[2][jb], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], bb[0][jb], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], bb[1][jb], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], bb[0][jb], acc[i][j], 0, 0, 0);
      }
      // the next step's split + store, one slice per MFMA row group, interleaved
      // with its MFMAs (unconditional: near the end it fills an unread buffer)
      sstore_q(buf ^ 1, i, rg, rx);
      if constexpr (SPREAD) gload_q(nb, i, rg, rx);  // slot i refilled as soon as it is stored
      if constexpr (!TWO) {
#pragma unroll
        for (int k = 0; k < 6; ++k) {
          __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);   // MFMA
          __builtin_amdgcn_sched_group_barrier(0x002, 10, 0);  // VALU
          __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);   // DS write
          if (SPREAD && (k == 2 || k == 5)) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM read
        }
      }
    }
    // refill the set just stored: DEPTH steps ahead (never past the split: row-fast loads are unmasked)
    if (!SPREAD && (ROWFAST || p0 + (DEPTH + 1) * BK < (int)pe))
      gload((uint32_t)(p0 + (DEPTH + 1) * BK), rg, rx, p0 + (DEPTH + 1) * BK < (int)pe);
    __syncthreads();
  };

  // steps run in pairs (with DEPTH 2 the two register sets alternate
  // statically); an odd count is padded with one all-zero step in front
  const int nsteps = pe > pb ? (int)((pe - pb + BK - 1) / BK) : 0;
  if constexpr (DEPTH == 3) {
    // three register sets rotate over steps in threes (LDS buffers alternate, so
    // the group's first buffer flips each group); the count is padded to a
    // multiple of three with all-zero steps in front (zero-page loads)
    const int q3 = (int)pb - ((3 - nsteps % 3) % 3) * BK;
    auto live = [&](int p) { return p >= (int)pb && p < (int)pe; };
    if (nsteps > 0) {
      gload((uint32_t)q3, g0r, x0r, live(q3));
      sstore(0, g0r, x0r);
      gload((uint32_t)(q3 + BK), g1r, x1r, live(q3 + BK));
      gload((uint32_t)(q3 + 2 * BK), g2r, x2r, live(q3 + 2 * BK));
      gload((uint32_t)(q3 + 3 * BK), g0r, x0r, live(q3 + 3 * BK));
    }
    __syncthreads();
    int b = 0;
    for (int p0 = q3; p0 < (int)pe; p0 += 3 * BK) {
      step(p0, b, g1r, x1r);
      step(p0 + BK, b ^ 1, g2r, x2r);
      step(p0 + 2 * BK, b, g0r, x0r);
      b ^= 1;
    }
  } else {
  auto& g1s = DEPTH == 2 ? g1r : g0r;
  auto& x1s = DEPTH == 2 ? x1r : x0r;
  const int q0 = (int)pb - ((nsteps & 1) ? BK : 0);
  if (nsteps > 0) {
    if (nsteps & 1) {
#pragma unroll
      for (int q = 0; q < QP; ++q) {
        g0r[q] = floatx4v{0.f, 0.f, 0.f, 0.f};
        x0r[q] = floatx4v{0.f, 0.f, 0.f, 0.f};
      }
    } else {
      gload((uint32_t)q0, g0r, x0r);
    }
    sstore(0, g0r, x0r);
    // unconditional (ROWFAST): every path into the loop then has the same loads in flight
    if (ROWFAST || q0 + BK < (int)pe) gload((uint32_t)(q0 + BK), g1s, x1s, q0 + BK < (int)pe);
    if (DEPTH == 2 && (ROWFAST || q0 + 2 * BK < (int)pe))
      gload((uint32_t)(q0 + 2 * BK), g0r, x0r, q0 + 2 * BK < (int)pe);
  }
  __syncthreads();
  for (int p0 = q0; p0 < (int)pe; p0 += 2 * BK) {
    step(p0, 0, g1s, x1s);
    step(p0 + BK, 1, g0r, x0r);
  }
  }

  float* slab = d.partial + ((long long)split * d.T + t) * (long long)d.Cg * d.ncols;
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



// Two waves per SIMD (WG_X3_DUAL): the split weight gradient with eight
// waves of 96 x 48 (g x c) tiles on v_mfma_f32_16x16x32_bf16 — 72 accumulator
// registers per wave instead of 144, so two waves share each SIMD and one
// hides the other's fragment reads, staging and barrier waits.  32-pixel K
// steps (one MFMA K), unpadded 192-bf16 rows whose 16-B chunks are XOR-
// swizzled by 4 on rows with bit 1 set and by 2 on rows with bit 3 set, so
// the four 4-row groups of a 16-column transposed read (rows 8lq + q) land on
// distinct banks; 144 KB of LDS for two stages, one block per CU.  Row-fast
// only (a step stays inside one output row: Wg % 32 == 0).
#ifndef WG_X3_DUAL
#define WG_X3_DUAL 1
#endif
#ifndef WG_X3G
#define WG_X3G 1  // 5x5 stride-2 192x192 weight gradients on the tap-group kernel (wg_x3p_kernel); 0: wg_x3d_kernel
#endif
#ifndef WG_X3P_DEEP  // bf16-copy producers keep three steps of loads in flight instead of two
#define WG_X3P_DEEP 1
#endif
#ifndef WG_X3P_B16
#define WG_X3P_B16 1  // bf16 weight gradients read the operands' bf16 copies when the caller passes them (C3)
#endif
#ifndef WG_X3P_PRIO
#define WG_X3P_PRIO 1  // s_setprio of the producer waves (0: hardware default; 1: g_a.2 wgrad 1.163 -> 1.107 ms, r07l)
#endif
#ifndef WG_X3P_ABL
#define WG_X3P_ABL 0  // diagnostic ablations of wg_x3p_kernel (wrong results): 1 no global loads, 2 no LDS stores, 4 no MFMAs, 8 every step loads the split's first pixels (L2-hot), 16 no split (one
// conversion per value), 32 every step loads step 0 (loop-invariant addresses), 64 G stored unsplit (one
// conversion per G value, X split as usual: round 6, what G pre-split into three planes could save)
#endif
#ifndef WG_X3_DUAL16
#define WG_X3_DUAL16 1  // the two-wave kernel also on maps 16 wide (two row segments per step)
#endif
// SEG16: maps 16 wide — a 32-pixel step spans two output rows, each 16-pixel half
// with its own row base (either half stays inside one row when Wg % 16 == 0).
// NP = 1: bf16 operands (round to nearest even) with fp32 accumulation, one product per
// tile and step (IC_MATH_BF16, config C3); only plane 0 of each operand image is used.
template <bool XSQ, bool SEG16, int NP = 3>
__global__ void __launch_bounds__(512, 1) wg_x3d_kernel(const WgDesc d) {
  typedef __bf16 b4 __attribute__((ext_vector_type(4)));
  typedef __bf16 b8 __attribute__((ext_vector_type(8)));
  constexpr int BM = 192, WM = 96, WN = 48, BK = 32;
  constexpr int TM = WM / 16, TN = WN / 16;  // 6 x 3 tiles of 16 x 16
  constexpr int PITCH = 192;
  constexpr int PLANE = BK * PITCH;
  constexpr int OPER = 3 * PLANE;
  constexpr int STAGE = 2 * OPER;
  constexpr int C4 = BM / 4;
  constexpr int NT = 512;
  constexpr int QP = BK * C4 / NT;  // 3 float4 per thread per operand
  static_assert(QP * NT == BK * C4 && 2 * QP == TM, "one staged slot per two row tiles");
  __shared__ __attribute__((aligned(16))) __bf16 lds[2 * STAGE];

  const int tiles = d.mtiles * d.ntiles;
  const int nblk = tiles * d.T * d.nsplit;
  const int b = blockIdx.x;
  const int wid = (b & 7) * (int)(gridDim.x >> 3) + (b >> 3);  // XCD-grouped; gridDim.x % 8 == 0
  if (wid >= nblk) return;
  const int per_split = tiles * d.T;
  const int split = wid / per_split;
  const int bx = wid - split * per_split;
  const int t = bx / tiles;
  const int rem = bx - t * tiles;
  const int mt = rem / d.ntiles, nt = rem - (rem / d.ntiles) * d.ntiles;
  const int g0 = mt * BM, c0 = nt * BM;
  const int pb = split * d.pps;
  int pe = pb + d.pps;
  if (pe > (int)d.P) pe = (int)d.P;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int dyt = d.dy[t], dxt = d.dx[t];

  auto swz = [](int row) { return ((((row >> 1) & 1) << 5) | (((row >> 3) & 1) << 4)); };
  int srow[QP], scol[QP];
#pragma unroll
  for (int q = 0; q < QP; ++q) {
    const int f = tid + NT * q;
    srow[q] = f / C4;
    scol[q] = (f - (f / C4) * C4) * 4;
  }
  floatx4v g0r[QP], x0r[QP], g1r[QP], x1r[QP];
  struct RowBase {
    const float* gb;
    const float* xb;
    int ix0;
    bool rowok, live;
  };
  auto row_base = [&](int p0, bool live) {
    const uint32_t img = fdiv((uint32_t)p0, d.fd_hw);
    const uint32_t rr = (uint32_t)p0 - img * d.fd_hw.d;
    const uint32_t gy = fdiv(rr, d.fd_w);
    const uint32_t gx0 = rr - gy * d.fd_w.d;
    const int iy = (int)gy * d.stride + dyt;
    return RowBase{d.g + (long long)img * d.gs_n + (long long)gy * d.gs_h + (long long)gx0 * d.gs_w,
                   d.x + (long long)img * d.xs_n + (long long)iy * d.xs_h, (int)gx0 * d.stride + dxt,
                   live && (unsigned)iy < (unsigned)d.Hx, live};
  };
  struct StepBase {
    RowBase lo, hi;  // pixels 0..15 and 16..31 of the step (SEG16), else lo only
  };
  auto step_base = [&](int p0, bool live) {
    StepBase sbs;
    sbs.lo = row_base(p0, live);
    if constexpr (SEG16) sbs.hi = row_base(p0 + 16, live);
    return sbs;
  };
  // branch-free: padding and out-of-range columns read a zero page
  auto gload_q = [&](const StepBase& sbs, int q, floatx4v (&rg)[QP], floatx4v (&rx)[QP]) {
    const bool upper = SEG16 && srow[q] >= 16;
    const RowBase& rb = upper ? sbs.hi : sbs.lo;
    const int sr = upper ? srow[q] - 16 : srow[q];
    const int gcol = g0 + scol[q], xcol = c0 + scol[q];
    const int ix = rb.ix0 + sr * d.stride;
    const float* gs = (rb.live && gcol < d.Cg) ? rb.gb + (long long)sr * d.gs_w + gcol : wg_zero_page;
    const float* xs = (rb.rowok && xcol < d.Cx && (unsigned)ix < (unsigned)d.Wx)
                          ? rb.xb + (long long)ix * d.xs_w + xcol : wg_zero_page;
    rg[q] = *(const floatx4v*)gs;
    floatx4v vx = *(const floatx4v*)xs;
    if (XSQ) vx = vx * vx;
    rx[q] = vx;
  };
  auto gload = [&](int p0, floatx4v (&rg)[QP], floatx4v (&rx)[QP], bool live) {
    const StepBase sbs = step_base(p0, live);
#pragma unroll
    for (int q = 0; q < QP; ++q) gload_q(sbs, q, rg, rx);
  };
  auto sstore_q = [&](int buf, int q, const floatx4v (&rg)[QP], const floatx4v (&rx)[QP]) {
    __bf16* base = lds + buf * STAGE;
#pragma unroll
    for (int op = 0; op < 2; ++op) {
      __bf16* dst = base + op * OPER + srow[q] * PITCH + (scol[q] ^ swz(srow[q]));
      const floatx4v v = op == 0 ? rg[q] : rx[q];
      if constexpr (NP == 1) {
        typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
        *(b4*)dst = __builtin_bit_cast(b4, u32x2{ic_cvt_pk_bf16(v[0], v[1]), ic_cvt_pk_bf16(v[2], v[3])});
        continue;
      }
      b4 vh, vm, vl;
      split3_bf16x4(v, vh, vm, vl);
      *(b4*)dst = vh;
      *(b4*)(dst + PLANE) = vm;
      *(b4*)(dst + 2 * PLANE) = vl;
    }
  };
  auto sstore = [&](int buf, const floatx4v (&rg)[QP], const floatx4v (&rx)[QP]) {
#pragma unroll
    for (int q = 0; q < QP; ++q) sstore_q(buf, q, rg, rx);
  };

  const int wm = w >> 2, wn = w & 3;
  const int li = lane & 15, lq = lane >> 4;
  // 16x16x32 operands: lane (li, lq) holds pixels 8lq .. 8lq+7 of channel li of its
  // tile; a transposed read gives a 16-lane group rows 8lq + (li >> 2) (+4), columns 4 (li & 3)
  const int tr_r = 8 * lq + (li >> 2);
  const int tr_off = tr_r * PITCH;
  const int tr_c = 4 * (li & 3);
  const int tr_sw = swz(tr_r);  // rows tr_r and tr_r + 4 share bits 1 and 3
  floatx4v acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = floatx4v{0.f, 0.f, 0.f, 0.f};

  auto step = [&](int p0, int buf, floatx4v (&rg)[QP], floatx4v (&rx)[QP]) {
    const __bf16* sb = lds + buf * STAGE;
    auto tr8 = [&](const __bf16* plane, int col) {
      const __bf16* src = plane + tr_off + ((col + tr_c) ^ tr_sw);
      const b4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) b4*)src);
      const b4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) b4*)(src + 4 * PITCH));
      return (b8)__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    };
    b8 bb[NP][TN];
#pragma unroll
    for (int q = 0; q < NP; ++q)
#pragma unroll
      for (int j = 0; j < TN; ++j) bb[q][j] = tr8(sb + OPER + q * PLANE, wn * WN + 16 * j);
    const int pn = p0 + 3 * BK;
    const StepBase nb = step_base(pn, pn < pe);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      b8 a[NP];
#pragma unroll
      for (int q = 0; q < NP; ++q) a[q] = tr8(sb + q * PLANE, wm * WM + 16 * i);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        floatx4v& c = acc[i][j];
        if constexpr (NP == 1) {
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], bb[0][j], c, 0, 0, 0);
          continue;
        }
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], bb[0][j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], bb[1][j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], bb[2][j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], bb[0][j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], bb[1][j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], bb[0][j], c, 0, 0, 0);
      }
      if (i & 1) {
        // the next step's split + store of slot i / 2, then its refill three steps ahead
        sstore_q(buf ^ 1, i >> 1, rg, rx);
        gload_q(nb, i >> 1, rg, rx);
        if constexpr (NP == 3)
#pragma unroll
        for (int k = 0; k < 6; ++k) {
          __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);   // MFMA (this and the previous row tile)
          __builtin_amdgcn_sched_group_barrier(0x002, 7, 0);   // VALU
          __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);   // DS write
          if (k == 2 || k == 5) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM read
        }
      }
    }
    __syncthreads();
  };

  // steps run in pairs (two register sets alternate statically); an odd count
  // is padded with one all-zero step in front
  const int nsteps = pe > pb ? (pe - pb) / BK : 0;
  const int q0 = pb - ((nsteps & 1) ? BK : 0);
  if (nsteps > 0) {
    if (nsteps & 1) {
#pragma unroll
      for (int q = 0; q < QP; ++q) {
        g0r[q] = floatx4v{0.f, 0.f, 0.f, 0.f};
        x0r[q] = floatx4v{0.f, 0.f, 0.f, 0.f};
      }
    } else {
      gload(q0, g0r, x0r, true);
    }
    sstore(0, g0r, x0r);
    gload(q0 + BK, g1r, x1r, q0 + BK < pe);
    gload(q0 + 2 * BK, g0r, x0r, q0 + 2 * BK < pe);
  }
  __syncthreads();
  for (int p0 = q0; p0 < pe; p0 += 2 * BK) {
    step(p0, 0, g1r, x1r);
    step(p0 + BK, 1, g0r, x0r);
  }

  // C/D map of the 16x16 MFMA: row (g) = 4 lq + r, col (c) = li
  float* slab = d.partial + ((long long)split * d.T + t) * (long long)d.Cg * d.ncols;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int gr = g0 + wm * WM + 16 * i + 4 * lq + r;
      if (gr >= d.Cg) continue;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = c0 + wn * WN + 16 * j + li;
        if (col < d.ncols) slab[(long long)gr * d.ncols + col] = acc[i][j][r];
      }
    }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(acc[i][j]));  // stores straight from held registers
}

// Tap groups (WG_X3G): a stride-2 conv's tap (ky, kx) reads X at input column 2 gx + kx - pad, so
// tap kx0 + 2j is tap kx0 shifted by j output pixels.  A block owns one kernel row ky, one parity
// group -- kx 0, 2, 4 with 64-channel column tiles, or kx 1, 3 with 96-channel ones, 192 columns of
// (tap, channel) either way -- and one pixel split.  Per 32-pixel step it stages G once (all 192
// g) and X once (32 + NTAP - 1 pixels of its CW channels, starting at the group's first tap) and
// runs every tap of the group from them: the B fragment of tap j is X's image read j rows further
// down.  Against wg_x3d_kernel (one tap per block) the staged bytes, the split work and the LDS
// writes per step fall by a third; the MFMAs, their order and the accumulation order per output
// element are the same, so the result is bitwise that kernel's.  Two groups run in one launch
// (the body is instantiated for NTAP = 3 and 2); 25 blocks per split, as before.  Round 4 ran this
// tiling with the staging inside the MFMA waves (wg_x3g_kernel, removed in round 6: 1.165 ms against
// wg_x3p's 1.107 on g_a.2, DESIGN_HISTORY.md).
// Producer / consumer tap groups (round 5): the tap-group tiles, LDS images, MFMAs and their
// order (bitwise wg_x3d_kernel's result), with the staging moved off the MFMA waves.  Twelve waves, three per
// SIMD: the eight consumer waves only read fragments and run the MFMAs of step s from one LDS stage;
// the four producer waves (one per SIMD) meanwhile split and store step s + 1 into the other stage
// and load step s + 3 into the register set it frees (two sets, loads two steps ahead).  One barrier
// per step for all twelve.  In wg_x3g the split + store of the next step sat in each MFMA wave's
// instruction stream (0.36 ms of a 1.19 ms g_a.2 wgrad: the round-4 kernel's ablations, profiles/r06k_*); a producer wave
// issues its VALU and LDS stores while its SIMD's MFMA pipe is busy with the consumers' work.
// B16 (with NP = 1, not XSQ): the producers read G and X from their bf16 copies (d.g16, d.x16: 8 B per
// four values, nothing converted).  The bf16 weight gradient is bound by the producers' loads (no
// MFMAs: the same time; no loads: half, profiles/r07x_*), so half the bytes is most of what it can gain.
template <bool XSQ, int NTAP, int NP, bool B16 = false>
__device__ __forceinline__ void wg_x3p_body(const WgDesc& d, __bf16* lds, int split, int ky, int ct) {
  static_assert(!B16 || (NP == 1 && !XSQ), "bf16 copies: one plane, plain X");
  typedef __bf16 b4 __attribute__((ext_vector_type(4)));
  typedef __bf16 b8 __attribute__((ext_vector_type(8)));
  constexpr int CW = 192 / NTAP;          // X channels per block
  constexpr int BM = 192, WM = 96, WN = 48, BK = 32;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int PITCH = 192;
  constexpr int XR = BK + NTAP - 1;       // X pixel rows per step
  constexpr int GPLANE = BK * PITCH, XPLANE = 34 * PITCH;
  constexpr int GOPER = NP * GPLANE;
  constexpr int STAGE = NP * (GPLANE + XPLANE);
  constexpr int NC = 512, NPR = 256;      // consumer / producer threads
  constexpr int QG = BK * (BM / 4) / NPR; // 6 float4 of G per producer thread and step
  constexpr int XQ4 = XR * (CW / 4);      // float4 of X per step
  constexpr int QX = (XQ4 + NPR - 1) / NPR;  // 3 (NTAP 3) or 4 (NTAP 2)
  static_assert(QG * NPR == BK * BM / 4, "G slots");
  const int kx0 = NTAP == 3 ? 0 : 1;
  const int t0 = ky * 5 + kx0;
  const int c0 = ct * CW;
  const int pb = split * d.pps;
  int pe = pb + d.pps;
  if (pe > (int)d.P) pe = (int)d.P;
  const int nsteps = pe > pb ? (pe - pb) / BK : 0;
  const int q0 = pb - ((nsteps & 1) ? BK : 0);  // an odd count starts with one all-zero (dead) step
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  auto swz = [](int row) { return ((((row >> 1) & 1) << 5) | (((row >> 3) & 1) << 4)); };

  if (w >= NC / 64) {
    // ---------------------------------------------------------------- producer waves
    // WG_X3P_PRIO: the producers' issue priority over the consumer waves of their SIMD (the younger
    // waves otherwise get only the VALU slots the older ones leave, and the barrier waits for them)
    if (WG_X3P_PRIO) __builtin_amdgcn_s_setprio(WG_X3P_PRIO);
    const int pt = tid - NC;
    const int dyt = d.dy[t0], dx0 = d.dx[t0];
    int grow[QG], gcol[QG], xrow[QX], xcol[QX];
#pragma unroll
    for (int q = 0; q < QG; ++q) {
      const int f = pt + NPR * q;
      grow[q] = f / (BM / 4);
      gcol[q] = (f - grow[q] * (BM / 4)) * 4;
    }
#pragma unroll
    for (int q = 0; q < QX; ++q) {
      const int f = min(pt + NPR * q, XQ4 - 1);  // past the image: a second copy of the last float4
      xrow[q] = f / (CW / 4);
      xcol[q] = (f - xrow[q] * (CW / 4)) * 4;
    }
    constexpr uint32_t ESZ = B16 ? 2u : 4u;  // bytes per element of the operands the producers read
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    typedef typename std::conditional<B16, u32x2, floatx4v>::type slot_t;  // four values
    uint32_t goff[QG];
#pragma unroll
    for (int q = 0; q < QG; ++q) goff[q] = ((uint32_t)grow[q] * (uint32_t)d.gs_w + (uint32_t)gcol[q]) * ESZ;
    slot_t ga[QG] = {}, xa[QX] = {}, gb[QG] = {}, xb[QX] = {};
    uint32_t oka = 0, okb = 0;
    // step k of the block (pixels q0 + k BK ..).  Branch-free: every load reads an in-range address
    // (dead steps pixel 0, padding a clamped column / row) and a select zeroes what must be zero; with
    // a zero-page pointer select the compiler branched around each load on the uniform step flag and
    // drained the loads in flight (s_waitcnt vmcnt(0)) inside the branches.
    // the zeroing select is applied at the store (store()), so no value is consumed before its step
    auto load = [&](int k, slot_t (&rg)[QG], slot_t (&rx)[QX], uint32_t& okm) {
      if (WG_X3P_ABL & 32) k = 0;  // the first step's addresses every step (hoisted address math, L2-hot)
      const int p0 = q0 + k * BK;
      const bool live = p0 >= pb && p0 < pe;
      const uint32_t pp = (WG_X3P_ABL & 8) ? (uint32_t)pb : live ? (uint32_t)p0 : 0u;
      const uint32_t img = fdiv(pp, d.fd_hw);
      const uint32_t rr = pp - img * d.fd_hw.d;
      const uint32_t gy = fdiv(rr, d.fd_w);
      const uint32_t gx0 = rr - gy * d.fd_w.d;
      const int iy = (int)gy * 2 + dyt;
      const bool rowok = live && (unsigned)iy < (unsigned)d.Hx;
      const int iyc = min(max(iy, 0), d.Hx - 1);
      // wave-uniform bases (SGPRs) + 32-bit per-lane byte offsets: the saddr form of global_load
      const long long goe = (long long)img * d.gs_n + (long long)gy * d.gs_h + (long long)gx0 * d.gs_w;
      const long long xoe = (long long)img * d.xs_n + (long long)iyc * d.xs_h + c0;
      const char* gbase = B16 ? (const char*)((const __bf16*)d.g16 + goe) : (const char*)(d.g + goe);
      const char* xbase = B16 ? (const char*)((const __bf16*)d.x16 + xoe) : (const char*)(d.x + xoe);
#pragma unroll
      for (int q = 0; q < QG; ++q)
        if (!(WG_X3P_ABL & 1)) rg[q] = *(const slot_t*)(gbase + goff[q]);
      okm = live ? 1u : 0u;
#pragma unroll
      for (int q = 0; q < QX; ++q) {
        const int ix = ((int)gx0 + xrow[q]) * 2 + dx0;
        const bool ok = rowok && (unsigned)ix < (unsigned)d.Wx;
        const uint32_t ixc = (uint32_t)min(max(ix, 0), d.Wx - 1);
        if (!(WG_X3P_ABL & 1)) rx[q] = *(const slot_t*)(xbase + (ixc * (uint32_t)d.xs_w + (uint32_t)xcol[q]) * ESZ);
        okm |= ok ? 2u << q : 0u;
      }
    };
    auto put = [&](__bf16* dst, int plane, floatx4v v, bool gop = false) {
      if (NP == 1 || (WG_X3P_ABL & 16) || ((WG_X3P_ABL & 64) && gop)) {  // ABL 64: G stored unsplit (diagnostic)
        typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
        *(b4*)dst = __builtin_bit_cast(b4, u32x2{ic_cvt_pk_bf16(v[0], v[1]), ic_cvt_pk_bf16(v[2], v[3])});
      } else {
        b4 vh, vm, vl;
        split3_bf16x4(v, vh, vm, vl);
        *(b4*)dst = vh;
        *(b4*)(dst + plane) = vm;
        *(b4*)(dst + 2 * plane) = vl;
      }
    };
    const floatx4v zero4 = {0.f, 0.f, 0.f, 0.f};
    auto store = [&](int buf, const slot_t (&rg)[QG], const slot_t (&rx)[QX], uint32_t okm) {
      if (WG_X3P_ABL & 2) return;
      __bf16* base = lds + buf * STAGE;
      if constexpr (B16) {  // bf16 copies: four values already rounded, 8 B straight to LDS
        const u32x2 z2 = {0u, 0u};
#pragma unroll
        for (int q = 0; q < QG; ++q)
          *(u32x2*)(base + grow[q] * PITCH + (gcol[q] ^ swz(grow[q]))) = (okm & 1u) ? rg[q] : z2;
#pragma unroll
        for (int q = 0; q < QX; ++q)
          *(u32x2*)(base + GOPER + xrow[q] * PITCH + (xcol[q] ^ swz(xrow[q]))) = (okm & (2u << q)) ? rx[q] : z2;
        return;
      } else {
#pragma unroll
      for (int q = 0; q < QG; ++q) {
        put(base + grow[q] * PITCH + (gcol[q] ^ swz(grow[q])), GPLANE, (okm & 1u) ? rg[q] : zero4, true);
        __builtin_amdgcn_sched_barrier(0);  // one slot at a time: the split temporaries of ten slots spilled
      }
#pragma unroll
      for (int q = 0; q < QX; ++q) {
        floatx4v v = (okm & (2u << q)) ? rx[q] : zero4;
        if (XSQ) v = v * v;
        put(base + GOPER + xrow[q] * PITCH + (xcol[q] ^ swz(xrow[q])), XPLANE, v);
        __builtin_amdgcn_sched_barrier(0);
      }
      }
    };
    const int L = (pe - q0) / BK;  // steps run (even)
    if constexpr (B16 && WG_X3P_DEEP) {
      // bf16 slots are half the registers: a third set keeps three steps of loads in flight
      // (the r07x ablation showed the bf16 kernel waits on its loads, not on its MFMAs)
      slot_t gc[QG] = {}, xc[QX] = {};
      uint32_t okc = 0;
      if (L > 0) {
        load(0, ga, xa, oka);
        load(1, gb, xb, okb);
        load(2, gc, xc, okc);
        store(0, ga, xa, oka);
        load(3, ga, xa, oka);
      }
      __syncthreads();
      // at sub-step j the consumers run step j; the producers store step j + 1 and load step j + 4
      for (int k = 0; k < L; k += 6) {
        store(1, gb, xb, okb);
        load(k + 4, gb, xb, okb);
        __syncthreads();
        if (k + 1 >= L) break;
        store(0, gc, xc, okc);
        load(k + 5, gc, xc, okc);
        __syncthreads();
        if (k + 2 >= L) break;
        store(1, ga, xa, oka);
        load(k + 6, ga, xa, oka);
        __syncthreads();
        if (k + 3 >= L) break;
        store(0, gb, xb, okb);
        load(k + 7, gb, xb, okb);
        __syncthreads();
        if (k + 4 >= L) break;
        store(1, gc, xc, okc);
        load(k + 8, gc, xc, okc);
        __syncthreads();
        if (k + 5 >= L) break;
        store(0, ga, xa, oka);
        load(k + 9, ga, xa, oka);
        __syncthreads();
      }
      return;
    }
    if (L > 0) {
      load(0, ga, xa, oka);
      load(1, gb, xb, okb);
      store(0, ga, xa, oka);
      load(2, ga, xa, oka);
    }
    __syncthreads();
    for (int k = 0; k < L; k += 2) {
      store(1, gb, xb, okb);  // step k + 1, while the consumers run step k
      load(k + 3, gb, xb, okb);
      __syncthreads();
      store(0, ga, xa, oka);  // step k + 2, while the consumers run step k + 1
      load(k + 4, ga, xa, oka);
      __syncthreads();
    }
    return;
  }

  // ------------------------------------------------------------------ consumer waves
  const int wm = w >> 2, wn = w & 3;
  const int li = lane & 15, lq = lane >> 4;
  const int tr_r = 8 * lq + (li >> 2);
  const int tr_c = 4 * (li & 3);
  floatx4v acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = floatx4v{0.f, 0.f, 0.f, 0.f};
  const int tr_sw = swz(tr_r);
  auto tr8a = [&](const __bf16* plane, int col) {
    const __bf16* src = plane + tr_r * PITCH + ((col + tr_c) ^ tr_sw);
    const b4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) b4*)src);
    const b4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) b4*)(src + 4 * PITCH));
    return (b8)__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  };
  int xo_lo[TN], xo_hi[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int vcol = wn * WN + 16 * j;
    const int tt = vcol / CW, cc = vcol - (vcol / CW) * CW;
    const int r0 = tr_r + tt;
    xo_lo[j] = r0 * PITCH + ((cc + tr_c) ^ swz(r0));
    xo_hi[j] = (r0 + 4) * PITCH + ((cc + tr_c) ^ swz(r0 + 4));
  }
  auto tr8b = [&](const __bf16* plane, int j) {
    const b4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) b4*)(plane + xo_lo[j]));
    const b4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) b4*)(plane + xo_hi[j]));
    return (b8)__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  };
  auto step = [&](int buf) {
    const __bf16* sb = lds + buf * STAGE;
    b8 bb[NP][TN];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int q = 0; q < NP; ++q) bb[q][j] = tr8b(sb + GOPER + q * XPLANE, j);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      b8 a[NP];
#pragma unroll
      for (int q = 0; q < NP; ++q) a[q] = tr8a(sb + q * GPLANE, wm * WM + 16 * i);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        floatx4v& c = acc[i][j];
        if constexpr (NP == 1) {
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], bb[0][j], c, 0, 0, 0);
        } else if (!(WG_X3P_ABL & 4)) {
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], bb[0][j], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], bb[1][j], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], bb[2][j], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], bb[0][j], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], bb[1][j], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], bb[0][j], c, 0, 0, 0);
        }
      }
    }
    __syncthreads();
  };
  const int L = (pe - q0) / BK;
  __syncthreads();
  for (int k = 0; k < L; k += 2) {
    step(0);
    step(1);
  }
  // C/D map of the 16x16 MFMA: row (g) = 4 lq + r, col = li; column tile j belongs to tap tt
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int vcol = wn * WN + 16 * j;
    const int tt = vcol / CW, cc = vcol - (vcol / CW) * CW;
    float* slab = d.partial + ((long long)split * d.T + t0 + 2 * tt) * (long long)d.Cg * d.ncols;
    const int col = c0 + cc + li;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gr = wm * WM + 16 * i + 4 * lq + r;
        slab[(long long)gr * d.ncols + col] = acc[i][j][r];
      }
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(acc[i][j]));
}

template <bool XSQ, int NP = 3, bool B16 = false>
__global__ void __launch_bounds__(768, 1) wg_x3p_kernel(const WgDesc d) {
  constexpr int STAGE = NP * (32 * 192 + 34 * 192);
  __shared__ __attribute__((aligned(16))) __bf16 lds[2 * STAGE];
  const int nblk = 25 * d.nsplit;
  const int b = blockIdx.x;
  const int wid = (b & 7) * (int)(gridDim.x >> 3) + (b >> 3);  // XCD-grouped; gridDim.x % 8 == 0
  if (wid >= nblk) return;
  const int split = wid / 25, rem = wid - (wid / 25) * 25;
  const int ky = rem / 5, u = rem - (rem / 5) * 5;
  if (u < 3) wg_x3p_body<XSQ, 3, NP, B16>(d, lds, split, ky, u);
  else wg_x3p_body<XSQ, 2, NP, B16>(d, lds, split, ky, u - 3);
}

struct WgRed {
  const float* partial;
  float* out;    // final [g][c][kk] (G == 1) or level-2 partial [G][g][t][c]
  int nsplit, Tp, T, Cg, Cx, ncols, kk, generic, spg, G;
  int kk_of_t[IC_MAXT];
};

// thread = one (g, t, c) element and one group of `spg` splits; 4 independent
// accumulators over the group (fixed order -> deterministic)
__global__ void wg_reduce_kernel(const WgRed r) {
  const long long total = (long long)r.Cg * r.Cx * r.T;
  const int grp = blockIdx.y;
  const int s0 = grp * r.spg;
  const int s1 = min(r.nsplit, s0 + r.spg);
  const long long sstride = (long long)r.Tp * r.Cg * r.ncols;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % r.Cx);
    const long long gt = i / r.Cx;
    const int t = (int)(gt % r.T);
    const int g = (int)(gt / r.T);
    const int tp = r.generic ? 0 : t;
    const int col = r.generic ? t * r.Cx + c : c;
    const float* src = r.partial + ((long long)tp * r.Cg + g) * r.ncols + col;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int sp = s0;
    for (; sp + 3 < s1; sp += 4) {
      a0 += src[(long long)sp * sstride];
      a1 += src[(long long)(sp + 1) * sstride];
      a2 += src[(long long)(sp + 2) * sstride];
      a3 += src[(long long)(sp + 3) * sstride];
    }
    for (; sp < s1; ++sp) a0 += src[(long long)sp * sstride];
    const float v = (a0 + a1) + (a2 + a3);
    if (r.G == 1)
      r.out[((long long)g * r.Cx + c) * r.kk + r.kk_of_t[t]] = v;
    else
      r.out[(long long)grp * total + i] = v;
  }
}

__global__ void wg_reduce2_kernel(const float* p2, int G, long long total, int Cx, int T, int kk,
                                  const WgRed r, float* out) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    float v = 0.f;
    for (int q = 0; q < G; ++q) v += p2[(long long)q * total + i];
    const int c = (int)(i % Cx);
    const long long gt = i / Cx;
    const int t = (int)(gt % T);
    const int g = (int)(gt / T);
    out[((long long)g * Cx + c) * kk + r.kk_of_t[t]] = v;
  }
}

// The final level of the reduction through LDS: out[g][c][kk] is the weight's PyTorch layout (taps
// fastest), while the partials run channels fastest, so a thread per (g, t, c) writes 4 B every kk
// floats -- each wave's stores then touch 64 different lines (15.7x the compulsory write bytes,
// r04b).  Here block (g, cb) sums the partials of channels [cb CB, cb CB + CB) of row g over every
// tap in the same fixed order (reads coalesced along c), transposes them in LDS to [c][kk] and
// writes out[g][cb CB .. + CB][0 .. kk) as one contiguous run.  Bitwise the result of
// wg_reduce_kernel / wg_reduce2_kernel.
__global__ void __launch_bounds__(256) wg_reduce_t_kernel(const WgRed r, int CB) {
  extern __shared__ float row[];  // [CB][kk]
  const int g = blockIdx.x, c0 = blockIdx.y * CB, cn = min(CB, r.Cx - c0);
  const long long sstride = (long long)r.Tp * r.Cg * r.ncols;
  for (int idx = threadIdx.x; idx < r.T * cn; idx += blockDim.x) {
    const int t = idx / cn, cl = idx - t * cn, c = c0 + cl;
    const int tp = r.generic ? 0 : t;
    const int col = r.generic ? t * r.Cx + c : c;
    const float* src = r.partial + ((long long)tp * r.Cg + g) * r.ncols + col;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int sp = 0;
    for (; sp + 3 < r.nsplit; sp += 4) {
      a0 += src[(long long)sp * sstride];
      a1 += src[(long long)(sp + 1) * sstride];
      a2 += src[(long long)(sp + 2) * sstride];
      a3 += src[(long long)(sp + 3) * sstride];
    }
    for (; sp < r.nsplit; ++sp) a0 += src[(long long)sp * sstride];
    row[cl * r.kk + r.kk_of_t[t]] = (a0 + a1) + (a2 + a3);
  }
  __syncthreads();
  float* o = r.out + ((long long)g * r.Cx + c0) * r.kk;
  for (int j = threadIdx.x; j < cn * r.kk; j += blockDim.x) o[j] = row[j];
}

__global__ void __launch_bounds__(256) wg_reduce2_t_kernel(const float* p2, int G, long long total, const WgRed r,
                                                           float* out, int CB) {
  extern __shared__ float row[];  // [CB][kk]
  const int g = blockIdx.x, c0 = blockIdx.y * CB, cn = min(CB, r.Cx - c0);
  for (int idx = threadIdx.x; idx < r.T * cn; idx += blockDim.x) {
    const int t = idx / cn, cl = idx - t * cn;
    const long long i = ((long long)g * r.T + t) * r.Cx + c0 + cl;
    float v = 0.f;
    for (int q = 0; q < G; ++q) v += p2[(long long)q * total + i];
    row[cl * r.kk + r.kk_of_t[t]] = v;
  }
  __syncthreads();
  float* o = out + ((long long)g * r.Cx + c0) * r.kk;
  for (int j = threadIdx.x; j < cn * r.kk; j += blockDim.x) o[j] = row[j];
}

template <int BM, int BN, int WM, int WN, bool GEN>
int wg_launch_t(const WgDesc& d, hipStream_t s) {
  const int Tp = GEN ? 1 : d.T;
  dim3 grid((d.mtiles * d.ntiles * Tp * d.nsplit + 7) / 8 * 8);
  hipLaunchKernelGGL((wg_kernel<BM, BN, WM, WN, GEN>), grid, dim3(256), 0, s, d);
  IC_CHECK_LAUNCH();
  return IC_OK;
}

template <int BM, int BN, int WM, int WN>
int wg_glds_launch_t(const WgDesc& d, hipStream_t s) {
  dim3 grid((d.mtiles * d.ntiles * d.T * d.nsplit + 7) / 8 * 8);
  if (d.x_op == AOP_SQUARE)
    hipLaunchKernelGGL((wg_glds_kernel<BM, BN, WM, WN, true>), grid, dim3(256), 0, s, d);
  else
    hipLaunchKernelGGL((wg_glds_kernel<BM, BN, WM, WN, false>), grid, dim3(256), 0, s, d);
  IC_CHECK_LAUNCH();
  return IC_OK;
}

// 5x5 stride-2 weight gradients of 192 x 192 channels on row-fast maps: the tap-group kernel
static bool wg_x3g_ok(const WgDesc& d) {
  return WG_X3G && WG_X3_DUAL && !d.generic && d.stride == 2 && d.T == 25 && d.Cg == 192 && d.Cx == 192 &&
         d.ncols == 192 && d.mtiles == 1 && d.ntiles == 1 && d.rowfast && d.Wg % 32 == 0 && d.pps % 32 == 0 &&
         d.P % 32 == 0;
}

int wg_x3_launch(const WgDesc& d, hipStream_t s) {
  const bool sq = d.x_op == AOP_SQUARE;
  dim3 grid((d.mtiles * d.ntiles * d.T * d.nsplit + 7) / 8 * 8);
  constexpr bool TWO = WG_X3_TWO;
  if (wg_x3g_ok(d)) {
    if (WG_X3P_B16 && d.bf16 && !sq && d.g16 && d.x16) {
      hipLaunchKernelGGL((wg_x3p_kernel<false, 1, true>), grid, dim3(768), 0, s, d);
    } else if (d.bf16) {
      if (sq) hipLaunchKernelGGL((wg_x3p_kernel<true, 1>), grid, dim3(768), 0, s, d);
      else hipLaunchKernelGGL((wg_x3p_kernel<false, 1>), grid, dim3(768), 0, s, d);
    } else if (sq) hipLaunchKernelGGL((wg_x3p_kernel<true>), grid, dim3(768), 0, s, d);
    else hipLaunchKernelGGL((wg_x3p_kernel<false>), grid, dim3(768), 0, s, d);
  } else if (WG_X3_DUAL && d.rowfast && d.Wg % 32 == 0 && d.pps % 32 == 0) {
    if (d.bf16) {
      if (sq) hipLaunchKernelGGL((wg_x3d_kernel<true, false, 1>), grid, dim3(512), 0, s, d);
      else hipLaunchKernelGGL((wg_x3d_kernel<false, false, 1>), grid, dim3(512), 0, s, d);
    } else if (sq) hipLaunchKernelGGL((wg_x3d_kernel<true, false>), grid, dim3(512), 0, s, d);
    else hipLaunchKernelGGL((wg_x3d_kernel<false, false>), grid, dim3(512), 0, s, d);
  } else if (WG_X3_DUAL16 && d.rowfast && d.Wg % 16 == 0 && d.pps % 32 == 0 && d.P % 32 == 0) {
    // whole 32-pixel steps only: with P % 32 == 16 the last split would end on half a step
    if (d.bf16) {
      if (sq) hipLaunchKernelGGL((wg_x3d_kernel<true, true, 1>), grid, dim3(512), 0, s, d);
      else hipLaunchKernelGGL((wg_x3d_kernel<false, true, 1>), grid, dim3(512), 0, s, d);
    } else if (sq) hipLaunchKernelGGL((wg_x3d_kernel<true, true>), grid, dim3(512), 0, s, d);
    else hipLaunchKernelGGL((wg_x3d_kernel<false, true>), grid, dim3(512), 0, s, d);
  } else if (d.bf16) {
    return IC_ERR_ARG;  // wg_plan keeps bf16 only where the two-wave kernel runs
  } else if (d.rowfast) {
    if (sq) hipLaunchKernelGGL((wg_x3_kernel<true, true, TWO>), grid, dim3(256), 0, s, d);
    else hipLaunchKernelGGL((wg_x3_kernel<true, false, TWO>), grid, dim3(256), 0, s, d);
  } else {
    if (sq) hipLaunchKernelGGL((wg_x3_kernel<false, true, TWO>), grid, dim3(256), 0, s, d);
    else hipLaunchKernelGGL((wg_x3_kernel<false, false, TWO>), grid, dim3(256), 0, s, d);
  }
  IC_CHECK_LAUNCH();
  return IC_OK;
}

// ---------------------------------------------------------------- colsum
// Generic strided form (small / non-NHWC tensors).
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

// Planar form (NCHW with contiguous H*W planes, e.g. the 3-channel image
// gradient): block (chunk, c, n) sums one contiguous run of a plane with
// float4 loads and a fixed-order block reduction.
__global__ void __launch_bounds__(256) colsum_planes_kernel(const float* t, long long s_n, long long s_c, int C,
                                                            int HW, int chunk, int nchunk, float* part) {
  __shared__ float lds[16];
  const int ck = blockIdx.x, c = blockIdx.y, n = blockIdx.z;
  const float* base = t + (long long)n * s_n + (long long)c * s_c;
  const int b0 = ck * chunk;
  const int b1 = min(HW, b0 + chunk);
  float acc[1] = {0.f};
  if (((uintptr_t)base & 15) == 0 && (b0 & 3) == 0) {
    const int n4 = (b1 - b0) >> 2;
    const floatx4v* p4 = (const floatx4v*)(base + b0);
    floatx4v a = {0.f, 0.f, 0.f, 0.f};
    for (int i = threadIdx.x; i < n4; i += 256) a += p4[i];
    acc[0] = (a[0] + a[1]) + (a[2] + a[3]);
    for (int i = b0 + 4 * n4 + threadIdx.x; i < b1; i += 256) acc[0] += base[i];
  } else {
    for (int i = b0 + threadIdx.x; i < b1; i += 256) acc[0] += base[i];
  }
  block_sum<1>(acc, lds);
  if (threadIdx.x == 0) part[((long long)n * nchunk + ck) * C + c] = acc[0];
}

// NHWC-dense form: rows x C, float4 per thread, rows interleaved over the
// block's thread groups, then a fixed-order LDS combine per column.
__global__ void __launch_bounds__(256) colsum_rows_kernel(const float* t, long long rows, int C, long long rpb,
                                                          float* part) {
  __shared__ float lds[8192];
  const int c4n = C >> 2;            // float4 per row
  const int groups = 256 / c4n;      // row groups
  const int tid = threadIdx.x;
  const int g = tid / c4n, c4 = tid - (tid / c4n) * c4n;
  const long long r0 = (long long)blockIdx.x * rpb;
  long long r1 = r0 + rpb;
  if (r1 > rows) r1 = rows;
  floatx4v acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
  if (g < groups) {
    const float* base = t + (size_t)c4 * 4;
    long long r = r0 + g;
    for (; r + 3 * groups < r1; r += 4 * groups) {  // four 16-B loads in flight per thread
      const floatx4v v0 = *(const floatx4v*)(base + (size_t)r * C);
      const floatx4v v1 = *(const floatx4v*)(base + (size_t)(r + groups) * C);
      const floatx4v v2 = *(const floatx4v*)(base + (size_t)(r + 2 * groups) * C);
      const floatx4v v3 = *(const floatx4v*)(base + (size_t)(r + 3 * groups) * C);
      acc0 += v0; acc1 += v1; acc2 += v2; acc3 += v3;
    }
    for (; r < r1; r += groups) acc0 += *(const floatx4v*)(base + (size_t)r * C);
    acc0 += acc1;
    acc2 += acc3;
    acc0 += acc2;
    *(floatx4v*)&lds[(g * c4n + c4) * 4] = acc0;
  }
  __syncthreads();
  for (int c = tid; c < C; c += 256) {
    float v = 0.f;
    for (int q = 0; q < groups; ++q) v += lds[q * C + c];
    part[(long long)blockIdx.x * C + c] = v;
  }
}

// one wave per column: lanes stride over the block partials, fixed-order tree
__global__ void colsum_final_kernel(const float* part, int nb, int C, float scale, float* out) {
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (c >= C) return;
  float acc = 0.f;
  for (int b = lane; b < nb; b += 64) acc += part[(long long)b * C + c];
  acc = wave_sum(acc);
  if (lane == 0) out[c] = acc * scale;
}

int colsum_blocks(long long rows) {
  long long nb = (rows + 255) / 256;
  if (nb > 512) nb = 512;
  if (nb < 1) nb = 1;
  return (int)nb;
}

}  // namespace

constexpr int WG_SPG = 32;  // splits summed per thread in the first reduce level
#ifndef WG_REDUCE_T
#define WG_REDUCE_T 1  // last reduce level through an LDS transpose (coalesced [g][c][kk] rows)
#endif

size_t wg_plan(WgDesc& d) {
  // split kernel: NHWC, 4-aligned channel rows, 192-wide tiles (wg_x3_kernel)
  auto a16 = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
  if (d.x3 && (d.generic || d.Cx < 128 || d.Cg < 128 || d.gs_c != 1 || d.xs_c != 1 || d.Cg % 4 || d.Cx % 4 ||
               !a16(d.g) || !a16(d.x) || d.gs_w % 4 || d.gs_h % 4 || d.gs_n % 4 || d.xs_w % 4 || d.xs_h % 4 ||
               d.xs_n % 4))
    d.x3 = 0;
  if (d.generic) { d.bm = 192; d.bn = 64; d.ncols = d.T * d.Cx; }
  else { d.bm = 192; d.bn = (d.Cx >= 128) ? 192 : 64; d.ncols = d.Cx; }
  d.mtiles = ic_cdiv(d.Cg, d.bm);
  d.ntiles = ic_cdiv(d.ncols, d.bn);
  d.P = (long long)d.N * d.Hg * d.Wg;
  const long long tiles = (long long)d.mtiles * d.ntiles *
                          (d.generic ? 1 : d.T);
  // one full wave of blocks: 256 CUs x 2 resident blocks = 512 slots, so a
  // grid of just over 512 equal blocks would run at half speed; never fewer
  // than 64 pixels per split
  const long long slots = (d.x3 && !WG_X3_TWO) ? 256 : 512;  // resident blocks: 1 or 2 per CU
  long long ns = tiles >= slots ? 1 : slots / tiles;
  long long maxs = (d.P + 63) / 64;
  if (ns > maxs) ns = maxs;
  if (ns < 1) ns = 1;
  long long pps = (d.P + ns - 1) / ns;
  pps = (pps + 31) / 32 * 32;
  d.pps = (int)pps;
  d.nsplit = (int)((d.P + pps - 1) / pps);
  if (d.nsplit < 1) d.nsplit = 1;
  // bf16 operands run on the two-wave kernel only (wg_x3_launch's row-fast conditions; pps is a
  // multiple of 32); elsewhere the split kernel when split arithmetic was asked for, else fp32
  if (d.bf16 && !(d.x3 && WG_X3_DUAL && WG_X3_DUAL16 && d.Wg % 16 == 0 && (d.Wg % 32 == 0 || d.P % 32 == 0) &&
                  (long long)d.gs_w * 16 < (1LL << 31) && (long long)d.stride * 16 * d.xs_w < (1LL << 31))) {
    d.bf16 = 0;
    if (!d.split_ok) d.x3 = 0;
  }
  const int Tp = d.generic ? 1 : d.T;
  const size_t slab = (size_t)d.nsplit * Tp * (size_t)d.Cg * d.ncols * sizeof(float);
  const int G = (d.nsplit + WG_SPG - 1) / WG_SPG;
  const size_t lvl2 = G > 1 ? (size_t)G * d.Cg * d.Cx * d.T * sizeof(float) : 0;
  return ic_align(slab, 256) + lvl2;
}

void wg_prepare(WgDesc& d) {
  d.fd_hw = make_fastdiv((uint32_t)((long long)d.Hg * d.Wg));
  d.rowfast = d.Wg % 16 == 0 && d.pps % 16 == 0 && d.gs_w * 16 < (1LL << 31) &&
              (long long)d.stride * 16 * d.xs_w < (1LL << 31);
  d.fd_w = make_fastdiv((uint32_t)d.Wg);
  d.g_vec = (d.gs_c == 1 && d.Cg % 4 == 0);
}

int wg_kernel_kind(const WgDesc& d) {
  // LDS-DMA path: 16-B aligned float4 rows in both operands
  auto a16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  const bool glds_ok = d.g_vec && !d.generic && a16(d.g) && a16(d.x) && d.gs_w % 4 == 0 && d.gs_h % 4 == 0 &&
                       d.gs_n % 4 == 0 && d.xs_w % 4 == 0 && d.xs_h % 4 == 0 && d.xs_n % 4 == 0;
  if (d.generic) return IC_KERNEL_WG_FP32_GATHER;
  if (d.x3) return d.bf16 ? IC_KERNEL_WG_BF16 : IC_KERNEL_WG_SPLIT;
  return glds_ok ? IC_KERNEL_WG_LDSDMA : IC_KERNEL_WG_FP32;
}

int wg_run(WgDesc& d, hipStream_t s) {
  if (d.P == 0) return IC_OK;
  if (d.P >= (1LL << 31)) return IC_ERR_ARG;  // 32-bit pixel indexing
  wg_prepare(d);
  if (!d.generic && (d.xs_c != 1 || d.Cx % 4 != 0)) return IC_ERR_ARG;
  switch (wg_kernel_kind(d)) {
    case IC_KERNEL_WG_FP32_GATHER:
      return wg_launch_t<192, 64, 96, 32, true>(d, s);
    case IC_KERNEL_WG_SPLIT:
    case IC_KERNEL_WG_BF16:
      if (!d.g_vec || d.bn != 192 || d.bm != 192) return IC_ERR_ARG;
      return wg_x3_launch(d, s);
    case IC_KERNEL_WG_LDSDMA:
      if (d.bn == 192) return wg_glds_launch_t<192, 192, 96, 96>(d, s);
      return wg_glds_launch_t<192, 64, 96, 32>(d, s);
    default:
      if (d.bn == 192) return wg_launch_t<192, 192, 96, 96, false>(d, s);
      return wg_launch_t<192, 64, 96, 32, false>(d, s);
  }
}

long long wg_grid_blocks(const WgDesc& d) {
  if (d.generic) return (d.mtiles * d.ntiles * d.nsplit + 7) / 8 * 8;
  return ((long long)d.mtiles * d.ntiles * d.T * d.nsplit + 7) / 8 * 8;
}

int wg_reduce(const WgDesc& d, float* out, const int* kk_of_t, int kk, hipStream_t s) {
  WgRed r;
  r.partial = d.partial; r.nsplit = d.nsplit; r.Tp = d.generic ? 1 : d.T; r.T = d.T;
  r.Cg = d.Cg; r.Cx = d.Cx; r.ncols = d.ncols; r.kk = kk; r.generic = d.generic;
  r.spg = WG_SPG;
  r.G = (d.nsplit + WG_SPG - 1) / WG_SPG;
  for (int t = 0; t < d.T; ++t) r.kk_of_t[t] = kk_of_t[t];
  const long long total = (long long)d.Cg * d.Cx * d.T;
  const size_t slab = (size_t)d.nsplit * r.Tp * (size_t)d.Cg * d.ncols * sizeof(float);
  float* p2 = (float*)((char*)d.partial + ic_align(slab, 256));
  r.out = r.G == 1 ? out : p2;
  long long blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) return IC_OK;
  // the last level transposes [CB channels][kk] slices of each g row through LDS (wg_reduce_t_kernel):
  // CB sized for about two (t, c) elements per thread
  const int CB = std::max(1, std::min(d.Cx, 512 / std::max(1, d.T)));
  const size_t rowb = (size_t)CB * kk * sizeof(float);
  const bool tr = WG_REDUCE_T && rowb <= 64 * 1024 && kk >= d.T;
  const dim3 tgrid((unsigned)d.Cg, (unsigned)((d.Cx + CB - 1) / CB));
  if (r.G == 1 && tr) {
    hipLaunchKernelGGL(wg_reduce_t_kernel, tgrid, dim3(256), rowb, s, r, CB);
    IC_CHECK_LAUNCH();
    return IC_OK;
  }
  hipLaunchKernelGGL(wg_reduce_kernel, dim3((unsigned)blocks, r.G), dim3(256), 0, s, r);
  IC_CHECK_LAUNCH();
  if (r.G > 1) {
    if (tr)
      hipLaunchKernelGGL(wg_reduce2_t_kernel, tgrid, dim3(256), rowb, s, p2, r.G, total, r, out, CB);
    else
      hipLaunchKernelGGL(wg_reduce2_kernel, dim3((unsigned)blocks), dim3(256), 0, s, p2, r.G, total, d.Cx, d.T, kk,
                         r, out);
    IC_CHECK_LAUNCH();
  }
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
  const bool nhwc = s_c == 1 && s_w == C && s_h == (long long)W * C && s_n == (long long)H * W * C;
  const long long HW = (long long)H * W;
  const bool planar = s_w == 1 && s_h == W && HW >= 1024 && HW < (1LL << 30) && (long long)N * C <= nb;
  if (nhwc && C % 4 == 0 && C / 4 <= 256 && (C / 4) * (256 / (C / 4)) * 4 <= 8192) {
    hipLaunchKernelGGL(colsum_rows_kernel, dim3(nb), dim3(256), 0, s, t, rows, C, rpb, part);
  } else if (planar) {
    // about nb blocks in total: chunks per plane = nb / (N*C), >= 1
    long long nchunk = nb / ((long long)N * C);
    if (nchunk < 1) nchunk = 1;
    long long chunk = (HW + nchunk - 1) / nchunk;
    chunk = (chunk + 1023) / 1024 * 1024;
    nchunk = (HW + chunk - 1) / chunk;
    hipLaunchKernelGGL(colsum_planes_kernel, dim3((unsigned)nchunk, C, N), dim3(256), 0, s, t, s_n, s_c, C, (int)HW,
                       (int)chunk, (int)nchunk, part);
    IC_CHECK_LAUNCH();
    hipLaunchKernelGGL(colsum_final_kernel, dim3((C + 3) / 4), dim3(256), 0, s, part, (int)(N * nchunk), C, scale,
                       out);
    IC_CHECK_LAUNCH();
    return IC_OK;
  } else {
    hipLaunchKernelGGL(colsum_partial_kernel, dim3(nb), dim3(256), 0, s, t, s_n, s_c, s_h, s_w, N, C, H,
                       W, rows, rpb, part);
  }
  IC_CHECK_LAUNCH();
  hipLaunchKernelGGL(colsum_final_kernel, dim3((C + 3) / 4), dim3(256), 0, s, part, nb, C, scale, out);
  IC_CHECK_LAUNCH();
  return IC_OK;
}
