// Implicit-GEMM convolution on fp32 MFMA (v_mfma_f32_32x32x2_f32), gfx950.
//
// Block = 256 threads = 4 waves; block tile BM (pixels) x BN (out channels);
// wave tile WM x WN made of 32x32 MFMA tiles.  K is walked in chunks of 32
// (one tap x 32 input channels on the fast path), register-staged into a
// single LDS image per operand ([rows][36]-float rows: 16-B aligned and
// conflict-free for the ds_read_b128 fragment reads below).
//
// K permutation: inside a 32-chunk, MFMA step (q,s) of lane-half h consumes
// logical k = 16h + 4q + s for BOTH operands, so each lane's 16 operand values
// per chunk are contiguous in LDS -> 4 x ds_read_b128 per operand tile.
#include "gemm.h"

#ifndef IG_X3_SGB
#define IG_X3_SGB 8  // ig_kernel_x3s: spread the next chunk's global loads, one per IG_X3_SGB MFMAs (0: compiler order, all loads up front)
#endif
#ifndef IG_BF16_SGB
#define IG_BF16_SGB 2  // bf16 kernels: one next-chunk global load per IG_BF16_SGB MFMAs (0: loads up front; 2: C3 fwd/dgrad 2.59 -> 2.53 ms)
#endif
#ifndef IG_BF16_S
// bf16 operands on small maps (64-row tiles) on ig_kernel_x3s's swizzled 16x16x32
// structure, one product: 0.056 vs 0.072-0.080 ms on g_a.6 / g_s.0 (the padded
// 64-channel-chunk kernel keeps the 128-row tiles: 0.378 vs 0.412 ms on g_a.2)
#define IG_BF16_S 1
#endif
#ifndef IG_BF16_NARROW
#define IG_BF16_NARROW 0  // 1: bf16 operands on the 32-channel-chunk kernel at 128-row tiles too
#endif

namespace {

constexpr int LDK = 36;

__device__ __forceinline__ void ig_store_out(const IgDesc& d, float v, uint32_t yoff, int n) {
  if (d.bias) v += d.bias[n];
  switch (d.epi) {
    case EPI_RELU:
      v = v > 0.f ? v : 0.f;
      break;
    case EPI_GDN: {
      const float xv = d.aux0[yoff];
      d.aux_out[yoff] = v;
      v = xv / sqrtf(v);
      break;
    }
    case EPI_IGDN: {
      const float xv = d.aux0[yoff];
      d.aux_out[yoff] = v;
      v = xv * sqrtf(v);
      break;
    }
    case EPI_GDN_BWD: {
      const float xv = d.aux0[yoff], nr = d.aux1[yoff], g = d.aux2[yoff];
      v = g / sqrtf(nr) + 2.f * xv * v;
      break;
    }
    case EPI_IGDN_BWD: {
      const float xv = d.aux0[yoff], nr = d.aux1[yoff], g = d.aux2[yoff];
      v = g * sqrtf(nr) + 2.f * xv * v;
      break;
    }
    default:
      break;
  }
  d.y[yoff] = v;
}

__device__ __forceinline__ uint32_t ig_out_offset(const IgDesc& d, const IgPhase& P, uint32_t m) {
  const uint32_t img = fdiv(m, P.fd_hw);
  const uint32_t rem = m - img * (uint32_t)P.fd_hw.d;
  const uint32_t gy = fdiv(rem, P.fd_w);
  const uint32_t gx = rem - gy * (uint32_t)P.Wg;
  const uint32_t oy = gy * P.oys + P.oy0, ox = gx * P.oxs + P.ox0;
  return img * (uint32_t)d.ys_n + oy * (uint32_t)d.ys_h + ox * (uint32_t)d.ys_w;
}

// keep every accumulator register live up to here: a store's data register
// is then never overwritten while the store is pending (which would wait for it)
template <int TM, int TN>
__device__ __forceinline__ void ig_hold32(floatx16 (&acc)[TM][TN]) {
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(acc[i][j]));
}

// epilogue shared by the fp32 and bf16 kernels.  C/D map of the 32x32 MFMA:
// col = lane&31, row = (reg&3)+8*(reg>>2)+4*(lane>>5)
template <int TM, int TN>
__device__ __forceinline__ void ig_epilogue(const IgDesc& d, const IgPhase& P, floatx16 (&acc)[TM][TN], uint32_t M,
                                            uint32_t m0, int n0, int wm, int wn, int WM, int WN, int r, int h,
                                            int split) {
  // stores straight from the held accumulators (see ig_epilogue16)
  if (d.ksplit > 1) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const uint32_t m = m0 + wm * WM + i * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
        if (m >= M) continue;
        float* prow = d.partial + ((size_t)split * d.Mtot + P.m_off + m) * d.Cout;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int n = n0 + wn * WN + j * 32 + r;
          if (n < d.Cout) prow[n] = acc[i][j][reg];
        }
      }
    ig_hold32<TM, TN>(acc);
    return;
  }
  const uint32_t ysc = (uint32_t)d.ys_c;
  if (d.epi == EPI_NONE || d.epi == EPI_RELU) {
    // plain conv epilogue: bias hoisted per column, optional ReLU
    float bj[TN];
    bool nok[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * WN + j * 32 + r;
      nok[j] = n < d.Cout;
      bj[j] = (d.bias && nok[j]) ? d.bias[n] : 0.f;
    }
    const bool relu = d.epi == EPI_RELU;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
          const float v = acc[i][j][reg] + bj[j];
          acc[i][j][reg] = (relu && !(v > 0.f)) ? 0.f : v;
        }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const uint32_t m = m0 + wm * WM + i * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
        if (m >= M) continue;
        float* yo = d.y + ig_out_offset(d, P, m);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          if (nok[j]) yo[(uint32_t)(n0 + wn * WN + j * 32 + r) * ysc] = acc[i][j][reg];
      }
    ig_hold32<TM, TN>(acc);
    return;
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const uint32_t m = m0 + wm * WM + i * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
      if (m >= M) continue;
      const uint32_t ob = ig_out_offset(d, P, m);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn * WN + j * 32 + r;
        if (n < d.Cout) ig_store_out(d, acc[i][j][reg], ob + (uint32_t)n * ysc, n);
      }
    }
}

__device__ __attribute__((aligned(16))) float ig_zero_page[4];

// SQ: square the A operand (GDN's x^2 on the non-fused GDN path); a template
// parameter so the conv main loop carries no per-element operand switch
template <int BM, int BN, int WM, int WN, bool GEN, bool SQ>
__global__ void __launch_bounds__(256, 2) ig_kernel(const IgDesc d) {
  constexpr int WAVES_N = BN / WN;
  constexpr int TM = WM / 32, TN = WN / 32;
  constexpr int APASS = BM / 32, BPASS = BN / 32;
  static_assert((BM / WM) * (BN / WN) == 4, "4 waves per block");
  __shared__ __attribute__((aligned(16))) float As[BM * LDK];
  __shared__ __attribute__((aligned(16))) float Bs[BN * LDK];

  const int zi = blockIdx.z;
  const int phase = zi / d.ksplit;
  const int split = zi - phase * d.ksplit;
  const IgPhase& P = d.ph[phase];
  // XCD-aware tile order: block b runs on XCD b % 8, so give each XCD a
  // contiguous range of m-tiles (neighbouring output rows share input rows,
  // which then hit that XCD's L2 instead of HBM)
  uint32_t bx = blockIdx.x;
  if ((gridDim.x & 7) == 0) bx = (bx & 7) * (gridDim.x >> 3) + (bx >> 3);
  if ((int)bx >= P.mtiles) return;

  const uint32_t M = (uint32_t)d.N * P.fd_hw.d;
  const uint32_t m0 = bx * BM;
  const int n0 = blockIdx.y * BN;
  const int nchunks = GEN ? (d.Kc >> 5) : P.T * (d.Cin >> 5);
  const int cb = split * d.kcps;
  const int ce = min(nchunks, cb + d.kcps);

  const int tid = threadIdx.x;
  const int lrow = tid >> 3, lc4 = tid & 7;
  const uint32_t xsh = (uint32_t)d.xs_h, xsw = (uint32_t)d.xs_w;

  // per-pass gather origin: pixel offset (32-bit) and input row/col of tap (0,0)
  uint32_t a_off[APASS];
  int a_iy[APASS], a_ix[APASS];
#pragma unroll
  for (int p = 0; p < APASS; ++p) {
    const uint32_t m = m0 + lrow + 32 * p;
    const bool ok = m < M;
    const uint32_t mm = ok ? m : 0u;
    const uint32_t img = fdiv(mm, P.fd_hw);
    const uint32_t rem = mm - img * (uint32_t)P.fd_hw.d;
    const uint32_t gy = fdiv(rem, P.fd_w);
    const uint32_t gx = rem - gy * (uint32_t)P.Wg;
    a_iy[p] = ok ? (int)gy * d.stride : -0x40000000;  // invalid rows fail the bounds test
    a_ix[p] = (int)gx * d.stride;
    a_off[p] = img * (uint32_t)d.xs_n + (uint32_t)a_iy[p] * xsh + (uint32_t)a_ix[p] * xsw;
  }
  const float* __restrict__ xg = d.x;

  floatx4v ra[APASS], rb[BPASS];

#define IG_GLOAD(c_)                                                                              \
  do {                                                                                            \
    const int c__ = (c_);                                                                         \
    if constexpr (!GEN) {                                                                         \
      /* channel chunk outer, tap inner: a pixel's chunk is re-read by the next */               \
      /* taps while it is still in L2 (tap-outer re-reads it ~T times from HBM) */                \
      const int cc = c__ / P.T, t = c__ - cc * P.T;                                               \
      const int dy = P.dy[t], dx = P.dx[t];                                                       \
      const uint32_t toff = (uint32_t)(dy * (int)xsh + dx * (int)xsw + cc * 32 + lc4 * 4);         \
      _Pragma("unroll") for (int p = 0; p < APASS; ++p) {                                         \
        const int iy = a_iy[p] + dy, ix = a_ix[p] + dx;                                           \
        /* branch-free gather: zero padding reads a zero page */                                  \
        const bool in = (unsigned)iy < (unsigned)d.Hx && (unsigned)ix < (unsigned)d.Wx;           \
        const float* src = in ? xg + (a_off[p] + toff) : ig_zero_page;                            \
        floatx4v v = *(const floatx4v*)src;                                                       \
        if constexpr (SQ) v = v * v;                                                              \
        ra[p] = v;                                                                                \
      }                                                                                           \
      const float* wb = P.wp + ((size_t)t * d.Npad + n0 + lrow) * d.Cin + cc * 32 + lc4 * 4;      \
      _Pragma("unroll") for (int p = 0; p < BPASS; ++p)                                           \
        rb[p] = *(const floatx4v*)(wb + (size_t)(32 * p) * d.Cin);                                  \
    } else {                                                                                      \
      _Pragma("unroll") for (int p = 0; p < APASS; ++p) {                                         \
        float v4[4];                                                                              \
        _Pragma("unroll") for (int e = 0; e < 4; ++e) {                                           \
          const int k = c__ * 32 + lc4 * 4 + e;                                                   \
          const int t = k / d.Cin, ci = k - t * d.Cin;                                            \
          float val = 0.f;                                                                        \
          if (t < P.T) {                                                                          \
            const int dy = P.dy[t], dx = P.dx[t];                                                 \
            const int iy = a_iy[p] + dy, ix = a_ix[p] + dx;                                       \
            if ((unsigned)iy < (unsigned)d.Hx && (unsigned)ix < (unsigned)d.Wx)                   \
              val = xg[a_off[p] + (uint32_t)(dy * (int)xsh + dx * (int)xsw) +                    \
                       (uint32_t)ci * (uint32_t)d.xs_c];                                         \
            if constexpr (SQ) val *= val;                                                         \
          }                                                                                       \
          v4[e] = val;                                                                            \
        }                                                                                         \
        ra[p] = floatx4v{v4[0], v4[1], v4[2], v4[3]};                                          \
      }                                                                                           \
      const float* wb = P.wp + (size_t)(n0 + lrow) * d.Kc + c__ * 32 + lc4 * 4;                   \
      _Pragma("unroll") for (int p = 0; p < BPASS; ++p)                                           \
        rb[p] = *(const floatx4v*)(wb + (size_t)(32 * p) * d.Kc);                                   \
    }                                                                                             \
  } while (0)

#define IG_SSTORE()                                                                               \
  do {                                                                                            \
    _Pragma("unroll") for (int p = 0; p < APASS; ++p)                                             \
      *(floatx4v*)&As[(lrow + 32 * p) * LDK + lc4 * 4] = ra[p];                                     \
    _Pragma("unroll") for (int p = 0; p < BPASS; ++p)                                             \
      *(floatx4v*)&Bs[(lrow + 32 * p) * LDK + lc4 * 4] = rb[p];                                     \
  } while (0)

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

  if (cb < ce) {
    IG_GLOAD(cb);
    IG_SSTORE();
  }
  __syncthreads();
  const float* Ard = &As[(wm * WM + r) * LDK + 16 * h];
  const float* Brd = &Bs[(wn * WN + r) * LDK + 16 * h];
  for (int c = cb; c < ce; ++c) {
    if (c + 1 < ce) IG_GLOAD(c + 1);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      floatx4v a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = *(const floatx4v*)(Ard + i * 32 * LDK + 4 * q);
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = *(const floatx4v*)(Brd + j * 32 * LDK + 4 * q);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][0], b[j][0], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][1], b[j][1], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][2], b[j][2], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][3], b[j][3], acc[i][j], 0, 0, 0);
        }
    }
    __syncthreads();
    if (c + 1 < ce) IG_SSTORE();
    __syncthreads();
  }
#undef IG_GLOAD
#undef IG_SSTORE

  ig_epilogue<TM, TN>(d, P, acc, M, m0, n0, wm, wn, WM, WN, r, h, split);
}

// ------------------------------------------------------------------ bf16
// Same implicit GEMM with bf16 operands and fp32 accumulation
// (v_mfma_f32_32x32x16_bf16): activations are read as fp32 and rounded to
// bf16 (round-to-nearest-even, v_cvt_pk_bf16_f32) on their way into LDS,
// weights come pre-packed in bf16.  K chunk = 64 channels of one tap
// (Cin % 64 == 0); LDS rows of 72 bf16 (144 B) make the 16-row fragment
// reads bank-conflict-free.  One MFMA consumes 16 k: lane (r, h) holds
// A[row r][k 8h..8h+7] and B[k 8h..8h+7][col r].
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

template <int BM, int BN, int WM, int WN>
__global__ void __launch_bounds__(256, 2) ig_kernel_bf16(const IgDesc d) {
  constexpr int LDKB = 72;
  constexpr int WAVES_N = BN / WN;
  constexpr int TM = WM / 32, TN = WN / 32;
  constexpr int APASS = BM / 16, BPASS = BN / 32;
  static_assert((BM / WM) * (BN / WN) == 4, "4 waves per block");
  __shared__ __attribute__((aligned(16))) __bf16 As[BM * LDKB];
  __shared__ __attribute__((aligned(16))) __bf16 Bs[BN * LDKB];

  const int zi = blockIdx.z;
  const int phase = zi / d.ksplit;
  const int split = zi - phase * d.ksplit;
  const IgPhase& P = d.ph[phase];
  uint32_t bx = blockIdx.x;
  if ((gridDim.x & 7) == 0) bx = (bx & 7) * (gridDim.x >> 3) + (bx >> 3);
  if ((int)bx >= P.mtiles) return;

  const uint32_t M = (uint32_t)d.N * P.fd_hw.d;
  const uint32_t m0 = bx * BM;
  const int n0 = blockIdx.y * BN;
  const int cpt = d.Cin >> 6;
  const int nchunks = P.T * cpt;
  const int cb = split * d.kcps;
  const int ce = min(nchunks, cb + d.kcps);

  const int tid = threadIdx.x;
  const int arow = tid >> 4, ac4 = tid & 15;   // A: 16 float4 per 64-wide row
  const int brow = tid >> 3, bc8 = tid & 7;    // B: 8 x 16 B per 64-wide bf16 row
  const uint32_t xsh = (uint32_t)d.xs_h, xsw = (uint32_t)d.xs_w;
  uint32_t a_off[APASS];
  int a_iy[APASS], a_ix[APASS];
#pragma unroll
  for (int p = 0; p < APASS; ++p) {
    const uint32_t m = m0 + arow + 16 * p;
    const bool ok = m < M;
    const uint32_t mm = ok ? m : 0u;
    const uint32_t img = fdiv(mm, P.fd_hw);
    const uint32_t rem = mm - img * (uint32_t)P.fd_hw.d;
    const uint32_t gy = fdiv(rem, P.fd_w);
    const uint32_t gx = rem - gy * (uint32_t)P.Wg;
    a_iy[p] = ok ? (int)gy * d.stride : -0x40000000;
    a_ix[p] = (int)gx * d.stride;
    a_off[p] = img * (uint32_t)d.xs_n + (uint32_t)a_iy[p] * xsh + (uint32_t)a_ix[p] * xsw;
  }
  const float* __restrict__ xg = d.x;
  const __bf16* __restrict__ wpb = (const __bf16*)P.wp;

  floatx4v ra[APASS];
  bf16x8 rb[BPASS];
  auto gload = [&](int c) {
    const int cc = c / P.T, t = c - cc * P.T;  // channel chunk outer, tap inner (L2 reuse)
    const int dy = P.dy[t], dx = P.dx[t];
    const uint32_t toff = (uint32_t)(dy * (int)xsh + dx * (int)xsw + cc * 64 + ac4 * 4);
#pragma unroll
    for (int p = 0; p < APASS; ++p) {
      const int iy = a_iy[p] + dy, ix = a_ix[p] + dx;
      const bool in = (unsigned)iy < (unsigned)d.Hx && (unsigned)ix < (unsigned)d.Wx;
      const float* src = in ? xg + (a_off[p] + toff) : ig_zero_page;
      ra[p] = *(const floatx4v*)src;
    }
    const __bf16* wb = wpb + ((size_t)t * d.Npad + n0 + brow) * d.Cin + cc * 64 + bc8 * 8;
#pragma unroll
    for (int p = 0; p < BPASS; ++p) rb[p] = *(const bf16x8*)(wb + (size_t)(32 * p) * d.Cin);
  };
  auto sstore = [&]() {
#pragma unroll
    for (int p = 0; p < APASS; ++p) {
      bf16x4 v;
      v[0] = (__bf16)ra[p][0]; v[1] = (__bf16)ra[p][1]; v[2] = (__bf16)ra[p][2]; v[3] = (__bf16)ra[p][3];
      *(bf16x4*)&As[(arow + 16 * p) * LDKB + ac4 * 4] = v;
    }
#pragma unroll
    for (int p = 0; p < BPASS; ++p) *(bf16x8*)&Bs[(brow + 32 * p) * LDKB + bc8 * 8] = rb[p];
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

  if (cb < ce) {
    gload(cb);
    sstore();
  }
  __syncthreads();
  const __bf16* Ard = &As[(wm * WM + r) * LDKB + 8 * h];
  const __bf16* Brd = &Bs[(wn * WN + r) * LDKB + 8 * h];
  for (int c = cb; c < ce; ++c) {
    // unconditional with IG_BF16_SGB (the last chunk reloads itself, unused): the
    // loads share the MFMAs' basic block and are spread among them
    if (IG_BF16_SGB) gload(c + 1 < ce ? c + 1 : c);
    else if (c + 1 < ce) gload(c + 1);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      bf16x8 a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = *(const bf16x8*)(Ard + i * 32 * LDKB + 16 * s);
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = *(const bf16x8*)(Brd + j * 32 * LDKB + 16 * s);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if constexpr (IG_BF16_SGB > 0) {
#pragma unroll
      for (int k = 0; k < APASS + BPASS; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);            // VMEM read
        __builtin_amdgcn_sched_group_barrier(0x008, IG_BF16_SGB, 0);  // MFMA
      }
    }
    __syncthreads();
    if (c + 1 < ce) sstore();
    __syncthreads();
  }
  ig_epilogue<TM, TN>(d, P, acc, M, m0, n0, wm, wn, WM, WN, r, h, split);
}

// ------------------------------------------------------------------ fp32 by exact bf16 split
// The fp32 implicit GEMM on the bf16 MFMA: every fp32 operand is split exactly
// into three bf16 terms (split3_bf16), and the six cross products that carry
// the product down to 2^-24 of its size are accumulated in fp32 on
// v_mfma_f32_16x16x32_bf16 (1/16 the cycles of the fp32 MFMA per product, so
// six of them cost 3/8 of v_mfma_f32_32x32x2_f32's time per MAC).
// Activations are read as fp32 and split on their way into LDS; weights
// arrive as three pre-split bf16 planes.  K chunk = 32 channels of one tap
// (Cin % 32 == 0), channel-chunk outer / tap inner as in ig_kernel.
// LDS rows are 64 B (32 bf16 of one K chunk) whose four 16-B chunks are
// XOR-swizzled by row: chunk c of row r sits at c ^ ig_swz(r),
// ig_swz(r) = (0, 2, 3, 1)[(r >> 2) & 3], which keeps the ds_read_b128
// fragment reads (lane (r16, g) holds 8 k of chunk g) on distinct banks in
// every 16-lane group, and the 8/16-lane write groups on distinct dword banks.
// The 16x16x32 shape runs 7-8 % faster than 32x32x16 at equal cycles per MAC:
// the chip holds a higher clock (MI355X_MICROARCH.md, DVFS item 7).
// keep every accumulator register live (and unread-for-reuse) up to here
template <int TM, int TN>
__device__ __forceinline__ void ig_hold(floatx4v (&acc)[TM][TN]) {
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(acc[i][j]));
}

__device__ __forceinline__ int ig_swz(int r) { return (0x78 >> (2 * ((r >> 2) & 3))) & 3; }

template <int TM, int TN>
__device__ __forceinline__ void ig_epilogue16(const IgDesc& d, const IgPhase& P, floatx4v (&acc)[TM][TN], uint32_t M,
                                              uint32_t m0, int n0, int wm, int wn, int WM, int WN, int lane,
                                              int split) {
  // C/D map of the 16x16 MFMA: col = lane & 15, row = 4 * (lane >> 4) + reg
  const int c16 = lane & 15, g = lane >> 4;
  // Stores go out straight from the accumulators, which stay live to the end
  // (ig_hold): overwriting a pending store's data register waits for that
  // store (s_waitcnt vmcnt), which otherwise serialises the epilogue on the
  // store latency, one store at a time.
  if (d.ksplit > 1) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const uint32_t m = m0 + wm * WM + i * 16 + 4 * g + reg;
        if (m >= M) continue;
        float* prow = d.partial + ((size_t)split * d.Mtot + P.m_off + m) * d.Cout;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int n = n0 + wn * WN + j * 16 + c16;
          if (n < d.Cout) prow[n] = acc[i][j][reg];
        }
      }
    ig_hold<TM, TN>(acc);
    return;
  }
  const uint32_t ysc = (uint32_t)d.ys_c;
  if (d.epi == EPI_NONE || d.epi == EPI_RELU) {
    float bj[TN];
    bool nok[TN];
    // the bias loads unconditional (index clamped; columns past Cout are never stored) under one uniform
    // test: a load per lane-dependent condition became a branch and a vmcnt(0) wait each, in series
    const float* __restrict__ bias = d.bias;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * WN + j * 16 + c16;
      nok[j] = n < d.Cout;
      bj[j] = bias ? bias[min(n, d.Cout - 1)] : 0.f;
    }
    const bool relu = d.epi == EPI_RELU;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
          const float v = acc[i][j][reg] + bj[j];
          acc[i][j][reg] = (relu && !(v > 0.f)) ? 0.f : v;
        }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const uint32_t m = m0 + wm * WM + i * 16 + 4 * g + reg;
        if (m >= M) continue;
        float* yo = d.y + ig_out_offset(d, P, m);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          if (nok[j]) yo[(uint32_t)(n0 + wn * WN + j * 16 + c16) * ysc] = acc[i][j][reg];
      }
    ig_hold<TM, TN>(acc);
    return;
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const uint32_t m = m0 + wm * WM + i * 16 + 4 * g + reg;
      if (m >= M) continue;
      const uint32_t ob = ig_out_offset(d, P, m);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn * WN + j * 16 + c16;
        if (n < d.Cout) ig_store_out(d, acc[i][j][reg], ob + (uint32_t)n * ysc, n);
      }
    }
}

// NT = 64 x (BM/WM) x (BN/WN) = 256 threads: 4 waves, two blocks per CU (three
// for 64-row tiles).  NP = 3: the exact split (six products); NP = 1: plain
// bf16 operands (RN of the activations, bf16-packed weights) with fp32
// accumulation, one product (C3 on maps <= 32^2)
template <int BM, int BN, int WM, int WN, int NP = 3>
__global__ void __launch_bounds__(64 * (BM / WM) * (BN / WN), (BM == 64 ? 3 : 2)) ig_kernel_x3s(const IgDesc d) {
  constexpr int LDB = 32;
  constexpr int WAVES_N = BN / WN;
  constexpr int NT = 64 * (BM / WM) * (BN / WN);
  constexpr int APASS = BM * 8 / NT;              // A: 8 float4 per 32-channel row
  constexpr int BSLOT = NP * BN * 4;              // B: 4 x 16 B per 32-wide bf16 row, NP planes
  constexpr int BPASS = (BSLOT + NT - 1) / NT;
  static_assert(BM * 8 % NT == 0, "whole A passes");
  __shared__ __attribute__((aligned(16))) __bf16 As[NP * BM * LDB];
  __shared__ __attribute__((aligned(16))) __bf16 Bs[NP * BN * LDB];

  const int zi = blockIdx.z;
  const int phase = zi / d.ksplit;
  const int split = zi - phase * d.ksplit;
  const IgPhase& P = d.ph[phase];
  uint32_t bx = blockIdx.x;
  if ((gridDim.x & 7) == 0) bx = (bx & 7) * (gridDim.x >> 3) + (bx >> 3);
  if ((int)bx >= P.mtiles) return;

  const uint32_t M = (uint32_t)d.N * P.fd_hw.d;
  const uint32_t m0 = bx * BM;
  const int n0 = blockIdx.y * BN;
  const int nchunks = P.T * (d.Cin >> 5);
  const int cb = split * d.kcps;
  const int ce = min(nchunks, cb + d.kcps);

  const int tid = threadIdx.x;
  const int lrow = tid >> 3, lc4 = tid & 7;   // A: 8 float4 per 32-channel row
  const uint32_t xsh = (uint32_t)d.xs_h, xsw = (uint32_t)d.xs_w;
  uint32_t a_off[APASS];
  int a_iy[APASS], a_ix[APASS];
#pragma unroll
  for (int p = 0; p < APASS; ++p) {
    const uint32_t m = m0 + lrow + (NT / 8) * p;
    const bool ok = m < M;
    const uint32_t mm = ok ? m : 0u;
    const uint32_t img = fdiv(mm, P.fd_hw);
    const uint32_t rem = mm - img * (uint32_t)P.fd_hw.d;
    const uint32_t gy = fdiv(rem, P.fd_w);
    const uint32_t gx = rem - gy * (uint32_t)P.Wg;
    a_iy[p] = ok ? (int)gy * d.stride : -0x40000000;
    a_ix[p] = (int)gx * d.stride;
    a_off[p] = img * (uint32_t)d.xs_n + (uint32_t)a_iy[p] * xsh + (uint32_t)a_ix[p] * xsw;
  }
  const float* __restrict__ xg = d.x;
  const __bf16* __restrict__ wpb = (const __bf16*)P.wp;
  const size_t wplane = (size_t)d.wplane;
  // swizzled store offsets (rows lrow + (NT/8) p keep bits 2..3 of the row)
  const int a_st = lrow * LDB + 8 * ((lc4 >> 1) ^ ig_swz(lrow)) + 4 * (lc4 & 1);
  // B: thread (brow, bq) stages 16-B chunk bq of (plane, row) pairs R = brow + (NT/4) p,
  // plane R / BN, row R % BN; NT/4 is a multiple of 64, so every such row keeps
  // bits 2..3 of brow and one swizzle serves all passes
  const int brow = tid >> 2, bq = tid & 3;
  const int b_sw = 8 * (bq ^ ig_swz(brow));
  auto b_plane = [&](int p, int& q, int& row) {
    if constexpr (NT == 256 && BN % 64 == 0) {  // compile-time plane / row block
      q = p / (BN / 64);
      row = brow + 64 * (p - q * (BN / 64));
    } else {
      const int R = brow + (NT / 4) * p;
      q = R / BN;
      row = R - q * BN;
    }
  };

  floatx4v ra[APASS];
  bf16x8 rb[BPASS];
  auto gload = [&](int c) {
    const int cc = c / P.T, t = c - cc * P.T;
    const int dy = P.dy[t], dx = P.dx[t];
    const uint32_t toff = (uint32_t)(dy * (int)xsh + dx * (int)xsw + cc * 32 + lc4 * 4);
#pragma unroll
    for (int p = 0; p < APASS; ++p) {
      const int iy = a_iy[p] + dy, ix = a_ix[p] + dx;
      const bool in = (unsigned)iy < (unsigned)d.Hx && (unsigned)ix < (unsigned)d.Wx;
      const float* src = in ? xg + (a_off[p] + toff) : ig_zero_page;
      ra[p] = *(const floatx4v*)src;
    }
    const __bf16* wb = wpb + (size_t)t * d.Npad * d.Cin + cc * 32 + bq * 8;
#pragma unroll
    for (int p = 0; p < BPASS; ++p) {
      int q, row;
      b_plane(p, q, row);
      if (BSLOT % NT == 0 || q < NP) rb[p] = *(const bf16x8*)(wb + q * wplane + (size_t)(n0 + row) * d.Cin);
    }
  };
  const bool sq = d.a_op == AOP_SQUARE;  // GDN's x^2 (uniform)
  auto sstore = [&]() {
#pragma unroll
    for (int p = 0; p < APASS; ++p) {
      if constexpr (NP == 1) {
        bf16x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = (__bf16)ra[p][e];
        *(bf16x4*)&As[a_st + (NT / 8) * p * LDB] = v;
        continue;
      }
      bf16x4 vh, vm, vl;
      if (IG_SPLIT_PK) {
        split3_bf16x4(sq ? ra[p] * ra[p] : ra[p], vh, vm, vl);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          __bf16 h, m, l;
          split3_bf16(sq ? ra[p][e] * ra[p][e] : ra[p][e], h, m, l);
          vh[e] = h; vm[e] = m; vl[e] = l;
        }
      }
      __bf16* dst = &As[a_st + (NT / 8) * p * LDB];
      *(bf16x4*)dst = vh;
      *(bf16x4*)(dst + BM * LDB) = vm;
      *(bf16x4*)(dst + 2 * BM * LDB) = vl;
    }
#pragma unroll
    for (int p = 0; p < BPASS; ++p) {
      int q, row;
      b_plane(p, q, row);
      if (BSLOT % NT == 0 || q < NP) *(bf16x8*)&Bs[(q * BN + row) * LDB + b_sw] = rb[p];
    }
  };

  const int lane = tid & 63, w = tid >> 6;
  const int wm = w / WAVES_N, wn = w - (w / WAVES_N) * WAVES_N;

  constexpr int TM = WM / 16, TN = WN / 16;
  const int r = lane & 15, g = lane >> 4;
  floatx4v acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = floatx4v{0.f, 0.f, 0.f, 0.f};
  if (cb < ce) {
    gload(cb);
    sstore();
  }
  __syncthreads();
  const int ch = 8 * (g ^ ig_swz(r));
  const __bf16* Ard = &As[(wm * WM + r) * LDB + ch];
  const __bf16* Brd = &Bs[(wn * WN + r) * LDB + ch];
  for (int c = cb; c < ce; ++c) {
    // unconditional (the last chunk reloads itself, unused): the loads then share
    // the MFMAs' basic block and can be spread among them (IG_X3_SGB)
    if (IG_X3_SGB) gload(c + 1 < ce ? c + 1 : c);
    else if (c + 1 < ce) gload(c + 1);
    bf16x8 a[NP][TM];
#pragma unroll
    for (int q = 0; q < NP; ++q)
#pragma unroll
      for (int i = 0; i < TM; ++i) a[q][i] = *(const bf16x8*)(Ard + (q * BM + i * 16) * LDB);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      bf16x8 b[NP];
#pragma unroll
      for (int q = 0; q < NP; ++q) b[q] = *(const bf16x8*)(Brd + (q * BN + j * 16) * LDB);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        if constexpr (NP == 1) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[0], acc[i][j], 0, 0, 0);
          continue;
        }
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2][i], b[0], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][i], b[1], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[2], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][i], b[0], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[1], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[0], acc[i][j], 0, 0, 0);
      }
    }
    if constexpr (IG_X3_SGB && (NP == 3 || IG_BF16_SGB)) {
      // one global load per IG_X3_SGB MFMAs (bf16, NP = 1: per IG_BF16_SGB)
#pragma unroll
      for (int k = 0; k < APASS + BPASS; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);         // VMEM read
        __builtin_amdgcn_sched_group_barrier(0x008, NP == 3 ? IG_X3_SGB : IG_BF16_SGB, 0);  // MFMA
      }
    }
    __syncthreads();
    if (c + 1 < ce) sstore();
    __syncthreads();
  }
  ig_epilogue16<TM, TN>(d, P, acc, M, m0, n0, wm, wn, WM, WN, lane, split);
}

// ------------------------------------------------------------------ split, every operand by LDS-DMA
// The split implicit GEMM on 256 x 192 tiles, eight waves of 32 x 192, one block per CU, with
// no register staging: per K chunk (32 channels of one tap) the block's 256 gathered fp32
// activation rows (32 KB) and the three pre-split weight planes (36 KB) arrive by LDS-DMA
// (global_load_lds_dwordx4 from inline asm, so the compiler does not wait for the DMA before
// LDS reads) into one of two stages; one barrier per chunk publishes chunk c and frees the
// stage that chunk c + 1's DMA, issued right after it, overwrites.  Each wave splits its own A
// fragments into three bf16 terms after reading them (8 fp32 per lane per 16-row tile) — the 32
// rows it DMAs, each split by one wave (64 x 96 wave tiles split every row in two waves: 2.6 %
// slower on the big layers, 1.4 % per C2 step, r03zw) — and runs
// ig_kernel_x3s's six products per (i, j) in the same order over the same chunk order, so the
// result is bitwise that kernel's.  Per chunk a 256-row tile stages the weights once for twice
// the rows of ig_kernel_x3s<128, ...> (68 vs 104 KB per 256 rows), and no VALU or ds_write
// staging sits between the MFMA phases.
// fp32 A rows are 128 B (eight 16-B chunks) with the chunks XOR-swizzled by row bits 1 and 3
// (ig_swa): the four 16-lane groups of a ds_read_b128 fragment read hit distinct bank slots.
#ifndef IG_X3D
#define IG_X3D 1
#endif
#ifndef IG_X3D_WM
#define IG_X3D_WM 32  // rows per wave: 32 x 192 wave tiles (64: 64 x 96, each A row split by two waves)
#endif
#ifndef IG_X3D_DMA_AT
#define IG_X3D_DMA_AT 2  // where the next chunk's DMA issues: 0 after the A split, 1 before it, 2 among the MFMAs
#endif
#ifndef IG_X3D_DMA_J
#define IG_X3D_DMA_J 4  // DMA_AT 2: before n-tile j's MFMAs (r03zx-r03zy: j = 4 of 12, 1.7-2.7 % per C2 step over 0)
#endif
#ifndef IG_X3D_MINT
#define IG_X3D_MINT 32  // smaller grids: 256-row tiles with K split to fill the chip (>= this many tiles)
#endif

// 16 B per lane, global -> LDS at byte offset lds + 16 * lane (wave-uniform lds; M0 restored)
__device__ __forceinline__ void ig_glds16(const void* src, uint32_t lds) {
  uint32_t save;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(save)
      : "v"(src), "s"(lds)
      : "memory");
}

__device__ __forceinline__ int ig_swa(int r) { return ((r >> 1) & 1) | (((r >> 3) & 1) << 2); }

__global__ void __launch_bounds__(512, 1) ig_kernel_x3d(const IgDesc d) {
  constexpr int BM = 256, BN = 192, WM = IG_X3D_WM, WN = BM * BN / 8 / WM, LDB = 32;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int ASTAGE = BM * 32 * 4;       // bytes of the fp32 A image (32 KB)
  constexpr int BSTAGE = 3 * BN * LDB * 2;  // bytes of the three bf16 B planes (36 KB)
  constexpr int STAGE = ASTAGE + BSTAGE;
  constexpr int NB = 3 * BN / 16;           // 1-KB B DMA pieces per stage (36)
  __shared__ __attribute__((aligned(16))) char lds[2 * STAGE];

  const int zi = blockIdx.z;
  const int phase = zi / d.ksplit;
  const int split = zi - phase * d.ksplit;
  const IgPhase& P = d.ph[phase];
  uint32_t bx = blockIdx.x;
  if ((gridDim.x & 7) == 0) bx = (bx & 7) * (gridDim.x >> 3) + (bx >> 3);
  if ((int)bx >= P.mtiles) return;
  const uint32_t M = (uint32_t)d.N * P.fd_hw.d;
  const uint32_t m0 = bx * BM;
  const int T = P.T;
  const int nchunks = T * (d.Cin >> 5);
  // split K: chunks [cb, ce) of this block's split (a split past the phase's chunks adds zeros)
  const int cb = split * d.kcps;
  const int ce = min(nchunks, cb + d.kcps);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t lbase = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)lds);

  // A: wave w DMAs rows 32w + 8k + (lane >> 3), k < 4 (1 KB = 8 rows per piece); lane's
  // physical chunk lane & 7 holds logical chunk (lane & 7) ^ ig_swa(row)
  const uint32_t xsh = (uint32_t)d.xs_h, xsw = (uint32_t)d.xs_w;
  uint32_t a_off[4];
  int a_iy[4], a_ix[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int row = 32 * w + 8 * k + (lane >> 3);
    const uint32_t m = m0 + row;
    const bool ok = m < M;
    const uint32_t mm = ok ? m : 0u;
    const uint32_t img = fdiv(mm, P.fd_hw);
    const uint32_t rem = mm - img * (uint32_t)P.fd_hw.d;
    const uint32_t gy = fdiv(rem, P.fd_w);
    const uint32_t gx = rem - gy * (uint32_t)P.Wg;
    a_iy[k] = ok ? (int)gy * d.stride : -0x40000000;
    a_ix[k] = (int)gx * d.stride;
    a_off[k] = img * (uint32_t)d.xs_n + (uint32_t)a_iy[k] * xsh + (uint32_t)a_ix[k] * xsw +
               4u * (uint32_t)((lane & 7) ^ ig_swa(row & 15));
  }
  // B: wave w DMAs pieces jj = w + 8 kb < 36: plane jj / 12, rows 16 (jj % 12) + (lane >> 2);
  // lane's physical chunk lane & 3 holds logical chunk (lane & 3) ^ ig_swz(row)
  const __bf16* __restrict__ wpb = (const __bf16*)P.wp;
  uint32_t b_off[5];
#pragma unroll
  for (int kb = 0; kb < 5; ++kb) {
    const int jj = w + 8 * kb;
    const int q = jj / 12, rb = 16 * (jj - 12 * q) + (lane >> 2);
    b_off[kb] = (uint32_t)q * (uint32_t)d.wplane + (uint32_t)rb * (uint32_t)d.Cin +
                8u * (uint32_t)((lane & 3) ^ ig_swz(rb));
  }
  const float* __restrict__ xg = d.x;
  auto issue = [&](int cc, int t, int st) {
    const uint32_t sb = lbase + (uint32_t)(st * STAGE);
    const int dy = P.dy[t], dx = P.dx[t];
    const uint32_t toff = (uint32_t)(dy * (int)xsh + dx * (int)xsw + cc * 32);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int iy = a_iy[k] + dy, ix = a_ix[k] + dx;
      const bool in = (unsigned)iy < (unsigned)d.Hx && (unsigned)ix < (unsigned)d.Wx;
      ig_glds16(in ? (const void*)(xg + (a_off[k] + toff)) : (const void*)ig_zero_page,
                sb + (uint32_t)((4 * w + k) * 1024));
    }
    const uint32_t boff = (uint32_t)(t * d.Npad * d.Cin + cc * 32);
#pragma unroll
    for (int kb = 0; kb < 5; ++kb) {
      if (w + 8 * kb < NB) ig_glds16(wpb + (b_off[kb] + boff), sb + (uint32_t)(ASTAGE + (w + 8 * kb) * 1024));
    }
  };

  const int wm = w / (BN / WN), wn = w % (BN / WN);
  int cn = cb / T, tn = cb - (cb / T) * T;  // channel chunk and tap of the next chunk to issue
  if (cb < ce) {
    issue(cn, tn, 0);
    if (++tn == T) { tn = 0; ++cn; }
  }
  const int r = lane & 15, g = lane >> 4;
  const int ach0 = ((2 * g) ^ ig_swa(r)) << 2, ach1 = ((2 * g + 1) ^ ig_swa(r)) << 2;
  const int bch = 8 * (g ^ ig_swz(r));
  floatx4v acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = floatx4v{0.f, 0.f, 0.f, 0.f};

  for (int c = cb; c < ce; ++c) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const float* As = (const float*)(lds + ((c - cb) & 1) * STAGE);
    const __bf16* Bs = (const __bf16*)(lds + ((c - cb) & 1) * STAGE + ASTAGE);
    if (IG_X3D_DMA_AT == 1 && c + 1 < ce) {
      issue(cn, tn, (c + 1 - cb) & 1);
      if (++tn == T) { tn = 0; ++cn; }
    }
    bf16x8 a[3][TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const float* ar = As + (wm * WM + i * 16 + r) * 32;
      const floatx4v lo = *(const floatx4v*)(ar + ach0);
      const floatx4v hi = *(const floatx4v*)(ar + ach1);
      bf16x4 h0, m0v, l0, h1, m1v, l1;
      split3_bf16x4(lo, h0, m0v, l0);
      split3_bf16x4(hi, h1, m1v, l1);
      a[0][i] = __builtin_shufflevector(h0, h1, 0, 1, 2, 3, 4, 5, 6, 7);
      a[1][i] = __builtin_shufflevector(m0v, m1v, 0, 1, 2, 3, 4, 5, 6, 7);
      a[2][i] = __builtin_shufflevector(l0, l1, 0, 1, 2, 3, 4, 5, 6, 7);
    }
    // the next chunk's DMA, between the split (VALU) and the MFMAs (r03p: 1 % faster than before the split)
    if (IG_X3D_DMA_AT == 0 && c + 1 < ce) {
      issue(cn, tn, (c + 1 - cb) & 1);
      if (++tn == T) { tn = 0; ++cn; }
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      if (IG_X3D_DMA_AT == 2 && j == IG_X3D_DMA_J && c + 1 < ce) {
        issue(cn, tn, (c + 1 - cb) & 1);
        if (++tn == T) { tn = 0; ++cn; }
      }
      bf16x8 b[3];
#pragma unroll
      for (int q = 0; q < 3; ++q) b[q] = *(const bf16x8*)(Bs + (q * BN + wn * WN + j * 16 + r) * LDB + bch);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2][i], b[0], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][i], b[1], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[2], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][i], b[0], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[1], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[0], acc[i][j], 0, 0, 0);
      }
    }
  }
  ig_epilogue16<TM, TN>(d, P, acc, M, m0, 0, wm, wn, WM, WN, lane, split);
}

// bf16 operands on 256 x 192 DMA tiles (C3, round 5): ig_kernel_x3d's block, waves, DMA pipeline and
// epilogue with both operands already bf16 in HBM -- the activations as a compact NHWC bf16 copy (d.xb)
// and one packed bf16 weight plane -- so nothing is converted or staged through registers.  K chunks of
// 64 channels of one tap: 128-B rows for both operands (A 32 KB + B 24 KB per stage, two stages), the
// 16-B pieces XOR-swizzled by row bits 1-3 (ig_swb: conflict-free ds_read_b128 fragments), two K steps
// of v_mfma_f32_16x16x32_bf16 per chunk.  Round 3 ran bf16 products on ig_kernel_x3d's fp32-A DMA tiles
// and was slower than ig_kernel_bf16 (the fp32 A bytes per MAC were six times the split kernel's).
#ifndef IG_B16D
#define IG_B16D 1
#endif
#ifndef IG_B16D_DMA_J
#define IG_B16D_DMA_J 4  // the next chunk's DMA issues before column tile j's MFMAs (as ig_kernel_x3d)
#endif
__device__ __forceinline__ int ig_swb(int r) { return (r >> 1) & 7; }

__global__ void __launch_bounds__(512, 1) ig_kernel_b16d(const IgDesc d) {
  constexpr int BM = 256, BN = 192, WM = 32, WN = 192, TM = WM / 16, TN = WN / 16;
  constexpr int ASTAGE = BM * 128;  // 32 KB: 256 rows x 64 bf16
  constexpr int BSTAGE = BN * 128;  // 24 KB: 192 rows x 64 bf16
  constexpr int STAGE = ASTAGE + BSTAGE;
  constexpr int NB = BN / 8;        // 1-KB B pieces per stage (24)
  __shared__ __attribute__((aligned(16))) char lds[2 * STAGE];

  const int zi = blockIdx.z;
  const int phase = zi / d.ksplit;
  const int split = zi - phase * d.ksplit;
  const IgPhase& P = d.ph[phase];
  uint32_t bx = blockIdx.x;
  if ((gridDim.x & 7) == 0) bx = (bx & 7) * (gridDim.x >> 3) + (bx >> 3);
  if ((int)bx >= P.mtiles) return;
  const uint32_t M = (uint32_t)d.N * P.fd_hw.d;
  const uint32_t m0 = bx * BM;
  const int T = P.T;
  const int nchunks = T * (d.Cin >> 6);
  const int cb = split * d.kcps;
  const int ce = min(nchunks, cb + d.kcps);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t lbase = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)lds);

  // A: wave w DMAs rows 32w + 8k + (lane >> 3), k < 4; lane's physical piece lane & 7 holds logical
  // piece (lane & 7) ^ ig_swb(row) (offsets in bf16 elements)
  const uint32_t xsh = (uint32_t)d.xs_h, xsw = (uint32_t)d.xs_w;
  uint32_t a_off[4];
  int a_iy[4], a_ix[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int row = 32 * w + 8 * k + (lane >> 3);
    const uint32_t m = m0 + row;
    const bool ok = m < M;
    const uint32_t mm = ok ? m : 0u;
    const uint32_t img = fdiv(mm, P.fd_hw);
    const uint32_t rem = mm - img * (uint32_t)P.fd_hw.d;
    const uint32_t gy = fdiv(rem, P.fd_w);
    const uint32_t gx = rem - gy * (uint32_t)P.Wg;
    a_iy[k] = ok ? (int)gy * d.stride : -0x40000000;
    a_ix[k] = (int)gx * d.stride;
    a_off[k] = img * (uint32_t)d.xs_n + (uint32_t)a_iy[k] * xsh + (uint32_t)a_ix[k] * xsw +
               8u * (uint32_t)((lane & 7) ^ ig_swb(row & 15));
  }
  // B: wave w DMAs pieces jj = w + 8 kb < 24: rows 8 jj + (lane >> 3)
  const __bf16* __restrict__ wpb = (const __bf16*)P.wp;
  uint32_t b_off[3];
#pragma unroll
  for (int kb = 0; kb < 3; ++kb) {
    const int rb = 8 * (w + 8 * kb) + (lane >> 3);
    b_off[kb] = (uint32_t)rb * (uint32_t)d.Cin + 8u * (uint32_t)((lane & 7) ^ ig_swb(rb & 15));
  }
  const __bf16* __restrict__ xg = (const __bf16*)d.xb;
  auto issue = [&](int cc, int t, int st) {
    const uint32_t sb = lbase + (uint32_t)(st * STAGE);
    const int dy = P.dy[t], dx = P.dx[t];
    const uint32_t toff = (uint32_t)(dy * (int)xsh + dx * (int)xsw + cc * 64);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int iy = a_iy[k] + dy, ix = a_ix[k] + dx;
      const bool in = (unsigned)iy < (unsigned)d.Hx && (unsigned)ix < (unsigned)d.Wx;
      ig_glds16(in ? (const void*)(xg + (a_off[k] + toff)) : (const void*)ig_zero_page,
                sb + (uint32_t)((4 * w + k) * 1024));
    }
    const uint32_t boff = (uint32_t)(t * d.Npad * d.Cin + cc * 64);
#pragma unroll
    for (int kb = 0; kb < 3; ++kb) ig_glds16(wpb + (b_off[kb] + boff), sb + (uint32_t)(ASTAGE + (w + 8 * kb) * 1024));
  };
  static_assert(NB == 24, "three B pieces per wave");

  const int wm = w, wn = 0;
  const int r = lane & 15, g = lane >> 4;
  const int ch0 = 16 * ((g) ^ ig_swb(r)), ch1 = 16 * ((4 + g) ^ ig_swb(r));  // byte offsets of K steps 0, 1
  floatx4v acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = floatx4v{0.f, 0.f, 0.f, 0.f};

  const int CC = d.Cin >> 6;
  int cn = cb / T, tn = cb - (cb / T) * T;  // channel chunk and tap of the next chunk to issue
  if (cb < ce) {
    issue(cn, tn, 0);
    if (++tn == T) { tn = 0; ++cn; }
  }
  (void)CC;
  for (int c = cb; c < ce; ++c) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const char* As = lds + ((c - cb) & 1) * STAGE;
    const char* Bs = As + ASTAGE;
    bf16x8 a[2][TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const char* ar = As + (wm * WM + i * 16 + r) * 128;
      a[0][i] = *(const bf16x8*)(ar + ch0);
      a[1][i] = *(const bf16x8*)(ar + ch1);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      if (j == IG_B16D_DMA_J && c + 1 < ce) {
        issue(cn, tn, (c + 1 - cb) & 1);
        if (++tn == T) { tn = 0; ++cn; }
      }
      const char* br = Bs + (wn * WN + j * 16 + r) * 128;
      const bf16x8 b0 = *(const bf16x8*)(br + ch0);
      const bf16x8 b1 = *(const bf16x8*)(br + ch1);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b0, acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][i], b1, acc[i][j], 0, 0, 0);
      }
    }
  }
  ig_epilogue16<TM, TN>(d, P, acc, M, m0, 0, wm, wn, WM, WN, lane, split);
}

__global__ void __launch_bounds__(256) ig_cvt_bf16_kernel(const float* __restrict__ x, __bf16* __restrict__ xb,
                                                          long long n8) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long long)gridDim.x * blockDim.x) {
    const floatx4v lo = *(const floatx4v*)(x + 8 * i), hi = *(const floatx4v*)(x + 8 * i + 4);
    *(u32x4*)(xb + 8 * i) = u32x4{ic_cvt_pk_bf16(lo[0], lo[1]), ic_cvt_pk_bf16(lo[2], lo[3]),
                                  ic_cvt_pk_bf16(hi[0], hi[1]), ic_cvt_pk_bf16(hi[2], hi[3])};
  }
}

// split-K reduction + epilogue: one thread per (row, channel)
__global__ void ig_reduce_kernel(const IgDesc d) {
  const long long total = d.Mtot * d.Cout;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long mg = i / d.Cout;
    const int n = (int)(i - mg * d.Cout);
    // eight independent loads in flight (a serial chain waits one memory
    // latency per split); fixed order, so the sum is deterministic
    const float* src = d.partial + i;
    const long long ss = d.Mtot * d.Cout;
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int s = 0;
    for (; s + 7 < d.ksplit; s += 8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += src[(s + j) * ss];
    }
    for (int j = 0; s < d.ksplit; ++s, ++j) a[j] += src[s * ss];
    const float v = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
    int ph = 0;
#pragma unroll
    for (int q = 1; q < IC_MAXPH; ++q)
      if (q < d.nphase && mg >= d.ph[q].m_off) ph = q;
    const IgPhase& P = d.ph[ph];
    const uint32_t m = (uint32_t)(mg - P.m_off);
    ig_store_out(d, v, ig_out_offset(d, P, m) + (uint32_t)n * (uint32_t)d.ys_c, n);
  }
}

#ifndef IG_REDUCE4
#define IG_REDUCE4 1
#endif
// the same reduction on float4 columns (Cout % 4 == 0): four channels per thread, the splits summed per
// channel in ig_reduce_kernel's order (split s into accumulator s & 7, then the fixed tree), so the result
// is bitwise the same; KS > 0: the split count at compile time (every load issued before the first add)
template <int KS>
__global__ void __launch_bounds__(256) ig_reduce4_kernel(const IgDesc d) {
  const int ks = KS ? KS : d.ksplit;
  const int c4n = d.Cout >> 2;
  const long long total4 = d.Mtot * c4n;
  const floatx4v* __restrict__ part = (const floatx4v*)d.partial;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total4;
       i += (long long)gridDim.x * blockDim.x) {
    floatx4v a[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = floatx4v{0.f, 0.f, 0.f, 0.f};
    if constexpr (KS > 0) {
      floatx4v v[KS];
#pragma unroll
      for (int s = 0; s < KS; ++s) v[s] = part[i + s * total4];
#pragma unroll
      for (int s = 0; s < KS; ++s) a[s & 7] += v[s];
    } else {
      int s = 0;
      for (; s + 7 < ks; s += 8) {
        floatx4v v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = part[i + (s + j) * total4];
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] += v[j];
      }
      // the rest (< 8, a uniform count): clamped loads, each added only where it exists
      floatx4v v[7];
#pragma unroll
      for (int j = 0; j < 7; ++j) v[j] = part[i + min(s + j, ks - 1) * total4];
#pragma unroll
      for (int j = 0; j < 7; ++j)
        if (s + j < ks) a[j] += v[j];
    }
    const floatx4v v = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
    const long long mg = i / c4n;
    const int n = (int)(i - mg * c4n) * 4;
    int ph = 0;
#pragma unroll
    for (int q = 1; q < IC_MAXPH; ++q)
      if (q < d.nphase && mg >= d.ph[q].m_off) ph = q;
    const IgPhase& P = d.ph[ph];
    const uint32_t m = (uint32_t)(mg - P.m_off);
    const uint32_t ob = ig_out_offset(d, P, m) + (uint32_t)n * (uint32_t)d.ys_c;
    if ((d.epi == EPI_NONE || d.epi == EPI_RELU) && d.ys_c == 1 && ((uintptr_t)(d.y + ob) & 15) == 0 &&
        ((uintptr_t)d.bias & 15) == 0) {
      floatx4v o = v;
      if (d.bias) o += *(const floatx4v*)(d.bias + n);
      if (d.epi == EPI_RELU)
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = o[e] > 0.f ? o[e] : 0.f;
      *(floatx4v*)(d.y + ob) = o;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) ig_store_out(d, v[e], ob + (uint32_t)e * (uint32_t)d.ys_c, n + e);
    }
  }
}

template <int BM, int BN, int WM, int WN>
int ig_launch_t(const IgDesc& d, hipStream_t s) {
  int mt = 0;
  for (int p = 0; p < d.nphase; ++p) mt = mt > d.ph[p].mtiles ? mt : d.ph[p].mtiles;
  dim3 grid(mt, d.Npad / BN, d.nphase * d.ksplit);
  const bool sq = d.a_op == AOP_SQUARE;
  switch (ig_kernel_kind(d)) {
    case IC_KERNEL_IG_SPLIT_BF16:
      if constexpr (BN % 64 == 0 && (BM == 64 || (IG_BF16_NARROW && BM == 128))) {
        if (sq) return IC_ERR_ARG;
        hipLaunchKernelGGL((ig_kernel_x3s<BM, BN, WM, WN, 1>), grid, dim3(256), 0, s, d);
        break;
      }
      return IC_ERR_ARG;
    case IC_KERNEL_IG_BF16:
      if constexpr (BM != 64) {
        if (sq) return IC_ERR_ARG;
        hipLaunchKernelGGL((ig_kernel_bf16<BM, BN, WM, WN>), grid, dim3(256), 0, s, d);
        break;
      }
      return IC_ERR_ARG;
    case IC_KERNEL_IG_SPLIT:
      if constexpr (BN % 64 == 0) {
        hipLaunchKernelGGL((ig_kernel_x3s<BM, BN, WM, WN>), grid, dim3(64 * (BM / WM) * (BN / WN)), 0, s, d);
        break;
      }
      return IC_ERR_ARG;
    case IC_KERNEL_IG_FP32_GATHER:
      if (sq) hipLaunchKernelGGL((ig_kernel<BM, BN, WM, WN, true, true>), grid, dim3(256), 0, s, d);
      else hipLaunchKernelGGL((ig_kernel<BM, BN, WM, WN, true, false>), grid, dim3(256), 0, s, d);
      break;
    default:
      if (sq) hipLaunchKernelGGL((ig_kernel<BM, BN, WM, WN, false, true>), grid, dim3(256), 0, s, d);
      else hipLaunchKernelGGL((ig_kernel<BM, BN, WM, WN, false, false>), grid, dim3(256), 0, s, d);
  }
  IC_CHECK_LAUNCH();
  return IC_OK;
}

}  // namespace

// bf16 operands on the padded 64-channel-chunk kernel (ig_kernel_bf16) rather
// than the swizzled 32-channel one (ig_kernel_x3s<..., 1>)
static bool ig_bf16_wide(const IgDesc& d) {
  return d.bf16 && !(IG_BF16_S && d.bn % 64 == 0 && (d.bm == 64 || (IG_BF16_NARROW && d.bm == 128)));
}

int ig_npad(int Cout) {
  if (Cout % 192 == 0) return Cout;
  if (Cout >= 64) return (Cout + 63) / 64 * 64;
  return (Cout + 31) / 32 * 32;
}

#ifndef IG_KSPLIT_MAX
#define IG_KSPLIT_MAX 32  // more splits cost more in the partial-sum pass than they save
#endif

size_t ig_plan(IgDesc& d) {
  long long mall = 0;
  for (int p = 0; p < d.nphase; ++p) mall += (long long)d.N * d.ph[p].Hg * d.ph[p].Wg;
  if (d.Cout % 192 == 0) {
    // small maps (hyperprior and <= 32x32 at batch 32): 64-row tiles double the tile
    // grid, so fewer K splits (and less split-K partial traffic) fill the chip
    d.bm = ((!d.bf16 || IG_BF16_S) && mall < 65536) ? 64 : 128;
    d.bn = 192;
    // big split maps: 256-row tiles on the all-DMA kernel (one block per CU) where they fill the chip
    d.dma = 0;
    if (IG_X3D && d.x3 && !d.bf16 && !d.generic && d.Cout == 192 && d.a_op == AOP_NONE && d.xs_c == 1 &&
        d.Cin % 32 == 0) {
      long long t256 = 0;
      for (int p = 0; p < d.nphase; ++p) t256 += ic_cdiv((long long)d.N * d.ph[p].Hg * d.ph[p].Wg, 256);
      // K split (below 256 tiles) only for one-phase maps: the phases of a transposed conv have
      // 9 / 6 / 6 / 4 taps, so equal chunk ranges leave one block per CU waiting on the longest
      if (t256 >= 256 || (d.nphase == 1 && t256 >= IG_X3D_MINT)) { d.bm = 256; d.dma = 1; }
    }
    // bf16 operands on one-phase maps: the DMA tiles (ig_kernel_b16d) on a compact NHWC input
    if (IG_B16D && d.b16d_ok && d.bf16 && !d.generic && d.Cout == 192 && d.a_op == AOP_NONE && d.xs_c == 1 &&
        d.Cin % 64 == 0 && d.xs_w == d.Cin && d.xs_h == (long long)d.Wx * d.Cin &&
        d.xs_n == (long long)d.Hx * d.Wx * d.Cin) {
      long long t256 = 0;
      for (int p = 0; p < d.nphase; ++p) t256 += ic_cdiv((long long)d.N * d.ph[p].Hg * d.ph[p].Wg, 256);
      // as ig_kernel_x3d: K split only for one-phase maps (a transposed conv's phases have unequal taps)
      if (t256 >= 256 || (d.nphase == 1 && t256 >= IG_X3D_MINT)) { d.bm = 256; d.dma = 1; }
    }
  }
  else if (d.Cout >= 64) { d.bm = 128; d.bn = 64; }
  else { d.bm = 256; d.bn = 32; }
  if (d.bn % 64 != 0) d.x3 = 0;  // the split kernel stages B 64 rows per pass; native fp32 instead
  d.Npad = ig_npad(d.Cout);
  long long mtot = 0;
  long long tiles = 0;
  int nchunks_max = 0;
  for (int p = 0; p < d.nphase; ++p) {
    IgPhase& P = d.ph[p];
    const long long M = (long long)d.N * P.Hg * P.Wg;
    P.mtiles = ic_cdiv(M, d.bm);
    P.fd_hw = make_fastdiv((uint32_t)((long long)P.Hg * P.Wg));
    P.fd_w = make_fastdiv((uint32_t)P.Wg);
    P.m_off = mtot;
    mtot += M;
    tiles += (long long)P.mtiles * (d.Npad / d.bn);
    const int nch = d.generic ? (d.Kc >> 5)
                  : P.T * (ig_bf16_wide(d) ? (d.Cin >> 6) : (d.Cin >> 5));
    nchunks_max = nch > nchunks_max ? nch : nchunks_max;
  }
  d.Mtot = mtot;
  // split K when the tile grid cannot fill 256 CUs x 2 blocks
  int ksplit = 1;
  if (d.dma && tiles < 256 && nchunks_max >= 4) {  // one block per CU
    ksplit = (int)((256 + tiles - 1) / tiles);
    int maxs = nchunks_max / 2;
    if (maxs > IG_KSPLIT_MAX) maxs = IG_KSPLIT_MAX;
    if (ksplit > maxs) ksplit = maxs;
    if (ksplit < 1) ksplit = 1;
  } else if (!d.dma && tiles < 512 && nchunks_max >= 4) {
    ksplit = (int)((1024 + tiles - 1) / tiles);
    int maxs = nchunks_max / 2;
    if (maxs > IG_KSPLIT_MAX) maxs = IG_KSPLIT_MAX;
    if (ksplit > maxs) ksplit = maxs;
    if (ksplit < 1) ksplit = 1;
  }
  d.kcps = (nchunks_max + ksplit - 1) / ksplit;
  d.ksplit = (nchunks_max + d.kcps - 1) / d.kcps;
  if (d.ksplit <= 1) {
    d.ksplit = 1;
    d.kcps = nchunks_max;
    return 0;
  }
  return (size_t)d.ksplit * (size_t)mtot * (size_t)d.Cout * sizeof(float);
}

int ig_kernel_kind(const IgDesc& d) {
  if (d.bf16) return d.dma ? IC_KERNEL_IG_BF16_DMA : ig_bf16_wide(d) ? IC_KERNEL_IG_BF16 : IC_KERNEL_IG_SPLIT_BF16;
  if (d.x3) return d.dma ? IC_KERNEL_IG_SPLIT_DMA : IC_KERNEL_IG_SPLIT;
  return d.generic ? IC_KERNEL_IG_FP32_GATHER : IC_KERNEL_IG_FP32;
}

long long ig_grid_blocks(const IgDesc& d) {
  int mt = 0;
  for (int p = 0; p < d.nphase; ++p) mt = mt > d.ph[p].mtiles ? mt : d.ph[p].mtiles;
  return (long long)mt * (d.Npad / d.bn) * d.nphase * d.ksplit;
}

int ig_run(IgDesc& d, hipStream_t s) {
  if (d.Mtot == 0) return IC_OK;
  if (!d.generic && (d.Cin % 32 != 0 || d.xs_c != 1)) return IC_ERR_ARG;
  if (d.bf16 && (d.generic || (ig_bf16_wide(d) && d.Cin % 64 != 0))) return IC_ERR_ARG;
  if (d.x3 && (d.generic || d.bf16 || d.Cin % 32 != 0 || d.a_op == AOP_ABS || d.bn % 64 != 0)) return IC_ERR_ARG;
  if (d.generic && (d.Kc % 32 != 0)) return IC_ERR_ARG;
  int rc;
  if (d.dma) {
    int mt = 0;
    for (int p = 0; p < d.nphase; ++p) mt = mt > d.ph[p].mtiles ? mt : d.ph[p].mtiles;
    if (d.bm != 256 || d.Npad != 192 || d.a_op != AOP_NONE) return IC_ERR_ARG;
    if (d.bf16) {
      if (!d.xb || d.Cin % 64 != 0) return IC_ERR_ARG;
      hipLaunchKernelGGL(ig_kernel_b16d, dim3(mt, 1, d.nphase * d.ksplit), dim3(512), 0, s, d);
    } else {
      hipLaunchKernelGGL(ig_kernel_x3d, dim3(mt, 1, d.nphase * d.ksplit), dim3(512), 0, s, d);
    }
    IC_CHECK_LAUNCH();
    rc = IC_OK;
  }
  else if (d.bn == 192 && d.bm == 64) rc = ig_launch_t<64, 192, 32, 96>(d, s);
  else if (d.bn == 192) rc = ig_launch_t<128, 192, 64, 96>(d, s);
  else if (d.bn == 64) rc = ig_launch_t<128, 64, 64, 32>(d, s);
  else rc = ig_launch_t<256, 32, 64, 32>(d, s);
  if (rc) return rc;
  if (d.ksplit > 1) {
    const long long total = d.Mtot * d.Cout;
    if (IG_REDUCE4 && d.Cout % 4 == 0 && ((uintptr_t)d.partial & 15) == 0) {
      long long blocks = (total / 4 + 255) / 256;
      if (blocks > 4096) blocks = 4096;
      const dim3 g((unsigned)blocks), b(256);
      switch (d.ksplit) {
        case 2: hipLaunchKernelGGL(ig_reduce4_kernel<2>, g, b, 0, s, d); break;
        case 3: hipLaunchKernelGGL(ig_reduce4_kernel<3>, g, b, 0, s, d); break;
        case 4: hipLaunchKernelGGL(ig_reduce4_kernel<4>, g, b, 0, s, d); break;
        case 8: hipLaunchKernelGGL(ig_reduce4_kernel<8>, g, b, 0, s, d); break;
        default: hipLaunchKernelGGL(ig_reduce4_kernel<0>, g, b, 0, s, d);
      }
      IC_CHECK_LAUNCH();
      return IC_OK;
    }
    long long blocks = (total + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(ig_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, s, d);
    IC_CHECK_LAUNCH();
  }
  return IC_OK;
}

int ig_cvt_bf16(const float* x, void* xb, long long n, hipStream_t s) {
  if (n % 8 != 0) return IC_ERR_ARG;
  const long long n8 = n / 8;
  long long blocks = (n8 + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) return IC_OK;
  hipLaunchKernelGGL(ig_cvt_bf16_kernel, dim3((unsigned)blocks), dim3(256), 0, s, x, (__bf16*)xb, n8);
  IC_CHECK_LAUNCH();
  return IC_OK;
}
