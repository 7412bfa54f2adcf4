// Fused GDN / IGDN forward and backward for NHWC-dense activations with
// C in {64, 128, 192} (modelling/layers/gdn.py:79-88):
//
//   norm[m][n] = beta[n] + sum_k gamma[n][k] * x[m][k]^2
//   y[m][n]    = x[m][n] * norm^-1/2            (IGDN: x * norm^1/2)
//
// backward (q = dL/dnorm):
//   q[m][n]      = -1/2 dy x norm^-3/2         (IGDN: +1/2 dy x norm^-1/2)
//   dx[m][k]     = dy norm^-1/2 (IGDN: dy norm^1/2) + 2 x[m][k] sum_n q[m][n] gamma[n][k]
//   dgamma[n][k] = sum_m q[m][n] x[m][k]^2,  dbeta[n] = sum_m q[m][n]
//
// Both are persistent kernels: 4 waves per block, wave w owns a C/4 slice of
// output channels and keeps its slice of gamma as MFMA B fragments in VGPRs for
// the whole launch, so gamma is read once per block.  Pixel tiles (BM rows of
// one contiguous NHWC run) stream in by LDS-DMA (global_load_lds_dwordx4) into
// two LDS buffers so tile i+1 lands while tile i computes.  Tile images are
// [row][C] with the 16-B chunks XOR-swizzled by row (chunk ^ (row & 15)) so the
// 16 rows of an MFMA fragment read distinct banks; the swizzle is applied to
// the DMA *source* address because the LDS-DMA destination is lane-linear.
// Results are written back into LDS and leave through one coalesced copy-out
// pass (whole 16-B chunks), so every HBM byte moves once:
//   fwd: read x, write y and norm               (3 C 4 B per pixel)
//   bwd: read x, norm, dy, write dx             (4 C 4 B per pixel)
// The backward also accumulates dgamma (C x C) in VGPRs across all of the
// block's tiles and writes one partial per block; a fixed-order reduction
// kernel sums the partials (deterministic, no atomics).
//
// MFMA: v_mfma_f32_16x16x4_f32 (exact f32).  Where an operand comes from a
// b128 LDS read, step s = 4u+v consumes logical channel 16u + 4*(lane>>4) + v in
// both operands.
#include "../../include/imgcomp.h"
#include "gemm.h"
#ifndef GDN_SPLIT_PK
#define GDN_SPLIT_PK 1  // split staging through split3_bf16x4 (paired conversions)
#endif

// per-block backward partials: dgamma (C x C), dbeta (C), column sums of dx (C)
#define GDN_SLAB(C) ((C) * (C) + 2 * (C))

namespace {

__device__ __attribute__((aligned(16))) float gdn_zero_page[4];

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef const __attribute__((address_space(1))) void* gbl_ptr_t;

// 16 B per lane global -> LDS (M0 = the wave's LDS base; M0 restored after).  Issued from
// inline asm rather than __builtin_amdgcn_global_load_lds: for the builtin, the compiler cannot
// tell the DMA's LDS target from the buffers being read and waits vmcnt(0) before the next LDS
// read, which puts the whole DMA latency of the next tile on the current tile's path.  The
// kernels wait for these loads explicitly (s_waitcnt vmcnt before the barrier that publishes a
// tile).
#ifndef GDN_BWD_DMA_B
#define GDN_BWD_DMA_B 1  // fused backward: group B issues the next tile's DMA (0: group A, after its first MFMAs)
#endif
#ifndef X3W_ABL
#define X3W_ABL 0  // diagnostic ablations of gdn_bwd_x3w_kernel (wrong results): 1 no loads in the loop, 2 no
                   // phase A, 4 no dgamma MFMAs, 8 no dx MFMAs, 16 no dx stores
#endif
#ifndef X3W_STAMP
#define X3W_STAMP 0  // diagnostic: per-iteration s_memtime stamps of gdn_bwd_x3w_kernel into the workspace
#endif
#ifndef X3W_SGB
#define X3W_SGB 1  // gdn_bwd_x3w_kernel: interleave phase A / epilogue with the MFMAs (sched_group_barrier)
#endif
#ifndef GDN_DMA_ASM
#define GDN_DMA_ASM 1
#endif
__device__ __forceinline__ void glds16(const float* src, float* lds_wave_base) {
  if (!GDN_DMA_ASM) {
    __builtin_amdgcn_global_load_lds((gbl_ptr_t)src, (lds_ptr_t)lds_wave_base, 16, 0, 0);
    return;
  }
  const uint32_t l = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_ptr_t)lds_wave_base);
  uint32_t save;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(save)
      : "v"(src), "s"(l)
      : "memory");
}

// element (m, n) of a swizzled [rows][C] tile image
template <int C>
__device__ __forceinline__ int swz(int m, int n) {
  return m * C + ((((n >> 2) ^ (m & 15)) << 2) | (n & 3));
}

// stage rows [m0, m0+BM) of a dense [P][C] tensor into a swizzled LDS image
template <int C, int BM, int NT>
__device__ __forceinline__ void stage_tile(const float* __restrict__ g, uint32_t m0, uint32_t P, float* img, int tid,
                                           int lane) {
  constexpr int CH = C / 4;
  constexpr int QPASS = BM * CH / NT;
  static_assert(BM * CH % NT == 0, "whole DMA passes");
#pragma unroll
  for (int q = 0; q < QPASS; ++q) {
    const int pos = tid + NT * q;  // lane-linear LDS chunk
    const int row = pos / CH, pc = pos - (pos / CH) * CH;
    const int lc = pc ^ (row & 15);  // logical chunk stored at pc
    const float* src = gdn_zero_page;
    if (m0 + row < P) src = g + (size_t)(m0 + row) * C + lc * 4;
    glds16(src, img + (pos - lane) * 4);
  }
}

// copy a swizzled LDS image out to rows [m0, m0+BM) of a dense [P][C] tensor
template <int C, int BM, int NT>
__device__ __forceinline__ void store_tile(float* __restrict__ g, uint32_t m0, uint32_t P, const float* img, int tid) {
  constexpr int CH = C / 4;
  constexpr int QPASS = BM * CH / NT;
#pragma unroll
  for (int q = 0; q < QPASS; ++q) {
    const int pos = tid + NT * q;
    const int row = pos / CH, lc = pos - (pos / CH) * CH;
    const floatx4v v = *(const floatx4v*)(img + row * C + ((lc ^ (row & 15)) << 2));
    if (m0 + row < P) *(floatx4v*)(g + (size_t)(m0 + row) * C + lc * 4) = v;
  }
}

// the same tile as bf16 (round to nearest even): 8 B per lane
template <int C, int BM, int NT>
__device__ __forceinline__ void store_tile_b16(__bf16* __restrict__ g, uint32_t m0, uint32_t P, const float* img,
                                               int tid) {
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  constexpr int CH = C / 4;
  constexpr int QPASS = BM * CH / NT;
#pragma unroll
  for (int q = 0; q < QPASS; ++q) {
    const int pos = tid + NT * q;
    const int row = pos / CH, lc = pos - (pos / CH) * CH;
    const floatx4v v = *(const floatx4v*)(img + row * C + ((lc ^ (row & 15)) << 2));
    if (m0 + row < P)
      *(u32x2*)(g + (size_t)(m0 + row) * C + lc * 4) = u32x2{ic_cvt_pk_bf16(v[0], v[1]), ic_cvt_pk_bf16(v[2], v[3])};
  }
}

// ============================================================== forward
// NW = C/32 waves (C=192: 6); wave w owns output channels [32w, 32w+32) of every
// row of a BM=32-pixel tile.  Two blocks share a CU (72 KB LDS each, three
// waves per SIMD), so one block's epilogue and copy-out overlap the other's
// MFMAs.
template <int C>
constexpr int fwd_waves() { return 4; }

template <int C, int BM>
__global__ void __launch_bounds__(256, 2)
    gdn_fwd_fused_kernel(const float* __restrict__ x, const float* __restrict__ gamma,
                         const float* __restrict__ beta, int inverse, float* __restrict__ y,
                         float* __restrict__ norm, uint32_t P) {
  constexpr int NW = fwd_waves<C>();
  constexpr int NT = 64 * NW;
  constexpr int NTW = C / 16 / NW;  // 16-wide n-tiles per wave
  constexpr int KU = C / 16;     // groups of 4 k-steps
  constexpr int MT = BM / 16;    // 16-row m-tiles
  constexpr int TILE = BM * C;
  constexpr int NSTORE = 2 * (BM * C / 4 / NT);  // vector-memory ops of one copy-out
  __shared__ __attribute__((aligned(16))) float lds[3 * TILE];  // 2 x-buffers + norm staging
  float* const nst = lds + 2 * TILE;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int li = lane & 15, lq = lane >> 4;
  const int nbase = w * (C / NW);
  const uint32_t ntiles = (P + BM - 1) / BM;

  // bfr[j][4u+v] = gamma[n = nbase+16j+li][k = 16u+4lq+v]
  float bfr[NTW][4 * KU];
#pragma unroll
  for (int j = 0; j < NTW; ++j)
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      const floatx4v g4 = *(const floatx4v*)(gamma + (size_t)(nbase + 16 * j + li) * C + 16 * u + 4 * lq);
#pragma unroll
      for (int v = 0; v < 4; ++v) bfr[j][4 * u + v] = g4[v];
    }
  float bet[NTW];
#pragma unroll
  for (int j = 0; j < NTW; ++j) bet[j] = beta[nbase + 16 * j + li];

  uint32_t tile = blockIdx.x;
  if (tile < ntiles) stage_tile<C, BM, NT>(x, tile * BM, P, lds, tid, lane);
  int buf = 0;
  bool first = true;
  for (; tile < ntiles; tile += gridDim.x) {
    // tile `buf` landed: its DMA is older than the previous copy-out's stores
    if (first) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(NSTORE) : "memory");
    __builtin_amdgcn_s_barrier();
    first = false;
    const uint32_t nxt = tile + gridDim.x;
    float* xs = lds + buf * TILE;

    floatx4v acc[MT][NTW];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int j = 0; j < NTW; ++j) acc[mt][j] = floatx4v{0.f, 0.f, 0.f, 0.f};
    // A fragments one k-group ahead (software pipeline); the scheduling
    // barrier keeps the compiler from hoisting all KU groups' LDS reads
    floatx4v a4[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) a4[mt] = *(const floatx4v*)(xs + (16 * mt + li) * C + ((lq ^ li) << 2));
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      floatx4v an[MT];
      if (u + 1 < KU) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
          an[mt] = *(const floatx4v*)(xs + (16 * mt + li) * C + (((4 * (u + 1) + lq) ^ li) << 2));
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) a4[mt] = a4[mt] * a4[mt];
#pragma unroll
      for (int v = 0; v < 4; ++v)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int j = 0; j < NTW; ++j)
            acc[mt][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[mt][v], bfr[j][4 * u + v], acc[mt][j], 0, 0, 0);
      if (u + 1 < KU) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) a4[mt] = an[mt];
      }
      __builtin_amdgcn_sched_barrier(0);
      // the next tile's DMA issues behind the first MFMAs, off the
      // barrier-to-barrier path (buffer buf^1 is free since the barrier)
      if (u == 0 && nxt < ntiles) {
        stage_tile<C, BM, NT>(x, nxt * BM, P, lds + (buf ^ 1) * TILE, tid, lane);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // every wave's x^2 reads are done before y overwrites x in place
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // epilogue into LDS (C/D map: col n = li, row m = 4*lq + r); y in place of x
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int j = 0; j < NTW; ++j) {
        const int n = nbase + 16 * j + li;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int off = swz<C>(16 * mt + 4 * lq + r, n);
          const float nv = acc[mt][j][r] + bet[j];
          const float xv = xs[off];
          xs[off] = inverse ? xv * __builtin_amdgcn_sqrtf(nv) : xv * __builtin_amdgcn_rsqf(nv);
          nst[off] = nv;
        }
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    store_tile<C, BM, NT>(y, tile * BM, P, xs, tid);
    store_tile<C, BM, NT>(norm, tile * BM, P, nst, tid);
    buf ^= 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}


// ============================================================== forward, split
// norm = beta + Gamma x^2 in split arithmetic (fp32 via three bf16 terms, six
// v_mfma_f32_16x16x32_bf16 products, fp32 accumulation), C = 192.  12 waves
// (768 threads), one block per CU: wave w owns output channels [16w, 16w+16)
// and keeps its slice of Gamma, split into three bf16 terms, as B fragments in
// 72 VGPRs for the whole launch.  Per 32-pixel tile one cooperative pass
// squares x and writes x^2 as three bf16 planes (384-B rows, 16-B chunks XOR
// (row >> 1) & 7: conflict-free 16x16x32 fragment reads), then the MFMAs and
// the epilogue.  Three x buffers and two sets of x^2 planes (144 KB), so one
// barrier per tile separates
//   loads of tile i+3 | split pass of tile i+1 | MFMAs + epilogue of tile i
// and the waves' split work (VALU, LDS) overlaps the other waves' MFMAs.  x is
// staged through registers (loaded three tiles ahead of its MFMAs, written to
// LDS one tile after its loads issued), not by LDS-DMA: the compiler cannot tell an LDS-DMA target
// from the buffers being read and would wait for the DMA before every LDS read.
// y and norm leave straight from the MFMA result registers (each 16-lane group
// writes 64 contiguous bytes of a pixel row; the 12 waves fill the row): no norm
// staging image and no copy-out pass.
//
// NP = 1 (IC_MATH_BF16, config C3): the same kernel on bf16 operands -- Gamma and x^2 rounded to
// nearest even, one plane each, one product, fp32 accumulation.
// YB (with NP = 1, config C3): y also as a compact bf16 copy (yb), the A operand of the next conv's
// bf16 DMA tiles (ig_kernel_b16d), so that conv reads 2 B per element and converts nothing.
// NORM = false (with NP = 1, config C3, round 6): norm is not stored -- the backward recomputes it
// (gdn_bwd_fused_kernel<..., RN>), 4 of the 14 bytes per element this HBM-bound kernel moves.
template <int C, int NP = 3, bool YB = false, bool NORM = true>
__global__ void __launch_bounds__(768, 1)
    gdn_fwd_x3s_kernel(const float* __restrict__ x, const float* __restrict__ gamma,
                       const float* __restrict__ beta, int inverse, float* __restrict__ y,
                       float* __restrict__ norm, uint32_t P, __bf16* __restrict__ yb = nullptr) {
  static_assert(C == 192, "12 waves x 16 channels");
  static_assert(NP == 3 || NP == 1, "split (3 planes) or bf16 (1 plane)");
  typedef __bf16 b4 __attribute__((ext_vector_type(4)));
  typedef __bf16 b8 __attribute__((ext_vector_type(8)));
  constexpr int BM = 32, NT = 768;
  constexpr int TILE = BM * C;
  constexpr int KU = C / 32;
  constexpr int QS = BM * C / 4 / NT;  // float4 per thread in staging and in the split pass
  __shared__ __attribute__((aligned(16))) float lds[3 * TILE];        // three x buffers
  __shared__ __attribute__((aligned(16))) __bf16 sq[2 * NP * TILE];  // two sets of NP x^2 planes

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int li = lane & 15, lg = lane >> 4;
  const int n = 16 * w + li;
  const uint32_t ntiles = (P + BM - 1) / BM;
  const uint32_t G = gridDim.x;

  b8 bg[NP][KU];
#pragma unroll
  for (int u = 0; u < KU; ++u) {
    const floatx4v g0 = *(const floatx4v*)(gamma + (size_t)n * C + 32 * u + 8 * lg);
    const floatx4v g1 = *(const floatx4v*)(gamma + (size_t)n * C + 32 * u + 8 * lg + 4);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float gv = e < 4 ? g0[e] : g1[e - 4];
      if constexpr (NP == 1) {
        bg[0][u][e] = (__bf16)gv;  // round to nearest even
      } else {
        __bf16 hh, mm, ll;
        split3_bf16(gv, hh, mm, ll);
        bg[0][u][e] = hh; bg[NP - 2][u][e] = mm; bg[NP - 1][u][e] = ll;
      }
    }
  }
  float bet = beta[n];
  // consume the prologue's loads here: a load still pending at the loop entry makes the compiler
  // wait for every store of the previous tile inside the loop
  asm volatile("" : "+v"(bet));
  const int fsw = (li >> 1) & 7;

  // staging: float4 `pos` of a swizzled image holds logical chunk (pos % (C/4)) ^ (row & 15)
  int srow[QS], scol[QS];
#pragma unroll
  for (int q = 0; q < QS; ++q) {
    const int pos = tid + NT * q;
    srow[q] = pos / (C / 4);
    scol[q] = ((pos - srow[q] * (C / 4)) ^ (srow[q] & 15)) * 4;
  }
  // rows past P load row P-1 (a row's x^2 feeds only that row's outputs, which are not stored)
  auto load = [&](uint32_t t, floatx4v* r) {
#pragma unroll
    for (int q = 0; q < QS; ++q) {
      const uint32_t m = min(t * BM + srow[q], P - 1);
      r[q] = *(const floatx4v*)(x + (size_t)m * C + scol[q]);
    }
  };
  auto put = [&](float* img, const floatx4v* r) {
#pragma unroll
    for (int q = 0; q < QS; ++q) *(floatx4v*)(img + (tid + NT * q) * 4) = r[q];
  };
  // x^2 split pass: float4 `pos` of a swizzled fp32 image -> 3 bf16 quads
  auto split_pass = [&](const float* xs, __bf16* sb) {
#pragma unroll
    for (int q = 0; q < QS; ++q) {
      const int pos = tid + NT * q;
      const int m = srow[q], lc = scol[q] >> 2;
      const floatx4v v = *(const floatx4v*)(xs + pos * 4);
      const int off = m * C + 8 * ((lc >> 1) ^ ((m >> 1) & 7)) + 4 * (lc & 1);
      if constexpr (NP == 1) {
        typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
        const floatx4v v2 = v * v;
        *(b4*)(sb + off) = __builtin_bit_cast(b4, u32x2{ic_cvt_pk_bf16(v2[0], v2[1]), ic_cvt_pk_bf16(v2[2], v2[3])});
      } else {
        b4 vh, vm, vl;
        split3_bf16x4(v * v, vh, vm, vl);
        *(b4*)(sb + off) = vh;
        *(b4*)(sb + TILE + off) = vm;
        *(b4*)(sb + 2 * TILE + off) = vl;
      }
    }
  };

  uint32_t tile = blockIdx.x;
  if (tile >= ntiles) return;
  floatx4v ra[QS], rb[QS];  // staging registers, two tiles in flight (loaded 2 tiles ahead of use)
  load(tile, ra);
  put(lds, ra);
  load(tile + G < ntiles ? tile + G : tile, ra);
  put(lds + TILE, ra);
  load(tile + 2 * G < ntiles ? tile + 2 * G : tile, rb);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  split_pass(lds, sq);
  int bx = 0, sb = 0;  // x buffer of `tile` (next: bx+1, staging: bx+2, mod 3); its plane set
  // one tile: load tile+3G into `ld` (a tile past the end reloads this one: no branch, so the
  // compiler counts the loads and stores and never waits for the stores), write `pt` (tile+2G,
  // loaded one tile earlier) into the free buffer at the end
  auto step = [&](floatx4v* ld, const floatx4v* pt) {
    // plane set sb and x buffer bx+1 complete; every wave's reads of the buffers written below done
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const int b1 = bx == 2 ? 0 : bx + 1, b2 = b1 == 2 ? 0 : b1 + 1;
    load(tile + 3 * G < ntiles ? tile + 3 * G : tile, ld);
    if (tile + G < ntiles) split_pass(lds + b1 * TILE, sq + (sb ^ 1) * NP * TILE);
    const float* xs = lds + bx * TILE;
    const __bf16* sp = sq + sb * NP * TILE;
    floatx4v acc[BM / 16];
#pragma unroll
    for (int mt = 0; mt < BM / 16; ++mt) {
      acc[mt] = floatx4v{0.f, 0.f, 0.f, 0.f};
      const __bf16* ar = sp + (16 * mt + li) * C;
#pragma unroll
      for (int u = 0; u < KU; ++u) {
        const int ch = 8 * ((4 * u + lg) ^ fsw);
        if constexpr (NP == 1) {
          acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*(const b8*)(ar + ch), bg[0][u], acc[mt], 0, 0, 0);
        } else {
          const b8 a0 = *(const b8*)(ar + ch), a1 = *(const b8*)(ar + TILE + ch), a2 = *(const b8*)(ar + 2 * TILE + ch);
          acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2, bg[0][u], acc[mt], 0, 0, 0);
          acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bg[1][u], acc[mt], 0, 0, 0);
          acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bg[2][u], acc[mt], 0, 0, 0);
          acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bg[0][u], acc[mt], 0, 0, 0);
          acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bg[1][u], acc[mt], 0, 0, 0);
          acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bg[0][u], acc[mt], 0, 0, 0);
        }
      }
    }
    // epilogue (C/D map: col n = li, row m = 16mt + 4g + r) straight to y and norm; rows past P
    // hold row P-1's x, so their results equal row P-1's and are stored there (the same values)
    const uint32_t m0 = tile * BM;
#pragma unroll
    for (int mt = 0; mt < BM / 16; ++mt)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int m = 16 * mt + 4 * lg + q;
        const float nv = acc[mt][q] + bet;
        const float xv = xs[swz<C>(m, n)];
        const float yv = inverse ? xv * __builtin_amdgcn_sqrtf(nv) : xv * __builtin_amdgcn_rsqf(nv);
        const size_t o = (size_t)min(m0 + m, P - 1) * C + n;
        y[o] = yv;
        if constexpr (NORM) norm[o] = nv;
        if constexpr (YB) yb[o] = (__bf16)yv;  // round to nearest even
      }
    put(lds + b2 * TILE, pt);
    bx = b1;
    sb ^= 1;
    tile += G;
    return tile < ntiles;
  };
  while (step(ra, rb) && step(rb, ra)) {
  }
}

// ============================================================== backward
// Split bf16 planes of the backward ([pixel][channel], C = 192 bf16 per row, no padding): the 8-channel
// (16-B) chunk k of row m (0..15) is stored at chunk k ^ pl_sw(m), pl_sw(m) = 4 bit1(m) + ((4 - (m>>2)) & 3)
// (within the row's aligned groups of 8 chunks).  Conflict-free for both readers: the dgamma GEMM's
// transposed reads (ds_read_b64_tr_b16: 4 consecutive rows x 32 channels per 32 lanes -- the rows differ
// in bank bits 5 (row parity, 384-B rows) and 4 (bit 1)) and the split dx GEMM's fragments (ds_read_b128:
// row li, chunk 4u + lg -- within each 16-lane bank group of b128 the 16 (row, chunk) pairs cover the 64
// banks); the phase-A stores of gdn_bwd_x3w_kernel (ds_write_b64, 16 rows of one channel group per 16
// lanes) are 2-way, the least any chunk-granular swizzle of 384-B rows allows (was 4-way with
// 4 bit1 + 2 bit2; bank simulation: tools/plane_banks.py).
__device__ __forceinline__ int pl_sw(int m) { return (((m >> 1) & 1) << 2) | ((4 - (m >> 2)) & 3); }
template <int C>
__device__ __forceinline__ int pl_off(int m, int n) {
  return m * C + ((((n >> 3) ^ pl_sw(m))) << 3) + (n & 7);
}

// phase A of one tile (elementwise, identical swizzled offsets in every image):
// q = dL/dnorm, and the direct term dy*norm^-1/2 (IGDN: dy*norm^1/2) over dy
// X3: also write q and x^2, split into three bf16 terms, as [pixel][channel]
// planes (sb: q planes then x^2 planes, swizzled by pl_off) for the split GEMMs
// BF: bf16 operands (config C3): only the first plane, q and x^2 rounded to nearest even
// one float4 chunk `pos` (lane-linear position in the swizzled images) with its norm values nv
template <int C, int BM, bool X3 = false, bool BF = false>
__device__ __forceinline__ void gdn_bwd_phase_a_chunk(int pos, const floatx4v nv, const float* xs, float* gs,
                                                      float* qs, uint32_t m0, uint32_t P, int inverse, __bf16* sb) {
  {
    const int off = pos * 4;
    const bool valid = m0 + (uint32_t)(pos / (C / 4)) < P;  // rows past P are zero-filled
    const floatx4v xv = *(const floatx4v*)(xs + off);
    const floatx4v gv = *(const floatx4v*)(gs + off);
    floatx4v qv, dv;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float rs = __builtin_amdgcn_rsqf(nv[e]);
      if (inverse) {
        qv[e] = 0.5f * gv[e] * xv[e] * rs;
        dv[e] = gv[e] * (nv[e] * rs);
      } else {
        qv[e] = -0.5f * gv[e] * xv[e] * (rs * rs * rs);
        dv[e] = gv[e] * rs;
      }
    }
    if (!valid) {  // keep 0 * inf out of dgamma
      qv = floatx4v{0.f, 0.f, 0.f, 0.f};
      dv = qv;
    }
    *(floatx4v*)(qs + off) = qv;
    *(floatx4v*)(gs + off) = dv;
    if constexpr (X3) {
      typedef __bf16 b4 __attribute__((ext_vector_type(4)));
      const int m = pos / (C / 4), lc = (pos - m * (C / 4)) ^ (m & 15);
      const int col = pl_off<C>(m, 4 * lc) - m * C;
      constexpr int PL = BM * C;  // one plane
#pragma unroll
      for (int op = 0; op < 2; ++op) {
        if constexpr (BF) {
          typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
          const floatx4v v = op == 0 ? qv : xv * xv;
          *(b4*)(sb + op * PL + m * C + col) =
              __builtin_bit_cast(b4, u32x2{ic_cvt_pk_bf16(v[0], v[1]), ic_cvt_pk_bf16(v[2], v[3])});
          continue;
        }
        b4 vh, vm, vl;
        if (GDN_SPLIT_PK) {
          split3_bf16x4(op == 0 ? qv : xv * xv, vh, vm, vl);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            __bf16 hh, mm, ll;
            split3_bf16(op == 0 ? qv[e] : xv[e] * xv[e], hh, mm, ll);
            vh[e] = hh; vm[e] = mm; vl[e] = ll;
          }
        }
        __bf16* dst = sb + op * 3 * PL + m * C + col;
        *(b4*)dst = vh;
        *(b4*)(dst + PL) = vm;
        *(b4*)(dst + 2 * PL) = vl;
      }
    }
  }
}

template <int C, int BM, bool X3 = false, bool BF = false>
__device__ __forceinline__ void gdn_bwd_phase_a(const float* xs, const float* ns, float* gs, float* qs, uint32_t m0,
                                                uint32_t P, int inverse, int tid, __bf16* sb = nullptr) {
  constexpr int NCH = BM * C / 4;
  for (int pos = tid; pos < NCH; pos += 512)
    gdn_bwd_phase_a_chunk<C, BM, X3, BF>(pos, *(const floatx4v*)(ns + pos * 4), xs, gs, qs, m0, P, inverse, sb);
}

// Keep a k-step's MFMAs inside that step: IR-level code motion otherwise sinks
// chains of them to the end of an unrolled loop, which keeps every step's
// operand fragments live (sched_barrier only constrains the machine
// scheduler).  Emits no instructions.
template <int N>
__device__ __forceinline__ void pin_acc(floatx4v* a) {
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+v"(a[i]));
}

__device__ __forceinline__ void bar_wait_lgkm() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}


// 8 waves, specialised (two per SIMD): waves 0-3 (group A) stage the tiles,
// form dx by a GEMM with gamma held in VGPRs and copy it out; waves 4-7
// (group B) accumulate dgamma (C x C, in VGPRs) and dbeta.  The groups run
// separate loops with the same barrier sequence per tile (B1 top, B2 after
// phase A, B3 before the copy-out), so each keeps only its own registers.
//
// X3 (C = 192, IC_MATH_SPLIT): group B's dgamma GEMM runs in split arithmetic
// (fp32 via three bf16 terms, six v_mfma_f32_32x32x16_bf16 products, fp32
// accumulation): phase A also writes q and x^2 as split bf16 [pixel][channel]
// images, read transposed (ds_read_b64_tr_b16, 8 pixels of one channel per
// lane); waves 4-7 own 96x96 quadrants of dgamma.  Group A's dx GEMM keeps
// gamma in VGPRs on the fp32 MFMA.
//
// BF (C = 192, with X3; IC_MATH_BF16, config C3): both GEMMs on bf16 operands with fp32
// accumulation — group A holds gamma as bf16 16x16x32 B fragments (72 VGPRs) and reads q's
// A fragments from the fp32 q image (8 channels per lane, rounded in registers); group B runs
// the quadrant GEMM with one product on single bf16 planes of q and x^2.
// XB (with BF): dx also as a compact bf16 copy (dxb), the A operand of the previous transposed conv's
// input gradient on the bf16 DMA tiles (ig_kernel_b16d).
// RN: one wave's share of phase A with the norm formed in registers.  The wave computes norm^T for its
// n-tiles tl0 .. tl0 + NT - 1 (16 channels each): norm[m][k] = beta[k] + sum_n bf16(gamma[k][n])
// bf16(x[m][n]^2) with Gamma's rows as the A operand (gfrag(j, s32), see gdn_norm_frags) and x^2 as B,
// over the six 16x16x32 K steps in order -- gdn_fwd_x3s_kernel<192, 1>'s products and order, so the
// forward's norm bitwise -- which leaves each lane the norm of 4 consecutive channels k = 16 tl + 4 lq ..
// of one pixel m = li: exactly one float4 chunk of phase A, which the lane then runs on its chunks
// (no norm image, no extra barrier).
template <int C, int BM, int NT, class GF>
__device__ __forceinline__ void gdn_norm_phase_a(const float* xs, float* gs, float* qs, __bf16* sb, GF gfrag,
                                                 const float (&bn)[NT][4], int tl0, int li, int lq, uint32_t m0,
                                                 uint32_t P, int inverse) {
  typedef __bf16 b8 __attribute__((ext_vector_type(8)));
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  floatx4v an[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) an[j] = floatx4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s32 = 0; s32 < C / 32; ++s32) {
    const int c0 = 8 * s32 + 2 * lq;
    floatx4v lo = *(const floatx4v*)(xs + li * C + ((c0 ^ li) << 2));
    floatx4v hi = *(const floatx4v*)(xs + li * C + (((c0 + 1) ^ li) << 2));
    lo = lo * lo;
    hi = hi * hi;
    const b8 b = __builtin_bit_cast(b8, u32x4{ic_cvt_pk_bf16(lo[0], lo[1]), ic_cvt_pk_bf16(lo[2], lo[3]),
                                               ic_cvt_pk_bf16(hi[0], hi[1]), ic_cvt_pk_bf16(hi[2], hi[3])});
#pragma unroll
    for (int j = 0; j < NT; ++j)
      an[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gfrag(j, s32), b, an[j], 0, 0, 0);
  }
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int pos = li * (C / 4) + ((4 * (tl0 + j) + lq) ^ li);  // chunk (m = li, k = 16 tl + 4 lq ..)
    gdn_bwd_phase_a_chunk<C, BM, true, true>(pos, an[j] + floatx4v{bn[j][0], bn[j][1], bn[j][2], bn[j][3]}, xs, gs,
                                             qs, m0, P, inverse, sb);
  }
}

// the bf16 rows of gamma an RN wave holds (A fragments: g[j][s32][e] = bf16(gamma[k = 16 (tl0 + j) + li][32 s32 +
// 8 lq + e])) and beta of the 4 output channels 16 (tl0 + j) + 4 lq .. each lane's results are
template <int C, int NT>
__device__ __forceinline__ void gdn_norm_frags(const float* __restrict__ gamma, const float* __restrict__ beta,
                                               __bf16 (&g)[NT][C / 32][8], float (&bn)[NT][4], int tl0, int li,
                                               int lq) {
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int k = 16 * (tl0 + j) + li;
#pragma unroll
    for (int r = 0; r < 4; ++r) bn[j][r] = beta[16 * (tl0 + j) + 4 * lq + r];  // the lane's output channels
#pragma unroll
    for (int s32 = 0; s32 < C / 32; ++s32) {
      const floatx4v g0 = *(const floatx4v*)(gamma + (size_t)k * C + 32 * s32 + 8 * lq);
      const floatx4v g1 = *(const floatx4v*)(gamma + (size_t)k * C + 32 * s32 + 8 * lq + 4);
#pragma unroll
      for (int e = 0; e < 8; ++e) g[j][s32][e] = (__bf16)(e < 4 ? g0[e] : g1[e - 4]);
    }
  }
}

// RN (with BF, round 6): norm is not read from HBM but recomputed per tile from the staged x, as the
// forward formed it (bitwise the forward's norm), inside phase A (gdn_norm_phase_a): each wave forms
// norm^T for its 16-channel n-tiles on the MFMA and runs phase A on the float4 chunks the result leaves in
// its lanes -- group A's waves two n-tiles each (the 2/3 of phase A they ran before; Gamma's rows as bf16
// A fragments, one tile's in 24 VGPRs, the other's in LDS), group B's one each from LDS (its 144 dgamma
// accumulators leave no registers; 48 KB of LDS in all).  No norm image and no extra barrier; the C3 GDN
// pair moves 10 + 14 bytes per element instead of 14 + 18.
template <int C, bool X3, bool BF = false, bool XB = false, bool RN = false>
__global__ void __launch_bounds__(512, 2)
    gdn_bwd_fused_kernel(const float* __restrict__ x, const float* __restrict__ norm, const float* __restrict__ dy,
                         const float* __restrict__ gamma, int inverse, float* __restrict__ dx,
                         float* __restrict__ slab, uint32_t P, __bf16* __restrict__ dxb = nullptr,
                         const float* __restrict__ beta = nullptr) {
  static_assert(!X3 || C == 192, "split dgamma tiles 192 x 192 as 2 x 2 quadrants of 96");
  static_assert(!BF || X3, "bf16 operands run on the split kernel's layout");
  static_assert(!RN || BF, "norm recomputed on the bf16 kernel only");
  constexpr int NP = BF ? 1 : 3;  // bf16 planes per operand image
  constexpr int BM = 16;
  constexpr int NTA = 256;       // threads of group A (staging / copy-out)
  constexpr int W4 = C / 4;      // channels per wave slice
  constexpr int NTW = C / 64;    // 16-wide tiles per wave slice
  constexpr int KT = C / 16;     // 16-wide tiles over all channels
  constexpr int KU = C / 16;
  constexpr int TILE = BM * C;
  constexpr int NSTORE = BM * C / 4 / NTA;
  // per buffer: x, norm (not with RN), dy images; plus the q image
  constexpr int BUF = RN ? 2 * TILE : 3 * TILE, DYO = RN ? TILE : 2 * TILE;
  __shared__ __attribute__((aligned(16))) float lds[2 * BUF + TILE];
  __shared__ __attribute__((aligned(16))) __bf16 sbf[X3 ? 2 * NP * TILE : 8];  // split q / x^2 images
  __shared__ __attribute__((aligned(16))) __bf16 gnrl[RN ? 12 * (C / 32) * 64 * 8 : 8];  // RN: Gamma's rows, 12 n-tiles
  float* const qs = lds + 2 * BUF;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int li = lane & 15, lq = lane >> 4;
  const int wbase = (w & 3) * W4;
  const uint32_t ntiles = (P + BM - 1) / BM;

  // group B issues the next tile's DMA (not in the fp32 C = 192 kernel, whose group B holds a
  // 144-register dgamma and would spill)
  constexpr bool DMA_B = GDN_BWD_DMA_B && (X3 || C < 192);
  // x, norm, dy of tile t into buffer b (256 threads; ti = thread index within the group)
  auto stage = [&](uint32_t t, int b, int ti) {
    float* base = lds + b * BUF;
    stage_tile<C, BM, NTA>(x, t * BM, P, base, ti, lane);
    if constexpr (!RN) stage_tile<C, BM, NTA>(norm, t * BM, P, base + TILE, ti, lane);
    stage_tile<C, BM, NTA>(dy, t * BM, P, base + DYO, ti, lane);
  };

  if (w < 4) {
    // ---------------- group A: dxg[m][k] = sum_n q[m][n] gamma[n][k], k = wbase + 16j + li
    // step s = 4u+v: n = 16u + 4lq + v  ->  bfr[j][4u+v] = gamma[n][k]
    // BF: 16x16x32 step s32: n = 32 s32 + 8 lq + e  ->  gbf[j][s32][e] = bf16(gamma[n][k])
    typedef __bf16 b8 __attribute__((ext_vector_type(8)));
    constexpr int K32 = C / 32;
    float bfr[BF ? 1 : NTW][BF ? 1 : 4 * KU];
    b8 gbf[BF ? NTW : 1][BF ? K32 : 1];
    // RN: Gamma's rows of n-tiles 2w, 2w + 1 for gdn_norm_phase_a, parked in LDS (this wave's slots in lane
    // order: conflict-free 16-B reads)
    float bnr[2][4];
    __bf16* gnl = gnrl + (size_t)w * 2 * K32 * 64 * 8;
    if constexpr (RN) {
      __bf16 g2[2][K32][8];
      gdn_norm_frags<C, 2>(gamma, beta, g2, bnr, 2 * w, li, lq);
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int s32 = 0; s32 < K32; ++s32) *(b8*)(gnl + ((j * K32 + s32) * 64 + lane) * 8) = *(const b8*)g2[j][s32];
    }
    if constexpr (BF) {
#pragma unroll
      for (int j = 0; j < NTW; ++j)
#pragma unroll
        for (int s32 = 0; s32 < K32; ++s32)
#pragma unroll
          for (int e = 0; e < 8; ++e)
            gbf[j][s32][e] = (__bf16)gamma[(size_t)(32 * s32 + 8 * lq + e) * C + wbase + 16 * j + li];
    } else {
#pragma unroll
    for (int j = 0; j < NTW; ++j)
#pragma unroll
      for (int u = 0; u < KU; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v)
          bfr[j][4 * u + v] = gamma[(size_t)(16 * u + 4 * lq + v) * C + wbase + 16 * j + li];
    }
    uint32_t tile = blockIdx.x;
    if (tile < ntiles) stage(tile, 0, tid);
    int buf = 0, it = 0;
    bool first = true;
    for (; tile < ntiles; tile += gridDim.x, ++it) {
      if (first) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(NSTORE) : "memory");
      __builtin_amdgcn_s_barrier();  // B1
      first = false;
      const uint32_t nxt = tile + gridDim.x;
      float* xs = lds + buf * BUF;
      float* gs = xs + DYO;  // dy, then the direct term of dx, then dx
      if constexpr (RN)
        gdn_norm_phase_a<C, BM, 2>(xs, gs, qs, sbf,
                                   [&](int j, int s32) { return *(const b8*)(gnl + ((j * K32 + s32) * 64 + lane) * 8); },
                                   bnr, 2 * w, li, lq, tile * BM, P, inverse);
      else
        gdn_bwd_phase_a<C, BM, X3, BF>(xs, xs + TILE, gs, qs, tile * BM, P, inverse, tid, sbf);
      bar_wait_lgkm();  // B2
      floatx4v acc[NTW];
#pragma unroll
      for (int j = 0; j < NTW; ++j) acc[j] = floatx4v{0.f, 0.f, 0.f, 0.f};
      if constexpr (BF) {
        // A fragment of step s32: q[m = li][32 s32 + 8 lq .. + 7] = logical chunks 8 s32 + 2 lq (+1)
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int s32 = 0; s32 < K32; ++s32) {
          const int c0 = 8 * s32 + 2 * lq;
          const floatx4v lo = *(const floatx4v*)(qs + li * C + ((c0 ^ li) << 2));
          const floatx4v hi = *(const floatx4v*)(qs + li * C + (((c0 + 1) ^ li) << 2));
          const b8 a = __builtin_bit_cast(b8, u32x4{ic_cvt_pk_bf16(lo[0], lo[1]), ic_cvt_pk_bf16(lo[2], lo[3]),
                                                     ic_cvt_pk_bf16(hi[0], hi[1]), ic_cvt_pk_bf16(hi[2], hi[3])});
#pragma unroll
          for (int j = 0; j < NTW; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, gbf[j][s32], acc[j], 0, 0, 0);
        }
      } else
#pragma unroll
      for (int u = 0; u < KU; ++u) {
        const floatx4v a4 = *(const floatx4v*)(qs + li * C + (((4 * u + lq) ^ li) << 2));
#pragma unroll
        for (int v = 0; v < 4; ++v)
#pragma unroll
          for (int j = 0; j < NTW; ++j)
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[v], bfr[j][4 * u + v], acc[j], 0, 0, 0);
        if (!DMA_B && u == 0) {
          // the next tile's DMA issues behind the first MFMAs instead of on the
          // barrier-to-barrier critical path (buffer buf^1 is free since B1)
          __builtin_amdgcn_sched_barrier(0);
          if (nxt < ntiles) stage(nxt, buf ^ 1, tid);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      // dx = direct + 2 x dxg over the direct term (each element owned by one lane); m = 4lq + r
#pragma unroll
      for (int j = 0; j < NTW; ++j) {
        const int k = wbase + 16 * j + li;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int off = swz<C>(4 * lq + r, k);
          gs[off] = gs[off] + 2.f * xs[off] * acc[j][r];
        }
      }
      bar_wait_lgkm();  // B3
      store_tile<C, BM, NTA>(dx, tile * BM, P, gs, tid);
      if constexpr (XB) store_tile_b16<C, BM, NTA>(dxb, tile * BM, P, gs, tid);
      buf ^= 1;
    }
  } else if constexpr (X3) {
    // ---------------- group B, split: dgamma[n][k] += sum_m q[m][n] x[m][k]^2 on 96x96 quadrants
    typedef __bf16 b4 __attribute__((ext_vector_type(4)));
    typedef __bf16 b8 __attribute__((ext_vector_type(8)));
    constexpr int PL = TILE;  // bf16 elements per plane
    const int wq = w - 4, wm2 = wq >> 1, wn2 = wq & 1;
    const int r = lane & 31, h = lane >> 5;
    // transposed read of rows 8h + (li >> 2) (lo) and that + 4 (hi), columns c0 + 16*(lane>>4 & 1) + 4*(li & 3)
    const int tr_row = 8 * h + (li >> 2);
    const int tr_col = 16 * ((lane >> 4) & 1) + 4 * (li & 3);
    auto tr8 = [&](const __bf16* plane, int c0) {
      const int c = c0 + tr_col;
      const b4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
          (__attribute__((address_space(3))) b4*)(plane + pl_off<C>(tr_row, c)));
      const b4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
          (__attribute__((address_space(3))) b4*)(plane + pl_off<C>(tr_row + 4, c)));
      return (b8)__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    };
    floatx16 acc[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    float db = 0.f, dxs = 0.f;
    const int t = tid - 256;
    int buf = 0;
    int it = 0;
    // RN: Gamma's rows of n-tile 8 + (w - 4) (gdn_norm_phase_a), parked in LDS (this wave's slot, lane order;
    // group B has no registers to spare beside its 144 dgamma accumulators)
    float bnr[1][4];
    __bf16* gnl = gnrl + (size_t)(8 + wq) * (C / 32) * 64 * 8;  // after group A's eight tiles
    if constexpr (RN) {
      __bf16 gnr[1][C / 32][8];
      gdn_norm_frags<C, 1>(gamma, beta, gnr, bnr, 8 + wq, li, lq);
#pragma unroll
      for (int s32 = 0; s32 < C / 32; ++s32) *(b8*)(gnl + (s32 * 64 + lane) * 8) = *(const b8*)gnr[0][s32];
    }
    for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x, ++it) {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // B1
      const float* xs = lds + buf * BUF;
      const uint32_t m0 = tile * BM;
      // group B (idle at B3 while group A finishes dx) issues the next tile's DMA; buffer buf^1
      // is free since B1, and this group's wait before the next B1 covers it
      if (DMA_B && tile + gridDim.x < ntiles) stage(tile + gridDim.x, buf ^ 1, tid - NTA);
      if constexpr (RN)
        gdn_norm_phase_a<C, BM, 1>(xs, (float*)xs + DYO, qs, sbf,
                                   [&](int, int s32) { return *(const b8*)(gnl + (s32 * 64 + lane) * 8); }, bnr, 8 + wq,
                                   li, lq, m0, P, inverse);
      else
        gdn_bwd_phase_a<C, BM, X3, BF>(xs, xs + TILE, (float*)xs + DYO, qs, m0, P, inverse, tid, sbf);
      bar_wait_lgkm();  // B2
      if (t < C) {
        const int rows = (P - m0) < (uint32_t)BM ? (int)(P - m0) : BM;
        for (int m = 0; m < rows; ++m) db += qs[swz<C>(m, t)];
      }
      b8 bb[NP][3];
#pragma unroll
      for (int q = 0; q < NP; ++q)
#pragma unroll
        for (int j = 0; j < 3; ++j) bb[q][j] = tr8(sbf + NP * PL + q * PL, 96 * wn2 + 32 * j);
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        b8 a[NP];
#pragma unroll
        for (int q = 0; q < NP; ++q) a[q] = tr8(sbf + q * PL, 96 * wm2 + 32 * i);
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          if constexpr (BF) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], bb[0][j], acc[i][j], 0, 0, 0);
            continue;
          }
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], bb[0][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], bb[1][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], bb[2][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], bb[0][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], bb[1][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], bb[0][j], acc[i][j], 0, 0, 0);
        }
      }
      bar_wait_lgkm();  // B3
      if (t < C) {  // column sums of this tile's dx (the producing conv's bias gradient)
        const float* gsd = xs + DYO;
        const int rows = (P - m0) < (uint32_t)BM ? (int)(P - m0) : BM;
        for (int m = 0; m < rows; ++m) dxs += gsd[swz<C>(m, t)];
      }
      buf ^= 1;
    }
    float* out = slab + (size_t)blockIdx.x * GDN_SLAB(C);
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        // C/D map of the 32x32 MFMA: row (A index n) = (reg&3) + 8(reg>>2) + 4h, col (B index k) = lane&31
        const int n = 96 * wm2 + 32 * i + (reg & 3) + 8 * (reg >> 2) + 4 * h;
#pragma unroll
        for (int j = 0; j < 3; ++j) out[(size_t)n * C + 96 * wn2 + 32 * j + r] = acc[i][j][reg];
      }
    if (t < C) {
      out[C * C + t] = db;
      out[C * C + C + t] = dxs;
    }
  } else {
    // ---------------- group B: dgamma[n][k] += sum_m q[m][n] x[m][k]^2, rows n = wbase + 16i + li
    floatx4v dg[NTW][KT];
#pragma unroll
    for (int i = 0; i < NTW; ++i)
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) dg[i][kt] = floatx4v{0.f, 0.f, 0.f, 0.f};
    float db = 0.f, dxs = 0.f;  // dbeta[t] and dx column-sum partials, t = tid - 256 < C
    const int t = tid - 256;
    int buf = 0;
    int it = 0;
    for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x, ++it) {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // B1
      const float* xs = lds + buf * BUF;
      const uint32_t m0 = tile * BM;
      // group B (idle at B3 while group A finishes dx) issues the next tile's DMA; buffer buf^1
      // is free since B1, and this group's wait before the next B1 covers it
      if (DMA_B && tile + gridDim.x < ntiles) stage(tile + gridDim.x, buf ^ 1, tid - NTA);
      gdn_bwd_phase_a<C, BM, X3, BF>(xs, xs + TILE, (float*)xs + 2 * TILE, qs, m0, P, inverse, tid, sbf);
      bar_wait_lgkm();  // B2
      if (t < C) {
        const int rows = (P - m0) < (uint32_t)BM ? (int)(P - m0) : BM;
        for (int m = 0; m < rows; ++m) db += qs[swz<C>(m, t)];
      }
      // k-step s2 of the pixel reduction takes pixel m = 4 lq + s2 (any order
      // works, A and B agree): the 4 lane quads then read rows differing in
      // bits 2-3, which the row swizzle sends to distinct banks.  Fragments
      // are read one k-step ahead of their MFMAs.
      float a[NTW], b[KT];
#pragma unroll
      for (int i = 0; i < NTW; ++i) a[i] = qs[swz<C>(4 * lq, wbase + 16 * i + li)];
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) b[kt] = xs[swz<C>(4 * lq, 16 * kt + li)];
#pragma unroll
      for (int s2 = 0; s2 < BM / 4; ++s2) {
        float an[NTW], bn[KT];
        if (s2 + 1 < BM / 4) {
          const int mn = 4 * lq + s2 + 1;
#pragma unroll
          for (int i = 0; i < NTW; ++i) an[i] = qs[swz<C>(mn, wbase + 16 * i + li)];
#pragma unroll
          for (int kt = 0; kt < KT; ++kt) bn[kt] = xs[swz<C>(mn, 16 * kt + li)];
        }
#pragma unroll
        for (int kt = 0; kt < KT; ++kt) {
          const float b2 = b[kt] * b[kt];
#pragma unroll
          for (int i = 0; i < NTW; ++i)
            dg[i][kt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b2, dg[i][kt], 0, 0, 0);
        }
        if (s2 + 1 < BM / 4) {
#pragma unroll
          for (int i = 0; i < NTW; ++i) a[i] = an[i];
#pragma unroll
          for (int kt = 0; kt < KT; ++kt) b[kt] = bn[kt];
        }
        pin_acc<NTW * KT>(&dg[0][0]);
        __builtin_amdgcn_sched_barrier(0);
      }
      bar_wait_lgkm();  // B3
      if (t < C) {  // column sums of this tile's dx (the producing conv's bias gradient)
        const float* gsd = xs + DYO;
        const int rows = (P - m0) < (uint32_t)BM ? (int)(P - m0) : BM;
        for (int m = 0; m < rows; ++m) dxs += gsd[swz<C>(m, t)];
      }
      buf ^= 1;
    }
    // partials: slab[block][n][k] (C*C), dbeta [C], dx column sums [C]
    float* out = slab + (size_t)blockIdx.x * GDN_SLAB(C);
#pragma unroll
    for (int i = 0; i < NTW; ++i)
#pragma unroll
      for (int kt = 0; kt < KT; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          // C/D map: row (A index n) = 4lq + r, col (B index k) = li
          const int n = wbase + 16 * i + 4 * lq + r;
          const int k = 16 * kt + li;
          out[(size_t)n * C + k] = dg[i][kt][r];
        }
    if (t < C) {
      out[C * C + t] = db;
      out[C * C + C + t] = dxs;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}


// ============================================================== backward, whole split, pipelined
// gdn_bwd_x3w_kernel (C = 192, IC_MATH_SPLIT): both contractions in split arithmetic, one wave per SIMD
// (4 waves, up to 512 registers each), software-pipelined over 16-pixel tiles with ONE barrier per tile.
// Wave w owns
//   * the dx columns k in [48w, 48w+48): gamma's three split planes as MFMA A fragments in 216 VGPRs,
//     dx^T tile = gamma^T q^T on v_mfma_f32_16x16x32_bf16 (six products), so each lane's results are
//     4 consecutive channels of one pixel -- the same (pixel li, channels 48w+16j+4lg..+3) elements the
//     lane loads, runs phase A on and stores: no LDS copy-out, 16-B global loads and stores;
//   * the 96x96 dgamma quadrant (w>>1, w&1) in 144 accumulators (v_mfma_f32_32x32x16_bf16, K = the
//     tile's 16 pixels, transposed plane reads), as group B of gdn_bwd_fused_kernel<192, true>.
// Iteration for tile t (planes / x,dv slots of t in buffer cb, written one iteration earlier):
//   dx GEMM(t) interleaved with phase A(t+G) (registers -> planes and x,dv slots of buffer cb^1) |
//   loads of tile t+2G into the landing registers | dgamma GEMM(t) | epilogue(t): dx = dv + 2 x s,
//   16-B stores | barrier.
// Global loads are register-staged (the landing registers are free once phase A has consumed them);
// rows past P load row P-1 with q = dv = 0, and their dx goes to a dump slot (no branches around
// memory operations, so the compiler's waitcnt pass never waits for the stores).
// dbeta and the dx column sums (the producing conv's bias gradient) accumulate in per-lane LDS slots.
// NP = 1 (IC_MATH_BF16, config C3, round 5): the same kernel on bf16 operands -- gamma, q and x^2
// rounded to nearest even, one plane each, one product per MFMA step; XB: dx also as a compact bf16
// copy (dxb) for the previous transposed conv's input gradient (ig_kernel_b16d).
template <int C, bool INV, int NP = 3, bool XB = false>
__global__ void __launch_bounds__(256, 1)
    gdn_bwd_x3w_kernel(const float* __restrict__ x, const float* __restrict__ norm, const float* __restrict__ dy,
                       const float* __restrict__ gamma, float* __restrict__ dx,
                       float* __restrict__ slab, uint32_t P, __bf16* __restrict__ dxb = nullptr) {
  static_assert(C == 192, "4 waves x 48 dx columns, 2 x 2 dgamma quadrants of 96");
  static_assert(NP == 3 || NP == 1, "split (3 planes) or bf16 (1 plane)");
  typedef __bf16 b4 __attribute__((ext_vector_type(4)));
  typedef __bf16 b8 __attribute__((ext_vector_type(8)));
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  constexpr int BM = 16, NT = 256, K32 = C / 32;
  constexpr int PL = BM * C;        // bf16 elements per plane
  constexpr int PSET = 2 * NP * PL; // q planes then x^2 planes
  __shared__ __attribute__((aligned(16))) __bf16 pls[2 * PSET];      // 72 KB (NP 3): two plane sets
  __shared__ __attribute__((aligned(16))) floatx4v xdv[2][6][NT];     // 48 KB: x (j) and dv (3 + j) per lane
  __shared__ __attribute__((aligned(16))) floatx4v acc_s[6][NT];      // 24 KB: dbeta (j), dx column sums (3 + j)

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int li = lane & 15, lg = lane >> 4;
  const uint32_t ntiles = (P + BM - 1) / BM;
  const uint32_t G = gridDim.x;
  uint32_t tile = blockIdx.x;
  if (tile >= ntiles) return;  // whole block: before any barrier

  // gamma^T fragments: gx[p][j][s] = plane p of gamma[n = 32s + 8lg + e][k = 48w + 16j + li]
  b8 gx[NP][3][K32];
#pragma unroll
  for (int j = 0; j < 3; ++j)
#pragma unroll
    for (int s = 0; s < K32; ++s)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float gv = gamma[(size_t)(32 * s + 8 * lg + e) * C + 48 * w + 16 * j + li];
        if constexpr (NP == 1) {
          gx[0][j][s][e] = (__bf16)gv;  // round to nearest even
        } else {
          __bf16 hh, mm, ll;
          split3_bf16(gv, hh, mm, ll);
          gx[0][j][s][e] = hh;
          gx[NP - 2][j][s][e] = mm;
          gx[NP - 1][j][s][e] = ll;
        }
      }
  // the 216 gamma registers live in AGPRs (MFMA A operands may be AGPRs): the 256 arch VGPRs of the
  // wave then hold the dgamma accumulators, the landing registers and phase A
#pragma unroll
  for (int p = 0; p < NP; ++p)
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int s = 0; s < K32; ++s) asm volatile("" : "+a"(gx[p][j][s]));
#pragma unroll
  for (int k = 0; k < 6; ++k) acc_s[k][tid] = floatx4v{0.f, 0.f, 0.f, 0.f};

  // this lane's elements: pixel li of the tile, channels n0(j) = 48w + 16j + 4lg .. +3
  const int cbase = 48 * w + 4 * lg;
  floatx4v lx[3], ln[3], ld[3];  // landing registers: x, norm, dy of the next tile to run phase A on
  auto load = [&](uint32_t t) {
    const uint32_t m = min(t * BM + li, P - 1);
    const size_t o = (size_t)m * C + cbase;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      lx[j] = *(const floatx4v*)(x + o + 16 * j);
      ln[j] = *(const floatx4v*)(norm + o + 16 * j);
      ld[j] = *(const floatx4v*)(dy + o + 16 * j);
    }
  };
  auto load_j = [&](uint32_t t, int j) {
    const size_t o = (size_t)min(t * BM + li, P - 1) * C + cbase + 16 * j;
    lx[j] = *(const floatx4v*)(x + o);
    ln[j] = *(const floatx4v*)(norm + o);
    ld[j] = *(const floatx4v*)(dy + o);
  };
  // a float4 into NP planes at dst (plane stride PL): the exact split, or rounded to nearest even
  auto put_planes = [&](__bf16* dst, floatx4v v) {
    if constexpr (NP == 1) {
      *(b4*)dst = __builtin_bit_cast(b4, u32x2{ic_cvt_pk_bf16(v[0], v[1]), ic_cvt_pk_bf16(v[2], v[3])});
    } else {
      b4 h, m, l;
      split3_bf16x4(v, h, m, l);
      *(b4*)dst = h;
      *(b4*)(dst + PL) = m;
      *(b4*)(dst + 2 * PL) = l;
    }
  };
  // phase A, element group j of tile t from the landing registers into buffer b
  auto phase_a = [&](uint32_t t, int b, int j) {
    // rows past P (and a tile past the end) contribute nothing: q = dv = 0 by selects (no branch)
    const bool valid = t < ntiles && t * BM + li < P;
    const floatx4v xv = lx[j], nv = ln[j], gv = ld[j];
    floatx4v qv, dv;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float rs = __builtin_amdgcn_rsqf(nv[e]);
      const float q = INV ? 0.5f * gv[e] * xv[e] * rs : -0.5f * gv[e] * xv[e] * (rs * rs * rs);
      const float d = INV ? gv[e] * (nv[e] * rs) : gv[e] * rs;
      qv[e] = valid ? q : 0.f;
      dv[e] = valid ? d : 0.f;
    }
    __bf16* sp = pls + b * PSET + pl_off<C>(li, cbase + 16 * j);
    put_planes(sp, qv);
    put_planes(sp + NP * PL, xv * xv);
    xdv[b][j][tid] = xv;
    xdv[b][3 + j][tid] = dv;
    acc_s[j][tid] += qv;
  };

  // dgamma quadrant
  const int wm2 = w >> 1, wn2 = w & 1;
  const int tr_row = 8 * (lane >> 5) + (li >> 2);
  const int tr_col = 16 * ((lane >> 4) & 1) + 4 * (li & 3);
  auto tr8 = [&](const __bf16* plane, int c0) {
    const int c = c0 + tr_col;
    const b4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
        (__attribute__((address_space(3))) b4*)(plane + pl_off<C>(tr_row, c)));
    const b4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
        (__attribute__((address_space(3))) b4*)(plane + pl_off<C>(tr_row + 4, c)));
    return (b8)__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  };
  floatx16 dg[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) dg[i][j][e] = 0.f;

  // prologue: phase A of the first tile, loads of the second
  load(tile);
#pragma unroll
  for (int j = 0; j < 3; ++j) phase_a(tile, 0, j);
  load(tile + G < ntiles ? tile + G : tile);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  float* const dump = slab + (size_t)gridDim.x * GDN_SLAB(C) + (size_t)blockIdx.x * NT * 4;
#if X3W_STAMP
  // diagnostic build: s_memtime at four points of each of the first 160 iterations, per wave
  uint64_t* const stp = (uint64_t*)(slab + (size_t)gridDim.x * (GDN_SLAB(C) + 1024)) +
                        ((size_t)blockIdx.x * 4 + w) * 160 * 4;
  int it = 0;
#define X3W_ST(k) \
  if (lane == 0 && it < 160) stp[it * 4 + (k)] = __builtin_amdgcn_s_memtime();
#else
#define X3W_ST(k)
#endif
  for (int cb = 0; tile < ntiles; tile += G, cb ^= 1) {
    X3W_ST(0)
    const uint32_t nx = tile + G;
    const uint32_t n2 = tile + 2 * G < ntiles ? tile + 2 * G : tile;  // past the end: reload this tile
    const __bf16* sp = pls + cb * PSET;
    // dx^T GEMM(t) (k rows 48w+16j+4lg+r, pixel column li), six K steps of 32 channels; phase A(t+G)
    // part j and the loads of part j of tile t+2G run between the MFMAs of steps 2j and 2j+1
    // (one wave per SIMD: the VALU and memory instructions issue in the MFMAs' shadow only when
    // interleaved with them, sched_group_barrier below)
    floatx4v acc[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) acc[j] = floatx4v{0.f, 0.f, 0.f, 0.f};
    auto qfrag = [&](int st, b8 (&f)[NP]) {
      const int off = pl_off<C>(li, 32 * st + 8 * lg);
#pragma unroll
      for (int p = 0; p < NP; ++p) f[p] = *(const b8*)(sp + p * PL + off);
    };
    b8 fa[NP], fb[NP];
    b8 av[3][NP], bb[2][NP];  // dgamma GEMM fragments (read during the dx GEMM's last K step)
    qfrag(0, fa);
    // phase A(t+G) part pr in six slices, one between each (K step, column tile) group of six MFMAs
    floatx4v pq, pd, pxv;
    auto pa_slice = [&](int pr, int k) {
      if (X3W_ABL & 2) return;
      const bool valid = nx < ntiles && nx * BM + li < P;
      __bf16* pp = pls + (cb ^ 1) * PSET + pl_off<C>(li, cbase + 16 * pr);
      if (k < 2) {  // elements 2k, 2k+1: q, dv
        if (k == 0) pxv = lx[pr];
#pragma unroll
        for (int e = 2 * k; e < 2 * k + 2; ++e) {
          const float xv = lx[pr][e], nv = ln[pr][e], gv = ld[pr][e];
          const float rs = __builtin_amdgcn_rsqf(nv);
          const float q = INV ? 0.5f * gv * xv * rs : -0.5f * gv * xv * (rs * rs * rs);
          const float d = INV ? gv * (nv * rs) : gv * rs;
          pq[e] = valid ? q : 0.f;
          pd[e] = valid ? d : 0.f;
        }
      } else if (k == 2) {  // q's split planes
        put_planes(pp, pq);
      } else if (k == 3) {  // x^2's split planes
        put_planes(pp + NP * PL, pxv * pxv);
      } else if (k == 4) {
        xdv[cb ^ 1][pr][tid] = pxv;
        xdv[cb ^ 1][3 + pr][tid] = pd;
        acc_s[pr][tid] += pq;
      } else if (!(X3W_ABL & 1)) {  // the landing registers of part pr are free: tile t+2G's
        load_j(n2, pr);
      }
    };
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int pr = 0; pr < K32 / 2; ++pr) {
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const int st = 2 * pr + h2;
        b8 (&cur)[NP] = h2 ? fb : fa;
        b8 (&nxt)[NP] = h2 ? fa : fb;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          if (j == 0 && st + 1 < K32) qfrag(st + 1, nxt);
          if constexpr (NP == 1) {
            if (!(X3W_ABL & 8)) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gx[0][j][st], cur[0], acc[j], 0, 0, 0);
          } else if (!(X3W_ABL & 8)) {
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gx[0][j][st], cur[2], acc[j], 0, 0, 0);
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gx[1][j][st], cur[1], acc[j], 0, 0, 0);
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gx[2][j][st], cur[0], acc[j], 0, 0, 0);
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gx[0][j][st], cur[1], acc[j], 0, 0, 0);
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gx[1][j][st], cur[0], acc[j], 0, 0, 0);
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gx[0][j][st], cur[0], acc[j], 0, 0, 0);
          }
          pa_slice(pr, 3 * h2 + j);
          if (X3W_SGB) {
#pragma unroll
            for (int k = 0; k < (NP == 1 ? 1 : 6); ++k) {
              __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
              __builtin_amdgcn_sched_group_barrier(0x002, NP == 1 ? 24 : 4, 0);  // VALU
            }
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
    X3W_ST(1)
    // dgamma GEMM(t) on the quadrant, with the epilogue of tile t (dx = dv + 2 x s, stored straight
    // from the registers) between its MFMAs
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int p = 0; p < NP; ++p) av[i][p] = tr8(sp + p * PL, 96 * wm2 + 32 * i);
#pragma unroll
    for (int p = 0; p < NP; ++p) bb[0][p] = tr8(sp + (NP + p) * PL, 96 * wn2);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      if (j + 1 < 3)
#pragma unroll
        for (int p = 0; p < NP; ++p) bb[(j + 1) & 1][p] = tr8(sp + (NP + p) * PL, 96 * wn2 + 32 * (j + 1));
      const b8 (&bc)[NP] = bb[j & 1];
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        if (X3W_ABL & 4) continue;
        if constexpr (NP == 1) {
          dg[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[i][0], bc[0], dg[i][j], 0, 0, 0);
          continue;
        } else {
        dg[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[i][2], bc[0], dg[i][j], 0, 0, 0);
        dg[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[i][1], bc[1], dg[i][j], 0, 0, 0);
        dg[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[i][0], bc[2], dg[i][j], 0, 0, 0);
        dg[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[i][1], bc[0], dg[i][j], 0, 0, 0);
        dg[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[i][0], bc[1], dg[i][j], 0, 0, 0);
        dg[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[i][0], bc[0], dg[i][j], 0, 0, 0);
        }
      }
      {  // epilogue, element group j
        const uint32_t m = tile * BM + li;
        float* dst = m < P ? dx + (size_t)m * C + cbase + 16 * j : dump + tid * 4;
        const floatx4v xv = xdv[cb][j][tid], dv = xdv[cb][3 + j][tid];
        const floatx4v d = dv + 2.f * xv * acc[j];
        if (!(X3W_ABL & 16)) *(floatx4v*)dst = d;
        if constexpr (XB) {  // the bf16 copy; rows past P to the (16-B) dump slot's first 8 B
          __bf16* db = m < P ? dxb + (size_t)m * C + cbase + 16 * j : (__bf16*)(dump + tid * 4);
          *(b4*)db = __builtin_bit_cast(b4, u32x2{ic_cvt_pk_bf16(d[0], d[1]), ic_cvt_pk_bf16(d[2], d[3])});
        }
        acc_s[3 + j][tid] += d;
      }
      if (X3W_SGB) {
#pragma unroll
        for (int k = 0; k < (NP == 1 ? 3 : 18); ++k) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
          if (k < 6) __builtin_amdgcn_sched_group_barrier(0x100, NP == 1 ? 2 : 1, 0);  // DS read (the next bb)
          __builtin_amdgcn_sched_group_barrier(0x002, NP == 1 ? 6 : 2, 0);  // VALU
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    X3W_ST(2)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    X3W_ST(3)
#if X3W_STAMP
    ++it;
#endif
  }
#undef X3W_ST
  // partials: dgamma quadrant, then dbeta and the dx column sums summed over the 16 pixels li in order
  float* out = slab + (size_t)blockIdx.x * GDN_SLAB(C);
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      // C/D map of the 32x32 MFMA: row (A index n) = (reg&3) + 8(reg>>2) + 4h, col (B index k) = lane&31
      const int n = 96 * wm2 + 32 * i + (reg & 3) + 8 * (reg >> 2) + 4 * h;
#pragma unroll
      for (int j = 0; j < 3; ++j) out[(size_t)n * C + 96 * wn2 + 32 * j + r] = dg[i][j][reg];
    }
  for (int k = tid; k < 2 * C; k += NT) {
    // k < C: dbeta[k]; C <= k < 2C: column sum of channel k - C.  Channel n lives in lane
    // (li, lg = (n % 16) / 4) of wave n / 48, slot j = (n % 48) / 16, element n % 4.
    const int n = k < C ? k : k - C, kind = k < C ? 0 : 3;
    const int wv = n / 48, j = (n % 48) / 16, lgn = (n % 16) / 4, e = n % 4;
    float sum = 0.f;
    for (int l = 0; l < 16; ++l) sum += acc_s[kind + j][64 * wv + 16 * lgn + l][e];
    out[C * C + k] = sum;
  }
}


// fixed-order sum of the per-block partials
// 64 elements x 4 groups of partials per block; each group sums a quarter of
// the partials with eight loads in flight, the quarters combine in LDS in a
// fixed order
__global__ void __launch_bounds__(256) gdn_slab_reduce_kernel(const float* __restrict__ slab, int nb, int C,
                                                              float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                              float* __restrict__ dxsum) {
  __shared__ float part[4][64];
  const int stride = GDN_SLAB(C);
  const int e = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + e;
  const int q = (nb + 3) >> 2, b0 = grp * q, b1 = min(nb, b0 + q);
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (i < stride) {
    const float* src = slab + i;
    int b = b0;
    for (; b + 7 < b1; b += 8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += src[(size_t)(b + j) * stride];
    }
    for (int j = 0; b < b1; ++b, ++j) a[j] += src[(size_t)b * stride];
  }
  part[grp][e] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  __syncthreads();
  if (grp == 0 && i < stride) {
    const float v = (part[0][e] + part[1][e]) + (part[2][e] + part[3][e]);
    if (i < C * C) {
      if (dgamma) dgamma[i] = v;
    } else if (i < C * C + C) {
      if (dbeta) dbeta[i - C * C] = v;
    } else if (dxsum) {
      dxsum[i - C * C - C] = v;
    }
  }
}

constexpr int FWD_BM = 16;

template <int C>
int gdn_fwd_fused_launch(const float* x, const float* gamma, const float* beta, int inverse, float* y, float* norm,
                         long long P, hipStream_t s) {
  const long long ntiles = (P + FWD_BM - 1) / FWD_BM;
  long long grid = ntiles < 512 ? ntiles : 512;  // two blocks per CU
  if (grid < 1) return IC_OK;
  hipLaunchKernelGGL((gdn_fwd_fused_kernel<C, FWD_BM>), dim3((unsigned)grid), dim3(64 * fwd_waves<C>()), 0, s, x, gamma, beta,
                     inverse, y, norm, (uint32_t)P);
  IC_CHECK_LAUNCH();
  return IC_OK;
}

int bwd_grid(long long P) {
  const long long ntiles = (P + 15) / 16;
  return (int)(ntiles < 256 ? ntiles : 256);
}

template <int C, bool X3 = false, bool BF = false, bool XB = false, bool RN = false>
int gdn_bwd_fused_launch(const float* x, const float* norm, const float* dy, const float* gamma, int inverse,
                         float* dx, float* dgamma, float* dbeta, float* dxsum, long long P, float* slab,
                         hipStream_t s, void* dxb = nullptr, const float* beta = nullptr) {
  const int grid = bwd_grid(P);
  if (grid < 1) return IC_OK;
  hipLaunchKernelGGL((gdn_bwd_fused_kernel<C, X3, BF, XB, RN>), dim3(grid), dim3(512), 0, s, x, norm, dy, gamma,
                     inverse, dx, slab, (uint32_t)P, (__bf16*)dxb, beta);
  IC_CHECK_LAUNCH();
  const int stride = GDN_SLAB(C);
  hipLaunchKernelGGL(gdn_slab_reduce_kernel, dim3((stride + 63) / 64), dim3(256), 0, s, slab, grid, C, dgamma,
                     dbeta, dxsum);
  IC_CHECK_LAUNCH();
  return IC_OK;
}

}  // namespace

// NHWC-dense (channel stride 1, pixel stride C), 16-B aligned, C in {64,128,192}
bool gdn_fused_ok(const float* x, const float* y, const float* norm, int C, long long sc, long long sw, long long sh,
                  long long sn, int H, int W, long long P) {
  if (!(C == 64 || C == 128 || C == 192)) return false;
  if (sc != 1 || sw != C || sh != (long long)W * C || sn != (long long)H * W * C) return false;
  if (P >= (1LL << 31) || P < 1) return false;
  auto a16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  return a16(x) && a16(y) && a16(norm);
}

int gdn_fwd_fused(const float* x, const float* gamma, const float* beta, int inverse, float* y, float* norm, int C,
                  long long P, hipStream_t s, int split, void* yb) {
  if (!norm && !(split == 2 && C == 192)) return IC_ERR_ARG;  // only the bf16 kernel can leave norm out
  if (split && C == 192) {  // split: 1 = fp32 by the exact split, 2 = bf16 operands (config C3)
    const long long ntiles = (P + 31) / 32;
    const long long grid = ntiles < 256 ? ntiles : 256;  // one block per CU
    if (grid < 1) return IC_OK;
    if (split == 2 && !norm && yb)  // norm recomputed by the backward (round 6)
      hipLaunchKernelGGL((gdn_fwd_x3s_kernel<192, 1, true, false>), dim3((unsigned)grid), dim3(768), 0, s, x, gamma,
                         beta, inverse, y, norm, (uint32_t)P, (__bf16*)yb);
    else if (split == 2 && !norm)
      hipLaunchKernelGGL((gdn_fwd_x3s_kernel<192, 1, false, false>), dim3((unsigned)grid), dim3(768), 0, s, x, gamma,
                         beta, inverse, y, norm, (uint32_t)P);
    else if (split == 2 && yb)
      hipLaunchKernelGGL((gdn_fwd_x3s_kernel<192, 1, true>), dim3((unsigned)grid), dim3(768), 0, s, x, gamma, beta,
                         inverse, y, norm, (uint32_t)P, (__bf16*)yb);
    else if (split == 2)
      hipLaunchKernelGGL((gdn_fwd_x3s_kernel<192, 1>), dim3((unsigned)grid), dim3(768), 0, s, x, gamma, beta, inverse,
                         y, norm, (uint32_t)P);
    else
      hipLaunchKernelGGL((gdn_fwd_x3s_kernel<192>), dim3((unsigned)grid), dim3(768), 0, s, x, gamma, beta, inverse, y,
                         norm, (uint32_t)P);
    IC_CHECK_LAUNCH();
    return IC_OK;
  }
  switch (C) {
    case 64: return gdn_fwd_fused_launch<64>(x, gamma, beta, inverse, y, norm, P, s);
    case 128: return gdn_fwd_fused_launch<128>(x, gamma, beta, inverse, y, norm, P, s);
    case 192: return gdn_fwd_fused_launch<192>(x, gamma, beta, inverse, y, norm, P, s);
    default: return IC_ERR_ARG;
  }
}

// per-block partial slabs, then (gdn_bwd_x3w_kernel) one 4 KB dump slot per block for the dx of rows past P
size_t gdn_bwd_fused_ws(int C, long long P) {
  return (size_t)bwd_grid(P) * (GDN_SLAB(C) + 1024) * sizeof(float) + (X3W_STAMP ? (size_t)256 * 4 * 160 * 4 * 8 : 0);
}

int gdn_bwd_fused(const float* x, const float* norm, const float* dy, const float* gamma, int inverse, float* dx,
                  float* dgamma, float* dbeta, int C, long long P, void* ws, hipStream_t s, int split, float* dxsum,
                  void* dxb, const float* beta) {
  float* slab = (float*)ws;
  if (split == 2 && C == 192 && !norm) {  // norm recomputed from x, gamma and beta (round 6)
    if (!beta) return IC_ERR_ARG;
    if (dxb)
      return gdn_bwd_fused_launch<192, true, true, true, true>(x, norm, dy, gamma, inverse, dx, dgamma, dbeta, dxsum,
                                                               P, slab, s, dxb, beta);
    return gdn_bwd_fused_launch<192, true, true, false, true>(x, norm, dy, gamma, inverse, dx, dgamma, dbeta, dxsum, P,
                                                              slab, s, nullptr, beta);
  }
  if (!norm) return IC_ERR_ARG;
  if (split == 2 && C == 192 && dxb)
    return gdn_bwd_fused_launch<192, true, true, true>(x, norm, dy, gamma, inverse, dx, dgamma, dbeta, dxsum, P, slab,
                                                       s, dxb);
  if (split == 2 && C == 192)
    return gdn_bwd_fused_launch<192, true, true>(x, norm, dy, gamma, inverse, dx, dgamma, dbeta, dxsum, P, slab, s);
  if (split && C == 192) {  // split arithmetic: the pipelined one-wave kernel
    const int grid = bwd_grid(P);
    if (grid < 1) return IC_OK;
    if (inverse)
      hipLaunchKernelGGL((gdn_bwd_x3w_kernel<192, true>), dim3(grid), dim3(256), 0, s, x, norm, dy, gamma, dx, slab,
                         (uint32_t)P);
    else
      hipLaunchKernelGGL((gdn_bwd_x3w_kernel<192, false>), dim3(grid), dim3(256), 0, s, x, norm, dy, gamma, dx, slab,
                         (uint32_t)P);
    IC_CHECK_LAUNCH();
    hipLaunchKernelGGL(gdn_slab_reduce_kernel, dim3((GDN_SLAB(192) + 63) / 64), dim3(256), 0, s, slab, grid, 192,
                       dgamma, dbeta, dxsum);
    IC_CHECK_LAUNCH();
    return IC_OK;
  }
  switch (C) {
    case 64: return gdn_bwd_fused_launch<64>(x, norm, dy, gamma, inverse, dx, dgamma, dbeta, dxsum, P, slab, s);
    case 128: return gdn_bwd_fused_launch<128>(x, norm, dy, gamma, inverse, dx, dgamma, dbeta, dxsum, P, slab, s);
    case 192: return gdn_bwd_fused_launch<192>(x, norm, dy, gamma, inverse, dx, dgamma, dbeta, dxsum, P, slab, s);
    default: return IC_ERR_ARG;
  }
}
