// The two image-edge convolutions (3-channel image <-> 192-channel maps),
// which dominate no FLOP count but move the largest tensors of the step:
//
//   edge_conv  : y[p][n] = bias[n] + sum_k xcol[p][k] * wp[n][k]
//                conv 3->192 5x5 s2 (g_a.0 forward; also the g_s.6 transposed
//                conv's dgrad, which is the same direct gather)
//   edge_wgrad : dW[g][k] = sum_p G[p][g] * xcol[p][k]   (+ bias column)
//                g_a.0 wgrad (G = dy, X = x) and g_s.6 wgrad (G = x, X = dy)
//
// with xcol[p][k], k = t*C + c, the (tap, channel) patch of the few-channel
// image X (NCHW, rows contiguous) at output pixel p.  Instead of materialising
// xcol in HBM (im2col: 100 B per pixel written and read back), each work unit
// = one 64-pixel segment of an output row stages the C x k x (63*s+k) input
// patch it needs in LDS (zero outside the image) and the MFMA operand for
// (pixel m, column k) is patch[off_k + s*m] — a table of per-lane offsets.
//
// Both kernels are persistent (a few blocks per CU loop over the units) and
// use v_mfma_f32_16x16x4_f32; wave w owns a C_out/4 channel slice.
//   edge_conv : weights live in VGPRs as B fragments for the whole launch;
//               output rows are written NHWC straight from the accumulators.
//   edge_wgrad: the G tile of the unit (64 pixels x 192 channels, one
//               contiguous NHWC run) arrives by LDS-DMA (row-swizzled, as in
//               gdn_fused.hip); dW accumulates in VGPRs across units and each
//               block writes one partial that a fixed-order kernel reduces.
//               An extra all-ones column k = T*C turns the same MFMAs into
//               the bias gradient sum_p G[p][g] when G is dy (conv wgrad).
#include "../../include/imgcomp.h"
#include "gemm.h"

namespace {

#ifndef EC_SPLIT
#define EC_SPLIT 1  // split arithmetic (IC_MATH_SPLIT) in the edge conv (edge_conv_x3_kernel)
#endif
#ifndef EW_SPLIT
#define EW_SPLIT 1  // split arithmetic (IC_MATH_SPLIT) in edge_wgrad_kernel
#endif
constexpr int SEG = 64;        // output pixels per work unit (one row segment)
constexpr int KMAX = 100;      // T*C <= 25 taps x 4 channels
constexpr int PMAX = 4 * 5 * (63 * 2 + 5);  // patch floats: C x k x (63 s + k)

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef const __attribute__((address_space(1))) void* gbl_ptr_t;

__device__ __attribute__((aligned(16))) float edge_zero_page[4];
__device__ __attribute__((aligned(16))) float edge_store_dump[128];  // written, never read
#ifndef EC_STAMP
#define EC_STAMP 0  // diagnostic build: s_memtime at six points of each unit of edge_conv_x3_kernel, per wave
#endif
#if EC_STAMP
constexpr int EC_ST_IT = 40, EC_ST_N = 8;
__device__ unsigned long long edge_stamps[256 * 8 * EC_ST_IT * EC_ST_N];
#endif

struct EdgeGeom {
  const float* x;            // few-channel image, NCHW strides (sw == 1)
  long long sn, sc, sh;
  int N, C, H, W;            // input image
  int Ho, Wo;                // output grid
  int k, stride, pad;
  int PW;                    // patch row length = (SEG-1)*stride + k
  int TC;                    // T*C real columns
  int units_per_row;         // ceil(Wo / SEG)
  long long units;
};

// the patch of unit u: patch[(c*k + ky)*PW + j] = x[n][c][iy0+ky][ix0+j] (0 outside
// the image).  Loaded into registers first (pr) and written to LDS later, so
// the global-load latency hides behind the current unit's MFMAs.
constexpr int PREG = (PMAX + 255) / 256;  // per thread of a 256-thread stager

// This thread's patch elements i = tid + NT q (NT stager threads), decomposed once per launch
// (the divisions by the runtime patch width and kernel size are not redone
// per unit) and packed into one register each: (c << 12) | (ky << 9) | j, or
// -1 for i >= C*k*PW.
template <int NT = 256>
struct EdgePatchMapT {
  static constexpr int R = (PMAX + NT - 1) / NT;
  int pk[R];
};
typedef EdgePatchMapT<256> EdgePatchMap;
template <int NT>
__device__ __forceinline__ void edge_patch_map(const EdgeGeom& g, EdgePatchMapT<NT>& m, int tid) {
  const int tot = g.C * g.k * g.PW;
#pragma unroll
  for (int q = 0; q < EdgePatchMapT<NT>::R; ++q) {
    const int i = tid + NT * q;
    const int row = i / g.PW, j = i - (i / g.PW) * g.PW;
    const int c = row / g.k, ky = row - (row / g.k) * g.k;
    m.pk[q] = i < tot ? (c << 12) | (ky << 9) | j : -1;
  }
}
// Branch-free (every lane loads and stores; out-of-image elements load the zero page, elements
// past the patch store their zero onto its first zero-run slot): with no exec-masked memory
// operations, and called unconditionally, the waitcnt pass tracks the loads exactly instead of
// waiting (vmcnt) at the loop head for everything in flight, the previous unit's output stores
// included (r03zl).  Unit and image offsets in 32 bits (edge_geom bounds them).
template <int NT>
__device__ __forceinline__ void edge_patch_load(const EdgeGeom& g, const EdgePatchMapT<NT>& m, long long u,
                                                float (&pr)[EdgePatchMapT<NT>::R]) {
  const unsigned uu = (unsigned)u, upr = (unsigned)g.units_per_row, ho = (unsigned)g.Ho;
  const unsigned r = uu / upr;
  const int seg = (int)(uu - r * upr);
  const unsigned n = r / ho;
  const int oy = (int)(r - n * ho);
  const int iy0 = oy * g.stride - g.pad, ix0 = seg * SEG * g.stride - g.pad;
  const float* xb = g.x + (long long)n * g.sn;
  const int sc = (int)g.sc, sh = (int)g.sh;
#pragma unroll
  for (int q = 0; q < EdgePatchMapT<NT>::R; ++q) {
    const int pk = m.pk[q];
    const int iy = iy0 + ((pk >> 9) & 7), ix = ix0 + (pk & 511);
    const bool ok = pk >= 0 && (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W;
    const int off = (pk >> 12) * sc + iy * sh + ix;
    pr[q] = *(ok ? xb + off : (const float*)edge_zero_page);  // no use of the value before the store
  }
}

template <int NT = 256>
__device__ __forceinline__ void edge_patch_store(const EdgeGeom& g, const float (&pr)[EdgePatchMapT<NT>::R],
                                                 float* patch, int tid) {
  const int tot = g.C * g.k * g.PW;
#pragma unroll
  for (int q = 0; q < EdgePatchMapT<NT>::R; ++q) {
    const int i = tid + NT * q;
    patch[i < tot ? i : tot] = pr[q];  // pr = 0 past the patch
  }
}

// The patch of unit u straight into LDS (global_load_lds_dword: each wave-instruction writes 64
// consecutive floats at M0 + 4 lane), element i = tid + 512 q as edge_patch_load / _store<512> place
// it; instructions whose 64 elements all lie past the patch are skipped (wave-uniform), the lanes of a
// partial one load the zero page into the zero run that follows the patch.  Counted by vmcnt like any
// load; the caller waits for it.
__device__ __forceinline__ void edge_patch_dma(const EdgeGeom& g, const EdgePatchMapT<512>& m, long long u,
                                               uint32_t buf_lds, int w) {
  const unsigned uu = (unsigned)u, upr = (unsigned)g.units_per_row, ho = (unsigned)g.Ho;
  const unsigned r = uu / upr;
  const int seg = (int)(uu - r * upr);
  const unsigned n = r / ho;
  const int oy = (int)(r - n * ho);
  const int iy0 = oy * g.stride - g.pad, ix0 = seg * SEG * g.stride - g.pad;
  const float* xb = g.x + (long long)n * g.sn;
  const int sc = (int)g.sc, sh = (int)g.sh;
  const int tot = g.C * g.k * g.PW;
#pragma unroll
  for (int q = 0; q < EdgePatchMapT<512>::R; ++q) {
    if (64 * w + 512 * q >= tot) break;
    const int pk = m.pk[q];
    const int iy = iy0 + ((pk >> 9) & 7), ix = ix0 + (pk & 511);
    const bool ok = pk >= 0 && (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W;
    const float* src = ok ? xb + ((pk >> 12) * sc + iy * sh + ix) : (const float*)edge_zero_page;
    const uint32_t dst = __builtin_amdgcn_readfirstlane(buf_lds + 4u * (uint32_t)(64 * w + 512 * q));
    uint32_t save;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dword %1, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(save)
        : "v"(src), "s"(dst)
        : "memory");
  }
}

// LDS offset of column k inside the patch (pixel 0); columns >= TC read the
// zero run after the patch; column TC reads the ones run when `ones`
__device__ __forceinline__ int edge_koff(const EdgeGeom& g, int k, int zero_off, int ones_off, bool ones) {
  if (k < g.TC) {
    const int t = k / g.C, c = k - (k / g.C) * g.C;
    const int ky = t / g.k, kx = t - (t / g.k) * g.k;
    return (c * g.k + ky) * g.PW + kx;
  }
  return (ones && k == g.TC) ? ones_off : zero_off;
}

// ------------------------------------------------------------------ conv
// y NHWC (channel stride 1, pixel stride ys_w), Cout = 64*NTW*... : wave slice = Cout/4
#ifndef EDGE_CONV_PER_CU
#define EDGE_CONV_PER_CU 2
#endif
template <int COUT>
__global__ void __launch_bounds__(256, EDGE_CONV_PER_CU)
    edge_conv_kernel(const EdgeGeom g, const float* __restrict__ wp, int Kp, const float* __restrict__ bias,
                     int relu, float* __restrict__ y, long long ys_n, long long ys_h, long long ys_w) {
  constexpr int NTW = COUT / 64;
  constexpr int KSMAX = (KMAX + 3) / 4;
  __shared__ __attribute__((aligned(16))) float lds[2 * (PMAX + 2 * SEG * 2)];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int li = lane & 15, lq = lane >> 4;
  const int nbase = w * (COUT / 4);
  const int KS = (g.TC + 3) / 4;
  const int PSZ = g.C * g.k * g.PW;
  const int zero_off = PSZ;  // 2*SEG*stride zeros follow the patch
  const int bufsz = PMAX + 2 * SEG * 2;

  // weights as B fragments: bfr[j][s] = wp[n = nbase+16j+li][k = 4s+lq]
  float bfr[NTW][KSMAX];
  int koff[KSMAX];
#pragma unroll
  for (int s = 0; s < KSMAX; ++s) {
    const int kk = 4 * s + lq;
    koff[s] = edge_koff(g, kk, zero_off, zero_off, false);
#pragma unroll
    for (int j = 0; j < NTW; ++j) bfr[j][s] = (s < KS && kk < Kp) ? wp[(size_t)(nbase + 16 * j + li) * Kp + kk] : 0.f;
  }
  // D = W * patch^T (weights as the A operand): lane (li, lq) then holds four
  // consecutive output channels n = nbase + 16j + 4lq + r of pixel li, so each
  // (pixel, channel quad) leaves as one 16-B store
  floatx4v bv[NTW];
#pragma unroll
  for (int j = 0; j < NTW; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[j][r] = bias ? bias[nbase + 16 * j + 4 * lq + r] : 0.f;
  // zero runs after both patch buffers
  for (int i = tid; i < 2 * SEG * 2; i += 256) {
    lds[PSZ + i] = 0.f;
    lds[bufsz + PSZ + i] = 0.f;
  }

  EdgePatchMap pm;
  edge_patch_map(g, pm, tid);
  long long u = blockIdx.x;
  int buf = 0;
  float pr[PREG];
  if (u < g.units) {
    edge_patch_load(g, pm, u, pr);
    edge_patch_store(g, pr, lds, tid);
  }
  for (; u < g.units; u += gridDim.x) {
    __syncthreads();  // patch `buf` complete; everyone is done with buf^1
    const long long un = u + gridDim.x;
    if (un < g.units) edge_patch_load(g, pm, un, pr);
    const float* patch = lds + buf * bufsz;
    floatx4v acc[SEG / 16][NTW];
#pragma unroll
    for (int mt = 0; mt < SEG / 16; ++mt)
#pragma unroll
      for (int j = 0; j < NTW; ++j) acc[mt][j] = floatx4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KSMAX; ++s) {
      if (s < KS) {
#pragma unroll
        for (int mt = 0; mt < SEG / 16; ++mt) {
          const float a = patch[koff[s] + g.stride * (16 * mt + li)];
#pragma unroll
          for (int j = 0; j < NTW; ++j)
            acc[mt][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(bfr[j][s], a, acc[mt][j], 0, 0, 0);
        }
      }
    }
    // the next patch into the free buffer before the epilogue's global stores
    // (waiting for its loads then never waits for stores)
    if (un < g.units) edge_patch_store(g, pr, lds + (buf ^ 1) * bufsz, tid);
    // epilogue: C/D map row n = 4lq + r (channel), col = li (pixel 16mt + li)
    const int seg = (int)(u % g.units_per_row);
    const long long rr = u / g.units_per_row;
    const int oy = (int)(rr % g.Ho);
    const int n = (int)(rr / g.Ho);
    const int ox0 = seg * SEG;
    float* yb = y + n * ys_n + (long long)oy * ys_h + nbase + 4 * lq;
#pragma unroll
    for (int mt = 0; mt < SEG / 16; ++mt) {
      const int ox = ox0 + 16 * mt + li;
      if (ox < g.Wo) {
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
          floatx4v v = acc[mt][j] + bv[j];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = (relu && !(v[r] > 0.f)) ? 0.f : v[r];  // branch-free ReLU
          *(floatx4v*)(yb + (long long)ox * ys_w + 16 * j) = v;
        }
      }
    }
    buf ^= 1;
  }
}

// ------------------------------------------------------------------ conv, split
// IC_MATH_SPLIT: fp32 by the exact three-term bf16 split on v_mfma_f32_16x16x32_bf16
// (six products per MAC), T*C <= 96 (three 32-wide k-steps).  One block of 8 waves per CU;
// wave w owns channel slice w & 3 (its split weights held as A fragments in 108 VGPRs for the
// launch) and m-tiles 2 (w >> 2), +1 of every unit.  The B operand of unit u — im2col of its
// patch, [pixel 64][k 96], split into three bf16 planes — is built once per unit by all 512
// threads (four consecutive k of one pixel per thread and pass: four patch reads, one paired
// split, three 8-B stores) one unit ahead of the MFMAs, into two plane buffers (16-B chunks
// XOR 2 on pixels with bit 3 set: conflict-free fragment reads), so each fragment is three
// ds_read_b128 and the split is done once per value instead of once per wave and tap that
// reads it (the per-wave gather-and-split cost 0.12 of 0.20 ms, r03zb; now 0.17 ms).
// Patches run two units ahead of the MFMAs (all 8 waves load them into registers and store them
// into two patch buffers); one barrier per unit.  The output leaves in one burst per unit after
// the MFMAs: streaming it out under them (one store per MFMA group, or two 4-wave blocks per CU
// drifting apart, or waves 4-7 storing a phase late) measured slower (r03zf-r03zj).
constexpr int EC3_S = 3;
constexpr int EC3_KP = 32 * EC3_S;       // k columns of the B planes (96)
constexpr int EC3_PL = SEG * EC3_KP;     // bf16 per plane
// NP = 1 (IC_MATH_BF16, config C3): bf16 operands (weights and patch values rounded to nearest
// even), one plane, one product per tile and k-step, fp32 accumulation.
// SC: the k-step count S = ceil(T*C / 32) when known at compile time (3: the 3-channel 5x5 edges of
// every config), 0 = read from the geometry.  A compile-time S leaves no branch between the k-steps'
// MFMA groups, so the next k-step's fragment reads issue under the current one's MFMAs.
template <int COUT, int NP = 3, int SC = 0>
__global__ void __launch_bounds__(512, 1)
    edge_conv_x3_kernel(const EdgeGeom g, const float* __restrict__ wp, int Kp, const float* __restrict__ bias,
                        int relu, float* __restrict__ y, long long ys_n, long long ys_h, long long ys_w) {
  typedef __bf16 eb4 __attribute__((ext_vector_type(4)));
  typedef __bf16 eb8 __attribute__((ext_vector_type(8)));
  static_assert(NP == 3 || NP == 1, "split (3 planes) or bf16 (1 plane)");
  constexpr int NTW = COUT / 64;
  __shared__ __attribute__((aligned(16))) __bf16 bpl[2 * NP * EC3_PL];  // two units' B planes
  __shared__ __attribute__((aligned(16))) float lds[2 * (PMAX + 2 * SEG * 2)];  // two patches
  __shared__ __attribute__((aligned(16))) float bl[COUT];  // bias (read per unit: frees 4 NTW VGPRs)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int li = lane & 15, lq = lane >> 4;
  const int nbase = (w & 3) * (COUT / 4);
  const int mt0 = 2 * (w >> 2);
  const int S = SC ? SC : (g.TC + 31) / 32;
  const int PSZ = g.C * g.k * g.PW;
  const int zero_off = PSZ;
  const int bufsz = PMAX + 2 * SEG * 2;

  // split weights as A fragments: aw[part][sx][j] = plane part of wp[n = nbase + 16 j + li][32 sx + 8 lq .. + 7].
  // All 72 loads first, unconditional (index clamped into the row), the zero fill after: a load under a
  // per-element condition became a branch and a vmcnt(0) wait each, 72 L2 round trips in series per block
  float wv[EC3_S][NTW][8];
#pragma unroll
  for (int sx = 0; sx < EC3_S; ++sx)
#pragma unroll
    for (int j = 0; j < NTW; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e)
        wv[sx][j][e] = wp[(size_t)(nbase + 16 * j + li) * Kp + min(32 * sx + 8 * lq + e, Kp - 1)];
  eb8 aw[NP][EC3_S][NTW];
#pragma unroll
  for (int sx = 0; sx < EC3_S; ++sx)
#pragma unroll
    for (int j = 0; j < NTW; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int kq = 32 * sx + 8 * lq + e;
        const float v = (sx < S && kq < Kp) ? wv[sx][j][e] : 0.f;
        if constexpr (NP == 1) {
          aw[0][sx][j][e] = (__bf16)v;  // round to nearest even
        } else {
          __bf16 hh, mm, ll;
          split3_bf16(v, hh, mm, ll);
          aw[0][sx][j][e] = hh;
          aw[NP - 2][sx][j][e] = mm;
          aw[NP - 1][sx][j][e] = ll;
        }
      }
  // plane build assignment: groups gi = tid + 512 q (q < 3) = (pixel gi / 24, k quad gi % 24)
  int bkoff[3][4], bdst[3];  // patch offsets of the group's 4 k at its pixel; plane offset
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int gi = tid + 512 * q;
    const int p = gi / 24, kq = gi - 24 * (gi / 24);
#pragma unroll
    for (int e = 0; e < 4; ++e) bkoff[q][e] = edge_koff(g, 4 * kq + e, zero_off, zero_off, false) + g.stride * p;
    const int c16 = kq >> 1;
    bdst[q] = p * EC3_KP + 8 * (c16 ^ (((p >> 3) & 1) << 1)) + 4 * (kq & 1);
  }
  for (int i = tid; i < COUT; i += 512) bl[i] = bias ? bias[i] : 0.f;
  for (int i = tid; i < 2 * SEG * 2; i += 512) {
    lds[PSZ + i] = 0.f;
    lds[bufsz + PSZ + i] = 0.f;
  }
  auto build = [&](const float* patch, __bf16* planes) {
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const floatx4v x = {patch[bkoff[q][0]], patch[bkoff[q][1]], patch[bkoff[q][2]], patch[bkoff[q][3]]};
      if constexpr (NP == 1) {
        typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
        *(eb4*)(planes + bdst[q]) = __builtin_bit_cast(eb4, u32x2{ic_cvt_pk_bf16(x[0], x[1]), ic_cvt_pk_bf16(x[2], x[3])});
      } else {
        eb4 h, m, l;
        split3_bf16x4(x, h, m, l);
        *(eb4*)(planes + bdst[q]) = h;
        *(eb4*)(planes + EC3_PL + bdst[q]) = m;
        *(eb4*)(planes + 2 * EC3_PL + bdst[q]) = l;
      }
    }
  };

  // all 512 threads stage patches, unconditionally: units past the end load the last one (into a
  // buffer nothing reads)
  EdgePatchMapT<512> pm;
  edge_patch_map(g, pm, tid);
  const long long u0 = blockIdx.x, gs = gridDim.x, ulast = g.units - 1;
  const int wu = __builtin_amdgcn_readfirstlane(w);  // wave index, known uniform (the DMA's skip is a scalar branch)
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(__attribute__((address_space(3))) float*)lds);
  // prologue: patch(u0) -> buffer 0, planes(u0) -> plane buffer 0, patch(u0 + gs) -> buffer 1
  edge_patch_dma(g, pm, u0, lds0, wu);
  edge_patch_dma(g, pm, min(u0 + gs, ulast), lds0 + 4u * (uint32_t)bufsz, wu);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  build(lds, bpl);
  floatx4v ob[2][NTW];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int j = 0; j < NTW; ++j) ob[t][j] = floatx4v{0.f, 0.f, 0.f, 0.f};
  int it = 0;
#if EC_STAMP
  unsigned long long* const stp = edge_stamps + ((size_t)(blockIdx.x & 255) * 8 + w) * EC_ST_IT * EC_ST_N;
#define EC_ST(k) \
  if (lane == 0 && it < EC_ST_IT) stp[it * EC_ST_N + (k)] = __builtin_amdgcn_s_memtime();
#else
#define EC_ST(k)
#endif
  for (long long u = u0; u < g.units; u += gs, ++it) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int j = 0; j < NTW; ++j) asm volatile("" ::"v"(ob[t][j]));  // keeps `ob` apart from `acc`
    EC_ST(0)
    // planes(u) and patch(u + gs) are in LDS; every read of plane buffer (it + 1) & 1 and patch
    // buffer it & 1 (the previous iteration's) is done
    __syncthreads();
    EC_ST(1)
    // patch(u + 2 gs) into the buffer patch(u) occupied (its planes were built last iteration)
    edge_patch_dma(g, pm, min(u + 2 * gs, ulast), lds0 + 4u * (uint32_t)((it & 1) * bufsz), wu);
    EC_ST(2)
    build(lds + ((it + 1) & 1) * bufsz, bpl + ((it + 1) & 1) * NP * EC3_PL);
    EC_ST(3)
    const __bf16* planes = bpl + (it & 1) * NP * EC3_PL;
    const int seg = (int)(u % g.units_per_row);
    const long long rr = u / g.units_per_row;
    float* yb = y + (rr / g.Ho) * ys_n + (rr % g.Ho) * ys_h + nbase + 4 * lq;
    // m-tile t outermost: t = 0's output stores issue while t = 1's MFMAs run (EC_T_OUTER; 0: all
    // MFMAs, then one burst of 2 NTW stores)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      floatx4v acc[NTW];
#pragma unroll
      for (int j = 0; j < NTW; ++j) acc[j] = floatx4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int sx = 0; sx < EC3_S; ++sx) {
        if (sx < S) {
          const int p = 16 * (mt0 + t) + li;
          const int off = p * EC3_KP + 8 * ((4 * sx + lq) ^ (((p >> 3) & 1) << 1));
          eb8 bf[NP];
#pragma unroll
          for (int q = 0; q < NP; ++q) bf[q] = *(const eb8*)(planes + q * EC3_PL + off);
          if constexpr (NP == 1) {
#pragma unroll
            for (int j = 0; j < NTW; ++j)
              acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aw[0][sx][j], bf[0], acc[j], 0, 0, 0);
          } else {
            // the six products, smallest first (a dependent MFMA issues back to back)
            constexpr int PA[6] = {2, 1, 0, 1, 0, 0}, PB[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
            for (int j = 0; j < NTW; ++j)
#pragma unroll
              for (int pr6 = 0; pr6 < 6; ++pr6)
                acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aw[PA[pr6]][sx][j], bf[PB[pr6]], acc[j], 0, 0, 0);
          }
        }
      }
      // epilogue of m-tile t: C/D map row n = 4lq + r (channel), col = li (pixel 16 (mt0 + t) + li).  The
      // stored values stay in registers of their own (`ob`, live across the unit loop): overwriting a
      // store's data registers waits for the store
#pragma unroll
      for (int j = 0; j < NTW; ++j) {
        const floatx4v bv = *(const floatx4v*)(bl + nbase + 16 * j + 4 * lq);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float x = acc[j][r] + bv[r];
          ob[t][j][r] = (relu && !(x > 0.f)) ? 0.f : x;  // branch-free ReLU
        }
      }
      EC_ST(4)
      const int ox = seg * SEG + 16 * (mt0 + t) + li;
      // branch-free: pixels past the row store into a dump slot (no exec-masked memory operation,
      // so the waitcnt pass counts the stores exactly)
      float* dst = ox < g.Wo ? yb + (long long)ox * ys_w : edge_store_dump + 48 * t;
#pragma unroll
      for (int j = 0; j < NTW; ++j) *(floatx4v*)(dst + 16 * j) = ob[t][j];
    }
    EC_ST(5)
    // the patch DMA issued at the top of this iteration must have landed before the barrier (the next
    // iteration builds from it); the 2 NTW output stores issued after it may stay in flight.  vmcnt
    // counts loads and stores in issue order: with the round-5 register-staged patch the compiler's
    // wait for the patch loads (vmcnt(0) at the loop's merge) also waited for the previous unit's
    // 48 KB of output stores (round 6: g_a.0 fwd 0.174 -> 0.170 ms alternating, r09e; the kernel is
    // bound by its MFMA and store energy rather than by that wait: profiles/r09c_x3d_edge_ablations.txt)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NTW + (EC_STAMP ? 4 : 0)) : "memory");
    EC_ST(6)
  }
#undef EC_ST
}

// ------------------------------------------------------------------ wgrad
// G NHWC-dense [N][Ho][Wo][CG] (pixel stride CG), 16-B aligned; CG in {64,128,192}
// KTMAX = 16-wide k-tiles compiled for (5 covers the 3-channel 5x5 edges plus
// the ones column: 76 columns)
// X3 (IC_MATH_SPLIT): fp32 by the exact three-term bf16 split on
// v_mfma_f32_16x16x32_bf16 (six products per MAC, 3/8 of the fp32 MFMA's cycles):
// the same LDS reads of G and of the patch as the fp32 loop (k-slot e of lane
// group lq takes pixel 32 ks + 4e + lq, so one read instruction spans four
// consecutive, differently swizzled G rows), split in registers.
// NP = 1 with X3 (IC_MATH_BF16, config C3): G and the patch values rounded to nearest even, one
// product per tile and 32-pixel step, fp32 accumulation.
template <int CG, int KTMAX, bool X3, int NP = 3>
__global__ void __launch_bounds__(256, KTMAX <= 5 ? 2 : 1)
    edge_wgrad_kernel(const EdgeGeom g, const float* __restrict__ G, int Kc, int ones, float* __restrict__ slab) {
  typedef __bf16 eb4 __attribute__((ext_vector_type(4)));
  typedef __bf16 eb8 __attribute__((ext_vector_type(8)));
  constexpr int NTW = CG / 64;            // 16-wide g-tiles per wave
  constexpr int CH = CG / 4;              // 16-B chunks per G row
  constexpr int GT = SEG * CG;            // G tile floats
  constexpr int QP = SEG * CH / 256;      // LDS-DMA pieces per thread
  constexpr int PB = PMAX + 2 * SEG * 2 + 2 * SEG * 2;  // patch + zero run + ones run
  // one G buffer (two blocks per CU cover each other's staging) and two patch buffers
  __shared__ __attribute__((aligned(16))) float lds[GT + 2 * PB];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int li = lane & 15, lq = lane >> 4;
  const int gbase = w * (CG / 4);
  const int KT = (Kc + 15) / 16;
  const int PSZ = g.C * g.k * g.PW;
  const int zero_off = PSZ, ones_off = PSZ + 2 * SEG * 2;
  float* const pbase = lds + GT;

  int koff[KTMAX];
#pragma unroll
  for (int kt = 0; kt < KTMAX; ++kt) koff[kt] = edge_koff(g, 16 * kt + li, zero_off, ones_off, ones != 0);
  for (int i = tid; i < 2 * SEG * 2; i += 256) {
    pbase[PSZ + i] = 0.f;
    pbase[PB + PSZ + i] = 0.f;
    pbase[ones_off + i] = 1.f;
    pbase[PB + ones_off + i] = 1.f;
  }
  floatx4v acc[NTW][KTMAX];
#pragma unroll
  for (int i = 0; i < NTW; ++i)
#pragma unroll
    for (int kt = 0; kt < KTMAX; ++kt) acc[i][kt] = floatx4v{0.f, 0.f, 0.f, 0.f};

  // G rows of unit u: pixels (n, oy, ox0 .. ox0+63) are one contiguous NHWC run
  auto stage_g = [&](long long u, float* img) {
    const int seg = (int)(u % g.units_per_row);
    const long long rr = u / g.units_per_row;
    const long long p0 = rr * g.Wo + (long long)seg * SEG;     // first pixel (n*Ho + oy)*Wo + ox0
    const int valid = min(SEG, g.Wo - seg * SEG);
    // the per-piece offsets are recomputed per unit, not hoisted out of the
    // unit loop into live registers (the split loop needs them)
    int t2 = tid;
    if (X3) asm volatile("" : "+v"(t2));
#pragma unroll
    for (int q = 0; q < QP; ++q) {
      const int pos = t2 + 256 * q;
      const int row = pos / CH, pc = pos - (pos / CH) * CH;
      const int lc = pc ^ (row & 15);
      const float* src = edge_zero_page;
      if (row < valid) src = G + (size_t)(p0 + row) * CG + lc * 4;
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)src, (lds_ptr_t)(img + (pos - (t2 & 63)) * 4), 16, 0, 0);
    }
  };

  EdgePatchMap pm;
  edge_patch_map(g, pm, tid);
  long long u = blockIdx.x;
  int buf = 0;
  float pr[PREG];
  if (u < g.units) {
    stage_g(u, lds);
    edge_patch_load(g, pm, u, pr);
    edge_patch_store(g, pr, pbase, tid);
  }
  for (; u < g.units; u += gridDim.x) {
    __syncthreads();  // vmcnt(0) + barrier: the G tile and patch `buf` are in LDS
    const long long un = u + gridDim.x;
    if (un < g.units) edge_patch_load(g, pm, un, pr);
    const float* gs = lds;
    const float* patch = pbase + buf * PB;
    if constexpr (X3) {
      auto split8 = [](const float (&v)[8], eb8& h, eb8& m, eb8& l) {
        if constexpr (NP == 1) {
          typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
          h = __builtin_bit_cast(eb8, u32x4{ic_cvt_pk_bf16(v[0], v[1]), ic_cvt_pk_bf16(v[2], v[3]),
                                            ic_cvt_pk_bf16(v[4], v[5]), ic_cvt_pk_bf16(v[6], v[7])});
          return;
        }
        eb4 h0, m0, l0, h1, m1, l1;
        split3_bf16x4(floatx4v{v[0], v[1], v[2], v[3]}, h0, m0, l0);
        split3_bf16x4(floatx4v{v[4], v[5], v[6], v[7]}, h1, m1, l1);
        h = __builtin_shufflevector(h0, h1, 0, 1, 2, 3, 4, 5, 6, 7);
        m = __builtin_shufflevector(m0, m1, 0, 1, 2, 3, 4, 5, 6, 7);
        l = __builtin_shufflevector(l0, l1, 0, 1, 2, 3, 4, 5, 6, 7);
      };
#pragma unroll 1
      for (int ks = 0; ks < SEG / 32; ++ks) {
        eb8 ah[NTW], am[NTW], al[NTW];
#pragma unroll
        for (int i = 0; i < NTW; ++i) {
          const int gc = gbase + 16 * i + li;
          float v[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const int m = 32 * ks + 4 * e + lq;
            v[e] = gs[m * CG + ((((gc >> 2) ^ (m & 15)) << 2) | (gc & 3))];
          }
          split8(v, ah[i], am[i], al[i]);
        }
#pragma unroll
        for (int kt = 0; kt < KTMAX; ++kt) {
          if (kt < KT) {
            float v[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = patch[koff[kt] + g.stride * (32 * ks + 4 * e + lq)];
            eb8 bh, bm, bl;
            split8(v, bh, bm, bl);
#pragma unroll
            for (int i = 0; i < NTW; ++i) {
              floatx4v& c = acc[i][kt];
              if constexpr (NP == 1) {
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh, c, 0, 0, 0);
                continue;
              }
              c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh, c, 0, 0, 0);
              c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am[i], bm, c, 0, 0, 0);
              c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl, c, 0, 0, 0);
              c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am[i], bh, c, 0, 0, 0);
              c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bm, c, 0, 0, 0);
              c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh, c, 0, 0, 0);
            }
          }
          __builtin_amdgcn_sched_barrier(0);  // one k-tile's operands live at a time
        }
      }
    }
    // k-step s2 of the pixel reduction: pixel m = 4 s2 + lq
#pragma unroll 4
    for (int s2 = 0; s2 < (X3 ? 0 : SEG / 4); ++s2) {
      const int m = 4 * s2 + lq;
      float a[NTW];
#pragma unroll
      for (int i = 0; i < NTW; ++i) {
        const int gc = gbase + 16 * i + li;
        a[i] = gs[m * CG + ((((gc >> 2) ^ (m & 15)) << 2) | (gc & 3))];
      }
#pragma unroll
      for (int kt = 0; kt < KTMAX; ++kt) {
        if (kt < KT) {
          const float b = patch[koff[kt] + g.stride * m];
#pragma unroll
          for (int i = 0; i < NTW; ++i) acc[i][kt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b, acc[i][kt], 0, 0, 0);
        }
      }
    }
    __syncthreads();  // every wave is done with the G tile
    if (un < g.units) {
      stage_g(un, lds);
      edge_patch_store(g, pr, pbase + (buf ^ 1) * PB, tid);
    }
    buf ^= 1;
  }
  // partial [CG][Kc] of this block (C/D map: row = g index 4lq + r, col = k index li)
  float* out = slab + (size_t)blockIdx.x * CG * Kc;
#pragma unroll
  for (int i = 0; i < NTW; ++i)
#pragma unroll
    for (int kt = 0; kt < KTMAX; ++kt)
      if (kt < KT) {
        const int kk = 16 * kt + li;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (kk < Kc) out[(size_t)(gbase + 16 * i + 4 * lq + r) * Kc + kk] = acc[i][kt][r];
      }
}

// fixed-order sum of the partials, scattered to dW[g][c][ky][kx] (+ db[g] from
// the ones column): 64 elements x 4 groups of partials per block, eight loads
// in flight per thread, the groups combined in LDS in a fixed order
__global__ void __launch_bounds__(256) edge_wgrad_reduce_kernel(const float* __restrict__ slab, int nb, int CG, int Kc,
                                                                int C, int T, float* __restrict__ dw,
                                                                float* __restrict__ db) {
  __shared__ float part[4][64];
  const int total = CG * Kc;
  const int e = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + e;
  const int q = (nb + 3) >> 2, b0 = grp * q, b1 = min(nb, b0 + q);
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (i < total) {
    const float* src = slab + i;
    int b = b0;
    for (; b + 7 < b1; b += 8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += src[(size_t)(b + j) * total];
    }
    for (int j = 0; b < b1; ++b, ++j) a[j] += src[(size_t)b * total];
  }
  part[grp][e] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  __syncthreads();
  if (grp != 0 || i >= total) return;
  const float v = (part[0][e] + part[1][e]) + (part[2][e] + part[3][e]);
  const int gg = i / Kc, kk = i - (i / Kc) * Kc;
  if (kk > T * C || (kk == T * C && !db)) return;
  if (kk == T * C) {
    db[gg] = v;
  } else {
    const int t = kk / C, c = kk - (kk / C) * C;
    dw[((size_t)gg * C + c) * T + t] = v;
  }
}

bool edge_geom(EdgeGeom& g, const float* x, long long sn, long long sc, long long sh, long long sw, int N, int C,
               int H, int W, int Ho, int Wo, int k, int stride, int pad) {
  if (sw != 1 || C < 1 || C > 4 || k < 1 || k > 5 || stride < 1 || stride > 2) return false;
  if (k * k * C > KMAX) return false;
  g.x = x; g.sn = sn; g.sc = sc; g.sh = sh;
  g.N = N; g.C = C; g.H = H; g.W = W; g.Ho = Ho; g.Wo = Wo;
  g.k = k; g.stride = stride; g.pad = pad;
  g.PW = (SEG - 1) * stride + k;
  g.TC = k * k * C;
  g.units_per_row = (Wo + SEG - 1) / SEG;
  g.units = (long long)N * Ho * g.units_per_row;
  // 32-bit unit indices and in-image offsets (edge_patch_load)
  if (g.units >= (1LL << 31) || (long long)(C - 1) * sc + (long long)(H - 1) * sh + W >= (1LL << 31)) return false;
  return g.C * g.k * g.PW <= PMAX;
}

int edge_grid(long long units, int per_cu) {
  const long long cap = 256LL * per_cu;
  return (int)(units < cap ? units : cap);
}


// ------------------------------------------------------------------ tconv to few channels
// Transposed conv, stride 2, wide NHWC input -> few-channel output (g_s.6:
// 192 -> 3, 5x5): output-row stationary, no column buffer in HBM.
//   out[n][o][Y][X] = b[o] + sum_{ky,kx,c} x[n][iy][ix][c] W[c][o][ky][kx],
//   Y = 2 iy - pad + ky,  X = 2 ix - pad + kx.
// Output row Y takes the taps ky = (Y + pad) mod 2, +2, ..., each from one
// input row iy; per (ky, iy) one small GEMM Cm[ix][(kx, o)] = x[n][iy][ix][:] .
// W[:, o, ky, kx] (M = input width, N = k*Cout <= 16 on one 16-wide MFMA tile,
// K = Cin) leaves its rows in LDS, and a fixed-order gather sums
// out[X][o] = sum_{ky, kx: X + pad - kx even} Cm_ky[(X + pad - kx)/2][(kx, o)].
// Every (ky, iy, ix) product is formed once (no padded MACs beyond N 15 -> 16).
// Blocks are persistent over rows of one parity of Y (their ky set), with that
// parity's weights staged once in LDS as B fragments [kyi][u][lq][col][v]:
// MFMA step s = 4u + v consumes channel 16u + 4lq + v on both sides, so a
// lane's A operand is one float4 of its pixel's channels.
constexpr int TF_KY = 3;  // taps per parity for k <= 5
#ifndef TCONV_FEW2
#define TCONV_FEW2 1  // stride-2 upsampling to few channels on the input-row-stationary kernel (Win <= 128)
#endif

template <int NWV, int MTW>  // waves, 16-pixel m-tiles per wave: input width <= 16 * NWV * MTW
__global__ void __launch_bounds__(64 * NWV, 2)
    tconv_few_kernel(const float* __restrict__ x, int N, int Hin, int Win, int Cin, const float* __restrict__ W,
                     int Cout, int k, int pad, const float* __restrict__ bias, int relu, float* __restrict__ y,
                     long long ysn, long long ysc, long long ysh, long long ysw, int Hout, int Wout) {
  constexpr int WMAX = 16 * NWV * MTW;
  constexpr int NT = 64 * NWV;
  __shared__ __attribute__((aligned(16))) float wl[TF_KY * 12 * 4 * 16 * 4];  // Cin <= 192
  __shared__ __attribute__((aligned(16))) float cm[TF_KY * WMAX * 16];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int li = lane & 15, lq = lane >> 4;
  const int U = Cin >> 4;
  const int par = blockIdx.x & 1;               // rows Y with Y % 2 == par
  const int ky0 = (par + pad) & 1;              // their first tap row
  const int nky = (k - ky0 + 1) >> 1;
  const int ncol = k * Cout;
  // weights of this parity: wl[((kyi*U + u)*4 + q)*16 + col][v] = W[c = 16u+4q+v][o][ky][kx], col = kx*Cout + o
  for (int i = tid; i < nky * U * 4 * 16 * 4; i += NT) {
    const int v = i & 3, col = (i >> 2) & 15, q = (i >> 6) & 3, r = i >> 8;
    const int u = r % U, kyi = r / U;
    const int c = 16 * u + 4 * q + v, ky = ky0 + 2 * kyi;
    float val = 0.f;
    if (col < ncol) {
      const int kx = col / Cout, o = col - (col / Cout) * Cout;
      val = W[(((size_t)c * Cout + o) * k + ky) * k + kx];
    }
    wl[i] = val;
  }
  const int rows_par = (Hout - par + 1) >> 1;   // rows of this parity per image
  const long long nrows = (long long)N * rows_par;
  for (long long rr = blockIdx.x >> 1; rr < nrows; rr += gridDim.x >> 1) {
    const int n = (int)(rr / rows_par);
    const int Y = 2 * (int)(rr - (long long)n * rows_par) + par;
    __syncthreads();  // weights staged / previous row's gather done with cm
    for (int kyi = 0; kyi < nky; ++kyi) {
      const int ky = ky0 + 2 * kyi;
      const int iy = (Y + pad - ky) >> 1;     // Y + pad - ky is even
      if (iy < 0 || iy >= Hin) continue;      // uniform: no contribution
      const float* xr = x + ((size_t)n * Hin + iy) * Win * Cin;
      floatx4v acc[MTW];
#pragma unroll
      for (int t = 0; t < MTW; ++t) acc[t] = floatx4v{0.f, 0.f, 0.f, 0.f};
      // the row's whole A operand (all channels of this wave's pixels) in
      // flight at once: one memory latency per (ky, iy) instead of one per
      // 16-channel step
      floatx4v a[MTW][12];
#pragma unroll
      for (int u = 0; u < 12; ++u)
#pragma unroll
        for (int t = 0; t < MTW; ++t) {
          const int px = 16 * (w + NWV * t) + li;
          a[t][u] = (u < U && px < Win) ? *(const floatx4v*)(xr + (size_t)px * Cin + 16 * u + 4 * lq)
                                        : floatx4v{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
      for (int u = 0; u < 12; ++u) {
        if (u < U) {
          const floatx4v b4 = *(const floatx4v*)(wl + ((((kyi * U + u) * 4 + lq) * 16 + li) << 2));
#pragma unroll
          for (int v = 0; v < 4; ++v)
#pragma unroll
            for (int t = 0; t < MTW; ++t)
              acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t][u][v], b4[v], acc[t], 0, 0, 0);
        }
      }
      // C/D map: row (pixel) 16*mtile + 4lq + r, col li
#pragma unroll
      for (int t = 0; t < MTW; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) cm[(kyi * WMAX + 16 * (w + NWV * t) + 4 * lq + r) * 16 + li] = acc[t][r];
    }
    __syncthreads();
    // gather, fixed order (ky ascending, kx ascending)
    for (int X = tid; X < Wout; X += NT) {
      float sum[4] = {0.f, 0.f, 0.f, 0.f};  // Cout <= 4 handled here (k*Cout <= 16)
      for (int kyi = 0; kyi < nky; ++kyi) {
        const int iy = (Y + pad - ky0 - 2 * kyi) >> 1;
        if (iy < 0 || iy >= Hin) continue;
        for (int kx = (X + pad) & 1; kx < k; kx += 2) {
          const int ix = (X + pad - kx) >> 1;
          if (ix < 0 || ix >= Win) continue;
          const float* cp = cm + (kyi * WMAX + ix) * 16 + kx * Cout;
          for (int o = 0; o < Cout; ++o) sum[o] += cp[o];
        }
      }
      for (int o = 0; o < Cout; ++o) {
        float v = sum[o] + (bias ? bias[o] : 0.f);
        if (relu) v = v > 0.f ? v : 0.f;
        y[n * ysn + o * ysc + (long long)Y * ysh + (long long)X * ysw] = v;
      }
    }
  }
}
// Input-row-stationary variant (stride 2, input width <= 16 * NWV): each
// block walks a run of input rows of one image; every input row is loaded
// once (one float4 of 16 channels per lane, all channels in flight, the next
// row prefetched into a second register set during this row's MFMAs) and
// multiplied by the weights of all k tap rows (k 16-column MFMA tiles: col =
// (kx, o)).  Tap row ky of input row r belongs to output row Y = 2r - pad + ky
// and lands in that row's slot of an LDS ring of pending output rows: the
// row's first contribution (ky = k - 1 or k - 2, by parity) stores, later
// ones add, in input-row order.  After input row r the rows 2r - pad and
// 2r - pad + 1 are complete; they are gathered (fixed order, kx ascending) and
// written during the next row's MFMAs, one barrier per input row.  A block
// starts (k - 1) / 2 rows before its run (halo: nothing emitted), and rows
// outside the image still store zeros, so every emitted row is exact.  Input
// traffic ~1.1x the tensor (vs ~2.5x for the output-row-stationary kernel).
#ifndef TF2_SPLIT
#define TF2_SPLIT 1  // split arithmetic (IC_MATH_SPLIT) on the input-row kernel
#endif
constexpr int TF2_RS = 8;  // ring slots: rows 2r - pad - 2 .. 2r - pad + k - 1 in flight
constexpr int TF2_HALO = 2;  // input columns loaded left of a column segment (k <= 5, pad >= 0)
// input columns a segment owns when the row is wider than the block (WMAX = 128): its output
// columns need input columns up to (2 (sg + 1) wseg - 1 + pad) / 2 <= base + WMAX - 1 for pad <= 5
constexpr int TF2_WSEG = 120;

// X3 (IC_MATH_SPLIT, Cin % 32 == 0): fp32 by the exact three-term bf16 split
// on v_mfma_f32_16x16x32_bf16 (six products per MAC, 3/8 of the fp32 MFMA's
// cycles): the weights are staged split, as B fragments
// [ky][s][part][lq][col][8] (8 consecutive channels 32s + 8lq + e of column
// col per lane: one b128 read per part), and each lane splits its pixel's
// 8-channel A fragment per 32-channel step from the same row registers.
// NP = 1 with X3 (IC_MATH_BF16, config C3): bf16 operands (weights and the pixel's channels rounded
// to nearest even), one product per tap row and 32-channel step, fp32 accumulation.
template <int NWV, bool X3, int NP = 3>
__global__ void __launch_bounds__(64 * NWV, 1)
    tconv_few2_kernel(const float* __restrict__ x, int N, int Hin, int Win, int Cin, const float* __restrict__ W,
                      int Cout, int k, int pad, const float* __restrict__ bias, int relu, float* __restrict__ y,
                      long long ysn, long long ysc, long long ysh, long long ysw, int Hout, int Wout, int run,
                      int wseg) {
  typedef __bf16 tb4 __attribute__((ext_vector_type(4)));
  typedef __bf16 tb8 __attribute__((ext_vector_type(8)));
  constexpr int WMAX = 16 * NWV;
  constexpr int NT = 64 * NWV;
  // fp32: [ky][u][q][col][v] floats; X3: [ky][s][part][lq][col][8] bf16 (the same 90 KB): Cin <= 192
  __shared__ __attribute__((aligned(16))) float wl[X3 ? 5 * 6 * 3 * 4 * 16 * 4 : 5 * 12 * 4 * 16 * 4];
  __shared__ __attribute__((aligned(16))) float ring[TF2_RS * WMAX * 16];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int li = lane & 15, lq = lane >> 4;
  const int U = Cin >> 4;
  const int S = Cin >> 5;
  const int ncol = k * Cout;
  __bf16* const wb = (__bf16*)wl;
  constexpr int PART = 4 * 16 * 8;  // bf16 per part of one (ky, s) B fragment set
  if constexpr (X3) {
    for (int i = tid; i < k * S * 4 * 16 * 8; i += NT) {
      const int e = i & 7, col = (i >> 3) & 15, q = (i >> 7) & 3, rr = i >> 9;
      const int sx = rr % S, ky = rr / S;
      const int c = 32 * sx + 8 * q + e;
      float val = 0.f;
      if (col < ncol) {
        const int kx = col / Cout, o = col - (col / Cout) * Cout;
        val = W[(((size_t)c * Cout + o) * k + ky) * k + kx];
      }
      const int o0 = (ky * S + sx) * 3 * PART + (q * 16 + col) * 8 + e;
      if constexpr (NP == 1) {
        wb[o0] = (__bf16)val;  // round to nearest even
      } else {
        __bf16 hh, mm, ll;
        split3_bf16(val, hh, mm, ll);
        wb[o0] = hh;
        wb[o0 + PART] = mm;
        wb[o0 + 2 * PART] = ll;
      }
    }
  } else {
    for (int i = tid; i < k * U * 4 * 16 * 4; i += NT) {
      const int v = i & 3, col = (i >> 2) & 15, q = (i >> 6) & 3, rr = i >> 8;
      const int u = rr % U, ky = rr / U;
      const int c = 16 * u + 4 * q + v;
      float val = 0.f;
      if (col < ncol) {
        const int kx = col / Cout, o = col - (col / Cout) * Cout;
        val = W[(((size_t)c * Cout + o) * k + ky) * k + kx];
      }
      wl[i] = val;
    }
  }
  __syncthreads();

  // rows wider than WMAX run in column segments: segment sg owns input columns [sg wseg, (sg + 1) wseg)
  // and output columns [2 sg wseg, 2 (sg + 1) wseg) (the last one: to Wout); it loads the WMAX
  // input columns from sg wseg - TF2_HALO, which hold every input column its output columns take
  // (2 ix = X + pad - kx, kx < k <= 5).  One segment (Win <= WMAX): base 0, all of Wout.
  const int nseg = (Win + wseg - 1) / wseg;
  const int sg = blockIdx.x % nseg;
  const int bq = blockIdx.x / nseg;
  const int base = nseg == 1 ? 0 : sg * wseg - TF2_HALO;
  const int X0 = 2 * sg * wseg;
  const int X1 = sg == nseg - 1 ? Wout : min(Wout, 2 * (sg + 1) * wseg);
  const int nrun = (Hin + run - 1) / run;
  const int n = bq / nrun;
  const int r0 = (bq - n * nrun) * run;
  const bool last = r0 + run >= Hin;
  const int rlast = last ? (Hout - 1 + pad) >> 1 : r0 + run - 1;   // last input row whose rows are emitted
  const int rfirst = r0 - (k - 1) / 2;
  const int px = 16 * w + li;  // this lane's column within the segment's WMAX
  const int gx = base + px;    // ... and in the image
  const float* xn = x + (size_t)n * Hin * Win * Cin;

  floatx4v a0[12], a1[12];
  // fp32: a[u] = channels 16u + 4lq .. +3; X3: a[2s + h] = channels 32s + 8lq + 4h .. +3
  auto load = [&](int r, floatx4v (&a)[12]) {
    const bool ok = r >= 0 && r < Hin && gx >= 0 && gx < Win;
    const float* xr = xn + ((size_t)(ok ? r : 0) * Win + (ok ? gx : 0)) * Cin + (X3 ? 8 : 4) * lq;
#pragma unroll
    for (int u = 0; u < 12; ++u) {
      const int off = X3 ? 32 * (u >> 1) + 4 * (u & 1) : 16 * u;
      a[u] = (ok && u < U) ? *(const floatx4v*)(xr + off) : floatx4v{0.f, 0.f, 0.f, 0.f};
    }
  };
  // the two rows completed by input row r (emitted from the block's run on)
  auto emit = [&](int r) {
    if (r < r0) return;
    for (int h = 0; h < 2; ++h) {
      const int Y = 2 * r - pad + h;
      if (Y < 0 || Y >= Hout) continue;
      const float* sl = ring + (Y & (TF2_RS - 1)) * WMAX * 16;
      for (int X = X0 + tid; X < X1; X += NT) {
        float sum[4] = {0.f, 0.f, 0.f, 0.f};
        for (int kx = (X + pad) & 1; kx < k; kx += 2) {
          const int ix = (X + pad - kx) >> 1;
          if (ix < 0 || ix >= Win) continue;
          const float* cp = sl + (ix - base) * 16 + kx * Cout;
          for (int o = 0; o < Cout; ++o) sum[o] += cp[o];
        }
        for (int o = 0; o < Cout; ++o) {
          float v = sum[o] + (bias ? bias[o] : 0.f);
          if (relu) v = v > 0.f ? v : 0.f;
          y[n * ysn + o * ysc + (long long)Y * ysh + (long long)X * ysw] = v;
        }
      }
    }
  };
  // one input row: its k tap-row tiles (MFMAs), the previous row's completed
  // rows emitted meanwhile, then the tiles stored / added into the ring
  auto row = [&](int r, const floatx4v (&a)[12]) {
    floatx4v acc[5];
#pragma unroll
    for (int ky = 0; ky < 5; ++ky) acc[ky] = floatx4v{0.f, 0.f, 0.f, 0.f};
    if (X3 && r >= 0 && r < Hin) {
#pragma unroll
      for (int sx = 0; sx < 6; ++sx) {
        if (sx < S && NP == 1) {
          typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
          const floatx4v v0 = a[2 * sx], v1 = a[2 * sx + 1];
          const tb8 ab = __builtin_bit_cast(tb8, u32x4{ic_cvt_pk_bf16(v0[0], v0[1]), ic_cvt_pk_bf16(v0[2], v0[3]),
                                                       ic_cvt_pk_bf16(v1[0], v1[1]), ic_cvt_pk_bf16(v1[2], v1[3])});
#pragma unroll
          for (int ky = 0; ky < 5; ++ky) {
            if (ky < k) {
              const tb8 b0 = *(const tb8*)(wb + (ky * S + sx) * 3 * PART + (lq * 16 + li) * 8);
              acc[ky] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, b0, acc[ky], 0, 0, 0);
            }
          }
        } else if (sx < S) {
          tb4 h0, m0, l0, h1, m1, l1;
          split3_bf16x4(a[2 * sx], h0, m0, l0);
          split3_bf16x4(a[2 * sx + 1], h1, m1, l1);
          const tb8 ah = __builtin_shufflevector(h0, h1, 0, 1, 2, 3, 4, 5, 6, 7);
          const tb8 am = __builtin_shufflevector(m0, m1, 0, 1, 2, 3, 4, 5, 6, 7);
          const tb8 al = __builtin_shufflevector(l0, l1, 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
          for (int ky = 0; ky < 5; ++ky) {
            if (ky < k) {
              const __bf16* bp = wb + (ky * S + sx) * 3 * PART + (lq * 16 + li) * 8;
              const tb8 b0 = *(const tb8*)bp, b1 = *(const tb8*)(bp + PART), b2 = *(const tb8*)(bp + 2 * PART);
              acc[ky] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, b0, acc[ky], 0, 0, 0);
              acc[ky] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, b1, acc[ky], 0, 0, 0);
              acc[ky] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, b2, acc[ky], 0, 0, 0);
              acc[ky] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, b0, acc[ky], 0, 0, 0);
              acc[ky] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, b1, acc[ky], 0, 0, 0);
              acc[ky] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, b0, acc[ky], 0, 0, 0);
            }
          }
        }
      }
    }
    if (!X3 && r >= 0 && r < Hin) {
#pragma unroll
      for (int u = 0; u < 12; ++u) {
        if (u < U) {
#pragma unroll
          for (int ky = 0; ky < 5; ++ky) {
            if (ky < k) {
              const floatx4v b4 = *(const floatx4v*)(wl + ((((ky * U + u) * 4 + lq) * 16 + li) << 2));
#pragma unroll
              for (int v = 0; v < 4; ++v)
                acc[ky] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][v], b4[v], acc[ky], 0, 0, 0);
            }
          }
        }
      }
    }
    emit(r - 1);  // its slots are not written by this row (ring of 8)
    // C/D map: pixel 16w + 4lq + e, column li; each (pixel, column) of a slot has one owner
#pragma unroll
    for (int ky = 0; ky < 5; ++ky) {
      const int Y = 2 * r - pad + ky;
      if (ky < k && Y >= 0 && Y < Hout) {
        float* sl = ring + ((Y & (TF2_RS - 1)) * WMAX + 16 * w + 4 * lq) * 16 + li;
        if (ky >= k - 2) {
#pragma unroll
          for (int e = 0; e < 4; ++e) sl[16 * e] = acc[ky][e];
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) sl[16 * e] += acc[ky][e];
        }
      }
    }
    __syncthreads();  // this row's ring writes before the next row's emission; emission reads before reuse
  };

  load(rfirst, a0);
  int r = rfirst;
  for (; r <= rlast; r += 2) {
    load(r + 1, a1);
    row(r, a0);
    if (r + 1 > rlast) { ++r; break; }
    load(r + 2, a0);
    row(r + 1, a1);
  }
  emit(rlast);
}
}  // namespace

// y (NHWC, channel stride 1) = conv(x few-channel, wp [Cout][Kp] with k = t*C + c)
int edge_conv_run(const float* x, long long sn, long long sc, long long sh, long long sw, int N, int C, int H, int W,
                  const float* wp, int Kp, const float* bias, int k, int stride, int pad, float* y, long long ys_n,
                  long long ys_c, long long ys_h, long long ys_w, int Cout, int Ho, int Wo, int relu, hipStream_t s,
                  int split) {
  EdgeGeom g;
  if (!edge_geom(g, x, sn, sc, sh, sw, N, C, H, W, Ho, Wo, k, stride, pad)) return IC_ERR_ARG;
  // 16-B channel-quad stores
  if (ys_c != 1 || Kp < g.TC || ((uintptr_t)y & 15) || ys_w % 4 || ys_h % 4 || ys_n % 4) return IC_ERR_ARG;
  if (edge_conv_split(split, g.TC, Cout)) {
    const int grid1 = edge_grid(g.units, 1);
    if (grid1 < 1) return IC_OK;
    const bool s3 = (g.TC + 31) / 32 == 3;
#define EDGE_CONV_X3(CO_)                                                                                      \
  do {                                                                                                         \
    if (split == 2 && s3)                                                                                      \
      hipLaunchKernelGGL((edge_conv_x3_kernel<CO_, 1, 3>), dim3(grid1), dim3(512), 0, s, g, wp, Kp, bias, relu, \
                         y, ys_n, ys_h, ys_w);                                                                 \
    else if (split == 2)                                                                                       \
      hipLaunchKernelGGL((edge_conv_x3_kernel<CO_, 1>), dim3(grid1), dim3(512), 0, s, g, wp, Kp, bias, relu, y, \
                         ys_n, ys_h, ys_w);                                                                    \
    else if (s3)                                                                                               \
      hipLaunchKernelGGL((edge_conv_x3_kernel<CO_, 3, 3>), dim3(grid1), dim3(512), 0, s, g, wp, Kp, bias, relu, \
                         y, ys_n, ys_h, ys_w);                                                                 \
    else                                                                                                       \
      hipLaunchKernelGGL((edge_conv_x3_kernel<CO_>), dim3(grid1), dim3(512), 0, s, g, wp, Kp, bias, relu, y,    \
                         ys_n, ys_h, ys_w);                                                                    \
  } while (0)
    if (Cout == 192) EDGE_CONV_X3(192);
    else if (Cout == 128) EDGE_CONV_X3(128);
    else EDGE_CONV_X3(64);
#undef EDGE_CONV_X3
    IC_CHECK_LAUNCH();
    return IC_OK;
  }
  const int grid = edge_grid(g.units, EDGE_CONV_PER_CU);
  if (grid < 1) return IC_OK;
  switch (Cout) {
    case 192:
      hipLaunchKernelGGL(edge_conv_kernel<192>, dim3(grid), dim3(256), 0, s, g, wp, Kp, bias, relu, y, ys_n, ys_h,
                         ys_w);
      break;
    case 128:
      hipLaunchKernelGGL(edge_conv_kernel<128>, dim3(grid), dim3(256), 0, s, g, wp, Kp, bias, relu, y, ys_n, ys_h,
                         ys_w);
      break;
    case 64:
      hipLaunchKernelGGL(edge_conv_kernel<64>, dim3(grid), dim3(256), 0, s, g, wp, Kp, bias, relu, y, ys_n, ys_h,
                         ys_w);
      break;
    default:
      return IC_ERR_ARG;
  }
  IC_CHECK_LAUNCH();
  return IC_OK;
}

bool edge_conv_split(int split, int TC, int Cout) {
  return EC_SPLIT && split && TC <= 32 * EC3_S && (Cout == 64 || Cout == 128 || Cout == 192);
}

bool edge_conv_ok(int C, int k, int stride, long long sw, long long ys_c, int Cout, long long ys_w, long long ys_h,
                  long long ys_n) {
  return C >= 1 && C <= 4 && k <= 5 && k * k * C <= KMAX && stride >= 1 && stride <= 2 && sw == 1 && ys_c == 1 &&
         (Cout == 64 || Cout == 128 || Cout == 192) && ys_w % 4 == 0 && ys_h % 4 == 0 && ys_n % 4 == 0;
}

// workspace of edge_wgrad_run
size_t edge_wgrad_ws(int CG, int Kc, long long units) {
  return (size_t)edge_grid(units, 2) * CG * Kc * sizeof(float);
}

bool edge_wgrad_ok(int C, int k, int stride, long long sw, const float* G, int CG, long long gs_c, long long gs_w,
                   long long gs_h, long long gs_n, int Ho, int Wo) {
  if (!(C >= 1 && C <= 4 && k <= 5 && k * k * C + 1 <= KMAX + 1 && stride >= 1 && stride <= 2 && sw == 1)) return false;
  if (!(CG == 64 || CG == 128 || CG == 192)) return false;
  if (gs_c != 1 || gs_w != CG || gs_h != (long long)Wo * CG || gs_n != (long long)Ho * Wo * CG) return false;
  return ((uintptr_t)G & 15) == 0;
}

long long edge_units(int N, int Ho, int Wo) { return (long long)N * Ho * ((Wo + SEG - 1) / SEG); }

// dW[g][c][ky][kx] = sum_p G[p][g] X[p*s + tap][c];  db[g] = sum_p G[p][g] when db != NULL
int edge_wgrad_run(const float* G, int CG, const float* x, long long sn, long long sc, long long sh, long long sw,
                   int N, int C, int H, int W, int Ho, int Wo, int k, int stride, int pad, float* dw, float* db,
                   void* ws, hipStream_t s, int split) {
  EdgeGeom g;
  if (!edge_geom(g, x, sn, sc, sh, sw, N, C, H, W, Ho, Wo, k, stride, pad)) return IC_ERR_ARG;
  const int Kc = g.TC + (db ? 1 : 0);
  const bool k5 = Kc <= 80;  // 5 k-tiles: two blocks per CU
  const int grid = edge_grid(g.units, k5 ? 2 : 1);
  if (grid < 1) return IC_OK;
  float* slab = (float*)ws;
  const bool x3 = EW_SPLIT && split;
#define EDGE_WG(CG_, KT_)                                                                                       \
  do {                                                                                                          \
    if (x3 && split == 2)                                                                                       \
      hipLaunchKernelGGL((edge_wgrad_kernel<CG_, KT_, true, 1>), dim3(grid), dim3(256), 0, s, g, G, Kc,         \
                         db ? 1 : 0, slab);                                                                     \
    else if (x3) hipLaunchKernelGGL((edge_wgrad_kernel<CG_, KT_, true>), dim3(grid), dim3(256), 0, s, g, G, Kc,\
                                    db ? 1 : 0, slab);                                                          \
    else hipLaunchKernelGGL((edge_wgrad_kernel<CG_, KT_, false>), dim3(grid), dim3(256), 0, s, g, G, Kc,       \
                            db ? 1 : 0, slab);                                                                  \
  } while (0)
  switch (CG) {
    case 192:
      if (k5) EDGE_WG(192, 5); else EDGE_WG(192, 7);
      break;
    case 128:
      if (k5) EDGE_WG(128, 5); else EDGE_WG(128, 7);
      break;
    case 64:
      if (k5) EDGE_WG(64, 5); else EDGE_WG(64, 7);
      break;
    default:
      return IC_ERR_ARG;
  }
#undef EDGE_WG
  IC_CHECK_LAUNCH();
  const int total = CG * Kc;
  hipLaunchKernelGGL(edge_wgrad_reduce_kernel, dim3((total + 63) / 64), dim3(256), 0, s, slab, grid, CG, Kc, C,
                     k * k, dw, db);
  IC_CHECK_LAUNCH();
  return IC_OK;
}

int tconv_few_kind(int Hin, int Win, int k, int pad, int Hout) {
  // any width (column segments past 128), pad <= 5 (the segment halo)
  return (TCONV_FEW2 && k <= 5 && pad <= 5 && (Hout - 1 + pad) / 2 <= Hin + 2 && Win <= 4096)
             ? IC_KERNEL_TCONV_FEW_ROWS
             : IC_KERNEL_TCONV_FEW;
}

// transposed conv 2x upsampling of a wide NHWC map to <= 4 channels (see tconv_few_kernel)
bool tconv_few_ok(int Cin, int Cout, int k, int stride, int pad, long long xsc, long long xsw, long long xsh,
                  long long xsn, int Hin, int Win) {
  return stride == 2 && k <= 5 && k >= 1 && Cout >= 1 && Cout <= 4 && k * Cout <= 16 && Cin % 16 == 0 &&
         Cin <= 192 && (Win <= 256 || (TCONV_FEW2 && pad <= 5 && Win <= 4096)) && xsc == 1 && xsw == Cin &&
         xsh == (long long)Win * Cin &&
         xsn == (long long)Hin * Win * Cin && pad >= 0;
}

int tconv_few_run(const float* x, int N, int Hin, int Win, int Cin, const float* W, int Cout, int k, int pad,
                  const float* bias, int relu, float* y, long long ysn, long long ysc, long long ysh, long long ysw,
                  int Hout, int Wout, hipStream_t s, int split) {
  if (((uintptr_t)x & 15) || Hout < 1 || Wout < 1) return IC_ERR_ARG;
  if (tconv_few_kind(Hin, Win, k, pad, Hout) == IC_KERNEL_TCONV_FEW_ROWS) {
    // input-row stationary: runs of input rows (x column segments past 128), about one block per CU
    const int wseg = Win <= 128 ? Win : TF2_WSEG;
    const long long nseg = (Win + wseg - 1) / wseg;
    // one block per CU (157 KB of LDS): split each (image, segment) row sequence into as many runs as
    // keep the grid within 256 blocks, so the grid runs in one round.  Rounding the row count per block
    // up instead (r08d: C5's 16 x 3 sequences of 256 rows in runs of 48 = 288 blocks) left 32 blocks
    // for a second round of full-length runs: 0.73 ms for C5's g_s.6 forward.
    const long long units = (long long)N * nseg;
    const long long per = units < 256 ? 256 / units : 1;
    long long run = (Hin + per - 1) / per;
    if (run < 4) run = 4;
    if (run > Hin) run = Hin;
    const long long blocks = (long long)N * ((Hin + run - 1) / run) * nseg;
    if (blocks >= (1LL << 31)) return IC_ERR_ARG;
    if (TF2_SPLIT && split == 2 && Cin % 32 == 0)
      hipLaunchKernelGGL((tconv_few2_kernel<8, true, 1>), dim3((unsigned)blocks), dim3(512), 0, s, x, N, Hin, Win, Cin,
                         W, Cout, k, pad, bias, relu, y, ysn, ysc, ysh, ysw, Hout, Wout, (int)run, wseg);
    else if (TF2_SPLIT && split && Cin % 32 == 0)
      hipLaunchKernelGGL((tconv_few2_kernel<8, true>), dim3((unsigned)blocks), dim3(512), 0, s, x, N, Hin, Win, Cin, W,
                         Cout, k, pad, bias, relu, y, ysn, ysc, ysh, ysw, Hout, Wout, (int)run, wseg);
    else
      hipLaunchKernelGGL((tconv_few2_kernel<8, false>), dim3((unsigned)blocks), dim3(512), 0, s, x, N, Hin, Win, Cin, W,
                         Cout, k, pad, bias, relu, y, ysn, ysc, ysh, ysw, Hout, Wout, (int)run, wseg);
    IC_CHECK_LAUNCH();
    return IC_OK;
  }
  if (Win > 256) return IC_ERR_ARG;  // the output-row kernels hold a row of <= 256 pixels
  const long long rows = (long long)N * ((Hout + 1) / 2);
  long long grid = 2 * (rows < 256 ? rows : 256);  // two parities, <= 2 blocks per CU
  if (Win <= 64)
    hipLaunchKernelGGL((tconv_few_kernel<4, 1>), dim3((unsigned)grid), dim3(256), 0, s, x, N, Hin, Win, Cin, W, Cout,
                       k, pad, bias, relu, y, ysn, ysc, ysh, ysw, Hout, Wout);
  else if (Win <= 128)
    hipLaunchKernelGGL((tconv_few_kernel<8, 1>), dim3((unsigned)grid), dim3(512), 0, s, x, N, Hin, Win, Cin, W, Cout,
                       k, pad, bias, relu, y, ysn, ysc, ysh, ysw, Hout, Wout);
  else
    hipLaunchKernelGGL((tconv_few_kernel<8, 2>), dim3((unsigned)grid), dim3(512), 0, s, x, N, Hin, Win, Cin, W, Cout,
                       k, pad, bias, relu, y, ysn, ysc, ysh, ysw, Hout, Wout);
  IC_CHECK_LAUNCH();
  return IC_OK;
}


#if EC_STAMP
// diagnostic build only (EC_STAMP): the edge conv's s_memtime stamps, for tools/edge_stamps.py
extern "C" int ic_debug_edge_stamps(void* host, size_t bytes) {
  if (bytes > sizeof(edge_stamps)) bytes = sizeof(edge_stamps);
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(edge_stamps), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 1;
}
#endif
