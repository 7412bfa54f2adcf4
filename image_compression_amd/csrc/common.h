// Shared device/host helpers for the gfx950 (CDNA4) kernels of imgcomp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4v __attribute__((ext_vector_type(4)));

#define IC_MAXT 25      // max taps of one (phase of a) convolution: 5x5
#define IC_MAXPH 4      // max sub-pixel phases per launch (stride 2)

// status codes returned by every extern "C" entry point (0 = ok)
#define IC_OK 0
#ifndef IC_ERR_ARG
#define IC_ERR_ARG 1001        // unsupported / inconsistent arguments
#define IC_ERR_WORKSPACE 1002  // workspace too small
#endif

#define IC_CHECK_LAUNCH()                                    \
  do {                                                       \
    hipError_t _e = hipGetLastError();                       \
    if (_e != hipSuccess) return (int)_e;                    \
  } while (0)

static inline size_t ic_align(size_t v, size_t a) { return (v + a - 1) / a * a; }
static inline int ic_cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

// Fast unsigned division for numerators < 2^31 (Granlund-Montgomery):
// q = (umulhi(n, m) + n) >> l, with l = ceil(log2 d), m = 2^32 (2^l - d) / d + 1.
struct FastDiv {
  uint32_t d, m, l;
};
static inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d ? d : 1;
  f.l = 0;
  while ((1ull << f.l) < f.d) ++f.l;
  f.m = (uint32_t)(((1ull << 32) * ((1ull << f.l) - f.d)) / f.d + 1);
  return f;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  return (__umulhi(n, f.m) + n) >> f.l;
}

// Exact three-term bf16 split of an fp32 value: a = h + m + l.  Each step
// rounds to nearest even (v_cvt_pk_bf16_f32) and the residual a - h (then
// minus m) is exact in fp32, so the three 8-bit significands carry all 24 of
// a's.  Products of split operands are exact in fp32; keeping the six terms
// h*h' + h*m' + m*h' + h*l' + m*m' + l*h' drops only terms below 2^-24 of the
// product, i.e. the error of an fp32 fma chain.
__device__ __forceinline__ void split3_bf16(float a, __bf16& h, __bf16& m, __bf16& l) {
  h = (__bf16)a;
  const float r1 = a - (float)h;
  m = (__bf16)r1;
  l = (__bf16)(r1 - (float)m);
}

// split staging through split3_bf16x4: on in wg_x3_kernel (g_a.2 / g_s.4 wgrad
// 1.28 -> 1.23 / 1.30 -> 1.27 ms) and in ig_kernel_x3s together with its
// spread global loads (IG_X3_SGB = 8: big fwd/dgrad ops 5.30 -> 5.13 ms, with
// the paired split 5.08; the paired split alone, loads up front, was slower)
#ifndef IG_SPLIT_PK
#define IG_SPLIT_PK 1
#endif
#ifndef WG_SPLIT_PK
#define WG_SPLIT_PK 1
#endif
// split3_bf16 of four values with the bf16 conversions paired
// (v_cvt_pk_bf16_f32 on two operands, round-to-nearest-even as the scalar
// cast); the residuals are written as two-wide vector subtractions, which the
// build lowers to scalar v_sub_f32 (every source is compiled without the
// packed-fp32 instructions, csrc/Makefile NOPK).  Bitwise identical to
// split3_bf16.  V4 is any 8-byte vector of four bf16.
__device__ __forceinline__ uint32_t ic_cvt_pk_bf16(float lo, float hi) {
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{lo, hi}, bf16x2));  // one v_cvt_pk_bf16_f32
}
template <class V4>
__device__ __forceinline__ void split3_bf16x4(floatx4v a, V4& h, V4& m, V4& l) {
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  u32x2 ph, pm, pl;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const f32x2 x = {a[2 * p], a[2 * p + 1]};
    const uint32_t hh = ic_cvt_pk_bf16(x[0], x[1]);
    const f32x2 r1 = x - f32x2{__uint_as_float(hh << 16), __uint_as_float(hh & 0xffff0000u)};
    const uint32_t mm = ic_cvt_pk_bf16(r1[0], r1[1]);
    const f32x2 r2 = r1 - f32x2{__uint_as_float(mm << 16), __uint_as_float(mm & 0xffff0000u)};
    ph[p] = hh;
    pm[p] = mm;
    pl[p] = ic_cvt_pk_bf16(r2[0], r2[1]);
  }
  h = __builtin_bit_cast(V4, ph);
  m = __builtin_bit_cast(V4, pm);
  l = __builtin_bit_cast(V4, pl);
}

// 64-lane wave reduction (gfx950 wave64)
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Block reduction of `nv` values per thread (blockDim.x multiple of 64,
// <= 1024).  Result valid in thread 0.  Deterministic order.
template <int NV>
__device__ __forceinline__ void block_sum(float (&v)[NV], float* lds /* >= 16*NV */) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = wave_sum(v[i]);
  __syncthreads();
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < NV; ++i) lds[wid * NV + i] = v[i];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      float s = 0.f;
      for (int w = 0; w < nw; ++w) s += lds[w * NV + i];
      v[i] = s;
    }
  }
  __syncthreads();
}

// Philox4x32-10 (Salmon, Moraes, Dror, Shaw, SC'11; the Random123 philox4x32_R with R = 10):
// per round (hi, lo) = mulhilo(M0, c0), mulhilo(M1, c2); c = {hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0};
// the key is bumped by the Weyl constants (0x9E3779B9, 0xBB67AE85) between rounds.
// Pinned to the published Random123 known-answer vectors (tests/test_noise_gpu.py via ic_philox_kat;
// oracle/philox.py restates it for the CPU tests).
__device__ __forceinline__ void philox4x32_10(uint32_t (&c)[4], uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(M0, c[0]), lo0 = M0 * c[0];
    const uint32_t hi1 = __umulhi(M1, c[2]), lo1 = M1 * c[2];
    const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
}

// The training-noise stream: element i of stream `seed` is word (i & 3) of
// Philox4x32-10(counter {i >> 2 (64 bit), 0, 0}, key = seed), mapped to U[0,1)
// by its top 24 bits.  Every Philox evaluation yields four consecutive
// elements; streams are drawn from 4-aligned offsets (noise.py) so a thread
// that handles elements 4j .. 4j+3 evaluates one block (philox_uniform4).
__device__ __forceinline__ float philox_u24(uint32_t w) { return (float)(w >> 8) * (1.0f / 16777216.0f); }

__device__ __forceinline__ floatx4v philox_uniform4(uint64_t seed, uint64_t blk) {
  uint32_t c[4] = {(uint32_t)blk, (uint32_t)(blk >> 32), 0u, 0u};
  philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  return floatx4v{philox_u24(c[0]), philox_u24(c[1]), philox_u24(c[2]), philox_u24(c[3])};
}

__device__ __forceinline__ float philox_uniform(uint64_t seed, uint64_t idx) {
  return philox_uniform4(seed, idx >> 2)[idx & 3];
}
