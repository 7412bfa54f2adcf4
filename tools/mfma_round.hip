// How the bf16 MFMAs of gfx950 sum their products: the exact sum of the
// products (and the accumulator) is compared with round-to-nearest-even (RNE)
// and round-toward-zero (RZ) of it, for each instruction the split kernels
// could use.  Probes: small products next to a large one in the same K group
// (are they truncated to the large one's grid?), and where in K a small product
// loses its bits (the adder-tree grouping).
// usage: hipcc --offload-arch=gfx950 -O2 tools/mfma_round.hip -o tools/_abl/mfma_round && tools/_abl/mfma_round
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short shortx4 __attribute__((ext_vector_type(4)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

// D[0][0] = c + sum_k a[k] b[k], K = 32 (two instructions for K 16 shapes)
// 16x16x32: lane l holds A[l&15][8(l>>4)..+8], B[8(l>>4)..+8][l&15]; D[0][0] in lane 0 reg 0
// 32x32x16: lane l holds A[l&31][8(l>>5)..+8], B[8(l>>5)..+8][l&31]; D[0][0] in lane 0 reg 0
// 16x16x16 (bf16_1k): lane l holds A[l&15][4(l>>4)..+4]
// 32x32x8 (bf16_1k): lane l holds A[l&31][4(l>>5)..+4]
__global__ void k(const float* a, const float* b, const float* c, float* out, int which) {
  const int l = threadIdx.x;
  float r = 0.f;
  if (which == 0) {
    const int row = l & 15, g = l >> 4;
    bf16x8 av, bv;
    for (int e = 0; e < 8; ++e) {
      av[e] = (__bf16)(row == 0 ? a[8 * g + e] : 0.f);
      bv[e] = (__bf16)(row == 0 ? b[8 * g + e] : 0.f);
    }
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    if (l == 0) acc[0] = c[0];
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc, 0, 0, 0);
    r = acc[0];
  } else if (which == 1) {
    const int row = l & 31, g = l >> 5;
    floatx16 acc;
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
    if (l == 0) acc[0] = c[0];
    for (int s = 0; s < 2; ++s) {
      bf16x8 av, bv;
      for (int e = 0; e < 8; ++e) {
        av[e] = (__bf16)(row == 0 ? a[16 * s + 8 * g + e] : 0.f);
        bv[e] = (__bf16)(row == 0 ? b[16 * s + 8 * g + e] : 0.f);
      }
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc, 0, 0, 0);
    }
    r = acc[0];
  } else if (which == 2) {
    const int row = l & 15, g = l >> 4;
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    if (l == 0) acc[0] = c[0];
    for (int s = 0; s < 2; ++s) {
      shortx4 av, bv;
      for (int e = 0; e < 4; ++e) {
        __bf16 x = (__bf16)(row == 0 ? a[16 * s + 4 * g + e] : 0.f);
        __bf16 y = (__bf16)(row == 0 ? b[16 * s + 4 * g + e] : 0.f);
        av[e] = __builtin_bit_cast(short, x);
        bv[e] = __builtin_bit_cast(short, y);
      }
      acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(av, bv, acc, 0, 0, 0);
    }
    r = acc[0];
  } else {
    const int row = l & 31, g = l >> 5;
    floatx16 acc;
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
    if (l == 0) acc[0] = c[0];
    for (int s = 0; s < 4; ++s) {
      shortx4 av, bv;
      for (int e = 0; e < 4; ++e) {
        __bf16 x = (__bf16)(row == 0 ? a[8 * s + 4 * g + e] : 0.f);
        __bf16 y = (__bf16)(row == 0 ? b[8 * s + 4 * g + e] : 0.f);
        av[e] = __builtin_bit_cast(short, x);
        bv[e] = __builtin_bit_cast(short, y);
      }
      acc = __builtin_amdgcn_mfma_f32_32x32x8bf16_1k(av, bv, acc, 0, 0, 0);
    }
    r = acc[0];
  }
  if (l == 0) out[0] = r;
}

static float *da, *db, *dc, *dout;

static float run(const float* a, const float* b, float c, int which) {
  float out;
  hipMemcpy(da, a, 128, hipMemcpyHostToDevice);
  hipMemcpy(db, b, 128, hipMemcpyHostToDevice);
  hipMemcpy(dc, &c, 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, da, db, dc, dout, which);
  hipMemcpy(&out, dout, 4, hipMemcpyDeviceToHost);
  return out;
}

static const char* NAMES[4] = {"16x16x32", "32x32x16", "16x16x16_1k", "32x32x8_1k"};

static void report(const char* name, const float* a, const float* b, float c) {
  long double ex = c;
  for (int i = 0; i < 32; ++i) ex += (long double)a[i] * b[i];
  const float rne = (float)ex;
  float rz = rne;
  if (fabsl((long double)rz) > fabsl(ex)) rz = nextafterf(rz, 0.f);
  printf("%-40s exact %.12Le |", name, ex);
  for (int w = 0; w < 4; ++w) {
    const float got = run(a, b, c, w);
    printf(" %s %.9e %s%s |", NAMES[w], got, got == rne ? "N" : "-", got == rz ? "Z" : "-");
  }
  printf("\n");
}

int main() {
  hipMalloc(&da, 128); hipMalloc(&db, 128); hipMalloc(&dc, 4); hipMalloc(&dout, 4);
  const float u = ldexpf(1.f, -23);  // ulp of 1.0
  float a[32], b[32];
  auto zero = [&]() { memset(a, 0, sizeof a); memset(b, 0, sizeof b); };
  zero(); a[0] = 0.75f * u; b[0] = 1.f; report("acc 1 + 0.75 ulp (one product)", a, b, 1.f);
  zero(); a[0] = 0.5f * u; b[0] = 1.f; report("acc 1 + 0.5 ulp (tie, even below)", a, b, 1.f);
  zero(); a[0] = 0.5f * u; b[0] = 1.f; report("acc 1+ulp + 0.5 ulp (tie, even above)", a, b, 1.f + u);
  zero(); for (int i = 0; i < 31; ++i) { a[i] = 1.f; b[i] = ldexpf(1.f, -28); } report("acc 1 + 31 x 2^-28", a, b, 1.f);
  zero(); a[0] = 1.f; b[0] = 1.f; for (int i = 1; i < 32; ++i) { a[i] = 1.f; b[i] = ldexpf(1.f, -28); }
  report("acc 0, products 1 + 31 x 2^-28", a, b, 0.f);
  zero(); a[0] = 1.f; b[0] = 1.f; for (int i = 1; i < 32; ++i) { a[i] = -1.f; b[i] = ldexpf(1.f, -28); }
  report("acc 0, products 1 - 31 x 2^-28", a, b, 0.f);
  zero(); a[0] = 1.f; b[0] = 1.f; a[1] = 1.f; b[1] = -1.f; a[2] = 0.75f * u; b[2] = 1.f;
  report("acc 0, 1 - 1 + 0.75 ulp (cancellation)", a, b, 0.f);
  zero(); a[0] = 0.75f * u; b[0] = 1.f; a[1] = 1.f; b[1] = 1.f; report("acc 0, products 1 + 0.75 ulp", a, b, 0.f);
  zero(); a[0] = 1.f; b[0] = ldexpf(1.f, -30); report("acc 1 + 2^-30 (lone product)", a, b, 1.f);
  // where does a small product lose its bits: a product 1 at k = 0, 1.5 x 2^-24 at k = j
  for (int j = 1; j < 32; ++j) {
    zero(); a[0] = 1.f; b[0] = 1.f; a[j] = 0.75f * u; b[j] = 1.f;
    char nm[64];
    snprintf(nm, sizeof nm, "acc 0, 1 @0 + 0.75 ulp @%d", j);
    report(nm, a, b, 0.f);
  }
  // a product 2^-9 next to 1 (bits below 2^-24 of 1 would be lost): exact in 24 bits?
  zero(); a[0] = 1.f; b[0] = 1.f; a[5] = 1.f + ldexpf(1.f, -7); b[5] = ldexpf(1.f + ldexpf(1.f, -7), -9);
  report("acc 0, 1 + (1+2^-7)^2 2^-9", a, b, 0.f);
  zero(); a[0] = 1.f; b[0] = 1.f; a[5] = 1.f + ldexpf(1.f, -7); b[5] = ldexpf(1.f + ldexpf(1.f, -7), -12);
  report("acc 0, 1 + (1+2^-7)^2 2^-12", a, b, 0.f);
  zero(); a[0] = 1.f; b[0] = 1.f; a[5] = -(1.f + ldexpf(1.f, -7)); b[5] = ldexpf(1.f + ldexpf(1.f, -7), -12);
  report("acc 0, 1 - (1+2^-7)^2 2^-12", a, b, 0.f);
  return 0;
}
