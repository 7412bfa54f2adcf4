// Multi-tensor AdamW with fused gradient value clipping (the optimizer step
// of the reference's training loop: torch.optim.AdamW built by
// solver/optim.py:20-45, after clip_grad_value_ in engine/trainer.py:189-190).
//
// Per element (torch.optim.AdamW, amsgrad=False, maximize=False):
//   g  = clamp(g, -clip, clip)            (when clip > 0; written back, as the
//                                          reference clips .grad in place)
//   p *= 1 - lr * wd
//   m  = m + (1 - b1) * (g - m)           (torch: exp_avg.lerp_(grad, 1 - b1))
//   v  = b2 * v + (1 - b2) * g * g
//   p -= (lr / bc1) * m / (sqrt(v) / sqrt(bc2) + eps)
//
// One launch covers up to IC_ADAMW_MAXT tensors: the tensor table travels in
// the kernel arguments (no device-side table to upload), each block owns a
// 4096-element chunk of one tensor and finds it by scanning the prefix table.
// The step is HBM-bound: 7 floats of traffic per element (read p, g, m, v;
// write p, m, v; + g when clipping).
#include "../../include/imgcomp.h"
#include "common.h"

namespace {

constexpr int MAXT = 48;          // tensors per launch (kernel-argument budget)
constexpr int CHUNK = 4096;

struct AdamWArgs {
  float* p[MAXT];
  float* g[MAXT];
  float* m[MAXT];
  float* v[MAXT];
  float lr[MAXT];
  float wd[MAXT];
  int chunk_begin[MAXT + 1];      // prefix sum of chunks per tensor
  long long n[MAXT];
  int nt;
  float omb1, b2, omb2, eps, clip, inv_bc1, inv_bc2_sqrt;  // omb = 1 - beta (formed in double)
};

__global__ void __launch_bounds__(256) adamw_kernel(const AdamWArgs a) {
  const int blk = blockIdx.x;
  int t = 0;
  while (t + 1 < a.nt && a.chunk_begin[t + 1] <= blk) ++t;
  const long long base = (long long)(blk - a.chunk_begin[t]) * CHUNK;
  const long long n = a.n[t];
  float* __restrict__ p = a.p[t];
  float* __restrict__ g = a.g[t];
  float* __restrict__ m = a.m[t];
  float* __restrict__ v = a.v[t];
  const float lr = a.lr[t], decay = 1.f - a.lr[t] * a.wd[t];
  const float step = lr * a.inv_bc1;
  for (long long i = base + threadIdx.x; i < base + CHUNK && i < n; i += 256) {
    float gi = g[i];
    if (a.clip > 0.f) {
      gi = fminf(fmaxf(gi, -a.clip), a.clip);
      g[i] = gi;
    }
    float pi = p[i] * decay;
    float mi = m[i];
    mi = mi + a.omb1 * (gi - mi);
    const float vi = a.b2 * v[i] + a.omb2 * gi * gi;
    const float denom = sqrtf(vi) * a.inv_bc2_sqrt + a.eps;
    pi = pi - step * (mi / denom);
    p[i] = pi;
    m[i] = mi;
    v[i] = vi;
  }
}

}  // namespace

extern "C" {

int ic_adamw_step(const ic_adamw_tensor* ts, int ntensors, double beta1, double beta2, float eps, float clip,
                  long long step, void* stream) {
  if (ntensors < 0 || step < 1) return IC_ERR_ARG;
  const double bc1 = 1.0 - pow((double)beta1, (double)step);
  const double bc2 = 1.0 - pow((double)beta2, (double)step);
  int cur = 0;
  while (cur < ntensors) {
    AdamWArgs a;
    a.nt = 0;
    int chunks = 0;
    for (; cur < ntensors && a.nt < MAXT; ++cur) {
      const ic_adamw_tensor& e = ts[cur];
      if (e.n <= 0) continue;
      const int k = a.nt++;
      a.p[k] = e.param; a.g[k] = e.grad; a.m[k] = e.exp_avg; a.v[k] = e.exp_avg_sq;
      a.lr[k] = e.lr; a.wd[k] = e.weight_decay; a.n[k] = e.n;
      a.chunk_begin[k] = chunks;
      chunks += (int)((e.n + CHUNK - 1) / CHUNK);
    }
    if (a.nt == 0) continue;
    a.chunk_begin[a.nt] = chunks;
    a.omb1 = (float)(1.0 - beta1);   // torch: lerp weight 1 - beta1 (Python double -> fp32)
    a.b2 = (float)beta2;
    a.omb2 = (float)(1.0 - beta2);
    a.eps = eps; a.clip = clip;
    a.inv_bc1 = (float)(1.0 / bc1);
    a.inv_bc2_sqrt = (float)(1.0 / sqrt(bc2));
    hipLaunchKernelGGL(adamw_kernel, dim3(chunks), dim3(256), 0, (hipStream_t)stream, a);
    IC_CHECK_LAUNCH();
  }
  return IC_OK;
}

}  // extern "C"
