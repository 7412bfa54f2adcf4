// Phase timing of the fused GDN backward: per-wave s_memtime stamps at each
// barrier (GDN_PROF build of gdn_fused.hip), averaged over blocks and tiles.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DGDN_PROF tools/gdn_prof.hip -o tools/_abl/gdn_prof
#include "../image_compression_amd/csrc/gdn_fused.hip"
#include <cstdio>
#include <vector>

template <bool X3>
void run() {
  const int C = 192;
  const long long P = 32LL * 128 * 128;
  std::vector<float> hx(P * C), hn(P * C), hg(C * C);
  for (size_t i = 0; i < hx.size(); ++i) {
    hx[i] = (float)((i * 2654435761u) % 1000) / 500.f - 1.f;
    hn[i] = 1.f + (float)((i * 40503u) % 1000) / 1000.f;
  }
  for (int i = 0; i < C * C; ++i) hg[i] = 0.001f * (float)(i % 7);
  float *x, *n, *dy, *g, *dx, *slab;
  hipMalloc(&x, P * C * 4); hipMalloc(&n, P * C * 4); hipMalloc(&dy, P * C * 4); hipMalloc(&dx, P * C * 4);
  hipMalloc(&g, C * C * 4); hipMalloc(&slab, 256 * (C * C + C) * 4);
  hipMemcpy(x, hx.data(), P * C * 4, hipMemcpyHostToDevice);
  hipMemcpy(dy, hx.data(), P * C * 4, hipMemcpyHostToDevice);
  hipMemcpy(n, hn.data(), P * C * 4, hipMemcpyHostToDevice);
  hipMemcpy(g, hg.data(), C * C * 4, hipMemcpyHostToDevice);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  float best = 1e9;
  for (int r = 0; r < 10; ++r) {
    hipEventRecord(e0);
    hipLaunchKernelGGL((gdn_bwd_fused_kernel<192, X3>), dim3(256), dim3(512), 0, 0, x, n, dy, g, 0, dx, slab, (uint32_t)P);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1); if (ms < best) best = ms;
  }
  std::vector<unsigned long long> pr(256 * 8 * 16 * 6);
  hipMemcpyFromSymbol(pr.data(), HIP_SYMBOL(gdn_prof), pr.size() * 8);
  printf("%s: kernel %.3f ms  (tiles/block %lld)\n", X3 ? "split dgamma" : "fp32", best, (P / 16 + 255) / 256);
  const char* names[6] = {"B1", "phaseA", "B2", "gemm", "epi", "B3"};
  for (int w : {0, 4}) {
    double d[6] = {0}, per = 0; int cnt = 0;
    for (int b = 0; b < 256; ++b)
      for (int it = 2; it < 15; ++it) {
        const unsigned long long* t = &pr[((b * 8 + w) * 16 + it) * 6];
        const unsigned long long* tn = &pr[((b * 8 + w) * 16 + it + 1) * 6];
        for (int e = 1; e < 6; ++e) d[e] += (double)(t[e] - t[e - 1]);
        d[0] += (double)(tn[0] - t[5]);
        per += (double)(tn[0] - t[0]); ++cnt;
      }
    printf("wave %d: tile period %.0f clk |", w, per / cnt);
    for (int e = 1; e < 6; ++e) printf(" %s->%s %.0f", names[e - 1], names[e], d[e] / cnt);
    printf(" | B3->B1 %.0f\n", d[0] / cnt);
  }
  hipFree(x); hipFree(n); hipFree(dy); hipFree(dx); hipFree(g); hipFree(slab);
}

int main() {
  run<false>();
  run<true>();
  return 0;
}
