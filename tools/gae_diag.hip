// Diagnostic harness (not shipped): times rai_gae variants built with -DGAE_DIAG=n.
#include "../rl-algo-impls_amd/csrc/gae.hip"
#include <cstdio>
#include <vector>
int main(int argc, char** argv) {
  int64_t T = argc > 1 ? atol(argv[1]) : 128, N = argc > 2 ? atol(argv[2]) : 4096;
  size_t n = T * N;
  float *r, *v, *nv, *adv, *ret;
  uint8_t *es, *nes;
  hipMalloc(&r, n * 4); hipMalloc(&v, n * 4); hipMalloc(&adv, n * 4); hipMalloc(&ret, n * 4);
  hipMalloc(&nv, N * 4); hipMalloc(&es, n); hipMalloc(&nes, N);
  hipMemset(r, 0, n * 4); hipMemset(v, 0, n * 4); hipMemset(nv, 0, N * 4); hipMemset(es, 0, n); hipMemset(nes, 0, N);
  double g = 0.99, l = 0.95;
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int i = 0; i < 10; ++i) rai_gae(r, v, es, nes, nv, T, N, 1, &g, &l, 0, 0, adv, ret, nullptr);
  hipEventRecord(e0);
  const int reps = 100;
  for (int i = 0; i < reps; ++i) rai_gae(r, v, es, nes, nv, T, N, 1, &g, &l, 0, 0, adv, ret, nullptr);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  printf("DIAG=%d T=%ld N=%ld: %.2f us/launch\n", GAE_DIAG, (long)T, (long)N, ms * 1e3 / reps);
#if GAE_DIAG & 8
  long long st[8];
  hipMemcpyFromSymbol(st, HIP_SYMBOL(gae_stamps), sizeof(st));
  const char* nm[] = {"load-wait+stage", "barrier1", "chain (wave0)", "barrier2", "stores", "cur=nxt wait"};
  for (int i = 0; i < 6; ++i) printf("  %-18s %10.1f cycles/launch\n", nm[i], (double)st[i] / (reps + 10));
#endif
  return 0;
}
