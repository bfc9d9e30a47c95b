// Diagnostic (not shipped): round-trip latency of an 8-byte {tag,value} granule
// exchange between two workgroups (the fused MLP kernel's grad-norm exchange).
// Variants: granule placement (same line / own 128-B lines), poll flavour
// (relaxed agent load vs. returning atomic), s_sleep in the spin, and partner
// placement (block 1 = other XCD vs block 8 = same XCD under round-robin dispatch).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned long long u64;

template <int POLL, int SLEEP>
__device__ u64 poll(u64* p, unsigned tag) {
  for (long long spins = 0; spins < (1ll << 26); ++spins) {
    u64 x;
    if (POLL == 0) x = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else x = __hip_atomic_fetch_or(p, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((unsigned)(x >> 32) == tag) return x;
    if (SLEEP) __builtin_amdgcn_s_sleep(1);
  }
  return 0;
}

template <int POLL, int SLEEP>
__global__ void pingpong(u64* g, int stride, int partner, int iters, long long* cyc) {
  const int b = blockIdx.x;
  if (b != 0 && b != partner) return;
  if (threadIdx.x != 0) return;
  const int me = b == 0 ? 0 : 1;
  u64* mine = g + me * stride;
  u64* other = g + (1 - me) * stride;
  long long t0 = clock64();
  for (int i = 1; i <= iters; ++i) {
    if (me == 0) {
      __hip_atomic_store(mine, ((u64)i << 32) | 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      poll<POLL, SLEEP>(other, i);
    } else {
      poll<POLL, SLEEP>(other, i);
      __hip_atomic_store(mine, ((u64)i << 32) | 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  long long t1 = clock64();
  if (me == 0) *cyc = t1 - t0;
}

template <int POLL, int SLEEP>
void run(const char* name, u64* g, long long* cyc, int stride, int partner) {
  const int iters = 2000;
  hipMemset(g, 0, 4096);
  hipLaunchKernelGGL((pingpong<POLL, SLEEP>), dim3(partner + 1), dim3(64), 0, 0, g, stride, partner, iters, cyc);
  hipDeviceSynchronize();
  long long h = 0;
  hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipMemset(g, 0, 4096);
  hipEventRecord(e0);
  hipLaunchKernelGGL((pingpong<POLL, SLEEP>), dim3(partner + 1), dim3(64), 0, 0, g, stride, partner, iters, cyc);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  printf("%-34s stride=%3d partner=%d: %8.1f clock64/round-trip  %6.3f us/round-trip\n", name, stride, partner,
         (double)h / iters, ms * 1e3 / iters);
}

int main() {
  u64* g;
  long long* cyc;
  hipMalloc(&g, 4096);
  hipMalloc(&cyc, 8);
  for (int partner : {1, 8}) {
    for (int stride : {1, 16}) {
      run<0, 1>("load poll + s_sleep(1)", g, cyc, stride, partner);
      run<0, 0>("load poll, no sleep", g, cyc, stride, partner);
      run<1, 1>("atomic fetch_or poll + s_sleep(1)", g, cyc, stride, partner);
      run<1, 0>("atomic fetch_or poll, no sleep", g, cyc, stride, partner);
    }
  }
  return 0;
}
