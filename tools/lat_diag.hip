// Diagnostic (not shipped): dependent-chain latency of x = d + c*x in f64 / f32 on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#pragma clang fp contract(off)
template <typename T>
__global__ void chain(T* out, T c, T d, int n, long long* cyc) {
  T x = (T)threadIdx.x;
  long long t0 = clock64();
  for (int i = 0; i < n; ++i) { x = d + c * x; }
  long long t1 = clock64();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}
int main() {
  double* o; float* of; long long* cyc; long long h;
  hipMalloc(&o, 64 * 8); hipMalloc(&of, 64 * 4); hipMalloc(&cyc, 8);
  const int n = 100000;
  chain<double><<<1, 64>>>(o, 0.5, 1.0, n, cyc); hipDeviceSynchronize();
  hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost); printf("f64 mul+add dependent: %.1f cycles/iter\n", (double)h / n);
  chain<float><<<1, 64>>>(of, 0.5f, 1.0f, n, cyc); hipDeviceSynchronize();
  hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost); printf("f32 mul+add dependent: %.1f cycles/iter\n", (double)h / n);
  return 0;
}
