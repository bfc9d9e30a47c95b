// Probe: does the f32 MFMA (v_mfma_f32_16x16x4_f32) overlap with independent f32 VALU work in the same wave,
// or do they share the SIMD's FP32 datapath?  One wave per SIMD (256-thread block, one block per CU), a loop
// of 4 independent MFMA accumulator chains with V independent v_fma_f32 per MFMA; shader cycles per loop
// iteration from s_memtime.  Diagnostic tool (hipcc --offload-arch=gfx950 -O3 tools/mfma_valu_overlap.hip).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));

template <int V, bool MF>
__global__ __launch_bounds__(256, 1) void probe(float* out, unsigned long long* cyc, int iters, float s) {
  f4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  float a = threadIdx.x * 1e-3f, b = s;
  float v[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = a + k;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (MF) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c3, 0, 0, 0);
      }
#pragma unroll
      for (int k = 0; k < V; ++k) v[k & 7] = fmaf(v[k & 7], 1.0001f, 0.5f);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float r = c0[0] + c1[1] + c2[2] + c3[3];
#pragma unroll
  for (int k = 0; k < 8; ++k) r += v[k];
  out[blockIdx.x * 256 + threadIdx.x] = r;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int V, bool MF>
void run(const char* name, float* out, unsigned long long* cyc, int iters) {
  hipLaunchKernelGGL((probe<V, MF>), dim3(256), dim3(256), 0, 0, out, cyc, iters, 1.0f);
  hipDeviceSynchronize();
  hipLaunchKernelGGL((probe<V, MF>), dim3(256), dim3(256), 0, 0, out, cyc, iters, 1.0f);
  unsigned long long h[256];
  hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < 256; ++i) m += h[i];
  m /= 256;
  printf("%-28s cycles per 16 MFMA-slots: %8.1f  (per MFMA %.1f)\n", name, m / iters, m / iters / 16.0);
}

int main() {
  float* out;
  unsigned long long* cyc;
  hipMalloc(&out, 256 * 256 * 4);
  hipMalloc(&cyc, 256 * 8);
  const int it = 20000;
  run<0, true>("mfma only", out, cyc, it);
  run<2, true>("mfma + 2 fma each", out, cyc, it);
  run<4, true>("mfma + 4 fma each", out, cyc, it);
  run<6, true>("mfma + 6 fma each", out, cyc, it);
  run<8, true>("mfma + 8 fma each", out, cyc, it);
  run<4, false>("4 fma each, no mfma", out, cyc, it);
  run<8, false>("8 fma each, no mfma", out, cyc, it);
  return 0;
}
