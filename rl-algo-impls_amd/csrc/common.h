// Shared device helpers for the gfx950 kernels (wave64, CDNA4).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rai_amd.h"

#define RAI_WAVE 64

#define RAI_LAUNCH_CHECK()                      \
  do {                                          \
    hipError_t e__ = hipGetLastError();         \
    if (e__ != hipSuccess) return (int)e__;     \
  } while (0)

static inline hipStream_t rai_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Workgroup barrier for LDS hand-offs only: drains this wave's LDS traffic and meets
// the other waves, but does NOT wait for outstanding global loads/stores
// (__syncthreads() adds s_waitcnt vmcnt(0), which exposes prefetch and store latency).
// Register results of global loads are still waited for by the compiler at first use.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// ---- bounded spins ----------------------------------------------------------
// Spin limits are wall-clock: s_memrealtime is the constant 100 MHz counter (s_memtime, the shader
// clock, was seen to jump under rocprofv3 kernel tracing and fail a healthy wait).  The elapsed
// time is compared signed, so a counter that steps backwards never expires a wait.
constexpr long long RAI_SPIN_LOCAL = 200000000LL;    // 2 s: partners on the same GPU
constexpr long long RAI_SPIN_REMOTE = 6000000000LL;  // 60 s: other ranks (they may still be launching)
// Cross-GPU exchange regions (rai_xdp_*): [0, 2048) u64 step flags [2 nets][8 ranks][16 workgroups],
// [2048, 4096) self-test flags, slots from 4096.  The wide whole-epoch kernel's slots
// (mlp_wide_epoch.hip): [2 parities][world][2 nets][16 workgroups][RAI_XDP_WIDE_SLOTF floats].
constexpr int RAI_XDP_SLOTS_OFF = 4096;
constexpr int RAI_XDP_WIDE_SLOTF = 5376;
__host__ __device__ constexpr long long rai_xdp_wide_bytes(int world) {
  return RAI_XDP_SLOTS_OFF + 2LL * world * 2 * 16 * RAI_XDP_WIDE_SLOTF * 4;
}
__device__ __forceinline__ unsigned long long rai_clock() { return __builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ bool rai_expired(unsigned long long t0, long long limit) {
  return (long long)(rai_clock() - t0) > limit;
}

// Branch-free tanh (libm's tanhf branches on |x| ranges, which diverges across a wave):
// |x| < 0.3: odd Taylor series to x^9 (truncation < 1e-7 relative); otherwise
// 1 - 2 / (exp(2|x|) + 1) with the sign restored (absolute error ~1 ulp of 1).
__device__ __forceinline__ float rai_tanh_bf(float x) {
  const float ax = fabsf(x);
  const float x2 = x * x;
  float p = fmaf(x2, 62.f / 2835.f, -17.f / 315.f);
  p = fmaf(x2, p, 2.f / 15.f);
  p = fmaf(x2, p, -1.f / 3.f);
  const float small = fmaf(x * x2, p, x);
  const float e = __builtin_amdgcn_exp2f(ax * 2.885390081777927f);  // exp(2|x|)
  const float big = fmaf(-2.f, __builtin_amdgcn_rcpf(e + 1.f), 1.f);
  return ax < 0.3f ? small : copysignf(big, x);
}

// ---- wave64 reductions (fixed order -> deterministic) ----------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// The same sums without LDS round trips (each __shfl_xor is a ds_bpermute, ~100+ cycles in a dependent
// chain): lanes pair up by DPP -- xor 1 and xor 2 (quad_perm), the 8-lane half mirror, the 16-lane row
// mirror -- then gfx950's v_permlane16_swap / v_permlane32_swap add the rows' and halves' sums.  Each
// step adds two commuted operands, so every lane ends with the same bits; the association differs from
// wave_sum's (pairing 1, 2, 4, 8, 16, 32 instead of 32 .. 1).  Requires all 64 lanes active.
template <int CTRL>
__device__ __forceinline__ int rai_dpp(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v += __int_as_float(rai_dpp<0xB1>(__float_as_int(v)));   // quad_perm [1,0,3,2]
  v += __int_as_float(rai_dpp<0x4E>(__float_as_int(v)));   // quad_perm [2,3,0,1]
  v += __int_as_float(rai_dpp<0x141>(__float_as_int(v)));  // row_half_mirror
  v += __int_as_float(rai_dpp<0x140>(__float_as_int(v)));  // row_mirror
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  const auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(q[0]) + __uint_as_float(q[1]);
}
template <int CTRL>
__device__ __forceinline__ double rai_dpp_d(double v) {
  const unsigned long long u = __double_as_longlong(v);
  const unsigned lo = (unsigned)rai_dpp<CTRL>((int)(unsigned)u);
  const unsigned hi = (unsigned)rai_dpp<CTRL>((int)(unsigned)(u >> 32));
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ double rai_swap_sum_d(double v, bool half32) {
  const unsigned long long u = __double_as_longlong(v);
  const unsigned lo = (unsigned)u, hi = (unsigned)(u >> 32);
  const auto l = half32 ? __builtin_amdgcn_permlane32_swap(lo, lo, false, false)
                        : __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto h = half32 ? __builtin_amdgcn_permlane32_swap(hi, hi, false, false)
                        : __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  const double a = __longlong_as_double((long long)(((unsigned long long)h[0] << 32) | l[0]));
  const double b = __longlong_as_double((long long)(((unsigned long long)h[1] << 32) | l[1]));
  return a + b;
}
__device__ __forceinline__ double wave_sum_dpp(double v) {
  v += rai_dpp_d<0xB1>(v);
  v += rai_dpp_d<0x4E>(v);
  v += rai_dpp_d<0x141>(v);
  v += rai_dpp_d<0x140>(v);
  v = rai_swap_sum_d(v, false);
  return rai_swap_sum_d(v, true);
}

// Block-wide sum of NV values per thread; every thread receives the totals.
// scratch: >= NV * (blockDim/64) doubles of LDS.
template <int NV>
__device__ __forceinline__ void block_sum(double (&v)[NV], double* scratch) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = wave_sum(v[i]);
  __syncthreads();
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < NV; ++i) scratch[i * nw + w] = v[i];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    double s = 0.0;
    for (int j = 0; j < nw; ++j) s += scratch[i * nw + j];
    v[i] = s;
  }
  __syncthreads();
}

// beta^n for the Adam bias corrections by binary exponentiation: <= 2*log2(n) double
// multiplies (a few ulps from libm's pow, far below fp32) instead of the double-precision
// pow() sequence, which costs tens of microseconds of FP64 work per launch.
__device__ __forceinline__ double ipow(double b, long long n) {
  double r = 1.0;
  while (n > 0) {
    if (n & 1) r *= b;
    b *= b;
    n >>= 1;
  }
  return r;
}

// ---- Philox4x32-10 counter RNG ---------------------------------------------
struct Philox4 {
  uint32_t x, y, z, w;
};
__device__ __forceinline__ Philox4 philox4x32_10(uint64_t ctr_hi, uint64_t ctr_lo, uint64_t key) {
  uint32_t c0 = (uint32_t)ctr_lo, c1 = (uint32_t)(ctr_lo >> 32);
  uint32_t c2 = (uint32_t)ctr_hi, c3 = (uint32_t)(ctr_hi >> 32);
  uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    uint32_t hi0 = __umulhi(M0, c0), lo0 = M0 * c0;
    uint32_t hi1 = __umulhi(M1, c2), lo1 = M1 * c2;
    uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return Philox4{c0, c1, c2, c3};
}
// uniform in (0, 1]  (never 0 -> safe for log)
__device__ __forceinline__ float u01_open0(uint32_t x) {
  return ((float)(x >> 8) + 1.0f) * (1.0f / 16777216.0f);
}
