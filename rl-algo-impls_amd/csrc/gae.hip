// GAE reverse scan + fused returns for gfx950.
//
// Restates rl_algo_impls/shared/gae.py:97-124 (compute_advantages) and
// rl_algo_impls/rollout/vec_rollout.py:88 (returns = advantages + values).
//
// Layout in HBM: rewards/values/adv/returns (T, C) fp32 with C = N*K columns,
// episode_starts (T, N) u8.  A block owns 64 consecutive columns (one wave-wide,
// so every row load/store is a coalesced 256-B segment) and walks T backwards
// in 32-row tiles:
//   * all four waves load a tile's rows (8 rows each) and compute the
//     carry-independent part delta_t and next_nonterminal into LDS
//     (double-buffered), and
//   * wave 0 runs the serial carry recurrence over the previous tile from LDS,
//     writing adv and returns, while the other waves' loads for the next tile
//     are in flight.
// Exact mode keeps the reference's numpy precision sequence bit for bit:
//   t1    = fp32(fp32(gamma) * V_next)          (gamma Python float; fp64 if ndarray)
//   delta = (f64(r_t) + f64(t1) * nn) - f64(V_t)
//   carry = delta + ((gamma*lambda)_f64 * nn) * carry      (fp64 carry)
//   adv_t = fp32(carry);  ret_t = adv_t + V_t (fp32)
// FP contraction is disabled for this file (-ffp-contract=off + pragma) so no
// multiply-add is fused differently from numpy.
#include "common.h"

#pragma clang fp contract(off)

namespace {

constexpr int GAE_COLS = 64;
constexpr int GAE_WAVES = 4;
constexpr int GAE_TT = 32;
constexpr int ROWS_PER_WAVE = GAE_TT / GAE_WAVES;

struct GaeArgs {
  const float* rewards;
  const float* values;
  const uint8_t* es;
  const uint8_t* next_es;
  const float* next_values;
  float* adv;
  float* ret;
  int64_t T, N, C;
  int32_t K;
  int32_t gamma_is_vector;
  double gamma[RAI_MAX_K];
  double gl[RAI_MAX_K];
  float gamma32[RAI_MAX_K];
  float gl32[RAI_MAX_K];
};

template <typename Acc>
__device__ __forceinline__ Acc gae_delta(float r, float v, float vn, uint8_t esn, bool gvec,
                                         float g32, double g64, Acc& nn_out);

template <>
__device__ __forceinline__ double gae_delta<double>(float r, float v, float vn, uint8_t esn,
                                                    bool gvec, float g32, double g64,
                                                    double& nn_out) {
  const double nn = 1.0 - (double)(esn != 0);
  double t1;
  if (gvec) {
    t1 = g64 * (double)vn;
  } else {
    const float t1f = g32 * vn;
    t1 = (double)t1f;
  }
  nn_out = nn;
  return ((double)r + t1 * nn) - (double)v;
}

template <>
__device__ __forceinline__ float gae_delta<float>(float r, float v, float vn, uint8_t esn,
                                                  bool /*gvec*/, float g32, double /*g64*/,
                                                  float& nn_out) {
  const float nn = esn ? 0.0f : 1.0f;
  nn_out = nn;
  return (r + (g32 * vn) * nn) - v;
}

template <typename Acc>
__global__ __launch_bounds__(256) void gae_kernel(const GaeArgs a) {
  __shared__ Acc delta_s[2][GAE_TT][GAE_COLS];
  __shared__ uint8_t nn_s[2][GAE_TT][GAE_COLS];
  __shared__ float v_s[2][GAE_TT][GAE_COLS];

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.x * GAE_COLS + lane;
  const bool valid = c < a.C;
  const int64_t cc = valid ? c : 0;
  const int64_t n = cc / a.K;
  const int k = (int)(cc - n * a.K);
  const bool gvec = a.gamma_is_vector != 0;
  const float g32 = a.gamma32[k];
  const double g64 = a.gamma[k];
  const Acc gl = (sizeof(Acc) == 8) ? (Acc)a.gl[k] : (Acc)a.gl32[k];
  const int64_t T = a.T;
  const int ntiles = (int)((T + GAE_TT - 1) / GAE_TT);

  float r_reg[ROWS_PER_WAVE], v_reg[ROWS_PER_WAVE], vn_reg[ROWS_PER_WAVE];
  uint8_t e_reg[ROWS_PER_WAVE];

  // Issue this wave's loads for tile `tile` into registers.
  auto issue_loads = [&](int tile) {
    const int64_t lo = T - (int64_t)(tile + 1) * GAE_TT;
#pragma unroll
    for (int j = 0; j < ROWS_PER_WAVE; ++j) {
      const int lr = wave + j * GAE_WAVES;
      const int64_t t = lo + lr;
      r_reg[j] = 0.f; v_reg[j] = 0.f; vn_reg[j] = 0.f; e_reg[j] = 0;
      if (t >= 0 && valid) {
        r_reg[j] = a.rewards[t * a.C + c];
        v_reg[j] = a.values[t * a.C + c];
        if (t == T - 1) {
          vn_reg[j] = a.next_values[c];
          e_reg[j] = a.next_es[n];
        } else {
          vn_reg[j] = a.values[(t + 1) * a.C + c];
          e_reg[j] = a.es[(t + 1) * a.N + n];
        }
      }
    }
  };
  // Carry-independent part -> LDS buffer `buf`.
  auto stage = [&](int buf) {
#pragma unroll
    for (int j = 0; j < ROWS_PER_WAVE; ++j) {
      const int lr = wave + j * GAE_WAVES;
      Acc nn;
      const Acc d = gae_delta<Acc>(r_reg[j], v_reg[j], vn_reg[j], e_reg[j], gvec, g32, g64, nn);
      delta_s[buf][lr][lane] = d;
      nn_s[buf][lr][lane] = (nn != (Acc)0) ? 1 : 0;
      v_s[buf][lr][lane] = v_reg[j];
    }
  };

  issue_loads(0);
  stage(0);
  __syncthreads();

  Acc carry = (Acc)0;
  for (int tile = 0; tile < ntiles; ++tile) {
    const int buf = tile & 1;
    const bool more = tile + 1 < ntiles;
    if (more) issue_loads(tile + 1);
    if (wave == 0) {
      const int64_t lo = T - (int64_t)(tile + 1) * GAE_TT;
      for (int lr = GAE_TT - 1; lr >= 0; --lr) {
        const int64_t t = lo + lr;
        if (t < 0) break;
        const Acc d = delta_s[buf][lr][lane];
        const Acc nn = nn_s[buf][lr][lane] ? (Acc)1 : (Acc)0;
        const Acc coef = gl * nn;
        carry = d + coef * carry;
        if (valid) {
          const float adv = (float)carry;
          a.adv[t * a.C + c] = adv;
          if (a.ret) a.ret[t * a.C + c] = adv + v_s[buf][lr][lane];
        }
      }
    }
    if (more) stage(buf ^ 1);
    __syncthreads();
  }
}

}  // namespace

extern "C" int rai_gae(const float* rewards, const float* values, const uint8_t* episode_starts,
                       const uint8_t* next_episode_starts, const float* next_values, int64_t T,
                       int64_t N, int32_t K, const double* gamma, const double* gae_lambda,
                       int32_t gamma_is_vector, int32_t mode, float* adv_out, float* returns_out,
                       void* stream) {
  if (T < 0 || N < 0 || K < 1) return RAI_E_SHAPE;
  if (K > RAI_MAX_K) return RAI_E_TOO_MANY_COLUMNS;
  if (mode != RAI_GAE_EXACT && mode != RAI_GAE_FAST) return RAI_E_MODE;
  if (T == 0 || N == 0) return RAI_OK;
  if (!rewards || !values || !episode_starts || !next_episode_starts || !next_values ||
      !gamma || !gae_lambda || !adv_out)
    return RAI_E_NULLPTR;
  GaeArgs a;
  a.rewards = rewards;
  a.values = values;
  a.es = episode_starts;
  a.next_es = next_episode_starts;
  a.next_values = next_values;
  a.adv = adv_out;
  a.ret = returns_out;
  a.T = T;
  a.N = N;
  a.K = K;
  a.C = N * (int64_t)K;
  a.gamma_is_vector = gamma_is_vector;
  for (int k = 0; k < RAI_MAX_K; ++k) {
    const int kk = k < K ? k : 0;
    a.gamma[k] = gamma[kk];
    a.gl[k] = gamma[kk] * gae_lambda[kk];  // Python/numpy f64 product
    a.gamma32[k] = (float)gamma[kk];
    a.gl32[k] = (float)a.gl[k];
  }
  const int64_t blocks = (a.C + GAE_COLS - 1) / GAE_COLS;
  if (mode == RAI_GAE_EXACT)
    hipLaunchKernelGGL(gae_kernel<double>, dim3((unsigned)blocks), dim3(256), 0, rai_stream(stream), a);
  else
    hipLaunchKernelGGL(gae_kernel<float>, dim3((unsigned)blocks), dim3(256), 0, rai_stream(stream), a);
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}
