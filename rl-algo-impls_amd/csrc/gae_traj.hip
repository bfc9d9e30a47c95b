// Ragged-batch GAE for per-trajectory rollouts on gfx950.
//
// Restates the two trajectory-level advantage operators of the reference:
//   kind 0  TrajectoryBuilder.trajectory   rl_algo_impls/rollout/trajectory.py:56-92
//           = compute_advantages (rl_algo_impls/shared/gae.py:97-124) over ONE trajectory with
//             episode_starts = [True, dones[:-1]], next_episode_starts = dones[-1],
//             next_values = the caller's or zeros.
//   kind 1  DiscreteSkipsTrajectoryBuilder.trajectory
//           rl_algo_impls/rollout/discrete_skips_trajectory_builder.py:64-109: semi-MDP GAE with
//           gamma ** steps_elapsed[t] in both the bootstrap and the carry, no episode cut inside a
//           trajectory, next value 0 when the trajectory ended in a terminal step.
// Many trajectories of different lengths are processed in one launch: the rows of all
// trajectories are concatenated ((sum L) x K row-major fp32, K value columns) and offsets[s]
// gives the first row of trajectory s.
//
// One 64-lane wave per trajectory walks it backwards in 64-row tiles: the wave loads the tile's
// rows x K contiguous floats (coalesced), forms every carry-independent term (delta_t and the
// carry coefficient) in parallel into LDS, then lanes k < K run the serial recurrence of column k
// out of LDS, and the wave stores adv (+ returns = adv + V) coalesced.
//
// Precision (mode 0 = exact): kind 0 follows rai_gae's numpy sequence bit for bit (fp32 gamma*V
// for a Python-float gamma, fp64 for an ndarray gamma, fp64 carry).  kind 1: gamma ** k is an
// np.float64 (numpy pow; the host passes the table gk[s][k] = gamma ** np.int32(s) computed by
// numpy itself and gkl = gk * lambda), so under numpy >= 2 (NEP 50) every term is fp64:
//   delta = (f64(r) + gk * f64(V_next)) - f64(V);  carry = delta + gkl * carry;  adv = fp32(carry).
// mode 1 (fast) is the same recurrence in fp32 with the coefficients rounded to fp32 first, which
// is also exactly numpy < 2's legacy value-based promotion for K-column values with a scalar
// gamma (np.float64 scalar * fp32 array -> fp32).
#include "common.h"

#pragma clang fp contract(off)

namespace {

constexpr int TG_ROWS = 64;  // rows per tile

struct TrajArgs {
  const float* rewards;
  const float* values;
  const uint8_t* dones;         // kind 0: per row
  const int32_t* steps;         // kind 1: per row (steps_elapsed)
  const int64_t* offsets;       // n_seg + 1
  const float* next_values;     // (n_seg, K) or null (zeros)
  const uint8_t* seg_done;      // kind 1: per trajectory, or null (none done)
  const double* gk;             // kind 1: (max_steps + 1, K) gamma ** s
  const double* gkl;            // kind 1: (max_steps + 1, K) (gamma ** s) * lambda
  float* adv;
  float* ret;
  int64_t n_seg;
  int32_t K;
  int32_t gamma_is_vector;
  int32_t max_steps;
  double gamma[RAI_MAX_K];
  double gl[RAI_MAX_K];
  float gamma32[RAI_MAX_K];
  float gl32[RAI_MAX_K];
};

template <typename Acc, int KIND>
__global__ __launch_bounds__(64) void gae_traj_kernel(const TrajArgs a) {
  __shared__ Acc delta_s[TG_ROWS * RAI_MAX_K];
  __shared__ Acc coef_s[TG_ROWS * RAI_MAX_K];
  const int64_t s = blockIdx.x;
  const int lane = threadIdx.x;
  const int K = a.K;
  const int64_t row0 = a.offsets[s];
  const int64_t L = a.offsets[s + 1] - row0;
  if (L <= 0) return;
  const bool gvec = a.gamma_is_vector != 0;
  const bool seg_done = KIND == 1 && a.seg_done && a.seg_done[s];
  const float* __restrict__ rw = a.rewards + row0 * K;
  const float* __restrict__ vl = a.values + row0 * K;
  float* __restrict__ adv = a.adv + row0 * K;
  float* __restrict__ ret = a.ret ? a.ret + row0 * K : nullptr;
  Acc carry = (Acc)0;  // lanes k < K own column k's carry
  const int ntiles = (int)((L + TG_ROWS - 1) / TG_ROWS);
  for (int tile = 0; tile < ntiles; ++tile) {
    const int64_t hi = L - (int64_t)tile * TG_ROWS;  // rows [lo, hi)
    const int64_t lo = hi - TG_ROWS < 0 ? 0 : hi - TG_ROWS;
    const int nrow = (int)(hi - lo);
    const int nel = nrow * K;
    for (int e = lane; e < nel; e += 64) {
      const int lr = e / K, k = e - lr * K;
      const int64_t t = lo + lr;
      const float r = rw[t * K + k];
      const float v = vl[t * K + k];
      float vn;
      if (t == L - 1) {
        vn = (a.next_values && !seg_done) ? a.next_values[s * K + k] : 0.f;
      } else {
        vn = vl[(t + 1) * K + k];
      }
      Acc d, cf;
      if (KIND == 0) {
        const uint8_t dn = a.dones[row0 + t];
        if (sizeof(Acc) == 8) {
          const double nn = 1.0 - (double)(dn != 0);
          const double t1 = gvec ? a.gamma[k] * (double)vn : (double)(a.gamma32[k] * vn);
          d = (Acc)(((double)r + t1 * nn) - (double)v);
          cf = dn ? (Acc)0 : (Acc)a.gl[k];
        } else {
          const float nn = dn ? 0.f : 1.f;
          d = (Acc)((r + (a.gamma32[k] * vn) * nn) - v);
          cf = dn ? (Acc)0 : (Acc)a.gl32[k];
        }
      } else {
        const int st0 = a.steps[row0 + t];  // host-validated; clamped so a bad row cannot read OOB
        const int st = st0 < 0 ? 0 : (st0 > a.max_steps ? a.max_steps : st0);
        const double g = a.gk[(int64_t)st * K + k];
        const double gl = a.gkl[(int64_t)st * K + k];
        if (sizeof(Acc) == 8) {
          d = (Acc)(((double)r + g * (double)vn) - (double)v);
          cf = (Acc)gl;
        } else {
          d = (Acc)((r + (float)g * vn) - v);
          cf = (Acc)(float)gl;
        }
      }
      delta_s[e] = d;
      coef_s[e] = cf;
    }
    __syncthreads();
    if (lane < K) {
      for (int lr = nrow - 1; lr >= 0; --lr) {
        const int e = lr * K + lane;
        carry = delta_s[e] + coef_s[e] * carry;
        delta_s[e] = carry;
      }
    }
    __syncthreads();
    for (int e = lane; e < nel; e += 64) {
      const int64_t idx = lo * K + e;
      const float av = (float)delta_s[e];
      adv[idx] = av;
      if (ret) ret[idx] = av + vl[idx];
    }
    __syncthreads();
  }
}

int launch(const TrajArgs& a, int kind, int mode, void* stream) {
  const dim3 grid((unsigned)a.n_seg), block(64);
  hipStream_t st = rai_stream(stream);
  if (kind == 0) {
    if (mode == RAI_GAE_EXACT) hipLaunchKernelGGL((gae_traj_kernel<double, 0>), grid, block, 0, st, a);
    else hipLaunchKernelGGL((gae_traj_kernel<float, 0>), grid, block, 0, st, a);
  } else {
    if (mode == RAI_GAE_EXACT) hipLaunchKernelGGL((gae_traj_kernel<double, 1>), grid, block, 0, st, a);
    else hipLaunchKernelGGL((gae_traj_kernel<float, 1>), grid, block, 0, st, a);
  }
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}

int common_args(TrajArgs& a, const float* rewards, const float* values, const int64_t* offsets,
                int64_t n_seg, int32_t K, const float* next_values, int32_t mode, float* adv_out,
                float* returns_out) {
  if (n_seg < 0 || K < 1) return RAI_E_SHAPE;
  if (K > RAI_MAX_K) return RAI_E_TOO_MANY_COLUMNS;
  if (mode != RAI_GAE_EXACT && mode != RAI_GAE_FAST) return RAI_E_MODE;
  if (n_seg > 0 && (!rewards || !values || !offsets || !adv_out)) return RAI_E_NULLPTR;
  if (n_seg > 0x7fffffffLL) return RAI_E_SHAPE;
  a = TrajArgs{};
  a.rewards = rewards;
  a.values = values;
  a.offsets = offsets;
  a.next_values = next_values;
  a.adv = adv_out;
  a.ret = returns_out;
  a.n_seg = n_seg;
  a.K = K;
  return RAI_OK;
}

}  // namespace

extern "C" int rai_gae_trajectories(const float* rewards, const float* values, const uint8_t* dones,
                                    const int64_t* offsets, int64_t n_traj, int32_t K,
                                    const float* next_values, const double* gamma,
                                    const double* gae_lambda, int32_t gamma_is_vector, int32_t mode,
                                    float* adv_out, float* returns_out, void* stream) {
  TrajArgs a;
  int rc = common_args(a, rewards, values, offsets, n_traj, K, next_values, mode, adv_out, returns_out);
  if (rc != RAI_OK) return rc;
  if (n_traj == 0) return RAI_OK;
  if (!dones || !gamma || !gae_lambda) return RAI_E_NULLPTR;
  a.dones = dones;
  a.gamma_is_vector = gamma_is_vector;
  for (int k = 0; k < RAI_MAX_K; ++k) {
    const int kk = gamma_is_vector ? (k < K ? k : 0) : 0;
    a.gamma[k] = gamma[kk];
    a.gl[k] = gamma[kk] * gae_lambda[kk];  // Python/numpy f64 product
    a.gamma32[k] = (float)gamma[kk];
    a.gl32[k] = (float)a.gl[k];
  }
  return launch(a, 0, mode, stream);
}

extern "C" int rai_gae_skips(const float* rewards, const float* values, const int32_t* steps_elapsed,
                             const int64_t* offsets, int64_t n_traj, int32_t K, const float* next_values,
                             const uint8_t* traj_done, const double* gk, const double* gkl,
                             int32_t max_steps, int32_t mode, float* adv_out, float* returns_out,
                             void* stream) {
  TrajArgs a;
  int rc = common_args(a, rewards, values, offsets, n_traj, K, next_values, mode, adv_out, returns_out);
  if (rc != RAI_OK) return rc;
  if (n_traj == 0) return RAI_OK;
  if (!steps_elapsed || !gk || !gkl) return RAI_E_NULLPTR;
  if (max_steps < 0) return RAI_E_SHAPE;
  a.steps = steps_elapsed;
  a.seg_done = traj_done;
  a.gk = gk;
  a.gkl = gkl;
  a.max_steps = max_steps;
  return launch(a, 1, mode, stream);
}
