/*
 * ORACLE — test infrastructure only (never linked into the product path).
 *
 * Scalar C restatement of rl_algo_impls/shared/gae.py:97-124 (compute_advantages)
 * with the exact numpy dtype-promotion sequence of the reference (numpy 1.24 /
 * NEP 50 agree on it), used by tests/ to pin the HIP kernel bit for bit:
 *   gae.py:115,118  next_nonterminal = 1.0 - bool           -> f64 (0.0 / 1.0)
 *   gae.py:121      gamma * next_value                       -> f32 if gamma is a Python
 *                                                               float, f64 if an ndarray
 *                   (... * next_nonterminal)                 -> f64
 *                   rewards[t] + (...) - values[t]           -> f64
 *   gae.py:122      gamma*gae_lambda (f64) * nn * last       -> f64 carry
 *   gae.py:123      advantages[t] = last                     -> cast to f32
 *   vec_rollout.py:88 returns = advantages + values          -> f32
 * Compiled with -ffp-contract=off so no multiply-add is fused.
 */
#include <stdint.h>

void gae_ref_f32(const float* rewards, const float* values, const uint8_t* episode_starts,
                 const uint8_t* next_episode_starts, const float* next_values, int64_t T,
                 int64_t N, int64_t K, const double* gamma, const double* gae_lambda,
                 int gamma_is_vector, float* adv_out, float* returns_out) {
  const int64_t C = N * K;
  for (int64_t c = 0; c < C; ++c) {
    const int64_t n = c / K, k = c % K;
    const double gl = gamma[k] * gae_lambda[k];
    const float g32 = (float)gamma[k];
    double last = 0.0;
    for (int64_t t = T - 1; t >= 0; --t) {
      float vn;
      uint8_t es;
      if (t == T - 1) {
        vn = next_values[c];
        es = next_episode_starts[n];
      } else {
        vn = values[(t + 1) * C + c];
        es = episode_starts[(t + 1) * N + n];
      }
      const double nn = 1.0 - (double)(es != 0);
      double t1;
      if (gamma_is_vector) {
        t1 = gamma[k] * (double)vn;
      } else {
        const float t1f = g32 * vn;
        t1 = (double)t1f;
      }
      const double delta = ((double)rewards[t * C + c] + t1 * nn) - (double)values[t * C + c];
      last = delta + (gl * nn) * last;
      const float a = (float)last;
      adv_out[t * C + c] = a;
      if (returns_out) returns_out[t * C + c] = a + values[t * C + c];
    }
  }
}
