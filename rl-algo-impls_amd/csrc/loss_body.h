// PPO / A2C loss body (rl_algo_impls/ppo/ppo.py:307-396; rl_algo_impls/a2c/a2c.py:132-158),
// shared by the standalone loss kernel (loss.hip, rai_ppo_loss) and the fused wide-MLP head + loss
// kernel (mlp_wide.hip, rai_mlp_wide_forward_loss).  Included inside each file's anonymous
// namespace.  The reference's rounding sequence is kept by compiling this code without FP
// contraction wherever it is included (a `#pragma clang fp contract(off)` opens every function
// with floating-point arithmetic; loss.hip additionally builds with -ffp-contract=off).
#pragma once

constexpr int LOSS_THREADS = 1024;

struct LossArgs {
  const float* new_logp;
  const float* entropy;
  const float* new_values;
  const float* old_logp;
  const float* old_values;
  const float* adv;
  const float* ret;
  const rai_ppo_hparams* hp;
  rai_train_state* state;
  float* d_logp;
  float* d_entropy;
  float* d_values;
  float* stats;
  int64_t B;
  int64_t n_entropy;
  int32_t K;
  int32_t max_stats;
};

struct AdvNorm {
  float mean[RAI_MAX_K];
  float inv_den[RAI_MAX_K];  // unused: keep (x - mean) / den as torch does
  float den[RAI_MAX_K];
  float smean, sden;  // scalar (normalize-after-scaling) moments
};

__device__ __forceinline__ float vf_elem_loss(int fn, float x) {
#pragma clang fp contract(off)
  if (fn == 0) return x * x;
  const float z = fabsf(x);
  return z < 1.f ? 0.5f * z * z : (z - 0.5f);
}
__device__ __forceinline__ float vf_elem_grad(int fn, float x) {  // d loss / d x
#pragma clang fp contract(off)
  if (fn == 0) return 2.f * x;
  return x <= -1.f ? -1.f : (x >= 1.f ? 1.f : x);
}

// Block sum of NV doubles: wave trees, then NV threads each add the nw wave partials in wave
// order (fixed order -> deterministic), result broadcast through LDS.  sc holds NV*(nw+1).
template <int NV>
__device__ __forceinline__ void block_sum_small(double (&v)[NV], double* sc) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = wave_sum(v[i]);
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < NV; ++i) sc[i * nw + w] = v[i];
  }
  __syncthreads();
  if (threadIdx.x < NV) {
    double s = 0.0;
    for (int j = 0; j < nw; ++j) s += sc[threadIdx.x * nw + j];
    sc[NV * nw + threadIdx.x] = s;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = sc[NV * nw + i];
  __syncthreads();
}

// KM: compile-time bound on the value columns (1 or RAI_MAX_K) so every per-column array is
// register-resident (indices unrolled; a runtime-indexed array would live in scratch).
template <int KM, class AdvF>
__device__ __forceinline__ float row_adv(const LossArgs& a, const rai_ppo_hparams& hp, const AdvNorm& nm,
                                         int64_t b, AdvF adv) {
#pragma clang fp contract(off)
  const int K = a.K;
  if (hp.normalize_after_scaling) {
    float x;
    if (hp.has_multi_reward_weights) {
      x = 0.f;
#pragma unroll
      for (int k = 0; k < KM; ++k)
        if (k < K) x += adv(b, k) * hp.multi_reward_weights[k];
    } else {
      x = adv(b, 0);
    }
    return (x - nm.smean) / nm.sden;
  }
  if (KM == 1 || (K == 1 && !hp.has_multi_reward_weights)) {
    const float x = adv(b, 0);
    float y = x;
    if (hp.normalize_advantage) y = (x - nm.mean[0]) / nm.den[0];
    else if (hp.standardize_advantage) y = x / nm.den[0];
    return hp.has_multi_reward_weights ? y * hp.multi_reward_weights[0] : y;
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    if (k < K) {
      float x = adv(b, k);
      if (hp.normalize_advantage) x = (x - nm.mean[k]) / nm.den[k];
      else if (hp.standardize_advantage) x = x / nm.den[k];
      s += x * (hp.has_multi_reward_weights ? hp.multi_reward_weights[k] : 1.f);
    }
  }
  return s;
}

// The loss body over one workgroup (blockDim.x threads) owning the minibatch: shared by
// pg_loss_kernel (loss.hip) and the wide-MLP head+loss kernel (mlp_wide.hip).
template <int KM>
__device__ __forceinline__ void pg_loss_body(const LossArgs& a) {
#pragma clang fp contract(off)
  constexpr int NR = 4 + 2 * KM;  // pi_sum, kl_sum, clip_cnt, ent_sum, vloss[KM], vclip[KM]
  __shared__ double red[NR * (LOSS_THREADS / 64 + 1)];
  __shared__ AdvNorm nm_s;
  // by value: one scalar load batch at entry (through a reference every field read after a barrier is a
  // fresh global load on the critical path); likewise the train-state words, which only thread 0 writes,
  // at the very end
  const rai_ppo_hparams hp = *a.hp;
  const int st_stat_index = a.state->stat_index, st_pi_coef_zero = a.state->pi_coef_zero;
  const int K = a.K;
  const int64_t B = a.B;
  const int tid = threadIdx.x, NT = blockDim.x;
  const bool ppo = hp.loss_kind == 0;

  // one row per thread (B <= blockDim.x: C3's 256-row minibatch): the row's inputs are loaded once, all
  // together, and every pass below reads them from registers -- one memory round trip instead of one per
  // pass.  Otherwise the accessors read memory, as before.  Same values, same arithmetic.
  const bool one_row = B <= NT;
  float c_adv[KM], c_v[KM], c_R[KM], c_vo[KM];
  float c_nl = 0.f, c_ol = 0.f, c_ent = 0.f;
#pragma unroll
  for (int k = 0; k < KM; ++k) c_adv[k] = c_v[k] = c_R[k] = c_vo[k] = 0.f;
  if (one_row && tid < B) {
#pragma unroll
    for (int k = 0; k < KM; ++k)
      if (k < K) {
        c_adv[k] = a.adv[tid * K + k];
        c_v[k] = a.new_values[tid * K + k];
        c_R[k] = a.ret[tid * K + k];
        c_vo[k] = a.old_values[tid * K + k];
      }
    c_nl = a.new_logp[tid];
    c_ol = a.old_logp[tid];
  }
  const bool one_ent = a.n_entropy <= NT;
  if (one_ent && tid < a.n_entropy) c_ent = a.entropy[tid];
  auto ADV = [&](int64_t b, int k) -> float { return one_row ? c_adv[k] : a.adv[b * K + k]; };
  auto NV = [&](int64_t b, int k) -> float { return one_row ? c_v[k] : a.new_values[b * K + k]; };
  auto RET = [&](int64_t b, int k) -> float { return one_row ? c_R[k] : a.ret[b * K + k]; };
  auto OV = [&](int64_t b, int k) -> float { return one_row ? c_vo[k] : a.old_values[b * K + k]; };
  auto NL = [&](int64_t b) -> float { return one_row ? c_nl : a.new_logp[b]; };
  auto OL = [&](int64_t b) -> float { return one_row ? c_ol : a.old_logp[b]; };

  // ---- pass 0: advantage moments (two-pass, fp64 accumulation; ppo.py:307-318) ---------
  const bool need_cols = !hp.normalize_after_scaling && (hp.normalize_advantage || hp.standardize_advantage);
  if (hp.ext_moments && (hp.normalize_after_scaling || need_cols)) {
    // data parallel: the global minibatch's moments, reduced across ranks by the host (ppo.py:307-318
    // over the union of the ranks' minibatch slices).  Row si holds K (mean, den) pairs per column,
    // or one pair of the weighted advantage under normalize_advantages_after_scaling.
    if (tid == 0) {
      const int si = st_stat_index;
      if (hp.normalize_after_scaling) {
        nm_s.smean = hp.ext_moments[2 * si];
        nm_s.sden = hp.ext_moments[2 * si + 1];
      } else {
#pragma unroll
        for (int k = 0; k < KM; ++k)
          if (k < K) {
            nm_s.mean[k] = hp.ext_moments[2 * (si * K + k)];
            nm_s.den[k] = hp.ext_moments[2 * (si * K + k) + 1];
          }
      }
    }
  } else if (hp.normalize_after_scaling) {
    double acc[1] = {0.0};
    for (int64_t b = tid; b < B; b += NT) {
      float x;
      if (hp.has_multi_reward_weights) {
        x = 0.f;
#pragma unroll
        for (int k = 0; k < KM; ++k)
          if (k < K) x += ADV(b, k) * hp.multi_reward_weights[k];
      } else {
        x = ADV(b, 0);
      }
      acc[0] += (double)x;
    }
    block_sum_small<1>(acc, red);
    const float mean = (float)(acc[0] / (double)B);
    acc[0] = 0.0;
    for (int64_t b = tid; b < B; b += NT) {
      float x;
      if (hp.has_multi_reward_weights) {
        x = 0.f;
#pragma unroll
        for (int k = 0; k < KM; ++k)
          if (k < K) x += ADV(b, k) * hp.multi_reward_weights[k];
      } else {
        x = ADV(b, 0);
      }
      const double d = (double)x - (double)mean;
      acc[0] += d * d;
    }
    block_sum_small<1>(acc, red);
    if (tid == 0) {
      nm_s.smean = mean;
      nm_s.sden = (float)sqrt(acc[0] / (double)(B - 1)) + 1e-8f;
    }
  } else if (need_cols) {
    double acc[KM];
#pragma unroll
    for (int k = 0; k < KM; ++k) acc[k] = 0.0;
    for (int64_t b = tid; b < B; b += NT) {
#pragma unroll
      for (int k = 0; k < KM; ++k)
        if (k < K) acc[k] += (double)ADV(b, k);
    }
    block_sum_small<KM>(acc, red);
    float mean[KM];
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      mean[k] = (float)(acc[k] / (double)B);
      acc[k] = 0.0;
    }
    for (int64_t b = tid; b < B; b += NT) {
#pragma unroll
      for (int k = 0; k < KM; ++k) {
        if (k < K) {
          const double d = (double)ADV(b, k) - (double)mean[k];
          acc[k] += d * d;
        }
      }
    }
    block_sum_small<KM>(acc, red);
    if (tid == 0) {
#pragma unroll
      for (int k = 0; k < KM; ++k) {
        nm_s.mean[k] = mean[k];
        nm_s.den[k] = (float)sqrt(acc[k] / (double)(B - 1)) + 1e-8f;
      }
    }
  }
  __syncthreads();
  const AdvNorm nm = nm_s;

  // ---- pass 1: forward statistics (ppo.py:326-361, 379-396) --------------------------
  const float lo = 1.f - hp.clip_range, hi = 1.f + hp.clip_range;
  const float vclip = hp.clip_range_vf;
  const bool vclip_on = ppo && hp.has_clip_range_vf;
  const int vfn = hp.vf_loss_fn;
  double acc[NR];
#pragma unroll
  for (int i = 0; i < NR; ++i) acc[i] = 0.0;
  for (int64_t b = tid; b < B; b += NT) {
    const float A = row_adv<KM>(a, hp, nm, b, ADV);
    if (ppo) {
      const float logratio = NL(b) - OL(b);
      const float ratio = expf(logratio);
      const float cr = fminf(fmaxf(ratio, lo), hi);
      acc[0] += (double)fminf(ratio * A, cr * A);
      acc[1] += (double)((ratio - 1.f) - logratio);
      acc[2] += (fabsf(ratio - 1.f) > hp.clip_range) ? 1.0 : 0.0;
    } else {
      acc[0] += (double)(A * NL(b));
    }
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      if (k < K) {
        const float v = NV(b, k), R = RET(b, k);
        float l = vf_elem_loss(vfn, v - R);
        if (vclip_on) {
          const float vo = OV(b, k);
          const float vc = vo + fminf(fmaxf(v - vo, -vclip), vclip);
          l = fmaxf(l, vf_elem_loss(vfn, vc - R));
          acc[4 + KM + k] += (fabsf(v - vo) > vclip) ? 1.0 : 0.0;
        }
        acc[4 + k] += (double)l;
      }
    }
  }
  if (one_ent) {
    if (tid < a.n_entropy) acc[3] += (double)c_ent;
  } else {
    for (int64_t i = tid; i < a.n_entropy; i += NT) acc[3] += (double)a.entropy[i];
  }
  block_sum_small<NR>(acc, red);

  const float invB = 1.f / (float)B;
  const float approx_kl = (float)(acc[1] / (double)B);
  int latched = st_pi_coef_zero;
  if (ppo && hp.has_kl_cutoff && approx_kl > hp.kl_cutoff) latched = 1;
  const float pi_coef = (ppo && latched) ? 0.f : 1.f;
  const float halve = hp.ppo2_vf_coef_halving ? 0.5f : 1.f;
  const float gs = hp.grad_scale;

  // ---- pass 2: gradients to the network outputs (torch.min/max tie split, clamp closed) --
  const float g_pi = (-pi_coef * invB) * gs;
  float gl[KM];
#pragma unroll
  for (int k = 0; k < KM; ++k) gl[k] = ((hp.vf_coef[k] * halve) * invB) * gs;  // d loss / d l_bk
  for (int64_t b = tid; b < B; b += NT) {
    const float A = row_adv<KM>(a, hp, nm, b, ADV);
    if (ppo) {
      const float logratio = NL(b) - OL(b);
      const float ratio = expf(logratio);
      const float cr = fminf(fmaxf(ratio, lo), hi);
      const float s1 = ratio * A, s2 = cr * A;
      float g1, g2;
      if (s1 < s2) { g1 = g_pi; g2 = 0.f; }
      else if (s1 > s2) { g1 = 0.f; g2 = g_pi; }
      else { g1 = g_pi * 0.5f; g2 = g_pi * 0.5f; }
      const float in_clip = (ratio >= lo && ratio <= hi) ? 1.f : 0.f;
      const float d_ratio = g1 * A + (g2 * A) * in_clip;
      a.d_logp[b] = d_ratio * ratio;
    } else {
      a.d_logp[b] = ((-invB) * gs) * A;
    }
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      if (k < K) {
        const float v = NV(b, k), R = RET(b, k);
        float dv;
        if (vclip_on) {
          const float vo = OV(b, k);
          const float dvo = v - vo;
          const float vc = vo + fminf(fmaxf(dvo, -vclip), vclip);
          const float l1 = vf_elem_loss(vfn, v - R);
          const float l2 = vf_elem_loss(vfn, vc - R);
          float w1, w2;
          if (l1 > l2) { w1 = gl[k]; w2 = 0.f; }
          else if (l1 < l2) { w1 = 0.f; w2 = gl[k]; }
          else { w1 = gl[k] * 0.5f; w2 = gl[k] * 0.5f; }
          const float in_vclip = (dvo >= -vclip && dvo <= vclip) ? 1.f : 0.f;
          dv = w1 * vf_elem_grad(vfn, v - R) + (w2 * vf_elem_grad(vfn, vc - R)) * in_vclip;
        } else {
          dv = gl[k] * vf_elem_grad(vfn, v - R);
        }
        a.d_values[b * K + k] = dv;
      }
    }
  }
  const float g_ent = (-hp.ent_coef / (float)a.n_entropy) * gs;
  for (int64_t i = tid; i < a.n_entropy; i += NT) a.d_entropy[i] = g_ent;

  // ---- stats row -------------------------------------------------------------------------
  if (tid == 0) {
    const float pi_loss = (float)(-acc[0] / (double)B);
    const float ent_loss = (float)(-acc[3] / (double)a.n_entropy);
    float vsum = 0.f;
    const int idx = st_stat_index;
    float* row = (a.stats && idx < a.max_stats) ? a.stats + (int64_t)idx * RAI_STAT_STRIDE : nullptr;
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      if (k < K) {
        const float vl = (float)(acc[4 + k] / (double)B) * halve;
        vsum += hp.vf_coef[k] * vl;
        if (row) {
          row[5 + k] = vl;
          row[5 + RAI_MAX_K + k] = vclip_on ? (float)(acc[4 + KM + k] / (double)B) : 0.f;
        }
      }
    }
    const float loss = (pi_coef * pi_loss + hp.ent_coef * ent_loss + vsum) * gs;
    if (row) {
      row[0] = loss;
      row[1] = pi_loss;
      row[2] = ent_loss;
      row[3] = ppo ? approx_kl : 0.f;
      row[4] = ppo ? (float)(acc[2] / (double)B) : 0.f;
    }
    a.state->stat_index = idx + 1;
    a.state->pi_coef_zero = latched;
  }
}

