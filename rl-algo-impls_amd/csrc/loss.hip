// Fused policy-gradient loss forward + backward for gfx950.
//
// Restates, per minibatch:
//   rl_algo_impls/ppo/ppo.py:307-318  advantage normalisation / standardisation /
//                                     multi_reward_weights (before or after scaling)
//   rl_algo_impls/ppo/ppo.py:326-361  ratio, clipped surrogate, (clipped) value loss,
//                                     vf_weights, ppo2 halving, entropy loss,
//                                     approx_kl, kl_cutoff latch, total loss
//   rl_algo_impls/ppo/ppo.py:373-374  gradient_accumulation scaling
//   rl_algo_impls/ppo/ppo.py:379-396  clipped_frac / val_clipped_frac
//   rl_algo_impls/a2c/a2c.py:132-158  A2C loss (loss_kind = 1)
// and emits dLoss/d(new_logp), dLoss/d(entropy), dLoss/d(new_values) with the
// autograd tie rules of torch.min/torch.max (ties split 1/2-1/2) and clamp
// (gradient passes on the closed interval), so PyTorch-ROCm backpropagates the
// network from these three tensors.  Stats are written as one row to a
// device-resident table (no host sync per minibatch; the reference does ~6
// `.item()` syncs here).
//
// One workgroup owns the whole minibatch (256 threads up to B = 2048, else 1024):
// the advantage moments, approx_kl (needed before the kl_cutoff decision) and
// every stat are block reductions in a fixed order -> the result is deterministic
// and needs no inter-workgroup protocol.  Per-column accumulators are sized by a
// compile-time column bound (K = 1 or RAI_MAX_K) so they stay in registers.
#include "common.h"

namespace {

#include "loss_body.h"

template <int KM>
__global__ __launch_bounds__(LOSS_THREADS) void pg_loss_kernel(const LossArgs a) {
  pg_loss_body<KM>(a);
}

}  // namespace

extern "C" int64_t rai_ppo_loss_workspace_bytes(int64_t /*B*/, int32_t /*K*/) { return 0; }

extern "C" int rai_ppo_loss(const float* new_logp, const float* entropy, int64_t n_entropy,
                            const float* new_values, const float* old_logp,
                            const float* old_values, const float* advantages,
                            const float* returns, int64_t B, int32_t K, const rai_ppo_hparams* hp,
                            rai_train_state* state, float* d_logp, float* d_entropy,
                            float* d_values, float* stats, int32_t max_stats, void* /*workspace*/,
                            int64_t /*workspace_bytes*/, void* stream) {
  if (B < 1 || K < 1 || n_entropy < 1) return RAI_E_SHAPE;
  if (K > RAI_MAX_K) return RAI_E_TOO_MANY_COLUMNS;
  if (!new_logp || !entropy || !new_values || !advantages || !returns || !hp || !state ||
      !d_logp || !d_entropy || !d_values)
    return RAI_E_NULLPTR;
  LossArgs a;
  a.new_logp = new_logp;
  a.entropy = entropy;
  a.new_values = new_values;
  a.old_logp = old_logp ? old_logp : new_logp;
  a.old_values = old_values ? old_values : new_values;
  a.adv = advantages;
  a.ret = returns;
  a.hp = hp;
  a.state = state;
  a.d_logp = d_logp;
  a.d_entropy = d_entropy;
  a.d_values = d_values;
  a.stats = stats;
  a.B = B;
  a.n_entropy = n_entropy;
  a.K = K;
  a.max_stats = max_stats;
  // one workgroup owns the minibatch; 256 threads while that is <= 8 rows per thread
  const unsigned nt = B <= 2048 ? 256u : (unsigned)LOSS_THREADS;
  if (K == 1) hipLaunchKernelGGL(pg_loss_kernel<1>, dim3(1), dim3(nt), 0, rai_stream(stream), a);
  else hipLaunchKernelGGL(pg_loss_kernel<RAI_MAX_K>, dim3(1), dim3(nt), 0, rai_stream(stream), a);
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}
