// Library-internal entry points shared between translation units (not part of the C ABI:
// C++ names in their own namespace, so include/rai_amd.h stays the whole exported surface).
#pragma once
#include "common.h"

namespace rai_internal {

// clip_grad_norm_ + Adam / RMSprop (optim.hip's clip_optim_kernel) over a flat buffer whose
// squared-norm partials (nparts fp64 values, fixed order) were already written by the caller's
// reduction kernel, which also advanced state->opt_step.
int optim_apply_partials(float* params, float* grads, float* state1, float* state2, int64_t P,
                         const rai_optim_hparams* hp, rai_train_state* state, const double* partial, int nparts,
                         float* norms, int32_t max_norms, hipStream_t stream);

// Large-minibatch PPO steps of the CartPole-class MLP actor-critic (mlp_large.hip): minibatches of
// more than 256 rows (SURVEY 8(d) batch policy (b), batch = T*N/4).  Epoch mode (grad_out == nullptr):
// every minibatch of rows [0, n_rows) -> forward / loss / backward partials over all CUs, a fixed-order
// reduction, clip_grad_norm_ + Adam.  Grads mode: minibatch mb_begin only (mb_count must be 1), raw
// gradients into grad_out, loss means over rows * world (the caller all-reduces, then steps).
// Data parallel over the in-kernel cross-GPU exchange (xdp != nullptr, epoch mode): each step's reduce
// launch pushes this rank's 64-parameter blocks into every rank's IPC-mapped region, waits for the
// other ranks' blocks and sums them in rank order (identical bits everywhere) before clip + Adam.
struct LargeXdp {
  void* const* peers;  // device array of the world's region pointers (own region at [rank])
  int32_t rank;
  int32_t world;
  int64_t step_base;   // optimizer steps already run through the regions (flags hold step ids)
};
int mlp_large(float* params, float* exp_avg, float* exp_avg_sq, const float* obs, const int64_t* actions,
              const float* old_logp, const float* old_values, const float* adv, const float* ret, int64_t n_rows,
              int32_t batch, int32_t in_dim, int32_t n_act, int32_t act_fn, int32_t mb_begin, int32_t mb_count,
              const float* moments, int32_t world, const rai_ppo_hparams* hp, const rai_optim_hparams* ohp,
              rai_train_state* state, float* stats, int32_t max_stats, float* norms, int32_t max_norms,
              float* grad_out, void* workspace, int64_t workspace_bytes, hipStream_t stream,
              const LargeXdp* xdp = nullptr);
// bytes of the exchange region the large-minibatch layout needs at `world` ranks
int64_t mlp_large_xdp_bytes(int32_t world);
int64_t mlp_large_workspace_bytes(int64_t n_rows, int32_t batch);
// shapes the large-minibatch kernels cover (the others fall back in the caller)
bool mlp_large_supported(int32_t in_dim, int32_t n_act, int32_t hidden);

}  // namespace rai_internal
