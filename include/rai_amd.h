/*
 * rai_amd.h — C ABI of the MI355X (gfx950) PPO/A2C rollout+update hot path.
 *
 * Drop-in boundary for toldo4/rl-algo-impls.  The reference is pure Python; every
 * entry point below replaces one eager NumPy/PyTorch region of its trainer and is
 * bound from Python through ctypes.  The signature style is
 * deliberately FFI-plain: device pointers, sizes, POD structs, and an opaque
 * `stream` (a hipStream_t; NULL = the null stream).  No allocation happens inside
 * any call: scratch memory is caller-owned (`workspace`), so every call can be
 * captured into a hipGraph.
 *
 * Return value: 0 on success; a negative RAI_E_* code for argument errors (checked
 * on the host before anything is launched); a positive hipError_t if a launch
 * failed.  rai_strerror() maps either to a message.
 *
 * All entry points are stream-ordered on `stream` and deterministic: fixed
 * reduction orders, no floating-point atomics.
 */
#ifndef RAI_AMD_H_
#define RAI_AMD_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RAI_ABI_VERSION 1
#define RAI_MAX_K 8 /* max value columns (multi-critic), reference value_shape (K,) */

enum {
  RAI_OK = 0,
  RAI_E_NULLPTR = -1,
  RAI_E_SHAPE = -2,
  RAI_E_MODE = -3,
  RAI_E_TOO_MANY_COLUMNS = -4,
  RAI_E_WORKSPACE = -5,
  RAI_E_UNSUPPORTED = -6,
  RAI_E_DP_BASE = -1000, /* RCCL failure r is reported as RAI_E_DP_BASE - r */
};

int rai_abi_version(void);
const char* rai_strerror(int code);

/* --------------------------------------------------------------------------
 * GAE / returns
 * Replaces rl_algo_impls/shared/gae.py:97-124 (compute_advantages) and the
 * fused `returns = advantages + values` of rl_algo_impls/rollout/vec_rollout.py:88.
 *
 * Layout: rewards/values/adv/returns are (T, N, K) row-major fp32; episode_starts
 * (T, N) and next_episode_starts (N) are uint8 booleans; next_values (N, K).
 * gamma/gae_lambda: host arrays of length K (or 1 when the reference argument is a
 * Python float).  gamma_is_vector selects the reference's numpy promotion path:
 *   0: gamma is a Python float -> gamma*V_next computed in fp32 (gae.py:121)
 *   1: gamma is an ndarray     -> gamma*V_next computed in fp64
 * mode: 0 = exact (fp64 carry in the reference's operation order; bit-exact),
 *       1 = fast  (fp32 carry; within 1e-5 relative of exact).
 * returns_out may be NULL.
 * ------------------------------------------------------------------------ */
#define RAI_GAE_EXACT 0
#define RAI_GAE_FAST 1
int rai_gae(const float* rewards, const float* values, const uint8_t* episode_starts,
            const uint8_t* next_episode_starts, const float* next_values, int64_t T, int64_t N,
            int32_t K, const double* gamma, const double* gae_lambda, int32_t gamma_is_vector,
            int32_t mode, float* adv_out, float* returns_out, void* stream);

/* --------------------------------------------------------------------------
 * Per-trajectory GAE over a ragged batch (one launch for many trajectories).
 * Rows of all trajectories are concatenated: rewards/values/adv/returns are
 * (sum L, K) row-major fp32; offsets (n_traj + 1, int64, device) gives each
 * trajectory's first row.  next_values (n_traj, K) may be NULL (zeros).
 *
 * rai_gae_trajectories replaces rl_algo_impls/rollout/trajectory.py:56-92
 * (TrajectoryBuilder.trajectory = compute_advantages over one trajectory with
 * episode_starts = [True, dones[:-1]], next_episode_starts = dones[-1]); dones is
 * per row (uint8).  gamma/gae_lambda/gamma_is_vector/mode as in rai_gae.
 *
 * rai_gae_skips replaces rl_algo_impls/rollout/discrete_skips_trajectory_builder.py:
 * 64-109 (semi-MDP GAE: gamma ** steps_elapsed[t] in the bootstrap and the carry).
 * steps_elapsed is per row (int32, 0..max_steps); traj_done (n_traj, uint8, may be
 * NULL) zeroes the last bootstrap; gk / gkl are device tables (max_steps + 1, K)
 * of gamma ** s and (gamma ** s) * lambda, computed by the caller exactly as numpy
 * evaluates them (the reference's own pow).  mode 0 = the numpy >= 2 fp64 sequence
 * (bit-exact), 1 = fp32 with fp32-rounded coefficients (= numpy < 2 promotion for
 * K-column values with a scalar gamma).  returns_out may be NULL.
 * ------------------------------------------------------------------------ */
int rai_gae_trajectories(const float* rewards, const float* values, const uint8_t* dones,
                         const int64_t* offsets, int64_t n_traj, int32_t K, const float* next_values,
                         const double* gamma, const double* gae_lambda, int32_t gamma_is_vector,
                         int32_t mode, float* adv_out, float* returns_out, void* stream);
int rai_gae_skips(const float* rewards, const float* values, const int32_t* steps_elapsed,
                  const int64_t* offsets, int64_t n_traj, int32_t K, const float* next_values,
                  const uint8_t* traj_done, const double* gk, const double* gkl, int32_t max_steps,
                  int32_t mode, float* adv_out, float* returns_out, void* stream);

/* --------------------------------------------------------------------------
 * GridNet masked-categorical head (MicroRTS per-cell sub-actions).
 * Replaces rl_algo_impls/shared/actor/gridnet.py:38-200 (GridnetDistribution.log_prob,
 * .entropy over MaskedCategorical, rl_algo_impls/shared/actor/categorical.py:12-54)
 * and their autograd backward.
 * logits / mask / d_logits: (B, C, A) row-major, A = sum(nvec) <= RAI_GRID_MAX_A,
 * C = cells (map H*W); actions (B, C, G) int64, G = len(nvec) <= RAI_GRID_MAX_G.
 * nvec / sub_ref / sub_val are host arrays of length G: group g's log-prob counts only
 * where actions[..., sub_ref[g]] == sub_val[g] (ValueDependentMask, gridnet.py:21-35;
 * sub_ref[g] = -1 or sub_ref = NULL: always counts).  Entropy is never gated.
 * logp_out / entropy_out (B,) fp32, either may be NULL (actions may be NULL when only
 * the entropy is wanted).  rai_gridnet_backward writes dL/dlogits for upstream
 * d_logp, d_entropy (B,).
 * ------------------------------------------------------------------------ */
#define RAI_GRID_MAX_G 8
#define RAI_GRID_MAX_A 256
int rai_gridnet_logp_entropy(const float* logits, const uint8_t* mask, const int64_t* actions, int64_t B,
                             int32_t C, int32_t G, const int32_t* nvec, const int32_t* sub_ref,
                             const int32_t* sub_val, float* logp_out, float* entropy_out, void* stream);
int rai_gridnet_backward(const float* logits, const uint8_t* mask, const int64_t* actions, int64_t B, int32_t C,
                         int32_t G, const int32_t* nvec, const int32_t* sub_ref, const int32_t* sub_val,
                         const float* d_logp, const float* d_entropy, float* d_logits, void* stream);
/* Rollout sampling of the same head: GridnetDistribution.sample() + log_prob(sample)
 * (rl_algo_impls/shared/actor/gridnet.py:195-205 then :101-160, as called by
 * actor_critic.py:306-318 / sync_step_rollout.py:193-201).  Each (cell, plane) draws from its
 * masked categorical by inverse CDF on Philox4x32-10 keyed (seed; counter (offset,
 * (b*C + c)*G + g)); a plane with no valid action draws uniformly over all its n values
 * (torch's equal finfo.min logits).  actions_out (B, C, G) int64; logp_out (B,) or NULL. */
int rai_gridnet_sample(const float* logits, const uint8_t* mask, int64_t B, int32_t C, int32_t G,
                       const int32_t* nvec, const int32_t* sub_ref, const int32_t* sub_val, uint64_t seed,
                       uint64_t offset, int64_t* actions_out, float* logp_out, void* stream);
/* Batch.num_actions of a GridNet rollout: rl_algo_impls/rollout/rollout.py:158-180
 * (per_position_num_actions, via num_actions :130-155 from VecRollout.__init__,
 * rl_algo_impls/rollout/vec_rollout.py:69-76).  For each of the B = T*N rows:
 *   per_group = 0 (no subaction_mask): out[b] = #cells whose A mask bytes hold any 1
 *                                      (np.sum(np.any(mask, -1), -1));
 *   per_group = 1: out[b] = sum over cells and groups g of any(mask[cell, group g]), group g
 *                  counted only where actions[b, cell, sub_ref[g]] == sub_val[g] (the
 *                  ValueDependentMask gate; sub_ref[g] = -1: always counted).
 * mask (B, C, A) u8/bool; actions (B, C, G) int64 (read only when per_group and a gate exists;
 * may be NULL otherwise).  out (B,) int32 when out_bytes == 4 (the reference's dtype with a
 * subaction mask), int64 when 8 (without).  Exact integer counts. */
int rai_gridnet_num_actions(const uint8_t* mask, const int64_t* actions, int64_t B, int32_t C, int32_t G,
                            const int32_t* nvec, const int32_t* sub_ref, const int32_t* sub_val,
                            int32_t per_group, int32_t out_bytes, void* out, void* stream);

/* --------------------------------------------------------------------------
 * Squeeze-excitation residual epilogue of the squeeze-U-Net backbone (config C5):
 * out = GELU(x + r * s[b, c]) and its backward in one pass each, replacing the
 * broadcast-multiply / add / GELU sequence of SEResidualBlock.forward
 * (rl_algo_impls/shared/policy/actor_critic_network/double_cone.py:43-47,85-86) and
 * its autograd.  x, r, out, dout, dx, dr: NHWC (channels_last) fp32, (B, HW, C) with C
 * fastest; s, ds: (B, C).  GELU is the exact erf form.  C % 4 == 0 and C / 4 must
 * divide 256 (RAI_E_SHAPE otherwise).
 * ------------------------------------------------------------------------ */
int rai_se_residual_fwd(const float* x, const float* r, const float* s, int64_t B, int32_t C, int32_t HW,
                        float* out, void* stream);
int rai_se_residual_bwd(const float* dout, const float* x, const float* r, const float* s, int64_t B, int32_t C,
                        int32_t HW, float* dx, float* dr, float* ds, void* stream);
/* Conv bias + GELU of the squeeze-U-Net's conv -> GELU pairs (squeeze_unet.py:56-70,117-137,
 * double_cone.py:58-70, backbone_actor_critic.py:114-133): out = GELU(x + b[c]) over NHWC rows,
 * and dx = dy * GELU'(x + b) (the bias gradient is dx summed over rows).  C % 4 == 0. */
int rai_bias_gelu_fwd(const float* x, const float* b, int64_t rows, int32_t C, float* out, void* stream);
int rai_bias_gelu_bwd(const float* dy, const float* x, const float* b, int64_t rows, int32_t C, float* dx,
                      void* stream);

/* Conv / Linear bias + ReLU of the NatureCNN encoder (rl_algo_impls/shared/encoder/nature_cnn.py:10-53:
 * Conv2d -> ReLU x3, then Linear -> ReLU) over NHWC (or (B, C) row-major) rows, C % 4 == 0, C / 4
 * dividing 256.  Forward: out = relu(x + b[c]) (x = the bias-free conv / GEMM output).  Backward, one
 * launch: dx = dy * (out > 0) (torch threshold_backward on the saved output) and the bias gradient
 * db[c] = sum_rows dx[row, c], written (accumulate == 0) or added to db (accumulate != 0, e.g. straight
 * into the flat .grad buffer), in one launch (the last workgroup to arrive sums the per-workgroup
 * partials).  The reduction order is fixed (deterministic).  workspace: at least
 * rai_bias_relu_workspace_bytes(C) bytes, 16-B aligned, ZEROED before its first use (its arrival
 * counters are re-armed by every launch); one workspace per concurrently running launch. */
int64_t rai_bias_relu_workspace_bytes(int32_t C);
int rai_bias_relu_fwd(const float* x, const float* b, int64_t rows, int32_t C, float* out, void* stream);
int rai_bias_relu_bwd(const float* dy, const float* y, int64_t rows, int32_t C, float* dx, float* db,
                      int32_t accumulate, void* workspace, int64_t workspace_bytes, void* stream);
/* The same pair for the layer whose output is flattened (NatureCNN conv3 -> nn.Flatten -> Linear,
 * nature_cnn.py:41-53): x is the bias-free conv output in NHWC (B, HW, C); the forward writes
 * out = relu(x + b) in the flattened NCHW order (B, C * HW) that nn.Flatten gives, the backward takes
 * dy and y in that order and writes dx in NHWC (B, HW, C) for the convolution's backward, with db as
 * rai_bias_relu_bwd (same workspace).  The two layout copies around the flatten disappear into the
 * passes.  (C + 1) * HW <= 8192, C % 4 == 0, C / 4 dividing 256; dx 16-B aligned. */
int rai_bias_relu_fwd_nchw(const float* x, const float* b, int64_t B, int32_t HW, int32_t C, float* out,
                           void* stream);
int rai_bias_relu_bwd_nchw(const float* dy, const float* y, int64_t B, int32_t HW, int32_t C, float* dx, float* db,
                           int32_t accumulate, void* workspace, int64_t workspace_bytes, void* stream);
/* NatureCNN Conv2d -> ReLU forward in ONE launch (nature_cnn.py:31-41; replaces MIOpen's bias-free
 * convolution + rai_bias_relu_fwd): a hand-written f32 MFMA implicit GEMM with the bias + ReLU in its
 * store.  x NHWC fp32 (B, H, W, Ci); w channels_last (Co, KH, KW, Ci); b (Co); padding 0, dilation 1.
 * y: NHWC (B, OH, OW, Co), or with out_nchw != 0 the nn.Flatten order (B, Co * OH * OW).
 * Ci % 4 == 0, Co % 16 == 0 (the NatureCNN layers: Co 32 / 64), KH * KW * Ci % 32 == 0 and <= 8192,
 * every pointer 16-B aligned.  f32 products, summation order of the kernel (fp32 tolerance vs
 * PyTorch); deterministic. */
int rai_conv2d_bias_relu_fwd(const float* x, const float* w, const float* b, int64_t B, int32_t H, int32_t W,
                             int32_t Ci, int32_t Co, int32_t KH, int32_t KW, int32_t stride, int32_t out_nchw,
                             float* y, void* stream);
/* Split-K form (round 5): where the default tiling leaves CUs idle (NatureCNN conv2 / conv3 at the update
 * minibatch B = 256), the reduction is cut in two halves run as separate workgroups (two per CU, half the
 * LDS-resident weights each) whose raw sums go to `part` (rai_conv2d_fwd_splitk_bytes(...) bytes, 0 when
 * the shape takes no split: the call is then rai_conv2d_bias_relu_fwd), and a second pass adds them in
 * order with the bias and the ReLU. Same results as the one-pass form up to fp32 summation order. */
int64_t rai_conv2d_fwd_splitk_bytes(int64_t B, int32_t H, int32_t W, int32_t Ci, int32_t Co, int32_t KH, int32_t KW,
                                    int32_t stride, int32_t out_nchw);
int rai_conv2d_bias_relu_fwd_splitk(const float* x, const float* w, const float* b, int64_t B, int32_t H, int32_t W,
                                    int32_t Ci, int32_t Co, int32_t KH, int32_t KW, int32_t stride, int32_t out_nchw,
                                    float* y, float* part, int64_t part_bytes, void* stream);
/* The same with a fixed workgroup blocking (variant 0 = chosen by shape, as above; 1-15 = the blockings, prefetch depths and LDS-resident-weight forms
 * in csrc/conv.hip, for same-box A/B timing in tools/conv_bench.py). */
int rai_conv2d_bias_relu_fwd_v(const float* x, const float* w, const float* b, int64_t B, int32_t H, int32_t W,
                               int32_t Ci, int32_t Co, int32_t KH, int32_t KW, int32_t stride, int32_t out_nchw,
                               float* y, int32_t variant, void* stream);
/* Weight gradient of the same convolution (the dW of Conv2d's autograd backward, nature_cnn.py:31-41):
 * dw[co][kh][kw][ci] (channels_last, as optim.FlatParams stores it) = sum over the B * OH * OW output
 * pixels p of dz[p][co] * x[receptive field of p][kh][kw][ci]; accumulate != 0 adds it to dw (the
 * flat .grad view).  dz NHWC (B, OH, OW, Co) (the bias + ReLU backward's output).  Co 32 or 64,
 * Ci % 4 == 0, KH * KW * Ci % 64 == 0, pointers 16-B aligned.  Hand-written f32 MFMA: per-workgroup
 * partial tiles in workspace (rai_conv2d_wgrad_workspace_bytes, no zeroing needed), summed in a fixed
 * order by a second launch (deterministic).  Replaces MIOpen's weight-gradient solver, its split-K
 * zero-fill and the gradient's accumulate. */
int64_t rai_conv2d_wgrad_workspace_bytes(int64_t B, int32_t H, int32_t W, int32_t Ci, int32_t Co, int32_t KH,
                                         int32_t KW, int32_t stride);
int rai_conv2d_wgrad(const float* x, const float* dz, int64_t B, int32_t H, int32_t W, int32_t Ci, int32_t Co,
                     int32_t KH, int32_t KW, int32_t stride, float* dw, int32_t accumulate, void* workspace,
                     int64_t workspace_bytes, void* stream);
/* rai_conv2d_wgrad in two parts, so the backward's convolutions share ONE reduction launch: the
 * partials launch per layer (workspace as above, kept until the reduce has run), then
 * rai_conv2d_wgrad_reduce over up to RAI_WGRAD_MAX_JOBS layers (host array of jobs; each job's
 * shape arguments as passed to its partials call). */
#define RAI_WGRAD_MAX_JOBS 4
typedef struct rai_conv2d_wgrad_job {
  const void* workspace;
  float* dw;
  float* db; /* NULL, or (after rai_conv2d_wgrad_relu_partials) the bias gradient, Co floats, 16-B aligned */
  int64_t B;
  int32_t H, W, Ci, Co, KH, KW, stride, reserved;
} rai_conv2d_wgrad_job;
int rai_conv2d_wgrad_partials(const float* x, const float* dz, int64_t B, int32_t H, int32_t W, int32_t Ci,
                              int32_t Co, int32_t KH, int32_t KW, int32_t stride, void* workspace,
                              int64_t workspace_bytes, void* stream);
int rai_conv2d_wgrad_reduce(const rai_conv2d_wgrad_job* jobs, int32_t n_jobs, int32_t accumulate, void* stream);
/* The partials with the layer's bias + ReLU backward folded in, for a convolution whose dz has no other
 * consumer (NatureCNN conv1, whose input needs no gradient): dz = y > 0 ? dy : 0 (threshold_backward on
 * the saved output y) is formed on the fly from dy and y (both NHWC (B, OH, OW, Co)), and the bias
 * gradient's per-split partials are written after the weight tiles; the job's db receives their sum
 * in the reduce.  Replaces rai_bias_relu_bwd + rai_conv2d_wgrad_partials for that layer. */
int rai_conv2d_wgrad_relu_partials(const float* dy, const float* y, const float* x, int64_t B, int32_t H, int32_t W,
                                   int32_t Ci, int32_t Co, int32_t KH, int32_t KW, int32_t stride, void* workspace,
                                   int64_t workspace_bytes, void* stream);
/* The first NatureCNN layer on uint8 frames (round 4): x is the gathered uint8 NHWC minibatch (B, H, W, 4)
 * (RAI_XFORM_U8_CHW_TO_U8_HWC) and the kernels read x = u8 / x_divisor (IEEE division: the value
 * cnn.py:24-27's obs.float() / range_size and RAI_XFORM_U8_CHW_TO_F32_HWC give), so the float32 input is
 * never materialised.  Ci == 4, x 4-B aligned, B * H * W * 4 < 2^31; otherwise as the float32 forms.
 * The forward is the LDS-weight form (RAI_E_UNSUPPORTED if the weight rows do not fit LDS). */
int rai_conv2d_bias_relu_fwd_u8(const uint8_t* x, float x_divisor, const float* w, const float* b, int64_t B,
                                int32_t H, int32_t W, int32_t Ci, int32_t Co, int32_t KH, int32_t KW, int32_t stride,
                                int32_t out_nchw, float* y, void* stream);
int rai_conv2d_wgrad_partials_u8(const uint8_t* x, float x_divisor, const float* dz, int64_t B, int32_t H, int32_t W,
                                 int32_t Ci, int32_t Co, int32_t KH, int32_t KW, int32_t stride, void* workspace,
                                 int64_t workspace_bytes, void* stream);
int rai_conv2d_wgrad_relu_partials_u8(const float* dy, const float* y, const uint8_t* x, float x_divisor, int64_t B,
                                      int32_t H, int32_t W, int32_t Ci, int32_t Co, int32_t KH, int32_t KW,
                                      int32_t stride, void* workspace, int64_t workspace_bytes, void* stream);
/* Input gradient of the same convolution (Conv2d's autograd dx; NatureCNN conv2 / conv3): dx (B, H, W, Ci)
 * NHWC = the transposed convolution of dz (B, OH, OW, Co) NHWC with w (Co, KH, KW, Ci) channels_last,
 * every element written (no accumulate, no zero-fill).  Ci 32 or 64, Co % 16 == 0, KH and KW multiples
 * of stride, padding 0, pointers 16-B aligned.  Hand-written f32 MFMA, deterministic. */
int rai_conv2d_dgrad(const float* dz, const float* w, int64_t B, int32_t H, int32_t W, int32_t Ci, int32_t Co,
                     int32_t KH, int32_t KW, int32_t stride, float* dx, void* stream);
/* The same with a fixed form (variant 0 = default; 1, 2 = weights resident in LDS, persistent workgroups;
 * 3 = per image, pointer loads; 4 = per image, weights staged through LDS; 5 / 6 / 7 = per image, buffer
 * loads, 2 / 3 / 4 quads in flight; tools/conv_bench.py, tools/dgrad_probe.py A/B). */
int rai_conv2d_dgrad_v(const float* dz, const float* w, int64_t B, int32_t H, int32_t W, int32_t Ci, int32_t Co,
                       int32_t KH, int32_t KW, int32_t stride, float* dx, int32_t variant, void* stream);
/* The input gradient with the layer's ReLU backward folded in (round 4; NatureCNN conv2, whose dz also feeds
 * rai_conv2d_wgrad_relu_partials): dz = y > 0 ? dy : 0 is formed on the fly from dy and the saved output y
 * (both NHWC (B, OH, OW, Co)), so no rai_bias_relu_bwd pass materialises it.  The per-image form only:
 * RAI_E_UNSUPPORTED for shapes it is not instantiated for. */
int rai_conv2d_dgrad_relu(const float* dy, const float* y, const float* w, int64_t B, int32_t H, int32_t W,
                          int32_t Ci, int32_t Co, int32_t KH, int32_t KW, int32_t stride, float* dx, void* stream);
/* The same with a fixed launch shape for same-box A/B (tools/conv_bench.py): target_wgs workgroups
 * (0 = 512, at most 1024), pf pixel steps in flight per wave (0 = 4; 4 or 8). */
int rai_conv2d_wgrad_v(const float* x, const float* dz, int64_t B, int32_t H, int32_t W, int32_t Ci, int32_t Co,
                       int32_t KH, int32_t KW, int32_t stride, float* dw, int32_t accumulate, void* workspace,
                       int64_t workspace_bytes, int32_t target_wgs, int32_t pf, void* stream);

/* --------------------------------------------------------------------------
 * Device-resident hyperparameters and training state.
 * These live in HBM so a captured hipGraph replays against values the host
 * rewrites once per update (schedules: rl_algo_impls/shared/callbacks/
 * hyperparam_transitions.py:19-31 mutate lr/clip/ent/vf coefficients).
 * ------------------------------------------------------------------------ */
typedef struct rai_ppo_hparams {
  float clip_range;      /* ppo.py:224,328 */
  float clip_range_vf;   /* ppo.py:233-237; used iff has_clip_range_vf */
  float ent_coef;        /* ppo.py:359 */
  float kl_cutoff;       /* ppo.py:354; used iff has_kl_cutoff */
  float grad_scale;      /* 1/num_minibatches under gradient_accumulation (ppo.py:373-374) */
  int32_t K;             /* value columns */
  int32_t has_clip_range_vf;
  int32_t has_kl_cutoff;
  int32_t normalize_advantage;       /* ppo.py:313-314 */
  int32_t standardize_advantage;     /* ppo.py:315-316 */
  int32_t normalize_after_scaling;   /* ppo.py:307-311 */
  int32_t ppo2_vf_coef_halving;      /* ppo.py:348-349 */
  int32_t has_vf_weights;            /* ppo.py:344-345 */
  int32_t has_multi_reward_weights;  /* ppo.py:308-309,317-318 */
  int32_t vf_loss_fn;                /* 0 mse_loss, 1 huber_loss(delta=1), 2 smooth_l1_loss(beta=1) */
  int32_t loss_kind;                 /* 0 PPO clipped surrogate, 1 A2C -(A*logp) (a2c.py:148-158) */
  float vf_coef[RAI_MAX_K];
  float vf_weights[RAI_MAX_K];
  float multi_reward_weights[RAI_MAX_K];
  /* Data parallel (K == 1, not normalize_after_scaling): device (n_steps, 2) table of the GLOBAL
   * minibatch's advantage (mean, den) for stats row stat_index (den includes +1e-8 and the
   * normalize / standardize choice), replacing the per-rank moments; NULL: the minibatch's own. */
  const float* ext_moments;
} rai_ppo_hparams;

typedef struct rai_optim_hparams {
  float lr;            /* ppo.py:223 update_learning_rate */
  float beta1;         /* Adam (0.9) */
  float beta2;         /* Adam (0.999) */
  float eps;           /* ppo.py:146 eps=1e-7 ; RMSprop a2c.py:46 eps=1e-5 */
  float alpha;         /* RMSprop smoothing (0.99) */
  float max_grad_norm; /* ppo.py:442-444; <= 0 disables clipping */
  int32_t kind;        /* 0 Adam, 1 RMSprop */
  int32_t pad;
  double beta1_d;      /* betas as the Python floats torch uses for its bias corrections */
  double beta2_d;
} rai_optim_hparams;

typedef struct rai_train_state {
  int64_t opt_step;      /* torch optimizer state['step'] */
  int32_t stat_index;    /* next per-minibatch stats row */
  int32_t pi_coef_zero;  /* kl_cutoff latch, reset per update (ppo.py:279,354-355) */
  int32_t norm_index;    /* next grad-norm slot */
  int32_t err;           /* sticky device-side error flag (e.g. a bounded spin gave up) */
} rai_train_state;

/* Per-minibatch stats row layout (floats), stride RAI_STAT_STRIDE:
 *  [0] loss [1] pi_loss [2] entropy_loss [3] approx_kl [4] clipped_frac
 *  [5 .. 5+K) v_loss  [5+RAI_MAX_K .. 5+RAI_MAX_K+K) val_clipped_frac       */
#define RAI_STAT_STRIDE (5 + 2 * RAI_MAX_K)

/* --------------------------------------------------------------------------
 * Fused policy-gradient loss forward + backward (to the network outputs).
 * Replaces rl_algo_impls/ppo/ppo.py:307-371,379-396 (advantage normalisation,
 * clipped surrogate, (clipped) value loss, entropy loss, approx_kl/clip stats)
 * and rl_algo_impls/a2c/a2c.py:132-158 when hp->loss_kind == 1.
 *
 * Inputs (device, fp32): new_logp (B), entropy (n_entropy: B or B*act_dim),
 * new_values/old_values/advantages/returns (B,K), old_logp (B; unused for A2C).
 * Outputs: d_logp (B), d_entropy (n_entropy), d_values (B,K) = dLoss/d(output),
 * and one stats row written at stats[state->stat_index] (then stat_index++).
 * workspace: >= rai_ppo_loss_workspace_bytes(B, K) bytes of device memory.
 * ------------------------------------------------------------------------ */
int64_t rai_ppo_loss_workspace_bytes(int64_t B, int32_t K);
int rai_ppo_loss(const float* new_logp, const float* entropy, int64_t n_entropy,
                 const float* new_values, const float* old_logp, const float* old_values,
                 const float* advantages, const float* returns, int64_t B, int32_t K,
                 const rai_ppo_hparams* hp, rai_train_state* state, float* d_logp,
                 float* d_entropy, float* d_values, float* stats, int32_t max_stats,
                 void* workspace, int64_t workspace_bytes, void* stream);

/* --------------------------------------------------------------------------
 * Fused clip_grad_norm_ + optimizer step over one flat fp32 parameter buffer.
 * Replaces rl_algo_impls/ppo/ppo.py:441-447 (clip_grad_norm_(...).item(),
 * Adam(eps=1e-7).step(), zero_grad) and rl_algo_impls/a2c/a2c.py:202-205
 * (RMSprop).  Grads are zeroed after use (zero_grad equivalent; the flat grad
 * buffer keeps its storage so parameter .grad views stay valid).
 * The total grad norm (pre-clip) is written to norms[state->norm_index++].
 * state->opt_step is incremented on device (bias corrections use it).
 * The workspace (rai_optim_workspace_bytes) holds the per-block fp64
 * partial sums of squares; it is scratch for one call at a time per stream.
 * ------------------------------------------------------------------------ */
int64_t rai_optim_workspace_bytes(int64_t P);
int rai_clip_optim_step(float* params, float* grads, float* state1, float* state2, int64_t P,
                        const rai_optim_hparams* hp, rai_train_state* state, float* norms,
                        int32_t max_norms, void* workspace, int64_t workspace_bytes,
                        void* stream);

/* --------------------------------------------------------------------------
 * Multi-field row gather: dst_f[i] = src_f[idx[i]] for up to RAI_MAX_FIELDS
 * fields of arbitrary row size (bytes).  Replaces the minibatch fancy-index
 * gather of rl_algo_impls/rollout/rollout.py:56-69 / vec_rollout.py:166-175;
 * the trainer uses it once per epoch to materialise the permuted rollout so
 * that minibatches become contiguous slices.
 * ------------------------------------------------------------------------ */
#define RAI_MAX_FIELDS 8
int rai_gather_rows(int32_t n_fields, const void* const* src, void* const* dst,
                    const int64_t* row_bytes, const int64_t* idx, int64_t n_rows, void* stream);

/* --------------------------------------------------------------------------
 * Rollout staging (the env-step loop of rl_algo_impls/rollout/sync_step_rollout.py:193-207):
 * rai_copy_d2h_sync copies device -> host (pinned) on the stream and waits for the stream (the
 * step's actions for the host env); rai_copy_h2d_multi issues n (<= RAI_MAX_FIELDS) asynchronous
 * host (pinned) -> device copies on the stream (rewards, terminations, next observations).
 * ------------------------------------------------------------------------ */
int rai_copy_d2h_sync(const void* src, void* dst, int64_t bytes, void* stream);
int rai_copy_h2d_multi(int32_t n, void* const* dst, const void* const* src, const int64_t* bytes, void* stream);

/* --------------------------------------------------------------------------
 * Epoch shuffle: out[i] = perm_key(i), a keyed bijection of [0, n) (6-round
 * Feistel network over the smallest even-bit power-of-two domain >= n with
 * cycle walking; round keys from the 64-bit key).  Stands in for
 * torch.randperm(total_steps) of rl_algo_impls/rollout/vec_rollout.py:166-170
 * as the epoch permutation: one independent kernel thread per index instead
 * of a device sort.  Same key -> same permutation.
 * ------------------------------------------------------------------------ */
int rai_feistel_permutation(int64_t n, uint64_t key, int64_t* out, void* stream);

/* --------------------------------------------------------------------------
 * Device-indexed minibatch gather for graph-replayed updates.  The source
 * fields, the epoch permutation and the minibatch counter live in a device
 * descriptor, so one captured launch sequence (gather -> forward -> loss ->
 * backward -> optimizer) is replayed for every minibatch of an epoch without
 * host work.  rai_gather_minibatch copies rows perm[mb*B + i] (identity order
 * when perm is NULL), i < min(B, n_rows - mb*B), of every field into dst;
 * rai_minibatch_advance then increments desc->mb (a separate launch, so every
 * block of the gather has read mb).  Same rows as Batch.__getitem__ over
 * VecRollout.minibatches (rl_algo_impls/rollout/vec_rollout.py:166-175,
 * rollout.py:56-69).  Row sizes: multiples of 16, 4 or 1 bytes.
 * ------------------------------------------------------------------------ */
typedef struct rai_minibatch_desc {
  const void* src[RAI_MAX_FIELDS];
  int64_t row_bytes[RAI_MAX_FIELDS];
  const int64_t* perm;  /* epoch permutation of [0, n_rows), or NULL */
  int64_t n_rows;       /* rows in the rollout (T*N) */
  int64_t batch_size;
  int64_t mb;           /* next minibatch, advanced on device */
  int32_t n_fields;
  int32_t arrivals;     /* rai_gather_minibatch_next's block-arrival counter; 0 between launches */
  int32_t group_arrivals[8 * 16]; /* its per-group counters (8 groups, 64 B apart); 0 between launches */
} rai_minibatch_desc;
int rai_gather_minibatch(const rai_minibatch_desc* desc, int32_t n_fields, void* const* dst,
                         const int64_t* row_bytes, int64_t batch_size, void* stream);
int rai_minibatch_advance(rai_minibatch_desc* desc, void* stream);
/* Gather + advance in ONE launch: the last workgroup to finish (after every workgroup has read
 * desc->mb) increments desc->mb and re-arms desc->arrivals. */
int rai_gather_minibatch_next(rai_minibatch_desc* desc, int32_t n_fields, void* const* dst,
                              const int64_t* row_bytes, int64_t batch_size, void* stream);

/* Actor-critic heads of the NatureCNN policy: a Categorical actor head Linear(D, A) and a critic head
 * Linear(D, 1) over the encoder output enc (B, D), with the Categorical log-prob of `actions` and the
 * entropy (rl_algo_impls/shared/actor/categorical.py:57-87, rl_algo_impls/shared/policy/critic.py:11-41,
 * actor_critic_network/connected_trio.py:83-92; torch.distributions.Categorical arithmetic).
 * Forward: logits_out (B, A) (kept for the backward), logp_out / entropy_out / v_out (B).
 * Backward, two launches: from the upstream d_logp, d_entropy, d_v (B): d_enc (B, D) written, and the
 * gradients of wpi (A, D), bpi (A), wv (D), bv (1) written (accumulate == 0) or added (accumulate != 0,
 * e.g. into the flat .grad buffer).  A in 2..10 or 12; workspace >= rai_categorical_critic_heads_
 * workspace_bytes(B, A).  Fixed reduction orders (deterministic). */
int rai_categorical_critic_heads_fwd(const float* enc, const float* wpi, const float* bpi, const float* wv,
                                     const float* bv, const int64_t* actions, int64_t B, int32_t D, int32_t A,
                                     float* logits_out, float* logp_out, float* entropy_out, float* v_out,
                                     void* stream);
int64_t rai_categorical_critic_heads_workspace_bytes(int64_t B, int32_t A);
int rai_categorical_critic_heads_bwd(const float* enc, const float* wpi, const float* bpi, const float* wv,
                                     const float* bv, const int64_t* actions, const float* logits, int64_t B,
                                     int32_t D, int32_t A, const float* d_logp, const float* d_entropy,
                                     const float* d_v, float* d_enc, float* g_wpi, float* g_bpi, float* g_wv,
                                     float* g_bv, int32_t accumulate, void* workspace, int64_t workspace_bytes,
                                     void* stream);
/* The same backward with the ReLU backward of the layer that produced enc folded in (round 4; NatureCNN's
 * fc -> ReLU, rl_algo_impls/shared/encoder/cnn.py:44-53): dz = enc <= 0 ? 0 : d_enc (threshold_backward on
 * the saved ReLU output) is written in place of d_enc, and g_benc (D floats) receives that layer's bias
 * gradient (the column sums of dz, fixed order; accumulate != 0 adds).  Replaces rai_bias_relu_bwd there. */
int rai_categorical_critic_heads_bwd_relu(const float* enc, const float* wpi, const float* bpi, const float* wv,
                                          const float* bv, const int64_t* actions, const float* logits, int64_t B,
                                          int32_t D, int32_t A, const float* d_logp, const float* d_entropy,
                                          const float* d_v, float* dz, float* g_wpi, float* g_bpi, float* g_wv,
                                          float* g_bv, float* g_benc, int32_t accumulate, void* workspace,
                                          int64_t workspace_bytes, void* stream);

/* Per-field output transform of the minibatch gather.
 *   RAI_XFORM_COPY: the row's bytes are copied (as above).
 *   RAI_XFORM_U8_CHW_TO_F32_HWC: the source row is `channels` (<= 4) planes of `hw` uint8 pixels
 *     (hw % 4 == 0; row_bytes = channels * hw), the rollout's NCHW frames; dst receives hw x channels
 *     float32 (NHWC, i.e. a channels_last (B, C, H, W) tensor, 16-B aligned) with
 *     out = (float)u8 / divisor (IEEE division).  This is the NatureCNN input prescale
 *     `obs.float() / range_size` of rl_algo_impls/shared/encoder/cnn.py:24-27 plus the channels_last
 *     conversion, fused into the gather of rl_algo_impls/rollout/rollout.py:56-69.
 *   RAI_XFORM_U8_CHW_TO_U8_HWC (round 4): the same source row (channels == 4), transposed only: dst
 *     receives hw x 4 uint8 (a channels_last uint8 tensor, 16-B aligned) for the uint8-input
 *     convolution (rai_conv2d_bias_relu_fwd_u8), which applies the prescale itself.
 * rai_gather_minibatch_x: rai_gather_minibatch (advance == 0) / _next (advance != 0) with one
 * rai_gather_xform per field (xform NULL: all copies).  Errors: RAI_E_SHAPE for a transform whose
 * shape or alignment does not fit, RAI_E_MODE for an unknown kind. */
#define RAI_XFORM_COPY 0
#define RAI_XFORM_U8_CHW_TO_F32_HWC 1
#define RAI_XFORM_U8_CHW_TO_U8_HWC 2
typedef struct rai_gather_xform {
  int32_t kind;
  int32_t channels;
  int64_t hw;
  float divisor;
  int32_t reserved;
} rai_gather_xform;
int rai_gather_minibatch_x(rai_minibatch_desc* desc, int32_t n_fields, void* const* dst, const int64_t* row_bytes,
                           const rai_gather_xform* xform, int64_t batch_size, int32_t advance, void* stream);

/* --------------------------------------------------------------------------
 * Rollout post-head: sample actions from the policy head and write the
 * rollout-buffer slot.  Replaces rl_algo_impls/shared/policy/actor_critic.py:
 * 306-318 (pi.sample, pi.log_prob, .cpu()) and the slot writes of
 * rl_algo_impls/rollout/sync_step_rollout.py:193-201.
 * Random numbers: Philox4x32-10 keyed by (seed), counter (offset, row).
 * ------------------------------------------------------------------------ */
int rai_categorical_sample(const float* logits, const uint8_t* mask, int64_t N, int32_t A,
                           uint64_t seed, uint64_t offset, int64_t* actions_out, float* logp_out,
                           const float* v_in, float* v_out, int32_t K, void* stream);
int rai_gaussian_sample(const float* mu, const float* log_std, int64_t N, int32_t A,
                        const float* low, const float* high, uint64_t seed, uint64_t offset,
                        float* actions_out, float* clamped_out, float* logp_out,
                        const float* v_in, float* v_out, int32_t K, void* stream);

/* --------------------------------------------------------------------------
 * Fused rollout step for CartPole-class MLP actor-critics (Flatten encoder,
 * [in_dim -> 64 -> 64 -> out] actor and critic, Categorical head; in_dim <= 8,
 * n_actions <= 8): both forward passes, the categorical sample and the slot
 * writes in one launch.  Replaces rl_algo_impls/shared/policy/actor_critic.py:
 * 306-318 + rl_algo_impls/rollout/sync_step_rollout.py:193-201 for this class
 * (and ActorCritic.value, actor_critic.py:298-304, when actions_out/logp_out are
 * NULL).  pi_params / v_params: host arrays of 6 device pointers {W1, b1, W2, b2,
 * W3, b3} (torch Linear layout, weight [out][in]).  Sampling is the stream of
 * rai_categorical_sample (same seed/offset/row keying).
 * ------------------------------------------------------------------------ */
int rai_mlp_policy_step(const float* const* pi_params, const float* const* v_params, const float* obs,
                        int64_t N, int32_t in_dim, int32_t hidden, int32_t n_actions,
                        int32_t activation, uint64_t seed, uint64_t offset, int64_t* actions_out,
                        float* logp_out, float* values_out, void* stream);
/* The same step with the env hand-off folded in (sync_step_rollout.py:193-207): obs_host / rew_host /
 * done_host are DEVICE addresses of host-mapped pinned buffers (rai_host_alloc) holding the env's next
 * observations (N x in_dim f32), rewards (N f32) and terminations (N u8); the kernel reads the
 * observations from there and writes them into obs_slot, copies rewards / terminations into rew_dst /
 * done_dst (either pair may be NULL), and writes the sampled actions to actions_out AND actions_host.
 * One launch + rai_stream_sync per env step instead of the copies. */
int rai_mlp_policy_step_mapped(const float* const* pi_params, const float* const* v_params, const float* obs_host,
                               float* obs_slot, int64_t N, int32_t in_dim, int32_t hidden, int32_t n_actions,
                               int32_t activation, uint64_t seed, uint64_t offset, int64_t* actions_out,
                               float* logp_out, float* values_out, int64_t* actions_host, const float* rew_host,
                               float* rew_dst, const uint8_t* done_host, uint8_t* done_dst, void* stream);
/* Host-mapped (coherent) pinned memory: host_out for the CPU, dev_out for kernels. */
int rai_host_alloc(int64_t bytes, void** host_out, void** dev_out);
int rai_host_free(void* host);
int rai_stream_sync(void* stream);

/* --------------------------------------------------------------------------
 * Fused PPO epoch for MLP actor-critics (Flatten encoder, separate
 * [in_dim -> 64 -> 64 -> out] actor and critic MLPs, Categorical head; the
 * CartPole-class policies of rl_algo_impls/shared/policy/actor_critic_network/
 * connected_trio.py).  One call = every minibatch of one epoch of
 * rl_algo_impls/ppo/ppo.py:290-411 (forward, loss, backward, clip_grad_norm_,
 * Adam) over rows [0, n_rows) of the (already permuted) rollout, minibatch i =
 * rows [i*batch_size, (i+1)*batch_size).  params / exp_avg / exp_avg_sq are the
 * flat buffers in torch parameters() order.  Requires hidden == 64,
 * in_dim <= 8, n_actions <= 8, batch_size <= 256, activation 0 tanh / 1 relu,
 * K == 1, no kl_cutoff and no gradient accumulation.
 * Stats rows: [0] holds the policy+entropy part of the loss; the caller adds
 * vf_coef * v_loss ([5]).
 * ------------------------------------------------------------------------ */
/* batch_size > 256 (SURVEY 8(d) batch policy (b), e.g. batch = n_steps * num_envs / 4; in_dim <= 4,
 * n_actions == 2, else RAI_E_UNSUPPORTED): the throughput-bound large-minibatch form.  Per epoch two
 * small launches compute every minibatch's advantage moments; per minibatch three launches: forward,
 * loss and backward partial gradients over all CUs (256 workgroups, 16-row MFMA tiles), a fixed-order
 * reduction of the 128 partials per network into the gradient + the stats row, clip_grad_norm_ + Adam.
 * Deterministic.  rai_mlp_ppo_grads takes the same form for batch_size > 256 (mb_count == 1).
 * Workspace: the inter-workgroup exchange words plus one (mean, den) pair per minibatch (<= 256
 * rows); the moments, partial gradients (~4.7 MB) and norm partials (> 256 rows). */
int64_t rai_mlp_ppo_workspace_bytes(int64_t n_rows, int32_t batch_size);
int rai_mlp_ppo_epoch(float* params, float* exp_avg, float* exp_avg_sq, const float* obs,
                      const int64_t* actions, const float* old_logp, const float* old_values,
                      const float* advantages, const float* returns, int64_t n_rows,
                      int32_t batch_size, int32_t in_dim, int32_t hidden, int32_t n_actions,
                      int32_t activation, const rai_ppo_hparams* hp, const rai_optim_hparams* ohp,
                      rai_train_state* state, float* stats, int32_t max_stats, float* norms,
                      int32_t max_norms, void* workspace, int64_t workspace_bytes, void* stream);

/* Data-parallel variant: processes minibatches [mb_begin, mb_begin+mb_count) of the
 * permuted rollout with the current parameters, normalising advantages with the given
 * global per-minibatch (mean, den) pairs (moments[2*mb], moments[2*mb+1]; den already
 * includes +1e-8 and the normalize/standardize choice) and averaging the loss over
 * rows*world samples, and writes the raw (pre-clip) gradients to grad_out in flat
 * parameter order.  The caller all-reduces grad_out across ranks (RCCL) and then runs
 * rai_clip_optim_step.  One stats row per minibatch holds this rank's share. */
int rai_mlp_ppo_grads(const float* params, const float* obs, const int64_t* actions,
                      const float* old_logp, const float* old_values, const float* advantages,
                      const float* returns, int64_t n_rows, int32_t batch_size, int32_t mb_begin,
                      int32_t mb_count, const float* moments, int32_t world, int32_t in_dim,
                      int32_t hidden, int32_t n_actions, int32_t activation,
                      const rai_ppo_hparams* hp, const rai_optim_hparams* ohp,
                      rai_train_state* state, float* grad_out, float* stats, int32_t max_stats,
                      void* workspace, int64_t workspace_bytes, void* stream);

/* --------------------------------------------------------------------------
 * Wide MLP actor-critic minibatch step (HalfCheetah-class policies: Flatten
 * encoder, separate [in -> H -> H -> out] actor and critic, H in {64,128,192,256},
 * Gaussian (head 1) or Categorical (head 0) actor, scalar critic).  Replaces the
 * per-minibatch PyTorch forward of rl_algo_impls/shared/policy/actor_critic_network/
 * connected_trio.py (+ shared/actor/gaussian.py:11-61, categorical.py, shared/policy/
 * critic.py) and its autograd backward inside rl_algo_impls/ppo/ppo.py:290-377.
 *   rai_mlp_wide_forward:  3 launches -> logp (B), entropy (B*out for Gaussian, B for
 *                          Categorical), v (B) for rai_ppo_loss
 *   rai_mlp_wide_backward: 2 launches -> gradients of every parameter (written, or added
 *                          when accumulate) from rai_ppo_loss's d_logp, d_entropy, d_v
 * w[n] / g[n]: network n (0 actor, 1 critic) W1 (H,in), b1, W2 (H,H), b2, W3 (out,H),
 * b3 and their gradient views; actions: (B, out) fp32 (Gaussian) or (B,) int64.
 * workspace: rai_mlp_wide_workspace_bytes(B, H) bytes, shared by the two calls.
 * ------------------------------------------------------------------------ */
#define RAI_WIDE_MAX_B 256
#define RAI_WIDE_MAX_H 256
#define RAI_WIDE_MAX_IN 64
#define RAI_WIDE_MAX_OUT 8
typedef struct rai_mlp_wide_desc {
  const float* w[2][6];
  float* g[2][6];
  const float* log_std; /* Gaussian head: (out) */
  float* g_log_std;
  int32_t in_dim;
  int32_t hidden;
  int32_t out_pi;
  int32_t head;       /* 0 Categorical, 1 Gaussian */
  int32_t activation; /* 0 tanh, 1 relu */
  int32_t accumulate; /* 1: gradients are added (gradient accumulation) */
} rai_mlp_wide_desc;
int64_t rai_mlp_wide_workspace_bytes(int64_t B, int32_t hidden);
int rai_mlp_wide_forward(const rai_mlp_wide_desc* desc, const float* obs, const void* actions, int64_t B,
                         float* logp_out, float* entropy_out, float* v_out, void* workspace,
                         int64_t workspace_bytes, void* stream);
/* Rollout forward of the wide MLP (rl_algo_impls/shared/policy/actor_critic.py:306-318 up to the
 * distribution): params_out (B, out_pi) = the Gaussian mean or the Categorical logits, v_out (B) the
 * critic value, for the sampler (rai_gaussian_sample / rai_categorical_sample).  3 launches instead
 * of the PyTorch module's GEMMs and elementwise kernels; desc->g is not used. */
int rai_mlp_wide_dist_params(const rai_mlp_wide_desc* desc, const float* obs, int64_t B, float* params_out,
                             float* v_out, void* workspace, int64_t workspace_bytes, void* stream);
/* rai_mlp_wide_forward followed by rai_ppo_loss (K = 1) with the head and the loss in ONE
 * workgroup launch: same arguments as the two calls, same results (the loss body is shared). */
int rai_mlp_wide_forward_loss(const rai_mlp_wide_desc* desc, const float* obs, const void* actions, int64_t B,
                              float* logp_out, float* entropy_out, float* v_out, const float* old_logp,
                              const float* old_values, const float* advantages, const float* returns,
                              const rai_ppo_hparams* hp, rai_train_state* state, float* d_logp, float* d_entropy,
                              float* d_values, float* stats, int32_t max_stats, void* workspace,
                              int64_t workspace_bytes, void* stream);
int rai_mlp_wide_backward(const rai_mlp_wide_desc* desc, const float* obs, const void* actions, int64_t B,
                          const float* d_logp, const float* d_entropy, const float* d_v, void* workspace,
                          int64_t workspace_bytes, void* stream);
/* One whole PPO epoch for the wide MLP actor-critic in ONE launch (persistent kernel,
 * csrc/mlp_wide_epoch.hip): for every minibatch of batch_size (<= 64) consecutive rows of the
 * epoch's permuted rollout copy, the forward, head log-prob / entropy, the clipped-surrogate /
 * value / entropy loss, the backward, clip_grad_norm_ and Adam -- replaces the per-minibatch loop
 * of rl_algo_impls/ppo/ppo.py:290-411 (forward + loss + backward + optimizer_step at :441-447).
 * The parameters (desc->w / log_std: views of the flat buffer `params`, P floats) and the Adam
 * moments (exp_avg / exp_avg_sq, same layout) are read at the start and written back at the end;
 * gradients never reach HBM (desc->g is unused).  Stats rows / grad norms / state as
 * rai_mlp_ppo_epoch (stats[0] excludes the value term: the host adds vf_coef * stats[5]).
 * Options outside K = 1, Adam, no gradient accumulation / kl_cutoff / multi-reward weights
 * are not covered (the caller keeps the per-minibatch path).  workspace:
 * rai_mlp_wide_epoch_workspace_bytes(hidden, in_dim, n_rows) (its counters are reset by the call; it
 * also holds the epoch's per-row records -- minibatch-normalized advantage, loss inputs, padded
 * observation -- built by a first small launch on the stream). */
int64_t rai_mlp_wide_epoch_workspace_bytes(int32_t hidden, int32_t in_dim, int64_t n_rows);
int rai_mlp_wide_epoch(const rai_mlp_wide_desc* desc, float* params, float* exp_avg, float* exp_avg_sq, int64_t P,
                       const float* obs, const void* actions, const float* old_logp, const float* old_values,
                       const float* advantages, const float* returns, int64_t n_rows, int32_t batch_size,
                       const rai_ppo_hparams* hp, const rai_optim_hparams* ohp, rai_train_state* state,
                       float* stats, int32_t max_stats, float* norms, int32_t max_norms, void* workspace,
                       int64_t workspace_bytes, void* stream);
/* Data-parallel form (one process per GPU, world 2..8): rank `rank` runs its batch_size-row slices of
 * the global minibatches (its own permuted rollout copy, n_rows rows); after each step's backward every
 * workgroup's owned gradient is summed over the ranks in rank order through the IPC-mapped exchange
 * regions (rai_xdp_alloc / rai_xdp_open; peers: device array of the world region pointers, rank order;
 * step_base: optimizer steps already run through them), so every rank applies the identical clip + Adam.
 * moments: the global minibatches' (mean, den) pairs with the normalize / standardize rule encoded
 * (A = (adv - mean) / den), as for rai_mlp_ppo_epoch_xdp; loss means and stats rows are over
 * batch_size x world rows (the caller sums the stats rows over the ranks). */
int rai_mlp_wide_epoch_xdp(const rai_mlp_wide_desc* desc, float* params, float* exp_avg, float* exp_avg_sq,
                           int64_t P, const float* obs, const void* actions, const float* old_logp,
                           const float* old_values, const float* advantages, const float* returns, int64_t n_rows,
                           int32_t batch_size, const float* moments, int32_t world, int32_t rank, void* const* peers,
                           int64_t step_base, const rai_ppo_hparams* hp, const rai_optim_hparams* ohp,
                           rai_train_state* state, float* stats, int32_t max_stats, float* norms, int32_t max_norms,
                           void* workspace, int64_t workspace_bytes, void* stream);

/* Timing hook of the large-minibatch form (bench.py's roofline): rai_mlp_large_timing(n) arms HIP
 * events around the next n gradient-kernel launches (0 disarms); rai_mlp_large_timing_read writes the
 * launches' durations in ms (in launch order, waiting for them) and their count. */
int rai_mlp_large_timing(int32_t capacity);
int rai_mlp_large_timing_read(float* ms_out, int32_t max_out, int32_t* count_out);

/* --------------------------------------------------------------------------
 * Data-parallel runtime: one process per GPU, an RCCL
 * communicator over xGMI, and the natively driven per-minibatch loop
 *   rai_mlp_ppo_grads -> in-place sum all-reduce of the flat gradient -> rai_clip_optim_step
 * for one epoch (replaces the single-process optimizer loop of
 * rl_algo_impls/ppo/ppo.py:290-411; every rank applies the identical update).
 * RCCL is resolved at run time from the process's librccl.so.1 (the one PyTorch-ROCm
 * maps); rai_dp_available() reports whether it was found.  The unique id is created
 * on rank 0 and shipped to the other ranks by the caller (e.g. torch.distributed).
 * grads: flat fp32 buffer of P elements (same order as params).  moments: global
 * per-minibatch (mean, den) pairs as for rai_mlp_ppo_grads.  grads_alt (optional, P
 * elements): with it, CartPole-class policies take the two-launch step (the multi-CU
 * kernel applies the previous all-reduced gradient, then computes the next partial one;
 * one RCCL all-reduce per step); without it, or for other shapes, each step is
 * rai_mlp_ppo_grads -> all-reduce -> rai_clip_optim_step.
 * ------------------------------------------------------------------------ */
#define RAI_DP_UID_BYTES 128
int rai_dp_available(void);
int rai_dp_unique_id(void* out, int32_t out_bytes);
int rai_dp_comm_init(void** comm_out, const void* uid_bytes, int32_t world, int32_t rank);
int rai_dp_comm_destroy(void* comm);
int rai_dp_allreduce_sum_f32(void* comm, float* buf, int64_t n, void* stream);
int rai_mlp_ppo_epoch_dp(float* params, float* grads, float* exp_avg, float* exp_avg_sq, int64_t P,
                         const float* obs, const int64_t* actions, const float* old_logp,
                         const float* old_values, const float* advantages, const float* returns,
                         int64_t n_rows, int32_t batch_size, const float* moments, int32_t world,
                         int32_t in_dim, int32_t hidden, int32_t n_actions, int32_t activation,
                         const rai_ppo_hparams* hp, const rai_optim_hparams* ohp,
                         rai_train_state* state, float* stats, int32_t max_stats, float* norms,
                         int32_t max_norms, void* comm, float* grads_alt, void* workspace,
                         int64_t workspace_bytes, void* optim_workspace, int64_t optim_workspace_bytes,
                         void* stream);

/* --------------------------------------------------------------------------
 * In-kernel cross-GPU gradient all-reduce over xGMI peer memory (CartPole-class
 * policies, the multi-CU epoch kernel).  Each rank allocates one exchange region
 * (uncached device memory, rai_xdp_alloc(rai_xdp_region_bytes(world))), exports
 * it by IPC handle, maps every other rank's region (rai_xdp_open) and passes the
 * device array of all world region pointers (own included, rank order) to
 * rai_mlp_ppo_epoch_xdp: one launch per epoch; per optimizer step the kernel
 * pushes this rank's gradient share into every region, waits for every rank's
 * step flag, sums the world slots in rank order and applies the identical
 * clip + Adam on every rank.  step_base = optimizer steps already run through the
 * regions (the flags hold monotonic step ids and are zeroed only at allocation).
 * world <= 8.  Replaces the per-step RCCL all-reduce of rai_mlp_ppo_epoch_dp for
 * this policy class (same semantics, no per-step launches).
 * batch_size > 256 (SURVEY 8(d) batch policy (b), in_dim <= 4, two actions): the large-minibatch
 * steps (rai_mlp_ppo_epoch's all-CU form, three launches per optimizer step, no host sync); the
 * exchange sits in each step's reduce launch: every 64-parameter block of this rank's reduced
 * gradient goes into every rank's region, each block waits for the world's flags of that block
 * and sums the slots in rank order, then clip + Adam run on the identical global gradient.
 * Replaces rai_mlp_ppo_grads -> host RCCL all-reduce -> rai_clip_optim_step per step.
 * ------------------------------------------------------------------------ */
int64_t rai_xdp_region_bytes(int32_t world);
int rai_xdp_handle_bytes(void);
int rai_xdp_alloc(int64_t bytes, void** region_out);
int rai_xdp_free(void* region);
int rai_xdp_handle(void* region, void* handle_out, int32_t out_bytes);
int rai_xdp_open(const void* handle, void** peer_region_out);
int rai_xdp_close(void* peer_region);
/* Setup canary: same memory, scopes and flag protocol on a known payload; bad[0] counts wrong
 * values, bad[1] timeouts (device int32[2], zeroed by the caller).  tag: a fresh id >= 1. */
int rai_xdp_selftest(void* const* peers, int32_t world, int32_t rank, int64_t tag, int32_t* bad,
                     void* stream);
int rai_mlp_ppo_epoch_xdp(float* params, float* exp_avg, float* exp_avg_sq, const float* obs,
                          const int64_t* actions, const float* old_logp, const float* old_values,
                          const float* advantages, const float* returns, int64_t n_rows,
                          int32_t batch_size, const float* moments, int32_t world, int32_t rank,
                          void* const* peers, int64_t step_base, int32_t in_dim, int32_t hidden,
                          int32_t n_actions, int32_t activation, const rai_ppo_hparams* hp,
                          const rai_optim_hparams* ohp, rai_train_state* state, float* stats,
                          int32_t max_stats, float* norms, int32_t max_norms, void* workspace,
                          int64_t workspace_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* RAI_AMD_H_ */
