// Fused clip_grad_norm_ + Adam / RMSprop over one flat fp32 parameter buffer.
//
// Restates rl_algo_impls/ppo/ppo.py:441-447 (optimizer_step: clip_grad_norm_ ->
// Adam(eps=1e-7).step() -> zero_grad) with torch's update formulas
// (torch/optim/adam.py _single_tensor_adam / _multi_tensor_adam):
//   m   = lerp(m, g, 1-b1)            v = v*b2 + (1-b2)*g*g
//   denom = sqrt(v)/sqrt(1-b2^t) + eps
//   p  += -(lr/(1-b1^t)) * (m/denom)
// and rl_algo_impls/a2c/a2c.py:45-50,202-205 (RMSprop, alpha=0.99):
//   s = s*alpha + (1-alpha)*g*g ;  p += -lr * g/(sqrt(s)+eps)
// clip: total = ||g||_2 ; coef = max_norm/(total+1e-6) clamped to 1 ; g *= coef.
//
// Two launches, no atomics, deterministic:
//   K1 per-block partial sum of squares (fp64) -> workspace
//   K2 every block re-reduces the partials in the same fixed order (identical
//      result in every block), then scales, updates, and zeroes its slice.
// The step counter and grad-norm slot live in device memory (rai_train_state)
// so a captured graph replays correctly.
#include "common.h"

#pragma clang fp contract(off)

namespace {

constexpr int OPT_THREADS = 256;
constexpr int OPT_MAX_BLOCKS = 512;
constexpr int OPT_VEC = 4;

__global__ __launch_bounds__(OPT_THREADS) void grad_sumsq_kernel(const float* __restrict__ g,
                                                                int64_t P, int aligned,
                                                                double* partial,
                                                                rai_train_state* state) {
  __shared__ double red[OPT_THREADS / 64];
  double s = 0.0;
  const int64_t stride = (int64_t)gridDim.x * OPT_THREADS;
  const int64_t nvec = aligned ? P / OPT_VEC : 0;
  const float4* g4 = reinterpret_cast<const float4*>(g);
  for (int64_t i = (int64_t)blockIdx.x * OPT_THREADS + threadIdx.x; i < nvec; i += stride) {
    const float4 x = g4[i];
    s += (double)x.x * x.x + (double)x.y * x.y + (double)x.z * x.z + (double)x.w * x.w;
  }
  for (int64_t i = nvec * OPT_VEC + (int64_t)blockIdx.x * OPT_THREADS + threadIdx.x; i < P;
       i += stride)
    s += (double)g[i] * g[i];
  double v[1] = {s};
  block_sum<1>(v, red);
  if (threadIdx.x == 0) {
    partial[blockIdx.x] = v[0];
    if (blockIdx.x == 0) state->opt_step += 1;  // K2 (next in stream order) reads the new step
  }
}

__global__ __launch_bounds__(OPT_THREADS) void clip_optim_kernel(
    float* __restrict__ p, float* __restrict__ g, float* __restrict__ s1, float* __restrict__ s2,
    int64_t P, const rai_optim_hparams* __restrict__ hpp, rai_train_state* state,
    const double* __restrict__ partial, int nparts, float* norms, int max_norms) {
  __shared__ double red[OPT_THREADS / 64];
  const rai_optim_hparams hp = *hpp;
  // identical fixed-order reduction in every block
  double t = 0.0;
  for (int i = threadIdx.x; i < nparts; i += OPT_THREADS) t += partial[i];
  double v[1] = {t};
  block_sum<1>(v, red);
  const float total_norm = (float)sqrt(v[0]);
  float coef = 1.f;
  if (hp.max_grad_norm > 0.f) {
    coef = hp.max_grad_norm / (total_norm + 1e-6f);
    coef = fminf(coef, 1.f);
  }
  const int64_t step = state->opt_step;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const int ni = state->norm_index;
    if (norms && ni < max_norms) norms[ni] = total_norm;
    state->norm_index = ni + 1;
  }
  const int64_t stride = (int64_t)gridDim.x * OPT_THREADS;
  if (hp.kind == 0) {
    const double bc1 = 1.0 - ipow(hp.beta1_d, step);
    const double bc2 = 1.0 - ipow(hp.beta2_d, step);
    const float w1 = (float)(1.0 - hp.beta1_d);   // lerp weight (torch: 1 - beta1 in Python)
    const float w2 = (float)(1.0 - hp.beta2_d);   // addcmul value
    const float bc2_sqrt = (float)sqrt(bc2);
    const float neg_step = (float)(-((double)hp.lr / bc1));
    for (int64_t i = (int64_t)blockIdx.x * OPT_THREADS + threadIdx.x; i < P; i += stride) {
      const float gi = g[i] * coef;
      g[i] = 0.f;  // zero_grad (storage kept so .grad views stay valid)
      float m = s1[i];
      m = m + w1 * (gi - m);
      float vv = s2[i] * hp.beta2;
      vv = vv + (w2 * gi) * gi;
      const float denom = sqrtf(vv) / bc2_sqrt + hp.eps;
      p[i] = p[i] + neg_step * (m / denom);
      s1[i] = m;
      s2[i] = vv;
    }
  } else {
    const float w = (float)(1.0 - hp.beta1_d);  // RMSprop: beta1_d carries alpha as a Python float
    const float neg_lr = -hp.lr;
    for (int64_t i = (int64_t)blockIdx.x * OPT_THREADS + threadIdx.x; i < P; i += stride) {
      const float gi = g[i] * coef;
      g[i] = 0.f;
      float sq = s1[i] * hp.alpha;
      sq = sq + (w * gi) * gi;
      const float avg = sqrtf(sq) + hp.eps;
      p[i] = p[i] + neg_lr * (gi / avg);
      s1[i] = sq;
    }
  }
}

inline int opt_blocks(int64_t P) {
  int64_t b = (P + OPT_THREADS * 8 - 1) / (OPT_THREADS * 8);
  if (b < 1) b = 1;
  if (b > OPT_MAX_BLOCKS) b = OPT_MAX_BLOCKS;
  return (int)b;
}

}  // namespace

extern "C" int64_t rai_optim_workspace_bytes(int64_t /*P*/) {
  return (int64_t)OPT_MAX_BLOCKS * sizeof(double);
}

extern "C" int rai_clip_optim_step(float* params, float* grads, float* state1, float* state2,
                                   int64_t P, const rai_optim_hparams* hp, rai_train_state* state,
                                   float* norms, int32_t max_norms, void* workspace,
                                   int64_t workspace_bytes, void* stream) {
  if (P < 1) return RAI_E_SHAPE;
  if (!params || !grads || !state1 || !hp || !state || !workspace) return RAI_E_NULLPTR;
  if (workspace_bytes < rai_optim_workspace_bytes(P)) return RAI_E_WORKSPACE;
  if (!state2) state2 = state1;  // RMSprop uses one state buffer
  const int blocks = opt_blocks(P);
  double* partial = reinterpret_cast<double*>(workspace);
  const int aligned = ((uintptr_t)grads % 16) == 0;
  hipLaunchKernelGGL(grad_sumsq_kernel, dim3(blocks), dim3(OPT_THREADS), 0, rai_stream(stream),
                     grads, P, aligned, partial, state);
  RAI_LAUNCH_CHECK();
  hipLaunchKernelGGL(clip_optim_kernel, dim3(blocks), dim3(OPT_THREADS), 0, rai_stream(stream),
                     params, grads, state1, state2, P, hp, state, partial, blocks, norms,
                     max_norms);
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}
