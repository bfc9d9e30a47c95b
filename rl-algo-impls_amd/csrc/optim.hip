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
// Deterministic.  Two-launch form (any alignment / size):
//   K1 per-block partial sum of squares (fp64) -> workspace
//   K2 every block re-reduces the partials in the same fixed order (identical
//      result in every block), then scales, updates, and zeroes its slice.
// The step counter and grad-norm slot live in device memory (rai_train_state)
// so a captured graph replays correctly.
#include "common.h"
#include "internal.h"

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
    const double* __restrict__ partial, int nparts, float* norms, int max_norms, int vec) {
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
  const int64_t gtid = (int64_t)blockIdx.x * OPT_THREADS + threadIdx.x;
  // the per-element update (torch's formulas, no contraction); g is zeroed (zero_grad)
  float c1, c2, c3, c4;  // Adam: w1, w2, bc2_sqrt, neg_step; RMSprop: w, neg_lr, -, -
  if (hp.kind == 0) {
    const double bc1 = 1.0 - ipow(hp.beta1_d, step);
    const double bc2 = 1.0 - ipow(hp.beta2_d, step);
    c1 = (float)(1.0 - hp.beta1_d);   // lerp weight (torch: 1 - beta1 in Python)
    c2 = (float)(1.0 - hp.beta2_d);   // addcmul value
    c3 = (float)sqrt(bc2);
    c4 = (float)(-((double)hp.lr / bc1));
  } else {
    c1 = (float)(1.0 - hp.beta1_d);  // RMSprop: beta1_d carries alpha as a Python float
    c2 = -hp.lr;
    c3 = c4 = 0.f;
  }
  const bool adam = hp.kind == 0;
  auto upd = [&](float graw, float& pp, float& m, float& vv) {
    const float gi = graw * coef;
    if (adam) {
      m = m + c1 * (gi - m);
      vv = vv * hp.beta2;
      vv = vv + (c2 * gi) * gi;
      const float denom = sqrtf(vv) / c3 + hp.eps;
      pp = pp + c4 * (m / denom);
    } else {
      float sq = m * hp.alpha;  // RMSprop keeps its square average in s1
      sq = sq + (c1 * gi) * gi;
      const float avg = sqrtf(sq) + hp.eps;
      pp = pp + c2 * (gi / avg);
      m = sq;
    }
  };
  // float4 body when every buffer is 16-B aligned: two vectors per thread in flight per iteration
  // (the scalar grid-stride loop was ~13 dependent round trips per thread at C3's 1.69M parameters:
  // 12.8 us per step); then the scalar tail.  Same arithmetic per element, same results.
  int64_t done = 0;
  if (vec) {
    const int64_t nv = P / 4;
    float4* p4 = reinterpret_cast<float4*>(p);
    float4* g4 = reinterpret_cast<float4*>(g);
    float4* m4 = reinterpret_cast<float4*>(s1);
    float4* v4 = reinterpret_cast<float4*>(s2);
    const float4 zero = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t i = gtid; i < nv; i += 2 * stride) {
      const int64_t i2 = i + stride;
      const bool two = i2 < nv;
      float4 ga = g4[i], pa = p4[i], ma = m4[i], va = adam ? v4[i] : zero;
      float4 gb = zero, pb = zero, mb = zero, vb = zero;
      if (two) {
        gb = g4[i2];
        pb = p4[i2];
        mb = m4[i2];
        if (adam) vb = v4[i2];
      }
      upd(ga.x, pa.x, ma.x, va.x);
      upd(ga.y, pa.y, ma.y, va.y);
      upd(ga.z, pa.z, ma.z, va.z);
      upd(ga.w, pa.w, ma.w, va.w);
      g4[i] = zero;
      p4[i] = pa;
      m4[i] = ma;
      if (adam) v4[i] = va;
      if (two) {
        upd(gb.x, pb.x, mb.x, vb.x);
        upd(gb.y, pb.y, mb.y, vb.y);
        upd(gb.z, pb.z, mb.z, vb.z);
        upd(gb.w, pb.w, mb.w, vb.w);
        g4[i2] = zero;
        p4[i2] = pb;
        m4[i2] = mb;
        if (adam) v4[i2] = vb;
      }
    }
    done = nv * 4;
  }
  for (int64_t i = done + gtid; i < P; i += stride) {
    float pp = p[i], m = s1[i], vv = adam ? s2[i] : 0.f;
    const float graw = g[i];
    g[i] = 0.f;
    upd(graw, pp, m, vv);
    p[i] = pp;
    s1[i] = m;
    if (adam) s2[i] = vv;
  }
}

inline int opt_blocks(int64_t P) {
  int64_t b = (P + OPT_THREADS * 8 - 1) / (OPT_THREADS * 8);
  if (b < 1) b = 1;
  if (b > OPT_MAX_BLOCKS) b = OPT_MAX_BLOCKS;
  return (int)b;
}

}  // namespace

// The per-block fp64 partials.  Round 2's opt-in one-launch form (an in-kernel arrival barrier
// over every workgroup) measured no faster (profiles/r2zs_optim_ab.txt) and could leave a partial
// step when a workgroup was held off the GPU past its bounded wait; it was removed in round 3.
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
  const int vec = aligned && ((uintptr_t)params % 16) == 0 && ((uintptr_t)state1 % 16) == 0 &&
                  ((uintptr_t)state2 % 16) == 0;
  hipLaunchKernelGGL(grad_sumsq_kernel, dim3(blocks), dim3(OPT_THREADS), 0, rai_stream(stream),
                     grads, P, aligned, partial, state);
  RAI_LAUNCH_CHECK();
  hipLaunchKernelGGL(clip_optim_kernel, dim3(blocks), dim3(OPT_THREADS), 0, rai_stream(stream),
                     params, grads, state1, state2, P, hp, state, partial, blocks, norms,
                     max_norms, vec);
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}

int rai_internal::optim_apply_partials(float* params, float* grads, float* state1, float* state2, int64_t P,
                                       const rai_optim_hparams* hp, rai_train_state* state, const double* partial,
                                       int nparts, float* norms, int32_t max_norms, hipStream_t stream) {
  if (P < 1 || nparts < 1) return RAI_E_SHAPE;
  if (!params || !grads || !state1 || !hp || !state || !partial) return RAI_E_NULLPTR;
  if (!state2) state2 = state1;
  const int vec = ((uintptr_t)grads % 16) == 0 && ((uintptr_t)params % 16) == 0 && ((uintptr_t)state1 % 16) == 0 &&
                  ((uintptr_t)state2 % 16) == 0;
  hipLaunchKernelGGL(clip_optim_kernel, dim3(opt_blocks(P)), dim3(OPT_THREADS), 0, stream, params, grads, state1,
                     state2, P, hp, state, partial, nparts, norms, max_norms, vec);
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}
