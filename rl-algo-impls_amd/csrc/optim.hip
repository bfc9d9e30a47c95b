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
// One-launch form (clip_optim_fused_kernel, opt-in, RAI_OPTIM_FUSED=1): the
// same two reductions around an in-kernel arrival barrier, bit-identical.
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

// One-launch form (opt-in; applies when the buffers are 16-B aligned and every thread holds at most
// OPT_FUSED_K float4 of the gradient): each workgroup loads its float4s of g ONCE into registers,
// forms the same per-thread / per-block fp64 partial as grad_sumsq_kernel (same element sets, same
// summation order, same block count), publishes it write-through and arrives on two-level counters;
// once every workgroup has arrived, each re-reduces the partials exactly as clip_optim_kernel does
// and updates its register-held elements.  Results are bit-identical to the two-launch form; it saves
// a launch and the second read of g, but not time (see opt_fused_enabled).
// The barrier needs every workgroup resident: the grid is at most OPT_MAX_BLOCKS = 2 per CU, and the
// wait is bounded (state->err on expiry).  Counters are monotonic (u64, zero-filled workspace): a
// workgroup's arrival value fixes its launch's generation, so no re-arming race.
constexpr int OPT_FUSED_K = 4;
constexpr int OPT_CTR_STRIDE = 8;  // u64 counters 64 B apart: the top one, then 8 group counters
constexpr int64_t OPT_CTR_BYTES = 9 * OPT_CTR_STRIDE * 8;
constexpr int OPT_SC1 = 16;  // cache-policy operand: sc1 (write-through stores, L1-bypassing loads)
typedef unsigned int opt_u2v __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(OPT_THREADS) void clip_optim_fused_kernel(
    float* __restrict__ p, float* __restrict__ g, float* __restrict__ s1, float* __restrict__ s2,
    int64_t P, const rai_optim_hparams* __restrict__ hpp, rai_train_state* state, double* partial,
    unsigned long long* ctr, float* norms, int max_norms) {
  __shared__ double red[OPT_THREADS / 64];
  const int nb = (int)gridDim.x;
  const int64_t stride = (int64_t)nb * OPT_THREADS;
  const int64_t gtid = (int64_t)blockIdx.x * OPT_THREADS + threadIdx.x;
  const int64_t nv = P / 4;
  const float4* g4 = reinterpret_cast<const float4*>(g);
  const float4 zero = make_float4(0.f, 0.f, 0.f, 0.f);
  const int64_t old_step = state->opt_step;  // drained by block_sum's barrier, before the arrival
  float4 gv[OPT_FUSED_K];
#pragma unroll
  for (int k = 0; k < OPT_FUSED_K; ++k) {
    const int64_t i = gtid + k * stride;
    gv[k] = i < nv ? g4[i] : zero;
  }
  const int64_t it = nv * 4 + gtid;  // the scalar tail: < 4 elements, one per thread
  const float gt = it < P ? g[it] : 0.f;
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < OPT_FUSED_K; ++k)
    if (gtid + k * stride < nv) {
      const float4 x = gv[k];
      s += (double)x.x * x.x + (double)x.y * x.y + (double)x.z * x.z + (double)x.w * x.w;
    }
  if (it < P) s += (double)gt * gt;
  double v[1] = {s};
  block_sum<1>(v, red);
  __shared__ int ok;
  if (threadIdx.x == 0) {
    const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(partial, 0, nb * 8, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(opt_u2v, v[0]), prs, blockIdx.x * 8, 0, OPT_SC1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long grp = blockIdx.x & 7, gsize = (nb - grp + 7) >> 3, ngroups = nb < 8 ? nb : 8;
    const unsigned long long old =
        __hip_atomic_fetch_add(&ctr[OPT_CTR_STRIDE * (1 + grp)], 1ULL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long gen = old / gsize;
    if (old % gsize == gsize - 1)
      __hip_atomic_fetch_add(&ctr[0], 1ULL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long want = (gen + 1) * ngroups;
    const unsigned long long t0 = rai_clock();
    ok = 1;
    while (__hip_atomic_load(&ctr[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
      if (rai_expired(t0, RAI_SPIN_LOCAL)) {
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  if (!ok) {  // a workgroup never arrived: flag it, leave the parameters untouched
    if (threadIdx.x == 0) __hip_atomic_store(&state->err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  // identical fixed-order re-reduction in every block (clip_optim_kernel's order)
  const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(partial, 0, nb * 8, 0x00020000);
  double t = 0.0;
  for (int i = threadIdx.x; i < nb; i += OPT_THREADS)
    t += __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(prs, i * 8, 0, OPT_SC1));
  v[0] = t;
  block_sum<1>(v, red);
  const rai_optim_hparams hp = *hpp;
  const float total_norm = (float)sqrt(v[0]);
  float coef = 1.f;
  if (hp.max_grad_norm > 0.f) {
    coef = hp.max_grad_norm / (total_norm + 1e-6f);
    coef = fminf(coef, 1.f);
  }
  const int64_t step = old_step + 1;
  if (blockIdx.x == 0 && threadIdx.x == 0) {  // every workgroup has read old_step (it arrived)
    state->opt_step = step;
    const int ni = state->norm_index;
    if (norms && ni < max_norms) norms[ni] = total_norm;
    state->norm_index = ni + 1;
  }
  float c1, c2, c3, c4;
  if (hp.kind == 0) {
    const double bc1 = 1.0 - ipow(hp.beta1_d, step);
    const double bc2 = 1.0 - ipow(hp.beta2_d, step);
    c1 = (float)(1.0 - hp.beta1_d);
    c2 = (float)(1.0 - hp.beta2_d);
    c3 = (float)sqrt(bc2);
    c4 = (float)(-((double)hp.lr / bc1));
  } else {
    c1 = (float)(1.0 - hp.beta1_d);
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
      float sq = m * hp.alpha;
      sq = sq + (c1 * gi) * gi;
      const float avg = sqrtf(sq) + hp.eps;
      pp = pp + c2 * (gi / avg);
      m = sq;
    }
  };
  float4* p4 = reinterpret_cast<float4*>(p);
  float4* gw4 = reinterpret_cast<float4*>(g);
  float4* m4 = reinterpret_cast<float4*>(s1);
  float4* v4 = reinterpret_cast<float4*>(s2);
  float4 pv[OPT_FUSED_K], mv[OPT_FUSED_K], vv4[OPT_FUSED_K];
#pragma unroll
  for (int k = 0; k < OPT_FUSED_K; ++k) {
    const int64_t i = gtid + k * stride;
    if (i < nv) {
      pv[k] = p4[i];
      mv[k] = m4[i];
      vv4[k] = adam ? v4[i] : zero;
    }
  }
#pragma unroll
  for (int k = 0; k < OPT_FUSED_K; ++k) {
    const int64_t i = gtid + k * stride;
    if (i < nv) {
      upd(gv[k].x, pv[k].x, mv[k].x, vv4[k].x);
      upd(gv[k].y, pv[k].y, mv[k].y, vv4[k].y);
      upd(gv[k].z, pv[k].z, mv[k].z, vv4[k].z);
      upd(gv[k].w, pv[k].w, mv[k].w, vv4[k].w);
      gw4[i] = zero;
      p4[i] = pv[k];
      m4[i] = mv[k];
      if (adam) v4[i] = vv4[k];
    }
  }
  if (it < P) {
    float pp = p[it], m = s1[it], vv = adam ? s2[it] : 0.f;
    g[it] = 0.f;
    upd(gt, pp, m, vv);
    p[it] = pp;
    s1[it] = m;
    if (adam) s2[it] = vv;
  }
}

inline int opt_blocks(int64_t P) {
  int64_t b = (P + OPT_THREADS * 8 - 1) / (OPT_THREADS * 8);
  if (b < 1) b = 1;
  if (b > OPT_MAX_BLOCKS) b = OPT_MAX_BLOCKS;
  return (int)b;
}

}  // namespace

// Partials, then the fused form's arrival counters.  The workspace must be zero-filled before its
// first use and then belongs to one parameter buffer (fixed P, hence a fixed grid).
extern "C" int64_t rai_optim_workspace_bytes(int64_t /*P*/) {
  return (int64_t)OPT_MAX_BLOCKS * sizeof(double) + OPT_CTR_BYTES;
}

// RAI_OPTIM_FUSED=1 selects the one-launch form.  Off by default: measured no faster (C4: 9.93 us
// against 4.7 + 5.6 us per minibatch, whole update 42.4k vs 43.3k env-steps/s; C3 137.6k vs 138.9k,
// profiles/r2zs_optim_ab.txt): the in-kernel barrier (write-through publish, two arrival levels,
// cross-XCD polling) costs what the launch boundary it replaces did.
static bool opt_fused_enabled() {
  const char* e = getenv("RAI_OPTIM_FUSED");
  return e && e[0] == '1';
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
  const int64_t per_thread = (P / 4 + (int64_t)blocks * OPT_THREADS - 1) / ((int64_t)blocks * OPT_THREADS);
  if (vec && per_thread <= OPT_FUSED_K && opt_fused_enabled()) {
    unsigned long long* ctr = reinterpret_cast<unsigned long long*>(
        reinterpret_cast<char*>(workspace) + (int64_t)OPT_MAX_BLOCKS * sizeof(double));
    hipLaunchKernelGGL(clip_optim_fused_kernel, dim3(blocks), dim3(OPT_THREADS), 0, rai_stream(stream), params,
                       grads, state1, state2, P, hp, state, partial, ctr, norms, max_norms);
    RAI_LAUNCH_CHECK();
    return RAI_OK;
  }
  hipLaunchKernelGGL(grad_sumsq_kernel, dim3(blocks), dim3(OPT_THREADS), 0, rai_stream(stream),
                     grads, P, aligned, partial, state);
  RAI_LAUNCH_CHECK();
  hipLaunchKernelGGL(clip_optim_kernel, dim3(blocks), dim3(OPT_THREADS), 0, rai_stream(stream),
                     params, grads, state1, state2, P, hp, state, partial, blocks, norms,
                     max_norms, vec);
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}
