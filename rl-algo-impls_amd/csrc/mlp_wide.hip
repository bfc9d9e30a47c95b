// Fused minibatch step for wide MLP actor-critics on gfx950 (HalfCheetah-class policies:
// separate [in -> H -> H -> out] actor and critic, H up to 256, Gaussian or Categorical head).
//
// Replaces, per minibatch of rl_algo_impls/ppo/ppo.py:290-377, the PyTorch-ROCm forward of
// rl_algo_impls/shared/policy/actor_critic_network/connected_trio.py (+ shared/actor/gaussian.py,
// categorical.py, shared/policy/critic.py) and its autograd backward, which at B = 64 rows is ~90
// small launches (hipBLASLt GEMMs picked for large tiles, ~75 elementwise kernels) per minibatch.
// Here it is five launches (each a graph node of the replayed minibatch step, graphs.py):
//
//   rai_mlp_wide_fwd1   grid (S, 2): H1[:, slice s] = act(X W1[slice]^T + b1)            (per net)
//   rai_mlp_wide_fwd2   grid (S, 2): H2[:, slice s] = act(H1 W2[slice]^T + b2), and the output
//                       layer's partial sums over the slice P[s] = H2[:, s] W3[:, s]^T
//   rai_mlp_wide_head   sum the S partials in slice order (+ b3): mu / logits and v; the head's
//                       log-prob and entropy (Normal: gaussian.py:11-16; Categorical) -> the loss
//   (rai_ppo_loss: clipped surrogate / value / entropy loss, unchanged)
//   rai_mlp_wide_bwd2   grid (S, 2): dOut from (d_logp, d_entropy, d_v); dZ2[:, s] =
//                       (dOut W3[:, s]) * act'(H2); dW3[:, s], db3, dW2[s, :], db2[s], dlog_std
//   rai_mlp_wide_bwd1   grid (S, 2): dZ1[:, s] = (dZ2 W2[:, s]) * act'(H1); dW1[s, :], db1[s]
//
// S = H / 16 column slices of 16 hidden units; every workgroup owns one (slice, network), so the
// dependent chain of a minibatch is these kernel boundaries and nothing else (no inter-workgroup
// protocol).  Weights are read through L2 (a 256-wide net is 280 KB; one slice of W2 is 16 KB).
// Activations live in the caller's workspace between launches (B x H per layer and network).
// Gradients are written into the flat gradient buffer views (or added, desc.accumulate, for
// gradient accumulation); rai_clip_optim_step then runs clip_grad_norm_ + Adam as before.
// All sums run in a fixed order: deterministic; fp32 like the reference (different association
// than hipBLASLt's, so parity is to fp32 tolerance, tests/test_gpu_trainer.py).
#include "common.h"

namespace {

constexpr int WT = 256;   // threads per workgroup
constexpr int SL = 16;    // hidden units per slice
constexpr int OUTM = RAI_WIDE_MAX_OUT;
constexpr int KC = 64;    // k-chunk staged through LDS

__device__ __forceinline__ float act_f(int act, float z) { return act ? fmaxf(z, 0.f) : tanhf(z); }
// derivative from the activation's OUTPUT h: relu: h > 0; tanh: 1 - h^2
__device__ __forceinline__ float act_d(int act, float h) { return act ? (h > 0.f ? 1.f : 0.f) : (1.f - h * h); }

struct WideWs {  // workspace layout (floats), per net n: offsets into ws
  float* H1;
  float* H2;
  float* P;    // [S][B][OUTM]
  float* OUT;  // [B][OUTM]
  float* DZ2;  // [B][H]
};
__device__ __host__ __forceinline__ int64_t wide_ws_net_floats(int64_t B, int H) {
  return 3 * B * H + (int64_t)(H / SL) * B * OUTM + B * OUTM;
}
__device__ __forceinline__ WideWs ws_of(float* ws, int n, int64_t B, int H) {
  float* base = ws + n * wide_ws_net_floats(B, H);
  WideWs w;
  w.H1 = base;
  w.H2 = base + B * H;
  w.DZ2 = base + 2 * B * H;
  w.P = base + 3 * B * H;
  w.OUT = w.P + (int64_t)(H / SL) * B * OUTM;
  return w;
}

struct WideArgs {
  rai_mlp_wide_desc d;
  const float* obs;       // (B, in)
  const void* actions;    // Gaussian: (B, out_pi) f32; Categorical: (B,) int64
  const float* d_logp;    // (B)
  const float* d_ent;     // (B*out_pi) Gaussian, (B) Categorical
  const float* d_v;       // (B)
  float* logp;            // (B)
  float* ent;             // (B*out_pi) Gaussian, (B) Categorical
  float* v;               // (B)
  float* ws;
  int32_t B;
};

__device__ __forceinline__ int out_dim(const rai_mlp_wide_desc& d, int n) { return n == 0 ? d.out_pi : 1; }

__device__ __forceinline__ void put(float* g, int64_t i, float val, int accumulate) {
  if (accumulate) g[i] += val;
  else g[i] = val;
}

// ---- layer 1 forward: H1[:, slice] ------------------------------------------------------------
__global__ __launch_bounds__(WT) void wide_fwd1_kernel(const WideArgs a) {
  __shared__ float w1s[SL][RAI_WIDE_MAX_IN + 1];
  __shared__ float b1s[SL];
  const int s = blockIdx.x, n = blockIdx.y, t = threadIdx.x;
  const rai_mlp_wide_desc& d = a.d;
  const int H = d.hidden, IN = d.in_dim, B = a.B;
  const float* W1 = d.w[n][0];
  for (int i = t; i < SL * IN; i += WT) w1s[i / IN][i % IN] = W1[(int64_t)(s * SL + i / IN) * IN + i % IN];
  if (t < SL) b1s[t] = d.w[n][1][s * SL + t];
  __syncthreads();
  const WideWs w = ws_of(a.ws, n, B, H);
  const int j = t % SL;
  for (int b = t / SL; b < B; b += WT / SL) {
    const float* x = a.obs + (int64_t)b * IN;
    float acc = 0.f;
    for (int i = 0; i < IN; ++i) acc += x[i] * w1s[j][i];
    w.H1[(int64_t)b * H + s * SL + j] = act_f(d.activation, acc + b1s[j]);
  }
}

// ---- layer 2 forward + output-layer partials ---------------------------------------------------
__global__ __launch_bounds__(WT) void wide_fwd2_kernel(const WideArgs a) {
  __shared__ float w2s[SL][KC + 4];
  __shared__ float hs[RAI_WIDE_MAX_B][KC + 4];  // H1 rows, one k-chunk
  __shared__ float h2s[RAI_WIDE_MAX_B][SL + 1];
  const int s = blockIdx.x, n = blockIdx.y, t = threadIdx.x;
  const rai_mlp_wide_desc& d = a.d;
  const int H = d.hidden, B = a.B, O = out_dim(d, n);
  const WideWs w = ws_of(a.ws, n, B, H);
  const float* W2 = d.w[n][2];
  const int j = t % SL, r0 = t / SL;  // rows r0, r0 + 16, ...
  constexpr int RMAX = RAI_WIDE_MAX_B / (WT / SL);
  float acc[RMAX];
#pragma unroll
  for (int q = 0; q < RMAX; ++q) acc[q] = 0.f;
  for (int k0 = 0; k0 < H; k0 += KC) {
    __syncthreads();
    for (int i = t; i < SL * KC; i += WT) w2s[i / KC][i % KC] = W2[(int64_t)(s * SL + i / KC) * H + k0 + i % KC];
    for (int i = t; i < B * KC; i += WT) hs[i / KC][i % KC] = w.H1[(int64_t)(i / KC) * H + k0 + i % KC];
    __syncthreads();
#pragma unroll
    for (int q = 0; q < RMAX; ++q) {
      const int b = r0 + q * (WT / SL);
      if (b < B) {
        float sacc = acc[q];
        for (int k = 0; k < KC; ++k) sacc += hs[b][k] * w2s[j][k];
        acc[q] = sacc;
      }
    }
  }
  const float bj = d.w[n][3][s * SL + j];
#pragma unroll
  for (int q = 0; q < RMAX; ++q) {
    const int b = r0 + q * (WT / SL);
    if (b < B) {
      const float h = act_f(d.activation, acc[q] + bj);
      h2s[b][j] = h;
      w.H2[(int64_t)b * H + s * SL + j] = h;
    }
  }
  __syncthreads();
  const float* W3 = d.w[n][4];
  for (int i = t; i < B * O; i += WT) {
    const int b = i / O, o = i % O;
    float p = 0.f;
#pragma unroll
    for (int jj = 0; jj < SL; ++jj) p += h2s[b][jj] * W3[(int64_t)o * H + s * SL + jj];
    w.P[((int64_t)s * B + b) * OUTM + o] = p;
  }
}

// ---- head: outputs, log-prob, entropy, value --------------------------------------------------
__global__ __launch_bounds__(WT) void wide_head_kernel(const WideArgs a) {
  const rai_mlp_wide_desc& d = a.d;
  const int H = d.hidden, B = a.B, S = H / SL, A = d.out_pi;
  const WideWs wp = ws_of(a.ws, 0, B, H), wv = ws_of(a.ws, 1, B, H);
  for (int b = blockIdx.x * WT + threadIdx.x; b < B; b += gridDim.x * WT) {
    float out[OUTM];
    for (int o = 0; o < A; ++o) {
      float acc = 0.f;
      for (int s = 0; s < S; ++s) acc += wp.P[((int64_t)s * B + b) * OUTM + o];
      out[o] = acc + d.w[0][5][o];
      wp.OUT[(int64_t)b * OUTM + o] = out[o];
    }
    float v = 0.f;
    for (int s = 0; s < S; ++s) v += wv.P[((int64_t)s * B + b) * OUTM];
    v += d.w[1][5][0];
    wv.OUT[(int64_t)b * OUTM] = v;
    a.v[b] = v;
    if (d.head == 1) {  // Normal(mu, exp(log_std)): torch.distributions.Normal.log_prob / entropy
      const float* act = static_cast<const float*>(a.actions) + (int64_t)b * A;
      float lp = 0.f;
      for (int o = 0; o < A; ++o) {
        const float scale = expf(d.log_std[o]);
        const float var = scale * scale;
        const float log_scale = logf(scale);
        const float x = act[o] - out[o];
        lp += -(x * x) / (2.f * var) - log_scale - 0.91893853320467274f;  // log(sqrt(2*pi))
        a.ent[(int64_t)b * A + o] = 1.4189385332046727f + log_scale;  // (0.5 + 0.5*log(2*pi)) + log(scale)
      }
      a.logp[b] = lp;
    } else {  // Categorical(logits)
      const int64_t ai = static_cast<const int64_t*>(a.actions)[b];
      float mx = out[0];
      for (int o = 1; o < A; ++o) mx = fmaxf(mx, out[o]);
      float se = 0.f;
      for (int o = 0; o < A; ++o) se += expf(out[o] - mx);
      const float lse = mx + logf(se);
      float h = 0.f;
      for (int o = 0; o < A; ++o) {
        const float l = out[o] - lse;
        h -= fmaxf(l, -3.4028234663852886e38f) * expf(l);
      }
      a.logp[b] = out[ai >= 0 && ai < A ? ai : 0] - lse;
      a.ent[b] = h;
    }
  }
}

// dLoss/dOut for row b of network n (recomputed by every workgroup that needs it)
__device__ __forceinline__ void d_out_row(const WideArgs& a, const WideWs& w, int n, int b, float* dout) {
  const rai_mlp_wide_desc& d = a.d;
  const int A = d.out_pi;
  if (n == 1) {
    dout[0] = a.d_v[b];
    return;
  }
  const float* out = w.OUT + (int64_t)b * OUTM;
  if (d.head == 1) {
    const float* act = static_cast<const float*>(a.actions) + (int64_t)b * A;
    for (int o = 0; o < A; ++o) {
      const float scale = expf(d.log_std[o]);
      dout[o] = a.d_logp[b] * ((act[o] - out[o]) / (scale * scale));
    }
  } else {
    const int64_t ai = static_cast<const int64_t*>(a.actions)[b];
    float mx = out[0];
    for (int o = 1; o < A; ++o) mx = fmaxf(mx, out[o]);
    float se = 0.f;
    for (int o = 0; o < A; ++o) se += expf(out[o] - mx);
    const float lse = mx + logf(se);
    float h = 0.f;
    for (int o = 0; o < A; ++o) {
      const float l = out[o] - lse;
      h -= l * expf(l);
    }
    const float gl = a.d_logp[b], ge = a.d_ent[b];
    for (int o = 0; o < A; ++o) {
      const float l = out[o] - lse, p = expf(l);
      dout[o] = gl * ((o == ai ? 1.f : 0.f) - p) - ge * p * (l + h);
    }
  }
}

// ---- backward through layers 3 and 2 ---------------------------------------------------------
__global__ __launch_bounds__(WT) void wide_bwd2_kernel(const WideArgs a) {
  __shared__ float douts[RAI_WIDE_MAX_B][OUTM];
  __shared__ float dz2s[RAI_WIDE_MAX_B][SL];
  __shared__ float w3s[OUTM][SL];
  const int s = blockIdx.x, n = blockIdx.y, t = threadIdx.x;
  const rai_mlp_wide_desc& d = a.d;
  const int H = d.hidden, B = a.B, O = out_dim(d, n), acc_mode = d.accumulate;
  const WideWs w = ws_of(a.ws, n, B, H);
  for (int b = t; b < B; b += WT) {
    float dout[OUTM];
    d_out_row(a, w, n, b, dout);
    for (int o = 0; o < O; ++o) douts[b][o] = dout[o];
  }
  for (int i = t; i < O * SL; i += WT) w3s[i / SL][i % SL] = d.w[n][4][(int64_t)(i / SL) * H + s * SL + i % SL];
  __syncthreads();
  // dZ2 slice
  for (int i = t; i < B * SL; i += WT) {
    const int b = i / SL, j = i % SL;
    float dh = 0.f;
    for (int o = 0; o < O; ++o) dh += douts[b][o] * w3s[o][j];
    const float h2 = w.H2[(int64_t)b * H + s * SL + j];
    const float dz = dh * act_d(d.activation, h2);
    dz2s[b][j] = dz;
    w.DZ2[(int64_t)b * H + s * SL + j] = dz;
  }
  __syncthreads();
  // dW3[:, slice] = dOut^T H2[:, slice]; db3 (slice 0)
  for (int i = t; i < O * SL; i += WT) {
    const int o = i / SL, j = i % SL;
    float g = 0.f;
    for (int b = 0; b < B; ++b) g += douts[b][o] * w.H2[(int64_t)b * H + s * SL + j];
    put(d.g[n][4], (int64_t)o * H + s * SL + j, g, acc_mode);
  }
  if (s == 0 && t < O) {
    float g = 0.f;
    for (int b = 0; b < B; ++b) g += douts[b][t];
    put(d.g[n][5], t, g, acc_mode);
  }
  // db2[slice]
  if (t < SL) {
    float g = 0.f;
    for (int b = 0; b < B; ++b) g += dz2s[b][t];
    put(d.g[n][3], s * SL + t, g, acc_mode);
  }
  // dW2[slice, :] = dZ2[:, slice]^T H1: thread k owns column k of every row in the slice
  for (int k = t; k < H; k += WT) {
    float g[SL];
#pragma unroll
    for (int j = 0; j < SL; ++j) g[j] = 0.f;
    for (int b = 0; b < B; ++b) {
      const float h1 = w.H1[(int64_t)b * H + k];
#pragma unroll
      for (int j = 0; j < SL; ++j) g[j] += dz2s[b][j] * h1;
    }
#pragma unroll
    for (int j = 0; j < SL; ++j) put(d.g[n][2], (int64_t)(s * SL + j) * H + k, g[j], acc_mode);
  }
  // dlog_std (Gaussian actor): sum_b d_logp * ((a - mu)^2 / var - 1) + d_entropy
  if (n == 0 && s == 0 && d.head == 1 && t < d.out_pi) {
    const int A = d.out_pi, o = t;
    const float scale = expf(d.log_std[o]);
    const float var = scale * scale;
    float g = 0.f;
    for (int b = 0; b < B; ++b) {
      const float x = static_cast<const float*>(a.actions)[(int64_t)b * A + o] - w.OUT[(int64_t)b * OUTM + o];
      g += a.d_logp[b] * ((x * x) / var - 1.f) + a.d_ent[(int64_t)b * A + o];
    }
    put(d.g_log_std, o, g, acc_mode);
  }
}

// ---- backward through layer 1 ----------------------------------------------------------------
__global__ __launch_bounds__(WT) void wide_bwd1_kernel(const WideArgs a) {
  __shared__ float w2s[KC][SL + 1];               // W2[k-chunk, slice]
  __shared__ float zs[RAI_WIDE_MAX_B][KC + 4];     // dZ2 rows, one k-chunk
  __shared__ float dz1s[RAI_WIDE_MAX_B][SL + 1];
  const int s = blockIdx.x, n = blockIdx.y, t = threadIdx.x;
  const rai_mlp_wide_desc& d = a.d;
  const int H = d.hidden, B = a.B, IN = d.in_dim, acc_mode = d.accumulate;
  const WideWs w = ws_of(a.ws, n, B, H);
  const float* W2 = d.w[n][2];
  const int j = t % SL, r0 = t / SL;
  constexpr int RMAX = RAI_WIDE_MAX_B / (WT / SL);
  float acc[RMAX];
#pragma unroll
  for (int q = 0; q < RMAX; ++q) acc[q] = 0.f;
  for (int k0 = 0; k0 < H; k0 += KC) {
    __syncthreads();
    for (int i = t; i < KC * SL; i += WT) w2s[i / SL][i % SL] = W2[(int64_t)(k0 + i / SL) * H + s * SL + i % SL];
    for (int i = t; i < B * KC; i += WT) zs[i / KC][i % KC] = w.DZ2[(int64_t)(i / KC) * H + k0 + i % KC];
    __syncthreads();
#pragma unroll
    for (int q = 0; q < RMAX; ++q) {
      const int b = r0 + q * (WT / SL);
      if (b < B) {
        float sacc = acc[q];
        for (int k = 0; k < KC; ++k) sacc += zs[b][k] * w2s[k][j];
        acc[q] = sacc;
      }
    }
  }
#pragma unroll
  for (int q = 0; q < RMAX; ++q) {
    const int b = r0 + q * (WT / SL);
    if (b < B) dz1s[b][j] = acc[q] * act_d(d.activation, w.H1[(int64_t)b * H + s * SL + j]);
  }
  __syncthreads();
  if (t < SL) {
    float g = 0.f;
    for (int b = 0; b < B; ++b) g += dz1s[b][t];
    put(d.g[n][1], s * SL + t, g, acc_mode);
  }
  for (int i = t; i < SL * IN; i += WT) {
    const int jj = i / IN, c = i % IN;
    float g = 0.f;
    for (int b = 0; b < B; ++b) g += dz1s[b][jj] * a.obs[(int64_t)b * IN + c];
    put(d.g[n][0], (int64_t)(s * SL + jj) * IN + c, g, acc_mode);
  }
}

int check(const rai_mlp_wide_desc* d, int64_t B, const float* obs, const void* ws, int64_t ws_bytes) {
  if (!d || !obs || !ws) return RAI_E_NULLPTR;
  if (B < 1 || B > RAI_WIDE_MAX_B) return RAI_E_SHAPE;
  if (d->hidden < SL || d->hidden > RAI_WIDE_MAX_H || d->hidden % 64 != 0) return RAI_E_UNSUPPORTED;
  if (d->in_dim < 1 || d->in_dim > RAI_WIDE_MAX_IN) return RAI_E_UNSUPPORTED;
  if (d->out_pi < 1 || d->out_pi > RAI_WIDE_MAX_OUT) return RAI_E_UNSUPPORTED;
  if (d->head != 0 && d->head != 1) return RAI_E_MODE;
  if (d->head == 1 && !d->log_std) return RAI_E_NULLPTR;
  for (int n = 0; n < 2; ++n)
    for (int i = 0; i < 6; ++i)
      if (!d->w[n][i]) return RAI_E_NULLPTR;
  if (ws_bytes < rai_mlp_wide_workspace_bytes(B, d->hidden)) return RAI_E_WORKSPACE;
  return RAI_OK;
}

WideArgs make_args(const rai_mlp_wide_desc* d, const float* obs, int64_t B, void* ws) {
  WideArgs a{};
  a.d = *d;
  a.obs = obs;
  a.B = (int32_t)B;
  a.ws = static_cast<float*>(ws);
  return a;
}

}  // namespace

extern "C" int64_t rai_mlp_wide_workspace_bytes(int64_t B, int32_t hidden) {
  return 2 * wide_ws_net_floats(B, hidden) * (int64_t)sizeof(float);
}

extern "C" int rai_mlp_wide_forward(const rai_mlp_wide_desc* desc, const float* obs, const void* actions, int64_t B,
                                    float* logp_out, float* entropy_out, float* v_out, void* workspace,
                                    int64_t workspace_bytes, void* stream) {
  int rc = check(desc, B, obs, workspace, workspace_bytes);
  if (rc != RAI_OK) return rc;
  if (!actions || !logp_out || !entropy_out || !v_out) return RAI_E_NULLPTR;
  WideArgs a = make_args(desc, obs, B, workspace);
  a.actions = actions;
  a.logp = logp_out;
  a.ent = entropy_out;
  a.v = v_out;
  const dim3 grid(desc->hidden / SL, 2);
  hipStream_t st = rai_stream(stream);
  hipLaunchKernelGGL(wide_fwd1_kernel, grid, dim3(WT), 0, st, a);
  RAI_LAUNCH_CHECK();
  hipLaunchKernelGGL(wide_fwd2_kernel, grid, dim3(WT), 0, st, a);
  RAI_LAUNCH_CHECK();
  hipLaunchKernelGGL(wide_head_kernel, dim3(1), dim3(WT), 0, st, a);
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}

extern "C" int rai_mlp_wide_backward(const rai_mlp_wide_desc* desc, const float* obs, const void* actions, int64_t B,
                                     const float* d_logp, const float* d_entropy, const float* d_v, void* workspace,
                                     int64_t workspace_bytes, void* stream) {
  int rc = check(desc, B, obs, workspace, workspace_bytes);
  if (rc != RAI_OK) return rc;
  if (!actions || !d_logp || !d_entropy || !d_v) return RAI_E_NULLPTR;
  for (int n = 0; n < 2; ++n)
    for (int i = 0; i < 6; ++i)
      if (!desc->g[n][i]) return RAI_E_NULLPTR;
  if (desc->head == 1 && !desc->g_log_std) return RAI_E_NULLPTR;
  WideArgs a = make_args(desc, obs, B, workspace);
  a.actions = actions;
  a.d_logp = d_logp;
  a.d_ent = d_entropy;
  a.d_v = d_v;
  const dim3 grid(desc->hidden / SL, 2);
  hipStream_t st = rai_stream(stream);
  hipLaunchKernelGGL(wide_bwd2_kernel, grid, dim3(WT), 0, st, a);
  RAI_LAUNCH_CHECK();
  hipLaunchKernelGGL(wide_bwd1_kernel, grid, dim3(WT), 0, st, a);
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}
