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

// Every operand a workgroup reuses is staged into LDS first with coalesced (float4 where the rows
// allow) loads; the arithmetic then runs out of LDS / registers only.  Rows are processed in chunks
// of RC = 64 (one chunk at the usual B = 64).
constexpr int RC = 64;
constexpr int HP = RAI_WIDE_MAX_H + 4;  // padded LDS row (floats) for H-long rows
constexpr int RPT = RC / (WT / SL);     // rows per thread in the (16 columns x 64 rows) tiles = 4

typedef float f4 __attribute__((ext_vector_type(4)));

// Cooperative copies into LDS.  Loads are issued in batches of U per thread before any LDS store,
// so a workgroup pays a few global round trips per staged tile, not one per element (a plain
// load -> ds_write loop waits on every load).
template <int U>
__device__ __forceinline__ void stage1(float* dst, int dst_ld, const float* src, int64_t src_ld, int rows, int cols) {
  const int total = rows * cols;
  for (int base = threadIdx.x; base < total; base += WT * U) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = base + u * WT;
      if (i < total) {
        const int r = i / cols, c = i - r * cols;
        v[u] = src[r * src_ld + c];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = base + u * WT;
      if (i < total) {
        const int r = i / cols, c = i - r * cols;
        dst[r * dst_ld + c] = v[u];
      }
    }
  }
}
// 16-B loads when the source rows are 16-B aligned (parameter views inside the flat buffer need not
// be), else the 4-B path
__device__ __forceinline__ void stage4(float* dst, int dst_ld, const float* src, int64_t src_ld, int rows, int cols) {
  if (((reinterpret_cast<uintptr_t>(src) & 15) != 0) || (src_ld & 3) || (cols & 3) || (dst_ld & 3)) {
    stage1<16>(dst, dst_ld, src, src_ld, rows, cols);
    return;
  }
  constexpr int U = 8;
  const int c4 = cols >> 2, total = rows * c4;
  for (int base = threadIdx.x; base < total; base += WT * U) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = base + u * WT;
      if (i < total) {
        const int r = i / c4, c = (i - r * c4) << 2;
        v[u] = *reinterpret_cast<const f4*>(src + r * src_ld + c);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = base + u * WT;
      if (i < total) {
        const int r = i / c4, c = (i - r * c4) << 2;
        *reinterpret_cast<f4*>(dst + r * dst_ld + c) = v[u];
      }
    }
  }
}

// One wave's 16-row x 16-column tile of  Rows[16w .. 16w+16) (LDS, ld HP) x Cols^T  over k in [0, H),
// with Cols[j][k] in LDS (ld HP): v_mfma_f32_16x16x4f32 (exact fp32 products, fp32 accumulation).
// Lane (li = lane & 15, g = lane >> 4) feeds A = Rows[li][k], B = Cols[li][k] for k in the lane
// group's contiguous quarter [g*H/4, (g+1)*H/4) (16-B LDS reads of 4 consecutive k); the result
// element r of the lane is row 4g + r, column li of the tile.  Two accumulators halve the chain.
__device__ __forceinline__ f4 tile_dot(const float* rows, const float* cols, int H, int lane) {
  const int li = lane & 15, g = lane >> 4, KQ = H >> 2;
  const float* ra = rows + li * HP + g * KQ;
  const float* cb = cols + li * HP + g * KQ;
  f4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  for (int kk = 0; kk < KQ; kk += 4) {
    const f4 av = *reinterpret_cast<const f4*>(ra + kk);
    const f4 bv = *reinterpret_cast<const f4*>(cb + kk);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, bv.x, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, bv.y, acc1, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.z, bv.z, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.w, bv.w, acc1, 0, 0, 0);
  }
  return acc0 + acc1;
}

// ---- layer 1 forward: H1[:, slice] ------------------------------------------------------------
__global__ __launch_bounds__(WT) void wide_fwd1_kernel(const WideArgs a) {
  __shared__ float w1s[SL][RAI_WIDE_MAX_IN + 1];
  __shared__ float xs[RC][RAI_WIDE_MAX_IN + 1];
  __shared__ float b1s[SL];
  const int s = blockIdx.x, n = blockIdx.y, t = threadIdx.x;
  const rai_mlp_wide_desc& d = a.d;
  const int H = d.hidden, IN = d.in_dim, B = a.B;
  stage1<16>(&w1s[0][0], RAI_WIDE_MAX_IN + 1, d.w[n][0] + (int64_t)s * SL * IN, IN, SL, IN);
  if (t < SL) b1s[t] = d.w[n][1][s * SL + t];
  const WideWs w = ws_of(a.ws, n, B, H);
  const int j = t % SL, r0 = t / SL;
  for (int c0 = blockIdx.z * RC; c0 < B; c0 += RC * gridDim.z) {  // row chunks over grid.z
    const int nr = min(RC, B - c0);
    __syncthreads();
    stage1<16>(&xs[0][0], RAI_WIDE_MAX_IN + 1, a.obs + (int64_t)c0 * IN, IN, nr, IN);
    __syncthreads();
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      const int b = r0 + q * (WT / SL);
      if (b < nr) {
        float acc = 0.f;
        for (int i = 0; i < IN; ++i) acc += xs[b][i] * w1s[j][i];
        w.H1[(int64_t)(c0 + b) * H + s * SL + j] = act_f(d.activation, acc + b1s[j]);
      }
    }
  }
}

// ---- layer 2 forward + output-layer partials ---------------------------------------------------
__global__ __launch_bounds__(WT) void wide_fwd2_kernel(const WideArgs a) {
  __shared__ float w2s[SL][HP];    // W2[slice, :]
  __shared__ float hs[RC][HP];     // H1 rows of the chunk
  __shared__ float h2s[RC][SL + 1];
  __shared__ float w3s[OUTM][SL];
  const int s = blockIdx.x, n = blockIdx.y, t = threadIdx.x;
  const rai_mlp_wide_desc& d = a.d;
  const int H = d.hidden, B = a.B, O = out_dim(d, n);
  const WideWs w = ws_of(a.ws, n, B, H);
  stage4(&w2s[0][0], HP, d.w[n][2] + (int64_t)s * SL * H, H, SL, H);
  for (int i = t; i < O * SL; i += WT) w3s[i / SL][i % SL] = d.w[n][4][(int64_t)(i / SL) * H + s * SL + i % SL];
  for (int c0 = blockIdx.z * RC; c0 < B; c0 += RC * gridDim.z) {  // row chunks over grid.z
    const int nr = min(RC, B - c0);
    __syncthreads();
    stage4(&hs[0][0], HP, w.H1 + (int64_t)c0 * H, H, nr, H);
    __syncthreads();
    {  // wave w: rows [16w, 16w + 16) of the chunk (the tile's rows >= nr are computed and dropped)
      const int wv = t >> 6, lane = t & 63;
      const f4 z = tile_dot(&hs[16 * wv][0], &w2s[0][0], H, lane);
      const int jj = lane & 15, g = lane >> 4;
      const float bjj = d.w[n][3][s * SL + jj];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int b = 16 * wv + 4 * g + r;
        if (b < nr) {
          const float h = act_f(d.activation, z[r] + bjj);
          h2s[b][jj] = h;
          w.H2[(int64_t)(c0 + b) * H + s * SL + jj] = h;
        }
      }
    }
    __syncthreads();
    for (int i = t; i < nr * O; i += WT) {
      const int b = i / O, o = i - b * O;
      float p = 0.f;
#pragma unroll
      for (int jj = 0; jj < SL; ++jj) p += h2s[b][jj] * w3s[o][jj];
      w.P[((int64_t)s * B + c0 + b) * OUTM + o] = p;
    }
  }
}

// ---- head: outputs, log-prob, entropy, value --------------------------------------------------
__device__ __forceinline__ void wide_head_body(const WideArgs& a) {
  __shared__ float outs[RAI_WIDE_MAX_B][OUTM + 1];
  const rai_mlp_wide_desc& d = a.d;
  const int H = d.hidden, B = a.B, S = H / SL, A = d.out_pi, t = threadIdx.x;
  constexpr int SMAX = RAI_WIDE_MAX_H / SL;
  const WideWs wp = ws_of(a.ws, 0, B, H), wv = ws_of(a.ws, 1, B, H);
  // (1) every (row, output) sums its S slice partials in slice order (loads issued together)
  const int per = A + 1;  // actor outputs, then the critic's value
  for (int i = t; i < B * per; i += WT) {
    const int b = i / per, o = i - b * per;
    const bool critic = o == A;
    const float* P = critic ? wv.P : wp.P;
    const int oo = critic ? 0 : o;
    float part[SMAX];
#pragma unroll
    for (int q = 0; q < SMAX; ++q) part[q] = q < S ? P[((int64_t)q * B + b) * OUTM + oo] : 0.f;
    float acc = 0.f;
#pragma unroll
    for (int q = 0; q < SMAX; ++q)
      if (q < S) acc += part[q];
    const float val = acc + (critic ? d.w[1][5][0] : d.w[0][5][o]);
    outs[b][o] = val;
    (critic ? wv.OUT : wp.OUT)[(int64_t)b * OUTM + oo] = val;
  }
  __syncthreads();
  // (2) one row per thread: the head's log-prob / entropy, and v
  for (int b = t; b < B; b += WT) {
    a.v[b] = outs[b][A];
    if (d.head == 1) {  // Normal(mu, exp(log_std)): torch.distributions.Normal.log_prob / entropy
      const float* act = static_cast<const float*>(a.actions) + (int64_t)b * A;
      float lp = 0.f;
      for (int o = 0; o < A; ++o) {
        const float scale = expf(d.log_std[o]);
        const float var = scale * scale;
        const float log_scale = logf(scale);
        const float x = act[o] - outs[b][o];
        lp += -(x * x) / (2.f * var) - log_scale - 0.91893853320467274f;  // log(sqrt(2*pi))
        a.ent[(int64_t)b * A + o] = 1.4189385332046727f + log_scale;     // (0.5 + 0.5*log(2*pi)) + log(scale)
      }
      a.logp[b] = lp;
    } else {  // Categorical(logits)
      const int64_t ai = static_cast<const int64_t*>(a.actions)[b];
      float mx = outs[b][0];
      for (int o = 1; o < A; ++o) mx = fmaxf(mx, outs[b][o]);
      float se = 0.f;
      for (int o = 0; o < A; ++o) se += expf(outs[b][o] - mx);
      const float lse = mx + logf(se);
      float h = 0.f;
      for (int o = 0; o < A; ++o) {
        const float l = outs[b][o] - lse;
        h -= fmaxf(l, -3.4028234663852886e38f) * expf(l);
      }
      a.logp[b] = outs[b][ai >= 0 && ai < A ? ai : 0] - lse;
      a.ent[b] = h;
    }
  }
}

__global__ __launch_bounds__(WT) void wide_head_kernel(const WideArgs a) { wide_head_body(a); }

// Rollout head: the actor's distribution parameters (Gaussian mean or Categorical logits, (B, out)
// contiguous) and the critic's value, the slice partials summed in slice order as wide_head_body;
// one thread per (row, output), no log-prob (the sampler draws the action from these).
__global__ __launch_bounds__(WT) void wide_head_params_kernel(const WideArgs a, float* params_out) {
  const rai_mlp_wide_desc& d = a.d;
  const int H = d.hidden, B = a.B, S = H / SL, A = d.out_pi;
  const WideWs wp = ws_of(a.ws, 0, B, H), wv = ws_of(a.ws, 1, B, H);
  const int per = A + 1;
  for (int i = blockIdx.x * WT + threadIdx.x; i < B * per; i += gridDim.x * WT) {
    const int b = i / per, o = i - b * per;
    const bool critic = o == A;
    const float* P = critic ? wv.P : wp.P;
    const int oo = critic ? 0 : o;
    float acc = 0.f;
    for (int q = 0; q < S; ++q) acc += P[((int64_t)q * B + b) * OUTM + oo];
    const float val = acc + (critic ? d.w[1][5][0] : d.w[0][5][o]);
    if (critic) a.v[b] = val;
    else params_out[(int64_t)b * A + o] = val;
  }
}

#include "loss_body.h"

// Head + PPO loss in one workgroup: the head's logp / entropy / v rows go to global memory and,
// after the workgroup barrier (workgroup-scope visibility of the block's own global stores), the
// loss body reads them back with the same code and order as rai_ppo_loss.  One launch fewer on
// the minibatch chain.
__global__ __launch_bounds__(WT) void wide_head_loss_kernel(const WideArgs a, const LossArgs la) {
  wide_head_body(a);
  __syncthreads();
  pg_loss_body<1>(la);
}

// dLoss/dOut for row b of network n (recomputed by every workgroup that needs it); for the Gaussian
// actor also the row's dLoss/dlog_std terms.  (Staging these operands through LDS first measured
// slower: the per-row loads of different threads already overlap.)
__device__ __forceinline__ void d_out_row(const WideArgs& a, const WideWs& w, int n, int b, float* dout,
                                          float* dls) {
  const rai_mlp_wide_desc& d = a.d;
  const int A = d.out_pi;
  if (n == 1) {
    dout[0] = a.d_v[b];
    return;
  }
  const float* out = w.OUT + (int64_t)b * OUTM;
  if (d.head == 1) {
    const float* act = static_cast<const float*>(a.actions) + (int64_t)b * A;
    const float gl = a.d_logp[b];
    for (int o = 0; o < A; ++o) {
      const float scale = expf(d.log_std[o]);
      const float var = scale * scale;
      const float x = act[o] - out[o];
      dout[o] = gl * (x / var);
      dls[o] = gl * ((x * x) / var - 1.f) + a.d_ent[(int64_t)b * A + o];
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
  __shared__ float dlss[RAI_WIDE_MAX_B][OUTM];
  __shared__ float hs[RC][HP];        // H1 rows of the chunk
  __shared__ float h2s[RC][SL + 1];   // H2[:, slice] rows of the chunk
  __shared__ float dz2s[RC][SL];
  __shared__ float w3s[OUTM][SL];
  const int s = blockIdx.x, n = blockIdx.y, t = threadIdx.x;
  const rai_mlp_wide_desc& d = a.d;
  const int H = d.hidden, B = a.B, O = out_dim(d, n), acc_mode = d.accumulate;
  const bool do_ls = n == 0 && s == 0 && d.head == 1;
  const WideWs w = ws_of(a.ws, n, B, H);
  for (int b = t; b < B; b += WT) {
    float dout[OUTM], dls[OUTM];
    d_out_row(a, w, n, b, dout, dls);
    for (int o = 0; o < O; ++o) {
      douts[b][o] = dout[o];
      if (do_ls) dlss[b][o] = dls[o];
    }
  }
  for (int i = t; i < O * SL; i += WT) w3s[i / SL][i % SL] = d.w[n][4][(int64_t)(i / SL) * H + s * SL + i % SL];
  // dW2[slice, :] = dZ2[:, slice]^T H1: thread k owns column k of the slice's 16 rows (VALU; an MFMA
  // version over 16-row k-tiles measured slower at B = 64: its chains are only 16 deep)
  float gw2v[SL];
#pragma unroll
  for (int jj = 0; jj < SL; ++jj) gw2v[jj] = 0.f;
  float gw3 = 0.f, gb = 0.f;  // dW3[o][j] for pair t < O*SL; db2[t] (t < SL)
  for (int c0 = 0; c0 < B; c0 += RC) {
    const int nr = min(RC, B - c0);
    __syncthreads();
    stage4(&hs[0][0], HP, w.H1 + (int64_t)c0 * H, H, nr, H);
    stage1<16>(&h2s[0][0], SL + 1, w.H2 + (int64_t)c0 * H + s * SL, H, nr, SL);
    __syncthreads();
    for (int i = t; i < nr * SL; i += WT) {
      const int b = i / SL, j = i - b * SL;
      float dh = 0.f;
      for (int o = 0; o < O; ++o) dh += douts[c0 + b][o] * w3s[o][j];
      const float dz = dh * act_d(d.activation, h2s[b][j]);
      dz2s[b][j] = dz;
      w.DZ2[(int64_t)(c0 + b) * H + s * SL + j] = dz;
    }
    __syncthreads();
    if (t < O * SL) {
      const int o = t / SL, j = t - o * SL;
      for (int b = 0; b < nr; ++b) gw3 += douts[c0 + b][o] * h2s[b][j];
    }
    if (t < SL)
      for (int b = 0; b < nr; ++b) gb += dz2s[b][t];
    if (t < H) {  // thread k owns column k of every row in the slice
      for (int b = 0; b < nr; ++b) {
        const float h1 = hs[b][t];
#pragma unroll
        for (int q = 0; q < SL / 4; ++q) {
          const f4 z = *reinterpret_cast<const f4*>(&dz2s[b][4 * q]);
          gw2v[4 * q + 0] += z.x * h1;
          gw2v[4 * q + 1] += z.y * h1;
          gw2v[4 * q + 2] += z.z * h1;
          gw2v[4 * q + 3] += z.w * h1;
        }
      }
    }
  }
  if (t < O * SL) put(d.g[n][4], (int64_t)(t / SL) * H + s * SL + t % SL, gw3, acc_mode);
  if (t < SL) put(d.g[n][3], s * SL + t, gb, acc_mode);
  if (t < H) {
#pragma unroll
    for (int jj = 0; jj < SL; ++jj) put(d.g[n][2], (int64_t)(s * SL + jj) * H + t, gw2v[jj], acc_mode);
  }
  if (s == 0 && t < O) {
    float sum = 0.f;
    for (int b = 0; b < B; ++b) sum += douts[b][t];
    put(d.g[n][5], t, sum, acc_mode);
  }
  if (do_ls && t < d.out_pi) {
    float sum = 0.f;
    for (int b = 0; b < B; ++b) sum += dlss[b][t];
    put(d.g_log_std, t, sum, acc_mode);
  }
}

// ---- backward through layer 1 ----------------------------------------------------------------
__global__ __launch_bounds__(WT) void wide_bwd1_kernel(const WideArgs a) {
  __shared__ float w2t[SL][HP];                     // W2[:, slice] transposed: [j][k]
  __shared__ float zs[RC][HP];                      // dZ2 rows of the chunk
  __shared__ float xs[RC][RAI_WIDE_MAX_IN + 1];     // obs rows of the chunk
  __shared__ float dz1s[RC][SL + 1];
  const int s = blockIdx.x, n = blockIdx.y, t = threadIdx.x;
  const rai_mlp_wide_desc& d = a.d;
  const int H = d.hidden, B = a.B, IN = d.in_dim, acc_mode = d.accumulate;
  const WideWs w = ws_of(a.ws, n, B, H);
  const float* W2 = d.w[n][2];
  for (int base = t; base < H * SL; base += WT * 16) {  // row k of W2 holds the slice's 16 floats
    float v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int i = base + u * WT;
      if (i < H * SL) v[u] = W2[(int64_t)(i / SL) * H + s * SL + i % SL];
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int i = base + u * WT;
      if (i < H * SL) w2t[i % SL][i / SL] = v[u];
    }
  }
  float gw1[(SL * RAI_WIDE_MAX_IN + WT - 1) / WT];
#pragma unroll
  for (int q = 0; q < (SL * RAI_WIDE_MAX_IN + WT - 1) / WT; ++q) gw1[q] = 0.f;
  float gb = 0.f;
  for (int c0 = 0; c0 < B; c0 += RC) {
    const int nr = min(RC, B - c0);
    __syncthreads();
    stage4(&zs[0][0], HP, w.DZ2 + (int64_t)c0 * H, H, nr, H);
    stage1<16>(&xs[0][0], RAI_WIDE_MAX_IN + 1, a.obs + (int64_t)c0 * IN, IN, nr, IN);
    __syncthreads();
    {  // dH1 tile of wave w on MFMA, then dZ1 = dH1 * act'(H1)
      const int wv = t >> 6, lane = t & 63;
      const f4 z = tile_dot(&zs[16 * wv][0], &w2t[0][0], H, lane);
      const int jj = lane & 15, g = lane >> 4;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int b = 16 * wv + 4 * g + r;
        if (b < nr) dz1s[b][jj] = z[r] * act_d(d.activation, w.H1[(int64_t)(c0 + b) * H + s * SL + jj]);
      }
    }
    __syncthreads();
    if (t < SL)
      for (int b = 0; b < nr; ++b) gb += dz1s[b][t];
#pragma unroll
    for (int q = 0; q < (SL * RAI_WIDE_MAX_IN + WT - 1) / WT; ++q) {
      const int i = t + q * WT;
      if (i < SL * IN) {
        const int jj = i / IN, c = i - jj * IN;
        float g = gw1[q];
        for (int b = 0; b < nr; ++b) g += dz1s[b][jj] * xs[b][c];
        gw1[q] = g;
      }
    }
  }
  if (t < SL) put(d.g[n][1], s * SL + t, gb, acc_mode);
#pragma unroll
  for (int q = 0; q < (SL * RAI_WIDE_MAX_IN + WT - 1) / WT; ++q) {
    const int i = t + q * WT;
    if (i < SL * IN) put(d.g[n][0], (int64_t)(s * SL + i / IN) * IN + i % IN, gw1[q], acc_mode);
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
  // the forward's row chunks (RC rows each) run on separate workgroups: the rollout's B = N envs
  const dim3 grid(desc->hidden / SL, 2, (unsigned)((B + RC - 1) / RC));
  hipStream_t st = rai_stream(stream);
  hipLaunchKernelGGL(wide_fwd1_kernel, grid, dim3(WT), 0, st, a);
  RAI_LAUNCH_CHECK();
  hipLaunchKernelGGL(wide_fwd2_kernel, grid, dim3(WT), 0, st, a);
  RAI_LAUNCH_CHECK();
  hipLaunchKernelGGL(wide_head_kernel, dim3(1), dim3(WT), 0, st, a);
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}

extern "C" int rai_mlp_wide_dist_params(const rai_mlp_wide_desc* desc, const float* obs, int64_t B, float* params_out,
                                        float* v_out, void* workspace, int64_t workspace_bytes, void* stream) {
  int rc = check(desc, B, obs, workspace, workspace_bytes);
  if (rc != RAI_OK) return rc;
  if (!params_out || !v_out) return RAI_E_NULLPTR;
  WideArgs a = make_args(desc, obs, B, workspace);
  a.v = v_out;
  // the forward's row chunks (RC rows each) run on separate workgroups: the rollout's B = N envs
  const dim3 grid(desc->hidden / SL, 2, (unsigned)((B + RC - 1) / RC));
  hipStream_t st = rai_stream(stream);
  hipLaunchKernelGGL(wide_fwd1_kernel, grid, dim3(WT), 0, st, a);
  RAI_LAUNCH_CHECK();
  hipLaunchKernelGGL(wide_fwd2_kernel, grid, dim3(WT), 0, st, a);
  RAI_LAUNCH_CHECK();
  const int nb = (int)((B * (desc->out_pi + 1) + WT - 1) / WT);
  hipLaunchKernelGGL(wide_head_params_kernel, dim3(nb), dim3(WT), 0, st, a, params_out);
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}

extern "C" int rai_mlp_wide_forward_loss(const rai_mlp_wide_desc* desc, const float* obs, const void* actions,
                                         int64_t B, float* logp_out, float* entropy_out, float* v_out,
                                         const float* old_logp, const float* old_values, const float* advantages,
                                         const float* returns, const rai_ppo_hparams* hp, rai_train_state* state,
                                         float* d_logp, float* d_entropy, float* d_values, float* stats,
                                         int32_t max_stats, void* workspace, int64_t workspace_bytes, void* stream) {
  int rc = check(desc, B, obs, workspace, workspace_bytes);
  if (rc != RAI_OK) return rc;
  if (!actions || !logp_out || !entropy_out || !v_out || !advantages || !returns || !hp || !state || !d_logp ||
      !d_entropy || !d_values)
    return RAI_E_NULLPTR;
  WideArgs a = make_args(desc, obs, B, workspace);
  a.actions = actions;
  a.logp = logp_out;
  a.ent = entropy_out;
  a.v = v_out;
  LossArgs la;
  la.new_logp = logp_out;
  la.entropy = entropy_out;
  la.new_values = v_out;
  la.old_logp = old_logp ? old_logp : logp_out;
  la.old_values = old_values ? old_values : v_out;
  la.adv = advantages;
  la.ret = returns;
  la.hp = hp;
  la.state = state;
  la.d_logp = d_logp;
  la.d_entropy = d_entropy;
  la.d_values = d_values;
  la.stats = stats;
  la.B = B;
  la.n_entropy = desc->head == 1 ? B * desc->out_pi : B;
  la.K = 1;
  la.max_stats = max_stats;
  // the forward's row chunks (RC rows each) run on separate workgroups: the rollout's B = N envs
  const dim3 grid(desc->hidden / SL, 2, (unsigned)((B + RC - 1) / RC));
  hipStream_t st = rai_stream(stream);
  hipLaunchKernelGGL(wide_fwd1_kernel, grid, dim3(WT), 0, st, a);
  RAI_LAUNCH_CHECK();
  hipLaunchKernelGGL(wide_fwd2_kernel, grid, dim3(WT), 0, st, a);
  RAI_LAUNCH_CHECK();
  hipLaunchKernelGGL(wide_head_loss_kernel, dim3(1), dim3(WT), 0, st, a, la);
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
