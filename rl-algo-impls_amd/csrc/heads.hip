// Actor-critic heads of the NatureCNN policy (config C3) on gfx950: a Categorical actor head and a
// scalar critic head, both single Linear layers over the encoder output, plus the Categorical
// log-prob / entropy.  Reference: rl_algo_impls/shared/actor/categorical.py:57-87
// (CategoricalActorHead: Linear(512, A) logits, torch.distributions.Categorical log_prob and
// entropy), rl_algo_impls/shared/policy/critic.py:11-41 (CriticHead: Linear(512, 1)), joined by
// rl_algo_impls/shared/policy/actor_critic_network/connected_trio.py:83-92.
//
// PyTorch runs this as two hipBLASLt GEMMs with bias, a dozen Categorical kernels, and in the
// backward two GEMMs for the weights, two for the input (then an add of the two input gradients),
// two bias reductions and four accumulates into .grad: ~20 launches per minibatch of B = 256 rows
// and 7 x 512 weights.  Here:
//   forward   one launch:  logits = enc Wpi^T + bpi, v = enc Wv^T + bv, logp(a), entropy
//                          (one wave per row, dot products as lane partials + a wave reduction)
//   backward  two launches: (1) per row: dlogits from (d_logp, d_entropy), and
//                          d_enc = dlogits Wpi + dv Wv;  (2) per 16-column slice of the weights:
//                          dWpi, dWv summed over the rows in row order, biases by slice 0;
//                          written or added (accumulate) into the caller's gradient buffers.
// Categorical arithmetic follows torch.distributions.Categorical: logits normalised by logsumexp,
// entropy = -sum(clamp(logits_n, min=finfo.min) * p).  Deterministic (fixed orders, no atomics).
#include "common.h"

namespace {

constexpr int HD_THREADS = 256;  // 4 waves, one row each
constexpr float HD_F32_MIN = -3.4028234663852886e38f;

struct HeadsArgs {
  const float* enc;    // (B, D)
  const float* wpi;    // (A, D)
  const float* bpi;    // (A)
  const float* wv;     // (D)
  const float* bv;     // (1)
  const int64_t* act;  // (B)
  int64_t B;
  int D, A;
};

__device__ __forceinline__ float wave_reduce(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int A>
__global__ __launch_bounds__(HD_THREADS) void heads_fwd_kernel(const HeadsArgs a, float* __restrict__ logits_out,
                                                              float* __restrict__ logp, float* __restrict__ ent,
                                                              float* __restrict__ v_out) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * (HD_THREADS / 64) + (threadIdx.x >> 6);
  if (b >= a.B) return;
  const int D = a.D;
  const float* e = a.enc + b * D;
  float acc[A + 1];
#pragma unroll
  for (int o = 0; o <= A; ++o) acc[o] = 0.f;
  constexpr int NPL = 8;
  if (D <= 64 * NPL) {  // NatureCNN (D = 512): all of the lane's loads first (one round trip, not eight)
    float xs[NPL], ws[NPL][A + 1];
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const int d = min(lane + 64 * k, D - 1);
      xs[k] = e[d];
#pragma unroll
      for (int o = 0; o < A; ++o) ws[k][o] = a.wpi[o * D + d];
      ws[k][A] = a.wv[d];
    }
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const bool in = lane + 64 * k < D;  // the same fma sequence as the loop below
#pragma unroll
      for (int o = 0; o <= A; ++o) acc[o] = in ? fmaf(xs[k], ws[k][o], acc[o]) : acc[o];
    }
  } else {
    for (int d = lane; d < D; d += 64) {
      const float x = e[d];
#pragma unroll
      for (int o = 0; o < A; ++o) acc[o] = fmaf(x, a.wpi[o * D + d], acc[o]);
      acc[A] = fmaf(x, a.wv[d], acc[A]);
    }
  }
  float z[A];
#pragma unroll
  for (int o = 0; o < A; ++o) z[o] = wave_reduce(acc[o]) + a.bpi[o];
  const float v = wave_reduce(acc[A]) + a.bv[0];
  if (lane == 0) {
    float m = z[0];
#pragma unroll
    for (int o = 1; o < A; ++o) m = fmaxf(m, z[o]);
    float se = 0.f;
#pragma unroll
    for (int o = 0; o < A; ++o) se += expf(z[o] - m);
    const float lse = m + logf(se);
    float H = 0.f;
    const int act = (int)a.act[b];
    float zact = z[0];
#pragma unroll
    for (int o = 0; o < A; ++o) {
      const float n = z[o] - lse;
      H -= fmaxf(n, HD_F32_MIN) * expf(n);
      if (o == act) zact = z[o];
      logits_out[b * A + o] = z[o];
    }
    logp[b] = zact - lse;
    ent[b] = H;
    v_out[b] = v;
  }
}

// (1) per row: dlogits and d_enc; dlogits (B, A) and dv (B) stored for pass (2).  RELU (round 4): enc is
// the output of the layer's ReLU and d_enc is written as that layer's dz = enc <= 0 ? 0 : d_enc (torch's
// threshold_backward on the saved result), so the ReLU backward needs no pass of its own
template <int A, bool RELU = false>
__global__ __launch_bounds__(HD_THREADS) void heads_bwd_rows_kernel(const HeadsArgs a, const float* __restrict__ logits,
                                                                   const float* __restrict__ d_logp,
                                                                   const float* __restrict__ d_ent,
                                                                   const float* __restrict__ d_v,
                                                                   float* __restrict__ dlogits, float* __restrict__ dvv,
                                                                   float* __restrict__ d_enc) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * (HD_THREADS / 64) + (threadIdx.x >> 6);
  if (b >= a.B) return;
  float z[A];
#pragma unroll
  for (int o = 0; o < A; ++o) z[o] = logits[b * A + o];
  float m = z[0];
#pragma unroll
  for (int o = 1; o < A; ++o) m = fmaxf(m, z[o]);
  float se = 0.f;
#pragma unroll
  for (int o = 0; o < A; ++o) se += expf(z[o] - m);
  const float lse = m + logf(se);
  float H = 0.f;
#pragma unroll
  for (int o = 0; o < A; ++o) {
    const float n = z[o] - lse;
    H -= fmaxf(n, HD_F32_MIN) * expf(n);
  }
  const int act = (int)a.act[b];
  const float gl = d_logp[b], ge = d_ent[b], gv = d_v[b];
  float dq[A];
#pragma unroll
  for (int o = 0; o < A; ++o) {
    const float n = z[o] - lse;
    const float p = expf(n);
    dq[o] = gl * ((o == act ? 1.f : 0.f) - p) + ge * (-p * (n + H));
  }
  if (lane == 0) {
#pragma unroll
    for (int o = 0; o < A; ++o) dlogits[b * A + o] = dq[o];
    dvv[b] = gv;
  }
  const int D = a.D;
  constexpr int NPL = 8;  // D <= 512 (NatureCNN): every load of the row first, then the stores (the
                          // stores may alias the weights for the compiler, so a fused loop serialises)
  if (D <= 64 * NPL) {
    float sv[NPL];
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const int d = min(lane + 64 * k, D - 1);  // branch-free (all loads batch); d >= D lanes are not stored
      float s = gv * a.wv[d];
#pragma unroll
      for (int o = 0; o < A; ++o) s = fmaf(dq[o], a.wpi[o * D + d], s);
      if (RELU) s = a.enc[b * D + d] <= 0.f ? 0.f : s;
      sv[k] = s;
    }
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const int d = lane + 64 * k;
      if (d < D) d_enc[b * D + d] = sv[k];
    }
    return;
  }
  for (int d = lane; d < D; d += 64) {
    float s = gv * a.wv[d];
#pragma unroll
    for (int o = 0; o < A; ++o) s = fmaf(dq[o], a.wpi[o * D + d], s);
    if (RELU) s = a.enc[b * D + d] <= 0.f ? 0.f : s;
    d_enc[b * D + d] = s;
  }
}

// (2) weight gradients: workgroup j owns columns [C j, C j + C) of Wpi / Wv (C = HW_COLS); its 256
// threads are C columns x HW_RL row lanes; each lane sums rows lane, lane + HW_RL, ... (row order), then
// the row lanes are added in order through LDS.  Workgroup 0 also sums the bias gradients.  FCB (round
// 4): the same column sums of pass (1)'s dz give the bias gradient of the layer whose ReLU output enc is
// (g_benc[d] = sum over rows of dz[:, d], row lanes in order, as the weights).  Round 4: 8 columns x 32
// row lanes (64 workgroups at D = 512, 8 rows per lane in one load batch) instead of 16 x 16 over 32.
constexpr int HW_COLS = 8, HW_RL = HD_THREADS / HW_COLS;
template <int A, bool FCB = false>
__global__ __launch_bounds__(HD_THREADS) void heads_bwd_weights_kernel(const HeadsArgs a,
                                                                      const float* __restrict__ dlogits,
                                                                      const float* __restrict__ dvv,
                                                                      float* __restrict__ g_wpi, float* __restrict__ g_bpi,
                                                                      float* __restrict__ g_wv, float* __restrict__ g_bv,
                                                                      int accumulate, const float* __restrict__ dz = nullptr,
                                                                      float* __restrict__ g_benc = nullptr) {
  __shared__ float red[A + 1][HW_RL][HW_COLS + 1];
  __shared__ float redb[FCB ? HW_RL : 1][HW_COLS + 1];
  __shared__ float redbias[A + 1][17];
  const int tid = threadIdx.x, col = tid % HW_COLS, rl = tid / HW_COLS;
  const int d = blockIdx.x * HW_COLS + col;
  const int D = a.D;
  const int64_t B = a.B;
  float acc[A + 1];
  float accb = 0.f;
#pragma unroll
  for (int o = 0; o <= A; ++o) acc[o] = 0.f;
  if (d < D) {
#pragma unroll 8  // B = 256: 8 rows per lane, their loads in one batch
    for (int64_t b = rl; b < B; b += HW_RL) {
      const float x = a.enc[b * D + d];
#pragma unroll
      for (int o = 0; o < A; ++o) acc[o] = fmaf(dlogits[b * A + o], x, acc[o]);
      acc[A] = fmaf(dvv[b], x, acc[A]);
      if (FCB) accb += dz[b * D + d];
    }
  }
#pragma unroll
  for (int o = 0; o <= A; ++o) red[o][rl][col] = acc[o];
  if (FCB) redb[rl][col] = accb;
  __syncthreads();
  if (FCB && tid < HW_COLS) {
    const int dd = blockIdx.x * HW_COLS + tid;
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < HW_RL; ++r) s += redb[r][tid];
    if (dd < D) g_benc[dd] = accumulate ? g_benc[dd] + s : s;
  }
  if (tid < HW_COLS * (A + 1)) {
    const int o = tid / HW_COLS, c = tid % HW_COLS;
    const int dd = blockIdx.x * HW_COLS + c;
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < HW_RL; ++r) s += red[o][r][c];
    if (dd < D) {
      float* dst = o < A ? g_wpi + o * D + dd : g_wv + dd;
      *dst = accumulate ? *dst + s : s;
    }
  }
  if (blockIdx.x == 0) {  // biases: 16 row lanes per output (rows lane, lane + 16, ...), lanes in order
    __syncthreads();
    const int o = tid >> 4, l = tid & 15;
    float s = 0.f;
    if (o <= A)
      for (int64_t b = l; b < B; b += 16) s += o < A ? dlogits[b * A + o] : dvv[b];
    if (o <= A) redbias[o][l] = s;
    __syncthreads();
    if (tid <= A) {
      float t = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) t += redbias[tid][r];
      float* dst = tid < A ? g_bpi + tid : g_bv;
      *dst = accumulate ? *dst + t : t;
    }
  }
}

// 16 x (A + 1) threads of the weight pass cover the outputs: A <= 12 (Atari: 6; 18 would need a
// second pass)
bool a_ok(int A) { return (A >= 2 && A <= 10) || A == 12; }

HeadsArgs make_args(const float* enc, const float* wpi, const float* bpi, const float* wv, const float* bv,
                    const int64_t* actions, int64_t B, int32_t D, int32_t A) {
  HeadsArgs a;
  a.enc = enc;
  a.wpi = wpi;
  a.bpi = bpi;
  a.wv = wv;
  a.bv = bv;
  a.act = actions;
  a.B = B;
  a.D = D;
  a.A = A;
  return a;
}

}  // namespace

extern "C" int rai_categorical_critic_heads_fwd(const float* enc, const float* wpi, const float* bpi, const float* wv,
                                                const float* bv, const int64_t* actions, int64_t B, int32_t D,
                                                int32_t A, float* logits_out, float* logp_out, float* entropy_out,
                                                float* v_out, void* stream) {
  if (B < 0 || D < 1 || !a_ok(A)) return RAI_E_SHAPE;
  if (B == 0) return RAI_OK;
  if (!enc || !wpi || !bpi || !wv || !bv || !actions || !logits_out || !logp_out || !entropy_out || !v_out)
    return RAI_E_NULLPTR;
  const HeadsArgs a = make_args(enc, wpi, bpi, wv, bv, actions, B, D, A);
  const dim3 grid((unsigned)((B + 3) / 4));
  hipStream_t st = rai_stream(stream);
  switch (A) {
#define RAI_HD_F(n) \
  case n: hipLaunchKernelGGL(heads_fwd_kernel<n>, grid, dim3(HD_THREADS), 0, st, a, logits_out, logp_out, entropy_out, v_out); break;
    RAI_HD_F(2) RAI_HD_F(3) RAI_HD_F(4) RAI_HD_F(5) RAI_HD_F(6) RAI_HD_F(7) RAI_HD_F(8) RAI_HD_F(9) RAI_HD_F(10)
    RAI_HD_F(12)
#undef RAI_HD_F
    default: return RAI_E_SHAPE;
  }
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}

extern "C" int rai_categorical_critic_heads_bwd_relu(const float* enc, const float* wpi, const float* bpi,
                                                     const float* wv, const float* bv, const int64_t* actions,
                                                     const float* logits, int64_t B, int32_t D, int32_t A,
                                                     const float* d_logp, const float* d_entropy, const float* d_v,
                                                     float* dz, float* g_wpi, float* g_bpi, float* g_wv, float* g_bv,
                                                     float* g_benc, int32_t accumulate, void* workspace,
                                                     int64_t workspace_bytes, void* stream);

extern "C" int64_t rai_categorical_critic_heads_workspace_bytes(int64_t B, int32_t A) {
  return B < 0 || A < 1 ? 0 : B * (int64_t)(A + 1) * 4;
}

extern "C" int rai_categorical_critic_heads_bwd(const float* enc, const float* wpi, const float* bpi, const float* wv,
                                                const float* bv, const int64_t* actions, const float* logits,
                                                int64_t B, int32_t D, int32_t A, const float* d_logp,
                                                const float* d_entropy, const float* d_v, float* d_enc,
                                                float* g_wpi, float* g_bpi, float* g_wv, float* g_bv,
                                                int32_t accumulate, void* workspace, int64_t workspace_bytes,
                                                void* stream) {
  if (B < 0 || D < 1 || !a_ok(A)) return RAI_E_SHAPE;
  if (!enc || !wpi || !bpi || !wv || !bv || !actions || !logits || !d_logp || !d_entropy || !d_v || !d_enc ||
      !g_wpi || !g_bpi || !g_wv || !g_bv || !workspace)
    return RAI_E_NULLPTR;
  if (workspace_bytes < rai_categorical_critic_heads_workspace_bytes(B, A)) return RAI_E_WORKSPACE;
  if (B == 0) return RAI_OK;
  const HeadsArgs a = make_args(enc, wpi, bpi, wv, bv, actions, B, D, A);
  float* dlogits = static_cast<float*>(workspace);
  float* dvv = dlogits + B * A;
  hipStream_t st = rai_stream(stream);
  const dim3 grid1((unsigned)((B + 3) / 4)), grid2((unsigned)((D + HW_COLS - 1) / HW_COLS));
  switch (A) {
#define RAI_HD_B(n)                                                                                          \
  case n:                                                                                                    \
    hipLaunchKernelGGL(heads_bwd_rows_kernel<n>, grid1, dim3(HD_THREADS), 0, st, a, logits, d_logp, d_entropy, \
                       d_v, dlogits, dvv, d_enc);                                                            \
    hipLaunchKernelGGL(heads_bwd_weights_kernel<n>, grid2, dim3(HD_THREADS), 0, st, a, dlogits, dvv, g_wpi,   \
                       g_bpi, g_wv, g_bv, accumulate);                                                       \
    break;
    RAI_HD_B(2) RAI_HD_B(3) RAI_HD_B(4) RAI_HD_B(5) RAI_HD_B(6) RAI_HD_B(7) RAI_HD_B(8) RAI_HD_B(9) RAI_HD_B(10)
    RAI_HD_B(12)
#undef RAI_HD_B
    default: return RAI_E_SHAPE;
  }
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}

// The heads' backward with the ReLU backward of the layer that produced enc folded in (round 4; NatureCNN's
// fc -> ReLU, nature_cnn.py / cnn.py:44-53): dz = enc <= 0 ? 0 : d_enc is written instead of d_enc, and
// g_benc (D floats) receives (accumulate: += ) that layer's bias gradient, the column sums of dz; the
// separate rai_bias_relu_bwd pass over the (B, D) gradient is gone.
extern "C" int rai_categorical_critic_heads_bwd_relu(const float* enc, const float* wpi, const float* bpi,
                                                     const float* wv, const float* bv, const int64_t* actions,
                                                     const float* logits, int64_t B, int32_t D, int32_t A,
                                                     const float* d_logp, const float* d_entropy, const float* d_v,
                                                     float* dz, float* g_wpi, float* g_bpi, float* g_wv, float* g_bv,
                                                     float* g_benc, int32_t accumulate, void* workspace,
                                                     int64_t workspace_bytes, void* stream) {
  if (B < 0 || D < 1 || !a_ok(A)) return RAI_E_SHAPE;
  if (!enc || !wpi || !bpi || !wv || !bv || !actions || !logits || !d_logp || !d_entropy || !d_v || !dz || !g_wpi ||
      !g_bpi || !g_wv || !g_bv || !g_benc || !workspace)
    return RAI_E_NULLPTR;
  if (workspace_bytes < rai_categorical_critic_heads_workspace_bytes(B, A)) return RAI_E_WORKSPACE;
  hipStream_t st = rai_stream(stream);
  if (B == 0) {
    if (!accumulate) {
      const hipError_t e = hipMemsetAsync(g_benc, 0, (size_t)D * 4, st);
      if (e != hipSuccess) return (int)e;
    }
    return RAI_OK;
  }
  const HeadsArgs a = make_args(enc, wpi, bpi, wv, bv, actions, B, D, A);
  float* dlogits = static_cast<float*>(workspace);
  float* dvv = dlogits + B * A;
  const dim3 grid1((unsigned)((B + 3) / 4)), grid2((unsigned)((D + HW_COLS - 1) / HW_COLS));
  switch (A) {
#define RAI_HD_BR(n)                                                                                            \
  case n:                                                                                                       \
    hipLaunchKernelGGL((heads_bwd_rows_kernel<n, true>), grid1, dim3(HD_THREADS), 0, st, a, logits, d_logp,      \
                       d_entropy, d_v, dlogits, dvv, dz);                                                       \
    hipLaunchKernelGGL((heads_bwd_weights_kernel<n, true>), grid2, dim3(HD_THREADS), 0, st, a, dlogits, dvv,     \
                       g_wpi, g_bpi, g_wv, g_bv, accumulate, dz, g_benc);                                       \
    break;
    RAI_HD_BR(2) RAI_HD_BR(3) RAI_HD_BR(4) RAI_HD_BR(5) RAI_HD_BR(6) RAI_HD_BR(7) RAI_HD_BR(8) RAI_HD_BR(9)
    RAI_HD_BR(10) RAI_HD_BR(12)
#undef RAI_HD_BR
    default: return RAI_E_SHAPE;
  }
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}
