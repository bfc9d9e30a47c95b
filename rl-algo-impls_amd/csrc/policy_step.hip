// Fused rollout step for CartPole-class MLP actor-critics: both networks' forward pass, the
// categorical sample and the rollout-slot writes (action, log-prob, value) in one launch per env
// step.  Replaces, for this policy class, rl_algo_impls/shared/policy/actor_critic.py:306-318
// (ActorCritic.step: _distribution_and_value -> pi.sample -> log_prob, v) and the slot writes of
// rl_algo_impls/rollout/sync_step_rollout.py:193-201 — the per-step sequence that otherwise is
// ~10 small PyTorch launches (3 linears + 2 activations per network) plus the sampling kernel.
//
// A workgroup owns 32 env rows: waves 0-1 run the critic on its two 16-row tiles while waves 2-3 run
// the actor on the same tiles (the two networks side by side instead of one after the other in every
// wave: half the dependent chain per wave, twice the workgroups).  Per network and tile: layer 1 (one
// v_mfma_f32_16x16x4f32 per 16-column tile, K = in_dim padded to 4/8), layer 2 (4 column tiles x 16
// k-steps), the output layer as DPP row sums; the weights of both networks are staged once per
// workgroup in LDS.  Sampling is the one of
// rai_categorical_sample (Philox4x32-10 keyed by seed, counter (offset, row); inverse CDF on the
// unnormalised mass), so the two paths draw from the same stream.
#include "common.h"

#pragma clang fp contract(off)

namespace {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

constexpr int HID = 64;
constexpr int LD = 66;
constexpr int NT = 256;        // 4 waves: (critic, actor) x two 16-row tiles
constexpr int ROWS = 32;

struct NetPtrs {
  const float* W1;  // [64][in]
  const float* b1;  // [64]
  const float* W2;  // [64][64]
  const float* b2;  // [64]
  const float* W3;  // [out][64]
  const float* b3;  // [out]
};
struct StepArgs {
  NetPtrs pi, v;
  const float* obs;  // [N][in]
  int64_t N;
  int32_t in_dim, n_act;
  uint64_t seed, offset;
  int64_t* actions;  // nullable (value-only call)
  float* logp;       // nullable
  float* values;     // [N]
  // host-mapped staging (rai_mlp_policy_step_mapped; all nullable): obs_host replaces obs as the input and
  // is copied into obs (the rollout slot); rew_host / done_host are copied into rew_dst / done_dst; the
  // sampled actions are also written to act_host
  const float* obs_host;
  const float* rew_host;
  float* rew_dst;
  const uint8_t* done_host;
  uint8_t* done_dst;
  int64_t* act_host;
};

template <int INP>
struct NetSmem {
  float W1[HID][INP];
  float b1[HID];
  float W2[HID][LD];
  float b2[HID];
};
template <int INP, int OUTP>
struct StepSmem {
  NetSmem<INP> n[2];
  float W3a[OUTP][HID];
  float W3v[HID];
  float b3a[8];
  float b3v;
  float X[ROWS][INP];
  float H1[2][ROWS][LD];  // per network
};

__device__ __forceinline__ int kmap(int g, int kk) { return (g & 1) * 32 + (g >> 1) * 16 + kk; }
__device__ __forceinline__ float tanh_bf(float x) {
  const float ax = fabsf(x);
  const float x2 = x * x;
  float p = fmaf(x2, 62.f / 2835.f, -17.f / 315.f);
  p = fmaf(x2, p, 2.f / 15.f);
  p = fmaf(x2, p, -1.f / 3.f);
  const float small = fmaf(x * x2, p, x);
  const float e = __builtin_amdgcn_exp2f(ax * 2.885390081777927f);
  const float big = fmaf(-2.f, __builtin_amdgcn_rcpf(e + 1.f), 1.f);
  return ax < 0.3f ? small : copysignf(big, x);
}
template <int RELU>
__device__ __forceinline__ float act_f(float z) { return RELU ? fmaxf(z, 0.f) : tanh_bf(z); }
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row_sum16(float v) {
  v += dpp<0xB1>(v);
  v += dpp<0x4E>(v);
  v += dpp<0x141>(v);
  v += dpp<0x140>(v);
  return v;
}

// A network's weights, fetched into registers (every load issued before any LDS store: one global
// round trip for the staging instead of one per element of a load -> ds_write loop), then stored.
template <int INP>
struct NetRegs {
  static constexpr int W2PT = HID * HID / NT;             // 16 floats of W2 per thread
  static constexpr int W1PT = (HID * INP + NT - 1) / NT;  // 1 (INP 4) or 2 (INP 8)
  float w2[W2PT], w1[W1PT], b1, b2;
};
template <int INP>
__device__ __forceinline__ NetRegs<INP> fetch_net(const NetPtrs& p, int IN, int tid) {
  NetRegs<INP> r;
#pragma unroll
  for (int u = 0; u < NetRegs<INP>::W2PT; ++u) r.w2[u] = p.W2[tid + u * NT];
#pragma unroll
  for (int u = 0; u < NetRegs<INP>::W1PT; ++u) {
    const int e = tid + u * NT, j = e / INP, k = e % INP;
    r.w1[u] = (e < HID * INP && k < IN) ? p.W1[j * IN + k] : 0.f;
  }
  r.b1 = tid < HID ? p.b1[tid] : 0.f;
  r.b2 = tid < HID ? p.b2[tid] : 0.f;
  return r;
}
template <int INP>
__device__ __forceinline__ void store_net(const NetRegs<INP>& r, NetSmem<INP>& S, int tid) {
#pragma unroll
  for (int u = 0; u < NetRegs<INP>::W2PT; ++u) {
    const int e = tid + u * NT;
    S.W2[e >> 6][e & 63] = r.w2[u];
  }
#pragma unroll
  for (int u = 0; u < NetRegs<INP>::W1PT; ++u) {
    const int e = tid + u * NT;
    if (e < HID * INP) S.W1[e / INP][e % INP] = r.w1[u];
  }
  if (tid < HID) {
    S.b1[tid] = r.b1;
    S.b2[tid] = r.b2;
  }
}

// hidden activations h2[t][r] (row 4g + r of the wave's tile, column 16t + li) of one network
template <int INP, int RELU>
__device__ __forceinline__ void mlp_hidden(const NetSmem<INP>& S, float (&H1)[ROWS][LD], const float (&X)[ROWS][INP],
                                           int R, int g, int li, float (&h2)[4][4]) {
  f4 z[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) z[t] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < INP / 4; ++q) {
    const float av = X[R + li][4 * q + g];
#pragma unroll
    for (int t = 0; t < 4; ++t)
      z[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, S.W1[16 * t + li][4 * q + g], z[t], 0, 0, 0);
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const float bj = S.b1[16 * t + li];
#pragma unroll
    for (int r = 0; r < 4; ++r) H1[R + g * 4 + r][16 * t + li] = act_f<RELU>(z[t][r] + bj);
  }
  f4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kk = 0; kk < 16; kk += 2) {
    const int kq = kmap(g, kk);
    const f2 av = *reinterpret_cast<const f2*>(&H1[R + li][kq]);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const f2 bv = *reinterpret_cast<const f2*>(&S.W2[16 * t + li][kq]);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, bv.x, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, bv.y, acc[t], 0, 0, 0);
    }
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const float bb = S.b2[16 * t + li];
#pragma unroll
    for (int r = 0; r < 4; ++r) h2[t][r] = act_f<RELU>(acc[t][r] + bb);
  }
}

template <int INP, int OUTP, int RELU>
__global__ __launch_bounds__(NT) void mlp_policy_step_kernel(const StepArgs a) {
  __shared__ StepSmem<INP, OUTP> S;
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, li = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int IN = a.in_dim, NA = a.n_act;
  const int64_t row0 = (int64_t)blockIdx.x * ROWS;
  const bool sample = a.actions != nullptr;

  // every staging load of the launch in flight together: both networks, the output layers, the rows
  const NetRegs<INP> rv = fetch_net<INP>(a.v, IN, tid);
  NetRegs<INP> rp;
  if (sample) rp = fetch_net<INP>(a.pi, IN, tid);
  constexpr int W3PT = (OUTP * HID + NT - 1) / NT, XPT = (ROWS * INP + NT - 1) / NT;
  float w3a[W3PT], xv[XPT];
#pragma unroll
  for (int u = 0; u < W3PT; ++u) {
    const int e = tid + u * NT;
    w3a[u] = (sample && e < OUTP * HID && (e >> 6) < NA) ? a.pi.W3[e] : 0.f;
  }
  const float w3v = tid < HID ? a.v.W3[tid] : 0.f;
  const float b3a = (sample && tid < NA && tid < 8) ? a.pi.b3[tid] : 0.f;
  const float b3v = tid == 0 ? a.v.b3[0] : 0.f;
  const float* xsrc = a.obs_host ? a.obs_host : a.obs;
#pragma unroll
  for (int u = 0; u < XPT; ++u) {
    const int e = tid + u * NT, r = e / INP, k = e % INP;
    const int64_t row = row0 + r;
    xv[u] = (e < ROWS * INP && row < a.N && k < IN) ? xsrc[row * IN + k] : 0.f;
  }
  if (a.obs_host) {  // the observations into the rollout slot (vector stores)
#pragma unroll
    for (int u = 0; u < XPT; ++u) {
      const int e = tid + u * NT, r = e / INP, k = e % INP;
      const int64_t row = row0 + r;
      if (e < ROWS * INP && row < a.N && k < IN) const_cast<float*>(a.obs)[row * IN + k] = xv[u];
    }
  }
  if (tid < ROWS && row0 + tid < a.N) {
    if (a.rew_host) a.rew_dst[row0 + tid] = a.rew_host[row0 + tid];
    if (a.done_host) a.done_dst[row0 + tid] = a.done_host[row0 + tid];
  }
  store_net<INP>(rv, S.n[1], tid);
  if (sample) store_net<INP>(rp, S.n[0], tid);
#pragma unroll
  for (int u = 0; u < W3PT; ++u) {
    const int e = tid + u * NT;
    if (e < OUTP * HID) S.W3a[e >> 6][e & 63] = w3a[u];
  }
  if (tid < HID) S.W3v[tid] = w3v;
  if (tid < 8) S.b3a[tid] = b3a;
  if (tid == 0) S.b3v = b3v;
#pragma unroll
  for (int u = 0; u < XPT; ++u) {
    const int e = tid + u * NT;
    if (e < ROWS * INP) S.X[e / INP][e % INP] = xv[u];
  }
  __syncthreads();

  const int R = (w & 1) * 16;  // this wave's 16-row tile; waves 0-1 the critic, 2-3 the actor
  const int q = li & 3;
  const int64_t my_row = row0 + R + g * 4 + q;  // the row whose outputs this lane writes (li < 4)
  float h2[4][4];
  if (w < 2) {
    // ---- critic: value of every row ----
    mlp_hidden<INP, RELU>(S.n[1], S.H1[1], S.X, R, g, li, h2);
    float val = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float p = h2[0][r] * S.W3v[li];
      p = fmaf(h2[1][r], S.W3v[16 + li], p);
      p = fmaf(h2[2][r], S.W3v[32 + li], p);
      p = fmaf(h2[3][r], S.W3v[48 + li], p);
      const float s = row_sum16(p);
      val = q == r ? s : val;
    }
    val += S.b3v;
    if (li < 4 && my_row < a.N) a.values[my_row] = val;
    return;
  }
  if (!sample) return;
  // ---- actor: logits, categorical sample, log-prob ----
  mlp_hidden<INP, RELU>(S.n[0], S.H1[0], S.X, R, g, li, h2);
  float z[OUTP];
#pragma unroll
  for (int o = 0; o < OUTP; ++o) {
    float sel = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float p = h2[0][r] * S.W3a[o][li];
      p = fmaf(h2[1][r], S.W3a[o][16 + li], p);
      p = fmaf(h2[2][r], S.W3a[o][32 + li], p);
      p = fmaf(h2[3][r], S.W3a[o][48 + li], p);
      const float s = row_sum16(p);
      sel = q == r ? s : sel;
    }
    z[o] = sel + S.b3a[o];
  }
  if (li < 4 && my_row < a.N) {
    float m = -INFINITY;
#pragma unroll
    for (int o = 0; o < OUTP; ++o)
      if (o < NA) m = fmaxf(m, z[o]);
    float s = 0.f;
#pragma unroll
    for (int o = 0; o < OUTP; ++o)
      if (o < NA) s += expf(z[o] - m);
    const float lse = m + logf(s);
    const Philox4 rnd = philox4x32_10(a.offset, (uint64_t)my_row, a.seed);
    const float u = u01_open0(rnd.x) * s;
    float c = 0.f;
    int act = -1;
#pragma unroll
    for (int o = 0; o < OUTP; ++o)
      if (o < NA) {
        c += expf(z[o] - m);
        if (act < 0 && u <= c) act = o;
      }
    if (act < 0) act = NA - 1;
    float zact = z[0];
#pragma unroll
    for (int o = 1; o < OUTP; ++o)
      if (o == act) zact = z[o];
    a.actions[my_row] = act;
    if (a.act_host) a.act_host[my_row] = act;
    a.logp[my_row] = zact - lse;
  }
}

template <int INP, int OUTP>
void launch_step(const StepArgs& a, int relu, hipStream_t s) {
  const dim3 grid((unsigned)((a.N + ROWS - 1) / ROWS));
  if (relu) hipLaunchKernelGGL((mlp_policy_step_kernel<INP, OUTP, 1>), grid, dim3(NT), 0, s, a);
  else hipLaunchKernelGGL((mlp_policy_step_kernel<INP, OUTP, 0>), grid, dim3(NT), 0, s, a);
}

}  // namespace

extern "C" int rai_mlp_policy_step(const float* const* pi_params, const float* const* v_params, const float* obs,
                                   int64_t N, int32_t in_dim, int32_t hidden, int32_t n_actions,
                                   int32_t activation, uint64_t seed, uint64_t offset, int64_t* actions_out,
                                   float* logp_out, float* values_out, void* stream) {
  if (!v_params || !obs || !values_out) return RAI_E_NULLPTR;
  if ((actions_out == nullptr) != (logp_out == nullptr) || (actions_out && !pi_params)) return RAI_E_NULLPTR;
  if (hidden != HID || in_dim < 1 || in_dim > 8 || n_actions < 1 || n_actions > 8 || N < 1 ||
      (activation != 0 && activation != 1))
    return RAI_E_SHAPE;
  for (int i = 0; i < 6; ++i)
    if (!v_params[i] || (actions_out && !pi_params[i])) return RAI_E_NULLPTR;
  StepArgs a = {};
  if (actions_out) a.pi = {pi_params[0], pi_params[1], pi_params[2], pi_params[3], pi_params[4], pi_params[5]};
  a.v = {v_params[0], v_params[1], v_params[2], v_params[3], v_params[4], v_params[5]};
  a.obs = obs;
  a.N = N;
  a.in_dim = in_dim;
  a.n_act = n_actions;
  a.seed = seed;
  a.offset = offset;
  a.actions = actions_out;
  a.logp = logp_out;
  a.values = values_out;
  hipStream_t s = rai_stream(stream);
  if (in_dim <= 4 && n_actions <= 2) launch_step<4, 2>(a, activation, s);
  else launch_step<8, 8>(a, activation, s);
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}

// The same step with the host hand-off folded in (the CartPole-class rollout loop,
// rl_algo_impls/rollout/sync_step_rollout.py:193-207): the env's next observations, rewards and
// terminations are read by the kernel straight from host-mapped pinned memory (rai_host_alloc) and
// written into their rollout slots, and the actions are written to host-mapped memory as well, so one
// launch and one stream wait replace three H2D copies, the D2H copy and their API calls per env step.
extern "C" int rai_mlp_policy_step_mapped(const float* const* pi_params, const float* const* v_params,
                                          const float* obs_host, float* obs_slot, int64_t N, int32_t in_dim,
                                          int32_t hidden, int32_t n_actions, int32_t activation, uint64_t seed,
                                          uint64_t offset, int64_t* actions_out, float* logp_out,
                                          float* values_out, int64_t* actions_host, const float* rew_host,
                                          float* rew_dst, const uint8_t* done_host, uint8_t* done_dst,
                                          void* stream) {
  if (!v_params || !obs_slot || !values_out || !pi_params || !actions_out || !logp_out) return RAI_E_NULLPTR;
  if ((rew_host == nullptr) != (rew_dst == nullptr) || (done_host == nullptr) != (done_dst == nullptr))
    return RAI_E_NULLPTR;
  if (hidden != HID || in_dim < 1 || in_dim > 8 || n_actions < 1 || n_actions > 8 || N < 1 ||
      (activation != 0 && activation != 1))
    return RAI_E_SHAPE;
  for (int i = 0; i < 6; ++i)
    if (!v_params[i] || !pi_params[i]) return RAI_E_NULLPTR;
  StepArgs a = {};
  a.pi = {pi_params[0], pi_params[1], pi_params[2], pi_params[3], pi_params[4], pi_params[5]};
  a.v = {v_params[0], v_params[1], v_params[2], v_params[3], v_params[4], v_params[5]};
  a.obs = obs_slot;
  a.N = N;
  a.in_dim = in_dim;
  a.n_act = n_actions;
  a.seed = seed;
  a.offset = offset;
  a.actions = actions_out;
  a.logp = logp_out;
  a.values = values_out;
  a.obs_host = obs_host;
  a.rew_host = rew_host;
  a.rew_dst = rew_dst;
  a.done_host = done_host;
  a.done_dst = done_dst;
  a.act_host = actions_host;
  hipStream_t s = rai_stream(stream);
  if (in_dim <= 4 && n_actions <= 2) launch_step<4, 2>(a, activation, s);
  else launch_step<8, 8>(a, activation, s);
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}

// Host-mapped pinned memory for the kernels above: coherent (fine-grained) host memory the GPU reads and
// writes over the bus, with its device-side address.
extern "C" int rai_host_alloc(int64_t bytes, void** host_out, void** dev_out) {
  if (bytes < 1) return RAI_E_SHAPE;
  if (!host_out || !dev_out) return RAI_E_NULLPTR;
  void* h = nullptr;
  hipError_t e = hipHostMalloc(&h, (size_t)bytes, hipHostMallocMapped | hipHostMallocCoherent);
  if (e != hipSuccess) return (int)e;
  void* d = nullptr;
  e = hipHostGetDevicePointer(&d, h, 0);
  if (e != hipSuccess) {
    (void)hipHostFree(h);
    return (int)e;
  }
  *host_out = h;
  *dev_out = d;
  return RAI_OK;
}

extern "C" int rai_host_free(void* host) {
  if (!host) return RAI_OK;
  const hipError_t e = hipHostFree(host);
  return e == hipSuccess ? RAI_OK : (int)e;
}

extern "C" int rai_stream_sync(void* stream) {
  const hipError_t e = hipStreamSynchronize(rai_stream(stream));
  return e == hipSuccess ? RAI_OK : (int)e;
}
