// Large-minibatch PPO step for CartPole-class MLP actor-critics (SURVEY 8(d) batch policy (b):
// batch_size = n_steps * num_envs / 4, i.e. 131,072 rows per optimizer step at config C2).
//
// Replaces rl_algo_impls/ppo/ppo.py:290-411 (minibatch forward, ppo.py:326-371 loss, ppo.py:375
// backward, ppo.py:441-447 clip_grad_norm_ + Adam) for the policy of
// rl_algo_impls/shared/policy/actor_critic_network/connected_trio.py with Flatten encoder and
// [in -> 64 -> 64 -> out] actor (Categorical, shared/actor/categorical.py:57-87) and critic
// (shared/policy/critic.py:11-41) MLPs, when a minibatch no longer fits the one-launch epoch kernels
// (<= 256 rows, mlp_mc8.h).  At this size one optimizer step is ~6.9 GFLOP of 64-wide contractions:
// throughput-bound, so the work spreads over every CU instead of a latency-bound dependent chain.
//
// Per minibatch, three launches on the caller's stream:
//  1. lb_grads_kernel: 256 persistent workgroups of 4 waves (128 per network; actor and critic share
//     no parameter and their loss terms are separable, ppo.py:361-371).  Each wave walks 16-row tiles
//     of the minibatch with no workgroup barrier:
//       layer 1, layer 2, dH1 = W2^T dZ2 on v_mfma_f32_16x16x4_f32 in the "hidden x rows" orientation,
//       so every layer's accumulator tile is the next layer's B operand in place (no data movement on
//       the forward / backward chain; the A operands are W2 permutations staged once in LDS);
//       the output layer and its backward as lane-group sums (v_permlane16/32_swap) in the epilogue;
//       the per-row loss and its gradient w.r.t. the head outputs (the arithmetic of mlp_ppo.hip);
//       dW2 += dZ2^T H1 and [dW1 | db1] += dZ1^T [x | 1] on MFMA with the rows as the reduction axis
//       (dZ2, H1, dZ1 transposed through a per-wave LDS tile; the x operand is loaded transposed);
//       dW3, db2, db3 as per-lane partial sums.
//     Accumulators persist over the wave's tiles; the LB_NW (= 4) waves add their partials in LDS in wave order
//     and the workgroup writes ONE partial gradient (its network's parameter block) + loss-statistic
//     partials.  Tiles are dealt to waves statically: the summation order is fixed (deterministic).
//  2. lb_reduce_kernel: every parameter's 128 workgroup partials summed in workgroup order -> the flat
//     gradient; per-block fp64 squared-norm partials; block 0 writes the minibatch's stats row.
//  3. optim.hip's clip_optim_kernel over those partials (clip_grad_norm_ + Adam, torch's formulas).
// Epoch mode adds, once per epoch, the per-minibatch advantage moments (ppo.py:313-316: mean and
// unbiased std, fp64 sums) in two small launches.
#include <algorithm>
#include <mutex>
#include <vector>

#include "common.h"
#include "internal.h"

// FP contraction stays ON here (mul + add -> fma): on gfx950 the f32 MFMAs and the VALU share the SIMD's f32
// datapath, so every VALU instruction is time taken from the MFMAs, and this kernel is checked against the
// reference at fp32 tolerance (its summation orders differ from torch's anyway), not bit for bit.

namespace {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned int u4v_lb __attribute__((ext_vector_type(4)));

constexpr int HID = 64;
constexpr int LB_NT = 256;            // 4 waves: one per SIMD (each pipelines two tiles)
constexpr int LB_NW = LB_NT / 64;
constexpr int LB_WG_PER_NET = 128;    // fixed: the partial-gradient summation order depends on it
constexpr int LB_GRID = 2 * LB_WG_PER_NET;
constexpr int LB_WAVES_PER_NET = LB_WG_PER_NET * LB_NW;
constexpr int LB_TS = 24;             // transpose-tile row stride (floats): conflict-free b128 reads
constexpr int LB_PSTRIDE = 4612;      // >= actor block 64*4+64+64*64+64+2*64+2 = 4610, multiple of 4
constexpr int LB_MOMP = 64;           // advantage-moment partial chunks per minibatch
constexpr int LB_RED_NT = 256;        // reduce kernel: 64 parameters x 4 partial quarters per block
constexpr float F32_MIN = -3.4028234663852886e38f;

struct LbSmem {
  float w2f[4][4][64][4];  // forward A operands   [m2][blk][lane][i] = W2[16 m2 + j][16 blk + 4 g + i]
  float w2b[4][4][64][4];  // backward A operands  [m1][blk][lane][i] = W2[16 blk + 4 g + i][16 m1 + j]
  float w1[HID][4];        // W1, inputs zero-padded to 4
  float b1[HID];
  float b2[HID];
  float b1c[HID];  // b * 2 log2(e) (lb_act_bias)
  float b2c[HID];
  float w3[2][HID];        // W3 rows (critic: row 1 zero)
  float b3[4];
  double st[LB_NW][4];     // per-wave loss-statistic partials
  // per-wave transpose tiles [c][row], two pipeline slots: H1 (then dZ1) and dZ2; after the tile loop
  // the workgroup's partial-gradient accumulator (hs0 onward)
  float hs0[LB_NW][HID][LB_TS];   // H1 of the slot's tile
  float tdz0[LB_NW][HID][LB_TS];  // dZ2 (and the other slot's dH1 in passing)
  float hs1[LB_NW][HID][LB_TS];
  float tdz1[LB_NW][HID][LB_TS];
};
static_assert(sizeof(float) * LB_NW * 4 * HID * LB_TS >= sizeof(float) * LB_PSTRIDE, "accumulator fits");

struct LbArgs {
  const float* params;
  const float* obs;
  const int64_t* actions;
  const float* old_logp;
  const float* old_values;
  const float* adv;
  const float* ret;
  const float* moments;  // this minibatch's (mean, den): A = (adv - mean) / den
  const rai_ppo_hparams* hp;
  float* part;           // [LB_GRID][LB_PSTRIDE] per-workgroup partial gradients (network-local order)
  double* statp;         // [LB_GRID][4]
  int64_t row0;          // first rollout row of the minibatch
  int32_t rows;          // rows in the minibatch
  int32_t in_dim;
  float inv_n;           // 1 / (rows * world)
};

// tanh(z + b) = 1 - 2 / (exp(2 (z + b)) + 1) with the bias folded into the exponent's FMA:
// exp2(z * 2 log2(e) + b * 2 log2(e)).  Absolute error ~2 ulp of 1 everywhere (no cancellation is
// compensated: tanh(x) ~ x below |x| ~ 1e-3 is consumed only through sums of O(1) terms, so the absolute
// error is what reaches the outputs); both tails saturate correctly (exp2 -> inf gives 1, -> 0 gives -1).
// Five VALU instructions, no branch: on gfx950 the f32 MFMAs and the VALU share the SIMD's f32 datapath
// (tools/mfma_valu_overlap.hip: VALU beside MFMAs is additive), so VALU instructions are the cost.
constexpr float LB_2LOG2E = 2.885390081777927f;
template <int RELU>
__device__ __forceinline__ float lb_act_bias(float z, float b, float bc) {  // bc = b * 2 log2(e)
  if (RELU) return fmaxf(z + b, 0.f);
  const float e = __builtin_amdgcn_exp2f(fmaf(z, LB_2LOG2E, bc));
  return fmaf(-2.f, __builtin_amdgcn_rcpf(e + 1.f), 1.f);
}
template <int RELU>
__device__ __forceinline__ float lb_act_d(float h) {  // derivative from the activation's output
  return RELU ? (h > 0.f ? 1.f : 0.f) : fmaf(-h, h, 1.f);
}
__device__ __forceinline__ float lb_exp(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }
__device__ __forceinline__ float lb_log(float x) { return __builtin_amdgcn_logf(x) * 0.6931471805599453f; }

// Sum over the four 16-lane groups at the same lane & 15 (every lane receives the same bits).
__device__ __forceinline__ float lb_sum_groups(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  const auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(q[0]) + __uint_as_float(q[1]);
}
template <int CTRL>
__device__ __forceinline__ float lb_dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
// Sum over the 16 lanes of a DPP row (every lane of the row receives the same bits).
__device__ __forceinline__ float lb_row_sum16(float v) {
  v += lb_dpp<0xB1>(v);
  v += lb_dpp<0x4E>(v);
  v += lb_dpp<0x141>(v);
  v += lb_dpp<0x140>(v);
  return v;
}

#ifdef RAI_STAMPS
// Diagnostic build only (never the shipped library): shader-clock stamps of every wave at the kernel's
// phase boundaries (last launch), plus the constant-rate clock at start / end; rai_mlp_large_debug_stamps
__device__ unsigned long long g_lb_stamps[LB_GRID][LB_NW][32];
#define LB_STAMP(k)                                                                               \
  do {                                                                                            \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();                                   \
    if ((threadIdx.x & 63) == 0) g_lb_stamps[blockIdx.x][threadIdx.x >> 6][k] = t_;               \
  } while (0)
#define LB_ACC(k, t0)                                                                             \
  do {                                                                                            \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();                                   \
    if ((threadIdx.x & 63) == 0) g_lb_stamps[blockIdx.x][threadIdx.x >> 6][k] += t_ - (t0);       \
    t0 = t_;                                                                                      \
  } while (0)
#define LB_PH()                                                                                   \
  do {                                                                                            \
    LB_ACC(ph, tr);                                                                               \
    ++ph;                                                                                         \
  } while (0)
#define LB_RSTAMP(k)                                                                              \
  do {                                                                                            \
    const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();                               \
    if ((threadIdx.x & 63) == 0) g_lb_stamps[blockIdx.x][threadIdx.x >> 6][k] = t_;               \
  } while (0)
#else
#define LB_STAMP(k) do { } while (0)
#define LB_RSTAMP(k) do { } while (0)
#define LB_ACC(k, t0) do { } while (0)
#define LB_PH() do { } while (0)
#endif

// Interleave an MFMA-heavy phase with a VALU-heavy one inside a scheduling region: N groups of one MFMA
// followed by V VALU instructions (the compiler otherwise clusters the MFMAs and exposes the VALU chain).
template <int N, int V>
__device__ __forceinline__ void lb_interleave() {
#ifndef LB_NO_IGLP
#pragma unroll
  for (int k = 0; k < N; ++k) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x002, V, 0);
  }
#endif
}

#ifdef LB_NO_FENCE  // A/B builds only
#define LB_FENCE() do { } while (0)
#else
#define LB_FENCE() __builtin_amdgcn_sched_barrier(0)
#endif

__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

struct LbIn {
  float xb;     // layer-1 B operand: x[row j][feature g]
  float u0, u1; // actor: old logp, advantage; critic: old value, return
  int act;      // actor: action
  bool valid;   // row j of the tile is inside the minibatch
};

// One tile's forward inputs for one lane (prefetched a tile ahead).  Loads are unconditional (row
// indices clamped into the minibatch) and masked afterwards, so the tile body is one basic block.
template <bool ACTOR>
__device__ __forceinline__ void lb_load(const LbArgs& a, int t, int g, int j, LbIn& in) {
  const int IN = a.in_dim, last = a.rows - 1;
  const int r = t * 16 + j;
  const bool valid = r <= last;
  const int64_t row = a.row0 + min(r, last);
  const float xb = a.obs[row * IN + min(g, IN - 1)];
  in.xb = (valid && g < IN) ? xb : 0.f;
  if (ACTOR) {
    in.act = (int)a.actions[row];
    in.u0 = a.old_logp[row];
    in.u1 = a.adv[row];
  } else {
    in.act = 0;
    in.u0 = a.old_values[row];
    in.u1 = a.ret[row];
  }
  in.valid = valid;
}
// [dW1 | db1]'s B operand of tile t: [x | 1][row 4g + s][column j] (zero past the minibatch)
__device__ __forceinline__ void lb_load_xw(const LbArgs& a, int t, int g, int j, float (&xw)[4]) {
  const int IN = a.in_dim, last = a.rows - 1;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int rs = t * 16 + 4 * g + s;
    const float x = a.obs[(a.row0 + min(rs, last)) * IN + min(j, IN - 1)];
    xw[s] = rs <= last ? (j < IN ? x : (j == 4 ? 1.f : 0.f)) : 0.f;
  }
}

template <int RELU, bool ACTOR>
__device__ __forceinline__ void lb_net(const LbArgs& a, LbSmem& S, int wgn) {
  constexpr int OUT = ACTOR ? 2 : 1;
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, j = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int IN = a.in_dim;
  const int szA = HID * IN + HID + HID * HID + HID + 2 * HID + 2;
  const int base = ACTOR ? 0 : szA;
  // network-local offsets (the partial-gradient layout) and flat offsets (base + local)
  const int oW1 = 0, ob1 = HID * IN, oW2 = ob1 + HID, ob2 = oW2 + HID * HID, oW3 = ob2 + HID,
            ob3 = oW3 + OUT * HID, P_net = ob3 + OUT;

  LB_RSTAMP(8);
  LB_STAMP(0);
#ifdef RAI_STAMPS
  if ((threadIdx.x & 63) == 0)
    for (int k = 10; k < 32; ++k) g_lb_stamps[blockIdx.x][threadIdx.x >> 6][k] = 0;
#endif
  // ---- stage the weights in LDS (operand permutations for the MFMA chains) -------------------
  {
    // W2 read once, coalesced (element e = tid + LB_NT u, row-major), every load in flight before the
    // first LDS store; each element then lands in both operand permutations:
    //   w2f[m][blk][16 lg + lj][i] = W2[16 m + lj][16 blk + 4 lg + i]
    //   w2b[m][blk][16 lg + lj][i] = W2[16 blk + 4 lg + i][16 m + lj]
    constexpr int PER = HID * HID / LB_NT;
    float wv[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) wv[u] = a.params[base + oW2 + tid + LB_NT * u];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int e = tid + LB_NT * u, r = e >> 6, c = e & 63;
      S.w2f[r >> 4][c >> 4][16 * ((c & 15) >> 2) + (r & 15)][c & 3] = wv[u];
      S.w2b[c >> 4][r >> 4][16 * ((r & 15) >> 2) + (c & 15)][r & 3] = wv[u];
    }
  }
  for (int e = tid; e < HID * 4; e += LB_NT) {
    const int c = e >> 2, f = e & 3;
    S.w1[c][f] = f < IN ? a.params[base + oW1 + c * IN + f] : 0.f;
  }
  if (tid < HID) {
    const float x1 = a.params[base + ob1 + tid], x2 = a.params[base + ob2 + tid];
    S.b1[tid] = x1;
    S.b2[tid] = x2;
    S.b1c[tid] = x1 * LB_2LOG2E;
    S.b2c[tid] = x2 * LB_2LOG2E;
  }
  if (tid < 2 * HID) {
    const int o = tid >> 6, c = tid & 63;
    S.w3[o][c] = o < OUT ? a.params[base + oW3 + o * HID + c] : 0.f;
  }
  if (tid < 4) S.b3[tid] = tid < OUT ? a.params[base + ob3 + tid] : 0.f;

  const rai_ppo_hparams* hp = a.hp;
  const float clip_range = hp->clip_range, ent_coef = hp->ent_coef, vf_coef0 = hp->vf_coef[0];
  const float clip_range_vf = hp->clip_range_vf;
  const bool has_vclip = hp->has_clip_range_vf != 0, huber = hp->vf_loss_fn != 0;
  const float halve = hp->ppo2_vf_coef_halving ? 0.5f : 1.f;
  const float amean = a.moments[0], aden = a.moments[1];
  const float inv_n = a.inv_n;
  __syncthreads();
  LB_STAMP(1);

  // constant per-lane operands: layer-1 A = W1[16 m + j][g].  The W2 permutations (layer 2 / dH1 A
  // operands) stay in LDS; each pipeline phase reads the next phase's block (lb_w2).
  // W3 stays in LDS too: a register copy (32 VGPRs for the actor) pushed the critic path into
  // VGPR<->AGPR shuffles and measured 2% slower.
  float w1a[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) w1a[m] = S.w1[16 * m + j][g];
  auto lb_w2 = [&](const float (&t)[4][4][64][4], int blk, f4 (&wv)[4]) {
#pragma unroll
    for (int m = 0; m < 4; ++m) wv[m] = *reinterpret_cast<const f4*>(&t[m][blk][lane][0]);
  };

  LB_STAMP(2);
  f4 acc2[4][4];  // dW2 tile [mc][mk]: lane (g, j), reg i -> dW2[16 mc + 4 g + i][16 mk + j]
  f4 acc1[4];     // [dW1 | db1] [mj]: lane (g, j = column), reg i -> row 16 mj + 4 g + i
  float aw3[OUT][16], ab2[16], ab3[OUT];
#pragma unroll
  for (int x = 0; x < 4; ++x) {
    acc1[x] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int y = 0; y < 4; ++y) acc2[x][y] = f4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    ab2[k] = 0.f;
#pragma unroll
    for (int o = 0; o < OUT; ++o) aw3[o][k] = 0.f;
  }
#pragma unroll
  for (int o = 0; o < OUT; ++o) ab3[o] = 0.f;
  float st0 = 0.f, st1 = 0.f, st2 = 0.f, st3 = 0.f;  // per-lane sums over its rows (<= a few hundred)

  // ---- the tile pipeline's phases.  Forward (tile k + 1, VALU-heavy): layer 1, layer 2, output layer,
  // loss, backward through the output layer; H1^T and dZ2^T go to the slot's LDS tiles (and dZ2 also in
  // registers to the next step).  Backward (tile k, MFMA-heavy): dH1^T = W2^T dZ2^T, dW2 += dZ2^T H1,
  // [dW1 | db1] += dZ1^T [x | 1] with the rows as the MFMA reduction axis (row 4 g + s of k-step s).
  // Branch-free (invalid rows carry zero gradients).
  auto l1_mfma = [&](const LbIn& in, f4 (&z1)[4]) {
#pragma unroll
    for (int m = 0; m < 4; ++m) z1[m] = mfma4(w1a[m], in.xb, f4{0.f, 0.f, 0.f, 0.f});
  };
  // h = act(z + b[16 m + 4 g + i]); bc: the same bias times 2 log2(e)
  auto act_rows = [&](const f4& z, const float* bias, const float* bc, int m, f4& h) {
    const f4 bb = *reinterpret_cast<const f4*>(&bias[16 * m + 4 * g]);
    const f4 cc = *reinterpret_cast<const f4*>(&bc[16 * m + 4 * g]);
#pragma unroll
    for (int i = 0; i < 4; ++i) h[i] = lb_act_bias<RELU>(z[i], bb[i], cc[i]);
  };
  auto put_t = [&](float(*t)[LB_TS], const f4& v, int m) {  // T-layout registers -> [c][row] tile
#pragma unroll
    for (int i = 0; i < 4; ++i) t[16 * m + 4 * g + i][j] = v[i];
  };
  auto dh1_blk = [&](const f4 (&dz2)[4], int blk, const f4 (&wv)[4], f4 (&dh1)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int m = 0; m < 4; ++m) dh1[m] = mfma4(wv[m][i], dz2[blk][i], dh1[m]);
  };
  auto l2_blk = [&](const f4 (&h1)[4], int blk, const f4 (&wv)[4], f4 (&z2)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int m = 0; m < 4; ++m) z2[m] = mfma4(wv[m][i], h1[blk][i], z2[m]);
  };
  auto dw2_s = [&](const f4 (&ar)[4], const f4 (&br)[4], int s) {
#pragma unroll
    for (int mc = 0; mc < 4; ++mc)
#pragma unroll
      for (int mk = 0; mk < 4; ++mk) acc2[mc][mk] = mfma4(ar[mc][s], br[mk][s], acc2[mc][mk]);
  };
  auto out_layer = [&](const f4 (&h2)[4], float (&zo)[OUT]) {
#pragma unroll
    for (int o = 0; o < OUT; ++o) {
      float p[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) {  // four independent chains, summed in a fixed order
        const f4 wv = *reinterpret_cast<const f4*>(&S.w3[o][16 * m + 4 * g]);
        p[m] = h2[m][0] * wv[0];
#pragma unroll
        for (int i = 1; i < 4; ++i) p[m] = fmaf(h2[m][i], wv[i], p[m]);
      }
      zo[o] = lb_sum_groups((p[0] + p[1]) + (p[2] + p[3])) + S.b3[o];
    }
  };
  // loss per row (ppo.py:326-371; the min/max tie rules of loss.hip): gradient w.r.t. the outputs
  auto loss = [&](const LbIn& in, const float (&zo)[OUT], float& d0, float& d1) {
    const bool valid = in.valid;
    const bool count = valid && g == 0;
    d1 = 0.f;
    if (ACTOR) {
      const float z0 = zo[0], z1 = zo[OUT - 1];
      const float mx = fmaxf(z0, z1);
      const float lse = mx + lb_log(lb_exp(z0 - mx) + lb_exp(z1 - mx));
      const float n0 = z0 - lse, n1 = z1 - lse;
      const float p0 = lb_exp(n0), p1 = lb_exp(n1);
      const float H = -(fmaxf(n0, F32_MIN) * p0) - fmaxf(n1, F32_MIN) * p1;
      const bool a1 = in.act == 1;
      const float logp = a1 ? n1 : n0;
      const float A = (in.u1 - amean) / aden;
      const float logratio = logp - in.u0;
      const float ratio = lb_exp(logratio);
      const float lo = 1.f - clip_range, hi = 1.f + clip_range;
      const float cr = fminf(fmaxf(ratio, lo), hi);
      const float s1 = ratio * A, s2 = cr * A;
      const float gpi = -inv_n;
      const float g1 = s1 < s2 ? gpi : (s1 > s2 ? 0.f : gpi * 0.5f);
      const float g2 = s1 < s2 ? 0.f : (s1 > s2 ? gpi : gpi * 0.5f);
      const float in_clip = (ratio >= lo && ratio <= hi) ? 1.f : 0.f;
      const float dlogp = (g1 * A + (g2 * A) * in_clip) * ratio;
      const float dent = -ent_coef * inv_n;
      d0 = dlogp * ((a1 ? 0.f : 1.f) - p0) + dent * (-p0 * (n0 + H));
      d1 = dlogp * ((a1 ? 1.f : 0.f) - p1) + dent * (-p1 * (n1 + H));
      d0 = valid ? d0 : 0.f;
      d1 = valid ? d1 : 0.f;
      st0 += count ? fminf(s1, s2) : 0.f;
      st1 += count ? (ratio - 1.f) - logratio : 0.f;
      st2 += (count && fabsf(ratio - 1.f) > clip_range) ? 1.f : 0.f;
      st3 += count ? H : 0.f;
    } else {
      const float v = zo[0], R = in.u1, vo = in.u0;
      const float gl = (vf_coef0 * halve) * inv_n;
      auto vloss = [&](float x) -> float {
        const float z = fabsf(x);
        return huber ? (z < 1.f ? 0.5f * z * z : (z - 0.5f)) : x * x;
      };
      auto vgrad = [&](float x) -> float {
        return huber ? (x <= -1.f ? -1.f : (x >= 1.f ? 1.f : x)) : 2.f * x;
      };
      const float e = v - R;
      const float l1 = vloss(e);
      const float dvo = v - vo;
      const float vcl = vo + fminf(fmaxf(dvo, -clip_range_vf), clip_range_vf);
      const float l2 = vloss(vcl - R);
      const float w1 = l1 > l2 ? gl : (l1 < l2 ? 0.f : gl * 0.5f);
      const float w2 = l1 > l2 ? 0.f : (l1 < l2 ? gl : gl * 0.5f);
      const float inside = (dvo >= -clip_range_vf && dvo <= clip_range_vf) ? 1.f : 0.f;
      const float dv_c = w1 * vgrad(e) + (w2 * vgrad(vcl - R)) * inside;
      const float dv = has_vclip ? dv_c : gl * vgrad(e);
      d0 = valid ? dv : 0.f;
      st0 += count ? (has_vclip ? fmaxf(l1, l2) : l1) : 0.f;
      st1 += (count && has_vclip && fabsf(v - vo) > clip_range_vf) ? 1.f : 0.f;
    }
  };
  // backward through the output layer for hidden block m: dZ2 = (W3^T d) * act'(H2); dW3, db2 partials
  auto out_bwd = [&](const f4& h2m, int m, float d0, float d1, f4& dz) {
    const f4 wa = *reinterpret_cast<const f4*>(&S.w3[0][16 * m + 4 * g]);
    const f4 wb = *reinterpret_cast<const f4*>(&S.w3[OUT - 1][16 * m + 4 * g]);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float h = h2m[i];
      const float dh = ACTOR ? fmaf(d1, wb[i], d0 * wa[i]) : d0 * wa[i];
      aw3[0][4 * m + i] = fmaf(d0, h, aw3[0][4 * m + i]);
      if (ACTOR) aw3[OUT - 1][4 * m + i] = fmaf(d1, h, aw3[OUT - 1][4 * m + i]);
      dz[i] = dh * lb_act_d<RELU>(h);
      ab2[4 * m + i] += dz[i];
    }
  };
  // the forward of one tile without interleaving (the pipeline's prologue)
  auto forward_alone = [&](const LbIn& in, float(*hs)[LB_TS], float(*tdz)[LB_TS], f4 (&dz2)[4]) {
    f4 z1[4], h1[4], z2[4], h2[4];
    l1_mfma(in, z1);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      act_rows(z1[m], S.b1, S.b1c, m, h1[m]);
      put_t(hs, h1[m], m);
      z2[m] = f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int blk = 0; blk < 4; ++blk) {
      f4 wv[4];
      lb_w2(S.w2f, blk, wv);
      l2_blk(h1, blk, wv, z2);
    }
#pragma unroll
    for (int m = 0; m < 4; ++m) act_rows(z2[m], S.b2, S.b2c, m, h2[m]);
    float zo[OUT], d0, d1;
    out_layer(h2, zo);
    loss(in, zo, d0, d1);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      out_bwd(h2[m], m, d0, d1, dz2[m]);
      put_t(tdz, dz2[m], m);
    }
    ab3[0] += d0;
    if (ACTOR) ab3[OUT - 1] += d1;
  };

  // One pipeline step: tile k's backward (slot B) beside tile k + 1's forward (slot F), hand-scheduled
  // as short regions (sched_barrier fences) that each pair one MFMA block with an independent VALU chunk;
  // the compiler interleaves inside a region.  dZ2 of tile k arrives in registers; dZ2 of tile k + 1
  // leaves in the same registers.
  auto step = [&](const LbIn& inF, float(*tdzF)[LB_TS], float(*hsF)[LB_TS], int tB, float(*tdzB)[LB_TS],
                  float(*hsB)[LB_TS], f4 (&dz2)[4]) {
#ifdef RAI_STAMPS
    unsigned long long tr = __builtin_amdgcn_s_memtime();
    int ph = 10;
#endif
    float xw[4];
    lb_load_xw(a, tB, g, j, xw);
    f4 z1[4], h1[4], dh1[4], z2[4], h2[4], ar[4], br[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      dh1[m] = f4{0.f, 0.f, 0.f, 0.f};
      z2[m] = f4{0.f, 0.f, 0.f, 0.f};
    }
    f4 wa[4], wb[4];
    lb_w2(S.w2b, 0, wa);
    l1_mfma(inF, z1);
    LB_FENCE();
    LB_PH();
    dh1_blk(dz2, 0, wa, dh1);  // P1
    lb_w2(S.w2b, 1, wb);
    act_rows(z1[0], S.b1, S.b1c, 0, h1[0]);
    act_rows(z1[1], S.b1, S.b1c, 1, h1[1]);
    LB_FENCE();
    LB_PH();
    dh1_blk(dz2, 1, wb, dh1);  // P2
    lb_w2(S.w2b, 2, wa);
    act_rows(z1[2], S.b1, S.b1c, 2, h1[2]);
    act_rows(z1[3], S.b1, S.b1c, 3, h1[3]);
    LB_FENCE();
    LB_PH();
    dh1_blk(dz2, 2, wa, dh1);  // P3
    lb_w2(S.w2b, 3, wb);
#pragma unroll
    for (int m = 0; m < 4; ++m) put_t(hsF, h1[m], m);
    LB_FENCE();
    LB_PH();
    dh1_blk(dz2, 3, wb, dh1);  // P4
    lb_w2(S.w2f, 0, wa);
    LB_FENCE();
    LB_PH();
    l2_blk(h1, 0, wa, z2);  // P5: layer 2 beside the dH1 transpose and the dW2 / dW1 operand reads
    lb_w2(S.w2f, 1, wb);
#pragma unroll
    for (int m = 0; m < 4; ++m) put_t(tdzF, dh1[m], m);  // dH1 through the forward slot's dZ2 tile
    LB_FENCE();
    LB_PH();
    l2_blk(h1, 1, wb, z2);
    lb_w2(S.w2f, 2, wa);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      ar[m] = *reinterpret_cast<const f4*>(&tdzB[16 * m + j][4 * g]);
      br[m] = *reinterpret_cast<const f4*>(&hsB[16 * m + j][4 * g]);
    }
    LB_FENCE();
    LB_PH();
    l2_blk(h1, 2, wa, z2);
    lb_w2(S.w2f, 3, wb);
    f4 az[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const f4 d = *reinterpret_cast<const f4*>(&tdzF[16 * m + j][4 * g]);
#pragma unroll
      for (int s = 0; s < 4; ++s) az[m][s] = d[s] * lb_act_d<RELU>(br[m][s]);
    }
    LB_FENCE();
    LB_PH();
    l2_blk(h1, 3, wb, z2);
    LB_FENCE();
    LB_PH();
    dw2_s(ar, br, 0);  // P6
    act_rows(z2[0], S.b2, S.b2c, 0, h2[0]);
    act_rows(z2[1], S.b2, S.b2c, 1, h2[1]);
    LB_FENCE();
    LB_PH();
    dw2_s(ar, br, 1);  // P7
    act_rows(z2[2], S.b2, S.b2c, 2, h2[2]);
    act_rows(z2[3], S.b2, S.b2c, 3, h2[3]);
    LB_FENCE();
    LB_PH();
    float zo[OUT], d0, d1;
    dw2_s(ar, br, 2);  // P8
    out_layer(h2, zo);
    LB_FENCE();
    LB_PH();
    dw2_s(ar, br, 3);  // P9
    loss(inF, zo, d0, d1);
    LB_FENCE();
    LB_PH();
#pragma unroll
    for (int s = 0; s < 4; ++s)  // P10: [dW1 | db1] beside the output layer's backward
#pragma unroll
      for (int m = 0; m < 4; ++m) acc1[m] = mfma4(az[m][s], xw[s], acc1[m]);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      out_bwd(h2[m], m, d0, d1, dz2[m]);
      put_t(tdzF, dz2[m], m);
    }
    ab3[0] += d0;
    if (ACTOR) ab3[OUT - 1] += d1;
    LB_FENCE();
    LB_PH();
  };

  // ---- two-stage software pipeline over the wave's tiles; tiles past the end are all-invalid (zero
  // gradients, never back-propagated).  Slots alternate; the loop body is unrolled over both.
  const int n_tiles = (a.rows + 15) >> 4;
  const int wave_id = wgn * LB_NW + w;
  const int n_my = wave_id < n_tiles ? (n_tiles - 1 - wave_id) / LB_WAVES_PER_NET + 1 : 0;
  float(*tdz0)[LB_TS] = S.tdz0[w];
  float(*tdz1)[LB_TS] = S.tdz1[w];
  float(*hs0)[LB_TS] = S.hs0[w];
  float(*hs1)[LB_TS] = S.hs1[w];
  if (n_my > 0) {
    LbIn in, nx;
    lb_load<ACTOR>(a, wave_id, g, j, in);
    lb_load<ACTOR>(a, wave_id + LB_WAVES_PER_NET, g, j, nx);
    f4 dz2[4];  // the forward stage's dZ2 tile, handed to the next step's dH1
    forward_alone(in, hs0, tdz0, dz2);  // prologue: tile 0's forward
    for (int k = 0; k < n_my; ++k) {
      const int t = wave_id + k * LB_WAVES_PER_NET;
      const bool odd = (k & 1) != 0;  // tile k's slot (backward) is k & 1, tile k + 1's (forward) the other
      in = nx;
      lb_load<ACTOR>(a, t + 2 * LB_WAVES_PER_NET, g, j, nx);
      step(in, odd ? tdz0 : tdz1, odd ? hs0 : hs1, t, odd ? tdz1 : tdz0, odd ? hs1 : hs0, dz2);
    }
  }

  // ---- per-wave sums over the 16 row lanes, then the workgroup's partial in wave order -----------
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    ab2[k] = lb_row_sum16(ab2[k]);
#pragma unroll
    for (int o = 0; o < OUT; ++o) aw3[o][k] = lb_row_sum16(aw3[o][k]);
  }
#pragma unroll
  for (int o = 0; o < OUT; ++o) ab3[o] = lb_row_sum16(ab3[o]);
  {
    double s[4] = {(double)st0, (double)st1, (double)st2, (double)st3};
#pragma unroll
    for (int q = 0; q < 4; ++q) s[q] = wave_sum(s[q]);
    if (lane == 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q) S.st[w][q] = s[q];
    }
  }
  // each wave stores its partial into a region of its own (plain stores: no read-modify-write chain),
  // then every thread sums the regions in wave order
  float* accv = &S.hs0[0][0][0];
  static_assert(sizeof(float) * LB_NW * LB_PSTRIDE <= sizeof(float) * 4 * LB_NW * HID * LB_TS, "regions fit");
  LB_STAMP(4);
  __syncthreads();  // every wave is past its last tile: the transpose tiles become the partial regions
  {
    float* mine = accv + w * LB_PSTRIDE;
#pragma unroll
    for (int mc = 0; mc < 4; ++mc)
#pragma unroll
      for (int mk = 0; mk < 4; ++mk)
#pragma unroll
        for (int i = 0; i < 4; ++i) mine[oW2 + (16 * mc + 4 * g + i) * HID + 16 * mk + j] = acc2[mc][mk][i];
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = 16 * m + 4 * g + i;
        if (j < IN) mine[oW1 + c * IN + j] = acc1[m][i];
        else if (j == 4) mine[ob1 + c] = acc1[m][i];
      }
    if (j == 0) {
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int c = 16 * m + 4 * g + i;
          mine[ob2 + c] = ab2[4 * m + i];
#pragma unroll
          for (int o = 0; o < OUT; ++o) mine[oW3 + o * HID + c] = aw3[o][4 * m + i];
        }
    }
    if (lane == 0) {
#pragma unroll
      for (int o = 0; o < OUT; ++o) mine[ob3 + o] = ab3[o];
    }
  }
  __syncthreads();
  LB_STAMP(5);
  const int slot = (ACTOR ? 0 : LB_WG_PER_NET) + wgn;
  float* dst = a.part + (int64_t)slot * LB_PSTRIDE;
  for (int e = tid; e < P_net; e += LB_NT) {
    float v = accv[e];
#pragma unroll
    for (int r = 1; r < LB_NW; ++r) v += accv[r * LB_PSTRIDE + e];
    dst[e] = v;
  }
  if (tid < 4) {
    double s = 0.0;
    for (int r = 0; r < LB_NW; ++r) s += S.st[r][tid];
    a.statp[slot * 4 + tid] = s;
  }
  LB_STAMP(6);
  LB_RSTAMP(9);
}

template <int RELU>
__global__ __launch_bounds__(LB_NT, 1) void lb_grads_kernel(LbArgs a) {
  extern __shared__ __align__(16) unsigned char lb_lds[];
  LbSmem& S = *reinterpret_cast<LbSmem*>(lb_lds);
  const int net = blockIdx.x & 1, wgn = blockIdx.x >> 1;
  if (net == 0) lb_net<RELU, true>(a, S, wgn);
  else lb_net<RELU, false>(a, S, wgn);
}

// Cross-GPU exchange layout of the large-minibatch reduce (data parallel, rai_mlp_ppo_epoch_xdp at batch
// > 256), inside each rank's IPC-mapped region past the words the setup canary writes (common.h; the
// canary's payload floats sit at [RAI_XDP_SLOTS_OFF, +2 KB): flag words there would read as huge step
// ids and never wait -- the flags are never re-zeroed, so they must live where only step ids are stored):
//   [LB_XF_OFF, +16 KB)  u64 flags[reduce block][sender rank]: step id of the last block pushed
//   [LB_XS_OFF, ...)     f32 slots[2 parities][world][LB_XSLOT]: each rank's reduced gradient of the step,
//                        64 parameters per reduce block
constexpr int LB_XMAXW = 8;
constexpr int LB_MAX_P = 2 * LB_PSTRIDE;
constexpr int LB_RED_MAX_BLOCKS = (LB_MAX_P + 63) / 64;
constexpr int64_t LB_XF_OFF = RAI_XDP_SLOTS_OFF + 4096;
constexpr int64_t LB_XS_OFF = LB_XF_OFF + 16384;
constexpr int LB_XSLOT = LB_RED_MAX_BLOCKS * 64;
constexpr int LB_XAUX = 17;  // sc0 | sc1: system-scope (cross-device) stores and loads
static_assert(LB_RED_MAX_BLOCKS * LB_XMAXW * 8 <= 16384, "flag words fit");
__host__ __device__ constexpr int64_t lb_xdp_bytes(int world) {
  return LB_XS_OFF + 2LL * world * LB_XSLOT * (int64_t)sizeof(float);
}

struct LbRed {
  const float* part;
  const double* statp;
  float* grad;           // the minibatch gradient (flat parameter order)
  double* sq_part;       // per-block fp64 squared-norm partials (epoch mode), or nullptr
  rai_train_state* state;
  float* stats;
  const rai_ppo_hparams* hp;
  int32_t P;
  int32_t szA;
  int32_t max_stats;
  int32_t bump_step;     // epoch mode: advance state->opt_step (read by the optimizer launch)
  double n_total;        // rows * world
  // data parallel over the exchange regions (xworld > 1): this step's id and slot parity
  void* const* xpeers;
  int32_t xrank;
  int32_t xworld;
  unsigned long long xstep;
};

// The exchange of one reduce block (wave 0 of it): this rank's 64 summed values (tot) go into slot
// [parity][xrank] of EVERY rank's region (16-B system-scope stores: 16 lanes x 16 B), the wave drains,
// one flag word per receiver; then the W flags of this block in the own region are polled and the W
// slots summed in rank order (the same bits on every rank).  Slot reuse: a rank writes parity p again
// two steps later, only after its own step in between passed this wait, i.e. after every peer pushed
// that step -- which each peer does only after it finished summing the parity-p slots.
__device__ void lb_exchange_block(const LbRed& r, float* tot) {
  const int lane = threadIdx.x & 63;
  const int W = r.xworld;
  const int par = (int)((r.xstep - 1) & 1);
  const int64_t rb = lb_xdp_bytes(W);
  const int64_t slot0 = LB_XS_OFF + ((int64_t)par * W * LB_XSLOT + (int64_t)blockIdx.x * 64) * 4;
  f4 mine = {0.f, 0.f, 0.f, 0.f};
  if (lane < 16) mine = reinterpret_cast<const f4*>(tot)[lane];
  for (int pr = 0; pr < W; ++pr) {
    const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(r.xpeers[pr], (short)0, (int)rb, 0x00020000);
    if (lane < 16)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v_lb, mine), prs,
                                             (int)(slot0 + (int64_t)r.xrank * LB_XSLOT * 4) + 16 * lane, 0, LB_XAUX);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the slot stores landed before any flag
  if (lane < W) {
    unsigned long long* fl = reinterpret_cast<unsigned long long*>(static_cast<char*>(r.xpeers[lane]) + LB_XF_OFF) +
                             blockIdx.x * LB_XMAXW + r.xrank;
    __hip_atomic_store(fl, r.xstep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  const unsigned long long* own =
      reinterpret_cast<const unsigned long long*>(static_cast<const char*>(r.xpeers[r.xrank]) + LB_XF_OFF) +
      blockIdx.x * LB_XMAXW;
  const unsigned long long t0 = rai_clock();
  for (;;) {
    const bool ok = lane >= W || __hip_atomic_load(own + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= r.xstep;
    if (__all(ok)) break;
    if (rai_expired(t0, RAI_SPIN_REMOTE)) {
      if (lane == 0) atomicExch(&r.state->err, 1);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  const __amdgpu_buffer_rsrc_t lrs = __builtin_amdgcn_make_buffer_rsrc(r.xpeers[r.xrank], (short)0, (int)rb, 0x00020000);
  f4 sum = {0.f, 0.f, 0.f, 0.f};
  if (lane < 16) {
    sum = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(lrs, (int)slot0 + 16 * lane, 0, LB_XAUX));
    for (int pr = 1; pr < W; ++pr)
      sum += __builtin_bit_cast(
          f4, __builtin_amdgcn_raw_buffer_load_b128(lrs, (int)(slot0 + (int64_t)pr * LB_XSLOT * 4) + 16 * lane, 0, LB_XAUX));
    reinterpret_cast<f4*>(tot)[lane] = sum;
  }
}

// Every parameter's LB_WG_PER_NET workgroup partials in a fixed order: a block owns 64 parameters and
// its four waves each sum one quarter of the partials (32 independent loads in flight per lane; one
// wave per parameter column with all 128 loads behind each other measured 17 us per launch), then wave
// 0 adds the quarters in order.  Block 0 also writes the minibatch's stats row (ppo.py:379-396 means;
// row[0] is the policy + entropy part, the host adds the value term, as for rai_mlp_ppo_epoch).
__global__ __launch_bounds__(LB_RED_NT) void lb_reduce_kernel(LbRed r) {
  __shared__ float quarter[LB_RED_NT / 64][64];
  const int c = threadIdx.x & 63, q4 = threadIdx.x >> 6;
  const int p = blockIdx.x * 64 + c;
  if (p < r.P) {
    const int net = p >= r.szA ? 1 : 0;
    const int loc = p - (net ? r.szA : 0);
    constexpr int KQ = LB_WG_PER_NET / (LB_RED_NT / 64);
    const float* src = r.part + ((int64_t)net * LB_WG_PER_NET + q4 * KQ) * LB_PSTRIDE + loc;
    float v[KQ];
#pragma unroll
    for (int k = 0; k < KQ; ++k) v[k] = src[(int64_t)k * LB_PSTRIDE];
#pragma unroll
    for (int w = KQ / 2; w >= 1; w /= 2)
#pragma unroll
      for (int k = 0; k < w; ++k) v[k] = v[k] + v[k + w];
    quarter[q4][c] = v[0];
  }
  __syncthreads();
  double sq = 0.0;
  if (r.xworld > 1) {  // data parallel: the block's 64 sums over every rank, in rank order
    __shared__ __align__(16) float tot[64];
    if (q4 == 0) tot[c] = p < r.P ? (quarter[0][c] + quarter[1][c]) + (quarter[2][c] + quarter[3][c]) : 0.f;
    __syncthreads();
    if (q4 == 0) lb_exchange_block(r, tot);
    __syncthreads();
    if (q4 == 0) quarter[0][c] = tot[c], quarter[1][c] = quarter[2][c] = quarter[3][c] = 0.f;
    __syncthreads();
  }
  if (q4 == 0) {
    if (p < r.P) {
      const float v = r.xworld > 1 ? quarter[0][c] : (quarter[0][c] + quarter[1][c]) + (quarter[2][c] + quarter[3][c]);
      r.grad[p] = v;
      sq = (double)v * (double)v;
    }
    if (r.sq_part) {
      sq = wave_sum(sq);
      if (c == 0) r.sq_part[blockIdx.x] = sq;
    }
  }
  if (blockIdx.x != 0) return;
  // stats: threads 0..3 the actor's four sums, 4..5 the critic's two, each in workgroup order
  __shared__ double tot[6];
  if (threadIdx.x < 6) {
    const int net = threadIdx.x < 4 ? 0 : 1, q = threadIdx.x < 4 ? threadIdx.x : threadIdx.x - 4;
    double t = 0.0;
    for (int k = 0; k < LB_WG_PER_NET; ++k) t += r.statp[(net * LB_WG_PER_NET + k) * 4 + q];
    tot[threadIdx.x] = t;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int idx = r.state->stat_index;
    if (r.stats && idx < r.max_stats) {
      const float halve = r.hp->ppo2_vf_coef_halving ? 0.5f : 1.f;
      const double Bd = r.n_total;
      float* row = r.stats + (int64_t)idx * RAI_STAT_STRIDE;
      const float pi_loss = (float)(-tot[0] / Bd);
      const float ent_loss = (float)(-tot[3] / Bd);
      row[0] = pi_loss + r.hp->ent_coef * ent_loss;  // host adds the value term
      row[1] = pi_loss;
      row[2] = ent_loss;
      row[3] = (float)(tot[1] / Bd);
      row[4] = (float)(tot[2] / Bd);
      row[5] = (float)(tot[4] / Bd) * halve;
      row[5 + RAI_MAX_K] = r.hp->has_clip_range_vf ? (float)(tot[5] / Bd) : 0.f;
    }
    r.state->stat_index = idx + 1;
    if (r.bump_step) r.state->opt_step += 1;
  }
}

// Advantage moments of every minibatch of the epoch: fp64 (sum, sum of squares) per chunk, then per
// minibatch mean (rounded to f32, as torch's f32 A.mean()) and unbiased std + 1e-8, encoded with the
// normalize / standardize choice as adv_moments_kernel (mlp_ppo.hip) does.
__global__ __launch_bounds__(256) void lb_moments_part_kernel(const float* __restrict__ adv, int64_t n_rows, int B,
                                                              double* mp) {
  __shared__ double red[2 * 4];
  const int mb = blockIdx.y, ch = blockIdx.x;
  const int64_t row0 = (int64_t)mb * B;
  const int64_t rows = min((int64_t)B, n_rows - row0);
  const int64_t lo = rows * ch / LB_MOMP, hi = rows * (ch + 1) / LB_MOMP;
  double s1 = 0.0, s2 = 0.0;
  for (int64_t i = lo + threadIdx.x; i < hi; i += 256) {
    const double x = (double)adv[row0 + i];
    s1 += x;
    s2 += x * x;
  }
  double v[2] = {s1, s2};
  block_sum<2>(v, red);
  if (threadIdx.x == 0) {
    mp[((int64_t)mb * LB_MOMP + ch) * 2] = v[0];
    mp[((int64_t)mb * LB_MOMP + ch) * 2 + 1] = v[1];
  }
}

__global__ __launch_bounds__(64) void lb_moments_final_kernel(const double* __restrict__ mp, int64_t n_rows, int B,
                                                              const rai_ppo_hparams* hp, float* moments) {
  const int mb = blockIdx.x;
  if (threadIdx.x != 0) return;
  const int64_t rows = min((int64_t)B, n_rows - (int64_t)mb * B);
  double s1 = 0.0, s2 = 0.0;
  for (int c = 0; c < LB_MOMP; ++c) {
    s1 += mp[((int64_t)mb * LB_MOMP + c) * 2];
    s2 += mp[((int64_t)mb * LB_MOMP + c) * 2 + 1];
  }
  const double n = (double)rows;
  const double md = s1 / n;
  const float mean = (float)md;
  const double var = fmax(s2 - n * md * md, 0.0) / (n - 1.0);
  const float den = (float)sqrt(var) + 1e-8f;
  float m0 = 0.f, m1 = 1.f;
  if (hp->normalize_advantage) { m0 = mean; m1 = den; }
  else if (hp->standardize_advantage) { m1 = den; }
  moments[2 * mb] = m0;
  moments[2 * mb + 1] = m1;
}

// ---- workspace -------------------------------------------------------------------------------
int64_t align256(int64_t b) { return (b + 255) / 256 * 256; }
struct LbWs {
  float* moments;
  double* momp;
  double* statp;
  double* sq;
  float* grad;
  float* part;
};
LbWs lb_carve(void* ws, int64_t nmb) {
  unsigned char* p = static_cast<unsigned char*>(ws);
  LbWs w;
  w.moments = reinterpret_cast<float*>(p);
  p += align256(8 * nmb);
  w.momp = reinterpret_cast<double*>(p);
  p += align256(16 * nmb * LB_MOMP);
  w.statp = reinterpret_cast<double*>(p);
  p += align256(8 * 4 * LB_GRID);
  w.sq = reinterpret_cast<double*>(p);
  p += align256(8 * LB_RED_MAX_BLOCKS);
  w.grad = reinterpret_cast<float*>(p);
  p += align256(4 * LB_MAX_P);
  w.part = reinterpret_cast<float*>(p);
  return w;
}

int lb_allow_lds(const void* kernel) {
  static std::mutex mu;
  static std::vector<const void*> done;
  std::lock_guard<std::mutex> lock(mu);
  for (const void* k : done)
    if (k == kernel) return RAI_OK;
  const hipError_t e = hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(LbSmem));
  if (e != hipSuccess) return (int)e;
  done.push_back(kernel);
  return RAI_OK;
}

// Timing hook (bench.py's roofline): HIP events around every lb_grads_kernel launch while armed.
struct LbTiming {
  std::mutex mu;
  std::vector<hipEvent_t> ev;  // pairs
  int next = 0;
  int cap = 0;
};
LbTiming& lb_timing() {
  static LbTiming t;
  return t;
}

}  // namespace

int64_t rai_internal::mlp_large_xdp_bytes(int32_t world) { return lb_xdp_bytes(world); }

bool rai_internal::mlp_large_supported(int32_t in_dim, int32_t n_act, int32_t hidden) {
  return hidden == HID && in_dim >= 1 && in_dim <= 4 && n_act == 2;
}

int64_t rai_internal::mlp_large_workspace_bytes(int64_t n_rows, int32_t batch) {
  const int64_t nmb = batch > 0 ? (n_rows + batch - 1) / batch : 0;
  return align256(8 * nmb) + align256(16 * nmb * LB_MOMP) + align256(8 * 4 * LB_GRID) +
         align256(8 * LB_RED_MAX_BLOCKS) + align256(4 * LB_MAX_P) + (int64_t)LB_GRID * LB_PSTRIDE * 4;
}

int rai_internal::mlp_large(float* params, float* exp_avg, float* exp_avg_sq, const float* obs,
                            const int64_t* actions, const float* old_logp, const float* old_values, const float* adv,
                            const float* ret, int64_t n_rows, int32_t batch, int32_t in_dim, int32_t n_act,
                            int32_t act_fn, int32_t mb_begin, int32_t mb_count, const float* moments, int32_t world,
                            const rai_ppo_hparams* hp, const rai_optim_hparams* ohp, rai_train_state* state,
                            float* stats, int32_t max_stats, float* norms, int32_t max_norms, float* grad_out,
                            void* workspace, int64_t workspace_bytes, hipStream_t s, const LargeXdp* xdp) {
  if (!mlp_large_supported(in_dim, n_act, HID)) return RAI_E_UNSUPPORTED;
  if (xdp && (grad_out || !moments || !xdp->peers || xdp->world < 2 || xdp->world > LB_XMAXW || xdp->rank < 0 ||
              xdp->rank >= xdp->world || xdp->world != world || xdp->step_base < 0))
    return RAI_E_SHAPE;
  if (batch < 2 || n_rows < 1 || world < 1 || (act_fn != 0 && act_fn != 1)) return RAI_E_SHAPE;
  if (!params || !obs || !actions || !old_logp || !old_values || !adv || !ret || !hp || !state || !workspace)
    return RAI_E_NULLPTR;
  const bool grads_mode = grad_out != nullptr;
  if (!grads_mode && (!exp_avg || !exp_avg_sq || !ohp)) return RAI_E_NULLPTR;
  if (workspace_bytes < mlp_large_workspace_bytes(n_rows, batch)) return RAI_E_WORKSPACE;
  const int64_t nmb = (n_rows + batch - 1) / batch;
  if (grads_mode && (mb_count != 1 || mb_begin < 0 || mb_begin >= nmb || !moments)) return RAI_E_SHAPE;
  if (!moments && n_rows % batch == 1) return RAI_E_SHAPE;  // a 1-row minibatch has no unbiased std
  const int szA = HID * in_dim + HID + HID * HID + HID + 2 * HID + 2;
  const int P = szA + HID * in_dim + HID + HID * HID + HID + HID + 1;
  LbWs w = lb_carve(workspace, nmb);
  int e = act_fn ? lb_allow_lds(reinterpret_cast<const void*>(&lb_grads_kernel<1>))
                 : lb_allow_lds(reinterpret_cast<const void*>(&lb_grads_kernel<0>));
  if (e != RAI_OK) return e;
  const float* mom = moments;
  if (!mom) {
    hipLaunchKernelGGL(lb_moments_part_kernel, dim3(LB_MOMP, (unsigned)nmb), dim3(256), 0, s, adv, n_rows, batch,
                       w.momp);
    RAI_LAUNCH_CHECK();
    hipLaunchKernelGGL(lb_moments_final_kernel, dim3((unsigned)nmb), dim3(64), 0, s, w.momp, n_rows, batch, hp,
                       w.moments);
    RAI_LAUNCH_CHECK();
    mom = w.moments;
  }
  const int red_blocks = (P + 63) / 64;
  const int64_t mb_end = grads_mode ? mb_begin + 1 : nmb;
  for (int64_t mb = grads_mode ? mb_begin : 0; mb < mb_end; ++mb) {
    LbArgs a;
    a.params = params;
    a.obs = obs;
    a.actions = actions;
    a.old_logp = old_logp;
    a.old_values = old_values;
    a.adv = adv;
    a.ret = ret;
    a.moments = mom + 2 * mb;
    a.hp = hp;
    a.part = w.part;
    a.statp = w.statp;
    a.row0 = mb * batch;
    a.rows = (int32_t)std::min<int64_t>(batch, n_rows - mb * batch);
    a.in_dim = in_dim;
    a.inv_n = 1.f / (float)((int64_t)a.rows * world);
    LbTiming& tm = lb_timing();
    hipEvent_t e0 = nullptr, e1 = nullptr;
    {
      std::lock_guard<std::mutex> lock(tm.mu);
      if (tm.next < tm.cap) {
        e0 = tm.ev[2 * tm.next];
        e1 = tm.ev[2 * tm.next + 1];
        ++tm.next;
      }
    }
    if (e0) (void)hipEventRecord(e0, s);
    if (act_fn) hipLaunchKernelGGL(lb_grads_kernel<1>, dim3(LB_GRID), dim3(LB_NT), sizeof(LbSmem), s, a);
    else hipLaunchKernelGGL(lb_grads_kernel<0>, dim3(LB_GRID), dim3(LB_NT), sizeof(LbSmem), s, a);
    RAI_LAUNCH_CHECK();
    if (e1) (void)hipEventRecord(e1, s);
    LbRed r;
    r.part = w.part;
    r.statp = w.statp;
    r.grad = grads_mode ? grad_out : w.grad;
    r.sq_part = grads_mode ? nullptr : w.sq;
    r.state = state;
    r.stats = stats;
    r.hp = hp;
    r.P = P;
    r.szA = szA;
    r.max_stats = max_stats;
    r.bump_step = grads_mode ? 0 : 1;
    r.n_total = (double)a.rows * (double)world;
    r.xpeers = xdp ? xdp->peers : nullptr;
    r.xrank = xdp ? xdp->rank : 0;
    r.xworld = xdp ? xdp->world : 1;
    r.xstep = xdp ? (unsigned long long)(xdp->step_base + (mb - (grads_mode ? mb_begin : 0)) + 1) : 0ull;
    hipLaunchKernelGGL(lb_reduce_kernel, dim3(red_blocks), dim3(LB_RED_NT), 0, s, r);
    RAI_LAUNCH_CHECK();
    if (!grads_mode) {
      e = rai_internal::optim_apply_partials(params, w.grad, exp_avg, exp_avg_sq, P, ohp, state, w.sq, red_blocks,
                                             norms, max_norms, s);
      if (e != RAI_OK) return e;
    }
  }
  return RAI_OK;
}

#ifdef RAI_STAMPS
extern "C" int rai_mlp_large_debug_stamps(unsigned long long* host_out) {  // LB_GRID x LB_NW x 32
  return (int)hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_lb_stamps), sizeof(g_lb_stamps));
}
#endif

extern "C" int rai_mlp_large_timing(int32_t capacity) {
  LbTiming& t = lb_timing();
  std::lock_guard<std::mutex> lock(t.mu);
  if (capacity < 0) return RAI_E_SHAPE;
  for (hipEvent_t ev : t.ev) (void)hipEventDestroy(ev);
  t.ev.clear();
  t.next = 0;
  t.cap = 0;
  for (int i = 0; i < 2 * capacity; ++i) {
    hipEvent_t ev;
    const hipError_t e = hipEventCreate(&ev);
    if (e != hipSuccess) return (int)e;
    t.ev.push_back(ev);
  }
  t.cap = capacity;
  return RAI_OK;
}

extern "C" int rai_mlp_large_timing_read(float* ms_out, int32_t max_out, int32_t* count_out) {
  if (!ms_out || !count_out) return RAI_E_NULLPTR;
  LbTiming& t = lb_timing();
  std::lock_guard<std::mutex> lock(t.mu);
  const int n = std::min(t.next, (int)max_out);
  for (int i = 0; i < n; ++i) {
    hipError_t e = hipEventSynchronize(t.ev[2 * i + 1]);
    if (e != hipSuccess) return (int)e;
    e = hipEventElapsedTime(&ms_out[i], t.ev[2 * i], t.ev[2 * i + 1]);
    if (e != hipSuccess) return (int)e;
  }
  *count_out = n;
  return RAI_OK;
}
