// Fused PPO epoch for small MLP actor-critics on gfx950 (CartPole-class policies).
//
// One launch runs EVERY minibatch of one epoch of rl_algo_impls/ppo/ppo.py:290-411
// for an ActorCritic whose encoder is Flatten and whose actor/critic heads are
// [in -> 64 -> 64 -> out] MLPs (rl_algo_impls/shared/policy/actor_critic_network/
// connected_trio.py + shared/actor/categorical.py + shared/policy/critic.py):
//   forward, categorical logp/entropy, clipped-surrogate + value loss gradients,
//   backward, clip_grad_norm_ and Adam(eps) — without leaving the chip.
//
// Why one launch: at the CartPole config an update is 40,960 *dependent* Adam steps
// of ~13 MFLOP each; per-step launches cost more than the arithmetic.  The floor of
// this design is the f32 MFMA work of one CU per network (3 x 64x64 contractions
// over the minibatch rows), so everything else is arranged to stay off that path:
//
//  * workgroup 0 = actor, workgroup 1 = critic (no shared parameters; the only
//    coupling is clip_grad_norm_'s global norm, exchanged once per minibatch as an
//    8-byte {tag,value} granule — ~0.5 us one way, measured by tools/xchg_diag.hip);
//  * weights live in LDS (W2 also transposed for the backward), Adam moments in the
//    registers of each parameter's owning lane, W2's gradient in MFMA accumulators;
//  * the three 64-wide contractions and layer 1 run on v_mfma_f32_16x16x4_f32
//    (exact f32); the output layer is folded into layer 2's epilogue (two column-
//    half partial sums, DPP row reductions);
//  * every sum over minibatch rows (dW3, db3, db2, db1, dW1) is a per-thread partial
//    over a row slice, reduced once per minibatch through LDS (no serial row loops);
//  * the next minibatch's rows are prefetched into registers, already in the MFMA
//    A-operand layout for layer 1;
//  * advantage normalisation moments (ppo.py:313-316) are computed for all the
//    epoch's minibatches by a small pre-kernel, off the dependent chain.
//
// The kernel is instantiated for padded (in_dim, n_actions) of (4, 2) — CartPole —
// and (8, 8); padded rows/columns carry zeros.
#include "common.h"
#include "internal.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>

#pragma clang fp contract(off)

namespace {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

constexpr int HID = 64;
constexpr int LD = 66;
constexpr int CH = 128;
constexpr int MAXIN = 8;
constexpr int MAXOUT = 8;
constexpr int MAXB = 256;
constexpr int NT = 1024;
constexpr int NW = NT / 64;
constexpr float F32_MIN = -3.4028234663852886e38f;

struct MlpArgs {
  float* params;
  float* exp_avg;
  float* exp_avg_sq;
  const float* obs;
  const int64_t* actions;
  const float* old_logp;
  const float* old_values;
  const float* adv;
  const float* ret;
  int64_t n_rows;
  int32_t batch;
  int32_t in_dim;
  int32_t n_act;
  int32_t act_fn;
  const rai_ppo_hparams* hp;
  const rai_optim_hparams* ohp;
  rai_train_state* state;
  float* stats;
  int32_t max_stats;
  float* norms;
  int32_t max_norms;
  unsigned long long* xchg;  // [0..3]: [2 nets][2 parities]; [4]: critic-done flag; zeroed per launch
  int32_t* err;
  // per-minibatch (mean, den) of the advantage normalisation: moments[2*mb], moments[2*mb+1]
  const float* moments;
  // row-tile layout: per-wave partial gradients [2 nets][NW][parts][64]; multi-CU layout: the
  // exchange slots (workspace)
  float* scratch;
  // multi-CU layout: per-CU loss-statistic partials [2 nets][minibatches][MC_G][4] (workspace)
  double* statp;
  // data-parallel "grads" mode (grad_out != nullptr): process minibatches
  // [mb_begin, mb_begin + mb_count), scale the loss means by 1/(rows*world), write the
  // raw gradients to grad_out and stop (the caller all-reduces them and runs
  // rai_clip_optim_step).
  float* grad_out;
  int32_t mb_begin;
  int32_t mb_count;
  int32_t world;
  // multi-CU data-parallel step (grads mode only): before the minibatch, apply clip_grad_norm_ +
  // Adam with the all-reduced flat gradient of the previous step (grad_in, P_total elements: both
  // networks); sync_base = number of earlier launches since the sync words were last zeroed
  const float* grad_in;
  int32_t P_total;
  int32_t sync_base;
  // in-kernel cross-GPU exchange (multi-CU layout, epoch mode): xpeers[r] = rank r's exchange
  // region (IPC-mapped device memory, uncached), xbase = optimizer steps already exchanged
  // through these regions (flags are monotonic step ids, never re-zeroed)
  void* const* xpeers;
  int32_t xrank;
  int32_t xworld;
  int64_t xbase;
};

#ifdef RAI_STAMPS
// Diagnostic build only (never the shipped library): per-phase cycle totals of wave 0 of
// each workgroup, accumulated over the launch and copied out by rai_mlp_debug_stamps().
__device__ unsigned long long g_stamps[2][32];
#define STAMP(i)                                                                 \
  do {                                                                           \
    if (threadIdx.x == 0) {                                                      \
      unsigned long long t_;                                                     \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
      S.stamps[i] += t_ - S.t_last;                                              \
      S.t_last = t_;                                                             \
    }                                                                            \
  } while (0)
#else
#define STAMP(i) \
  do {           \
  } while (0)
#endif

// Re-derive the lane coordinates inside each phase from a freshly computed lane id (mbcnt, so
// threadIdx.x's register need not stay live) and an opaque copy of the wave index, so the
// compiler recomputes per-phase LDS addresses where they are used instead of hoisting them all
// out of the minibatch loop (which overflows 128 VGPRs and spills).
#define RELANE()                                                                     \
  int tid_l_ = (w << 6) | (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); \
  asm volatile("" : "+v"(tid_l_));                                                   \
  int w_l_ = w;                                                                      \
  asm volatile("" : "+s"(w_l_));                                                     \
  const int tid = tid_l_, lane = tid & 63, g = lane >> 4, li = lane & 15, w = w_l_;  \
  (void)tid; (void)lane; (void)g; (void)li; (void)w

template <int INP, int OUTP>
struct Smem {
#ifdef RAI_STAMPS
  unsigned long long stamps[32];
  unsigned long long t_last;
#endif
  double red[NW];
  double pw[2];
  double st[16];  // loss statistics: [4 row waves][4]
  float bcast[8];
  float W1[HID][INP];  // [out j][in k]
  float b1[HID];
  float b2[HID];
  float b3[MAXOUT];
  float W2[HID][LD];   // [out j][in k]
  float W2T[HID][LD];  // [in k][out j]
  float W3[OUTP][LD];  // [out o][in k]
  float X[CH][INP];
  float H1[CH][LD];    // act(z1), later dZ1, at minibatch end: partial-gradient scratch
  float H2[CH][LD];    // act(z2), later dZ2, at minibatch end: partial-gradient scratch
  float outp[2][CH][OUTP];  // output-layer partial sums of the two column halves of H2
  float dout[CH][OUTP];
  float db3p[4][OUTP];
};

__device__ __forceinline__ int kmap(int g, int kk) { return (g & 1) * 32 + (g >> 1) * 16 + kk; }
__device__ __forceinline__ int smap(int g, int kk) {
  return (kk >> 3) * 32 + (g >> 1) * 16 + (g & 1) * 8 + (kk & 7);
}
// Branch-free tanh (libm's tanhf branches on |x| ranges, which diverges across a wave):
// |x| < 0.3: odd Taylor series to x^9 (truncation < 1e-7 relative); otherwise
// 1 - 2 / (exp(2|x|) + 1) with the sign restored (absolute error ~1 ulp of 1).
__device__ __forceinline__ float tanh_bf(float x) {
  const float ax = fabsf(x);
  const float x2 = x * x;
  float p = fmaf(x2, 62.f / 2835.f, -17.f / 315.f);
  p = fmaf(x2, p, 2.f / 15.f);
  p = fmaf(x2, p, -1.f / 3.f);
  const float small = fmaf(x * x2, p, x);
  const float e = __builtin_amdgcn_exp2f(ax * 2.885390081777927f);  // exp(2|x|)
  const float big = fmaf(-2.f, __builtin_amdgcn_rcpf(e + 1.f), 1.f);
  return ax < 0.3f ? small : copysignf(big, x);
}
__device__ __forceinline__ float act_f(const int relu, float z) { return relu ? fmaxf(z, 0.f) : tanh_bf(z); }
__device__ __forceinline__ float act_d(int relu, float h) { return relu ? (h > 0.f ? 1.f : 0.f) : 1.f - h * h; }

__device__ __forceinline__ float vf_loss(int fn, float x) {
  if (fn == 0) return x * x;
  const float z = fabsf(x);
  return z < 1.f ? 0.5f * z * z : (z - 0.5f);
}
__device__ __forceinline__ float vf_grad(int fn, float x) {
  if (fn == 0) return 2.f * x;
  return x <= -1.f ? -1.f : (x >= 1.f ? 1.f : x);
}

// Sum over the 16 lanes of a DPP row; every lane of the row receives the same bits.
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row_sum16(float v) {
  v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp<0x141>(v);  // row_half_mirror
  v += dpp<0x140>(v);  // row_mirror
  return v;
}

__device__ __forceinline__ void adam_update(float& p, float& m, float& v, float g, float w1, float w2,
                                            float beta2, float bc2_sqrt, float neg_step, float eps) {
  m = m + w1 * (g - m);
  v = v * beta2;
  v = v + (w2 * g) * g;
  const float denom = sqrtf(v) / bc2_sqrt + eps;
  p = p + neg_step * (m / denom);
}

// Advantage-normalisation moments of every minibatch (one workgroup per minibatch), in the
// operation order of the loss kernel: fp64 sums, mean rounded to f32, unbiased std
// (ppo.py:313-316: (A - A.mean()) / (A.std() + 1e-8); standardize: A / (A.std() + 1e-8)).
__global__ __launch_bounds__(256) void adv_moments_kernel(const float* __restrict__ adv, int64_t n_rows, int B,
                                                          const rai_ppo_hparams* hp, float* moments) {
  __shared__ double scratch[4];
  const int mb = blockIdx.x;
  const int64_t row0 = (int64_t)mb * B;
  const int rows = (int)min((int64_t)B, n_rows - row0);
  const int tid = threadIdx.x;
  const float x = tid < rows ? adv[row0 + tid] : 0.f;
  double v1[1] = {tid < rows ? (double)x : 0.0};
  block_sum<1>(v1, scratch);
  const float mean = (float)(v1[0] / (double)rows);
  const double d = tid < rows ? (double)x - (double)mean : 0.0;
  double v2[1] = {d * d};
  block_sum<1>(v2, scratch);
  if (tid == 0) {
    const float den = (float)sqrt(v2[0] / (double)(rows - 1)) + 1e-8f;
    float m0 = 0.f, m1 = 1.f;
    if (hp->normalize_advantage) { m0 = mean; m1 = den; }
    else if (hp->standardize_advantage) { m1 = den; }
    moments[2 * mb] = m0;
    moments[2 * mb + 1] = m1;
  }
}

// One network (ACTOR: the policy head; else the value head) of the fused epoch.
template <int INP, int OUTP, bool ACTOR, int RELU>
__device__ __forceinline__ void mlp_net(const MlpArgs& a, Smem<INP, OUTP>& S) {
  constexpr int net = ACTOR ? 0 : 1;
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, li = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int IN = a.in_dim;
  const int NA = a.n_act;
  const int OUT = ACTOR ? NA : 1;
  constexpr int relu = RELU;  // compile-time: keeps the activation epilogues in one basic block
  const float clip_range = a.hp->clip_range, ent_coef = a.hp->ent_coef, vf_coef0 = a.hp->vf_coef[0];
  const float clip_range_vf = a.hp->clip_range_vf;
  const int has_vclip = a.hp->has_clip_range_vf, vf_fn = a.hp->vf_loss_fn;
  const float halve = a.hp->ppo2_vf_coef_halving ? 0.5f : 1.f;
  const float beta2 = a.ohp->beta2, adam_eps = a.ohp->eps, lr = a.ohp->lr;
  const double beta1_d = a.ohp->beta1_d, beta2_d = a.ohp->beta2_d;
  const bool grads_mode = a.grad_out != nullptr;
  const float max_grad_norm = a.ohp->max_grad_norm;

  // ---- flat parameter offsets (torch parameters() order: actor block, critic block) -------
  const int szA = HID * IN + HID + HID * HID + HID + NA * HID + NA;
  const int base = net == 0 ? 0 : szA;
  const int oW1 = base, ob1 = oW1 + HID * IN, oW2 = ob1 + HID, ob2 = oW2 + HID * HID, oW3 = ob2 + HID,
            ob3 = oW3 + OUT * HID;

  for (int e = tid; e < HID * INP; e += NT) {
    const int j = e / INP, k = e % INP;
    S.W1[j][k] = k < IN ? a.params[oW1 + j * IN + k] : 0.f;
  }
  if (tid < HID) {
    S.b1[tid] = a.params[ob1 + tid];
    S.b2[tid] = a.params[ob2 + tid];
  }
  for (int e = tid; e < HID * HID; e += NT) {
    const int j = e >> 6, k = e & 63;
    const float x = a.params[oW2 + e];
    S.W2[j][k] = x;
    S.W2T[k][j] = x;
  }
  for (int e = tid; e < OUTP * HID; e += NT) {
    const int o = e >> 6, k = e & 63;
    S.W3[o][k] = o < OUT ? a.params[oW3 + o * HID + k] : 0.f;
  }
  if (tid < MAXOUT) S.b3[tid] = tid < OUT ? a.params[ob3 + tid] : 0.f;

  // ---- ownership: W2 tile element (jt,kt) from the dW2 MFMA layout; slot A / slot B ---------
  const int jt = w >> 2, kt = w & 3;
  int w2_idx[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) w2_idx[r] = (jt * 16 + g * 4 + r) * HID + kt * 16 + li;
  // grads mode carries no optimizer state (exp_avg/exp_avg_sq are null there)
  float w2_m[4] = {0.f, 0.f, 0.f, 0.f}, w2_v[4] = {0.f, 0.f, 0.f, 0.f};
  if (!grads_mode) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      w2_m[r] = a.exp_avg[oW2 + w2_idx[r]];
      w2_v[r] = a.exp_avg_sq[oW2 + w2_idx[r]];
    }
  }
  // slot A: W3 (tid < OUT*64) | b3 (512..512+OUT) | b2 (576..639) | b1 (640..703)
  int a_flat = -1;
  if (tid < OUT * HID) a_flat = oW3 + tid;
  else if (tid >= 512 && tid < 512 + OUT) a_flat = ob3 + (tid - 512);
  else if (tid >= 576 && tid < 640) a_flat = ob2 + (tid - 576);
  else if (tid >= 640 && tid < 704) a_flat = ob1 + (tid - 640);
  // slot B: W1 (tid < 64*IN)
  const int b_flat = tid < HID * IN ? oW1 + tid : -1;
  float a_m = 0.f, a_v = 0.f, b_m = 0.f, b_v = 0.f;
  if (!grads_mode && a_flat >= 0) { a_m = a.exp_avg[a_flat]; a_v = a.exp_avg_sq[a_flat]; }
  if (!grads_mode && b_flat >= 0) { b_m = a.exp_avg[b_flat]; b_v = a.exp_avg_sq[b_flat]; }

  const int B = a.batch;
  const int64_t n_rows = a.n_rows;
  const int nmb_total = (int)((n_rows + B - 1) / B);
  const int mb_begin = a.mb_begin;
  const int mb_end = min(nmb_total, a.mb_begin + a.mb_count);
  const int nmb = mb_end - mb_begin;
  const int64_t step0 = a.state->opt_step;
  const int stat0 = a.state->stat_index;
  const int norm0 = a.state->norm_index;
  const int latched = a.state->pi_coef_zero;
  const float pi_coef = latched ? 0.f : 1.f;

  // ---- per-minibatch inputs, prefetched into registers one minibatch ahead ------------------
  // thread t < rows: row t's (action, old logp, adv | old value, return);
  // px[c][q]: X[c*CH + (w>>1)*16 + li][4q + g] = the layer-1 MFMA A operand of chunk c
  constexpr int NQ = INP / 4;
  int r_act = 0;
  float r_a = 0.f, r_b = 0.f, r_c = 0.f, r_d = 1.f;
  float px[2][NQ];
  auto prefetch = [&](int mb) {
    const int64_t row0 = (int64_t)mb * B;
    const int rows = (int)min((int64_t)B, n_rows - row0);
    if (tid < rows) {
      const int64_t r = row0 + tid;
      if (ACTOR) {
        r_act = (int)a.actions[r];
        r_a = a.old_logp[r];
        r_b = a.adv[r];
      } else {
        r_a = a.old_values[r];
        r_b = a.ret[r];
      }
    }
    if (ACTOR) {
      r_c = a.moments[2 * mb];
      r_d = a.moments[2 * mb + 1];
    }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int s = c * CH + (w >> 1) * 16 + li;
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int k = 4 * q + g;
        px[c][q] = (s < rows && k < IN) ? a.obs[(row0 + s) * IN + k] : 0.f;
      }
    }
  };
  prefetch(mb_begin);
  if (tid == 0) {  // running powers beta^step (bias corrections), advanced once per minibatch
    S.pw[0] = ipow(beta1_d, step0);
    S.pw[1] = ipow(beta2_d, step0);
  }
#ifdef RAI_STAMPS
  if (tid < 32) S.stamps[tid] = 0;
  if (tid == 0) S.t_last = __builtin_amdgcn_s_memtime();
#endif
  lds_barrier();

  for (int mb = mb_begin; mb < mb_end; ++mb) {
    const int64_t row0 = (int64_t)mb * B;
    const int rows = (int)min((int64_t)B, n_rows - row0);
    // take this minibatch's inputs out of the prefetch registers
    const int c_act = r_act;
    const float c_a = r_a, c_b = r_b;
    float cx[2][NQ];
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int q = 0; q < NQ; ++q) cx[c][q] = px[c][q];
    const float amean = r_c, aden = r_d;
    if (mb + 1 < mb_end) prefetch(mb + 1);
    const float invB = 1.f / (float)(rows * a.world);

    // per-thread partial gradients over this minibatch's rows
    f4 gw2 = {0.f, 0.f, 0.f, 0.f};   // dW2 tile (MFMA accumulator)
    float p_w3[OUTP], p_b2 = 0.f;    // B1 layout: column k = lane, rows w + 16 i
    float p_b1[2] = {0.f, 0.f};      // B3 layout: columns k0, k0 + 16, rows of tile (w>>1)
    float p_w1 = 0.f;                // B4 layout: (j = lane, k, row slice)
    float my_dout[OUTP];             // this thread's row (L layout), for db3
    float st[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int o = 0; o < OUTP; ++o) { p_w3[o] = 0.f; my_dout[o] = 0.f; }

    const int nch = (rows + CH - 1) / CH;
    for (int c = 0; c < nch; ++c) {
      const int crows = min(CH, rows - c * CH);
      // ---- F1: layer 1 on MFMA (K = in_dim padded to 4/8), act -> H1; X -> LDS for dW1 ----------
      {
        RELANE();
        const int mt = w >> 1, ntb = (w & 1) * 2;
        f4 z0 = {0.f, 0.f, 0.f, 0.f}, z1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          const float av = c == 0 ? cx[0][q] : cx[1][q];
          const float b0 = S.W1[ntb * 16 + li][4 * q + g];
          const float b1 = S.W1[(ntb + 1) * 16 + li][4 * q + g];
          z0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, b0, z0, 0, 0, 0);
          z1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, b1, z1, 0, 0, 0);
          if ((w & 1) == 0) S.X[mt * 16 + li][4 * q + g] = av;
        }
        const int j0 = ntb * 16 + li;
        const float bb0 = S.b1[j0], bb1 = S.b1[j0 + 16];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int s = mt * 16 + g * 4 + r;
          S.H1[s][j0] = act_f(relu, z0[r] + bb0);
          S.H1[s][j0 + 16] = act_f(relu, z1[r] + bb1);
        }
      }
      lds_barrier();
      STAMP(1);
      // ---- F2: layer 2 on MFMA, act -> H2; output layer folded into the epilogue -----------------
      {
        RELANE();
        const int mt = w >> 1, nt0 = (w & 1) * 2;
        f4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < 16; kk += 2) {
          const int kq = kmap(g, kk);
          const f2 av = *reinterpret_cast<const f2*>(&S.H1[mt * 16 + li][kq]);
          const f2 b0 = *reinterpret_cast<const f2*>(&S.W2[nt0 * 16 + li][kq]);
          const f2 b1 = *reinterpret_cast<const f2*>(&S.W2[(nt0 + 1) * 16 + li][kq]);
          acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, b0.x, acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, b1.x, acc1, 0, 0, 0);
          acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, b0.y, acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, b1.y, acc1, 0, 0, 0);
        }
        const int j0 = nt0 * 16 + li;
        const float bb0 = S.b2[j0], bb1 = S.b2[j0 + 16];
        float w3a[OUTP], w3b[OUTP];
#pragma unroll
        for (int o = 0; o < OUTP; ++o) {
          w3a[o] = S.W3[o][j0];
          w3b[o] = S.W3[o][j0 + 16];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int s = mt * 16 + g * 4 + r;
          const float h0 = act_f(relu, acc0[r] + bb0);
          const float h1 = act_f(relu, acc1[r] + bb1);
          S.H2[s][j0] = h0;
          S.H2[s][j0 + 16] = h1;
#pragma unroll
          for (int o = 0; o < OUTP; ++o) {
            const float part = row_sum16(fmaf(h1, w3b[o], h0 * w3a[o]));
            if (li == ((r * OUTP + o) & 15)) S.outp[w & 1][s][o] = part;
          }
        }
      }
      lds_barrier();
      STAMP(2);
      // ---- L: per-row loss gradient w.r.t. the head outputs (ppo.py:326-371 semantics; autograd
      //      tie rules of min/max and closed-interval clamp, as loss.hip) ---------------------------
      {
        RELANE();
        const int s = tid - c * CH;
        if (s >= 0 && s < CH) {
          float d[OUTP];
#pragma unroll
          for (int o = 0; o < OUTP; ++o) d[o] = 0.f;
          if (s < crows) {
            float z[OUTP];
#pragma unroll
            for (int o = 0; o < OUTP; ++o) z[o] = (S.outp[0][s][o] + S.outp[1][s][o]) + S.b3[o];
            if (ACTOR) {
              float m = F32_MIN;
#pragma unroll
              for (int o = 0; o < OUTP; ++o)
                if (o < NA) m = fmaxf(m, z[o]);
              float se = 0.f;
#pragma unroll
              for (int o = 0; o < OUTP; ++o)
                if (o < NA) se += expf(z[o] - m);
              const float lse = m + logf(se);
              float H = 0.f;
#pragma unroll
              for (int o = 0; o < OUTP; ++o)
                if (o < NA) {
                  const float n = z[o] - lse;
                  H -= fmaxf(n, F32_MIN) * expf(n);
                }
              const int act = min(max(c_act, 0), NA - 1);
              float zact = z[0];
#pragma unroll
              for (int o = 1; o < OUTP; ++o)
                if (o == act) zact = z[o];
              const float logp = zact - lse;
              const float A = (c_b - amean) / aden;
              const float logratio = logp - c_a;
              const float ratio = expf(logratio);
              const float lo = 1.f - clip_range, hi = 1.f + clip_range;
              const float cr = fminf(fmaxf(ratio, lo), hi);
              const float s1 = ratio * A, s2 = cr * A;
              const float gpi = -pi_coef * invB;
              float g1, g2;
              if (s1 < s2) { g1 = gpi; g2 = 0.f; }
              else if (s1 > s2) { g1 = 0.f; g2 = gpi; }
              else { g1 = gpi * 0.5f; g2 = gpi * 0.5f; }
              const float in_clip = (ratio >= lo && ratio <= hi) ? 1.f : 0.f;
              const float dlogp = (g1 * A + (g2 * A) * in_clip) * ratio;
              const float dent = -ent_coef * invB;
#pragma unroll
              for (int o = 0; o < OUTP; ++o)
                if (o < NA) {
                  const float n = z[o] - lse;
                  const float p = expf(n);
                  d[o] = dlogp * ((o == act ? 1.f : 0.f) - p) + dent * (-p * (n + H));
                }
              st[0] += fminf(s1, s2);
              st[1] += (ratio - 1.f) - logratio;
              st[2] += (fabsf(ratio - 1.f) > clip_range) ? 1.f : 0.f;
              st[3] += H;
            } else {
              const float v = z[0], R = c_b;
              const float gl = (vf_coef0 * halve) * invB;
              float l = vf_loss(vf_fn, v - R), dv;
              if (has_vclip) {
                const float vc_ = clip_range_vf;
                const float dvo = v - c_a;
                const float vcl = c_a + fminf(fmaxf(dvo, -vc_), vc_);
                const float l2 = vf_loss(vf_fn, vcl - R);
                float w1, w2;
                if (l > l2) { w1 = gl; w2 = 0.f; }
                else if (l < l2) { w1 = 0.f; w2 = gl; }
                else { w1 = gl * 0.5f; w2 = gl * 0.5f; }
                const float inv = (dvo >= -vc_ && dvo <= vc_) ? 1.f : 0.f;
                dv = w1 * vf_grad(vf_fn, v - R) + (w2 * vf_grad(vf_fn, vcl - R)) * inv;
                st[1] += (fabsf(v - c_a) > vc_) ? 1.f : 0.f;
                l = fmaxf(l, l2);
              } else {
                dv = gl * vf_grad(vf_fn, v - R);
              }
              st[0] += l;
              d[0] = dv;
            }
          }
#pragma unroll
          for (int o = 0; o < OUTP; ++o) {
            S.dout[s][o] = d[o];
            my_dout[o] = d[o];
          }
        }
      }
      lds_barrier();
      STAMP(3);
      // ---- B1: dZ2 = (dout . W3) * act'(H2) in place over H2; dW3, db2 partials (column k) ------
      {
        RELANE();
        const int k = lane;
        float w3[OUTP];
#pragma unroll
        for (int o = 0; o < OUTP; ++o) w3[o] = S.W3[o][k];
#pragma unroll
        for (int i = 0; i < CH / NW; ++i) {
          const int s = w + NW * i;
          const float h = S.H2[s][k];
          float dh = 0.f;
#pragma unroll
          for (int o = 0; o < OUTP; ++o) {
            const float dv = S.dout[s][o];
            dh = fmaf(dv, w3[o], dh);
            p_w3[o] = fmaf(dv, h, p_w3[o]);
          }
          const float dz = dh * act_d(relu, h);
          p_b2 += dz;
          S.H2[s][k] = dz;
        }
      }
      lds_barrier();
      STAMP(4);
      // ---- B2: dW2 += dZ2^T H1 (accumulators persist over chunks), dH1 = dZ2 W2 (held) ---------
      f4 h0 = {0.f, 0.f, 0.f, 0.f}, h1 = {0.f, 0.f, 0.f, 0.f};
      {
        RELANE();
#pragma unroll 8
        for (int kk = 0; kk < 32; ++kk) {
          const int s = smap(g, kk);
          const int jt = w >> 2, kt = w & 3;
          gw2 = __builtin_amdgcn_mfma_f32_16x16x4f32(S.H2[s][jt * 16 + li], S.H1[s][kt * 16 + li], gw2, 0, 0, 0);
        }
        const int mt = w >> 1, nt0 = (w & 1) * 2;
#pragma unroll
        for (int kk = 0; kk < 16; kk += 2) {
          const int kq = kmap(g, kk);
          const f2 av = *reinterpret_cast<const f2*>(&S.H2[mt * 16 + li][kq]);
          const f2 b0 = *reinterpret_cast<const f2*>(&S.W2T[nt0 * 16 + li][kq]);
          const f2 b1 = *reinterpret_cast<const f2*>(&S.W2T[(nt0 + 1) * 16 + li][kq]);
          h0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, b0.x, h0, 0, 0, 0);
          h1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, b1.x, h1, 0, 0, 0);
          h0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, b0.y, h0, 0, 0, 0);
          h1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, b1.y, h1, 0, 0, 0);
        }
      }
      lds_barrier();
      STAMP(5);
      // ---- B3: dZ1 = dH1 * act'(H1) in place over H1; db1 partials -------------------------------
      {
        RELANE();
        const int mt = w >> 1, k0 = (w & 1) * 32 + li;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int s = mt * 16 + g * 4 + r;
          const float da = h0[r] * act_d(relu, S.H1[s][k0]);
          const float db = h1[r] * act_d(relu, S.H1[s][k0 + 16]);
          S.H1[s][k0] = da;
          S.H1[s][k0 + 16] = db;
          p_b1[0] += da;
          p_b1[1] += db;
        }
      }
      lds_barrier();
      STAMP(6);
      // ---- B4: dW1 partial over a row slice (j = lane, k = w % INP, slice = w / INP) -------------
      {
        RELANE();
        constexpr int NSL = NW / INP, RS = CH / NSL;
        const int k = w % INP, sl = w / INP;
        float acc = 0.f;
#pragma unroll 8
        for (int i = 0; i < RS; ++i) {
          const int s = sl * RS + i;
          acc = fmaf(S.H1[s][lane], S.X[s][k], acc);
        }
        p_w1 += acc;
      }
      lds_barrier();
      STAMP(7);
    }

    // ---- E1: per-thread partials -> LDS (H1/H2 are free now) -------------------------------------
    float* R3 = &S.H2[0][0];           // [NW][OUTP][64]
    float* Rb2 = &S.H1[0][0];          // [NW][64]
    float* Rb1 = Rb2 + NW * HID;       // [8 row tiles][64]
    float* RW1 = Rb1 + 8 * HID;        // [NW / INP slices][INP][64]
    {
      RELANE();
#pragma unroll
      for (int o = 0; o < OUTP; ++o) R3[(w * OUTP + o) * HID + lane] = p_w3[o];
      Rb2[w * HID + lane] = p_b2;
      float b1a = p_b1[0] + __shfl_xor(p_b1[0], 16, 64);
      float b1b = p_b1[1] + __shfl_xor(p_b1[1], 16, 64);
      b1a += __shfl_xor(b1a, 32, 64);
      b1b += __shfl_xor(b1b, 32, 64);
      if (g == 0) {
        const int mt = w >> 1, k0 = (w & 1) * 32 + li;
        Rb1[mt * HID + k0] = b1a;
        Rb1[mt * HID + k0 + 16] = b1b;
      }
      RW1[((w / INP) * INP + (w % INP)) * HID + lane] = p_w1;
      if (w < 4) {  // rows live in threads 0..255: db3 and the loss statistics
#pragma unroll
        for (int o = 0; o < OUTP; ++o) {
          const float t = wave_sum(my_dout[o]);
          if (lane == 0) S.db3p[w][o] = t;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const double t = wave_sum((double)st[i]);
          if (lane == 0) S.st[w * 4 + i] = t;
        }
      }
    }
    lds_barrier();
    STAMP(8);
    // ---- E2: owners sum partials in fixed order; squared norm of this network's gradient ----------
    float ga = 0.f, gb = 0.f;
    {
      RELANE();
      if (tid < OUT * HID) {
        const int o = tid >> 6, k = tid & 63;
        float t = 0.f;
#pragma unroll
        for (int q = 0; q < NW; ++q) t += R3[(q * OUTP + o) * HID + k];
        ga = t;
      } else if (tid >= 512 && tid < 512 + OUT) {
        const int o = tid - 512;
        ga = ((S.db3p[0][o] + S.db3p[1][o]) + S.db3p[2][o]) + S.db3p[3][o];
      } else if (tid >= 576 && tid < 640) {
        const int j = tid - 576;
        float t = 0.f;
#pragma unroll
        for (int q = 0; q < NW; ++q) t += Rb2[q * HID + j];
        ga = t;
      } else if (tid >= 640 && tid < 704) {
        const int j = tid - 640;
        float t = 0.f;
#pragma unroll
        for (int q = 0; q < 8; ++q) t += Rb1[q * HID + j];
        ga = t;
      }
      if (b_flat >= 0) {
        const int j = tid / IN, k = tid % IN;
        float t = 0.f;
#pragma unroll
        for (int q = 0; q < NW / INP; ++q) t += RW1[(q * INP + k) * HID + j];
        gb = t;
      }
      double ss = (double)gw2.x * gw2.x + (double)gw2.y * gw2.y + (double)gw2.z * gw2.z + (double)gw2.w * gw2.w;
      if (a_flat >= 0) ss += (double)ga * ga;
      if (b_flat >= 0) ss += (double)gb * gb;
      ss = wave_sum(ss);
      if (lane == 0) S.red[w] = ss;
      if (grads_mode) {
        // raw gradients out (same flat indices as the parameters)
#pragma unroll
        for (int r = 0; r < 4; ++r) a.grad_out[oW2 + w2_idx[r]] = gw2[r];
        if (a_flat >= 0) a.grad_out[a_flat] = ga;
        if (b_flat >= 0) a.grad_out[b_flat] = gb;
      }
    }
    lds_barrier();
    STAMP(9);
    // ---- E3: stats row, grad-norm exchange with the other network, bias corrections ---------------
    if (tid == 0) {
      double ssum = 0.0;
      for (int q = 0; q < NW; ++q) ssum += S.red[q];
      const double* stp = S.st;
      double sv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) sv[i] = ((stp[0 * 4 + i] + stp[1 * 4 + i]) + stp[2 * 4 + i]) + stp[3 * 4 + i];
      const int srow = stat0 + (mb - mb_begin);
      if (a.stats && srow < a.max_stats) {
        float* row = a.stats + (int64_t)srow * RAI_STAT_STRIDE;
        const double Bd = (double)rows * (double)a.world;
        if (ACTOR) {
          const float pi_loss = (float)(-sv[0] / Bd);
          const float ent_loss = (float)(-sv[3] / Bd);
          row[0] = pi_coef * pi_loss + ent_coef * ent_loss;  // host adds the value term
          row[1] = pi_loss;
          row[2] = ent_loss;
          row[3] = (float)(sv[1] / Bd);
          row[4] = (float)(sv[2] / Bd);
        } else {
          row[5] = (float)(sv[0] / Bd) * halve;
          row[5 + RAI_MAX_K] = has_vclip ? (float)(sv[1] / Bd) : 0.f;
        }
      }
      if (!grads_mode) {
        const float mine = (float)ssum;
        const unsigned tag = (unsigned)(mb + 1);
        const int par = mb & 1;
        const unsigned long long gr = ((unsigned long long)tag << 32) | (unsigned long long)__float_as_uint(mine);
        __hip_atomic_store(&a.xchg[net * 2 + par], gr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        float other = 0.f;
        unsigned long long spins = 0;
        for (;;) {
          const unsigned long long x =
              __hip_atomic_load(&a.xchg[(1 - net) * 2 + par], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if ((unsigned)(x >> 32) == tag) { other = __uint_as_float((unsigned)x); break; }
          if (++spins > (1ull << 26)) { atomicExch(a.err, 1); break; }  // bounded: never hangs
          __builtin_amdgcn_s_sleep(1);
        }
        S.bcast[0] = net == 0 ? mine : other;
        S.bcast[1] = net == 0 ? other : mine;
        S.pw[0] *= beta1_d;
        S.pw[1] *= beta2_d;
        const double bc1 = 1.0 - S.pw[0];
        const double bc2 = 1.0 - S.pw[1];
        S.bcast[2] = (float)sqrt(bc2);
        S.bcast[3] = (float)(-((double)lr / bc1));
      }
    }
    lds_barrier();
    STAMP(10);
    if (grads_mode) continue;
    const float total_norm = (float)sqrt((double)S.bcast[0] + (double)S.bcast[1]);
    float coef = 1.f;
    if (max_grad_norm > 0.f) coef = fminf(max_grad_norm / (total_norm + 1e-6f), 1.f);
    const float bc2_sqrt = S.bcast[2], neg_step = S.bcast[3];
    const float w1 = (float)(1.0 - beta1_d), w2 = (float)(1.0 - beta2_d);

    // ---- E4: Adam on owned parameters; refresh the LDS copies --------------------------------------
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = w2_idx[r] >> 6, k = w2_idx[r] & 63;
      float p = S.W2[j][k];
      adam_update(p, w2_m[r], w2_v[r], gw2[r] * coef, w1, w2, beta2, bc2_sqrt, neg_step, adam_eps);
      S.W2[j][k] = p;
      S.W2T[k][j] = p;
    }
    if (a_flat >= 0) {
      float* slot;
      if (tid < OUT * HID) slot = &S.W3[tid >> 6][tid & 63];
      else if (tid < 576) slot = &S.b3[tid - 512];
      else if (tid < 640) slot = &S.b2[tid - 576];
      else slot = &S.b1[tid - 640];
      float p = *slot;
      adam_update(p, a_m, a_v, ga * coef, w1, w2, beta2, bc2_sqrt, neg_step, adam_eps);
      *slot = p;
    }
    if (b_flat >= 0) {
      const int j = tid / IN, k = tid % IN;
      float p = S.W1[j][k];
      adam_update(p, b_m, b_v, gb * coef, w1, w2, beta2, bc2_sqrt, neg_step, adam_eps);
      S.W1[j][k] = p;
    }
    if (tid == 0) {
      if (ACTOR && a.norms && norm0 + (mb - mb_begin) < a.max_norms) a.norms[norm0 + (mb - mb_begin)] = total_norm;
    }
    lds_barrier();
    STAMP(11);
  }

  // ---- write back parameters and optimizer moments (torch parameter order) -----------------------
  if (!grads_mode) {
    int t2 = tid;
    asm volatile("" : "+v"(t2));
    const int lane2 = t2 & 63, w_2 = t2 >> 6, g2 = lane2 >> 4, li2 = lane2 & 15;
    const int jt2 = w_2 >> 2, kt2 = w_2 & 3;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = jt2 * 16 + g2 * 4 + r, k = kt2 * 16 + li2;
      const int idx = oW2 + j * HID + k;
      a.params[idx] = S.W2[j][k];
      a.exp_avg[idx] = w2_m[r];
      a.exp_avg_sq[idx] = w2_v[r];
    }
    int af = -1;
    float p = 0.f;
    if (t2 < OUT * HID) { af = oW3 + t2; p = S.W3[t2 >> 6][t2 & 63]; }
    else if (t2 >= 512 && t2 < 512 + OUT) { af = ob3 + (t2 - 512); p = S.b3[t2 - 512]; }
    else if (t2 >= 576 && t2 < 640) { af = ob2 + (t2 - 576); p = S.b2[t2 - 576]; }
    else if (t2 >= 640 && t2 < 704) { af = ob1 + (t2 - 640); p = S.b1[t2 - 640]; }
    if (af >= 0) {
      a.params[af] = p;
      a.exp_avg[af] = a_m;
      a.exp_avg_sq[af] = a_v;
    }
    if (t2 < HID * IN) {
      a.params[oW1 + t2] = S.W1[t2 / IN][t2 % IN];
      a.exp_avg[oW1 + t2] = b_m;
      a.exp_avg_sq[oW1 + t2] = b_v;
    }
  }
#ifdef RAI_STAMPS
  if (tid < 32) g_stamps[net][tid] = S.stamps[tid];
#endif
  // grads mode has no per-minibatch exchange, so the actor must not advance the shared
  // stat_index before the critic has read it: the critic posts a done flag, the actor waits.
  if (grads_mode && tid == 0) {
    if (!ACTOR) {
      __hip_atomic_store(&a.xchg[4], 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      unsigned long long spins = 0;
      while (__hip_atomic_load(&a.xchg[4], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == 0ull) {
        if (++spins > (1ull << 26)) { atomicExch(a.err, 1); break; }
        __builtin_amdgcn_s_sleep(1);
      }
    }
  }
  if (ACTOR && tid == 0) {
    a.state->stat_index = stat0 + nmb;
    if (!grads_mode) {
      a.state->opt_step = step0 + nmb;
      a.state->norm_index = norm0 + nmb;
    }
  }
}

// ================================================================================================
// Row-tile layout for in_dim <= 4, n_actions <= 2 (the CartPole class; the bench configuration).
// The whole minibatch (<= 256 rows) is one pass: wave w owns rows [16w, 16w + 16) end to end —
// layer 1, layer 2 (all 64 columns: 4 MFMA tiles), the output layer and the loss, dZ2, dH1 and
// dZ1 — so the forward, the loss and most of the backward need no workgroup barrier at all
// (every LDS hand-off in that stretch is wave-local).  The only cross-wave steps per minibatch are
// dW2 = dZ2^T H1 over all rows (one MFMA tile of dW2 per wave) and the owner reductions of the
// per-wave partial gradients (staged in a global scratch slab: LDS holds H1 and dZ2 for 256 rows).
// 4 barriers per minibatch instead of 18.
// ================================================================================================
constexpr int RB = 256;  // rows per pass = NW waves x 16

template <int OUTP>
struct SmemR {
#ifdef RAI_STAMPS
  unsigned long long stamps[32];
  unsigned long long t_last;
#endif
  double red[NW];
  double pw[2];
  double st[NW][4];
  float bcast[8];
  float db3p[NW][OUTP];
  float W1[HID][4];    // [out j][in k]
  float b1[HID];
  float b2[HID];
  float b3[MAXOUT];
  float W2[HID][LD];   // [out j][in k]
  float W3[OUTP][LD];  // [out o][in k]
  float X[RB][4];
  float H1[RB][LD];    // act(z1) of every row
  float Z2[RB][LD];    // dZ2 of every row
};

template <int OUTP>
struct RowParts {
  static constexpr int N = OUTP + 2 + 4;  // dW3[o], db2, db1, dW1[k] per column
};

template <int OUTP, bool ACTOR, int RELU>
__device__ __forceinline__ void mlp_rows(const MlpArgs& a, SmemR<OUTP>& S) {
  constexpr int net = ACTOR ? 0 : 1;
  constexpr int relu = RELU;
  constexpr int NPART = RowParts<OUTP>::N;
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, li = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int IN = a.in_dim;
  const int NA = a.n_act;
  const int OUT = ACTOR ? NA : 1;
  const float clip_range = a.hp->clip_range, ent_coef = a.hp->ent_coef, vf_coef0 = a.hp->vf_coef[0];
  const float clip_range_vf = a.hp->clip_range_vf;
  const int has_vclip = a.hp->has_clip_range_vf, vf_fn = a.hp->vf_loss_fn;
  const float halve = a.hp->ppo2_vf_coef_halving ? 0.5f : 1.f;
  const float beta2 = a.ohp->beta2, adam_eps = a.ohp->eps, lr = a.ohp->lr;
  const double beta1_d = a.ohp->beta1_d, beta2_d = a.ohp->beta2_d;
  const bool grads_mode = a.grad_out != nullptr;
  const float max_grad_norm = a.ohp->max_grad_norm;
  float* const scr = a.scratch + (size_t)net * NW * (MAXOUT + 6) * HID;  // fixed per-net stride

  // ---- flat parameter offsets (torch parameters() order: actor block, critic block) -------
  const int szA = HID * IN + HID + HID * HID + HID + NA * HID + NA;
  const int base = net == 0 ? 0 : szA;
  const int oW1 = base, ob1 = oW1 + HID * IN, oW2 = ob1 + HID, ob2 = oW2 + HID * HID, oW3 = ob2 + HID,
            ob3 = oW3 + OUT * HID;

  if (tid < HID * 4) {
    const int j = tid >> 2, k = tid & 3;
    S.W1[j][k] = k < IN ? a.params[oW1 + j * IN + k] : 0.f;
  }
  if (tid < HID) {
    S.b1[tid] = a.params[ob1 + tid];
    S.b2[tid] = a.params[ob2 + tid];
  }
  for (int e = tid; e < HID * HID; e += NT) S.W2[e >> 6][e & 63] = a.params[oW2 + e];
  if (tid < OUTP * HID) S.W3[tid >> 6][tid & 63] = (tid >> 6) < OUT ? a.params[oW3 + tid] : 0.f;
  if (tid < MAXOUT) S.b3[tid] = tid < OUT ? a.params[ob3 + tid] : 0.f;

  // ---- ownership (as the chunked layout): W2 tile element of the dW2 MFMA; slot A; slot B ----
  const int jt = w >> 2, kt = w & 3;
  int w2_idx[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) w2_idx[r] = (jt * 16 + g * 4 + r) * HID + kt * 16 + li;
  float w2_m[4] = {0.f, 0.f, 0.f, 0.f}, w2_v[4] = {0.f, 0.f, 0.f, 0.f};
  if (!grads_mode) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      w2_m[r] = a.exp_avg[oW2 + w2_idx[r]];
      w2_v[r] = a.exp_avg_sq[oW2 + w2_idx[r]];
    }
  }
  int a_flat = -1;
  if (tid < OUT * HID) a_flat = oW3 + tid;
  else if (tid >= 512 && tid < 512 + OUT) a_flat = ob3 + (tid - 512);
  else if (tid >= 576 && tid < 640) a_flat = ob2 + (tid - 576);
  else if (tid >= 640 && tid < 704) a_flat = ob1 + (tid - 640);
  const int b_flat = tid < HID * IN ? oW1 + tid : -1;
  float a_m = 0.f, a_v = 0.f, b_m = 0.f, b_v = 0.f;
  if (!grads_mode && a_flat >= 0) { a_m = a.exp_avg[a_flat]; a_v = a.exp_avg_sq[a_flat]; }
  if (!grads_mode && b_flat >= 0) { b_m = a.exp_avg[b_flat]; b_v = a.exp_avg_sq[b_flat]; }

  const int B = a.batch;
  const int64_t n_rows = a.n_rows;
  const int nmb_total = (int)((n_rows + B - 1) / B);
  const int mb_begin = a.mb_begin;
  const int mb_end = min(nmb_total, a.mb_begin + a.mb_count);
  const int nmb = mb_end - mb_begin;
  const int64_t step0 = a.state->opt_step;
  const int stat0 = a.state->stat_index;
  const int norm0 = a.state->norm_index;
  const int latched = a.state->pi_coef_zero;
  const float pi_coef = latched ? 0.f : 1.f;

  // ---- per-minibatch inputs, prefetched into registers one minibatch ahead ------------------
  // lane (g, li) of wave w: the loss inputs of row 16w + 4g + (li & 3) and the layer-1 MFMA
  // A operand X[16w + li][g]
  int r_act = 0;
  float r_a = 0.f, r_b = 0.f, r_c = 0.f, r_d = 1.f, r_x = 0.f;
  auto prefetch = [&](int mb) {
    const int64_t row0 = (int64_t)mb * B;
    const int rows = (int)min((int64_t)B, n_rows - row0);
    // lane coordinates recomputed here (mbcnt) and made opaque: keeps per-lane addresses from
    // being hoisted out of the minibatch loop — kept live they spill, and a spill reload's
    // vmcnt(0) would then wait for these very prefetch loads
    int ln = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    asm volatile("" : "+v"(ln));
    const int xr = w * 16 + (ln & 15), xg = ln >> 4;
    r_x = (xr < rows && xg < IN) ? a.obs[(row0 + xr) * IN + xg] : 0.f;
    const int rr = w * 16 + (ln >> 4) * 4 + (ln & 3);
    if (rr < rows) {
      const int64_t r = row0 + rr;
      if (ACTOR) {
        r_act = (int)a.actions[r];
        r_a = a.old_logp[r];
        r_b = a.adv[r];
      } else {
        r_a = a.old_values[r];
        r_b = a.ret[r];
      }
    }
    if (ACTOR) {
      r_c = a.moments[2 * mb];
      r_d = a.moments[2 * mb + 1];
    }
  };
  prefetch(mb_begin);
  if (tid == 0) {
    S.pw[0] = ipow(beta1_d, step0);
    S.pw[1] = ipow(beta2_d, step0);
  }
#ifdef RAI_STAMPS
  if (tid < 32) S.stamps[tid] = 0;
  if (tid == 0) S.t_last = __builtin_amdgcn_s_memtime();
#endif
  lds_barrier();

  for (int mb = mb_begin; mb < mb_end; ++mb) {
    const int64_t row0 = (int64_t)mb * B;
    const int rows = (int)min((int64_t)B, n_rows - row0);
    const int c_act = r_act;
    const float c_a = r_a, c_b = r_b, amean = r_c, aden = r_d, c_x = r_x;
    if (mb + 1 < mb_end) prefetch(mb + 1);
    const float invB = 1.f / (float)(rows * a.world);
    const int R = w * 16;  // first row of this wave's tile

    // ============ P_A: wave-local forward, loss and backward of rows [R, R + 16) ============
    float h2[4][4];  // [col tile t][row r] = act(z2) at row R + 4g + r, column 16t + li
    {
      RELANE();
      // layer 1 (K = in_dim padded to 4): one MFMA per column tile
      f4 z[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const f4 zero = {0.f, 0.f, 0.f, 0.f};
        z[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(c_x, S.W1[16 * t + li][g], zero, 0, 0, 0);
      }
      S.X[R + li][g] = c_x;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float bj = S.b1[16 * t + li];
#pragma unroll
        for (int r = 0; r < 4; ++r) S.H1[R + g * 4 + r][16 * t + li] = act_f(relu, z[t][r] + bj);
      }
      STAMP(1);
      // layer 2 over all 64 columns (A = this wave's H1 rows, written just above)
      f4 acc[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 16; kk += 2) {
        const int kq = kmap(g, kk);
        const f2 av = *reinterpret_cast<const f2*>(&S.H1[R + li][kq]);
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
        for (int r = 0; r < 4; ++r) h2[t][r] = act_f(relu, acc[t][r] + bb);
      }
      STAMP(2);
    }
    float pw3[4][OUTP], pb2[4];  // per-lane partials over this lane's 4 rows (column 16t + li)
    float dq[OUTP];              // dL/d(out) of this lane's loss row (li & 3)
    float st[4] = {0.f, 0.f, 0.f, 0.f};
    {
      RELANE();
      float w3[4][OUTP];
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int o = 0; o < OUTP; ++o) w3[t][o] = S.W3[o][16 * t + li];
      // output layer: logits of rows R + 4g + r, summed over the 16 lanes of the DPP row
      // per-row loss gradient (ppo.py:326-371; tie rules as loss.hip) for row q = li & 3
      const int q = li & 3;
      const bool valid = R + g * 4 + q < rows;
      float z[OUTP];
#pragma unroll
      for (int o = 0; o < OUTP; ++o) {
        // logit o of rows R + 4g + r (r = 0..3), each summed over the 16 lanes of the DPP row;
        // this lane keeps row q's (scalar selects: no indexable array, which would go to scratch)
        float sel = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float p = h2[0][r] * w3[0][o];
          p = fmaf(h2[1][r], w3[1][o], p);
          p = fmaf(h2[2][r], w3[2][o], p);
          p = fmaf(h2[3][r], w3[3][o], p);
          const float lgr = row_sum16(p);
          sel = q == r ? lgr : sel;
        }
        z[o] = sel + S.b3[o];
        dq[o] = 0.f;
      }
      if (valid) {
        if (ACTOR) {
          float m = F32_MIN;
#pragma unroll
          for (int o = 0; o < OUTP; ++o)
            if (o < NA) m = fmaxf(m, z[o]);
          float se = 0.f;
#pragma unroll
          for (int o = 0; o < OUTP; ++o)
            if (o < NA) se += expf(z[o] - m);
          const float lse = m + logf(se);
          float H = 0.f;
#pragma unroll
          for (int o = 0; o < OUTP; ++o)
            if (o < NA) {
              const float n = z[o] - lse;
              H -= fmaxf(n, F32_MIN) * expf(n);
            }
          const int act = min(max(c_act, 0), NA - 1);
          float zact = z[0];
#pragma unroll
          for (int o = 1; o < OUTP; ++o)
            if (o == act) zact = z[o];
          const float logp = zact - lse;
          const float A = (c_b - amean) / aden;
          const float logratio = logp - c_a;
          const float ratio = expf(logratio);
          const float lo = 1.f - clip_range, hi = 1.f + clip_range;
          const float cr = fminf(fmaxf(ratio, lo), hi);
          const float s1 = ratio * A, s2 = cr * A;
          const float gpi = -pi_coef * invB;
          float g1, g2;
          if (s1 < s2) { g1 = gpi; g2 = 0.f; }
          else if (s1 > s2) { g1 = 0.f; g2 = gpi; }
          else { g1 = gpi * 0.5f; g2 = gpi * 0.5f; }
          const float in_clip = (ratio >= lo && ratio <= hi) ? 1.f : 0.f;
          const float dlogp = (g1 * A + (g2 * A) * in_clip) * ratio;
          const float dent = -ent_coef * invB;
#pragma unroll
          for (int o = 0; o < OUTP; ++o)
            if (o < NA) {
              const float n = z[o] - lse;
              const float p = expf(n);
              dq[o] = dlogp * ((o == act ? 1.f : 0.f) - p) + dent * (-p * (n + H));
            }
          if (li < 4) {
            st[0] = fminf(s1, s2);
            st[1] = (ratio - 1.f) - logratio;
            st[2] = (fabsf(ratio - 1.f) > clip_range) ? 1.f : 0.f;
            st[3] = H;
          }
        } else {
          const float v = z[0], Rt = c_b;
          const float gl = (vf_coef0 * halve) * invB;
          float l = vf_loss(vf_fn, v - Rt), dv;
          float vcf = 0.f;
          if (has_vclip) {
            const float vc_ = clip_range_vf;
            const float dvo = v - c_a;
            const float vcl = c_a + fminf(fmaxf(dvo, -vc_), vc_);
            const float l2 = vf_loss(vf_fn, vcl - Rt);
            float w1, w2;
            if (l > l2) { w1 = gl; w2 = 0.f; }
            else if (l < l2) { w1 = 0.f; w2 = gl; }
            else { w1 = gl * 0.5f; w2 = gl * 0.5f; }
            const float inv = (dvo >= -vc_ && dvo <= vc_) ? 1.f : 0.f;
            dv = w1 * vf_grad(vf_fn, v - Rt) + (w2 * vf_grad(vf_fn, vcl - Rt)) * inv;
            vcf = (fabsf(v - c_a) > vc_) ? 1.f : 0.f;
            l = fmaxf(l, l2);
          } else {
            dv = gl * vf_grad(vf_fn, v - Rt);
          }
          dq[0] = dv;
          if (li < 4) {
            st[0] = l;
            st[1] = vcf;
          }
        }
      }
      // dL/d(out) of the 4 rows of this lane's D-layout: quad broadcast from lane r of each quad
      float dr[4][OUTP];
#pragma unroll
      for (int o = 0; o < OUTP; ++o) {
        dr[0][o] = dpp<0x00>(dq[o]);
        dr[1][o] = dpp<0x55>(dq[o]);
        dr[2][o] = dpp<0xAA>(dq[o]);
        dr[3][o] = dpp<0xFF>(dq[o]);
      }
      // dZ2 = (dout . W3) * act'(H2) -> LDS (wave-local rows); dW3 / db2 partials
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        pb2[t] = 0.f;
#pragma unroll
        for (int o = 0; o < OUTP; ++o) pw3[t][o] = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float dh = 0.f;
#pragma unroll
          for (int o = 0; o < OUTP; ++o) {
            dh = fmaf(dr[r][o], w3[t][o], dh);
            pw3[t][o] = fmaf(dr[r][o], h2[t][r], pw3[t][o]);
          }
          const float dz = dh * act_d(relu, h2[t][r]);
          pb2[t] += dz;
          S.Z2[R + g * 4 + r][16 * t + li] = dz;
        }
      }
      STAMP(3);
    }
    float pb1[4], pw1[4][4];  // db1 / dW1 partials (column 16t + li; dW1 also per input k)
    {
      RELANE();
      // dH1 = dZ2 W2 for this wave's rows (A = dZ2 rows written above; B = W2[j][16t + li])
      f4 dh1[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) dh1[t] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 16; kk += 2) {
        const int kq = kmap(g, kk);
        const f2 av = *reinterpret_cast<const f2*>(&S.Z2[R + li][kq]);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const float bx = S.W2[kq][16 * t + li], by = S.W2[kq + 1][16 * t + li];
          dh1[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, bx, dh1[t], 0, 0, 0);
          dh1[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, by, dh1[t], 0, 0, 0);
        }
      }
      STAMP(4);
      // dZ1 = dH1 * act'(H1); db1 and dW1 partials over this lane's 4 rows
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        pb1[t] = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) pw1[t][k] = 0.f;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const f4 xr = *reinterpret_cast<const f4*>(&S.X[R + g * 4 + r][0]);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const float dz1 = dh1[t][r] * act_d(relu, S.H1[R + g * 4 + r][16 * t + li]);
          pb1[t] += dz1;
#pragma unroll
          for (int k = 0; k < 4; ++k) pw1[t][k] = fmaf(dz1, xr[k], pw1[t][k]);
        }
      }
    }
    // ---- partials: reduce over the 4 lane groups, lane group g stores column tile t == g ---------
    {
      RELANE();
      auto red4 = [&](float v) {
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        return v;
      };
      float* sp = scr + (size_t)w * NPART * HID + 16 * g + li;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        float v[NPART];
#pragma unroll
        for (int o = 0; o < OUTP; ++o) v[o] = red4(pw3[t][o]);
        v[OUTP] = red4(pb2[t]);
        v[OUTP + 1] = red4(pb1[t]);
#pragma unroll
        for (int k = 0; k < 4; ++k) v[OUTP + 2 + k] = red4(pw1[t][k]);
        if (t == g) {
#pragma unroll
          for (int p = 0; p < NPART; ++p) sp[p * HID] = v[p];
        }
      }
      // db3 and the loss statistics: lanes li < 4 hold the wave's 16 distinct rows
#pragma unroll
      for (int o = 0; o < OUTP; ++o) {
        const float t3 = wave_sum(li < 4 ? dq[o] : 0.f);
        if (lane == 0) S.db3p[w][o] = t3;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const double t = wave_sum((double)st[i]);
        if (lane == 0) S.st[w][i] = t;
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // partial-gradient stores are out
    lds_barrier();
    STAMP(5);
    // ============ P_B: dW2 = dZ2^T H1 over all rows (wave w: tile jt, kt) ============
    f4 gw2;
    {
      RELANE();
      const int jt = w >> 2, kt = w & 3;
      f4 g0 = {0.f, 0.f, 0.f, 0.f}, g1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
      for (int kk = 0; kk < RB / 4; kk += 2) {
        const int s0 = smap(g, kk), s1 = smap(g, kk + 1);
        g0 = __builtin_amdgcn_mfma_f32_16x16x4f32(S.Z2[s0][jt * 16 + li], S.H1[s0][kt * 16 + li], g0, 0, 0, 0);
        g1 = __builtin_amdgcn_mfma_f32_16x16x4f32(S.Z2[s1][jt * 16 + li], S.H1[s1][kt * 16 + li], g1, 0, 0, 0);
      }
      gw2 = g0 + g1;
    }
    STAMP(6);
    // ============ E2: owners sum the per-wave partials (fixed order); this network's |g|^2 ============
    float ga = 0.f, gb = 0.f;
    {
      RELANE();
      auto ld = [&](int wv, int p, int col) {
        return __hip_atomic_load(scr + ((size_t)wv * NPART + p) * HID + col, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
      };
      if (tid < OUT * HID) {
        const int o = tid >> 6, k = tid & 63;
        float t = 0.f;
#pragma unroll
        for (int q = 0; q < NW; ++q) t += ld(q, o, k);
        ga = t;
      } else if (tid >= 512 && tid < 512 + OUT) {
        const int o = tid - 512;
        float t = 0.f;
#pragma unroll
        for (int q = 0; q < NW; ++q) t += S.db3p[q][o];
        ga = t;
      } else if (tid >= 576 && tid < 640) {
        float t = 0.f;
#pragma unroll
        for (int q = 0; q < NW; ++q) t += ld(q, OUTP, tid - 576);
        ga = t;
      } else if (tid >= 640 && tid < 704) {
        float t = 0.f;
#pragma unroll
        for (int q = 0; q < NW; ++q) t += ld(q, OUTP + 1, tid - 640);
        ga = t;
      }
      if (tid < HID * IN) {
        const int j = tid / IN, k = tid % IN;
        float t = 0.f;
#pragma unroll
        for (int q = 0; q < NW; ++q) t += ld(q, OUTP + 2 + k, j);
        gb = t;
      }
      double ss = (double)gw2.x * gw2.x + (double)gw2.y * gw2.y + (double)gw2.z * gw2.z + (double)gw2.w * gw2.w;
      if (a_flat >= 0) ss += (double)ga * ga;
      if (b_flat >= 0) ss += (double)gb * gb;
      ss = wave_sum(ss);
      if (lane == 0) S.red[w] = ss;
      if (grads_mode) {
#pragma unroll
        for (int r = 0; r < 4; ++r) a.grad_out[oW2 + w2_idx[r]] = gw2[r];
        if (a_flat >= 0) a.grad_out[a_flat] = ga;
        if (b_flat >= 0) a.grad_out[b_flat] = gb;
      }
    }
    lds_barrier();
    STAMP(7);
    // ============ E3: stats row, grad-norm exchange, bias corrections (thread 0) ============
    if (tid == 0) {
      double ssum = 0.0;
      for (int q = 0; q < NW; ++q) ssum += S.red[q];
      double sv[4] = {0.0, 0.0, 0.0, 0.0};
      for (int q = 0; q < NW; ++q)
#pragma unroll
        for (int i = 0; i < 4; ++i) sv[i] += S.st[q][i];
      const int srow = stat0 + (mb - mb_begin);
      if (a.stats && srow < a.max_stats) {
        float* row = a.stats + (int64_t)srow * RAI_STAT_STRIDE;
        const double Bd = (double)rows * (double)a.world;
        if (ACTOR) {
          const float pi_loss = (float)(-sv[0] / Bd);
          const float ent_loss = (float)(-sv[3] / Bd);
          row[0] = pi_coef * pi_loss + ent_coef * ent_loss;  // host adds the value term
          row[1] = pi_loss;
          row[2] = ent_loss;
          row[3] = (float)(sv[1] / Bd);
          row[4] = (float)(sv[2] / Bd);
        } else {
          row[5] = (float)(sv[0] / Bd) * halve;
          row[5 + RAI_MAX_K] = has_vclip ? (float)(sv[1] / Bd) : 0.f;
        }
      }
      if (!grads_mode) {
        const float mine = (float)ssum;
        const unsigned tag = (unsigned)(mb + 1);
        const int par = mb & 1;
        const unsigned long long gr = ((unsigned long long)tag << 32) | (unsigned long long)__float_as_uint(mine);
        __hip_atomic_store(&a.xchg[net * 2 + par], gr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        float other = 0.f;
        unsigned long long spins = 0;
        for (;;) {
          const unsigned long long x =
              __hip_atomic_load(&a.xchg[(1 - net) * 2 + par], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if ((unsigned)(x >> 32) == tag) { other = __uint_as_float((unsigned)x); break; }
          if (++spins > (1ull << 26)) { atomicExch(a.err, 1); break; }  // bounded: never hangs
          __builtin_amdgcn_s_sleep(1);
        }
        S.bcast[0] = net == 0 ? mine : other;
        S.bcast[1] = net == 0 ? other : mine;
        S.pw[0] *= beta1_d;
        S.pw[1] *= beta2_d;
        const double bc1 = 1.0 - S.pw[0];
        const double bc2 = 1.0 - S.pw[1];
        S.bcast[2] = (float)sqrt(bc2);
        S.bcast[3] = (float)(-((double)lr / bc1));
      }
    }
    lds_barrier();
    STAMP(8);
    if (grads_mode) continue;
    const float total_norm = (float)sqrt((double)S.bcast[0] + (double)S.bcast[1]);
    float coef = 1.f;
    if (max_grad_norm > 0.f) coef = fminf(max_grad_norm / (total_norm + 1e-6f), 1.f);
    const float bc2_sqrt = S.bcast[2], neg_step = S.bcast[3];
    const float w1 = (float)(1.0 - beta1_d), w2 = (float)(1.0 - beta2_d);
    // ============ E4: Adam on owned parameters; refresh the LDS copies ============
    {
      RELANE();
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = (w >> 2) * 16 + g * 4 + r, k = (w & 3) * 16 + li;
        float p = S.W2[j][k];
        adam_update(p, w2_m[r], w2_v[r], gw2[r] * coef, w1, w2, beta2, bc2_sqrt, neg_step, adam_eps);
        S.W2[j][k] = p;
      }
      if (a_flat >= 0) {
        float* slot;
        if (tid < OUT * HID) slot = &S.W3[tid >> 6][tid & 63];
        else if (tid < 576) slot = &S.b3[tid - 512];
        else if (tid < 640) slot = &S.b2[tid - 576];
        else slot = &S.b1[tid - 640];
        float p = *slot;
        adam_update(p, a_m, a_v, ga * coef, w1, w2, beta2, bc2_sqrt, neg_step, adam_eps);
        *slot = p;
      }
      if (b_flat >= 0) {
        const int j = tid / IN, k = tid % IN;
        float p = S.W1[j][k];
        adam_update(p, b_m, b_v, gb * coef, w1, w2, beta2, bc2_sqrt, neg_step, adam_eps);
        S.W1[j][k] = p;
      }
      if (tid == 0) {
        if (ACTOR && a.norms && norm0 + (mb - mb_begin) < a.max_norms) a.norms[norm0 + (mb - mb_begin)] = total_norm;
      }
    }
    lds_barrier();
    STAMP(9);
  }

  // ---- write back parameters and optimizer moments (torch parameter order) -----------------------
  if (!grads_mode) {
    int t2 = tid;
    asm volatile("" : "+v"(t2));
    const int lane2 = t2 & 63, w_2 = t2 >> 6, g2 = lane2 >> 4, li2 = lane2 & 15;
    const int jt2 = w_2 >> 2, kt2 = w_2 & 3;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = jt2 * 16 + g2 * 4 + r, k = kt2 * 16 + li2;
      const int idx = oW2 + j * HID + k;
      a.params[idx] = S.W2[j][k];
      a.exp_avg[idx] = w2_m[r];
      a.exp_avg_sq[idx] = w2_v[r];
    }
    int af = -1;
    float p = 0.f;
    if (t2 < OUT * HID) { af = oW3 + t2; p = S.W3[t2 >> 6][t2 & 63]; }
    else if (t2 >= 512 && t2 < 512 + OUT) { af = ob3 + (t2 - 512); p = S.b3[t2 - 512]; }
    else if (t2 >= 576 && t2 < 640) { af = ob2 + (t2 - 576); p = S.b2[t2 - 576]; }
    else if (t2 >= 640 && t2 < 704) { af = ob1 + (t2 - 640); p = S.b1[t2 - 640]; }
    if (af >= 0) {
      a.params[af] = p;
      a.exp_avg[af] = a_m;
      a.exp_avg_sq[af] = a_v;
    }
    if (t2 < HID * IN) {
      a.params[oW1 + t2] = S.W1[t2 / IN][t2 % IN];
      a.exp_avg[oW1 + t2] = b_m;
      a.exp_avg_sq[oW1 + t2] = b_v;
    }
  }
#ifdef RAI_STAMPS
  if (tid < 32) g_stamps[net][tid] = S.stamps[tid];
#endif
  if (grads_mode && tid == 0) {
    if (!ACTOR) {
      __hip_atomic_store(&a.xchg[4], 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      unsigned long long spins = 0;
      while (__hip_atomic_load(&a.xchg[4], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == 0ull) {
        if (++spins > (1ull << 26)) { atomicExch(a.err, 1); break; }
        __builtin_amdgcn_s_sleep(1);
      }
    }
  }
  if (ACTOR && tid == 0) {
    a.state->stat_index = stat0 + nmb;
    if (!grads_mode) {
      a.state->opt_step = step0 + nmb;
      a.state->norm_index = norm0 + nmb;
    }
  }
}

template <int RELU>
__global__ __launch_bounds__(NT) void mlp_ppo_rows_kernel(const MlpArgs a) {
  static_assert(sizeof(SmemR<2>) <= 160 * 1024, "LDS budget");
  __shared__ __attribute__((aligned(16))) unsigned char smem_raw[sizeof(SmemR<2>)];
  if (blockIdx.x == 0) mlp_rows<2, true, RELU>(a, *reinterpret_cast<SmemR<2>*>(smem_raw));
  else mlp_rows<1, false, RELU>(a, *reinterpret_cast<SmemR<1>*>(smem_raw));
}

#include "mlp_mc.h"
#include "mlp_mc8.h"

template <int INP, int NAP, int RELU>
__global__ __launch_bounds__(NT) void mlp_ppo_epoch_kernel(const MlpArgs a) {
  static_assert(sizeof(Smem<INP, NAP>) <= 160 * 1024, "LDS budget");
  __shared__ __attribute__((aligned(16))) unsigned char smem_raw[sizeof(Smem<INP, NAP>)];
  if (blockIdx.x == 0) mlp_net<INP, NAP, true, RELU>(a, *reinterpret_cast<Smem<INP, NAP>*>(smem_raw));
  else mlp_net<INP, 1, false, RELU>(a, *reinterpret_cast<Smem<INP, 1>*>(smem_raw));
}

template <int INP, int NAP>
void launch_epoch(const MlpArgs& a, hipStream_t s) {
  if (a.act_fn == 1) hipLaunchKernelGGL((mlp_ppo_epoch_kernel<INP, NAP, 1>), dim3(2), dim3(NT), 0, s, a);
  else hipLaunchKernelGGL((mlp_ppo_epoch_kernel<INP, NAP, 0>), dim3(2), dim3(NT), 0, s, a);
}

}  // namespace

#ifdef RAI_STAMPS
extern "C" int rai_mlp_debug_stamps(unsigned long long* host_out) {
  return (int)hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_stamps), sizeof(g_stamps));
}
#endif

namespace {
constexpr int64_t XCHG_BYTES = 256;  // exchange words (first 64 B zeroed per launch), padded
constexpr int64_t SCRATCH_ROWS = 2LL * NW * (MAXOUT + 2 + 4) * HID * sizeof(float);
constexpr int64_t SCRATCH_MC = 2LL * 2 * MC_G * MC_SLOT * sizeof(float);
constexpr int64_t SCRATCH_MAX2 = SCRATCH_ROWS > SCRATCH_MC ? SCRATCH_ROWS : SCRATCH_MC;
constexpr int64_t SCRATCH_BYTES = SCRATCH_MAX2 > M8_SCRATCH ? SCRATCH_MAX2 : M8_SCRATCH;

// Kernel layout for the CartPole class (diagnostics / A-B only: RAI_MLP_LAYOUT=rows|chunk|mc4)
int mlp_layout() {
  const char* e = getenv("RAI_MLP_LAYOUT");
  if (e && !strcmp(e, "rows")) return 1;
  if (e && !strcmp(e, "chunk")) return 2;
  if (e && !strcmp(e, "mc4")) return 3;
  return 0;  // multi-CU: 8 CUs per network (epoch mode), 4 (data-parallel grads mode)
}

// CUs per network of the default epoch kernel (A-B: RAI_MLP_CUS=8|16)
int mlp_cus_per_net() {
  const char* e = getenv("RAI_MLP_CUS");
  return (e && !strcmp(e, "8")) ? 8 : 16;
}

// Per-rank geometry for minibatches of <= 128 rows (A-B: RAI_MLP_PER_RANK_GEO=0 keeps 16 CUs)
bool mlp_per_rank_geometry() {
  const char* e = getenv("RAI_MLP_PER_RANK_GEO");
  return !(e && !strcmp(e, "0"));
}

int64_t num_minibatches(int64_t n_rows, int32_t batch_size) {
  return batch_size > 0 ? (n_rows + batch_size - 1) / batch_size : 0;
}
int64_t moments_bytes(int64_t n_rows, int32_t batch_size) {
  return ((8 * num_minibatches(n_rows, batch_size) + 255) / 256) * 256;
}
int64_t statp_bytes(int64_t n_rows, int32_t batch_size) {
  return 2 * num_minibatches(n_rows, batch_size) * (MC_G > M8_GMAX ? MC_G : M8_GMAX) * 4 * (int64_t)sizeof(double);
}

int mlp_launch(MlpArgs& a, int32_t hidden, int32_t batch_size, int64_t n_rows, void* workspace,
               int64_t workspace_bytes, void* stream) {
  if (hidden != HID || a.in_dim < 1 || a.in_dim > MAXIN || a.n_act < 1 || a.n_act > MAXOUT ||
      batch_size < 2 || batch_size > MAXB || n_rows < 1 || (a.act_fn != 0 && a.act_fn != 1) ||
      a.world < 1)
    return RAI_E_SHAPE;
  if (!a.params || !a.obs || !a.actions || !a.old_logp || !a.old_values || !a.adv || !a.ret ||
      !a.hp || !a.ohp || !a.state || !workspace)
    return RAI_E_NULLPTR;
  if (!a.grad_out && (!a.exp_avg || !a.exp_avg_sq)) return RAI_E_NULLPTR;
  if (workspace_bytes < rai_mlp_ppo_workspace_bytes(n_rows, batch_size)) return RAI_E_WORKSPACE;
  if (n_rows % batch_size == 1 && !a.moments) return RAI_E_SHAPE;  // 1-row minibatch: no std
  if (a.grad_out && a.mb_count > 0 && (int64_t)a.mb_begin * batch_size >= n_rows) return RAI_E_SHAPE;
  a.n_rows = n_rows;
  a.batch = batch_size;
  a.xchg = reinterpret_cast<unsigned long long*>(workspace);
  a.err = &a.state->err;
  hipStream_t s = rai_stream(stream);
  if (a.sync_base == 0) {  // later launches of a data-parallel epoch keep counting on the same words
    hipError_t e = hipMemsetAsync(workspace, 0, XCHG_BYTES, s);
    if (e != hipSuccess) return (int)e;
  }
  a.scratch = reinterpret_cast<float*>(static_cast<unsigned char*>(workspace) + XCHG_BYTES);
  if (!a.moments) {
    float* mom = reinterpret_cast<float*>(static_cast<unsigned char*>(workspace) + XCHG_BYTES + SCRATCH_BYTES);
    const int64_t nmb = num_minibatches(n_rows, batch_size);
    hipLaunchKernelGGL(adv_moments_kernel, dim3((unsigned)nmb), dim3(256), 0, s, a.adv, n_rows, batch_size, a.hp,
                       mom);
    RAI_LAUNCH_CHECK();
    a.moments = mom;
  }
  a.statp = reinterpret_cast<double*>(static_cast<unsigned char*>(workspace) + XCHG_BYTES + SCRATCH_BYTES +
                                      moments_bytes(n_rows, batch_size));
  const int layout = mlp_layout();
  if (a.in_dim <= 4 && a.n_act <= 2 && layout == 0 && !a.grad_out) {
    // multi-CU layout, G CUs per network: reduce-scatter + all-gather per minibatch
    if (mlp_cus_per_net() == 16 && batch_size <= 128 && mlp_per_rank_geometry()) {
      // <= 128 rows (256 / world per rank at world 2): 8 CUs of 16 rows, not 16 CUs of which half hold no rows
      if (a.act_fn == 1) hipLaunchKernelGGL((mlp_ppo_mc8_kernel<1, 8, 16>), dim3(M8Geo<8, 16>::GRID), dim3(M8_NT), 0, s, a);
      else hipLaunchKernelGGL((mlp_ppo_mc8_kernel<0, 8, 16>), dim3(M8Geo<8, 16>::GRID), dim3(M8_NT), 0, s, a);
    } else if (mlp_cus_per_net() == 16) {
      if (a.act_fn == 1) hipLaunchKernelGGL((mlp_ppo_mc8_kernel<1, 16>), dim3(M8Geo<16>::GRID), dim3(M8_NT), 0, s, a);
      else hipLaunchKernelGGL((mlp_ppo_mc8_kernel<0, 16>), dim3(M8Geo<16>::GRID), dim3(M8_NT), 0, s, a);
    } else {
      if (a.act_fn == 1) hipLaunchKernelGGL((mlp_ppo_mc8_kernel<1, 8>), dim3(M8Geo<8>::GRID), dim3(M8_NT), 0, s, a);
      else hipLaunchKernelGGL((mlp_ppo_mc8_kernel<0, 8>), dim3(M8Geo<8>::GRID), dim3(M8_NT), 0, s, a);
    }
  } else if (a.in_dim <= 4 && a.n_act <= 2 && (layout == 0 || layout == 3)) {
    // multi-CU layout, MC_G CUs per network, partial-gradient all-reduce per minibatch
    if (a.act_fn == 1) hipLaunchKernelGGL((mlp_ppo_mc_kernel<1>), dim3(MC_GRID), dim3(MC_NT), 0, s, a);
    else hipLaunchKernelGGL((mlp_ppo_mc_kernel<0>), dim3(MC_GRID), dim3(MC_NT), 0, s, a);
  } else if (a.in_dim <= 4 && a.n_act <= 2 && layout == 1) {
    // row-tile layout on one CU per network (one pass over <= 256 rows)
    if (a.act_fn == 1) hipLaunchKernelGGL((mlp_ppo_rows_kernel<1>), dim3(2), dim3(NT), 0, s, a);
    else hipLaunchKernelGGL((mlp_ppo_rows_kernel<0>), dim3(2), dim3(NT), 0, s, a);
  } else if (a.in_dim <= 4 && a.n_act <= 2) {
    launch_epoch<4, 2>(a, s);
  } else {
    launch_epoch<8, 8>(a, s);
  }
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}
}  // namespace

extern "C" int64_t rai_mlp_ppo_workspace_bytes(int64_t n_rows, int32_t batch_size) {
  if (batch_size > MAXB) return rai_internal::mlp_large_workspace_bytes(n_rows, batch_size);
  return XCHG_BYTES + SCRATCH_BYTES + moments_bytes(n_rows, batch_size) + statp_bytes(n_rows, batch_size);
}

extern "C" int rai_mlp_ppo_epoch(float* params, float* exp_avg, float* exp_avg_sq, const float* obs,
                                 const int64_t* actions, const float* old_logp, const float* old_values,
                                 const float* advantages, const float* returns, int64_t n_rows,
                                 int32_t batch_size, int32_t in_dim, int32_t hidden, int32_t n_actions,
                                 int32_t activation, const rai_ppo_hparams* hp, const rai_optim_hparams* ohp,
                                 rai_train_state* state, float* stats, int32_t max_stats, float* norms,
                                 int32_t max_norms, void* workspace, int64_t workspace_bytes,
                                 void* stream) {
  if (batch_size > MAXB) {  // SURVEY 8(d) batch policy (b): the all-CU large-minibatch step (mlp_large.hip)
    if (!rai_internal::mlp_large_supported(in_dim, n_actions, hidden)) return RAI_E_UNSUPPORTED;
    return rai_internal::mlp_large(params, exp_avg, exp_avg_sq, obs, actions, old_logp, old_values, advantages,
                                   returns, n_rows, batch_size, in_dim, n_actions, activation, 0, 1 << 30, nullptr,
                                   1, hp, ohp, state, stats, max_stats, norms, max_norms, nullptr, workspace,
                                   workspace_bytes, rai_stream(stream));
  }
  MlpArgs a = {};
  a.params = params; a.exp_avg = exp_avg; a.exp_avg_sq = exp_avg_sq;
  a.obs = obs; a.actions = actions; a.old_logp = old_logp; a.old_values = old_values;
  a.adv = advantages; a.ret = returns;
  a.in_dim = in_dim; a.n_act = n_actions; a.act_fn = activation;
  a.hp = hp; a.ohp = ohp; a.state = state;
  a.stats = stats; a.max_stats = max_stats; a.norms = norms; a.max_norms = max_norms;
  a.grad_out = nullptr; a.moments = nullptr;
  a.mb_begin = 0; a.mb_count = 1 << 30; a.world = 1;
  a.grad_in = nullptr; a.P_total = 0; a.sync_base = 0;
  return mlp_launch(a, hidden, batch_size, n_rows, workspace, workspace_bytes, stream);
}

extern "C" int rai_mlp_ppo_epoch_xdp(float* params, float* exp_avg, float* exp_avg_sq, const float* obs,
                                     const int64_t* actions, const float* old_logp, const float* old_values,
                                     const float* advantages, const float* returns, int64_t n_rows,
                                     int32_t batch_size, const float* moments, int32_t world, int32_t rank,
                                     void* const* peers, int64_t step_base, int32_t in_dim, int32_t hidden,
                                     int32_t n_actions, int32_t activation, const rai_ppo_hparams* hp,
                                     const rai_optim_hparams* ohp, rai_train_state* state, float* stats,
                                     int32_t max_stats, float* norms, int32_t max_norms, void* workspace,
                                     int64_t workspace_bytes, void* stream) {
  if (!moments || !peers) return RAI_E_NULLPTR;
  if (world < 2 || world > XDP_MAXW || rank < 0 || rank >= world || step_base < 0) return RAI_E_SHAPE;
  if (batch_size > MAXB) {  // large minibatches (mlp_large.hip): the exchange inside each step's reduce launch
    if (!rai_internal::mlp_large_supported(in_dim, n_actions, hidden)) return RAI_E_UNSUPPORTED;
    const rai_internal::LargeXdp x = {peers, rank, world, step_base};
    return rai_internal::mlp_large(params, exp_avg, exp_avg_sq, obs, actions, old_logp, old_values, advantages,
                                   returns, n_rows, batch_size, in_dim, n_actions, activation, 0, 1 << 30, moments,
                                   world, hp, ohp, state, stats, max_stats, norms, max_norms, nullptr, workspace,
                                   workspace_bytes, rai_stream(stream), &x);
  }
  if (!(in_dim <= 4 && n_actions <= 2 && (mlp_layout() == 0 || mlp_layout() == 3))) return RAI_E_UNSUPPORTED;
  MlpArgs a = {};
  a.params = params; a.exp_avg = exp_avg; a.exp_avg_sq = exp_avg_sq;
  a.obs = obs; a.actions = actions; a.old_logp = old_logp; a.old_values = old_values;
  a.adv = advantages; a.ret = returns;
  a.in_dim = in_dim; a.n_act = n_actions; a.act_fn = activation;
  a.hp = hp; a.ohp = ohp; a.state = state;
  a.stats = stats; a.max_stats = max_stats; a.norms = norms; a.max_norms = max_norms;
  a.grad_out = nullptr; a.moments = moments;
  a.mb_begin = 0; a.mb_count = 1 << 30; a.world = world;
  a.grad_in = nullptr; a.P_total = 0; a.sync_base = 0;
  a.xpeers = peers; a.xrank = rank; a.xworld = world; a.xbase = step_base;
  return mlp_launch(a, hidden, batch_size, n_rows, workspace, workspace_bytes, stream);
}

// Setup-time canary for the cross-GPU regions: the same memory, scopes and flag protocol as
// the epoch kernel on a known payload.  bad[0] counts wrong values, bad[1] timeouts.
__global__ __launch_bounds__(64) void xdp_selftest_kernel(void* const* peers, int W, int rank,
                                                          unsigned long long tag, int* bad) {
  const int lane = threadIdx.x;
  for (int p = 0; p < W; ++p) {
    float* dst = reinterpret_cast<float*>(static_cast<char*>(peers[p]) + XDP_FLAGS_BYTES) + rank * 64 + lane;
    __hip_atomic_store(dst, (float)(rank * 1000 + lane) + (float)tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (lane < W) {
    unsigned long long* fl = reinterpret_cast<unsigned long long*>(static_cast<char*>(peers[lane]) + XDP_TEST_OFF) + rank;
    __hip_atomic_store(fl, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  const unsigned long long* own = reinterpret_cast<const unsigned long long*>(static_cast<char*>(peers[rank]) + XDP_TEST_OFF);
  unsigned long long spins = 0;
  for (;;) {
    bool ok = lane >= W || __hip_atomic_load(own + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= tag;
    if (__all(ok)) break;
    if (++spins > (1ull << 22)) {
      if (lane == 0) atomicAdd(&bad[1], 1);
      return;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  const float* src = reinterpret_cast<const float*>(static_cast<const char*>(peers[rank]) + XDP_FLAGS_BYTES);
  for (int r = 0; r < W; ++r) {
    const float v = __hip_atomic_load(src + r * 64 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (v != (float)(r * 1000 + lane) + (float)tag) atomicAdd(&bad[0], 1);
  }
}

extern "C" int rai_xdp_selftest(void* const* peers, int32_t world, int32_t rank, int64_t tag, int32_t* bad,
                                void* stream) {
  if (!peers || !bad) return RAI_E_NULLPTR;
  if (world < 1 || world > XDP_MAXW || rank < 0 || rank >= world || tag < 1) return RAI_E_SHAPE;
  hipLaunchKernelGGL(xdp_selftest_kernel, dim3(1), dim3(64), 0, rai_stream(stream), peers, (int)world, (int)rank,
                     (unsigned long long)tag, bad);
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}

extern "C" int64_t rai_xdp_region_bytes(int32_t world) {
  if (world < 1 || world > XDP_MAXW) return 0;
  static_assert(XDP_FLAGS_BYTES == RAI_XDP_SLOTS_OFF, "one region layout");
  // one region serves the CartPole-class epoch kernels (<= 256 rows and the large-minibatch steps) and the
  // wide whole-epoch kernel
  return std::max<int64_t>(std::max<int64_t>(xdp_region_bytes(world), rai_xdp_wide_bytes(world)),
                           rai_internal::mlp_large_xdp_bytes(world));
}

// Multi-CU data-parallel step (used by rai_mlp_ppo_epoch_dp): apply the previous all-reduced
// gradient (grad_in; nullptr on the first step) then compute minibatch mb's partial gradient into
// grad_out (mb_count 0: apply only).  Returns RAI_E_UNSUPPORTED for shapes outside the multi-CU
// layout; the caller then uses the three-call sequence.
int rai_mlp_ppo_dp_step(float* params, float* exp_avg, float* exp_avg_sq, const float* grad_in, int32_t P_total,
                        const float* obs, const int64_t* actions, const float* old_logp, const float* old_values,
                        const float* advantages, const float* returns, int64_t n_rows, int32_t batch_size,
                        int32_t mb, int32_t mb_count, const float* moments, int32_t world, int32_t in_dim,
                        int32_t hidden, int32_t n_actions, int32_t activation, const rai_ppo_hparams* hp,
                        const rai_optim_hparams* ohp, rai_train_state* state, float* grad_out, float* stats,
                        int32_t max_stats, float* norms, int32_t max_norms, int32_t sync_base, void* workspace,
                        int64_t workspace_bytes, void* stream) {
  if (!(in_dim <= 4 && n_actions <= 2 && (mlp_layout() == 0 || mlp_layout() == 3)) || batch_size > MAXB)
    return RAI_E_UNSUPPORTED;
  if (!grad_out || !moments || !exp_avg || !exp_avg_sq) return RAI_E_NULLPTR;
  if (mb < 0 || mb_count < 0 || sync_base < 0) return RAI_E_SHAPE;
  MlpArgs a = {};
  a.params = params; a.exp_avg = exp_avg; a.exp_avg_sq = exp_avg_sq;
  a.obs = obs; a.actions = actions; a.old_logp = old_logp; a.old_values = old_values;
  a.adv = advantages; a.ret = returns;
  a.in_dim = in_dim; a.n_act = n_actions; a.act_fn = activation;
  a.hp = hp; a.ohp = ohp; a.state = state;
  a.stats = stats; a.max_stats = max_stats; a.norms = norms; a.max_norms = max_norms;
  a.grad_out = grad_out; a.moments = moments;
  a.mb_begin = mb; a.mb_count = mb_count; a.world = world;
  a.grad_in = grad_in; a.P_total = P_total; a.sync_base = sync_base;
  return mlp_launch(a, hidden, batch_size, n_rows, workspace, workspace_bytes, stream);
}

extern "C" int rai_mlp_ppo_grads(const float* params, const float* obs, const int64_t* actions,
                                 const float* old_logp, const float* old_values,
                                 const float* advantages, const float* returns, int64_t n_rows,
                                 int32_t batch_size, int32_t mb_begin, int32_t mb_count,
                                 const float* moments, int32_t world, int32_t in_dim, int32_t hidden,
                                 int32_t n_actions, int32_t activation, const rai_ppo_hparams* hp,
                                 const rai_optim_hparams* ohp, rai_train_state* state, float* grad_out,
                                 float* stats, int32_t max_stats, void* workspace,
                                 int64_t workspace_bytes, void* stream) {
  if (!grad_out) return RAI_E_NULLPTR;
  if (mb_begin < 0 || mb_count < 1) return RAI_E_SHAPE;
  if (batch_size > MAXB) {  // large minibatches: one minibatch per call (mlp_large.hip)
    if (!rai_internal::mlp_large_supported(in_dim, n_actions, hidden)) return RAI_E_UNSUPPORTED;
    return rai_internal::mlp_large(const_cast<float*>(params), nullptr, nullptr, obs, actions, old_logp, old_values,
                                   advantages, returns, n_rows, batch_size, in_dim, n_actions, activation, mb_begin,
                                   mb_count, moments, world, hp, ohp, state, stats, max_stats, nullptr, 0, grad_out,
                                   workspace, workspace_bytes, rai_stream(stream));
  }
  MlpArgs a = {};
  a.grad_in = nullptr; a.P_total = 0; a.sync_base = 0;
  a.params = const_cast<float*>(params);
  a.obs = obs; a.actions = actions; a.old_logp = old_logp; a.old_values = old_values;
  a.adv = advantages; a.ret = returns;
  a.in_dim = in_dim; a.n_act = n_actions; a.act_fn = activation;
  a.hp = hp; a.ohp = ohp; a.state = state;
  a.stats = stats; a.max_stats = max_stats; a.norms = nullptr; a.max_norms = 0;
  a.grad_out = grad_out; a.moments = moments;
  a.mb_begin = mb_begin; a.mb_count = mb_count; a.world = world;
  return mlp_launch(a, hidden, batch_size, n_rows, workspace, workspace_bytes, stream);
}
