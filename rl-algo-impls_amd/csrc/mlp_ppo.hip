// Fused PPO epoch for small MLP actor-critics on gfx950 (CartPole-class policies).
//
// One launch runs EVERY minibatch of one epoch of rl_algo_impls/ppo/ppo.py:290-411
// for an ActorCritic whose encoder is Flatten and whose actor/critic heads are
// [in -> 64 -> 64 -> out] MLPs (rl_algo_impls/shared/policy/actor_critic_network/
// connected_trio.py + shared/actor/categorical.py + shared/policy/critic.py):
//   forward, categorical logp/entropy, clipped-surrogate + value loss gradients,
//   backward, clip_grad_norm_ and Adam(eps) — without leaving the chip.
//
// Layout: workgroup 0 owns the actor, workgroup 1 the critic (the two networks
// share no parameters; the only coupling is the global grad norm of
// clip_grad_norm_, exchanged once per minibatch as an 8-byte {tag,value} granule
// with agent-scope relaxed atomics, double-buffered by minibatch parity).  Each
// 1024-thread workgroup keeps its network's weights in LDS (W2 also transposed
// for the backward), processes the minibatch in 128-row chunks, and runs the
// three 64x64 contractions (forward, dW2, dH1) on v_mfma_f32_16x16x4_f32 — exact
// fp32 (a k-ordered fmaf chain), at the CU's full fp32 rate.  Gradients of W2
// stay in the MFMA accumulators of the wave that owns the tile, and the Adam
// moments of every parameter live in the registers of its owning lane for the
// whole launch; only the next minibatch's inputs are fetched from HBM
// (prefetched into registers one minibatch ahead).
//
// LDS banking: activations/weights use a 66-float row stride with the K index
// permuted per lane group (kmap / smap below) so the b64 A/B-operand reads of
// the forward/dH1 products and the b32 reads of the dW2 product are
// conflict-free.
#include "common.h"

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
  unsigned long long* xchg;  // [2 nets][2 parities], zeroed before every launch
  int32_t* err;
  // data-parallel "grads" mode (grad_out != nullptr): process minibatches
  // [mb_begin, mb_begin + mb_count), normalise advantages with the given global
  // per-minibatch (mean, den) pairs, scale the loss means by 1/(rows*world), write the
  // raw gradients to grad_out and stop (the caller all-reduces them and runs
  // rai_clip_optim_step).
  float* grad_out;
  const float* moments;
  int32_t mb_begin;
  int32_t mb_count;
  int32_t world;
};

#ifdef RAI_STAMPS
// Diagnostic build only (never the shipped library): per-phase cycle totals of wave 0 of
// each workgroup, accumulated over the launch and copied out by rai_mlp_debug_stamps().
__device__ unsigned long long g_stamps[2][32];
#define STAMP(i)                                                        \
  do {                                                                  \
    if (threadIdx.x == 0) {                                             \
      unsigned long long t_;                                            \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
      S.stamps[i] += t_ - S.t_last;                                     \
      S.t_last = t_;                                                    \
    }                                                                   \
  } while (0)
#else
#define STAMP(i) \
  do {           \
  } while (0)
#endif

struct Smem {
#ifdef RAI_STAMPS
  unsigned long long stamps[32];
  unsigned long long t_last;
#endif
  float W1[HID][MAXIN];
  float b1[HID];
  float W2[HID][LD];   // [out j][in k]
  float W2T[HID][LD];  // [in k][out j]
  float b2[HID];
  float W3[MAXOUT][LD];
  float b3[MAXOUT];
  float X[CH][MAXIN];
  float H1[CH][LD];    // act(z1), later dZ1
  float H2[CH][LD];    // act(z2), later dZ2
  float out[CH][MAXOUT];
  float dout[CH][MAXOUT];
  double red[8 * NW];
  double pw[2];
  float bcast[8];
};

__device__ __forceinline__ int kmap(int g, int kk) { return (g & 1) * 32 + (g >> 1) * 16 + kk; }
__device__ __forceinline__ int smap(int g, int kk) {
  return (kk >> 3) * 32 + (g >> 1) * 16 + (g & 1) * 8 + (kk & 7);
}
__device__ __forceinline__ float act_f(int relu, float z) { return relu ? fmaxf(z, 0.f) : tanhf(z); }
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

template <int NV>
__device__ __forceinline__ void bsum(double (&v)[NV], double* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = wave_sum(v[i]);
  lds_barrier();
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < NV; ++i) red[i * NW + w] = v[i];
  }
  lds_barrier();
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    double t = 0.0;
    for (int j = 0; j < NW; ++j) t += red[i * NW + j];
    v[i] = t;
  }
  lds_barrier();
}

__device__ __forceinline__ void adam_update(float& p, float& m, float& v, float g, float w1, float w2,
                                            float beta2, float bc2_sqrt, float neg_step, float eps) {
  m = m + w1 * (g - m);
  v = v * beta2;
  v = v + (w2 * g) * g;
  const float denom = sqrtf(v) / bc2_sqrt + eps;
  p = p + neg_step * (m / denom);
}

__global__ __launch_bounds__(NT) void mlp_ppo_epoch_kernel(const MlpArgs a) {
  __shared__ Smem S;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, li = lane & 15;
  const int net = blockIdx.x;  // 0 actor, 1 critic
  const int IN = a.in_dim;
  const int NA = a.n_act;
  const int OUT = net == 0 ? NA : 1;
  const int relu = a.act_fn;
  // only the hyperparameters this path uses (kept uniform / scalar)
  const float clip_range = a.hp->clip_range, ent_coef = a.hp->ent_coef, vf_coef0 = a.hp->vf_coef[0];
  const float clip_range_vf = a.hp->clip_range_vf;
  const int has_vclip = a.hp->has_clip_range_vf, vf_fn = a.hp->vf_loss_fn;
  const int norm_adv = a.hp->normalize_advantage, std_adv = a.hp->standardize_advantage;
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

  for (int e = tid; e < HID * MAXIN; e += NT) {
    const int j = e / MAXIN, k = e % MAXIN;
    S.W1[j][k] = k < IN ? a.params[oW1 + j * IN + k] : 0.f;
  }
  for (int e = tid; e < HID; e += NT) {
    S.b1[e] = a.params[ob1 + e];
    S.b2[e] = a.params[ob2 + e];
  }
  for (int e = tid; e < HID * HID; e += NT) {
    const int j = e >> 6, k = e & 63;
    const float x = a.params[oW2 + e];
    S.W2[j][k] = x;
    S.W2T[k][j] = x;
  }
  for (int e = tid; e < MAXOUT * HID; e += NT) {
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
  // thread t < B: row t's (action, old logp, old value, adv, return); X elements t and t+NT
  int64_t r_act = 0;
  float r_olp = 0.f, r_ov = 0.f, r_adv = 0.f, r_ret = 0.f, r_x0 = 0.f, r_x1 = 0.f;
  auto prefetch = [&](int mb) {
    const int64_t row0 = (int64_t)mb * B;
    const int rows = (int)min((int64_t)B, n_rows - row0);
    if (tid < rows) {
      const int64_t r = row0 + tid;
      if (net == 0) {
        r_act = a.actions[r];
        r_olp = a.old_logp[r];
        r_adv = a.adv[r];
      } else {
        r_ov = a.old_values[r];
        r_ret = a.ret[r];
      }
    }
    const int nx = rows * IN;
    r_x0 = tid < nx ? a.obs[row0 * IN + tid] : 0.f;
    r_x1 = tid + NT < nx ? a.obs[row0 * IN + tid + NT] : 0.f;
  };
  prefetch(mb_begin);
  if (tid == 0) {  // running powers beta^step (bias corrections), advanced once per minibatch
    S.pw[0] = pow(beta1_d, (double)step0);
    S.pw[1] = pow(beta2_d, (double)step0);
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
    const int64_t c_act = r_act;
    const float c_olp = r_olp, c_ov = r_ov, c_adv = r_adv, c_ret = r_ret, c_x0 = r_x0, c_x1 = r_x1;
    if (mb + 1 < mb_end) prefetch(mb + 1);

    // advantage normalisation moments over the minibatch (ppo.py:313-316), actor only
    float amean = 0.f, aden = 1.f;
    if (net == 0 && a.moments) {
      amean = a.moments[2 * mb];
      aden = a.moments[2 * mb + 1];
    } else if (net == 0 && (norm_adv || std_adv)) {
      double v1[1] = {tid < rows ? (double)c_adv : 0.0};
      bsum<1>(v1, S.red);
      const float mean = (float)(v1[0] / (double)rows);
      const double d = tid < rows ? (double)c_adv - (double)mean : 0.0;
      double v2[1] = {d * d};
      bsum<1>(v2, S.red);
      const float den = (float)sqrt(v2[0] / (double)(rows - 1)) + 1e-8f;
      if (norm_adv) { amean = mean; aden = den; }
      else { aden = den; }
    }
    const float invB = 1.f / (float)(rows * a.world);

    f4 gw2 = {0.f, 0.f, 0.f, 0.f};
    float ga = 0.f, gb = 0.f;
    float st[4] = {0.f, 0.f, 0.f, 0.f};

    for (int c = 0; c * CH < rows; ++c) {
      // Re-derive the (tid & 63) coordinates from a laundered tid every chunk so per-(tid & 63) LDS
      // addresses are computed where they are used instead of being hoisted out of the
      // loops and kept alive (that hoisting alone overflowed the 128-VGPR budget).
      int tid = threadIdx.x;
      const int crows = min(CH, rows - c * CH);
      asm volatile("" : "+v"(tid));
      // P0: minibatch X elements of this chunk -> LDS
      for (int e = tid; e < CH * MAXIN; e += NT) S.X[e / MAXIN][e % MAXIN] = 0.f;
      lds_barrier();
      STAMP(1);
      {
        const int e0 = tid, e1 = tid + NT;
        const int s0 = e0 / IN - c * CH, s1 = e1 / IN - c * CH;
        if (s0 >= 0 && s0 < crows) S.X[s0][e0 % IN] = c_x0;
        if (s1 >= 0 && s1 < crows) S.X[s1][e1 % IN] = c_x1;
      }
      lds_barrier();
      STAMP(2);
      asm volatile("" : "+v"(tid));
      // P1: layer 1 (VALU; K = in_dim <= 8)
      {
        const int j = tid & 63;
        float wv[MAXIN];
#pragma unroll
        for (int k = 0; k < MAXIN; ++k) wv[k] = S.W1[j][k];
        const float bj = S.b1[j];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int s = (tid >> 6) * 8 + i;
          float z = 0.f;
#pragma unroll
          for (int k = 0; k < MAXIN; ++k) z = fmaf(S.X[s][k], wv[k], z);
          S.H1[s][j] = act_f(relu, z + bj);
        }
      }
      lds_barrier();
      STAMP(3);
      asm volatile("" : "+v"(tid));
      // P2: layer 2 forward on MFMA: Z2[s][j] = sum_k H1[s][k] W2[j][k]
      {
        const int mt = (tid >> 6) >> 1, nt0 = ((tid >> 6) & 1) * 2;
        f4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < 16; kk += 2) {
          const int kq = kmap(((tid >> 4) & 3), kk);
          const f2 av = *reinterpret_cast<const f2*>(&S.H1[mt * 16 + (tid & 15)][kq]);
          const f2 b0 = *reinterpret_cast<const f2*>(&S.W2[nt0 * 16 + (tid & 15)][kq]);
          const f2 b1 = *reinterpret_cast<const f2*>(&S.W2[(nt0 + 1) * 16 + (tid & 15)][kq]);
          acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, b0.x, acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, b1.x, acc1, 0, 0, 0);
          acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, b0.y, acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, b1.y, acc1, 0, 0, 0);
        }
        const int j0 = nt0 * 16 + (tid & 15);
        const float bb0 = S.b2[j0], bb1 = S.b2[j0 + 16];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int s = mt * 16 + ((tid >> 4) & 3) * 4 + r;
          S.H2[s][j0] = act_f(relu, acc0[r] + bb0);
          S.H2[s][j0 + 16] = act_f(relu, acc1[r] + bb1);
        }
      }
      lds_barrier();
      STAMP(4);
      asm volatile("" : "+v"(tid));
      // P3: output layer (VALU)
      {
        const int s = tid >> 3, o = tid & 7;
        if (o < OUT) {
          float z = 0.f;
          for (int k = 0; k < HID; k += 2) {
            const f2 h = *reinterpret_cast<const f2*>(&S.H2[s][k]);
            z = fmaf(h.x, S.W3[o][k], z);
            z = fmaf(h.y, S.W3[o][k + 1], z);
          }
          S.out[s][o] = z + S.b3[o];
        }
      }
      lds_barrier();
      STAMP(5);
      asm volatile("" : "+v"(tid));
      // P4: per-sample loss gradient (tid >> 6).r.t. the head outputs (ppo.py:307-361 semantics;
      //     autograd tie rules of min/max and closed-interval clamp, as loss.hip)
      {
        const int s = tid - c * CH;
        if (s >= 0 && s < CH) {
          if (s < crows) {
            if (net == 0) {
              float m = F32_MIN;
              for (int o = 0; o < NA; ++o) m = fmaxf(m, S.out[s][o]);
              float se = 0.f;
              for (int o = 0; o < NA; ++o) se += expf(S.out[s][o] - m);
              const float lse = m + logf(se);
              float H = 0.f;
              for (int o = 0; o < NA; ++o) {
                const float n = S.out[s][o] - lse;
                H -= fmaxf(n, F32_MIN) * expf(n);
              }
              const int act = min(max((int)c_act, 0), NA - 1);
              const float logp = S.out[s][act] - lse;
              const float A = (c_adv - amean) / aden;
              const float logratio = logp - c_olp;
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
              for (int o = 0; o < MAXOUT; ++o) {
                float d = 0.f;
                if (o < NA) {
                  const float n = S.out[s][o] - lse;
                  const float p = expf(n);
                  d = dlogp * ((o == act ? 1.f : 0.f) - p) + dent * (-p * (n + H));
                }
                S.dout[s][o] = d;
              }
              st[0] += fminf(s1, s2);
              st[1] += (ratio - 1.f) - logratio;
              st[2] += (fabsf(ratio - 1.f) > clip_range) ? 1.f : 0.f;
              st[3] += H;
            } else {
              const float v = S.out[s][0], R = c_ret;
              const float gl = (vf_coef0 * halve) * invB;
              float l = vf_loss(vf_fn, v - R), dv;
              if (has_vclip) {
                const float vc_ = clip_range_vf;
                const float dvo = v - c_ov;
                const float vcl = c_ov + fminf(fmaxf(dvo, -vc_), vc_);
                const float l2 = vf_loss(vf_fn, vcl - R);
                float w1, w2;
                if (l > l2) { w1 = gl; w2 = 0.f; }
                else if (l < l2) { w1 = 0.f; w2 = gl; }
                else { w1 = gl * 0.5f; w2 = gl * 0.5f; }
                const float inv = (dvo >= -vc_ && dvo <= vc_) ? 1.f : 0.f;
                dv = w1 * vf_grad(vf_fn, v - R) + (w2 * vf_grad(vf_fn, vcl - R)) * inv;
                st[1] += (fabsf(v - c_ov) > vc_) ? 1.f : 0.f;
                l = fmaxf(l, l2);
              } else {
                dv = gl * vf_grad(vf_fn, v - R);
              }
              st[0] += l;
              for (int o = 0; o < MAXOUT; ++o) S.dout[s][o] = o == 0 ? dv : 0.f;
            }
          } else {
            for (int o = 0; o < MAXOUT; ++o) S.dout[s][o] = 0.f;
          }
        }
      }
      lds_barrier();
      STAMP(6);
      asm volatile("" : "+v"(tid));
      // P5: output-layer weight/bias grads (slot A owners)
      if (tid < OUT * HID) {
        const int o = tid >> 6, k = tid & 63;
        float acc = 0.f;
        for (int s = 0; s < CH; ++s) acc = fmaf(S.dout[s][o], S.H2[s][k], acc);
        ga += acc;
      } else if (tid >= 512 && tid < 512 + OUT) {
        const int o = tid - 512;
        float acc = 0.f;
        for (int s = 0; s < CH; ++s) acc += S.dout[s][o];
        ga += acc;
      }
      lds_barrier();
      STAMP(7);
      asm volatile("" : "+v"(tid));
      // P6: dZ2 = (dout . W3) * act'(H2), in place over H2
      {
        const int k = tid & 63;
        float w3[MAXOUT];
#pragma unroll
        for (int o = 0; o < MAXOUT; ++o) w3[o] = S.W3[o][k];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int s = (tid >> 6) + 16 * i;
          float dh = 0.f;
#pragma unroll
          for (int o = 0; o < MAXOUT; ++o) dh = fmaf(S.dout[s][o], w3[o], dh);
          S.H2[s][k] = dh * act_d(relu, S.H2[s][k]);
        }
      }
      lds_barrier();
      STAMP(8);
      asm volatile("" : "+v"(tid));
      // P7: dW2 += dZ2^T H1 (accumulators persist over chunks), dH1 = dZ2 W2 (held), db2
      f4 h0 = {0.f, 0.f, 0.f, 0.f}, h1 = {0.f, 0.f, 0.f, 0.f};
      {
#pragma unroll 8
        for (int kk = 0; kk < 32; ++kk) {
          const int s = smap(((tid >> 4) & 3), kk);
          gw2 = __builtin_amdgcn_mfma_f32_16x16x4f32(S.H2[s][(tid >> 8) * 16 + (tid & 15)], S.H1[s][((tid >> 6) & 3) * 16 + (tid & 15)], gw2, 0, 0, 0);
        }
        const int mt = (tid >> 6) >> 1, nt0 = ((tid >> 6) & 1) * 2;
#pragma unroll
        for (int kk = 0; kk < 16; kk += 2) {
          const int kq = kmap(((tid >> 4) & 3), kk);
          const f2 av = *reinterpret_cast<const f2*>(&S.H2[mt * 16 + (tid & 15)][kq]);
          const f2 b0 = *reinterpret_cast<const f2*>(&S.W2T[nt0 * 16 + (tid & 15)][kq]);
          const f2 b1 = *reinterpret_cast<const f2*>(&S.W2T[(nt0 + 1) * 16 + (tid & 15)][kq]);
          h0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, b0.x, h0, 0, 0, 0);
          h1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, b1.x, h1, 0, 0, 0);
          h0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, b0.y, h0, 0, 0, 0);
          h1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, b1.y, h1, 0, 0, 0);
        }
        if (tid >= 576 && tid < 640) {
          const int j = tid - 576;
          float acc = 0.f;
          for (int s = 0; s < CH; ++s) acc += S.H2[s][j];
          ga += acc;
        }
      }
      lds_barrier();
      STAMP(9);
      asm volatile("" : "+v"(tid));
      // P8: dZ1 = dH1 * act'(H1), in place over H1
      {
        const int mt = (tid >> 6) >> 1, k0 = ((tid >> 6) & 1) * 32 + (tid & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int s = mt * 16 + ((tid >> 4) & 3) * 4 + r;
          S.H1[s][k0] = h0[r] * act_d(relu, S.H1[s][k0]);
          S.H1[s][k0 + 16] = h1[r] * act_d(relu, S.H1[s][k0 + 16]);
        }
      }
      lds_barrier();
      STAMP(10);
      asm volatile("" : "+v"(tid));
      // P9: layer-1 weight (slot B) and bias (slot A) grads
      if (tid < HID * IN) {
        const int j = tid / IN, k = tid % IN;
        float acc = 0.f;
        for (int s = 0; s < CH; ++s) acc = fmaf(S.H1[s][j], S.X[s][k], acc);
        gb += acc;
      }
      if (tid >= 640 && tid < 704) {
        const int j = tid - 640;
        float acc = 0.f;
        for (int s = 0; s < CH; ++s) acc += S.H1[s][j];
        ga += acc;
      }
      lds_barrier();
      STAMP(11);
    }

    // ---- global grad norm (both networks), clip coefficient ---------------------------------
    double red[5];
    {
      double ss = (double)gw2.x * gw2.x + (double)gw2.y * gw2.y + (double)gw2.z * gw2.z +
                  (double)gw2.w * gw2.w;
      if (a_flat >= 0) ss += (double)ga * ga;
      if (b_flat >= 0) ss += (double)gb * gb;
      red[0] = ss; red[1] = (double)st[0]; red[2] = (double)st[1]; red[3] = (double)st[2]; red[4] = (double)st[3];
    }
    bsum<5>(red, S.red);
    if (grads_mode) {
      // raw gradients out (same flat indices as the parameters), stats row, next minibatch
#pragma unroll
      for (int r = 0; r < 4; ++r) a.grad_out[oW2 + w2_idx[r]] = gw2[r];
      if (a_flat >= 0) a.grad_out[a_flat] = ga;
      if (b_flat >= 0) a.grad_out[b_flat] = gb;
    }
    if (tid == 0) {
      const int srow = stat0 + (mb - mb_begin);
      if (a.stats && srow < a.max_stats) {
        float* row = a.stats + (int64_t)srow * RAI_STAT_STRIDE;
        const double Bd = (double)rows * (double)a.world;
        if (net == 0) {
          const float pi_loss = (float)(-red[1] / Bd);
          const float ent_loss = (float)(-red[4] / Bd);
          row[0] = pi_coef * pi_loss + ent_coef * ent_loss;  // host adds the value term
          row[1] = pi_loss;
          row[2] = ent_loss;
          row[3] = (float)(red[2] / Bd);
          row[4] = (float)(red[3] / Bd);
        } else {
          row[5] = (float)(red[1] / Bd) * halve;
          row[5 + RAI_MAX_K] = has_vclip ? (float)(red[2] / Bd) : 0.f;
        }
      }
    }
    if (grads_mode) {
      lds_barrier();
      continue;
    }
    if (tid == 0) {
      const float mine = (float)red[0];
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
    lds_barrier();
      STAMP(12);
    const float total_norm = (float)sqrt((double)S.bcast[0] + (double)S.bcast[1]);
    float coef = 1.f;
    if (max_grad_norm > 0.f) coef = fminf(max_grad_norm / (total_norm + 1e-6f), 1.f);
    const float bc2_sqrt = S.bcast[2], neg_step = S.bcast[3];
    const float w1 = (float)(1.0 - beta1_d), w2 = (float)(1.0 - beta2_d);

    // ---- Adam on owned parameters; refresh the LDS copies ----------------------------------------
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
      if (net == 0 && a.norms && norm0 + (mb - mb_begin) < a.max_norms) a.norms[norm0 + (mb - mb_begin)] = total_norm;
    }
    lds_barrier();
      STAMP(13);
  }

  // ---- write back parameters and optimizer moments (torch parameter order) -----------------------
  // Indices are recomputed from a laundered copy of tid so the compiler does not keep the
  // prologue's 64-bit addresses alive (in VGPRs) across the whole minibatch loop.
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
    if (net == 1) {
      __hip_atomic_store(&a.xchg[4], 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      unsigned long long spins = 0;
      while (__hip_atomic_load(&a.xchg[4], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == 0ull) {
        if (++spins > (1ull << 26)) { atomicExch(a.err, 1); break; }
        __builtin_amdgcn_s_sleep(1);
      }
    }
  }
  if (net == 0 && tid == 0) {
    a.state->stat_index = stat0 + nmb;
    if (!grads_mode) {
      a.state->opt_step = step0 + nmb;
      a.state->norm_index = norm0 + nmb;
    }
  }
}

}  // namespace

extern "C" int64_t rai_mlp_ppo_workspace_bytes(void) { return 64; }

#ifdef RAI_STAMPS
extern "C" int rai_mlp_debug_stamps(unsigned long long* host_out) {
  return (int)hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_stamps), sizeof(g_stamps));
}
#endif

namespace {
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
  if (workspace_bytes < rai_mlp_ppo_workspace_bytes()) return RAI_E_WORKSPACE;
  if (n_rows % batch_size == 1 && !a.moments) return RAI_E_SHAPE;  // 1-row minibatch: no std
  if (a.grad_out && (int64_t)a.mb_begin * batch_size >= n_rows) return RAI_E_SHAPE;
  a.n_rows = n_rows;
  a.batch = batch_size;
  a.xchg = reinterpret_cast<unsigned long long*>(workspace);
  a.err = &a.state->err;
  hipError_t e = hipMemsetAsync(workspace, 0, 64, rai_stream(stream));
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(mlp_ppo_epoch_kernel, dim3(2), dim3(NT), 0, rai_stream(stream), a);
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}
}  // namespace

extern "C" int rai_mlp_ppo_epoch(float* params, float* exp_avg, float* exp_avg_sq, const float* obs,
                                 const int64_t* actions, const float* old_logp, const float* old_values,
                                 const float* advantages, const float* returns, int64_t n_rows,
                                 int32_t batch_size, int32_t in_dim, int32_t hidden, int32_t n_actions,
                                 int32_t activation, const rai_ppo_hparams* hp, const rai_optim_hparams* ohp,
                                 rai_train_state* state, float* stats, int32_t max_stats, float* norms,
                                 int32_t max_norms, void* workspace, int64_t workspace_bytes,
                                 void* stream) {
  MlpArgs a = {};
  a.params = params; a.exp_avg = exp_avg; a.exp_avg_sq = exp_avg_sq;
  a.obs = obs; a.actions = actions; a.old_logp = old_logp; a.old_values = old_values;
  a.adv = advantages; a.ret = returns;
  a.in_dim = in_dim; a.n_act = n_actions; a.act_fn = activation;
  a.hp = hp; a.ohp = ohp; a.state = state;
  a.stats = stats; a.max_stats = max_stats; a.norms = norms; a.max_norms = max_norms;
  a.grad_out = nullptr; a.moments = nullptr;
  a.mb_begin = 0; a.mb_count = 1 << 30; a.world = 1;
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
  MlpArgs a = {};
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
