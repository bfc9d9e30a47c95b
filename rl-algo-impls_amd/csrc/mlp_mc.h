// Multi-CU fused PPO epoch for CartPole-class MLP actor-critics (in_dim <= 4, n_actions <= 2).
// Included once, inside mlp_ppo.hip's anonymous namespace (shares MlpArgs and the helpers).
//
// Why more than one CU per network: one CU per network is bound by its own MFMA pipe and by
// the latency of a long dependent chain per minibatch (~33 us per minibatch at 256 rows).  Here
// each network runs on G = 4 CUs; CU c owns minibatch rows [64c, 64c + 64), one 16-row tile per
// wave, computed end to end as in the row-tile layout (forward, loss, dZ2, dH1, dZ1 wave-local).
// Per minibatch the G CUs of a network all-reduce their partial gradients:
//   * each CU writes its partial (in the LDS weight layout, 19 KB) to a global slot with 16-B
//     write-through (sc1) stores, drains (vmcnt(0)), meets its workgroup barrier and bumps the
//     network's arrival counter with one agent-scope atomic (MI355X_MICROARCH.md's hand-off
//     table, first row; cdna_hip_programming.md Guideline 16, R1);
//   * one wave polls the counter, the workgroup meets a barrier, and every thread sums its 5
//     float4 chunks of all G slots in CU order (sc1 buffer loads) — so every CU of a network
//     holds the bitwise-identical full gradient and applies the identical clip + Adam to its own
//     LDS copy of the weights (no parameter broadcast);
//   * the two networks swap their squared gradient norms CU-pairwise as 8-byte {tag,value}
//     granules (R2) for clip_grad_norm_'s global norm.
// Slots are double-buffered by minibatch parity: a CU can run at most one minibatch ahead of
// the slowest CU of its network (it cannot pass the next counter wait before every CU has
// published, i.e. finished reading the previous parity).  Every spin is bounded and sets the
// state's err flag instead of hanging.  The 8 workgroups are placed by blockIdx on two XCDs
// (blocks b with b % 8 in {0, 1}; round-robin dispatch), a locality bonus, never a correctness
// requirement.

constexpr int MC_G = 4;              // CUs per network
constexpr int MC_NT = 256;           // threads per CU (4 waves, one per SIMD)
constexpr int MC_NW = MC_NT / 64;
constexpr int MC_RC = 64;            // minibatch rows per CU (MC_NW 16-row tiles)
constexpr int MC_GRID = 8 * MC_G;    // blocks launched; only b % 8 < 2 work

// Weight layout shared by LDS, the partial-gradient buffers and the exchange slots (floats).
constexpr int WL_W1 = 0;                   // [64][4]
constexpr int WL_B1 = WL_W1 + HID * 4;     // [64]
constexpr int WL_W2 = WL_B1 + HID;         // [64][LD]
constexpr int WL_B2 = WL_W2 + HID * LD;    // [64]
constexpr int WL_W3 = WL_B2 + HID;         // [OUTP][LD]
constexpr int WL_N = 4752;                 // >= WL_W3 + 2 * LD + 8, multiple of 16
constexpr int WL_CH = WL_N / 4;            // float4 chunks
constexpr int MC_CPT = (WL_CH + MC_NT - 1) / MC_NT;  // chunks owned per thread
constexpr int MC_SLOT = WL_N;
static_assert(WL_W3 + 2 * LD + 8 <= WL_N, "weight layout");

// Cross-GPU exchange region (one per rank, IPC-mapped by every other rank):
//   [0, 2048)    u64 flags[2 nets][XDP_MAXW ranks][CUs per network]: step id of the last share pushed
//   [2048, 2112) u64 self-test flags[XDP_MAXW ranks]
//   [4096, ...)  floats slots[2 parities][world][2 nets][WL_N]: each rank's gradient of the step
constexpr int XDP_MAXW = 8;
constexpr int XDP_TEST_OFF = 2048;     // self-test flags
constexpr int XDP_FLAGS_BYTES = 4096;  // slots start here
static_assert(2 * XDP_MAXW * MC_G * 8 <= XDP_TEST_OFF, "xdp flags");
__host__ __device__ constexpr long long xdp_region_bytes(int world) {
  return XDP_FLAGS_BYTES + 2LL * world * 2 * WL_N * (long long)sizeof(float);
}
constexpr int XDP_AUX = 17;  // sc0 | sc1: system-scope (cross-device) stores and loads

// sync words (u64) at the start of the workspace, zeroed before every launch
constexpr int MC_CNT = 0;     // [2 nets] arrival counters
constexpr int MC_XG = 8;      // [2 nets][MC_G][2 parities] norm granules
constexpr int MC_DONE = 24;   // critic-done counter (grads mode)

template <int OUTP>
struct SmemM {
#ifdef RAI_STAMPS
  unsigned long long stamps[32];
  unsigned long long t_last;
#endif
  double red[MC_NW];
  double pw[2];
  double st[MC_NW][4];
  float bcast[8];
  int bail;  // set when a spin timed out: every later wait would too, so the CU stops
  float db3p[MC_NW][OUTP];
  float Wt[WL_N];   // weights
  float Gb[WL_N];   // this CU's partial gradient
  float X[MC_RC][4];
  float H1[MC_RC][LD];
  float Z2[MC_RC][LD];
  float Ps[MC_NW][OUTP + 6][HID];  // per-wave partials: dW3[o], db2, db1, dW1[k]
};

template <int OUTP>
__device__ __forceinline__ int wl_b3() { return WL_W3 + OUTP * LD; }

// weight-layout index -> flat torch parameters() index of this network (-1: padding).
// Branch-free (every region computed, the right one selected): per-lane branches here split the
// gathers that use it into separate basic blocks, each waiting for its own load.
template <int OUTP>
__device__ __forceinline__ int wl_to_flat(int e, int IN, int OUT, int base) {
  const int fW1 = base, fb1 = fW1 + HID * IN, fW2 = fb1 + HID, fb2 = fW2 + HID * HID, fW3 = fb2 + HID,
            fb3 = fW3 + OUT * HID;
  constexpr int WL_B3 = WL_W3 + OUTP * LD;
  const int j1 = e >> 2, k1 = e & 3;
  const int r1 = k1 < IN ? fW1 + j1 * IN + k1 : -1;
  const int r_b1 = fb1 + (e - WL_B1);
  const int q2 = e - WL_W2, j2 = q2 / LD, k2 = q2 - j2 * LD;
  const int r2 = k2 < HID ? fW2 + j2 * HID + k2 : -1;
  const int r_b2 = fb2 + (e - WL_B2);
  const int q3 = e - WL_W3, o3 = q3 / LD, k3 = q3 - o3 * LD;
  const int r3 = (o3 < OUT && k3 < HID) ? fW3 + o3 * HID + k3 : -1;
  const int o4 = e - WL_B3;
  const int r4 = (o4 >= 0 && o4 < OUT) ? fb3 + o4 : -1;
  int f = -1;
  f = e < WL_B3 + 8 ? r4 : f;
  f = e < WL_B3 ? r3 : f;
  f = e < WL_W3 ? r_b2 : f;
  f = e < WL_B2 ? r2 : f;
  f = e < WL_W2 ? r_b1 : f;
  f = e < WL_B1 ? r1 : f;
  return f;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t mc_rsrc(const void* p, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, bytes, 0x00020000);
}
typedef unsigned int u4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f4 as_f4(u4v v) { return __builtin_bit_cast(f4, v); }
__device__ __forceinline__ u4v as_u4(f4 v) { return __builtin_bit_cast(u4v, v); }

// Wave-wide sums on the VALU (DPP row butterflies + lane swaps) instead of ds_bpermute shuffles:
// a fixed combination order in which every lane ends with the same bits (common.h wave_sum_dpp).
__device__ __forceinline__ float wave_sum_v(float v) { return wave_sum_dpp(v); }
__device__ __forceinline__ double wave_sum_v(double v) { return wave_sum_dpp(v); }

// torch Adam step (m, v, denom = sqrt(v)/sqrt(bc2) + eps, p -= lr/bc1 * m/denom) with the
// hardware sqrt / reciprocal (1 ulp each) instead of the IEEE-exact sequences: ~1e-7 relative
// on the update, inside the fp32 tolerance the parity tests state.
__device__ __forceinline__ void adam_update_fast(float& p, float& m, float& v, float g, float w1, float w2,
                                                 float beta2, float inv_bc2_sqrt, float neg_step, float eps) {
  m = m + w1 * (g - m);
  v = v * beta2;
  v = v + (w2 * g) * g;
  const float denom = __builtin_amdgcn_sqrtf(v) * inv_bc2_sqrt + eps;
  p = p + neg_step * (m * __builtin_amdgcn_rcpf(denom));
}

// The same update on an element pair in packed fp32 (v_pk_mul_f32 / v_pk_fma_f32 / v_pk_add_f32: two
// elements per VALU op; per element the identical IEEE operations, so identical results), the square
// root and reciprocal per element.  The 8-CU epoch kernel's whole-network Adam is on every step's
// critical path.
typedef float f2a __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void adam_update_fast2(f2a& p, f2a& m, f2a& v, f2a g, float w1, float w2, float beta2,
                                                  float inv_bc2_sqrt, float neg_step, float eps) {
  const f2a W1 = {w1, w1}, W2 = {w2, w2}, B2 = {beta2, beta2}, IB = {inv_bc2_sqrt, inv_bc2_sqrt}, EP = {eps, eps},
            NS = {neg_step, neg_step};
  m = m + W1 * (g - m);
  v = v * B2;
  v = v + (W2 * g) * g;
  const f2a sq = {__builtin_amdgcn_sqrtf(v.x), __builtin_amdgcn_sqrtf(v.y)};
  const f2a denom = sq * IB + EP;
  const f2a rc = {__builtin_amdgcn_rcpf(denom.x), __builtin_amdgcn_rcpf(denom.y)};
  p = p + NS * (m * rc);
}

// Branch-free gather: the load is issued unconditionally (clamped index) and masked after, so
// a run of them stays in one basic block with all loads in flight (a guarded load becomes a
// branch, and the wait for its data is then placed before the next one is issued).
__device__ __forceinline__ float ld_or0(const float* p, int f) {
  const float v = p[f >= 0 ? f : 0];
  return f >= 0 ? v : 0.f;
}

template <int OUTP, bool ACTOR, int RELU>
__device__ __forceinline__ void mlp_mc(const MlpArgs& a, SmemM<OUTP>& S, const int c) {
  constexpr int net = ACTOR ? 0 : 1;
  constexpr int relu = RELU;
  constexpr int NPART = OUTP + 6;
  constexpr int WL_B3 = WL_W3 + OUTP * LD;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
#ifdef RAI_STAMPS
  const unsigned long long t_entry = __builtin_amdgcn_s_memtime();
#endif
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
  const bool apply_in = grads_mode && a.grad_in != nullptr;  // data-parallel step: apply grad_in first
  const float max_grad_norm = a.ohp->max_grad_norm;
  const unsigned long long sbase = (unsigned long long)a.sync_base;
  unsigned long long* const sync = a.xchg;
  float* const slots = a.scratch;  // [2 nets][2 parities][MC_G][MC_SLOT]
  const int slot_bytes = 2 * 2 * MC_G * MC_SLOT * (int)sizeof(float);
  const __amdgpu_buffer_rsrc_t srs = mc_rsrc(slots, slot_bytes);
  const int nmb_all = (int)((a.n_rows + a.batch - 1) / a.batch);
  const __amdgpu_buffer_rsrc_t str = mc_rsrc(a.statp, 2 * nmb_all * MC_G * 32);

  const int szA = HID * IN + HID + HID * HID + HID + NA * HID + NA;
  const int base = net == 0 ? 0 : szA;

  // ---- weights -> LDS (weight layout); partial-gradient buffer zeroed (padding stays 0) -------
  {
    // fully unrolled so all ~19 loads per thread are in flight at once (a rolled loop waits for
    // each load before the next: ~19 memory latencies, paid on every data-parallel launch)
    constexpr int NE = (WL_N + MC_NT - 1) / MC_NT;
    float wv[NE];
#pragma unroll
    for (int i = 0; i < NE; ++i) {
      const int e = tid + MC_NT * i;
      const int f = e < WL_N ? wl_to_flat<OUTP>(e, IN, OUT, base) : -1;
      wv[i] = ld_or0(a.params, f);
    }
#pragma unroll
    for (int i = 0; i < NE; ++i) {
      const int e = tid + MC_NT * i;
      if (e < WL_N) {
        S.Wt[e] = wv[i];
        S.Gb[e] = 0.f;
      }
    }
  }
  // ---- Adam moments of the owned chunks (chunk ch = tid + MC_NT * i), in registers -----------
#ifdef RAI_STAMPS
  const unsigned long long t_w = __builtin_amdgcn_s_memtime();
#endif
  f4 mreg[MC_CPT], vreg[MC_CPT];
#pragma unroll
  for (int i = 0; i < MC_CPT; ++i) {
    mreg[i] = f4{0.f, 0.f, 0.f, 0.f};
    vreg[i] = f4{0.f, 0.f, 0.f, 0.f};
    const int ch = tid + MC_NT * i;
    if (!grads_mode || apply_in) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int f = ch < WL_CH ? wl_to_flat<OUTP>(4 * ch + q, IN, OUT, base) : -1;
        mreg[i][q] = ld_or0(a.exp_avg, f);
        vreg[i][q] = ld_or0(a.exp_avg_sq, f);
      }
    }
  }

#ifdef RAI_STAMPS
  const unsigned long long t_mv = __builtin_amdgcn_s_memtime();
#endif
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

  int r_act = 0;
  float r_a = 0.f, r_b = 0.f, r_c = 0.f, r_d = 1.f, r_x = 0.f;
  auto prefetch = [&](int mb) {
    const int64_t row0 = (int64_t)mb * B;
    const int rows = (int)min((int64_t)B, n_rows - row0);
    int ln = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    asm volatile("" : "+v"(ln));
    const int xr = c * MC_RC + w * 16 + (ln & 15), xg = ln >> 4;
    r_x = (xr < rows && xg < IN) ? a.obs[(row0 + xr) * IN + xg] : 0.f;
    const int rr = c * MC_RC + w * 16 + (ln >> 4) * 4 + (ln & 3);
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
  if (nmb > 0) prefetch(mb_begin);
  if (tid == 0) {
    S.pw[0] = ipow(beta1_d, step0);
    S.pw[1] = ipow(beta2_d, step0);
    S.bail = 0;
  }
  __syncthreads();
#ifdef RAI_STAMPS
  const unsigned long long t_pre = __builtin_amdgcn_s_memtime();
  unsigned long long t_ss = t_pre;
#endif
  if (apply_in) {
    // ---- data-parallel step: clip_grad_norm_ + Adam with the previous step's all-reduced gradient.
    // Every CU of both networks computes the same global norm over the same flat vector in the
    // same order, so every copy of the weights gets the identical update. -----------------------
    double ss = 0.0;
    {
      constexpr int U = 16;  // loads in flight per thread per batch
      for (int i0 = tid; i0 < a.P_total; i0 += MC_NT * U) {
        float gv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int i = i0 + u * MC_NT;
          gv[u] = ld_or0(a.grad_in, i < a.P_total ? i : -1);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) ss += (double)gv[u] * gv[u];
      }
    }
    ss = wave_sum_v(ss);
    if (lane == 0) S.red[w] = ss;
    __syncthreads();
#ifdef RAI_STAMPS
    t_ss = __builtin_amdgcn_s_memtime();
#endif
    double tot = 0.0;
    for (int q = 0; q < MC_NW; ++q) tot += S.red[q];
    const float total_norm = (float)sqrt(tot);
    float coef = 1.f;
    if (max_grad_norm > 0.f) coef = fminf(max_grad_norm / (total_norm + 1e-6f), 1.f);
    const double bc1 = 1.0 - ipow(beta1_d, step0 + 1);
    const double bc2 = 1.0 - ipow(beta2_d, step0 + 1);
    const float inv_bc2_sqrt = 1.f / (float)sqrt(bc2), neg_step = (float)(-((double)lr / bc1));
    const float w1 = (float)(1.0 - beta1_d), w2 = (float)(1.0 - beta2_d);
    f4 gin[MC_CPT];  // all gathers first (one batch in flight), then the updates
#pragma unroll
    for (int i = 0; i < MC_CPT; ++i) {
      const int ch = tid + MC_NT * i;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        gin[i][q] = ld_or0(a.grad_in, ch < WL_CH ? wl_to_flat<OUTP>(4 * ch + q, IN, OUT, base) : -1);
    }
#pragma unroll
    for (int i = 0; i < MC_CPT; ++i) {
      const int ch = tid + MC_NT * i;
      if (ch < WL_CH) {
        f4 p = *reinterpret_cast<const f4*>(&S.Wt[4 * ch]);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int f = wl_to_flat<OUTP>(4 * ch + q, IN, OUT, base);
          const float gq = gin[i][q];
          float pq = p[q], mq = mreg[i][q], vq = vreg[i][q];
          adam_update_fast(pq, mq, vq, gq * coef, w1, w2, beta2, inv_bc2_sqrt, neg_step, adam_eps);
          if (f >= 0) {
            p[q] = pq;
            mreg[i][q] = mq;
            vreg[i][q] = vq;
          }
        }
        *reinterpret_cast<f4*>(&S.Wt[4 * ch]) = p;
      }
    }
    if (ACTOR && c == 0 && tid == 0 && a.norms && norm0 < a.max_norms) a.norms[norm0] = total_norm;
    __syncthreads();
  }
#ifdef RAI_STAMPS
  const unsigned long long t_ap = __builtin_amdgcn_s_memtime();
#endif
#ifdef RAI_STAMPS
  if (tid < 32) S.stamps[tid] = 0;
  if (tid == 0) {
    S.stamps[14] = t_w - t_entry;      // weights -> LDS
    S.stamps[15] = t_mv - t_w;         // Adam moments -> registers
    S.stamps[16] = t_pre - t_mv;       // prefetch issue, pw, barrier
    S.stamps[17] = apply_in ? t_ss - t_pre : 0;  // apply: global |g|^2
    S.stamps[18] = t_ap - (apply_in ? t_ss : t_pre);  // apply: Adam
    S.t_last = __builtin_amdgcn_s_memtime();
  }
#endif
  __syncthreads();

  // Bounded waits, by elapsed s_memrealtime ticks (the constant 100 MHz counter, common.h
  // rai_clock): 2 s for partners on this GPU (they are co-resident and a minibatch apart at most),
  // 60 s for other GPUs (their ranks can start an epoch later by host-side jitter: rollouts,
  // collectives).  A timeout sets err and stops the CU.
  constexpr long long MC_WAIT_LOCAL = RAI_SPIN_LOCAL, MC_WAIT_REMOTE = RAI_SPIN_REMOTE;
  for (int mb = mb_begin; mb < mb_end; ++mb) {
    const int kk_mb = mb - mb_begin;
    const int par = mb & 1;
    const int64_t row0 = (int64_t)mb * B;
    const int rows = (int)min((int64_t)B, n_rows - row0);
    const int c_act = r_act;
    const float c_a = r_a, c_b = r_b, amean = r_c, aden = r_d, c_x = r_x;
    if (mb + 1 < mb_end) prefetch(mb + 1);
    const float invB = 1.f / (float)(rows * a.world);
    const int R = w * 16;               // first local row of this wave's tile
    const int RG = c * MC_RC + R;       // ... and its row within the minibatch

    // ============ P_A: wave-local forward, loss and backward of rows [RG, RG + 16) ============
    float h2[4][4];
    {
      RELANE();
      f4 z[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const f4 zero = {0.f, 0.f, 0.f, 0.f};
        z[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(c_x, S.Wt[WL_W1 + (16 * t + li) * 4 + g], zero, 0, 0, 0);
      }
      S.X[R + li][g] = c_x;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float bj = S.Wt[WL_B1 + 16 * t + li];
#pragma unroll
        for (int r = 0; r < 4; ++r) S.H1[R + g * 4 + r][16 * t + li] = act_f(relu, z[t][r] + bj);
      }
      f4 acc[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 16; kk += 2) {
        const int kq = kmap(g, kk);
        const f2 av = *reinterpret_cast<const f2*>(&S.H1[R + li][kq]);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const f2 bv = *reinterpret_cast<const f2*>(&S.Wt[WL_W2 + (16 * t + li) * LD + kq]);
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, bv.x, acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, bv.y, acc[t], 0, 0, 0);
        }
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float bb = S.Wt[WL_B2 + 16 * t + li];
#pragma unroll
        for (int r = 0; r < 4; ++r) h2[t][r] = act_f(relu, acc[t][r] + bb);
      }
    }
    STAMP(1);
    float pw3[4][OUTP], pb2[4];
    float dq[OUTP];
    float st[4] = {0.f, 0.f, 0.f, 0.f};
    {
      RELANE();
      float w3[4][OUTP];
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int o = 0; o < OUTP; ++o) w3[t][o] = S.Wt[WL_W3 + o * LD + 16 * t + li];
      const int q = li & 3;
      const bool valid = RG + g * 4 + q < rows;
      float z[OUTP];
#pragma unroll
      for (int o = 0; o < OUTP; ++o) {
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
        z[o] = sel + S.Wt[WL_B3 + o];
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
      float dr[4][OUTP];
#pragma unroll
      for (int o = 0; o < OUTP; ++o) {
        dr[0][o] = dpp<0x00>(dq[o]);
        dr[1][o] = dpp<0x55>(dq[o]);
        dr[2][o] = dpp<0xAA>(dq[o]);
        dr[3][o] = dpp<0xFF>(dq[o]);
      }
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
    }
    STAMP(2);
    float pb1[4], pw1[4][4];
    {
      RELANE();
      f4 dh1[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) dh1[t] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 16; kk += 2) {
        const int kq = kmap(g, kk);
        const f2 av = *reinterpret_cast<const f2*>(&S.Z2[R + li][kq]);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const float bx = S.Wt[WL_W2 + kq * LD + 16 * t + li];
          const float by = S.Wt[WL_W2 + (kq + 1) * LD + 16 * t + li];
          dh1[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, bx, dh1[t], 0, 0, 0);
          dh1[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, by, dh1[t], 0, 0, 0);
        }
      }
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
    {
      RELANE();
      // sum over the 4 lane groups (lanes l, l^16, l^32, l^48) with VALU lane swaps
      auto red4 = [&](float v) {
        const auto a16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
        v = __uint_as_float(a16[0]) + __uint_as_float(a16[1]);
        const auto a32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
        return __uint_as_float(a32[0]) + __uint_as_float(a32[1]);
      };
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
          for (int p = 0; p < NPART; ++p) S.Ps[w][p][16 * g + li] = v[p];
        }
      }
#pragma unroll
      for (int o = 0; o < OUTP; ++o) {
        const float t3 = wave_sum_v(li < 4 ? dq[o] : 0.f);
        if (lane == 0) S.db3p[w][o] = t3;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const double t = wave_sum_v((double)st[i]);
        if (lane == 0) S.st[w][i] = t;
      }
    }
    lds_barrier();
    STAMP(3);
    // ============ P_B: this CU's dW2 partial (wave w: row tile jt = w of dW2, 4 column tiles) =====
    {
      RELANE();
      f4 gacc[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) gacc[t] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
      for (int kk = 0; kk < MC_RC / 4; ++kk) {
        const int s = smap(g, kk);
        const float av = S.Z2[s][w * 16 + li];
#pragma unroll
        for (int t = 0; t < 4; ++t)
          gacc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, S.H1[s][t * 16 + li], gacc[t], 0, 0, 0);
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) S.Gb[WL_W2 + (w * 16 + g * 4 + r) * LD + t * 16 + li] = gacc[t][r];
      // the other tensors: sum the per-wave partials in wave order
      for (int e = tid; e < HID * 4 + 2 * HID + OUTP * HID + OUTP; e += MC_NT) {
        float sum = 0.f;
        int dst;
        if (e < HID * 4) {  // W1[j][k]
          const int j = e >> 2, k = e & 3;
#pragma unroll
          for (int q = 0; q < MC_NW; ++q) sum += S.Ps[q][OUTP + 2 + k][j];
          dst = WL_W1 + e;
        } else if (e < HID * 5) {  // b1
          const int j = e - HID * 4;
#pragma unroll
          for (int q = 0; q < MC_NW; ++q) sum += S.Ps[q][OUTP + 1][j];
          dst = WL_B1 + j;
        } else if (e < HID * 6) {  // b2
          const int j = e - HID * 5;
#pragma unroll
          for (int q = 0; q < MC_NW; ++q) sum += S.Ps[q][OUTP][j];
          dst = WL_B2 + j;
        } else if (e < HID * 6 + OUTP * HID) {  // W3[o][k]
          const int o = (e - HID * 6) >> 6, k = (e - HID * 6) & 63;
#pragma unroll
          for (int q = 0; q < MC_NW; ++q) sum += S.Ps[q][o][k];
          dst = WL_W3 + o * LD + k;
        } else {  // b3
          const int o = e - HID * 6 - OUTP * HID;
#pragma unroll
          for (int q = 0; q < MC_NW; ++q) sum += S.db3p[q][o];
          dst = WL_B3 + o;
        }
        S.Gb[dst] = sum;
      }
    }
    lds_barrier();
    STAMP(4);
    // ============ publish this CU's partial (sc1 16-B stores), arrive on the network counter ======
    {
      RELANE();
      const int sbase = ((net * 2 + par) * MC_G + c) * MC_SLOT * (int)sizeof(float);
#pragma unroll
      for (int i = 0; i < MC_CPT; ++i) {
        const int ch = tid + MC_NT * i;
        if (ch < WL_CH) {
          const f4 v = *reinterpret_cast<const f4*>(&S.Gb[4 * ch]);
          __builtin_amdgcn_raw_buffer_store_b128(as_u4(v), srs, sbase + 16 * ch, 0, 16);
        }
      }
      if (tid == 0) {  // this CU's loss statistics (4 doubles); CU 0 turns them into rows at the end
        double sv[4] = {0.0, 0.0, 0.0, 0.0};
        for (int q = 0; q < MC_NW; ++q)
#pragma unroll
          for (int i = 0; i < 4; ++i) sv[i] += S.st[q][i];
        const u4v p0 = __builtin_bit_cast(u4v, (double __attribute__((ext_vector_type(2)))){sv[0], sv[1]});
        const u4v p1 = __builtin_bit_cast(u4v, (double __attribute__((ext_vector_type(2)))){sv[2], sv[3]});
        const int so = ((net * nmb + kk_mb) * MC_G + c) * 32;
        __builtin_amdgcn_raw_buffer_store_b128(p0, str, so, 0, 16);
        __builtin_amdgcn_raw_buffer_store_b128(p1, str, so + 16, 0, 16);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // EVERY storing wave drains its stores
    }
    __syncthreads();
    if (tid == 0) {
      __hip_atomic_fetch_add(&sync[MC_CNT + net], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long want = (unsigned long long)MC_G * (sbase + (unsigned long long)(kk_mb + 1));
      const unsigned long long t0 = rai_clock();
      while (__hip_atomic_load(&sync[MC_CNT + net], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
        if (rai_expired(t0, MC_WAIT_LOCAL)) { atomicExch(a.err, 1); S.bail = 1; break; }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __syncthreads();
    if (S.bail) break;
    STAMP(5);
    // ============ reduce: every thread sums its chunks over the G slots in CU order ============
    f4 gr[MC_CPT];
    {
      RELANE();
      const int pbase = (net * 2 + par) * MC_G * MC_SLOT * (int)sizeof(float);
      double ss = 0.0;
      // every load of the phase issued up front (clamped chunk index, masked after the sums)
      f4 v[MC_CPT][MC_G];
#pragma unroll
      for (int i = 0; i < MC_CPT; ++i) {
        const int chl = min(tid + MC_NT * i, WL_CH - 1);
#pragma unroll
        for (int cc = 0; cc < MC_G; ++cc)
          v[i][cc] = as_f4(__builtin_amdgcn_raw_buffer_load_b128(
              srs, pbase + cc * MC_SLOT * (int)sizeof(float) + 16 * chl, 0, 16));
      }
#pragma unroll
      for (int i = 0; i < MC_CPT; ++i) {
        const int ch = tid + MC_NT * i;
        gr[i] = f4{0.f, 0.f, 0.f, 0.f};
        if (ch < WL_CH) {
          f4 sum = v[i][0];
#pragma unroll
          for (int cc = 1; cc < MC_G; ++cc) sum += v[i][cc];
          gr[i] = sum;
        }
      }
      if (a.xworld > 1) {
        // ---- cross-GPU sum over xGMI peer memory: CU c pushes its 1/G share of this rank's
        // gradient into every rank's region (system-scope 16-B stores), drains, then stamps one
        // flag per receiver; each CU waits for all world*G flags of this step in its own region
        // and sums the world slots in rank order (identical bits on every rank). ------------------
        const int W = a.xworld;
        const unsigned long long step_id = (unsigned long long)(a.xbase + kk_mb + 1);
        const int xpar = (int)((a.xbase + kk_mb) & 1);  // global-step parity: mb restarts at 0 every launch
        const int slot_off = XDP_FLAGS_BYTES + ((xpar * W + a.xrank) * 2 + net) * WL_N * (int)sizeof(float);
        for (int pr = 0; pr < W; ++pr) {
          const __amdgpu_buffer_rsrc_t prs = mc_rsrc(a.xpeers[pr], (int)xdp_region_bytes(W));
#pragma unroll
          for (int i = 0; i < MC_CPT; ++i) {
            const int ch = tid + MC_NT * i;
            if (ch < WL_CH && ch % MC_G == c)
              __builtin_amdgcn_raw_buffer_store_b128(as_u4(gr[i]), prs, slot_off + 16 * ch, 0, XDP_AUX);
          }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave: shares landed
        __syncthreads();
        if (tid < W) {  // one flag store per receiver, after the whole workgroup drained
          unsigned long long* fl = reinterpret_cast<unsigned long long*>(a.xpeers[tid]) +
                                   (net * XDP_MAXW + a.xrank) * MC_G + c;
          __hip_atomic_store(fl, step_id, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        if (w == 0) {  // one wave polls this rank's W*G flags of this network
          const unsigned long long* fl = reinterpret_cast<const unsigned long long*>(a.xpeers[a.xrank]) +
                                         net * XDP_MAXW * MC_G;
          const unsigned long long t0 = rai_clock();
          for (;;) {
            bool ok = true;
            if (lane < W * MC_G)
              ok = __hip_atomic_load(fl + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= step_id;
            if (__all(ok)) break;
            if (rai_expired(t0, MC_WAIT_REMOTE)) {
              if (lane == 0) { atomicExch(a.err, 1); S.bail = 1; }
              break;
            }
            __builtin_amdgcn_s_sleep(1);
          }
        }
        __syncthreads();
        const __amdgpu_buffer_rsrc_t lrs = mc_rsrc(a.xpeers[a.xrank], (int)xdp_region_bytes(W));
#pragma unroll
        for (int i = 0; i < MC_CPT; ++i) {
          const int chl = min(tid + MC_NT * i, WL_CH - 1);
          f4 sum = f4{0.f, 0.f, 0.f, 0.f};
          for (int pr = 0; pr < W; ++pr) {
            const int off = XDP_FLAGS_BYTES + ((xpar * W + pr) * 2 + net) * WL_N * (int)sizeof(float);
            sum += as_f4(__builtin_amdgcn_raw_buffer_load_b128(lrs, off + 16 * chl, 0, XDP_AUX));
          }
          if (tid + MC_NT * i < WL_CH) gr[i] = sum;
        }
      }
#pragma unroll
      for (int i = 0; i < MC_CPT; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) ss += (double)gr[i][q] * gr[i][q];
      ss = wave_sum_v(ss);
      if (lane == 0) S.red[w] = ss;
      if (grads_mode) {  // raw gradients out in flat order (every CU holds them: each writes 1/G)
#pragma unroll
        for (int i = 0; i < MC_CPT; ++i) {
          const int ch = tid + MC_NT * i;
          if (ch < WL_CH && ch % MC_G == c) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int f = wl_to_flat<OUTP>(4 * ch + q, IN, OUT, base);
              if (f >= 0) a.grad_out[f] = gr[i][q];
            }
          }
        }
      }
    }
    lds_barrier();
    if (S.bail) break;
    STAMP(6);
    // ============ stats row (CU 0), norm exchange with the other network, bias corrections ============
    if (tid == 0) {
      double ssum = 0.0;
      for (int q = 0; q < MC_NW; ++q) ssum += S.red[q];
      if (!grads_mode) {
        const float mine = (float)ssum;
        const unsigned tag = (unsigned)(kk_mb + 1);
        const unsigned long long gv = ((unsigned long long)tag << 32) | (unsigned long long)__float_as_uint(mine);
        __hip_atomic_store(&sync[MC_XG + (net * MC_G + c) * 2 + par], gv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        float other = 0.f;
        const unsigned long long t0 = rai_clock();
        for (;;) {
          const unsigned long long x = __hip_atomic_load(&sync[MC_XG + ((1 - net) * MC_G + c) * 2 + par],
                                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if ((unsigned)(x >> 32) == tag) { other = __uint_as_float((unsigned)x); break; }
          if (rai_expired(t0, MC_WAIT_LOCAL)) { atomicExch(a.err, 1); S.bail = 1; break; }
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
    if (S.bail) break;
    STAMP(7);
    if (grads_mode) continue;
    {
      const float total_norm = (float)sqrt((double)S.bcast[0] + (double)S.bcast[1]);
      float coef = 1.f;
      if (max_grad_norm > 0.f) coef = fminf(max_grad_norm / (total_norm + 1e-6f), 1.f);
      const float inv_bc2_sqrt = 1.f / S.bcast[2], neg_step = S.bcast[3];
      const float w1 = (float)(1.0 - beta1_d), w2 = (float)(1.0 - beta2_d);
      RELANE();
#pragma unroll
      for (int i = 0; i < MC_CPT; ++i) {
        const int ch = tid + MC_NT * i;
        if (ch < WL_CH) {
          f4 p = *reinterpret_cast<const f4*>(&S.Wt[4 * ch]);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            float pq = p[q], mq = mreg[i][q], vq = vreg[i][q];
            adam_update_fast(pq, mq, vq, gr[i][q] * coef, w1, w2, beta2, inv_bc2_sqrt, neg_step, adam_eps);
            p[q] = pq;
            mreg[i][q] = mq;
            vreg[i][q] = vq;
          }
          *reinterpret_cast<f4*>(&S.Wt[4 * ch]) = p;
        }
      }
      if (ACTOR && c == 0 && tid == 0 && a.norms && norm0 + kk_mb < a.max_norms) a.norms[norm0 + kk_mb] = total_norm;
    }
    lds_barrier();
    STAMP(8);
  }

  STAMP(12);
  // ---- stats rows of every minibatch (CU 0): sum the CUs' partials in CU order ---------------------
  // (every CU published minibatch k's partial before the counter wait CU 0 passed for k)
  if (c == 0 && !S.bail && a.stats) {
    for (int k = tid; k < nmb; k += MC_NT) {
      const int srow = stat0 + k;
      if (srow >= a.max_stats) continue;
      const int64_t r0 = (int64_t)(mb_begin + k) * B;
      const int rws = (int)min((int64_t)B, n_rows - r0);
      double sv[4] = {0.0, 0.0, 0.0, 0.0};
      for (int cc = 0; cc < MC_G; ++cc) {
        const int so = ((net * nmb + k) * MC_G + cc) * 32;
        const auto d0 = __builtin_bit_cast(double __attribute__((ext_vector_type(2))),
                                           __builtin_amdgcn_raw_buffer_load_b128(str, so, 0, 16));
        const auto d1 = __builtin_bit_cast(double __attribute__((ext_vector_type(2))),
                                           __builtin_amdgcn_raw_buffer_load_b128(str, so + 16, 0, 16));
        sv[0] += d0[0];
        sv[1] += d0[1];
        sv[2] += d1[0];
        sv[3] += d1[1];
      }
      float* row = a.stats + (int64_t)srow * RAI_STAT_STRIDE;
      const double Bd = (double)rws * (double)a.world;
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
  }
  // ---- write back parameters and optimizer moments -----------------------------------------------
  if ((!grads_mode || apply_in) && !S.bail) {  // identical copies on every CU: each writes 1/G
#pragma unroll
    for (int i = 0; i < MC_CPT; ++i) {
      const int ch = tid + MC_NT * i;
      if (ch < WL_CH && ch % MC_G == c) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int f = wl_to_flat<OUTP>(4 * ch + q, IN, OUT, base);
          if (f >= 0) {
            a.params[f] = S.Wt[4 * ch + q];
            a.exp_avg[f] = mreg[i][q];
            a.exp_avg_sq[f] = vreg[i][q];
          }
        }
      }
    }
  }
  STAMP(13);
#ifdef RAI_STAMPS
  if (c == 0 && tid < 32) atomicAdd(&g_stamps[net][tid], S.stamps[tid]);  // summed over launches
#endif
  if (grads_mode && tid == 0) {  // the actor's CU 0 advances stat_index after every critic CU read it
    if (!ACTOR) {
      __hip_atomic_fetch_add(&sync[MC_DONE], 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else if (c == 0) {
      const unsigned long long t0 = rai_clock();
      while (__hip_atomic_load(&sync[MC_DONE], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) <
             (unsigned long long)MC_G * (sbase + 1)) {
        if (rai_expired(t0, MC_WAIT_LOCAL)) { atomicExch(a.err, 1); break; }
        __builtin_amdgcn_s_sleep(1);
      }
    }
  }
  if (ACTOR && c == 0 && tid == 0) {
    a.state->stat_index = stat0 + nmb;
    if (!grads_mode) {
      a.state->opt_step = step0 + nmb;
      a.state->norm_index = norm0 + nmb;
    } else if (apply_in) {
      a.state->opt_step = step0 + 1;
      a.state->norm_index = norm0 + 1;
    }
  }
}

template <int RELU>
__global__ __launch_bounds__(MC_NT) void mlp_ppo_mc_kernel(const MlpArgs a) {
  static_assert(sizeof(SmemM<2>) <= 160 * 1024, "LDS budget");
  __shared__ __attribute__((aligned(16))) unsigned char smem_raw[sizeof(SmemM<2>)];
  const int b = blockIdx.x, xcd = b & 7, c = b >> 3;
  if (xcd >= 2) return;  // only two XCDs' worth of blocks work (locality, not correctness)
  if (xcd == 0) mlp_mc<2, true, RELU>(a, *reinterpret_cast<SmemM<2>*>(smem_raw), c);
  else mlp_mc<1, false, RELU>(a, *reinterpret_cast<SmemM<1>*>(smem_raw), c);
}
