// Eight-CU-per-network fused PPO epoch for CartPole-class MLP actor-critics (in_dim <= 4,
// n_actions <= 2): the default epoch kernel (single GPU and in-kernel cross-GPU exchange).
// Included once, after mlp_mc.h, inside mlp_ppo.hip's anonymous namespace (shares MlpArgs, the
// weight layout WL_* and the helpers).
//
// Why 8 CUs and two exchange rounds.  With 4 CUs per network (mlp_mc.h) a minibatch step is ~65 %
// wave-serial compute: each wave carries one 16-row tile through ~200 dependent MFMAs plus the
// activation / loss / reduction VALU work, one wave per SIMD, nothing to hide latency behind.
// Here each network runs on G = 8 CUs owning 32 minibatch rows each; the two 16-row tiles of a CU
// are each split by hidden-unit column halves over a pair of waves (wave w: tile w >> 1, columns
// [32 (w & 1), +32)), which halves every wave's MFMA chain (forward, dH1, dW2 partial) and its
// activation work, at the price of three more LDS barriers per step (the halves meet at H1, at the
// output-layer partial sums and at dZ2).
//
// Reading all G partial slots (the 4-CU design's all-reduce) would double to 152 KB per CU per
// step at G = 8 — and those sc1 loads run at the cross-XCD rate (~60 GB/s per CU), so the
// gradient is all-reduced as reduce-scatter + all-gather instead:
//   round 1  every CU stores its 19 KB partial (16-B sc1 stores), drains, arrives on the
//            network's counter; CU c then sums share c (149 float4 chunks) over the G slots in CU
//            order (19 KB read) and, with several GPUs, adds the other ranks' share c through
//            xGMI peer memory (rank order);
//   round 2  CU c stores its summed share plus the share's squared norm, drains, arrives on a
//            second counter; every CU waits for both networks' round-2 counters, reads the summed
//            gradient of its network (19 KB) and the 16 share norms of both networks (fixed
//            order: every CU on every rank forms the bit-identical clip_grad_norm_ total), and
//            applies the identical clip + Adam to its own LDS copy of the weights.
// The norm needs no separate exchange.  Publish form: write-through (sc1) by default; when the step-0
// arrival shows every CU of the network on ONE XCC (HW_REG_XCC_ID, registered by each CU before it
// arrives), the partial and summed-share slots go out as plain stores drained into that XCC's L2 (the
// lines stay there; write-through drops them and the readers then fetch past the L2).  The readers'
// loads stay sc1 (past their own L1 only) and the share norms, read by the other network's XCC, stay
// write-through.  Placement decides only the store form, never correctness.  Slots are
// double-buffered by minibatch parity; the reuse argument is the 4-CU one per round (a CU cannot pass round r of step k + 1 before every
// CU that reads its round-r slot of step k has published round r + 1 of step k, or round 1 of
// step k + 1).  Every spin is bounded by elapsed clock and sets state.err.

constexpr int M8_GMAX = 16;                          // largest CUs-per-network instantiation
constexpr int M8_NT = 256;                           // threads per CU (4 waves)
constexpr int M8_NW = M8_NT / 64;
// Geometry for G CUs per network: RC rows per CU in NTILE 16-row tiles, WPT waves per tile, each
// wave owning CT 16-column tiles of the hidden layers; SH float4 chunks per gradient share.  RC defaults
// to MAXB / G (a 256-row minibatch over all G CUs); the per-rank geometry of data parallel keeps RC = 16
// at G = 8 for minibatches of <= 128 rows (256 / world rows per rank at world 2), so no CU of the
// network idles through the exchange.
template <int G, int RCV = MAXB / G>
struct M8Geo {
  static constexpr int RC = RCV;
  static constexpr int NTILE = RC / 16;
  static constexpr int WPT = M8_NW / NTILE;
  static constexpr int CT = HID / 16 / WPT;
  static constexpr int SH = (WL_CH + G - 1) / G;
  static constexpr int GRID = 8 * G;                 // blocks launched; only b % 8 < 2 work
  static_assert(RC % 16 == 0 && NTILE * WPT == M8_NW && CT * WPT * 16 == HID, "geometry");
  static_assert(SH <= M8_NT, "one share chunk per thread");
};
// sync words (u64, zeroed per launch): round-1 and round-2 arrival counters per network; per network
// the set of XCCs its CUs run on (one bit per HW_REG_XCC_ID)
constexpr int M8_CNT1 = 0;
constexpr int M8_CNT2 = 2;
constexpr int M8_XCC = 6;
// Adam's bias corrections are tabulated in LDS for the first M8_BC_MAX steps of a launch (C2: 2,048
// minibatches per epoch launch); later steps form them in the loop
constexpr int M8_BC_MAX = 2048;
// scratch (workspace) layout, bytes (sized for M8_GMAX; smaller G use a prefix of each region)
constexpr int64_t M8_S1_BYTES = 2LL * 2 * M8_GMAX * WL_N * sizeof(float);  // [net][par][c][WL_N] partials
constexpr int64_t M8_S2_OFF = M8_S1_BYTES;                                  // [net][par][WL_N] summed gradient
constexpr int64_t M8_SQ_OFF = M8_S2_OFF + 2LL * 2 * WL_N * sizeof(float);   // [par][net][c][hi, lo] share |g|^2 granules
constexpr int64_t M8_SCRATCH = M8_SQ_OFF + 2LL * 2 * M8_GMAX * M8_NW * sizeof(double);
static_assert(2 * XDP_MAXW * M8_GMAX * 8 <= XDP_TEST_OFF, "xdp share flags");

template <int OUTP, int G, int RCV>
struct SmemM8 {
  using Geo = M8Geo<G, RCV>;
#ifdef RAI_STAMPS
  unsigned long long stamps[32];
  unsigned long long t_last;
#endif
  double sq[M8_NW];  // round 2: the wave parts of this CU's share |g|^2
  float strow[Geo::RC][4];  // per-row loss statistics, reduced off the critical path (round-1 wait)
  int bail;
  int xl;            // every CU of this network on one XCC: gradient slots published with plain stores
  float bc[M8_BC_MAX][2];  // per step of the launch: Adam's 1 / sqrt(1 - beta2^t) and -lr / (1 - beta1^t)
  float db3p[Geo::NTILE][OUTP];
  float Wt[WL_N];    // weights
  float Gb[WL_N];    // this CU's partial gradient
  // this step's rows (staged by wave 3 in the previous step's waits): observations zero-padded to 4
  // columns (the F1 operand and dW1's X), actions, old log-prob / value, advantage / return, and the
  // normalized advantage
  alignas(16) float px[Geo::RC][4];
  int pact[Geo::RC];
  float pa[Geo::RC], pb[Geo::RC], pA[Geo::RC];
  float H1[Geo::RC][LD];
  float Z2[Geo::RC][LD];
  float Zp[Geo::WPT][Geo::RC][OUTP];  // output-layer partial sums of the column parts
  float Ps[Geo::NTILE][OUTP + 6][HID];  // per-tile partials: dW3[o], db2, db1, dW1[k]
};

// Per-row PPO loss gradient (reference: rl_algo_impls/ppo/ppo.py:326-377) for one row's logits
// (actor) or value (critic): dq = dLoss/dz, st = the row's statistics contributions.
struct RowLossHp {
  float clip_range, ent_coef, pi_coef, invB, vf_coef0, halve, clip_range_vf;
  int has_vclip, vf_fn, NA;
};
template <int OUTP, bool ACTOR>
__device__ __forceinline__ void ppo_row_loss(const float (&z)[OUTP], const RowLossHp& h, int c_act, float c_a,
                                             float c_b, float A, float (&dq)[OUTP], float (&st)[4]) {
  if (ACTOR) {
    const int NA = h.NA;
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
    const float logratio = logp - c_a;
    const float ratio = expf(logratio);
    const float lo = 1.f - h.clip_range, hi = 1.f + h.clip_range;
    const float cr = fminf(fmaxf(ratio, lo), hi);
    const float s1 = ratio * A, s2 = cr * A;
    const float gpi = -h.pi_coef * h.invB;
    float g1, g2;
    if (s1 < s2) { g1 = gpi; g2 = 0.f; }
    else if (s1 > s2) { g1 = 0.f; g2 = gpi; }
    else { g1 = gpi * 0.5f; g2 = gpi * 0.5f; }
    const float in_clip = (ratio >= lo && ratio <= hi) ? 1.f : 0.f;
    const float dlogp = (g1 * A + (g2 * A) * in_clip) * ratio;
    const float dent = -h.ent_coef * h.invB;
#pragma unroll
    for (int o = 0; o < OUTP; ++o)
      if (o < NA) {
        const float n = z[o] - lse;
        const float p = expf(n);
        dq[o] = dlogp * ((o == act ? 1.f : 0.f) - p) + dent * (-p * (n + H));
      }
    st[0] = fminf(s1, s2);
    st[1] = (ratio - 1.f) - logratio;
    st[2] = (fabsf(ratio - 1.f) > h.clip_range) ? 1.f : 0.f;
    st[3] = H;
  } else {
    const float v = z[0], Rt = c_b;
    const float gl = (h.vf_coef0 * h.halve) * h.invB;
    float l = vf_loss(h.vf_fn, v - Rt), dv;
    float vcf = 0.f;
    if (h.has_vclip) {
      const float vc_ = h.clip_range_vf;
      const float dvo = v - c_a;
      const float vcl = c_a + fminf(fmaxf(dvo, -vc_), vc_);
      const float l2 = vf_loss(h.vf_fn, vcl - Rt);
      float w1, w2;
      if (l > l2) { w1 = gl; w2 = 0.f; }
      else if (l < l2) { w1 = 0.f; w2 = gl; }
      else { w1 = gl * 0.5f; w2 = gl * 0.5f; }
      const float inv = (dvo >= -vc_ && dvo <= vc_) ? 1.f : 0.f;
      dv = w1 * vf_grad(h.vf_fn, v - Rt) + (w2 * vf_grad(h.vf_fn, vcl - Rt)) * inv;
      vcf = (fabsf(v - c_a) > vc_) ? 1.f : 0.f;
      l = fmaxf(l, l2);
    } else {
      dv = gl * vf_grad(h.vf_fn, v - Rt);
    }
    dq[0] = dv;
    st[0] = l;
    st[1] = vcf;
  }
}

// bounded spin of one lane until sync[i0] and sync[i1] both reach `want`
__device__ __forceinline__ bool m8_wait2(unsigned long long* sync, int i0, int i1, unsigned long long want,
                                         long long limit) {
  const unsigned long long t0 = rai_clock();
  while (__hip_atomic_load(&sync[i0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want ||
         __hip_atomic_load(&sync[i1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
    if (rai_expired(t0, limit)) return false;
    __builtin_amdgcn_s_sleep(1);
  }
  return true;
}

template <int OUTP, bool ACTOR, int RELU, int G, int RCV>
__device__ __forceinline__ void mlp_mc8(const MlpArgs& a, SmemM8<OUTP, G, RCV>& S, const int c) {
  using Geo = M8Geo<G, RCV>;
  constexpr int RC = Geo::RC, WPT = Geo::WPT, CT = Geo::CT, NTILE = Geo::NTILE, SH = Geo::SH;
  constexpr int net = ACTOR ? 0 : 1;
  constexpr int relu = RELU;
  constexpr int NPART = OUTP + 6;
  constexpr int WL_B3 = WL_W3 + OUTP * LD;
  const int tid = threadIdx.x;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int T = w / WPT;  // this wave's row tile (its hidden-column part: w % WPT)
#ifdef RAI_STAMPS
  if (tid < 32) S.stamps[tid] = 0;
#endif
  const int IN = a.in_dim;
  const int NA = a.n_act;
  const int OUT = ACTOR ? NA : 1;
  RowLossHp lh;
  lh.clip_range = a.hp->clip_range;
  lh.ent_coef = a.hp->ent_coef;
  lh.vf_coef0 = a.hp->vf_coef[0];
  lh.clip_range_vf = a.hp->clip_range_vf;
  lh.has_vclip = a.hp->has_clip_range_vf;
  lh.vf_fn = a.hp->vf_loss_fn;
  lh.halve = a.hp->ppo2_vf_coef_halving ? 0.5f : 1.f;
  lh.NA = NA;
  float beta2 = a.ohp->beta2, adam_eps = a.ohp->eps;
  const float lr = a.ohp->lr;
  const double beta1_d = a.ohp->beta1_d, beta2_d = a.ohp->beta2_d;
  float max_grad_norm = a.ohp->max_grad_norm;
  float w1c = (float)(1.0 - beta1_d), w2c = (float)(1.0 - beta2_d);  // Adam's lerp / addcmul weights
  unsigned long long* const sync = a.xchg;
  const __amdgpu_buffer_rsrc_t srs = mc_rsrc(a.scratch, (int)M8_SCRATCH);
  // [par][net][c][hi, lo] share-norm granules (within the share-norm region)
  unsigned long long* const sq_gran =
      reinterpret_cast<unsigned long long*>(reinterpret_cast<unsigned char*>(a.scratch) + M8_SQ_OFF);
  const int nmb_all = (int)((a.n_rows + a.batch - 1) / a.batch);
  const __amdgpu_buffer_rsrc_t str = mc_rsrc(a.statp, 2 * nmb_all * G * 32);

  const int szA = HID * IN + HID + HID * HID + HID + NA * HID + NA;
  const int base = net == 0 ? 0 : szA;

  // ---- weights -> LDS (weight layout); partial-gradient buffer zeroed (padding stays 0) -------
  {
    constexpr int NE = (WL_N + M8_NT - 1) / M8_NT;
    float wv[NE];
#pragma unroll
    for (int i = 0; i < NE; ++i) {
      const int e = tid + M8_NT * i;
      wv[i] = ld_or0(a.params, e < WL_N ? wl_to_flat<OUTP>(e, IN, OUT, base) : -1);
    }
#pragma unroll
    for (int i = 0; i < NE; ++i) {
      const int e = tid + M8_NT * i;
      if (e < WL_N) {
        S.Wt[e] = wv[i];
        S.Gb[e] = 0.f;
      }
    }
  }
  // ---- Adam moments of chunks ch = tid + M8_NT * i (every CU updates the whole network) -------
  f4 mreg[MC_CPT], vreg[MC_CPT];
#pragma unroll
  for (int i = 0; i < MC_CPT; ++i) {
    const int ch = tid + M8_NT * i;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int f = ch < WL_CH ? wl_to_flat<OUTP>(4 * ch + q, IN, OUT, base) : -1;
      mreg[i][q] = ld_or0(a.exp_avg, f);
      vreg[i][q] = ld_or0(a.exp_avg_sq, f);
    }
  }

  const int B = a.batch;
  const int64_t n_rows = a.n_rows;
  const int nmb = nmb_all;
  const int64_t step0 = a.state->opt_step;
  const int stat0 = a.state->stat_index;
  const int norm0 = a.state->norm_index;
  lh.pi_coef = a.state->pi_coef_zero ? 0.f : 1.f;

  // The step's rows are staged by wave 3 off the critical path: its loads issue in the previous step's
  // round-1 wait and land in LDS in its round-2 wait (step 0's before the loop), so the step itself only
  // reads LDS -- no global address arithmetic or load issue ahead of F1.
  constexpr int PXN = (RC * 4 + 63) / 64;  // observation floats per lane of wave 3
  float q_x[PXN], q_a = 0.f, q_b = 0.f, q_c = 0.f, q_d = 1.f;
  int q_act = 0;
  auto pf_issue = [&](int m) {
    const int64_t r0 = (int64_t)m * B;
    const int rws = (int)min((int64_t)B, n_rows - r0);
    const int ln = tid & 63;
#pragma unroll
    for (int k = 0; k < PXN; ++k) {
      const int e = ln + 64 * k, row = c * RC + (e >> 2), col = e & 3;
      q_x[k] = (e < RC * 4 && row < rws && col < IN) ? a.obs[(r0 + row) * IN + col] : 0.f;
    }
    q_act = 0;
    q_a = q_b = 0.f;
    if (ln < RC && c * RC + ln < rws) {
      const int64_t r = r0 + c * RC + ln;
      if (ACTOR) {
        q_act = (int)a.actions[r];
        q_a = a.old_logp[r];
        q_b = a.adv[r];
      } else {
        q_a = a.old_values[r];
        q_b = a.ret[r];
      }
    }
    if (ACTOR) {
      q_c = a.moments[2 * m];
      q_d = a.moments[2 * m + 1];
    }
  };
  auto pf_store = [&]() {
    const int ln = tid & 63;
#pragma unroll
    for (int k = 0; k < PXN; ++k) {
      const int e = ln + 64 * k;
      if (e < RC * 4) S.px[e >> 2][e & 3] = q_x[k];
    }
    if (ln < RC) {
      S.pact[ln] = q_act;
      S.pa[ln] = q_a;
      S.pb[ln] = q_b;
      if (ACTOR) S.pA[ln] = (q_b - q_c) / q_d;  // (adv - mean) / (std + eps): the loss's divide, staged
    }
  };
  if (w == 3 && nmb > 0) {
    pf_issue(0);
    pf_store();
  }
  // Adam's bias corrections of every step of the launch, t = step0 + mb + 1, as the per-minibatch
  // optimizer forms them (ipow, fp64): tabulated here, so no fp64 divide sits in the step loop
  auto bias_corr = [&](int mb, float& inv_bc2_sqrt, float& neg_step) {
    const long long t = step0 + mb + 1;
    inv_bc2_sqrt = 1.f / (float)sqrt(1.0 - ipow(beta2_d, t));
    neg_step = (float)(-((double)lr / (1.0 - ipow(beta1_d, t))));
  };
  for (int k = tid; k < min(nmb, M8_BC_MAX); k += M8_NT) bias_corr(k, S.bc[k][0], S.bc[k][1]);
  if (tid == 0) {
    S.bail = 0;
    S.xl = 0;
    // register this CU's XCC (completed before its first round-1 arrival: the vmcnt wait below)
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
    __hip_atomic_fetch_or(&sync[M8_XCC + net], 1ull << (xcc & 15), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
#ifdef RAI_STAMPS
  if (tid == 0) S.t_last = __builtin_amdgcn_s_memtime();
#endif

  // the loss's 1 / (rows x world) off the step's critical path, for a full and for the last minibatch
  float invB_full = 1.f / (float)(B * a.world);
  float invB_last = nmb > 0 ? 1.f / (float)((int)(n_rows - (int64_t)(nmb - 1) * B) * a.world) : 0.f;
  // loop-invariant floats held in VGPRs: uniform, but the kernel runs at the SGPR limit, and kept in SGPRs
  // they are spilled to VGPR lanes and restored with v_readlane inside the step
  asm volatile("" : "+v"(beta2), "+v"(adam_eps), "+v"(max_grad_norm), "+v"(w1c), "+v"(w2c), "+v"(invB_full),
               "+v"(invB_last));
  asm volatile("" : "+v"(lh.clip_range), "+v"(lh.ent_coef), "+v"(lh.vf_coef0), "+v"(lh.halve), "+v"(lh.clip_range_vf),
               "+v"(lh.pi_coef));

  constexpr long long MC_WAIT_LOCAL = RAI_SPIN_LOCAL, MC_WAIT_REMOTE = RAI_SPIN_REMOTE;
  for (int mb = 0; mb < nmb; ++mb) {
    const int par = mb & 1;
    const int64_t row0 = (int64_t)mb * B;
    const int rows = (int)min((int64_t)B, n_rows - row0);
    int ln0 = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    asm volatile("" : "+v"(ln0));
    const float c_x = S.px[T * 16 + (ln0 & 15)][ln0 >> 4];
    const int lrow = T * 16 + (ln0 >> 4) * 4 + (ln0 & 3);  // the loss's row of this lane
    const int c_act = S.pact[lrow];
    const float c_a = S.pa[lrow], c_b = S.pb[lrow], c_A = ACTOR ? S.pA[lrow] : 0.f;
    lh.invB = mb + 1 < nmb ? invB_full : invB_last;
    const int R = T * 16;              // first local row of this wave's tile
    const int RG = c * RC + R;         // ... and its row within the minibatch

    // ============ F1: H1 = act(X W1^T + b1) for this wave's columns of its tile ============
    {
      RELANE();
      const int T_ = w / WPT, hf_ = w % WPT;
      f4 z[CT];
#pragma unroll
      for (int tt = 0; tt < CT; ++tt) {
        const f4 zero = {0.f, 0.f, 0.f, 0.f};
        z[tt] = __builtin_amdgcn_mfma_f32_16x16x4f32(c_x, S.Wt[WL_W1 + (16 * (CT * hf_ + tt) + li) * 4 + g], zero,
                                                     0, 0, 0);
      }
#pragma unroll
      for (int tt = 0; tt < CT; ++tt) {
        const int t = CT * hf_ + tt;
        const float bj = S.Wt[WL_B1 + 16 * t + li];
#pragma unroll
        for (int r = 0; r < 4; ++r) S.H1[16 * T_ + g * 4 + r][16 * t + li] = act_f(relu, z[tt][r] + bj);
      }
    }
    STAMP(15);  // work done; the barrier wait follows
    lds_barrier();
    STAMP(1);
    // ============ F2: H2 = act(H1 W2^T + b2), own columns; output-layer partial sums ============
    float h2[CT][4];
    float w3[CT][OUTP];
    {
      RELANE();
      const int T_ = w / WPT, hf_ = w % WPT;
      f4 acc[CT];
#pragma unroll
      for (int tt = 0; tt < CT; ++tt) acc[tt] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 16; kk += 2) {
        const int kq = kmap(g, kk);
        const f2 av = *reinterpret_cast<const f2*>(&S.H1[16 * T_ + li][kq]);
#pragma unroll
        for (int tt = 0; tt < CT; ++tt) {
          const f2 bv = *reinterpret_cast<const f2*>(&S.Wt[WL_W2 + (16 * (CT * hf_ + tt) + li) * LD + kq]);
          acc[tt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, bv.x, acc[tt], 0, 0, 0);
          acc[tt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, bv.y, acc[tt], 0, 0, 0);
        }
      }
#pragma unroll
      for (int tt = 0; tt < CT; ++tt) {
        const int t = CT * hf_ + tt;
        const float bb = S.Wt[WL_B2 + 16 * t + li];
#pragma unroll
        for (int r = 0; r < 4; ++r) h2[tt][r] = act_f(relu, acc[tt][r] + bb);
#pragma unroll
        for (int o = 0; o < OUTP; ++o) w3[tt][o] = S.Wt[WL_W3 + o * LD + 16 * t + li];
      }
      const int q = li & 3;
#pragma unroll
      for (int o = 0; o < OUTP; ++o) {
        float sel = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float p = h2[0][r] * w3[0][o];
#pragma unroll
          for (int tt = 1; tt < CT; ++tt) p = fmaf(h2[tt][r], w3[tt][o], p);
          const float s16 = row_sum16(p);
          sel = q == r ? s16 : sel;
        }
        if (li < 4) S.Zp[hf_][16 * T_ + g * 4 + li][o] = sel;
      }
    }
    STAMP(16);  // work done; the barrier wait follows
    lds_barrier();
    STAMP(2);
    // ============ loss (both halves, identical), dZ2 on own columns ============
    float pw3[CT][OUTP], pb2[CT];
    float dq[OUTP];
    {
      RELANE();
      const int T_ = w / WPT, hf_ = w % WPT;
      const int q = li & 3;
      const int lr_ = 16 * T_ + g * 4 + q;
      float z[OUTP];
#pragma unroll
      for (int o = 0; o < OUTP; ++o) {
        float zs = S.Zp[0][lr_][o];
#pragma unroll
        for (int h = 1; h < WPT; ++h) zs += S.Zp[h][lr_][o];
        z[o] = zs + S.Wt[WL_B3 + o];
        dq[o] = 0.f;
      }
      float sr[4] = {0.f, 0.f, 0.f, 0.f};
      if (RG + g * 4 + q < rows) ppo_row_loss<OUTP, ACTOR>(z, lh, c_act, c_a, c_b, c_A, dq, sr);
      if (li < 4 && hf_ == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) S.strow[lr_][i] = sr[i];
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
      for (int tt = 0; tt < CT; ++tt) {
        const int t = CT * hf_ + tt;
        pb2[tt] = 0.f;
#pragma unroll
        for (int o = 0; o < OUTP; ++o) pw3[tt][o] = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float dh = 0.f;
#pragma unroll
          for (int o = 0; o < OUTP; ++o) {
            dh = fmaf(dr[r][o], w3[tt][o], dh);
            pw3[tt][o] = fmaf(dr[r][o], h2[tt][r], pw3[tt][o]);
          }
          const float dz = dh * act_d(relu, h2[tt][r]);
          pb2[tt] += dz;
          S.Z2[16 * T_ + g * 4 + r][16 * t + li] = dz;
        }
      }
    }
    STAMP(17);  // work done; the barrier wait follows
    lds_barrier();
    STAMP(3);
    // ============ dH1 = dZ2 W2 (own columns), dZ1, per-tile partials ============
    {
      RELANE();
      const int T_ = w / WPT, hf_ = w % WPT;
      f4 dh1[CT];
#pragma unroll
      for (int tt = 0; tt < CT; ++tt) dh1[tt] = f4{0.f, 0.f, 0.f, 0.f};
      // every operand read before the first MFMA (one LDS latency instead of one per k step)
      f2 avs[8];
      float bxs[8][CT], bys[8][CT];
#pragma unroll
      for (int k2 = 0; k2 < 8; ++k2) {
        const int kq = kmap(g, 2 * k2);
        avs[k2] = *reinterpret_cast<const f2*>(&S.Z2[16 * T_ + li][kq]);
#pragma unroll
        for (int tt = 0; tt < CT; ++tt) {
          const int t = CT * hf_ + tt;
          bxs[k2][tt] = S.Wt[WL_W2 + kq * LD + 16 * t + li];
          bys[k2][tt] = S.Wt[WL_W2 + (kq + 1) * LD + 16 * t + li];
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k2 = 0; k2 < 8; ++k2) {
#pragma unroll
        for (int tt = 0; tt < CT; ++tt) {
          dh1[tt] = __builtin_amdgcn_mfma_f32_16x16x4f32(avs[k2].x, bxs[k2][tt], dh1[tt], 0, 0, 0);
          dh1[tt] = __builtin_amdgcn_mfma_f32_16x16x4f32(avs[k2].y, bys[k2][tt], dh1[tt], 0, 0, 0);
        }
      }
      float pb1[CT], pw1[CT][4];
#pragma unroll
      for (int tt = 0; tt < CT; ++tt) {
        pb1[tt] = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) pw1[tt][k] = 0.f;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const f4 xr = *reinterpret_cast<const f4*>(&S.px[16 * T_ + g * 4 + r][0]);
#pragma unroll
        for (int tt = 0; tt < CT; ++tt) {
          const int t = CT * hf_ + tt;
          const float dz1 = dh1[tt][r] * act_d(relu, S.H1[16 * T_ + g * 4 + r][16 * t + li]);
          pb1[tt] += dz1;
#pragma unroll
          for (int k = 0; k < 4; ++k) pw1[tt][k] = fmaf(dz1, xr[k], pw1[tt][k]);
        }
      }
      // sum over the 4 lane groups (rows of the tile) with VALU lane swaps
      auto red4 = [&](float v) {
        const auto a16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
        v = __uint_as_float(a16[0]) + __uint_as_float(a16[1]);
        const auto a32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
        return __uint_as_float(a32[0]) + __uint_as_float(a32[1]);
      };
#pragma unroll
      for (int tt = 0; tt < CT; ++tt) {
        float v[NPART];
#pragma unroll
        for (int o = 0; o < OUTP; ++o) v[o] = red4(pw3[tt][o]);
        v[OUTP] = red4(pb2[tt]);
        v[OUTP + 1] = red4(pb1[tt]);
#pragma unroll
        for (int k = 0; k < 4; ++k) v[OUTP + 2 + k] = red4(pw1[tt][k]);
        if (g == tt) {
          const int j = 16 * (CT * hf_ + tt) + li;
          if constexpr (NTILE == 1) {  // one tile: its partials are the CU's sums (P_B copies nothing)
#pragma unroll
            for (int o = 0; o < OUTP; ++o) S.Gb[WL_W3 + o * LD + j] = v[o];
            S.Gb[WL_B2 + j] = v[OUTP];
            S.Gb[WL_B1 + j] = v[OUTP + 1];
            *reinterpret_cast<f4*>(&S.Gb[WL_W1 + 4 * j]) = f4{v[OUTP + 2], v[OUTP + 3], v[OUTP + 4], v[OUTP + 5]};
          } else {
#pragma unroll
            for (int p = 0; p < NPART; ++p) S.Ps[T_][p][j] = v[p];
          }
        }
      }
      if (hf_ == 0) {  // per-tile loss sums, once per tile
#pragma unroll
        for (int o = 0; o < OUTP; ++o) {
          const float t3 = wave_sum_v(li < 4 ? dq[o] : 0.f);
          if (lane == 0) {
            if constexpr (NTILE == 1) S.Gb[WL_B3 + o] = t3;
            else S.db3p[T_][o] = t3;
          }
        }
      }
    }
    STAMP(18);  // work done; the barrier wait follows
    lds_barrier();
    STAMP(4);
    // ============ P_B: dW2 partial over the CU's RC rows (wave w: dW2 rows [16w, 16w + 16)) =====
    {
      RELANE();
      f4 gacc[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) gacc[t] = f4{0.f, 0.f, 0.f, 0.f};
      float avs[RC / 4], bvs[RC / 4][4];
#pragma unroll
      for (int kk = 0; kk < RC / 4; ++kk) {
        const int s = g * (RC / 4) + kk;  // lane group g: rows [g RC/4, +RC/4)
        avs[kk] = S.Z2[s][w * 16 + li];
#pragma unroll
        for (int t = 0; t < 4; ++t) bvs[kk][t] = S.H1[s][t * 16 + li];
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int kk = 0; kk < RC / 4; ++kk) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
          gacc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(avs[kk], bvs[kk][t], gacc[t], 0, 0, 0);
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) S.Gb[WL_W2 + (w * 16 + g * 4 + r) * LD + t * 16 + li] = gacc[t][r];
      // the other tensors: sum of the tiles' partials in tile order (one tile: already in S.Gb)
      if constexpr (NTILE > 1) {
      auto tsum = [&](int p, int j) {
        float v = S.Ps[0][p][j];
#pragma unroll
        for (int q = 1; q < NTILE; ++q) v += S.Ps[q][p][j];
        return v;
      };
      for (int e = tid; e < HID * 4 + 2 * HID + OUTP * HID + OUTP; e += M8_NT) {
        float sum;
        int dst;
        if (e < HID * 4) {  // W1[j][k]
          const int j = e >> 2, k = e & 3;
          sum = tsum(OUTP + 2 + k, j);
          dst = WL_W1 + e;
        } else if (e < HID * 5) {  // b1
          const int j = e - HID * 4;
          sum = tsum(OUTP + 1, j);
          dst = WL_B1 + j;
        } else if (e < HID * 6) {  // b2
          const int j = e - HID * 5;
          sum = tsum(OUTP, j);
          dst = WL_B2 + j;
        } else if (e < HID * 6 + OUTP * HID) {  // W3[o][k]
          const int o = (e - HID * 6) >> 6, k = (e - HID * 6) & 63;
          sum = tsum(o, k);
          dst = WL_W3 + o * LD + k;
        } else {  // b3
          const int o = e - HID * 6 - OUTP * HID;
          float v = S.db3p[0][o];
#pragma unroll
          for (int q = 1; q < NTILE; ++q) v += S.db3p[q][o];
          sum = v;
          dst = WL_B3 + o;
        }
        S.Gb[dst] = sum;
      }
      }
    }
    STAMP(19);  // work done; the barrier wait follows
    lds_barrier();
    STAMP(5);
    // ============ round 1: publish the partial (sc1), arrive; sum share c over the G slots ============
    {
      RELANE();
      const int sbase = ((net * 2 + par) * G + c) * WL_N * (int)sizeof(float);
      f4 pv[MC_CPT];
#pragma unroll
      for (int i = 0; i < MC_CPT; ++i) pv[i] = *reinterpret_cast<const f4*>(&S.Gb[4 * min(tid + M8_NT * i, WL_CH - 1)]);
      if (__builtin_amdgcn_readfirstlane(S.xl)) {  // one XCC: plain stores, the lines stay in its L2
#pragma unroll
        for (int i = 0; i < MC_CPT; ++i) {
          const int ch = tid + M8_NT * i;
          if (ch < WL_CH) __builtin_amdgcn_raw_buffer_store_b128(as_u4(pv[i]), srs, sbase + 16 * ch, 0, 0);
        }
      } else {
#pragma unroll
        for (int i = 0; i < MC_CPT; ++i) {
          const int ch = tid + M8_NT * i;
          if (ch < WL_CH) __builtin_amdgcn_raw_buffer_store_b128(as_u4(pv[i]), srs, sbase + 16 * ch, 0, 16);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // EVERY storing wave drains its stores
    }
    STAMP(9);
    __syncthreads();
    STAMP(10);
    if (tid == 0) {
      __hip_atomic_fetch_add(&sync[M8_CNT1 + net], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (!m8_wait2(sync, M8_CNT1 + net, M8_CNT1 + net, (unsigned long long)G * (mb + 1), MC_WAIT_LOCAL)) {
        atomicExch(a.err, 1);
        S.bail = 1;
      }
#ifndef RAI_M8_NO_XCC_LOCAL
      if (mb == 0) {
        // every CU of the network registered its XCC before its step-0 arrival: from step 1 on, when they
        // all share one XCC (one L2), the gradient slots go out as plain stores (drained into that L2)
        // instead of write-through; the readers' sc1 loads bypass only their L1, so they read that L2
        const unsigned long long m =
            __hip_atomic_fetch_or(&sync[M8_XCC + net], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        S.xl = m != 0 && (m & (m - 1)) == 0;
      }
#endif
    } else if (w == 1) {
      // while wave 0 waits for the other CUs: this CU's loss statistics (fp64 sums over its rows in
      // row order of the lanes); CU 0 turns them into rows at the end.  Off the gradient's path.
      const int ln = tid & 63;
      double sv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) sv[i] = wave_sum_v(ln < RC ? (double)S.strow[ln < RC ? ln : 0][i] : 0.0);
      if (ln == 0) {
        const u4v p0 = __builtin_bit_cast(u4v, (double __attribute__((ext_vector_type(2)))){sv[0], sv[1]});
        const u4v p1 = __builtin_bit_cast(u4v, (double __attribute__((ext_vector_type(2)))){sv[2], sv[3]});
        const int so = ((net * nmb + mb) * G + c) * 32;
        __builtin_amdgcn_raw_buffer_store_b128(p0, str, so, 0, 16);
        __builtin_amdgcn_raw_buffer_store_b128(p1, str, so + 16, 0, 16);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if (w == 3 && mb + 1 < nmb) {
      pf_issue(mb + 1);  // the next step's rows: loads in flight through round 2
    }
    __syncthreads();
    if (S.bail) break;
    STAMP(6);
    // this step's Adam bias corrections: the launch's table (an LDS read), or formed here past its end
    float inv_bc2_sqrt, neg_step;
    if (mb < M8_BC_MAX) {
      inv_bc2_sqrt = S.bc[mb][0];
      neg_step = S.bc[mb][1];
    } else {
      bias_corr(mb, inv_bc2_sqrt, neg_step);
    }
    const float w1 = w1c, w2 = w2c;
    {
      RELANE();
      const int ch = c * SH + tid;
      const bool own = tid < SH && ch < WL_CH;
      const int chl = min(ch, WL_CH - 1);
      const int pbase = (net * 2 + par) * G * WL_N * (int)sizeof(float);
      f4 v[G];
#ifdef RAI_M8_ALL_LOAD  // A/B builds only: every lane loads (clamped), as before round 4
      const bool ld = true;
#else
      // only the share's owner lanes load (tid < SH: 75 of 256 at G = 16): the other lanes' clamped loads
      // were a second copy of the request stream through the CU's address unit, results unused
      const bool ld = tid < SH;
#endif
      if (ld) {
#pragma unroll
        for (int cc = 0; cc < G; ++cc)
          v[cc] = as_f4(__builtin_amdgcn_raw_buffer_load_b128(srs, pbase + (cc * WL_N + 4 * chl) * (int)sizeof(float),
                                                              0, 16));
      } else {
#pragma unroll
        for (int cc = 0; cc < G; ++cc) v[cc] = f4{0.f, 0.f, 0.f, 0.f};
      }
      f4 s = v[0];
#pragma unroll
      for (int cc = 1; cc < G; ++cc) s += v[cc];
      if (a.xworld > 1) {
        // ---- cross-GPU: push share c to every rank's region (system-scope 16-B stores), drain,
        // one flag per receiver; wait for every rank's share c in this rank's region and sum them
        // in rank order (identical bits on every rank) ---------------------------------------
        const int W = a.xworld;
        const unsigned long long step_id = (unsigned long long)(a.xbase + mb + 1);
        const int xpar = (int)((a.xbase + mb) & 1);  // global-step parity: mb restarts at 0 every launch
        const int slot_off = XDP_FLAGS_BYTES + ((xpar * W + a.xrank) * 2 + net) * WL_N * (int)sizeof(float);
        for (int pr = 0; pr < W; ++pr) {
          const __amdgpu_buffer_rsrc_t prs = mc_rsrc(a.xpeers[pr], (int)xdp_region_bytes(W));
          if (own) __builtin_amdgcn_raw_buffer_store_b128(as_u4(s), prs, slot_off + 16 * ch, 0, XDP_AUX);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid < W) {
          unsigned long long* fl = reinterpret_cast<unsigned long long*>(a.xpeers[tid]) +
                                   (net * XDP_MAXW + a.xrank) * G + c;
          __hip_atomic_store(fl, step_id, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        if (w == 0) {
          const unsigned long long* fl = reinterpret_cast<const unsigned long long*>(a.xpeers[a.xrank]) +
                                         (net * XDP_MAXW + lane) * G + c;
          const unsigned long long t0 = rai_clock();
          for (;;) {
            bool ok = true;
            if (lane < W) ok = __hip_atomic_load(fl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= step_id;
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
        f4 sum = f4{0.f, 0.f, 0.f, 0.f};
        for (int pr = 0; pr < W; ++pr) {
          const int off = XDP_FLAGS_BYTES + ((xpar * W + pr) * 2 + net) * WL_N * (int)sizeof(float);
          sum += as_f4(__builtin_amdgcn_raw_buffer_load_b128(lrs, off + 16 * chl, 0, XDP_AUX));
        }
        s = sum;
      }
      STAMP(11);
      // ---- round 2: publish the summed share and its squared norm ----
      const int s2 = (int)M8_S2_OFF + ((net * 2 + par) * WL_N + 4 * chl) * (int)sizeof(float);
      if (__builtin_amdgcn_readfirstlane(S.xl)) {
        if (own) __builtin_amdgcn_raw_buffer_store_b128(as_u4(s), srs, s2, 0, 0);
      } else {
        if (own) __builtin_amdgcn_raw_buffer_store_b128(as_u4(s), srs, s2, 0, 16);
      }
      double ss = 0.0;
      if (own) {
#pragma unroll
        for (int q = 0; q < 4; ++q) ss = __builtin_fma((double)s[q], (double)s[q], ss);
      }
      ss = wave_sum_v(ss);
      if (lane == 0) S.sq[w] = ss;  // the CU's share norm: its four wave parts, summed below in wave order
      // the waves that stored share chunks drain them (the others -- wave 3 with the next step's row loads in
      // flight -- have nothing to drain)
      if (64 * w < SH) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    STAMP(12);
    __syncthreads();
    STAMP(13);
    if (tid == 0) {
      // the share norm goes out as two tagged 8-B granules (hi / lo words of the double; agent-scope
      // atomic stores, the data is the flag: no drain), read by every CU of both networks after the
      // round-2 wait; the tag is the global optimizer step (unique across launches)
      const double cu = ((S.sq[0] + S.sq[1]) + S.sq[2]) + S.sq[3];
      const unsigned long long u = __double_as_longlong(cu), tg = (unsigned long long)(unsigned)(step0 + mb + 1) << 32;
      unsigned long long* gq = sq_gran + ((par * 2 + net) * G + c) * 2;
      __hip_atomic_store(gq, tg | (u >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(gq + 1, tg | (u & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(&sync[M8_CNT2 + net], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (!m8_wait2(sync, M8_CNT2, M8_CNT2 + 1, (unsigned long long)G * (mb + 1), MC_WAIT_LOCAL)) {
        atomicExch(a.err, 1);
        S.bail = 1;
      }
    } else if (w == 3 && mb + 1 < nmb) {
      pf_store();  // the next step's rows -> LDS (this step's px / p* reads all preceded round 1)
    }
    __syncthreads();
    if (S.bail) break;
    STAMP(7);
    // ============ all-gather: the summed gradient, the global norm, clip + Adam ============
    {
      RELANE();
      f4 gr[MC_CPT];
      const int gbase = (int)M8_S2_OFF + (net * 2 + par) * WL_N * (int)sizeof(float);
#pragma unroll
      for (int i = 0; i < MC_CPT; ++i) {
        const int chl = min(tid + M8_NT * i, WL_CH - 1);
        gr[i] = as_f4(__builtin_amdgcn_raw_buffer_load_b128(srs, gbase + 16 * chl, 0, 16));
      }
      // the 2G share norms (net-major, CU order), lane l polling the granules of number l until both
      // carry this step's tag (they were stored before their CU's round-2 arrival); fixed-order wave sum
      static_assert(M8_NW == 4, "four wave parts per share norm");
      const unsigned long long* gq = sq_gran + (par * 2 * G + min(lane, 2 * G - 1)) * 2;
      const unsigned tag = (unsigned)(step0 + mb + 1);
      unsigned long long qh, ql;
      {
        const unsigned long long t0 = rai_clock();
        for (;;) {
          qh = __hip_atomic_load(gq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ql = __hip_atomic_load(gq + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (__all((unsigned)(qh >> 32) == tag && (unsigned)(ql >> 32) == tag)) break;
          if (rai_expired(t0, MC_WAIT_LOCAL)) {
            if (lane == 0) {
              atomicExch(a.err, 1);
              S.bail = 1;
            }
            break;
          }
        }
      }
      const double sq = __longlong_as_double((long long)((qh << 32) | (ql & 0xffffffffull)));
      const double tot = wave_sum_v(lane < 2 * G ? sq : 0.0);
      const float total_norm = (float)sqrt(tot);
      STAMP(14);
      float coef = 1.f;
      if (max_grad_norm > 0.f) coef = fminf(max_grad_norm / (total_norm + 1e-6f), 1.f);
      // branch-free over the chunks (one basic block: the transcendentals of all chunks interleave); a lane
      // past the last chunk updates a clamped copy and stores nothing (its moments are never written back)
#pragma unroll
      for (int i = 0; i < MC_CPT; ++i) {
        const int ch = tid + M8_NT * i;
        {
          f4 p = *reinterpret_cast<const f4*>(&S.Wt[4 * min(ch, WL_CH - 1)]);
#ifdef RAI_M8_SCALAR_ADAM  // A/B builds only: one element per VALU op
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            float pq = p[q], mq = mreg[i][q], vq = vreg[i][q];
            adam_update_fast(pq, mq, vq, gr[i][q] * coef, w1, w2, beta2, inv_bc2_sqrt, neg_step, adam_eps);
            p[q] = pq;
            mreg[i][q] = mq;
            vreg[i][q] = vq;
          }
#else
          const f2a C2 = {coef, coef};
#pragma unroll
          for (int h = 0; h < 2; ++h) {  // element pairs (0, 1), (2, 3)
            f2a pp = {p[2 * h], p[2 * h + 1]}, mm = {mreg[i][2 * h], mreg[i][2 * h + 1]},
                vv = {vreg[i][2 * h], vreg[i][2 * h + 1]};
            const f2a gg = f2a{gr[i][2 * h], gr[i][2 * h + 1]} * C2;
            adam_update_fast2(pp, mm, vv, gg, w1, w2, beta2, inv_bc2_sqrt, neg_step, adam_eps);
            p[2 * h] = pp.x;
            p[2 * h + 1] = pp.y;
            mreg[i][2 * h] = mm.x;
            mreg[i][2 * h + 1] = mm.y;
            vreg[i][2 * h] = vv.x;
            vreg[i][2 * h + 1] = vv.y;
          }
#endif
          if (ch < WL_CH) *reinterpret_cast<f4*>(&S.Wt[4 * ch]) = p;
        }
      }
      if (ACTOR && c == 0 && tid == 0 && a.norms && norm0 + mb < a.max_norms) a.norms[norm0 + mb] = total_norm;
    }
    lds_barrier();
    STAMP(8);
  }

  // ---- stats rows of every minibatch (CU 0): sum the CUs' partials in CU order ---------------------
  if (c == 0 && !S.bail && a.stats) {
    for (int k = tid; k < nmb; k += M8_NT) {
      const int srow = stat0 + k;
      if (srow >= a.max_stats) continue;
      const int64_t r0 = (int64_t)k * B;
      const int rws = (int)min((int64_t)B, n_rows - r0);
      double sv[4] = {0.0, 0.0, 0.0, 0.0};
      for (int cc = 0; cc < G; ++cc) {
        const int so = ((net * nmb + k) * G + cc) * 32;
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
        row[0] = lh.pi_coef * pi_loss + lh.ent_coef * ent_loss;  // host adds the value term
        row[1] = pi_loss;
        row[2] = ent_loss;
        row[3] = (float)(sv[1] / Bd);
        row[4] = (float)(sv[2] / Bd);
      } else {
        row[5] = (float)(sv[0] / Bd) * lh.halve;
        row[5 + RAI_MAX_K] = lh.has_vclip ? (float)(sv[1] / Bd) : 0.f;
      }
    }
  }
  // ---- write back parameters and optimizer moments (identical copies: each CU writes 1/G) ------
  if (!S.bail) {
#pragma unroll
    for (int i = 0; i < MC_CPT; ++i) {
      const int ch = tid + M8_NT * i;
      if (ch < WL_CH && ch % G == c) {
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
#ifdef RAI_STAMPS
  if (c == 0 && tid == 0) S.stamps[31] = (unsigned long long)S.xl;  // launches with the one-XCC store form
  __syncthreads();
  if (c == 0 && tid < 32) atomicAdd(&g_stamps[net][tid], S.stamps[tid]);  // summed over launches
#endif
  if (ACTOR && c == 0 && tid == 0) {
    a.state->stat_index = stat0 + nmb;
    a.state->opt_step = step0 + nmb;
    a.state->norm_index = norm0 + nmb;
  }
}

template <int RELU, int G, int RCV = MAXB / G>
__global__ __launch_bounds__(M8_NT) void mlp_ppo_mc8_kernel(const MlpArgs a) {
  static_assert(sizeof(SmemM8<2, G, RCV>) <= 160 * 1024, "LDS budget");
  __shared__ __attribute__((aligned(16))) unsigned char smem_raw[sizeof(SmemM8<2, G, RCV>)];
  const int b = blockIdx.x, xcd = b & 7, c = b >> 3;
  if (xcd >= 2) return;  // only two XCDs' worth of blocks work (locality, not correctness)
  if (xcd == 0) mlp_mc8<2, true, RELU, G, RCV>(a, *reinterpret_cast<SmemM8<2, G, RCV>*>(smem_raw), c);
  else mlp_mc8<1, false, RELU, G, RCV>(a, *reinterpret_cast<SmemM8<1, G, RCV>*>(smem_raw), c);
}
