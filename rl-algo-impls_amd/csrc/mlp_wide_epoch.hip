// Persistent PPO epoch for wide MLP actor-critics on gfx950 (HalfCheetah class: separate
// [in -> H -> H -> out] actor and critic, H <= 256 in 16-unit slices, Gaussian or Categorical
// head).  ONE launch runs every minibatch step of an epoch of rl_algo_impls/ppo/ppo.py:290-411:
// forward, head log-prob / entropy, the clipped-surrogate / value / entropy loss, the backward,
// clip_grad_norm_ and Adam(eps) -- where the per-minibatch path (mlp_wide.hip + rai_ppo_loss +
// rai_clip_optim_step) is a chain of 8 dependent launches per optimizer step.
//
// Layout: each network runs on G = H / 16 workgroups (one per CU; the grid is launched 8 G wide
// and only blocks b % 8 == 0 (actor) / == 1 (critic) work, so each network's workgroups share one
// XCD's L2 -- placement is a speed choice only, the hand-offs below are placement-independent).
// Workgroup j OWNS hidden units [16 j, 16 j + 16) of both hidden layers and keeps in LDS, updated
// by its own Adam every step: W1 rows j, b1 j, W2 rows j, b2 j, W3 columns j, and copies of b3 /
// log_std.  Its Adam moments live in registers.  W2 is held once, by its row owner.
//
// Before the epoch, we_pack_kernel builds one record per row (minibatch-normalized advantage, loss
// inputs, zero-padded observation), so each step's inputs are one contiguous prefetched block.
//
// One optimizer step = four hand-offs:
//   A  H1[:, j] published (16-B write-through (sc1) stores, every storing wave drained, one
//      agent-scope arrival per workgroup on a monotonic counter -- MI355X_MICROARCH.md "Valid forms",
//      row 1); every workgroup gathers H1 (B x H) by LDS-DMA sc1 loads
//   B  output-layer partials H2[:, j] W3[:, j]^T published (as A); every workgroup sums them in slice
//      order and runs the head + loss for all rows (identical everywhere), then dZ2[:, j]
//   C  dZ2[:, j] published (as A); every workgroup gathers dZ2 and forms dH1[:, j] = dZ2 W2[:, j]
//      from W2's column slice, which the row owners publish each step after their H1 gather (drained
//      before their B arrival) and the column owners load by LDS-DMA after the B wait
//   D  (both networks) each workgroup's share of the squared gradient norm as two tagged 8-B
//      granules (agent-scope atomic store / load, no drain or counter); every workgroup sums the 2 G
//      shares in a fixed order (clip_grad_norm_ over all parameters, bit-identical on every
//      workgroup) and applies clip + Adam to what it owns.
// Data parallel (rai_mlp_wide_epoch_xdp, world W > 1): after the backward, each workgroup pushes the
// gradient it owns (its W2 rows, W1 rows and small parameters, 21 KB) to slot [rank] of every rank's
// IPC-mapped region (16-B system-scope stores, drained, one step-id flag per receiver), waits for all W
// ranks' flags of its slice and sums the W slots in rank order, so every rank holds the bit-identical
// global gradient before D; the loss means are over rows x W and the advantage moments are the global
// minibatch's (computed by the caller).  Every spin is bounded and sets state->err.  Numerics: fp32 like the reference, exact-f32 MFMA
// (v_mfma_f32_16x16x4f32), Adam with the hardware sqrt / rcp (as the CartPole epoch kernel); parity
// to fp32 tolerance against the per-minibatch path and the reference (tests/test_gpu_trainer.py).
#include "common.h"

// RAI_WE_NO_DEFER (A/B builds only): the W2 Adam at the end of its own step instead of in the next
// step's A wait
#ifdef RAI_WE_NO_DEFER
constexpr bool WE_DEFER_W2 = false;
#else
constexpr bool WE_DEFER_W2 = true;
#endif

namespace {

constexpr int WE_NT = 256;                  // threads per workgroup (4 waves)
constexpr int WE_SL = 16;                   // hidden units per workgroup
constexpr int WE_B = 64;                    // max minibatch rows (4 row tiles of 16)
constexpr int WE_HMAX = RAI_WIDE_MAX_H;     // 256
constexpr int WE_GMAX = WE_HMAX / WE_SL;    // 16
constexpr int WE_HP = WE_HMAX + 4;          // LDS row stride of H-long rows (16-B aligned)
constexpr int WE_INMAX = RAI_WIDE_MAX_IN;   // 64
constexpr int WE_XLD = WE_INMAX + 4;        // LDS row stride of obs rows
constexpr int WE_OUTM = RAI_WIDE_MAX_OUT;   // 8
constexpr int WE_SP = WE_SL + 4;            // stride of [rows][16] slices: 16-B rows, 4 rows = 16 banks
constexpr int WE_NSMALL = 2 * WE_SL + WE_OUTM * WE_SL + 2 * WE_OUTM;  // b1 j, b2 j, W3 cols j, b3, log_std
constexpr int WE_SC1 = 16;                  // buffer cache policy: sc1
constexpr int WE_XDP_AUX = 17;              // sc0 | sc1: system-scope (cross-device) stores and loads
static_assert(4096 + 1024 + WE_NSMALL <= RAI_XDP_WIDE_SLOTF && WE_NSMALL % 4 == 0, "xdp slot");
static_assert(2 * 8 * WE_GMAX * 8 <= 2048, "xdp flags");

typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned int u4v __attribute__((ext_vector_type(4)));
typedef unsigned int u2v __attribute__((ext_vector_type(2)));

// workspace layout (bytes)
constexpr int64_t WE_CTR_STRIDE = 128;                                  // one counter per 128-B line
constexpr int64_t WE_CTR_BYTES = 8 * WE_CTR_STRIDE;                     // A0 A1 B0 B1 C0 C1 D
constexpr int64_t WE_ACT_SLOT = (int64_t)WE_B * WE_HMAX * 4;            // one [64][H] f32 slot
// the D exchange as granules (8-B {tag = step + 1, 32-bit value} words, agent-scope atomic stores and
// loads: the data is the flag -- no drain, no counter), zeroed with the counters before every launch.
// (The B exchange measured 3x slower as granules -- 24 polled words per lane -- and keeps the counter.)
constexpr int64_t WE_GD_OFF = WE_CTR_BYTES;                             // D: [par][net][slice][hi, lo]
constexpr int64_t WE_STATE_BYTES = WE_GD_OFF + 2 * 2 * WE_GMAX * 2 * 8;  // the memset block
constexpr int64_t WE_H1_OFF = WE_STATE_BYTES;                           // [net][par] H1 slots
constexpr int64_t WE_Z2_OFF = WE_H1_OFF + 4 * WE_ACT_SLOT;              // [net][par] dZ2 slots
// W2 as its row owners publish it each step (after the H1 gather: the last Adam step's rows), for
// the column owners' dH1 (loaded after the B wait): [net][producer
// p][unit tile ct] transposed 16 x 16 tiles of 1 KB, tile (p, ct)[u][kk] = W2[16 p + kk][16 ct + u]
constexpr int64_t WE_W2T_NET = (int64_t)WE_GMAX * WE_GMAX * 1024;
constexpr int64_t WE_W2T_OFF = WE_Z2_OFF + 4 * WE_ACT_SLOT;
constexpr int64_t WE_P_SLOT = (int64_t)WE_GMAX * WE_B * WE_OUTM * 4;    // [slice][64][8] f32
constexpr int64_t WE_P_OFF = WE_W2T_OFF + 2 * WE_W2T_NET;              // [net][par] output-layer partial slots
// per-row records of the epoch, built by we_pack_kernel before the epoch: [0] normalized advantage,
// [1] old log-prob, [2] return, [3] old value, [4, 12) action (Gaussian: O floats; Categorical: the
// index's int32 bits), [12, 12 + IN4) observation (zero-padded): one contiguous 16-B-aligned block per
// minibatch, staged by WE_RU 16-B loads per thread
constexpr int WE_LIN = 12;
constexpr int64_t WE_REC_OFF = WE_P_OFF + 4 * WE_P_SLOT;
inline int we_rec_floats(int in_dim) { return WE_LIN + ((in_dim + 3) & ~3); }
inline int64_t we_ws_bytes(int in_dim, int64_t n_rows) {
  return WE_REC_OFF + ((n_rows * we_rec_floats(in_dim) * 4 + 255) & ~(int64_t)255);
}
constexpr int WE_RU = (WE_B * (WE_LIN + WE_INMAX) / 4 + 255) / 256;  // 16-B record loads per thread
enum { WE_CA = 0, WE_CB = 2, WE_CC = 4, WE_CXCC = 6 };  // counters (A: H1, B: head partials, C: dH1 tiles;
                                                      // line 6: per network the set of XCCs); D: granules
static_assert(WE_STATE_BYTES % 16 == 0, "memset block");

typedef __attribute__((address_space(1))) unsigned long long we_gu64;
__device__ __forceinline__ we_gu64* we_gptr(unsigned char* p) { return (we_gu64*)p; }  // global, never flat
__device__ __forceinline__ void we_put(we_gu64* g, unsigned tag, unsigned value) {
  __hip_atomic_store(g, ((unsigned long long)tag << 32) | value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long we_get(we_gu64* g) {
  return __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct WeArgs {
  rai_mlp_wide_desc d;
  float* params;       // flat parameter buffer (desc.w point into it)
  float* exp_avg;      // Adam state, same layout as params
  float* exp_avg_sq;
  const float* rec;    // (n_rows, we_rec_floats(in)) per-row records (we_pack_kernel)
  int64_t n_rows;
  int32_t batch;
  const rai_ppo_hparams* hp;
  const rai_optim_hparams* ohp;
  rai_train_state* state;
  float* stats;
  int32_t max_stats;
  float* norms;
  int32_t max_norms;
  unsigned char* ws;
  // data parallel (rai_mlp_wide_epoch_xdp): world ranks, this one xrank; every workgroup's owned
  // gradient is summed over the ranks in rank order through the IPC-mapped regions xpeers[] each step
  int32_t world;         // loss means over rows x world (1: single process)
  int32_t xrank;
  void* const* xpeers;   // device array of the world regions (rank order), nullptr when world == 1
  int64_t xbase;         // optimizer steps already run through the regions (flags hold step ids)
};

struct WeSmem {
  float Act[WE_B][WE_HP];     // H1 of the minibatch (all columns), later dZ2
  float W2r[WE_SL][WE_HP];    // W2[16 j + i][:]
  alignas(16) float W2cT[WE_GMAX][WE_SL][WE_SL];  // W2[:, 16 j ..] as [k / 16][u][k % 16] (this step's)
  // minibatch observations, row stride IN4 (zero-padded), then the loss inputs [64][12] (record words 0-11)
  alignas(16) float Xl[WE_B * WE_INMAX + WE_B * WE_LIN];
  float W1j[WE_SL][WE_XLD];   // W1[16 j + i][:]
  float H1j[WE_B][WE_SP];
  float H2j[WE_B][WE_SP];
  float Z2j[WE_B][WE_SP];
  float Z1j[WE_B][WE_SP];
  alignas(16) float dOut[WE_B][WE_OUTM];
  float dls[WE_B][WE_OUTM];
  float Pw[4][WE_B][WE_OUTM];  // per-wave sums of 4 slices' output partials
  alignas(16) float small[WE_NSMALL];  // b1 j | b2 j | W3[:, j] (o-major) | b3 | log_std
  alignas(16) float gsm[WE_NSMALL];  // small-parameter gradients (MFMA column sums), by small index
  double st[4][WE_B];         // per-row loss statistics, reduced off the critical path (D wait)
  float ginv[WE_OUTM], glsc[WE_OUTM], entc;  // Gaussian 1 / variance, log scale, per-row entropy
  float adamc[2];             // this step's Adam bias-correction constants (formed during the D wait)
  float coef;                 // this step's clip coefficient
  alignas(16) float db1[WE_SL];      // db1 j (wave 3)
  double red[4][8];
  float adv_mean, adv_den;
  int bail;
  int xl;  // every workgroup of this network on one XCC: hand-off slots published with plain stores
};

#ifdef RAI_STAMPS
// diagnostic build only (lib/librai_amd_stamps.so, tools/wide_stamps.py): per-phase shader-clock ticks
// of workgroup 0 of each network, accumulated over launches
__device__ unsigned long long g_we_stamps[2][24];
#define WSTAMP(i)                                                             \
  do {                                                                        \
    if (j == 0 && threadIdx.x == 0) {                                         \
      const unsigned long long t_ = __builtin_amdgcn_s_memtime();            \
      st_acc[i] += t_ - t_last;                                               \
      t_last = t_;                                                            \
    }                                                                         \
  } while (0)
#else
#define WSTAMP(i) \
  do {            \
  } while (0)
#endif

__device__ __forceinline__ __amdgpu_buffer_rsrc_t we_rsrc(const void* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float we_act(int act, float z) { return act ? fmaxf(z, 0.f) : tanhf(z); }
__device__ __forceinline__ float we_actd(int act, float h) { return act ? (h > 0.f ? 1.f : 0.f) : (1.f - h * h); }

__device__ __forceinline__ float we_vf_loss(int fn, float x) {
#pragma clang fp contract(off)
  if (fn == 0) return x * x;
  const float z = fabsf(x);
  return z < 1.f ? 0.5f * z * z : (z - 0.5f);
}
__device__ __forceinline__ float we_vf_grad(int fn, float x) {
#pragma clang fp contract(off)
  if (fn == 0) return 2.f * x;
  return x <= -1.f ? -1.f : (x >= 1.f ? 1.f : x);
}

// 16 x 16 tile of  Rows[16 tiles rows][k] . Cols[16][k]^T  over k in [0, H) (LDS, ld WE_HP): lane
// group g takes the contiguous quarter [g H/4, (g+1) H/4), four accumulator chains (one per f4
// component).  For the common widths (KQ = H / 4 a compile-time constant) the loop is unrolled and
// the next 16-B operands are read while the current four MFMAs issue.
template <int KQ>
__device__ __forceinline__ f4 we_tile_dot_k(const float* ra, const float* cb) {
  f4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
  f4 av = *reinterpret_cast<const f4*>(ra), bv = *reinterpret_cast<const f4*>(cb);
  __builtin_amdgcn_sched_barrier(0);  // the prologue reads stay outside the loop's schedule groups
#pragma unroll
  for (int kk = 0; kk < KQ; kk += 4) {
    f4 an = av, bn = bv;
    if (kk + 4 < KQ) {
      an = *reinterpret_cast<const f4*>(ra + kk + 4);
      bn = *reinterpret_cast<const f4*>(cb + kk + 4);
    }
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, bv.x, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, bv.y, acc1, 0, 0, 0);
    acc2 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.z, bv.z, acc2, 0, 0, 0);
    acc3 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.w, bv.w, acc3, 0, 0, 0);
    if (kk + 4 < KQ) {
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // DS reads of the next step
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);  // this step's MFMAs
    }
    av = an;
    bv = bn;
  }
  return (acc0 + acc1) + (acc2 + acc3);
}
__device__ __forceinline__ f4 we_tile_dot(const float* rows, const float* cols, int H, int lane) {
  const int li = lane & 15, g = lane >> 4, KQ = H >> 2;
  const float* ra = rows + li * WE_HP + g * KQ;
  const float* cb = cols + li * WE_HP + g * KQ;
  if (H == 256) return we_tile_dot_k<64>(ra, cb);
  if (H == 128) return we_tile_dot_k<32>(ra, cb);
  if (H == 64) return we_tile_dot_k<16>(ra, cb);
  f4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
  for (int kk = 0; kk < KQ; kk += 4) {
    const f4 av = *reinterpret_cast<const f4*>(ra + kk);
    const f4 bv = *reinterpret_cast<const f4*>(cb + kk);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, bv.x, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, bv.y, acc1, 0, 0, 0);
    acc2 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.z, bv.z, acc2, 0, 0, 0);
    acc3 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.w, bv.w, acc3, 0, 0, 0);
  }
  return (acc0 + acc1) + (acc2 + acc3);
}

// Minibatch row fed by lane group g to the kk-th MFMA of a row-reduction: rows come in blocks of 8,
// two MFMAs per block, lane groups g = 0..3 taking offsets 0, 4, 2, 6 (+1 in the odd MFMA).  The two
// lane groups of one ds_read_b32 half-wave (g, g + 1) then read rows 4 apart: with a row stride of
// 4 (mod 32) dwords (WE_HP, WE_XLD, WE_SP) they sit 16 banks apart -- no bank conflicts.
__device__ __forceinline__ int we_krow(int kk, int g) {
  return 8 * (kk >> 1) + (kk & 1) + ((g & 1) << 2) + ((g >> 1) << 1);
}

// Four dW2 tiles t = 0..3: D_t[i][jj] = sum over the 64 minibatch rows k of A[k][t as + i] *
// Bm[k][t bs + jj], k = we_krow(kk, g), one accumulator chain per tile, the four chains interleaved
// (each kk step reads the shared operand once).  The row owner calls it with A = its dZ2 slice (as = 0),
// Bm = H1 columns 16 (4 w + t) (bs = 16); the column owner with A = dZ2 columns 16 (4 w + t)
// (as = 16), Bm = its H1 slice (bs = 0): the same products in the same order, so both copies of a W2
// element receive the same gradient bits.  Tiles past H read in-bounds stale LDS; callers mask them.
template <int as, int bs>
__device__ __forceinline__ void we_dw2_tiles4(const float* A, int lda, const float* Bm, int ldb, int lane, f4 out[4]) {
  const int li = lane & 15, g = lane >> 4;
  const float* a0 = A + we_krow(0, g) * lda + li;
  const float* b0 = Bm + we_krow(0, g) * ldb + li;
  f4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f4{0.f, 0.f, 0.f, 0.f};
  // operands one kk step ahead: step kk + 1's reads issue before step kk's MFMAs
  float av[4], bv[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    av[t] = a0[t * as];
    bv[t] = b0[t * bs];
  }
#pragma unroll
  for (int kk = 0; kk < WE_B / 4; ++kk) {
    const int dk = 8 * ((kk + 1) >> 1) + ((kk + 1) & 1);  // we_krow(kk + 1, g) - we_krow(0, g)
    float an[4], bn[4];
    if (kk + 1 < WE_B / 4) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        an[t] = a0[dk * lda + t * as];
        bn[t] = b0[dk * ldb + t * bs];
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[t], bv[t], acc[t], 0, 0, 0);
    if (kk + 1 < WE_B / 4) {
      __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);  // DS reads of step kk + 1
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);  // MFMAs of step kk
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        av[t] = an[t];
        bv[t] = bn[t];
      }
    }
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) out[t] = acc[t];
}

// One 16 x 16 MFMA tile over the 64 minibatch rows, D[i][jj] = sum_k A[k][i] B[k][jj], for the
// small-parameter gradients: lane (li, g) feeds A = a0[k LDA] and B = b0[k WE_SP] (ONES: B = 1) at
// rows k = we_krow(kk, g); every operand is read first, then two MFMA chains.  Rows i of D that come
// from padding lanes are never stored, so no operand needs masking.
template <int LDA, bool ONES>
__device__ __forceinline__ f4 we_small_tile(const float* a0, const float* b0, int g) {
  const int k0 = we_krow(0, g);
  a0 += k0 * LDA;
  b0 += k0 * WE_SP;
  float av[WE_B / 4], bv[WE_B / 4];
#pragma unroll
  for (int kk = 0; kk < WE_B / 4; ++kk) {
    const int dk = 8 * (kk >> 1) + (kk & 1);
    av[kk] = a0[dk * LDA];
    bv[kk] = ONES ? 1.f : b0[dk * WE_SP];
  }
  __builtin_amdgcn_sched_barrier(0);
  f4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
#pragma unroll
  for (int kk = 0; kk < WE_B / 4; ++kk) {
    if (kk & 1) acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[kk], bv[kk], acc1, 0, 0, 0);
    else acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[kk], bv[kk], acc0, 0, 0, 0);
  }
  return acc0 + acc1;
}

// sum over the 64 minibatch rows of f(r), as four interleaved partial sums (rows r = q mod 4) added
// in a fixed order: four independent dependency chains instead of one, identical on every workgroup
template <typename F>
__device__ __forceinline__ float we_rowsum(F f) {
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int r = 0; r < WE_B; r += 4) {
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] += f(r + q);
  }
  return ((acc[0] + acc[1]) + acc[2]) + acc[3];
}

// Adam with the hardware square root and reciprocal (as the CartPole epoch kernel's
// adam_update_fast): a few ulps from torch's IEEE sequence, far inside the fp32 tolerances
__device__ __forceinline__ void adam_fast(float& p, float& m, float& v, float g, float c1, float c2, float beta2,
                                          float inv_c3, float c4, float eps) {
  m = m + c1 * (g - m);
  v = v * beta2;
  v = v + (c2 * g) * g;
  const float denom = __builtin_amdgcn_sqrtf(v) * inv_c3 + eps;
  p = p + c4 * (m * __builtin_amdgcn_rcpf(denom));
}

typedef float f2a __attribute__((ext_vector_type(2)));
// adam_fast on an element pair (packed f32 VALU; the same operations per element)
__device__ __forceinline__ void adam_fast2(f2a& p, f2a& m, f2a& v, f2a g, float c1, float c2, float beta2, float inv_c3,
                                           float c4, float eps) {
  const f2a C1 = {c1, c1}, Cb = {c2, c2}, B2 = {beta2, beta2}, IC = {inv_c3, inv_c3}, EP = {eps, eps}, C4 = {c4, c4};
  m = m + C1 * (g - m);
  v = v * B2;
  v = v + (Cb * g) * g;
  const f2a sq = {__builtin_amdgcn_sqrtf(v.x), __builtin_amdgcn_sqrtf(v.y)};
  const f2a denom = sq * IC + EP;
  const f2a rc = {__builtin_amdgcn_rcpf(denom.x), __builtin_amdgcn_rcpf(denom.y)};
  p = p + C4 * (m * rc);
}

// arrive on counter `ci` after every wave's stores drained (caller: s_waitcnt vmcnt(0) in every
// storing wave, then this); lane 0 polls until ctr[ci] >= want.
// dH1 tile of wave w: D[i][u] = sum_k dZ2[16 w + i][k] W2[k][16 j + u] over k in [0, H): lane group g
// takes k in [g KQ, (g + 1) KQ), four at a time: A from the Act row (16-B reads), B from W2cT[k / 16][u]
// (16-B reads); four accumulator chains, unrolled and read one step ahead for the common widths
// W2cT rows are stored swizzled (we_w2t_src): unit u's 16-B piece kk4 sits at slot kk4 ^ ((u >> 2) & 3),
// so the 16 units' reads of one piece spread over all 16 bank groups (a plain [u][16] row stride of
// 64 B put four units on every bank group)
__device__ __forceinline__ int we_w2t_slot(int u, int kk4) { return kk4 ^ ((u >> 2) & 3); }
template <int KQ>
__device__ __forceinline__ f4 we_dh1_tile_k(const float* ra, const float* wt, int k0, int u) {
  f4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
  // k0 is a multiple of 16 here (KQ >= 16): the four swizzled piece bases once, then every read is
  // one of them plus a compile-time offset (no per-step address arithmetic between the reads)
  const float* bp[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) bp[c] = wt + (k0 >> 4) * (WE_SL * WE_SL) + 4 * we_w2t_slot(u, c);
  auto bptr = [&](int kk) { return bp[(kk >> 2) & 3] + (kk >> 4) * (WE_SL * WE_SL); };
  f4 av = *reinterpret_cast<const f4*>(ra), bv = *reinterpret_cast<const f4*>(bptr(0));
  __builtin_amdgcn_sched_barrier(0);  // the prologue reads stay outside the loop's schedule groups
#pragma unroll
  for (int kk = 0; kk < KQ; kk += 4) {
    f4 an = av, bn = bv;
    if (kk + 4 < KQ) {
      an = *reinterpret_cast<const f4*>(ra + kk + 4);
      bn = *reinterpret_cast<const f4*>(bptr(kk + 4));
    }
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, bv.x, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, bv.y, acc1, 0, 0, 0);
    acc2 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.z, bv.z, acc2, 0, 0, 0);
    acc3 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.w, bv.w, acc3, 0, 0, 0);
    if (kk + 4 < KQ) {
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
    }
    av = an;
    bv = bn;
  }
  return (acc0 + acc1) + (acc2 + acc3);
}
__device__ __forceinline__ f4 we_dh1_tile(const float* act_row, const float* w2t_u, int H, int g, int u) {
  const int KQ = H >> 2, k0 = g * KQ;
  const float* ra = act_row + k0;
  if (H == 256) return we_dh1_tile_k<64>(ra, w2t_u, k0, u);
  if (H == 128) return we_dh1_tile_k<32>(ra, w2t_u, k0, u);
  if (H == 64) return we_dh1_tile_k<16>(ra, w2t_u, k0, u);
  f4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
  for (int kk = 0; kk < KQ; kk += 4) {
    const int k = k0 + kk;
    const f4 av = *reinterpret_cast<const f4*>(ra + kk);
    const f4 bv = *reinterpret_cast<const f4*>(w2t_u + (k >> 4) * (WE_SL * WE_SL) + 4 * we_w2t_slot(u, (k & 15) >> 2));
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, bv.x, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, bv.y, acc1, 0, 0, 0);
    acc2 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.z, bv.z, acc2, 0, 0, 0);
    acc3 = __builtin_amdgcn_mfma_f32_16x16x4f32(av.w, bv.w, acc3, 0, 0, 0);
  }
  return (acc0 + acc1) + (acc2 + acc3);
}

// A within-network hand-off store: write-through (sc1), or plain when every workgroup of the network runs
// on one XCC (xl: the data then stays in that XCC's L2, where the readers' sc1 loads -- past their own L1
// only -- find it; write-through drops the line and the readers fetch past the L2).  xl is wave-uniform.
__device__ __forceinline__ void we_st16(u4v v, __amdgpu_buffer_rsrc_t rs, int off, bool xl) {
  if (xl) __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 0);
  else __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, WE_SC1);
}

// Publish W2 rows j for the column owners as transposed 16 x 16 tiles (16-B sc1 stores; no drain
// here: the next H1 publish's drain covers them, before the A arrival their readers wait on).  Wave
// w writes tiles ct = w + 4 m; lane (u = lane >> 2, kk4 = lane & 3) one 16-B row piece of each.
__device__ __forceinline__ void we_publish_w2(const float (*W2r)[WE_HP], __amdgpu_buffer_rsrc_t wrs, int64_t base,
                                              int G, int w, int lane, bool xl) {
  const int u = lane >> 2, kk4 = lane & 3;
#pragma unroll
  for (int m = 0; m < WE_GMAX / 4; ++m) {
    const int ct = w + 4 * m;
    if (ct < G) {
      const f4 v = {W2r[4 * kk4][WE_SL * ct + u], W2r[4 * kk4 + 1][WE_SL * ct + u], W2r[4 * kk4 + 2][WE_SL * ct + u],
                    W2r[4 * kk4 + 3][WE_SL * ct + u]};
      we_st16(__builtin_bit_cast(u4v, v), wrs, (int)(base + (int64_t)ct * 1024 + (u * WE_SL + 4 * kk4) * 4), xl);
    }
  }
}

// fwd1 tile: sum over k = 4 kk + g < IN4 of X[row][k] W1j[unit][k]; operands read first, then the
// MFMAs in two chains (unrolled for each K-step count up to 16)
template <int NK>
__device__ __forceinline__ f4 we_fwd1_k(const float* xa, const float* wa) {
  float xv[NK], wv[NK];
#pragma unroll
  for (int kk = 0; kk < NK; ++kk) {
    xv[kk] = xa[4 * kk];
    wv[kk] = wa[4 * kk];
  }
  __builtin_amdgcn_sched_barrier(0);
  f4 z0 = {0.f, 0.f, 0.f, 0.f}, z1 = z0;
#pragma unroll
  for (int kk = 0; kk < NK; ++kk) {
    if (kk & 1) z1 = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[kk], wv[kk], z1, 0, 0, 0);
    else z0 = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[kk], wv[kk], z0, 0, 0, 0);
  }
  return z0 + z1;
}
__device__ __forceinline__ f4 we_fwd1(const float* xa, const float* wa, int nk) {
  switch (nk) {
#define WE_FWD1_CASE(n) \
  case n:               \
    return we_fwd1_k<n>(xa, wa);
    WE_FWD1_CASE(1) WE_FWD1_CASE(2) WE_FWD1_CASE(3) WE_FWD1_CASE(4) WE_FWD1_CASE(5) WE_FWD1_CASE(6)
    WE_FWD1_CASE(7) WE_FWD1_CASE(8) WE_FWD1_CASE(9) WE_FWD1_CASE(10) WE_FWD1_CASE(11) WE_FWD1_CASE(12)
    WE_FWD1_CASE(13) WE_FWD1_CASE(14) WE_FWD1_CASE(15)
#undef WE_FWD1_CASE
    default:
      return we_fwd1_k<16>(xa, wa);  // IN4 <= 64
  }
}

// Gather a published 64 x H exchange slot (workspace byte offset `base`) into Act (LDS rows of WE_HP
// floats) by LDS-DMA: one global_load_lds_dwordx4 per row (H / 4 lanes x 16 B, landing contiguously
// at the row's start), sc1 like every load of handed-off bytes; wave w takes rows w, w + 4, ...  The
// data lands without VGPRs or ds_write instructions; the caller's barrier follows the vmcnt(0) here.
__device__ __forceinline__ void we_gather_lds(const unsigned char* ws, int64_t base, int H, float (*Act)[WE_HP], int w,
                                              int lane, bool drain = true, bool own_tile = false) {
  if (lane < (H >> 2)) {
    const float* src = reinterpret_cast<const float*>(ws + base) + 4 * lane;
    if (own_tile) {  // rows [16 w, 16 w + 16): this wave's row tile
#pragma unroll
      for (int r = 16 * w; r < 16 * w + 16; ++r)
        __builtin_amdgcn_global_load_lds(src + (int64_t)r * H, &Act[r][0], 16, 0, WE_SC1);
    } else {
#pragma unroll
      for (int r = w; r < WE_B; r += 4)
        __builtin_amdgcn_global_load_lds(src + (int64_t)r * H, &Act[r][0], 16, 0, WE_SC1);
    }
  }
  if (drain) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Wave 1 runs `side` (work off the critical path: LDS in, LDS / plain global out) while lane 0 polls.
template <typename F>
__device__ __forceinline__ bool we_arrive_wait(unsigned long long* ctr, int ci, unsigned long long want,
                                               rai_train_state* state, int& bail, int w, F side) {
  __syncthreads();
  if (w == 1) side();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(&ctr[ci * (WE_CTR_STRIDE / 8)], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long t0 = rai_clock();
    while (__hip_atomic_load(&ctr[ci * (WE_CTR_STRIDE / 8)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
      if (rai_expired(t0, RAI_SPIN_LOCAL)) {
        __hip_atomic_store(&state->err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bail = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  return !bail;
}

// we_arrive_wait split in two, so the workgroup can work between its own arrival and the wait for the
// others' (the deferred W2 Adam below): every wave's stores were drained before the barrier that precedes
// the arrival (as in we_arrive_wait), and the wait's closing barrier releases the waves.
__device__ __forceinline__ void we_arrive(unsigned long long* ctr, int ci) {
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_fetch_add(&ctr[ci * (WE_CTR_STRIDE / 8)], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool we_wait(unsigned long long* ctr, int ci, unsigned long long want,
                                        rai_train_state* state, int& bail) {
  if (threadIdx.x == 0) {
    const unsigned long long t0 = rai_clock();
    while (__hip_atomic_load(&ctr[ci * (WE_CTR_STRIDE / 8)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
      if (rai_expired(t0, RAI_SPIN_LOCAL)) {
        __hip_atomic_store(&state->err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bail = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  return !bail;
}

template <int HEAD>  // 0 Categorical, 1 Gaussian
__device__ void we_epoch(const WeArgs& a, WeSmem& S, const int net, const int j) {
  const rai_mlp_wide_desc& d = a.d;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, g = lane >> 4;
  const int H = d.hidden, G = H / WE_SL, IN = d.in_dim, IN4 = (IN + 3) & ~3;
  const int O = net == 0 ? d.out_pi : 1;
  const int act = d.activation;
  const rai_ppo_hparams& hp = *a.hp;
  const rai_optim_hparams& ohp = *a.ohp;
  unsigned long long* ctr = reinterpret_cast<unsigned long long*>(a.ws);
  const __amdgpu_buffer_rsrc_t wrs = we_rsrc(a.ws, WE_REC_OFF);  // the exchange region
  const float* const* W = d.w[net];
  const int64_t pbase_off = 0;
  (void)pbase_off;
  auto foff = [&](const float* p) -> int64_t { return p - a.params; };  // offset in the flat buffer

  // ---- parameters -> LDS, Adam moments -> registers -------------------------------------------
  for (int e = tid; e < WE_SL * WE_XLD; e += WE_NT) {
    const int i = e / WE_XLD, k = e - i * WE_XLD;
    S.W1j[i][k] = k < IN ? W[0][(int64_t)(WE_SL * j + i) * IN + k] : 0.f;
  }
  for (int e = tid; e < WE_SL * H; e += WE_NT) {
    const int i = e / H, k = e - i * H;
    S.W2r[i][k] = W[2][(int64_t)(WE_SL * j + i) * H + k];
  }
  // small parameters: index e -> (tensor, element) in the flat buffer (-1: padding)
  auto small_flat = [&](int e) -> int64_t {
    if (e < WE_SL) return foff(W[1]) + WE_SL * j + e;                         // b1
    e -= WE_SL;
    if (e < WE_SL) return foff(W[3]) + WE_SL * j + e;                         // b2
    e -= WE_SL;
    if (e < WE_OUTM * WE_SL) {                                                 // W3[o][16 j + c]
      const int o = e / WE_SL, c = e - o * WE_SL;
      return o < O ? foff(W[4]) + (int64_t)o * H + WE_SL * j + c : -1;
    }
    e -= WE_OUTM * WE_SL;
    if (e < WE_OUTM) return e < O ? foff(W[5]) + e : -1;                     // b3
    e -= WE_OUTM;
    return (net == 0 && HEAD == 1 && e < O) ? foff(d.log_std) + e : -1;       // log_std
  };
  float m_s = 0.f, v_s = 0.f;
  int64_t fs = -1;
  if (tid < WE_NSMALL) {
    fs = small_flat(tid);
    S.small[tid] = fs >= 0 ? a.params[fs] : 0.f;
    m_s = fs >= 0 ? a.exp_avg[fs] : 0.f;
    v_s = fs >= 0 ? a.exp_avg_sq[fs] : 0.f;
  }
  // W2 row slice: wave w holds column tiles 4 w + t (t < 4) of row tile j: lane element (t, r) =
  // W2[16 j + 4 g + r][16 (4 w + t) + li].  Tiles beyond H are inactive.
  float m_r[4][4], v_r[4][4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int ct = 4 * w + t;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool on = ct < G;
      const int64_t fr = foff(W[2]) + (int64_t)(WE_SL * j + 4 * g + r) * H + WE_SL * ct + li;
      m_r[t][r] = on ? a.exp_avg[fr] : 0.f;
      v_r[t][r] = on ? a.exp_avg_sq[fr] : 0.f;
    }
  }
  // W1 rows j: wave w holds column tile w: lane element r = W1[16 j + 4 g + r][16 w + li]
  float m_1[4], v_1[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int col = WE_SL * w + li;
    const int64_t f = foff(W[0]) + (int64_t)(WE_SL * j + 4 * g + r) * IN + col;
    m_1[r] = col < IN ? a.exp_avg[f] : 0.f;
    v_1[r] = col < IN ? a.exp_avg_sq[f] : 0.f;
  }

  const int B = a.batch;
  const int64_t n_rows = a.n_rows;
  const int nmb = (int)((n_rows + B - 1) / B);
  const int64_t step0 = a.state->opt_step;
  const int stat0 = a.state->stat_index;
  const int norm0 = a.state->norm_index;
  const float beta2 = ohp.beta2, eps = ohp.eps, lr = ohp.lr;
  const double beta1_d = ohp.beta1_d, beta2_d = ohp.beta2_d;
  const float c1 = (float)(1.0 - beta1_d), c2 = (float)(1.0 - beta2_d);
  double pw1 = ipow(beta1_d, step0), pw2 = ipow(beta2_d, step0);
  if (tid == 0) {
    S.bail = 0;
    S.xl = 0;
    // register this workgroup's XCC (completed long before its step-0 A arrival: the drains between)
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
    __hip_atomic_fetch_or(&ctr[WE_CXCC * (WE_CTR_STRIDE / 8) + net], 1ull << (xcc & 15), __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  bool xl = false;  // the store form of the B / C / W2 hand-offs from step 0 on and of A from step 1 on
  const int64_t w2t_mine = WE_W2T_OFF + net * WE_W2T_NET + (int64_t)j * WE_GMAX * 1024;  // my published tiles
  we_publish_w2(S.W2r, wrs, w2t_mine, G, w, lane, false);  // the initial W2, for step 0's column owners

  // the next minibatch's records are loaded into registers one step ahead: one contiguous block of
  // rws x R floats (R = 12 + IN4), WE_RU 16-B loads per thread (those past the block not issued:
  // wave-uniform skip); the staging destination of each (Lin row or Xl row, both 16-B aligned) is
  // fixed per thread and computed once
  const int R = WE_LIN + IN4, R4 = R >> 2;
  f4 xr[WE_RU];
  int dst[WE_RU];  // LDS float index of the 16 B this thread stages (-1: none); Lin words 0-11, Xl beyond
#pragma unroll
  for (int u = 0; u < WE_RU; ++u) {
    const int e4 = tid + WE_NT * u;
    const int row = e4 / R4, c4 = e4 - row * R4;
    dst[u] = row >= WE_B ? -1 : (c4 < WE_LIN / 4 ? WE_B * WE_INMAX + row * WE_LIN + 4 * c4 : row * IN4 + 4 * (c4 - WE_LIN / 4));
  }
  // buffer loads: the minibatch's block offset joins each thread's fixed 16-B offset in the VECTOR offset,
  // so a record past the rollout's last row reads 0 (the buffer's bound applies to voffset only -- soffset
  // is excluded from the range check -- which covers the rows [rws, B) of the last, partial minibatch)
  const __amdgpu_buffer_rsrc_t rrs = we_rsrc(a.rec, n_rows * R * 4);
  auto prefetch = [&](int m) {
    const int64_t r0 = (int64_t)m * B;
    const int rws = (int)min((int64_t)B, n_rows - r0);
    const int n4 = rws * R4;
    const int boff = (int)(r0 * R * 4);
#pragma unroll
    for (int u = 0; u < WE_RU; ++u) {
      xr[u] = f4{0.f, 0.f, 0.f, 0.f};
      if (WE_NT * u + 64 * w < n4)  // wave-uniform skip of the 16-B pieces past the block
        xr[u] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rrs, boff + 16 * (tid + WE_NT * u), 0, 0));
    }
  };
  if (nmb > 0) prefetch(0);
  // the loss's divides by the minibatch size (rows x world) and the entropy count, for a full and for the
  // last minibatch: off the step's critical path
  const int rows_last = nmb > 0 ? (int)(n_rows - (int64_t)(nmb - 1) * B) : 0;
  const float invB_full = 1.f / (float)(B * a.world), invB_last = 1.f / (float)(rows_last * a.world);
  const float dent_full = -hp.ent_coef / (float)((HEAD == 1 ? B * O : B) * a.world);
  const float dent_last = -hp.ent_coef / (float)((HEAD == 1 ? rows_last * O : rows_last) * a.world);
#ifdef RAI_STAMPS
  unsigned long long st_acc[24] = {0}, t_last = __builtin_amdgcn_s_memtime();
#endif
  // clip + Adam on this workgroup's W2 row slice with the last D phase's clip coefficient and bias
  // corrections (S.coef / S.adamc, rewritten only by the next D phase) and the gradient rows g_r
  float g_r[4][4];  // this step's W2-row gradient, kept for the deferred Adam
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) g_r[t][r] = 0.f;
  // (element pairs in packed f32 math; branch-free over the column tiles: a tile past H has zero moments
  // and gradient, so its update leaves those padding columns of W2r -- never read -- as they are.  All the
  // LDS reads first, then the arithmetic, then the stores, so the pairs' latencies overlap.)
  auto adam_w2 = [&](int t0, int t1) {  // the column tiles t in [t0, t1) of each wave
    const float coef = S.coef;
    const float inv_c3 = S.adamc[0], c4 = S.adamc[1];
    const f2a C2 = {coef, coef};
    f2a pp[4][2];
#pragma unroll
    for (int t = t0; t < t1; ++t)
#pragma unroll
      for (int h = 0; h < 2; ++h)
        pp[t][h] = f2a{S.W2r[4 * g + 2 * h][WE_SL * (4 * w + t) + li], S.W2r[4 * g + 2 * h + 1][WE_SL * (4 * w + t) + li]};
#pragma unroll
    for (int t = t0; t < t1; ++t) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        f2a mm = {m_r[t][2 * h], m_r[t][2 * h + 1]}, vv = {v_r[t][2 * h], v_r[t][2 * h + 1]};
        const f2a gg = f2a{g_r[t][2 * h], g_r[t][2 * h + 1]} * C2;
        adam_fast2(pp[t][h], mm, vv, gg, c1, c2, beta2, inv_c3, c4, eps);
        m_r[t][2 * h] = mm.x;
        m_r[t][2 * h + 1] = mm.y;
        v_r[t][2 * h] = vv.x;
        v_r[t][2 * h + 1] = vv.y;
      }
    }
#pragma unroll
    for (int t = t0; t < t1; ++t)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        S.W2r[4 * g + 2 * h][WE_SL * (4 * w + t) + li] = pp[t][h].x;
        S.W2r[4 * g + 2 * h + 1][WE_SL * (4 * w + t) + li] = pp[t][h].y;
      }
  };

  for (int mb = 0; mb < nmb; ++mb) {
    const int par = mb & 1;
    const int64_t row0 = (int64_t)mb * B;
    const int rows = (int)min((int64_t)B, n_rows - row0);
    const unsigned long long want = (unsigned long long)G * (mb + 1);
    // ---- the minibatch's records -> LDS: loss inputs to Lin, observations to Xl (rows beyond the
    // data are zero) ----------------------------------------------------------------------------
#pragma unroll
    for (int u = 0; u < WE_RU; ++u)
      if (dst[u] >= 0) *reinterpret_cast<f4*>(&S.Xl[dst[u]]) = xr[u];
    lds_barrier();
    // wave 1 during the A wait: the Gaussian head's per-step constants of Normal(mu, exp(log_std)) --
    // variance, log scale (lane o) and the per-row entropy summed over dims in order
    auto side_a = [&]() {
      if (net != 0 || HEAD != 1) return;
      const float* ls = &S.small[2 * WE_SL + WE_OUTM * WE_SL + WE_OUTM];
      const float scale = expf(ls[lane < O ? lane : 0]);
      const float lsc = logf(scale);
      if (lane < WE_OUTM) {
        S.ginv[lane] = 1.f / (scale * scale);
        S.glsc[lane] = lsc;
      }
      float ent = 0.f;
      for (int o = 0; o < O; ++o)
        ent += 1.4189385332046727f + __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, lsc), o));
      if (lane == 0) S.entc = ent;
    };
    // wave 1 during the D wait: the minibatch's loss statistics (per-row values left in S.st)
    auto side_d = [&]() {
      pw1 *= beta1_d;
      pw2 *= beta2_d;
      if (lane == 0) {
        S.adamc[0] = 1.f / (float)sqrt(1.0 - pw2);
        S.adamc[1] = (float)(-((double)lr / (1.0 - pw1)));
      }
      double st[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) st[i] = wave_sum_dpp(S.st[i][lane]);
      if (j == 0 && lane == 0 && a.stats) {
        const int srow = stat0 + mb;
        if (srow < a.max_stats) {
          float* row = a.stats + (int64_t)srow * RAI_STAT_STRIDE;
          const double Bd = (double)rows * (double)a.world;
          if (net == 0) {
            const float pi_loss = (float)(-st[0] / Bd);
            const float ent_loss = (float)(-st[3] / ((double)(HEAD == 1 ? rows * O : rows) * (double)a.world));
            row[0] = pi_loss + hp.ent_coef * ent_loss;  // the host adds vf_coef * v_loss
            row[1] = pi_loss;
            row[2] = ent_loss;
            row[3] = (float)(st[1] / Bd);
            row[4] = (float)(st[2] / Bd);
          } else {
            row[5] = (float)(st[0] / Bd) * (hp.ppo2_vf_coef_halving ? 0.5f : 1.f);
            row[5 + RAI_MAX_K] = hp.has_clip_range_vf ? (float)(st[1] / Bd) : 0.f;
          }
        }
      }
    };
    // ============ fwd1: H1[:, j] = act(X W1[j]^T + b1[j]); wave w: row tile w =============
    {
      // k in [IN, IN4) reads the observation's zero padding against W1j's
      const f4 z = we_fwd1(&S.Xl[(16 * w + li) * IN4 + g], &S.W1j[li][g], IN4 / 4);
      const float bj = S.small[li];
#pragma unroll
      for (int r = 0; r < 4; ++r) S.H1j[16 * w + 4 * g + r][li] = we_act(act, z[r] + bj);
    }
    lds_barrier();
    {  // publish H1[:, j]: row tid >> 2, columns 4 (tid & 3) ..
      const int r = tid >> 2, q = tid & 3;
      const f4 v = {S.H1j[r][4 * q], S.H1j[r][4 * q + 1], S.H1j[r][4 * q + 2], S.H1j[r][4 * q + 3]};
      const int64_t off = WE_H1_OFF + (int64_t)(net * 2 + par) * WE_ACT_SLOT + ((int64_t)r * H + WE_SL * j + 4 * q) * 4;
      we_st16(__builtin_bit_cast(u4v, v), wrs, (int)off, xl);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    WSTAMP(0);
    // A: arrive, then -- while the other workgroups' H1 slices land -- the previous step's Adam on this
    // workgroup's W2 rows (deferred from its D phase: only fwd2 and the W2 publish below read them), then
    // wait.  Same values as applying it at the end of the previous step.
    we_arrive(ctr, WE_CA + net);
    if (w == 1) side_a();
    // (half of it: the other half runs under the H1 gather's LDS-DMA below)
    if (WE_DEFER_W2 && mb > 0) adam_w2(0, 2);
    WSTAMP(22);  // (stamps: the A wait split into the deferred Adam and the rest of the wait)
    if (!we_wait(ctr, WE_CA + net, want, a.state, S.bail)) break;
#ifndef RAI_WE_NO_XCC_LOCAL
    if (mb == 0) {  // every workgroup of the network registered its XCC before its step-0 A arrival
      if (tid == 0) {
        const unsigned long long m = __hip_atomic_fetch_or(&ctr[WE_CXCC * (WE_CTR_STRIDE / 8) + net], 0ull,
                                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        S.xl = m != 0 && (m & (m - 1)) == 0;
      }
      __syncthreads();
      xl = __builtin_amdgcn_readfirstlane(S.xl) != 0;
    }
#endif
    WSTAMP(1);
    // H1 -> Act by LDS-DMA, and while it lands the deferred W2 Adam's other half (LDS rows W2r, disjoint
    // from Act); then the drain and the barrier
    we_gather_lds(a.ws, WE_H1_OFF + (int64_t)(net * 2 + par) * WE_ACT_SLOT, H, S.Act, w, lane, false);
    if (WE_DEFER_W2 && mb > 0) adam_w2(2, 4);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
    // W2 rows j (as updated by the last Adam step, every wave's tiles: after the barrier) for this step's
    // column owners: drained in the background during fwd2 -- by the B publish's drain, before this
    // workgroup's B arrival, after which the column owners load them (step 0: the tiles published before
    // the loop)
    if (mb > 0) we_publish_w2(S.W2r, wrs, w2t_mine, G, w, lane, xl);
    WSTAMP(2);
    // ============ fwd2: H2[:, j] = act(H1 W2[j]^T + b2[j]); wave w: row tile w =============
    {
      const f4 z = we_tile_dot(&S.Act[16 * w][0], &S.W2r[0][0], H, lane);
      const float bj = S.small[WE_SL + li];
#pragma unroll
      for (int r = 0; r < 4; ++r) S.H2j[16 * w + 4 * g + r][li] = we_act(act, z[r] + bj);
    }
    lds_barrier();
    WSTAMP(3);
    {  // output-layer partials over the slice: P[row][o] = sum_c H2[row][c] W3[o][16 j + c]
      if (tid < WE_B * 2) {
        const int r = tid >> 1, o0 = 4 * (tid & 1);
        // 16-B LDS reads, no per-output branches: W3 rows o >= O are zero, so those sums are 0
        f4 p = {0.f, 0.f, 0.f, 0.f};
        const f4* h4 = reinterpret_cast<const f4*>(&S.H2j[r][0]);
        const f4 h[4] = {h4[0], h4[1], h4[2], h4[3]};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f4* w4 = reinterpret_cast<const f4*>(&S.small[2 * WE_SL + (o0 + q) * WE_SL]);
          float s = 0.f;
#pragma unroll
          for (int c4 = 0; c4 < 4; ++c4) {
            const f4 wv = w4[c4];
            s += h[c4].x * wv.x;
            s += h[c4].y * wv.y;
            s += h[c4].z * wv.z;
            s += h[c4].w * wv.w;
          }
          p[q] = s;
        }
        const int64_t off = WE_P_OFF + (int64_t)(net * 2 + par) * WE_P_SLOT + (((int64_t)j * WE_B + r) * WE_OUTM + o0) * 4;
        we_st16(__builtin_bit_cast(u4v, p), wrs, (int)off, xl);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    WSTAMP(4);
    if (!we_arrive_wait(ctr, WE_CB + net, want, a.state, S.bail, w, [] {})) break;
    WSTAMP(5);
    // ============ head + loss, all rows (identical on every workgroup of the network) ========
    {  // slice partials: wave w sums slices [4 w, 4 w + 4) for row = lane (loads issued together)
      const int64_t base = WE_P_OFF + (int64_t)(net * 2 + par) * WE_P_SLOT;
      f4 qa[4], qb[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int ss = min(4 * w + u, G - 1);
        const int64_t off = base + (((int64_t)ss * WE_B + lane) * WE_OUTM) * 4;
        qa[u] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(wrs, (int)off, 0, WE_SC1));
        qb[u] = O > 4 ? __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(wrs, (int)off + 16, 0, WE_SC1))
                      : f4{0.f, 0.f, 0.f, 0.f};
      }
#ifdef RAI_WE_W2T_EARLY  // A/B: the W2 column tiles issued before the partials land
      // after the partials landed (in-order vmcnt: issued earlier, they would delay them): W2's column
      // slice j (16 tiles of 1 KB, one LDS-DMA load each; needed at dH1, drained by the
      // dZ2 gather's vmcnt).  Lane l lands at LDS slot (u = l >> 2, s = l & 3) and fetches piece
      // we_w2t_slot(u, s) of row u (the swizzle is an involution: pre-swizzled source, as LDS-DMA needs)
      {
        const int u = lane >> 2;
        const unsigned char* src =
            a.ws + WE_W2T_OFF + net * WE_W2T_NET + (int64_t)j * 1024 + (u * WE_SL + 4 * we_w2t_slot(u, lane & 3)) * 4;
#pragma unroll
        for (int m = 0; m < WE_GMAX / 4; ++m) {
          const int p = w + 4 * m;
          if (p < G)
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const float*>(src + (int64_t)p * WE_GMAX * 1024),
                                             &S.W2cT[p][0][0], 16, 0, WE_SC1);
        }
      }
#endif
      f4 sa = {0.f, 0.f, 0.f, 0.f}, sb = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (4 * w + u < G) {
          sa += qa[u];
          sb += qb[u];
        }
      *reinterpret_cast<f4*>(&S.Pw[w][lane][0]) = sa;
      *reinterpret_cast<f4*>(&S.Pw[w][lane][4]) = sb;
#ifndef RAI_WE_W2T_EARLY
      // after the partials landed (in-order vmcnt: issued earlier, they would delay them): W2's column
      // slice j (16 tiles of 1 KB, one LDS-DMA load each; needed at dH1, drained by the
      // dZ2 gather's vmcnt).  Lane l lands at LDS slot (u = l >> 2, s = l & 3) and fetches piece
      // we_w2t_slot(u, s) of row u (the swizzle is an involution: pre-swizzled source, as LDS-DMA needs)
      {
        const int u = lane >> 2;
        const unsigned char* src =
            a.ws + WE_W2T_OFF + net * WE_W2T_NET + (int64_t)j * 1024 + (u * WE_SL + 4 * we_w2t_slot(u, lane & 3)) * 4;
#pragma unroll
        for (int m = 0; m < WE_GMAX / 4; ++m) {
          const int p = w + 4 * m;
          if (p < G)
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const float*>(src + (int64_t)p * WE_GMAX * 1024),
                                             &S.W2cT[p][0][0], 16, 0, WE_SC1);
        }
      }
#endif
    }
    lds_barrier();
    WSTAMP(6);
#ifndef RAI_WE_LOSS_ONE_WAVE
    if (HEAD == 1 && net == 0) {
      // Gaussian actor: every wave, 16 rows each, four lanes per row (lane & 3 = dimension pair dp: dims
      // 2 dp, 2 dp + 1).  The log-prob's eight per-dimension terms are gathered across the quad and summed
      // in dimension order (the one-wave form's order), so every lane of the quad forms the identical row
      // values; each lane then writes the loss gradient of its two dimensions.
#pragma clang fp contract(off)
      const int rq = lane >> 2, dp = lane & 3;
      const int r = 16 * w + rq;
      const bool valid = r < rows;
      const float* lr_ = &S.Xl[WE_B * WE_INMAX + r * WE_LIN];
      const float c_adv = lr_[0], c_lpold = lr_[1];
      const int o0 = 2 * dp;
      const float2 ca = *reinterpret_cast<const float2*>(&lr_[4 + o0]);  // the action's dims o0, o0 + 1
      float outv[2], term[2], ginv2[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int o = o0 + e;
        outv[e] = (((S.Pw[0][r][o] + S.Pw[1][r][o]) + S.Pw[2][r][o]) + S.Pw[3][r][o]) +
                  S.small[2 * WE_SL + WE_OUTM * WE_SL + o];
        ginv2[e] = S.ginv[o];
        const float xo = (e ? ca.y : ca.x) - outv[e];
        const float tm = -(xo * xo) * (0.5f * ginv2[e]) - S.glsc[o] - 0.91893853320467274f;
        term[e] = o < O ? tm : 0.f;
      }
      // the eight terms in every lane of the quad (quad_perm broadcasts), summed in dimension order
      auto qb = [](float v, int k) {
        const int x = __float_as_int(v);
        int y;
        switch (k) {
          case 0: y = __builtin_amdgcn_mov_dpp(x, 0x00, 0xF, 0xF, false); break;
          case 1: y = __builtin_amdgcn_mov_dpp(x, 0x55, 0xF, 0xF, false); break;
          case 2: y = __builtin_amdgcn_mov_dpp(x, 0xAA, 0xF, 0xF, false); break;
          default: y = __builtin_amdgcn_mov_dpp(x, 0xFF, 0xF, 0xF, false); break;
        }
        return __int_as_float(y);
      };
      float lp = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        lp += qb(term[0], k);
        lp += qb(term[1], k);
      }
      const float A = c_adv;  // normalized per minibatch by we_pack_kernel before the epoch
      const float ent = S.entc;
      const float invB = mb + 1 < nmb ? invB_full : invB_last;
      const float logratio = lp - c_lpold;
      const float ratio = expf(logratio);
      const float lo = 1.f - hp.clip_range, hi = 1.f + hp.clip_range;
      const float cr = fminf(fmaxf(ratio, lo), hi);
      const float s1 = ratio * A, s2 = cr * A;
      const float g_pi = -invB;
      float g1, g2;
      if (s1 < s2) { g1 = g_pi; g2 = 0.f; }
      else if (s1 > s2) { g1 = 0.f; g2 = g_pi; }
      else { g1 = g_pi * 0.5f; g2 = g_pi * 0.5f; }
      const float in_clip = (ratio >= lo && ratio <= hi) ? 1.f : 0.f;
      const float d_logp = valid ? (g1 * A + (g2 * A) * in_clip) * ratio : 0.f;
      const float d_ent = valid ? (mb + 1 < nmb ? dent_full : dent_last) : 0.f;
      float dd[2], dlv[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const bool on = o0 + e < O;
        const float xo = (e ? ca.y : ca.x) - outv[e];
        dd[e] = on ? d_logp * (xo * ginv2[e]) : 0.f;
        dlv[e] = on ? d_logp * ((xo * xo) * ginv2[e] - 1.f) + d_ent : 0.f;
      }
      *reinterpret_cast<float2*>(&S.dOut[r][o0]) = float2{dd[0], dd[1]};
      *reinterpret_cast<float2*>(&S.dls[r][o0]) = float2{dlv[0], dlv[1]};
      if (dp == 0) {
        S.st[0][r] = valid ? (double)fminf(s1, s2) : 0.0;
        S.st[1][r] = valid ? (double)((ratio - 1.f) - logratio) : 0.0;
        S.st[2][r] = valid ? ((fabsf(ratio - 1.f) > hp.clip_range) ? 1.0 : 0.0) : 0.0;
        S.st[3][r] = valid ? (double)ent : 0.0;
      }
      WSTAMP(7);
    } else
#endif
    if (w == 0) {
      const int r = lane;
      const bool valid = r < rows;
      const f4* lin = reinterpret_cast<const f4*>(&S.Xl[WE_B * WE_INMAX + r * WE_LIN]);
      const f4 l0 = lin[0], l1 = lin[1], l2 = lin[2];
      const float c_adv = l0.x, c_lpold = l0.y, c_ret = l0.z, c_vold = l0.w;
      const float c_act[WE_OUTM] = {l1.x, l1.y, l1.z, l1.w, l2.x, l2.y, l2.z, l2.w};
      const int64_t c_ai = __float_as_int(l1.x);
      // head outputs: the four waves' slice sums in order, + b3 (16-B LDS reads; entries o >= O are
      // zero throughout -- partials, W3 columns and b3 padding -- so no per-dimension branches)
      float out[WE_OUTM];
      {
        const f4* pw = reinterpret_cast<const f4*>(&S.Pw[0][r][0]);
        constexpr int WS = WE_B * WE_OUTM / 4;  // f4 stride between the waves' copies
        const f4 lo = ((pw[0] + pw[WS]) + pw[2 * WS]) + pw[3 * WS];
        const f4 hi = ((pw[1] + pw[WS + 1]) + pw[2 * WS + 1]) + pw[3 * WS + 1];
        const f4* b3 = reinterpret_cast<const f4*>(&S.small[2 * WE_SL + WE_OUTM * WE_SL]);
        const f4 ol = lo + b3[0], oh = hi + b3[1];
#pragma unroll
        for (int o = 0; o < 4; ++o) {
          out[o] = ol[o];
          out[4 + o] = oh[o];
        }
      }
      float dout[WE_OUTM], dl[WE_OUTM];
#pragma unroll
      for (int o = 0; o < WE_OUTM; ++o) dout[o] = dl[o] = 0.f;
      // statistics: [0] sum min(s1, s2) | loss, [1] sum kl | vclipped, [2] clipped, [3] entropy
      double st[4] = {0.0, 0.0, 0.0, 0.0};  // per row; summed by side_d
      const bool full = mb + 1 < nmb;  // the loss's per-step divides, formed before the loop
      const float invB = full ? invB_full : invB_last;
      if (net == 0) {
#pragma clang fp contract(off)
        const float A = c_adv;  // normalized per minibatch by we_adv_norm_kernel before the epoch
        float lp = 0.f, ent = 0.f;  // log-prob of the action, entropy (summed over dims)
        // Normal.log_prob's divisions by var and 2 var as products with the per-step reciprocal
        // (within an ulp of torch's quotients)
        float ginv[WE_OUTM];
        if (HEAD == 1) {
#pragma unroll
          for (int o = 0; o < WE_OUTM; ++o) ginv[o] = S.ginv[o];
#pragma unroll
          for (int o = 0; o < WE_OUTM; ++o) {  // dimensions o >= O masked (no uniform branches)
            const float xo = c_act[o] - out[o];
            const float term = -(xo * xo) * (0.5f * ginv[o]) - S.glsc[o] - 0.91893853320467274f;
            lp += o < O ? term : 0.f;
          }
          ent = S.entc;
        } else {
          const int64_t ai = c_ai;
          float mx = out[0];
#pragma unroll
          for (int o = 1; o < WE_OUTM; ++o)
            if (o < O) mx = fmaxf(mx, out[o]);
          float se = 0.f;
#pragma unroll
          for (int o = 0; o < WE_OUTM; ++o)
            if (o < O) se += expf(out[o] - mx);
          const float lse = mx + logf(se);
          float h = 0.f;
          float za = out[0];
#pragma unroll
          for (int o = 0; o < WE_OUTM; ++o)
            if (o < O) {
              const float l = out[o] - lse;
              h -= fmaxf(l, -3.4028234663852886e38f) * expf(l);
              if (o == (ai >= 0 && ai < O ? ai : 0)) za = out[o];
            }
          lp = za - lse;
          ent = h;
        }
        const float logratio = lp - c_lpold;
        const float ratio = expf(logratio);
        const float lo = 1.f - hp.clip_range, hi = 1.f + hp.clip_range;
        const float cr = fminf(fmaxf(ratio, lo), hi);
        const float s1 = ratio * A, s2 = cr * A;
        const float g_pi = -invB;
        float g1, g2;
        if (s1 < s2) { g1 = g_pi; g2 = 0.f; }
        else if (s1 > s2) { g1 = 0.f; g2 = g_pi; }
        else { g1 = g_pi * 0.5f; g2 = g_pi * 0.5f; }
        const float in_clip = (ratio >= lo && ratio <= hi) ? 1.f : 0.f;
        const float d_logp = valid ? (g1 * A + (g2 * A) * in_clip) * ratio : 0.f;
        const float d_ent = valid ? (full ? dent_full : dent_last) : 0.f;
        if (HEAD == 1) {
#pragma unroll
          for (int o = 0; o < WE_OUTM; ++o) {
            const float xo = c_act[o] - out[o];
            const bool on = o < O;
            dout[o] = on ? d_logp * (xo * ginv[o]) : 0.f;
            dl[o] = on ? d_logp * ((xo * xo) * ginv[o] - 1.f) + d_ent : 0.f;
          }
        } else {
          const int64_t ai = c_ai;
          float mx = out[0];
#pragma unroll
          for (int o = 1; o < WE_OUTM; ++o)
            if (o < O) mx = fmaxf(mx, out[o]);
          float se = 0.f;
#pragma unroll
          for (int o = 0; o < WE_OUTM; ++o)
            if (o < O) se += expf(out[o] - mx);
          const float lse = mx + logf(se);
          float h = 0.f;
#pragma unroll
          for (int o = 0; o < WE_OUTM; ++o)
            if (o < O) {
              const float l = out[o] - lse;
              h -= l * expf(l);
            }
#pragma unroll
          for (int o = 0; o < WE_OUTM; ++o)
            if (o < O) {
              const float l = out[o] - lse, p = expf(l);
              dout[o] = d_logp * ((o == ai ? 1.f : 0.f) - p) - d_ent * p * (l + h);
            }
        }
        if (valid) {
          st[0] = (double)fminf(s1, s2);
          st[1] = (double)((ratio - 1.f) - logratio);
          st[2] = (fabsf(ratio - 1.f) > hp.clip_range) ? 1.0 : 0.0;
          st[3] = (double)ent;
        }
      } else {
#pragma clang fp contract(off)
        const float v = out[0], R = c_ret;
        const float halve = hp.ppo2_vf_coef_halving ? 0.5f : 1.f;
        const float gl = (hp.vf_coef[0] * halve) * invB;
        const int vfn = hp.vf_loss_fn;
        float l = we_vf_loss(vfn, v - R), dv;
        float vcf = 0.f;
        if (hp.has_clip_range_vf) {
          const float vc_ = hp.clip_range_vf, vo = c_vold;
          const float dvo = v - vo;
          const float vcl = vo + fminf(fmaxf(dvo, -vc_), vc_);
          const float l2 = we_vf_loss(vfn, vcl - R);
          float w1, w2;
          if (l > l2) { w1 = gl; w2 = 0.f; }
          else if (l < l2) { w1 = 0.f; w2 = gl; }
          else { w1 = gl * 0.5f; w2 = gl * 0.5f; }
          const float inv = (dvo >= -vc_ && dvo <= vc_) ? 1.f : 0.f;
          dv = w1 * we_vf_grad(vfn, v - R) + (w2 * we_vf_grad(vfn, vcl - R)) * inv;
          vcf = (fabsf(v - vo) > vc_) ? 1.f : 0.f;
          l = fmaxf(l, l2);
        } else {
          dv = gl * we_vf_grad(vfn, v - R);
        }
        dout[0] = valid ? dv : 0.f;
        if (valid) {
          st[0] = (double)l;
          st[1] = (double)vcf;
        }
      }
      WSTAMP(7);
      *reinterpret_cast<f4*>(&S.dOut[r][0]) = f4{dout[0], dout[1], dout[2], dout[3]};
      *reinterpret_cast<f4*>(&S.dOut[r][4]) = f4{dout[4], dout[5], dout[6], dout[7]};
      *reinterpret_cast<f4*>(&S.dls[r][0]) = f4{dl[0], dl[1], dl[2], dl[3]};
      *reinterpret_cast<f4*>(&S.dls[r][4]) = f4{dl[4], dl[5], dl[6], dl[7]};
#pragma unroll
      for (int i = 0; i < 4; ++i) S.st[i][r] = st[i];
    }
    lds_barrier();
    WSTAMP(8);
    // ============ bwd2 (local): dZ2[:, j], publish; dW2 rows j; small gradients ===============
    {
      const int r = tid >> 2, q = tid & 3;
      const f4 d0 = *reinterpret_cast<const f4*>(&S.dOut[r][0]), d1 = *reinterpret_cast<const f4*>(&S.dOut[r][4]);
      const float dr[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
      f4 dh = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int o = 0; o < WE_OUTM; ++o)
        if (o < O) dh += dr[o] * *reinterpret_cast<const f4*>(&S.small[2 * WE_SL + o * WE_SL + 4 * q]);
      const f4 h2 = *reinterpret_cast<const f4*>(&S.H2j[r][4 * q]);
      f4 z;
#pragma unroll
      for (int u = 0; u < 4; ++u) z[u] = dh[u] * we_actd(act, h2[u]);
      *reinterpret_cast<f4*>(&S.Z2j[r][4 * q]) = z;
      const int64_t off = WE_Z2_OFF + (int64_t)(net * 2 + par) * WE_ACT_SLOT + ((int64_t)r * H + WE_SL * j + 4 * q) * 4;
      we_st16(__builtin_bit_cast(u4v, z), wrs, (int)off, xl);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (tid == 0) __hip_atomic_fetch_add(&ctr[(WE_CC + net) * (WE_CTR_STRIDE / 8)], 1ull, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    WSTAMP(9);
    // while dZ2 lands: small-parameter gradients and dW2 rows j (H1 still in Act)
    // small-parameter gradients as three MFMA tiles over the 64 rows (D[i][jj] = sum_k A[k][i] B[k][jj]),
    // one per wave: wave 0 dW3 = dOut^T H2 (i = o), wave 1 the column sums of [dOut | dls] (db3,
    // dlog_std), wave 2 those of dZ2 (db2); b1 j is formed after dZ1 (below).  Every workgroup forms
    // db3 / dlog_std with the same code on the same rows, so their copies stay identical.
    if (w < 3) {
      // row offsets are compile-time, so the reads use immediate offsets from one base
      f4 dsm;
      if (w == 0) dsm = we_small_tile<WE_OUTM, false>(&S.dOut[0][li & 7], &S.H2j[0][li], g);
      else if (w == 1)
        dsm = we_small_tile<WE_OUTM, true>(li < WE_OUTM ? &S.dOut[0][li] : &S.dls[0][li - WE_OUTM], nullptr, g);
      else dsm = we_small_tile<WE_SP, true>(&S.Z2j[0][li], nullptr, g);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 4 * g + r;  // D row; column jj = li
        if (w == 0) {
          if (i < WE_OUTM) S.gsm[2 * WE_SL + i * WE_SL + li] = dsm[r];
        } else if (li == 0) {
          if (w == 1) S.gsm[2 * WE_SL + WE_OUTM * WE_SL + i] = dsm[r];  // db3 (i < 8), dlog_std (i >= 8)
          else S.gsm[WE_SL + i] = dsm[r];                               // db2
        }
      }
    }
    WSTAMP(10);
    f4 g_rv[4];
    we_dw2_tiles4<0, WE_SL>(&S.Z2j[0][0], WE_SP, &S.Act[0][WE_SL * 4 * w], WE_HP, lane, g_rv);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) g_r[t][r] = 4 * w + t >= G ? 0.f : g_rv[t][r];
    WSTAMP(11);
    // wait for every workgroup's dZ2 slice
    if (tid == 0) {
      const unsigned long long t0 = rai_clock();
      while (__hip_atomic_load(&ctr[(WE_CC + net) * (WE_CTR_STRIDE / 8)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
             want) {
        if (rai_expired(t0, RAI_SPIN_LOCAL)) {
          __hip_atomic_store(&a.state->err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          S.bail = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __syncthreads();
    if (S.bail) break;
    WSTAMP(12);
    // dZ2 -> Act: wave w gathers the 16 rows of its own dH1 row tile (the only rows it reads below), so its
    // own drain suffices -- no workgroup barrier (the W2 column tiles it also reads were drained before the
    // C arrival's barrier)
    we_gather_lds(a.ws, WE_Z2_OFF + (int64_t)(net * 2 + par) * WE_ACT_SLOT, H, S.Act, w, lane, true, true);
    WSTAMP(13);
    // ============ bwd1: dH1[:, j] = dZ2 W2[:, slice j] -> dZ1, dW1 rows j, db1 j ==================
    {
      // wave w: row tile w; lane (li, g) holds dH1[16 w + 4 g + r][16 j + li], r < 4 (MFMA layout)
      const f4 z = we_dh1_tile(&S.Act[16 * w + li][0], &S.W2cT[0][li][0], H, g, li);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * w + 4 * g + r;
        S.Z1j[row][li] = z[r] * we_actd(act, S.H1j[row][li]);
      }
      WSTAMP(14);
    }
    lds_barrier();
    WSTAMP(15);
    f4 g_1 = {0.f, 0.f, 0.f, 0.f};  // dW1[16 j + 4 g + r][16 w + li]
    if (WE_SL * w < IN) {
      // all 32 operands read first (the observation rows' stride IN4 is a runtime value, so their
      // addresses are formed here, outside the MFMA sequence), then two accumulator chains
      const float* za = &S.Z1j[we_krow(0, g)][li];
      const float* xa = &S.Xl[we_krow(0, g) * IN4 + min(WE_SL * w + li, IN - 1)];
      float zv[WE_B / 4], xv[WE_B / 4];
#pragma unroll
      for (int kk = 0; kk < WE_B / 4; ++kk) {
        const int dk = 8 * (kk >> 1) + (kk & 1);  // we_krow(kk, g) - we_krow(0, g)
        zv[kk] = za[dk * WE_SP];
        xv[kk] = xa[dk * IN4];
      }
      __builtin_amdgcn_sched_barrier(0);
      f4 g_1b = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < WE_B / 4; ++kk) {
        if (kk & 1) g_1b = __builtin_amdgcn_mfma_f32_16x16x4f32(zv[kk], xv[kk], g_1b, 0, 0, 0);
        else g_1 = __builtin_amdgcn_mfma_f32_16x16x4f32(zv[kk], xv[kk], g_1, 0, 0, 0);
      }
      g_1 += g_1b;
    }
    WSTAMP(16);
    // db1 (wave 3, all lanes): lane (c = lane & 15, q = lane >> 4) sums rows [16 q, 16 q + 16) of
    // column c in four chains; the quarters are added by the row / half swaps
    float db1_sq = 0.f;
    if (w == 3) {
      const int c = lane & 15, q = lane >> 4;
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int r = 0; r < 16; r += 4)
#pragma unroll
        for (int u = 0; u < 4; ++u) acc[u] += S.Z1j[16 * q + r + u][c];
      float v = ((acc[0] + acc[1]) + acc[2]) + acc[3];
      const auto r16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
      v = __uint_as_float(r16[0]) + __uint_as_float(r16[1]);
      const auto r32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
      v = __uint_as_float(r32[0]) + __uint_as_float(r32[1]);
      if (lane < WE_SL) {
        S.db1[lane] = v;
        db1_sq = v;  // its square joins wave 3's norm share
      }
    }
    WSTAMP(17);
    // ============ X (data parallel): the owned gradient summed over the ranks in rank order ==========
    if (a.world > 1) {
      __syncthreads();  // S.gsm (waves 0-2) and S.db1 (wave 3) complete
      const int W = a.world;
      const unsigned long long step_id = (unsigned long long)(a.xbase + mb + 1);
      // the cross-rank slots alternate with the GLOBAL step (not mb, which restarts every launch): with an
      // odd minibatch count a rank entering the next launch early would otherwise reuse the parity a slow
      // peer is still summing
      const int xpar = (int)((a.xbase + mb) & 1);
      const int rb = (int)rai_xdp_wide_bytes(W);
      // slot floats: [0, 4096) W2 rows j as f4 (w 4 + t) 64 + lane; [4096, 5120) W1 rows j, f4 w 64 + lane;
      // [5120, 5296) the small gradients by small index (db1 j from S.db1)
      auto slot_off = [&](int sender) {
        return RAI_XDP_SLOTS_OFF + ((((xpar * W + sender) * 2 + net) * WE_GMAX + j) * RAI_XDP_WIDE_SLOTF) * 4;
      };
      const bool w1_on = WE_SL * w < IN;
      const bool sm_on = tid < WE_NSMALL / 4;
      f4 psm = {0.f, 0.f, 0.f, 0.f};
      if (sm_on) psm = *reinterpret_cast<const f4*>(tid < WE_SL / 4 ? &S.db1[4 * tid] : &S.gsm[4 * tid]);
      const int my = slot_off(a.xrank);
      for (int pr = 0; pr < W; ++pr) {
        const __amdgpu_buffer_rsrc_t prs = we_rsrc(a.xpeers[pr], rb);
#pragma unroll
        for (int t = 0; t < 4; ++t)
          if (4 * w + t < G) {
            const f4 v = {g_r[t][0], g_r[t][1], g_r[t][2], g_r[t][3]};
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, v), prs, my + ((w * 4 + t) * 64 + lane) * 16,
                                                   0, WE_XDP_AUX);
          }
        if (w1_on)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, g_1), prs, my + (4096 + (w * 64 + lane) * 4) * 4,
                                                 0, WE_XDP_AUX);
        if (sm_on)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, psm), prs, my + (5120 + 4 * tid) * 4, 0,
                                                 WE_XDP_AUX);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains
      __syncthreads();
      if (tid < W) {
        unsigned long long* fl = reinterpret_cast<unsigned long long*>(a.xpeers[tid]) + (net * 8 + a.xrank) * WE_GMAX + j;
        __hip_atomic_store(fl, step_id, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      if (w == 0) {
        const unsigned long long* fl =
            reinterpret_cast<const unsigned long long*>(a.xpeers[a.xrank]) + (net * 8 + (lane < W ? lane : 0)) * WE_GMAX + j;
        const unsigned long long t0 = rai_clock();
        for (;;) {
          const bool ok = lane >= W || __hip_atomic_load(fl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= step_id;
          if (__all(ok)) break;
          if (rai_expired(t0, RAI_SPIN_REMOTE)) {
            if (lane == 0) {
              __hip_atomic_store(&a.state->err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              S.bail = 1;
            }
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      __syncthreads();
      if (S.bail) break;
      const __amdgpu_buffer_rsrc_t lrs = we_rsrc(a.xpeers[a.xrank], rb);
      f4 s2[4], s1 = {0.f, 0.f, 0.f, 0.f}, ssm = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < 4; ++t) s2[t] = f4{0.f, 0.f, 0.f, 0.f};
      for (int pr = 0; pr < W; ++pr) {
        const int off = slot_off(pr);
#pragma unroll
        for (int t = 0; t < 4; ++t)
          if (4 * w + t < G)
            s2[t] += __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(lrs, off + ((w * 4 + t) * 64 + lane) * 16,
                                                                                 0, WE_XDP_AUX));
        if (w1_on)
          s1 += __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(lrs, off + (4096 + (w * 64 + lane) * 4) * 4, 0,
                                                                            WE_XDP_AUX));
        if (sm_on)
          ssm += __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(lrs, off + (5120 + 4 * tid) * 4, 0, WE_XDP_AUX));
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
        if (4 * w + t < G)
#pragma unroll
          for (int r = 0; r < 4; ++r) g_r[t][r] = s2[t][r];
      if (w1_on) g_1 = s1;
      if (sm_on) *reinterpret_cast<f4*>(tid < WE_SL / 4 ? &S.db1[4 * tid] : &S.gsm[4 * tid]) = ssm;
      __syncthreads();
      if (w == 3 && lane < WE_SL) db1_sq = S.db1[lane];
    }
    // ============ D: this workgroup's share of |g|^2, then clip_grad_norm_ + Adam =============
    {
      double ss = 0.0;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const double gv = (double)g_r[t][r];
          ss += gv * gv;
        }
      if (WE_SL * w + li < IN) {
#pragma unroll
        for (int r = 0; r < 4; ++r) ss += (double)g_1[r] * (double)g_1[r];
      }
      // b3 and log_std are counted once, by workgroup 0
      const bool count_small = tid < WE_NSMALL && fs >= 0 &&
                               (tid < 2 * WE_SL + WE_OUTM * WE_SL || j == 0);
      const float g_s = tid < WE_SL ? 0.f : S.gsm[min(tid, WE_NSMALL - 1)];
      if (count_small && tid >= WE_SL) ss += (double)g_s * (double)g_s;  // db1: wave 3 below
      ss += (double)db1_sq * (double)db1_sq;
      ss = wave_sum_dpp(ss);
      if (lane == 0) S.red[0][w] = ss;
      __syncthreads();
      we_gu64* gd = we_gptr(a.ws + WE_GD_OFF);
      if (tid == 0) {  // the share as two granules (hi, lo words of the double)
        const double tot = ((S.red[0][0] + S.red[0][1]) + S.red[0][2]) + S.red[0][3];
        const unsigned long long u = __double_as_longlong(tot);
        we_gu64* gs = gd + ((int64_t)(par * 2 + net) * WE_GMAX + j) * 2;
        we_put(gs, (unsigned)mb + 1, (unsigned)(u >> 32));
        we_put(gs + 1, (unsigned)mb + 1, (unsigned)u);
      }
    }
    WSTAMP(18);
    // the next minibatch's inputs: they land during the D sweep and Adam
    if (mb + 1 < nmb) prefetch(mb + 1);
    WSTAMP(19);
    // D: wave 0 sweeps the 2 G shares (both networks: clip_grad_norm_ is over all parameters) and
    // forms the clip coefficient; wave 1 meanwhile runs the stats / Adam-constant side job
    if (w == 0) {
      const int l = lane < 2 * G ? lane : 0;
      const int nn = l / G, jj = l - nn * G;
      we_gu64* gs = we_gptr(a.ws + WE_GD_OFF) + ((int64_t)(par * 2 + nn) * WE_GMAX + jj) * 2;
      const unsigned tag = (unsigned)mb + 1;
      unsigned long long hi, lo;
      const unsigned long long t0 = rai_clock();
      for (;;) {
        hi = we_get(gs);
        lo = we_get(gs + 1);
        if (__all((unsigned)(hi >> 32) == tag && (unsigned)(lo >> 32) == tag)) break;
        if (rai_expired(t0, RAI_SPIN_LOCAL)) {
          if (lane == 0) {
            __hip_atomic_store(&a.state->err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            S.bail = 1;
          }
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      const double sh = __longlong_as_double((long long)((hi << 32) | (lo & 0xffffffffull)));
      // the 2 G shares, net-major then slice order, fixed-order wave sum
      const double tot = wave_sum_dpp(lane < 2 * G ? sh : 0.0);
      const float total_norm = (float)sqrt(tot);
      float coef = 1.f;
      if (ohp.max_grad_norm > 0.f) coef = fminf(ohp.max_grad_norm / (total_norm + 1e-6f), 1.f);
      if (lane == 0) S.coef = coef;
      if (net == 0 && j == 0 && lane == 0 && a.norms && norm0 + mb < a.max_norms) a.norms[norm0 + mb] = total_norm;
    } else if (w == 1) {
#ifndef RAI_WE_SKIP_SIDE_D  // timing experiments only: stale Adam constants and no stats rows
      side_d();
#endif
    }
    __syncthreads();
    if (S.bail) break;
    WSTAMP(20);
    {
      const float coef = S.coef;
      const float inv_c3 = S.adamc[0], c4 = S.adamc[1];
      // (the W2 row slice: deferred to the next step's A wait, adam_w2)
      if (!WE_DEFER_W2) adam_w2(0, 4);
      if (WE_SL * w + li < IN) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float& p = S.W1j[4 * g + r][WE_SL * w + li];
          float pv = p;
          adam_fast(pv, m_1[r], v_1[r], g_1[r] * coef, c1, c2, beta2, inv_c3, c4, eps);
          p = pv;
        }
      }
      if (tid < WE_NSMALL && fs >= 0) {
        float pv = S.small[tid];
        adam_fast(pv, m_s, v_s, (tid < WE_SL ? S.db1[tid] : S.gsm[tid]) * coef, c1, c2, beta2, inv_c3, c4, eps);
        S.small[tid] = pv;
      }
    }
    lds_barrier();
    WSTAMP(21);
  }
  if (WE_DEFER_W2 && !S.bail && nmb > 0) {  // the last step's deferred W2 Adam
    adam_w2(0, 4);
    lds_barrier();
  }
#ifdef RAI_STAMPS
  if (j == 0 && tid == 0)
    for (int i = 0; i < 24; ++i) atomicAdd(&g_we_stamps[net][i], i == 23 ? (unsigned long long)xl : st_acc[i]);
#endif

  // ---- write back what this workgroup owns: parameters and Adam moments ----------------------
  if (!S.bail) {
    for (int e = tid; e < WE_SL * IN; e += WE_NT) {
      const int i = e / IN, k = e - i * IN;
      a.params[foff(W[0]) + (int64_t)(WE_SL * j + i) * IN + k] = S.W1j[i][k];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int col = WE_SL * w + li;
      if (col < IN) {
        const int64_t f = foff(W[0]) + (int64_t)(WE_SL * j + 4 * g + r) * IN + col;
        a.exp_avg[f] = m_1[r];
        a.exp_avg_sq[f] = v_1[r];
      }
    }
    for (int e = tid; e < WE_SL * H; e += WE_NT) {
      const int i = e / H, k = e - i * H;
      a.params[foff(W[2]) + (int64_t)(WE_SL * j + i) * H + k] = S.W2r[i][k];
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int ct = 4 * w + t;
      if (ct < G) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t f = foff(W[2]) + (int64_t)(WE_SL * j + 4 * g + r) * H + WE_SL * ct + li;
          a.exp_avg[f] = m_r[t][r];
          a.exp_avg_sq[f] = v_r[t][r];
        }
      }
    }
    // small parameters: b3 / log_std copies are identical everywhere; workgroup 0 writes them
    if (tid < WE_NSMALL && fs >= 0 && (tid < 2 * WE_SL + WE_OUTM * WE_SL || j == 0)) {
      a.params[fs] = S.small[tid];
      a.exp_avg[fs] = m_s;
      a.exp_avg_sq[fs] = v_s;
    }
  }
  if (net == 0 && j == 0 && tid == 0 && !S.bail) {
    a.state->stat_index = stat0 + nmb;
    a.state->opt_step = step0 + nmb;
    a.state->norm_index = norm0 + nmb;
  }
}

// The epoch's per-row records (layout at WE_REC_OFF) from its permuted rollout copy, one wave per
// minibatch (lane = row), before the epoch: the advantage normalized over the minibatch
// (ppo.py:313-316: mean and the unbiased std, fp64 two-pass sums; copied when neither normalization
// is on) -- it depends on no parameter, so the epoch kernel reads it instead of forming it on its
// critical path -- then the loss inputs and the zero-padded observation.
__global__ __launch_bounds__(256) void we_pack_kernel(const float* obs, const void* actions, const float* old_logp,
                                                      const float* old_values, const float* adv, const float* ret,
                                                      int64_t n_rows, int B, int IN, int O, int head,
                                                      const rai_ppo_hparams* hpp, const float* moments, float* rec) {
#pragma clang fp contract(off)
  const int64_t mb = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int64_t r0 = mb * B;
  if (r0 >= n_rows) return;  // wave-uniform
  const rai_ppo_hparams& hp = *hpp;
  const int rows = (int)min((int64_t)B, n_rows - r0);
  const bool valid = lane < rows;
  const int64_t gr = r0 + (valid ? lane : 0);
  const float x = valid ? adv[gr] : 0.f;
  float A = x;
  if (moments) {  // data parallel: the global minibatch's (mean, den), the normalize / standardize rule encoded
    A = (x - moments[2 * mb]) / moments[2 * mb + 1];
  } else if (hp.normalize_advantage || hp.standardize_advantage) {
    const double s1 = wave_sum_dpp(valid ? (double)x : 0.0);
    const float mean = (float)(s1 / (double)rows);
    const double dv = (double)x - (double)mean;
    const double s2 = wave_sum_dpp(valid ? dv * dv : 0.0);
    const float den = (float)sqrt(s2 / (double)(rows - 1)) + 1e-8f;
    A = hp.normalize_advantage ? (x - mean) / den : x / den;
  }
  if (!valid) return;
  const int IN4 = (IN + 3) & ~3, R = WE_LIN + IN4;
  float* out = rec + gr * R;
  out[0] = A;
  out[1] = old_logp[gr];
  out[2] = ret[gr];
  out[3] = old_values[gr];
  for (int o = 0; o < 8; ++o) {
    float v = 0.f;
    if (head == 1) v = o < O ? static_cast<const float*>(actions)[gr * O + o] : 0.f;
    else if (o == 0) v = __int_as_float((int)static_cast<const int64_t*>(actions)[gr]);
    out[4 + o] = v;
  }
  for (int k = 0; k < IN4; ++k) out[WE_LIN + k] = k < IN ? obs[gr * IN + k] : 0.f;
}

template <int HEAD>
__global__ __launch_bounds__(WE_NT) __attribute__((amdgpu_waves_per_eu(1, 1))) void mlp_wide_epoch_kernel(const WeArgs a) {
  static_assert(sizeof(WeSmem) <= 160 * 1024, "LDS budget");
  __shared__ __attribute__((aligned(16))) unsigned char smem_raw[sizeof(WeSmem)];
  const int b = blockIdx.x, grp = b & 7, j = b >> 3;
  if (grp >= 2) return;  // two XCDs' worth of blocks work (locality, not correctness)
  we_epoch<HEAD>(a, *reinterpret_cast<WeSmem*>(smem_raw), grp, j);
}

}  // namespace

#ifdef RAI_STAMPS
extern "C" int rai_wide_epoch_debug_stamps(unsigned long long* host_out) {
  return (int)hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_we_stamps), sizeof(g_we_stamps));
}
#endif

extern "C" int64_t rai_mlp_wide_epoch_workspace_bytes(int32_t hidden, int32_t in_dim, int64_t n_rows) {
  (void)hidden;
  return (n_rows < 0 || in_dim < 1 || in_dim > WE_INMAX) ? -1 : we_ws_bytes(in_dim, n_rows);
}

static int wide_epoch(const rai_mlp_wide_desc* desc, float* params, float* exp_avg, float* exp_avg_sq, int64_t P,
                      const float* obs, const void* actions, const float* old_logp, const float* old_values,
                      const float* advantages, const float* returns, int64_t n_rows, int32_t batch_size,
                      const float* moments, int32_t world, int32_t rank, void* const* peers, int64_t step_base,
                      const rai_ppo_hparams* hp, const rai_optim_hparams* ohp, rai_train_state* state, float* stats,
                      int32_t max_stats, float* norms, int32_t max_norms, void* workspace, int64_t workspace_bytes,
                      void* stream) {
  if (!desc || !params || !exp_avg || !exp_avg_sq || !obs || !actions || !old_logp || !old_values || !advantages ||
      !returns || !hp || !ohp || !state || !workspace)
    return RAI_E_NULLPTR;
  if (n_rows < 2 || batch_size < 2 || batch_size > WE_B) return RAI_E_SHAPE;
  if (desc->in_dim < 1 || desc->in_dim > WE_INMAX) return RAI_E_UNSUPPORTED;
  if (workspace_bytes < we_ws_bytes(desc->in_dim, n_rows)) return RAI_E_WORKSPACE;
  if (!moments && n_rows % batch_size == 1) return RAI_E_SHAPE;  // a 1-row minibatch has no unbiased std
  const int H = desc->hidden;
  if (H < WE_SL || H > WE_HMAX || H % WE_SL != 0) return RAI_E_UNSUPPORTED;
  if (desc->in_dim < 1 || desc->in_dim > WE_INMAX || desc->out_pi < 1 || desc->out_pi > WE_OUTM)
    return RAI_E_UNSUPPORTED;
  if (desc->head != 0 && desc->head != 1) return RAI_E_MODE;
  if (desc->head == 1 && !desc->log_std) return RAI_E_NULLPTR;
  if (desc->accumulate) return RAI_E_UNSUPPORTED;
  // the per-row records are read through one buffer resource (32-bit byte bound)
  if (n_rows * we_rec_floats(desc->in_dim) * 4 >= (1LL << 31)) return RAI_E_UNSUPPORTED;
  for (int n = 0; n < 2; ++n)
    for (int i = 0; i < 6; ++i) {
      if (!desc->w[n][i]) return RAI_E_NULLPTR;
      if (desc->w[n][i] < params || desc->w[n][i] >= params + P) return RAI_E_SHAPE;  // views of the flat buffer
    }
  if (desc->head == 1 && (desc->log_std < params || desc->log_std >= params + P)) return RAI_E_SHAPE;
  WeArgs a{};
  a.d = *desc;
  a.params = params;
  a.exp_avg = exp_avg;
  a.exp_avg_sq = exp_avg_sq;
  a.rec = reinterpret_cast<const float*>(static_cast<unsigned char*>(workspace) + WE_REC_OFF);
  a.n_rows = n_rows;
  a.batch = batch_size;
  a.hp = hp;
  a.ohp = ohp;
  a.state = state;
  a.stats = stats;
  a.max_stats = max_stats;
  a.norms = norms;
  a.max_norms = max_norms;
  a.ws = static_cast<unsigned char*>(workspace);
  a.world = world;
  a.xrank = rank;
  a.xpeers = peers;
  a.xbase = step_base;
  hipStream_t s = rai_stream(stream);
  // monotonic counters and granule tags start at 0 (tags are step + 1 >= 1)
  const hipError_t e = hipMemsetAsync(workspace, 0, WE_STATE_BYTES, s);
  if (e != hipSuccess) return (int)e;
  const int64_t nmb = (n_rows + batch_size - 1) / batch_size;
  hipLaunchKernelGGL(we_pack_kernel, dim3((unsigned)((nmb + 3) / 4)), dim3(256), 0, s, obs, actions, old_logp, old_values,
                     advantages, returns, n_rows, (int)batch_size, desc->in_dim, desc->out_pi, desc->head, hp, moments,
                     const_cast<float*>(a.rec));
  RAI_LAUNCH_CHECK();
  const dim3 grid(8 * (H / WE_SL));
  if (desc->head == 1) hipLaunchKernelGGL(mlp_wide_epoch_kernel<1>, grid, dim3(WE_NT), 0, s, a);
  else hipLaunchKernelGGL(mlp_wide_epoch_kernel<0>, grid, dim3(WE_NT), 0, s, a);
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}

extern "C" int rai_mlp_wide_epoch(const rai_mlp_wide_desc* desc, float* params, float* exp_avg, float* exp_avg_sq,
                                  int64_t P, const float* obs, const void* actions, const float* old_logp,
                                  const float* old_values, const float* advantages, const float* returns,
                                  int64_t n_rows, int32_t batch_size, const rai_ppo_hparams* hp,
                                  const rai_optim_hparams* ohp, rai_train_state* state, float* stats,
                                  int32_t max_stats, float* norms, int32_t max_norms, void* workspace,
                                  int64_t workspace_bytes, void* stream) {
  return wide_epoch(desc, params, exp_avg, exp_avg_sq, P, obs, actions, old_logp, old_values, advantages, returns,
                    n_rows, batch_size, nullptr, 1, 0, nullptr, 0, hp, ohp, state, stats, max_stats, norms, max_norms,
                    workspace, workspace_bytes, stream);
}

extern "C" int rai_mlp_wide_epoch_xdp(const rai_mlp_wide_desc* desc, float* params, float* exp_avg, float* exp_avg_sq,
                                      int64_t P, const float* obs, const void* actions, const float* old_logp,
                                      const float* old_values, const float* advantages, const float* returns,
                                      int64_t n_rows, int32_t batch_size, const float* moments, int32_t world,
                                      int32_t rank, void* const* peers, int64_t step_base, const rai_ppo_hparams* hp,
                                      const rai_optim_hparams* ohp, rai_train_state* state, float* stats,
                                      int32_t max_stats, float* norms, int32_t max_norms, void* workspace,
                                      int64_t workspace_bytes, void* stream) {
  if (world < 2 || world > 8 || rank < 0 || rank >= world || step_base < 0) return RAI_E_SHAPE;
  if (!peers || !moments) return RAI_E_NULLPTR;
  return wide_epoch(desc, params, exp_avg, exp_avg_sq, P, obs, actions, old_logp, old_values, advantages, returns,
                    n_rows, batch_size, moments, world, rank, peers, step_base, hp, ohp, state, stats, max_stats, norms,
                    max_norms, workspace, workspace_bytes, stream);
}
