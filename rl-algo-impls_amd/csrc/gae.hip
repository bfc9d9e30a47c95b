// GAE reverse scan + fused returns for gfx950.
//
// Restates rl_algo_impls/shared/gae.py:97-124 (compute_advantages) and
// rl_algo_impls/rollout/vec_rollout.py:88 (returns = advantages + values).
//
// Layout in HBM: rewards/values/adv/returns (T, C) fp32 with C = N*K columns,
// episode_starts (T, N) u8.  A 512-thread block owns COLS consecutive columns (64: one
// wave-wide coalesced 256-B row segment per load; 16 when C is small, so that the grid still
// has a block per CU — at C2's 4096 columns 256 blocks instead of 64: 9.4 -> 5.9 us) and walks
// T backwards in 64-row tiles:
//   (1) all 8 waves hold 8 rows each in registers and write the carry-independent
//       part delta_t (+ next_nonterminal) to LDS,
//   (2) wave 0 runs the serial carry recurrence (two dependent FP64 ops per row,
//       operands batched out of LDS 4 rows at a time) while the NEXT tile's loads,
//       issued one tile ahead (two tiles in flight from the start), are arriving,
//   (3) every wave stores its rows of adv and returns (= adv + V, from registers).
// So per tile the exposed latency is one HBM round trip shared by all 64 rows.
// Exact mode keeps the reference's numpy precision sequence bit for bit:
//   t1    = fp32(fp32(gamma) * V_next)          (gamma Python float; fp64 if ndarray)
//   delta = (f64(r_t) + f64(t1) * nn) - f64(V_t)
//   carry = delta + ((gamma*lambda)_f64 * nn) * carry      (fp64 carry)
//   adv_t = fp32(carry);  ret_t = adv_t + V_t (fp32)
// FP contraction is disabled for this file (-ffp-contract=off + pragma) so no
// multiply-add is fused differently from numpy.
#include "common.h"

#include <cstdlib>
#include <type_traits>

#pragma clang fp contract(off)

namespace {

#ifndef GAE_DIAG
#define GAE_DIAG 0  // diagnostic builds only (tools/gae_diag.hip): 1 no chain, 2 no stores, 4 no prefetch,
                    // 8 phase stamps of block 0 wave 0 into gae_stamps[]
#endif
#if GAE_DIAG & 8
__device__ long long gae_stamps[8];
#define GSTAMP(i) do { if (blockIdx.x == 0 && threadIdx.x == 0) { long long t_ = clock64(); gae_stamps[i] += t_ - t_last; t_last = t_; } } while (0)
#else
#define GSTAMP(i) do { } while (0)
#endif

constexpr int GAE_WAVES = 8;   // 512 threads
constexpr int GAE_TT = 64;     // rows per tile
constexpr int RPW = GAE_TT / GAE_WAVES;  // rows per wave per tile
// COLS columns per block: 64 (one wave-wide 256-B row segment per load) when there are enough
// columns to fill the chip; 32 / 16 at smaller N (C2: 4096 columns are 64 blocks at 64 but 256 at
// 16), a wave then covering 64 / COLS rows per load instruction.

struct GaeArgs {
  const float* rewards;
  const float* values;
  const uint8_t* es;
  const uint8_t* next_es;
  const float* next_values;
  float* adv;
  float* ret;
  int64_t T, N, C;
  int32_t K;
  int32_t gamma_is_vector;
  double gamma[RAI_MAX_K];
  double gl[RAI_MAX_K];
  float gamma32[RAI_MAX_K];
  float gl32[RAI_MAX_K];
};

template <typename Acc>
__device__ __forceinline__ Acc gae_delta(float r, float v, float vn, uint8_t esn, bool gvec,
                                         float g32, double g64);

template <>
__device__ __forceinline__ double gae_delta<double>(float r, float v, float vn, uint8_t esn,
                                                    bool gvec, float g32, double g64) {
  const double nn = 1.0 - (double)(esn != 0);
  double t1;
  if (gvec) {
    t1 = g64 * (double)vn;
  } else {
    const float t1f = g32 * vn;
    t1 = (double)t1f;
  }
  return ((double)r + t1 * nn) - (double)v;
}

template <>
__device__ __forceinline__ float gae_delta<float>(float r, float v, float vn, uint8_t esn,
                                                  bool /*gvec*/, float g32, double /*g64*/) {
  const float nn = esn ? 0.0f : 1.0f;
  return (r + (g32 * vn) * nn) - v;
}

struct Rows {
  float r[RPW], v[RPW], vn[RPW];
  uint8_t e[RPW];
};

template <typename Acc, int COLS>
__global__ __launch_bounds__(GAE_WAVES * 64) void gae_kernel(const GaeArgs a) {
  __shared__ Acc delta_s[GAE_TT][COLS];  // delta_t, overwritten in place by the carry
  // (gamma*lambda) * next_nonterminal per row, formed as the select nn ? gl : 0 (exactly the product,
  // nn in {0, 1}).  The 64-column blocks (large N) keep nn as a byte: 36 KB of LDS instead of 64 KB,
  // four blocks per CU instead of two (512 x 262144 x 3: 1,382 -> 1,304 us).  The narrow blocks (small
  // N, chain-latency bound) keep the Acc coefficient, read in the chain without a select (C2 shape:
  // 6.2 us, against 7.2 with the byte and select on the chain's operand path).
  using CoefT = typename std::conditional<COLS == 64, uint8_t, Acc>::type;
  __shared__ CoefT coef_s[GAE_TT][COLS];
  constexpr int LPR = 64 / COLS;          // rows one wave instruction covers

  const int lane64 = threadIdx.x & 63;
  const int lane = lane64 % COLS;         // column within the block
  const int sub = lane64 / COLS;          // row within the instruction's row group
  // wave index made provably wave-uniform: row indices/addresses then live in SGPRs
  // (scalar base + per-lane column offset) instead of one 64-bit VGPR pair per row.
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // XCD-aware column groups: the dispatcher deals blocks round-robin over the 8 XCDs (block b ->
  // XCD b % 8), so with the identity mapping the COLS-wide segments sharing one 128-B line of
  // r / V / adv (and the 8-16 segments sharing a line of the u8 starts) land on different XCDs,
  // each fetching the whole line into its own L2.  Remapped, XCD x owns a contiguous run of
  // column groups and every line is fetched once.
  const int nb = (int)gridDim.x, b = (int)blockIdx.x;
  const int grp = (nb % 8 == 0) ? (b % 8) * (nb / 8) + b / 8 : b;
  const int64_t c = (int64_t)grp * COLS + lane;
  const bool valid = c < a.C;
  const int64_t cc = valid ? c : 0;
  const int64_t n = cc / a.K;
  const int k = (int)(cc - n * a.K);
  const bool gvec = a.gamma_is_vector != 0;
  const float g32 = a.gamma32[k];
  const double g64 = a.gamma[k];
  const Acc gl = (sizeof(Acc) == 8) ? (Acc)a.gl[k] : (Acc)a.gl32[k];
  auto put_coef = [&](int r, uint8_t e) {
    if constexpr (COLS == 64) coef_s[r][lane] = e ? 0 : 1;
    else coef_s[r][lane] = e ? (Acc)0 : gl;
  };
  auto get_coef = [&](int r) -> Acc {
    if constexpr (COLS == 64) return coef_s[r][lane] ? gl : (Acc)0;
    else return coef_s[r][lane];
  };
  const int64_t T = a.T;
  const int ntiles = (int)((T + GAE_TT - 1) / GAE_TT);

  // Kernel arguments copied to locals once (they live in SGPRs; re-reading the large
  // by-value struct from the kernarg segment in every row branch cost a scalar-load wait
  // per row).  Loads are branch-free: clamped row index + pointer select, masked after.
  const float* __restrict__ rewards = a.rewards;
  const float* __restrict__ values = a.values;
  const uint8_t* __restrict__ es = a.es;
  const uint8_t* __restrict__ next_es = a.next_es;
  const float* __restrict__ next_values = a.next_values;
  const int64_t C = a.C, N = a.N;
  auto load = [&](Rows& R, int tile) {
    const int64_t lo = T - (int64_t)(tile + 1) * GAE_TT;
#pragma unroll
    for (int j = 0; j < RPW / LPR; ++j) {
      const int64_t t = lo + wave * RPW + j * LPR + sub;
      const int64_t tc = t < 0 ? 0 : t;
      const bool last = tc == T - 1;
      const float* vn_p = last ? next_values + cc : values + (tc + 1) * C + cc;
      const uint8_t* e_p = last ? next_es + n : es + (tc + 1) * N + n;
      const bool ok = t >= 0;
      const float r = rewards[tc * C + cc];
      const float v = values[tc * C + cc];
      const float vn = *vn_p;
      const uint8_t e = *e_p;
      R.r[j] = ok ? r : 0.f;
      R.v[j] = ok ? v : 0.f;
      R.vn[j] = ok ? vn : 0.f;
      R.e[j] = ok ? e : 0;
    }
  };

  float* __restrict__ adv_out = a.adv;
  float* __restrict__ ret_out = a.ret;
  Rows cur, nxt;
#if GAE_DIAG & 8
  long long t_last = clock64();
#endif
  // two tiles in flight from the start: tile 1's loads are not left waiting behind tile 0's
  // round trip (at C2's T = 128 that is every load of the launch up front)
  load(cur, 0);
  if (!(GAE_DIAG & 4) && ntiles > 1) load(nxt, 1);
  Acc carry = (Acc)0;
  for (int tile = 0; tile < ntiles; ++tile) {
    const int64_t lo = T - (int64_t)(tile + 1) * GAE_TT;
    // (1) carry-independent part of every row -> LDS
#pragma unroll
    for (int j = 0; j < RPW / LPR; ++j) {
      const int lr = wave * RPW + j * LPR + sub;
      delta_s[lr][lane] = gae_delta<Acc>(cur.r[j], cur.v[j], cur.vn[j], cur.e[j], gvec, g32, g64);
      put_coef(lr, cur.e[j]);
    }
    GSTAMP(0);
    lds_barrier();
    GSTAMP(1);
    // (2) wave 0 runs the serial recurrence while the next tile's loads are in flight
    if (!(GAE_DIAG & 1) && wave == 0 && sub == 0) {
      // The only serial work: carry = delta + coef*carry (two dependent FP64 ops per row),
      // operands batched out of LDS, carries written back in place.  Rows with t < 0 (only in
      // the last-processed partial tile) lie below every valid row and are never stored.
      constexpr int QB = 4;  // rows per LDS batch; batch h-1 is read while batch h is chained
      Acc d[QB], cf[QB], dn[QB], cfn[QB];
#pragma unroll
      for (int q = 0; q < QB; ++q) {
        d[q] = delta_s[GAE_TT - QB + q][lane];
        cf[q] = get_coef(GAE_TT - QB + q);
      }
#pragma unroll
      for (int h = GAE_TT / QB - 1; h >= 0; --h) {
        if (h > 0) {
#pragma unroll
          for (int q = 0; q < QB; ++q) {
            dn[q] = delta_s[(h - 1) * QB + q][lane];
            cfn[q] = get_coef((h - 1) * QB + q);
          }
        }
#pragma unroll
        for (int q = QB - 1; q >= 0; --q) {
          carry = d[q] + cf[q] * carry;
          d[q] = carry;
        }
#pragma unroll
        for (int q = 0; q < QB; ++q) delta_s[h * QB + q][lane] = d[q];
        if (h > 0) {
#pragma unroll
          for (int q = 0; q < QB; ++q) {
            d[q] = dn[q];
            cf[q] = cfn[q];
          }
        }
      }
    }
    GSTAMP(2);
    lds_barrier();
    GSTAMP(3);
    // (3) every wave stores its rows: adv and returns = adv + V (fp32), coalesced 256-B rows
#pragma unroll
    for (int j = 0; j < RPW / LPR; ++j) {
      const int lr = wave * RPW + j * LPR + sub;
      const int64_t t = lo + lr;
      if (!(GAE_DIAG & 2) && t >= 0 && valid) {
        const float adv = (float)delta_s[lr][lane];
        adv_out[t * C + c] = adv;
        if (ret_out) ret_out[t * C + c] = adv + cur.v[j];
      }
    }
    GSTAMP(4);
    if (!(GAE_DIAG & 4) && tile + 1 < ntiles) {
      cur = nxt;
      if (tile + 2 < ntiles) load(nxt, tile + 2);
    }
    GSTAMP(5);
  }
}

// Bandwidth regime (C >= GAE_STREAM_MIN_C columns): one thread owns 4 consecutive columns and walks
// T backwards on its own -- 16-B loads of r and V and 16-B stores of adv and returns (the tiled
// kernel above moves 4 B per lane per instruction), four independent carry chains per lane, and no
// LDS or workgroup barrier.  Rows are processed in chunks of D with the next chunk's loads in
// flight.  Per column the arithmetic and its order are the tiled kernel's (gae_delta, the select
// coefficient, the fp64 carry), so exact mode stays bit-identical to the reference.
constexpr int GAE_STREAM_NT = 256;
constexpr int64_t GAE_STREAM_MIN_C = 1LL << 18;

template <typename Acc, int D, bool K1, int NT, bool NTM = false>
__global__ __launch_bounds__(NT) void gae_stream_kernel(const GaeArgs a) {
  typedef float f4v __attribute__((ext_vector_type(4)));
  const int64_t C = a.C, N = a.N, T = a.T;
  const int64_t c0 = 4 * ((int64_t)blockIdx.x * NT + threadIdx.x);
  if (c0 >= C) return;
  const int K = a.K;
  const bool gvec = a.gamma_is_vector != 0;
  float g32[4];
  double g64[4];
  Acc gl[4];
  int64_t env[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t c = c0 + i;
    env[i] = K1 ? c : c / K;
    const int k = K1 ? 0 : (int)(c - env[i] * K);
    g32[i] = a.gamma32[k];
    g64[i] = a.gamma[k];
    gl[i] = (sizeof(Acc) == 8) ? (Acc)a.gl[k] : (Acc)a.gl32[k];
  }
  const float* __restrict__ rewards = a.rewards;
  const float* __restrict__ values = a.values;
  const uint8_t* __restrict__ es = a.es;
  auto load_e = [&](const uint8_t* row, uint8_t (&e)[4]) {
    if (K1) {
      const uint32_t w = *reinterpret_cast<const uint32_t*>(row + c0);
#pragma unroll
      for (int i = 0; i < 4; ++i) e[i] = (uint8_t)(w >> (8 * i));
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) e[i] = row[env[i]];
    }
  };
  f4v vprev = *reinterpret_cast<const f4v*>(a.next_values + c0);
  uint8_t eprev[4];
  load_e(a.next_es, eprev);
  Acc carry[4] = {(Acc)0, (Acc)0, (Acc)0, (Acc)0};
  struct Chunk {
    f4v r[D], v[D];
    uint8_t e[D][4];
  };
  auto load_chunk = [&](Chunk& ch, int64_t top) {  // rows top, top - 1, ..., clamped at 0
#pragma unroll
    for (int i = 0; i < D; ++i) {
      const int64_t t = top - i < 0 ? 0 : top - i;
      // NTM: the streams (read once, written once, each far larger than L2) carry the nontemporal
      // hint; the values are the same either way
      if (NTM) {
        ch.r[i] = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(rewards + t * C + c0));
        ch.v[i] = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(values + t * C + c0));
      } else {
        ch.r[i] = *reinterpret_cast<const f4v*>(rewards + t * C + c0);
        ch.v[i] = *reinterpret_cast<const f4v*>(values + t * C + c0);
      }
      load_e(es + t * N, ch.e[i]);
    }
  };
  Chunk cur, nxt;
  load_chunk(cur, T - 1);
  const int64_t nch = (T + D - 1) / D;
  for (int64_t ch = 0; ch < nch; ++ch) {
    const int64_t top = T - 1 - ch * D;
    if (ch + 1 < nch) load_chunk(nxt, top - D);
#pragma unroll
    for (int i = 0; i < D; ++i) {
      const int64_t t = top - i;
      if (t < 0) break;
      f4v adv4, ret4;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const Acc dl = gae_delta<Acc>(cur.r[i][q], cur.v[i][q], vprev[q], eprev[q], gvec, g32[q], g64[q]);
        const Acc cf = eprev[q] ? (Acc)0 : gl[q];
        carry[q] = dl + cf * carry[q];
        adv4[q] = (float)carry[q];
        ret4[q] = adv4[q] + cur.v[i][q];
      }
      if (NTM) {
        __builtin_nontemporal_store(adv4, reinterpret_cast<f4v*>(a.adv + t * C + c0));
        if (a.ret) __builtin_nontemporal_store(ret4, reinterpret_cast<f4v*>(a.ret + t * C + c0));
      } else {
        *reinterpret_cast<f4v*>(a.adv + t * C + c0) = adv4;
        if (a.ret) *reinterpret_cast<f4v*>(a.ret + t * C + c0) = ret4;
      }
      vprev = cur.v[i];
#pragma unroll
      for (int q = 0; q < 4; ++q) eprev[q] = cur.e[i][q];
    }
    cur = nxt;
  }
}

// Fast mode (RAI_GAE_FAST, fp32) at latency-bound shapes: a chunked affine
// scan over T instead of T serial steps per column.  Row t's step is the affine map
// x -> delta_t + c_t x (c_t = gamma*lambda*next_nonterminal); a 512-thread block owns COLS columns and
// cuts T into P = 512 / COLS segments of L <= GAE_SCAN_LMAX rows, one thread per (segment, column):
//   (1) each thread loads its L rows, forms delta_t / c_t (gae_delta<float>: the serial fast mode's
//       per-row arithmetic) and composes its segment's map (D, Cc) bottom-up, to LDS;
//   (2) the carry entering segment s is the composition of the segments above it applied to 0
//       (at most P - 1 dependent multiply-adds, operands from LDS);
//   (3) each thread re-runs its rows from that carry (the serial chain's own operations) and stores
//       adv and returns = adv + V.
// The dependent chain is 2 L + P steps instead of T (C2, T = 128 at 4096 columns: 4 + 32 + 4).  Only
// the grouping of the fp32 chain differs from the serial fast mode; the tolerance is fast mode's
// (tests/test_gpu_kernels.py: rtol 1e-5 against the exact oracle).
constexpr int GAE_SCAN_LMAX = 32;

template <int COLS, int LM>
__global__ __launch_bounds__(512) void gae_scan_kernel(const GaeArgs a) {
  constexpr int P = 512 / COLS;
  __shared__ float seg_d[P][COLS], seg_c[P][COLS];
  const int tid = threadIdx.x;
  const int lane = tid % COLS;
  const int s = tid / COLS;  // segment
  // XCD-aware column groups (as gae_kernel)
  const int nb = (int)gridDim.x, b = (int)blockIdx.x;
  const int grp = (nb % 8 == 0) ? (b % 8) * (nb / 8) + b / 8 : b;
  const int64_t c = (int64_t)grp * COLS + lane;
  const int64_t C = a.C, N = a.N, T = a.T;
  const bool valid = c < C;
  const int64_t cc = valid ? c : 0;
  const int64_t n = cc / a.K;
  const int k = (int)(cc - n * a.K);
  const float g32 = a.gamma32[k], gl = a.gl32[k];
  const int64_t L = (T + P - 1) / P;
  const int64_t t_lo = (int64_t)s * L;
  const int64_t t_hi = t_lo + L < T ? t_lo + L : T;  // rows [t_lo, t_hi); empty when t_lo >= T
  float d[LM], cf[LM], vv[LM];
#pragma unroll
  for (int i = 0; i < LM; ++i) {
    const int64_t t = t_lo + i;
    d[i] = 0.f;
    cf[i] = 1.f;
    vv[i] = 0.f;
    if (t < t_hi) {
      const bool last = t == T - 1;
      const float r = a.rewards[t * C + cc];
      const float v = a.values[t * C + cc];
      const float vn = last ? a.next_values[cc] : a.values[(t + 1) * C + cc];
      const uint8_t e = last ? a.next_es[n] : a.es[(t + 1) * N + n];
      d[i] = gae_delta<float>(r, v, vn, e, false, g32, 0.0);
      cf[i] = e ? 0.f : gl;
      vv[i] = v;
    }
  }
  // (1) the segment's map, composed from its last row upwards: x -> D + Cc x
  float D = 0.f, Cc = 1.f;
#pragma unroll
  for (int i = LM - 1; i >= 0; --i) {
    if (t_lo + i < t_hi) {
      D = d[i] + cf[i] * D;
      Cc = cf[i] * Cc;
    }
  }
  seg_d[s][lane] = D;
  seg_c[s][lane] = Cc;
  __syncthreads();
  // (2) carry entering the segment from below it in time order (rows >= t_hi)
  float x = 0.f;
  for (int q = P - 1; q > s; --q) x = seg_d[q][lane] + seg_c[q][lane] * x;
  // (3) the segment's rows from that carry
#pragma unroll
  for (int i = LM - 1; i >= 0; --i) {
    const int64_t t = t_lo + i;
    if (t < t_hi) {
      x = d[i] + cf[i] * x;
      if (valid) {
        a.adv[t * C + c] = x;
        if (a.ret) a.ret[t * C + c] = x + vv[i];
      }
    }
  }
}

}  // namespace

extern "C" int rai_gae(const float* rewards, const float* values, const uint8_t* episode_starts,
                       const uint8_t* next_episode_starts, const float* next_values, int64_t T,
                       int64_t N, int32_t K, const double* gamma, const double* gae_lambda,
                       int32_t gamma_is_vector, int32_t mode, float* adv_out, float* returns_out,
                       void* stream) {
  if (T < 0 || N < 0 || K < 1) return RAI_E_SHAPE;
  if (K > RAI_MAX_K) return RAI_E_TOO_MANY_COLUMNS;
  if (mode != RAI_GAE_EXACT && mode != RAI_GAE_FAST) return RAI_E_MODE;
  if (T == 0 || N == 0) return RAI_OK;
  if (!rewards || !values || !episode_starts || !next_episode_starts || !next_values ||
      !gamma || !gae_lambda || !adv_out)
    return RAI_E_NULLPTR;
  GaeArgs a;
  a.rewards = rewards;
  a.values = values;
  a.es = episode_starts;
  a.next_es = next_episode_starts;
  a.next_values = next_values;
  a.adv = adv_out;
  a.ret = returns_out;
  a.T = T;
  a.N = N;
  a.K = K;
  a.C = N * (int64_t)K;
  a.gamma_is_vector = gamma_is_vector;
  for (int k = 0; k < RAI_MAX_K; ++k) {
    const int kk = k < K ? k : 0;
    a.gamma[k] = gamma[kk];
    a.gl[k] = gamma[kk] * gae_lambda[kk];  // Python/numpy f64 product
    a.gamma32[k] = (float)gamma[kk];
    a.gl32[k] = (float)a.gl[k];
  }
  hipStream_t st = rai_stream(stream);
  // bandwidth regime: the 4-columns-per-lane streaming kernel (16-B accesses need C % 4 == 0 and
  // 16-B aligned float buffers; the K = 1 start bytes are read 4 at a time: N % 4 == 0)
  const bool aligned16 = ((uintptr_t)rewards | (uintptr_t)values | (uintptr_t)next_values | (uintptr_t)adv_out |
                          (uintptr_t)(returns_out ? returns_out : adv_out)) % 16 == 0;
  const char* sf = getenv("RAI_GAE_STREAM");  // diagnostics: 0 forces the tiled kernel
  if (a.C >= GAE_STREAM_MIN_C && a.C % 4 == 0 && aligned16 && !(sf && sf[0] == '0')) {
    const bool k1 = K == 1 && N % 4 == 0 && (uintptr_t)episode_starts % 4 == 0 &&
                    (uintptr_t)next_episode_starts % 4 == 0;
    // diagnostics: rows in flight per chunk (RAI_GAE_STREAM_D = 4 or 8) and threads per block
    // (RAI_GAE_STREAM_NT = 256 or 1024: 4 KB or 16 KB of each row per block)
    const char* sd = getenv("RAI_GAE_STREAM_D");
    const char* sn = getenv("RAI_GAE_STREAM_NT");
    const bool d4 = sd && sd[0] == '4';
    // default: K = 1 -> 1024 threads (16 KB of every row per block; 128 x 2^20: 446-449 us against
    // 455-482 at 256 threads, profiles/r3b_gae_bench.txt); K > 1 -> 256 threads, 8 rows in flight
    // (the 1024-thread form spills there)
    int nt = k1 ? 1024 : GAE_STREAM_NT;
    if (sn && atoi(sn) == 256) nt = 256;
    if (sn && atoi(sn) == 512) nt = 512;
    if (sn && atoi(sn) == 1024 && k1) nt = 1024;
    const dim3 grid((unsigned)((a.C / 4 + nt - 1) / nt)), block(nt);
#define RAI_GAE_STREAM_LAUNCH(ACC, DD, NTT)                                                          \
  do {                                                                                               \
    if (k1) hipLaunchKernelGGL((gae_stream_kernel<ACC, DD, true, NTT>), grid, block, 0, st, a);     \
    else hipLaunchKernelGGL((gae_stream_kernel<ACC, DD, false, NTT>), grid, block, 0, st, a);       \
  } while (0)
    // K = 1, 1024 threads: nontemporal loads / stores (the streams are read or written once, each far
    // larger than L2): 128 x 2^20 at 5.63 TB/s against 4.81 with the default policy
    // (profiles/r3h_gae_bench.txt); RAI_GAE_NT=0 turns it off (diagnostics, tools/gae_bench.py)
    const char* ntm = getenv("RAI_GAE_NT");
    if (nt == 1024 && !(ntm && atoi(ntm) == 0)) {
      if (mode == RAI_GAE_EXACT) hipLaunchKernelGGL((gae_stream_kernel<double, 4, true, 1024, true>), grid, block, 0, st, a);
      else hipLaunchKernelGGL((gae_stream_kernel<float, 4, true, 1024, true>), grid, block, 0, st, a);
    } else if (nt == 1024) {  // 128 VGPRs per lane at 4 waves per SIMD: 4 rows in flight
      if (mode == RAI_GAE_EXACT) hipLaunchKernelGGL((gae_stream_kernel<double, 4, true, 1024>), grid, block, 0, st, a);
      else hipLaunchKernelGGL((gae_stream_kernel<float, 4, true, 1024>), grid, block, 0, st, a);
    } else if (nt == 512) {  // 256 VGPRs per lane at 2 waves per SIMD: 8 rows in flight
      if (mode == RAI_GAE_EXACT) RAI_GAE_STREAM_LAUNCH(double, 8, 512);
      else RAI_GAE_STREAM_LAUNCH(float, 8, 512);
    } else if (mode == RAI_GAE_EXACT) {
      if (d4) RAI_GAE_STREAM_LAUNCH(double, 4, 256);
      else RAI_GAE_STREAM_LAUNCH(double, 8, 256);
    } else {
      if (d4) RAI_GAE_STREAM_LAUNCH(float, 4, 256);
      else RAI_GAE_STREAM_LAUNCH(float, 8, 256);
    }
#undef RAI_GAE_STREAM_LAUNCH
    RAI_LAUNCH_CHECK();
    return RAI_OK;
  }
  // fast mode: the chunked affine scan where T fits its segments (RAI_GAE_SCAN=0: the serial fp32 chain)
  const char* sc = getenv("RAI_GAE_SCAN");
  if (mode == RAI_GAE_FAST && !(sc && sc[0] == '0')) {
    // columns per block: the widest of 64 / 32 / 16 that still gives >= 256 blocks; P = 512 / cols segments
    const int scols = a.C >= 256LL * 64 ? 64 : (a.C >= 256LL * 32 ? 32 : 16);
    const int64_t L = (T + 512 / scols - 1) / (512 / scols);  // rows per segment
    if (L <= GAE_SCAN_LMAX) {
      const dim3 grid((unsigned)((a.C + scols - 1) / scols)), block(512);
#define RAI_GAE_SCAN_LAUNCH(CO)                                                                    \
  do {                                                                                             \
    if (L <= 8) hipLaunchKernelGGL((gae_scan_kernel<CO, 8>), grid, block, 0, st, a);              \
    else hipLaunchKernelGGL((gae_scan_kernel<CO, GAE_SCAN_LMAX>), grid, block, 0, st, a);         \
  } while (0)
      if (scols == 64) RAI_GAE_SCAN_LAUNCH(64);
      else if (scols == 32) RAI_GAE_SCAN_LAUNCH(32);
      else RAI_GAE_SCAN_LAUNCH(16);
#undef RAI_GAE_SCAN_LAUNCH
      RAI_LAUNCH_CHECK();
      return RAI_OK;
    }
  }
  // columns per block: the widest of 64 / 32 / 16 that still gives >= 256 blocks (one per CU)
  int cols = 64;
  if (const char* f = getenv("RAI_GAE_COLS")) cols = atoi(f);  // diagnostics (tools/gae_bench.py)
  else if (a.C < 256LL * 64) cols = a.C < 256LL * 32 ? 16 : 32;
  if (cols != 16 && cols != 32) cols = 64;
  const int64_t blocks = (a.C + cols - 1) / cols;
  const dim3 grid((unsigned)blocks), block(GAE_WAVES * 64);
  if (mode == RAI_GAE_EXACT) {
    if (cols == 16) hipLaunchKernelGGL((gae_kernel<double, 16>), grid, block, 0, st, a);
    else if (cols == 32) hipLaunchKernelGGL((gae_kernel<double, 32>), grid, block, 0, st, a);
    else hipLaunchKernelGGL((gae_kernel<double, 64>), grid, block, 0, st, a);
  } else {
    if (cols == 16) hipLaunchKernelGGL((gae_kernel<float, 16>), grid, block, 0, st, a);
    else if (cols == 32) hipLaunchKernelGGL((gae_kernel<float, 32>), grid, block, 0, st, a);
    else hipLaunchKernelGGL((gae_kernel<float, 64>), grid, block, 0, st, a);
  }
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}
