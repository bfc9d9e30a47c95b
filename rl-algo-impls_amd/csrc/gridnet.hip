// GridNet masked-categorical head (MicroRTS) on gfx950: fused log-prob + entropy and their
// backward, for every cell and sub-action of a minibatch in one launch each.
//
// Restates rl_algo_impls/shared/actor/gridnet.py:38-200 (GridnetDistribution.log_prob / entropy)
// over rl_algo_impls/shared/actor/categorical.py:12-54 (MaskedCategorical).  Per sample b, per cell
// c (C = H*W cells) the A = sum(nvec) logits are split into G sub-action groups (MicroRTS:
// nvec = [6, 4, 4, 4, 4, 7, 49]); group g of cell c is a categorical over its masked logits
//   zm = mask ? z : FLT_MIN_NORMAL_NEG (torch.finfo(f32).min),  l = zm - logsumexp(zm),  p = exp(l)
//   logp_g = l[a_g]  (x 0 when a ValueDependentMask gates it: actions[ref] != value)
//   H_g    = -sum_j mask_j * l_j * p_j          (the masked entropy approximation)
// and logp(b) = sum over cells and groups of logp_g, entropy(b) = sum of H_g.  A group with no
// valid action has l = 0 (torch's logsumexp of all-finfo.min rows), logp 0 and H 0.
// Backward for upstream (dL/dlogp(b), dL/dH(b)) = (gl, ge), through torch.where's zero gradient
// on masked entries:
//   dz_j = mask_j * ( gl * gate * ([j == a] - p_j)  -  ge * p_j * (l_j + H_g) )
// (closed form of autograd through logsumexp/softmax; within fp32 rounding of torch's).
//
// Layout: logits / masks / d_logits are (B, C, A) row-major (A fastest), actions (B, C, G) int64.
// One 256-thread workgroup per sample walks its cells in 64-cell tiles: the tile's 64*A logits and
// mask bytes are one contiguous span, loaded coalesced into LDS; the 64*G (cell, group) items are
// spread over the threads; the backward writes dz into the LDS tile in place and stores the span
// coalesced.  Sums over a sample's items are fixed-order block reductions (deterministic).
#include <algorithm>

#include "common.h"

namespace {

constexpr int GN_THREADS = 256;
constexpr int GN_CELLS = 64;  // cells per LDS tile
constexpr float GN_NEG = -3.4028234663852886e38f;  // torch.finfo(torch.float32).min

struct GridArgs {
  const float* logits;
  const uint8_t* mask;
  const int64_t* actions;
  int64_t* actions_out;  // sample mode
  uint64_t seed, offset;
  const float* d_logp;
  const float* d_ent;
  float* logp;
  float* ent;
  float* d_logits;
  int64_t B;
  int32_t C, A, G;
  int32_t off[RAI_GRID_MAX_G + 1];  // group g: logits [off[g], off[g+1])
  int32_t sub_ref[RAI_GRID_MAX_G];  // -1: no gate
  int32_t sub_val[RAI_GRID_MAX_G];
};

struct GroupStats {
  float lse;  // logsumexp of the masked logits (torch: max + log(sum(exp(x - max))))
  float H;    // masked entropy
  int nvalid;
};

__device__ __forceinline__ GroupStats group_stats(const float* z, const uint8_t* m, int n) {
  float mx = GN_NEG;
  int nv = 0;
  for (int j = 0; j < n; ++j) {
    const float v = m[j] ? z[j] : GN_NEG;
    mx = fmaxf(mx, v);
    nv += m[j] ? 1 : 0;
  }
  float s = 0.f;
  for (int j = 0; j < n; ++j) {
    const float v = m[j] ? z[j] : GN_NEG;
    s += expf(v - mx);
  }
  GroupStats g;
  g.lse = mx + logf(s);
  g.nvalid = nv;
  float h = 0.f;
  if (nv > 0) {
    for (int j = 0; j < n; ++j) {
      if (m[j]) {
        const float l = z[j] - g.lse;
        h -= l * expf(l);
      }
    }
  }
  g.H = h;
  return g;
}

// Stage one tile's logits and mask bytes into LDS.  The loads are issued in batches of GN_BATCH per
// thread before any LDS store: a load -> store loop waits out one HBM round trip per element
// (measured: 298 us per 64-sample rollout launch with the plain loop).
constexpr int GN_BATCH = 8;
constexpr int GN_REG = 64;  // planes up to this size are sampled from registers
__device__ __forceinline__ void load_tile(const GridArgs& a, int64_t base, int span, float* zt, uint8_t* mt,
                                          int tid) {
  for (int i0 = tid; i0 < span; i0 += GN_BATCH * GN_THREADS) {
    float zv[GN_BATCH];
    uint8_t mv[GN_BATCH];
#pragma unroll
    for (int k = 0; k < GN_BATCH; ++k) {
      const int i = min(i0 + k * GN_THREADS, span - 1);
      zv[k] = a.logits[base + i];
      mv[k] = a.mask[base + i];
    }
#pragma unroll
    for (int k = 0; k < GN_BATCH; ++k) {
      const int i = i0 + k * GN_THREADS;
      if (i < span) {
        zt[i] = zv[k];
        mt[i] = mv[k];
      }
    }
  }
}

template <bool BWD>
__global__ __launch_bounds__(GN_THREADS) void gridnet_kernel(const GridArgs a) {
  extern __shared__ float smem[];
  const int A = a.A, G = a.G, C = a.C;
  float* zt = smem;                                                     // [GN_CELLS][A]
  uint8_t* mt = reinterpret_cast<uint8_t*>(smem + GN_CELLS * A);       // [GN_CELLS][A]
  __shared__ double red[2 * (GN_THREADS / 64)];
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x;
  const float gl = BWD ? a.d_logp[b] : 0.f;
  const float ge = BWD ? a.d_ent[b] : 0.f;
  double acc_lp = 0.0, acc_h = 0.0;
  for (int c0 = 0; c0 < C; c0 += GN_CELLS) {
    const int nc = min(GN_CELLS, C - c0);
    const int64_t base = (b * C + c0) * (int64_t)A;
    const int span = nc * A;
    load_tile(a, base, span, zt, mt, tid);
    __syncthreads();
    const int items = nc * G;
    for (int it = tid; it < items; it += GN_THREADS) {
      const int cl = it / G, g = it - cl * G;
      const int o = a.off[g], n = a.off[g + 1] - o;
      float* z = zt + cl * A + o;
      const uint8_t* m = mt + cl * A + o;
      const int64_t* act = a.actions ? a.actions + (b * C + c0 + cl) * (int64_t)G : nullptr;
      const GroupStats s = group_stats(z, m, n);
      const int ag = act ? (int)act[g] : 0;
      const bool gate = !act || a.sub_ref[g] < 0 || act[a.sub_ref[g]] == (int64_t)a.sub_val[g];
      if (!BWD) {
        if (act && gate) {
          const bool ok = ag >= 0 && ag < n;
          const float za = ok ? (m[ag] ? z[ag] : GN_NEG) : 0.f;
          acc_lp += (double)(s.nvalid > 0 ? za - s.lse : 0.f);  // all-masked: l = 0
        }
        acc_h += (double)s.H;
      } else {
        for (int j = 0; j < n; ++j) {
          float d = 0.f;
          if (m[j]) {
            const float l = z[j] - s.lse;
            const float p = expf(l);
            if (act && gate) d = gl * ((j == ag ? 1.f : 0.f) - p);
            d -= ge * p * (l + s.H);
          }
          z[j] = d;  // the item owns these LDS slots: dz overwrites its logits in place
        }
      }
    }
    __syncthreads();
    if (BWD) {
      for (int i = tid; i < span; i += GN_THREADS) a.d_logits[base + i] = zt[i];
      __syncthreads();
    }
  }
  if (!BWD) {
    const int lane = tid & 63, w = tid >> 6;
    acc_lp = wave_sum(acc_lp);
    acc_h = wave_sum(acc_h);
    if (lane == 0) {
      red[w] = acc_lp;
      red[GN_THREADS / 64 + w] = acc_h;
    }
    __syncthreads();
    if (tid == 0) {
      double lp = 0.0, h = 0.0;
      for (int i = 0; i < GN_THREADS / 64; ++i) {
        lp += red[i];
        h += red[GN_THREADS / 64 + i];
      }
      if (a.logp) a.logp[b] = (float)lp;
      if (a.ent) a.ent[b] = (float)h;
    }
  }
}

// Rollout sampling (gridnet.py:195-205 sample() + log_prob): every (cell, group) draws its action
// from its masked categorical by inverse CDF on a Philox4x32-10 uniform keyed (seed; counter
// (offset, item)), item = (b * C + c) * G + g; a group with no valid action samples uniformly over
// all n (torch: equal finfo.min logits).  Then, after the tile's actions are in LDS, the log-prob of
// the sampled action under the same gating as log_prob (the ValueDependentMask reads the cell's
// other sampled planes).  One workgroup per sample, 64-cell tiles as in the forward.
__global__ __launch_bounds__(GN_THREADS) void gridnet_sample_kernel(const GridArgs a) {
  extern __shared__ float smem[];
  const int A = a.A, G = a.G, C = a.C;
  float* zt = smem;                                                     // [GN_CELLS][A]
  uint8_t* mt = reinterpret_cast<uint8_t*>(smem + GN_CELLS * A);       // [GN_CELLS][A]
  __shared__ int act_s[GN_CELLS * RAI_GRID_MAX_G];
  __shared__ float lp_s[GN_CELLS * RAI_GRID_MAX_G];  // log-prob of each drawn value (before gating)
  __shared__ double red[GN_THREADS / 64];
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x;
  double acc_lp = 0.0;
  for (int c0 = 0; c0 < C; c0 += GN_CELLS) {
    const int nc = min(GN_CELLS, C - c0);
    const int64_t base = (b * C + c0) * (int64_t)A;
    const int span = nc * A;
    load_tile(a, base, span, zt, mt, tid);
    __syncthreads();
    const int items = nc * G;
    for (int it = tid; it < items; it += GN_THREADS) {
      const int cl = it / G, g = it - cl * G;
      const int o = a.off[g], n = a.off[g + 1] - o;
      const float* z = zt + cl * A + o;
      const uint8_t* m = mt + cl * A + o;
      const uint64_t item = (uint64_t)((b * C + c0 + cl) * (int64_t)G + g);
      const Philox4 r = philox4x32_10(a.offset, item, a.seed);
      int pick;
      float lp;
      if (n <= GN_REG) {
        // the plane's masked logits in registers: one pipelined sweep of LDS reads instead of three
        // dependent sweeps (each iteration of the LDS loops below waits out an LDS round trip)
        float v[GN_REG];
        bool any = false;
#pragma unroll
        for (int j = 0; j < GN_REG; ++j) {
          const bool on = j < n && m[j];
          v[j] = on ? z[j] : GN_NEG;
          any = any || on;
        }
        float mx = GN_NEG;
#pragma unroll
        for (int j = 0; j < GN_REG; ++j)
          if (j < n) mx = fmaxf(mx, v[j]);
        float tot = 0.f;
#pragma unroll
        for (int j = 0; j < GN_REG; ++j) {
          v[j] = j < n ? expf(v[j] - mx) : 0.f;
          tot += v[j];
        }
        const float target = u01_open0(r.x) * tot;
        int last = 0;
        float cum = 0.f;
        pick = -1;
#pragma unroll
        for (int j = 0; j < GN_REG; ++j) {
          if (v[j] > 0.f) last = j;
          cum += v[j];
          if (pick < 0 && cum >= target && v[j] > 0.f) pick = j;
        }
        if (pick < 0) pick = last;  // rounding at the top of the CDF
        // log-prob exactly as group_stats + the forward kernel: lse = max + log(sum exp(x - max))
        lp = any ? (m[pick] ? z[pick] : GN_NEG) - (mx + logf(tot)) : 0.f;
      } else {
        float mx = GN_NEG;
        for (int j = 0; j < n; ++j) mx = fmaxf(mx, m[j] ? z[j] : GN_NEG);
        float tot = 0.f;
        for (int j = 0; j < n; ++j) tot += expf((m[j] ? z[j] : GN_NEG) - mx);
        const float target = u01_open0(r.x) * tot;
        int last = 0;
        float cum = 0.f;
        pick = -1;
        for (int j = 0; j < n; ++j) {
          const float pj = expf((m[j] ? z[j] : GN_NEG) - mx);
          if (pj > 0.f) last = j;
          cum += pj;
          if (pick < 0 && cum >= target && pj > 0.f) pick = j;
        }
        if (pick < 0) pick = last;  // rounding at the top of the CDF
        const GroupStats st = group_stats(z, m, n);
        lp = st.nvalid > 0 ? (m[pick] ? z[pick] : GN_NEG) - st.lse : 0.f;
      }
      act_s[cl * G + g] = pick;
      lp_s[cl * G + g] = lp;
      a.actions_out[(b * C + c0 + cl) * (int64_t)G + g] = pick;
    }
    __syncthreads();
    for (int it = tid; it < items; it += GN_THREADS) {
      const int cl = it / G, g = it - cl * G;
      const int ref = a.sub_ref[g];
      const bool gate = ref < 0 || act_s[cl * G + ref] == a.sub_val[g];
      if (gate) acc_lp += (double)lp_s[cl * G + g];
    }
    __syncthreads();
  }
  const int lane = tid & 63, w = tid >> 6;
  acc_lp = wave_sum(acc_lp);
  if (lane == 0) red[w] = acc_lp;
  __syncthreads();
  if (tid == 0) {
    double lp = 0.0;
    for (int i = 0; i < GN_THREADS / 64; ++i) lp += red[i];
    if (a.logp) a.logp[b] = (float)lp;
  }
}

int setup(GridArgs& a, const float* logits, const uint8_t* mask, const int64_t* actions, int64_t B, int32_t C,
          int32_t G, const int32_t* nvec, const int32_t* sub_ref, const int32_t* sub_val, bool need_logits = true) {
  if (B < 0 || C < 1 || G < 1) return RAI_E_SHAPE;
  if (G > RAI_GRID_MAX_G) return RAI_E_UNSUPPORTED;
  if (!nvec) return RAI_E_NULLPTR;
  a = GridArgs{};
  a.logits = logits;
  a.mask = mask;
  a.actions = actions;
  a.B = B;
  a.C = C;
  a.G = G;
  int A = 0;
  for (int g = 0; g < G; ++g) {
    if (nvec[g] < 1) return RAI_E_SHAPE;
    a.off[g] = A;
    A += nvec[g];
    const int r = sub_ref ? sub_ref[g] : -1;
    if (r >= G || r == g) return RAI_E_SHAPE;
    a.sub_ref[g] = r;
    a.sub_val[g] = sub_val && r >= 0 ? sub_val[g] : 0;
  }
  if (A > RAI_GRID_MAX_A) return RAI_E_UNSUPPORTED;
  a.off[G] = A;
  a.A = A;
  if (B > 0 && ((need_logits && !logits) || !mask)) return RAI_E_NULLPTR;
  return RAI_OK;
}

size_t smem_bytes(int A) { return (size_t)GN_CELLS * A * (sizeof(float) + 1); }

}  // namespace

extern "C" int rai_gridnet_logp_entropy(const float* logits, const uint8_t* mask, const int64_t* actions,
                                        int64_t B, int32_t C, int32_t G, const int32_t* nvec,
                                        const int32_t* sub_ref, const int32_t* sub_val, float* logp_out,
                                        float* entropy_out, void* stream) {
  GridArgs a;
  int rc = setup(a, logits, mask, actions, B, C, G, nvec, sub_ref, sub_val);
  if (rc != RAI_OK) return rc;
  if (logp_out && !actions) return RAI_E_NULLPTR;
  if (B == 0) return RAI_OK;
  a.logp = logp_out;
  a.ent = entropy_out;
  hipLaunchKernelGGL(gridnet_kernel<false>, dim3((unsigned)B), dim3(GN_THREADS), smem_bytes(a.A),
                     rai_stream(stream), a);
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}

extern "C" int rai_gridnet_backward(const float* logits, const uint8_t* mask, const int64_t* actions, int64_t B,
                                    int32_t C, int32_t G, const int32_t* nvec, const int32_t* sub_ref,
                                    const int32_t* sub_val, const float* d_logp, const float* d_entropy,
                                    float* d_logits, void* stream) {
  GridArgs a;
  int rc = setup(a, logits, mask, actions, B, C, G, nvec, sub_ref, sub_val);
  if (rc != RAI_OK) return rc;
  if (B == 0) return RAI_OK;
  if (!actions || !d_logp || !d_entropy || !d_logits) return RAI_E_NULLPTR;
  a.d_logp = d_logp;
  a.d_ent = d_entropy;
  a.d_logits = d_logits;
  hipLaunchKernelGGL(gridnet_kernel<true>, dim3((unsigned)B), dim3(GN_THREADS), smem_bytes(a.A),
                     rai_stream(stream), a);
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}

extern "C" int rai_gridnet_sample(const float* logits, const uint8_t* mask, int64_t B, int32_t C, int32_t G,
                                  const int32_t* nvec, const int32_t* sub_ref, const int32_t* sub_val,
                                  uint64_t seed, uint64_t offset, int64_t* actions_out, float* logp_out,
                                  void* stream) {
  GridArgs a;
  int rc = setup(a, logits, mask, nullptr, B, C, G, nvec, sub_ref, sub_val);
  if (rc != RAI_OK) return rc;
  if (B == 0) return RAI_OK;
  if (!actions_out) return RAI_E_NULLPTR;
  a.actions_out = actions_out;
  a.logp = logp_out;
  a.seed = seed;
  a.offset = offset;
  hipLaunchKernelGGL(gridnet_sample_kernel, dim3((unsigned)B), dim3(GN_THREADS), smem_bytes(a.A),
                     rai_stream(stream), a);
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}

// ---- Batch.num_actions (rl_algo_impls/rollout/rollout.py:158-180) ------------------------------
// HBM-bound byte work: one 256-thread workgroup per row b streams the row's C*A mask bytes through
// LDS in tiles of NA_CELLS cells (dword loads when the row is 4-B aligned), then one thread per cell
// scans its A bytes group by group.  C5: 256 cells x 78 B = 19,968 B per row, 262,144 rows.
namespace {
constexpr int NA_THREADS = 256;
constexpr int NA_CELLS = 256;

__global__ void __launch_bounds__(NA_THREADS) gridnet_num_actions_kernel(GridArgs a, int per_group, int out_bytes,
                                                                         int tile_cells, void* out) {
  extern __shared__ uint8_t na_tile[];
  __shared__ int na_part[NA_THREADS / RAI_WAVE];
  const int64_t b = blockIdx.x;
  const int A = a.A, C = a.C, G = a.G;
  const uint8_t* row = a.mask + b * (int64_t)C * A;
  const bool dw = ((reinterpret_cast<uintptr_t>(row) | (uintptr_t)((int64_t)C * A)) & 3) == 0;
  int count = 0;
  for (int c0 = 0; c0 < C; c0 += tile_cells) {
    const int nc = min(tile_cells, C - c0);
    const int nbytes = nc * A;
    const uint8_t* src = row + (int64_t)c0 * A;
    __syncthreads();
    if (dw && (nbytes & 3) == 0) {
      const uint32_t* s4 = reinterpret_cast<const uint32_t*>(src);
      uint32_t* d4 = reinterpret_cast<uint32_t*>(na_tile);
      for (int i = threadIdx.x; i < nbytes / 4; i += NA_THREADS) d4[i] = __builtin_nontemporal_load(s4 + i);
    } else {
      for (int i = threadIdx.x; i < nbytes; i += NA_THREADS) na_tile[i] = src[i];
    }
    __syncthreads();
    for (int cl = threadIdx.x; cl < nc; cl += NA_THREADS) {
      const uint8_t* m = na_tile + cl * A;
      if (!per_group) {
        int any = 0;
        for (int j = 0; j < A; ++j) any |= m[j];
        count += any != 0;
      } else {
        const int64_t* act = a.actions ? a.actions + (b * C + c0 + cl) * G : nullptr;
        for (int g = 0; g < G; ++g) {
          int any = 0;
          for (int j = a.off[g]; j < a.off[g + 1]; ++j) any |= m[j];
          const int r = a.sub_ref[g];
          const bool gate = r < 0 || act[r] == (int64_t)a.sub_val[g];
          count += (any != 0) && gate;
        }
      }
    }
  }
  // fixed-order block sum (integers: any order is exact)
  for (int o = RAI_WAVE / 2; o > 0; o >>= 1) count += __shfl_xor(count, o);
  if ((threadIdx.x & (RAI_WAVE - 1)) == 0) na_part[threadIdx.x / RAI_WAVE] = count;
  __syncthreads();
  if (threadIdx.x == 0) {
    int tot = 0;
    for (int w = 0; w < NA_THREADS / RAI_WAVE; ++w) tot += na_part[w];
    if (out_bytes == 8) static_cast<int64_t*>(out)[b] = tot;
    else static_cast<int32_t*>(out)[b] = tot;
  }
}
}  // namespace

extern "C" int rai_gridnet_num_actions(const uint8_t* mask, const int64_t* actions, int64_t B, int32_t C, int32_t G,
                                       const int32_t* nvec, const int32_t* sub_ref, const int32_t* sub_val,
                                       int32_t per_group, int32_t out_bytes, void* out, void* stream) {
  GridArgs a;
  int rc = setup(a, nullptr, mask, actions, B, C, G, nvec, per_group ? sub_ref : nullptr, sub_val, false);
  if (rc != RAI_OK) return rc;
  if (out_bytes != 4 && out_bytes != 8) return RAI_E_SHAPE;
  if (B > 0x7fffffff) return RAI_E_SHAPE;
  if (B == 0) return RAI_OK;
  if (!out) return RAI_E_NULLPTR;
  bool gated = false;
  for (int g = 0; g < G; ++g) gated |= a.sub_ref[g] >= 0;
  if (per_group && gated && !actions) return RAI_E_NULLPTR;
  // the cell tile fits the default 64 KiB of LDS beside the kernel's static words for any A <= RAI_GRID_MAX_A
  const int tile_cells = std::min(NA_CELLS, (65536 - 256) / a.A);
  hipLaunchKernelGGL(gridnet_num_actions_kernel, dim3((unsigned)B), dim3(NA_THREADS), (size_t)tile_cells * a.A,
                     rai_stream(stream), a, (int)per_group, (int)out_bytes, tile_cells, out);
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}
