// Rollout-buffer side kernels for gfx950:
//  * multi-field row gather (minibatch / epoch permutation),
//  * categorical and diagonal-Gaussian post-head sampling that writes the
//    rollout slot (action, log-prob, value) in one pass.
//
// Reference regions replaced:
//   rl_algo_impls/rollout/rollout.py:56-69      Batch.__getitem__ (fancy-index gather)
//   rl_algo_impls/rollout/vec_rollout.py:166-175 minibatches()
//   rl_algo_impls/shared/policy/actor_critic.py:306-318  step(): pi.sample(), log_prob
//   rl_algo_impls/shared/actor/categorical.py:12-54      MaskedCategorical
//   rl_algo_impls/shared/actor/gaussian.py:11-16         GaussianDistribution
//   rl_algo_impls/shared/policy/actor_critic.py:62-87    clamp_actions (Box clip)
//   rl_algo_impls/rollout/sync_step_rollout.py:193-201   slot writes
#include "common.h"

namespace {

struct GatherField {
  const uint8_t* src;
  uint8_t* dst;
  int64_t units;  // granules per row
  int32_t gran;   // 16, 4 or 1 bytes
};
struct GatherArgs {
  GatherField f[RAI_MAX_FIELDS];
  const int64_t* idx;
  int64_t n_rows;
};

__global__ __launch_bounds__(256) void gather_rows_kernel(const GatherArgs a) {
  const GatherField f = a.f[blockIdx.y];
  const int64_t total = a.n_rows * f.units;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < total; u += stride) {
    const int64_t r = u / f.units;
    const int64_t j = u - r * f.units;
    const int64_t sr = a.idx[r];
    if (f.gran == 16) {
      reinterpret_cast<uint4*>(f.dst)[u] = reinterpret_cast<const uint4*>(f.src)[sr * f.units + j];
    } else if (f.gran == 4) {
      reinterpret_cast<uint32_t*>(f.dst)[u] =
          reinterpret_cast<const uint32_t*>(f.src)[sr * f.units + j];
    } else {
      f.dst[u] = f.src[sr * f.units + j];
    }
  }
}

// Keyed permutation of [0, n) (the epoch shuffle).  A 6-round unbalanced Feistel network over the
// smallest domain 2^b >= n (b >= 2), split into a high part of h1 = b/2 bits and a low part of
// h2 = b - h1 bits whose widths swap every round; the round function is the lowbias32 integer hash of
// (low part ^ round key) masked to the high part's width, with cycle walking back into [0, n): a
// bijection for every key, computed independently per index (no sort).  Replaces the device torch.randperm (a radix sort
// of n random keys plus merge passes, ~0.27 ms per epoch at n = 524,288 on the scaled batch policy,
// where the epoch kernels fill every CU and the side-stream overlap of the 32-CU epoch kernel is gone).
// (The first version used a balanced network over the even-bit domain 2^(2h), up to 4n: at n = 2^19
// that is 2n, and a wave waits for its longest cycle walk: 31.2 us per epoch against 6.8 us now.)
// The reference draws torch.randperm on the host CPU generator (vec_rollout.py:166-175); the shuffle is
// a different random stream either way, and parity tests inject the reference's permutations.
__device__ __forceinline__ uint32_t perm_mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
constexpr int PERM_ROUNDS = 6;
struct PermArgs {
  uint32_t k[PERM_ROUNDS];
  int32_t h1, h2;  // high / low part widths, h1 + h2 = b
  int64_t n;
  int64_t* out;
};
__global__ __launch_bounds__(256) void feistel_perm_kernel(const PermArgs a) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.n) return;
  const uint32_t m1 = (1u << a.h1) - 1u, m2 = (1u << a.h2) - 1u;
  uint64_t x = (uint64_t)i;
  do {  // the domain 2^b is < 2n: walks twice on average, never when n is a power of two
    uint32_t hi = (uint32_t)(x >> a.h2), lo = (uint32_t)x & m2;  // h1 and h2 bits
#pragma unroll
    for (int r = 0; r < PERM_ROUNDS; r += 2) {
      const uint32_t t = hi ^ (perm_mix32(lo ^ a.k[r]) & m1);  // (h1, h2) -> (h2, h1)
      hi = lo;
      lo = t;
      const uint32_t u = hi ^ (perm_mix32(lo ^ a.k[r + 1]) & m2);  // (h2, h1) -> (h1, h2)
      hi = lo;
      lo = u;
    }
    x = ((uint64_t)hi << a.h2) | lo;
  } while (x >= (uint64_t)a.n);
  a.out[i] = (int64_t)x;
}

// Minibatch gather driven by a device descriptor (graph replay: the launch is fixed, the
// minibatch index advances on device).  Workgroup b owns rows b, b + G, ... and its threads stride
// the (row, unit) pairs of those rows over the concatenated units of all fields with GM_BATCH loads
// in flight before the stores.  A unit is 16, 4 or 1 bytes of a copied field, or one QUAD of a frame
// field (below).  The grid is at most one workgroup per row and <= 1024, so few workgroups arrive on
// the advance counter (a device-scope atomic on one address, serialised across the XCDs); rows of
// more than 256 units take 1024-thread workgroups so that a whole Pong row (1,764 frame quads) is
// in flight at once instead of seven dependent 256-thread passes (43.8 us per Pong minibatch with
// 256 threads; the first version, (rows x units / 256) x fields workgroups each arriving on the
// counter, took 202 us).
//
// Frame fields (RAI_XFORM_U8_CHW_TO_F32_HWC): a source row of C <= 4 planes of HW uint8 pixels
// (the rollout's NCHW frames) becomes HW x C float32 (NHWC, channels_last) with
// out = (float)u8 / divisor: the NatureCNN input prescale obs.float() / range_size
// (rl_algo_impls/shared/encoder/cnn.py:24-27) and the channels_last conversion fused into the
// gather.  One unit = 4 consecutive pixels: C 4-byte loads (one per plane) and C float4 stores.
// The division is IEEE-correct (hipcc's default), as the reference's CPU path divides; torch on a
// GPU multiplies by the rounded reciprocal instead.
struct MbDst {
  uint8_t* dst[RAI_MAX_FIELDS];
  int64_t units[RAI_MAX_FIELDS];
  int32_t gran[RAI_MAX_FIELDS];  // 16 / 4 / 1: copy; 0: frame quads -> f32; -1: frame quads -> u8 (4 planes)
  int32_t planes[RAI_MAX_FIELDS];
  int64_t hw[RAI_MAX_FIELDS];
  float divisor[RAI_MAX_FIELDS];
  int32_t n_fields;
};
constexpr int GM_BATCH = 4;
template <int NT>
__global__ __launch_bounds__(NT) void gather_minibatch_kernel(rai_minibatch_desc* __restrict__ d, const MbDst o,
                                                              const int advance) {
  const int64_t mb = d->mb, B = d->batch_size;
  const int64_t row0 = mb * B;
  const int rows = (int)min(B, d->n_rows - row0);
  const int64_t* perm = d->perm;
  const int nf = o.n_fields;
  int total = 0;  // a row's units over all fields: the threads stride (row, unit) pairs of the
  for (int f = 0; f < nf; ++f) total += (int)o.units[f];  // workgroup's rows jointly
  const int G = (int)gridDim.x, b = (int)blockIdx.x;
  const int my_rows = rows > b ? (rows - b + G - 1) / G : 0;  // rows b, b + G, b + 2G, ...
  const int work = my_rows * total;  // < 2^31: checked at launch (batch_size x total)
  for (int i0 = threadIdx.x; i0 < work; i0 += GM_BATCH * NT) {
    uint4 v[GM_BATCH];
    int64_t doff[GM_BATCH];
    int fk[GM_BATCH];
#pragma unroll
    for (int k = 0; k < GM_BATCH; ++k) {
      const int i = i0 + k * NT;
      fk[k] = -1;
      if (i < work) {
        const int ri = (int)((unsigned)i / (unsigned)total);
        int j = i - ri * total;
        const int64_t r = b + (int64_t)ri * G;
        const int64_t sr = perm ? perm[row0 + r] : row0 + r;
        int f = 0;
        while (j >= (int)o.units[f]) j -= (int)o.units[f++];
        fk[k] = f;
        const uint8_t* src = static_cast<const uint8_t*>(d->src[f]);
        if (o.gran[f] <= 0) {  // frame quad j of row sr: one word per plane
          const int C = o.planes[f];
          const int64_t hw4 = o.hw[f] >> 2;
          const uint32_t* s32 = reinterpret_cast<const uint32_t*>(src) + sr * C * hw4 + j;
          v[k].x = s32[0];
          v[k].y = C > 1 ? s32[hw4] : 0u;
          v[k].z = C > 2 ? s32[2 * hw4] : 0u;
          v[k].w = C > 3 ? s32[3 * hw4] : 0u;
          doff[k] = (r * o.hw[f] + 4LL * j) * C;  // element (float or byte) index of the quad's first pixel
        } else {
          const int64_t so = sr * o.units[f] + j;
          doff[k] = r * o.units[f] + j;
          if (o.gran[f] == 16) v[k] = reinterpret_cast<const uint4*>(src)[so];
          else if (o.gran[f] == 4) v[k].x = reinterpret_cast<const uint32_t*>(src)[so];
          else v[k].x = src[so];
        }
      }
    }
#pragma unroll
    for (int k = 0; k < GM_BATCH; ++k) {
      const int f = fk[k];
      if (f < 0) continue;
      if (o.gran[f] == 0) {
        const int C = o.planes[f];
        const float div = o.divisor[f];
        const uint32_t w[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
        float4* out = reinterpret_cast<float4*>(reinterpret_cast<float*>(o.dst[f]) + doff[k]);
        for (int q = 0; q < C; ++q) {  // float4 q holds elements m = 4q..4q+3 of (pixel p, plane c), m = p*C + c
          float e[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int m = 4 * q + u, p = m / C, c = m - p * C;
            e[u] = (float)((w[c] >> (8 * p)) & 0xffu) / div;
          }
          out[q] = make_float4(e[0], e[1], e[2], e[3]);
        }
      } else if (o.gran[f] == -1) {  // 4 pixels x 4 planes of bytes, transposed to pixel-major (NHWC)
        const uint32_t w[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
        uint32_t px[4];
#pragma unroll
        for (int p = 0; p < 4; ++p)
          px[p] = ((w[0] >> (8 * p)) & 0xffu) | (((w[1] >> (8 * p)) & 0xffu) << 8) |
                  (((w[2] >> (8 * p)) & 0xffu) << 16) | (((w[3] >> (8 * p)) & 0xffu) << 24);
        *reinterpret_cast<uint4*>(o.dst[f] + doff[k]) = make_uint4(px[0], px[1], px[2], px[3]);
      } else if (o.gran[f] == 16) {
        reinterpret_cast<uint4*>(o.dst[f])[doff[k]] = v[k];
      } else if (o.gran[f] == 4) {
        reinterpret_cast<uint32_t*>(o.dst[f])[doff[k]] = v[k].x;
      } else {
        o.dst[f][doff[k]] = (uint8_t)v[k].x;
      }
    }
  }
  if (advance) {
    // every wave read mb at its start and used it for its loop bounds, so after the barrier the
    // workgroup's reads of it are complete: the last workgroup to arrive may then advance the
    // minibatch for the next launch (which sees it across the kernel boundary) and re-arm the
    // counter.  No fences: a __threadfence() here is an L2 write-back (buffer_wbl2) right after the
    // workgroup's 28 KB of output, 256 times a launch (26.3 us per C3 minibatch with them).
    // Two-level arrival (same-address agent atomics serialise at ~10 ns each: 256 arrivals on one
    // counter cost ~2.4 us): workgroup w counts in group w % 8, the last of a group in the top one.
    __syncthreads();
    if (threadIdx.x == 0) {
      const int nb = (int)gridDim.x, w = (int)blockIdx.x;
      const int grp = w & 7, gsize = (nb - grp + 7) >> 3, ngroups = nb < 8 ? nb : 8;
      int* cg = &d->group_arrivals[16 * grp];
      if (__hip_atomic_fetch_add(cg, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gsize - 1) {
        __hip_atomic_store(cg, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (__hip_atomic_fetch_add(&d->arrivals, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ngroups - 1) {
          __hip_atomic_store(&d->arrivals, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(&d->mb, mb + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
  }
}

__global__ void minibatch_advance_kernel(rai_minibatch_desc* d) { d->mb += 1; }

// One thread per env row.  Masked logits follow MaskedCategorical
// (torch.where(mask, logits, finfo.min)); torch.distributions normalises
// logits by logsumexp; log_prob(a) = logits[a] - logsumexp.
__global__ __launch_bounds__(256) void categorical_sample_kernel(
    const float* __restrict__ logits, const uint8_t* __restrict__ mask, int64_t N, int A,
    uint64_t seed, uint64_t offset, int64_t* __restrict__ actions, float* __restrict__ logp,
    const float* __restrict__ v_in, float* __restrict__ v_out, int K) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= N) return;
  const float* l = logits + r * A;
  const uint8_t* mk = mask ? mask + r * A : nullptr;
  const float NEG = -3.4028234663852886e38f;  // torch.finfo(float32).min
  float m = -INFINITY;
  for (int i = 0; i < A; ++i) {
    const float x = (mk && !mk[i]) ? NEG : l[i];
    m = fmaxf(m, x);
  }
  float s = 0.f;
  for (int i = 0; i < A; ++i) {
    const float x = (mk && !mk[i]) ? NEG : l[i];
    s += expf(x - m);
  }
  const float lse = m + logf(s);
  const Philox4 rnd = philox4x32_10(offset, (uint64_t)r, seed);
  const float u = u01_open0(rnd.x) * s;  // inverse CDF on unnormalised mass
  float c = 0.f;
  int act = -1, last_valid = 0;
  for (int i = 0; i < A; ++i) {
    const bool ok = !(mk && !mk[i]);
    if (!ok) continue;
    last_valid = i;
    c += expf(l[i] - m);
    if (act < 0 && u <= c) act = i;
  }
  if (act < 0) act = last_valid;
  actions[r] = act;
  logp[r] = l[act] - lse;
  if (v_in && v_out)
    for (int k = 0; k < K; ++k) v_out[r * K + k] = v_in[r * K + k];
}

// a = mu + std*eps (rsample); logp = sum_d Normal.log_prob; clamped = clip(a, low, high)
__global__ __launch_bounds__(256) void gaussian_sample_kernel(
    const float* __restrict__ mu, const float* __restrict__ log_std, int64_t N, int A,
    const float* __restrict__ low, const float* __restrict__ high, uint64_t seed,
    uint64_t offset, float* __restrict__ actions, float* __restrict__ clamped,
    float* __restrict__ logp, const float* __restrict__ v_in, float* __restrict__ v_out, int K) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= N) return;
  const float LOG_SQRT_2PI = 0.91893853320467274178f;  // log(sqrt(2*pi))
  float lp = 0.f;
  for (int d = 0; d < A; d += 2) {
    const Philox4 rnd = philox4x32_10(offset, ((uint64_t)r << 16) | (uint64_t)(d >> 1), seed);
    const float u1 = u01_open0(rnd.x), u2 = u01_open0(rnd.y);
    const float rad = sqrtf(-2.f * logf(u1));
    float s, c;
    sincosf(6.283185307179586f * u2, &s, &c);
    const float e2[2] = {rad * c, rad * s};
    for (int q = 0; q < 2 && d + q < A; ++q) {
      const int dd = d + q;
      const float ls = log_std[dd];
      const float sd = expf(ls);
      const float m = mu[r * A + dd];
      const float a = m + sd * e2[q];
      const float var = sd * sd;
      const float diff = a - m;
      lp += -(diff * diff) / (2.f * var) - ls - LOG_SQRT_2PI;
      actions[r * A + dd] = a;
      if (clamped) {
        float x = a;
        if (low) x = fmaxf(x, low[dd]);
        if (high) x = fminf(x, high[dd]);
        clamped[r * A + dd] = x;
      }
    }
  }
  logp[r] = lp;
  if (v_in && v_out)
    for (int k = 0; k < K; ++k) v_out[r * K + k] = v_in[r * K + k];
}

}  // namespace

// Rollout host <-> device staging in one native call each (the env-step loop of
// rl_algo_impls/rollout/sync_step_rollout.py:193-207: actions to the host env, then its rewards,
// terminations and next observations back).  Issued here rather than as separate torch copies, whose
// per-call dispatch costs ~10 us each on the 128-step C2 loop.
extern "C" int rai_copy_d2h_sync(const void* src, void* dst, int64_t bytes, void* stream) {
  if (bytes < 0) return RAI_E_SHAPE;
  if (bytes == 0) return RAI_OK;
  if (!src || !dst) return RAI_E_NULLPTR;
  hipStream_t s = rai_stream(stream);
  hipError_t e = hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToHost, s);
  if (e != hipSuccess) return (int)e;
  e = hipStreamSynchronize(s);
  return e == hipSuccess ? RAI_OK : (int)e;
}

extern "C" int rai_copy_h2d_multi(int32_t n, void* const* dst, const void* const* src, const int64_t* bytes,
                                  void* stream) {
  if (n < 0 || n > RAI_MAX_FIELDS) return RAI_E_SHAPE;
  if (n == 0) return RAI_OK;
  if (!dst || !src || !bytes) return RAI_E_NULLPTR;
  hipStream_t s = rai_stream(stream);
  for (int i = 0; i < n; ++i) {
    if (bytes[i] < 0) return RAI_E_SHAPE;
    if (bytes[i] == 0) continue;
    if (!dst[i] || !src[i]) return RAI_E_NULLPTR;
    const hipError_t e = hipMemcpyAsync(dst[i], src[i], (size_t)bytes[i], hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return (int)e;
  }
  return RAI_OK;
}

extern "C" int rai_gather_rows(int32_t n_fields, const void* const* src, void* const* dst,
                               const int64_t* row_bytes, const int64_t* idx, int64_t n_rows,
                               void* stream) {
  if (n_fields < 1 || n_fields > RAI_MAX_FIELDS || n_rows < 0) return RAI_E_SHAPE;
  if (n_rows == 0) return RAI_OK;
  if (!src || !dst || !row_bytes || !idx) return RAI_E_NULLPTR;
  GatherArgs a;
  int64_t max_units = 0;
  for (int i = 0; i < n_fields; ++i) {
    if (!src[i] || !dst[i]) return RAI_E_NULLPTR;
    if (row_bytes[i] < 1) return RAI_E_SHAPE;
    const uintptr_t al = (uintptr_t)src[i] | (uintptr_t)dst[i];
    int gran = 1;
    if (row_bytes[i] % 16 == 0 && al % 16 == 0) gran = 16;
    else if (row_bytes[i] % 4 == 0 && al % 4 == 0) gran = 4;
    a.f[i].src = static_cast<const uint8_t*>(src[i]);
    a.f[i].dst = static_cast<uint8_t*>(dst[i]);
    a.f[i].gran = gran;
    a.f[i].units = row_bytes[i] / gran;
    if (a.f[i].units > max_units) max_units = a.f[i].units;
  }
  a.idx = idx;
  a.n_rows = n_rows;
  int64_t blocks = (n_rows * max_units + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)blocks, (unsigned)n_fields), dim3(256), 0,
                     rai_stream(stream), a);
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}

static uint32_t perm_mix32_host(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

extern "C" int rai_feistel_permutation(int64_t n, uint64_t key, int64_t* out, void* stream) {
  if (n < 0 || n > ((int64_t)1 << 60)) return RAI_E_SHAPE;
  if (n == 0) return RAI_OK;
  if (!out) return RAI_E_NULLPTR;
  PermArgs a;
  int bits = 0;
  while (bits < 62 && ((int64_t)1 << bits) < n) ++bits;
  if (bits < 2) bits = 2;
  a.h1 = bits / 2;
  a.h2 = bits - a.h1;
  const uint32_t lo = (uint32_t)key, hi = (uint32_t)(key >> 32);
  for (int r = 0; r < PERM_ROUNDS; ++r) a.k[r] = perm_mix32_host(lo ^ perm_mix32_host(hi + 0x9e3779b9u * (uint32_t)(r + 1)));
  a.n = n;
  a.out = out;
  hipLaunchKernelGGL(feistel_perm_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, rai_stream(stream), a);
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}

static int gather_minibatch(rai_minibatch_desc* desc, int32_t n_fields, void* const* dst, const int64_t* row_bytes,
                            const rai_gather_xform* xform, int64_t batch_size, int advance, void* stream) {
  if (n_fields < 1 || n_fields > RAI_MAX_FIELDS || batch_size < 1) return RAI_E_SHAPE;
  if (!desc || !dst || !row_bytes) return RAI_E_NULLPTR;
  MbDst o;
  for (int i = 0; i < n_fields; ++i) {
    if (!dst[i] || row_bytes[i] < 1) return RAI_E_NULLPTR;
    o.dst[i] = static_cast<uint8_t*>(dst[i]);
    o.planes[i] = 0;
    o.hw[i] = 0;
    o.divisor[i] = 1.f;
    const int kind = xform ? xform[i].kind : RAI_XFORM_COPY;
    if (kind == RAI_XFORM_U8_CHW_TO_F32_HWC) {
      const rai_gather_xform& x = xform[i];
      // C <= 4 planes of HW pixels, HW % 4 == 0 (quads of 4-byte source words), 16-B aligned output
      if (x.channels < 1 || x.channels > 4 || x.hw < 4 || x.hw % 4 || (int64_t)x.channels * x.hw != row_bytes[i] ||
          !(x.divisor > 0.f) || ((uintptr_t)dst[i] & 15))
        return RAI_E_SHAPE;
      o.gran[i] = 0;
      o.planes[i] = x.channels;
      o.hw[i] = x.hw;
      o.divisor[i] = x.divisor;
      o.units[i] = x.hw / 4;
    } else if (kind == RAI_XFORM_U8_CHW_TO_U8_HWC) {
      const rai_gather_xform& x = xform[i];
      // exactly 4 planes (one 16-B pixel-major quad per unit), 16-B aligned output
      if (x.channels != 4 || x.hw < 4 || x.hw % 4 || 4 * x.hw != row_bytes[i] || ((uintptr_t)dst[i] & 15))
        return RAI_E_SHAPE;
      o.gran[i] = -1;
      o.planes[i] = 4;
      o.hw[i] = x.hw;
      o.units[i] = x.hw / 4;
    } else if (kind == RAI_XFORM_COPY) {
      const int gran = (row_bytes[i] % 16 == 0) ? 16 : ((row_bytes[i] % 4 == 0) ? 4 : 1);
      o.gran[i] = gran;
      o.units[i] = row_bytes[i] / gran;
    } else {
      return RAI_E_MODE;
    }
  }
  o.n_fields = n_fields;
  int64_t total = 0;
  for (int i = 0; i < n_fields; ++i) total += o.units[i];
  if (batch_size * total >= (1LL << 31)) return RAI_E_SHAPE;  // 32-bit (row, unit) indexing
  // rows of more than 256 units: one 1024-thread workgroup per row (the row in flight at once);
  // else ~256 (row, unit) pairs per 256-thread workgroup, at most one workgroup per row (<= 1024)
  const bool wide = total > 256;
  const int nt = wide ? 1024 : 256;
  int64_t blocks = (batch_size * total + nt - 1) / nt;
  if (blocks > batch_size) blocks = batch_size;
  if (blocks > 1024) blocks = 1024;
  if (blocks < 1) blocks = 1;
  // (two rows per workgroup measured 23.7 us per C3 minibatch, two and four workgroups per row
  // 21.9 / 25.9 us, against 19.3 us for one workgroup per row: tools/gather_bench.py, profiles/r2zi_*)
  if (wide)
    hipLaunchKernelGGL(gather_minibatch_kernel<1024>, dim3((unsigned)blocks), dim3(1024), 0, rai_stream(stream), desc,
                       o, advance);
  else
    hipLaunchKernelGGL(gather_minibatch_kernel<256>, dim3((unsigned)blocks), dim3(256), 0, rai_stream(stream), desc,
                       o, advance);
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}

extern "C" int rai_gather_minibatch(const rai_minibatch_desc* desc, int32_t n_fields, void* const* dst,
                                    const int64_t* row_bytes, int64_t batch_size, void* stream) {
  return gather_minibatch(const_cast<rai_minibatch_desc*>(desc), n_fields, dst, row_bytes, nullptr, batch_size, 0,
                          stream);
}

extern "C" int rai_gather_minibatch_next(rai_minibatch_desc* desc, int32_t n_fields, void* const* dst,
                                         const int64_t* row_bytes, int64_t batch_size, void* stream) {
  return gather_minibatch(desc, n_fields, dst, row_bytes, nullptr, batch_size, 1, stream);
}

extern "C" int rai_gather_minibatch_x(rai_minibatch_desc* desc, int32_t n_fields, void* const* dst,
                                      const int64_t* row_bytes, const rai_gather_xform* xform, int64_t batch_size,
                                      int32_t advance, void* stream) {
  return gather_minibatch(desc, n_fields, dst, row_bytes, xform, batch_size, advance ? 1 : 0, stream);
}

extern "C" int rai_minibatch_advance(rai_minibatch_desc* desc, void* stream) {
  if (!desc) return RAI_E_NULLPTR;
  hipLaunchKernelGGL(minibatch_advance_kernel, dim3(1), dim3(1), 0, rai_stream(stream), desc);
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}

extern "C" int rai_categorical_sample(const float* logits, const uint8_t* mask, int64_t N,
                                      int32_t A, uint64_t seed, uint64_t offset,
                                      int64_t* actions_out, float* logp_out, const float* v_in,
                                      float* v_out, int32_t K, void* stream) {
  if (N < 0 || A < 1 || K < 0) return RAI_E_SHAPE;
  if (N == 0) return RAI_OK;
  if (!logits || !actions_out || !logp_out) return RAI_E_NULLPTR;
  const unsigned blocks = (unsigned)((N + 255) / 256);
  hipLaunchKernelGGL(categorical_sample_kernel, dim3(blocks), dim3(256), 0, rai_stream(stream),
                     logits, mask, N, A, seed, offset, actions_out, logp_out, v_in, v_out, K);
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}

extern "C" int rai_gaussian_sample(const float* mu, const float* log_std, int64_t N, int32_t A,
                                   const float* low, const float* high, uint64_t seed,
                                   uint64_t offset, float* actions_out, float* clamped_out,
                                   float* logp_out, const float* v_in, float* v_out, int32_t K,
                                   void* stream) {
  if (N < 0 || A < 1 || K < 0) return RAI_E_SHAPE;
  if (N == 0) return RAI_OK;
  if (!mu || !log_std || !actions_out || !logp_out) return RAI_E_NULLPTR;
  const unsigned blocks = (unsigned)((N + 255) / 256);
  hipLaunchKernelGGL(gaussian_sample_kernel, dim3(blocks), dim3(256), 0, rai_stream(stream), mu,
                     log_std, N, A, low, high, seed, offset, actions_out, clamped_out, logp_out,
                     v_in, v_out, K);
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}
