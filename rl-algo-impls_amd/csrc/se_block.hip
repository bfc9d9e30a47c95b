// Squeeze-excitation residual epilogue of the squeeze-U-Net backbone (config C5) on gfx950.
//
// SEResidualBlock.forward (rl_algo_impls/shared/policy/actor_critic_network/double_cone.py:85-86)
// ends with   out = GELU(x + r * s)   where r is the second 3x3 conv's output, s = sigmoid(fc(mean_hw r))
// the squeeze-excitation scale (double_cone.py:43-47).  PyTorch runs that as a broadcast multiply,
// an add and a GELU (three passes over the activation, two intermediates) and the backward as four
// more kernels plus a reduction for ds.  Here:
//   forward   one pass:  out = gelu(x + r * s[b, c])                          (reads x, r; writes out)
//   backward  one pass:  g = dout * gelu'(x + r * s);  dx = g;  dr = g * s;  ds[b, c] = sum_hw g * r
// GELU is the exact (erf) form of torch.nn.GELU(): gelu(t) = t * Phi(t), gelu'(t) = Phi(t) + t * phi(t).
//
// Layout: NHWC (channels_last) activations, (B, HW, C) row-major with C fastest; s, ds (B, C).
// Forward: grid-stride float4 elementwise pass.  Backward: one 256-thread workgroup per sample; a
// thread owns one float4 channel group (c4 = tid % C4) for HW rows tid / C4 + k * (256 / C4), keeps
// its ds partial in registers, and the 256 / C4 row-groups are summed in a fixed order through LDS
// (deterministic).  Needs C % 4 == 0 and C / 4 dividing 256 (C in {4, 8, ..., 1024}).
#include "common.h"

namespace {

constexpr int SE_THREADS = 256;
using f4 = float __attribute__((ext_vector_type(4)));
typedef unsigned int u4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float gelu_f(float t) { return 0.5f * t * (1.f + erff(t * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_grad(float t) {
  const float cdf = 0.5f * (1.f + erff(t * 0.70710678118654752f));
  const float pdf = expf(-0.5f * t * t) * 0.39894228040143268f;
  return cdf + t * pdf;
}

__global__ __launch_bounds__(SE_THREADS) void se_fwd_kernel(const f4* __restrict__ x, const f4* __restrict__ r,
                                                            const f4* __restrict__ s, int C4, int64_t HWC4,
                                                            int64_t n4, f4* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)SE_THREADS + threadIdx.x; i < n4; i += (int64_t)gridDim.x * SE_THREADS) {
    const int64_t b = i / HWC4;
    const int c4 = (int)(i % C4);
    const f4 xv = x[i], rv = r[i], sv = s[b * C4 + c4];
    f4 o;
#pragma unroll
    for (int q = 0; q < 4; ++q) o[q] = gelu_f(xv[q] + rv[q] * sv[q]);
    out[i] = o;
  }
}

__global__ __launch_bounds__(SE_THREADS) void se_bwd_kernel(const f4* __restrict__ dout, const f4* __restrict__ x,
                                                            const f4* __restrict__ r, const f4* __restrict__ s,
                                                            int C4, int HW, f4* __restrict__ dx, f4* __restrict__ dr,
                                                            f4* __restrict__ ds) {
  __shared__ f4 part[SE_THREADS];
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x;
  const int c4 = tid % C4, row0 = tid / C4, rstep = SE_THREADS / C4;
  const f4 sv = s[b * C4 + c4];
  f4 acc = f4{0.f, 0.f, 0.f, 0.f};
  const int64_t base = b * (int64_t)HW * C4;
  for (int h = row0; h < HW; h += rstep) {
    const int64_t i = base + (int64_t)h * C4 + c4;
    const f4 g0 = dout[i], xv = x[i], rv = r[i];
    f4 g, dri;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      g[q] = g0[q] * gelu_grad(xv[q] + rv[q] * sv[q]);
      dri[q] = g[q] * sv[q];
      acc[q] += g[q] * rv[q];
    }
    dx[i] = g;
    dr[i] = dri;
  }
  part[tid] = acc;
  __syncthreads();
  if (tid < C4) {
    f4 t = part[tid];
    for (int k = 1; k < rstep; ++k) t += part[tid + k * C4];
    ds[b * C4 + tid] = t;
  }
}

bool shape_ok(int64_t B, int32_t C, int32_t HW) {
  if (B < 0 || C < 4 || HW < 1 || C % 4) return false;
  const int C4 = C / 4;
  return C4 <= SE_THREADS && SE_THREADS % C4 == 0;
}

}  // namespace

extern "C" int rai_se_residual_fwd(const float* x, const float* r, const float* s, int64_t B, int32_t C, int32_t HW,
                                   float* out, void* stream) {
  if (!shape_ok(B, C, HW)) return RAI_E_SHAPE;
  if (B == 0) return RAI_OK;
  if (!x || !r || !s || !out) return RAI_E_NULLPTR;
  const int C4 = C / 4;
  const int64_t n4 = B * (int64_t)HW * C4;
  const int64_t blocks = std::min<int64_t>((n4 + SE_THREADS - 1) / SE_THREADS, 256 * 64);
  hipLaunchKernelGGL(se_fwd_kernel, dim3((unsigned)blocks), dim3(SE_THREADS), 0, rai_stream(stream),
                     reinterpret_cast<const f4*>(x), reinterpret_cast<const f4*>(r), reinterpret_cast<const f4*>(s),
                     C4, (int64_t)HW * C4, n4, reinterpret_cast<f4*>(out));
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}

extern "C" int rai_se_residual_bwd(const float* dout, const float* x, const float* r, const float* s, int64_t B,
                                   int32_t C, int32_t HW, float* dx, float* dr, float* ds, void* stream) {
  if (!shape_ok(B, C, HW)) return RAI_E_SHAPE;
  if (B == 0) return RAI_OK;
  if (!dout || !x || !r || !s || !dx || !dr || !ds) return RAI_E_NULLPTR;
  hipLaunchKernelGGL(se_bwd_kernel, dim3((unsigned)B), dim3(SE_THREADS), 0, rai_stream(stream),
                     reinterpret_cast<const f4*>(dout), reinterpret_cast<const f4*>(x),
                     reinterpret_cast<const f4*>(r), reinterpret_cast<const f4*>(s), C / 4, HW,
                     reinterpret_cast<f4*>(dx), reinterpret_cast<f4*>(dr), reinterpret_cast<f4*>(ds));
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}

// ---- conv bias + GELU epilogue (squeeze-U-Net conv -> GELU pairs) ------------------------------
// y = gelu(x + b[c]) over NHWC rows (rows = B*H*W, C fastest): MIOpen's separate bias pass
// (SubTensorOpWithScalar1d) and the GELU kernel become one pass.  Backward: dx = dy * gelu'(x + b);
// the bias gradient is dx summed over rows (the caller's one reduction).
namespace {
// b is read as scalars: a bias is a view into the flat parameter buffer, 4-byte aligned only
__device__ __forceinline__ f4 ld_bias4(const float* __restrict__ b, int c4) {
  return f4{b[4 * c4], b[4 * c4 + 1], b[4 * c4 + 2], b[4 * c4 + 3]};
}
__global__ __launch_bounds__(SE_THREADS) void bias_gelu_fwd_kernel(const f4* __restrict__ x, const float* __restrict__ b,
                                                                   int C4, int64_t n4, f4* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)SE_THREADS + threadIdx.x; i < n4; i += (int64_t)gridDim.x * SE_THREADS) {
    const f4 xv = x[i], bv = ld_bias4(b, (int)(i % C4));
    f4 o;
#pragma unroll
    for (int q = 0; q < 4; ++q) o[q] = gelu_f(xv[q] + bv[q]);
    out[i] = o;
  }
}
__global__ __launch_bounds__(SE_THREADS) void bias_gelu_bwd_kernel(const f4* __restrict__ dy, const f4* __restrict__ x,
                                                                   const float* __restrict__ b, int C4, int64_t n4,
                                                                   f4* __restrict__ dx) {
  for (int64_t i = blockIdx.x * (int64_t)SE_THREADS + threadIdx.x; i < n4; i += (int64_t)gridDim.x * SE_THREADS) {
    const f4 g = dy[i], xv = x[i], bv = ld_bias4(b, (int)(i % C4));
    f4 o;
#pragma unroll
    for (int q = 0; q < 4; ++q) o[q] = g[q] * gelu_grad(xv[q] + bv[q]);
    dx[i] = o;
  }
}
int64_t ew_blocks(int64_t n4) { return std::min<int64_t>((n4 + SE_THREADS - 1) / SE_THREADS, 256 * 64); }
}  // namespace

extern "C" int rai_bias_gelu_fwd(const float* x, const float* b, int64_t rows, int32_t C, float* out, void* stream) {
  if (rows < 0 || C < 4 || C % 4) return RAI_E_SHAPE;
  if (rows == 0) return RAI_OK;
  if (!x || !b || !out) return RAI_E_NULLPTR;
  const int64_t n4 = rows * (C / 4);
  hipLaunchKernelGGL(bias_gelu_fwd_kernel, dim3((unsigned)ew_blocks(n4)), dim3(SE_THREADS), 0, rai_stream(stream),
                     reinterpret_cast<const f4*>(x), b, C / 4, n4, reinterpret_cast<f4*>(out));
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}

extern "C" int rai_bias_gelu_bwd(const float* dy, const float* x, const float* b, int64_t rows, int32_t C, float* dx,
                                 void* stream) {
  if (rows < 0 || C < 4 || C % 4) return RAI_E_SHAPE;
  if (rows == 0) return RAI_OK;
  if (!dy || !x || !b || !dx) return RAI_E_NULLPTR;
  const int64_t n4 = rows * (C / 4);
  hipLaunchKernelGGL(bias_gelu_bwd_kernel, dim3((unsigned)ew_blocks(n4)), dim3(SE_THREADS), 0, rai_stream(stream),
                     reinterpret_cast<const f4*>(dy), reinterpret_cast<const f4*>(x), b, C / 4, n4,
                     reinterpret_cast<f4*>(dx));
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}

// ---- conv / linear bias + ReLU epilogue (NatureCNN, config C3) --------------------------------
// The NatureCNN encoder (rl_algo_impls/shared/encoder/nature_cnn.py:10-53) is three conv -> ReLU
// pairs and a Linear -> ReLU.  PyTorch runs each as conv, a bias add (broadcast over NHWC rows) and a
// clamp; backward as threshold_backward, a column-sum reduction for the bias gradient and an
// accumulate of that gradient into .grad: five launches per layer around the MIOpen / hipBLASLt
// contraction.  Here, per layer:
//   forward   one pass:  out = relu(x + b[c])                       (x: bias-free conv / GEMM output)
//   backward  dx = dy * (out > 0) and db[c] (+)= sum_rows dx[row, c]: one pass over the rows whose
//             last-arriving workgroup sums the per-workgroup column sums
// The bias-gradient reduction is deterministic (fixed row runs per workgroup, fixed summation
// orders).  relu(NaN) = NaN and dx = 0 where out <= 0, as torch's clamp_min / threshold_backward.
namespace {
constexpr int BR_THREADS = 256;
constexpr int BR_MAX_BLOCKS = 512;  // two workgroups per CU
constexpr int BR_UNROLL = 4;      // rows in flight per lane before the first use
constexpr int BR_ROWS_PER_LANE = 8;  // conv1 at C3: 400 workgroups of 256 rows
constexpr int BR_TAIL = 16;       // partial loads in flight per thread in the last arriver
constexpr int BR_CTR_STRIDE = 16;  // arrival counters 64 B apart: the top one, then 8 group counters
constexpr int BR_CTR_BYTES = 9 * BR_CTR_STRIDE * 4;

__global__ __launch_bounds__(BR_THREADS) void bias_relu_fwd_kernel(const f4* __restrict__ x, const float* __restrict__ b,
                                                                  int C4, int64_t n4, f4* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)BR_THREADS + threadIdx.x; i < n4; i += (int64_t)gridDim.x * BR_THREADS) {
    const f4 xv = x[i], bv = ld_bias4(b, (int)(i % C4));
    f4 o;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float t = xv[q] + bv[q];
      o[q] = t < 0.f ? 0.f : t;
    }
    out[i] = o;
  }
}

// Workgroup w owns rows [w * rpb, (w + 1) * rpb); its threads are (row lane, float4 channel group)
// pairs, each lane keeping BR_UNROLL rows' loads in flight; dx is stored and the workgroup's column
// sums (a pairwise tree over the row lanes) go to partial[w].  The workgroup whose arrival comes last
// then sums the partials: thread (lane, c4) adds partials lane, lane + lanes, ... of channel group c4
// with BR_TAIL 16-B loads in flight, and the lanes are tree-summed again -> db.  Every order is fixed
// by (rows, C), so db is deterministic.  (Round 2, first form: serial lane sums and 4-B tail loads
// four in flight, 8-13 us per C3 layer against ~5 us for torch's threshold_backward alone;
// tools/bias_relu_bench.py, profiles/r2t_bias_relu_bench.txt.)
// Hand-off without fences (MI355X_MICROARCH.md, inter-workgroup visibility, valid forms): the partials
// are 16-B write-through (sc1) buffer stores drained by every storing wave (vmcnt(0)) before the
// workgroup barrier and the agent-scope arrival atomics (group counter, then the top counter for the
// last of a group); the last arriver's waves read them with sc1 buffer loads after a barrier.  (Two launches, the row pass then a one-workgroup finalize, cost a second
// ~4.8 us launch per layer; a last-arriver variant with __threadfence() in every thread ~30 us.)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t br_rsrc(const void* p, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, bytes, 0x00020000);
}
constexpr int BR_SC1 = 16;  // cache-policy operand: sc1 (write-through stores, L1-bypassing loads)

// part[lane * C4 + c4] (lanes a power of two) -> part[c4]: a pairwise tree over the lanes, the same
// order on every launch.  Called with part written and the workgroup synchronised.
__device__ __forceinline__ void lane_tree_sum(f4* part, int lane, int C4, int lanes) {
  for (int h = lanes / 2; h >= 1; h /= 2) {
    if (lane < h) part[threadIdx.x] += part[threadIdx.x + h * C4];
    __syncthreads();
  }
}

// The end of every bias-gradient pass: this workgroup's column sums (thread tid < C4 holds channels
// 4 tid .. 4 tid + 3 in wsum) go to partial[blockIdx.x] (write-through), the workgroup arrives on
// the two-level counters, and the last arriver sums the nb partials in a fixed order into db
// (db0: db as read at the kernel's start, for accumulate).
__device__ __forceinline__ void br_finish(f4 wsum, f4* part, int* last, float* partial, int* counter, float* db,
                                          const float* db0, int accumulate, int C4) {
  const int tid = threadIdx.x, lanes = BR_THREADS / C4, c4 = tid % C4, lane = tid / C4, C = 4 * C4;
  const int nb = (int)gridDim.x;
  const __amdgpu_buffer_rsrc_t prs = br_rsrc(partial, nb * C * 4);
  if (tid < C4)
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, wsum), prs, (blockIdx.x * C + 4 * tid) * 4, 0,
                                           BR_SC1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its stores
  __syncthreads();
  // arrival in two levels: workgroup w counts in group w % 8 (same-address atomics serialise at
  // ~10 ns each: one counter for 400 workgroups cost ~3.6 us), the last of each group in the top one
  if (tid == 0) {
    const int g = blockIdx.x & 7, gsize = (nb - g + 7) >> 3, ngroups = nb < 8 ? nb : 8;
    int* cg = counter + BR_CTR_STRIDE * (1 + g);
    *last = 0;
    if (__hip_atomic_fetch_add(cg, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gsize - 1) {
      __hip_atomic_store(cg, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-armed
      *last = __hip_atomic_fetch_add(counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ngroups - 1;
    }
  }
  __syncthreads();
  if (!*last) return;
  // the last arriver: thread (lane, c4) sums partials lane, lane + lanes, ... of channel group c4 with
  // BR_TAIL loads in flight (one round for every C3 layer), then the lanes are tree-summed
  f4 s[BR_TAIL];
#pragma unroll
  for (int u = 0; u < BR_TAIL; ++u) s[u] = f4{0.f, 0.f, 0.f, 0.f};
  for (int w0 = lane; w0 < nb; w0 += BR_TAIL * lanes) {
    f4 v[BR_TAIL];
#pragma unroll
    for (int u = 0; u < BR_TAIL; ++u) {  // past nb: num_records bounds the resource, the load returns 0
      const int w = w0 + u * lanes;
      v[u] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(prs, (w * C + 4 * c4) * 4, 0, BR_SC1));
    }
#pragma unroll
    for (int u = 0; u < BR_TAIL; ++u)
      if (w0 + u * lanes < nb) s[u] += v[u];
  }
#pragma unroll
  for (int h = BR_TAIL / 2; h >= 1; h /= 2)
#pragma unroll
    for (int u = 0; u < h; ++u) s[u] += s[u + h];
  part[tid] = s[0];
  __syncthreads();
  lane_tree_sum(part, lane, C4, lanes);
  if (tid < C4) {
    const f4 t = part[tid];
#pragma unroll
    for (int q = 0; q < 4; ++q) db[4 * tid + q] = accumulate ? db0[q] + t[q] : t[q];
  }
  if (tid == 0) __hip_atomic_store(counter, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-armed
}

__device__ __forceinline__ void br_load_db(const float* db, int accumulate, int C4, float* db0) {
  if (accumulate && (int)threadIdx.x < C4) {  // db read now: the last arriver's update is then one store
#pragma unroll
    for (int q = 0; q < 4; ++q) db0[q] = db[4 * threadIdx.x + q];
  }
}

__global__ __launch_bounds__(BR_THREADS) void bias_relu_bwd_kernel(const f4* __restrict__ dy, const f4* __restrict__ y,
                                                                  int C4, int64_t rows, int64_t rows_per_block,
                                                                  f4* __restrict__ dx, float* partial,
                                                                  int* counter, float* __restrict__ db,
                                                                  int accumulate) {
  __shared__ f4 part[BR_THREADS];
  __shared__ int last;
  const int tid = threadIdx.x;
  const int lanes = BR_THREADS / C4;  // row lanes; C4 divides 256
  const int c4 = tid % C4, lane = tid / C4;
  const int64_t r0 = blockIdx.x * rows_per_block;
  const int64_t r1 = min(rows, r0 + rows_per_block);
  float db0[4] = {0.f, 0.f, 0.f, 0.f};
  br_load_db(db, accumulate, C4, db0);
  f4 acc = f4{0.f, 0.f, 0.f, 0.f};
  for (int64_t r = r0 + lane; r < r1; r += (int64_t)lanes * BR_UNROLL) {
    f4 g[BR_UNROLL], yv[BR_UNROLL];
#pragma unroll
    for (int u = 0; u < BR_UNROLL; ++u) {
      const int64_t rr = r + (int64_t)u * lanes;
      const int64_t i = (rr < r1 ? rr : r) * C4 + c4;
      g[u] = dy[i];
      yv[u] = y[i];
    }
#pragma unroll
    for (int u = 0; u < BR_UNROLL; ++u) {
      const int64_t rr = r + (int64_t)u * lanes;
      if (rr < r1) {
        f4 o;
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = yv[u][q] <= 0.f ? 0.f : g[u][q];
        dx[rr * C4 + c4] = o;
        acc += o;
      }
    }
  }
  part[tid] = acc;
  __syncthreads();
  lane_tree_sum(part, lane, C4, lanes);
  br_finish(part[tid], part, &last, partial, counter, db, db0, accumulate, C4);
}

// ---- the flattening layer's epilogue (NatureCNN conv3 -> Flatten -> Linear) ---------------------
// nn.Flatten after a channels_last convolution flattens in NCHW order (c, h, w), so torch copies the
// NHWC activation into that order before the fc GEMM and copies the fc's input gradient back to NHWC
// for the convolution's backward: two layout copies per minibatch (19 us per C3 minibatch, r2x
// stats).  These two kernels do the transposes inside the bias + ReLU passes instead:
//   forward   out[b, c * HW + p] = relu(x[b, p, c] + bias[c])      (x NHWC, out flat NCHW)
//   backward  dx[b, p, c] = y[b, c * HW + p] > 0 ? dy[b, c * HW + p] : 0   (dx NHWC), db as above
// Workgroup w handles samples w, w + G, ...: the sample's HW x C plane is staged in LDS with rows of
// C + 1 floats (the transposed reads walk 65-float strides: conflict-free) so that both the global
// reads and the global writes are contiguous.  Needs (C + 1) * HW <= BRT_MAX_ELEMS.
constexpr int BRT_MAX_ELEMS = 8192;  // (C + 1) * HW floats of LDS: 32 KB

__global__ __launch_bounds__(BR_THREADS) void bias_relu_fwd_nchw_kernel(const float* __restrict__ x,
                                                                       const float* __restrict__ b, int64_t B, int HW,
                                                                       int C, float* __restrict__ out) {
  __shared__ float t[BRT_MAX_ELEMS];
  const int n = HW * C, ld = C + 1;
  for (int64_t s = blockIdx.x; s < B; s += gridDim.x) {
    const float* xs = x + s * n;
    for (int m = threadIdx.x; m < n; m += BR_THREADS) {  // NHWC element m = p * C + c
      const int p = m / C, c = m - p * C;
      const float v = xs[m] + b[c];
      t[p * ld + c] = v < 0.f ? 0.f : v;
    }
    __syncthreads();
    float* os = out + s * n;
    for (int e = threadIdx.x; e < n; e += BR_THREADS) {  // NCHW element e = c * HW + p
      const int c = e / HW, p = e - c * HW;
      os[e] = t[p * ld + c];
    }
    __syncthreads();
  }
}

// VEC (round 4, 16-B aligned dy / y): the sample's NCHW plane is read as float4s, all of a thread's loads
// issued before the first use (one memory round trip per sample instead of one per loop trip), and the
// channel of element e is e * ceil(2^32 / HW) >> 32 (exact for e < 8192) instead of an integer division.
template <bool VEC = false>
__global__ __launch_bounds__(BR_THREADS) void bias_relu_bwd_nchw_kernel(const float* __restrict__ dy,
                                                                       const float* __restrict__ y, int64_t B, int HW,
                                                                       int C, float* __restrict__ dx, float* partial,
                                                                       int* counter, float* __restrict__ db,
                                                                       int accumulate) {
  __shared__ float t[BRT_MAX_ELEMS];
  __shared__ f4 part[BR_THREADS];
  __shared__ int last;
  const int tid = threadIdx.x, C4 = C / 4, lanes = BR_THREADS / C4, c4 = tid % C4, lane = tid / C4;
  const int n = HW * C, ld = C + 1;
  const unsigned magic = (unsigned)((0x100000000ULL + (unsigned)HW - 1) / (unsigned)HW);
  float db0[4] = {0.f, 0.f, 0.f, 0.f};
  br_load_db(db, accumulate, C4, db0);
  f4 wsum = f4{0.f, 0.f, 0.f, 0.f};  // thread tid < C4: this workgroup's samples, in sample order
  for (int64_t s = blockIdx.x; s < B; s += gridDim.x) {
    const float* dys = dy + s * n;
    const float* ys = y + s * n;
    if (VEC) {
      constexpr int NV = BRT_MAX_ELEMS / 4 / BR_THREADS;  // float4s per thread at most
      const int n4 = n >> 2;
      f4 yv[NV], gv[NV];
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int m4 = tid + i * BR_THREADS;
        if (m4 < n4) {
          yv[i] = reinterpret_cast<const f4*>(ys)[m4];
          gv[i] = reinterpret_cast<const f4*>(dys)[m4];
        }
      }
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int m4 = tid + i * BR_THREADS;
        if (m4 < n4) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {  // NCHW element e = c * HW + p
            const unsigned e = 4u * (unsigned)m4 + q;
            const int c = (int)__umulhi(e, magic), p = (int)e - c * HW;
            t[p * ld + c] = yv[i][q] <= 0.f ? 0.f : gv[i][q];
          }
        }
      }
    } else {
      for (int e = tid; e < n; e += BR_THREADS) {  // NCHW element e = c * HW + p
        const int c = e / HW, p = e - c * HW;
        t[p * ld + c] = ys[e] <= 0.f ? 0.f : dys[e];
      }
    }
    __syncthreads();
    float* dxs = dx + s * n;
    for (int m4 = tid; m4 < n / 4; m4 += BR_THREADS) {  // NHWC float4 m4: pixel p, channels 4 q .. 4 q + 3
      const int p = m4 / C4, q = m4 - p * C4;
      const float* r = t + p * ld + 4 * q;
      reinterpret_cast<f4*>(dxs)[m4] = f4{r[0], r[1], r[2], r[3]};
    }
    f4 acc = f4{0.f, 0.f, 0.f, 0.f};  // thread (lane, c4): pixels lane, lane + lanes, ...
    for (int p = lane; p < HW; p += lanes) {
      const float* r = t + p * ld + 4 * c4;
      acc += f4{r[0], r[1], r[2], r[3]};
    }
    part[tid] = acc;
    __syncthreads();
    lane_tree_sum(part, lane, C4, lanes);
    if (tid < C4) wsum += part[tid];
    __syncthreads();  // t and part are rewritten by the next sample
  }
  br_finish(wsum, part, &last, partial, counter, db, db0, accumulate, C4);
}

bool br_shape_ok(int64_t rows, int32_t C) {
  if (rows < 0 || C < 4 || C % 4) return false;
  const int C4 = C / 4;
  return C4 <= BR_THREADS && BR_THREADS % C4 == 0;
}
}  // namespace

extern "C" int64_t rai_bias_relu_workspace_bytes(int32_t C) {
  return (int64_t)BR_MAX_BLOCKS * (C > 0 ? C : 0) * 4 + BR_CTR_BYTES;  // partials, then the arrival counters
}

extern "C" int rai_bias_relu_fwd(const float* x, const float* b, int64_t rows, int32_t C, float* out, void* stream) {
  if (!br_shape_ok(rows, C)) return RAI_E_SHAPE;
  if (rows == 0) return RAI_OK;
  if (!x || !b || !out) return RAI_E_NULLPTR;
  const int64_t n4 = rows * (C / 4);
  hipLaunchKernelGGL(bias_relu_fwd_kernel, dim3((unsigned)ew_blocks(n4)), dim3(BR_THREADS), 0, rai_stream(stream),
                     reinterpret_cast<const f4*>(x), b, C / 4, n4, reinterpret_cast<f4*>(out));
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}

static bool brt_shape_ok(int64_t B, int32_t HW, int32_t C) {
  return B >= 0 && HW >= 1 && br_shape_ok(1, C) && (int64_t)(C + 1) * HW <= BRT_MAX_ELEMS;
}

extern "C" int rai_bias_relu_fwd_nchw(const float* x, const float* b, int64_t B, int32_t HW, int32_t C, float* out,
                                      void* stream) {
  if (!brt_shape_ok(B, HW, C)) return RAI_E_SHAPE;
  if (B == 0) return RAI_OK;
  if (!x || !b || !out) return RAI_E_NULLPTR;
  const int64_t blocks = B < 1024 ? B : 1024;
  hipLaunchKernelGGL(bias_relu_fwd_nchw_kernel, dim3((unsigned)blocks), dim3(BR_THREADS), 0, rai_stream(stream), x, b,
                     B, HW, C, out);
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}

extern "C" int rai_bias_relu_bwd_nchw(const float* dy, const float* y, int64_t B, int32_t HW, int32_t C, float* dx,
                                      float* db, int32_t accumulate, void* workspace, int64_t workspace_bytes,
                                      void* stream) {
  if (!brt_shape_ok(B, HW, C)) return RAI_E_SHAPE;
  if (!dy || !y || !dx || !db || !workspace) return RAI_E_NULLPTR;
  if (workspace_bytes < rai_bias_relu_workspace_bytes(C) || ((uintptr_t)workspace & 15) || ((uintptr_t)dx & 15))
    return RAI_E_WORKSPACE;
  hipStream_t st = rai_stream(stream);
  if (B == 0) {
    if (!accumulate) {
      const hipError_t e = hipMemsetAsync(db, 0, (size_t)C * 4, st);
      if (e != hipSuccess) return (int)e;
    }
    return RAI_OK;
  }
  const int64_t blocks = B < BR_MAX_BLOCKS ? B : BR_MAX_BLOCKS;
  float* partial = static_cast<float*>(workspace);
  int* counter = reinterpret_cast<int*>(static_cast<uint8_t*>(workspace) + (int64_t)BR_MAX_BLOCKS * C * 4);
  const char* bv = getenv("RAI_BRT_VEC");  // A/B: 0 keeps the scalar form
  if ((((uintptr_t)dy | (uintptr_t)y) & 15) == 0 && !(bv && bv[0] == '0'))
    hipLaunchKernelGGL(bias_relu_bwd_nchw_kernel<true>, dim3((unsigned)blocks), dim3(BR_THREADS), 0, st, dy, y, B, HW,
                       C, dx, partial, counter, db, accumulate);
  else
    hipLaunchKernelGGL(bias_relu_bwd_nchw_kernel<false>, dim3((unsigned)blocks), dim3(BR_THREADS), 0, st, dy, y, B,
                       HW, C, dx, partial, counter, db, accumulate);
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}

extern "C" int rai_bias_relu_bwd(const float* dy, const float* y, int64_t rows, int32_t C, float* dx, float* db,
                                 int32_t accumulate, void* workspace, int64_t workspace_bytes, void* stream) {
  if (!br_shape_ok(rows, C)) return RAI_E_SHAPE;
  if (!dy || !y || !dx || !db || !workspace) return RAI_E_NULLPTR;
  if (workspace_bytes < rai_bias_relu_workspace_bytes(C) || ((uintptr_t)workspace & 15)) return RAI_E_WORKSPACE;
  hipStream_t st = rai_stream(stream);
  if (rows == 0) {
    if (!accumulate) {
      const hipError_t e = hipMemsetAsync(db, 0, (size_t)C * 4, st);
      if (e != hipSuccess) return (int)e;
    }
    return RAI_OK;
  }
  const int C4 = C / 4, lanes = BR_THREADS / C4;
  // ~BR_ROWS_PER_LANE rows per row lane, at most BR_MAX_BLOCKS workgroups
  int64_t blocks = (rows + (int64_t)BR_ROWS_PER_LANE * lanes - 1) / ((int64_t)BR_ROWS_PER_LANE * lanes);
  if (blocks > BR_MAX_BLOCKS) blocks = BR_MAX_BLOCKS;
  if (blocks < 1) blocks = 1;
  const int64_t rpb = (rows + blocks - 1) / blocks;
  blocks = (rows + rpb - 1) / rpb;
  float* partial = static_cast<float*>(workspace);
  int* counter = reinterpret_cast<int*>(static_cast<uint8_t*>(workspace) + (int64_t)BR_MAX_BLOCKS * C * 4);
  hipLaunchKernelGGL(bias_relu_bwd_kernel, dim3((unsigned)blocks), dim3(BR_THREADS), 0, st,
                     reinterpret_cast<const f4*>(dy), reinterpret_cast<const f4*>(y), C4, rows, rpb,
                     reinterpret_cast<f4*>(dx), partial, counter, db, accumulate);
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}
