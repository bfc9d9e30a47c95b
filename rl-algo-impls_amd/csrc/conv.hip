// NatureCNN convolutions (config C3) as hand-written f32 MFMA implicit GEMMs on gfx950.
//
// Reference: rl_algo_impls/shared/encoder/nature_cnn.py:31-41 (Conv2d 8x8/4, 4x4/2, 3x3/1, each
// followed by ReLU) and cnn.py:24-27; the bias + ReLU of the reference's Conv2d -> ReLU pair is the
// store epilogue here, so one launch replaces MIOpen's convolution plus rai_bias_relu_fwd.
//
// Layouts (what the C3 trainer already holds in HBM): activations NHWC fp32 (the minibatch gather
// writes obs / 255 as NHWC), weights channels_last [Co][KH][KW][Ci] (optim.FlatParams stores the
// conv weights that way), bias [Co].  Output NHWC [B][OH][OW][Co], or, for the layer nn.Flatten
// follows, the NCHW-flattened (B, Co*OH*OW) that Linear consumes.
//
// GEMM view: y^T[co][p] = sum_k W[co][k] * im2col(x)[p][k], k = (kh, kw, ci) -- the order of both
// the NHWC input and the channels_last weight, so 4 consecutive k (Ci % 4 == 0) are one 16-B load
// of either operand.  v_mfma_f32_16x16x4f32 takes lane (i, g) = (lane % 16, lane / 16) as row i of A
// and column i of B at reduction index g.  A "quad" is 16 consecutive k = 4 chunks of 4: lane group g
// loads chunk 4*quad + g of its weight row (A) and of its pixel's im2col row (B) as float4, and the
// quad's four MFMAs take component j of both -- every k pairs the same weight and input element, so
// the products are exact f32 and only the summation order differs from MIOpen's (fp32 tolerance).
// The chunk -> im2col offset table (independent of the pixel) sits in LDS.
//
// The output of one MFMA is co rows 4g..4g+3 at pixel column i: a lane adds the bias, applies the
// ReLU (t < 0 ? 0 : t, NaN kept, as rai_bias_relu_fwd) and stores one float4 of the NHWC row.
//
// Blocking: a wave computes TCO x TPX 16x16 output blocks (co x pixels); per quad it loads TCO + TPX
// float4 and issues 4 * TCO * TPX MFMAs.  Operands are read straight from global memory (L1/L2:
// the weights are shared by every workgroup, overlapping receptive fields re-read the same lines),
// two quads in flight per wave.
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <unordered_map>
#include <unordered_set>

#include "common.h"

namespace {

typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int CV_THREADS = 256;
constexpr int CV_MAXCHUNK = 2048;  // K <= 8192

struct ConvFwdArgs {
  const float* x;
  const uint8_t* xu8;  // U8 forms: the uint8 NHWC input (Ci = 4), read as x = u8 / xdiv
  float xdiv;
  float xinv;          // U8 == 2: the rounded 1 / xdiv of the multiply + fma-correction quotient
  const float* w;
  const float* b;
  float* y;
  int64_t M;  // B * OH * OW output pixels
  int H, W, Ci, Co, KW, S, OH, OW, K;
  // split-K (conv_fwd_lds_kernel only): blockIdx.z takes quads [nq z / ksplit, nq (z + 1) / ksplit) of the
  // reduction and, with ksplit > 1, stores its raw partial sums to part[z][p][co] (no bias / ReLU);
  // conv_fwd_splitk_reduce_kernel then adds the splits in order, the bias and the ReLU
  int ksplit = 1;
  float* part = nullptr;
  int xcd_map = 0;  // conv_fwd_lds_kernel: the co tiles of one pixel-tile stream on ONE XCD (fwd_tile)
};

// The uint8 forms' x = u / d for the four bytes of a dword.  U8 == 1: a 256-entry LDS table of the IEEE
// quotients (four dependent, bank-conflicting LDS reads per dword).  U8 == 2: the quotient q0 = u * inv
// corrected by one fused multiply-add step, q = q0 + (u - q0 d) inv (two FMAs, exact residual) — four
// VALU operations per byte and no LDS; the host launches it only when u8_div_valu_exact(d) has
// checked it equal, bit for bit, to u / d for all 256 bytes (true for d = 255).
__device__ __forceinline__ f4 u8x4_div(unsigned u, float d, float inv) {
#ifdef RAI_U8_FAKE_CVT  // diagnostic builds only (wrong values): the dword operand path without the quotient
  return f4{__uint_as_float(u), __uint_as_float(u >> 8), __uint_as_float(u >> 16), __uint_as_float(u >> 24)};
#endif
  // packed-fp32 pairs (v_pk_mul_f32 / v_pk_fma_f32: two lanes' worth per VALU op, per-element IEEE results
  // identical to the scalar ops the host check runs)
  typedef float f2v __attribute__((ext_vector_type(2)));
  const f2v iv = {inv, inv}, dv = {d, d};
  const f2v x01 = {(float)(u & 255u), (float)((u >> 8) & 255u)};
  const f2v x23 = {(float)((u >> 16) & 255u), (float)(u >> 24)};
  const f2v q01 = x01 * iv, q23 = x23 * iv;
  const f2v r01 = __builtin_elementwise_fma(__builtin_elementwise_fma(-q01, dv, x01), iv, q01);
  const f2v r23 = __builtin_elementwise_fma(__builtin_elementwise_fma(-q23, dv, x23), iv, q23);
  return f4{r01.x, r01.y, r23.x, r23.y};
}

// host: does the U8 == 2 quotient equal the IEEE u / d for every byte?  (RAI_CONV_U8_LUT=1: the table)
static bool u8_div_valu_exact(float d, float* inv_out) {
  const char* e = getenv("RAI_CONV_U8_LUT");  // read per launch (the tests switch it in-process)
  if ((e && e[0] == '1') || !(d > 0.f)) return false;
  const float inv = 1.f / d;
  for (int i = 0; i < 256; ++i) {
    const float x = (float)i;
    volatile float q0 = x * inv;  // a rounded product, as the device's v_mul_f32
    const float q = std::fmaf(std::fmaf(-q0, d, x), inv, q0);
    const float ref = x / d;
    if (__builtin_bit_cast(uint32_t, q) != __builtin_bit_cast(uint32_t, ref)) return false;
  }
  *inv_out = inv;
  return true;
}

template <int TCO, int TPX, int WCO, int WPX, bool NCHW, int PF>
__global__ __launch_bounds__(CV_THREADS) void conv_fwd_kernel(const ConvFwdArgs a) {
  static_assert(WCO * WPX == CV_THREADS / 64, "four waves");
  __shared__ int xoff[CV_MAXCHUNK];
  const int nch = a.K >> 2;
  for (int q = threadIdx.x; q < nch; q += CV_THREADS) {
    const int k = 4 * q, kpos = k / a.Ci, ci0 = k - kpos * a.Ci, kh = kpos / a.KW, kw = kpos - kh * a.KW;
    xoff[q] = (kh * a.W + kw) * a.Ci + ci0;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int wco = wv % WCO, wpx = wv / WCO;
  const int64_t px0 = (int64_t)blockIdx.x * (16 * TPX * WPX) + 16 * TPX * wpx;
  const int co0 = blockIdx.y * (16 * TCO * WCO) + 16 * TCO * wco;
  const int OHW = a.OH * a.OW;

  const float* xb[TPX];
#pragma unroll
  for (int tp = 0; tp < TPX; ++tp) {
    int64_t p = px0 + 16 * tp + li;
    p = p < a.M ? p : a.M - 1;
    const int64_t n = p / OHW;
    const int r = (int)(p - n * OHW), oh = r / a.OW, ow = r - oh * a.OW;
    xb[tp] = a.x + ((n * a.H + (int64_t)oh * a.S) * a.W + (int64_t)ow * a.S) * a.Ci;
  }
  const float* wb[TCO];
#pragma unroll
  for (int tc = 0; tc < TCO; ++tc) wb[tc] = a.w + (int64_t)(co0 + 16 * tc + li) * a.K;

  f4 acc[TCO][TPX];
#pragma unroll
  for (int tc = 0; tc < TCO; ++tc)
#pragma unroll
    for (int tp = 0; tp < TPX; ++tp) acc[tc][tp] = f4{0.f, 0.f, 0.f, 0.f};

  auto load = [&](int qd, f4(&A)[TCO], f4(&Bv)[TPX]) {
    const int q = 4 * qd + g;
    const int xo = xoff[q];
#pragma unroll
    for (int tc = 0; tc < TCO; ++tc) A[tc] = *reinterpret_cast<const f4*>(wb[tc] + 4 * q);
#pragma unroll
    for (int tp = 0; tp < TPX; ++tp) Bv[tp] = *reinterpret_cast<const f4*>(xb[tp] + xo);
  };
  auto mma = [&](const f4(&A)[TCO], const f4(&Bv)[TPX]) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int tc = 0; tc < TCO; ++tc)
#pragma unroll
        for (int tp = 0; tp < TPX; ++tp)
          acc[tc][tp] = __builtin_amdgcn_mfma_f32_16x16x4f32(A[tc][j], Bv[tp][j], acc[tc][tp], 0, 0, 0);
  };

  const int nq = nch >> 2;  // quads (host guarantees K % 32 == 0)
  f4 Ar[PF][TCO], Br[PF][TPX];
#pragma unroll
  for (int u = 0; u < PF; ++u)
    if (u < nq) load(u, Ar[u], Br[u]);
  for (int qd = 0; qd < nq; qd += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      if (qd + u < nq) mma(Ar[u], Br[u]);
      if (qd + u + PF < nq) load(qd + u + PF, Ar[u], Br[u]);
    }
  }

#pragma unroll
  for (int tc = 0; tc < TCO; ++tc) {
    const int co = co0 + 16 * tc + 4 * g;
    const f4 bv = *reinterpret_cast<const f4*>(a.b + co);
#pragma unroll
    for (int tp = 0; tp < TPX; ++tp) {
      const int64_t p = px0 + 16 * tp + li;
      if (p >= a.M) continue;
      f4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float t = acc[tc][tp][r] + bv[r];
        v[r] = t < 0.f ? 0.f : t;
      }
      if (!NCHW) {
        *reinterpret_cast<f4*>(a.y + p * a.Co + co) = v;
      } else {
        const int64_t n = p / OHW;
        float* yb = a.y + n * (int64_t)a.Co * OHW + (p - n * OHW) + (int64_t)co * OHW;
#pragma unroll
        for (int r = 0; r < 4; ++r) yb[(int64_t)r * OHW] = v[r];
      }
    }
  }
}

// Compute units of the current device (256 on MI355X), queried once per device.
static int num_cus() {
  static std::mutex mu;
  static std::unordered_map<int, int> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  std::lock_guard<std::mutex> lock(mu);
  auto it = cache.find(dev);
  if (it != cache.end()) return it->second;
  int n = 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 1) n = 256;
  cache[dev] = n;
  return n;
}

// Raise a kernel's dynamic-LDS limit to the 160 KB of a CU (minus its static LDS) once per kernel (a host call; not repeated per
// launch, so a graph-captured or eager step pays it only on its first launch).
static int allow_lds(const void* kernel) {
  static std::mutex mu;
  static std::unordered_set<const void*> done;
  std::lock_guard<std::mutex> lock(mu);
  if (done.count(kernel)) return RAI_OK;
  hipFuncAttributes fa;
  hipError_t e = hipFuncGetAttributes(&fa, kernel);
  if (e != hipSuccess) return (int)e;
  e = hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - (int)fa.sharedSizeBytes);
  if (e != hipSuccess) return (int)e;
  done.insert(kernel);
  return RAI_OK;
}

// The same forward with the workgroup's weight rows resident in LDS: a persistent workgroup (8 waves,
// one per CU) copies its COT rows x K once (row stride K + 4 floats: the 16 lanes of a ds_read_b128
// group land on distinct banks), then loops over pixel tiles; only the im2col operand is read from
// L1/L2 per quad.
template <int TCO, int TPX, int WCO, int WPX, bool NCHW, int PF, bool BUF = false, int U8 = 0>
__global__ __launch_bounds__(512) void conv_fwd_lds_kernel(const ConvFwdArgs a) {
  static_assert(WCO * WPX == 8, "eight waves");
  static_assert(!U8 || BUF, "the uint8 input is read through a buffer resource");
  constexpr int COT = 16 * TCO * WCO, PXT = 16 * TPX * WPX;
  extern __shared__ __attribute__((aligned(16))) float wl[];  // [COT][K + 4]
  __shared__ int xoff[CV_MAXCHUNK];
  __shared__ float lut[U8 == 1 ? 256 : 1];  // U8 == 1: lut[u] = u / xdiv (IEEE division, as the gather's prescale)
  if (U8 == 1)
    for (int i = threadIdx.x; i < 256; i += 512) lut[i] = (float)i / a.xdiv;
  const int K = a.K;
  // this split's chunk range [c0, c0 + nch) of the K / 4 chunks, in whole quads
  const int zs = blockIdx.z, nq_all = K >> 4;
  const int q0 = (int)((int64_t)nq_all * zs / a.ksplit), q1 = (int)((int64_t)nq_all * (zs + 1) / a.ksplit);
  const int c0 = 4 * q0, nch = 4 * (q1 - q0), KP = 4 * nch + 4;
  // (pixel-tile stream, co tile) of this workgroup.  The workgroups of one stream read the same input
  // pixels; dispatch deals consecutive workgroups round-robin over the 8 XCDs (speed only, never
  // correctness), so with the natural order and a stream count that is not a multiple of 8 (conv2 at
  // B = 256: 81) the co tiles of a stream sit on different XCDs and each fetches the pixels past its L2.
  // xcd_map (host: gridDim.x a multiple of 8): workgroup lin keeps XCD slot lin % 8, and the gridDim.y co
  // tiles of stream 8 (lin / 8 / cot) + lin % 8 are consecutive slots of that XCD.
  int sx = (int)blockIdx.x, sy = (int)blockIdx.y;
  if (a.xcd_map) {
    const int lin = (int)(blockIdx.x + blockIdx.y * gridDim.x), slot = lin >> 3, cot = (int)gridDim.y;
    sx = 8 * (slot / cot) + (lin & 7);
    sy = slot % cot;
  }
  const int co_wg = sy * COT;
  for (int q = threadIdx.x; q < nch; q += 512) {
    const int k = 4 * (c0 + q), kpos = k / a.Ci, ci0 = k - kpos * a.Ci, kh = kpos / a.KW, kw = kpos - kh * a.KW;
    xoff[q] = (kh * a.W + kw) * a.Ci + ci0;
  }
  for (int e = threadIdx.x; e < COT * nch; e += 512) {
    const int r = e / nch, q = e - r * nch;
    *reinterpret_cast<f4*>(wl + r * KP + 4 * q) =
        *reinterpret_cast<const f4*>(a.w + (int64_t)(co_wg + r) * K + 4 * (c0 + q));
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int wco = wv % WCO, wpx = wv / WCO;
  const int OHW = a.OH * a.OW;
  const float* wrow[TCO];
#pragma unroll
  for (int tc = 0; tc < TCO; ++tc) wrow[tc] = wl + (16 * (TCO * wco + tc) + li) * KP;
  const int64_t ntiles = (a.M + PXT - 1) / PXT;
  const int nq = nch >> 2;
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      U8 ? (void*)const_cast<uint8_t*>(a.xu8) : (void*)const_cast<float*>(a.x), 0,
      BUF ? (int)((a.M / (a.OH * a.OW)) * a.H * a.W * a.Ci * (U8 ? 1 : 4)) : 0, 0x00020000);
  for (int64_t tile = sx; tile < ntiles; tile += gridDim.x) {
    const int64_t px0 = tile * PXT + 16 * TPX * wpx;
    const float* xb[TPX];
    int xbo[TPX];  // BUF: the same base as an element offset into x (host: x < 2 GB)
#pragma unroll
    for (int tp = 0; tp < TPX; ++tp) {
      int64_t p = px0 + 16 * tp + li;
      p = p < a.M ? p : a.M - 1;
      const int64_t n = p / OHW;
      const int r = (int)(p - n * OHW), oh = r / a.OW, ow = r - oh * a.OW;
      const int64_t base = ((n * a.H + (int64_t)oh * a.S) * a.W + (int64_t)ow * a.S) * a.Ci;
      xb[tp] = a.x + base;
      xbo[tp] = (int)base;
    }
    f4 acc[TCO][TPX];
#pragma unroll
    for (int tc = 0; tc < TCO; ++tc)
#pragma unroll
      for (int tp = 0; tp < TPX; ++tp) acc[tc][tp] = f4{0.f, 0.f, 0.f, 0.f};
    f4 Br[PF][TPX];
    unsigned Ur[U8 ? PF : 1][TPX];  // U8: the raw dwords, converted when the stage is consumed (no early wait)
    auto ldb = [&](int qd, int slot) {
      f4(&Bv)[TPX] = Br[slot];
      const int xo = xoff[4 * qd + g];
      if (U8) {  // one pixel's 4 channels per chunk (Ci = 4): one dword
#pragma unroll
        for (int tp = 0; tp < TPX; ++tp) Ur[slot][tp] = __builtin_amdgcn_raw_buffer_load_b32(xrs, xbo[tp] + xo, 0, 0);
        return;
      }
      if (BUF) {
#pragma unroll
        for (int tp = 0; tp < TPX; ++tp)
          Bv[tp] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(xrs, 4 * (xbo[tp] + xo), 0, 0));
        return;
      }
#pragma unroll
      for (int tp = 0; tp < TPX; ++tp) Bv[tp] = *reinterpret_cast<const f4*>(xb[tp] + xo);
    };
    // BUF: every ring load is issued (a chunk index past the end re-reads the last chunk, an L1 hit), so
    // the loop's loads are straight-line code and each wait leaves the PF - 1 younger stages in flight
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      if (BUF || u < nq) ldb(BUF ? min(u, nq - 1) : u, u);
      __builtin_amdgcn_sched_barrier(0);
    }
    auto stage = [&](int q, int u) {  // chunk quad q from ring slot u
      if (U8) {
#pragma unroll
        for (int tp = 0; tp < TPX; ++tp) {
          const unsigned w4 = Ur[u][tp];
          if (U8 == 2) Br[u][tp] = u8x4_div(w4, a.xdiv, a.xinv);
          else Br[u][tp] = f4{lut[w4 & 255u], lut[(w4 >> 8) & 255u], lut[(w4 >> 16) & 255u], lut[w4 >> 24]};
        }
      }
      f4 A[TCO];
#pragma unroll
      for (int tc = 0; tc < TCO; ++tc) A[tc] = *reinterpret_cast<const f4*>(wrow[tc] + 4 * (4 * q + g));
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int tc = 0; tc < TCO; ++tc)
#pragma unroll
          for (int tp = 0; tp < TPX; ++tp)
            acc[tc][tp] = __builtin_amdgcn_mfma_f32_16x16x4f32(A[tc][j], Br[u][tp][j], acc[tc][tp], 0, 0, 0);
    };
    if (BUF) {  // full PF blocks as straight-line code (stages interleave), then the remainder
      int qd = 0;
      for (; qd + PF <= nq; qd += PF) {
#pragma unroll
        for (int u = 0; u < PF; ++u) {
          stage(qd + u, u);
          ldb(min(qd + u + PF, nq - 1), u);
          __builtin_amdgcn_sched_barrier(0);  // slot u's reload right behind its MFMAs, not clustered at the end
        }
      }
#pragma unroll
      for (int u = 0; u < PF; ++u)
        if (qd + u < nq) stage(qd + u, u);
    } else {
      for (int qd = 0; qd < nq; qd += PF) {
#pragma unroll
        for (int u = 0; u < PF; ++u) {
          if (qd + u < nq) stage(qd + u, u);
          if (qd + u + PF < nq) ldb(qd + u + PF, u);
        }
      }
    }
    if (a.ksplit > 1) {  // raw partial sums of this split, [z][p][co]
#pragma unroll
      for (int tc = 0; tc < TCO; ++tc) {
        const int co = co_wg + 16 * (TCO * wco + tc) + 4 * g;
#pragma unroll
        for (int tp = 0; tp < TPX; ++tp) {
          const int64_t p = px0 + 16 * tp + li;
          if (p < a.M) *reinterpret_cast<f4*>(a.part + ((int64_t)zs * a.M + p) * a.Co + co) = acc[tc][tp];
        }
      }
      continue;
    }
#pragma unroll
    for (int tc = 0; tc < TCO; ++tc) {
      const int co = co_wg + 16 * (TCO * wco + tc) + 4 * g;
      const f4 bv = *reinterpret_cast<const f4*>(a.b + co);
#pragma unroll
      for (int tp = 0; tp < TPX; ++tp) {
        const int64_t p = px0 + 16 * tp + li;
        if (p >= a.M) continue;
        f4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float t = acc[tc][tp][r] + bv[r];
          v[r] = t < 0.f ? 0.f : t;
        }
        if (!NCHW) {
          *reinterpret_cast<f4*>(a.y + p * a.Co + co) = v;
        } else {
          const int64_t n = p / OHW;
          float* yb = a.y + n * (int64_t)a.Co * OHW + (p - n * OHW) + (int64_t)co * OHW;
#pragma unroll
          for (int r = 0; r < 4; ++r) yb[(int64_t)r * OHW] = v[r];
        }
      }
    }
  }
}

template <int TCO, int TPX, int WCO, int WPX, int PF, bool BUF = false, int U8 = 0>
int launch_fwd_lds(const ConvFwdArgs& a, bool nchw, hipStream_t st) {
  constexpr int PXT = 16 * TPX * WPX, COT = 16 * TCO * WCO;
  if (a.Co % COT) return RAI_E_SHAPE;
  if (BUF && (a.M / ((int64_t)a.OH * a.OW)) * a.H * a.W * a.Ci * (U8 ? 1 : 4) >= (1LL << 31)) return RAI_E_SHAPE;
  const int nq_all = a.K >> 4, ks = a.ksplit < 1 ? 1 : a.ksplit;
  if (ks > 1 && (!a.part || ks > nq_all)) return RAI_E_SHAPE;
  const int ksplit_k = 16 * ((nq_all + ks - 1) / ks);  // the largest split's K
  const size_t lds = (size_t)COT * (ksplit_k + 4) * sizeof(float);
  if (lds + CV_MAXCHUNK * 4 > 160 * 1024) return RAI_E_SHAPE;
  const int64_t ntiles = (a.M + PXT - 1) / PXT;
  const int64_t cot = a.Co / COT;
  // persistent workgroups: two per CU for the small-K layer (conv1: 33 KB of weight rows; every
  // instantiation stays under 128 VGPRs), so its 400 tiles at B = 256 run as one round of co-resident
  // workgroups instead of two rounds of one: conv1 23.8 vs 25.5 us (u8 26.9 vs 27.9) at B = 256, 68.1 vs
  // 76.8 us at 1,024.  Not for the 66-75 KB layers: conv2 at B = 1,024 took 73.0 vs 59.8 us with two
  // (profiles/r5l_conv_bench_*.txt).  RAI_CONV_FWD_WPC=1 / 2 forces one / two.
  const char* we = getenv("RAI_CONV_FWD_WPC");
  const int wpc = (we && !strcmp(we, "1")) ? 1 : (we && !strcmp(we, "2")) ? 2 : (lds <= 40 * 1024 ? 2 : 1);
  int64_t gx = (int64_t)wpc * num_cus() / cot;  // per split
  if (gx > ntiles) gx = ntiles;
  if (gx < 1) gx = 1;
  // XCD-aware stream order (conv_fwd_lds_kernel): gx rounded up to a multiple of 8 (a stream past the
  // tiles runs no iteration).  RAI_CONV_FWD_XCD=0 keeps the natural order (A/B)
  static const int env_xcd = [] {
    const char* e = getenv("RAI_CONV_FWD_XCD");
    return e ? atoi(e) : 1;
  }();
  ConvFwdArgs ax = a;
  if (env_xcd != 0 && cot > 1) {
    gx = (gx + 7) / 8 * 8;
    ax.xcd_map = 1;
  }
  const dim3 grid((unsigned)gx, (unsigned)cot, (unsigned)ks);
  if (nchw) {
    auto k = conv_fwd_lds_kernel<TCO, TPX, WCO, WPX, true, PF, BUF, U8>;
    const int e = allow_lds(reinterpret_cast<const void*>(k));
    if (e != RAI_OK) return e;
    hipLaunchKernelGGL(k, grid, dim3(512), lds, st, ax);
  } else {
    auto k = conv_fwd_lds_kernel<TCO, TPX, WCO, WPX, false, PF, BUF, U8>;
    const int e = allow_lds(reinterpret_cast<const void*>(k));
    if (e != RAI_OK) return e;
    hipLaunchKernelGGL(k, grid, dim3(512), lds, st, ax);
  }
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}

template <int TCO, int TPX, int WCO, int WPX, int PF = 2>
int launch_fwd(const ConvFwdArgs& a, bool nchw, hipStream_t st) {
  constexpr int PXT = 16 * TPX * WPX, COT = 16 * TCO * WCO;
  if (a.Co % COT) return RAI_E_SHAPE;
  const int64_t gx = (a.M + PXT - 1) / PXT;
  if (gx > 0x7fffffffLL) return RAI_E_SHAPE;
  const dim3 grid((unsigned)gx, (unsigned)(a.Co / COT));
  if (nchw)
    hipLaunchKernelGGL((conv_fwd_kernel<TCO, TPX, WCO, WPX, true, PF>), grid, dim3(CV_THREADS), 0, st, a);
  else
    hipLaunchKernelGGL((conv_fwd_kernel<TCO, TPX, WCO, WPX, false, PF>), grid, dim3(CV_THREADS), 0, st, a);
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}

// Split-K forward's second pass: y = ReLU(sum over the splits in order of part[z] + b).  NHWC output: one
// float4 of 4 channels per thread (the partials' own layout).  NCHW output (the layer nn.Flatten follows):
// one workgroup per image, the image's OH*OW x Co tile summed into LDS, then written in the flattened
// (co, oh, ow) order, coalesced both ways.
constexpr int CV_RED_NCHW_MAX = 8192;  // floats of one image's output tile in LDS
__global__ __launch_bounds__(256) void conv_fwd_splitk_reduce_kernel(const float* __restrict__ part, int S, int64_t M,
                                                                     int Co, const float* __restrict__ b, float* y,
                                                                     int nchw, int OHW) {
  if (!nchw) {
    const int64_t n4 = M * Co / 4;
    const f4* p4 = reinterpret_cast<const f4*>(part);
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
      f4 v = p4[i];
      for (int z = 1; z < S; ++z) v += p4[z * n4 + i];
      const f4 bv = *reinterpret_cast<const f4*>(b + (int)((4 * i) % Co));
      f4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float t = v[r] + bv[r];
        o[r] = t < 0.f ? 0.f : t;
      }
      reinterpret_cast<f4*>(y)[i] = o;
    }
    return;
  }
  __shared__ float t[CV_RED_NCHW_MAX];
  const int64_t n = blockIdx.x;
  const int e4 = OHW * Co / 4;
  const f4* p4 = reinterpret_cast<const f4*>(part + n * OHW * Co);
  const int64_t zs4 = M * Co / 4;
  for (int i = threadIdx.x; i < e4; i += 256) {  // [r][co] order, 4 channels per thread
    f4 v = p4[i];
    for (int z = 1; z < S; ++z) v += p4[z * zs4 + i];
    const int r = (4 * i) / Co, co = (4 * i) - r * Co;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float tt = v[q] + b[co + q];
      t[(co + q) * OHW + r] = tt < 0.f ? 0.f : tt;
    }
  }
  __syncthreads();
  float* yn = y + n * OHW * Co;
  for (int i = threadIdx.x; i < OHW * Co; i += 256) yn[i] = t[i];
}

// ---------------------------------------------------------------------------------------------
// Weight gradient: dW[co][k] = sum_p dz[p][co] * im2col(x)[p][k] (the reduction runs over the
// B * OH * OW output pixels).  MFMA rows = co, columns = k, reduction index = pixel.  The 4-wide
// trick runs along the OUTPUT dimensions here: lane (i, g) loads VC consecutive co of dz at pixel
// p_g (VC = 4: 16 B) and 4 consecutive k of x's im2col row (16 B).  MFMA (j, j') takes component j of
// the first and j' of the second, so it accumulates the 16 x 16 block of co = VC*i + j, k = k0 + 4i + j':
// one pixel step (4 pixels) is 4 * VC MFMAs fed by two loads per lane.  A wave owns all Co = 16 * VC
// output channels x one 64-wide k tile (grid.y); the workgroup's four waves split its pixels (each
// 256-pixel chunk: 64 per wave) and add their tiles through LDS in wave order; grid.x splits the
// pixels over workgroups.  Every workgroup writes one partial tile; conv_wrw_reduce sums the S splits
// in a fixed order (deterministic, no atomics) and writes or adds dW (accumulate: straight into the
// flat .grad).
constexpr int WR_MAXPX = 8192;  // pixels per split (their base offsets sit in LDS)

struct ConvWrwArgs {
  const float* x;
  const uint8_t* xu8;  // U8 forms: uint8 NHWC input (Ci = 4), x = u8 / xdiv
  float xdiv;
  float xinv;          // U8 == 2: the rounded 1 / xdiv (see u8x4_div)
  const float* dz;  // RB: dy, the gradient of the ReLU's output
  const float* y;   // RB: the forward output (dz = y > 0 ? dy : 0, as threshold_backward)
  float* part;      // [S][Co][K], then (RB) the bias-gradient partials [S][Co]
  int64_t M;    // pixels
  int64_t per;  // pixels per split
  int H, W, Ci, Co, KW, S_, OH, OW, K;
  int xcd_map;  // 1: the k tiles of one pixel split run back to back on ONE XCD (see wrw_tile)
};

// The (pixel split, k tile) a workgroup works on.  Dispatch deals consecutive workgroups round-robin over the
// 8 XCDs (MI355X_MICROARCH.md, workgroup dispatch: blocks b and b + 8 share one; speed only, never
// correctness).  With the grid's natural order the KT k tiles of split s are dispatched S workgroups apart,
// so each reads the split's dz / y rows (and its input rows) from beyond its XCD's L2 again.  xcd_map
// renumbers: workgroup lin -> XCD slot lin % 8 keeps split s = 8 (slot / KT) + lin % 8, k tile slot % KT, so
// a split's k tiles are dispatched consecutively on the same XCD and the later ones read its rows from L2.
struct WrwTile {
  int s, kt;
};
__device__ __forceinline__ WrwTile wrw_tile(int xcd_map) {
  if (!xcd_map) return WrwTile{(int)blockIdx.x, (int)blockIdx.y};
  const int lin = (int)(blockIdx.x + blockIdx.y * gridDim.x);
  const int slot = lin >> 3, KT = (int)gridDim.y;
  return WrwTile{8 * (slot / KT) + (lin & 7), slot % KT};
}

template <int VC, int PF, bool RB, bool BUF = false, int U8 = 0>
__global__ __launch_bounds__(CV_THREADS) void conv_wrw_kernel(const ConvWrwArgs a) {
  static_assert(!U8 || BUF, "the uint8 input is read through a buffer resource");
  constexpr int NB = VC * 4;  // 16x16 accumulator blocks per wave
  __shared__ float dbl[RB ? 4 * 16 * VC : 1];  // RB: the waves' bias-gradient sums
  __shared__ float lut[U8 == 1 ? 256 : 1];     // U8 == 1: lut[u] = u / xdiv
  if (U8 == 1) lut[threadIdx.x] = (float)threadIdx.x / a.xdiv;  // CV_THREADS == 256
  // LDS: the split's pixel -> input offset table, later reused for the cross-wave sum of the tiles
  constexpr int TAB_BYTES = WR_MAXPX * 4, RED_BYTES = 3 * NB * 64 * 16;
  __shared__ __attribute__((aligned(16))) unsigned char lds[TAB_BYTES > RED_BYTES ? TAB_BYTES : RED_BYTES];
  int* const xbase_l = reinterpret_cast<int*>(lds);
  f4* const red = reinterpret_cast<f4*>(lds);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int li = lane & 15, g = lane >> 4;
  const WrwTile tile = wrw_tile(a.xcd_map);
  const int k0 = tile.kt * 64 + 4 * li;  // this lane's 4 k (one chunk: Ci % 4 == 0)
  int xo;
  {
    const int kpos = k0 / a.Ci, ci0 = k0 - kpos * a.Ci, kh = kpos / a.KW, kw = kpos - kh * a.KW;
    xo = (kh * a.W + kw) * a.Ci + ci0;
  }
  const int64_t pbeg = (int64_t)tile.s * a.per;
  const int n_p = (int)max((int64_t)0, min(a.per, a.M - pbeg));
  const int OHW = a.OH * a.OW;
  const int64_t n0 = pbeg / OHW;  // offsets are relative to the split's first sample
  for (int t = threadIdx.x; t < n_p; t += CV_THREADS) {
    const int64_t p = pbeg + t;
    const int64_t n = p / OHW;
    const int r = (int)(p - n * OHW), oh = r / a.OW, ow = r - oh * a.OW;
    xbase_l[t] = (int)((((n - n0) * a.H + (int64_t)oh * a.S_) * a.W + (int64_t)ow * a.S_) * a.Ci);
  }
  __syncthreads();
  typedef float fv __attribute__((ext_vector_type(VC)));
  f4 acc[VC][4];
#pragma unroll
  for (int j = 0; j < VC; ++j)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) acc[j][jj] = f4{0.f, 0.f, 0.f, 0.f};
  {
    // wave w: the split's pixels [lo, hi), in steps of 4 (lane group g: pixel lo + 4 st + g)
    const int q4 = (((n_p + 3) >> 2) + 3) >> 2;  // steps per wave
    const int lo = min(4 * q4 * wv, n_p), hi = min(lo + 4 * q4, n_p);
    const float* xc = a.x + n0 * (int64_t)a.H * a.W * a.Ci + xo;
    const float* dzc = a.dz + pbeg * a.Co + VC * li;
    const float* yc = RB ? a.y + pbeg * a.Co + VC * li : nullptr;
    const int nst = (hi - lo + 3) >> 2;
    // BUF: 32-bit element offsets into buffer resources (host: x, dz < 2 GB) instead of 64-bit pointers
    const int dzo = (int)(pbeg * a.Co) + VC * li, xco = (int)(n0 * a.H * a.W * a.Ci) + xo;
    const __amdgpu_buffer_rsrc_t zrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.dz), 0,
                                                                         BUF ? (int)(a.M * a.Co * 4) : 0, 0x00020000);
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(RB ? a.y : a.dz), 0,
                                                                         BUF ? (int)(a.M * a.Co * 4) : 0, 0x00020000);
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
        U8 ? (void*)const_cast<uint8_t*>(a.xu8) : (void*)const_cast<float*>(a.x), 0,
        BUF ? (int)((a.M / (a.OH * a.OW)) * a.H * a.W * a.Ci * (U8 ? 1 : 4)) : 0, 0x00020000);
    auto ldz = [&](const __amdgpu_buffer_rsrc_t& rs, int off) -> fv {
      if constexpr (VC == 4) return __builtin_bit_cast(fv, __builtin_amdgcn_raw_buffer_load_b128(rs, 4 * off, 0, 0));
      else return __builtin_bit_cast(fv, __builtin_amdgcn_raw_buffer_load_b64(rs, 4 * off, 0, 0));
    };
    // the PF-deep ring holds the loads as they arrive (raw dz, y, the uint8 dword): the ReLU mask and the
    // byte conversion are applied when a step is consumed, so no load is waited for PF - 1 steps early
    fv dv[PF];
    fv yv[RB ? PF : 1];
    f4 xv[PF];
    unsigned xu[U8 ? PF : 1];
    auto ld = [&](int st, int u) {
      const int pl = lo + 4 * st + g;
      if (BUF) {
        // unconditional, so the loop's loads are straight-line code and each wait leaves the PF - 1 younger
        // steps in flight: a lane past the wave's pixels re-reads its last pixel (an L1 hit), zeroed when
        // consumed
        const int plc = min(min(pl, max(hi - 1, lo)), WR_MAXPX - 1);
        dv[u] = ldz(zrs, dzo + plc * a.Co);
        if (RB) yv[u] = ldz(yrs, dzo + plc * a.Co);
        if (U8) xu[u] = __builtin_amdgcn_raw_buffer_load_b32(xrs, xco + xbase_l[plc], 0, 0);
        else xv[u] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(xrs, 4 * (xco + xbase_l[plc]), 0, 0));
      } else if (pl < hi) {
        dv[u] = *reinterpret_cast<const fv*>(dzc + (int64_t)pl * a.Co);
        if (RB) yv[u] = *reinterpret_cast<const fv*>(yc + (int64_t)pl * a.Co);
        xv[u] = *reinterpret_cast<const f4*>(xc + xbase_l[pl]);
      } else {
        dv[u] = fv{};
        if (RB) yv[u] = fv{};
        if (U8) xu[u] = 0u;
        else xv[u] = f4{0.f, 0.f, 0.f, 0.f};
      }
    };
    auto mma = [&](const fv& dv, const f4& xv) {
#pragma unroll
      for (int j = 0; j < VC; ++j)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          acc[j][jj] = __builtin_amdgcn_mfma_f32_16x16x4f32(dv[j], xv[jj], acc[j][jj], 0, 0, 0);
    };
    fv dsum = fv{};  // RB: this lane's bias-gradient sum (its pixels, in step order)
    // prologue loads in slot order (the scheduler may not interleave them): the loop-entry wait state then
    // matches the back edge's, and each step waits for its own slot only
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      ld(u, u);
      __builtin_amdgcn_sched_barrier(0);
    }
    auto step = [&](int sq, int u) {  // pixel step sq from ring slot u
      fv d = dv[u];
      if (RB) {
#pragma unroll
        for (int j = 0; j < VC; ++j) d[j] = yv[u][j] > 0.f ? d[j] : 0.f;
      }
      f4 x;
      if (U8 == 2) x = u8x4_div(xu[u], a.xdiv, a.xinv);
      else if (U8 == 1) x = f4{lut[xu[u] & 255u], lut[(xu[u] >> 8) & 255u], lut[(xu[u] >> 16) & 255u], lut[xu[u] >> 24]};
      else x = xv[u];
      if (BUF && lo + 4 * sq + g >= hi) {  // past the wave's pixels: zero, as the pointer form loads
        d = fv{};
        x = f4{0.f, 0.f, 0.f, 0.f};
      }
      mma(d, x);
      if (RB) dsum += d;
    };
    if (BUF) {  // full PF blocks as straight-line code (steps interleave), then the remainder
      int st = 0;
      for (; st + PF <= nst; st += PF) {
#pragma unroll
        for (int u = 0; u < PF; ++u) {
          step(st + u, u);
          ld(st + u + PF, u);
          __builtin_amdgcn_sched_barrier(0);  // slot u's reload right behind its MFMAs, not clustered at the end
        }
      }
#pragma unroll
      for (int u = 0; u < PF; ++u)
        if (st + u < nst) step(st + u, u);
    } else {
      for (int st = 0; st < nst; st += PF) {
#pragma unroll
        for (int u = 0; u < PF; ++u) {
          if (st + u < nst) step(st + u, u);
          if (st + u + PF < nst) ld(st + u + PF, u);
        }
      }
    }
    if (RB) {  // the four lane groups (rows of the step), then the waves in order through LDS
#pragma unroll
      for (int j = 0; j < VC; ++j) {
        float v = dsum[j];
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        if (g == 0) dbl[(wv * 16 + li) * VC + j] = v;
      }
    }
  }
  __syncthreads();  // the table's last readers are done: its LDS becomes the reduction buffer
  // the four waves' tiles, added in wave order
  if (wv > 0) {
#pragma unroll
    for (int j = 0; j < VC; ++j)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) red[((wv - 1) * NB + j * 4 + jj) * 64 + lane] = acc[j][jj];
  }
  __syncthreads();
  if (wv > 0) return;
  if (RB && tile.kt == 0 && g == 0) {  // this split's bias-gradient partial (one k tile writes it)
    float* dp = a.part + (int64_t)gridDim.x * a.Co * a.K + (int64_t)tile.s * a.Co;
#pragma unroll
    for (int j = 0; j < VC; ++j) {
      float v = dbl[li * VC + j];
#pragma unroll
      for (int q = 1; q < 4; ++q) v += dbl[(q * 16 + li) * VC + j];
      dp[VC * li + j] = v;
    }
  }
#pragma unroll
  for (int q = 0; q < 3; ++q)
#pragma unroll
    for (int j = 0; j < VC; ++j)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) acc[j][jj] += red[(q * NB + j * 4 + jj) * 64 + lane];
  // partial tile: lane (i, g) holds co = VC*(4g + r) + j, k = k0 .. k0 + 3 (one float4 per (j, r))
  float* pp = a.part + (int64_t)tile.s * a.Co * a.K;
#pragma unroll
  for (int j = 0; j < VC; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = VC * (4 * g + r) + j;
      *reinterpret_cast<f4*>(pp + (int64_t)co * a.K + k0) = f4{acc[j][0][r], acc[j][1][r], acc[j][2][r], acc[j][3][r]};
    }
}

// dW (+)= sum over s of part[s] (fixed order: 16 lane groups each add S / 16 consecutive splits, then
// the 16 group sums are added in group order through LDS).  One launch serves up to RAI_WGRAD_MAX_JOBS
// layers (the backward's convolutions, reduced together once the backward has ended): block b works
// on the job whose block range holds it.
struct WrwReduceJob {
  const f4* part;
  f4* dw;
  int64_t n4;
  int S;
  int blk0;  // first block of this job
};
struct WrwReduceArgs {
  WrwReduceJob j[2 * RAI_WGRAD_MAX_JOBS];  // a layer with a bias gradient is two jobs
  int n;
  int accumulate;
};

__global__ __launch_bounds__(CV_THREADS) void conv_wrw_reduce_kernel(const WrwReduceArgs a) {
  __shared__ f4 red[16][16];
  int jb = 0;
#pragma unroll
  for (int q = 1; q < 2 * RAI_WGRAD_MAX_JOBS; ++q)
    if (q < a.n && (int)blockIdx.x >= a.j[q].blk0) jb = q;
  const f4* __restrict__ part = a.j[jb].part;
  f4* __restrict__ dw = a.j[jb].dw;
  const int64_t n4 = a.j[jb].n4;
  const int S = a.j[jb].S;
  const int o = threadIdx.x & 15, sg = threadIdx.x >> 4;
  const int64_t i = (int64_t)(blockIdx.x - a.j[jb].blk0) * 16 + o;
  const int per = S >> 4;
  f4 s = f4{0.f, 0.f, 0.f, 0.f};
  if (i < n4) {
    f4 v[8];
    for (int b = 0; b < per; b += 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u)
        v[u] = b + u < per ? part[(int64_t)(sg * per + b + u) * n4 + i] : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
  }
  red[sg][o] = s;
  __syncthreads();
  if (sg == 0 && i < n4) {
    f4 t = red[0][o];
#pragma unroll
    for (int q = 1; q < 16; ++q) t += red[q][o];
    dw[i] = a.accumulate ? dw[i] + t : t;
  }
}

struct WrwPlan {
  int VC, S, KT;
  int64_t per;
};

// target_wgs workgroups in all (default 512: two per CU), S a multiple of 16, each split at most
// WR_MAXPX pixels and at least 64
static WrwPlan wrw_plan(int64_t M, int Co, int K, int target_wgs) {
  WrwPlan p;
  p.VC = Co / 16;
  p.KT = K / 64;  // k tiles (grid.y)
  // default: 512 workgroups (measured best of 256 / 512 / 768 / 1024 at B = 256, r3r), 1024 for K <= 256
  // (NatureCNN conv1: 26.5 vs 28.6 us at B = 256, 71.3 vs 84.4 at B = 1024; profiles/r4g_conv_bench.txt)
  static const int env_wgs = [] {  // A/B: RAI_WRW_WGS=512 restores the single default (read once)
    const char* e = getenv("RAI_WRW_WGS");
    return e ? atoi(e) : 0;
  }();
  if (target_wgs <= 0) target_wgs = env_wgs > 0 && env_wgs <= 1024 ? env_wgs : (K <= 256 ? 1024 : 512);
  int64_t S = target_wgs / p.KT;
  S = S < 16 ? 16 : (S / 16) * 16;
  while (S > 16 && (M + S - 1) / S < 64) S -= 16;
  while ((M + S - 1) / S > WR_MAXPX) S += 16;
  p.S = (int)S;
  p.per = (M + S - 1) / S;
  return p;
}

// ---------------------------------------------------------------------------------------------
// Input gradient (the dx of Conv2d's autograd backward; conv2 / conv3 of NatureCNN, whose inputs
// need gradients): dx[n][ih][iw][ci] = sum over taps (kh, kw) with oh = (ih - kh) / S, ow = (iw - kw) / S
// integral and in range, and over co, of dz[n][oh][ow][co] * W[co][kh][kw][ci].  Input pixels are
// grouped into S x S classes (ih % S, iw % S): every pixel of a class sees the same taps
// kh = ih % S + S * th (th < KH / S), so a column block of 16 same-class pixels shares the A operand.
// MFMA rows = ci, columns = input pixels, reduction = (tap, co).  Both 4-wide tricks: lane (i, g)
// loads VC consecutive ci of W at co = c0 + 4g + m (m = 0..3: four loads) and 4 consecutive co of dz
// at its pixel's output position (one float4 per column block); MFMA (m, j) takes W component j of
// load m and dz component m, accumulating rows ci = VC * i + j.  A wave owns all Ci = 16 * VC rows x
// TQ column blocks; invalid taps (outside the output) load zeros.  Every dx element is written once
// (no split, no zero-fill, deterministic).
struct ConvDgradArgs {
  const float* dz;  // (B, OH, OW, Co); with a ReLU folded in: dy, the gradient of the ReLU's output
  const float* y;   // ReLU folded in: the forward output (dz = y > 0 ? dz : 0), else unused
  const float* w;   // (Co, KH, KW, Ci)
  float* dx;        // (B, H, W, Ci)
  int64_t B;
  int H, W, Ci, Co, KH, KW, S, OH, OW;
};

template <int VC, int TQ>
__global__ __launch_bounds__(CV_THREADS) void conv_dgrad_kernel(const ConvDgradArgs a) {
  typedef float fv __attribute__((ext_vector_type(VC)));
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int cls = blockIdx.y, ph = cls / a.S, pw = cls - ph * a.S;
  const int Hc = (a.H - ph + a.S - 1) / a.S, Wc = (a.W - pw + a.S - 1) / a.S;  // this class's grid
  const int64_t ncls = a.B * Hc * Wc;
  const int TH = a.KH / a.S, TW = a.KW / a.S;
  int64_t pix[TQ];   // this lane's class pixel per column block (clamped), -1 past the end
  int ihc[TQ], iwc[TQ];
  int64_t dzb[TQ];   // dz pixel index of tap (0, 0)
#pragma unroll
  for (int tq = 0; tq < TQ; ++tq) {
    const int64_t c = (int64_t)blockIdx.x * (64 * TQ) + (int64_t)(wv * TQ + tq) * 16 + li;
    const int64_t cc = c < ncls ? c : ncls - 1;
    pix[tq] = c < ncls ? c : -1;
    const int64_t n = cc / (Hc * Wc);
    const int r = (int)(cc - n * Hc * Wc);
    ihc[tq] = r / Wc;
    iwc[tq] = r - ihc[tq] * Wc;
    dzb[tq] = (n * a.OH + ihc[tq]) * a.OW + iwc[tq];
  }
  f4 acc[VC][TQ];
#pragma unroll
  for (int j = 0; j < VC; ++j)
#pragma unroll
    for (int tq = 0; tq < TQ; ++tq) acc[j][tq] = f4{0.f, 0.f, 0.f, 0.f};
  const int ncc = a.Co >> 4;
  const int nsteps = TH * TW * ncc;  // (tap, 16-co chunk) steps
  auto ld = [&](int stp, fv (&A)[4], f4 (&Bv)[TQ]) {
    const int t = stp / ncc, c0 = (stp - t * ncc) * 16;
    const int th = t / TW, tw = t - th * TW;
    const int kh = ph + a.S * th, kw = pw + a.S * tw;
    const float* wp = a.w + ((int64_t)((c0 + 4 * g) * a.KH + kh) * a.KW + kw) * a.Ci + VC * li;
    const int64_t wco = (int64_t)a.KH * a.KW * a.Ci;  // one co further
#pragma unroll
    for (int m = 0; m < 4; ++m) A[m] = *reinterpret_cast<const fv*>(wp + m * wco);
#pragma unroll
    for (int tq = 0; tq < TQ; ++tq) {
      const int oh = ihc[tq] - th, ow = iwc[tq] - tw;
      if (pix[tq] >= 0 && oh >= 0 && oh < a.OH && ow >= 0 && ow < a.OW)
        Bv[tq] = *reinterpret_cast<const f4*>(a.dz + (dzb[tq] - (int64_t)th * a.OW - tw) * a.Co + c0 + 4 * g);
      else
        Bv[tq] = f4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto mma = [&](const fv (&A)[4], const f4 (&Bv)[TQ]) {
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int j = 0; j < VC; ++j)
#pragma unroll
        for (int tq = 0; tq < TQ; ++tq)
          acc[j][tq] = __builtin_amdgcn_mfma_f32_16x16x4f32(A[m][j], Bv[tq][m], acc[j][tq], 0, 0, 0);
  };
  constexpr int PF = 2;
  fv A[PF][4];
  f4 Bv[PF][TQ];
#pragma unroll
  for (int u = 0; u < PF; ++u)
    if (u < nsteps) ld(u, A[u], Bv[u]);
  for (int st = 0; st < nsteps; st += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      if (st + u < nsteps) mma(A[u], Bv[u]);
      if (st + u + PF < nsteps) ld(st + u + PF, A[u], Bv[u]);
    }
  }
  // lane (i, g), block tq: rows ci = VC * (4g + r) + j for pixel column i -> VC consecutive ci per r
#pragma unroll
  for (int tq = 0; tq < TQ; ++tq) {
    if (pix[tq] < 0) continue;
    const int64_t n = pix[tq] / (Hc * Wc);
    const int ih = ph + a.S * ihc[tq], iw = pw + a.S * iwc[tq];
    float* dp = a.dx + ((n * a.H + ih) * a.W + iw) * a.Ci;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      fv v;
#pragma unroll
      for (int j = 0; j < VC; ++j) v[j] = acc[j][tq][r];
      *reinterpret_cast<fv*>(dp + VC * (4 * g + r)) = v;
    }
  }
}

// The input gradient with the whole weight tensor resident in LDS (<= ~150 KB: NatureCNN conv2 128 KB,
// conv3 147 KB), persistent 8-wave workgroups looping over (class, pixel tile) work items: only dz is
// read from L1/L2 per step.  Waves split the rows (WCI groups of 16 * VC ci) and the pixel blocks.
template <int VC, int TQ, int WCI>
__global__ __launch_bounds__(512) void conv_dgrad_lds_kernel(const ConvDgradArgs a) {
  typedef float fv __attribute__((ext_vector_type(VC)));
  constexpr int WQ = 8 / WCI;             // waves along pixels
  constexpr int PXT = 16 * TQ * WQ;       // pixels per work item
  extern __shared__ __attribute__((aligned(16))) float wl[];  // (Co, KH, KW, Ci)
  const int64_t wn = (int64_t)a.Co * a.KH * a.KW * a.Ci;
  for (int64_t e = threadIdx.x; e < wn / 4; e += 512)
    reinterpret_cast<f4*>(wl)[e] = reinterpret_cast<const f4*>(a.w)[e];
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int wci = wv % WCI, wq = wv / WCI;
  const int ci0 = 16 * VC * wci;
  const int TH = a.KH / a.S, TW = a.KW / a.S;
  const int ncc = a.Co >> 4;
  const int nsteps = TH * TW * ncc;
  const int wco = a.KH * a.KW * a.Ci;
  // work items: class-major, tiles of PXT pixels of the class
  const int Hc0 = (a.H + a.S - 1) / a.S, Wc0 = (a.W + a.S - 1) / a.S;
  const int64_t tiles_per_cls = (a.B * Hc0 * Wc0 + PXT - 1) / PXT;
  const int64_t nitems = tiles_per_cls * a.S * a.S;
  for (int64_t item = blockIdx.x; item < nitems; item += gridDim.x) {
    const int cls = (int)(item / tiles_per_cls);
    const int64_t tile = item - (int64_t)cls * tiles_per_cls;
    const int ph = cls / a.S, pw = cls - ph * a.S;
    const int Hc = (a.H - ph + a.S - 1) / a.S, Wc = (a.W - pw + a.S - 1) / a.S;
    const int64_t ncls = a.B * Hc * Wc;
    if (tile * PXT >= ncls) continue;  // uniform over the workgroup
    int64_t pix[TQ];
    int ihc[TQ], iwc[TQ];
    int64_t dzb[TQ];
#pragma unroll
    for (int tq = 0; tq < TQ; ++tq) {
      const int64_t c = tile * PXT + (int64_t)(wq * TQ + tq) * 16 + li;
      const int64_t cc = c < ncls ? c : ncls - 1;
      pix[tq] = c < ncls ? c : -1;
      const int64_t n = cc / (Hc * Wc);
      const int r = (int)(cc - n * Hc * Wc);
      ihc[tq] = r / Wc;
      iwc[tq] = r - ihc[tq] * Wc;
      dzb[tq] = (n * a.OH + ihc[tq]) * a.OW + iwc[tq];
    }
    f4 acc[VC][TQ];
#pragma unroll
    for (int j = 0; j < VC; ++j)
#pragma unroll
      for (int tq = 0; tq < TQ; ++tq) acc[j][tq] = f4{0.f, 0.f, 0.f, 0.f};
    auto ldb = [&](int stp, f4 (&Bv)[TQ]) {
      const int t = stp / ncc, c0 = (stp - t * ncc) * 16;
      const int th = t / TW, tw = t - th * TW;
#pragma unroll
      for (int tq = 0; tq < TQ; ++tq) {
        const int oh = ihc[tq] - th, ow = iwc[tq] - tw;
        if (pix[tq] >= 0 && oh >= 0 && oh < a.OH && ow >= 0 && ow < a.OW)
          Bv[tq] = *reinterpret_cast<const f4*>(a.dz + (dzb[tq] - (int64_t)th * a.OW - tw) * a.Co + c0 + 4 * g);
        else
          Bv[tq] = f4{0.f, 0.f, 0.f, 0.f};
      }
    };
    constexpr int PF = 3;
    f4 Bv[PF][TQ];
#pragma unroll
    for (int u = 0; u < PF; ++u)
      if (u < nsteps) ldb(u, Bv[u]);
    for (int st = 0; st < nsteps; st += PF) {
#pragma unroll
      for (int u = 0; u < PF; ++u) {
        if (st + u < nsteps) {
          const int stp = st + u;
          const int t = stp / ncc, c0 = (stp - t * ncc) * 16;
          const int th = t / TW, tw = t - th * TW;
          const int kh = ph + a.S * th, kw = pw + a.S * tw;
          const float* wp = wl + ((c0 + 4 * g) * a.KH + kh) * a.KW * a.Ci + kw * a.Ci + ci0 + VC * li;
          fv A[4];
#pragma unroll
          for (int m = 0; m < 4; ++m) A[m] = *reinterpret_cast<const fv*>(wp + m * wco);
#pragma unroll
          for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int j = 0; j < VC; ++j)
#pragma unroll
              for (int tq = 0; tq < TQ; ++tq)
                acc[j][tq] = __builtin_amdgcn_mfma_f32_16x16x4f32(A[m][j], Bv[u][tq][m], acc[j][tq], 0, 0, 0);
        }
        if (st + u + PF < nsteps) ldb(st + u + PF, Bv[u]);
      }
    }
#pragma unroll
    for (int tq = 0; tq < TQ; ++tq) {
      if (pix[tq] < 0) continue;
      const int64_t n = pix[tq] / (Hc * Wc);
      const int ih = ph + a.S * ihc[tq], iw = pw + a.S * iwc[tq];
      float* dp = a.dx + ((n * a.H + ih) * a.W + iw) * a.Ci + ci0;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        fv v;
#pragma unroll
        for (int j = 0; j < VC; ++j) v[j] = acc[j][tq][r];
        *reinterpret_cast<fv*>(dp + VC * (4 * g + r)) = v;
      }
    }
  }
}

template <int VC, int TQ, int WCI>
int launch_dgrad_lds(const ConvDgradArgs& a, hipStream_t st) {
  const size_t lds = (size_t)a.Co * a.KH * a.KW * a.Ci * sizeof(float);
  if (lds > 160 * 1024 || 16 * VC * WCI != a.Ci) return RAI_E_SHAPE;
  constexpr int PXT = 16 * TQ * (8 / WCI);
  const int64_t Hc0 = (a.H + a.S - 1) / a.S, Wc0 = (a.W + a.S - 1) / a.S;
  const int64_t nitems = (a.B * Hc0 * Wc0 + PXT - 1) / PXT * a.S * a.S;
  const int64_t gx = nitems < num_cus() ? nitems : num_cus();
  auto k = conv_dgrad_lds_kernel<VC, TQ, WCI>;
  const int e = allow_lds(reinterpret_cast<const void*>(k));
  if (e != RAI_OK) return e;
  hipLaunchKernelGGL(k, dim3((unsigned)gx), dim3(512), lds, st, a);
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}

// The input gradient per IMAGE, as a GEMM over the image's output pixels followed by col2im in LDS
// (round 4).  For image n: dxc[(tap, ci)][p] = sum_co W[co][tap][ci] * dz[n][p][co] over the OH*OW
// output pixels p -- every (pixel, tap) product lands inside the input (no border taps computed as
// zeros, unlike the pixel-class form above) -- then dx[n][p*S + tap] += dxc, summed over the taps in
// a fixed (kh, kw) order.  The workgroup's waves own disjoint (16-ci block, tap-parity class (kh % S,
// kw % S)) pairs: a class's taps write only input pixels of that parity, so no two waves touch the same
// dx element and one wave's adds run in program order -- deterministic without atomics or barriers.
// MFMA rows = ci, columns = output pixels, reduction = co (16 per quad, the 4-wide trick along co: one
// float4 of dz per lane, four strided W loads per tap); a wave holds TC taps x MT pixel tiles of
// accumulators.  The image's dx is assembled in LDS (pixel stride Ci + 4 floats: the 16 pixel lanes of
// an add land on distinct banks) and written once, coalesced.  NatureCNN: conv2 (4x4/2, 64 -> 32 ch,
// 9x9 -> 20x20) = 8 waves x 4 taps x 6 tiles, conv3 (3x3/1, 64 -> 64, 7x7 -> 9x9) = 4 waves x 9 x 4.
template <int TC, int MT, int NT, int PF, bool BUF = false, bool RELU = false>
__global__ __launch_bounds__(NT) void conv_dgrad_img_kernel(const ConvDgradArgs a) {
  extern __shared__ __attribute__((aligned(16))) float dxl[];  // [H * W][Ci + 4]
  const int n = blockIdx.x;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int NCB = a.Ci >> 4;
  const int cb = wv % NCB, cls = wv / NCB;
  const int ph = cls / a.S, pw = cls - ph * a.S;
  const int TW = a.KW / a.S;
  const int CP = a.Ci + 4;
  const int HW = a.H * a.W, OHW = a.OH * a.OW;
  for (int e = threadIdx.x; e < HW * CP / 4; e += NT) reinterpret_cast<f4*>(dxl)[e] = f4{0.f, 0.f, 0.f, 0.f};
  const float* dzn = a.dz + (int64_t)n * OHW * a.Co;
  const int64_t wco = (int64_t)a.KH * a.KW * a.Ci;  // W stride of one co
  int woff[TC];
#pragma unroll
  for (int t = 0; t < TC; ++t) {
    const int th = t / TW, tw = t - th * TW;
    woff[t] = ((ph + a.S * th) * a.KW + pw + a.S * tw) * a.Ci + 16 * cb + li;
  }
  int poff[MT];
  bool pv[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int p = 16 * mt + li;
    pv[mt] = p < OHW;
    poff[mt] = (pv[mt] ? p : 0) * a.Co;
  }
  f4 acc[TC][MT];
#pragma unroll
  for (int t = 0; t < TC; ++t)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[t][mt] = f4{0.f, 0.f, 0.f, 0.f};
  // BUF: buffer loads with the lane-invariant part of every offset in a scalar register (no per-load
  // 64-bit address arithmetic); a masked pixel's offset points past the image's dz, which reads 0
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.w), 0,
                                                                       (int)(a.Co * wco * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t drs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(dzn), 0,
                                                                       OHW * a.Co * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(RELU ? a.y + (int64_t)n * OHW * a.Co : dzn), 0, OHW * a.Co * 4, 0x00020000);
  int wvo[TC], dvo[MT];
#pragma unroll
  for (int t = 0; t < TC; ++t) wvo[t] = 4 * (int)(4 * g * wco + woff[t]);
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) dvo[mt] = pv[mt] ? 4 * (poff[mt] + 4 * g) : OHW * a.Co * 4;
  auto load = [&](int q, float (&Wv)[TC][4], f4 (&Dv)[MT]) {
    if (BUF) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int so = 4 * (int)((16 * q + j) * wco);
#pragma unroll
        for (int t = 0; t < TC; ++t) Wv[t][j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(wrs, wvo[t], so, 0));
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        Dv[mt] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(drs, dvo[mt], 64 * q, 0));
        if (RELU) {  // threshold_backward on the saved output: dz = y > 0 ? dy : 0
          const f4 yv = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(yrs, dvo[mt], 64 * q, 0));
#pragma unroll
          for (int j = 0; j < 4; ++j) Dv[mt][j] = yv[j] > 0.f ? Dv[mt][j] : 0.f;
        }
      }
      return;
    }
    const int co0 = 4 * (4 * q + g);
    const float* wq = a.w + (int64_t)co0 * wco;
#pragma unroll
    for (int t = 0; t < TC; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) Wv[t][j] = wq[j * wco + woff[t]];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
      Dv[mt] = pv[mt] ? *reinterpret_cast<const f4*>(dzn + poff[mt] + co0) : f4{0.f, 0.f, 0.f, 0.f};
  };
  const int nq = a.Co >> 4;
  float Wv[PF][TC][4];
  f4 Dv[PF][MT];
#pragma unroll
  for (int u = 0; u < PF; ++u)
    if (u < nq) load(u, Wv[u], Dv[u]);
  for (int q = 0; q < nq; q += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      if (q + u < nq) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int t = 0; t < TC; ++t)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
              acc[t][mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(Wv[u][t][j], Dv[u][mt][j], acc[t][mt], 0, 0, 0);
      }
      if (q + u + PF < nq) load(q + u + PF, Wv[u], Dv[u]);
    }
  }
  __syncthreads();  // LDS zeroed by every thread
  // col2im: lane (i, g) holds ci rows 16 cb + 4g .. +3 of output pixel p = 16 mt + i; taps in order
  int pbase[MT];  // this lane's dx LDS offset of tap (0, 0) per pixel tile
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int p = 16 * mt + li;
    const int oh = p / a.OW, ow = p - oh * a.OW;
    pbase[mt] = ((oh * a.S + ph) * a.W + ow * a.S + pw) * CP + 16 * cb + 4 * g;
  }
#pragma unroll
  for (int t = 0; t < TC; ++t) {
    const int th = t / TW, tw = t - th * TW;
    const int toff = (a.S * th * a.W + a.S * tw) * CP;
#ifdef RAI_DGRAD_BATCH_COL2IM
    // one tap's tiles touch distinct dx pixels: all their reads, then the adds, then the writes (one LDS
    // round trip per tap instead of one per tile)
    f4 cur[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
      if (pv[mt]) cur[mt] = *reinterpret_cast<const f4*>(dxl + pbase[mt] + toff);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
      if (pv[mt]) *reinterpret_cast<f4*>(dxl + pbase[mt] + toff) = cur[mt] + acc[t][mt];
#else
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      if (!pv[mt]) continue;
      f4* d = reinterpret_cast<f4*>(dxl + pbase[mt] + toff);
      *d += acc[t][mt];
    }
#endif
  }
  __syncthreads();
  float* dxn = a.dx + (int64_t)n * HW * a.Ci;
  const int c4 = a.Ci >> 2;
  for (int e = threadIdx.x; e < HW * c4; e += NT) {
    const int px = e / c4, c = e - px * c4;
    reinterpret_cast<f4*>(dxn)[e] = *reinterpret_cast<const f4*>(dxl + px * CP + 4 * c);
  }
}

// The same per-image input gradient with the weight operand staged through LDS, transposed to
// [tap][ci][co] one 16-co quad at a time (double-buffered): per quad the workgroup loads the contiguous
// 16 x KH*KW*Ci block of W with 16-B loads and writes it with 16-B LDS stores along co, and the MFMA's
// weight operand is one ds_read_b128 per tap (instead of four strided 4-B global loads per tap).  Row
// stride 16 + 4 floats: the 16 ci lanes of a read land on distinct banks.
template <int TC, int MT, int NT, int SI>
__global__ __launch_bounds__(NT) void conv_dgrad_img_lds_kernel(const ConvDgradArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int WR = 20;  // floats per (tap, ci) row of a staged quad
  const int KK = a.KH * a.KW;
  const int CP = a.Ci + 4;
  const int HW = a.H * a.W, OHW = a.OH * a.OW;
  float* const dxl = lds;                          // [HW][CP]
  float* const wb0 = lds + ((HW * CP + 3) & ~3);  // [2][KK][Ci][WR]
  const int wbuf = KK * a.Ci * WR;
  const int n = blockIdx.x;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int NCB = a.Ci >> 4;
  const int cb = wv % NCB, cls = wv / NCB;
  const int ph = cls / a.S, pw = cls - ph * a.S;
  const int TW = a.KW / a.S;
  for (int e = threadIdx.x; e < HW * CP / 4; e += NT) reinterpret_cast<f4*>(dxl)[e] = f4{0.f, 0.f, 0.f, 0.f};
  // staging items of a quad: (tap, 4-ci group, 4-co group): 4 global float4 (co m = 0..3) -> 4 LDS float4
  const int ci4n = a.Ci >> 2;
  const int nitems = KK * ci4n * 4;
  const int64_t wco = (int64_t)KK * a.Ci;
  auto stage_load = [&](int q, int item, f4 (&r)[4]) {
    const int cg = item & 3, rest = item >> 2, c4 = rest % ci4n, tap = rest / ci4n;
    const float* src = a.w + (int64_t)(16 * q + 4 * cg) * wco + tap * a.Ci + 4 * c4;
#pragma unroll
    for (int m = 0; m < 4; ++m) r[m] = *reinterpret_cast<const f4*>(src + m * wco);
  };
  auto stage_store = [&](int buf, int item, const f4 (&r)[4]) {
    const int cg = item & 3, rest = item >> 2, c4 = rest % ci4n, tap = rest / ci4n;
    float* dst = wb0 + buf * wbuf + (tap * a.Ci + 4 * c4) * WR + 4 * cg;
#pragma unroll
    for (int c = 0; c < 4; ++c)
      *reinterpret_cast<f4*>(dst + c * WR) = f4{r[0][c], r[1][c], r[2][c], r[3][c]};
  };
  const float* dzn = a.dz + (int64_t)n * OHW * a.Co;
  int woff[TC];
#pragma unroll
  for (int t = 0; t < TC; ++t) {
    const int th = t / TW, tw = t - th * TW;
    woff[t] = (((ph + a.S * th) * a.KW + pw + a.S * tw) * a.Ci + 16 * cb + li) * WR + 4 * g;
  }
  int poff[MT];
  bool pv[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int p = 16 * mt + li;
    pv[mt] = p < OHW;
    poff[mt] = (pv[mt] ? p : 0) * a.Co;
  }
  auto load_dz = [&](int q, f4 (&Dv)[MT]) {
    const int co0 = 4 * (4 * q + g);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
      Dv[mt] = pv[mt] ? *reinterpret_cast<const f4*>(dzn + poff[mt] + co0) : f4{0.f, 0.f, 0.f, 0.f};
  };
  f4 acc[TC][MT];
#pragma unroll
  for (int t = 0; t < TC; ++t)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[t][mt] = f4{0.f, 0.f, 0.f, 0.f};
  const int nq = a.Co >> 4;
  f4 sr[SI][4];
#pragma unroll
  for (int u = 0; u < SI; ++u) {
    const int item = threadIdx.x + u * NT;
    if (item < nitems) stage_load(0, item, sr[u]);
  }
  f4 Dv[MT];
  load_dz(0, Dv);
#pragma unroll
  for (int u = 0; u < SI; ++u) {
    const int item = threadIdx.x + u * NT;
    if (item < nitems) stage_store(0, item, sr[u]);
  }
  __syncthreads();
  for (int q = 0; q < nq; ++q) {
    const int buf = q & 1;
    if (q + 1 < nq) {
#pragma unroll
      for (int u = 0; u < SI; ++u) {
        const int item = threadIdx.x + u * NT;
        if (item < nitems) stage_load(q + 1, item, sr[u]);
      }
    }
    f4 Dn[MT];
    if (q + 1 < nq) load_dz(q + 1, Dn);
    f4 A[TC];
#pragma unroll
    for (int t = 0; t < TC; ++t) A[t] = *reinterpret_cast<const f4*>(wb0 + buf * wbuf + woff[t]);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int t = 0; t < TC; ++t)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
          acc[t][mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(A[t][j], Dv[mt][j], acc[t][mt], 0, 0, 0);
    if (q + 1 < nq) {
#pragma unroll
      for (int u = 0; u < SI; ++u) {
        const int item = threadIdx.x + u * NT;
        if (item < nitems) stage_store(buf ^ 1, item, sr[u]);
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) Dv[mt] = Dn[mt];
    }
    __syncthreads();
  }
  int pbase[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int p = 16 * mt + li;
    const int oh = p / a.OW, ow = p - oh * a.OW;
    pbase[mt] = ((oh * a.S + ph) * a.W + ow * a.S + pw) * CP + 16 * cb + 4 * g;
  }
#pragma unroll
  for (int t = 0; t < TC; ++t) {
    const int th = t / TW, tw = t - th * TW;
    const int toff = (a.S * th * a.W + a.S * tw) * CP;
    f4 cur[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
      if (pv[mt]) cur[mt] = *reinterpret_cast<const f4*>(dxl + pbase[mt] + toff);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
      if (pv[mt]) *reinterpret_cast<f4*>(dxl + pbase[mt] + toff) = cur[mt] + acc[t][mt];
  }
  __syncthreads();
  float* dxn = a.dx + (int64_t)n * HW * a.Ci;
  const int c4 = a.Ci >> 2;
  for (int e = threadIdx.x; e < HW * c4; e += NT) {
    const int px = e / c4, c = e - px * c4;
    reinterpret_cast<f4*>(dxn)[e] = *reinterpret_cast<const f4*>(dxl + px * CP + 4 * c);
  }
}

// SI: staging items per thread per quad (conv3: 576 items / 256 threads -> 3; conv2: 512 / 512 -> 1)
template <int TC, int MT, int NT, int SI>
int launch_dgrad_img_lds(const ConvDgradArgs& a, hipStream_t st) {
  const int KK = a.KH * a.KW;
  const size_t lds = ((size_t)a.H * a.W * (a.Ci + 4) + 3) / 4 * 4 * sizeof(float) + 2 * (size_t)KK * a.Ci * 20 * sizeof(float);
  if (lds > 160 * 1024 || KK * (a.Ci / 4) * 4 > SI * NT || a.Co % 16) return RAI_E_SHAPE;
  auto k = conv_dgrad_img_lds_kernel<TC, MT, NT, SI>;
  const int e = allow_lds(reinterpret_cast<const void*>(k));
  if (e != RAI_OK) return e;
  if (a.B > 0x7fffffffLL) return RAI_E_SHAPE;
  hipLaunchKernelGGL(k, dim3((unsigned)a.B), dim3(NT), lds, st, a);
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}

template <int TC, int MT, int NT, int PF = 2, bool BUF = false, bool RELU = false>
int launch_dgrad_img(const ConvDgradArgs& a, hipStream_t st) {
  static_assert(BUF || !RELU, "the ReLU-folded form uses buffer loads");
  const size_t lds = (size_t)a.H * a.W * (a.Ci + 4) * sizeof(float);
  if (lds > 160 * 1024) return RAI_E_SHAPE;
  if (BUF && (int64_t)a.Co * a.KH * a.KW * a.Ci * 4 >= (1LL << 31)) return RAI_E_SHAPE;
  auto k = conv_dgrad_img_kernel<TC, MT, NT, PF, BUF, RELU>;
  const int e = allow_lds(reinterpret_cast<const void*>(k));
  if (e != RAI_OK) return e;
  if (a.B > 0x7fffffffLL) return RAI_E_SHAPE;
  hipLaunchKernelGGL(k, dim3((unsigned)a.B), dim3(NT), lds, st, a);
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}

// the per-image form's instantiation for this shape: 1 = conv3-like, 2 = conv2-like, 0 = none
static int dgrad_img_kind(const ConvDgradArgs& a) {
  if (a.Ci % 16 || a.Co % 16 || a.KH % a.S || a.KW % a.S) return 0;
  const int nw = (a.Ci / 16) * a.S * a.S, tc = (a.KH / a.S) * (a.KW / a.S), mt = (a.OH * a.OW + 15) / 16;
  if ((size_t)a.H * a.W * (a.Ci + 4) * sizeof(float) > 160 * 1024) return 0;
  if (nw == 4 && tc == 9 && mt == 4) return 1;
  if (nw == 8 && tc == 4 && mt == 6) return 2;
  return 0;
}

}  // namespace

extern "C" int64_t rai_conv2d_wgrad_workspace_bytes(int64_t B, int32_t H, int32_t W, int32_t Ci, int32_t Co,
                                                    int32_t KH, int32_t KW, int32_t stride) {
  if (B < 1 || H < KH || W < KW || stride < 1 || Co < 16 || KH < 1 || KW < 1 || Ci < 4) return 0;
  const int64_t M = B * ((H - KH) / stride + 1) * ((W - KW) / stride + 1);
  const int K = KH * KW * Ci;
  // the largest split count any target_wgs <= 1024 gives (the _v variants share the workspace size)
  int64_t mx = 0;
  for (int t = 256; t <= 1024; t += 256) {
    const WrwPlan p = wrw_plan(M, Co, K, t);
    mx = p.S > mx ? p.S : mx;
  }
  return mx * Co * (K + 1) * (int64_t)sizeof(float);  // + the bias-gradient partials (relu_partials)
}

static bool wgrad_shape_ok(int64_t B, int32_t H, int32_t W, int32_t Ci, int32_t Co, int32_t KH, int32_t KW,
                           int32_t stride) {
  if (B < 0 || H < 1 || W < 1 || Ci < 4 || Ci % 4 || (Co != 32 && Co != 64) || KH < 1 || KW < 1 || stride < 1 ||
      KH > H || KW > W)
    return false;
  const int64_t K = (int64_t)KH * KW * Ci;
  return K % 64 == 0 && K <= (1 << 20);
}

// the first launch of rai_conv2d_wgrad: every workgroup's partial tile into workspace (B >= 1)
static int wgrad_partials(const float* x, const float* dz, const float* y, int64_t B, int32_t H, int32_t W,
                          int32_t Ci, int32_t Co, int32_t KH, int32_t KW, int32_t stride, void* workspace,
                          int64_t workspace_bytes, int32_t target_wgs, int32_t pf, hipStream_t st,
                          const uint8_t* xu8 = nullptr, float xdiv = 1.f) {
  const int64_t K = (int64_t)KH * KW * Ci;
  if (xu8) {  // uint8 input: one dword per pixel (Ci = 4), buffer loads
    if (Ci != 4 || !(xdiv > 0.f) || (int64_t)B * H * W * Ci >= (1LL << 31)) return RAI_E_SHAPE;
    if ((uintptr_t)xu8 & 3) return RAI_E_SHAPE;
    x = reinterpret_cast<const float*>(xu8);  // never dereferenced as float
  }
  if (!x || !dz || !workspace) return RAI_E_NULLPTR;
  if (((uintptr_t)(xu8 ? nullptr : x) | (uintptr_t)dz | (uintptr_t)workspace) & 15) return RAI_E_SHAPE;
  if ((int64_t)H * W * Ci > (1LL << 30)) return RAI_E_SHAPE;  // per-chunk offsets are int32
  if (workspace_bytes < rai_conv2d_wgrad_workspace_bytes(B, H, W, Ci, Co, KH, KW, stride)) return RAI_E_WORKSPACE;
  ConvWrwArgs a;
  a.x = x;
  a.xu8 = xu8;
  a.xdiv = xdiv;
  a.xinv = 0.f;
  a.dz = dz;
  a.y = y;
  a.part = static_cast<float*>(workspace);
  a.H = H;
  a.W = W;
  a.Ci = Ci;
  a.Co = Co;
  a.KW = KW;
  a.S_ = stride;
  a.OH = (H - KH) / stride + 1;
  a.OW = (W - KW) / stride + 1;
  a.K = (int)K;
  a.M = B * a.OH * a.OW;
  if (target_wgs < 0 || target_wgs > 1024) return RAI_E_SHAPE;
  const WrwPlan p = wrw_plan(a.M, Co, a.K, target_wgs);
  a.per = p.per;
  static const int env_xcd = [] {  // A/B: RAI_WRW_XCD=0 keeps the grid's natural order (read once)
    const char* e = getenv("RAI_WRW_XCD");
    return e ? atoi(e) : 1;
  }();
  a.xcd_map = (env_xcd != 0 && p.S % 8 == 0) ? 1 : 0;
  // a split's offsets from its first sample fit int32
  if ((int64_t)(WR_MAXPX / (a.OH * a.OW) + 2) * H * W * Ci > 0x7fffffffLL) return RAI_E_SHAPE;
  const dim3 grid((unsigned)p.S, (unsigned)p.KT);
  const bool buf_ok = (int64_t)B * H * W * Ci * (xu8 ? 1 : 4) < (1LL << 31) && a.M * Co * 4 < (1LL << 31);
  // default: buffer loads with 4 pixel steps in flight where the operands fit 2 GB buffers (NatureCNN
  // B = 256: 2-4 % faster than pointer loads, B = 1024: 8-21 %; profiles/r4g_conv_bench.txt)
  if (pf <= 0) pf = buf_ok ? 104 : 4;
  if (pf >= 100 && !buf_ok) return RAI_E_SHAPE;
  if (xu8) {  // buffer loads, 4 pixel steps in flight (the default form), uint8 input
    if (!buf_ok) return RAI_E_SHAPE;
    if (y && (((uintptr_t)y) & 15)) return RAI_E_SHAPE;
    if (u8_div_valu_exact(xdiv, &a.xinv)) {
      if (y && p.VC == 2) hipLaunchKernelGGL((conv_wrw_kernel<2, 4, true, true, 2>), grid, dim3(CV_THREADS), 0, st, a);
      else if (y) hipLaunchKernelGGL((conv_wrw_kernel<4, 4, true, true, 2>), grid, dim3(CV_THREADS), 0, st, a);
      else if (p.VC == 2) hipLaunchKernelGGL((conv_wrw_kernel<2, 4, false, true, 2>), grid, dim3(CV_THREADS), 0, st, a);
      else hipLaunchKernelGGL((conv_wrw_kernel<4, 4, false, true, 2>), grid, dim3(CV_THREADS), 0, st, a);
    } else {
      if (y && p.VC == 2) hipLaunchKernelGGL((conv_wrw_kernel<2, 4, true, true, 1>), grid, dim3(CV_THREADS), 0, st, a);
      else if (y) hipLaunchKernelGGL((conv_wrw_kernel<4, 4, true, true, 1>), grid, dim3(CV_THREADS), 0, st, a);
      else if (p.VC == 2) hipLaunchKernelGGL((conv_wrw_kernel<2, 4, false, true, 1>), grid, dim3(CV_THREADS), 0, st, a);
      else hipLaunchKernelGGL((conv_wrw_kernel<4, 4, false, true, 1>), grid, dim3(CV_THREADS), 0, st, a);
    }
  } else if (y) {  // the ReLU backward and the bias gradient fused in (rai_conv2d_wgrad_relu_partials)
    if (((uintptr_t)y) & 15) return RAI_E_SHAPE;
    if (pf == 104 && p.VC == 2) hipLaunchKernelGGL((conv_wrw_kernel<2, 4, true, true>), grid, dim3(CV_THREADS), 0, st, a);
    else if (pf == 104) hipLaunchKernelGGL((conv_wrw_kernel<4, 4, true, true>), grid, dim3(CV_THREADS), 0, st, a);
    else if (p.VC == 2) hipLaunchKernelGGL((conv_wrw_kernel<2, 4, true>), grid, dim3(CV_THREADS), 0, st, a);
    else hipLaunchKernelGGL((conv_wrw_kernel<4, 4, true>), grid, dim3(CV_THREADS), 0, st, a);
  } else if (pf >= 100) {  // buffer loads, 4 or 8 pixel steps in flight (A/B)
    if (p.VC == 2 && pf == 104) hipLaunchKernelGGL((conv_wrw_kernel<2, 4, false, true>), grid, dim3(CV_THREADS), 0, st, a);
    else if (p.VC == 2) hipLaunchKernelGGL((conv_wrw_kernel<2, 8, false, true>), grid, dim3(CV_THREADS), 0, st, a);
    else if (pf == 104) hipLaunchKernelGGL((conv_wrw_kernel<4, 4, false, true>), grid, dim3(CV_THREADS), 0, st, a);
    else hipLaunchKernelGGL((conv_wrw_kernel<4, 8, false, true>), grid, dim3(CV_THREADS), 0, st, a);
  } else if (p.VC == 2) {
    if (pf == 4) hipLaunchKernelGGL((conv_wrw_kernel<2, 4, false>), grid, dim3(CV_THREADS), 0, st, a);
    else hipLaunchKernelGGL((conv_wrw_kernel<2, 8, false>), grid, dim3(CV_THREADS), 0, st, a);
  } else {
    if (pf == 4) hipLaunchKernelGGL((conv_wrw_kernel<4, 4, false>), grid, dim3(CV_THREADS), 0, st, a);
    else hipLaunchKernelGGL((conv_wrw_kernel<4, 8, false>), grid, dim3(CV_THREADS), 0, st, a);
  }
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}

static int wgrad_reduce(const rai_conv2d_wgrad_job* jobs, int32_t n_jobs, int32_t accumulate, hipStream_t st) {
  WrwReduceArgs ra;
  ra.n = 0;
  ra.accumulate = accumulate ? 1 : 0;
  int blocks = 0;
  for (int q = 0; q < n_jobs; ++q) {
    const rai_conv2d_wgrad_job& jb = jobs[q];
    if (!wgrad_shape_ok(jb.B, jb.H, jb.W, jb.Ci, jb.Co, jb.KH, jb.KW, jb.stride)) return RAI_E_SHAPE;
    const int64_t K = (int64_t)jb.KH * jb.KW * jb.Ci;
    if (jb.B == 0) {
      if (!accumulate) {
        if (!jb.dw) return RAI_E_NULLPTR;
        const hipError_t e = hipMemsetAsync(jb.dw, 0, (size_t)jb.Co * K * 4, st);
        if (e != hipSuccess) return (int)e;
      }
      continue;
    }
    if (!jb.dw || !jb.workspace) return RAI_E_NULLPTR;
    if (((uintptr_t)jb.dw | (uintptr_t)jb.workspace) & 15) return RAI_E_SHAPE;
    const int64_t M = jb.B * ((jb.H - jb.KH) / jb.stride + 1) * ((jb.W - jb.KW) / jb.stride + 1);
    const WrwPlan p = wrw_plan(M, jb.Co, (int)K, 0);
    WrwReduceJob& r = ra.j[ra.n++];
    r.part = static_cast<const f4*>(jb.workspace);
    r.dw = reinterpret_cast<f4*>(jb.dw);
    r.n4 = (int64_t)jb.Co * K / 4;
    r.S = p.S;
    r.blk0 = blocks;
    blocks += (int)((r.n4 + 15) / 16);
    if (jb.db) {  // the bias-gradient partials of rai_conv2d_wgrad_relu_partials, after the weight tiles
      if (((uintptr_t)jb.db) & 15) return RAI_E_SHAPE;
      WrwReduceJob& rb = ra.j[ra.n++];
      rb.part = reinterpret_cast<const f4*>(static_cast<const float*>(jb.workspace) + (int64_t)p.S * jb.Co * K);
      rb.dw = reinterpret_cast<f4*>(jb.db);
      rb.n4 = jb.Co / 4;
      rb.S = p.S;
      rb.blk0 = blocks;
      blocks += (int)((rb.n4 + 15) / 16);
    }
  }
  if (ra.n == 0) return RAI_OK;
  hipLaunchKernelGGL(conv_wrw_reduce_kernel, dim3((unsigned)blocks), dim3(CV_THREADS), 0, st, ra);
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}

extern "C" int rai_conv2d_wgrad_v(const float* x, const float* dz, int64_t B, int32_t H, int32_t W, int32_t Ci,
                                  int32_t Co, int32_t KH, int32_t KW, int32_t stride, float* dw, int32_t accumulate,
                                  void* workspace, int64_t workspace_bytes, int32_t target_wgs, int32_t pf,
                                  void* stream) {
  if (!wgrad_shape_ok(B, H, W, Ci, Co, KH, KW, stride)) return RAI_E_SHAPE;
  hipStream_t st = rai_stream(stream);
  if (B > 0) {
    if (!dw) return RAI_E_NULLPTR;
    const int rc = wgrad_partials(x, dz, nullptr, B, H, W, Ci, Co, KH, KW, stride, workspace, workspace_bytes,
                                  target_wgs, pf, st);
    if (rc != RAI_OK) return rc;
    if (target_wgs != 0) {  // the reduce below follows the default plan: re-derive S for this one
      // (A/B only) the reduction reads the split count the partials were launched with
      const int64_t K = (int64_t)KH * KW * Ci;
      const int64_t M = B * ((H - KH) / stride + 1) * ((W - KW) / stride + 1);
      const WrwPlan p = wrw_plan(M, Co, (int)K, target_wgs);
      WrwReduceArgs ra;
      ra.n = 1;
      ra.accumulate = accumulate ? 1 : 0;
      ra.j[0].part = static_cast<const f4*>(workspace);
      ra.j[0].dw = reinterpret_cast<f4*>(dw);
      ra.j[0].n4 = (int64_t)Co * K / 4;
      ra.j[0].S = p.S;
      ra.j[0].blk0 = 0;
      hipLaunchKernelGGL(conv_wrw_reduce_kernel, dim3((unsigned)((ra.j[0].n4 + 15) / 16)), dim3(CV_THREADS), 0, st,
                         ra);
      RAI_LAUNCH_CHECK();
      return RAI_OK;
    }
  }
  rai_conv2d_wgrad_job jb = {workspace, dw, nullptr, B, H, W, Ci, Co, KH, KW, stride, 0};
  return wgrad_reduce(&jb, 1, accumulate, st);
}

extern "C" int rai_conv2d_wgrad_partials(const float* x, const float* dz, int64_t B, int32_t H, int32_t W,
                                         int32_t Ci, int32_t Co, int32_t KH, int32_t KW, int32_t stride,
                                         void* workspace, int64_t workspace_bytes, void* stream) {
  if (!wgrad_shape_ok(B, H, W, Ci, Co, KH, KW, stride)) return RAI_E_SHAPE;
  if (B == 0) return RAI_OK;
  return wgrad_partials(x, dz, nullptr, B, H, W, Ci, Co, KH, KW, stride, workspace, workspace_bytes, 0, 0,
                        rai_stream(stream));
}

extern "C" int rai_conv2d_wgrad_relu_partials(const float* dy, const float* y, const float* x, int64_t B, int32_t H,
                                              int32_t W, int32_t Ci, int32_t Co, int32_t KH, int32_t KW,
                                              int32_t stride, void* workspace, int64_t workspace_bytes,
                                              void* stream) {
  if (!wgrad_shape_ok(B, H, W, Ci, Co, KH, KW, stride)) return RAI_E_SHAPE;
  if (B == 0) return RAI_OK;
  if (!y) return RAI_E_NULLPTR;
  return wgrad_partials(x, dy, y, B, H, W, Ci, Co, KH, KW, stride, workspace, workspace_bytes, 0, 0,
                        rai_stream(stream));
}

// uint8-input forms of the two partial passes (the first NatureCNN layer: x = u8 / x_divisor, Ci = 4)
extern "C" int rai_conv2d_wgrad_partials_u8(const uint8_t* x, float x_divisor, const float* dz, int64_t B, int32_t H,
                                            int32_t W, int32_t Ci, int32_t Co, int32_t KH, int32_t KW, int32_t stride,
                                            void* workspace, int64_t workspace_bytes, void* stream) {
  if (!wgrad_shape_ok(B, H, W, Ci, Co, KH, KW, stride) || Ci != 4) return RAI_E_SHAPE;
  if (B == 0) return RAI_OK;
  if (!x) return RAI_E_NULLPTR;
  return wgrad_partials(nullptr, dz, nullptr, B, H, W, Ci, Co, KH, KW, stride, workspace, workspace_bytes, 0, 0,
                        rai_stream(stream), x, x_divisor);
}

extern "C" int rai_conv2d_wgrad_relu_partials_u8(const float* dy, const float* y, const uint8_t* x, float x_divisor,
                                                 int64_t B, int32_t H, int32_t W, int32_t Ci, int32_t Co, int32_t KH,
                                                 int32_t KW, int32_t stride, void* workspace, int64_t workspace_bytes,
                                                 void* stream) {
  if (!wgrad_shape_ok(B, H, W, Ci, Co, KH, KW, stride) || Ci != 4) return RAI_E_SHAPE;
  if (B == 0) return RAI_OK;
  if (!x || !y) return RAI_E_NULLPTR;
  return wgrad_partials(nullptr, dy, y, B, H, W, Ci, Co, KH, KW, stride, workspace, workspace_bytes, 0, 0,
                        rai_stream(stream), x, x_divisor);
}

extern "C" int rai_conv2d_wgrad_reduce(const rai_conv2d_wgrad_job* jobs, int32_t n_jobs, int32_t accumulate,
                                       void* stream) {
  if (n_jobs < 0 || n_jobs > RAI_WGRAD_MAX_JOBS) return RAI_E_SHAPE;
  if (n_jobs > 0 && !jobs) return RAI_E_NULLPTR;
  return wgrad_reduce(jobs, n_jobs, accumulate, rai_stream(stream));
}

// variant: 0 = by shape (the shipped choice); 1.. = a fixed blocking (tools/conv_bench.py A/B)
extern "C" int rai_conv2d_bias_relu_fwd_v(const float* x, const float* w, const float* b, int64_t B, int32_t H,
                                         int32_t W, int32_t Ci, int32_t Co, int32_t KH, int32_t KW, int32_t stride,
                                         int32_t out_nchw, float* y, int32_t variant, void* stream) {
  if (B < 0 || H < 1 || W < 1 || Ci < 4 || Ci % 4 || Co < 16 || Co % 16 || KH < 1 || KW < 1 || stride < 1 ||
      KH > H || KW > W)
    return RAI_E_SHAPE;
  const int64_t K = (int64_t)KH * KW * Ci;
  if (K % 32 || K / 4 > CV_MAXCHUNK) return RAI_E_SHAPE;
  if (B == 0) return RAI_OK;
  if (!x || !w || !b || !y) return RAI_E_NULLPTR;
  if (((uintptr_t)x | (uintptr_t)w | (uintptr_t)b | (uintptr_t)y) & 15) return RAI_E_SHAPE;
  ConvFwdArgs a;
  a.x = x;
  a.xu8 = nullptr;
  a.xdiv = 1.f;
  a.xinv = 1.f;
  a.w = w;
  a.b = b;
  a.y = y;
  a.H = H;
  a.W = W;
  a.Ci = Ci;
  a.Co = Co;
  a.KW = KW;
  a.S = stride;
  a.OH = (H - KH) / stride + 1;
  a.OW = (W - KW) / stride + 1;
  a.K = (int)K;
  a.M = B * a.OH * a.OW;
  if ((int64_t)H * W * Ci * B > (1LL << 40)) return RAI_E_SHAPE;
  hipStream_t st = rai_stream(stream);
  const bool nchw = out_nchw != 0;
  if (variant == 0) {
    // measured (profiles/r3v_conv_bench.txt): the LDS-resident-weight forms win wherever the weight rows
    // fit (<= ~150 KB); 32 co x 256 px tiles once they give >= 256 workgroup tiles, else 64 co x 64 px
    const size_t lds32 = (size_t)32 * (K + 4) * 4, lds64 = (size_t)64 * (K + 4) * 4;
    // buffer-load forms (16 / 17 = 14 / 13 with raw_buffer_load, scalar offsets) where the input fits a
    // 2 GB buffer: 3-6 % faster at B = 256 and 1024 (profiles/r4g_conv_bench.txt).  Between the 32 x 256
    // and the 64 x 64 tile: the fewer rounds of tiles over the persistent workgroups (one per CU), a
    // 32 x 256 tile costing two 64 x 64 ones, ties to the wider tile (it measured faster at equal rounds:
    // conv2 at B = 256 24.2 vs 26.1 us, conv2 / conv3 at B = 1024; conv3 at B = 256 takes the 64 x 64
    // tile, 17.6 vs 24.8 us; profiles/r4n_conv_bench.txt)
    const int ncu = num_cus();
    const int64_t wg32 = ncu / (Co / 32 > 0 ? Co / 32 : 1), wg64 = ncu / (Co / 64 > 0 ? Co / 64 : 1);
    const int64_t rounds32 = ((a.M + 255) / 256 + wg32 - 1) / (wg32 > 0 ? wg32 : 1);
    const int64_t rounds64 = ((a.M + 63) / 64 + wg64 - 1) / (wg64 > 0 ? wg64 : 1);
    const bool buf = B * H * W * (int64_t)Ci * 4 < (1LL << 31);
    if (Co % 32 == 0 && lds32 + CV_MAXCHUNK * 4 <= 160 * 1024 && (Co % 64 != 0 || 2 * rounds32 <= rounds64))
      variant = buf ? 16 : 14;
    else if (Co % 64 == 0 && lds64 + CV_MAXCHUNK * 4 <= 160 * 1024)
      variant = buf ? 17 : 13;
    else
      variant = (Co % 64 == 0) ? 10 : (Co % 32 == 0) ? 11 : 7;
  }
  switch (variant) {
    case 1: return launch_fwd<2, 2, 1, 4>(a, nchw, st);  // 32 co x 128 px
    case 2: return launch_fwd<1, 2, 2, 2>(a, nchw, st);  // 32 co x 64 px
    case 3: return launch_fwd<2, 1, 2, 2>(a, nchw, st);  // 64 co x 32 px
    case 4: return launch_fwd<4, 1, 1, 4>(a, nchw, st);  // 64 co x 64 px
    case 5: return launch_fwd<2, 2, 2, 2>(a, nchw, st);  // 64 co x 64 px
    case 6: return launch_fwd<1, 1, 2, 2>(a, nchw, st);  // 32 co x 32 px
    case 7: return launch_fwd<1, 1, 1, 4>(a, nchw, st);  // 16 co x 64 px
    case 8: return launch_fwd<2, 2, 1, 4, 4>(a, nchw, st);  // variant 1, four quads in flight
    case 9: return launch_fwd<2, 2, 2, 2, 4>(a, nchw, st);  // variant 5, four quads in flight
    case 10: return launch_fwd<2, 2, 2, 2, 3>(a, nchw, st);  // variant 5, three quads in flight
    case 11: return launch_fwd<2, 2, 1, 4, 3>(a, nchw, st);  // variant 1, three quads in flight
    case 12: return launch_fwd_lds<2, 2, 2, 4, 3>(a, nchw, st);  // LDS weights, 64 co x 128 px, 8 waves
    case 13: return launch_fwd_lds<2, 1, 2, 4, 4>(a, nchw, st);  // LDS weights, 64 co x 64 px, 8 waves
    case 14: return launch_fwd_lds<2, 2, 1, 8, 3>(a, nchw, st);  // LDS weights, 32 co x 256 px, 8 waves
    case 15: return launch_fwd_lds<1, 2, 2, 4, 4>(a, nchw, st);  // LDS weights, 32 co x 128 px, 8 waves
    case 16: return launch_fwd_lds<2, 2, 1, 8, 3, true>(a, nchw, st);  // variant 14, buffer loads
    case 17: return launch_fwd_lds<2, 1, 2, 4, 4, true>(a, nchw, st);  // variant 13, buffer loads
    case 18: return launch_fwd_lds<2, 2, 2, 4, 3, true>(a, nchw, st);  // variant 12, buffer loads
    // 64 co x 32 px (one 16 x 16 block per wave): twice variant 17's pixel tiles, for grids whose tile
    // count is just above the CU count (NatureCNN conv2 at B = 256: 648 tiles instead of 324 on 256 CUs)
    case 19: return launch_fwd_lds<1, 1, 4, 2, 4, true>(a, nchw, st);
    case 20: return launch_fwd_lds<1, 1, 4, 2, 8, true>(a, nchw, st);
    default: return RAI_E_SHAPE;
  }
}

// The first NatureCNN layer on the rollout's uint8 frames (NHWC, Ci = 4): x = u8 / x_divisor formed in the
// kernel (IEEE division, the value the gather's prescale writes), so the f32 input tensor (4x the
// bytes) is never written or read.  The LDS-weight forms with buffer loads (variants 16 / 17's blocking).
extern "C" int rai_conv2d_bias_relu_fwd_u8(const uint8_t* x, float x_divisor, const float* w, const float* b,
                                          int64_t B, int32_t H, int32_t W, int32_t Ci, int32_t Co, int32_t KH,
                                          int32_t KW, int32_t stride, int32_t out_nchw, float* y, void* stream) {
  if (B < 0 || H < 1 || W < 1 || Ci != 4 || Co < 16 || Co % 16 || KH < 1 || KW < 1 || stride < 1 || KH > H ||
      KW > W || !(x_divisor > 0.f))
    return RAI_E_SHAPE;
  const int64_t K = (int64_t)KH * KW * Ci;
  if (K % 32 || K / 4 > CV_MAXCHUNK) return RAI_E_SHAPE;
  if (B == 0) return RAI_OK;
  if (!x || !w || !b || !y) return RAI_E_NULLPTR;
  if ((((uintptr_t)w | (uintptr_t)b | (uintptr_t)y) & 15) || ((uintptr_t)x & 3)) return RAI_E_SHAPE;
  if (B * H * W * (int64_t)Ci >= (1LL << 31)) return RAI_E_SHAPE;
  ConvFwdArgs a;
  a.x = nullptr;
  a.xu8 = x;
  a.xdiv = x_divisor;
  a.xinv = 0.f;
  const bool valu = u8_div_valu_exact(x_divisor, &a.xinv);
  a.w = w;
  a.b = b;
  a.y = y;
  a.H = H;
  a.W = W;
  a.Ci = Ci;
  a.Co = Co;
  a.KW = KW;
  a.S = stride;
  a.OH = (H - KH) / stride + 1;
  a.OW = (W - KW) / stride + 1;
  a.K = (int)K;
  a.M = B * a.OH * a.OW;
  hipStream_t st = rai_stream(stream);
  const bool nchw = out_nchw != 0;
  const size_t lds32 = (size_t)32 * (K + 4) * 4, lds64 = (size_t)64 * (K + 4) * 4;
  const int64_t t14 = (a.M + 255) / 256 * (Co / 32);
  if (Co % 32 == 0 && lds32 + CV_MAXCHUNK * 4 <= 160 * 1024 && (t14 >= 256 || Co % 64 != 0))
    return valu ? launch_fwd_lds<2, 2, 1, 8, 3, true, 2>(a, nchw, st) : launch_fwd_lds<2, 2, 1, 8, 3, true, 1>(a, nchw, st);
  if (Co % 64 == 0 && lds64 + CV_MAXCHUNK * 4 <= 160 * 1024)
    return valu ? launch_fwd_lds<2, 1, 2, 4, 4, true, 2>(a, nchw, st) : launch_fwd_lds<2, 1, 2, 4, 4, true, 1>(a, nchw, st);
  return RAI_E_UNSUPPORTED;
}

// Split-K factor the forward takes for a shape (1: none): 2 where the default LDS-weight variant's tiles
// leave CUs idle (fewer tile workgroups than CUs) and each half keeps >= 8 quads of the reduction, so the
// two halves run as twice the workgroups, two per CU (half the LDS each); then a second pass adds them.
// Opt-in (RAI_CONV_FWD_SPLITK=1): measured SLOWER than the one-pass forward at the C3 update's B = 256
// (conv2 27.8 vs 23.1 us, conv3 24.7 vs 17.8 us, profiles/r5l_conv_bench_*.txt): the partials' extra
// 2 x 3-6 MB and the second launch cost more than the idle CUs the split fills.
static int fwd_splitk_factor(int64_t B, int32_t H, int32_t W, int32_t Ci, int32_t Co, int32_t KH, int32_t KW,
                             int32_t stride, int32_t out_nchw) {
  const char* e = getenv("RAI_CONV_FWD_SPLITK");
  if (!(e && !strcmp(e, "1"))) return 1;
  if (B < 1 || Ci % 4 || Co % 64 || stride < 1 || KH > H || KW > W) return 1;
  const int64_t K = (int64_t)KH * KW * Ci;
  if (K % 32 || K / 4 > CV_MAXCHUNK || K / 16 < 16) return 1;
  const int64_t OH = (H - KH) / stride + 1, OW = (W - KW) / stride + 1, M = B * OH * OW;
  if (out_nchw && OH * OW * Co > CV_RED_NCHW_MAX) return 1;
  // the default variant's workgroup tiles (16: 32 co x 256 px, 17: 64 co x 64 px; see rai_conv2d_bias_relu_fwd_v)
  const int ncu = num_cus();
  const size_t lds32 = (size_t)32 * (K + 4) * 4;
  const int64_t wg32 = ncu / (Co / 32), wg64 = ncu / (Co / 64);
  const int64_t rounds32 = ((M + 255) / 256 + wg32 - 1) / wg32, rounds64 = ((M + 63) / 64 + wg64 - 1) / wg64;
  const bool v32 = lds32 + CV_MAXCHUNK * 4 <= 160 * 1024 && 2 * rounds32 <= rounds64;
  const int64_t tiles = v32 ? (M + 255) / 256 * (Co / 32) : (M + 63) / 64 * (Co / 64);
  return tiles < ncu ? 2 : 1;
}

extern "C" int64_t rai_conv2d_fwd_splitk_bytes(int64_t B, int32_t H, int32_t W, int32_t Ci, int32_t Co, int32_t KH,
                                               int32_t KW, int32_t stride, int32_t out_nchw) {
  const int S = fwd_splitk_factor(B, H, W, Ci, Co, KH, KW, stride, out_nchw);
  if (S < 2) return 0;
  const int64_t OH = (H - KH) / stride + 1, OW = (W - KW) / stride + 1;
  return (int64_t)S * B * OH * OW * Co * (int64_t)sizeof(float);
}

extern "C" int rai_conv2d_bias_relu_fwd_splitk(const float* x, const float* w, const float* b, int64_t B, int32_t H,
                                               int32_t W, int32_t Ci, int32_t Co, int32_t KH, int32_t KW,
                                               int32_t stride, int32_t out_nchw, float* y, float* part,
                                               int64_t part_bytes, void* stream) {
  const int S = fwd_splitk_factor(B, H, W, Ci, Co, KH, KW, stride, out_nchw);
  if (S < 2) return rai_conv2d_bias_relu_fwd_v(x, w, b, B, H, W, Ci, Co, KH, KW, stride, out_nchw, y, 0, stream);
  if (!x || !w || !b || !y || !part) return RAI_E_NULLPTR;
  if (part_bytes < rai_conv2d_fwd_splitk_bytes(B, H, W, Ci, Co, KH, KW, stride, out_nchw)) return RAI_E_WORKSPACE;
  if (((uintptr_t)x | (uintptr_t)w | (uintptr_t)b | (uintptr_t)y | (uintptr_t)part) & 15) return RAI_E_SHAPE;
  if ((int64_t)H * W * Ci * B > (1LL << 40)) return RAI_E_SHAPE;
  ConvFwdArgs a;
  a.x = x;
  a.xu8 = nullptr;
  a.xdiv = 1.f;
  a.xinv = 1.f;
  a.w = w;
  a.b = b;
  a.y = y;
  a.H = H;
  a.W = W;
  a.Ci = Ci;
  a.Co = Co;
  a.KW = KW;
  a.S = stride;
  a.OH = (H - KH) / stride + 1;
  a.OW = (W - KW) / stride + 1;
  a.K = KH * KW * Ci;
  a.M = B * a.OH * a.OW;
  a.ksplit = S;
  a.part = part;
  hipStream_t st = rai_stream(stream);
  const bool buf = B * H * W * (int64_t)Ci * 4 < (1LL << 31);
  const size_t lds32 = (size_t)32 * (a.K + 4) * 4;
  const int ncu = num_cus();
  const int64_t wg32 = ncu / (Co / 32), wg64 = ncu / (Co / 64);
  const int64_t rounds32 = ((a.M + 255) / 256 + wg32 - 1) / wg32, rounds64 = ((a.M + 63) / 64 + wg64 - 1) / wg64;
  int e;
  if (lds32 + CV_MAXCHUNK * 4 <= 160 * 1024 && 2 * rounds32 <= rounds64)
    e = buf ? launch_fwd_lds<2, 2, 1, 8, 3, true>(a, false, st) : launch_fwd_lds<2, 2, 1, 8, 3>(a, false, st);
  else
    e = buf ? launch_fwd_lds<2, 1, 2, 4, 4, true>(a, false, st) : launch_fwd_lds<2, 1, 2, 4, 4>(a, false, st);
  if (e != RAI_OK) return e;
  const int OHW = a.OH * a.OW;
  if (out_nchw) {
    hipLaunchKernelGGL(conv_fwd_splitk_reduce_kernel, dim3((unsigned)B), dim3(256), 0, st, part, S, a.M, Co, b, y, 1,
                       OHW);
  } else {
    int64_t blocks = (a.M * Co / 4 + 255) / 256;
    if (blocks > 4 * ncu) blocks = 4 * ncu;
    hipLaunchKernelGGL(conv_fwd_splitk_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, st, part, S, a.M, Co, b, y,
                       0, OHW);
  }
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}

extern "C" int rai_conv2d_bias_relu_fwd(const float* x, const float* w, const float* b, int64_t B, int32_t H,
                                       int32_t W, int32_t Ci, int32_t Co, int32_t KH, int32_t KW, int32_t stride,
                                       int32_t out_nchw, float* y, void* stream) {
  return rai_conv2d_bias_relu_fwd_v(x, w, b, B, H, W, Ci, Co, KH, KW, stride, out_nchw, y, 0, stream);
}

extern "C" int rai_conv2d_wgrad(const float* x, const float* dz, int64_t B, int32_t H, int32_t W, int32_t Ci,
                                int32_t Co, int32_t KH, int32_t KW, int32_t stride, float* dw, int32_t accumulate,
                                void* workspace, int64_t workspace_bytes, void* stream) {
  return rai_conv2d_wgrad_v(x, dz, B, H, W, Ci, Co, KH, KW, stride, dw, accumulate, workspace, workspace_bytes, 0, 0,
                            stream);
}

extern "C" int rai_conv2d_dgrad_v(const float* dz, const float* w, int64_t B, int32_t H, int32_t W, int32_t Ci,
                                  int32_t Co, int32_t KH, int32_t KW, int32_t stride, float* dx, int32_t variant,
                                  void* stream) {
  if (B < 0 || H < 1 || W < 1 || Ci < 1 || Co < 1 || KH < 1 || KW < 1 || stride < 1 || KH > H || KW > W)
    return RAI_E_SHAPE;  // not a convolution
  if ((Ci != 32 && Ci != 64) || Co % 16 || KH % stride || KW % stride)
    return RAI_E_UNSUPPORTED;  // a valid shape these kernels are not instantiated for (the caller falls back)
  if (B == 0) return RAI_OK;
  if (!dz || !w || !dx) return RAI_E_NULLPTR;
  if (((uintptr_t)dz | (uintptr_t)w | (uintptr_t)dx) & 15) return RAI_E_SHAPE;
  ConvDgradArgs a;
  a.dz = dz;
  a.y = nullptr;
  a.w = w;
  a.dx = dx;
  a.B = B;
  a.H = H;
  a.W = W;
  a.Ci = Ci;
  a.Co = Co;
  a.KH = KH;
  a.KW = KW;
  a.S = stride;
  a.OH = (H - KH) / stride + 1;
  a.OW = (W - KW) / stride + 1;
  const int64_t maxcls = B * ((H + stride - 1) / stride) * ((W + stride - 1) / stride);
  hipStream_t st = rai_stream(stream);
  // variant 0: the per-image GEMM + col2im form where it is instantiated (NatureCNN conv2 / conv3), with
  // buffer loads (B = 256: conv2 21.9 us with 2 quads in flight, conv3 18.2 us with 3, against 26.0 /
  // 19.1 us with pointer loads and MIOpen's 33.2 / 27.7; profiles/r4f_dgrad_probe.txt), else the
  // pixel-class form; 3: the per-image form with pointer loads (RAI_E_UNSUPPORTED where not instantiated)
  const int kind = dgrad_img_kind(a);
  if (variant == 0 && kind == 1) return launch_dgrad_img<9, 4, 256, 3, true>(a, st);
  if (variant == 0 && kind == 2) return launch_dgrad_img<4, 6, 512, 2, true>(a, st);
  if (variant == 3) {
    if (kind == 1) return launch_dgrad_img<9, 4, 256>(a, st);
    if (kind == 2) return launch_dgrad_img<4, 6, 512>(a, st);
    if (variant == 3) return RAI_E_UNSUPPORTED;
  }
  if (variant >= 5 && variant <= 7) {  // the per-image form: buffer loads (5), + 3 / 4 quads in flight (6 / 7)
    if (kind == 1 && variant == 5) return launch_dgrad_img<9, 4, 256, 2, true>(a, st);
    if (kind == 1 && variant == 6) return launch_dgrad_img<9, 4, 256, 3, true>(a, st);
    if (kind == 1 && variant == 7) return launch_dgrad_img<9, 4, 256, 4, true>(a, st);
    if (kind == 2 && variant == 5) return launch_dgrad_img<4, 6, 512, 2, true>(a, st);
    if (kind == 2 && variant == 6) return launch_dgrad_img<4, 6, 512, 3, true>(a, st);
    if (kind == 2 && variant == 7) return launch_dgrad_img<4, 6, 512, 4, true>(a, st);
    return RAI_E_UNSUPPORTED;
  }
  if (variant == 4) {  // the per-image form with the weight operand staged through LDS
    if (kind == 1) return launch_dgrad_img_lds<9, 4, 256, 3>(a, st);
    if (kind == 2) return launch_dgrad_img_lds<4, 6, 512, 1>(a, st);
    return RAI_E_UNSUPPORTED;
  }
  if (variant == 1 && Ci == 32) return launch_dgrad_lds<2, 2, 1>(a, st);  // LDS weights, 32 ci x 32 px per wave
  if (variant == 2 && Ci == 32) return launch_dgrad_lds<2, 1, 1>(a, st);  // LDS weights, 32 ci x 16 px per wave
  if (variant == 1 && Ci == 64) return launch_dgrad_lds<2, 1, 2>(a, st);  // LDS weights, ci halves over waves
  if (variant == 2 && Ci == 64) return launch_dgrad_lds<4, 1, 1>(a, st);  // LDS weights, 64 ci x 16 px per wave
  if (Ci == 32) {  // 32 rows: four column blocks per wave
    const int64_t gx = (maxcls + 255) / 256;
    hipLaunchKernelGGL((conv_dgrad_kernel<2, 4>), dim3((unsigned)gx, (unsigned)(stride * stride)), dim3(CV_THREADS),
                       0, st, a);
  } else {  // 64 rows: one column block per wave
    const int64_t gx = (maxcls + 63) / 64;
    hipLaunchKernelGGL((conv_dgrad_kernel<4, 1>), dim3((unsigned)gx, (unsigned)(stride * stride)), dim3(CV_THREADS),
                       0, st, a);
  }
  RAI_LAUNCH_CHECK();
  return RAI_OK;
}

extern "C" int rai_conv2d_dgrad(const float* dz, const float* w, int64_t B, int32_t H, int32_t W, int32_t Ci,
                                int32_t Co, int32_t KH, int32_t KW, int32_t stride, float* dx, void* stream) {
  return rai_conv2d_dgrad_v(dz, w, B, H, W, Ci, Co, KH, KW, stride, dx, 0, stream);
}

extern "C" int rai_conv2d_dgrad_relu(const float* dy, const float* y, const float* w, int64_t B, int32_t H, int32_t W,
                                     int32_t Ci, int32_t Co, int32_t KH, int32_t KW, int32_t stride, float* dx,
                                     void* stream) {
  if (B < 0 || H < 1 || W < 1 || Ci < 1 || Co < 1 || KH < 1 || KW < 1 || stride < 1 || KH > H || KW > W)
    return RAI_E_SHAPE;  // not a convolution
  if (Ci < 16 || Co % 16 || KH % stride || KW % stride) return RAI_E_UNSUPPORTED;  // not instantiated: fall back
  if (B == 0) return RAI_OK;
  if (!dy || !y || !w || !dx) return RAI_E_NULLPTR;
  if (((uintptr_t)dy | (uintptr_t)y | (uintptr_t)w | (uintptr_t)dx) & 15) return RAI_E_SHAPE;
  ConvDgradArgs a;
  a.dz = dy;
  a.y = y;
  a.w = w;
  a.dx = dx;
  a.B = B;
  a.H = H;
  a.W = W;
  a.Ci = Ci;
  a.Co = Co;
  a.KH = KH;
  a.KW = KW;
  a.S = stride;
  a.OH = (H - KH) / stride + 1;
  a.OW = (W - KW) / stride + 1;
  hipStream_t st = rai_stream(stream);
  const int kind = dgrad_img_kind(a);
  if (kind == 1) return launch_dgrad_img<9, 4, 256, 3, true, true>(a, st);
  if (kind == 2) return launch_dgrad_img<4, 6, 512, 2, true, true>(a, st);
  return RAI_E_UNSUPPORTED;
}
