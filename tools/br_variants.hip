// Diagnostic microbenchmark (not part of the product or the tests): where the time of the bias +
// ReLU backward (csrc/se_block.hip, rai_bias_relu_bwd) goes at the C3 conv1 shape (256 x 20 x 20
// rows, 32 channels).  Variants of the row pass, each timed with HIP events over 200 launches:
//   ew        dx = dy * (y > 0) only, one float4 per thread (the elementwise yardstick)
//   pass      the row pass + per-workgroup partial stores, no arrival counter, no tail
//   counter   pass + the drained stores + one agent-scope atomic per workgroup, no tail
//   full      the shipped kernel's structure (pass + counter + last-arriver tail)
// at several (rows per lane, max workgroups).
//   hipcc -O3 --offload-arch=gfx950 -o tools/br_variants tools/br_variants.hip && tools/br_variants
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

using f4 = float __attribute__((ext_vector_type(4)));
typedef unsigned int u4v __attribute__((ext_vector_type(4)));
#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);      \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

constexpr int T = 256;
constexpr int SC1 = 16;

__global__ __launch_bounds__(T) void ew_kernel(const f4* dy, const f4* y, int64_t n4, f4* dx) {
  const int64_t i = blockIdx.x * (int64_t)T + threadIdx.x;
  if (i < n4) {
    const f4 g = dy[i], yv = y[i];
    f4 o;
    for (int q = 0; q < 4; ++q) o[q] = yv[q] <= 0.f ? 0.f : g[q];
    dx[i] = o;
  }
}

template <int MODE, int UNROLL, int NT = T, int TAIL = 16>  // MODE 0 pass, 1 counter, 2 full, 3 full two-level
__global__ __launch_bounds__(NT) void rows_kernel(const f4* __restrict__ dy, const f4* __restrict__ y, int C4,
                                                 int64_t rows, int64_t rpb, f4* __restrict__ dx, float* partial,
                                                 int* counter, float* db) {
  __shared__ f4 part[NT];
  __shared__ int last;
  const int tid = threadIdx.x, lanes = NT / C4, c4 = tid % C4, lane = tid / C4, C = 4 * C4;
  const int nb = gridDim.x;
  const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(partial, 0, nb * C * 4, 0x00020000);
  const int64_t r0 = blockIdx.x * rpb, r1 = min(rows, r0 + rpb);
  f4 acc = f4{0.f, 0.f, 0.f, 0.f};
  for (int64_t r = r0 + lane; r < r1; r += (int64_t)lanes * UNROLL) {
    f4 g[UNROLL], yv[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int64_t rr = r + (int64_t)u * lanes;
      const int64_t i = (rr < r1 ? rr : r) * C4 + c4;
      g[u] = dy[i];
      yv[u] = y[i];
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int64_t rr = r + (int64_t)u * lanes;
      if (rr < r1) {
        f4 o;
        for (int q = 0; q < 4; ++q) o[q] = yv[u][q] <= 0.f ? 0.f : g[u][q];
        dx[rr * C4 + c4] = o;
        acc += o;
      }
    }
  }
  part[tid] = acc;
  __syncthreads();
  for (int h = lanes / 2; h >= 1; h /= 2) {
    if (lane < h) part[tid] += part[tid + h * C4];
    __syncthreads();
  }
  if (tid < C4)
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, part[tid]), prs, (blockIdx.x * C + 4 * tid) * 4, 0,
                                           SC1);
  if (MODE == 0) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (MODE == 3) {  // counters 1..8 per group blockIdx % 8 (64 B apart), counter 0 the groups
    if (tid == 0) {
      const int g = blockIdx.x & 7, gsize = (nb - g + 7) >> 3, ng = nb < 8 ? nb : 8;
      int* cg = counter + 16 * (1 + g);
      last = 0;
      if (__hip_atomic_fetch_add(cg, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gsize - 1) {
        __hip_atomic_store(cg, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = __hip_atomic_fetch_add(counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ng - 1;
      }
    }
  } else if (tid == 0) {
    last = __hip_atomic_fetch_add(counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nb - 1;
  }
  __syncthreads();
  if (MODE == 1 || !last) {
    if (MODE == 1 && last && tid == 0) __hip_atomic_store(counter, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  f4 s[TAIL];
  for (int u = 0; u < TAIL; ++u) s[u] = f4{0.f, 0.f, 0.f, 0.f};
  for (int w0 = lane; w0 < nb; w0 += TAIL * lanes) {
    f4 v[TAIL];
#pragma unroll
    for (int u = 0; u < TAIL; ++u)
      v[u] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(prs, ((w0 + u * lanes) * C + 4 * c4) * 4, 0,
                                                                          SC1));
#pragma unroll
    for (int u = 0; u < TAIL; ++u)
      if (w0 + u * lanes < nb) s[u] += v[u];
  }
  for (int h = TAIL / 2; h >= 1; h /= 2)
    for (int u = 0; u < h; ++u) s[u] += s[u + h];
  part[tid] = s[0];
  __syncthreads();
  for (int h = lanes / 2; h >= 1; h /= 2) {
    if (lane < h) part[tid] += part[tid + h * C4];
    __syncthreads();
  }
  if (tid < C4)
    for (int q = 0; q < 4; ++q) db[4 * tid + q] += part[tid][q];
  if (tid == 0) __hip_atomic_store(counter, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <typename F>
float timeit(F&& launch, int reps = 200) {
  for (int i = 0; i < 5; ++i) launch();
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventRecord(a, 0);
  for (int i = 0; i < reps; ++i) launch();
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  return ms * 1e3f / reps;
}

int main() {
  struct Shape {
    const char* name;
    int64_t rows;
    int C;
  } shapes[] = {{"conv1", 256 * 400, 32}, {"conv2", 256 * 81, 64}, {"conv3", 256 * 49, 64}};
  for (const Shape& sh : shapes) {
    const int64_t n = sh.rows * sh.C, n4 = n / 4;
    const int C4 = sh.C / 4, lanes = T / C4;
    float *dy, *y, *dx, *part, *db;
    int* counter;
    CK(hipMalloc(&dy, n * 4));
    CK(hipMalloc(&y, n * 4));
    CK(hipMalloc(&dx, n * 4));
    CK(hipMalloc(&part, 4096 * sh.C * 4));
    CK(hipMalloc(&db, sh.C * 4));
    CK(hipMalloc(&counter, 1024));
    CK(hipMemset(counter, 0, 1024));
    CK(hipMemset(db, 0, sh.C * 4));
    std::vector<float> h(n);
    for (int64_t i = 0; i < n; ++i) h[i] = (float)((i * 2654435761u) % 1000) / 500.f - 1.f;
    CK(hipMemcpy(dy, h.data(), n * 4, hipMemcpyHostToDevice));
    for (int64_t i = 0; i < n; ++i) h[i] = (float)((i * 40503u + 7) % 1000) / 500.f - 1.f;
    CK(hipMemcpy(y, h.data(), n * 4, hipMemcpyHostToDevice));
    const float t_ew = timeit([&] {
      hipLaunchKernelGGL(ew_kernel, dim3((unsigned)((n4 + T - 1) / T)), dim3(T), 0, 0, (const f4*)dy, (const f4*)y,
                         n4, (f4*)dx);
    });
    std::printf("%s rows %lld C %d  (%.1f MB moved)  ew %.2f us\n", sh.name, (long long)sh.rows, sh.C, 3.0 * n * 4 / 1e6,
                t_ew);
    for (int NTsel : {256, 1024}) {
      const int nt = NTsel, lanes_nt = nt / C4;
      for (int rpl : {4, 8}) {
        for (int maxb : {128, 256, 512, 1024}) {
          int64_t blocks = (sh.rows + (int64_t)rpl * lanes_nt - 1) / ((int64_t)rpl * lanes_nt);
          if (blocks > maxb) blocks = maxb;
          const int64_t rpb = (sh.rows + blocks - 1) / blocks;
          blocks = (sh.rows + rpb - 1) / rpb;
          auto L = [&](auto kern) {
            return timeit([&] {
              hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(nt), 0, 0, (const f4*)dy, (const f4*)y, C4,
                                 sh.rows, rpb, (f4*)dx, part, counter, db);
            });
          };
          float p, c, f, h;
          if (nt == 256) {
            p = L(rows_kernel<0, 4>), c = L(rows_kernel<1, 4>), f = L(rows_kernel<2, 4>), h = L(rows_kernel<3, 4>);
          } else {
            p = L(rows_kernel<0, 4, 1024, 8>), c = L(rows_kernel<1, 4, 1024, 8>), f = L(rows_kernel<2, 4, 1024, 8>),
            h = L(rows_kernel<3, 4, 1024, 8>);
          }
          std::printf("  threads %4d rows/lane %2d maxb %4d -> %4lld wg: pass %6.2f counter %6.2f full %6.2f "
                      "two-level %6.2f us\n", nt, rpl, maxb, (long long)blocks, p, c, f, h);
        }
      }
    }
    CK(hipFree(dy));
    CK(hipFree(y));
    CK(hipFree(dx));
    CK(hipFree(part));
    CK(hipFree(db));
    CK(hipFree(counter));
  }
  return 0;
}
