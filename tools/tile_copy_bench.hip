// Ceiling study for the pass-kernel structure (not part of the product):
// read+write 8 GiB with (a) a grid-stride float4 copy, (b) the pass kernel's
// tile shape: 256 lanes x 16 x 16-B loads of a 4096-amplitude tile, k LDS
// re-layouts through 64 KiB of LDS, 16 stores, 2 workgroups per CU.
// Build: hipcc --offload-arch=gfx950 -O3 tools/tile_copy_bench.hip -o /tmp/tcb
#include <hip/hip_runtime.h>

#include <cstdio>

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      printf("%s: %s\n", #x, hipGetErrorString(e));                                   \
      return 1;                                                                       \
    }                                                                                 \
  } while (0)

__global__ void copy_stream(const double2* __restrict__ a, double2* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    b[i] = a[i];
}

typedef double d2v __attribute__((ext_vector_type(2)));
template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_unroll(const d2v* __restrict__ a,
                                                   d2v* __restrict__ b) {
  const unsigned base = blockIdx.x * (256u * U) + threadIdx.x;
  d2v v[U];
#pragma unroll
  for (int u = 0; u < U; ++u)
    v[u] = NT ? __builtin_nontemporal_load(&a[base + 256u * u]) : a[base + 256u * u];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (NT) __builtin_nontemporal_store(v[u], &b[base + 256u * u]);
    else b[base + 256u * u] = v[u];
  }
}

template <int EXCH, int LDS_KB>
__global__ __launch_bounds__(256, 2) void copy_tile(const double2* a, double2* b) {
  __shared__ double2 s[LDS_KB * 64];
  const int t = threadIdx.x;
  const size_t base = (size_t)blockIdx.x * 4096;
  double2 v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = a[base + t + 256 * r];
  for (int e = 0; e < EXCH; ++e) {
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) s[(t + 256 * r) ^ ((t >> 4) & 15)] = v[r];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = s[((t << 4) | r) ^ (t & 15)];
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) b[base + t + 256 * r] = v[r];
}

template <typename F>
float time_it(F f, int reps) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  f();
  (void)hipEventRecord(e0);
  for (int i = 0; i < reps; ++i) f();
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms / reps;
}

int main() {
  const size_t n = (size_t)1 << 28;  // 4 GiB per array, 8 GiB moved
  double2 *a, *b;
  CHECK(hipMalloc(&a, n * 16));
  CHECK(hipMalloc(&b, n * 16));
  CHECK(hipMemset(a, 0, n * 16));
  const double bytes = 2.0 * n * 16;
  auto report = [&](const char* name, float ms) {
    printf("%-28s %8.3f ms  %7.0f GB/s\n", name, ms, bytes / ms / 1e6);
  };
  report("stream copy (2048x256)", time_it([&] {
    hipLaunchKernelGGL(copy_stream, dim3(2048), dim3(256), 0, 0, a, b, n);
  }, 10));
  report("stream copy (8192x256)", time_it([&] {
    hipLaunchKernelGGL(copy_stream, dim3(8192), dim3(256), 0, 0, a, b, n);
  }, 10));
  report("unroll4", time_it([&] {
    hipLaunchKernelGGL((copy_unroll<4, false>), dim3(n / 1024), dim3(256), 0, 0, (const d2v*)a, (d2v*)b);
  }, 10));
  report("unroll16", time_it([&] {
    hipLaunchKernelGGL((copy_unroll<16, false>), dim3(n / 4096), dim3(256), 0, 0, (const d2v*)a, (d2v*)b);
  }, 10));
  report("unroll4 nt", time_it([&] {
    hipLaunchKernelGGL((copy_unroll<4, true>), dim3(n / 1024), dim3(256), 0, 0, (const d2v*)a, (d2v*)b);
  }, 10));
  report("unroll16 nt", time_it([&] {
    hipLaunchKernelGGL((copy_unroll<16, true>), dim3(n / 4096), dim3(256), 0, 0, (const d2v*)a, (d2v*)b);
  }, 10));
  const dim3 g(n / 4096);
  report("tile, 0 exchanges, 64KiB", time_it([&] {
    hipLaunchKernelGGL((copy_tile<0, 64>), g, dim3(256), 0, 0, a, b);
  }, 10));
  report("tile, 0 exchanges, 1KiB", time_it([&] {
    hipLaunchKernelGGL((copy_tile<0, 1>), g, dim3(256), 0, 0, a, b);
  }, 10));
  report("tile, 1 exchange", time_it([&] {
    hipLaunchKernelGGL((copy_tile<1, 64>), g, dim3(256), 0, 0, a, b);
  }, 10));
  report("tile, 2 exchanges", time_it([&] {
    hipLaunchKernelGGL((copy_tile<2, 64>), g, dim3(256), 0, 0, a, b);
  }, 10));
  report("tile, 4 exchanges", time_it([&] {
    hipLaunchKernelGGL((copy_tile<4, 64>), g, dim3(256), 0, 0, a, b);
  }, 10));
  return 0;
}
