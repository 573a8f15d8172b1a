// Ceiling study (not part of the product): which streaming structures reach
// the most read+write bandwidth on this box, from HBM (4 GiB arrays) and from
// the Infinity Cache (in-place sweeps of 128 MiB), to decide whether a
// persistent, software-pipelined pass kernel can beat the current
// 2-workgroups-per-CU tile structure.
//   read      : sum of 16-B loads (read bandwidth alone)
//   write     : 16-B stores
//   copy/U    : out-of-place, U x 16 B per lane, one tile per workgroup
//   inplace/U : a[i] = c * a[i], U x 16 B per lane, one tile per workgroup
//   tile2wg   : the pass shape: 16 loads/lane, 4 LDS re-layouts of 64 KiB,
//               24 FMA layers, 16 stores, 2 workgroups per CU (in place)
//   pipe      : persistent, 2 workgroups per CU, the next tile's 16 loads
//               issued before the current tile's FMA layers / re-layouts /
//               stores (register double buffer), in place
// Build: hipcc --offload-arch=gfx950 -O3 tools/hbm_ceiling.hip -o tools/hbm_ceiling
#include <hip/hip_runtime.h>

#include <cstdio>

#define CHECK(x)                                                         \
  do {                                                                   \
    hipError_t e = (x);                                                  \
    if (e != hipSuccess) {                                               \
      printf("%s: %s\n", #x, hipGetErrorString(e));                      \
      return 1;                                                          \
    }                                                                    \
  } while (0)

typedef double d2v __attribute__((ext_vector_type(2)));

template <int U>
__global__ __launch_bounds__(256) void k_read(const d2v* __restrict__ a, double* out) {
  const size_t base = (size_t)blockIdx.x * (256 * U) + threadIdx.x;
  d2v s = {0, 0};
#pragma unroll
  for (int u = 0; u < U; ++u) s += __builtin_nontemporal_load(&a[base + 256 * u]);
  if (s.x == 12345.0) out[0] = s.y;
}

template <int U>
__global__ __launch_bounds__(256) void k_write(d2v* __restrict__ a) {
  const size_t base = (size_t)blockIdx.x * (256 * U) + threadIdx.x;
  d2v z = {1.0, 2.0};
#pragma unroll
  for (int u = 0; u < U; ++u) __builtin_nontemporal_store(z, &a[base + 256 * u]);
}

template <int U>
__global__ __launch_bounds__(256) void k_copy(const d2v* __restrict__ a, d2v* __restrict__ b) {
  const size_t base = (size_t)blockIdx.x * (256 * U) + threadIdx.x;
  d2v v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(&a[base + 256 * u]);
#pragma unroll
  for (int u = 0; u < U; ++u) __builtin_nontemporal_store(v[u], &b[base + 256 * u]);
}

template <int U>
__global__ __launch_bounds__(256) void k_inplace(d2v* __restrict__ a, double c) {
  const size_t base = (size_t)blockIdx.x * (256 * U) + threadIdx.x;
  d2v v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(&a[base + 256 * u]);
#pragma unroll
  for (int u = 0; u < U; ++u) __builtin_nontemporal_store(v[u] * c, &a[base + 256 * u]);
}


template <int U>
__global__ __launch_bounds__(256) void k_write_plain(d2v* __restrict__ a) {
  const size_t base = (size_t)blockIdx.x * (256 * U) + threadIdx.x;
  d2v z = {1.0, 2.0};
#pragma unroll
  for (int u = 0; u < U; ++u) a[base + 256 * u] = z;
}

template <int U>
__global__ __launch_bounds__(256) void k_inplace_plain(d2v* __restrict__ a, double c) {
  const size_t base = (size_t)blockIdx.x * (256 * U) + threadIdx.x;
  d2v v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = a[base + 256 * u];
#pragma unroll
  for (int u = 0; u < U; ++u) a[base + 256 * u] = v[u] * c;
}

// loads nontemporal, stores plain (and the reverse)
template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k_inplace_mix(d2v* __restrict__ a, double c) {
  const size_t base = (size_t)blockIdx.x * (256 * U) + threadIdx.x;
  d2v v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = NTL ? __builtin_nontemporal_load(&a[base + 256 * u]) : a[base + 256 * u];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (NTS) __builtin_nontemporal_store(v[u] * c, &a[base + 256 * u]);
    else a[base + 256 * u] = v[u] * c;
  }
}

template <int LAYERS>
__device__ __forceinline__ void fma_layers(d2v (&v)[16], double f) {
#pragma unroll
  for (int l = 0; l < LAYERS; ++l) {
    const int q = l & 3;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (r & (1 << q)) continue;
      d2v& u = v[r];
      d2v& w = v[r | (1 << q)];
      d2v nu, nw;
      nu.x = fma(-f, w.y, u.x); nu.y = fma(f, w.x, u.y);
      nw.x = fma(-f, u.y, w.x); nw.y = fma(f, u.x, w.y);
      u = nu;
      w = nw;
    }
  }
}

template <int E>
__device__ __forceinline__ void relayout(d2v (&v)[16], d2v* s, int t) {
  constexpr int e = E;
  // alternate between two conflict-free layouts
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int y = (e & 1) ? ((t << 4) | r) : (t + 256 * r);
    s[y ^ ((y >> 4) & 15)] = v[r];
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int y = (e & 1) ? (t + 256 * r) : ((t << 4) | r);
    v[r] = s[y ^ ((y >> 4) & 15)];
  }
  __syncthreads();
}

template <int LAYERS, int EXCH>
__device__ __forceinline__ void body(d2v (&v)[16], double f, d2v* s, int t) {
  constexpr int per = LAYERS / (EXCH + 1);
  fma_layers<per>(v, f);
  if constexpr (EXCH > 0) { relayout<0>(v, s, t); fma_layers<per>(v, f); }
  if constexpr (EXCH > 1) { relayout<1>(v, s, t); fma_layers<per>(v, f); }
  if constexpr (EXCH > 2) { relayout<0>(v, s, t); fma_layers<per>(v, f); }
  if constexpr (EXCH > 3) { relayout<1>(v, s, t); fma_layers<per>(v, f); }
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] *= (1.0 + f);  // never elided: a runtime scale
}

template <int LAYERS, int EXCH>
__global__ __launch_bounds__(256, 2) void k_tile2wg(d2v* __restrict__ a, double f) {
  __shared__ d2v s[4096];
  const int t = threadIdx.x;
  const size_t base = (size_t)blockIdx.x * 4096;
  d2v v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = __builtin_nontemporal_load(&a[base + t + 256 * r]);
  body<LAYERS, EXCH>(v, f, s, t);
#pragma unroll
  for (int r = 0; r < 16; ++r) __builtin_nontemporal_store(v[r], &a[base + t + 256 * r]);
}

// persistent, register double buffer: loads of tile i+1 in flight while tile i
// computes and stores
template <int LAYERS, int EXCH>
__global__ __launch_bounds__(256, 2) void k_pipe(d2v* __restrict__ a, double f, int n_tiles) {
  __shared__ d2v s[4096];
  const int t = threadIdx.x;
  int tile = blockIdx.x;
  if (tile >= n_tiles) return;
  d2v nx[16];
#pragma unroll
  for (int r = 0; r < 16; ++r)
    nx[r] = __builtin_nontemporal_load(&a[(size_t)tile * 4096 + t + 256 * r]);
  for (; tile < n_tiles; tile += gridDim.x) {
    d2v v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = nx[r];
    const int nt = tile + gridDim.x;
    if (nt < n_tiles) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        nx[r] = __builtin_nontemporal_load(&a[(size_t)nt * 4096 + t + 256 * r]);
    }
    body<LAYERS, EXCH>(v, f, s, t);
#pragma unroll
    for (int r = 0; r < 16; ++r) __builtin_nontemporal_store(v[r], &a[(size_t)tile * 4096 + t + 256 * r]);
  }
}

template <typename F>
float time_it(F f, int reps) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  f();
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
  int dev = 0, ncu = 0;
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const size_t n = (size_t)1 << 28;  // 4 GiB per array
  d2v *a, *b;
  double* out;
  CHECK(hipMalloc(&a, n * 16));
  CHECK(hipMalloc(&b, n * 16));
  CHECK(hipMalloc(&out, 64));
  CHECK(hipMemset(a, 0, n * 16));
  CHECK(hipMemset(b, 0, n * 16));
  auto rep = [&](const char* name, double bytes, float ms) {
    printf("%-40s %9.3f ms  %7.0f GB/s\n", name, ms, bytes / ms / 1e6);
  };
  const double rw = 2.0 * n * 16;
  rep("read U=16", n * 16.0, time_it([&] { hipLaunchKernelGGL((k_read<16>), dim3(n / 4096), dim3(256), 0, 0, a, out); }, 10));
  rep("read U=4", n * 16.0, time_it([&] { hipLaunchKernelGGL((k_read<4>), dim3(n / 1024), dim3(256), 0, 0, a, out); }, 10));
  rep("write U=16", n * 16.0, time_it([&] { hipLaunchKernelGGL((k_write<16>), dim3(n / 4096), dim3(256), 0, 0, b); }, 10));
  rep("copy U=4", rw, time_it([&] { hipLaunchKernelGGL((k_copy<4>), dim3(n / 1024), dim3(256), 0, 0, a, b); }, 10));
  rep("copy U=16", rw, time_it([&] { hipLaunchKernelGGL((k_copy<16>), dim3(n / 4096), dim3(256), 0, 0, a, b); }, 10));
  rep("inplace U=4", rw, time_it([&] { hipLaunchKernelGGL((k_inplace<4>), dim3(n / 1024), dim3(256), 0, 0, a, 1.0); }, 10));
  rep("write plain U=16", n * 16.0, time_it([&] { hipLaunchKernelGGL((k_write_plain<16>), dim3(n / 4096), dim3(256), 0, 0, b); }, 10));
  rep("write plain U=4", n * 16.0, time_it([&] { hipLaunchKernelGGL((k_write_plain<4>), dim3(n / 1024), dim3(256), 0, 0, b); }, 10));
  rep("inplace plain U=4", rw, time_it([&] { hipLaunchKernelGGL((k_inplace_plain<4>), dim3(n / 1024), dim3(256), 0, 0, a, 1.0); }, 10));
  rep("inplace plain U=16", rw, time_it([&] { hipLaunchKernelGGL((k_inplace_plain<16>), dim3(n / 4096), dim3(256), 0, 0, a, 1.0); }, 10));
  rep("inplace ntload/plainstore U=16", rw, time_it([&] { hipLaunchKernelGGL((k_inplace_mix<16, true, false>), dim3(n / 4096), dim3(256), 0, 0, a, 1.0); }, 10));
  rep("inplace plainload/ntstore U=16", rw, time_it([&] { hipLaunchKernelGGL((k_inplace_mix<16, false, true>), dim3(n / 4096), dim3(256), 0, 0, a, 1.0); }, 10));
  rep("inplace U=16", rw, time_it([&] { hipLaunchKernelGGL((k_inplace<16>), dim3(n / 4096), dim3(256), 0, 0, a, 1.0); }, 10));
  const int tiles = (int)(n / 4096);
#define RUN2(LY, EX)                                                                           \
  rep("tile2wg L=" #LY " X=" #EX, rw, time_it([&] { hipLaunchKernelGGL((k_tile2wg<LY, EX>), dim3(tiles), dim3(256), 0, 0, a, 0.0); }, 10)); \
  rep("pipe    L=" #LY " X=" #EX, rw, time_it([&] { hipLaunchKernelGGL((k_pipe<LY, EX>), dim3(2 * ncu), dim3(256), 0, 0, a, 0.0, tiles); }, 10));
  RUN2(0, 0)
  RUN2(24, 0)
  RUN2(0, 4)
  RUN2(24, 4)
  // Infinity-Cache resident: 128 MiB in place, repeated
  const int small = (int)((128u << 20) / (4096 * 16));
  const double rws = 2.0 * (128u << 20);
#define RUNS(LY, EX)                                                                           \
  rep("IC128 tile2wg L=" #LY " X=" #EX, rws, time_it([&] { hipLaunchKernelGGL((k_tile2wg<LY, EX>), dim3(small), dim3(256), 0, 0, a, 0.0); }, 50)); \
  rep("IC128 pipe    L=" #LY " X=" #EX, rws, time_it([&] { hipLaunchKernelGGL((k_pipe<LY, EX>), dim3(2 * ncu), dim3(256), 0, 0, a, 0.0, small); }, 50));
  RUNS(0, 0)
  RUNS(24, 4)
  rep("IC128 inplace U=16", rws, time_it([&] { hipLaunchKernelGGL((k_inplace<16>), dim3(small), dim3(256), 0, 0, a, 1.0); }, 50));
  return 0;
}
