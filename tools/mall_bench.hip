// Residency study (not part of the product): in-place read+write sweeps of a
// buffer of S bytes repeated back to back, for S from 16 MiB (Infinity-Cache
// resident) to 4 GiB (HBM), in the pass kernel's tile shape (4096 complex128
// amplitudes per workgroup, 16 per lane, optional LDS re-layouts).  Answers:
// does a state batch that stays resident in the 256 MiB Infinity Cache across
// consecutive passes stream faster than HBM?  Plain launches and a hipGraph of
// the same launches (launch-gap check).
// Build: hipcc --offload-arch=gfx950 -O3 tools/mall_bench.hip -o /tmp/mallb
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      printf("%s: %s\n", #x, hipGetErrorString(e));                                   \
      return 1;                                                                       \
    }                                                                                 \
  } while (0)

template <int EXCH>
__global__ __launch_bounds__(256, 2) void tile_rw(double2* a, double s) {
  __shared__ double2 sh[4096];
  const int t = threadIdx.x;
  const size_t base = (size_t)blockIdx.x * 4096;
  double2 v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = a[base + t + 256 * r];
  for (int e = 0; e < EXCH; ++e) {
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) sh[(t + 256 * r) ^ ((t >> 4) & 15)] = v[r];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = sh[((t << 4) | r) ^ (t & 15)];
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    v[r].x *= s;
    v[r].y *= s;
    a[base + t + 256 * r] = v[r];
  }
}

int main() {
  const size_t max_bytes = (size_t)4 << 30;
  double2* a;
  CHECK(hipMalloc(&a, max_bytes));
  CHECK(hipMemset(a, 0, max_bytes));
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const size_t mib[] = {16, 32, 64, 96, 128, 160, 192, 224, 256, 384, 1024, 4096};
  const int reps = 40;
  printf("%8s %6s %10s %10s %10s %10s\n", "MiB", "exch", "us/launch", "GB/s", "graph_us", "graph_GB/s");
  for (size_t m : mib) {
    const size_t bytes = m << 20;
    const unsigned grid = (unsigned)(bytes / 16 / 4096);
    for (int ex : {0, 4}) {
      auto launch = [&]() {
        if (ex == 0) hipLaunchKernelGGL(tile_rw<0>, dim3(grid), dim3(256), 0, st, a, 1.0);
        else hipLaunchKernelGGL(tile_rw<4>, dim3(grid), dim3(256), 0, st, a, 1.0);
      };
      for (int w = 0; w < 5; ++w) launch();
      CHECK(hipEventRecord(e0, st));
      for (int i = 0; i < reps; ++i) launch();
      CHECK(hipEventRecord(e1, st));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      const double us = 1000.0 * ms / reps;
      // same launches captured into a graph
      hipGraph_t g;
      hipGraphExec_t ge;
      CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
      for (int i = 0; i < reps; ++i) launch();
      CHECK(hipStreamEndCapture(st, &g));
      CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      CHECK(hipGraphLaunch(ge, st));
      CHECK(hipStreamSynchronize(st));
      CHECK(hipEventRecord(e0, st));
      CHECK(hipGraphLaunch(ge, st));
      CHECK(hipEventRecord(e1, st));
      CHECK(hipEventSynchronize(e1));
      float gms = 0;
      CHECK(hipEventElapsedTime(&gms, e0, e1));
      const double gus = 1000.0 * gms / reps;
      printf("%8zu %6d %10.2f %10.0f %10.2f %10.0f\n", m, ex, us, 2.0 * bytes / us / 1e3, gus,
             2.0 * bytes / gus / 1e3);
      CHECK(hipGraphExecDestroy(ge));
      CHECK(hipGraphDestroy(g));
    }
  }
  return 0;
}
