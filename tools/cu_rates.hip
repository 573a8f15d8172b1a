// Per-CU rate study (not part of the product): FP64 FMA issue rate and the
// cost of the pass kernel's LDS re-layout (16 x ds_write_b128, barrier, 16 x
// ds_read_b128 per lane over a 64 KiB tile), with 1 or 2 workgroups of 256
// threads per CU, no global memory in the loop.
// Build: hipcc --offload-arch=gfx950 -O3 tools/cu_rates.hip -o tools/cu_rates
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

// 16 independent complex amplitudes per lane, ITER butterfly layers of 8
// pairs x 4 FMAs (the factored kick) -> 32 FMAs per layer per lane.
template <int LDS_KB>
__global__ __launch_bounds__(256, 2) void fma_loop(double* out, double f, int iters) {
  __shared__ double pad[LDS_KB * 128];
  double2 v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = make_double2(threadIdx.x + r, r * 0.5);
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (r & (1 << q)) continue;
        double2& u = v[r];
        double2& w = v[r | (1 << q)];
        double2 nu, nw;
        nu.x = fma(-f, w.y, u.x); nu.y = fma(f, w.x, u.y);
        nw.x = fma(-f, u.y, w.x); nw.y = fma(f, u.x, w.y);
        u = nu;
        w = nw;
      }
    }
  }
  double acc = 0;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc += v[r].x + v[r].y;
  if (LDS_KB) pad[threadIdx.x] = acc;
  __syncthreads();
  if (LDS_KB) acc += pad[(threadIdx.x + 1) & 255];
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

__device__ __forceinline__ int slot(int y) { return y ^ ((y >> 4) & 15); }

template <bool LEAD_BARRIER>
__global__ __launch_bounds__(256, 2) void lds_loop(double2* out, int iters) {
  __shared__ double2 s[4096];
  const int t = threadIdx.x;
  double2 v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = make_double2(t, r);
  for (int it = 0; it < iters; ++it) {
    // layout 2 -> 0 -> 2 (two exchanges per iteration)
    if (LEAD_BARRIER) __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) s[slot(t | (r << 8))] = v[r];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = s[slot((t << 4) | r)];
    if (LEAD_BARRIER) __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) s[slot((t << 4) | r)] = v[r];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = s[slot(t | (r << 8))];
  }
  double2 acc = make_double2(0, 0);
#pragma unroll
  for (int r = 0; r < 16; ++r) acc = make_double2(acc.x + v[r].x, acc.y + v[r].y);
  out[blockIdx.x * 256 + t] = acc;
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const double clk_ghz = prop.clockRate / 1e6;
  printf("CUs %d, clockRate %.3f GHz\n", cus, clk_ghz);
  double* out;
  CHECK(hipMalloc(&out, (size_t)cus * 8 * 256 * 16));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  auto timed = [&](auto launch) -> double {
    launch();
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return (double)ms;
  };
  const int iters = 2000;
  for (int wg_per_cu : {1, 2}) {
    const int grid = cus * wg_per_cu;
    double ms = timed([&] {
      hipLaunchKernelGGL((fma_loop<64>), dim3(grid), dim3(256), 0, 0, out, 0.3, iters);
      return 0;
    });
    const double fmas = (double)grid * 256 * iters * 4 * 8 * 4;  // lanes x layers x pairs x 4
    const double per_cu_clk = fmas / cus / (ms * 1e-3 * clk_ghz * 1e9);
    printf("fma_loop  %d WG/CU: %.3f ms  %.1f FP64 FMA lanes/clk/CU (%.1f TFLOP/s)\n", wg_per_cu,
           ms, per_cu_clk, 2 * fmas / (ms * 1e-3) / 1e12);
  }
  for (int wg_per_cu : {1, 2}) {
    for (int lead : {1, 0}) {
      const int grid = cus * wg_per_cu;
      const int it2 = 500;
      double ms = timed([&] {
        if (lead) hipLaunchKernelGGL((lds_loop<true>), dim3(grid), dim3(256), 0, 0, (double2*)out, it2);
        else hipLaunchKernelGGL((lds_loop<false>), dim3(grid), dim3(256), 0, 0, (double2*)out, it2);
        return 0;
      });
      const double exch = (double)wg_per_cu * it2 * 2;  // exchanges per CU
      printf("lds_loop  %d WG/CU lead_barrier=%d: %.3f ms  %.0f clk per 64 KiB exchange per CU\n",
             wg_per_cu, lead, ms, ms * 1e-3 * clk_ghz * 1e9 / exch);
    }
  }
  return 0;
}
