// HBM ceiling study, round 3 (not part of the product): which simple
// streaming kernels reach the guide's 6.29 TB/s float4 copy
// (MI355X_MICROARCH.md, chip table) on this box, and what the read+write mix
// of the pass kernels can expect.  Sweeps, for 8 GiB arrays (far past the
// 256 MiB Infinity Cache):
//   copy   b[i] = a[i]          (out of place)    U x 16 B per lane
//   inpl   a[i] = c a[i]        (in place)
//   write  a[i] = const
//   read   sum a[i]
// with plain or nontemporal ("nt") loads / stores, U = 1, 2, 4, 8 amplitudes
// per lane spaced one workgroup-width apart (coalesced 1 KiB per wave
// instruction), 256 / 512 / 1024 threads per workgroup, one tile per
// workgroup or grid-stride over a fixed grid, plus hipMemcpyAsync D2D.
// Bytes counted: read + written (copy/inpl: 2 x array bytes).
// Build: hipcc --offload-arch=gfx950 -O3 tools/hbm_ceiling2.hip -o tools/hbm_ceiling2
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

#define CHECK(x)                                                         \
  do {                                                                   \
    hipError_t e = (x);                                                  \
    if (e != hipSuccess) {                                               \
      printf("%s: %s\n", #x, hipGetErrorString(e));                      \
      return 1;                                                          \
    }                                                                    \
  } while (0)

typedef double d2v __attribute__((ext_vector_type(2)));

template <bool NT>
__device__ __forceinline__ d2v ld(const d2v* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(d2v v, d2v* p) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// MODE 0 copy, 1 in place, 2 write, 3 read
template <int MODE, int U, int TPB, bool NTL, bool NTS>
__global__ __launch_bounds__(TPB) void k_tile(const d2v* __restrict__ a, d2v* __restrict__ b,
                                             double c, double* out) {
  const size_t base = (size_t)blockIdx.x * (TPB * U) + threadIdx.x;
  d2v v[U];
  if constexpr (MODE != 2) {
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld<NTL>(&a[base + TPB * u]);
  }
  if constexpr (MODE == 3) {
    d2v s = {0, 0};
#pragma unroll
    for (int u = 0; u < U; ++u) s += v[u];
    if (s.x == 12345.0) out[0] = s.y;
  } else {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      d2v w = MODE == 2 ? d2v{1.0, 2.0} : (MODE == 1 ? v[u] * c : v[u]);
      st<NTS>(w, (MODE == 0 ? b : (d2v*)a) + base + TPB * u);
    }
  }
}

// grid-stride: a fixed grid sweeps the array in U-amplitude tiles per lane
template <int MODE, int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k_stride(const d2v* __restrict__ a, d2v* __restrict__ b,
                                               double c, size_t n_tiles) {
  for (size_t t = blockIdx.x; t < n_tiles; t += gridDim.x) {
    const size_t base = t * (256 * U) + threadIdx.x;
    d2v v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld<NTL>(&a[base + 256 * u]);
#pragma unroll
    for (int u = 0; u < U; ++u)
      st<NTS>(MODE == 1 ? v[u] * c : v[u], (MODE == 0 ? b : (d2v*)a) + base + 256 * u);
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
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return ms / reps;
}

static d2v *g_a, *g_b;
static double* g_out;
static size_t g_n;

static void rep(const char* name, double bytes, float ms) {
  printf("%-44s %9.3f ms  %7.0f GB/s\n", name, ms, bytes / ms / 1e6);
  fflush(stdout);
}

template <int MODE, int U, int TPB, bool NTL, bool NTS>
void run_tile(const char* tag) {
  const size_t blocks = g_n / (TPB * U);
  const double bytes = (MODE <= 1 ? 2.0 : 1.0) * g_n * 16;
  char name[96];
  snprintf(name, sizeof name, "%s U=%d tpb=%d ld=%s st=%s", tag, U, TPB, NTL ? "nt" : "pl",
           NTS ? "nt" : "pl");
  rep(name, bytes, time_it([&] {
        hipLaunchKernelGGL((k_tile<MODE, U, TPB, NTL, NTS>), dim3((unsigned)blocks), dim3(TPB), 0, 0,
                           g_a, g_b, 1.0, g_out);
      }, 8));
}

template <int MODE, int U, bool NTL, bool NTS>
void run_stride(const char* tag, int grid) {
  const size_t tiles = g_n / (256 * U);
  char name[96];
  snprintf(name, sizeof name, "%s U=%d grid=%d ld=%s st=%s", tag, U, grid, NTL ? "nt" : "pl",
           NTS ? "nt" : "pl");
  rep(name, 2.0 * g_n * 16, time_it([&] {
        hipLaunchKernelGGL((k_stride<MODE, U, NTL, NTS>), dim3(grid), dim3(256), 0, 0, g_a, g_b,
                           1.0, tiles);
      }, 8));
}

template <int MODE, int U>
void run_hints(const char* tag) {
  run_tile<MODE, U, 256, false, false>(tag);
  run_tile<MODE, U, 256, true, false>(tag);
  run_tile<MODE, U, 256, false, true>(tag);
  run_tile<MODE, U, 256, true, true>(tag);
}

int main() {
  g_n = (size_t)1 << 29;  // 8 GiB per array
  CHECK(hipMalloc(&g_a, g_n * 16));
  CHECK(hipMalloc(&g_b, g_n * 16));
  CHECK(hipMalloc(&g_out, 64));
  CHECK(hipMemset(g_a, 0, g_n * 16));
  CHECK(hipMemset(g_b, 0, g_n * 16));
  printf("# arrays 2 x %.1f GiB\n", g_n * 16.0 / (1 << 30));
  rep("hipMemcpyAsync D2D", 2.0 * g_n * 16, time_it([&] {
        (void)hipMemcpyAsync(g_b, g_a, g_n * 16, hipMemcpyDeviceToDevice, 0);
      }, 8));
  run_hints<0, 1>("copy");
  run_hints<0, 2>("copy");
  run_hints<0, 4>("copy");
  run_hints<0, 8>("copy");
  run_hints<1, 1>("inpl");
  run_hints<1, 2>("inpl");
  run_hints<1, 4>("inpl");
  run_hints<1, 8>("inpl");
  run_hints<2, 1>("write");
  run_hints<2, 4>("write");
  run_tile<3, 4, 256, false, false>("read");
  run_tile<3, 4, 256, true, false>("read");
  run_tile<0, 4, 512, false, false>("copy");
  run_tile<0, 4, 1024, false, false>("copy");
  run_tile<0, 4, 512, true, true>("copy");
  run_tile<0, 2, 1024, false, false>("copy");
  run_tile<1, 4, 512, false, false>("inpl");
  run_tile<1, 4, 1024, false, false>("inpl");
  for (int grid : {512, 1024, 2048, 4096}) {
    run_stride<0, 4, false, false>("copy stride", grid);
    run_stride<1, 4, false, false>("inpl stride", grid);
    run_stride<1, 4, true, true>("inpl stride", grid);
  }
  return 0;
}
