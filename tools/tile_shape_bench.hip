// Tile-shape study, round 3 (not part of the product).  hbm_ceiling2 showed a
// 16-B-per-lane in-place sweep reaching 6.59 TB/s with ONE amplitude per lane
// (4 KiB per workgroup) but only 5.4-5.7 TB/s with 4-16 per lane.  The pass
// kernels hold a 64 KiB tile per workgroup (16 amplitudes per lane, two
// workgroups per CU).  This sweeps, for an 8 GiB array in place with
// nontemporal 16-B loads/stores and 16 amplitudes per lane:
//   MAP 0  tile b = blockIdx (contiguous 64 KiB per workgroup, in order)
//   MAP 1  XCD bands: workgroup b works in band (b % 8) of 8 contiguous bands
//          (blocks are dealt round-robin over the 8 XCDs)
//   MAP 2  interleaved: load u of workgroup b at 4 KiB piece (u * nblocks + b)
//          (the instantaneous footprint of a one-amplitude-per-lane sweep)
//   MAP 3  XCD-interleaved pieces: piece u of workgroup b lands where the
//          eight XCDs' concurrent workgroups are contiguous
// with LDS forcing 1, 2 or 3 workgroups per CU, and 0 or 4 LDS re-layouts of
// the tile (the pass's structure).
// Build: hipcc --offload-arch=gfx950 -O3 tools/tile_shape_bench.hip -o tools/tile_shape_bench
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

template <int MAP>
__device__ __forceinline__ size_t piece(size_t b, size_t nb, int u) {
  // index of the 4 KiB piece (256 amplitudes) that load u of workgroup b covers
  if constexpr (MAP == 0) return b * 16 + u;
  if constexpr (MAP == 1) {
    const size_t band = nb / 8;
    return ((b % 8) * band + b / 8) * 16 + u;
  }
  if constexpr (MAP == 2) return (size_t)u * nb + b;
  // MAP 3: the 8 consecutive blocks (one per XCD) take 8 consecutive pieces
  if constexpr (MAP == 3) return ((b / 8) * 16 + u) * 8 + (b % 8);
  // MAP 4: as 3, residues permuted among the eight
  if constexpr (MAP == 4) return ((b / 8) * 16 + u) * 8 + ((b % 8) * 3 % 8);
  // MAP 5: adjacent like 3, but each workgroup's residue rotates per load
  if constexpr (MAP == 5) return ((b / 8) * 16 + u) * 8 + ((b + u) % 8);
  // MAP 6: residue b % 8 like 3, the eight far apart (1/16 of the array)
  return ((size_t)u * (nb / 8) + b / 8) * 8 + (b % 8);
}

template <int MAP, int LDSKB, int EXCH, int WPC>
__global__ __launch_bounds__(256, WPC) void k_tile(d2v* __restrict__ a, double f) {
  __shared__ d2v s[LDSKB > 0 ? LDSKB * 64 : 1];
  const int t = threadIdx.x;
  const size_t b = blockIdx.x, nb = gridDim.x;
  d2v v[16];
#pragma unroll
  for (int u = 0; u < 16; ++u) v[u] = __builtin_nontemporal_load(&a[piece<MAP>(b, nb, u) * 256 + t]);
#pragma unroll
  for (int e = 0; e < EXCH; ++e) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int y = (e & 1) ? ((t << 4) | u) : (t + 256 * u);
      s[(y ^ ((y >> 4) & 15)) & (LDSKB * 64 - 1)] = v[u];
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int y = (e & 1) ? (t + 256 * u) : ((t << 4) | u);
      v[u] = s[(y ^ ((y >> 4) & 15)) & (LDSKB * 64 - 1)];
    }
    __syncthreads();
  }
  if (LDSKB > 0 && EXCH == 0 && f == 12345.0) s[t] = v[0];  // keep the LDS allocation
#pragma unroll
  for (int u = 0; u < 16; ++u)
    __builtin_nontemporal_store(v[u] * (1.0 + f), &a[piece<MAP>(b, nb, u) * 256 + t]);
}

__global__ __launch_bounds__(256) void k_u1(d2v* __restrict__ a, double f) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  __builtin_nontemporal_store(__builtin_nontemporal_load(&a[i]) * (1.0 + f), &a[i]);
}

template <typename F>
float time_it(F fn, int reps) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  fn();
  fn();
  (void)hipEventRecord(e0);
  for (int i = 0; i < reps; ++i) fn();
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms / reps;
}

static d2v* g_a;
static size_t g_n;

template <int MAP, int LDSKB, int EXCH, int WPC>
void run(const char* what) {
  const size_t nb = g_n / 4096;
  const float ms = time_it([&] {
    hipLaunchKernelGGL((k_tile<MAP, LDSKB, EXCH, WPC>), dim3((unsigned)nb), dim3(256), 0, 0, g_a, 0.0);
  }, 8);
  printf("MAP=%d lds=%3d KiB exch=%d  %-28s %8.3f ms %7.0f GB/s\n", MAP, LDSKB, EXCH, what, ms,
         2.0 * g_n * 16 / ms / 1e6);
  fflush(stdout);
}

int main() {
  g_n = (size_t)1 << 29;  // 8 GiB
  CHECK(hipMalloc(&g_a, g_n * 16));
  CHECK(hipMemset(g_a, 0, g_n * 16));
  const float u1 = time_it([&] { hipLaunchKernelGGL(k_u1, dim3((unsigned)(g_n / 256)), dim3(256), 0, 0, g_a, 0.0); }, 8);
  printf("one amplitude per lane (reference)                        %8.3f ms %7.0f GB/s\n", u1,
         2.0 * g_n * 16 / u1 / 1e6);
  run<0, 64, 0, 2>("2 WG/CU");
  run<1, 64, 0, 2>("2 WG/CU");
  run<2, 64, 0, 2>("2 WG/CU");
  run<3, 64, 0, 2>("2 WG/CU");
  run<4, 64, 0, 2>("2 WG/CU");
  run<5, 64, 0, 2>("2 WG/CU");
  run<6, 64, 0, 2>("2 WG/CU");
  run<0, 64, 4, 2>("2 WG/CU");
  run<1, 64, 4, 2>("2 WG/CU");
  run<2, 64, 4, 2>("2 WG/CU");
  run<3, 64, 4, 2>("2 WG/CU");
  run<0, 128, 0, 1>("1 WG/CU");
  run<2, 128, 0, 1>("1 WG/CU");
  run<0, 48, 0, 3>("3 WG/CU");
  run<2, 48, 0, 3>("3 WG/CU");
  run<0, 32, 0, 4>("4 WG/CU");
  run<2, 32, 0, 4>("4 WG/CU");
  run<0, 0, 0, 2>("no LDS (VGPR-limited)");
  run<2, 0, 0, 2>("no LDS (VGPR-limited)");
  return 0;
}
