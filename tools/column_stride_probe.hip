// Timing probe, round 5 (not part of the product): why C4's K-D-K on the top
// 8-site group (tile = index bits 0..3 + sites 20..27, rows 16 MiB apart)
// runs 57 ms against 47 ms for the group below it (sites 12..19, rows 64 KiB
// apart) on the same work (r5k_c4 kernel trace).  A bare in-place tile
// pass over NS states of 2^28 amplitudes: 256 threads load 16 x 16 B each
// (a 4096-amplitude tile = 256 rows of 256 B at bit position S), write them
// back; 52 KiB of LDS held so three workgroups share a CU as in the product.
// Tile ids run over the non-tile bits in ascending order, state index last.
// Allocation: hipMalloc, or hipExtMallocWithFlags(hipDeviceMallocContiguous).
// Build: hipcc --offload-arch=gfx950 -O3 tools/column_stride_probe.hip -o gpu_bin/column_stride_probe
#include <hip/hip_runtime.h>

#include <cstdio>

#define CHECK(x)                                                    \
  do {                                                              \
    hipError_t e = (x);                                             \
    if (e != hipSuccess) {                                          \
      printf("%s: %s\n", #x, hipGetErrorString(e));                 \
      return 1;                                                     \
    }                                                               \
  } while (0)

typedef double d2v __attribute__((ext_vector_type(2)));
constexpr int kL = 28;

// tile id -> base amplitude: bits [4, S) then [S + 8, kL) then the state
__device__ __forceinline__ int64_t tile_base(int64_t id, int S) {
  const int64_t lo_n = S - 4;
  const int64_t lo = id & ((1ll << lo_n) - 1);
  const int64_t hi = id >> lo_n;  // bits above the rows, and the state
  return (lo << 4) | (hi << (S + 8));
}

template <bool NT, int WORK>
__global__ __launch_bounds__(256) void tile_pass(d2v* st, int S, int order) {
  __shared__ d2v pad[52 * 64];
  const int t = threadIdx.x;
  int64_t id = blockIdx.x;
  if (order == 1) {
    // XCD-aware: consecutive ids on one XCD (blocks go round-robin over 8)
    const int64_t n = gridDim.x;
    id = (blockIdx.x & 7) * (n >> 3) + (blockIdx.x >> 3);
  }
  const int64_t base = tile_base(id, S);
  const int col = t & 15;
  d2v v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t row = (t >> 4) + 16 * r;
    d2v* p = st + base + col + (row << S);
    v[r] = NT ? __builtin_nontemporal_load(p) : *p;
  }
  // WORK > 0: the K-D-K's in-register work between the loads and the stores,
  // emulated by WORK rounds of (LDS re-layout of the tile's 2 x 32 KiB halves +
  // 64 dependent-chain FMAs per amplitude register pair)
  for (int w = 0; w < WORK; ++w) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      __syncthreads();
#pragma unroll
      for (int r = 8 * h; r < 8 * h + 8; ++r) pad[((t + 256 * (r & 7)) ^ ((t >> 4) & 15))] = v[r];
      __syncthreads();
#pragma unroll
      for (int r = 8 * h; r < 8 * h + 8; ++r) v[r] = pad[(((t << 3) | (r & 7)) ^ (t & 15)) & 2047];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        const d2v a = v[r], c = v[r + 1];
        v[r].x = fma(0.7, a.x, -0.7 * c.y);
        v[r].y = fma(0.7, a.y, 0.7 * c.x);
        v[r + 1].x = fma(0.7, c.x, -0.7 * a.y);
        v[r + 1].y = fma(0.7, c.y, 0.7 * a.x);
      }
  }
  if (WORK == 0 && S < 0) pad[t] = v[0];  // never: keeps the LDS allocation
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t row = (t >> 4) + 16 * r;
    d2v* p = st + base + col + (row << S);
    v[r].x += 1.0;
    if (NT) __builtin_nontemporal_store(v[r], p);
    else *p = v[r];
  }
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
  const int NS = 8;  // 8 states of 2^28 amplitudes = 32 GiB
  const size_t n = (size_t)NS << kL;
  const int64_t tiles = (int64_t)n >> 12;
  for (int alloc = 0; alloc < 1; ++alloc) {
    d2v* st = nullptr;
    hipError_t e = alloc == 0 ? hipMalloc(&st, n * 16)
                              : hipExtMallocWithFlags((void**)&st, n * 16, hipDeviceMallocContiguous);
    if (e != hipSuccess) {
      printf("alloc %d: %s\n", alloc, hipGetErrorString(e));
      (void)hipGetLastError();
      continue;
    }
    CHECK(hipMemset(st, 0, n * 16));
    const double bytes = 2.0 * n * 16;
    for (int work = 0; work < 3; ++work) {
      for (int S : {4, 12, 20}) {
        for (int order = 0; order < 2; ++order) {
          const float ms = time_it([&] {
            if (work == 0) hipLaunchKernelGGL((tile_pass<true, 0>), dim3(tiles), dim3(256), 0, 0, st, S, order);
            else if (work == 1) hipLaunchKernelGGL((tile_pass<true, 2>), dim3(tiles), dim3(256), 0, 0, st, S, order);
            else hipLaunchKernelGGL((tile_pass<true, 4>), dim3(tiles), dim3(256), 0, 0, st, S, order);
          }, 5);
          printf("%s work=%d S=%2d (rows %8lld B apart) order=%d  %8.3f ms  %6.0f GB/s\n",
                 alloc ? "contig " : "hipMalloc", work == 0 ? 0 : 2 * work, S, 16ll << S, order, ms,
                 bytes / ms / 1e6);
        }
      }
    }
    CHECK(hipDeviceSynchronize());
    CHECK(hipFree(st));
  }
  return 0;
}
