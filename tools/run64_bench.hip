// Read-only access patterns of the light-cone passes (development tool),
// with nontemporal and with ordinary loads.
// 1024 L=20 states in the octet layout (16 GiB); each 256-thread workgroup
// reads one 4096-amplitude tile of one state, 16 amplitudes per lane, with
// nontemporal 16-B loads, and reduces them (one double per workgroup, so
// nothing is dead code).  The tile's index bits:
//   R64   dtc_lcw2_final's load layout at j = 10: lanes = bits 0, 1, 5, 6, 7, 14
//         (64-B runs), waves = 12, 13, registers = 8..11, tile id = 2, 3, 4, 15..19
//   R128  lanes 0, 1, 2, 6, 7, 14 (128-B runs), id 3, 4, 5, 15..19
//   R256  lanes 0..3, 6, 7 (256-B runs), id 4, 5, 14..19
//   RC    lanes 0..5, waves 6, 7 (contiguous tiles), id 12..19
//   R16   lanes 4..9, waves 10, 11, registers 12..15, id 0..3, 16..19: no run at
//         all (16-B pieces; each 128-B line is read by 8 tiles, consecutive blocks)
// Prints time and GB/s per pattern; run under rocprofv3 --pmc FETCH_SIZE to
// compare the counter with the bytes read (16 GiB per launch).
// build: hipcc --offload-arch=gfx950 -O3 tools/run64_bench.hip -o tools/run64_bench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x)                                                             \
  do {                                                                       \
    hipError_t e_ = (x);                                                     \
    if (e_ != hipSuccess) {                                                  \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
      return 1;                                                              \
    }                                                                        \
  } while (0)

typedef double d2v __attribute__((ext_vector_type(2)));
static constexpr int kL = 20, kOg = 6, kStates = 1024;
static constexpr int64_t kLen = (int64_t)1 << kL;

__device__ __forceinline__ int64_t spread(int64_t x) {
  return ((x >> kOg) << (kOg + 3)) | (x & ((1 << kOg) - 1));
}

template <int P>
struct Pat;
template <>
struct Pat<0> {
  static constexpr int lane[6] = {0, 1, 5, 6, 7, 14}, wave[2] = {12, 13}, reg[4] = {8, 9, 10, 11};
  static constexpr int id[8] = {2, 3, 4, 15, 16, 17, 18, 19};
};
template <>
struct Pat<1> {
  static constexpr int lane[6] = {0, 1, 2, 6, 7, 14}, wave[2] = {12, 13}, reg[4] = {8, 9, 10, 11};
  static constexpr int id[8] = {3, 4, 5, 15, 16, 17, 18, 19};
};
template <>
struct Pat<2> {
  static constexpr int lane[6] = {0, 1, 2, 3, 6, 7}, wave[2] = {12, 13}, reg[4] = {8, 9, 10, 11};
  static constexpr int id[8] = {4, 5, 14, 15, 16, 17, 18, 19};
};
template <>
struct Pat<4> {  // R16: a 12-site window without column bits (16-B pieces)
  static constexpr int lane[6] = {4, 5, 6, 7, 8, 9}, wave[2] = {10, 11}, reg[4] = {12, 13, 14, 15};
  static constexpr int id[8] = {0, 1, 2, 3, 16, 17, 18, 19};
};
template <>
struct Pat<3> {
  static constexpr int lane[6] = {0, 1, 2, 3, 4, 5}, wave[2] = {6, 7}, reg[4] = {8, 9, 10, 11};
  static constexpr int id[8] = {12, 13, 14, 15, 16, 17, 18, 19};
};

template <int P, bool NT>
__global__ __launch_bounds__(256) void k_read(const double2* __restrict__ src, double* out) {
  using T = Pat<P>;
  const int t = threadIdx.x;
  const int64_t b = ((int64_t)blockIdx.y << 3) | (blockIdx.x & 7);
  const int tile = blockIdx.x >> 3;
  int64_t x = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) x |= (int64_t)((tile >> i) & 1) << T::id[i];
#pragma unroll
  for (int i = 0; i < 6; ++i) x |= (int64_t)((t >> i) & 1) << T::lane[i];
#pragma unroll
  for (int i = 0; i < 2; ++i) x |= (int64_t)((t >> (6 + i)) & 1) << T::wave[i];
  const char* base = (const char*)(src + ((b >> 3) << 3) * kLen + ((b & 7) << kOg));
  const int64_t vofs = spread(x) << 4;
  double acc = 0.0;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    int64_t y = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) y |= (int64_t)((r >> i) & 1) << T::reg[i];
    const d2v* a = (const d2v*)(base + (spread(y) << 4) + vofs);
    const d2v w = NT ? __builtin_nontemporal_load(a) : *a;
    acc += w.x + w.y;
  }
  if (acc == 12345.678) out[blockIdx.x + blockIdx.y * gridDim.x] = acc;  // keeps the loads
}

int main() {
  const size_t bytes = (size_t)kStates * kLen * 16;
  double2* s = nullptr;
  double* out = nullptr;
  CHECK(hipMalloc(&s, bytes));
  CHECK(hipMalloc(&out, 1 << 22));
  CHECK(hipMemset(s, 0, bytes));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const dim3 grid(8 * 256, kStates / 8), block(256);
  const char* names[10] = {"R64  nt (lcw2 load: 64-B runs)", "R128 nt (128-B runs)",
                           "R256 nt (256-B runs)", "RC   nt (contiguous tiles)",
                           "R64  temporal", "R128 temporal", "R256 temporal", "RC   temporal",
                           "R16  nt (16-B pieces)", "R16  temporal"};
  for (int rep = 0; rep < 2; ++rep) {
    for (int p = 0; p < 10; ++p) {
      auto launch = [&]() {
        if (p == 0) hipLaunchKernelGGL((k_read<0, true>), grid, block, 0, 0, s, out);
        if (p == 1) hipLaunchKernelGGL((k_read<1, true>), grid, block, 0, 0, s, out);
        if (p == 2) hipLaunchKernelGGL((k_read<2, true>), grid, block, 0, 0, s, out);
        if (p == 3) hipLaunchKernelGGL((k_read<3, true>), grid, block, 0, 0, s, out);
        if (p == 4) hipLaunchKernelGGL((k_read<0, false>), grid, block, 0, 0, s, out);
        if (p == 5) hipLaunchKernelGGL((k_read<1, false>), grid, block, 0, 0, s, out);
        if (p == 6) hipLaunchKernelGGL((k_read<2, false>), grid, block, 0, 0, s, out);
        if (p == 7) hipLaunchKernelGGL((k_read<3, false>), grid, block, 0, 0, s, out);
        if (p == 8) hipLaunchKernelGGL((k_read<4, true>), grid, block, 0, 0, s, out);
        if (p == 9) hipLaunchKernelGGL((k_read<4, false>), grid, block, 0, 0, s, out);
      };
      launch();
      CHECK(hipDeviceSynchronize());
      CHECK(hipEventRecord(e0, 0));
      for (int i = 0; i < 5; ++i) launch();
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      ms /= 5;
      printf("%-34s %8.3f ms  %6.0f GB/s (16 GiB read)\n", names[p], ms, bytes / (ms * 1e-3) / 1e9);
    }
  }
  CHECK(hipFree(s));
  CHECK(hipFree(out));
  return 0;
}
