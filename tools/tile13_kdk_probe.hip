// Timing probe, round 5 (not part of the product): the
// 13-bit-tile split of an L=20 period -- a 13-site group A (tile = index bits
// 0..12) and a 7-site group B in 1 KiB columns (index bits 0..5 + sites
// 13..19) -- against the product's 12 / 8 split (bits 0..11; 256-B columns
// 0..3 + sites 12..19), as synthetic K-D-K passes with the product's
// structure: 16 nontemporal 16-B loads per lane in place, the group's kicks
// (2 per site, readlane'd coefficients, register butterflies in 4-site
// rounds) with LDS re-layouts between rounds (half-tile buffer, real then
// imaginary parts, or the full tile), one diagonal lookup per amplitude, 16
// nontemporal stores.  Octet state layout at 1 KiB (the product's), the eight
// states of an octet on consecutive blocks.  Results are wrong by design.
//   A12: 4096 amplitudes, 256 threads, 24 kicks, 4 re-layouts, 3 WG/CU
//        (product dtc_kdk_pass3<7>: 5.41 ms at B = 1024)
//   B12: 4096 amplitudes, 256 threads, 16 kicks, 2 re-layouts, full 64 KiB
//        tile, 2 WG/CU (product dtc_kdk_pass<6>: 5.83 ms)
//   A13: 8192 amplitudes, 512 threads, 26 kicks, 4 re-layouts + 2 row swaps
//   B13: 8192 amplitudes, 512 threads, 14 kicks, 2 re-layouts
// each 13-bit form at one workgroup per CU (full 128 KiB tile) and at two
// (64 KiB half-tile buffer).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I<pkg>/csrc tools/tile13_kdk_probe.hip -o gpu_bin/tile13_kdk_probe
#include <hip/hip_runtime.h>

#include <cstdio>

#include "dtc_device.h"

using namespace dtc;

#define CHECK(x)                                                    \
  do {                                                              \
    hipError_t e = (x);                                             \
    if (e != hipSuccess) {                                          \
      printf("%s: %s\n", #x, hipGetErrorString(e));                 \
      return 1;                                                     \
    }                                                               \
  } while (0)

// layout P: registers = tile bits [P, P + 4), threads = the other bits in order
template <int P>
__device__ __forceinline__ int ybase_p(int t) {
  return (t & ((1 << P) - 1)) | ((t >> P) << (P + 4));
}
__host__ __device__ constexpr int swz(int y) { return y ^ ((y >> 5) & 31) ^ ((y >> 10) & 7); }

// TB-bit tile, C column bits (C = TB: contiguous), the rest = sites from bit S
template <int TB, int C, bool HALF, int IOP>
struct Tile {
  static constexpr int NT = 1 << (TB - 4);
  static constexpr int S = C == TB ? TB : 20 - (TB - C);  // first site bit of the columns form
  static constexpr int IDB = 20 - TB;                      // tile-id bits
};

template <int TB, int C, bool HALF, int IOP, int PROG>
__device__ __forceinline__ void kdk_probe(double2* __restrict__ st, int og, int batch,
                                          const double* __restrict__ coefs,
                                          const double2* __restrict__ tabs, double* s_x,
                                          double2* s_full, double2* s_tab) {
  using T = Tile<TB, C, HALF, IOP>;
  const int t = threadIdx.x;
  const int64_t b = ((int64_t)blockIdx.y << 3) | (blockIdx.x & 7);
  const int64_t tile = blockIdx.x >> 3;
  if (b >= batch) return;
  RecRegs R;
  {
    const int lane = t & 63;
    R.rv[0] = coefs[(b * 64 + lane) * 4 % 4096];
    R.rv[1] = coefs[(b * 64 + lane) * 4 % 4096 + 1];
    R.rv[2] = coefs[(b * 64 + lane) * 4 % 4096 + 2];
    R.rv[3] = coefs[(b * 64 + lane) * 4 % 4096 + 3];
  }
  const double2 tv = tabs[t & 255];
  char* base = (char*)(st + state_base(b, (int64_t)1 << 20, og));
  // tile-local y -> state index x
  auto xof = [&](int y) -> int64_t {
    if constexpr (C == TB) return (tile << TB) | y;
    return (int64_t)(y & ((1 << C) - 1)) | (tile << C) | ((int64_t)(y >> C) << T::S);
  };
  const int yb = ybase_p<IOP>(t);
  auto addr = [&](int r) { return base + (octet_spread(xof(yb | (r << IOP)), og) << 4); };
  double2 v[kRegs];
#pragma unroll
  for (int r = 0; r < kRegs; ++r) {
    const d2v w = __builtin_nontemporal_load((const d2v*)addr(r));
    v[r] = make_double2(w.x, w.y);
  }
  if (t < 256) s_tab[t] = tv;
  auto kick = [&](auto q_tag) {
    constexpr int Q = decltype(q_tag)::value;
    layer_f<kKindRX, 0, Q & 3>(v, R.d(0, (Q * 3) & 127));
  };
  auto kicks = [&](auto n_tag) {
    constexpr int N = decltype(n_tag)::value;
    if constexpr (N >= 1) kick(std::integral_constant<int, 0>{});
    if constexpr (N >= 2) kick(std::integral_constant<int, 1>{});
    if constexpr (N >= 3) kick(std::integral_constant<int, 2>{});
    if constexpr (N >= 4) kick(std::integral_constant<int, 3>{});
  };
  auto xch = [&](auto f_tag, auto t_tag) {
    constexpr int F = decltype(f_tag)::value, TO = decltype(t_tag)::value;
    int bf = ybase_p<F>(t), bt = ybase_p<TO>(t);
    asm volatile("" : "+v"(bf), "+v"(bt));
    if constexpr (HALF) {
      __syncthreads();
#pragma unroll
      for (int r = 0; r < kRegs; ++r) s_x[swz(bf | (r << F))] = v[r].x;
      __syncthreads();
#pragma unroll
      for (int r = 0; r < kRegs; ++r) v[r].x = s_x[swz(bt | (r << TO))];
      __syncthreads();
#pragma unroll
      for (int r = 0; r < kRegs; ++r) s_x[swz(bf | (r << F))] = v[r].y;
      __syncthreads();
#pragma unroll
      for (int r = 0; r < kRegs; ++r) v[r].y = s_x[swz(bt | (r << TO))];
    } else {
      __syncthreads();
#pragma unroll
      for (int r = 0; r < kRegs; ++r) s_full[swz(bf | (r << F))] = v[r];
      __syncthreads();
#pragma unroll
      for (int r = 0; r < kRegs; ++r) v[r] = s_full[swz(bt | (r << TO))];
    }
  };
  auto diag = [&]() {
    int ba = t & 255;
    asm volatile("" : "+v"(ba));
#pragma unroll
    for (int r = 0; r < kRegs; ++r) v[r] = cmul(v[r], s_tab[(ba ^ (r * 7)) & 255]);
  };
  auto swap16 = [&]() {
#pragma unroll
    for (int r = 0; r < kRegs; r += 2) {
      swap_rows<16>(v[r].x, v[r + 1].x);
      swap_rows<16>(v[r].y, v[r + 1].y);
    }
  };
  using K1 = std::integral_constant<int, 1>;
  using K3 = std::integral_constant<int, 3>;
  using K4 = std::integral_constant<int, 4>;
#define P_(x) std::integral_constant<int, x>{}
  if constexpr (PROG == 0) {  // A12: IO 4 -> 0 -> 8 | D | 8 -> 0 -> 4
    kicks(K4{}); xch(P_(4), P_(0)); kicks(K4{}); xch(P_(0), P_(8)); kicks(K4{});
    diag();
    kicks(K4{}); xch(P_(8), P_(0)); kicks(K4{}); xch(P_(0), P_(4)); kicks(K4{});
  } else if constexpr (PROG == 1) {  // B12: IO 8 -> 4 | D | 4 -> 8
    kicks(K4{}); xch(P_(8), P_(4)); kicks(K4{});
    diag();
    kicks(K4{}); xch(P_(4), P_(8)); kicks(K4{});
  } else if constexpr (PROG == 2) {  // A13: IO 4 -> 0 -> 8 (+ site 12 by a row swap) | D | back
    kicks(K4{}); xch(P_(4), P_(0)); kicks(K4{}); xch(P_(0), P_(8)); kicks(K4{});
    swap16(); kicks(K1{});
    diag();
    kicks(K1{}); swap16();
    kicks(K4{}); xch(P_(8), P_(0)); kicks(K4{}); xch(P_(0), P_(4)); kicks(K4{});
  } else if constexpr (PROG == 3) {  // B13: IO 9 (sites 16..19) -> 5 (col 5, sites 13..15) | D | back
    kicks(K4{}); xch(P_(9), P_(5)); kicks(K3{});
    diag();
    kicks(K3{}); xch(P_(5), P_(9)); kicks(K4{});
  } else if constexpr (PROG == 4) {  // B13c5 (round 6): 8 sites 12..19 over 512-B columns: IO 9 (sites 16..19) -> 5 (12..15) | D | back
    kicks(K4{}); xch(P_(9), P_(5)); kicks(K4{});
    diag();
    kicks(K4{}); xch(P_(5), P_(9)); kicks(K4{});
  } else {  // B12c5 (round 6): 12-bit tile, 7 sites 13..19 over 512-B columns: IO 8 (16..19) -> 4 (col 4, 13..15) | D | back
    kicks(K4{}); xch(P_(8), P_(4)); kicks(K3{});
    diag();
    kicks(K3{}); xch(P_(4), P_(8)); kicks(K4{});
  }
#undef P_
#pragma unroll
  for (int r = 0; r < kRegs; ++r) {
    d2v w = {v[r].x, v[r].y};
    __builtin_nontemporal_store(w, (d2v*)addr(r));
  }
}

template <int TB, int C, bool HALF, int IOP, int PROG, int WPC>
__global__ __launch_bounds__(1 << (TB - 4)) __attribute__((amdgpu_waves_per_eu(
    WPC * (1 << (TB - 4)) / 256, WPC * (1 << (TB - 4)) / 256))) void k_probe(double2* __restrict__ st, int og,
                                                              int batch,
                                                              const double* __restrict__ coefs,
                                                              const double2* __restrict__ tabs) {
  __shared__ double s_x[HALF ? (1 << TB) : 1];
  __shared__ double2 s_full[HALF ? 1 : (1 << TB)];
  __shared__ double2 s_tab[256];
  kdk_probe<TB, C, HALF, IOP, PROG>(st, og, batch, coefs, tabs, s_x, s_full, s_tab);
}

// round 6: state filled with normalised pseudo-random amplitudes (argv[3] =
// "rand"): do the passes' times depend on the data (zeros vs dense values)?
__global__ void fill_rand(double2* st, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t h = i * 0x9E3779B97F4A7C15ull;
  h ^= h >> 31;
  h *= 0xBF58476D1CE4E5B9ull;
  h ^= h >> 29;
  const double a = (double)(h & 0xFFFFF) / 1048576.0 - 0.5, c = (double)((h >> 20) & 0xFFFFF) / 1048576.0 - 0.5;
  st[i] = make_double2(a * 1e-3, c * 1e-3);
}

// round 6: what precedes a pass -- an idle gap (one sleeping wave) or a
// VALU-heavy burner on every CU (FP64 FMA chains, no memory) of ~us microseconds
__global__ void k_sleep(int us) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
  while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)us * 100) __builtin_amdgcn_s_sleep(10);
}
__global__ void k_burn(int us, double* sink) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  double a = threadIdx.x * 1e-3, b = 0.999, c = 1e-3;
  while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)us * 100) {
#pragma unroll
    for (int i = 0; i < 64; ++i) a = fma(a, b, c);
  }
  if (a == 12345.0) sink[0] = a;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 1024, og = 6;
  const size_t n = (size_t)B << 20;
  double2* st;
  double* coefs;
  double2* tabs;
  CHECK(hipMalloc(&st, n * 16));
  CHECK(hipMemset(st, 0, n * 16));
  if (argc > 3) {
    hipLaunchKernelGGL(fill_rand, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, st, n);
    CHECK(hipDeviceSynchronize());
  }
  CHECK(hipMalloc(&coefs, 4096 * 8));
  CHECK(hipMemset(coefs, 0, 4096 * 8));
  CHECK(hipMalloc(&tabs, 256 * 16));
  CHECK(hipMemset(tabs, 0, 256 * 16));
  if (argc > 3) {
    double2 ht[256];
    double hc[4096];
    for (int i = 0; i < 256; ++i) ht[i] = make_double2(0.6, 0.8);
    for (int i = 0; i < 4096; ++i) hc[i] = 0.05;
    CHECK(hipMemcpy(tabs, ht, sizeof(ht), hipMemcpyHostToDevice));
    CHECK(hipMemcpy(coefs, hc, sizeof(hc), hipMemcpyHostToDevice));
  }
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const unsigned oct = (unsigned)((B + 7) / 8);
  auto run = [&](const char* name, auto launch) -> int {
    launch();
    launch();
    CHECK(hipDeviceSynchronize());
    const int reps = 10;
    CHECK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) launch();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    printf("%-58s %8.3f ms  %7.0f GB/s\n", name, ms, n * 32.0 / (ms * 1e6));
    return 0;
  };
  // round 6: two passes alternating (the product's chains alternate the row
  // and the column group): each one's own time when it follows the other
  hipEvent_t ev[41];
  for (auto& evx : ev) CHECK(hipEventCreate(&evx));
  auto pair = [&](const char* na, auto la, const char* nb, auto lb) -> int {
    la();
    lb();
    CHECK(hipDeviceSynchronize());
    for (int i = 0; i < 20; ++i) {
      CHECK(hipEventRecord(ev[2 * i]));
      la();
      CHECK(hipEventRecord(ev[2 * i + 1]));
      lb();
    }
    CHECK(hipEventRecord(ev[40]));
    CHECK(hipEventSynchronize(ev[40]));
    float ta = 0, tb = 0;
    for (int i = 0; i < 20; ++i) {
      float x = 0, y = 0;
      CHECK(hipEventElapsedTime(&x, ev[2 * i], ev[2 * i + 1]));
      CHECK(hipEventElapsedTime(&y, ev[2 * i + 1], ev[2 * i + 2]));
      ta += x / 20;
      tb += y / 20;
    }
    printf("alternating: %-34s %8.3f ms | %-34s %8.3f ms\n", na, ta, nb, tb);
    return 0;
  };
#define LNCH(TB, C, HALF, IOP, PROG, WPC)                                                            \
  [&] {                                                                                            \
    hipLaunchKernelGGL((k_probe<TB, C, HALF, IOP, PROG, WPC>), dim3(8u << (20 - TB), oct),         \
                       dim3(1 << (TB - 4)), 0, 0, st, og, B, coefs, tabs);                         \
  }
  if (argc > 2 && argv[2][0] == 'p') {
    // A13 after an idle gap / after a burner / back to back (argv[2] = "pre")
    double* sink;
    CHECK(hipMalloc(&sink, 8));
    auto a13 = LNCH(13, 13, true, 4, 2, 2);
    auto a12 = LNCH(12, 12, true, 4, 0, 3);
    for (int us : {0, 500, 2000}) {
      auto sl = [&] { hipLaunchKernelGGL(k_sleep, dim3(1), dim3(64), 0, 0, us); };
      auto bu = [&] { hipLaunchKernelGGL(k_burn, dim3(2048), dim3(256), 0, 0, us, sink); };
      char na[64], nb[64];
      snprintf(na, sizeof na, "sleep %d us", us);
      snprintf(nb, sizeof nb, "burn %d us", us);
      if (pair(na, sl, "A13 half, 2 WG/CU", a13)) return 1;
      if (pair(nb, bu, "A13 half, 2 WG/CU", a13)) return 1;
      if (pair(na, sl, "A12 (kdk3<7>)", a12)) return 1;
      if (pair(nb, bu, "A12 (kdk3<7>)", a12)) return 1;
    }
    return 0;
  }
  if (argc > 2) {
    for (int rep = 0; rep < 2; ++rep) {
      if (pair("A12 (kdk3<7>)", LNCH(12, 12, true, 4, 0, 3), "B12 (kdk<6>)", LNCH(12, 4, false, 8, 1, 2)))
        return 1;
      if (pair("A13 half, 2 WG/CU", LNCH(13, 13, true, 4, 2, 2), "B12c5 full, 2 WG/CU",
               LNCH(12, 5, false, 8, 5, 2)))
        return 1;
      if (pair("A13 half, 2 WG/CU", LNCH(13, 13, true, 4, 2, 2), "A13 half, 2 WG/CU",
               LNCH(13, 13, true, 4, 2, 2)))
        return 1;
      if (pair("B12c5 full, 2 WG/CU", LNCH(12, 5, false, 8, 5, 2), "B12c5 full, 2 WG/CU",
               LNCH(12, 5, false, 8, 5, 2)))
        return 1;
    }
    return 0;
  }
#define RUN(NAME, TB, C, HALF, IOP, PROG, WPC)                                                   \
  if (run(NAME, [&] {                                                                            \
        hipLaunchKernelGGL((k_probe<TB, C, HALF, IOP, PROG, WPC>), dim3(8u << (20 - TB), oct),   \
                           dim3(1 << (TB - 4)), 0, 0, st, og, B, coefs, tabs);                   \
      }))                                                                                        \
    return 1;
  for (int rep = 0; rep < 2; ++rep) {
    RUN("A12 c=12, half-tile LDS, 3 WG/CU (product: kdk3<7>)", 12, 12, true, 4, 0, 3);
    RUN("B12 c=4 s=12, full-tile LDS, 2 WG/CU (product: kdk<6>)", 12, 4, false, 8, 1, 2);
    RUN("A13 c=13, full-tile LDS, 1 WG/CU", 13, 13, false, 4, 2, 1);
    RUN("A13 c=13, half-tile LDS, 2 WG/CU", 13, 13, true, 4, 2, 2);
    RUN("B13 c=6 s=13, full-tile LDS, 1 WG/CU", 13, 6, false, 9, 3, 1);
    RUN("B13 c=6 s=13, half-tile LDS, 2 WG/CU", 13, 6, true, 9, 3, 2);
    // round 6: the 12/8 split kept, only the 8-site column pass on a 13-bit
    // tile (5 column bits: 512-B runs, half an octet run)
    RUN("B13c5 c=5 s=12 (8 sites), half-tile LDS, 2 WG/CU", 13, 5, true, 9, 4, 2);
    RUN("B13c5 c=5 s=12 (8 sites), full-tile LDS, 1 WG/CU", 13, 5, false, 9, 4, 1);
    RUN("B12 c=4 s=12, half-tile LDS, 3 WG/CU", 12, 4, true, 8, 1, 3);
    // round 6: the 13/7 split's column pass on a 12-bit tile (7 sites + 5
    // column bits: 512-B runs): is the gain the site count or the 1 KiB runs?
    RUN("B12c5 c=5 s=13 (7 sites), full-tile LDS, 2 WG/CU", 12, 5, false, 8, 5, 2);
    RUN("B12c5 c=5 s=13 (7 sites), half-tile LDS, 3 WG/CU", 12, 5, true, 8, 5, 3);
  }
  return 0;
}
