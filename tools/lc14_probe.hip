// Timing probe, round 5 (not part of the product): would a
// 14-site light-cone end (the echo chain's last SEVEN passes merged: eight kick
// layers of radius 7 .. 0, 58 site kicks, seven cone diagonals, a 16384-
// amplitude tile per workgroup = 1024 threads x 16 registers, re-layouts
// through a 128 KiB half-tile LDS buffer, one workgroup per CU) cost less than
// what it replaces -- dtc_lcw3_final (7.8 ms at B = 1024) plus one K-D-K pass
// (5.9 ms)?  Results are wrong by design: the probe runs the instruction mix
// (butterflies on register bits with readlane'd coefficients, permlane row
// swaps, cone-table lookups from LDS, half-tile re-layouts, the probe sum)
// and the memory pattern (16-B pieces of L=20 octet-layout states, tile bits =
// global bits W0 .. W0+TB-1, ordinary loads) of the two kernels:
//   E = 0: the 12-bit program of dtc_lcw3_final (41 kicks, 6 row swaps, 4
//          two-table + 2 one-table diagonals, 3 re-layouts), 4 workgroups / CU
//          -- the calibration against the product kernel's measured time
//   E = 2: a 14-bit program (58 kicks, 8 row swaps, 5 + 2 diagonals, 4
//          re-layouts), 1 workgroup / CU
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I<pkg>/csrc tools/lc14_probe.hip -o gpu_bin/lc14_probe
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

// layout n: registers = tile bits [P(n), P(n) + 4), threads = the other bits
// in order (lane bits first)
template <int TB, int N>
__device__ __forceinline__ constexpr int reg_pos() {
  return TB == 12 ? (N % 3) * 4 : (N % 4 == 3 ? 10 : (N % 4) * 4);
}
template <int TB, int N>
__device__ __forceinline__ int ybase_n(int t) {
  constexpr int P = reg_pos<TB, N>();
  return (t & ((1 << P) - 1)) | ((t >> P) << (P + 4));
}
// XOR swizzle: lane bits spread over the banks in every layout
__host__ __device__ constexpr int swz(int y) { return y ^ ((y >> 5) & 31) ^ ((y >> 10) & 15); }

template <int TB>
__device__ __forceinline__ void lc_body(const double2* __restrict__ st, int L, int w0, int og,
                                        int batch, const double* __restrict__ coefs,
                                        const double2* __restrict__ tabs, double* __restrict__ out,
                                        double* s_x, double2* s_tab, unsigned bx, unsigned by) {
  constexpr int NT = 1 << (TB - 4);
  const int t = threadIdx.x;
  const int tile_bits = L - TB;
  const int64_t b = ((int64_t)by << 3) | (bx & 7);
  const int64_t tile = bx >> 3;
  if (b >= batch) return;
  // tile id: global bits 0 .. w0-1 and w0+TB .. L-1
  const int64_t tbase = (tile & ((1 << w0) - 1)) | ((tile >> w0) << (w0 + TB));
  (void)tile_bits;
  RecRegs R;
  {
    const int lane = t & 63;
    R.rv[0] = coefs[(b * 64 + lane) * 4 % 4096];
    R.rv[1] = coefs[(b * 64 + lane) * 4 % 4096 + 1];
    R.rv[2] = coefs[(b * 64 + lane) * 4 % 4096 + 2];
    R.rv[3] = coefs[(b * 64 + lane) * 4 % 4096 + 3];
  }
  // the tile in layout 2 (registers = tile bits 8..11): 16-B pieces
  double2 v[kRegs];
  {
    const int y0 = ybase_n<TB, 2>(t);
    const char* base = (const char*)(st + state_base(b, (int64_t)1 << L, og));
#pragma unroll
    for (int r = 0; r < kRegs; ++r) {
      const int64_t x = tbase | ((int64_t)(y0 | (r << reg_pos<TB, 2>())) << w0);
      const d2v w = *(const d2v*)(base + (octet_spread(x, og) << 4));
      v[r] = make_double2(w.x, w.y);
    }
  }
  for (int e = t; e < 512; e += NT) s_tab[e] = tabs[e];
  __syncthreads();
  // kicks<N>(): N site kicks on register bits 0, 1, 2, 3, 0, ... with
  // readlane'd coefficients (all indices compile-time)
  auto kick = [&](auto q_tag) {
    constexpr int Q = decltype(q_tag)::value;
    layer_f<kKindRX, 0, Q & 3>(v, R.d(0, (Q * 5) & 127));
  };
  auto kicks = [&](auto n_tag) {
    constexpr int N = decltype(n_tag)::value;
    if constexpr (N >= 1) kick(std::integral_constant<int, 0>{});
    if constexpr (N >= 2) kick(std::integral_constant<int, 1>{});
    if constexpr (N >= 3) kick(std::integral_constant<int, 2>{});
    if constexpr (N >= 4) kick(std::integral_constant<int, 3>{});
    if constexpr (N >= 5) kick(std::integral_constant<int, 4>{});
  };
  auto swap16 = [&]() {
#pragma unroll
    for (int r = 0; r < kRegs; r += 2) {
      swap_rows<16>(v[r].x, v[r + 1].x);
      swap_rows<16>(v[r].y, v[r + 1].y);
    }
  };
  auto swap32 = [&]() {
#pragma unroll
    for (int r = 0; r < kRegs; r += 4) {
      swap_rows<32>(v[r].x, v[r + 2].x);
      swap_rows<32>(v[r].y, v[r + 2].y);
    }
  };
  int dk = 0;
  auto diag2 = [&]() {
    int ba = (t * 37 + dk * 11) & 255, bb = (t * 53 + dk * 7) & 255;
    asm volatile("" : "+v"(ba), "+v"(bb));
    ++dk;
#pragma unroll
    for (int r = 0; r < kRegs; ++r)
      v[r] = cmul(v[r], cmul(s_tab[ba ^ (r * 9)], s_tab[256 + (bb ^ (r * 5))]));
  };
  auto diag1 = [&]() {
    int ba = (t * 29 + dk * 13) & 255;
    asm volatile("" : "+v"(ba));
    ++dk;
#pragma unroll
    for (int r = 0; r < kRegs; ++r) v[r] = cmul(v[r], s_tab[ba ^ (r * 3)]);
  };
  auto xch = [&](auto f_tag, auto t_tag) {
    constexpr int F = decltype(f_tag)::value, T = decltype(t_tag)::value;
    int bf = ybase_n<TB, F>(t), bt = ybase_n<TB, T>(t);
    asm volatile("" : "+v"(bf), "+v"(bt));
#pragma unroll
    for (int r = 0; r < kRegs; ++r) s_x[swz(bf | (r << reg_pos<TB, F>()))] = v[r].x;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kRegs; ++r) v[r].x = s_x[swz(bt | (r << reg_pos<TB, T>()))];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kRegs; ++r) s_x[swz(bf | (r << reg_pos<TB, F>()))] = v[r].y;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kRegs; ++r) v[r].y = s_x[swz(bt | (r << reg_pos<TB, T>()))];
  };
  using C0 = std::integral_constant<int, 0>;
  using C1 = std::integral_constant<int, 1>;
  using C2 = std::integral_constant<int, 2>;
  using C3 = std::integral_constant<int, 3>;
  if constexpr (TB == 12) {
    // dtc_lcw3_final's program
    kicks(std::integral_constant<int, 4>{}); swap16(); kicks(std::integral_constant<int, 1>{}); diag2();
    kicks(std::integral_constant<int, 4>{}); swap32(); kicks(std::integral_constant<int, 1>{});
    xch(C2{}, C0{});
    kicks(std::integral_constant<int, 4>{}); swap16(); swap32(); kicks(std::integral_constant<int, 2>{}); diag2(); kicks(std::integral_constant<int, 4>{});
    xch(C0{}, C1{});
    kicks(std::integral_constant<int, 4>{}); swap16(); kicks(std::integral_constant<int, 1>{}); diag2(); kicks(std::integral_constant<int, 3>{});
    xch(C1{}, C2{});
    kicks(std::integral_constant<int, 4>{}); diag2(); kicks(std::integral_constant<int, 4>{}); swap16(); kicks(std::integral_constant<int, 1>{}); diag1(); kicks(std::integral_constant<int, 3>{}); diag1(); kicks(std::integral_constant<int, 1>{});
  } else {
    // 58 kicks, 8 row swaps, 5 + 2 diagonals, 4 re-layouts
    kicks(std::integral_constant<int, 4>{}); swap16(); swap32(); kicks(std::integral_constant<int, 5>{}); diag2();     // l-1 (9)
    kicks(std::integral_constant<int, 4>{}); swap16(); kicks(std::integral_constant<int, 2>{});
    xch(C2{}, C0{});
    kicks(std::integral_constant<int, 4>{}); swap32(); kicks(std::integral_constant<int, 3>{}); diag2();               // l0 (13)
    kicks(std::integral_constant<int, 4>{}); swap16(); kicks(std::integral_constant<int, 2>{});
    xch(C0{}, C1{});
    kicks(std::integral_constant<int, 5>{}); diag2(); kicks(std::integral_constant<int, 4>{}); swap32(); kicks(std::integral_constant<int, 1>{});     // l1 (11)
    xch(C1{}, C3{});
    kicks(std::integral_constant<int, 4>{}); swap16(); kicks(std::integral_constant<int, 2>{}); diag2(); kicks(std::integral_constant<int, 4>{});     // l2 (9)
    xch(C3{}, C2{});
    kicks(std::integral_constant<int, 3>{}); diag2(); kicks(std::integral_constant<int, 4>{}); swap16(); kicks(std::integral_constant<int, 1>{}); diag1(); kicks(std::integral_constant<int, 3>{}); diag1(); kicks(std::integral_constant<int, 1>{});
  }
  double tot = 0.0, z = 0.0;
#pragma unroll
  for (int r = 0; r < kRegs; ++r) {
    const double p = fma(v[r].x, v[r].x, v[r].y * v[r].y);
    tot += p;
    z += (r & 4) ? -p : p;
  }
  tot = wave_sum(tot);
  z = wave_sum(z);
  if ((t & 63) == 0) {
    out[(by * 4096 + bx) * 2 % (1 << 22)] = tot + z;
  }
}

template <int TB, int WPC>
__global__ __launch_bounds__(1 << (TB - 4), WPC) void k_lc(const double2* __restrict__ st, int L,
                                                          int w0, int og, int batch,
                                                          const double* __restrict__ coefs,
                                                          const double2* __restrict__ tabs,
                                                          double* __restrict__ out) {
  __shared__ double s_x[1 << TB];
  __shared__ double2 s_tab[512];
  lc_body<TB>(st, L, w0, og, batch, coefs, tabs, out, s_x, s_tab, blockIdx.x, blockIdx.y);
}

// A synthetic 12-site K-D-K (the product's dtc_kdk_pass3<7> shape): 16
// nontemporal 16-B loads of a contiguous 4096-amplitude tile in layout 1
// (lanes = tile bits 0..3, 8..11), 24 kicks in six 4-site rounds with four
// half-tile re-layouts, one diagonal lookup per amplitude, 16 nontemporal
// stores in place.
__device__ __forceinline__ void kdk_body(double2* __restrict__ st, int L, int og, int batch,
                                         const double* __restrict__ coefs,
                                         const double2* __restrict__ tabs, double* s_x,
                                         double2* s_tab, unsigned bx, unsigned by) {
  const int t = threadIdx.x;
  const int64_t b = ((int64_t)by << 3) | (bx & 7);
  const int64_t tile = bx >> 3;
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
  char* base = (char*)(st + state_base(b, (int64_t)1 << L, og));
  const int64_t tb = tile << 12;
  auto addr = [&](int r) { return base + (octet_spread(tb | tile_y<1>(t, r), og) << 4); };
  double2 v[kRegs];
#pragma unroll
  for (int r = 0; r < kRegs; ++r) {
    const d2v w = __builtin_nontemporal_load((const d2v*)addr(r));
    v[r] = make_double2(w.x, w.y);
  }
  s_tab[t] = tv;
  auto nib = [&](auto q0) {
    constexpr int K = decltype(q0)::value;
    layer_f<kKindRX, 0, 0>(v, R.d(0, K + 0));
    layer_f<kKindRX, 0, 1>(v, R.d(0, K + 1));
    layer_f<kKindRX, 0, 2>(v, R.d(0, K + 2));
    layer_f<kKindRX, 0, 3>(v, R.d(0, K + 3));
  };
  nib(std::integral_constant<int, 0>{});
  exchange_split<1, 0>(v, s_x, t);
  nib(std::integral_constant<int, 4>{});
  exchange_split<0, 2>(v, s_x, t);
  nib(std::integral_constant<int, 8>{});
  {
    int ba = t & 255;
    asm volatile("" : "+v"(ba));
#pragma unroll
    for (int r = 0; r < kRegs; ++r) v[r] = cmul(v[r], s_tab[(ba ^ (r * 7)) & 255]);
  }
  nib(std::integral_constant<int, 12>{});
  exchange_split<2, 0>(v, s_x, t);
  nib(std::integral_constant<int, 16>{});
  exchange_split<0, 1>(v, s_x, t);
  nib(std::integral_constant<int, 20>{});
#pragma unroll
  for (int r = 0; r < kRegs; ++r) {
    d2v w = {v[r].x, v[r].y};
    __builtin_nontemporal_store(w, (d2v*)addr(r));
  }
}

__global__ __launch_bounds__(256, 3) void k_kdk(double2* __restrict__ st, int L, int og, int batch,
                                                 const double* __restrict__ coefs,
                                                 const double2* __restrict__ tabs) {
  __shared__ double s_x[4096];
  __shared__ double2 s_tab[512];
  kdk_body(st, L, og, batch, coefs, tabs, s_x, s_tab, blockIdx.x, blockIdx.y);
}

// Both in one launch: groups of eight blocks (one octet tile, one block per
// XCD) alternate between a K-D-K tile of `kst` and a light-cone tile of `lst`,
// so every CU holds a mix of memory-bound and VALU-bound workgroups.
__global__ __launch_bounds__(256, 3) void k_fused(double2* __restrict__ kst,
                                                   const double2* __restrict__ lst, int L, int og,
                                                   int batch, const double* __restrict__ coefs,
                                                   const double2* __restrict__ tabs,
                                                   double* __restrict__ out) {
  __shared__ double s_x[4096];
  __shared__ double2 s_tab[512];
  const unsigned g = blockIdx.x >> 3, bx = ((g >> 1) << 3) | (blockIdx.x & 7);
  if (g & 1) lc_body<12>(lst, L, 5, og, batch, coefs, tabs, out, s_x, s_tab, bx, blockIdx.y);
  else kdk_body(kst, L, og, batch, coefs, tabs, s_x, s_tab, bx, blockIdx.y);
}

int main(int argc, char** argv) {
  const int L = 20, B = argc > 1 ? atoi(argv[1]) : 1024, og = 6;
  const size_t n = (size_t)B << L;
  double2* st;
  double *coefs, *out;
  double2* tabs;
  double2* st2;
  CHECK(hipMalloc(&st, n * 16));
  CHECK(hipMemset(st, 0, n * 16));
  CHECK(hipMalloc(&st2, n * 16));
  CHECK(hipMemset(st2, 0, n * 16));
  CHECK(hipMalloc(&coefs, 4096 * 8));
  CHECK(hipMemset(coefs, 0, 4096 * 8));
  CHECK(hipMalloc(&tabs, 512 * 16));
  CHECK(hipMemset(tabs, 0, 512 * 16));
  CHECK(hipMalloc(&out, (1 << 22) * 8));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
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
    printf("%-48s %8.3f ms  %7.0f GB/s read\n", name, ms, n * 16.0 / (ms * 1e6));
    return 0;
  };
  const unsigned oct = (unsigned)((B + 7) / 8);
  // 12-bit: window j-5 .. j+6 at j = 10 -> global bits 5 .. 16
  if (run("12-bit lcw3 program, 4 WG/CU (w0 = 5)", [&] {
        hipLaunchKernelGGL((k_lc<12, 4>), dim3(8u << (L - 12), oct), dim3(256), 0, 0, st, L, 5, og,
                           B, coefs, tabs, out);
      }))
    return 1;
  // 14-bit: window j-7 .. j+6 -> global bits 3 .. 16
  if (run("14-bit program, 1 WG/CU (w0 = 3)", [&] {
        hipLaunchKernelGGL((k_lc<14, 1>), dim3(8u << (L - 14), oct), dim3(1024), 0, 0, st, L, 3, og,
                           B, coefs, tabs, out);
      }))
    return 1;
  if (run("synthetic 12-site K-D-K, 3 WG/CU", [&] {
        hipLaunchKernelGGL(k_kdk, dim3(8u << (L - 12), oct), dim3(256), 0, 0, st2, L, og, B, coefs,
                           tabs);
      }))
    return 1;
  if (run("K-D-K then lcw3 program (two launches)", [&] {
        hipLaunchKernelGGL(k_kdk, dim3(8u << (L - 12), oct), dim3(256), 0, 0, st2, L, og, B, coefs,
                           tabs);
        hipLaunchKernelGGL((k_lc<12, 4>), dim3(8u << (L - 12), oct), dim3(256), 0, 0, st, L, 5, og,
                           B, coefs, tabs, out);
      }))
    return 1;
  if (run("K-D-K + lcw3 program fused (one launch, 3 WG/CU)", [&] {
        hipLaunchKernelGGL(k_fused, dim3(16u << (L - 12), oct), dim3(256), 0, 0, st2, st, L, og, B,
                           coefs, tabs, out);
      }))
    return 1;
  if (run("12-bit lcw3 program, 4 WG/CU (again)", [&] {
        hipLaunchKernelGGL((k_lc<12, 4>), dim3(8u << (L - 12), oct), dim3(256), 0, 0, st, L, 5, og,
                           B, coefs, tabs, out);
      }))
    return 1;
  if (run("14-bit program, 1 WG/CU (again)", [&] {
        hipLaunchKernelGGL((k_lc<14, 1>), dim3(8u << (L - 14), oct), dim3(1024), 0, 0, st, L, 3, og,
                           B, coefs, tabs, out);
      }))
    return 1;
  return 0;
}
