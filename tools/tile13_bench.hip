// Tile-shape study, round 4 (not part of the product):
// the bare in-place access pattern (16 nontemporal 16-B loads and stores per
// lane, octet layout at 1 KiB, the eight states of an octet on consecutive
// blocks) of tiles of 2^(12+E) amplitudes = c column bits (index bits
// 0 .. c-1) + the sites s0 .. s0+12+E-c-1, threads = the low tile bits, at a
// fixed number of workgroups per CU (LDS padding, as the pass kernels' tiles
// limit them).  The question: does a 13-bit tile (a 13-site group A and a
// 7-site group B with 1 KiB columns at L=20) stream faster than the 12/8
// split's 256-B columns (pass_pattern_bench: 5.8-5.95 TB/s)?
// Build: hipcc --offload-arch=gfx950 -O3 tools/tile13_bench.hip -o tools/tile13_bench
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double d2v __attribute__((ext_vector_type(2)));

template <int E, int WPC>
__global__ __launch_bounds__(256 << E) void k_tile(d2v* __restrict__ a, int L, int c, int s0,
                                                  double f) {
  constexpr int TB = 12 + E;
  __shared__ double s_pad[(160 * 1024 / WPC - 1024) / 8];  // WPC workgroups per CU
  const int t = threadIdx.x;
  const int tile_bits = L - TB;
  const int64_t n_tiles = (int64_t)1 << tile_bits;
  const int64_t b = blockIdx.x;
  const int64_t tile = (b >> 3) & (n_tiles - 1);
  const int64_t st = ((b >> (3 + tile_bits)) << 3) | (b & 7);
  const int mid_bits = s0 - c;
  const int64_t mid_mask = ((int64_t)1 << mid_bits) - 1;
  const int64_t tbase = ((tile & mid_mask) << c) | ((tile >> mid_bits) << (s0 + TB - c));
  auto rel = [&](int y) -> int64_t {
    return (int64_t)(y & ((1 << c) - 1)) | ((int64_t)(y >> c) << s0);
  };
  auto addr = [&](int64_t x) -> int64_t {
    return ((st >> 3) << (L + 3)) + ((x >> 6) << 9) + ((st & 7) << 6) + (x & 63);
  };
  d2v v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = __builtin_nontemporal_load(&a[addr(tbase | rel(t | (r << (8 + E))))]);
  if (f == 12345.0) s_pad[t] = v[0].x;
#pragma unroll
  for (int r = 0; r < 16; ++r)
    __builtin_nontemporal_store(v[r] * (1.0 + f), &a[addr(tbase | rel(t | (r << (8 + E))))]);
}

// Alternating layouts (round 4): a pass reads its tile from a layout where
// the tile is contiguous and writes it to the other layout, where it is the
// 256-B-column pattern (the next pass's tile is contiguous there): both passes
// "read contiguous, write columns" instead of the 12/8 split's one contiguous
// and one column pass.  RD/WR: 0 = the tile at c = 12 (contiguous), 1 = the
// same tile indices placed as a c = 4, s = 12 tile; out of place (a -> b).
template <int RD, int WR>
__global__ __launch_bounds__(256) void k_alt(const d2v* __restrict__ a, d2v* __restrict__ bo, int L,
                                              double f) {
  __shared__ double s_pad[(160 * 1024 / 2 - 1024) / 8];  // 2 workgroups per CU
  const int t = threadIdx.x;
  const int tile_bits = L - 12;
  const int64_t n_tiles = (int64_t)1 << tile_bits;
  const int64_t b = blockIdx.x;
  const int64_t tile = (b >> 3) & (n_tiles - 1);
  const int64_t st = ((b >> (3 + tile_bits)) << 3) | (b & 7);
  auto addr = [&](int64_t x) -> int64_t {
    return ((st >> 3) << (L + 3)) + ((x >> 6) << 9) + ((st & 7) << 6) + (x & 63);
  };
  // tile index y (12 bits) of tile `tile`: layout 0 -> x = tile << 12 | y;
  // layout 1 -> bits 0..3 of y stay, y's bits 4..11 go to x bits 12..19 and the
  // tile id fills x bits 4..11 (the tile's sites 4..11 at memory bits 12..19)
  auto place = [&](int lay, int y) -> int64_t {
    if (lay == 0) return (tile << 12) | y;
    return (int64_t)(y & 15) | ((int64_t)(y >> 4) << 12) | ((tile & 255) << 4) |
           ((tile >> 8) << 20);
  };
  d2v v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int y = RD == 0 ? ((t & 15) | (r << 4) | ((t >> 4) << 8)) : (t | (r << 8));
    v[r] = __builtin_nontemporal_load(&a[addr(place(RD, y))]);
  }
  if (f == 12345.0) s_pad[t] = v[0].x;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int y = RD == 0 ? ((t & 15) | (r << 4) | ((t >> 4) << 8)) : (t | (r << 8));
    __builtin_nontemporal_store(v[r] * (1.0 + f), &bo[addr(place(WR, y))]);
  }
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

int main() {
  const int L = 20, B = 512;  // 8 GiB, octets of L=20 states
  const size_t n = (size_t)B << L;
  d2v* a;
  if (hipMalloc(&a, n * 16) != hipSuccess) return 1;
  (void)hipMemset(a, 0, n * 16);
  auto run = [&](const char* name, auto kern, int E, int c, int s0) {
    const unsigned blocks = (unsigned)(n >> (12 + E));
    const float ms = time_it([&] { hipLaunchKernelGGL(kern, dim3(blocks), dim3(256 << E), 0, 0, a, L, c, s0, 0.0); }, 8);
    printf("%-44s %8.3f ms %7.0f GB/s\n", name, ms, 2.0 * n * 16 / ms / 1e6);
    fflush(stdout);
  };
  d2v* a2;
  if (hipMalloc(&a2, n * 16) != hipSuccess) return 1;
  (void)hipMemset(a2, 0, n * 16);
  auto run_alt = [&](const char* name, auto kern) {
    const unsigned blocks = (unsigned)(n >> 12);
    const float ms = time_it([&] { hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, a, a2, L, 0.0); }, 8);
    printf("%-44s %8.3f ms %7.0f GB/s\n", name, ms, 2.0 * n * 16 / ms / 1e6);
    fflush(stdout);
  };
  for (int rep = 0; rep < 2; ++rep) {
    run_alt("alt: read contiguous, write 256-B columns", k_alt<0, 1>);
    run_alt("alt: read 256-B columns, write contiguous", k_alt<1, 0>);
    run_alt("alt: contiguous -> contiguous (copy ref)", k_alt<0, 0>);
    run_alt("alt: columns -> columns (copy ref)", k_alt<1, 1>);
    run("12-bit B c=4  s 12..19 1 WG/CU ( 4 waves)", k_tile<0, 1>, 0, 4, 12);
    run("12-bit A c=12          1 WG/CU ( 4 waves)", k_tile<0, 1>, 0, 12, 12);
  }
  for (int rep = 0; rep < 2; ++rep) {
    run("12-bit A c=12          2 WG/CU ( 8 waves)", k_tile<0, 2>, 0, 12, 12);
    run("12-bit A c=12          3 WG/CU (12 waves)", k_tile<0, 3>, 0, 12, 12);
    run("12-bit B c=4  s 12..19 2 WG/CU ( 8 waves)", k_tile<0, 2>, 0, 4, 12);
    run("12-bit B c=4  s 12..19 3 WG/CU (12 waves)", k_tile<0, 3>, 0, 4, 12);
    run("12-bit B c=5  s 13..19 2 WG/CU ( 8 waves)", k_tile<0, 2>, 0, 5, 13);
    run("12-bit B c=6  s 14..19 2 WG/CU ( 8 waves)", k_tile<0, 2>, 0, 6, 14);
    run("13-bit A c=13          1 WG/CU ( 8 waves)", k_tile<1, 1>, 1, 13, 13);
    run("13-bit A c=13          2 WG/CU (16 waves)", k_tile<1, 2>, 1, 13, 13);
    run("13-bit B c=6  s 13..19 1 WG/CU ( 8 waves)", k_tile<1, 1>, 1, 6, 13);
    run("13-bit B c=6  s 13..19 2 WG/CU (16 waves)", k_tile<1, 2>, 1, 6, 13);
    run("13-bit B c=5  s 12..19 1 WG/CU ( 8 waves)", k_tile<1, 1>, 1, 5, 12);
    run("13-bit B c=5  s 12..19 2 WG/CU (16 waves)", k_tile<1, 2>, 1, 5, 12);
  }
  return 0;
}
