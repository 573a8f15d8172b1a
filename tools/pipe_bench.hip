// Feasibility study (not part of the product): a persistent, LDS-DMA double-
// buffered variant of the pass kernel's tile structure.  One 256-thread
// workgroup per CU walks a contiguous range of 4096-amplitude tiles; the
// next tile's 64 KiB arrive by global_load_lds (swizzle on the source address)
// while the current tile does R kick-like FMA layers and X LDS re-layouts;
// raw s_barrier + counted vmcnt so the prefetch stays in flight.  Compared with
// the non-persistent 2-workgroups-per-CU structure on the same work, from the
// Infinity Cache (in-place sweeps of <= 256 MiB) and from HBM (4 GiB).
// Build: hipcc --offload-arch=gfx950 -O3 tools/pipe_bench.hip -o tools/pipe_bench
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

__device__ __forceinline__ int slot(int y) { return y ^ ((y >> 4) & 15); }

template <int LAYERS>
__device__ __forceinline__ void layers(double2 (&v)[16], double f) {
#pragma unroll
  for (int l = 0; l < LAYERS; ++l) {
    const int q = l & 3;
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

__device__ __forceinline__ void bar_lds() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// baseline: one tile per workgroup, register loads, 2 WG/CU
template <int LAYERS, int EXCH>
__global__ __launch_bounds__(256, 2) void tile_plain(double2* a, double f) {
  __shared__ double2 s[4096];
  const int t = threadIdx.x;
  const size_t base = (size_t)blockIdx.x * 4096;
  double2 v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = a[base + t + 256 * r];
  layers<LAYERS / (EXCH + 1)>(v, f);
#pragma unroll
  for (int e = 0; e < EXCH; ++e) {
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) s[slot(t + 256 * r)] = v[r];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = s[slot((t << 4) | r)];
    layers<LAYERS / (EXCH + 1)>(v, f);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) s[slot((t << 4) | r)] = v[r];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = s[slot(t + 256 * r)];
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) a[base + t + 256 * r] = v[r];
}

// persistent, DMA double buffer, 1 WG/CU
template <int LAYERS, int EXCH>
__global__ __launch_bounds__(256, 1) void tile_pipe(double2* a, double f, int n_tiles) {
  __shared__ double2 s[2 * 4096];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int per = (n_tiles + gridDim.x - 1) / gridDim.x;
  const int first = blockIdx.x * per;
  const int last = min(first + per, n_tiles);
  if (first >= last) return;
  // DMA one tile into buffer `buf`: wave w, instruction i fills slots
  // (16 w + i) * 64 + lane with tile index slot^-1 (swizzle on the source)
  // inline-asm LDS-DMA: hipcc neither counts it nor drains it at LDS
  // accesses of the other buffer; completion is waited for by hand (vmcnt)
  const unsigned s_lds = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)s;
  auto dma = [&](int tile, int buf) {
    const double2* src = a + (size_t)tile * 4096;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int k = (wave * 16 + i) * 64 + lane;
      const int y = k ^ ((k >> 4) & 15);
      const double2* g = src + y;
      const unsigned dst = __builtin_amdgcn_readfirstlane(
          s_lds + (unsigned)((buf * 4096 + (wave * 16 + i) * 64) * 16));
      unsigned keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                   "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(g), "s"(dst) : "memory");
    }
  };
  dma(first, 0);
  for (int tile = first; tile < last; ++tile) {
    const int cur = (tile - first) & 1;
    double2* sb = s + cur * 4096;
    // this tile's DMA (issued one iteration ago, before 16 stores) has landed
    if (tile == first) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    bar_lds();
    double2 v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = sb[slot(t + 256 * r)];
    if (tile + 1 < last) dma(tile + 1, cur ^ 1);
    layers<LAYERS / (EXCH + 1)>(v, f);
#pragma unroll
    for (int e = 0; e < EXCH; ++e) {
#pragma unroll
      for (int r = 0; r < 16; ++r) sb[slot(t + 256 * r)] = v[r];
      bar_lds();
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = sb[slot((t << 4) | r)];
      layers<LAYERS / (EXCH + 1)>(v, f);
#pragma unroll
      for (int r = 0; r < 16; ++r) sb[slot((t << 4) | r)] = v[r];
      bar_lds();
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = sb[slot(t + 256 * r)];
    }
    double2* dst = a + (size_t)tile * 4096;
#pragma unroll
    for (int r = 0; r < 16; ++r) dst[t + 256 * r] = v[r];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const size_t max_bytes = (size_t)4 << 30;
  double2* a;
  CHECK(hipMalloc(&a, max_bytes));
  CHECK(hipMemset(a, 0, max_bytes));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int reps = 20;
  auto run = [&](const char* name, size_t mib, auto launch) {
    for (int w = 0; w < 3; ++w) launch();
    (void)hipEventRecord(e0);
    for (int i = 0; i < reps; ++i) launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double us = 1000.0 * ms / reps;
    printf("%-34s %6zu MiB  %9.1f us  %6.0f GB/s\n", name, mib, us, 2.0 * (mib << 20) / us / 1e3);
  };
  for (size_t mib : {128, 192, 4096}) {
    const int nt = (int)((mib << 20) / 65536);
    run("plain  24 layers 4 exch (2 WG/CU)", mib, [&] {
      hipLaunchKernelGGL((tile_plain<24, 2>), dim3(nt), dim3(256), 0, 0, a, 0.01);
    });
    run("pipe   24 layers 4 exch (1 WG/CU)", mib, [&] {
      hipLaunchKernelGGL((tile_pipe<24, 2>), dim3(cus), dim3(256), 0, 0, a, 0.01, nt);
    });
    run("plain   0 layers 4 exch", mib, [&] {
      hipLaunchKernelGGL((tile_plain<0, 2>), dim3(nt), dim3(256), 0, 0, a, 0.01);
    });
    run("pipe    0 layers 4 exch", mib, [&] {
      hipLaunchKernelGGL((tile_pipe<0, 2>), dim3(cus), dim3(256), 0, 0, a, 0.01, nt);
    });
  }
  return 0;
}
