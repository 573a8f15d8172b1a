// dtc_tile13.hip — gfx950 passes over a 13-site group (the 13 / 7 split of an
// L = 20 period, round 6).
//
// The 12 / 8 split of dtc_kernels.hip gives the high group 8 sites over 256-B
// columns; that column pass runs 5.8 ms per period against 5.4 for the 12-site
// pass (r5w).  Moving site 12 into the low group leaves the high group 7 sites
// over 512-B columns (tile bits 0..4 + 13..19, a 12-bit tile: dtc_kernels.hip
// pass_body with geometry kGeoB7) and makes the low group 13 sites, a 13-bit
// tile of 8192 contiguous amplitudes: this file.  The synthetic passes of
// tools/tile13_kdk_probe.hip measured the pair at 5.14 + 5.42 ms against
// 5.06 + 6.10 for the 12 / 8 pair (profiles/r6c_tile13_kdk_probe.txt).
//
// A workgroup: 512 threads (8 waves) x 16 amplitudes in registers, re-layouts
// through a 64 KiB half-tile LDS buffer (real parts, then imaginary parts), two
// workgroups per CU (128 VGPRs).  Layouts (tile bit at register position 0..3,
// lane bit 0..5, wave bit 0..2):
//   LIO  regs 4 5 6 7 | lanes 0 1 2 3 8 9 | waves 10 11 12   (load / store:
//                                                              256-B runs)
//   LIOs regs 8 5 6 7 | lanes 0 1 2 3 4 9 | waves 10 11 12   (LIO after a row
//                                                              swap of register
//                                                              bit 0, lane bit 4)
//   L0   regs 0 1 2 3 | lanes 4 .. 9      | waves 10 11 12
//   L9   regs 9 .. 12 | lanes 0 .. 5      | waves 6 7 8       (the diagonal)
// K-D-K program: LIO kick 4..7, swap, kick 8 | L0 kick 0..3 | L9 kick 9..12,
// D, measure, kick 9..12 | L0 kick 0..3 | LIOs kick 8, swap back, kick 4..7:
// four re-layouts and two row swaps for 26 site kicks (the 12-site pass: four
// re-layouts for 24).  Kick records: pre-kick of tile bit k at rec k, post at
// 13 + k, the total (global factor, 1 / w_post^2) at 26 (prep_kernel, tb 13).
#include <type_traits>

#include "dtc_device.h"
#include "dtc_kernels.h"

namespace dtc {
namespace t13 {

static constexpr int kBits = 13;
static constexpr int kNT = 512;  // threads
static constexpr int kWaves = kNT / 64;
static constexpr int kRecTot = 2 * kBits;
static_assert(kRecTot + 1 <= kRecPerState, "13-bit kick records fit the record block");

enum : int { LIO = 0, LIOs, L0, L9 };
// tile bit at position p of layout li (0..3 registers, 4..9 lanes, 10..12 waves)
__host__ __device__ constexpr int lay_bit(int li, int p) {
  constexpr int tab[4][13] = {{4, 5, 6, 7, 0, 1, 2, 3, 8, 9, 10, 11, 12},
                              {8, 5, 6, 7, 0, 1, 2, 3, 4, 9, 10, 11, 12},
                              {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12},
                              {9, 10, 11, 12, 0, 1, 2, 3, 4, 5, 6, 7, 8}};
  return tab[li][p];
}
// tile index of register r (thread bits zero) and of thread t (register bits zero)
__host__ __device__ constexpr int yreg(int li, int r) {
  return ((r & 1) << lay_bit(li, 0)) | (((r >> 1) & 1) << lay_bit(li, 1)) |
         (((r >> 2) & 1) << lay_bit(li, 2)) | (((r >> 3) & 1) << lay_bit(li, 3));
}
template <int LI>
__device__ __forceinline__ int ythr(int t) {
  int y = 0;
#pragma unroll
  for (int p = 4; p < 13; ++p) y |= ((t >> (p - 4)) & 1) << lay_bit(LI, p);
  return y;
}
// half-tile LDS slot (8-B): the tile index XOR-swizzled, linear over XOR.
// ds_write_b64 serves 16 contiguous lanes per LDS cycle (bank = slot mod 16
// in 8-B units), ds_read_b64 32 (slot mod 32; MI355X_MICROARCH.md §LDS).  Slot
// vector of tile bit k: k < 4: 1 << k; 4..8: (1 << k) ^ (1 << (k - 4)); 9..12:
// 1 << k.  Lane bits 0..3 of every layout written (LIO, LIOs, L9: tile bits
// 0..3; L0: 4..7) are independent mod 16, lane bits 0..4 of every layout read
// (L0: 4..8; L9, LIOs: 0..4; LIO: 0..3, 8) mod 32: conflict-free (checked by
// simulating the lane groups; the first map, y ^ ((y >> 5) & 15) ^ (y >> 8 &
// 1) << 4, made L0's writes two-way: 256 conflict cycles per wave, r6e).
__host__ __device__ constexpr int slot(int y) { return y ^ ((y >> 4) & 31); }

template <int FROM, int TO>
__device__ __forceinline__ void xch(double2 (&v)[kRegs], double* s_half, int t, int xw = 0, int xr = 0) {
  // xw, xr: the Pauli frame's X bits flushed by the pass's re-layouts before
  // and including this one (frame13_records, cumulative): index y is written
  // at slot(y ^ xw), read from slot(y ^ xr) (slot is linear over XOR), so the
  // tile comes out X^(xw ^ xr)-permuted and no barrier precedes the writes: a
  // thread writes exactly the slots it read itself in the previous re-layout
  // (which ended in layout FROM, read with this one's xw)
  int bf = slot(ythr<FROM>(t)) ^ slot(xw), bt = slot(ythr<TO>(t)) ^ slot(xr);
  asm volatile("" : "+v"(bf), "+v"(bt));
#pragma unroll
  for (int r = 0; r < kRegs; ++r) s_half[bf ^ slot(yreg(FROM, r))] = v[r].x;
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kRegs; ++r) v[r].x = s_half[bt ^ slot(yreg(TO, r))];
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kRegs; ++r) s_half[bf ^ slot(yreg(FROM, r))] = v[r].y;
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kRegs; ++r) v[r].y = s_half[bt ^ slot(yreg(TO, r))];
}

// one site kick: register bit Q, record k -- the form-B butterfly with the
// frame-signed coefficient (frame13_records), no variant branch
template <int Q, int KIND, typename Rec>
__device__ __forceinline__ void kick(double2 (&v)[kRegs], const Rec& R, int k) {
  layer_f<KIND, 2, Q>(v, R.d(k, 0));
}
// the four register sites of layout LI (records rec0 + tile bit)
template <int LI, int KIND, typename Rec>
__device__ __forceinline__ void kick4(double2 (&v)[kRegs], const Rec& R, int rec0) {
  kick<0, KIND>(v, R, rec0 + lay_bit(LI, 0));
  kick<1, KIND>(v, R, rec0 + lay_bit(LI, 1));
  kick<2, KIND>(v, R, rec0 + lay_bit(LI, 2));
  kick<3, KIND>(v, R, rec0 + lay_bit(LI, 3));
}

}  // namespace t13

template <int SHAPE, int KIND, int MC, bool NS>
__device__ __forceinline__ void pass13_body(const PassArgs& A) {
  using namespace t13;
  constexpr bool PRE = SHAPE == kShapeK || SHAPE == kShapeKD || SHAPE == kShapeKDK;
  constexpr bool DIAG = SHAPE == kShapeKD || SHAPE == kShapeDK || SHAPE == kShapeKDK || SHAPE == kShapeD;
  constexpr bool POST = SHAPE == kShapeDK || SHAPE == kShapeKDK;
  static_assert(KIND == kKindRX || KIND == kKindRY, "13-site passes: factored kicks");
  __shared__ double s_half[1 << kBits];
  __shared__ double2 s_chunk[DIAG ? kMaxChunks * 64 : 1];
  __shared__ double2 s_win[DIAG ? 64 : 1];
  __shared__ double s_red[kWaves][2];

  const int t = threadIdx.x;
  const int64_t n_tiles = (int64_t)1 << (A.L_eff - kBits);
  const int og = A.octet_bits;
  const int64_t b = og ? (((int64_t)blockIdx.y << 3) | (blockIdx.x & 7)) : (int64_t)blockIdx.y;
  const int64_t tile = og ? (int64_t)(blockIdx.x >> 3)
                          : ((gridDim.x & 7) ? (int64_t)blockIdx.x
                                             : (int64_t)(blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3));
  if (og && b >= A.batch) return;
  const int inst = (int)((A.batch_start + b) / A.n_traj);
#ifdef DTC_T13_RECREGS
  // the state's kick records, lane-distributed (RecRegs: 27 records)
  RecRegs R;
  {
    const int lane = t & 63;
    const double2* rp = (const double2*)(A.recs + b * kRecPerState) + 2 * lane;
    double2 r0 = make_double2(0.0, 0.0), r1 = make_double2(0.0, 0.0);
    if (4 * lane < 8 * kRecPerState) {
      r0 = rp[0];
      r1 = rp[1];
    }
    R.rv[0] = r0.x; R.rv[1] = r0.y; R.rv[2] = r1.x; R.rv[3] = r1.y;
  }
#else
  // the state's kick records through the scalar data cache (RecScalar): the
  // 128-VGPR budget of two 512-thread workgroups per CU has no room for the
  // lane-distributed form
  const RecScalar R(A.recs + b * kRecPerState);
#endif
  // the tile: global bits 0..12, its id above
  const int64_t tbase = tile << kBits;
  // diagonal tables (issued before the tile's loads: vector memory returns in order)
  constexpr int kG0 = 9;  // window of L9's register bits 9..12
  double2 dchunk = make_double2(0.0, 0.0), dwin = make_double2(1.0, 0.0);
  const double2* dt = A.diag + (int64_t)inst * A.diag_stride;
  if (DIAG) {
    if (t < A.n_chunks * 64) dchunk = dt[t];
    if (t < 64) dwin = dt[(A.n_chunks + kG0) * 64 + t];
  }
  const int64_t vofs64 = octet_spread((int64_t)ythr<LIO>(t), og) << 4;
  const uint32_t vofs = (uint32_t)vofs64;  // lane bits <= global 12: always 32-bit
  auto tile_ofs = [&](int r) -> int64_t { return octet_spread(tbase | yreg(LIO, r), og) << 4; };
  const int64_t sbase = state_base(b, A.state_len, og);
  double2 v[kRegs];
  {
    const char* src = (const char*)(A.src + sbase);
#pragma unroll
    for (int r = 0; r < kRegs; ++r) {
      const d2v w = __builtin_nontemporal_load((const d2v*)(src + tile_ofs(r) + vofs));
      v[r] = make_double2(w.x, w.y);
    }
  }
  // vmcnt(16): records and tables landed, the tile's 16 loads in flight
  __builtin_amdgcn_s_waitcnt(0x4F70);
  // the Pauli frame's Z flush (frame13_records), a sign per amplitude at the
  // diagonal: tile bits 0..8 are L9's thread bits (zt), 9..12 its registers
  const int zm = R.i(kRecTot, kT13MaskZ);
  const bool zt = __builtin_popcount(ythr<L9>(t) & zm) & 1;
  if (DIAG) {
    const double cs = A.diag_conj ? -1.0 : 1.0;
    if (t < A.n_chunks * 64) s_chunk[t] = make_double2(dchunk.x, cs * dchunk.y);
    // the window entry of register bits (t >> 1) & 15 (tile bits 9..12) takes
    // their share of the Z flush
    const double zs = (__builtin_popcount((t >> 1) & (zm >> 9) & 15) & 1) ? -1.0 : 1.0;
    if (t < 64) s_win[t] = make_double2(zs * dwin.x, zs * cs * dwin.y);
    // made visible by the first re-layout's barriers (every shape re-lays out
    // before its diagonal: L9 is not the load layout)
  }
  const double2 gph = make_double2(R.d(kRecTot, 0), R.d(kRecTot, 1));
  const double inv_w2_mid = R.d(kRecTot, 2);

  // probe partials (MC 1): each thread's (|a|^2, z_j |a|^2) sums in layout LI;
  // the wave / workgroup reduction runs after the stores
  double pm_tot = 0.0, pm_z = 0.0, pm_inv = 1.0;
  bool pm_on = false;
  auto measure = [&](auto lay_tag, double inv_w2) {
    constexpr int LI = decltype(lay_tag)::value;
    double tot = 0.0, zq[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int r = 0; r < kRegs; ++r) {
      const double p = fma(v[r].x, v[r].x, v[r].y * v[r].y);
      tot += p;
#pragma unroll
      for (int q = 0; q < 4; ++q) zq[q] += ((r >> q) & 1) ? -p : p;
    }
    const int j = A.probe;
    double z = 0.0;
    if (j < kBits) {
      int q = -1;
#pragma unroll
      for (int p = 0; p < 4; ++p)
        if (lay_bit(LI, p) == j) q = p;
      if (q >= 0) z = q == 0 ? zq[0] : (q == 1 ? zq[1] : (q == 2 ? zq[2] : zq[3]));
      else z = ((ythr<LI>(t) >> j) & 1) ? -tot : tot;
    }
    pm_tot = tot;
    pm_z = z;
    pm_inv = inv_w2;
    pm_on = true;
  };

  using CLIO = std::integral_constant<int, LIO>;
  using CL9 = std::integral_constant<int, L9>;
  // ---- pre-kick: LIO 4..7, (swap) 8, L0 0..3, L9 9..12 ----
  if constexpr (PRE) {
    kick4<LIO, KIND>(v, R, 0);
    swap_reg_lane<0, 16>(v);
    kick<0, KIND>(v, R, 8);
    xch<LIOs, L0>(v, s_half, t, 0, R.i(kRecTot, kT13MaskX1));
    kick4<L0, KIND>(v, R, 0);
    xch<L0, L9>(v, s_half, t, R.i(kRecTot, kT13MaskX1), R.i(kRecTot, kT13MaskX2));
    kick4<L9, KIND>(v, R, 0);
  } else if constexpr (DIAG) {
    xch<LIO, L9>(v, s_half, t);
  }
  if constexpr (!DIAG) {
    // the global factor and the Z flush (L9: register bits = tile bits 9..12)
    const double2 g = zt ? make_double2(-gph.x, -gph.y) : gph;
    const double2 gn = make_double2(-g.x, -g.y);
    const int zr = (zm >> 9) & 15;
#pragma unroll
    for (int r = 0; r < kRegs; ++r) v[r] = cmul(v[r], (__builtin_popcount(r & zr) & 1) ? gn : g);
  } else {
    // D(x) = P_C * W[x]: P_C = D(x0) / W(x0) per thread, W indexed by bits
    // 8..13 of x (the 64-entry window table of start bit 9)
    const int64_t x0 = tbase | ythr<L9>(t);
    const int w0i = (int)(((x0 << 1) >> kG0) & 63);
    const double2 w0 = s_win[w0i];
    const double2 pc0 = cmul(cmul(diag_phase(s_chunk, A.n_chunks, x0), make_double2(w0.x, -w0.y)), gph);
    const double2 pc = zt ? make_double2(-pc0.x, -pc0.y) : pc0;
    // four window entries in flight at a time: all sixteen at once (64 VGPRs
    // next to the tile's 64) spilled at the 128-VGPR budget; the empty asm
    // (memory clobber) keeps the next group's reads below this group's products
#pragma unroll
    for (int r0 = 0; r0 < kRegs; r0 += 4) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[r0 + j] = cmul(v[r0 + j], cmul(pc, s_win[w0i | ((r0 + j) << 1)]));
      asm volatile("" : "+v"(v[r0].x), "+v"(v[r0].y), "+v"(v[r0 + 1].x), "+v"(v[r0 + 1].y),
                   "+v"(v[r0 + 2].x), "+v"(v[r0 + 2].y), "+v"(v[r0 + 3].x), "+v"(v[r0 + 3].y)
                   :: "memory");
    }
  }
  if constexpr (MC == 1) {
    if (A.meas != kMeasNone && !A.meas_at_end) {
      if constexpr (PRE || DIAG) measure(CL9{}, inv_w2_mid);
      else measure(CLIO{}, inv_w2_mid);
    }
  }
  // ---- post-kick: L9 9..12, L0 0..3, (LIOs) 8, swap back, LIO 4..7 ----
  if constexpr (POST) {
    kick4<L9, KIND>(v, R, kBits);
    xch<L9, L0>(v, s_half, t, R.i(kRecTot, kT13MaskX2), R.i(kRecTot, kT13MaskX3));
    kick4<L0, KIND>(v, R, kBits);
    xch<L0, LIOs>(v, s_half, t, R.i(kRecTot, kT13MaskX3), R.i(kRecTot, kT13MaskX4));
    kick<0, KIND>(v, R, kBits + 8);
    swap_reg_lane<0, 16>(v);
    kick4<LIO, KIND>(v, R, kBits);
  } else if constexpr (PRE || DIAG) {
    // (no flush of its own: the slot map the pre-kick's re-layouts left)
    xch<L9, LIO>(v, s_half, t, R.i(kRecTot, kT13MaskX2), R.i(kRecTot, kT13MaskX2));
  }
  if constexpr (MC == 1) {
    if (A.meas != kMeasNone && A.meas_at_end) measure(CLIO{}, 1.0);
  }
  if constexpr (!NS) {
    char* dst = (char*)(A.dst + sbase);
#pragma unroll
    for (int r = 0; r < kRegs; ++r) {
      d2v w = {v[r].x, v[r].y};
      __builtin_nontemporal_store(w, (d2v*)(dst + tile_ofs(r) + vofs));
    }
  }
  if constexpr (MC == 1) {
    if (pm_on) {  // workgroup-uniform (A.meas)
      const int wave = t >> 6, lane = t & 63;
      const int j = A.probe;
      const bool zin = j < kBits;
      const double tot = wave_sum(pm_tot);
      if (lane == 0) s_red[wave][0] = tot;
      if (zin) {
        const double z = wave_sum(pm_z);
        if (lane == 0) s_red[wave][1] = z;
      }
      __syncthreads();
      if (t < 2) {
        double acc = 0.0;
        const int ws = (t == 0 || zin) ? t : 0;
        for (int w = 0; w < kWaves; ++w) acc += s_red[w][ws];
        if (ws != t && ((tbase >> j) & 1)) acc = -acc;
        A.partial[(b * n_tiles + tile) * A.n_obs + t] = acc * pm_inv;
      }
    }
  }
}

// 512 threads, two workgroups per CU: four waves per SIMD, 128 VGPRs
// (launch_bounds' second argument alone leaves the compiler at three)
#define DTC_T13_BOUNDS __launch_bounds__(t13::kNT) __attribute__((amdgpu_waves_per_eu(4, 4)))
template <int SHAPE, int KIND, int MC>
__global__ DTC_T13_BOUNDS void dtc_pass13(PassArgs A) {
  pass13_body<SHAPE, KIND, MC, false>(A);
}
// the last pass of an echo chain (measure only, no store)
template <int SHAPE, int KIND>
__global__ DTC_T13_BOUNDS void dtc_final13(PassArgs A) {
  pass13_body<SHAPE, KIND, 1, true>(A);
}

template <int KIND, int MC>
hipError_t launch13_kind(const PassArgs& a, dim3 grid, int shape, hipStream_t stream) {
  const dim3 block(t13::kNT);
  if (a.no_store) {
    if constexpr (MC != 1) {
      return hipErrorInvalidValue;
    } else {
      switch (shape) {
        case kShapeKDK: hipLaunchKernelGGL((dtc_final13<kShapeKDK, KIND>), grid, block, 0, stream, a); break;
        case kShapeKD: hipLaunchKernelGGL((dtc_final13<kShapeKD, KIND>), grid, block, 0, stream, a); break;
        case kShapeDK: hipLaunchKernelGGL((dtc_final13<kShapeDK, KIND>), grid, block, 0, stream, a); break;
        case kShapeK: hipLaunchKernelGGL((dtc_final13<kShapeK, KIND>), grid, block, 0, stream, a); break;
        default: return hipErrorInvalidValue;
      }
      return hipGetLastError();
    }
  }
  switch (shape) {
    case kShapeKDK: hipLaunchKernelGGL((dtc_pass13<kShapeKDK, KIND, MC>), grid, block, 0, stream, a); break;
    case kShapeKD: hipLaunchKernelGGL((dtc_pass13<kShapeKD, KIND, MC>), grid, block, 0, stream, a); break;
    case kShapeDK: hipLaunchKernelGGL((dtc_pass13<kShapeDK, KIND, MC>), grid, block, 0, stream, a); break;
    case kShapeK: hipLaunchKernelGGL((dtc_pass13<kShapeK, KIND, MC>), grid, block, 0, stream, a); break;
    case kShapeD: hipLaunchKernelGGL((dtc_pass13<kShapeD, KIND, MC>), grid, block, 0, stream, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_pass13(const PassArgs& a, int batch, int shape, int kind, hipStream_t stream) {
  using namespace t13;
  // contiguous 13-site group at tile bits 0..12, no column split, unitary
  // factored kicks, the probe at most, no dual, no basis source
  if (a.tile_bits != kBits || a.c != kBits || a.act != (1 << kBits) - 1 || a.L_eff < kBits ||
      a.L_eff > 32 || a.batch != batch || batch > 65535 || a.n_chunks > kMaxChunks ||
      a.dst2 || a.basis || a.lc_layers > 0 || (a.meas != kMeasNone && a.meas != kMeasProbe) ||
      (kind != kKindRX && kind != kKindRY))
    return hipErrorInvalidValue;
  const int n_tiles = 1 << (a.L_eff - kBits);
  if (a.octet_bits && (a.octet_bits < 4 || a.octet_bits > a.L_eff)) return hipErrorInvalidValue;
  const dim3 grid = a.octet_bits ? dim3(n_tiles * 8, (batch + 7) / 8) : dim3(n_tiles, batch);
#ifdef DTC_T13_MC1_PROBE  // development A/B: the measuring instantiation for every pass
  const int mc = 1;
#else
  const int mc = a.meas == kMeasNone ? 0 : 1;
#endif
  if (kind == kKindRX)
    return mc ? launch13_kind<kKindRX, 1>(a, grid, shape, stream)
              : launch13_kind<kKindRX, 0>(a, grid, shape, stream);
  return mc ? launch13_kind<kKindRY, 1>(a, grid, shape, stream)
            : launch13_kind<kKindRY, 0>(a, grid, shape, stream);
}

}  // namespace dtc
