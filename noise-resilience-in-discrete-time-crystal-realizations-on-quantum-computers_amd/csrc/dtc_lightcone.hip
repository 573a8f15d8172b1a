// dtc_lightcone.hip -- the light-cone ends of the echo chains (kShapeLC):
// measure-only passes that replace an echo chain's last two to five passes
// (dtc_engine.cpp lc_merge / lc_merge_wide; the echo end of
// autocorr-delta-a-single-qiskit-fast.py:140-147).  A separate translation
// unit from the streaming pass kernels (dtc_kernels.hip) so the two compile in
// parallel.
#include <cstdlib>
#include <type_traits>

#include "dtc_device.h"
#include "dtc_kernels.h"

// dtc_lcw2_final: workgroups per CU (its 38.7 KB of LDS allow four; four cap
// the kernel at 128 VGPRs, three at 168)
#ifndef DTC_LCW3_WPS
#if defined(DTC_LCW3_ADD) || defined(DTC_LCW3_MERGE)
#define DTC_LCW3_WPS 3  // 41.2 KB of LDS with the padded additive slots, 49.7 with whole tables
#else
#define DTC_LCW3_WPS 4
#endif
#endif
#ifndef DTC_LCW2_WPS
#define DTC_LCW2_WPS 4
#endif

namespace dtc {

static constexpr int kLcTilesPerGroup = 2;

// ---- the light-cone end of an echo chain (kShapeLC) ------------------------
// The chain ends with <Z_j>.  Going backward from the measurement, the last
// kick layer matters only on j, the one before on j-1..j+1, the r-th from the
// end on j-r..j+r (kicks are unitary and D is diagonal with nearest-neighbour
// terms), so the chain's last few passes collapse into one measure-only pass
// over tiles that hold the window w0..w0+7 (tile bits 4..11; bits 0..3 =
// sites 0..3 as columns, c = 4): layer l = 0 .. lc_layers-1 kicks the window
// sites its mask keeps -- nibble 2 then 1 for even l, 1 then 2 for odd l, one
// LDS re-layout between them -- with the cone diagonal (conjugated: echo)
// between consecutive layers; then the probe.  Kicks in Pauli-frame form
// (dtc_kernels.h): one butterfly variant; a site of a layer runs only when the
// layer's mask kicks it (scalar branches on the kernel argument).
// A workgroup takes TPB consecutive tiles of one state: the records and tables
// are staged once, and the next tile's 16 loads are issued before the current
// tile's layers (register double buffer: the pass is VALU/LDS-heavy per byte).
template <int KIND, int TPB, bool SPLIT = false>
__device__ __forceinline__ void lc_body(const PassArgs& A) {
  static_assert(KIND == kKindRX || KIND == kKindRY, "light-cone pass: factored kicks");
  __shared__ double2 s_tile[SPLIT ? 1 : kTile];
  __shared__ double s_half[SPLIT ? kHalfSlots : 1];
  __shared__ double2 s_cone[kLcTab4];
  __shared__ double s_red[kThreads / 64][2];
  const int t = threadIdx.x;
  const int c = A.c, s = A.s;  // c = 4, s = w0
  const int64_t n_tiles = (int64_t)1 << (A.L_eff - kTileBits);
  const int og = A.octet_bits;  // state layout, as pass_body
  const int64_t b = og ? (((int64_t)blockIdx.y << 3) | (blockIdx.x & 7)) : (int64_t)blockIdx.y;
  const int64_t tile0 = (og ? (int64_t)(blockIdx.x >> 3) : (int64_t)blockIdx.x) * TPB;
  if (og && b >= A.batch) return;
  const int inst = (int)((A.batch_start + b) / A.n_traj);
  // the state's records through the scalar data cache (RecScalar): these
  // ends are VALU-bound, a v_readlane pair per coefficient is an issue slot
  const RecScalar R(A.recs + b * kRecPerState);
  const int64_t mid_mask = ((int64_t)1 << A.tile_bits_mid) - 1;
  TileMap M;
  M.c = c;
  M.s = s;
  M.cmask = (1 << c) - 1;
  auto tbase_of = [&](int64_t tile) {
    return ((tile & mid_mask) << c) | ((tile >> A.tile_bits_mid) << (s + kTileBits - c));
  };
  M.tbase = tbase_of(tile0);
  constexpr int kConePerThread = (kLcTab4 + kThreads - 1) / kThreads;
  double2 cv[kConePerThread];
  const double2* ct = A.lc_diag + (int64_t)inst * kLcTab;
#pragma unroll
  for (int j = 0; j < kConePerThread; ++j) {
    const int i = t + j * kThreads;
    if (i < kLcTab4) cv[j] = ct[i];
  }
  // the tile in layout 2 (threads = tile bits 0..7: 16-amplitude runs)
  // (layout 2: lanes = tile bits 0..3 (columns) and window sites 0..3; a
  // 64-bit lane offset: the window may sit high in a large state)
  const int64_t vofs = octet_spread(M.rel(ybase<2>(t)), og) << 4;
  const char* src = (const char*)(A.src + state_base(b, A.state_len, og));
  auto load_tile = [&](double2 (&dst)[kRegs], int64_t tb) {
#pragma unroll
    for (int r = 0; r < kRegs; ++r) {
      const char* a = src + (octet_spread(tb | M.rel(r << 8), og) << 4) + vofs;
      const d2v w = __builtin_nontemporal_load((const d2v*)a);
      dst[r] = make_double2(w.x, w.y);
    }
  };
  double2 v[kRegs];
  load_tile(v, M.tbase);
  __builtin_amdgcn_s_waitcnt(0x4F70);  // records and tables landed, the tile's 16 loads in flight
  const double cs = A.diag_conj ? -1.0 : 1.0;
#pragma unroll
  for (int j = 0; j < kConePerThread; ++j) {
    const int i = t + j * kThreads;
    if (i < kLcTab4) s_cone[i] = make_double2(cv[j].x, cs * cv[j].y);
  }
  // (visible after the first re-layout's barrier)
  const double g2 = R.d(0, kLcG2);
  const long long packed = R.bits(kLcPacked);
  const int nl = A.lc_layers;
  const int jp = A.probe;

  // kicks of nibble N (window sites 4 (N-1) .. 4 (N-1) + 3) in layer l
  auto kick = [&](double2 (&v)[kRegs], auto n_tag, auto l_tag) {
    constexpr int N = decltype(n_tag)::value;
    constexpr int l = decltype(l_tag)::value;
    constexpr int k0 = kLcSites * l + 4 * (N - 1);
    // per site: the cone leaves most layers' nibbles partly idle (the last
    // layer kicks j alone), and an idle site's f = 0 butterfly is the
    // identity; the mask is a kernel argument, so these are scalar branches
    const int m = (int)((A.lc_mask >> k0) & 0xFull);
    if (m & 1) layer_f<KIND, 0, 0>(v, R.d(0, k0));
    if (m & 2) layer_f<KIND, 0, 1>(v, R.d(0, k0 + 1));
    if (m & 4) layer_f<KIND, 0, 2>(v, R.d(0, k0 + 2));
    if (m & 8) layer_f<KIND, 0, 3>(v, R.d(0, k0 + 3));
  };
  // cone diagonal after layer l, applied in layout LAY: D_r(x ^ m_l), one
  // table lookup and one complex product per amplitude
  auto diag = [&](double2 (&v)[kRegs], auto lay_tag, int l) {
    constexpr int LAY = decltype(lay_tag)::value;
    const int rad = nl - 1 - l;
    const int lo = max(0, jp - rad), hi = min(A.L_real - 1, jp + rad);
    const int msk = (1 << (hi - lo + 1)) - 1;
    const int g0 = s + 4 * LAY - c;  // global bit of register bit 0
    const int64_t m = (int64_t)((packed >> (8 * l)) & 0xFF) << s;
    const int base = (int)(((M.at(ybase<LAY>(t)) ^ m) >> lo) & msk);
    const double2* tab = s_cone + lc_tab_off(rad);
#pragma unroll
    for (int r = 0; r < kRegs; ++r) {
      const int off = (g0 >= lo ? (r << (g0 - lo)) : (r >> (lo - g0))) & msk;
      const int i = base ^ off;
      v[r] = cmul(v[r], tab[rad == 4 ? lc_pos4(i) : i]);  // (the radius-4 table's storage)
    }
  };
  using L1 = std::integral_constant<int, 1>;
  using L2 = std::integral_constant<int, 2>;
  auto lc_xch_impl = [&](double2 (&v)[kRegs], auto from_tag, auto to_tag) {
    constexpr int F = decltype(from_tag)::value, T = decltype(to_tag)::value;
    if constexpr (SPLIT) exchange_split<F, T>(v, s_half, t);
    else exchange<F, T>(v, s_tile, t);
  };
  // one tile, its amplitudes in v (layout 2)
  auto process = [&](double2 (&v)[kRegs], int64_t tile) {
    M.tbase = tbase_of(tile);
    // layer 0: nibble 2 (layout 2), re-layout, nibble 1 (layout 1), D
    kick(v, L2{}, std::integral_constant<int, 0>{});
    lc_xch_impl(v, std::integral_constant<int, 2>{}, std::integral_constant<int, 1>{});
    kick(v, L1{}, std::integral_constant<int, 0>{});
    if (nl > 1) {  // layer 1: 1 -> 2
      diag(v, L1{}, 0);
      kick(v, L1{}, std::integral_constant<int, 1>{});
      lc_xch_impl(v, std::integral_constant<int, 1>{}, std::integral_constant<int, 2>{});
      kick(v, L2{}, std::integral_constant<int, 1>{});
    }
    if (nl > 2) {  // layer 2: 2 -> 1
      diag(v, L2{}, 1);
      kick(v, L2{}, std::integral_constant<int, 2>{});
      lc_xch_impl(v, std::integral_constant<int, 2>{}, std::integral_constant<int, 1>{});
      kick(v, L1{}, std::integral_constant<int, 2>{});
    }
    if (nl > 3) {  // layer 3: 1 -> 2
      diag(v, L1{}, 2);
      kick(v, L1{}, std::integral_constant<int, 3>{});
      lc_xch_impl(v, std::integral_constant<int, 1>{}, std::integral_constant<int, 2>{});
      kick(v, L2{}, std::integral_constant<int, 3>{});
    }
    if (nl > 4) {  // layer 4: 2 -> 1
      diag(v, L2{}, 3);
      kick(v, L2{}, std::integral_constant<int, 4>{});
      lc_xch_impl(v, std::integral_constant<int, 2>{}, std::integral_constant<int, 1>{});
      kick(v, L1{}, std::integral_constant<int, 4>{});
    }
    // probe: layout 1 after an odd number of layers, 2 after an even number;
    // the frame's X on j flips it
    const int lay = (nl & 1) ? 1 : 2;
    double ptot = 0.0, pz = 0.0;
    {
      const int64_t x0 = lay == 1 ? M.at(ybase<1>(t)) : M.at(ybase<2>(t));
      const int tb = jp < c ? jp : ((jp >= s && jp < s + kTileBits - c) ? c + jp - s : -1);
      const int jr = tb - 4 * lay;  // register bit of the probe, if in the nibble in registers
#pragma unroll
      for (int r = 0; r < kRegs; ++r) {
        const double p2 = fma(v[r].x, v[r].x, v[r].y * v[r].y);
        ptot += p2;
        pz += (jr >= 0 && jr < 4 && ((r >> jr) & 1)) ? -p2 : p2;
      }
      if (!(jr >= 0 && jr < 4)) pz = ((x0 >> jp) & 1) ? -ptot : ptot;
      if ((packed >> (32 + jp - s)) & 1) pz = -pz;
    }
    const int wave = t >> 6, lane = t & 63;
    const double tot = wave_sum(ptot) * g2;
    const double z = wave_sum(pz) * g2;
    if (lane == 0) {
      s_red[wave][0] = tot;
      s_red[wave][1] = z;
    }
    __syncthreads();
    if (t < 2) {
      double acc = 0.0;
      for (int k = 0; k < kThreads / 64; ++k) acc += s_red[k][t];
      A.partial[(b * n_tiles + tile) * A.n_obs + t] = acc;
    }
  };
  // two register buffers, no copies: the loads of tile i+1 fly while tile i runs
  static_assert(TPB == 1 || TPB == 2 || TPB == 4, "tiles per workgroup");
  if constexpr (TPB == 1) {
    process(v, tile0);
  } else {
    double2 w[kRegs];
    load_tile(w, tbase_of(tile0 + 1));
    process(v, tile0);
    if constexpr (TPB == 4) {
      load_tile(v, tbase_of(tile0 + 2));
      process(w, tile0 + 1);
      load_tile(w, tbase_of(tile0 + 3));
      process(v, tile0 + 2);
      process(w, tile0 + 3);
    } else {
      process(w, tile0 + 1);
    }
  }
}

template <int KIND, int TPB>
__global__ __launch_bounds__(kThreads, 2) void dtc_lc_final(PassArgs A) {
  lc_body<KIND, TPB>(A);
}
// One tile per workgroup, re-layouts through half the LDS: three per CU (the
// pass is bound by its per-workgroup chain, so a third chain per CU pays more
// than the two extra barriers per re-layout cost; the default)
template <int KIND>
__global__ __launch_bounds__(kThreads, 3) void dtc_lc_final_split(PassArgs A) {
  lc_body<KIND, 1, true>(A);
}

// ---- the 10-site light-cone end (kShapeLC, lc_wide) ------------------------
// The chain's last five passes as six kick layers (r = 5 .. 0 diagonals before
// the probe) on a 10-site window (dtc_kernels.h, kLcw*).  Tile bits 0, 1 =
// global bits 0, 1 (64-B runs), tile bit k >= 2 = site lc_gb[k]: nibble 1 =
// j-2 .. j+1 (the cone of r <= 1), nibble 2 = j+2, j+3, j-4, j-3 (with nibble
// 1, r <= 3), nibble 0 = the columns and the two outer sites.  Program (the
// nibble in registers; the host checks every layer's sites against it):
//   r=5: 2 1 0 | D5 | r=4: 0 2 1 | D4 | r=3: 1 2 | D3 | r=2: 2 1 | D2 |
//   r=1: 1 | D1 | r=0: 1 | probe (j = tile bit 6 = register bit 2)
// — six re-layouts through the 32 KiB half-tile buffer for five passes (the
// 8-site pass: five for four), three workgroups per CU.  D5 is two lookups
// in the split radius-5 tables.  Global indices fit 32 bits (L_eff <= 32).
// MASK: the layers' kick mask when known at compile time (0: read A.lc_mask).
// The chains of the C2 sweep (two site groups split at j+2, the first merged
// pass on j's group) all have kLcwMaskJ2 (lc_merge_wide): its instantiation
// runs exactly the 32 kicked sites with no per-site branches, so the compiler
// keeps the butterflies' results in renamed registers instead of copying them
// back for the branch merges.
static constexpr uint64_t kLcwMaskJ2 =
    // l = 0: tile bits 2, 4..7, 10, 11 (sites j-5, j-2..j+1, j-4, j-3)
    (0x33Dull) |
    // l = 1: tile bits 3..11 (j+4, j-2..j+3, j-4, j-3)
    (0x3FEull << 10) |
    // l = 2: tile bits 4..9, 11 (j-2..j+3, j-3)
    (0x2FCull << 20) |
    // l = 3: tile bits 4..8 (j-2..j+2)
    (0x07Cull << 30) |
    // l = 4: tile bits 5..7 (j-1..j+1)
    (0x038ull << 40) |
    // l = 5: tile bit 6 (j)
    (0x010ull << 50);

template <int KIND, uint64_t MASK = 0>
__global__ __launch_bounds__(kThreads, 3) void dtc_lcw_final(PassArgs A) {
  static_assert(KIND == kKindRX || KIND == kKindRY, "light-cone pass: factored kicks");
  __shared__ double s_half[kHalfSlots];
  __shared__ double2 s_cone[kLcTab5b + 64];  // the r = 1 .. 4 and 5a / 5b tables
  __shared__ double s_red[kThreads / 64][2];
  const int t = threadIdx.x;
  const int64_t n_tiles = (int64_t)1 << (A.L_eff - kTileBits);
  const int og = A.octet_bits;
  const int64_t b = og ? (((int64_t)blockIdx.y << 3) | (blockIdx.x & 7)) : (int64_t)blockIdx.y;
  const int64_t tile = og ? (int64_t)(blockIdx.x >> 3) : (int64_t)blockIdx.x;
  if (og && b >= A.batch) return;
  const int inst = (int)((A.batch_start + b) / A.n_traj);
  // the state's records through the scalar data cache (RecScalar): these
  // ends are VALU-bound, a v_readlane pair per coefficient is an issue slot
  const RecScalar R(A.recs + b * kRecPerState);
  constexpr int kConePerThread = (kLcTab5b + 64 + kThreads - 1) / kThreads;
  double2 cv[kConePerThread];
  const double2* ct = A.lc_diag + (int64_t)inst * kLcTab;
#pragma unroll
  for (int j = 0; j < kConePerThread; ++j) {
    const int i = t + j * kThreads;
    if (i < kLcTab5b + 64) cv[j] = ct[i];
  }
  // tile bit -> global bit (wave-uniform), the window, the tile's base: the
  // tile id's bits deposited, in order, into the global bits off the window
  uint32_t gbit[kTileBits];
  uint32_t win = 0;
#pragma unroll
  for (int k = 0; k < kTileBits; ++k) {
    gbit[k] = 1u << A.lc_gb[k];
    win |= gbit[k];
  }
  uint32_t tbase = 0;
  {
    uint32_t rest = (uint32_t)tile;
    for (int g = 0; g < A.L_eff; ++g) {
      if ((win >> g) & 1u) continue;
      tbase |= (rest & 1u) << g;
      rest >>= 1;
    }
  }
  // the thread's part of the global index in layout LAY (register bits zero)
  auto lane_part = [&](auto lay_tag) -> uint32_t {
    constexpr int LAY = decltype(lay_tag)::value;
    const int y = ybase<LAY>(t);
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < kTileBits; ++k)
      if (k < 4 * LAY || k >= 4 * LAY + 4) x |= ((y >> k) & 1) ? gbit[k] : 0u;
    return x;
  };
  using L0 = std::integral_constant<int, 0>;
  using L1 = std::integral_constant<int, 1>;
  using L2 = std::integral_constant<int, 2>;
  // register r's part in layout LAY (uniform)
  auto reg_part = [&](auto lay_tag, int r) -> uint32_t {
    constexpr int LAY = decltype(lay_tag)::value;
    return ((r & 1) ? gbit[4 * LAY] : 0u) | ((r & 2) ? gbit[4 * LAY + 1] : 0u) |
           ((r & 4) ? gbit[4 * LAY + 2] : 0u) | ((r & 8) ? gbit[4 * LAY + 3] : 0u);
  };
  // the tile in layout 2 (threads = tile bits 0 .. 7: the columns in lane bits 0, 1)
  double2 v[kRegs];
  {
    const int64_t vofs = octet_spread((int64_t)lane_part(L2{}), og) << 4;
    const char* src = (const char*)(A.src + state_base(b, A.state_len, og));
#pragma unroll
    for (int r = 0; r < kRegs; ++r) {
      const char* a = src + (octet_spread((int64_t)(tbase | reg_part(L2{}, r)), og) << 4) + vofs;
      const d2v w = *(const d2v*)a;  // ordinary load: 64-B runs (note above dtc_lcw2_final)
      v[r] = make_double2(w.x, w.y);
    }
  }
  __builtin_amdgcn_s_waitcnt(0x4F70);  // records and tables landed, the tile's 16 loads in flight
  const double cs = A.diag_conj ? -1.0 : 1.0;
#pragma unroll
  for (int j = 0; j < kConePerThread; ++j) {
    const int i = t + j * kThreads;
    if (i < kLcTab5b + 64) s_cone[i] = make_double2(cv[j].x, cs * cv[j].y);
  }
  // (visible after the first re-layout's barrier)
  const int jp = A.probe;
  const int Lr = A.L_real;

  // kicks of layer l on the kicked sites of nibble N (in registers)
  auto kick = [&](auto n_tag, auto l_tag) {
    constexpr int N = decltype(n_tag)::value;
    constexpr int l = decltype(l_tag)::value;
    if constexpr (MASK != 0) {
      constexpr uint32_t m = (uint32_t)(MASK >> (10 * l));
      if constexpr (4 * N + 0 >= 2 && ((m >> (4 * N + 0 - 2)) & 1u))
        layer_f<KIND, 0, 0>(v, R.d(0, 12 * l + 4 * N + 0));
      if constexpr (4 * N + 1 >= 2 && ((m >> (4 * N + 1 - 2)) & 1u))
        layer_f<KIND, 0, 1>(v, R.d(0, 12 * l + 4 * N + 1));
      if constexpr ((m >> (4 * N + 2 - 2)) & 1u) layer_f<KIND, 0, 2>(v, R.d(0, 12 * l + 4 * N + 2));
      if constexpr ((m >> (4 * N + 3 - 2)) & 1u) layer_f<KIND, 0, 3>(v, R.d(0, 12 * l + 4 * N + 3));
    } else {
      const uint32_t m = (uint32_t)(A.lc_mask >> (10 * l));
      if constexpr (4 * N + 0 >= 2)
        if ((m >> (4 * N + 0 - 2)) & 1u) layer_f<KIND, 0, 0>(v, R.d(0, 12 * l + 4 * N + 0));
      if constexpr (4 * N + 1 >= 2)
        if ((m >> (4 * N + 1 - 2)) & 1u) layer_f<KIND, 0, 1>(v, R.d(0, 12 * l + 4 * N + 1));
      if ((m >> (4 * N + 2 - 2)) & 1u) layer_f<KIND, 0, 2>(v, R.d(0, 12 * l + 4 * N + 2));
      if ((m >> (4 * N + 3 - 2)) & 1u) layer_f<KIND, 0, 3>(v, R.d(0, 12 * l + 4 * N + 3));
    }
  };
  // one cone-table factor in layout LAY: tab[((x ^ m) >> lo) & msk] per amplitude
  // sw: the table's storage swizzle (0 none, 4 lc_pos4, 5 lc_pos5a), applied to
  // the thread's base and the register offsets once (linear)
  auto diag_tab = [&](auto lay_tag, uint32_t xm, int lo, int hi, const double2* tab, auto sw_tag) {
    constexpr int LAY = decltype(lay_tag)::value;
    constexpr int SW = decltype(sw_tag)::value;
    auto pos = [](int i) { return SW == 4 ? lc_pos4(i) : (SW == 5 ? lc_pos5a(i) : i); };
    const uint32_t msk = (1u << (hi - lo + 1)) - 1u;
    const int base = pos((int)((xm >> lo) & msk));
    const int o0 = pos((int)((gbit[4 * LAY] >> lo) & msk)), o1 = pos((int)((gbit[4 * LAY + 1] >> lo) & msk));
    const int o2 = pos((int)((gbit[4 * LAY + 2] >> lo) & msk)), o3 = pos((int)((gbit[4 * LAY + 3] >> lo) & msk));
#pragma unroll
    for (int r = 0; r < kRegs; ++r) {
      const int off = ((r & 1) ? o0 : 0) ^ ((r & 2) ? o1 : 0) ^ ((r & 4) ? o2 : 0) ^ ((r & 8) ? o3 : 0);
      v[r] = cmul(v[r], tab[base ^ off]);
    }
  };
  // the cone diagonal after layer l (r = 5 - l), frame X mask m_l
  auto diag = [&](auto lay_tag, auto l_tag) {
    constexpr int l = decltype(l_tag)::value;
    constexpr int rad = kLcwLayers - 1 - l;
    const uint32_t xm = (tbase | lane_part(lay_tag)) ^ (uint32_t)R.bits(kLcwMask + l);
    using S0 = std::integral_constant<int, 0>;
    if constexpr (rad == 5) {
      diag_tab(lay_tag, xm, max(0, jp - 5), jp, s_cone + kLcTab5a, std::integral_constant<int, 5>{});
      diag_tab(lay_tag, xm, jp, min(Lr - 1, jp + 5), s_cone + kLcTab5b, S0{});
    } else if constexpr (rad == 4) {
      diag_tab(lay_tag, xm, max(0, jp - 4), min(Lr - 1, jp + 4), s_cone + lc_tab_off(4),
               std::integral_constant<int, 4>{});
    } else {
      diag_tab(lay_tag, xm, max(0, jp - rad), min(Lr - 1, jp + rad), s_cone + lc_tab_off(rad), S0{});
    }
  };
  using C0 = std::integral_constant<int, 0>;
  using C1 = std::integral_constant<int, 1>;
  using C2 = std::integral_constant<int, 2>;
  using C3 = std::integral_constant<int, 3>;
  using C4 = std::integral_constant<int, 4>;
  using C5 = std::integral_constant<int, 5>;
  // r = 5: nibbles 2, 1, 0
  kick(L2{}, C0{});
  exchange_split<2, 1>(v, s_half, t);
  kick(L1{}, C0{});
  exchange_split<1, 0>(v, s_half, t);
  kick(L0{}, C0{});
  diag(L0{}, C0{});
  // r = 4: nibbles 0, 2, 1
  kick(L0{}, C1{});
  exchange_split<0, 2>(v, s_half, t);
  kick(L2{}, C1{});
  exchange_split<2, 1>(v, s_half, t);
  kick(L1{}, C1{});
  diag(L1{}, C1{});
  // r = 3: nibbles 1, 2
  kick(L1{}, C2{});
  exchange_split<1, 2>(v, s_half, t);
  kick(L2{}, C2{});
  diag(L2{}, C2{});
  // r = 2: nibbles 2, 1
  kick(L2{}, C3{});
  exchange_split<2, 1>(v, s_half, t);
  kick(L1{}, C3{});
  diag(L1{}, C3{});
  // r = 1, r = 0: nibble 1
  kick(L1{}, C4{});
  diag(L1{}, C4{});
  kick(L1{}, C5{});
  // probe: j at register bit 2 of layout 1; the frame's final X on j flips it
  double ptot = 0.0, pz = 0.0;
#pragma unroll
  for (int r = 0; r < kRegs; ++r) {
    const double p2 = fma(v[r].x, v[r].x, v[r].y * v[r].y);
    ptot += p2;
    pz += ((r >> 2) & 1) ? -p2 : p2;
  }
  if ((R.bits(kLcwMask + kLcwLayers - 1) >> jp) & 1) pz = -pz;
  const double g2 = R.d(0, kLcwG2);
  const int wave = t >> 6, lane = t & 63;
  const double tot = wave_sum(ptot) * g2;
  const double z = wave_sum(pz) * g2;
  if (lane == 0) {
    s_red[wave][0] = tot;
    s_red[wave][1] = z;
  }
  __syncthreads();
  if (t < 2) {
    double acc = 0.0;
    for (int k = 0; k < kThreads / 64; ++k) acc += s_red[k][t];
    A.partial[(b * n_tiles + tile) * A.n_obs + t] = acc;
  }
}

// Tile loads of the 10-site passes (dtc_lcw_final, dtc_lcw2_final) are
// ordinary, not nontemporal: their tiles read 64-B runs (global bits 0, 1),
// so each 128-B line's other half belongs to the partner tile (global bit 2,
// the next block on the same XCD).  With the nontemporal hint L2 does not keep
// the line for it and HBM serves it twice: tools/run64_bench.hip (r4g) reads
// that pattern at 4.45-4.67 TB/s, FETCH_SIZE x2 = 1.38 x the bytes, against
// 5.68-5.91 TB/s and x1.02 with ordinary loads; the pass's own PMC went
// x1.44 -> x1.0001 and its time 5.61 -> 5.43 ms (same box).  Runs of 128 B
// and more keep the nontemporal hint (no partner: x1.000 either way, and
// faster: 256-B runs 6.96 vs 6.59 TB/s).

// ---- the 10-site light-cone end, C2 form (dtc_lcw2_final) ------------------
// The same six layers on the same window as dtc_lcw_final (kLcwMaskJ2, the
// canonical lc_gb of lc_merge_wide, 7 <= j <= L-6: no cone clipped), with the
// tile re-laid-out three times instead of six.  Between two LDS re-layouts a
// site enters the registers by a gfx950 row swap: v_permlane16_swap /
// v_permlane32_swap of a register pair exchanges register bit q with lane bit
// 4 / 5 (32 VALU ops for the tile, no LDS, no barrier), so each layout has six
// "near" sites (four register bits, lane bits 4 and 5).  Program (sites by
// offset from j; c0, c1 = global bits 0, 1):
//   L0  regs -2 -1  0 +1 | l0: -2 -1 0 +1                       (load layout)
//   L1  regs -5 -4 -3 +4 | l0: -5 -4 -3 | D5 | l1: -4 -3 +4
//   L2  regs -2 -1  0 +1 | l1: -2 -1 0 +1, swap +2 +3 in, l1: +2 +3 | D4 |
//                          l2: +2 +3 0 +1
//   L3  regs -3 -2 -1  0 | l2: -3 -2 -1 | D3 | l3: -2 -1 0, swap +1 in, +1,
//                          swap +2 in, +2 | D2 | l4: -1 0 +1 | D1 | l5: 0 | probe
// Re-layout slots are additive in the sites' bits (lcw2::kW): a slot is the
// thread's base plus a compile-time register offset, i.e. the ds_write_b64 /
// ds_read_b64 immediate, no address VALU per access; the weights' 2-adic
// valuations make every write (lane bits 0..3) and read (lane bits 0..4) of the
// layouts used conflict-free.  The cone tables are staged with the layer's
// Pauli-frame X mask applied (T'[i] = T[i ^ m]) and their index bits permuted
// so the lane-varying sites hit distinct banks: a lookup is likewise a base
// plus an immediate.  D5 and D4 are two 6- / 5-bit tables each (10 and 18
// lookups), D1 has 8 distinct entries: 68 lookups instead of 112, and 38.6 KB
// of LDS (four workgroups per CU under a 128-VGPR cap).
namespace lcw2 {
enum : int { c0 = 0, c1, m5, m4, m3, m2, m1, z0, p1, p2, p3, p4, p5, kNSite };
// offset from j of each window site (c0, c1: not in any cone)
__host__ __device__ constexpr int off_of(int s) { return s == c0 || s == c1 ? -99 : s - z0; }
// the record index (tile bit of lc_merge_wide's lc_gb order) of each site
__host__ __device__ constexpr int rec_of(int s) {
  return s == c0 ? 0 : s == c1 ? 1 : s == m5 ? 2 : s == p4 ? 3 : s == m2 ? 4 : s == m1 ? 5
       : s == z0 ? 6 : s == p1 ? 7 : s == p2 ? 8 : s == p3 ? 9 : s == m4 ? 10 : 11;
}
// re-layout slot weights (8-B slots; slot = sum of the set sites' weights):
// valuations c0 0, c1 1, m5 / m2 2, m4 / m1 3, p2 4 -- injective over the
// 4096 tile indices, max slot 4107 (tools/lcw2_design.py checks both)
__host__ __device__ constexpr int wt(int s) {
  return s == c0 ? 1 : s == c1 ? 2 : s == m5 ? 4 : s == m4 ? 8 : s == p2 ? 16 : s == m3 ? 32
       : s == z0 ? 64 : s == p1 ? 128 : s == p3 ? 256 : s == p4 ? 512 : s == m2 ? 1028 : 2056;
}
static constexpr int kSlots = 4108;
// layouts: positions 0..3 registers, 4..9 lane bits 0..5, 10..11 wave bits
enum : int { kL0 = 0, kL1, kL2s, kL2e, kL3s, kL3e };
__host__ __device__ constexpr int lay_site(int li, int pos) {
  constexpr int tab[6][12] = {
      {m2, m1, z0, p1, c0, c1, m5, m4, m3, p4, p2, p3},   // L0
      {m5, m4, m3, p4, c0, c1, m2, m1, p2, z0, p1, p3},   // L1
      {m2, m1, z0, p1, c0, c1, m5, m4, p2, p3, m3, p4},   // L2s
      {p2, p3, z0, p1, c0, c1, m5, m4, m2, m1, m3, p4},   // L2e (L2s after two swaps)
      {m3, m2, m1, z0, c0, c1, m5, m4, p2, p1, p3, p4},   // L3s
      {p1, p2, m1, z0, c0, c1, m5, m4, m2, m3, p3, p4}};  // L3e (L3s after two swaps)
  return tab[li][pos];
}
// register part of a slot: the weights of register r's set bits
__host__ __device__ constexpr int reg_slot(int li, int r) {
  return ((r & 1) ? wt(lay_site(li, 0)) : 0) + ((r & 2) ? wt(lay_site(li, 1)) : 0) +
         ((r & 4) ? wt(lay_site(li, 2)) : 0) + ((r & 8) ? wt(lay_site(li, 3)) : 0);
}
template <int LI>
__device__ __forceinline__ int slot_base(int t) {
  int b = 0;
#pragma unroll
  for (int p = 4; p < 12; ++p) b += ((t >> (p - 4)) & 1) * wt(lay_site(LI, p));
  return b;
}
// cone tables in LDS (double2 entries): [offset, bits, first site] and each
// index bit's position bit (lane-varying sites low: conflict-free lookups)
enum : int { kT5a = 0, kT5b, kT4a, kT4b, kT3, kT2, kT1, kNTab };
__host__ __device__ constexpr int tab_off(int k) {
  return k == kT5a ? 0 : k == kT5b ? 64 : k == kT4a ? 128 : k == kT4b ? 160 : k == kT3 ? 192
       : k == kT2 ? 320 : 352;
}
static constexpr int kTabEntries = 360;
__host__ __device__ constexpr int tab_bits(int k) {
  return k == kT5a || k == kT5b ? 6 : k == kT4a || k == kT4b ? 5 : k == kT3 ? 7 : k == kT2 ? 5 : 3;
}
__host__ __device__ constexpr int tab_lo(int k) {  // offset from j of index bit 0
  return k == kT5a ? -5 : k == kT5b ? 0 : k == kT4a ? -4 : k == kT4b ? 0 : k == kT3 ? -3
       : k == kT2 ? -2 : -1;
}
// position bit of index bit i (5a: -2 -1 0 first; 3: +1 +2 first; others natural)
__host__ __device__ constexpr int pos_bit(int k, int i) {
  return k == kT5a ? (i < 3 ? i + 3 : i - 3) : k == kT3 ? (i < 4 ? i + 2 : (i < 6 ? i - 4 : 6)) : i;
}
__host__ __device__ constexpr int pos_of(int k, int idx) {
  int p = 0;
  for (int i = 0; i < tab_bits(k); ++i) p |= ((idx >> i) & 1) << pos_bit(k, i);
  return p;
}
// position weight of site s in table k (0: not an index bit)
__host__ __device__ constexpr int tab_wt(int k, int s) {
  const int d = off_of(s) - tab_lo(k);
  return (s == c0 || s == c1 || d < 0 || d >= tab_bits(k)) ? 0 : 1 << pos_bit(k, d);
}
// the table's layer (frame mask after it) and its source in the instance's
// global cone table set (kLcTab layout; the j-5 .. j table stored lc_pos5a)
__host__ __device__ constexpr int tab_layer(int k) {
  return k == kT5a || k == kT5b ? 0 : k == kT4a || k == kT4b ? 1 : k == kT3 ? 2 : k == kT2 ? 3 : 4;
}
__host__ __device__ constexpr int tab_src(int k) {
  return k == kT5a ? kLcTab5a : k == kT5b ? kLcTab5b : k == kT4a ? kLcTab4a : k == kT4b ? kLcTab4b
       : lc_tab_off(k == kT3 ? 3 : k == kT2 ? 2 : 1);
}
template <int LI, int K>
__device__ __forceinline__ int tab_reg(int r) {
  return ((r & 1) ? tab_wt(K, lay_site(LI, 0)) : 0) + ((r & 2) ? tab_wt(K, lay_site(LI, 1)) : 0) +
         ((r & 4) ? tab_wt(K, lay_site(LI, 2)) : 0) + ((r & 8) ? tab_wt(K, lay_site(LI, 3)) : 0);
}
// a thread's table base: its lane / wave sites in the table, plus the tile's
// bit j+5 (table 5b's last index bit, outside the window)
template <int LI, int K>
__device__ __forceinline__ int tab_base(int t, int bit_p5) {
  int b = 0;
#pragma unroll
  for (int p = 4; p < 12; ++p) b += ((t >> (p - 4)) & 1) * tab_wt(K, lay_site(LI, p));
  return b + (K == kT5b ? bit_p5 * tab_wt(K, p5) : 0);
}
}  // namespace lcw2

template <int KIND>
__global__ __launch_bounds__(kThreads, DTC_LCW2_WPS) void dtc_lcw2_final(PassArgs A) {
  static_assert(KIND == kKindRX || KIND == kKindRY, "light-cone pass: factored kicks");
  using namespace lcw2;
  __shared__ double s_x[kSlots];
  __shared__ double2 s_tab[kTabEntries];
  __shared__ double s_red[kThreads / 64][2];
  const int t = threadIdx.x;
  const int64_t n_tiles = (int64_t)1 << (A.L_eff - kTileBits);
  const int og = A.octet_bits;
  const int64_t b = og ? (((int64_t)blockIdx.y << 3) | (blockIdx.x & 7)) : (int64_t)blockIdx.y;
  const int64_t tile = og ? (int64_t)(blockIdx.x >> 3) : (int64_t)blockIdx.x;
  if (og && b >= A.batch) return;
  const int inst = (int)((A.batch_start + b) / A.n_traj);
  const int j = A.probe;
  // the state's records through the scalar data cache (RecScalar): these
  // ends are VALU-bound, a v_readlane pair per coefficient is an issue slot
  const RecScalar R(A.recs + b * kRecPerState);
  // global bit of each window site; the tile's base (its id deposited into
  // the bits off the window, as lc_merge_wide's lc_gb)
  auto gpos = [&](int s) { return s == c0 ? 0 : (s == c1 ? 1 : j + off_of(s)); };
  // (the bits off the window are 2 .. j-6 and j+5 .. L_eff-1: two shifts)
  const uint32_t tbase = (((uint32_t)tile & ((1u << (j - 7)) - 1u)) << 2) |
                         (((uint32_t)tile >> (j - 7)) << (j + 5));
  const int bit_p5 = (int)((tbase >> (j + 5)) & 1u);  // table 5b's bit j+5
  double2 v[kRegs];  // the tile: 16 amplitudes per thread
  // re-layout through the 4108-slot half buffer (real parts, then imaginary)
  auto xch = [&](auto from_tag, auto to_tag) {
    constexpr int F = decltype(from_tag)::value, T = decltype(to_tag)::value;
    int bf = slot_base<F>(t), bt = slot_base<T>(t);
    asm volatile("" : "+v"(bf), "+v"(bt));
#pragma unroll
    for (int r = 0; r < kRegs; ++r) s_x[bf + reg_slot(F, r)] = v[r].x;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kRegs; ++r) v[r].x = s_x[bt + reg_slot(T, r)];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kRegs; ++r) s_x[bf + reg_slot(F, r)] = v[r].y;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kRegs; ++r) v[r].y = s_x[bt + reg_slot(T, r)];
  };
  // kick of site S (register bit Q) in layer l
  auto kick = [&](auto q_tag, auto l_tag, auto s_tag) {
    constexpr int Q = decltype(q_tag)::value, l = decltype(l_tag)::value, S = decltype(s_tag)::value;
    layer_f<KIND, 0, Q>(v, R.d(0, 12 * l + rec_of(S)));
  };
  // v[r] *= T_k[base + reg part]: 16 lookups (or the distinct ones)
  auto diag1 = [&](auto lay_tag, auto k_tag) {
    constexpr int LI = decltype(lay_tag)::value, K = decltype(k_tag)::value;
    int base = tab_base<LI, K>(t, bit_p5);
    asm volatile("" : "+v"(base));
    const double2* tab = s_tab + tab_off(K) + base;
#pragma unroll
    for (int r = 0; r < kRegs; ++r) v[r] = cmul(v[r], tab[tab_reg<LI, K>(r)]);  // (D1: 8 distinct)
  };
  using C0 = std::integral_constant<int, 0>;
  using C1 = std::integral_constant<int, 1>;
  using C2 = std::integral_constant<int, 2>;
  using C3 = std::integral_constant<int, 3>;
  using C4 = std::integral_constant<int, 4>;
  using C5 = std::integral_constant<int, 5>;
#define LCW2_SITE(s) std::integral_constant<int, s>{}
  // the tile in layout L0 (lane bits 0, 1 = global bits 0, 1: 64-B runs)
  {
    uint32_t xl = 0;
#pragma unroll
    for (int p = 4; p < 12; ++p) xl |= (uint32_t)((t >> (p - 4)) & 1) << gpos(lay_site(kL0, p));
    const int64_t vofs = octet_spread((int64_t)xl, og) << 4;
    const char* src = (const char*)(A.src + state_base(b, A.state_len, og));
    // register offsets: the spread is linear over disjoint bits, so one per
    // register bit, summed (uniform)
    const int64_t sp0 = octet_spread((int64_t)tbase, og) << 4;
    int64_t spq[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) spq[q] = octet_spread((int64_t)1 << gpos(lay_site(kL0, q)), og) << 4;
#pragma unroll
    for (int r = 0; r < kRegs; ++r) {
      int64_t o = sp0;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if ((r >> q) & 1) o += spq[q];
      const d2v w = *(const d2v*)(src + o + vofs);  // ordinary load (note above this section)
      v[r] = make_double2(w.x, w.y);
    }
  }
  // the cone tables' entries this thread stages (e = t, t + 256 of the 360):
  // loaded behind the tile: first used after the first re-layout
  const double2* ct = A.lc_diag + (int64_t)inst * kLcTab;
  auto tab_of = [](int e) {
    return e >= tab_off(kT1) ? kT1 : e >= tab_off(kT2) ? kT2 : e >= tab_off(kT3) ? kT3
         : e >= tab_off(kT4b) ? kT4b : e >= tab_off(kT4a) ? kT4a : e >= tab_off(kT5b) ? kT5b : kT5a;
  };
  auto tab_start = [](int k) {
    return k == kT5a ? tab_off(kT5a) : k == kT5b ? tab_off(kT5b) : k == kT4a ? tab_off(kT4a)
         : k == kT4b ? tab_off(kT4b) : k == kT3 ? tab_off(kT3) : k == kT2 ? tab_off(kT2) : tab_off(kT1);
  };
  auto src_of = [](int k) {
    return k == kT5a ? tab_src(kT5a) : k == kT5b ? tab_src(kT5b) : k == kT4a ? tab_src(kT4a)
         : k == kT4b ? tab_src(kT4b) : k == kT3 ? tab_src(kT3) : k == kT2 ? tab_src(kT2) : tab_src(kT1);
  };
  const int e1 = t + kThreads;
  const int k0 = tab_of(t), k1 = tab_of(e1);
  const int i0 = t - tab_start(k0), i1 = e1 - tab_start(k1);
  const double2 tv0 = ct[src_of(k0) + (k0 == kT5a ? lc_pos5a(i0) : i0)];
  double2 tv1 = make_double2(0.0, 0.0);
  if (e1 < kTabEntries) tv1 = ct[src_of(k1) + i1];
  // ---- L0: l0 on -2 -1 0 +1 (the staging below waits for the tables) ----
  kick(C0{}, C0{}, LCW2_SITE(m2));
  kick(C1{}, C0{}, LCW2_SITE(m1));
  kick(C2{}, C0{}, LCW2_SITE(z0));
  kick(C3{}, C0{}, LCW2_SITE(p1));
  // stage the tables: entry i of table k at pos(i ^ m_k), m_k the frame's X
  // mask after the table's layer on the table's bits; conjugated for D*
  {
    const double cs = A.diag_conj ? -1.0 : 1.0;
    const uint64_t m0 = (uint64_t)R.bits(kLcwMask + 0), m1 = (uint64_t)R.bits(kLcwMask + 1);
    const uint64_t m2 = (uint64_t)R.bits(kLcwMask + 2), m3 = (uint64_t)R.bits(kLcwMask + 3);
    const uint64_t m4 = (uint64_t)R.bits(kLcwMask + 4);
    auto stage = [&](int k, int i, double2 tv) {
      const int l = tab_layer(k);
      const uint64_t m = l == 0 ? m0 : l == 1 ? m1 : l == 2 ? m2 : l == 3 ? m3 : m4;
      const int lo = k == kT5a ? -5 : k == kT4a ? -4 : k == kT3 ? -3 : k == kT2 ? -2 : k == kT1 ? -1 : 0;
      const int nb = k == kT3 ? 7 : (k == kT5a || k == kT5b) ? 6 : k == kT1 ? 3 : 5;
      const int x = i ^ (int)((m >> (j + lo)) & ((1u << nb) - 1u));
      // the position bit permutations (pos_of): 5a rotates by 3, 3 puts bits 4, 5 first
      const int pos = k == kT5a ? (((x & 7) << 3) | (x >> 3))
                    : k == kT3 ? (((x & 15) << 2) | ((x >> 4) & 3) | (x & 64)) : x;
      s_tab[tab_start(k) + pos] = make_double2(tv.x, cs * tv.y);
    };
    stage(k0, i0, tv0);
    if (e1 < kTabEntries) stage(k1, i1, tv1);
  }
  // (visible after the first re-layout's barriers)

  xch(std::integral_constant<int, kL0>{}, std::integral_constant<int, kL1>{});
  // ---- L1: l0 on -5 -4 -3, D5, l1 on -4 -3 +4 ----
  kick(C0{}, C0{}, LCW2_SITE(m5));
  kick(C1{}, C0{}, LCW2_SITE(m4));
  kick(C2{}, C0{}, LCW2_SITE(m3));
  {  // D5 = T5a(-5 .. 0) T5b(0 .. +5): registers -5 -4 -3 in 5a, +4 in 5b
    int ba = tab_base<kL1, kT5a>(t, bit_p5), bb = tab_base<kL1, kT5b>(t, bit_p5);
    asm volatile("" : "+v"(ba), "+v"(bb));
    const double2* ta = s_tab + tab_off(kT5a) + ba;
    const double2* tb = s_tab + tab_off(kT5b) + bb;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const double2 f = ta[tab_reg<kL1, kT5a>(r)];
      v[r] = cmul(v[r], f);
      v[r + 8] = cmul(v[r + 8], f);
    }
    const double2 f0 = tb[0], f1 = tb[tab_reg<kL1, kT5b>(8)];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      v[r] = cmul(v[r], f0);
      v[r + 8] = cmul(v[r + 8], f1);
    }
  }
  kick(C1{}, C1{}, LCW2_SITE(m4));
  kick(C2{}, C1{}, LCW2_SITE(m3));
  kick(C3{}, C1{}, LCW2_SITE(p4));
  xch(std::integral_constant<int, kL1>{}, std::integral_constant<int, kL2s>{});
  // ---- L2: l1 on -2 -1 0 +1, swap +2 +3 in, l1 on +2 +3, D4, l2 on +2 +3 0 +1 ----
  kick(C0{}, C1{}, LCW2_SITE(m2));
  kick(C1{}, C1{}, LCW2_SITE(m1));
  kick(C2{}, C1{}, LCW2_SITE(z0));
  kick(C3{}, C1{}, LCW2_SITE(p1));
  swap_reg_lane<0, 16>(v);  // register bit 0: +2 (lane bit 4: -2)
  swap_reg_lane<1, 32>(v);  // register bit 1: +3 (lane bit 5: -1)
  kick(C0{}, C1{}, LCW2_SITE(p2));
  kick(C1{}, C1{}, LCW2_SITE(p3));
  {  // D4 = T4a(-4 .. 0) T4b(0 .. +4): register 0 (bit 2) in 4a, all four in 4b
    int ba = tab_base<kL2e, kT4a>(t, bit_p5), bb = tab_base<kL2e, kT4b>(t, bit_p5);
    asm volatile("" : "+v"(ba), "+v"(bb));
    const double2* ta = s_tab + tab_off(kT4a) + ba;
    const double2* tb = s_tab + tab_off(kT4b) + bb;
    const double2 a0 = ta[0], a1 = ta[tab_reg<kL2e, kT4a>(4)];
#pragma unroll
    for (int r = 0; r < kRegs; ++r) v[r] = cmul(v[r], cmul((r & 4) ? a1 : a0, tb[tab_reg<kL2e, kT4b>(r)]));
  }
  kick(C0{}, C2{}, LCW2_SITE(p2));
  kick(C1{}, C2{}, LCW2_SITE(p3));
  kick(C2{}, C2{}, LCW2_SITE(z0));
  kick(C3{}, C2{}, LCW2_SITE(p1));
  xch(std::integral_constant<int, kL2e>{}, std::integral_constant<int, kL3s>{});
  // ---- L3: l2 on -3 -2 -1, D3, l3 on -2 -1 0 (+1, +2 swapped in), D2, l4, D1, l5 ----
  kick(C0{}, C2{}, LCW2_SITE(m3));
  kick(C1{}, C2{}, LCW2_SITE(m2));
  kick(C2{}, C2{}, LCW2_SITE(m1));
  diag1(std::integral_constant<int, kL3s>{}, std::integral_constant<int, kT3>{});
  kick(C1{}, C3{}, LCW2_SITE(m2));
  kick(C2{}, C3{}, LCW2_SITE(m1));
  kick(C3{}, C3{}, LCW2_SITE(z0));
  swap_reg_lane<0, 32>(v);  // register bit 0: +1 (lane bit 5: -3)
  kick(C0{}, C3{}, LCW2_SITE(p1));
  swap_reg_lane<1, 16>(v);  // register bit 1: +2 (lane bit 4: -2)
  kick(C1{}, C3{}, LCW2_SITE(p2));
  diag1(std::integral_constant<int, kL3e>{}, std::integral_constant<int, kT2>{});
  kick(C2{}, C4{}, LCW2_SITE(m1));
  kick(C3{}, C4{}, LCW2_SITE(z0));
  kick(C0{}, C4{}, LCW2_SITE(p1));
  diag1(std::integral_constant<int, kL3e>{}, std::integral_constant<int, kT1>{});
  kick(C3{}, C5{}, LCW2_SITE(z0));
#undef LCW2_SITE
  // probe: j at register bit 3 of L3e; the frame's final X on j flips it
  double ptot = 0.0, pz = 0.0;
#pragma unroll
  for (int r = 0; r < kRegs; ++r) {
    const double p2v = fma(v[r].x, v[r].x, v[r].y * v[r].y);
    ptot += p2v;
    pz += ((r >> 3) & 1) ? -p2v : p2v;
  }
  if ((R.bits(kLcwMask + kLcwLayers - 1) >> j) & 1) pz = -pz;
  const double g2 = R.d(0, kLcwG2);
  const int wave = t >> 6, lane = t & 63;
  const double tot = wave_sum(ptot) * g2;
  const double z = wave_sum(pz) * g2;
  if (lane == 0) {
    s_red[wave][0] = tot;
    s_red[wave][1] = z;
  }
  __syncthreads();
  if (t < 2) {
    double acc = 0.0;
    for (int k = 0; k < kThreads / 64; ++k) acc += s_red[k][t];
    A.partial[(b * n_tiles + tile) * A.n_obs + t] = acc;
  }
}

// ---- the 12-site light-cone end, C2 form (dtc_lcw3_final) ------------------
// One more pass of the echo chain merged: seven layers l0 .. l6 (cone radius
// 6 .. 0) over the window j-5 .. j+6 (sites m5 .. p6; the C2 chains' first
// layer is group B's pre-kick, p2 .. p6), tile bit k = global bit j-5+k.  No
// column bits: the tile reads 16-B pieces, each 128-B line shared by eight
// consecutive tiles of the same XCD (ordinary loads: L2 serves the partners,
// tools/run64_bench.hip R16: 3.1 TB/s at x1.00 of the bytes, the pass needs
// less).  Program (register sites, swaps into lane bits 4 / 5):
//   X1  p3 p4 p5 p6 | l0: p3 p4 p5 p6, swap p2 in, p2 | D6 | l1: p3 p4 p5 p2,
//                     swap m5 in, m5
//   X2  m4 m3 m2 m1 | l1: m4 m3 m2 m1, swap z0 p1 in, z0 p1 | D5 | l2: z0 p1
//                     m2 m1
//   X3  p2 p3 p4 m3 | l2: p2 p3 p4 m3, swap m4 in, m4 | D4 | l3: p2 p3 m3
//   X4  m2 m1 z0 p1 | l3: m2 m1 z0 p1 | D3 | l4: m2 m1 z0 p1, swap p2 in, p2 |
//                     D2 | l5: m1 z0 p1 | D1 | l6: z0 | probe
// 41 site kicks, three LDS re-layouts, six row swaps (a seventh, swapping
// m4 m3 back in X2, cost 1.7 % of the pass: r4m).  Re-layout slots are
// the tile index mapped by an invertible GF(2) matrix (lcw3::cv: 4096 slots,
// the thread's base XOR a compile-time register part): the low four bits of
// the lane 0..3 sites' vectors are independent in every layout written, the
// low five of lanes 0..4 in every layout read, so the accesses are
// conflict-free (ds_write_b64: 16-lane groups, ds_read_b64: 32).  The cone
// diagonals r = 6, 5, 4, 3 are split at j (two tables each, 456 entries with
// r = 2 and 1; the r = 6 left table staged for the workgroup's bit j-6 only):
// 40.1 KB of LDS, four workgroups per CU.
namespace lcw3 {
enum : int { m5 = 0, m4, m3, m2, m1, z0, p1, p2, p3, p4, p5, p6, kNSite };
__host__ __device__ constexpr int off_of(int s) { return s - z0; }
#ifdef DTC_LCW3_ADD
// Development variant (round 6): additive slots, so a slot is the thread's
// base plus a compile-time register part -- the ds_write_b64 / ds_read_b64
// immediate, no address VALU per access.  Site -> position k of the padded
// index y + (y >> 5) + (y >> 10) (strictly increasing in y: injective, 4226
// slots); position k weighs 2^k + 2^(k-5) [k >= 5] + 2^(k-10) [k >= 10], so
// its 2-adic valuation is k mod 5, and every layout's lane sites 0..4 (reads)
// carry distinct valuations below 5 (the writes' lane 0..3 sites would need
// distinct ones below 4: this variant leaves some writes two-way).
__host__ __device__ constexpr int pos_of_site(int s) {
  return s == m4 ? 0 : s == m3 ? 1 : s == m2 ? 2 : s == m1 ? 3 : s == z0 ? 4 : s == p3 ? 5
       : s == p1 ? 6 : s == p5 ? 7 : s == p6 ? 8 : s == p2 ? 9 : s == m5 ? 10 : 11;
}
__host__ __device__ constexpr int cv(int s) {
  return (1 << pos_of_site(s)) + (pos_of_site(s) >= 5 ? 1 << (pos_of_site(s) - 5) : 0) +
         (pos_of_site(s) >= 10 ? 1 << (pos_of_site(s) - 10) : 0);
}
static constexpr int kSlots = 4226;
#define LCW3_SLOT(a, b) ((a) + (b))
#else
// (ds_write_b64 serves 16 contiguous lanes per LDS cycle: bank = slot mod 16;
// ds_read_b64 32: slot mod 32.  The low four bits of the written layouts'
// lane 0..3 sites and the low five of the read layouts' lane 0..4 sites are
// independent -- checked by simulating the lane groups.  Round 6: z0's vector
// had no low-four bits (16), so X3e's writes were two-way, 128 conflict cycles
// per wave of the 276 SQ_LDS_BANK_CONFLICT counted, r6c)
__host__ __device__ constexpr int cv(int s) {
  return s == m4 ? 1 : s == m3 ? 2 : s == m2 ? 4 : s == m1 ? 8 : s == z0 ? 16 | 1
       : s == p3 ? 32 | 2 : s == p4 ? 64 | 1 : s == p1 ? 128 | 2 : s == p5 ? 256 | 14
       : s == p6 ? 512 | 8 : s == p2 ? 1024 | 16 : 2048;
}
static constexpr int kSlots = kTile;
#define LCW3_SLOT(a, b) ((a) ^ (b))
#endif
// layouts: positions 0..3 registers, 4..9 lane bits 0..5, 10..11 wave bits
enum : int { kX1 = 0, kX1e, kX1f, kX2, kX2s, kX3, kX3e, kX4, kX4e };
__host__ __device__ constexpr int lay_site(int li, int pos) {
  constexpr int tab[9][12] = {
      {p3, p4, p5, p6, m4, m3, m2, m1, p2, m5, z0, p1},   // X1 (load)
      {p3, p4, p5, p2, m4, m3, m2, m1, p6, m5, z0, p1},   // X1e: R3 <-> lane 4
      {m5, p4, p5, p2, m4, m3, m2, m1, p6, p3, z0, p1},   // X1f: R0 <-> lane 5
      {m4, m3, m2, m1, p3, p4, p5, p6, z0, p1, m5, p2},   // X2
      {z0, p1, m2, m1, p3, p4, p5, p6, m4, m3, m5, p2},   // X2s: R0 <-> lane 4, R1 <-> lane 5
      {p2, p3, p4, m3, p1, m2, m1, z0, m4, m5, p5, p6},   // X3
      {p2, p3, m4, m3, p1, m2, m1, z0, p4, m5, p5, p6},   // X3e: R2 <-> lane 4
      {m2, m1, z0, p1, m4, m3, p5, p6, p2, m5, p3, p4},   // X4
      {p2, m1, z0, p1, m4, m3, p5, p6, m2, m5, p3, p4}};  // X4e: R0 <-> lane 4
  return tab[li][pos];
}
__host__ __device__ constexpr int reg_slot(int li, int r) {
  return LCW3_SLOT(LCW3_SLOT(LCW3_SLOT((r & 1) ? cv(lay_site(li, 0)) : 0,
                                       (r & 2) ? cv(lay_site(li, 1)) : 0),
                             (r & 4) ? cv(lay_site(li, 2)) : 0),
                   (r & 8) ? cv(lay_site(li, 3)) : 0);
}
template <int LI>
__device__ __forceinline__ int slot_base(int t) {
  int b = 0;
#pragma unroll
  for (int p = 4; p < 12; ++p) b = LCW3_SLOT(b, ((t >> (p - 4)) & 1) * cv(lay_site(LI, p)));
  return b;
}
// cone tables in LDS (double2 entries), natural index order from bit lo
// kT4 / kT3: the r = 4 and r = 3 diagonals whole (9 and 7 bits), formed in
// LDS from their staged halves (T4[y] = T4a[y & 31] T4b[y >> 4], the halves
// overlapping at j): one lookup and product per amplitude instead of two
enum : int { kT6a = 0, kT6b, kT5a, kT5b, kT4a, kT4b, kT3a, kT3b, kT2, kT1, kT4, kT3, kNTab };
__host__ __device__ constexpr int tab_off(int k) {
  return k == kT6a ? 0 : k == kT6b ? 64 : k == kT5a ? 192 : k == kT5b ? 256 : k == kT4a ? 320
       : k == kT4b ? 352 : k == kT3a ? 384 : k == kT3b ? 400 : k == kT2 ? 416 : k == kT1 ? 448
       : k == kT4 ? 456 : 968;
}
static constexpr int kTabStaged = 456;  // entries staged from the instance's tables
#ifdef DTC_LCW3_MERGE
static constexpr int kTabEntries = 1096;
#else
static constexpr int kTabEntries = 456;
#endif
__host__ __device__ constexpr int tab_bits(int k) {
  return k == kT6a ? 6 : k == kT6b ? 7 : (k == kT5a || k == kT5b) ? 6 : (k == kT4a || k == kT4b) ? 5
       : (k == kT3a || k == kT3b) ? 4 : k == kT2 ? 5 : k == kT1 ? 3 : k == kT4 ? 9 : 7;
}
__host__ __device__ constexpr int tab_lo(int k) {  // offset from j of index bit 0
  return k == kT6a ? -5 : k == kT5a ? -5 : (k == kT4a || k == kT4) ? -4 : (k == kT3a || k == kT3) ? -3
       : k == kT2 ? -2 : k == kT1 ? -1 : 0;
}
__host__ __device__ constexpr int tab_layer(int k) {
  return (k == kT6a || k == kT6b) ? 0 : (k == kT5a || k == kT5b) ? 1 : (k == kT4a || k == kT4b) ? 2
       : (k == kT3a || k == kT3b) ? 3 : k == kT2 ? 4 : 5;
}
__host__ __device__ constexpr int tab_src(int k) {
  return k == kT6a ? kLcTab6a : k == kT6b ? kLcTab6b : k == kT5a ? kLcTab5a : k == kT5b ? kLcTab5b
       : k == kT4a ? kLcTab4a : k == kT4b ? kLcTab4b : k == kT3a ? kLcTab3a : k == kT3b ? kLcTab3b
       : lc_tab_off(k == kT2 ? 2 : 1);
}
__host__ __device__ constexpr int tab_wt(int k, int s) {
  const int d = off_of(s) - tab_lo(k);
  return (d < 0 || d >= tab_bits(k)) ? 0 : 1 << d;
}
template <int LI, int K>
__device__ __forceinline__ int tab_reg(int r) {
  return ((r & 1) ? tab_wt(K, lay_site(LI, 0)) : 0) + ((r & 2) ? tab_wt(K, lay_site(LI, 1)) : 0) +
         ((r & 4) ? tab_wt(K, lay_site(LI, 2)) : 0) + ((r & 8) ? tab_wt(K, lay_site(LI, 3)) : 0);
}
template <int LI, int K>
__device__ __forceinline__ int tab_base(int t) {
  int b = 0;
#pragma unroll
  for (int p = 4; p < 12; ++p) b += ((t >> (p - 4)) & 1) * tab_wt(K, lay_site(LI, p));
  return b;
}
}  // namespace lcw3

template <int KIND>
__global__ __launch_bounds__(kThreads, DTC_LCW3_WPS) void dtc_lcw3_final(PassArgs A) {
  static_assert(KIND == kKindRX || KIND == kKindRY, "light-cone pass: factored kicks");
  using namespace lcw3;
  __shared__ double s_x[kSlots];
  __shared__ double2 s_tab[kTabEntries];
  __shared__ double s_red[kThreads / 64][2];
  const int t = threadIdx.x;
  const int64_t n_tiles = (int64_t)1 << (A.L_eff - kTileBits);
  const int og = A.octet_bits;
  const int64_t b = og ? (((int64_t)blockIdx.y << 3) | (blockIdx.x & 7)) : (int64_t)blockIdx.y;
  const int64_t tile = og ? (int64_t)(blockIdx.x >> 3) : (int64_t)blockIdx.x;
  if (og && b >= A.batch) return;
  const int inst = (int)((A.batch_start + b) / A.n_traj);
  const int j = A.probe;
  // the state's records through the scalar data cache (RecScalar): these
  // ends are VALU-bound, a v_readlane pair per coefficient is an issue slot
  const RecScalar R(A.recs + b * kRecPerState);
  // global bit of each window site; the tile's base: its id in bits
  // 0 .. j-6 and j+7 .. (the host checks j >= 6: bit j-6 is an id bit)
  auto gpos = [&](int s) { return j + off_of(s); };
  const uint32_t tbase = ((uint32_t)tile & ((1u << (j - 5)) - 1u)) |
                         (((uint32_t)tile >> (j - 5)) << (j + 7));
  const int b6 = (int)((tbase >> (j - 6)) & 1u);  // table 6a's bit j-6
  double2 v[kRegs];
  auto xch = [&](auto from_tag, auto to_tag) {
    constexpr int F = decltype(from_tag)::value, T = decltype(to_tag)::value;
    int bf = slot_base<F>(t), bt = slot_base<T>(t);
    asm volatile("" : "+v"(bf), "+v"(bt));
#pragma unroll
    for (int r = 0; r < kRegs; ++r) s_x[LCW3_SLOT(bf, reg_slot(F, r))] = v[r].x;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kRegs; ++r) v[r].x = s_x[LCW3_SLOT(bt, reg_slot(T, r))];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kRegs; ++r) s_x[LCW3_SLOT(bf, reg_slot(F, r))] = v[r].y;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kRegs; ++r) v[r].y = s_x[LCW3_SLOT(bt, reg_slot(T, r))];
  };
  auto kick = [&](auto q_tag, auto l_tag, auto s_tag) {
    constexpr int Q = decltype(q_tag)::value, l = decltype(l_tag)::value, S = decltype(s_tag)::value;
    layer_f<KIND, 0, Q>(v, R.d(0, 12 * l + S));
  };
  // v[r] *= TA[reg part] * TB[reg part] (two tables of one diagonal)
  auto diag2 = [&](auto lay_tag, auto ka_tag, auto kb_tag) {
    constexpr int LI = decltype(lay_tag)::value, KA = decltype(ka_tag)::value,
                  KB = decltype(kb_tag)::value;
    int ba = tab_base<LI, KA>(t), bb = tab_base<LI, KB>(t);
    asm volatile("" : "+v"(ba), "+v"(bb));
    const double2* ta = s_tab + tab_off(KA) + ba;
    const double2* tb = s_tab + tab_off(KB) + bb;
#pragma unroll
    for (int r = 0; r < kRegs; ++r)
      v[r] = cmul(v[r], cmul(ta[tab_reg<LI, KA>(r)], tb[tab_reg<LI, KB>(r)]));
  };
  auto diag1 = [&](auto lay_tag, auto k_tag) {
    constexpr int LI = decltype(lay_tag)::value, K = decltype(k_tag)::value;
    int base = tab_base<LI, K>(t);
    asm volatile("" : "+v"(base));
    const double2* tab = s_tab + tab_off(K) + base;
#pragma unroll
    for (int r = 0; r < kRegs; ++r) v[r] = cmul(v[r], tab[tab_reg<LI, K>(r)]);
  };
  using C0 = std::integral_constant<int, 0>;
  using C1 = std::integral_constant<int, 1>;
  using C2 = std::integral_constant<int, 2>;
  using C3 = std::integral_constant<int, 3>;
  using C4 = std::integral_constant<int, 4>;
  using C5 = std::integral_constant<int, 5>;
  using C6 = std::integral_constant<int, 6>;
#define LCW3_S(s) std::integral_constant<int, s>{}
#define LCW3_L(x) std::integral_constant<int, x>{}
  // the tile in layout X1 (ordinary loads: 16-B pieces, note above dtc_lcw2_final)
  {
    uint32_t xl = 0;
#pragma unroll
    for (int p = 4; p < 12; ++p) xl |= (uint32_t)((t >> (p - 4)) & 1) << gpos(lay_site(kX1, p));
    const int64_t vofs = octet_spread((int64_t)xl, og) << 4;
    const char* src = (const char*)(A.src + state_base(b, A.state_len, og));
    const int64_t sp0 = octet_spread((int64_t)tbase, og) << 4;
    int64_t spq[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) spq[q] = octet_spread((int64_t)1 << gpos(lay_site(kX1, q)), og) << 4;
    // uniform base + one 32-bit lane offset (global_load with an SGPR base:
    // no 64-bit address add per load) while the lane bits' byte offsets fit
    const bool vofs32 = vofs < ((int64_t)1 << 32);
#pragma unroll
    for (int r = 0; r < kRegs; ++r) {
      int64_t o = sp0;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if ((r >> q) & 1) o += spq[q];
      const d2v w = vofs32 ? *(const d2v*)(src + o + (uint32_t)vofs) : *(const d2v*)(src + o + vofs);
      v[r] = make_double2(w.x, w.y);
    }
  }
  // the cone-table entries this thread stages (e = t, t + 256 of the 456):
  // loaded behind the tile, staged after the first layer.  Wave w's entries t
  // lie in one table (6a, 6b, 6b, 5a) and its entries t + 256 in at most
  // three (5b | 4a 4b | 3a 3b 2 | 1): the wave index is made uniform, so each
  // wave runs only its own tables' index arithmetic (compile-time offsets,
  // bit counts and layers), with lane selects where a wave spans two or three
  const double2* ct = A.lc_diag + (int64_t)inst * kLcTab;
  // entry i of table K in the instance's tables (6a: the workgroup's bit j-6
  // is index bit 0 there; 5a is stored lc_pos5a-swizzled) and its staged slot
  // (i ^ m_K, m_K the frame's X mask after the table's layer on its bits)
  auto src_of = [&](auto k_tag, int i) {
    constexpr int K = decltype(k_tag)::value;
    return tab_src(K) + (K == kT6a ? ((i << 1) | b6) : K == kT5a ? lc_pos5a(i) : i);
  };
  auto dst_of = [&](auto k_tag, int i) {
    constexpr int K = decltype(k_tag)::value;
    const uint64_t m = (uint64_t)R.bits(kLcw3Mask + tab_layer(K));
    return tab_off(K) + (i ^ (int)((m >> (j + tab_lo(K))) & ((1u << tab_bits(K)) - 1u)));
  };
  using K6a = std::integral_constant<int, kT6a>;
  using K6b = std::integral_constant<int, kT6b>;
  using K5a = std::integral_constant<int, kT5a>;
  using K5b = std::integral_constant<int, kT5b>;
  using K4a = std::integral_constant<int, kT4a>;
  using K4b = std::integral_constant<int, kT4b>;
  using K3a = std::integral_constant<int, kT3a>;
  using K3b = std::integral_constant<int, kT3b>;
  using K2 = std::integral_constant<int, kT2>;
  using K1 = std::integral_constant<int, kT1>;
  static_assert(tab_off(kT6b) == 64 && tab_off(kT5a) == 192 && tab_off(kT5b) == 256 &&
                    tab_off(kT4a) == 320 && tab_off(kT4b) == 352 && tab_off(kT3a) == 384 &&
                    tab_off(kT3b) == 400 && tab_off(kT2) == 416 && tab_off(kT1) == 448 &&
                    kTabStaged == 456 && kThreads == 256,
                "the per-wave table split below");
  const int wv = __builtin_amdgcn_readfirstlane(t >> 6), ln = t & 63;
  int s0, d0, s1 = -1, d1 = 0;
  if (wv == 0) {
    s0 = src_of(K6a{}, ln); d0 = dst_of(K6a{}, ln);
    s1 = src_of(K5b{}, ln); d1 = dst_of(K5b{}, ln);
  } else if (wv == 1) {
    s0 = src_of(K6b{}, ln); d0 = dst_of(K6b{}, ln);
    const bool a = ln < 32;
    s1 = a ? src_of(K4a{}, ln) : src_of(K4b{}, ln - 32);
    d1 = a ? dst_of(K4a{}, ln) : dst_of(K4b{}, ln - 32);
  } else if (wv == 2) {
    s0 = src_of(K6b{}, 64 + ln); d0 = dst_of(K6b{}, 64 + ln);
    s1 = ln < 16 ? src_of(K3a{}, ln) : ln < 32 ? src_of(K3b{}, ln - 16) : src_of(K2{}, ln - 32);
    d1 = ln < 16 ? dst_of(K3a{}, ln) : ln < 32 ? dst_of(K3b{}, ln - 16) : dst_of(K2{}, ln - 32);
  } else {
    s0 = src_of(K5a{}, ln); d0 = dst_of(K5a{}, ln);
    if (ln < 8) {
      s1 = src_of(K1{}, ln);
      d1 = dst_of(K1{}, ln);
    }
  }
  const double2 tv0 = ct[s0];
  double2 tv1 = make_double2(0.0, 0.0);
  if (s1 >= 0) tv1 = ct[s1];
  // ---- X1: l0 on p3 p4 p5 p6, p2 (swapped in) ----
  kick(C0{}, C0{}, LCW3_S(p3));
  kick(C1{}, C0{}, LCW3_S(p4));
  kick(C2{}, C0{}, LCW3_S(p5));
  kick(C3{}, C0{}, LCW3_S(p6));
  swap_reg_lane<3, 16>(v);  // register bit 3: p2 (lane bit 4: p6)
  // (the 13 / 7 split's chains start with group B = sites j+3 ..: no p2 kick
  // in l0; workgroup-uniform)
  if ((A.lc_mask >> p2) & 1ull) kick(C3{}, C0{}, LCW3_S(p2));
  // stage the tables at their frame-masked slots, conjugated for D*
  {
    const double cs = A.diag_conj ? -1.0 : 1.0;
    s_tab[d0] = make_double2(tv0.x, cs * tv0.y);
    if (s1 >= 0) s_tab[d1] = make_double2(tv1.x, cs * tv1.y);
  }
  __syncthreads();  // the tables, before D6 (the first re-layout comes later)
  // ---- D6 in X1e, l1 on p3 p4 p5 p2, m5 (swapped in) ----
  diag2(LCW3_L(kX1e), LCW3_L(kT6a), LCW3_L(kT6b));
  kick(C0{}, C1{}, LCW3_S(p3));
  kick(C1{}, C1{}, LCW3_S(p4));
  kick(C2{}, C1{}, LCW3_S(p5));
  kick(C3{}, C1{}, LCW3_S(p2));
  swap_reg_lane<0, 32>(v);  // register bit 0: m5 (lane bit 5: p3)
  kick(C0{}, C1{}, LCW3_S(m5));
#ifdef DTC_LCW3_MERGE
  // the whole r = 4 / r = 3 tables from their staged halves (read after the
  // staging barrier, used after the next re-layout's barriers)
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int y = t + e * kThreads;
    s_tab[tab_off(kT4) + y] = cmul(s_tab[tab_off(kT4a) + (y & 31)], s_tab[tab_off(kT4b) + (y >> 4)]);
  }
  if (t < 128) s_tab[tab_off(kT3) + t] = cmul(s_tab[tab_off(kT3a) + (t & 15)], s_tab[tab_off(kT3b) + (t >> 3)]);
#endif
  xch(LCW3_L(kX1f), LCW3_L(kX2));
  // ---- X2: l1 on m4 m3 m2 m1, z0 p1 (swapped in), D5, l2 ----
  kick(C0{}, C1{}, LCW3_S(m4));
  kick(C1{}, C1{}, LCW3_S(m3));
  kick(C2{}, C1{}, LCW3_S(m2));
  kick(C3{}, C1{}, LCW3_S(m1));
  swap_reg_lane<0, 16>(v);  // register bit 0: z0 (lane bit 4: m4)
  swap_reg_lane<1, 32>(v);  // register bit 1: p1 (lane bit 5: m3)
  kick(C0{}, C1{}, LCW3_S(z0));
  kick(C1{}, C1{}, LCW3_S(p1));
  diag2(LCW3_L(kX2s), LCW3_L(kT5a), LCW3_L(kT5b));
  kick(C0{}, C2{}, LCW3_S(z0));
  kick(C1{}, C2{}, LCW3_S(p1));
  kick(C2{}, C2{}, LCW3_S(m2));
  kick(C3{}, C2{}, LCW3_S(m1));
  xch(LCW3_L(kX2s), LCW3_L(kX3));
  // ---- X3: l2 on p2 p3 p4 m3, m4 (swapped in), D4, l3 on p2 p3 m3 ----
  kick(C0{}, C2{}, LCW3_S(p2));
  kick(C1{}, C2{}, LCW3_S(p3));
  kick(C2{}, C2{}, LCW3_S(p4));
  kick(C3{}, C2{}, LCW3_S(m3));
  swap_reg_lane<2, 16>(v);  // register bit 2: m4 (lane bit 4: p4)
  kick(C2{}, C2{}, LCW3_S(m4));
#ifdef DTC_LCW3_MERGE
  diag1(LCW3_L(kX3e), LCW3_L(kT4));
#else
  diag2(LCW3_L(kX3e), LCW3_L(kT4a), LCW3_L(kT4b));
#endif
  kick(C0{}, C3{}, LCW3_S(p2));
  kick(C1{}, C3{}, LCW3_S(p3));
  kick(C3{}, C3{}, LCW3_S(m3));
  xch(LCW3_L(kX3e), LCW3_L(kX4));
  // ---- X4: l3 on m2 m1 z0 p1, D3, l4, D2, l5, D1, l6 ----
  kick(C0{}, C3{}, LCW3_S(m2));
  kick(C1{}, C3{}, LCW3_S(m1));
  kick(C2{}, C3{}, LCW3_S(z0));
  kick(C3{}, C3{}, LCW3_S(p1));
#ifdef DTC_LCW3_MERGE
  diag1(LCW3_L(kX4), LCW3_L(kT3));
#else
  diag2(LCW3_L(kX4), LCW3_L(kT3a), LCW3_L(kT3b));
#endif
  kick(C0{}, C4{}, LCW3_S(m2));
  kick(C1{}, C4{}, LCW3_S(m1));
  kick(C2{}, C4{}, LCW3_S(z0));
  kick(C3{}, C4{}, LCW3_S(p1));
  swap_reg_lane<0, 16>(v);  // register bit 0: p2 (lane bit 4: m2)
  kick(C0{}, C4{}, LCW3_S(p2));
  diag1(LCW3_L(kX4e), LCW3_L(kT2));
  kick(C1{}, C5{}, LCW3_S(m1));
  kick(C2{}, C5{}, LCW3_S(z0));
  kick(C3{}, C5{}, LCW3_S(p1));
  diag1(LCW3_L(kX4e), LCW3_L(kT1));
  kick(C2{}, C6{}, LCW3_S(z0));
#undef LCW3_S
#undef LCW3_L
  // probe: j at register bit 2 of X4e; the frame's final X on j flips it
  double ptot = 0.0, pz = 0.0;
#pragma unroll
  for (int r = 0; r < kRegs; ++r) {
    const double p2v = fma(v[r].x, v[r].x, v[r].y * v[r].y);
    ptot += p2v;
    pz += ((r >> 2) & 1) ? -p2v : p2v;
  }
  if ((R.bits(kLcw3Mask + kLcw3Layers - 1) >> j) & 1) pz = -pz;
  const double g2 = R.d(0, kLcw3G2);
  const int wave = t >> 6, lane = t & 63;
  const double tot = wave_sum(ptot) * g2;
  const double z = wave_sum(pz) * g2;
  if (lane == 0) {
    s_red[wave][0] = tot;
    s_red[wave][1] = z;
  }
  __syncthreads();
  // (an opaque copy of t: the compiler would otherwise keep the 8 t of the
  // slot bases alive to here at the 128-VGPR cap -- a 4-byte spill per thread,
  // 1 KB of scratch writes per workgroup, r6e)
  int t2 = t;
  asm volatile("" : "+v"(t2));
  if (t2 < 2) {
    double acc = 0.0;
    for (int k = 0; k < kThreads / 64; ++k) acc += s_red[k][t2];
    A.partial[(b * n_tiles + tile) * A.n_obs + t2] = acc;
  }
}

hipError_t launch_lightcone(const PassArgs& a, dim3 grid, int kind, hipStream_t stream,
                            int* variant) {
  int vdummy = 0;
  if (!variant) variant = &vdummy;
  const int n_tiles = 1 << (a.L_eff - kTileBits);
  if (a.lc_wide == 2) {
    // 12-site light-cone pass (C2 form): seven layers, tile bit k = global
    // bit j-5+k, bits j-6 and j+6 inside the state
    const int j = a.probe;
    if (a.meas != kMeasProbe || !a.no_store || a.lc_layers != kLcw3Layers || a.n_obs < 2 ||
        !a.lc_diag || j < 6 || j + 6 > a.L_real - 1 || a.L_eff > 32 ||
        (kind != kKindRX && kind != kKindRY))
      return hipErrorInvalidValue;
    for (int k = 0; k < kTileBits; ++k)
      if (a.lc_gb[k] != j - 5 + k) return hipErrorInvalidValue;
    *variant = kLcVariantWide3;
    hipLaunchKernelGGL((kind == kKindRX ? dtc_lcw3_final<kKindRX> : dtc_lcw3_final<kKindRY>), grid,
                       dim3(kThreads), 0, stream, a);
    return hipGetLastError();
  }
  if (a.lc_wide) {
    // 10-site light-cone pass: six layers, tile bits 0, 1 = global 0, 1, the
    // probe at tile bit 6, twelve distinct global bits inside the state
    if (a.meas != kMeasProbe || !a.no_store || a.lc_layers != kLcwLayers || a.n_obs < 2 ||
        !a.lc_diag || a.lc_gb[0] != 0 || a.lc_gb[1] != 1 || a.lc_gb[6] != a.probe ||
        (kind != kKindRX && kind != kKindRY))
      return hipErrorInvalidValue;
    uint64_t seen = 0;
    for (int k = 0; k < kTileBits; ++k) {
      if (a.lc_gb[k] < 0 || a.lc_gb[k] >= a.L_eff || ((seen >> a.lc_gb[k]) & 1)) return hipErrorInvalidValue;
      seen |= 1ull << a.lc_gb[k];
    }
    // the C2 chains' form: canonical window order (lc_merge_wide) with no cone
    // clipped -> the three-re-layout kernel (dtc_lcw2_final); lc_tpb < 0 (dev
    // builds, DTC_LC_TPB=-1) keeps the six-re-layout one for A/B
    const int j = a.probe;
    const int8_t canon[kTileBits] = {0, 1, (int8_t)(j - 5), (int8_t)(j + 4), (int8_t)(j - 2),
                                     (int8_t)(j - 1), (int8_t)j, (int8_t)(j + 1), (int8_t)(j + 2),
                                     (int8_t)(j + 3), (int8_t)(j - 4), (int8_t)(j - 3)};
    bool lcw2 = a.lc_mask == kLcwMaskJ2 && j >= 7 && j + 5 <= a.L_real - 1 && a.lc_tpb >= 0;
    for (int k = 0; k < kTileBits && lcw2; ++k) lcw2 = a.lc_gb[k] == canon[k];
    *variant = lcw2 ? kLcVariantWide2 : kLcVariantWide;
    if (lcw2)
      hipLaunchKernelGGL((kind == kKindRX ? dtc_lcw2_final<kKindRX> : dtc_lcw2_final<kKindRY>), grid,
                         dim3(kThreads), 0, stream, a);
    else if (a.lc_mask == kLcwMaskJ2)
      hipLaunchKernelGGL((kind == kKindRX ? dtc_lcw_final<kKindRX, kLcwMaskJ2>
                                          : dtc_lcw_final<kKindRY, kLcwMaskJ2>),
                         grid, dim3(kThreads), 0, stream, a);
    else
      hipLaunchKernelGGL((kind == kKindRX ? dtc_lcw_final<kKindRX> : dtc_lcw_final<kKindRY>), grid,
                         dim3(kThreads), 0, stream, a);
    return hipGetLastError();
  }
  {
    // measure-only light-cone pass: probe, window at tile bits 4..11 (c = 4)
    *variant = kLcVariant8;
    if (a.c != 4 || a.act != 0xFF0 || a.meas != kMeasProbe || !a.no_store || a.lc_layers < 1 ||
        a.lc_layers > kLcLayers || a.n_obs < 2 || !a.lc_diag)
      return hipErrorInvalidValue;
    // several tiles per workgroup (register double buffer) when they divide the state
    // default: one tile per workgroup, re-layouts through half the LDS, three
    // workgroups per CU (r2ar: 6.15 -> 5.42 ms); lc_split = 0 keeps the
    // 64 KiB exchange with lc_tpb tiles per workgroup (development A/B:
    // DTC_LC_SPLIT / DTC_LC_TPB, read once by dtc_open)
    int tpb = a.lc_tpb > 0 ? a.lc_tpb : kLcTilesPerGroup;
    if (a.lc_split) {
      if (kind != kKindRX && kind != kKindRY) return hipErrorInvalidValue;
      hipLaunchKernelGGL((kind == kKindRX ? dtc_lc_final_split<kKindRX> : dtc_lc_final_split<kKindRY>),
                         grid, dim3(kThreads), 0, stream, a);
      return hipGetLastError();
    }
    while (tpb > 1 && n_tiles % tpb) tpb >>= 1;
    if (tpb != 1 && tpb != 2 && tpb != 4) tpb = 1;
    grid.x = (a.octet_bits ? 8 : 1) * n_tiles / tpb;
    if (kind != kKindRX && kind != kKindRY) return hipErrorInvalidValue;
    const bool rx = kind == kKindRX;
    if (tpb == 4)
      hipLaunchKernelGGL((rx ? dtc_lc_final<kKindRX, 4> : dtc_lc_final<kKindRY, 4>), grid, dim3(kThreads), 0, stream, a);
    else if (tpb == 2)
      hipLaunchKernelGGL((rx ? dtc_lc_final<kKindRX, 2> : dtc_lc_final<kKindRY, 2>), grid, dim3(kThreads), 0, stream, a);
    else
      hipLaunchKernelGGL((rx ? dtc_lc_final<kKindRX, 1> : dtc_lc_final<kKindRY, 1>), grid, dim3(kThreads), 0, stream, a);
    return hipGetLastError();
  }
}

}  // namespace dtc
