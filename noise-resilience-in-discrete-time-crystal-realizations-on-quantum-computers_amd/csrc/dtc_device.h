// dtc_device.h -- device helpers shared by the gfx950 kernel translation
// units (dtc_kernels.hip: prep / pass / reduce kernels; dtc_lightcone.hip: the
// light-cone ends of the echo chains): complex arithmetic, the factored kick
// butterflies, the lane-distributed kick records, the tile layouts and their
// LDS re-layouts, and the cross-lane (DPP / permlane) exchanges.
#pragma once
#include <type_traits>

#include "dtc_kernels.h"

namespace dtc {

typedef double d2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
  return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}

// General: (u, v) <- (m00 u + m01 v, m10 u + m11 v)
__device__ __forceinline__ void bfly_general(double2& u, double2& v, const double2* m) {
  const double2 m00 = m[0], m01 = m[1], m10 = m[2], m11 = m[3];
  double2 nu, nv;
  nu.x = m00.x * u.x - m00.y * u.y + m01.x * v.x - m01.y * v.y;
  nu.y = m00.x * u.y + m00.y * u.x + m01.x * v.y + m01.y * v.x;
  nv.x = m10.x * u.x - m10.y * u.y + m11.x * v.x - m11.y * v.y;
  nv.y = m10.x * u.y + m10.y * u.x + m11.x * v.y + m11.y * v.x;
  u = nu;
  v = nv;
}

// Tile layouts: register r of lane-thread t holds tile index Y(t, r) =
// ybase<LAY>(t) | (r << 4 LAY).
// Layout 2: registers = tile bits 8..11, threads = bits 0..7 (coalesced).
// Layout 1: registers = tile bits 4..7.  Layout 0: registers = bits 0..3.
template <int LAY>
__device__ __forceinline__ int ybase(int t) {
  if (LAY == 2) return t;
  if (LAY == 1) return (t & 15) | ((t >> 4) << 8);
  return t << 4;
}
template <int LAY>
__device__ __forceinline__ int tile_y(int t, int r) {
  return ybase<LAY>(t) | (r << (4 * LAY));
}

// XOR swizzle over 16-B slots: conflict-free ds_write_b128 / ds_read_b128 for
// every layout transition used here (MI355X_MICROARCH.md §LDS lane groups).
__device__ __forceinline__ int lds_slot(int y) { return y ^ ((y >> 4) & 15); }

// Factored RX-family butterfly (see SiteMat): (u, v) <- diag(1, sigma) S (u, v)
template <int VAR>
__device__ __forceinline__ void bfly_rx_f(double2& u, double2& v, double f) {
  double2 nu, nv;
  if (VAR == 0) {  // S = [[1, i f], [i f, 1]]
    nu.x = fma(-f, v.y, u.x); nu.y = fma(f, v.x, u.y);
    nv.x = fma(-f, u.y, v.x); nv.y = fma(f, u.x, v.y);
  } else if (VAR == 1) {  // sigma = -1
    nu.x = fma(-f, v.y, u.x); nu.y = fma(f, v.x, u.y);
    nv.x = fma(f, u.y, -v.x); nv.y = fma(-f, u.x, -v.y);
  } else if (VAR == 2) {  // S = [[f, i], [i, f]]
    nu.x = fma(f, u.x, -v.y); nu.y = fma(f, u.y, v.x);
    nv.x = fma(f, v.x, -u.y); nv.y = fma(f, v.y, u.x);
  } else {
    nu.x = fma(f, u.x, -v.y); nu.y = fma(f, u.y, v.x);
    nv.x = fma(-f, v.x, u.y); nv.y = fma(-f, v.y, -u.x);
  }
  u = nu;
  v = nv;
}

// Factored RY-family butterfly: (u, v) <- diag(1, sigma) R (u, v)
template <int VAR>
__device__ __forceinline__ void bfly_ry_f(double2& u, double2& v, double f) {
  double2 nu, nv;
  if (VAR == 0) {  // R = [[1, f], [-f, 1]]
    nu.x = fma(f, v.x, u.x); nu.y = fma(f, v.y, u.y);
    nv.x = fma(-f, u.x, v.x); nv.y = fma(-f, u.y, v.y);
  } else if (VAR == 1) {
    nu.x = fma(f, v.x, u.x); nu.y = fma(f, v.y, u.y);
    nv.x = fma(f, u.x, -v.x); nv.y = fma(f, u.y, -v.y);
  } else if (VAR == 2) {  // R = [[f, 1], [-1, f]]
    nu.x = fma(f, u.x, v.x); nu.y = fma(f, u.y, v.y);
    nv.x = fma(f, v.x, -u.x); nv.y = fma(f, v.y, -u.y);
  } else {
    nu.x = fma(f, u.x, v.x); nu.y = fma(f, u.y, v.y);
    nv.x = fma(-f, v.x, u.x); nv.y = fma(-f, v.y, u.y);
  }
  u = nu;
  v = nv;
}

template <int KIND, int VAR, int Q>
__device__ __forceinline__ void layer_f(double2 (&v)[kRegs], double f) {
#pragma unroll
  for (int r = 0; r < kRegs; ++r) {
    if (r & (1 << Q)) continue;
    if (KIND == kKindRX) bfly_rx_f<VAR>(v[r], v[r | (1 << Q)], f);
    else bfly_ry_f<VAR>(v[r], v[r | (1 << Q)], f);
  }
}

// The kick records of a (pass, state) — 25 x 64 B — live in the VGPRs of
// every wave: lane l holds doubles [4l, 4l + 4) of the block (loaded with the
// setup, before the tile); a coefficient is two v_readlane_b32 with static
// lane and register indices: no LDS, no scalar-memory round trip per layer.
struct RecRegs {
  double rv[4];
  __device__ __forceinline__ long long bits(int j) const {
    const long long x = __double_as_longlong(rv[j & 3]);
    const int lo = __builtin_amdgcn_readlane((int)(x & 0xffffffffll), j >> 2);
    const int hi = __builtin_amdgcn_readlane((int)(x >> 32), j >> 2);
    return ((long long)hi << 32) | (unsigned int)lo;
  }
  __device__ __forceinline__ double d(int rec, int e) const {
    return __longlong_as_double(bits(8 * rec + e));
  }
  __device__ __forceinline__ int i(int rec, int e) const { return (int)bits(8 * rec + e); }
};

// The same records read through the scalar data cache instead: the block's
// address is uniform, so with the constant address space every value is an
// s_load into SGPRs (batched by the compiler) and a butterfly takes it as an
// SGPR operand -- no v_readlane_b32 pair per value.  For the VALU-bound
// light-cone ends (dtc_lcw3_final: 98 readlanes of 2818 VALU per wave).  The
// records are written by an earlier kernel of the stream (prep_kernel); the
// scalar cache is invalidated at every dispatch.
struct RecScalar {
  typedef __attribute__((address_space(4))) const long long* cptr;
  cptr p;
  __device__ __forceinline__ explicit RecScalar(const KickRec* rec)
      : p((cptr)(const void*)rec) {}
  __device__ __forceinline__ long long bits(int j) const { return p[j]; }
  __device__ __forceinline__ double d(int rec, int e) const {
    return __longlong_as_double(p[8 * rec + e]);
  }
  __device__ __forceinline__ int i(int rec, int e) const { return (int)p[8 * rec + e]; }
};

// FRAME (unitary RX / RY kicks of a Pauli-frame pass, dtc_kernels.hip
// frame12_records): every kick runs the form-B butterfly with the frame-signed
// coefficient of d[3], no variant branch
template <int N, int KIND, int QM = 15, bool FRAME = false, typename Rec>
__device__ __forceinline__ void apply_nibble(double2 (&v)[kRegs], const Rec& R, int rec0) {
  // Every site of an active nibble runs (inactive sites carry the identity):
  // no data-dependent branches, so no register shuffles at merge points; the
  // RX/RY variant branch is wave-uniform.  QM: the register bits that hold
  // sites at all (the 7-site column group's nibble 1 starts with a column bit)
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (!((QM >> q) & 1)) continue;
    const int k = rec0 + 4 * N + q;
    if (KIND == kKindGen) {
      double2 m[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) m[e] = make_double2(R.d(k, 2 * e), R.d(k, 2 * e + 1));
#pragma unroll
      for (int r = 0; r < kRegs; ++r)
        if (!(r & (1 << q))) bfly_general(v[r], v[r | (1 << q)], m);
    } else if (KIND == kKindRXU || KIND == kKindRYU) {
      // S of form A or B only (the sign and the Kraus factor: the deferred
      // diag(1, rho), rho_apply)
      constexpr int BK = KIND == kKindRXU ? kKindRX : kKindRY;
      const double f = R.d(k, 0);
      const int var = R.i(k, 1);
      auto run = [&](auto qtag) {
        constexpr int Q = decltype(qtag)::value;
        if (var == 0) layer_f<BK, 0, Q>(v, f);
        else layer_f<BK, 2, Q>(v, f);
      };
      if (q == 0) run(std::integral_constant<int, 0>{});
      else if (q == 1) run(std::integral_constant<int, 1>{});
      else if (q == 2) run(std::integral_constant<int, 2>{});
      else run(std::integral_constant<int, 3>{});
    } else if constexpr (FRAME) {
      static_assert(KIND == kKindRX || KIND == kKindRY, "Pauli-frame kicks: the unitary families");
      const double f = R.d(k, 3);
      auto run = [&](auto qtag) { layer_f<KIND, 2, decltype(qtag)::value>(v, f); };
      if (q == 0) run(std::integral_constant<int, 0>{});
      else if (q == 1) run(std::integral_constant<int, 1>{});
      else if (q == 2) run(std::integral_constant<int, 2>{});
      else run(std::integral_constant<int, 3>{});
    } else {
      const double f = R.d(k, 0);
#ifdef DTC_VAR_PROBE
      // timing probe only (wrong results by design): one butterfly variant
      auto run = [&](auto qtag) { layer_f<KIND, 2, decltype(qtag)::value>(v, f); };
#else
      const int var = R.i(k, 1);
      auto run = [&](auto qtag) {
        constexpr int Q = decltype(qtag)::value;
        if (var == 0) layer_f<KIND, 0, Q>(v, f);
        else if (var == 1) layer_f<KIND, 1, Q>(v, f);
        else if (var == 2) layer_f<KIND, 2, Q>(v, f);
        else layer_f<KIND, 3, Q>(v, f);
      };
#endif
      if (q == 0) run(std::integral_constant<int, 0>{});
      else if (q == 1) run(std::integral_constant<int, 1>{});
      else if (q == 2) run(std::integral_constant<int, 2>{});
      else run(std::integral_constant<int, 3>{});
    }
  }
}

// Tile re-layout through LDS.  No barrier before the writes: a thread writes
// exactly the slots it read itself in the previous exchange (that one ended in
// layout FROM), so no other thread can still need them.
// xw, xr (Pauli-frame passes): the frame's X bits this re-layout flushes,
// on the write side (thread bits of FROM) and the read side (thread bits of
// TO): index y is written at slot(y ^ xw), read from slot(y ^ xr), so the
// tile comes out X^(xw ^ xr)-permuted, and the register offsets stay
// compile-time immediates.  A thread then no longer writes only slots it read
// itself in the previous re-layout when xw or that one's xr is nonzero: the
// caller passes sync for those.
template <int FROM, int TO>
__device__ __forceinline__ void exchange(double2 (&v)[kRegs], double2* s_tile, int t, int xw = 0,
                                         int xr = 0, bool sync = false) {
  if (FROM == TO) return;
  constexpr int kThrF = (kTile - 1) & ~(15 << (4 * FROM)), kThrT = (kTile - 1) & ~(15 << (4 * TO));
  const int yw = ybase<FROM>(t) ^ (xw & kThrF), yr = ybase<TO>(t) ^ (xr & kThrT);
  if (sync) __syncthreads();
#pragma unroll
  for (int r = 0; r < kRegs; ++r) s_tile[lds_slot(yw | (r << (4 * FROM)))] = v[r];
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kRegs; ++r) v[r] = s_tile[lds_slot(yr | (r << (4 * TO)))];
}

// The same re-layout through a half-tile buffer, real parts then imaginary
// parts (8-B slots): about half the LDS, so three workgroups fit a CU; two
// more barriers (the imaginary writes reuse the slots the real reads just
// left).  Slots are the tile index XOR-swizzled,
//   slot(y) = y ^ ((y >> 4) & 15) ^ (((y >> 8) & 1) << 4),
// linear over XOR, so a slot is the thread's base XOR a compile-time register
// offset (one VALU op per access); the compiler merges register pairs into
// ds_read2_b64 / ds_write2st64_b64.  Development builds with -DDTC_ADD_SLOTS
// use additive slots, y[0:4) + 17 y[4:8) + 272 y[8:12) (4351 slots): base +
// immediate offset, no address VALU, but either merged into ds_read2 pairs or
// (Makefile KNOMERGE=1) issued one by one they ran slower on the same box --
// C2 -2.0 % (r4c, merged) and -1.9 % (r4d, unmerged), energy -2.4 %.
#ifdef DTC_ADD_SLOTS
static constexpr int kHalfSlots = 15 + 17 * 15 + 272 * 15 + 1;
__host__ __device__ constexpr int slot_add(int y) {
  return (y & 15) + 17 * ((y >> 4) & 15) + 272 * (y >> 8);
}
#define DTC_SLOT(base, LAY, r) ((base) + slot_add((r) << (4 * (LAY))))
#else
static constexpr int kHalfSlots = kTile;
__host__ __device__ constexpr int slot_add(int y) { return y ^ ((y >> 4) & 15) ^ (((y >> 8) & 1) << 4); }
#define DTC_SLOT(base, LAY, r) ((base) ^ slot_add((r) << (4 * (LAY))))
#endif
template <int FROM, int TO>
__device__ __forceinline__ void exchange_split(double2 (&v)[kRegs], double* s_half, int t, int xw = 0,
                                               int xr = 0) {
  if (FROM == TO) return;
  // the two per-thread bases are made opaque here, so every exchange forms
  // them afresh instead of the compiler keeping addresses live across the
  // kernel (the 12-site K-D-K at three workgroups per CU once spilled 80 B/lane
  // for 16 slot addresses per layout, r3h)
  int bf = slot_add(ybase<FROM>(t)), bt = slot_add(ybase<TO>(t));
#ifndef DTC_ADD_SLOTS
  bf ^= slot_add(xw);  // the frame's X flushes (exchange above)
  bt ^= slot_add(xr);
#endif
  asm volatile("" : "+v"(bf), "+v"(bt));
#pragma unroll
  for (int r = 0; r < kRegs; ++r) s_half[DTC_SLOT(bf, FROM, r)] = v[r].x;
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kRegs; ++r) v[r].x = s_half[DTC_SLOT(bt, TO, r)];
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kRegs; ++r) s_half[DTC_SLOT(bf, FROM, r)] = v[r].y;
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kRegs; ++r) v[r].y = s_half[DTC_SLOT(bt, TO, r)];
}

// Two tiles re-laid out together (the dual pass's forward and echo tiles),
// each through its own half-tile buffer with the same slots: three barriers
// for both.  Each buffer follows exchange_split's slot discipline.
// (each tile with its own frame's flushes: vw, vr and ww, wr, exchange above)
template <int FROM, int TO>
__device__ __forceinline__ void exchange_split2(double2 (&v)[kRegs], double2 (&w)[kRegs],
                                                double* s_a, double* s_b, int t, int vw = 0,
                                                int vr = 0, int ww = 0, int wr = 0) {
  if (FROM == TO) return;
  int bf = slot_add(ybase<FROM>(t)), bt = slot_add(ybase<TO>(t));
  int bw = bf, bu = bt;
#ifndef DTC_ADD_SLOTS
  bf ^= slot_add(vw);
  bt ^= slot_add(vr);
  bw ^= slot_add(ww);
  bu ^= slot_add(wr);
#endif
  asm volatile("" : "+v"(bf), "+v"(bt), "+v"(bw), "+v"(bu));
#pragma unroll
  for (int r = 0; r < kRegs; ++r) {
    s_a[DTC_SLOT(bf, FROM, r)] = v[r].x;
    s_b[DTC_SLOT(bw, FROM, r)] = w[r].x;
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kRegs; ++r) {
    v[r].x = s_a[DTC_SLOT(bt, TO, r)];
    w[r].x = s_b[DTC_SLOT(bu, TO, r)];
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kRegs; ++r) {
    s_a[DTC_SLOT(bf, FROM, r)] = v[r].y;
    s_b[DTC_SLOT(bw, FROM, r)] = w[r].y;
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kRegs; ++r) {
    v[r].y = s_a[DTC_SLOT(bt, TO, r)];
    w[r].y = s_b[DTC_SLOT(bu, TO, r)];
  }
}

// (Pauli-frame masks: xw, xr, sync as exchange takes them; cw, cr the
// cumulative ones exchange_split takes)
template <bool SPLIT, int FROM, int TO>
__device__ __forceinline__ void xch_tile(double2 (&v)[kRegs], double2* s_tile, double* s_half,
                                         int t, int xw = 0, int xr = 0, int cw = 0, int cr = 0,
                                         bool sync = false) {
  if constexpr (SPLIT) exchange_split<FROM, TO>(v, s_half, t, cw, cr);
  else exchange<FROM, TO>(v, s_tile, t, xw, xr, sync);
}

__device__ __forceinline__ double2 diag_phase(const double2* s_chunk, int n_chunks, int64_t x) {
  double2 ph = s_chunk[x & 63];
  for (int k = 1; k < n_chunks; ++k) {
    ph = cmul(ph, s_chunk[k * 64 + ((x >> (kChunkBits * k)) & 63)]);
  }
  return ph;
}

// Value of lane (l ^ M) for every lane l, M = 1 .. 32, without LDS: DPP
// quad permutes (1, 2) and row rotations (4, 8) on the VALU, and gfx950's
// v_permlane16_swap / v_permlane32_swap (16, 32).  A row rotation by n gives
// lane l the value of lane ((l - n) mod 16); l ^ 8 is one such rotation, l ^ 4
// is (l + 4) or (l - 4) by lane bit 2.  permlane{16,32}_swap(x, x) returns
// (x with its even rows/lower half copied up, x with its odd rows/upper half
// copied down): the xor partner is the first for lanes with the bit set.
template <int M>
__device__ __forceinline__ int xor_lane_b32(int x) {
  static_assert(M == 1 || M == 2 || M == 4 || M == 8 || M == 16 || M == 32, "lane xor");
  if constexpr (M == 1) {
    return __builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
  } else if constexpr (M == 2) {
    return __builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
  } else if constexpr (M == 8) {
    return __builtin_amdgcn_update_dpp(0, x, 0x128, 0xF, 0xF, false);  // row_ror:8
  } else if constexpr (M == 4) {
    const int up = __builtin_amdgcn_update_dpp(0, x, 0x12C, 0xF, 0xF, false);  // l - 12 = l + 4
    const int dn = __builtin_amdgcn_update_dpp(0, x, 0x124, 0xF, 0xF, false);  // l - 4
    return (__lane_id() & 4) ? dn : up;
  } else if constexpr (M == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    return (__lane_id() & 16) ? (int)r[0] : (int)r[1];
  } else {
    const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    return (__lane_id() & 32) ? (int)r[0] : (int)r[1];
  }
}

template <int M>
__device__ __forceinline__ double xor_lane(double x) {
  const long long b = __double_as_longlong(x);
  const int lo = xor_lane_b32<M>((int)(b & 0xffffffffll));
  const int hi = xor_lane_b32<M>((int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ __forceinline__ double wave_sum(double x) {
  x += xor_lane<32>(x);
  x += xor_lane<16>(x);
  x += xor_lane<8>(x);
  x += xor_lane<4>(x);
  x += xor_lane<2>(x);
  x += xor_lane<1>(x);
  return x;
}

// One butterfly stage of a Walsh-Hadamard transform over the wave's lanes:
// lane l ends with h(l) + h(l ^ M) or h(l ^ M) - h(l) by lane bit M.
template <int M>
__device__ __forceinline__ double wht_stage(double h) {
  const double o = xor_lane<M>(h);
  return fma((__lane_id() & M) ? -1.0 : 1.0, h, o);
}

// permlane{32,16}_swap of a pair of doubles (both 32-bit halves): with
// vdst = a, src0 = b, a becomes (a's lower half-wave / even rows, b's lower /
// even) and b becomes (a's upper / odd, b's upper / odd).  For a pair whose
// first member is kept by the lanes without the bit and the second by the
// lanes with it, a + b afterwards is, in every lane, its kept vector summed
// with the partner lane's copy: one swap pair and one add per stage, no
// selects, no copies.
template <int M>
__device__ __forceinline__ void swap_rows(double& a, double& b) {
  const long long ab = __double_as_longlong(a), bb = __double_as_longlong(b);
  const int alo = (int)(ab & 0xffffffffll), ahi = (int)(ab >> 32);
  const int blo = (int)(bb & 0xffffffffll), bhi = (int)(bb >> 32);
  if constexpr (M == 32) {
    const auto lo = __builtin_amdgcn_permlane32_swap(alo, blo, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap(ahi, bhi, false, false);
    a = __longlong_as_double(((long long)(int)hi[0] << 32) | (unsigned int)lo[0]);
    b = __longlong_as_double(((long long)(int)hi[1] << 32) | (unsigned int)lo[1]);
  } else {
    static_assert(M == 16, "row swap");
    const auto lo = __builtin_amdgcn_permlane16_swap(alo, blo, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap(ahi, bhi, false, false);
    a = __longlong_as_double(((long long)(int)hi[0] << 32) | (unsigned int)lo[0]);
    b = __longlong_as_double(((long long)(int)hi[1] << 32) | (unsigned int)lo[1]);
  }
}

// register bit Q <-> lane bit 4 (M = 16) or 5 (M = 32), for the whole tile
// (32 permlane swaps, no LDS, no barrier): the light-cone ends' row swaps and
// the 13-site pass's fifth register site (dtc_tile13.hip)
template <int Q, int M>
__device__ __forceinline__ void swap_reg_lane(double2 (&v)[kRegs]) {
#pragma unroll
  for (int r = 0; r < kRegs; ++r) {
    if (r & (1 << Q)) continue;
    swap_rows<M>(v[r].x, v[r | (1 << Q)].x);
    swap_rows<M>(v[r].y, v[r | (1 << Q)].y);
  }
}

// Sum of NV per-lane vectors over the wave (NV = 4 or 8), halving the vector
// count per lane at each of the first stages: afterwards every lane of the
// group of 8 with lane bits (5, 4, 3) = v (NV = 8; NV = 4: bits (5, 4)
// and every bit-3 value) holds the wave sum of vector v.
template <int NV>
__device__ __forceinline__ double wave_sum_multi(const double (&x)[NV]) {
  const int lane = __lane_id();
  double a[NV / 2];
#pragma unroll
  for (int m = 0; m < NV / 2; ++m) {
    double u = x[m], w = x[NV / 2 + m];
    swap_rows<32>(u, w);
    a[m] = u + w;
  }
  double b[NV / 4];
#pragma unroll
  for (int m = 0; m < NV / 4; ++m) {
    double u = a[m], w = a[NV / 4 + m];
    swap_rows<16>(u, w);
    b[m] = u + w;
  }
  double c;
  if constexpr (NV == 8) {
    const bool h3 = lane & 8;
    c = (h3 ? b[1] : b[0]) + xor_lane<8>(h3 ? b[0] : b[1]);
  } else {
    c = b[0] + xor_lane<8>(b[0]);
  }
  c += xor_lane<4>(c);
  c += xor_lane<2>(c);
  c += xor_lane<1>(c);
  return c;
}

// Lane patterns kept from a wave's Walsh-Hadamard transform (s_red entries):
// 0, the single bits 1 .. 32 and the adjacent pairs 3 .. 48 — every site or
// bond observable needs one of them.  -1: not kept.
__device__ __forceinline__ int lane_pattern(int m) {
  if (m == 0) return 0;
  const int k = __ffs(m) - 1;
  if (m == (1 << k)) return 1 + k;
  if (k < 5 && m == (3 << k)) return 7 + k;
  return -1;
}

// Per-layout global index of register r: x(r) = x0(t) | off(r), off uniform.
struct TileMap {
  int64_t tbase;
  int c, s, cmask;
  __device__ __forceinline__ int64_t rel(int y) const {
    return (int64_t)(y & cmask) | ((int64_t)(y >> c) << s);
  }
  __device__ __forceinline__ int64_t at(int y) const { return tbase | rel(y); }
};

}  // namespace dtc
