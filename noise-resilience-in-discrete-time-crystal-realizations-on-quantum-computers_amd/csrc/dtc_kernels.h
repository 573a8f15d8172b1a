// dtc_kernels.h — launch interface between the host engine and the gfx950
// kernels in dtc_kernels.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dtc {

// Tile geometry: one workgroup owns 2^kTileBits amplitudes of one state,
// 256 threads x 16 amplitudes in registers, staged through 64 KiB of LDS.
static constexpr int kTileBits = 12;
static constexpr int kTile = 1 << kTileBits;
static constexpr int kThreads = 256;
static constexpr int kWaveSize = 64;
static constexpr int kRegs = 16;          // amplitudes per thread (4 register bits)
static constexpr int kChunkBits = 5;      // diagonal factor tables: 5 sites + next bit
static constexpr int kMaxChunks = 8;      // L_eff <= 40
// Per-wave reduction slots (s_red): 8 parity vectors x 12 lane patterns for
// the Z-type observables, then <X> partials of the 12 tile bits at the entry
// (pre-kick) and mid-pass (post-kick) points of an energy pass.
static constexpr int kRedLanes = 12;
static constexpr int kSlotXPre = 8 * kRedLanes;
static constexpr int kSlotXPost = kSlotXPre + kTileBits;
static constexpr int kRedSlots = kSlotXPost + kTileBits;

// Load/store register layout of a pass over the register nibbles `nibs`
// (bit n = nibble n holds active sites): 1 (threads = tile bits 0..3, 8..11:
// 256-B row segments per 16 lanes) for the nibble sets in DTC_IO1_NIBS, else 2
// (threads = tile bits 0..7).  Same-box A/B (profiles/r1s_io_ab.json): the
// 12-site low group of C2 runs 1.60 -> 1.56 ms from layout 1.
#ifndef DTC_IO1_NIBS
#define DTC_IO1_NIBS (1 << 7)
#endif
constexpr int io_layout(int nibs) { return ((DTC_IO1_NIBS >> nibs) & 1) ? 1 : 2; }

enum DiagMode { kDiagNone = 0, kDiagFwd = 1, kDiagConj = 2 };
// Tile geometries of the 12-bit passes (pass_body GEO): the plan's standard
// groups, and the 7-site column group of the 13 / 7 split (c = 5, s = 13:
// tile bits 0..4 = global 0..4, 5..11 = sites 13..19; act 0xFE0).
enum TileGeo { kGeoStd = 0, kGeoB7 = 1 };
static constexpr int kB7Cols = 5;
enum MeasMode {
  kMeasNone = 0,
  kMeasProbe = 1,   // (norm, Z_probe)
  kMeasSites = 2,   // (norm, Z_0 .. Z_{L-1})
  kMeasEnergy = 3,  // (norm, Z_i, Z_i Z_i+1, X_i mid-pass, X_i entry): 4 L values
};
// Parts of a kMeasEnergy pass (PassArgs::meas_parts).  X_i of a site is the
// pair product 2 Re sum conj(a_0) a_1 over its register bit, taken in the
// layout that holds the site in registers just before the site's kick:
//   kPartZ     norm, Z_i, Z_i Z_i+1 after the diagonal        (obs [0, 2L))
//   kPartXPost X_i of the kicked sites before the post-kick    (obs [2L, 3L))
//   kPartXPre  X_i of the kicked sites before the pre-kick     (obs [3L, 4L))
// Kicks on other sites commute with X_i, so both X points see the state of
// the time the engine assigns them to (dtc_energy).
enum MeasPart { kPartZ = 1, kPartXPost = 2, kPartXPre = 4 };
// Which parts a pass runs: pre-kick (K), diagonal (D), post-kick (K).
// kShapeLC: the light-cone end of an echo chain (lc_body in dtc_kernels.hip):
// up to kLcLayers kick layers with D between them on the 8-site window at
// tile bits 4..11 (c = 4), each layer only on the sites its mask keeps, then
// the probe; measure-only (no store).
enum PassShape { kShapeK = 0, kShapeKD = 1, kShapeDK = 2, kShapeKDK = 3, kShapeD = 4,
                 kShapeLC = 5 };
static constexpr int kLcLayers = 5;
static constexpr int kLcSites = 8;
// LC records (in the state's KickRec block read as doubles), Pauli frame form:
// every kick i^k w Z^a X^b A(f) is applied as A(f^) (A = I + i f X for the RX
// family, I + f ZX for RY), its Paulis carried to the probe: they flip the
// sign of later coefficients on the site (f^), XOR the index of later
// diagonals (x -> x ^ m) and the sign of Z_j.  Doubles [0, kLcCoefs): f^ of
// (layer l, window site b) at 8 l + b (0: identity); kLcG2: prod w^2;
// kLcPacked (as integer): bits 8 l .. 8 l + 7 = the frame's X mask after layer
// l (window sites), bits 32..39 = the final one.
static constexpr int kLcCoefs = kLcLayers * kLcSites;
static constexpr int kLcG2 = kLcCoefs;
static constexpr int kLcPacked = kLcCoefs + 1;
// Cone diagonals: the D after layer l of M only matters through its terms on
// sites j-r+1 .. j+r-1 (r = M - 1 - l; the terms elsewhere commute with
// everything after it), a function of bits j-r .. j+r (clipped to [0, L)):
// per instance one table per r = 1 .. 4 at offset (2^(2r+1) - 8) / 3.
static constexpr int kLcTab4 = 680;  // the r = 1 .. 4 tables (what the 8-site pass stages)
__host__ __device__ constexpr int lc_tab_off(int r) { return ((1 << (2 * r + 1)) - 8) / 3; }
// The 10-site pass (kShapeLC with lc_wide) also needs r = 5, a function of 11
// bits: split at j into two 6-bit tables, bits j-5 .. j (fields j-4 .. j,
// bonds (j-5, j-4) .. (j-1, j)) and bits j .. j+5 (fields j+1 .. j+4, bonds
// (j, j+1) .. (j+4, j+5)), clipped to [0, L): two lookups instead of a
// 2048-entry table (which would leave LDS for two workgroups per CU only).
// Storage swizzles of the tables whose lookups in the 10-site pass index by
// lane bits 256 B apart (one LDS bank group): entry i of the radius-4 table
// sits at lc_pos4(i), of the j-5 .. j table at lc_pos5a(i) -- XOR folds of the
// lane-varying index bits into the low bits, linear, so a lookup base ^ offset
// becomes pos(base) ^ pos(offset) at no cost per amplitude.
__host__ __device__ constexpr int lc_pos4(int i) { return i ^ ((i >> 8) & 1); }
__host__ __device__ constexpr int lc_pos5a(int i) { return i ^ ((i >> 4) & 3); }
static constexpr int kLcTab5a = kLcTab4;
static constexpr int kLcTab5b = kLcTab4 + 64;
// The radius-4 cone diagonal split at j like r = 5 (dtc_lcw2_final): bits
// j-4 .. j (fields j-3 .. j, bonds (j-4, j-3) .. (j-1, j)) and bits j .. j+4
// (fields j+1 .. j+3, bonds (j, j+1) .. (j+3, j+4)), natural order, so the
// kernel's tables fit four workgroups per CU.
static constexpr int kLcTab4a = kLcTab4 + 128;
static constexpr int kLcTab4b = kLcTab4 + 160;
// The 12-site pass (dtc_lcw3_final) adds r = 6 split at j (bits j-6 .. j:
// fields j-5 .. j, bonds (j-6, j-5) .. (j-1, j); bits j .. j+6: fields j+1 ..
// j+5, bonds (j, j+1) .. (j+5, j+6)) and r = 3 split at j (bits j-3 .. j and
// j .. j+3), natural order.
static constexpr int kLcTab6a = kLcTab4 + 192;
static constexpr int kLcTab6b = kLcTab4 + 320;
static constexpr int kLcTab3a = kLcTab4 + 448;
static constexpr int kLcTab3b = kLcTab4 + 464;
static constexpr int kLcTab = kLcTab4 + 480;  // per-instance stride of PassArgs::lc_diag
// kShapeLC with lc_wide: six kick layers over a 10-site window (one more
// pass of the echo chain merged).  Tile bits 0, 1 = global bits 0, 1 (64-B
// runs), tile bits 2 .. 11 = window sites lc_gb[2 .. 11] (host-chosen: nibble
// 1 = j-2 .. j+1, nibble 2 = j+2, j+3, j-4, j-3, bits 2, 3 = the other two),
// so the cone's inner layers stay in one or two register nibbles.  lc_mask
// bit 10 l + k - 2 = tile bit k kicked in layer l.  Records (doubles): f^ of
// (layer l, tile bit k) at 12 l + k; kLcwG2: prod w^2; kLcwMask + l (as
// integer): the frame's X mask after layer l in global bit positions
// (l = 5: the final one, for the probe's sign).
static constexpr int kLcwLayers = 6;
static constexpr int kLcwG2 = 12 * kLcwLayers;
static constexpr int kLcwMask = kLcwG2 + 1;
// kShapeLC with lc_wide = 2 (dtc_lcw3_final): seven layers over a 12-site
// window, tile bit k = global bit j-5+k (no column bits), one more pass of
// the echo chain merged; kick of (layer l, tile bit k) when bit 12 l + k of
// the 84-bit mask (lc_mask: bits 0..63, lc_mask2: 64..83) is set.  Records:
// f^ of (l, k) at 12 l + k, kLcw3G2: prod w^2, kLcw3Mask + l: the frame's X
// mask after layer l in global bit positions.
static constexpr int kLcw3Layers = 7;
static constexpr int kLcw3G2 = 12 * kLcw3Layers;
static constexpr int kLcw3Mask = kLcw3G2 + 1;
static constexpr int kLcMaxLayers = kLcw3Layers;
// Matrix family of every kick in a pass (chosen by the host from the kick
// table): Pauli x RX(theta) = i^k [[a, ib], [ic, d]], Pauli x RY(theta) =
// i^k [[a, b], [c, d]] (4 flops per amplitude), anything else general (8).
// kKindRXU / kKindRYU: the same families under device-like noise (one sub-gate
// per kick): a real Kraus diagonal times the unitary, factored as
// i^k w diag(rho0, rho1) S, the diagonal deferred to one per-amplitude factor per layer
// (SiteMat in dtc_kernels.hip), 2 flops per amplitude like RX / RY.
enum KickKind { kKindRX = 0, kKindRY = 1, kKindGen = 2, kKindRXU = 3, kKindRYU = 4 };

// One layer of single-site kicks on the sites of a pass.
enum KickMode {
  kKickForward = 0,  // M = P_n G_n ... P_1 G_1            (forward period, noisy)
  kKickInverse = 1,  // M = P_n G_1^+ ... P_1 G_n^+        (UF.inverse(), noisy)
  kKickUndo = 2,     // M = (forward M)^+                  (exact undo, same draws)
  kKickBasisX = 3,   // M = H                              (X-basis measurement, noiseless)
  kKickUndoBasisX = 4,  // M = H (forward M)^+             (undo a pending kick, then H)
};

struct KickDesc {
  int enabled;
  int row;              // kick table row (period - 1)
  int mode;             // KickMode
  uint32_t stream;      // RNG stream (0 forward, 1 + t echo branch at t)
  uint32_t rng_period;  // RNG period counter
  uint32_t skip;        // tile bits of the pass left unkicked (identity); 0 = none
};

// Kick records.  Every noisy kick of a pass is a pure function of (pass,
// state, site): the prep kernel evaluates them once per (pass, state) — the
// Pauli draws, the sub-gate products and the factored form (SiteMat in
// dtc_kernels.hip) — instead of once per tile.  Per (pass, state):
//   rec[k], rec[12 + k]  pre / post kick of tile bit k
//       RX/RY family: d[0] = coefficient, i[1] = variant, d[2] = w^2 (the
//       site's share of the global factor, squared), RXU/RYU: d[3], d[4] = rho0,
//       rho1 (the deferred Kraus diagonal);  general: d[0..7] = 2x2
//   rec[24]              d[0], d[1] = global factor (i^k * prod of scales),
//                        d[2] = 1 / w_post^2 (measurement before the post-kick)
union KickRec {
  double d[8];
  long long i[8];
};
// (blocks of 27 records: room for the 13-bit tile of dtc_tile13.hip, whose
// records are pre k, post 13 + k, total 26; the 12-bit passes use 0..24)
static constexpr int kMaxTileBits = 13;
static constexpr int kRecPerState = 2 * kMaxTileBits + 1;
static constexpr int kRecTotal = 2 * kTileBits;
// 13-site passes (Pauli-frame records, dtc_kernels.hip frame13_records): every
// kick record holds the signed form-B coefficient; the total record (26) adds
// the X masks the four re-layouts flush (tile bits) and the Z mask of the
// diagonal
enum : int { kT13MaskX1 = 3, kT13MaskX2 = 4, kT13MaskX3 = 5, kT13MaskX4 = 6, kT13MaskZ = 7 };
// 12-bit passes of the unitary RX / RY families (frame12_records, pass_body
// with FR): every kick record also holds the frame-signed form-B coefficient
// in d[3] (d[0], i[1] keep the variant form for the passes that measure X in
// flight), the total record the X masks of the pass's real re-layouts in
// program order (i[3 ..]: write side in bits 0..11, read side in 16..27) and
// the diagonal's Z mask with the frame's extra power of i in bits 16, 17 (i[7])
static constexpr int kFrameCoef = 3;
enum : int { kT12MaskX0 = 3, kT12MaskZ = 7, kT12PhShift = 16 };

// One pass's kick layers, as the prep kernel needs them.
struct PassKick {
  KickDesc pre, post;   // enabled = 0: no such layer
  int kind;             // KickKind of the pass
  int c, s, act;        // tile geometry (see PassArgs)
  int tb;               // tile bits (12; 13: dtc_tile13.hip's records 13 + k, 26)
  int lc_layers;        // kShapeLC: layers lc[0 .. lc_layers), site b of layer l kicked
  KickDesc lc[kLcMaxLayers];  // when bit 8 l + b of lc_mask is set (window site b = tile
  uint64_t lc_mask;     // bit 4 + b); Pauli-frame records (kLcCoefs ..)
  int lc_wide;          // the 10-site form: lc_mask bit 10 l + k - 2 = tile bit k of
  int8_t lc_gb[kTileBits];  // layer l, tile bit k = global bit lc_gb[k] (kLcw* records)
  uint64_t lc_mask2;    // lc_wide = 2: bits 64..83 of the 12-site form's mask
};

struct PrepArgs {
  const PassKick* passes;  // [n_pass] (device), or null: use `one`
  PassKick one;
  int n_pass;
  int batch;
  int64_t batch_start;
  int n_traj;
  int64_t traj_offset;
  const double2* kick;     // [n_periods][L_kick][n_sub][4]
  int n_sub;
  int L_kick;              // sites per kick-table row (logical chain length)
  int L_real;              // physical sites of the state
  const int* site_of;      // physical index bit -> logical site (sharded states); null = identity
  uint32_t thr1, thr2, thr3;
  uint64_t seed;
  int noisy;
  // device-like noise (null = depolarizing only): per logical site, Pauli
  // thresholds [L][3], amplitude-damping jump threshold [L], and the
  // importance-weighted Kraus factors [L][3] = (K0 00, K0 11, K1 01)
  const uint32_t* dev_thr;
  const uint32_t* dev_thr_jump;
  const double* dev_kraus;
  KickRec* out;            // [n_pass][batch][kRecPerState]
};

// One streaming pass over a batch of states.  A tile covers index bits
// [0, c) ∪ [s, s + 12 - c); tile bit k < c is global bit k, tile bit k >= c is
// global bit s + k - c.  The pass applies, in order:
//   pre-kick on the active tile bits -> diagonal D or D^* -> (measure) ->
//   post-kick on the active tile bits
// (any part optional), so one pass can finish period p on its sites, close
// the period with the diagonal and start period p+1 ("K-D-K" pass).
struct PassArgs {
  const double2* src;      // batch base, state b at src + b * state_len
  double2* dst;            // may alias src (in-place)
  int64_t state_len;       // 2^L_eff
  int L_eff;               // padded number of index bits (>= kTileBits)
  int L_real;              // physical sites
  int c, s;                // tile geometry
  int tile_bits_mid;       // s - c  (tile-id bits deposited at [c, s))
  int tile_bits;           // 12 (dtc_kernels.hip), 13 (dtc_tile13.hip: c = 13, the
                           // low 13-site group of the 13 / 7 split)
  int act;                 // active tile-bit mask (sites kicked by this pass)
  // batch -> instance: inst = (batch_start + b) / n_traj
  int batch;               // states in this launch
  int64_t batch_start;
  int n_traj;
  const KickRec* recs;     // [batch][kRecPerState] of this pass (prep kernel)
  // diagonal factor tables, per instance: n_chunks chunk tables then one
  // 64-entry window table per start bit g0 = 0 .. L_eff-1
  const double2* diag;
  int n_chunks;
  int diag_stride;         // double2 entries per instance
  // measurement
  int diag_conj;           // apply D^* instead of D
  int meas;                // MeasMode
  int probe;
  int meas_at_end;         // measure after the post-kick instead of after the diagonal
  int n_obs;               // kMeasProbe: 2; kMeasSites: 1 + L_real; kMeasEnergy: 4 L_real
  int meas_parts;          // kMeasEnergy: MeasPart bits
  int no_store;            // measure only: the tile is not written back (dst unused)
  int lc_layers;           // kShapeLC: kick layers; lc_mask bit 8 l + b = site b of layer l
  uint64_t lc_mask;
  const double2* lc_diag;  // kShapeLC: cone diagonals, [n_inst][kLcTab]
  int lc_wide;             // kShapeLC: the 10-site form (dtc_lcw_final), tile bit k =
  int8_t lc_gb[kTileBits]; // global bit lc_gb[k]; 2: the 12-site form (dtc_lcw3_final)
  uint64_t lc_mask2;       // lc_wide = 2: bits 64..83 of its mask
  int zx_reg, zx_lane;      // kMeasEnergy: the bond between register bit zx_reg and lane
                           // bit zx_lane of the measured layout (-1: none), host-computed
  double* partial;         // [B][n_tiles][n_obs]
  const int64_t* basis;    // kick-only passes: non-null = the source is the basis state
                           // |basis[b]> (synthesised in registers: src is not read)
  int octet_bits;          // state layout in HBM (state_addr below); 0 = contiguous
  int lc_split, lc_tpb;    // light-cone pass variant (dev A/B, read once in dtc_open)
  int kdk_split;           // K-D-K at three workgroups per CU (dtc_kdk_pass3): bit NIBS for
                           // measurement classes 0/1, bit 8 + NIBS for 2/3
  // non-null: a dual pass (dtc_kdk_dual) -- the tile after the pre-kick also
  // takes recs2's post-kick (the echo chain's first layer) and goes to dst2
  const KickRec* recs2;
  double2* dst2;
  uint64_t* dbg_ts;        // development builds (-DDTC_PHASE_TIMING) only; null otherwise
};

// Where amplitude x of state b of a batch lives (in amplitudes from the batch
// base).  octet_bits g = 0: b * state_len + x (contiguous states).  g > 0:
// the states of an octet (b >> 3) are interleaved in runs of 2^g amplitudes,
//   (b >> 3) * 8 * state_len + (b & 7) * 2^g + spread(x),
//   spread(x) = ((x >> g) << (g + 3)) | (x & (2^g - 1)),
// and the launch deals the eight states of an octet to consecutive blocks
// (grid.x = 8 * tiles, grid.y = octets), i.e. one per XCD: the eight XCDs'
// concurrent tiles then cover whole 8 * 2^g runs of memory instead of each
// XCD streaming its own 64 KiB tiles (tools/tile_shape_bench.hip,
// tools/pass_pattern_bench.hip: the 12-site pass's access pattern 6.2 -> 6.5
// TB/s, the 8-site pass's 5.45 -> 5.85 at g = 6).  spread is linear over
// disjoint bit sets, so per-register and per-lane offsets spread separately.
__host__ __device__ __forceinline__ int64_t octet_spread(int64_t x, int g) {
  return g ? (((x >> g) << (g + 3)) | (x & (((int64_t)1 << g) - 1))) : x;
}
__host__ __device__ __forceinline__ int64_t state_base(int64_t b, int64_t state_len, int g) {
  return g ? (((b >> 3) << 3) * state_len + ((b & 7) << g)) : b * state_len;
}
// states a batch buffer of n states must hold (octets are padded to 8)
__host__ __device__ __forceinline__ int64_t octet_padded(int64_t n, int g) {
  return g ? ((n + 7) & ~(int64_t)7) : n;
}

// Kick records of n_pass passes x batch states.
hipError_t launch_prep(const PrepArgs& a, hipStream_t stream);

// act must cover nibble sets {2}, {1,2} or {0,1,2}; L_eff in [12, 32].
// lc_variant (kShapeLC passes, nullable): which light-cone kernel ran
// (kLcVariant* below)
hipError_t launch_pass(const PassArgs& a, int batch, int shape, int kind, hipStream_t stream,
                       int* lc_variant = nullptr);

// Passes over a 13-site group at tile bits 0..12 (dtc_tile13.hip; tile_bits 13,
// c = 13): K-D-K, K-D, D-K, K, D shapes, factored RX / RY kicks, the probe
// measurement at most, no dual pass, no basis source.
hipError_t launch_pass13(const PassArgs& a, int batch, int shape, int kind, hipStream_t stream);

// kShapeLC passes (dtc_lightcone.hip), from launch_pass with its grid
enum LcVariant { kLcVariant8 = 0, kLcVariantWide = 1, kLcVariantWide2 = 2, kLcVariantWide3 = 3 };
hipError_t launch_lightcone(const PassArgs& a, dim3 grid, int kind, hipStream_t stream,
                            int* variant);

// out[b * out_stride + o] = sum over tiles of partial[b][tile][o_first + o],
// o < n_out (fixed order); accumulate: += instead of =.  Large states
// (reduce_splits(n_tiles) > 1) sum in two stages, split sums into `scratch`
// ([batch][splits][n_out] doubles): the order depends on n_tiles only, so a
// state's result does not depend on the batch it ran in.
__host__ __device__ constexpr int reduce_splits(int n_tiles) { return n_tiles >= 1024 ? n_tiles / 512 : 1; }
hipError_t launch_reduce(const double* partial, int n_tiles, int n_obs, int batch,
                         double* out, int64_t out_stride, hipStream_t stream,
                         int o_first = 0, int n_out = -1, int accumulate = 0,
                         double* scratch = nullptr);

// Per-instance trajectory sums of a batch's per-state rows: vals [nb][cols],
// state b of instance (batch_start + b) / n_traj; out [instances of the
// batch, first = batch_start / n_traj][cols] (fixed summation order).
hipError_t launch_traj_sum(const double* vals, int nb, int cols, int64_t batch_start, int n_traj,
                           double* out, hipStream_t stream);

// amplitude idx[b] of state b = 1 (after the caller zeroed the batch), in the
// batch layout of octet_bits (state_base / octet_spread)
hipError_t launch_set_basis(double2* state, int64_t state_len, const int64_t* idx,
                            int batch, hipStream_t stream, int octet_bits = 0);

// A kick-only pass over the W^2 slice pieces of 2^k_bits shards (batch
// b = r W + c, contiguous, in place) that stores piece (r, c) at (c, r): the
// slice's last pre-exchange kick fused with the in-place all-to-all below.
// Unitary kick kinds (RX, RY, general) only.
hipError_t launch_kick_swap(const PassArgs& a, int k_bits, int kind, hipStream_t stream);

// Virtual ranks' in-place all-to-all of one slice: 2^k shards of 2^nl
// amplitudes, chunk = top k local bits, slice = the next nl - k - nsub bits;
// piece (shard r, chunk c, slice) <-> piece (shard c, chunk r, slice), r != c.
// Requires nsub >= 10 (1024 amplitudes per workgroup).
hipError_t launch_exchange_swap(double2* state, int nl, int k, int nsub, int slice,
                                hipStream_t stream);

}  // namespace dtc
