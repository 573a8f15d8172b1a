// dtc_engine.cpp — host-side engine behind the C ABI (include/dtc.h).
//
// Replaces the reference's per-circuit loop
//   for inst: for t in range(T): qc_qiskit(...) -> backend.run(...)
//   (fast.py:217-239, 124-214)
// with one schedule over a batch of state vectors resident in HBM:
//   forward trajectory  F: init -> period 1 -> period 2 -> ...   (measure at each t)
//   echo branch at t    E: F(t) -> U^-1_p ... U^-1_1             (measure at the end)
// so the forward sweep costs T-1+t_offset periods per trajectory instead of
// sum_t t, and each echo point branches off the forward prefix (same
// per-t marginal distribution as the reference's independent circuits).
//
// Both sweeps are "layer chains" X_0 D X_1 D ... (X = a layer of single-site
// kicks, D = the RZZ/RZ diagonal or its conjugate).  The sites are split in
// groups that fit a tile; the scheduler (next_pass) emits passes that each
// finish the pending kick layer on one group, apply D if that completed the
// layer on every group, and start the next layer on the same group.  With two
// groups (L <= 21) every pass applies one D: one HBM round trip per period.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/dtc.h"
#include "dtc_kernels.h"
#include "dtc_rng.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define DTC_HIP(expr)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      return fail(e_ == hipErrorOutOfMemory ? DTC_ENOMEM : DTC_EHIP,                    \
                  std::string(#expr) + ": " + hipGetErrorString(e_));                   \
  } while (0)

#define DTC_TRY(expr)        \
  do {                       \
    int rc_ = (expr);        \
    if (rc_ != DTC_OK) return rc_; \
  } while (0)

struct DevBuf {
  void* p = nullptr;
  size_t n = 0;
};

// Pinned host staging for the per-trajectory results copied back after a
// batch (direct DMA, no zero-filled pageable vector per call).
struct HostBuf {
  double* p = nullptr;
  size_t n = 0;  // doubles
};


struct Group {
  int c, s;  // tile = bits [0, c) + [s, s + tb - c)
  int act;   // active tile-bit mask
  int tb = dtc::kTileBits;  // tile bits: 12, or 13 (the 13-site group, dtc_tile13.hip)
};

struct Pending {
  int kind;
  hipEvent_t e0, e1;
  double bytes;
};

}  // namespace

struct dtc_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  DevBuf F, E, partial, vals_f, vals_e, diag, kick, basis, sitemap;
  DevBuf lc_diag;  // cone diagonals of the light-cone pass, [n_inst][kLcTab]
  DevBuf red_scratch;  // split sums of the two-stage tile reduction (large states)
  DevBuf recs, recs1, pk;               // kick records (batch schedule / single pass), pass list
  DevBuf dev_thr, dev_jump, dev_kraus;  // device-like noise tables (dtc_autocorr_device)
  std::vector<dtc::PassKick> pk_host;   // staged pass list (alive until the stream syncs)
  // forward prefix (dtc_prefix_build): every trajectory's state after
  // prefix_periods periods, and what it was built from
  DevBuf prefix;
  std::vector<int64_t> prefix_masks;
  int prefix_periods = -1;  // -1: none
  int64_t prefix_states = 0, prefix_traj_offset = 0, prefix_len = 0;
  int prefix_n_traj = 0, prefix_device = 0;
  uint64_t prefix_hash = 0;
  bool prof = false;
  // options fixed at dtc_open (environment read once there; development A/B
  // switches, documented in DESIGN.md): batch state layout, light-cone pass
  // variant, the basis-synthesising first pass, the light-cone merge, batch
  // memory budget, verbose batch report
  int octet_bits = 6;        // DTC_OCTET_BITS (0 = contiguous states)
  int lc_split = 1;          // DTC_LC_SPLIT
  int lc_tpb = 0;            // DTC_LC_TPB (0 = default)
  bool lc_wide = true;       // DTC_NO_LCW unset: five-pass (10-site) light-cone ends
  bool lc_wide3 = true;      // DTC_NO_LCW3 unset: six-pass (12-site) ends where they fit
  HostBuf host_f, host_e;    // pinned result staging (autocorr / energy)
  uint64_t tables_key = 0;   // upload_tables: the problem whose tables are in place
  bool tables_valid = false;
  // DTC_KDK_SPLIT: which K-D-K passes run three workgroups per CU (dtc_kernels.h
  // PassArgs::kdk_split): the 12-site probe passes, every per-site/energy pass
  int kdk_split = (1 << 7) | (1 << (8 + 7)) | (1 << (8 + 6));
  bool basis_synth = true;   // DTC_NO_BASIS_SYNTH
  bool lightcone = true;     // DTC_NO_LIGHTCONE
  double batch_bytes = 0.0;  // DTC_BATCH_BYTES (0 = automatic)
  bool verbose = false;      // DTC_VERBOSE
  int prefix_octet = 0;      // layout the prefix states were built in
  int64_t st_n[DTC_KERNEL_KINDS] = {};
  int64_t lc_launches[4] = {};  // light-cone passes by kernel (dtc_lightcone_counts)
  bool dual = true;  // DTC_NO_DUAL: echo chains start with a pass of their own
  bool runahead = true;  // DTC_NO_RUNAHEAD: device-noise forward closes periods with K-D
  // DTC_SPLIT13=1: L = 20 sweeps run the 13 / 7 site groups (round 6: built
  // and parity-tested, slower than the 12 / 8 split on the power-capped chip,
  // profiles/r6q_*; the 12 / 8 split stays the default)
  bool split13 = false;
  int64_t sched_counts[4] = {};  // dtc_schedule_counts: folds, run-ahead, rebuilt, 13 / 7
  double st_ms[DTC_KERNEL_KINDS] = {};
  double st_bytes[DTC_KERNEL_KINDS] = {};
  std::vector<Pending> pending;
  std::vector<hipEvent_t> pool;
  // sharded state (dtc_shard_*): device tables per bit map, cached so that
  // the asynchronous steps of a sweep never re-upload from host memory
  struct ShardTables {
    uint64_t key = 0;
    DevBuf diag;
  };
  std::vector<ShardTables> shard_cache;  // most recent last, at most 4
  std::vector<ShardTables> shard_maps;   // bit -> site maps (diag = the map), at most 4
  DevBuf shard_kick;
  uint64_t shard_kick_key = 0;
};

namespace {

int ensure(DevBuf& b, size_t bytes) {
  if (bytes == 0) bytes = 16;
  if (b.n >= bytes) return DTC_OK;
  if (b.p) {
    (void)hipFree(b.p);
    b.p = nullptr;
    b.n = 0;
  }
  DTC_HIP(hipMalloc(&b.p, bytes));
  b.n = bytes;
  return DTC_OK;
}

int ensure_host(HostBuf& b, size_t n) {
  if (n == 0) n = 1;
  if (b.n >= n) return DTC_OK;
  if (b.p) (void)hipHostFree(b.p);
  b.p = nullptr;
  b.n = 0;
  DTC_HIP(hipHostMalloc((void**)&b.p, n * sizeof(double), hipHostMallocDefault));
  b.n = n;
  return DTC_OK;
}

void release(DevBuf& b) {
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.n = 0;
}

hipEvent_t get_event(dtc_ctx* ctx) {
  if (!ctx->pool.empty()) {
    hipEvent_t e = ctx->pool.back();
    ctx->pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}

int resolve_pending(dtc_ctx* ctx) {
  for (auto& p : ctx->pending) {
    float ms = 0.f;
    DTC_HIP(hipEventSynchronize(p.e1));
    DTC_HIP(hipEventElapsedTime(&ms, p.e0, p.e1));
    ctx->st_n[p.kind] += 1;
    ctx->st_ms[p.kind] += ms;
    ctx->st_bytes[p.kind] += p.bytes;
    ctx->pool.push_back(p.e0);
    ctx->pool.push_back(p.e1);
  }
  ctx->pending.clear();
  return DTC_OK;
}

// Profiling: a call leaves its launches' events pending (resolving them costs
// an elapsed-time query per launch while the GPU idles between calls); they
// are resolved by dtc_kernel_stats / dtc_reset_stats, or here once many wait.
int settle_pending(dtc_ctx* ctx) {
  return ctx->pending.size() > 16384 ? resolve_pending(ctx) : DTC_OK;
}

struct Plan {
  int L = 0, L_eff = 0, n_chunks = 0, n_tiles = 0, diag_stride = 0;
  int64_t len = 0;
  std::vector<Group> groups;
};

// Site groups: group 0 = sites [0, a0) in a contiguous 4096-amplitude tile;
// further groups take up to `hi_max` sites each (tile = 12 - a column bits of
// >= 128-B rows + the group's sites).  Defaults: 11 + 9 for L = 20.
// Site groups: the low group (tile bits 0..11 = sites 0..a_lo-1) and higher
// groups of a sites each (tile = a_lo.. column bits 0..c-1 + the group's a
// sites, c = 12 - a).  Sizes are chosen so that the register nibble the
// diagonal is applied in never straddles the column boundary c (kernel
// diag_in: one window-table lookup per amplitude): the low group holds 9..12
// sites, a higher group 9, 8 or 4 (c = 3, 4, 8).  Fewest groups first, then
// the largest low group, then the largest higher groups.
// largest_top (sharded states): the high groups in increasing size, so the
// group holding the top bits (the bits an exchange swaps with the rank bits)
// is a large one and the pre-exchange kicks stay below a few free bits of it
// (the slices of dtc_shard_kick_slice).
// split13 (round 6, L = 20 only): a 13-site group at tile bits 0..12
// (dtc_tile13.hip) and a 7-site column group, tile bits 0..4 + sites 13..19
// (pass_body kGeoB7) -- the column pass kicks 7 sites over 512-B runs instead
// of 8 over 256-B runs (tools/tile13_kdk_probe.hip, profiles/r6c_*).
// pl.n_tiles is then the larger group's tile count (buffer sizes); a pass's
// own is 2^(L_eff - tb).
Plan make_plan(int L, bool largest_top = false, bool split13 = false) {
  Plan pl;
  pl.L = L;
  pl.L_eff = std::max(L, dtc::kTileBits);
  pl.len = (int64_t)1 << pl.L_eff;
  pl.n_tiles = 1 << (pl.L_eff - dtc::kTileBits);
  pl.n_chunks = (pl.L_eff + dtc::kChunkBits - 1) / dtc::kChunkBits;
  pl.diag_stride = (pl.n_chunks + pl.L_eff) * 64;
  if (split13 && L == 20) {
    pl.groups.push_back(Group{dtc::kMaxTileBits, dtc::kMaxTileBits, (1 << dtc::kMaxTileBits) - 1,
                              dtc::kMaxTileBits});
    pl.groups.push_back(Group{dtc::kB7Cols, dtc::kMaxTileBits, 0xFE0, dtc::kTileBits});
    return pl;
  }
  if (L <= dtc::kTileBits) {
    // one group; the padding sites L..11 get identity kicks (kernel) so the
    // whole 12-bit tile runs the standard round plan
    pl.groups.push_back(Group{0, 0, (1 << dtc::kTileBits) - 1});
    return pl;
  }
  static const int kHi[3] = {9, 8, 4};
  for (int n_hi = (L - dtc::kTileBits + 8) / 9;; ++n_hi) {
    for (int a_lo = dtc::kTileBits; a_lo >= 9; --a_lo) {
      const int need = L - a_lo;
      // n9 nines, n8 eights, the rest fours
      for (int n9 = n_hi; n9 >= 0; --n9) {
        for (int n8 = n_hi - n9; n8 >= 0; --n8) {
          const int n4 = n_hi - n9 - n8;
          if (9 * n9 + 8 * n8 + 4 * n4 != need) continue;
          pl.groups.push_back(Group{0, 0, (1 << a_lo) - 1});
          int s = a_lo;
          for (int kk = 0; kk < 3; ++kk) {
            const int k = largest_top ? 2 - kk : kk;
            const int cnt = k == 0 ? n9 : (k == 1 ? n8 : n4);
            for (int i = 0; i < cnt; ++i) {
              const int a = kHi[k], c = dtc::kTileBits - a;
              pl.groups.push_back(Group{c, s, ((1 << a) - 1) << c});
              s += a;
            }
          }
          return pl;
        }
      }
    }
  }
}

// Diagonal factor tables (RZZ even/odd bonds + RZ, fast.py:115-120):
// D(x) = exp(-i/2 (sum_i h_i z_i + sum_i phi_i z_i z_{i+1})), z_i = 1 - 2 bit_i(x).
// Per instance: n_chunks chunk tables, D(x) = prod_k C_k[(x >> 5k) & 63] (C_k covers
// sites 5k..5k+4 and the bond to site 5k+5 = index bit 5), followed by one window
// table W_g0[v] per start bit g0, v = bits [g0-1, g0+5) of x, holding the terms of
// sites g0..g0+3 and of every bond touching them (the kernel factors
// D(x) = D(x0) / W(x0) * W(x) over the 16 amplitudes of a thread).
double diag_angle(int L, const double* hh, const double* pp, int lo_site, int hi_site,
                  int bond_lo, int bond_hi, int bit0, int v) {
  auto z = [&](int i) -> double { return ((v >> (i - bit0)) & 1) ? -1.0 : 1.0; };
  double ang = 0.0;
  for (int i = lo_site; i < hi_site && i < L; ++i) ang += hh[i] * z(i);
  for (int i = std::max(bond_lo, 0); i < bond_hi && i + 1 < L; ++i) ang += pp[i] * z(i) * z(i + 1);
  return ang;
}

void build_diag_tables(const Plan& pl, int n_inst, const double* h, const double* phi,
                       std::vector<double>& out, const double* const_angle = nullptr) {
  const int L = pl.L;
  out.assign((size_t)n_inst * pl.diag_stride * 2, 0.0);
  for (int in = 0; in < n_inst; ++in) {
    const double* hh = h + (size_t)in * L;
    const double* pp = phi + (size_t)in * (L > 1 ? L - 1 : 0);
    double* o = out.data() + (size_t)in * pl.diag_stride * 2;
    auto put = [&](int e, double ang) {
      o[e * 2] = std::cos(-0.5 * ang);
      o[e * 2 + 1] = std::sin(-0.5 * ang);
    };
    for (int k = 0; k < pl.n_chunks; ++k) {
      const int b0 = dtc::kChunkBits * k;
      const double c0 = (k == 0 && const_angle) ? const_angle[in] : 0.0;
      for (int v = 0; v < 64; ++v)
        put(k * 64 + v, c0 + diag_angle(L, hh, pp, b0, b0 + dtc::kChunkBits, b0,
                                        b0 + dtc::kChunkBits, b0, v));
    }
    for (int g0 = 0; g0 < pl.L_eff; ++g0) {
      for (int v = 0; v < 64; ++v) {
        if (g0 == 0 && (v & 1)) continue;  // bit -1 does not exist
        put((pl.n_chunks + g0) * 64 + v,
            diag_angle(L, hh, pp, g0, g0 + 4, g0 - 1, g0 + 4, g0 - 1, v));
      }
    }
  }
}

struct RunCfg {
  const dtc_problem* prob;
  Plan pl;
  std::vector<int> row_kind;  // KickKind of every kick-table row
  uint64_t seed;
  int64_t traj_offset;
  int n_traj;
  int noisy;
  uint32_t thr1, thr2, thr3;
  const int* site_of = nullptr;  // device: physical bit -> logical site (shards)
  int octet_bits = 0;            // batch state layout (dtc_kernels.h state_base)
  // sharded state: the tables live in ctx->shard_cache / shard_kick, and a
  // chunk pass covers the low L_eff_override bits of states stride_override apart
  const double2* diag_tab = nullptr;
  const double2* kick_tab = nullptr;
  int L_eff_override = 0;
  int64_t stride_override = 0;
  // device-like noise (dtc_autocorr_device): general non-unitary kicks, no
  // forward pass runs ahead of a branch point (a jump cannot be undone)
  bool device = false;
  std::vector<uint32_t> dev_thr_host;  // [L][3] per-site Pauli thresholds (prep X)
  const uint32_t* dev_thr = nullptr;   // device copies
  const uint32_t* dev_jump = nullptr;
  const double* dev_kraus = nullptr;
};

// ---- layer chains ---------------------------------------------------------
using dtc::KickDesc;

KickDesc no_kick() { return KickDesc{0, 0, 0, 0u, 0u}; }

struct Chain {
  std::vector<KickDesc> X;  // kick layers X_0..X_n
  bool trailing_d = false;  // a D after X_n too
  int diag = dtc::kDiagFwd;
  std::vector<int> kc;      // layers applied per group
  int nd = 0;               // diagonals applied
  bool post_after_d = true; // a pass that applies D may start the next layer
  std::vector<int> prio;    // tie-break between groups with equal kc (lower first); empty = index
  int n() const { return (int)X.size() - 1; }
  int n_d() const { return trailing_d ? n() + 1 : n(); }
  bool done() const {
    if (nd != n_d()) return false;
    for (int k : kc)
      if (k != n() + 1) return false;
    return true;
  }
};

struct PassSpec {
  int group;
  KickDesc pre, post;
  int diag;    // DiagMode
  int d_index; // diagonals applied after this pass (valid when diag)
  // light-cone end of an echo chain (kShapeLC): tile = bits 0..3 + sites
  // lc_w0..lc_w0+7; layers lc[0] D* lc[1] ... D* lc[lc_layers-1] on the window
  // sites of lc_mask (bit 8 l + b: site lc_w0 + b in layer l), then the probe
  int lc_w0 = -1;
  int lc_layers = 0;
  KickDesc lc[dtc::kLcMaxLayers] = {};
  uint64_t lc_mask = 0;
  // the 10-site form (lc_merge_wide): tile bit k = global bit lc_gb[k], lc_mask
  // bit 10 l + k - 2 = tile bit k kicked in layer l
  int lc_wide = 0;
  int8_t lc_gb[dtc::kTileBits] = {};
  // the 12-site form (lc_wide = 2, lc_merge_wide7): tile bit k = global bit
  // j-5+k, bit 12 l + k of the 84-bit mask lc_mask | lc_mask2 << 64
  uint64_t lc_mask2 = 0;
};

// the tile bits a light-cone pass kicks in layer l (nonzero: the layer runs)
uint64_t lc_layer_bits(const PassSpec& ps, int l) {
  if (ps.lc_wide == 2) {
    uint64_t m = 0;
    for (int k = 0; k < dtc::kTileBits; ++k) {
      const int bit = 12 * l + k;
      const uint64_t on = bit < 64 ? (ps.lc_mask >> bit) & 1ull : (ps.lc_mask2 >> (bit - 64)) & 1ull;
      m |= on << k;
    }
    return m;
  }
  return ps.lc_wide ? (ps.lc_mask >> (10 * l)) & 0x3FFull
                    : (ps.lc_mask >> (dtc::kLcSites * l)) & 0xFFull;
}

// The tile geometry of a pass (the plan's group, or the light-cone window).
Group pass_group(const Plan& pl, const PassSpec& ps) {
  if (ps.lc_w0 >= 0) return Group{4, ps.lc_w0, 0xFF0};
  return pl.groups[ps.group];
}

// Emit the next pass of a chain (greedy, deterministic).
PassSpec next_pass(Chain& ch) {
  int G = 0;
  for (int g = 1; g < (int)ch.kc.size(); ++g) {
    const int pg = ch.prio.empty() ? g : ch.prio[g], pG = ch.prio.empty() ? G : ch.prio[G];
    if (ch.kc[g] < ch.kc[G] || (ch.kc[g] == ch.kc[G] && pg < pG)) G = g;
  }
  PassSpec ps{G, no_kick(), no_kick(), dtc::kDiagNone, ch.nd};
  const int n = ch.n();
  if (ch.kc[G] == ch.nd && ch.kc[G] <= n) ps.pre = ch.X[ch.kc[G]++];
  bool level = true;
  for (int k : ch.kc)
    if (k != ch.nd + 1) level = false;
  if (level && ch.nd < ch.n_d()) {
    ps.diag = ch.diag;
    ps.d_index = ++ch.nd;
    if (ch.post_after_d && ch.kc[G] == ch.nd && ch.kc[G] <= n) ps.post = ch.X[ch.kc[G]++];
  }
  return ps;
}

dtc::PassArgs base_args(dtc_ctx* ctx, const RunCfg& rc, int64_t batch_start) {
  dtc::PassArgs A{};
  A.state_len = rc.stride_override ? rc.stride_override : rc.pl.len;
  A.L_eff = rc.L_eff_override ? rc.L_eff_override : rc.pl.L_eff;
  A.L_real = rc.pl.L;
  A.batch_start = batch_start;
  A.n_traj = rc.n_traj;
  A.diag = rc.diag_tab ? rc.diag_tab : (const double2*)ctx->diag.p;
  A.n_chunks = rc.pl.n_chunks;
  A.diag_stride = rc.pl.diag_stride;
  A.probe = rc.prob->probe_site;
  A.partial = (double*)ctx->partial.p;
  A.octet_bits = rc.octet_bits;
  A.lc_split = ctx->lc_split;
  A.lc_tpb = ctx->lc_tpb;
  A.kdk_split = ctx->kdk_split;
#ifdef DTC_PHASE_TIMING
  if (const char* e = std::getenv("DTC_DBG_PTR")) A.dbg_ts = (uint64_t*)std::strtoull(e, nullptr, 0);
#endif
  return A;
}

dtc::PrepArgs prep_args(dtc_ctx* ctx, const RunCfg& rc, int64_t batch_start, int batch) {
  dtc::PrepArgs P{};
  P.batch = batch;
  P.batch_start = batch_start;
  P.n_traj = rc.n_traj;
  P.traj_offset = rc.traj_offset;
  P.kick = rc.kick_tab ? rc.kick_tab : (const double2*)ctx->kick.p;
  P.n_sub = rc.prob->n_sub;
  P.L_kick = rc.prob->L;
  P.L_real = rc.pl.L;
  P.site_of = rc.site_of;
  P.thr1 = rc.thr1;
  P.thr2 = rc.thr2;
  P.thr3 = rc.thr3;
  P.seed = rc.seed;
  P.noisy = rc.noisy;
  P.dev_thr = rc.dev_thr;
  P.dev_thr_jump = rc.dev_jump;
  P.dev_kraus = rc.dev_kraus;
  return P;
}

int launch_reduce_prof(dtc_ctx* ctx, int n_tiles, int n_obs, int batch, double* out,
                       int64_t out_stride, int o_first = 0, int n_out = -1,
                       int accumulate = 0) {
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (ctx->prof) {
    e0 = get_event(ctx);
    e1 = get_event(ctx);
    DTC_HIP(hipEventRecord(e0, ctx->stream));
  }
  double* scratch = nullptr;
  if (dtc::reduce_splits(n_tiles) > 1) {
    // split sums of a large state's tiles ([batch][splits][n_out])
    const int no = n_out < 0 ? n_obs - o_first : n_out;
    const size_t need = (size_t)batch * dtc::reduce_splits(n_tiles) * no * sizeof(double);
    if (ctx->red_scratch.n < need) {
      DTC_HIP(hipStreamSynchronize(ctx->stream));  // the previous scratch may be in use
      DTC_TRY(ensure(ctx->red_scratch, need));
    }
    scratch = (double*)ctx->red_scratch.p;
  }
  DTC_HIP(dtc::launch_reduce((const double*)ctx->partial.p, n_tiles, n_obs, batch, out,
                             out_stride, ctx->stream, o_first, n_out, accumulate, scratch));
  if (ctx->prof) {
    DTC_HIP(hipEventRecord(e1, ctx->stream));
    ctx->pending.push_back(
        Pending{DTC_KERNEL_REDUCE, e0, e1,
                8.0 * (double)n_tiles * (n_out < 0 ? n_obs - o_first : n_out) * batch});
  }
  return DTC_OK;
}

// Shape and matrix family of a pass.
int pass_shape(const PassSpec& ps) {
  if (ps.lc_w0 >= 0) return dtc::kShapeLC;
  const bool has_d = ps.diag != dtc::kDiagNone;
  if (ps.pre.enabled && has_d && ps.post.enabled) return dtc::kShapeKDK;
  if (ps.pre.enabled && has_d) return dtc::kShapeKD;
  if (has_d && ps.post.enabled) return dtc::kShapeDK;
  if (ps.pre.enabled && !has_d && !ps.post.enabled) return dtc::kShapeK;
  if (has_d) return dtc::kShapeD;
  return -1;
}

int pass_kind(const RunCfg& rc, const PassSpec& ps, int shape) {
  int kind = shape == dtc::kShapeD ? dtc::kKindRX : -1;
  std::vector<const KickDesc*> ks{&ps.pre, &ps.post};
  for (int l = 0; l < ps.lc_layers; ++l)
    if (lc_layer_bits(ps, l)) ks.push_back(&ps.lc[l]);
  for (const KickDesc* k : ks) {
    if (!k->enabled) continue;
    const bool basis_x = k->mode == dtc::kKickBasisX || k->mode == dtc::kKickUndoBasisX;
    int rk = basis_x ? dtc::kKindGen : rc.row_kind[k->row];
    // device-like noise: Kraus x Pauli x gate is not unitary; with one
    // sub-gate per kick it is a real diagonal times a unitary of the family
    // (SiteMat in dtc_kernels.hip: factored, the diagonal deferred); Kraus
    // factors between sub-gates, or a dagger (undo) putting the diagonal on
    // the right, leave only the general form
    if (rc.device && (rk == dtc::kKindRX || rk == dtc::kKindRY)) {
      const bool left_diag = rc.prob->n_sub == 1 && k->mode != dtc::kKickUndo &&
                             k->mode != dtc::kKickUndoBasisX;
      rk = !left_diag ? dtc::kKindGen : (rk == dtc::kKindRX ? dtc::kKindRXU : dtc::kKindRYU);
    }
    kind = (kind < 0 || kind == rk) ? rk : dtc::kKindGen;
  }
  return kind;
}

dtc::PassKick pass_kick(const RunCfg& rc, const PassSpec& ps) {
  const Group g = pass_group(rc.pl, ps);
  dtc::PassKick pk{};
  pk.pre = ps.pre;
  pk.post = ps.post;
  pk.lc_layers = ps.lc_layers;
  for (int l = 0; l < dtc::kLcMaxLayers; ++l) pk.lc[l] = ps.lc[l];
  pk.lc_mask = ps.lc_mask;
  pk.lc_mask2 = ps.lc_mask2;
  pk.lc_wide = ps.lc_wide;
  for (int k = 0; k < dtc::kTileBits; ++k) pk.lc_gb[k] = ps.lc_gb[k];
  pk.kind = pass_kind(rc, ps, pass_shape(ps));
  pk.c = g.c;
  pk.s = g.s;
  pk.act = g.act;
  pk.tb = g.tb;
  return pk;
}

// Launch one pass whose kick records are `recs` ([batch][kRecPerState]; null:
// build them first with a one-pass prep launch); if meas_mode != none, reduce
// its observables into meas_out.
int launch_pass_spec(dtc_ctx* ctx, const RunCfg& rc, int64_t batch_start, int batch,
                     const PassSpec& ps, const double2* src, double2* dst, int meas_mode,
                     int meas_at_end, int n_obs, double* meas_out, int64_t meas_stride,
                     const dtc::KickRec* recs = nullptr, int meas_parts = 0,
                     int no_store = 0, const int64_t* basis = nullptr, int swap_k = 0,
                     const dtc::KickRec* recs2 = nullptr, double2* dst2 = nullptr) {
  const int shape = pass_shape(ps);
  if (shape < 0) return fail(DTC_EINVAL, "internal: empty pass");
  const int kind = pass_kind(rc, ps, shape);
  if (!recs) {
    DTC_TRY(ensure(ctx->recs1, (size_t)batch * dtc::kRecPerState * sizeof(dtc::KickRec)));
    dtc::PrepArgs P = prep_args(ctx, rc, batch_start, batch);
    P.passes = nullptr;
    P.one = pass_kick(rc, ps);
    P.n_pass = 1;
    P.out = (dtc::KickRec*)ctx->recs1.p;
    DTC_HIP(dtc::launch_prep(P, ctx->stream));
    recs = P.out;
  }
  dtc::PassArgs A = base_args(ctx, rc, batch_start);
  const Group g = pass_group(rc.pl, ps);
#ifdef DTC_PHASE_TIMING
  if (const char* e = std::getenv("DTC_DBG_GROUP"))
    if (std::atoi(e) != ps.group) A.dbg_ts = nullptr;
#endif
  A.zx_reg = -1;
  A.zx_lane = -1;
  if (meas_mode == dtc::kMeasEnergy) {
    // the layout the kernel measures Z, ZZ in (RoundPlan::d_lay, or the IO
    // layout at the end): its one bond between a register bit and a lane bit
    const int nibs = ((g.act & 0xF) ? 1 : 0) | ((g.act & 0xF0) ? 2 : 0) | ((g.act & 0xF00) ? 4 : 0);
    const int io = dtc::io_layout(nibs), o = 3 - io;
    const bool n0 = nibs & 1, n_o = (nibs >> o) & 1;
    const bool pre = shape == dtc::kShapeK || shape == dtc::kShapeKD || shape == dtc::kShapeKDK;
    const int lay = meas_at_end ? io : (pre ? (n_o ? o : (n0 ? 0 : io)) : io);
    auto tile_bit = [&](int site) {
      return site < g.c ? site : ((site >= g.s && site < g.s + dtc::kTileBits - g.c) ? g.c + site - g.s : -1);
    };
    for (int i = 0; i + 1 < rc.pl.L; ++i) {
      int reg = -1, lane = -1;
      for (int site : {i, i + 1}) {
        const int tb = tile_bit(site);
        if (tb < 0) continue;
        if (tb >= 4 * lay && tb < 4 * lay + 4) {
          reg = tb - 4 * lay;
        } else {
          const int q = lay == 2 ? tb : (lay == 1 ? (tb < 4 ? tb : tb - 4) : tb - 4);
          if (q < 6) lane = q;
        }
      }
      if (reg >= 0 && lane >= 0) {
        if (A.zx_reg >= 0) return fail(DTC_EINVAL, "internal: two register-lane bonds in one layout");
        A.zx_reg = reg;
        A.zx_lane = lane;
      }
    }
  }
  if (ps.diag != dtc::kDiagNone && g.tb == dtc::kTileBits && g.c != dtc::kB7Cols) {
    // the kernel's diagonal uses the window table of the register nibble it
    // is applied in (RoundPlan::d_lay): that nibble must not straddle c
    // (same rule as RoundPlan: load/store layout IO, other high nibble O)
    const int nibs = ((g.act & 0xF) ? 1 : 0) | ((g.act & 0xF0) ? 2 : 0) | ((g.act & 0xF00) ? 4 : 0);
    const int io = dtc::io_layout(nibs), o = 3 - io;
    const bool n0 = nibs & 1, n_o = (nibs >> o) & 1;
    const bool pre = shape == dtc::kShapeK || shape == dtc::kShapeKD || shape == dtc::kShapeKDK ||
                     shape == dtc::kShapeLC;
    const int tb = 4 * (pre ? (n_o ? o : (n0 ? 0 : io)) : io);
    if (!(tb >= g.c || tb + 4 <= g.c))
      return fail(DTC_EINVAL, "internal: diagonal nibble straddles the column bits");
  }
  A.src = src;
  A.dst = dst;
  // the source is the basis state (synthesised by the kernel): kick-only passes
  if (basis && shape != dtc::kShapeK) return fail(DTC_EINVAL, "internal: basis source on a non-kick pass");
  A.basis = basis;
  A.c = g.c;
  A.s = g.s;
  A.tile_bits_mid = g.s - g.c;
  A.tile_bits = g.tb;
  A.act = g.act;
  A.recs = recs;
  A.diag_conj = ps.diag == dtc::kDiagConj;
#ifdef DTC_DEV_KNOBS
  // development builds, timing probes only (wrong results): DTC_DBG_CONJ=0 / 1
  // runs every diagonal unconjugated / conjugated
  if (const char* e = std::getenv("DTC_DBG_CONJ")) A.diag_conj = std::atoi(e) != 0;
#endif
  A.meas = meas_mode;
  A.meas_at_end = meas_at_end;
  A.meas_parts = meas_parts;
  A.no_store = no_store;
  A.lc_layers = ps.lc_layers;
  A.lc_mask = ps.lc_mask;
  A.lc_mask2 = ps.lc_mask2;
  A.lc_diag = (const double2*)ctx->lc_diag.p;
  A.lc_wide = ps.lc_wide;
  for (int k = 0; k < dtc::kTileBits; ++k) A.lc_gb[k] = ps.lc_gb[k];
  A.batch = batch;
  A.n_obs = n_obs;
  A.recs2 = recs2;
  A.dst2 = dst2;
  if (dst2 && (!recs2 || (shape != dtc::kShapeKDK && shape != dtc::kShapeKD) || no_store || basis))
    return fail(DTC_EINVAL, "internal: a dual pass is a stored K-D-K / K-D with its branch's records");
  const int kernel = no_store ? DTC_KERNEL_FINAL_PASS
                              : (ps.diag != dtc::kDiagNone ? DTC_KERNEL_LO_PASS : DTC_KERNEL_HI_PASS);
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (ctx->prof) {
    e0 = get_event(ctx);
    e1 = get_event(ctx);
    DTC_HIP(hipEventRecord(e0, ctx->stream));
  }
  int lc_variant = -1;
  if (swap_k > 0) {
    // the slice's last pre-exchange kick, stored at the partner piece
    if (shape != dtc::kShapeK || meas_mode != dtc::kMeasNone || basis)
      return fail(DTC_EINVAL, "internal: kick+exchange pass must be a plain kick pass");
    DTC_HIP(dtc::launch_kick_swap(A, swap_k, kind, ctx->stream));
  } else {
    DTC_HIP(dtc::launch_pass(A, batch, shape, kind, ctx->stream, &lc_variant));
  }
  if (lc_variant >= 0 && lc_variant < 4) ++ctx->lc_launches[lc_variant];
  if (ctx->prof) {
    DTC_HIP(hipEventRecord(e1, ctx->stream));
    // algorithmic bytes: a read and a store per amplitude, or one of them
    // (measure-only passes store nothing, a basis-synthesising pass reads nothing)
    const double per_amp = (no_store || basis) ? 16.0 : (dst2 ? 48.0 : 32.0);
    ctx->pending.push_back(Pending{kernel, e0, e1, per_amp * (double)((int64_t)1 << A.L_eff) * batch});
  }
  if (meas_mode != dtc::kMeasNone && meas_out)
    DTC_TRY(launch_reduce_prof(ctx, 1 << (A.L_eff - g.tb), n_obs, batch, meas_out, meas_stride));
  return DTC_OK;
}

// A scheduled pass of a batch (dtc_autocorr builds the whole batch schedule,
// prepares every kick record with one prep launch per segment, then streams
// the passes).
struct Launch {
  PassSpec ps;
  const double2* src;
  double2* dst;
  int meas_mode, meas_at_end, n_obs;
  double* meas_out;
  int64_t meas_stride;
  int no_store = 0;  // the pass's output is never read again (last pass of an echo chain)
  const int64_t* basis = nullptr;  // first pass of a sweep: src = the basis states (synthesised)
  // dual pass (dtc_kdk_dual): ps is a forward K-D-K that also starts an echo
  // chain -- ps2 = {ps's pre-kick, the echo's first kick layer as post}, its
  // tile after the pre-kick, kicked by ps2's post, goes to dst2
  double2* dst2 = nullptr;
  PassSpec ps2{};
};

int run_launches(dtc_ctx* ctx, const RunCfg& rc, int64_t batch_start, int batch,
                 const std::vector<Launch>& L) {
#ifdef DTC_DEV_KNOBS
  // development builds: DTC_PRINT_SCHED=1 lists the batch's schedule on stderr
  if (std::getenv("DTC_PRINT_SCHED")) {
    auto role = [&](const void* p) {
      return p == ctx->F.p ? "F" : (p == ctx->E.p ? "E" : (p ? "?" : "-"));
    };
    for (size_t i = 0; i < L.size(); ++i)
      std::fprintf(stderr, "sched %zu g%d shape%d diag%d pre%d post%d lc%d %s->%s%s meas%d%s%s\n", i,
                   L[i].ps.group, pass_shape(L[i].ps), L[i].ps.diag, L[i].ps.pre.enabled,
                   L[i].ps.post.enabled, L[i].ps.lc_w0, role(L[i].src), role(L[i].dst),
                   L[i].dst2 ? "+E" : "", L[i].meas_mode, L[i].no_store ? " nostore" : "",
                   L[i].basis ? " basis" : "");
  }
#endif
  // one record row per launch, two for a dual pass (its echo branch's kicks)
  std::vector<size_t> row0(L.size() + 1);
  ctx->pk_host.clear();
  for (size_t i = 0; i < L.size(); ++i) {
    row0[i] = ctx->pk_host.size();
    ctx->pk_host.push_back(pass_kick(rc, L[i].ps));
    if (L[i].dst2) ctx->pk_host.push_back(pass_kick(rc, L[i].ps2));
  }
  row0[L.size()] = ctx->pk_host.size();
  const size_t n_rows = ctx->pk_host.size();
  const size_t per_pass = (size_t)batch * dtc::kRecPerState * sizeof(dtc::KickRec);
  const size_t seg = std::max<size_t>(2, std::min<size_t>(n_rows, (size_t)(256u << 20) / per_pass));
  DTC_TRY(ensure(ctx->recs, seg * per_pass));
  DTC_TRY(ensure(ctx->pk, n_rows * sizeof(dtc::PassKick)));
  DTC_HIP(hipMemcpyAsync(ctx->pk.p, ctx->pk_host.data(), n_rows * sizeof(dtc::PassKick),
                         hipMemcpyHostToDevice, ctx->stream));
  // segments of whole launches whose rows fit the record buffer
  for (size_t i0 = 0; i0 < L.size();) {
    size_t i1 = i0;
    while (i1 < L.size() && row0[i1 + 1] - row0[i0] <= seg) ++i1;
    dtc::PrepArgs P = prep_args(ctx, rc, batch_start, batch);
    P.passes = (const dtc::PassKick*)ctx->pk.p + row0[i0];
    P.n_pass = (int)(row0[i1] - row0[i0]);
    P.out = (dtc::KickRec*)ctx->recs.p;
    DTC_HIP(dtc::launch_prep(P, ctx->stream));
    for (size_t i = i0; i < i1; ++i) {
      const Launch& l = L[i];
      const dtc::KickRec* rec = P.out + (row0[i] - row0[i0]) * batch * dtc::kRecPerState;
      DTC_TRY(launch_pass_spec(ctx, rc, batch_start, batch, l.ps, l.src, l.dst, l.meas_mode,
                               l.meas_at_end, l.n_obs, l.meas_out, l.meas_stride, rec, 0,
                               l.no_store, l.basis, 0,
                               l.dst2 ? rec + batch * dtc::kRecPerState : nullptr, l.dst2));
    }
    i0 = i1;
  }
  return DTC_OK;
}

// The basis states of a batch (masks already in ctx->basis) as the source of
// its schedule: a first pass that only kicks forms them in registers (no
// zero-fill of F, no read of it); any other first pass reads F, filled here.
template <class LaunchT>
int basis_source(dtc_ctx* ctx, std::vector<LaunchT>& sched, double2* F, int64_t len, int nb,
                 int octet_bits) {
  if (!sched.empty() && pass_shape(sched[0].ps) == dtc::kShapeK && ctx->basis_synth) {
    sched[0].basis = (const int64_t*)ctx->basis.p;
    return DTC_OK;
  }
  DTC_HIP(hipMemsetAsync(F, 0, (size_t)dtc::octet_padded(nb, octet_bits) * len * 16, ctx->stream));
  DTC_HIP(dtc::launch_set_basis(F, len, (const int64_t*)ctx->basis.p, nb, ctx->stream, octet_bits));
  return DTC_OK;
}

// Batch size and state layout of a batched run: B states per launch within
// the memory budget (per_state bytes each), the octet layout (dtc_kernels.h)
// when a batch holds at least one octet; then B is a multiple of 8 unless one
// batch takes every state.
// Batch size and state layout.  The octet layout (eight states interleaved
// at 2^octet_bits amplitudes, one state per XCD) serves states below 1 GiB;
// larger states (L_eff >= 26: C4) stay contiguous, the pass kernels then
// giving each XCD an eighth of a state's tiles (r5r: C4 +3.5 %, the top
// 8-site group's rows 16 MiB apart instead of 128 MiB)
constexpr int kOctetMaxLeff = 25;
void batch_layout(const dtc_ctx* ctx, int L_eff, int64_t S, int64_t& B, int& octet) {
  B = std::min<int64_t>(std::min<int64_t>(B, S), 65535);
  octet = (ctx->octet_bits > 0 && B >= 8 && L_eff <= kOctetMaxLeff) ? ctx->octet_bits : 0;
  if (octet && B < S) B &= ~(int64_t)7;
}

// Matrix family of each kick-table row: RX if every sub-gate is
// [[real, imag], [imag, real]], RY if every sub-gate is real, else general.
// Both families are closed under products, Paulis and daggers.
std::vector<int> classify_rows(const dtc_problem* pr) {
  const int n_rows = std::max(1, pr->T - 1 + pr->t_offset);
  std::vector<int> out(n_rows);
  const size_t per_row = (size_t)pr->L * pr->n_sub;
  for (int r = 0; r < n_rows; ++r) {
    bool rx = true, ry = true;
    for (size_t e = 0; e < per_row; ++e) {
      const double* m = pr->kick + ((size_t)r * per_row + e) * 8;
      // m = {m00.re, m00.im, m01.re, m01.im, m10.re, m10.im, m11.re, m11.im}
      if (!(m[1] == 0.0 && m[2] == 0.0 && m[4] == 0.0 && m[7] == 0.0)) rx = false;
      if (!(m[1] == 0.0 && m[3] == 0.0 && m[5] == 0.0 && m[7] == 0.0)) ry = false;
    }
    out[r] = rx ? dtc::kKindRX : (ry ? dtc::kKindRY : dtc::kKindGen);
  }
  return out;
}

// Forward chain over periods first .. first + n - 1 (rows period-1, RNG counter
// = period, stream `stream`), a diagonal after every layer (fast.py:111-121).
Chain forward_chain(const Plan& pl, int first, int n, uint32_t stream) {
  Chain ch;
  for (int k = 0; k < n; ++k)
    ch.X.push_back(KickDesc{1, first + k - 1, dtc::kKickForward, stream, (uint32_t)(first + k)});
  ch.trailing_d = true;
  ch.diag = dtc::kDiagFwd;
  ch.kc.assign(pl.groups.size(), 0);
  return ch;
}

// Echo chain (fast.py:140-143, UF.inverse() per period, periods in reverse):
// D^* K'_p D^* K'_{p-1} ... D^* K'_1, RNG stream `stream`, counter = step k.
// `ahead[g]` marks groups whose state already carries the forward layer
// K_{p+1} (row p): X_0 undoes it exactly before the first D^*.
Chain echo_chain(const Plan& pl, int p, uint32_t stream, const std::vector<int>& ahead) {
  Chain ch;
  ch.X.push_back(KickDesc{1, p, dtc::kKickUndo, dtc::kStreamForward, (uint32_t)(p + 1)});
  for (int k = 1; k <= p; ++k)
    ch.X.push_back(KickDesc{1, p - k, dtc::kKickInverse, stream, (uint32_t)k});
  ch.trailing_d = false;
  ch.diag = dtc::kDiagConj;
  ch.kc.resize(pl.groups.size());
  for (size_t g = 0; g < pl.groups.size(); ++g) ch.kc[g] = ahead[g] ? 0 : 1;
  return ch;
}

// Run a whole chain; the first pass reads src, every pass writes dst; the
// observables of the final state are reduced into meas_out (if meas_mode).
int run_chain(dtc_ctx* ctx, const RunCfg& rc, int64_t batch_start, int batch, Chain& ch,
              const double2* src, double2* dst, int meas_mode, int n_obs, double* meas_out,
              int64_t meas_stride) {
  const double2* s = src;
  while (!ch.done()) {
    PassSpec ps = next_pass(ch);
    const bool last = ch.done();
    DTC_TRY(launch_pass_spec(ctx, rc, batch_start, batch, ps, s, dst,
                             last ? meas_mode : dtc::kMeasNone, 1, n_obs, meas_out,
                             meas_stride));
    s = dst;
  }
  return DTC_OK;
}

int check_problem(const dtc_problem* pr, const dtc_noise* nz, int max_L = 32) {
  if (!pr || !nz) return fail(DTC_EINVAL, "null problem/noise");
  if (pr->L < 1 || pr->L > max_L)
    return fail(DTC_EINVAL, max_L == 32 ? "L must be in [1, 32] per device (larger: dtc_shard_*)"
                                        : "L out of range");
  if (pr->T < 1) return fail(DTC_EINVAL, "T must be >= 1");
  if (pr->n_inst < 1) return fail(DTC_EINVAL, "n_inst must be >= 1");
  if (pr->probe_site < 0 || pr->probe_site >= pr->L)
    return fail(DTC_EINVAL, "probe_site out of range");
  if (pr->t_offset < 0) return fail(DTC_EINVAL, "t_offset must be >= 0");
  if (pr->t_first < 0 || pr->t_first >= pr->T) return fail(DTC_EINVAL, "t_first out of range");
  if (pr->n_sub < 1 || pr->n_sub > 8) return fail(DTC_EINVAL, "n_sub must be in [1, 8]");
  if (!pr->h || (!pr->phi && pr->L > 1) || !pr->kick)
    return fail(DTC_EINVAL, "null h/phi/kick");
  if (pr->L < 64 && (pr->init_mask >> pr->L) != 0)
    return fail(DTC_EINVAL, "init_mask has bits beyond L");
  if (!(nz->p >= 0.0) || nz->p > 4.0 / 3.0) return fail(DTC_EINVAL, "noise p out of range");
  return DTC_OK;
}

void thresholds(double p, uint32_t* t1, uint32_t* t2, uint32_t* t3) {
  auto thr = [&](int k) -> uint32_t {
    double v = std::floor(k * p / 4.0 * 4294967296.0 + 0.5);
    if (v >= 4294967295.0) v = 4294967295.0;
    if (v < 0) v = 0;
    return (uint32_t)v;
  };
  *t1 = thr(1);
  *t2 = thr(2);
  *t3 = thr(3);
}

// Initial product state of one trajectory: neel X gates (fast.py:127-130)
// followed by their depolarizing draw; X or Y after X returns the site to |0>.
uint64_t init_state_mask(const RunCfg& rc, uint64_t traj) {
  uint64_t m = rc.prob->init_mask;
  if (!rc.noisy) return m;
  for (int i = 0; i < rc.pl.L; ++i) {
    if (!((rc.prob->init_mask >> i) & 1ull)) continue;
    int jump = 0;
    int pz = rc.device ? dtc::sample_device(rc.seed, traj, dtc::kStreamPrep, 0u, (uint32_t)i, 0u,
                                            rc.dev_thr_host.data() + 3 * i, 0u, &jump)
                       : dtc::sample_pauli(rc.seed, traj, dtc::kStreamPrep, 0u, (uint32_t)i, 0u,
                                           rc.thr1, rc.thr2, rc.thr3);
    if (pz == 1 || pz == 2) m &= ~(1ull << i);
  }
  return m;
}

// Cone diagonals of the light-cone pass (dtc_kernels.h, kLcTab): for r = 1..4
// the terms of D on sites j-r+1 .. j+r-1 and every bond touching them, as a
// function of bits lo..hi = j-r .. j+r (clipped to [0, L)); r = 5 split at j
// into bits j-5 .. j (fields j-4 .. j, bonds from j-5) and j .. j+5 (fields
// j+1 .. j+4, bonds from j to j+5).
void build_cone_tables(int L, int j, int n_inst, const double* h, const double* phi,
                       std::vector<double>& out) {
  out.assign((size_t)n_inst * dtc::kLcTab * 2, 0.0);
  for (int in = 0; in < n_inst; ++in) {
    const double* hh = h + (size_t)in * L;
    const double* pp = phi + (size_t)in * (L > 1 ? L - 1 : 0);
    for (int r = 1; r <= 4; ++r) {
      const int lo = std::max(0, j - r), hi = std::min(L - 1, j + r);
      double* o = out.data() + ((size_t)in * dtc::kLcTab + dtc::lc_tab_off(r)) * 2;
      for (int v = 0; v < (1 << (hi - lo + 1)); ++v) {
        const double ang = diag_angle(L, hh, pp, std::max(0, j - r + 1), j + r, j - r, j + r, lo, v);
        const int e = r == 4 ? dtc::lc_pos4(v) : v;  // the radius-4 table's storage swizzle
        o[2 * e] = std::cos(-0.5 * ang);
        o[2 * e + 1] = std::sin(-0.5 * ang);
      }
    }
    for (int part = 0; part < 2; ++part) {
      const int lo = part == 0 ? std::max(0, j - 5) : j;
      const int hi = part == 0 ? j : std::min(L - 1, j + 5);
      double* o = out.data() + ((size_t)in * dtc::kLcTab + (part == 0 ? dtc::kLcTab5a : dtc::kLcTab5b)) * 2;
      for (int v = 0; v < (1 << (hi - lo + 1)); ++v) {
        const double ang = part == 0
                               ? diag_angle(L, hh, pp, std::max(0, j - 4), j + 1, j - 5, j, lo, v)
                               : diag_angle(L, hh, pp, j + 1, j + 5, j, j + 5, lo, v);
        const int e = part == 0 ? dtc::lc_pos5a(v) : v;  // storage swizzle of the j-5 .. j table
        o[2 * e] = std::cos(-0.5 * ang);
        o[2 * e + 1] = std::sin(-0.5 * ang);
      }
    }
    // r = 6 and r = 3 split at j (dtc_lcw3_final; j - 6 >= 0 and j + 6 < L,
    // the only geometry that kernel runs): bits j-6 .. j (fields j-5 .. j,
    // bonds from j-6) and j .. j+6 (fields j+1 .. j+5, bonds up to j+6); bits
    // j-3 .. j and j .. j+3 likewise
    if (j - 6 >= 0 && j + 6 <= L - 1) {
      for (int part = 0; part < 4; ++part) {
        const int off = part == 0 ? dtc::kLcTab6a : part == 1 ? dtc::kLcTab6b
                      : part == 2 ? dtc::kLcTab3a : dtc::kLcTab3b;
        const int r = part < 2 ? 6 : 3;
        double* o = out.data() + ((size_t)in * dtc::kLcTab + off) * 2;
        for (int v = 0; v < (1 << (r + 1)); ++v) {
          const double ang = (part % 2 == 0)
                                 ? diag_angle(L, hh, pp, j - r + 1, j + 1, j - r, j, j - r, v)
                                 : diag_angle(L, hh, pp, j + 1, j + r, j, j + r, j, v);
          o[2 * v] = std::cos(-0.5 * ang);
          o[2 * v + 1] = std::sin(-0.5 * ang);
        }
      }
    }
    // r = 4 split at j (dtc_lcw2_final): the product of the two is the r = 4
    // table (dtc_kernels.h kLcTab4a / kLcTab4b; j - 4 >= 0 and j + 4 < L, the
    // only geometry that kernel runs)
    if (j - 4 >= 0 && j + 4 <= L - 1) {
      for (int part = 0; part < 2; ++part) {
        double* o = out.data() + ((size_t)in * dtc::kLcTab + (part == 0 ? dtc::kLcTab4a : dtc::kLcTab4b)) * 2;
        for (int v = 0; v < 32; ++v) {
          const double ang = part == 0 ? diag_angle(L, hh, pp, j - 3, j + 1, j - 4, j, j - 4, v)
                                       : diag_angle(L, hh, pp, j + 1, j + 4, j, j + 4, j, v);
          o[2 * v] = std::cos(-0.5 * ang);
          o[2 * v + 1] = std::sin(-0.5 * ang);
        }
      }
    }
  }
}

uint64_t fnv(uint64_t h, const void* p, size_t n);

// The problem's device tables (diagonal factors, cone diagonals, kick table),
// uploaded when they differ from the ones in place: a repeated sweep of the
// same problem (the bench's steps, a controller's evaluations) neither
// rebuilds nor re-uploads them, nor waits for the stream.
int upload_tables(dtc_ctx* ctx, const dtc_problem* pr, const Plan& pl) {
  const int n_periods = std::max(1, pr->T - 1 + pr->t_offset);
  const size_t kb = (size_t)n_periods * pr->L * pr->n_sub * 8 * sizeof(double);
  const int32_t shape[6] = {pr->L, pl.L_eff, pr->n_inst, pr->probe_site, n_periods, pr->n_sub};
  uint64_t key = fnv(1469598103934665603ull, shape, sizeof(shape));
  key = fnv(key, pr->h, sizeof(double) * pr->n_inst * pr->L);
  if (pr->L > 1) key = fnv(key, pr->phi, sizeof(double) * pr->n_inst * (pr->L - 1));
  key = fnv(key, pr->kick, kb);
  if (ctx->tables_valid && key == ctx->tables_key) return DTC_OK;
  ctx->tables_valid = false;
  std::vector<double> dt;
  build_diag_tables(pl, pr->n_inst, pr->h, pr->phi, dt);
  DTC_TRY(ensure(ctx->diag, dt.size() * sizeof(double)));
  DTC_HIP(hipMemcpyAsync(ctx->diag.p, dt.data(), dt.size() * sizeof(double),
                         hipMemcpyHostToDevice, ctx->stream));
  if (pr->probe_site >= 0 && pr->probe_site < pr->L) {
    std::vector<double> ct;
    build_cone_tables(pr->L, pr->probe_site, pr->n_inst, pr->h, pr->phi, ct);
    DTC_TRY(ensure(ctx->lc_diag, ct.size() * sizeof(double)));
    DTC_HIP(hipMemcpyAsync(ctx->lc_diag.p, ct.data(), ct.size() * sizeof(double),
                           hipMemcpyHostToDevice, ctx->stream));
  }
  DTC_TRY(ensure(ctx->kick, kb));
  DTC_HIP(hipMemcpyAsync(ctx->kick.p, pr->kick, kb, hipMemcpyHostToDevice, ctx->stream));
  DTC_HIP(hipStreamSynchronize(ctx->stream));
  ctx->tables_key = key;
  ctx->tables_valid = true;
  return DTC_OK;
}


// ---- sharded state (include/dtc.h: dtc_shard) ---------------------------------

int check_shard(const dtc_problem* pr, const dtc_shard* sh) {
  if (!sh) return fail(DTC_EINVAL, "null shard");
  const int L = pr->L, nl = sh->n_local, ng = sh->n_global;
  if (ng < 0 || ng > 16 || nl + ng != L) return fail(DTC_EINVAL, "n_local + n_global must equal L");
  if (nl < dtc::kTileBits || nl > 32) return fail(DTC_EINVAL, "n_local must be in [12, 32]");
  if (sh->n_shards < 1 || sh->first_rank < 0 ||
      (int64_t)sh->first_rank + sh->n_shards > ((int64_t)1 << ng))
    return fail(DTC_EINVAL, "shard ranks outside [0, 2^n_global)");
  std::vector<int> seen(L, 0);
  for (int q = 0; q < L; ++q) {
    const int v = sh->site_of[q];
    if (v < 0 || v >= L || seen[v]++) return fail(DTC_EINVAL, "site_of is not a permutation");
  }
  // every bond between two local sites must join adjacent physical bits
  std::vector<int> bit_of(L);
  for (int q = 0; q < L; ++q) bit_of[sh->site_of[q]] = q;
  for (int i = 0; i + 1 < L; ++i) {
    const int a = bit_of[i], b = bit_of[i + 1];
    if (a < nl && b < nl && std::abs(a - b) != 1)
      return fail(DTC_EINVAL, "a bond between two local sites is not physically adjacent");
  }
  return DTC_OK;
}

// Effective chain of one shard: local fields/bonds over physical bits plus the
// constant angle of the rank's global sites (fields, bonds to and among them).
void shard_chain(const dtc_problem* pr, const dtc_shard* sh, int inst, int rank,
                 double* h_eff, double* phi_eff, double* c_angle) {
  const int L = pr->L, nl = sh->n_local;
  const double* h = pr->h + (size_t)inst * L;
  const double* phi = pr->phi + (size_t)inst * (L > 1 ? L - 1 : 0);
  std::vector<int> bit_of(L);
  for (int q = 0; q < L; ++q) bit_of[sh->site_of[q]] = q;
  auto zg = [&](int site) {  // z of a global site on this rank
    return ((rank >> (bit_of[site] - nl)) & 1) ? -1.0 : 1.0;
  };
  double c = 0.0;
  for (int q = 0; q < nl; ++q) h_eff[q] = h[sh->site_of[q]];
  for (int q = 0; q + 1 < nl; ++q) phi_eff[q] = 0.0;
  for (int i = 0; i < L; ++i)
    if (bit_of[i] >= nl) c += h[i] * zg(i);
  for (int i = 0; i + 1 < L; ++i) {
    const int a = bit_of[i], b = bit_of[i + 1];
    if (a < nl && b < nl) phi_eff[std::min(a, b)] = phi[i];
    else if (a < nl) h_eff[a] += phi[i] * zg(i + 1);
    else if (b < nl) h_eff[b] += phi[i] * zg(i);
    else c += phi[i] * zg(i) * zg(i + 1);
  }
  *c_angle = c;
}

uint64_t group_bits(const Group& g) {
  uint64_t m = 0;
  for (int k = 0; k < g.tb; ++k)
    if (g.act & (1 << k)) m |= 1ull << (k < g.c ? k : g.s + k - g.c);
  return m;
}

// The kick sites of layer `k` in a pass over group g (tile bits outside
// k.skip), below L.
uint64_t layer_sites(const Group& g, const KickDesc& k, int L) {
  uint64_t m = 0;
  for (int b = 0; b < g.tb; ++b) {
    if (!(g.act & ~(int)k.skip & (1 << b))) continue;
    const int site = b < g.c ? b : g.s + b - g.c;
    if (site < L) m |= 1ull << site;
  }
  return m;
}

// tile bits of group g that are NOT in mask (left identity by a kick layer)
uint32_t skip_bits(const Group& g, uint64_t mask) {
  uint32_t sk = 0;
  for (int k = 0; k < g.tb; ++k) {
    if (!(g.act & (1 << k))) continue;
    const int bit = k < g.c ? k : g.s + k - g.c;
    if (!((mask >> bit) & 1)) sk |= 1u << k;
  }
  return sk;
}

// The kick layers of a chain's last k passes, in order, separated by the
// D*'s (a layer of one period spans two passes: the post-kick of one group and
// the pre-kick of the next); trailing diagonals are dropped.  False when the
// passes do not form such layers (not a D* chain, a light-cone pass already).
bool lc_layers_of(const RunCfg& rc, const std::vector<Launch>& sched, int k,
                  std::vector<KickDesc>& desc, std::vector<uint64_t>& sites) {
  const Plan& pl = rc.pl;
  auto same_layer = [](const KickDesc& a, const KickDesc& b) {
    return a.row == b.row && a.mode == b.mode && a.stream == b.stream &&
           a.rng_period == b.rng_period;
  };
  desc.assign(1, no_kick());
  sites.assign(1, 0);
  bool ok = true;
  int pending_d = 0;  // diagonals not yet followed by a kick (trailing ones are dropped)
  auto kick = [&](const Group& g, const KickDesc& kd) {
    for (; pending_d > 0; --pending_d) {
      desc.push_back(no_kick());
      sites.push_back(0);
    }
    if (desc.back().enabled && !same_layer(desc.back(), kd)) ok = false;
    desc.back() = kd;
    desc.back().skip = 0;
    sites.back() |= layer_sites(g, kd, pl.L);
  };
  for (size_t i = sched.size() - k; i < sched.size(); ++i) {
    const PassSpec& ps = sched[i].ps;
    if (ps.lc_w0 >= 0) ok = false;
    if (!ok) break;
    const Group& g = pl.groups[ps.group];
    if (ps.pre.enabled) kick(g, ps.pre);
    if (ps.diag != dtc::kDiagNone) {
      if (ps.diag != dtc::kDiagConj) ok = false;
      ++pending_d;
    }
    if (ps.post.enabled) kick(g, ps.post);
  }
  return ok;
}

// The sites of j's cone (radius r), clipped to [0, L).
uint64_t cone_sites(int L, int j, int r) {
  uint64_t cone = 0;
  for (int i = std::max(0, j - r); i <= std::min(L - 1, j + r); ++i) cone |= 1ull << i;
  return cone;
}

// The 10-site light-cone end (dtc_lcw_final): the chain's last five passes
// as six layers r = 5 .. 0 on the window j-5 .. j+4 or j-4 .. j+5 (the cone
// of r = 4 plus the first layer's group), tile bits 0, 1 = global bits 0, 1.
// The kernel's fixed nibble program needs layers r <= 1 on j-2 .. j+1 (nibble
// 1), r <= 3 on nibbles 1 and 2 (+ j+2, j+3, j-4, j-3): checked here, as the
// window's bounds; false leaves the chain to lc_merge's 8-site form.
bool lc_merge_wide(const RunCfg& rc, std::vector<Launch>& sched, size_t chain0, int j) {
  const Plan& pl = rc.pl;
  const int L = pl.L;
  if ((int)(sched.size() - chain0) < 5) return false;
  if (j - 4 < 2 || j + 3 > L - 1) return false;
  std::vector<KickDesc> desc;
  std::vector<uint64_t> sites;
  if (!lc_layers_of(rc, sched, 5, desc, sites) || (int)desc.size() != dtc::kLcwLayers) return false;
  uint64_t u = 1ull << j;
  for (int l = 0; l < dtc::kLcwLayers; ++l) {
    sites[l] &= cone_sites(L, j, dtc::kLcwLayers - 1 - l);
    u |= sites[l];
  }
  const uint64_t nib1 = 0xFull << (j - 2);
  const uint64_t nib2 = (3ull << (j + 2)) | (3ull << (j - 4));
  if ((sites[4] | sites[5]) & ~nib1) return false;
  if ((sites[2] | sites[3]) & ~(nib1 | nib2)) return false;
  uint64_t rest = u & ~(nib1 | nib2);
  if (__builtin_popcountll(rest) > 2 || (rest & 3ull)) return false;
  // the two low tile bits beside the columns: the outer sites, padded with
  // free bits of the state (their kicks stay off)
  for (int g = 2; g < pl.L_eff && __builtin_popcountll(rest) < 2; ++g)
    if (!(((nib1 | nib2 | rest) >> g) & 1ull)) rest |= 1ull << g;
  if (__builtin_popcountll(rest) != 2) return false;
  PassSpec lc{sched.back().ps.group, no_kick(), no_kick(), dtc::kDiagConj, sched.back().ps.d_index};
  const int r0 = __builtin_ctzll(rest), r1 = 63 - __builtin_clzll(rest);
  const int gb[dtc::kTileBits] = {0, 1, r0, r1, j - 2, j - 1, j, j + 1, j + 2, j + 3, j - 4, j - 3};
  lc.lc_w0 = j - 4;  // (marks the light-cone pass; the tile is lc_gb)
  lc.lc_wide = 1;
  lc.lc_layers = dtc::kLcwLayers;
  for (int k = 0; k < dtc::kTileBits; ++k) lc.lc_gb[k] = (int8_t)gb[k];
  for (int l = 0; l < dtc::kLcwLayers; ++l) {
    lc.lc[l] = desc[l];
    for (int k = 2; k < dtc::kTileBits; ++k)
      if ((sites[l] >> gb[k]) & 1ull) lc.lc_mask |= 1ull << (10 * l + k - 2);
  }
  const int kind = pass_kind(rc, lc, dtc::kShapeLC);
  if (kind != dtc::kKindRX && kind != dtc::kKindRY) return false;
  const Launch first = sched[sched.size() - 5];
  sched.resize(sched.size() - 5 + 1);
  sched.back() = Launch{lc, first.src, first.dst, dtc::kMeasProbe, 1, 2, nullptr, first.meas_stride};
  return true;
}

// The 12-site light-cone end (dtc_lcw3_final): the chain's last six passes
// as seven layers r = 6 .. 0 on the window j-5 .. j+6, tile bit k = global
// bit j-5+k (no column bits).  The kernel runs a fixed program: layer l may
// kick only sites of its cone that the program visits (l0: j+2 .. j+6 -- the
// C2 chains' first layer is group B's pre-kick; l1: j-5 .. j+5; then the
// cones of radius 4 .. 0); a site the chain leaves unkicked gets the identity
// record.  False leaves the chain to lc_merge_wide.
bool lc_merge_wide7(const RunCfg& rc, std::vector<Launch>& sched, size_t chain0, int j) {
  const Plan& pl = rc.pl;
  const int L = pl.L;
  if ((int)(sched.size() - chain0) < 6) return false;
  if (j - 6 < 0 || j + 6 > L - 1 || pl.L_eff != L || pl.L_eff > 32) return false;
  std::vector<KickDesc> desc;
  std::vector<uint64_t> sites;
  if (!lc_layers_of(rc, sched, 6, desc, sites) || (int)desc.size() != dtc::kLcw3Layers) return false;
  auto span = [&](int a, int b) {  // sites j+a .. j+b
    uint64_t m = 0;
    for (int i = j + a; i <= j + b; ++i) m |= 1ull << i;
    return m;
  };
  const uint64_t prog[dtc::kLcw3Layers] = {span(2, 6), span(-5, 5), span(-4, 4), span(-3, 3),
                                           span(-2, 2), span(-1, 1), span(0, 0)};
  for (int l = 0; l < dtc::kLcw3Layers; ++l) {
    sites[l] &= cone_sites(L, j, dtc::kLcw3Layers - 1 - l);
    if (sites[l] & ~prog[l]) return false;
  }
  PassSpec lc{sched.back().ps.group, no_kick(), no_kick(), dtc::kDiagConj, sched.back().ps.d_index};
  lc.lc_w0 = j - 5;  // (marks the light-cone pass; the tile is lc_gb)
  lc.lc_wide = 2;
  lc.lc_layers = dtc::kLcw3Layers;
  for (int k = 0; k < dtc::kTileBits; ++k) lc.lc_gb[k] = (int8_t)(j - 5 + k);
  for (int l = 0; l < dtc::kLcw3Layers; ++l) {
    lc.lc[l] = desc[l];
    for (int k = 0; k < dtc::kTileBits; ++k)
      if ((sites[l] >> (j - 5 + k)) & 1ull) {
        const int bit = 12 * l + k;
        if (bit < 64) lc.lc_mask |= 1ull << bit;
        else lc.lc_mask2 |= 1ull << (bit - 64);
      }
  }
  const int kind = pass_kind(rc, lc, dtc::kShapeLC);
  if (kind != dtc::kKindRX && kind != dtc::kKindRY) return false;
  const Launch first = sched[sched.size() - 6];
  sched.resize(sched.size() - 6 + 1);
  sched.back() = Launch{lc, first.src, first.dst, dtc::kMeasProbe, 1, 2, nullptr, first.meas_stride};
  return true;
}

// Light-cone end of the echo chain sched[chain0 ..) measuring Z_j: replace
// its last k passes by one kShapeLC pass -- six (lc_merge_wide7) or five
// (lc_merge_wide), when enabled and they fit, else k = 4 .. 2 (the first that
// fits) over an 8-site window.
// Layer l of M (r = M - 1 - l diagonals before the probe) only matters on
// sites j-r .. j+r, and the layers' remaining sites must fit the window
// w0 .. w0+7 (4 <= w0 <= L - 8: clear of tile bits 0..3).
void lc_merge(const RunCfg& rc, std::vector<Launch>& sched, size_t chain0, int j, bool wide,
              bool wide3) {
  const Plan& pl = rc.pl;
  const int L = pl.L;
  if (wide3 && lc_merge_wide7(rc, sched, chain0, j)) return;
  if (wide && lc_merge_wide(rc, sched, chain0, j)) return;
  const int n_chain = (int)(sched.size() - chain0);
  for (int k = std::min(4, n_chain); k >= 2; --k) {
    std::vector<KickDesc> desc;
    std::vector<uint64_t> sites;
    const bool ok = lc_layers_of(rc, sched, k, desc, sites);
    const int M = (int)desc.size();
    if (!ok || M > dtc::kLcLayers) continue;
    uint64_t u = 1ull << j;
    for (int l = 0; l < M; ++l) {
      sites[l] &= cone_sites(L, j, M - 1 - l);
      u |= sites[l];
    }
    const int lo = __builtin_ctzll(u), hi = 63 - __builtin_clzll(u);
    const int w0 = std::max(4, std::min(lo, L - 8));
    if (w0 > lo || hi > w0 + 7 || w0 + 8 > pl.L_eff) continue;
    const PassSpec& last = sched.back().ps;
    PassSpec lc{last.group, no_kick(), no_kick(), dtc::kDiagConj, last.d_index};
    lc.lc_w0 = w0;
    lc.lc_layers = M;
    for (int l = 0; l < M; ++l) {
      lc.lc[l] = desc[l];
      lc.lc_mask |= ((sites[l] >> w0) & 0xFFull) << (dtc::kLcSites * l);
    }
    const int kind = pass_kind(rc, lc, dtc::kShapeLC);
    if (kind != dtc::kKindRX && kind != dtc::kKindRY) continue;
    const Launch first = sched[sched.size() - k];
    sched.resize(sched.size() - k + 1);
    sched.back() = Launch{lc, first.src, first.dst, dtc::kMeasProbe, 1, 2, nullptr, first.meas_stride};
    return;
  }
}
}  // namespace

extern "C" {

const char* dtc_last_error(void) { return g_err.c_str(); }

int32_t dtc_abi_version(void) { return DTC_ABI_VERSION; }

int dtc_open(int32_t device, dtc_ctx** out) {
  if (!out) return fail(DTC_EINVAL, "null out");
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(DTC_ENODEV, "no HIP device");
  if (device < 0 || device >= n) return fail(DTC_EINVAL, "device ordinal out of range");
  hipDeviceProp_t prop;
  DTC_HIP(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(DTC_ENODEV, std::string("libdtc_hip is built for gfx950, device is ") +
                                prop.gcnArchName);
  DTC_HIP(hipSetDevice(device));
  dtc_ctx* c = new dtc_ctx();
  c->device = device;
#ifdef DTC_DEV_KNOBS
  // development A/B builds only (make DEV=1): layout and launch-geometry
  // overrides.  The product library ignores these variables, so a stray one
  // cannot change the HBM layout or the kernels' geometry.
  if (const char* e = std::getenv("DTC_OCTET_BITS")) c->octet_bits = std::atoi(e);
  if (c->octet_bits != 0 && (c->octet_bits < 4 || c->octet_bits > 12)) c->octet_bits = 6;
  if (const char* e = std::getenv("DTC_LC_SPLIT")) c->lc_split = e[0] != '0';
  if (const char* e = std::getenv("DTC_LC_TPB")) c->lc_tpb = std::atoi(e);
  if (const char* e = std::getenv("DTC_KDK_SPLIT")) c->kdk_split = std::atoi(e);
  c->basis_synth = std::getenv("DTC_NO_BASIS_SYNTH") == nullptr;
  if (const char* e = std::getenv("DTC_BATCH_BYTES")) c->batch_bytes = std::atof(e);
#endif
  // documented test switches (the parity tests compare the light-cone ends
  // with the full passes, each form on its own engine)
  c->lightcone = std::getenv("DTC_NO_LIGHTCONE") == nullptr;
  c->lc_wide = std::getenv("DTC_NO_LCW") == nullptr;
  c->lc_wide3 = c->lc_wide && std::getenv("DTC_NO_LCW3") == nullptr;
  c->dual = std::getenv("DTC_NO_DUAL") == nullptr;
  c->runahead = std::getenv("DTC_NO_RUNAHEAD") == nullptr;
  if (const char* e = std::getenv("DTC_SPLIT13")) c->split13 = std::atoi(e) != 0;
  c->verbose = std::getenv("DTC_VERBOSE") != nullptr;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return fail(DTC_EHIP, "hipStreamCreate failed");
  }
  *out = c;
  return DTC_OK;
}

int dtc_close(dtc_ctx* ctx) {
  if (!ctx) return DTC_OK;
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  for (auto& p : ctx->pending) {
    (void)hipEventDestroy(p.e0);
    (void)hipEventDestroy(p.e1);
  }
  for (auto e : ctx->pool) (void)hipEventDestroy(e);
  release(ctx->F);
  release(ctx->E);
  release(ctx->prefix);
  release(ctx->partial);
  release(ctx->vals_f);
  release(ctx->vals_e);
  release(ctx->diag);
  release(ctx->lc_diag);
  release(ctx->red_scratch);
  if (ctx->host_f.p) (void)hipHostFree(ctx->host_f.p);
  if (ctx->host_e.p) (void)hipHostFree(ctx->host_e.p);
  release(ctx->kick);
  release(ctx->basis);
  release(ctx->sitemap);
  release(ctx->recs);
  release(ctx->recs1);
  release(ctx->pk);
  release(ctx->dev_thr);
  release(ctx->dev_jump);
  release(ctx->dev_kraus);
  for (auto& e : ctx->shard_cache) release(e.diag);
  for (auto& e : ctx->shard_maps) release(e.diag);
  release(ctx->shard_kick);
  (void)hipStreamDestroy(ctx->stream);
  delete ctx;
  return DTC_OK;
}

int dtc_release_buffers(dtc_ctx* ctx) {
  if (!ctx) return fail(DTC_EINVAL, "null ctx");
  DTC_HIP(hipSetDevice(ctx->device));
  DTC_HIP(hipStreamSynchronize(ctx->stream));
  DTC_TRY(resolve_pending(ctx));
  release(ctx->F);
  release(ctx->E);
  release(ctx->partial);
  release(ctx->red_scratch);
  release(ctx->recs);
  release(ctx->recs1);
  release(ctx->pk);
  return DTC_OK;
}

int dtc_set_profiling(dtc_ctx* ctx, int32_t on) {
  if (!ctx) return fail(DTC_EINVAL, "null ctx");
  ctx->prof = on != 0;
  return DTC_OK;
}

int dtc_reset_stats(dtc_ctx* ctx) {
  if (!ctx) return fail(DTC_EINVAL, "null ctx");
  DTC_TRY(resolve_pending(ctx));
  for (int k = 0; k < DTC_KERNEL_KINDS; ++k) {
    ctx->st_n[k] = 0;
    ctx->st_ms[k] = 0;
    ctx->st_bytes[k] = 0;
  }
  return DTC_OK;
}

int dtc_lightcone_counts(dtc_ctx* ctx, int64_t* counts) {
  if (!ctx || !counts) return fail(DTC_EINVAL, "null ctx / counts");
  for (int k = 0; k < 4; ++k) counts[k] = ctx->lc_launches[k];
  return DTC_OK;
}

int dtc_schedule_counts(dtc_ctx* ctx, int64_t* counts) {
  if (!ctx || !counts) return fail(DTC_EINVAL, "null ctx / counts");
  for (int k = 0; k < 4; ++k) counts[k] = ctx->sched_counts[k];
  return DTC_OK;
}

int dtc_kernel_stats(dtc_ctx* ctx, int32_t kind, int64_t* launches, double* total_ms,
                     double* total_bytes) {
  if (!ctx || kind < 0 || kind >= DTC_KERNEL_KINDS) return fail(DTC_EINVAL, "bad args");
  DTC_TRY(resolve_pending(ctx));
  if (launches) *launches = ctx->st_n[kind];
  if (total_ms) *total_ms = ctx->st_ms[kind];
  if (total_bytes) *total_bytes = ctx->st_bytes[kind];
  return DTC_OK;
}

int dtc_device_info(dtc_ctx* ctx, char* name, int32_t name_len, int32_t* n_cu,
                    double* hbm_bytes) {
  if (!ctx) return fail(DTC_EINVAL, "null ctx");
  hipDeviceProp_t prop;
  DTC_HIP(hipGetDeviceProperties(&prop, ctx->device));
  if (name && name_len > 0) {
    std::snprintf(name, (size_t)name_len, "%s (%s)", prop.name, prop.gcnArchName);
  }
  if (n_cu) *n_cu = prop.multiProcessorCount;
  if (hbm_bytes) *hbm_bytes = (double)prop.totalGlobalMem;
  return DTC_OK;
}

}  // extern "C"

namespace {

// Host-side tables of dtc_device_noise (see include/dtc.h for the model).
int setup_device_noise(dtc_ctx* ctx, const dtc_problem* pr, const dtc_device_noise* dv,
                       RunCfg& rc) {
  const int L = pr->L;
  if (!dv->p_gate || !dv->t1_us || !dv->t2_us) return fail(DTC_EINVAL, "null device-noise arrays");
  if (!(dv->gate_ns >= 0.0)) return fail(DTC_EINVAL, "gate_ns must be >= 0");
  if (!(dv->readout_p01 >= 0.0 && dv->readout_p01 <= 1.0 && dv->readout_p10 >= 0.0 &&
        dv->readout_p10 <= 1.0))
    return fail(DTC_EINVAL, "read-out errors must be in [0, 1]");
  auto u32 = [](double prob) -> uint32_t {
    double v = std::floor(prob * 4294967296.0 + 0.5);
    if (v >= 4294967295.0) v = 4294967295.0;
    if (v < 0) v = 0;
    return (uint32_t)v;
  };
  std::vector<uint32_t> jump(L);
  std::vector<double> kraus((size_t)3 * L);
  rc.dev_thr_host.assign((size_t)3 * L, 0u);
  for (int i = 0; i < L; ++i) {
    const double p = dv->p_gate[i];
    if (!(p >= 0.0 && p <= 4.0 / 3.0)) return fail(DTC_EINVAL, "p_gate out of range");
    const double t1 = dv->t1_us[i] > 0.0 ? dv->t1_us[i] * 1e3 : INFINITY;  // ns
    double t2 = dv->t2_us[i] > 0.0 ? dv->t2_us[i] * 1e3 : INFINITY;
    t2 = std::min(t2, 2.0 * t1);
    const double tg = dv->gate_ns;
    const double gamma = std::isinf(t1) ? 0.0 : 1.0 - std::exp(-tg / t1);
    // coherence left by amplitude damping: exp(-tg/(2 T1)); the rest is pure
    // dephasing: Z with probability (1 - r)/2, r = exp(-tg (1/T2 - 1/(2 T1)))
    const double rate = (std::isinf(t2) ? 0.0 : 1.0 / t2) - (std::isinf(t1) ? 0.0 : 0.5 / t1);
    const double pz_deph = 0.5 * (1.0 - std::exp(-tg * std::max(0.0, rate)));
    // dephasing then depolarizing(p): X, Y w.p. p/4, Z w.p. (1-d) p/4 + d (1 - 3p/4)
    const double px = p / 4.0, py = p / 4.0;
    const double pzz = (1.0 - pz_deph) * p / 4.0 + pz_deph * (1.0 - 3.0 * p / 4.0);
    rc.dev_thr_host[3 * i + 0] = u32(px);
    rc.dev_thr_host[3 * i + 1] = u32(px + py);
    rc.dev_thr_host[3 * i + 2] = u32(px + py + pzz);
    const double q1 = gamma / 2.0, q0 = 1.0 - q1;
    jump[i] = u32(q1);
    kraus[3 * i + 0] = 1.0 / std::sqrt(q0);
    kraus[3 * i + 1] = std::sqrt(1.0 - gamma) / std::sqrt(q0);
    kraus[3 * i + 2] = q1 > 0.0 ? std::sqrt(gamma / q1) : 0.0;
  }
  DTC_TRY(ensure(ctx->dev_thr, rc.dev_thr_host.size() * sizeof(uint32_t)));
  DTC_TRY(ensure(ctx->dev_jump, jump.size() * sizeof(uint32_t)));
  DTC_TRY(ensure(ctx->dev_kraus, kraus.size() * sizeof(double)));
  DTC_HIP(hipMemcpyAsync(ctx->dev_thr.p, rc.dev_thr_host.data(),
                         rc.dev_thr_host.size() * sizeof(uint32_t), hipMemcpyHostToDevice,
                         ctx->stream));
  DTC_HIP(hipMemcpyAsync(ctx->dev_jump.p, jump.data(), jump.size() * sizeof(uint32_t),
                         hipMemcpyHostToDevice, ctx->stream));
  DTC_HIP(hipMemcpyAsync(ctx->dev_kraus.p, kraus.data(), kraus.size() * sizeof(double),
                         hipMemcpyHostToDevice, ctx->stream));
  DTC_HIP(hipStreamSynchronize(ctx->stream));
  rc.device = true;
  rc.noisy = 1;
  rc.dev_thr = (const uint32_t*)ctx->dev_thr.p;
  rc.dev_jump = (const uint32_t*)ctx->dev_jump.p;
  rc.dev_kraus = (const double*)ctx->dev_kraus.p;
  return DTC_OK;
}

// What a prefix must match: the instances' angles and the kick rows of its
// periods (FNV-1a over the bytes), so a continuation inverts the same periods.
uint64_t prefix_hash(const dtc_problem* pr, int n_periods) {
  uint64_t h = 1469598103934665603ull;
  auto mix = [&](const void* p, size_t n) {
    const unsigned char* c = (const unsigned char*)p;
    for (size_t i = 0; i < n; ++i) h = (h ^ c[i]) * 1099511628211ull;
  };
  mix(&pr->L, sizeof(pr->L));
  mix(&pr->n_inst, sizeof(pr->n_inst));
  mix(&pr->n_sub, sizeof(pr->n_sub));
  mix(&pr->init_mask, sizeof(pr->init_mask));
  mix(pr->h, sizeof(double) * (size_t)pr->n_inst * pr->L);
  if (pr->L > 1) mix(pr->phi, sizeof(double) * (size_t)pr->n_inst * (pr->L - 1));
  mix(pr->kick, sizeof(double) * 8 * (size_t)n_periods * pr->L * pr->n_sub);
  return h;
}

int autocorr_impl(dtc_ctx* ctx, const dtc_problem* pr, const dtc_noise* nz,
                  const dtc_device_noise* dv, uint64_t seed, int64_t traj_offset, int32_t n_traj,
                  double* fwd, double* echo, double* zsite, bool use_prefix = false) {
  if (!ctx) return fail(DTC_EINVAL, "null ctx");
  DTC_TRY(check_problem(pr, nz));
  if (n_traj < 1) return fail(DTC_EINVAL, "n_traj must be >= 1");
  if (traj_offset < 0) return fail(DTC_EINVAL, "traj_offset must be >= 0");
  if (pr->want_fwd && !fwd) return fail(DTC_EINVAL, "want_fwd but fwd is null");
  if (pr->want_echo && !echo) return fail(DTC_EINVAL, "want_echo but echo is null");
  DTC_HIP(hipSetDevice(ctx->device));

  RunCfg rc;
  rc.prob = pr;
  rc.seed = seed;
  rc.traj_offset = traj_offset;
  rc.n_traj = n_traj;
  rc.noisy = nz->p > 0.0 ? 1 : 0;
  rc.row_kind = classify_rows(pr);
  {
    // the 13 / 7 split where its kernels cover every pass: L = 20, unitary
    // factored kicks (RX / RY rows), the probe measurement only, no prefix
    bool s13 = ctx->split13 && pr->L == 20 && !dv && !zsite && !use_prefix;
    for (int k : rc.row_kind) s13 = s13 && (k == dtc::kKindRX || k == dtc::kKindRY);
    rc.pl = make_plan(pr->L, false, s13);
  }
  thresholds(nz->p, &rc.thr1, &rc.thr2, &rc.thr3);
  if (dv) DTC_TRY(setup_device_noise(ctx, pr, dv, rc));
  const Plan& pl = rc.pl;
  const int T = pr->T, L = pr->L;
  const int P = T - 1 + pr->t_offset;
  const bool want_z = zsite != nullptr;
  const bool want_f = pr->want_fwd || want_z;
  const bool want_e = pr->want_echo != 0;
  const int n_obs_f = want_z ? 1 + L : 2;
  const int meas_f = want_z ? dtc::kMeasSites : dtc::kMeasProbe;
  const double fac = dv ? dv->anc_factor : std::pow(1.0 - nz->p, (double)nz->n_anc);
  // read-out: measured = ro_a * a + ro_b (identity without device noise)
  const double ro_a = dv ? 1.0 - dv->readout_p01 - dv->readout_p10 : 1.0;
  const double ro_b = dv ? dv->readout_p10 - dv->readout_p01 : 0.0;

  DTC_TRY(upload_tables(ctx, pr, pl));

  // batch size: F (+ E for echo) resident in HBM
  const int64_t S = (int64_t)pr->n_inst * n_traj;
  // continuation of a prefix: periods 1..n_pre come from dtc_prefix_build
  const int n_pre = use_prefix ? ctx->prefix_periods : 0;
  if (use_prefix) {
    if (ctx->prefix_periods < 0) return fail(DTC_EINVAL, "no prefix built");
    if (ctx->prefix_states != S || ctx->prefix_n_traj != n_traj ||
        ctx->prefix_traj_offset != traj_offset || ctx->prefix_len != pl.len ||
        ctx->prefix_device != (dv ? 1 : 0))
      return fail(DTC_EINVAL, "prefix built for other trajectories / size / noise kind");
    if (pr->t_first + pr->t_offset <= n_pre || P <= n_pre)
      return fail(DTC_EINVAL, "prefixed run must measure only after the prefix's periods");
    if (prefix_hash(pr, n_pre) != ctx->prefix_hash)
      return fail(DTC_EINVAL, "problem differs from the prefix's in angles or kick rows");
  }
  const double per_state = (double)pl.len * 16.0 * (want_e ? 2.0 : 1.0);
  int64_t B = pr->batch;
  if (B <= 0) {
    size_t free_b = 0, total_b = 0;
    DTC_HIP(hipMemGetInfo(&free_b, &total_b));
    free_b += ctx->F.n + ctx->E.n;  // the batch buffers this call may reuse or regrow
    // small states: ~64 GiB of batch saturates the device; large states
    // (L >= 24, C4-style instance batches) may use most of the 288 GB
    double budget = per_state >= (double)(256ull << 20)
                        ? 0.7 * (double)free_b
                        : std::min(0.6 * (double)free_b, 64.0 * (1ull << 30));
    if (ctx->batch_bytes > 0) budget = ctx->batch_bytes;
    B = (int64_t)(budget / per_state);
    B = std::max<int64_t>(1, std::min<int64_t>(B, 4096));
  }
  int octet = 0;
  batch_layout(ctx, rc.pl.L_eff, S, B, octet);
  if (use_prefix) {
    // the prefix's states are in the layout they were built in
    octet = ctx->prefix_octet;
    if (octet && B < S) {
      B &= ~(int64_t)7;
      if (B < 8) return fail(DTC_EINVAL, "batch too small for the prefix's octet layout");
    }
  }
  rc.octet_bits = octet;
  const int64_t Bp = dtc::octet_padded(B, octet);
  if (ctx->verbose) {
    size_t fr = 0, to = 0;
    (void)hipMemGetInfo(&fr, &to);
    std::fprintf(stderr, "[dtc] L=%d states=%lld batch=%lld state=%.3f GiB free=%.1f/%.1f GiB\n",
                 L, (long long)S, (long long)B, per_state / (1 << 30), fr / 1073741824.0,
                 to / 1073741824.0);
  }

  DTC_TRY(ensure(ctx->F, (size_t)(Bp * pl.len * 16)));
  if (want_e) DTC_TRY(ensure(ctx->E, (size_t)(Bp * pl.len * 16)));
  const int max_obs = std::max(n_obs_f, 2);
  DTC_TRY(ensure(ctx->partial, (size_t)B * pl.n_tiles * max_obs * sizeof(double)));
  DTC_TRY(ensure(ctx->vals_f, (size_t)B * T * n_obs_f * sizeof(double)));
  if (want_e) DTC_TRY(ensure(ctx->vals_e, (size_t)B * T * 2 * sizeof(double)));
  DTC_TRY(ensure(ctx->basis, (size_t)B * sizeof(int64_t)));

  DTC_TRY(ensure_host(ctx->host_f, (size_t)B * T * n_obs_f));
  if (want_e) DTC_TRY(ensure_host(ctx->host_e, (size_t)B * T * 2));
  double* const hv_f = ctx->host_f.p;
  double* const hv_e = ctx->host_e.p;
  std::vector<int64_t> masks(B);

  for (int64_t bs = 0; bs < S; bs += B) {
    const int nb = (int)std::min<int64_t>(B, S - bs);
    for (int b = 0; b < nb; ++b) {
      const int64_t g = bs + b;
      masks[b] = use_prefix ? ctx->prefix_masks[g]
                            : (int64_t)init_state_mask(rc, (uint64_t)(traj_offset + g % n_traj));
    }
    double2* F = (double2*)ctx->F.p;
    double2* E = (double2*)ctx->E.p;
#ifdef DTC_DEV_KNOBS
    // development builds: DTC_FE_SWAP=1 runs the forward in the echo buffer and
    // the echo chains in the forward buffer (buffer-placement A/B)
    if (want_e && !use_prefix && std::getenv("DTC_FE_SWAP")) std::swap(F, E);
#endif
    // the first forward pass reads the prefix states (or the basis states in F)
    // (bs is a multiple of 8 in the octet layout: the batch starts an octet)
    const double2* F0 = use_prefix ? (const double2*)ctx->prefix.p + (size_t)bs * pl.len : F;
    if (!use_prefix) {
      DTC_HIP(hipMemcpyAsync(ctx->basis.p, masks.data(), nb * sizeof(int64_t),
                             hipMemcpyHostToDevice, ctx->stream));
    }
    DTC_HIP(hipMemsetAsync(ctx->vals_f.p, 0, (size_t)nb * T * n_obs_f * sizeof(double),
                           ctx->stream));
    if (want_e)
      DTC_HIP(hipMemsetAsync(ctx->vals_e.p, 0, (size_t)nb * T * 2 * sizeof(double),
                             ctx->stream));

    // DTC_NO_LIGHTCONE=1: keep the chains' last two passes (development A/B)
    const bool lc_enabled = ctx->lightcone;
    // Forward chain K_1 D K_2 D ... K_P D; after each D_p: measure t = p - t_offset
    // and branch the echo at t off F.  The whole batch schedule is built first.
    // Device-like noise (r5): the forward runs one kick layer ahead, one pass
    // per period as in the unitary case, when every echo chain's first pass
    // folds into the forward's dual pass -- the chain's echo start is then
    // taken before that layer, so the layer (a Kraus kick, not invertible) is
    // never undone; if any chain does not fold, the schedule is rebuilt with
    // K-D forward passes (two passes per period, nothing run ahead).
    std::vector<Launch> sched;
    bool dev_ahead = rc.device && ctx->dual && ctx->runahead;
    for (;;) {
    sched.clear();
    bool all_folded = true;
    const bool dev_kd = rc.device && !dev_ahead;  // device-like noise, K-D forward
    if (P > n_pre) {
      Chain fw = forward_chain(pl, n_pre + 1, P - n_pre, dtc::kStreamForward);
      fw.post_after_d = !dev_kd;
      // start on a group without the probe site: every echo chain then ends
      // with its kick-only pass on such a group, which the probe does not need
      // (two groups: the closing groups alternate with p, see below)
      fw.prio.resize(pl.groups.size());
      for (size_t g = 0; g < pl.groups.size(); ++g)
        fw.prio[g] = (int)g + (((group_bits(pl.groups[g]) >> pr->probe_site) & 1ull)
                                   ? (int)pl.groups.size() : 0);
      while (!fw.done()) {
        PassSpec ps = next_pass(fw);
        const int p = ps.d_index + n_pre;  // the chain counts its own periods
        const int t = p - pr->t_offset;
        const bool closes = ps.diag != dtc::kDiagNone;
        const bool meas = closes && want_f && t >= 0 && t >= pr->t_first;
        sched.push_back(Launch{ps, sched.empty() ? F0 : F, F, meas ? meas_f : dtc::kMeasNone, 0,
                               n_obs_f,
                               meas ? (double*)ctx->vals_f.p + (size_t)t * n_obs_f : nullptr,
                               (int64_t)T * n_obs_f});
        if (!closes || !want_e || t < 0 || t < pr->t_first) continue;
        std::vector<int> ahead(pl.groups.size());
        for (size_t g = 0; g < pl.groups.size(); ++g) ahead[g] = fw.kc[g] > ps.d_index;
        Chain ec = echo_chain(pl, p, (uint32_t)(1 + t), ahead);
        // run ahead under device-like noise, a chain whose first pass undoes
        // the forward's run-ahead layer must fold (the undo of a Kraus kick
        // cannot run); the sweep's last chain, after a K-D, has none
        bool must_fold = false;
        for (size_t g = 0; g < pl.groups.size(); ++g) must_fold |= dev_ahead && ahead[g];
        if (rc.device && ctx->dual) {
          // device-like noise: the chain starts on the group whose forward
          // K-D closed the period (the dual pass below)
          ec.prio.resize(pl.groups.size());
          for (size_t g = 0; g < pl.groups.size(); ++g)
            ec.prio[g] = (int)g == ps.group ? -1 : (int)g;
        }
        const double2* src = F;
        const size_t chain0 = sched.size();
        while (!ec.done()) {
          PassSpec es = next_pass(ec);
          sched.push_back(Launch{es, src, E, dtc::kMeasNone, 1, 2, nullptr, (int64_t)T * 2});
          src = E;
        }
        // A chain that ends with a kick-only pass on a group without the probe
        // site: unitary single-site kicks on other sites leave <Z_j> unchanged
        // (K_i^+ Z_j K_i = Z_j), so that pass is dropped and the probe is read
        // after the previous one.  Not for device-like noise: its Kraus kicks
        // are not unitary and change the trajectory weight.
        if (!rc.device && sched.size() - chain0 >= 2) {
          const Launch& l = sched.back();
          const bool kick_only = l.ps.diag == dtc::kDiagNone && !l.ps.post.enabled;
          if (kick_only && !((group_bits(pl.groups[l.ps.group]) >> pr->probe_site) & 1ull))
            sched.pop_back();
        }
        // Light cone of <Z_j> through the chain's last kick layers (unitary
        // single-site kicks, D diagonal with nearest-neighbour couplings): the
        // last layer X_n matters only on j, X_{n-1} on j-1..j+1, X_{n-r} on
        // j-r..j+r.  The chain's last k passes (k = 4 .. 2, the most that fit)
        // become one measure-only pass over a tile holding the 8-site window
        // of the kicks left: their layers, restricted to the cone, with D*
        // between them, then the probe.
        if (!rc.device && lc_enabled && sched.size() - chain0 >= 2)
          lc_merge(rc, sched, chain0, pr->probe_site, ctx->lc_wide, ctx->lc_wide3);
        sched.back().meas_mode = dtc::kMeasProbe;
        sched.back().meas_out = (double*)ctx->vals_e.p + (size_t)t * 2;
        // the echo state is only measured: the chain's last pass reads its
        // tiles and stores nothing (the next chain starts from F again)
        sched.back().no_store = 1;
        // Dual pass: the forward K-D-K on G just before the chain computes
        // K_{p+1} D K_p (input); the chain's first pass, on the same G, is
        // undo(K_{p+1}) D^* K'_1 of that -- so K'_1 K_p (input), which the
        // forward pass forms from its own tile after the pre-kick and stores
        // to E: the chain's first read of F and its own pass go away (48 B
        // per amplitude instead of 64).  Not when the chain is one pass (the
        // light-cone end reads F itself).
        // Device-like noise (no forward layer runs ahead): the forward K-D
        // on G gives D_p K_p (input), the chain's first pass is D^* K'_1 of
        // that on G -- K'_1 K_p (input) again, formed by a K-D dual pass.
        if (ctx->dual && sched.size() - chain0 >= 2 && chain0 >= 1) {
          Launch& f = sched[chain0 - 1];
          const Launch& e = sched[chain0];
          const int fs = dev_kd ? dtc::kShapeKD : dtc::kShapeKDK;
          const int es = dev_kd ? dtc::kShapeDK : dtc::kShapeKDK;
          // (the dual kernels carry the probe at most: not with per-site Z)
          const bool fok = pass_shape(f.ps) == fs && !f.basis && f.src == F &&
                           pl.groups[f.ps.group].tb == dtc::kTileBits &&
                           (f.meas_mode == dtc::kMeasNone || f.meas_mode == dtc::kMeasProbe);
          const bool eok =
              pass_shape(e.ps) == es && e.ps.lc_w0 < 0 && e.ps.group == f.ps.group &&
              e.ps.post.enabled &&
              (dev_kd ? e.ps.post.skip == 0 && f.ps.pre.skip == 0
                      : e.ps.pre.mode == dtc::kKickUndo && e.ps.pre.skip == 0 &&
                            f.ps.post.skip == 0);
          // the fold is exact only when the chain's first pass conjugates the
          // forward's diagonal (one table per instance; d_index only counts
          // each chain's own periods) and, in the unitary case, undoes exactly
          // the forward's post-kick: check it, so a different chain order
          // falls back to the separate passes instead of folding wrongly
          const bool same_d = f.ps.diag == dtc::kDiagFwd && e.ps.diag == dtc::kDiagConj;
          const bool undoes_post =
              dev_kd || (f.ps.post.enabled && f.ps.post.mode == dtc::kKickForward &&
                            e.ps.pre.row == f.ps.post.row &&
                            e.ps.pre.stream == f.ps.post.stream &&
                            e.ps.pre.rng_period == f.ps.post.rng_period);
          const int fk = (fok && same_d && undoes_post) ? pass_kind(rc, f.ps, fs) : -1;
          const bool kind_ok = rc.device ? (fk == dtc::kKindRXU || fk == dtc::kKindRYU ||
                                            fk == dtc::kKindGen)
                                         : (fk == dtc::kKindRX || fk == dtc::kKindRY ||
                                            fk == dtc::kKindGen);
          const PassSpec branch{f.ps.group, f.ps.pre, e.ps.post, dtc::kDiagNone, 0};
          // (run ahead under device-like noise, the chain's first pass holds an
          // undo of a Kraus kick: its own kind is not a factored one, and it
          // never runs)
          if (fok && eok && kind_ok && (dev_ahead || fk == pass_kind(rc, e.ps, es)) &&
              fk == pass_kind(rc, branch, -1)) {
            f.ps2 = branch;
            f.dst2 = E;
            sched.erase(sched.begin() + (std::ptrdiff_t)chain0);
          } else if (must_fold) {
            all_folded = false;
          }
        } else if (must_fold) {
          all_folded = false;
        }
      }
    }
    if (!dev_ahead || all_folded) break;
    dev_ahead = false;
    if (ctx->verbose)
      std::fprintf(stderr, "[dtc] device-noise schedule rebuilt with K-D forward passes "
                           "(an echo chain did not fold into the dual pass)\n");
    }
    for (const Launch& l : sched) ctx->sched_counts[0] += l.dst2 != nullptr;
    if (rc.device) ++ctx->sched_counts[dev_ahead ? 1 : 2];
    if (pl.groups[0].tb == dtc::kMaxTileBits) ++ctx->sched_counts[3];
    if (!use_prefix) DTC_TRY(basis_source(ctx, sched, F, pl.len, nb, octet));
    DTC_TRY(run_launches(ctx, rc, bs, nb, sched));
    DTC_HIP(hipMemcpyAsync(hv_f, ctx->vals_f.p, (size_t)nb * T * n_obs_f * sizeof(double),
                           hipMemcpyDeviceToHost, ctx->stream));
    if (want_e)
      DTC_HIP(hipMemcpyAsync(hv_e, ctx->vals_e.p, (size_t)nb * T * 2 * sizeof(double),
                             hipMemcpyDeviceToHost, ctx->stream));
    DTC_HIP(hipStreamSynchronize(ctx->stream));
    DTC_TRY(settle_pending(ctx));

    const int j = pr->probe_site;
    for (int b = 0; b < nb; ++b) {
      const int64_t g = bs + b;
      const uint64_t m = (uint64_t)masks[b];
      const double zinit = ((m >> j) & 1ull) ? -1.0 : 1.0;
      for (int t = std::max(0, pr->t_first); t < T; ++t) {
        const bool at_init = (t + pr->t_offset == 0);
        const double* vf = hv_f + ((size_t)b * T + t) * n_obs_f;
        const double zj_f = at_init ? zinit : (want_z ? vf[1 + j] : vf[1]);
        if (pr->want_fwd) fwd[(size_t)g * T + t] = ro_a * (fac * zinit * zj_f) + ro_b;
        if (want_z) {
          double* zo = zsite + ((size_t)g * T + t) * L;
          for (int i = 0; i < L; ++i)
            zo[i] = at_init ? (((m >> i) & 1ull) ? -1.0 : 1.0) : vf[1 + i];
        }
        if (want_e) {
          const double zj_e = at_init ? zinit : hv_e[((size_t)b * T + t) * 2 + 1];
          echo[(size_t)g * T + t] = ro_a * (fac * zinit * zj_e) + ro_b;
        }
      }
    }
  }
  return DTC_OK;
}

// Forward prefix: the initial states of all n_inst * n_traj trajectories
// taken through periods 1..n_periods (post_after_d as the forward chain of
// autocorr_impl, so no kick is pending) into ctx->prefix, in batches in place.
int prefix_build_impl(dtc_ctx* ctx, const dtc_problem* pr, const dtc_noise* nz,
                      const dtc_device_noise* dv, uint64_t seed, int64_t traj_offset,
                      int32_t n_traj, int32_t n_periods) {
  if (!ctx) return fail(DTC_EINVAL, "null ctx");
  DTC_TRY(check_problem(pr, nz));
  if (n_traj < 1) return fail(DTC_EINVAL, "n_traj must be >= 1");
  if (traj_offset < 0) return fail(DTC_EINVAL, "traj_offset must be >= 0");
  if (n_periods < 1 || n_periods > pr->T - 1 + pr->t_offset)
    return fail(DTC_EINVAL, "n_periods must be in [1, T - 1 + t_offset]");
  DTC_HIP(hipSetDevice(ctx->device));
  RunCfg rc;
  rc.prob = pr;
  rc.pl = make_plan(pr->L);
  rc.seed = seed;
  rc.traj_offset = traj_offset;
  rc.n_traj = n_traj;
  rc.noisy = nz->p > 0.0 ? 1 : 0;
  rc.row_kind = classify_rows(pr);
  thresholds(nz->p, &rc.thr1, &rc.thr2, &rc.thr3);
  if (dv) DTC_TRY(setup_device_noise(ctx, pr, dv, rc));
  const Plan& pl = rc.pl;
  DTC_TRY(upload_tables(ctx, pr, pl));
  const int64_t S = (int64_t)pr->n_inst * n_traj;
  ctx->prefix_periods = -1;
  // batches of up to 4096 states (multiples of 8): the octet layout whenever
  // there is an octet; autocorr_prefixed reads them in this layout
  int64_t B = 4096;
  int octet = 0;
  batch_layout(ctx, pl.L_eff, S, B, octet);
  rc.octet_bits = octet;
  DTC_TRY(ensure(ctx->prefix, (size_t)dtc::octet_padded(S, octet) * pl.len * 16));
  ctx->prefix_masks.resize(S);
  for (int64_t g = 0; g < S; ++g)
    ctx->prefix_masks[g] = (int64_t)init_state_mask(rc, (uint64_t)(traj_offset + g % n_traj));
  DTC_TRY(ensure(ctx->basis, (size_t)B * sizeof(int64_t)));
  for (int64_t bs = 0; bs < S; bs += B) {
    const int nb = (int)std::min<int64_t>(B, S - bs);
    double2* F = (double2*)ctx->prefix.p + (size_t)bs * pl.len;
    DTC_HIP(hipMemcpyAsync(ctx->basis.p, ctx->prefix_masks.data() + bs, nb * sizeof(int64_t),
                           hipMemcpyHostToDevice, ctx->stream));
    Chain fw = forward_chain(pl, 1, n_periods, dtc::kStreamForward);
    fw.post_after_d = !rc.device;
    std::vector<Launch> sched;
    while (!fw.done())
      sched.push_back(Launch{next_pass(fw), F, F, dtc::kMeasNone, 0, 2, nullptr, 0});
    DTC_TRY(basis_source(ctx, sched, F, pl.len, nb, octet));
    DTC_TRY(run_launches(ctx, rc, bs, nb, sched));
    DTC_HIP(hipStreamSynchronize(ctx->stream));  // the staged pass list is reused
  }
  DTC_TRY(settle_pending(ctx));
  ctx->prefix_periods = n_periods;
  ctx->prefix_states = S;
  ctx->prefix_traj_offset = traj_offset;
  ctx->prefix_n_traj = n_traj;
  ctx->prefix_len = pl.len;
  ctx->prefix_device = dv ? 1 : 0;
  ctx->prefix_octet = octet;
  ctx->prefix_hash = prefix_hash(pr, n_periods);
  return DTC_OK;
}

}  // namespace

extern "C" {

int dtc_autocorr(dtc_ctx* ctx, const dtc_problem* pr, const dtc_noise* nz, uint64_t seed,
                 int64_t traj_offset, int32_t n_traj, double* fwd, double* echo,
                 double* zsite) {
  return autocorr_impl(ctx, pr, nz, nullptr, seed, traj_offset, n_traj, fwd, echo, zsite);
}

int dtc_autocorr_device(dtc_ctx* ctx, const dtc_problem* pr, const dtc_device_noise* dv,
                        uint64_t seed, int64_t traj_offset, int32_t n_traj, double* fwd,
                        double* echo, double* zsite) {
  if (!dv) return fail(DTC_EINVAL, "null device noise");
  const dtc_noise nz{0.0, 0, 0};
  return autocorr_impl(ctx, pr, &nz, dv, seed, traj_offset, n_traj, fwd, echo, zsite);
}

int dtc_prefix_build(dtc_ctx* ctx, const dtc_problem* pr, const dtc_noise* nz,
                     const dtc_device_noise* dv, uint64_t seed, int64_t traj_offset,
                     int32_t n_traj, int32_t n_periods) {
  const dtc_noise none{0.0, 0, 0};
  if (!dv && !nz) return fail(DTC_EINVAL, "null noise");
  return prefix_build_impl(ctx, pr, dv ? &none : nz, dv, seed, traj_offset, n_traj, n_periods);
}

int dtc_autocorr_prefixed(dtc_ctx* ctx, const dtc_problem* pr, const dtc_noise* nz,
                          const dtc_device_noise* dv, uint64_t seed, int64_t traj_offset,
                          int32_t n_traj, double* fwd, double* echo) {
  const dtc_noise none{0.0, 0, 0};
  if (!dv && !nz) return fail(DTC_EINVAL, "null noise");
  return autocorr_impl(ctx, pr, dv ? &none : nz, dv, seed, traj_offset, n_traj, fwd, echo,
                       nullptr, true);
}

int dtc_prefix_release(dtc_ctx* ctx) {
  if (!ctx) return fail(DTC_EINVAL, "null ctx");
  DTC_HIP(hipStreamSynchronize(ctx->stream));
  release(ctx->prefix);
  ctx->prefix_masks.clear();
  ctx->prefix_periods = -1;
  return DTC_OK;
}

int dtc_apply_periods(dtc_ctx* ctx, const dtc_problem* pr, const dtc_noise* nz, uint64_t seed,
                      int32_t inst, int64_t traj, uint32_t stream, int32_t first_period,
                      int32_t n_periods, int32_t inverse, double* state, double* zsite_out) {
  if (!ctx || !state) return fail(DTC_EINVAL, "null ctx/state");
  DTC_TRY(check_problem(pr, nz));
  if (inst < 0 || inst >= pr->n_inst) return fail(DTC_EINVAL, "inst out of range");
  if (traj < 0) return fail(DTC_EINVAL, "traj must be >= 0");
  if (n_periods < 0) return fail(DTC_EINVAL, "n_periods must be >= 0");
  const int n_rows = std::max(1, pr->T - 1 + pr->t_offset);
  if (n_periods > 0) {
    const int lo = inverse ? first_period - n_periods + 1 : first_period;
    const int hi = inverse ? first_period : first_period + n_periods - 1;
    if (lo < 1 || hi > n_rows) return fail(DTC_EINVAL, "period range outside kick table");
  }
  DTC_HIP(hipSetDevice(ctx->device));
  RunCfg rc;
  rc.prob = pr;
  rc.pl = make_plan(pr->L);
  rc.seed = seed;
  rc.traj_offset = traj;
  rc.n_traj = 1;
  rc.noisy = nz->p > 0.0 ? 1 : 0;
  rc.row_kind = classify_rows(pr);
  thresholds(nz->p, &rc.thr1, &rc.thr2, &rc.thr3);
  const Plan& pl = rc.pl;
  const int L = pr->L;
  DTC_TRY(upload_tables(ctx, pr, pl));
  DTC_TRY(ensure(ctx->F, (size_t)pl.len * 16));
  DTC_TRY(ensure(ctx->partial, (size_t)pl.n_tiles * (1 + L) * sizeof(double)));
  DTC_TRY(ensure(ctx->vals_f, (size_t)(1 + L) * sizeof(double)));
  double2* F = (double2*)ctx->F.p;
  DTC_HIP(hipMemsetAsync(F, 0, (size_t)pl.len * 16, ctx->stream));
  DTC_HIP(hipMemcpyAsync(F, state, ((size_t)1 << L) * 16, hipMemcpyHostToDevice, ctx->stream));
  const int64_t batch_start = inst;  // n_traj = 1: g = inst -> (inst, traj)
  if (n_periods > 0) {
    Chain ch;
    if (inverse) {
      ch = echo_chain(pl, first_period, stream, std::vector<int>(pl.groups.size(), 0));
      // echo_chain counts periods p..1; re-base so the first inverse period is
      // first_period and there are n_periods of them
      ch.X.resize(1);
      for (int k = 1; k <= n_periods; ++k)
        ch.X.push_back(dtc::KickDesc{1, first_period - k, dtc::kKickInverse, stream,
                                     (uint32_t)k});
    } else {
      ch = forward_chain(pl, first_period, n_periods, stream);
    }
    DTC_TRY(run_chain(ctx, rc, batch_start, 1, ch, F, F,
                      zsite_out ? dtc::kMeasSites : dtc::kMeasNone, 1 + L,
                      (double*)ctx->vals_f.p, 1 + L));
  }
  DTC_HIP(hipMemcpyAsync(state, F, ((size_t)1 << L) * 16, hipMemcpyDeviceToHost, ctx->stream));
  if (zsite_out && n_periods > 0)
    DTC_HIP(hipMemcpyAsync(zsite_out, ctx->vals_f.p, (size_t)(1 + L) * sizeof(double),
                           hipMemcpyDeviceToHost, ctx->stream));
  DTC_HIP(hipStreamSynchronize(ctx->stream));
  DTC_TRY(settle_pending(ctx));
  if (zsite_out && n_periods == 0) {
    // no kernel ran: reduce on the host copy
    std::vector<double> acc(1 + L, 0.0);
    for (size_t x = 0; x < ((size_t)1 << L); ++x) {
      const double pr2 = state[2 * x] * state[2 * x] + state[2 * x + 1] * state[2 * x + 1];
      acc[0] += pr2;
      for (int i = 0; i < L; ++i) acc[1 + i] += ((x >> i) & 1) ? -pr2 : pr2;
    }
    for (int i = 0; i <= L; ++i) zsite_out[i] = acc[i];
  }
  return DTC_OK;
}


namespace {

// sums: z, zz, x are per-instance sums over the trajectories ([n_inst][T][.],
// dtc_energy_sums) instead of per-trajectory rows
int energy_impl(dtc_ctx* ctx, const dtc_problem* pr, const dtc_noise* nz,
                const dtc_device_noise* dv, uint64_t seed, int64_t traj_offset, int32_t n_traj,
                double* z, double* zz, double* x, bool sums = false) {
  if (!ctx || !z || !x || (!zz && pr && pr->L > 1)) return fail(DTC_EINVAL, "null ctx/outputs");
  DTC_TRY(check_problem(pr, nz));
  if (n_traj < 1) return fail(DTC_EINVAL, "n_traj must be >= 1");
  if (traj_offset < 0) return fail(DTC_EINVAL, "traj_offset must be >= 0");
  DTC_HIP(hipSetDevice(ctx->device));

  RunCfg rc;
  rc.prob = pr;
  rc.pl = make_plan(pr->L);
  rc.seed = seed;
  rc.traj_offset = traj_offset;
  rc.n_traj = n_traj;
  rc.noisy = nz->p > 0.0 ? 1 : 0;
  rc.row_kind = classify_rows(pr);
  thresholds(nz->p, &rc.thr1, &rc.thr2, &rc.thr3);
  if (dv) DTC_TRY(setup_device_noise(ctx, pr, dv, rc));
  const Plan& pl = rc.pl;
  const int T = pr->T, L = pr->L;
  const int P = T - 1 + pr->t_offset;
  const int n_v = 3 * L;    // per time: norm, Z_i, Z_i Z_i+1, X_i
  const int n_obs = 4 * L;  // per pass: the above (mid-pass) + X_i before the pre-kick
  if (n_obs > dtc::kThreads) return fail(DTC_EINVAL, "dtc_energy: L > 64");
  DTC_TRY(upload_tables(ctx, pr, pl));

  const int64_t S = (int64_t)pr->n_inst * n_traj;
  const double per_state = (double)pl.len * 16.0;
  int64_t B = pr->batch;
  if (B <= 0) {
    size_t free_b = 0, total_b = 0;
    DTC_HIP(hipMemGetInfo(&free_b, &total_b));
    free_b += ctx->F.n + (dv ? ctx->E.n : 0);
    const double budget = std::min(0.6 * (double)free_b, 64.0 * (1ull << 30));
    B = std::max<int64_t>(1, std::min<int64_t>((int64_t)(budget / (dv ? 2 * per_state : per_state)),
                                               4096));
  }
  int octet = 0;
  batch_layout(ctx, rc.pl.L_eff, S, B, octet);
  rc.octet_bits = octet;
  const int64_t Bp = dtc::octet_padded(B, octet);
  DTC_TRY(ensure(ctx->F, (size_t)(Bp * pl.len * 16)));
  if (dv) DTC_TRY(ensure(ctx->E, (size_t)(Bp * pl.len * 16)));
  DTC_TRY(ensure(ctx->partial, (size_t)B * pl.n_tiles * n_obs * sizeof(double)));
  DTC_TRY(ensure(ctx->vals_f, (size_t)B * T * n_v * sizeof(double)));
  DTC_TRY(ensure(ctx->basis, (size_t)B * sizeof(int64_t)));
  // per-instance sums: at most (B - 1) / n_traj + 2 instances per batch
  const int64_t max_inst_b = std::min<int64_t>(pr->n_inst, (B - 1) / n_traj + 2);
  if (sums) {
    DTC_TRY(ensure(ctx->vals_e, (size_t)max_inst_b * T * n_v * sizeof(double)));
    const size_t n_out = (size_t)pr->n_inst * T;
    std::fill(z, z + n_out * L, 0.0);
    std::fill(x, x + n_out * L, 0.0);
    if (L > 1) std::fill(zz, zz + n_out * (L - 1), 0.0);
  }
  DTC_TRY(ensure_host(ctx->host_f, (size_t)(sums ? max_inst_b : B) * T * n_v));
  double* const hv_f = ctx->host_f.p;
  std::vector<int64_t> masks(B);

  // The schedule: the forward chain one kick layer past the last period
  // (X_P, no D after it), every pass measuring in flight (meas_parts):
  //  * a pass closing period p: Z, ZZ after the diagonal and X of its sites
  //    before their post-kick X_p -> time p - t_offset;
  //  * a pass whose pre-kick is X_nd (nd diagonals applied): X of its sites
  //    before that kick -> time nd - t_offset, unless its sites' X at that
  //    time is already taken (one group: the post-kick of the previous pass).
  // Each group's X at a time is taken exactly once (checked below); the
  // reduce accumulates the X ranges into the zeroed per-time rows.
  //
  // Device-like noise: a non-unitary kick on one site changes <X> of the
  // others, so nothing is measured across a kick.  The chain starts no layer
  // in a pass that applies D (2 passes per period); after the pass closing
  // period p the state is exactly the state at p: Z, ZZ mid-pass, then X by
  // one noiseless basis-change pass per site group (E = H^L F).
  struct EPass {
    PassSpec ps;
    int parts, t_mid, t_pre;
    bool xbasis;
    const int64_t* basis = nullptr;
    int no_store = 0;
  };
  std::vector<EPass> sched;
  if (P > 0 && dv) {
    Chain fw = forward_chain(pl, 1, P, dtc::kStreamForward);
    fw.post_after_d = false;
    while (!fw.done()) {
      EPass e{next_pass(fw), 0, -1, -1, false};
      if (e.ps.diag != dtc::kDiagNone) {
        const int t = e.ps.d_index - pr->t_offset;
        if (t >= 0 && t < T) {
          e.parts = dtc::kPartZ;
          e.t_mid = t;
          e.xbasis = true;
        }
      }
      sched.push_back(e);
    }
  } else if (P > 0) {
    const int G = (int)pl.groups.size();
    Chain fw = forward_chain(pl, 1, P + 1, dtc::kStreamForward);
    fw.trailing_d = false;
    fw.X[P].row = P - 1;  // never observed: any valid table row
    std::vector<char> x_done((size_t)T * G, 0);
    while (!fw.done()) {
      const int nd = fw.nd;
      EPass e{next_pass(fw), 0, -1, -1, false};
      const int g = e.ps.group;
      if (e.ps.diag != dtc::kDiagNone) {
        const int t = e.ps.d_index - pr->t_offset;
        if (t >= 0 && t < T) {
          e.parts |= dtc::kPartZ;
          e.t_mid = t;
          if (e.ps.post.enabled) {
            e.parts |= dtc::kPartXPost;
            x_done[(size_t)t * G + g] = 1;
          }
        }
      }
      const int te = nd - pr->t_offset;
      if (e.ps.pre.enabled && nd >= 1 && te >= 0 && te < T && !x_done[(size_t)te * G + g]) {
        e.parts |= dtc::kPartXPre;
        e.t_pre = te;
        x_done[(size_t)te * G + g] = 1;
      }
      sched.push_back(e);
    }
    for (int t = 0; t < T; ++t)
      for (int g = 0; g < G; ++g)
        if (t + pr->t_offset >= 1 && !x_done[(size_t)t * G + g])
          return fail(DTC_EINVAL, "internal: dtc_energy left an X group unmeasured");
    // the extra kick layer's pass only measures X: its state is never read
    if (sched.size() >= 2 && pass_shape(sched.back().ps) == dtc::kShapeK &&
        (sched.back().parts & dtc::kPartXPre) && !(sched.back().parts & dtc::kPartZ))
      sched.back().no_store = 1;
  }

  for (int64_t bs = 0; bs < S; bs += B) {
    const int nb = (int)std::min<int64_t>(B, S - bs);
    for (int b = 0; b < nb; ++b)
      masks[b] = (int64_t)init_state_mask(rc, (uint64_t)(traj_offset + (bs + b) % n_traj));
    double2* F = (double2*)ctx->F.p;
    double* vals = (double*)ctx->vals_f.p;
    DTC_HIP(hipMemcpyAsync(ctx->basis.p, masks.data(), nb * sizeof(int64_t),
                           hipMemcpyHostToDevice, ctx->stream));
    DTC_TRY(basis_source(ctx, sched, F, pl.len, nb, octet));
    DTC_HIP(hipMemsetAsync(vals, 0, (size_t)nb * T * n_v * sizeof(double), ctx->stream));
    const int64_t vs = (int64_t)T * n_v;
    // kick records of the schedule's passes: one prep launch per segment
    // (the X-basis passes of the device path build their own)
    const size_t per_pass = (size_t)nb * dtc::kRecPerState * sizeof(dtc::KickRec);
    const size_t seg = std::max<size_t>(1, std::min<size_t>(sched.size(), (size_t)(256u << 20) / per_pass));
    DTC_TRY(ensure(ctx->recs, seg * per_pass));
    ctx->pk_host.resize(sched.size());
    for (size_t i = 0; i < sched.size(); ++i) ctx->pk_host[i] = pass_kick(rc, sched[i].ps);
    DTC_TRY(ensure(ctx->pk, sched.size() * sizeof(dtc::PassKick)));
    DTC_HIP(hipMemcpyAsync(ctx->pk.p, ctx->pk_host.data(), sched.size() * sizeof(dtc::PassKick),
                           hipMemcpyHostToDevice, ctx->stream));
    for (size_t i = 0; i < sched.size(); ++i) {
      const EPass& e = sched[i];
      if (i % seg == 0) {
        dtc::PrepArgs Pp = prep_args(ctx, rc, bs, nb);
        Pp.passes = (const dtc::PassKick*)ctx->pk.p + i;
        Pp.n_pass = (int)std::min(seg, sched.size() - i);
        Pp.out = (dtc::KickRec*)ctx->recs.p;
        DTC_HIP(dtc::launch_prep(Pp, ctx->stream));
      }
      const dtc::KickRec* recs = (const dtc::KickRec*)ctx->recs.p + (i % seg) * nb * dtc::kRecPerState;
      DTC_TRY(launch_pass_spec(ctx, rc, bs, nb, e.ps, F, F,
                               e.parts ? dtc::kMeasEnergy : dtc::kMeasNone, 0, n_obs, nullptr,
                               0, recs, e.parts, e.no_store, e.basis));
      if (e.parts & dtc::kPartZ)
        DTC_TRY(launch_reduce_prof(ctx, pl.n_tiles, n_obs, nb, vals + (size_t)e.t_mid * n_v, vs,
                                   0, (e.parts & dtc::kPartXPost) ? 3 * L : 2 * L, 1));
      if (e.parts & dtc::kPartXPre)
        DTC_TRY(launch_reduce_prof(ctx, pl.n_tiles, n_obs, nb,
                                   vals + (size_t)e.t_pre * n_v + 2 * L, vs, 3 * L, L, 1));
      if (e.xbasis) {
        double2* E = (double2*)ctx->E.p;
        const int G = (int)pl.groups.size();
        for (int g = 0; g < G; ++g) {
          PassSpec xs{g, no_kick(), no_kick(), dtc::kDiagNone, 0};
          xs.pre = dtc::KickDesc{1, 0, dtc::kKickBasisX, 0u, 0u, 0u};
          const bool last = g == G - 1;
          DTC_TRY(launch_pass_spec(ctx, rc, bs, nb, xs, g == 0 ? F : E, E,
                                   last ? dtc::kMeasSites : dtc::kMeasNone, 1, 1 + L, nullptr, 0));
        }
        DTC_TRY(launch_reduce_prof(ctx, pl.n_tiles, 1 + L, nb,
                                   vals + (size_t)e.t_mid * n_v + 2 * L, vs, 1, L, 1));
      }
    }
    if (sums) {
      // the batch's rows summed per instance on the device (the rows of the
      // initial time are formed from the masks below, not read)
      const int64_t i0 = bs / n_traj, n_ib = (bs + nb - 1) / n_traj - i0 + 1;
      DTC_HIP(dtc::launch_traj_sum(vals, nb, (int)vs, bs, n_traj, (double*)ctx->vals_e.p,
                                   ctx->stream));
      DTC_HIP(hipMemcpyAsync(hv_f, ctx->vals_e.p, (size_t)n_ib * vs * sizeof(double),
                             hipMemcpyDeviceToHost, ctx->stream));
      DTC_HIP(hipStreamSynchronize(ctx->stream));
      DTC_TRY(settle_pending(ctx));
      for (int64_t i = 0; i < n_ib; ++i) {
        const int64_t inst = i0 + i;
        for (int t = 0; t < T; ++t) {
          if (t + pr->t_offset == 0) continue;
          const double* vf = hv_f + ((size_t)i * T + t) * n_v;
          const double* vx = vf + 2 * L - 1;
          double* zo = z + ((size_t)inst * T + t) * L;
          double* xo = x + ((size_t)inst * T + t) * L;
          for (int k = 0; k < L; ++k) {
            zo[k] += vf[1 + k];
            xo[k] += vx[1 + k];
          }
          if (L > 1) {
            double* zzo = zz + ((size_t)inst * T + t) * (L - 1);
            for (int k = 0; k + 1 < L; ++k) zzo[k] += vf[1 + L + k];
          }
        }
      }
      if (pr->t_offset == 0) {
        for (int b = 0; b < nb; ++b) {
          const int64_t inst = (bs + b) / n_traj;
          const uint64_t m = (uint64_t)masks[b];
          double* zo = z + (size_t)inst * T * L;
          for (int k = 0; k < L; ++k) zo[k] += ((m >> k) & 1ull) ? -1.0 : 1.0;
          if (L > 1) {
            double* zzo = zz + (size_t)inst * T * (L - 1);
            for (int k = 0; k + 1 < L; ++k)
              zzo[k] += (((m >> k) ^ (m >> (k + 1))) & 1ull) ? -1.0 : 1.0;
          }
        }
      }
      continue;
    }
    DTC_HIP(hipMemcpyAsync(hv_f, vals, (size_t)nb * T * n_v * sizeof(double),
                           hipMemcpyDeviceToHost, ctx->stream));
    DTC_HIP(hipStreamSynchronize(ctx->stream));
    DTC_TRY(settle_pending(ctx));
    for (int b = 0; b < nb; ++b) {
      const int64_t g = bs + b;
      const uint64_t m = (uint64_t)masks[b];
      for (int t = 0; t < T; ++t) {
        const bool at_init = (t + pr->t_offset == 0);
        const double* vf = hv_f + ((size_t)b * T + t) * n_v;
        const double* vx = vf + 2 * L - 1;  // X_i at vx[1 + i]
        double* zo = z + ((size_t)g * T + t) * L;
        double* xo = x + ((size_t)g * T + t) * L;
        for (int i = 0; i < L; ++i) {
          zo[i] = at_init ? (((m >> i) & 1ull) ? -1.0 : 1.0) : vf[1 + i];
          xo[i] = at_init ? 0.0 : vx[1 + i];
        }
        if (L > 1) {
          double* zzo = zz + ((size_t)g * T + t) * (L - 1);
          for (int i = 0; i + 1 < L; ++i)
            zzo[i] = at_init ? ((((m >> i) ^ (m >> (i + 1))) & 1ull) ? -1.0 : 1.0)
                             : vf[1 + L + i];
        }
      }
    }
  }
  return DTC_OK;
}

}  // namespace

int dtc_energy(dtc_ctx* ctx, const dtc_problem* pr, const dtc_noise* nz, uint64_t seed,
               int64_t traj_offset, int32_t n_traj, double* z, double* zz, double* x) {
  return energy_impl(ctx, pr, nz, nullptr, seed, traj_offset, n_traj, z, zz, x);
}

int dtc_energy_device(dtc_ctx* ctx, const dtc_problem* pr, const dtc_device_noise* dv,
                      uint64_t seed, int64_t traj_offset, int32_t n_traj, double* z, double* zz,
                      double* x) {
  if (!dv) return fail(DTC_EINVAL, "null device noise");
  const dtc_noise nz{0.0, 0, 0};
  return energy_impl(ctx, pr, &nz, dv, seed, traj_offset, n_traj, z, zz, x);
}

int dtc_energy_sums(dtc_ctx* ctx, const dtc_problem* pr, const dtc_noise* nz,
                    const dtc_device_noise* dv, uint64_t seed, int64_t traj_offset,
                    int32_t n_traj, double* z_sum, double* zz_sum, double* x_sum) {
  if (dv) {
    const dtc_noise none{0.0, 0, 0};
    return energy_impl(ctx, pr, &none, dv, seed, traj_offset, n_traj, z_sum, zz_sum, x_sum, true);
  }
  if (!nz) return fail(DTC_EINVAL, "null noise");
  return energy_impl(ctx, pr, nz, nullptr, seed, traj_offset, n_traj, z_sum, zz_sum, x_sum, true);
}

int32_t dtc_plan_groups(int32_t n_bits, uint64_t* masks, int32_t max_groups) {
  if (n_bits < 1 || n_bits > 40 || !masks) return fail(DTC_EINVAL, "bad arguments");
  Plan pl = make_plan(n_bits, true);
  if ((int)pl.groups.size() > max_groups) return fail(DTC_EINVAL, "max_groups too small");
  for (size_t g = 0; g < pl.groups.size(); ++g)
    masks[g] = group_bits(pl.groups[g]) & ((n_bits >= 64) ? ~0ull : ((1ull << n_bits) - 1));
  return (int32_t)pl.groups.size();
}

int dtc_shard_set_basis(dtc_ctx* ctx, const dtc_problem* pr, const dtc_noise* nz,
                        const dtc_shard* sh, uint64_t seed, int64_t traj, double* state) {
  if (!ctx || !state) return fail(DTC_EINVAL, "null ctx/state");
  DTC_TRY(check_problem(pr, nz, 64));
  DTC_TRY(check_shard(pr, sh));
  if (traj < 0) return fail(DTC_EINVAL, "traj must be >= 0");
  DTC_HIP(hipSetDevice(ctx->device));
  uint64_t mask = pr->init_mask;
  if (nz->p > 0.0) {  // as init_state_mask: X/Y errors after a prep X undo the flip
    uint32_t t1, t2, t3;
    thresholds(nz->p, &t1, &t2, &t3);
    for (int i = 0; i < pr->L; ++i) {
      if (!((pr->init_mask >> i) & 1ull)) continue;
      const int pz = dtc::sample_pauli(seed, (uint64_t)traj, dtc::kStreamPrep, 0u, (uint32_t)i,
                                       0u, t1, t2, t3);
      if (pz == 1 || pz == 2) mask &= ~(1ull << i);
    }
  }
  const int nl = sh->n_local;
  const size_t len = (size_t)1 << nl;
  DTC_HIP(hipMemsetAsync(state, 0, len * 16 * sh->n_shards, ctx->stream));
  uint64_t local = 0, rank = 0;
  for (int q = 0; q < pr->L; ++q) {
    const uint64_t bit = (mask >> sh->site_of[q]) & 1;
    if (q < nl) local |= bit << q;
    else rank |= bit << (q - nl);
  }
  const int64_t b = (int64_t)rank - sh->first_rank;
  static const double one[2] = {1.0, 0.0};
  if (b >= 0 && b < sh->n_shards)
    DTC_HIP(hipMemcpyAsync(state + 2 * ((size_t)b * len + local), one, 16,
                           hipMemcpyHostToDevice, ctx->stream));
  DTC_HIP(hipStreamSynchronize(ctx->stream));
  return DTC_OK;
}

}  // extern "C"

namespace {

uint64_t fnv(uint64_t h, const void* p, size_t n) {
  const unsigned char* c = (const unsigned char*)p;
  for (size_t i = 0; i < n; ++i) h = (h ^ c[i]) * 1099511628211ull;
  return h;
}

// A small device-table cache (most recent last, at most 4 entries): the entry
// for `key`, built by `fill` (host bytes) on a miss.  Evicting an entry waits
// for the stream (its table may be in use); a sweep alternates two bit maps,
// so that happens only when a caller switches problems.
template <class Fill>
int cached_table(dtc_ctx* ctx, std::vector<dtc_ctx::ShardTables>& cache, uint64_t key,
                 Fill fill, const void** out) {
  for (auto& e : cache)
    if (e.key == key) {
      *out = e.diag.p;
      return DTC_OK;
    }
  std::vector<double> host;
  fill(host);
  if (cache.size() >= 4) {
    DTC_HIP(hipStreamSynchronize(ctx->stream));
    release(cache.front().diag);
    cache.erase(cache.begin());
  }
  cache.emplace_back();
  auto& e = cache.back();
  DTC_TRY(ensure(e.diag, host.size() * sizeof(double)));
  DTC_HIP(hipMemcpy(e.diag.p, host.data(), host.size() * sizeof(double), hipMemcpyHostToDevice));
  e.key = key;
  *out = e.diag.p;
  return DTC_OK;
}

// The kick-side tables of a shard bit map: the bit -> site map (cached per
// map) and the logical kick table.  dtc_shard_kick_slice needs only these.
int shard_kick_tables(dtc_ctx* ctx, const dtc_problem* pr, const dtc_shard* sh, RunCfg& rc) {
  const int L = pr->L;
  const int n_rows = std::max(1, pr->T - 1 + pr->t_offset);
  uint64_t mkey = fnv(1469598103934665603ull, sh->site_of, sizeof(int32_t) * 64);
  const void* map = nullptr;
  DTC_TRY(cached_table(ctx, ctx->shard_maps, mkey,
                       [&](std::vector<double>& h) {
                         h.assign(32, 0.0);  // 64 int32 in 32 doubles
                         std::memcpy(h.data(), sh->site_of, 64 * sizeof(int32_t));
                       },
                       &map));
  rc.site_of = (const int*)map;
  const size_t kb = (size_t)n_rows * L * pr->n_sub * 8 * sizeof(double);
  uint64_t kkey = fnv(1469598103934665603ull, &kb, sizeof(kb));
  kkey = fnv(kkey, pr->kick, kb);
  if (kkey != ctx->shard_kick_key || !ctx->shard_kick.p) {
    DTC_HIP(hipStreamSynchronize(ctx->stream));  // the previous table may be in use
    DTC_TRY(ensure(ctx->shard_kick, kb));
    DTC_HIP(hipMemcpy(ctx->shard_kick.p, pr->kick, kb, hipMemcpyHostToDevice));
    ctx->shard_kick_key = kkey;
  }
  rc.kick_tab = (const double2*)ctx->shard_kick.p;
  return DTC_OK;
}

// Device tables of one shard bit map and instance: the effective diagonal per
// held shard (cached per map, instance and angles) plus the kick-side tables.
int shard_tables(dtc_ctx* ctx, const dtc_problem* pr, const dtc_shard* sh, int inst,
                 const Plan& pl, RunCfg& rc) {
  const int L = pr->L, nl = sh->n_local, B = sh->n_shards;
  uint64_t key = 1469598103934665603ull;
  key = fnv(key, &L, sizeof(L));
  key = fnv(key, &sh->n_local, sizeof(int32_t) * 4);
  key = fnv(key, sh->site_of, sizeof(int32_t) * L);
  key = fnv(key, &inst, sizeof(inst));
  key = fnv(key, pr->h + (size_t)inst * L, sizeof(double) * L);
  if (L > 1) key = fnv(key, pr->phi + (size_t)inst * (L - 1), sizeof(double) * (L - 1));
  const void* tab = nullptr;
  DTC_TRY(cached_table(ctx, ctx->shard_cache, key,
                       [&](std::vector<double>& dt) {
                         std::vector<double> he((size_t)B * nl),
                             pe((size_t)B * std::max(nl - 1, 1)), ca(B);
                         for (int b = 0; b < B; ++b)
                           shard_chain(pr, sh, inst, sh->first_rank + b,
                                       he.data() + (size_t)b * nl,
                                       pe.data() + (size_t)b * std::max(nl - 1, 1), &ca[b]);
                         build_diag_tables(pl, B, he.data(), pe.data(), dt, ca.data());
                       },
                       &tab));
  rc.diag_tab = (const double2*)tab;
  return shard_kick_tables(ctx, pr, sh, rc);
}

int shard_check_common(dtc_ctx* ctx, const dtc_problem* pr, const dtc_noise* nz,
                       const dtc_shard* sh, int64_t traj, int32_t inst) {
  if (!ctx) return fail(DTC_EINVAL, "null ctx");
  DTC_TRY(check_problem(pr, nz, 64));
  DTC_TRY(check_shard(pr, sh));
  if (inst < 0 || inst >= pr->n_inst) return fail(DTC_EINVAL, "inst out of range");
  if (traj < 0) return fail(DTC_EINVAL, "traj must be >= 0");
  return DTC_OK;
}

RunCfg shard_runcfg(const dtc_problem* pr, const dtc_noise* nz, const dtc_shard* sh,
                    uint64_t seed, int64_t traj) {
  RunCfg rc;
  rc.prob = pr;
  rc.pl = make_plan(sh->n_local, true);
  rc.seed = seed;
  rc.traj_offset = traj;
  rc.n_traj = 1;  // batch index b = shard b -> diag table b
  rc.noisy = nz->p > 0.0 ? 1 : 0;
  rc.row_kind = classify_rows(pr);
  thresholds(nz->p, &rc.thr1, &rc.thr2, &rc.thr3);
  return rc;
}

// dtc_shard_step / dtc_shard_step_async: obs is a host array (copied, then
// the stream is synchronised) or, when obs_on_device, a device array the
// reduction writes directly (nothing waits).
int shard_step_impl(dtc_ctx* ctx, const dtc_problem* pr, const dtc_noise* nz,
                    const dtc_shard* sh, uint64_t seed, int64_t traj, int32_t inst,
                    int32_t period, uint64_t pre_mask, int32_t diag, uint64_t post_mask,
                    const double* src, double* dst, double* obs, bool obs_on_device) {
  if (!src || !dst) return fail(DTC_EINVAL, "null src/dst");
  DTC_TRY(shard_check_common(ctx, pr, nz, sh, traj, inst));
  const int nl = sh->n_local;
  const uint64_t all = nl >= 64 ? ~0ull : (1ull << nl) - 1;
  if ((pre_mask | post_mask) & ~all) return fail(DTC_EINVAL, "kick mask has non-local bits");
  if (post_mask && !diag) return fail(DTC_EINVAL, "post_mask needs diag");
  const int n_rows = std::max(1, pr->T - 1 + pr->t_offset);
  if (pre_mask && (period < 1 || period > n_rows))
    return fail(DTC_EINVAL, "period outside kick table");
  if (post_mask && period + 1 > n_rows) return fail(DTC_EINVAL, "period + 1 outside kick table");
  DTC_HIP(hipSetDevice(ctx->device));

  RunCfg rc = shard_runcfg(pr, nz, sh, seed, traj);
  const Plan& pl = rc.pl;
  const int B = sh->n_shards;
  DTC_TRY(shard_tables(ctx, pr, sh, inst, pl, rc));
  const int n_obs = 1 + nl;
  DTC_TRY(ensure(ctx->partial, (size_t)B * pl.n_tiles * n_obs * sizeof(double)));
  DTC_TRY(ensure(ctx->vals_f, (size_t)B * n_obs * sizeof(double)));
  double* meas_out = obs_on_device ? obs : (double*)ctx->vals_f.p;

  auto layer = [&](int p, uint64_t mask, const Group& g) {
    dtc::KickDesc k{1, p - 1, dtc::kKickForward, dtc::kStreamForward, (uint32_t)p,
                    skip_bits(g, mask)};
    return k;
  };
  // main group: holds the highest kicked bit (the bits an exchange just made local)
  const uint64_t any = pre_mask | post_mask;
  int main_g = (int)pl.groups.size() - 1;
  if (any) {
    const int top = 63 - __builtin_clzll(any);
    for (size_t g = 0; g < pl.groups.size(); ++g)
      if ((group_bits(pl.groups[g]) >> top) & 1) main_g = (int)g;
  }
  std::vector<PassSpec> passes;
  for (size_t g = 0; g < pl.groups.size(); ++g) {
    const uint64_t gb = group_bits(pl.groups[g]);
    if ((int)g != main_g && (pre_mask & gb))
      passes.push_back(PassSpec{(int)g, layer(period, pre_mask, pl.groups[g]), no_kick(),
                                dtc::kDiagNone, 0});
  }
  const Group& mg = pl.groups[main_g];
  const uint64_t mb = group_bits(mg);
  PassSpec mp{main_g, no_kick(), no_kick(), diag ? dtc::kDiagFwd : dtc::kDiagNone, 1};
  if (pre_mask & mb) mp.pre = layer(period, pre_mask, mg);
  if (post_mask & mb) mp.post = layer(period + 1, post_mask, mg);
  const int main_idx = (int)passes.size();
  if (mp.pre.enabled || mp.post.enabled || diag) passes.push_back(mp);
  const int meas_idx = diag ? main_idx : (int)passes.size() - 1;
  for (size_t g = 0; g < pl.groups.size(); ++g) {
    const uint64_t gb = group_bits(pl.groups[g]);
    if ((int)g != main_g && (post_mask & gb))
      passes.push_back(PassSpec{(int)g, layer(period + 1, post_mask, pl.groups[g]), no_kick(),
                                dtc::kDiagNone, 0});
  }
  const double2* s2 = (const double2*)src;
  double2* d2 = (double2*)dst;
  const size_t len = (size_t)1 << nl;
  if (passes.empty()) {
    if (src != dst)
      DTC_HIP(hipMemcpyAsync(d2, s2, len * 16 * B, hipMemcpyDeviceToDevice, ctx->stream));
  }
  for (size_t i = 0; i < passes.size(); ++i) {
    const bool meas = obs && (int)i == meas_idx;
    DTC_TRY(launch_pass_spec(ctx, rc, 0, B, passes[i], i == 0 ? s2 : d2, d2,
                             meas ? dtc::kMeasSites : dtc::kMeasNone, diag ? 0 : 1, n_obs,
                             meas ? meas_out : nullptr, n_obs));
  }
  if (obs && passes.empty()) {
    // no pass ran: measure with an identity-only kick pass over group 0
    PassSpec ps{0, layer(1, 0, pl.groups[0]), no_kick(), dtc::kDiagNone, 0};
    ps.pre.row = 0;
    DTC_TRY(launch_pass_spec(ctx, rc, 0, B, ps, d2, d2, dtc::kMeasSites, 1, n_obs, meas_out,
                             n_obs));
  }
  if (obs_on_device) return DTC_OK;
  if (obs)
    DTC_HIP(hipMemcpyAsync(obs, ctx->vals_f.p, (size_t)B * n_obs * sizeof(double),
                           hipMemcpyDeviceToHost, ctx->stream));
  DTC_HIP(hipStreamSynchronize(ctx->stream));
  DTC_TRY(settle_pending(ctx));
  return DTC_OK;
}

}  // namespace

extern "C" {

int dtc_shard_step(dtc_ctx* ctx, const dtc_problem* pr, const dtc_noise* nz,
                   const dtc_shard* sh, uint64_t seed, int64_t traj, int32_t inst,
                   int32_t period, uint64_t pre_mask, int32_t diag, uint64_t post_mask,
                   const double* src, double* dst, double* obs) {
  return shard_step_impl(ctx, pr, nz, sh, seed, traj, inst, period, pre_mask, diag, post_mask,
                         src, dst, obs, false);
}

int dtc_shard_step_async(dtc_ctx* ctx, const dtc_problem* pr, const dtc_noise* nz,
                         const dtc_shard* sh, uint64_t seed, int64_t traj, int32_t inst,
                         int32_t period, uint64_t pre_mask, int32_t diag, uint64_t post_mask,
                         const double* src, double* dst, double* obs_dev) {
  return shard_step_impl(ctx, pr, nz, sh, seed, traj, inst, period, pre_mask, diag, post_mask,
                         src, dst, obs_dev, true);
}

int dtc_shard_kick_slice(dtc_ctx* ctx, const dtc_problem* pr, const dtc_noise* nz,
                         const dtc_shard* sh, uint64_t seed, int64_t traj, int32_t period,
                         uint64_t pre_mask, int32_t chunk_bits, int32_t slice_bits, int32_t slice,
                         double* state) {
  if (!state) return fail(DTC_EINVAL, "null state");
  DTC_TRY(shard_check_common(ctx, pr, nz, sh, traj, 0));
  const int nl = sh->n_local;
  if (chunk_bits < 0 || slice_bits < 0 || chunk_bits + slice_bits > 16 ||
      nl - chunk_bits - slice_bits < dtc::kTileBits)
    return fail(DTC_EINVAL, "chunk_bits + slice_bits must leave >= 12 bits per slice");
  if (slice < 0 || slice >= (1 << slice_bits)) return fail(DTC_EINVAL, "slice out of range");
  const int nsub = nl - chunk_bits - slice_bits;
  const uint64_t low = (1ull << nsub) - 1;
  if (pre_mask & ~low) return fail(DTC_EINVAL, "slice kick mask reaches the chunk/slice bits");
  const int n_rows = std::max(1, pr->T - 1 + pr->t_offset);
  if (!pre_mask) return DTC_OK;
  if (period < 1 || period > n_rows) return fail(DTC_EINVAL, "period outside kick table");
  const int64_t n_pieces = (int64_t)sh->n_shards << chunk_bits;
  if (n_pieces > 65535) return fail(DTC_EINVAL, "too many chunks x shards for one launch");
  DTC_HIP(hipSetDevice(ctx->device));
  RunCfg rc = shard_runcfg(pr, nz, sh, seed, traj);
  const Plan& pl = rc.pl;
  DTC_TRY(shard_kick_tables(ctx, pr, sh, rc));  // kick-only passes read no diagonal
  // one launch: the slice of every (shard, chunk) piece is a 2^nsub-amplitude
  // state, pieces 2^(nl - chunk_bits) apart (the same trajectory: identical
  // kick records for every piece)
  rc.L_eff_override = nsub;
  rc.stride_override = (int64_t)1 << (nl - chunk_bits);
  double2* base = (double2*)state + ((size_t)slice << nsub);
  for (size_t g = 0; g < pl.groups.size(); ++g) {
    const Group& G = pl.groups[g];
    const uint64_t gb = group_bits(G);
    if (!(pre_mask & gb)) continue;
    if (gb & ~low) return fail(DTC_EINVAL, "a site group of the kick mask reaches the slice bits");
    PassSpec ps{(int)g, no_kick(), no_kick(), dtc::kDiagNone, 0};
    ps.pre = dtc::KickDesc{1, period - 1, dtc::kKickForward, dtc::kStreamForward,
                           (uint32_t)period, skip_bits(G, pre_mask)};
    DTC_TRY(launch_pass_spec(ctx, rc, 0, (int)n_pieces, ps, base, base, dtc::kMeasNone, 1, 2,
                             nullptr, 0));
  }
  return DTC_OK;
}

int dtc_shard_kick_exchange_slice(dtc_ctx* ctx, const dtc_problem* pr, const dtc_noise* nz,
                                  const dtc_shard* sh, uint64_t seed, int64_t traj,
                                  int32_t period, uint64_t pre_mask, int32_t slice_bits,
                                  int32_t slice, double* state) {
  if (!ctx || !sh || !state) return fail(DTC_EINVAL, "null ctx/shard/state");
  const int k = sh->n_global, nl = sh->n_local;
  if (sh->n_shards != (1 << k) || sh->first_rank != 0)
    return fail(DTC_EINVAL, "the in-place exchange needs every shard in this buffer");
  DTC_TRY(shard_check_common(ctx, pr, nz, sh, traj, 0));
  if (slice_bits < 0 || k + slice_bits > 16 || nl - k - slice_bits < dtc::kTileBits)
    return fail(DTC_EINVAL, "chunk_bits + slice_bits must leave >= 12 bits per slice");
  if (slice < 0 || slice >= (1 << slice_bits)) return fail(DTC_EINVAL, "slice out of range");
  const int nsub = nl - k - slice_bits;
  const uint64_t low = (1ull << nsub) - 1;
  if (pre_mask & ~low) return fail(DTC_EINVAL, "slice kick mask reaches the chunk/slice bits");
  RunCfg rc = shard_runcfg(pr, nz, sh, seed, traj);
  const Plan& pl = rc.pl;
  const int n_rows = std::max(1, pr->T - 1 + pr->t_offset);
  if (period < 1 || period > n_rows) return fail(DTC_EINVAL, "period outside kick table");
  // the group whose pass goes last carries the exchange (a unitary kick kind,
  // classified on the row that pass actually launches; launch_kick_swap takes
  // 1 <= k <= 6 chunk bits, other shapes run the two calls)
  int last = -1;
  for (size_t g = 0; g < pl.groups.size(); ++g)
    if (pre_mask & group_bits(pl.groups[g])) last = (int)g;
  bool fuse = last >= 0 && k >= 1 && k <= 6;
  if (fuse) {
    const Group& G = pl.groups[last];
    PassSpec ps{last, no_kick(), no_kick(), dtc::kDiagNone, 0};
    ps.pre = dtc::KickDesc{1, period - 1, dtc::kKickForward, dtc::kStreamForward,
                           (uint32_t)period, skip_bits(G, pre_mask)};
    const int kind = pass_kind(rc, ps, dtc::kShapeK);
    fuse = kind == dtc::kKindRX || kind == dtc::kKindRY || kind == dtc::kKindGen;
  }
  if (!fuse) {
    DTC_TRY(dtc_shard_kick_slice(ctx, pr, nz, sh, seed, traj, period, pre_mask, k, slice_bits,
                                 slice, state));
    return dtc_shard_exchange_slice(ctx, sh, slice_bits, slice, state);
  }
  DTC_HIP(hipSetDevice(ctx->device));
  DTC_TRY(shard_kick_tables(ctx, pr, sh, rc));
  rc.L_eff_override = nsub;
  rc.stride_override = (int64_t)1 << (nl - k);
  double2* base = (double2*)state + ((size_t)slice << nsub);
  const int n_pieces = 1 << (2 * k);
  for (size_t g = 0; g < pl.groups.size(); ++g) {
    const Group& G = pl.groups[g];
    const uint64_t gb = group_bits(G);
    if (!(pre_mask & gb)) continue;
    if (gb & ~low) return fail(DTC_EINVAL, "a site group of the kick mask reaches the slice bits");
    PassSpec ps{(int)g, no_kick(), no_kick(), dtc::kDiagNone, 0};
    ps.pre = dtc::KickDesc{1, period - 1, dtc::kKickForward, dtc::kStreamForward,
                           (uint32_t)period, skip_bits(G, pre_mask)};
    DTC_TRY(launch_pass_spec(ctx, rc, 0, n_pieces, ps, base, base, dtc::kMeasNone, 1, 2, nullptr,
                             0, nullptr, 0, 0, nullptr, (int)g == last ? k : 0));
  }
  return DTC_OK;
}

int dtc_shard_exchange_slice(dtc_ctx* ctx, const dtc_shard* sh, int32_t slice_bits,
                             int32_t slice, double* state) {
  if (!ctx || !sh || !state) return fail(DTC_EINVAL, "null ctx/shard/state");
  const int nl = sh->n_local, k = sh->n_global;
  if (k < 1 || k > 6 || nl < 2 * k || nl > 40)
    return fail(DTC_EINVAL, "need 1 <= n_global <= 6 and n_local >= 2 n_global");
  if (sh->n_shards != (1 << k) || sh->first_rank != 0)
    return fail(DTC_EINVAL, "the in-place exchange needs every shard in this buffer");
  if (slice_bits < 0 || nl - k - slice_bits < dtc::kTileBits)
    return fail(DTC_EINVAL, "slice_bits must leave >= 12 bits per slice");
  if (slice < 0 || slice >= (1 << slice_bits)) return fail(DTC_EINVAL, "slice out of range");
  DTC_HIP(hipSetDevice(ctx->device));
  const int nsub = nl - k - slice_bits;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (ctx->prof) {
    e0 = get_event(ctx);
    e1 = get_event(ctx);
    DTC_HIP(hipEventRecord(e0, ctx->stream));
  }
  DTC_HIP(dtc::launch_exchange_swap((double2*)state, nl, k, nsub, slice, ctx->stream));
  if (ctx->prof) {
    DTC_HIP(hipEventRecord(e1, ctx->stream));
    // every off-diagonal piece read once and written once
    const double moved = (double)((1 << k) * ((1 << k) - 1)) * (double)((int64_t)1 << nsub);
    ctx->pending.push_back(Pending{DTC_KERNEL_EXCHANGE, e0, e1, 32.0 * moved});
  }
  return DTC_OK;
}

int dtc_get_stream(dtc_ctx* ctx, void** stream) {
  if (!ctx || !stream) return fail(DTC_EINVAL, "null ctx/stream");
  *stream = (void*)ctx->stream;
  return DTC_OK;
}

int dtc_synchronize(dtc_ctx* ctx) {
  if (!ctx) return fail(DTC_EINVAL, "null ctx");
  DTC_HIP(hipSetDevice(ctx->device));
  DTC_HIP(hipStreamSynchronize(ctx->stream));
  DTC_TRY(settle_pending(ctx));
  return DTC_OK;
}

}  // extern "C"
