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
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <complex>
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

struct Geom {
  int c, s, a;
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
  DevBuf F, E, partial, vals_f, vals_e, diag, kick, basis;
  bool prof = false;
  int64_t st_n[DTC_KERNEL_KINDS] = {0, 0, 0, 0};
  double st_ms[DTC_KERNEL_KINDS] = {0, 0, 0, 0};
  double st_bytes[DTC_KERNEL_KINDS] = {0, 0, 0, 0};
  std::vector<Pending> pending;
  std::vector<hipEvent_t> pool;
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

struct Plan {
  int L = 0, L_eff = 0, n_chunks = 0, n_tiles = 0;
  int64_t len = 0;
  Geom lo{0, 0, dtc::kTileBits};
  std::vector<Geom> hi;
};

Plan make_plan(int L) {
  Plan pl;
  pl.L = L;
  pl.L_eff = std::max(L, dtc::kTileBits);
  pl.len = (int64_t)1 << pl.L_eff;
  pl.n_tiles = 1 << (pl.L_eff - dtc::kTileBits);
  pl.n_chunks = (pl.L_eff + dtc::kChunkBits - 1) / dtc::kChunkBits;
  int rem = pl.L_eff - dtc::kTileBits;
  int n_hi = (rem + 7) / 8;
  int s = dtc::kTileBits;
  for (int i = 0; i < n_hi; ++i) {
    int a = (rem + (n_hi - i) - 1) / (n_hi - i);  // even split, larger first
    pl.hi.push_back(Geom{dtc::kTileBits - a, s, a});
    s += a;
    rem -= a;
  }
  return pl;
}

// Diagonal factor tables (RZZ even/odd bonds + RZ, fast.py:115-120):
// D(x) = exp(-i/2 (sum_i h_i z_i + sum_i phi_i z_i z_{i+1})), z_i = 1 - 2 bit_i(x).
// Per instance: n_chunks chunk tables, D(x) = prod_k C_k[(x >> 5k) & 63] (C_k covers
// sites 5k..5k+4 and the bond to site 5k+5 = index bit 5), followed by 3 register-
// nibble tables N_n[v], v = bits [4n-1, 4n+5) of x, holding the terms of sites
// 4n..4n+3 and of the bonds touching them (the kernel's apply_diag_nibble<n>).
double diag_angle(int L, const double* hh, const double* pp, int lo_site, int hi_site,
                  int bond_lo, int bond_hi, int bit0, int v) {
  auto z = [&](int i) -> double { return ((v >> (i - bit0)) & 1) ? -1.0 : 1.0; };
  double ang = 0.0;
  for (int i = lo_site; i < hi_site && i < L; ++i) ang += hh[i] * z(i);
  for (int i = std::max(bond_lo, 0); i < bond_hi && i + 1 < L; ++i) ang += pp[i] * z(i) * z(i + 1);
  return ang;
}

void build_diag_tables(const Plan& pl, int n_inst, const double* h, const double* phi,
                       std::vector<double>& out) {
  const int L = pl.L;
  const int per_inst = (pl.n_chunks + 3) * 64;
  out.assign((size_t)n_inst * per_inst * 2, 0.0);
  for (int in = 0; in < n_inst; ++in) {
    const double* hh = h + (size_t)in * L;
    const double* pp = phi + (size_t)in * (L > 1 ? L - 1 : 0);
    double* o = out.data() + (size_t)in * per_inst * 2;
    for (int k = 0; k < pl.n_chunks; ++k) {
      const int b0 = dtc::kChunkBits * k;
      for (int v = 0; v < 64; ++v) {
        const double ang = diag_angle(L, hh, pp, b0, b0 + dtc::kChunkBits, b0,
                                      b0 + dtc::kChunkBits, b0, v);
        o[(k * 64 + v) * 2] = std::cos(-0.5 * ang);
        o[(k * 64 + v) * 2 + 1] = std::sin(-0.5 * ang);
      }
    }
    for (int n = 0; n < 3; ++n) {
      const int b0 = 4 * n - 1;
      for (int v = 0; v < 64; ++v) {
        if (n == 0 && (v & 1)) continue;  // bit -1 does not exist
        const double ang = diag_angle(L, hh, pp, 4 * n, 4 * n + 4, 4 * n - 1, 4 * n + 4, b0, v);
        const int e = (pl.n_chunks + n) * 64 + v;
        o[e * 2] = std::cos(-0.5 * ang);
        o[e * 2 + 1] = std::sin(-0.5 * ang);
      }
    }
  }
}

struct RunCfg {
  const dtc_problem* prob;
  Plan pl;
  uint64_t seed;
  int64_t traj_offset;
  int n_traj;
  int noisy;
  uint32_t thr1, thr2, thr3;
};

dtc::PassArgs base_args(dtc_ctx* ctx, const RunCfg& rc, int64_t batch_start) {
  dtc::PassArgs A{};
  A.state_len = rc.pl.len;
  A.L_eff = rc.pl.L_eff;
  A.L_real = rc.pl.L;
  A.batch_start = batch_start;
  A.n_traj = rc.n_traj;
  A.traj_offset = rc.traj_offset;
  A.kick = (const double2*)ctx->kick.p;
  A.n_sub = rc.prob->n_sub;
  A.thr1 = rc.thr1;
  A.thr2 = rc.thr2;
  A.thr3 = rc.thr3;
  A.seed = rc.seed;
  A.noisy = rc.noisy;
  A.diag = (const double2*)ctx->diag.p;
  A.n_chunks = rc.pl.n_chunks;
  A.probe = rc.prob->probe_site;
  A.partial = (double*)ctx->partial.p;
  return A;
}

int launch_one(dtc_ctx* ctx, dtc::PassArgs A, const Geom& g, int batch, int diag_mode,
               int meas_mode, int kind) {
  A.c = g.c;
  A.s = g.s;
  A.a = g.a;
  A.tile_bits_mid = g.s - g.c;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (ctx->prof) {
    e0 = get_event(ctx);
    e1 = get_event(ctx);
    DTC_HIP(hipEventRecord(e0, ctx->stream));
  }
  DTC_HIP(dtc::launch_pass(A, batch, diag_mode, meas_mode, ctx->stream));
  if (ctx->prof) {
    DTC_HIP(hipEventRecord(e1, ctx->stream));
    ctx->pending.push_back(Pending{kind, e0, e1, 32.0 * (double)A.state_len * batch});
  }
  return DTC_OK;
}

int launch_reduce_prof(dtc_ctx* ctx, int n_tiles, int n_obs, int batch, double* out,
                       int64_t out_stride) {
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (ctx->prof) {
    e0 = get_event(ctx);
    e1 = get_event(ctx);
    DTC_HIP(hipEventRecord(e0, ctx->stream));
  }
  DTC_HIP(dtc::launch_reduce((const double*)ctx->partial.p, n_tiles, n_obs, batch, out,
                             out_stride, ctx->stream));
  if (ctx->prof) {
    DTC_HIP(hipEventRecord(e1, ctx->stream));
    ctx->pending.push_back(
        Pending{DTC_KERNEL_REDUCE, e0, e1, 8.0 * (double)n_tiles * n_obs * batch});
  }
  return DTC_OK;
}

// One forward period p (1-based) on `batch` states: K_hi passes, then the fused
// K_lo + diagonal pass (fast.py:111-121 order: kicks, RZZ, RZ).
int forward_period(dtc_ctx* ctx, const RunCfg& rc, int64_t batch_start, int batch,
                   const double2* src, double2* dst, int p, uint32_t stream, int meas_mode,
                   int n_obs, double* meas_out, int64_t meas_stride) {
  dtc::PassArgs A = base_args(ctx, rc, batch_start);
  A.kick_row = p - 1;
  A.inverse = 0;
  A.stream = stream;
  A.rng_period = (uint32_t)p;
  A.n_obs = n_obs;
  const double2* s = src;
  for (const Geom& g : rc.pl.hi) {
    A.src = s;
    A.dst = dst;
    DTC_TRY(launch_one(ctx, A, g, batch, dtc::kDiagNone, dtc::kMeasNone, DTC_KERNEL_HI_PASS));
    s = dst;
  }
  A.src = s;
  A.dst = dst;
  DTC_TRY(launch_one(ctx, A, rc.pl.lo, batch, dtc::kDiagAfter, meas_mode, DTC_KERNEL_LO_PASS));
  if (meas_mode != dtc::kMeasNone)
    DTC_TRY(launch_reduce_prof(ctx, rc.pl.n_tiles, n_obs, batch, meas_out, meas_stride));
  return DTC_OK;
}

// One inverse period (fast.py:140-143, UF.inverse()): diagonal^-1 fused into
// the K_lo pass, then K_hi passes; rng counter = echo step k.
int inverse_period(dtc_ctx* ctx, const RunCfg& rc, int64_t batch_start, int batch,
                   const double2* src, double2* dst, int p, int step, uint32_t stream,
                   int meas_mode, int n_obs, double* meas_out, int64_t meas_stride) {
  dtc::PassArgs A = base_args(ctx, rc, batch_start);
  A.kick_row = p - 1;
  A.inverse = 1;
  A.stream = stream;
  A.rng_period = (uint32_t)step;
  A.n_obs = n_obs;
  const bool lo_last = rc.pl.hi.empty();
  A.src = src;
  A.dst = dst;
  DTC_TRY(launch_one(ctx, A, rc.pl.lo, batch, dtc::kDiagBeforeConj,
                     lo_last ? meas_mode : dtc::kMeasNone, DTC_KERNEL_LO_PASS));
  for (size_t i = 0; i < rc.pl.hi.size(); ++i) {
    A.src = dst;
    A.dst = dst;
    const bool last = (i + 1 == rc.pl.hi.size());
    DTC_TRY(launch_one(ctx, A, rc.pl.hi[i], batch, dtc::kDiagNone,
                       last ? meas_mode : dtc::kMeasNone, DTC_KERNEL_HI_PASS));
  }
  if (meas_mode != dtc::kMeasNone)
    DTC_TRY(launch_reduce_prof(ctx, rc.pl.n_tiles, n_obs, batch, meas_out, meas_stride));
  return DTC_OK;
}

int check_problem(const dtc_problem* pr, const dtc_noise* nz) {
  if (!pr || !nz) return fail(DTC_EINVAL, "null problem/noise");
  if (pr->L < 1 || pr->L > 36) return fail(DTC_EINVAL, "L must be in [1, 36]");
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
    int pz = dtc::sample_pauli(rc.seed, traj, dtc::kStreamPrep, 0u, (uint32_t)i, 0u, rc.thr1,
                               rc.thr2, rc.thr3);
    if (pz == 1 || pz == 2) m &= ~(1ull << i);
  }
  return m;
}

int upload_tables(dtc_ctx* ctx, const dtc_problem* pr, const Plan& pl) {
  std::vector<double> dt;
  build_diag_tables(pl, pr->n_inst, pr->h, pr->phi, dt);
  DTC_TRY(ensure(ctx->diag, dt.size() * sizeof(double)));
  DTC_HIP(hipMemcpyAsync(ctx->diag.p, dt.data(), dt.size() * sizeof(double),
                         hipMemcpyHostToDevice, ctx->stream));
  const int n_periods = std::max(1, pr->T - 1 + pr->t_offset);
  const size_t kb = (size_t)n_periods * pr->L * pr->n_sub * 8 * sizeof(double);
  DTC_TRY(ensure(ctx->kick, kb));
  DTC_HIP(hipMemcpyAsync(ctx->kick.p, pr->kick, kb, hipMemcpyHostToDevice, ctx->stream));
  DTC_HIP(hipStreamSynchronize(ctx->stream));
  return DTC_OK;
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
  release(ctx->partial);
  release(ctx->vals_f);
  release(ctx->vals_e);
  release(ctx->diag);
  release(ctx->kick);
  release(ctx->basis);
  (void)hipStreamDestroy(ctx->stream);
  delete ctx;
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

int dtc_autocorr(dtc_ctx* ctx, const dtc_problem* pr, const dtc_noise* nz, uint64_t seed,
                 int64_t traj_offset, int32_t n_traj, double* fwd, double* echo,
                 double* zsite) {
  if (!ctx) return fail(DTC_EINVAL, "null ctx");
  DTC_TRY(check_problem(pr, nz));
  if (n_traj < 1) return fail(DTC_EINVAL, "n_traj must be >= 1");
  if (traj_offset < 0) return fail(DTC_EINVAL, "traj_offset must be >= 0");
  if (pr->want_fwd && !fwd) return fail(DTC_EINVAL, "want_fwd but fwd is null");
  if (pr->want_echo && !echo) return fail(DTC_EINVAL, "want_echo but echo is null");
  DTC_HIP(hipSetDevice(ctx->device));

  RunCfg rc;
  rc.prob = pr;
  rc.pl = make_plan(pr->L);
  rc.seed = seed;
  rc.traj_offset = traj_offset;
  rc.n_traj = n_traj;
  rc.noisy = nz->p > 0.0 ? 1 : 0;
  thresholds(nz->p, &rc.thr1, &rc.thr2, &rc.thr3);
  const Plan& pl = rc.pl;
  const int T = pr->T, L = pr->L;
  const int P = T - 1 + pr->t_offset;
  const bool want_z = zsite != nullptr;
  const bool want_f = pr->want_fwd || want_z;
  const bool want_e = pr->want_echo != 0;
  const int n_obs_f = want_z ? 1 + L : 2;
  const int meas_f = want_z ? dtc::kMeasSites : dtc::kMeasProbe;
  const double fac = std::pow(1.0 - nz->p, (double)nz->n_anc);

  DTC_TRY(upload_tables(ctx, pr, pl));

  // batch size: F (+ E for echo) resident in HBM
  const int64_t S = (int64_t)pr->n_inst * n_traj;
  const double per_state = (double)pl.len * 16.0 * (want_e ? 2.0 : 1.0);
  int64_t B = pr->batch;
  if (B <= 0) {
    size_t free_b = 0, total_b = 0;
    DTC_HIP(hipMemGetInfo(&free_b, &total_b));
    double budget = std::min(0.6 * (double)free_b, 64.0 * (1ull << 30));
    if (const char* env = std::getenv("DTC_BATCH_BYTES")) budget = std::atof(env);
    B = (int64_t)(budget / per_state);
    B = std::max<int64_t>(1, std::min<int64_t>(B, 4096));
  }
  B = std::min<int64_t>(B, S);
  B = std::min<int64_t>(B, 65535);

  DTC_TRY(ensure(ctx->F, (size_t)(B * pl.len * 16)));
  if (want_e) DTC_TRY(ensure(ctx->E, (size_t)(B * pl.len * 16)));
  const int max_obs = std::max(n_obs_f, 2);
  DTC_TRY(ensure(ctx->partial, (size_t)B * pl.n_tiles * max_obs * sizeof(double)));
  DTC_TRY(ensure(ctx->vals_f, (size_t)B * T * n_obs_f * sizeof(double)));
  if (want_e) DTC_TRY(ensure(ctx->vals_e, (size_t)B * T * 2 * sizeof(double)));
  DTC_TRY(ensure(ctx->basis, (size_t)B * sizeof(int64_t)));

  std::vector<double> hv_f((size_t)B * T * n_obs_f), hv_e(want_e ? (size_t)B * T * 2 : 0);
  std::vector<int64_t> masks(B);

  for (int64_t bs = 0; bs < S; bs += B) {
    const int nb = (int)std::min<int64_t>(B, S - bs);
    for (int b = 0; b < nb; ++b) {
      const int64_t g = bs + b;
      masks[b] = (int64_t)init_state_mask(rc, (uint64_t)(traj_offset + g % n_traj));
    }
    double2* F = (double2*)ctx->F.p;
    double2* E = (double2*)ctx->E.p;
    DTC_HIP(hipMemcpyAsync(ctx->basis.p, masks.data(), nb * sizeof(int64_t),
                           hipMemcpyHostToDevice, ctx->stream));
    DTC_HIP(hipMemsetAsync(F, 0, (size_t)nb * pl.len * 16, ctx->stream));
    DTC_HIP(dtc::launch_set_basis(F, pl.len, (const int64_t*)ctx->basis.p, nb, ctx->stream));
    DTC_HIP(hipMemsetAsync(ctx->vals_f.p, 0, (size_t)nb * T * n_obs_f * sizeof(double),
                           ctx->stream));
    if (want_e)
      DTC_HIP(hipMemsetAsync(ctx->vals_e.p, 0, (size_t)nb * T * 2 * sizeof(double),
                             ctx->stream));

    for (int p = 0; p <= P; ++p) {
      const int t = p - pr->t_offset;
      if (p > 0) {
        const bool meas = want_f && t >= 0 && t >= pr->t_first;
        DTC_TRY(forward_period(ctx, rc, bs, nb, F, F, p, dtc::kStreamForward,
                               meas ? meas_f : dtc::kMeasNone, n_obs_f,
                               meas ? (double*)ctx->vals_f.p + (size_t)t * n_obs_f : nullptr,
                               (int64_t)T * n_obs_f));
      }
      if (t < 0 || t < pr->t_first || !want_e || p == 0) continue;
      double* vout = (double*)ctx->vals_e.p + (size_t)t * 2;
      for (int k = 1; k <= p; ++k) {
        const bool last = (k == p);
        DTC_TRY(inverse_period(ctx, rc, bs, nb, k == 1 ? F : E, E, p - k + 1, k,
                               (uint32_t)(1 + t), last ? dtc::kMeasProbe : dtc::kMeasNone, 2,
                               last ? vout : nullptr, (int64_t)T * 2));
      }
    }
    DTC_HIP(hipMemcpyAsync(hv_f.data(), ctx->vals_f.p, (size_t)nb * T * n_obs_f * sizeof(double),
                           hipMemcpyDeviceToHost, ctx->stream));
    if (want_e)
      DTC_HIP(hipMemcpyAsync(hv_e.data(), ctx->vals_e.p, (size_t)nb * T * 2 * sizeof(double),
                             hipMemcpyDeviceToHost, ctx->stream));
    DTC_HIP(hipStreamSynchronize(ctx->stream));
    if (ctx->prof) DTC_TRY(resolve_pending(ctx));

    const int j = pr->probe_site;
    for (int b = 0; b < nb; ++b) {
      const int64_t g = bs + b;
      const uint64_t m = (uint64_t)masks[b];
      const double zinit = ((m >> j) & 1ull) ? -1.0 : 1.0;
      for (int t = std::max(0, pr->t_first); t < T; ++t) {
        const bool at_init = (t + pr->t_offset == 0);
        const double* vf = hv_f.data() + ((size_t)b * T + t) * n_obs_f;
        const double zj_f = at_init ? zinit : (want_z ? vf[1 + j] : vf[1]);
        if (pr->want_fwd) fwd[(size_t)g * T + t] = fac * zinit * zj_f;
        if (want_z) {
          double* zo = zsite + ((size_t)g * T + t) * L;
          for (int i = 0; i < L; ++i)
            zo[i] = at_init ? (((m >> i) & 1ull) ? -1.0 : 1.0) : vf[1 + i];
        }
        if (want_e) {
          const double zj_e = at_init ? zinit : hv_e[((size_t)b * T + t) * 2 + 1];
          echo[(size_t)g * T + t] = fac * zinit * zj_e;
        }
      }
    }
  }
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
  for (int k = 1; k <= n_periods; ++k) {
    const bool last = (k == n_periods) && zsite_out;
    const int meas = last ? dtc::kMeasSites : dtc::kMeasNone;
    if (inverse) {
      DTC_TRY(inverse_period(ctx, rc, batch_start, 1, F, F, first_period - k + 1, k, stream, meas,
                             1 + L, (double*)ctx->vals_f.p, 1 + L));
    } else {
      const int p = first_period + k - 1;
      DTC_TRY(forward_period(ctx, rc, batch_start, 1, F, F, p, stream, meas, 1 + L,
                             (double*)ctx->vals_f.p, 1 + L));
    }
  }
  DTC_HIP(hipMemcpyAsync(state, F, ((size_t)1 << L) * 16, hipMemcpyDeviceToHost, ctx->stream));
  if (zsite_out && n_periods > 0)
    DTC_HIP(hipMemcpyAsync(zsite_out, ctx->vals_f.p, (size_t)(1 + L) * sizeof(double),
                           hipMemcpyDeviceToHost, ctx->stream));
  DTC_HIP(hipStreamSynchronize(ctx->stream));
  if (ctx->prof) DTC_TRY(resolve_pending(ctx));
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

}  // extern "C"
