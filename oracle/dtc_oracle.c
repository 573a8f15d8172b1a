/*
 * dtc_oracle.c — CPU restatement of the reference's DTC autocorrelator path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product path links, loads or
 * calls this file: only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg use it, and only as the checker / CPU baseline.
 *
 * What it restates (reference = /root/reference, read as text):
 *   create_UF_subcircuit        autocorr-delta-a-single-qiskit-fast.py:111-121
 *     - RX(pi g) on every site i (circuit qubit i+1)                 :113-114
 *     - RZZ(phi_i) on bonds (i, i+1), even i first, then odd i         :115-118
 *     - RZ(h_i) on every site                                         :119-120
 *     generalised kick (per period, per site, sub-gate list):
 *       ...-polarization.py:110-129, ...-circular-polarization.py:110-142,
 *       ...-polarization-xy-cycle.py:141-155, ...-controlled-g.py:196-241
 *   UF.inverse() for the echo   fast.py:140-143 (reverse order, negated
 *                               angles; RX -> RX^dagger)
 *   noise                       fast.py:84-86: depolarizing_error(p,1) on
 *                               u1/u2/u3; RX/RY/X transpile to noisy u3, H and
 *                               the CZ wrappers on the ancilla to noisy u2,
 *                               RZZ -> cx.rz.cx and RZ -> rz are noiseless
 *                               (pinned by the reference's gate_counts_*.csv).
 *                               Aer's channel = Pauli I w.p. 1-3p/4, X/Y/Z w.p.
 *                               p/4 each, applied after the gate.
 *   estimator                   fast.py:92-109, 211-213: (n0 - n1)/shots of the
 *                               ancilla; folded here to (1-p)^6 z_j(init)
 *                               <Z_j(t)> (checked against the
 *                               full (L+1)-qubit density matrix in
 *                               oracle/dm_oracle.py).
 *
 * Unlike the engine, every gate is applied one by one on a 2^L statevector,
 * with the RZZ/RZ phases computed directly from exp(-i theta/2 z z), and no
 * tiling, batching or factor tables.  The trajectory schedule and the
 * counter-based Philox4x32-10 draws follow the engine's RNG contract
 * (documented in include/dtc.h) so per-trajectory outputs can be compared
 * to ~1e-12.  Written independently of the HIP sources.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* Same layout as dtc_problem / dtc_noise in include/dtc.h. */
typedef struct orc_problem {
  int32_t L, T, n_inst, probe_site, t_offset, n_sub;
  uint64_t init_mask;
  const double* h;
  const double* phi;
  const double* kick;
  int32_t want_fwd, want_echo, batch, t_first;
} orc_problem;

typedef struct orc_noise {
  double p;
  int32_t n_anc, reserved;
} orc_noise;

/* Same layout as dtc_device_noise in include/dtc.h. */
typedef struct orc_device_noise {
  const double* p_gate;
  const double* t1_us;
  const double* t2_us;
  double gate_ns, anc_factor, readout_p01, readout_p10;
} orc_device_noise;

typedef struct { double re, im; } cpx;

static inline cpx cx(double r, double i) { cpx z = {r, i}; return z; }
static inline cpx cadd(cpx a, cpx b) { return cx(a.re + b.re, a.im + b.im); }
static inline cpx cmul(cpx a, cpx b) {
  return cx(a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re);
}
static inline cpx cconj(cpx a) { return cx(a.re, -a.im); }

/* ---- Philox4x32-10 (Salmon, Moraes, Dror, Shaw, SC'11) ---------------- */
static uint32_t orc_philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    uint32_t y0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
    uint32_t y1 = (uint32_t)p1;
    uint32_t y2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    uint32_t y3 = (uint32_t)p0;
    c[0] = y0; c[1] = y1; c[2] = y2; c[3] = y3;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c[0];
}

typedef struct {
  uint32_t thr[3];
  int noisy;
  uint64_t seed;
  /* device-like noise (NULL dev_thr: depolarizing only) */
  const uint32_t* dev_thr;   /* [L][3] */
  const uint32_t* dev_jump;  /* [L] */
  const double* dev_kraus;   /* [L][3] K0 00, K0 11, K1 01 */
} orc_rng;

static void orc_rng_init(orc_rng* r, double p, uint64_t seed) {
  for (int k = 1; k <= 3; ++k) {
    double v = floor(k * p / 4.0 * 4294967296.0 + 0.5);
    if (v > 4294967295.0) v = 4294967295.0;
    r->thr[k - 1] = (uint32_t)v;
  }
  r->noisy = p > 0.0;
  r->seed = seed;
  r->dev_thr = NULL;
  r->dev_jump = NULL;
  r->dev_kraus = NULL;
}

/* 0 = I, 1 = X, 2 = Y, 3 = Z */
static int orc_pauli(const orc_rng* r, uint64_t traj, uint32_t stream, uint32_t period,
                     uint32_t site, uint32_t sub) {
  if (!r->noisy) return 0;
  uint32_t c[4] = {site | (sub << 16), period, stream, (uint32_t)traj};
  uint32_t x = orc_philox(c, (uint32_t)r->seed, (uint32_t)(r->seed >> 32) ^ (uint32_t)(traj >> 32));
  if (x < r->thr[0]) return 1;
  if (x < r->thr[1]) return 2;
  if (x < r->thr[2]) return 3;
  return 0;
}

/* Device-like noise draw: Philox word 0 -> Pauli against the site's
 * thresholds, word 1 -> amplitude-damping jump (include/dtc.h). */
static int orc_device_draw(const orc_rng* r, uint64_t traj, uint32_t stream, uint32_t period,
                           uint32_t site, uint32_t sub, uint32_t thr_jump, int* jump) {
  uint32_t c[4] = {site | (sub << 16), period, stream, (uint32_t)traj};
  uint32_t x = orc_philox(c, (uint32_t)r->seed, (uint32_t)(r->seed >> 32) ^ (uint32_t)(traj >> 32));
  *jump = c[1] < thr_jump;
  const uint32_t* t = r->dev_thr + 3 * site;
  if (x < t[0]) return 1;
  if (x < t[1]) return 2;
  if (x < t[2]) return 3;
  return 0;
}

/* ---- gates on a 2^L statevector (bit i = site i) ------------------------ */
/* States of 2^22 amplitudes and more (the L = 28 parity runs) are swept by
 * all threads, one trajectory at a time (autocorr_run does not split such
 * runs over trajectories); the loops are element-wise, so the result does not
 * depend on the thread count, except measure_z's sums (per-thread partials
 * added in thread order). */
#define ORC_INNER_PAR(n) ((n) >= ((size_t)1 << 22))
static void gate_1q(cpx* psi, int L, int site, const cpx m[4]) {
  const size_t n = (size_t)1 << L, bit = (size_t)1 << site;
#ifdef _OPENMP
#pragma omp parallel for schedule(static) if (ORC_INNER_PAR(n))
#endif
  for (size_t x = 0; x < n; ++x) {
    if (x & bit) continue;
    cpx a = psi[x], b = psi[x | bit];
    psi[x] = cadd(cmul(m[0], a), cmul(m[1], b));
    psi[x | bit] = cadd(cmul(m[2], a), cmul(m[3], b));
  }
}

static void gate_pauli(cpx* psi, int L, int site, int pauli) {
  static const cpx X[4] = {{0, 0}, {1, 0}, {1, 0}, {0, 0}};
  static const cpx Y[4] = {{0, 0}, {0, -1}, {0, 1}, {0, 0}};
  static const cpx Z[4] = {{1, 0}, {0, 0}, {0, 0}, {-1, 0}};
  if (pauli == 1) gate_1q(psi, L, site, X);
  else if (pauli == 2) gate_1q(psi, L, site, Y);
  else if (pauli == 3) gate_1q(psi, L, site, Z);
}

/* qiskit RZZ(theta) = exp(-i theta/2 Z(x)Z) */
static void gate_rzz(cpx* psi, int L, int i, int j, double theta) {
  const size_t n = (size_t)1 << L;
  const cpx same = cx(cos(-theta / 2), sin(-theta / 2));
  const cpx diff = cconj(same);
#ifdef _OPENMP
#pragma omp parallel for schedule(static) if (ORC_INNER_PAR(n))
#endif
  for (size_t x = 0; x < n; ++x) {
    int zz = (((x >> i) ^ (x >> j)) & 1) ? -1 : 1;
    psi[x] = cmul(psi[x], zz > 0 ? same : diff);
  }
}

/* qiskit RZ(theta) = diag(e^{-i theta/2}, e^{+i theta/2}) */
static void gate_rz(cpx* psi, int L, int i, double theta) {
  const size_t n = (size_t)1 << L;
  const cpx up = cx(cos(-theta / 2), sin(-theta / 2));
  const cpx dn = cconj(up);
#ifdef _OPENMP
#pragma omp parallel for schedule(static) if (ORC_INNER_PAR(n))
#endif
  for (size_t x = 0; x < n; ++x) psi[x] = cmul(psi[x], ((x >> i) & 1) ? dn : up);
}

/* The noise after one kick sub-gate: depolarizing Pauli (fast.py:84-86), or
 * the device-like channel -- importance-weighted amplitude-damping Kraus
 * operator, then the composite dephasing + depolarizing Pauli. */
static void gate_noise(cpx* psi, int L, int site, const orc_rng* rng, uint64_t traj,
                       uint32_t stream, uint32_t period, uint32_t q) {
  if (rng->dev_thr) {
    int jump = 0;
    int pz = orc_device_draw(rng, traj, stream, period, (uint32_t)site, q, rng->dev_jump[site],
                             &jump);
    const double* kr = rng->dev_kraus + 3 * site;
    cpx k[4];
    if (jump) {
      k[0] = cx(0, 0); k[1] = cx(kr[2], 0); k[2] = cx(0, 0); k[3] = cx(0, 0);
    } else {
      k[0] = cx(kr[0], 0); k[1] = cx(0, 0); k[2] = cx(0, 0); k[3] = cx(kr[1], 0);
    }
    gate_1q(psi, L, site, k);
    gate_pauli(psi, L, site, pz);
    return;
  }
  gate_pauli(psi, L, site, orc_pauli(rng, traj, stream, period, (uint32_t)site, q));
}

static void kick_gate(const orc_problem* pr, int row, int site, int q, int dagger, cpx m[4]) {
  const double* g = pr->kick + (((size_t)row * pr->L + site) * pr->n_sub + q) * 8;
  if (!dagger) {
    m[0] = cx(g[0], g[1]); m[1] = cx(g[2], g[3]);
    m[2] = cx(g[4], g[5]); m[3] = cx(g[6], g[7]);
  } else {
    m[0] = cx(g[0], -g[1]); m[1] = cx(g[4], -g[5]);
    m[2] = cx(g[2], -g[3]); m[3] = cx(g[6], -g[7]);
  }
}

/* One forward period (fast.py:111-121), kick row = period - 1. */
static void period_forward(const orc_problem* pr, const orc_rng* rng, int inst, cpx* psi,
                           int period, uint64_t traj, uint32_t stream) {
  const int L = pr->L;
  const double* h = pr->h + (size_t)inst * L;
  const double* phi = pr->phi + (size_t)inst * (L - 1);
  cpx m[4];
  for (int i = 0; i < L; ++i)
    for (int q = 0; q < pr->n_sub; ++q) {
      kick_gate(pr, period - 1, i, q, 0, m);
      gate_1q(psi, L, i, m);
      gate_noise(psi, L, i, rng, traj, stream, (uint32_t)period, (uint32_t)q);
    }
  for (int i = 0; i < L - 1; i += 2) gate_rzz(psi, L, i, i + 1, phi[i]);
  for (int i = 1; i < L - 1; i += 2) gate_rzz(psi, L, i, i + 1, phi[i]);
  for (int i = 0; i < L; ++i) gate_rz(psi, L, i, h[i]);
}

/* UF.inverse() (fast.py:140-143): gates reversed, angles negated; noise after
 * every (inverted) kick gate, rng period counter = echo step. */
static void period_inverse(const orc_problem* pr, const orc_rng* rng, int inst, cpx* psi,
                           int period, int step, uint64_t traj, uint32_t stream) {
  const int L = pr->L;
  const double* h = pr->h + (size_t)inst * L;
  const double* phi = pr->phi + (size_t)inst * (L - 1);
  cpx m[4];
  for (int i = L - 1; i >= 0; --i) gate_rz(psi, L, i, -h[i]);
  int last_odd = ((L - 2) % 2 == 1) ? L - 2 : L - 3;
  for (int i = last_odd; i >= 1; i -= 2) gate_rzz(psi, L, i, i + 1, -phi[i]);
  int last_even = ((L - 2) % 2 == 0) ? L - 2 : L - 3;
  for (int i = last_even; i >= 0; i -= 2) gate_rzz(psi, L, i, i + 1, -phi[i]);
  for (int i = L - 1; i >= 0; --i)
    for (int q = 0; q < pr->n_sub; ++q) {
      kick_gate(pr, period - 1, i, pr->n_sub - 1 - q, 1, m);
      gate_1q(psi, L, i, m);
      gate_noise(psi, L, i, rng, traj, stream, (uint32_t)step, (uint32_t)q);
    }
}

static void measure_z(const cpx* psi, int L, double* out /* [1+L] */) {
  const size_t n = (size_t)1 << L;
  for (int i = 0; i <= L; ++i) out[i] = 0.0;
#ifdef _OPENMP
  if (ORC_INNER_PAR(n)) {
    const int nt = omp_get_max_threads();
    double* part = (double*)calloc((size_t)nt * (L + 1), sizeof(double));
    if (part) {
#pragma omp parallel num_threads(nt)
      {
        // blocks of 4096 amplitudes summed on their own, then added to the
        // thread's partial: no long running sums (the GPU reduces in trees)
        double* o = part + (size_t)omp_get_thread_num() * (L + 1);
        double blk[65];
#pragma omp for schedule(static)
        for (size_t x0 = 0; x0 < n; x0 += 4096) {
          for (int i = 0; i <= L; ++i) blk[i] = 0.0;
          for (size_t x = x0; x < x0 + 4096; ++x) {
            const double p = psi[x].re * psi[x].re + psi[x].im * psi[x].im;
            blk[0] += p;
            for (int i = 0; i < L; ++i) blk[1 + i] += ((x >> i) & 1) ? -p : p;
          }
          for (int i = 0; i <= L; ++i) o[i] += blk[i];
        }
      }
      for (int t = 0; t < nt; ++t)
        for (int i = 0; i <= L; ++i) out[i] += part[(size_t)t * (L + 1) + i];
      free(part);
      return;
    }
  }
#endif
  for (size_t x = 0; x < n; ++x) {
    double p = psi[x].re * psi[x].re + psi[x].im * psi[x].im;
    out[0] += p;
    for (int i = 0; i < L; ++i) out[1 + i] += ((x >> i) & 1) ? -p : p;
  }
}

static uint64_t init_mask(const orc_problem* pr, const orc_rng* rng, uint64_t traj) {
  uint64_t m = pr->init_mask;
  for (int i = 0; i < pr->L; ++i) {
    if (!((pr->init_mask >> i) & 1ull)) continue;
    int jump = 0;
    int pz = rng->dev_thr ? orc_device_draw(rng, traj, 0xFFFFFFFFu, 0u, (uint32_t)i, 0u, 0u, &jump)
                          : orc_pauli(rng, traj, 0xFFFFFFFFu, 0u, (uint32_t)i, 0u);
    if (pz == 1 || pz == 2) m &= ~(1ull << i); /* X.X = I, Y.X ~ Z: back to |0> */
  }
  return m;
}

int orc_apply_periods(const orc_problem* pr, const orc_noise* nz, uint64_t seed, int32_t inst,
                      int64_t traj, uint32_t stream, int32_t first_period, int32_t n_periods,
                      int32_t inverse, double* state, double* zsite_out) {
  orc_rng rng;
  orc_rng_init(&rng, nz->p, seed);
  cpx* psi = (cpx*)state;
  for (int k = 1; k <= n_periods; ++k) {
    if (inverse)
      period_inverse(pr, &rng, inst, psi, first_period - k + 1, k, (uint64_t)traj, stream);
    else
      period_forward(pr, &rng, inst, psi, first_period + k - 1, (uint64_t)traj, stream);
  }
  if (zsite_out) measure_z(psi, pr->L, zsite_out);
  return 0;
}

/* Trajectory schedule of the engine: forward prefix reused for every t, echo
 * at t branches off the forward state after p = t + t_offset periods. */
static int autocorr_run(const orc_problem* pr, const orc_rng* rngp, double fac, double ro_a,
                        double ro_b, int64_t traj_offset, int32_t n_traj, double* fwd,
                        double* echo, double* zsite, int32_t n_threads) {
  const int L = pr->L, T = pr->T;
  const int P = T - 1 + pr->t_offset;
  const size_t n = (size_t)1 << L;
  const int64_t S = (int64_t)pr->n_inst * n_traj;
  const orc_rng rng = *rngp;
  int err = 0;
#ifdef _OPENMP
  if (n_threads > 0) omp_set_num_threads(n_threads);
#pragma omp parallel for schedule(dynamic, 1) if (!ORC_INNER_PAR(n))
#endif
  for (int64_t g = 0; g < S; ++g) {
    const int inst = (int)(g / n_traj);
    const uint64_t traj = (uint64_t)(traj_offset + g % n_traj);
    cpx* F = (cpx*)calloc(n, sizeof(cpx));
    cpx* E = pr->want_echo ? (cpx*)malloc(n * sizeof(cpx)) : NULL;
    double* z = (double*)malloc((size_t)(L + 1) * sizeof(double));
    if (!F || (pr->want_echo && !E) || !z) {
      err = 1;
      free(F); free(E); free(z);
      continue;
    }
    const uint64_t m0 = init_mask(pr, &rng, traj);
    const double zinit = ((m0 >> pr->probe_site) & 1ull) ? -1.0 : 1.0;
    F[m0] = cx(1.0, 0.0);
    for (int p = 0; p <= P; ++p) {
      const int t = p - pr->t_offset;
      if (p > 0) period_forward(pr, &rng, inst, F, p, traj, 0u);
      if (t < 0 || t < pr->t_first) continue;
      if (pr->want_fwd || zsite) {
        measure_z(F, L, z);
        if (pr->want_fwd) fwd[(size_t)g * T + t] = ro_a * (fac * zinit * z[1 + pr->probe_site]) + ro_b;
        if (zsite)
          for (int i = 0; i < L; ++i) zsite[((size_t)g * T + t) * L + i] = z[1 + i];
      }
      if (pr->want_echo) {
        memcpy(E, F, n * sizeof(cpx));
        for (int k = 1; k <= p; ++k)
          period_inverse(pr, &rng, inst, E, p - k + 1, k, traj, (uint32_t)(1 + t));
        measure_z(E, L, z);
        echo[(size_t)g * T + t] = ro_a * (fac * zinit * z[1 + pr->probe_site]) + ro_b;
      }
    }
    free(F); free(E); free(z);
  }
  return err ? -3 : 0;
}

int orc_autocorr(const orc_problem* pr, const orc_noise* nz, uint64_t seed, int64_t traj_offset,
                 int32_t n_traj, double* fwd, double* echo, double* zsite, int32_t n_threads) {
  orc_rng rng;
  orc_rng_init(&rng, nz->p, seed);
  return autocorr_run(pr, &rng, pow(1.0 - nz->p, (double)nz->n_anc), 1.0, 0.0, traj_offset,
                      n_traj, fwd, echo, zsite, n_threads);
}

static uint32_t orc_u32(double prob) {
  double v = floor(prob * 4294967296.0 + 0.5);
  if (v >= 4294967295.0) v = 4294967295.0;
  if (v < 0) v = 0;
  return (uint32_t)v;
}

/* Device-like noise (include/dtc.h dtc_device_noise), restated: per site
 * gamma = 1 - exp(-tg/T1); pure dephasing Z w.p. (1 - exp(-tg (1/T2 - 1/2T1)))/2
 * (T2 <= 2 T1); composite with depolarizing(p): X, Y p/4, Z (1-d) p/4 + d (1-3p/4);
 * jump w.p. q1 = gamma/2 with K1/sqrt(q1), else K0/sqrt(1 - q1). */
typedef struct {
  orc_rng rng;
  uint32_t* thr;
  uint32_t* jmp;
  double* kr;
} orc_device_rng;

static void device_rng_free(orc_device_rng* d) {
  free(d->thr); free(d->jmp); free(d->kr);
}

static int device_rng_init(orc_device_rng* d, const orc_device_noise* dv, int L, uint64_t seed) {
  d->thr = (uint32_t*)malloc(sizeof(uint32_t) * 3 * L);
  d->jmp = (uint32_t*)malloc(sizeof(uint32_t) * L);
  d->kr = (double*)malloc(sizeof(double) * 3 * L);
  if (!d->thr || !d->jmp || !d->kr) { device_rng_free(d); return -3; }
  for (int i = 0; i < L; ++i) {
    const double p = dv->p_gate[i];
    const double t1 = dv->t1_us[i] > 0.0 ? dv->t1_us[i] * 1e3 : INFINITY;
    double t2 = dv->t2_us[i] > 0.0 ? dv->t2_us[i] * 1e3 : INFINITY;
    if (t2 > 2.0 * t1) t2 = 2.0 * t1;
    const double tg = dv->gate_ns;
    const double gamma = isinf(t1) ? 0.0 : 1.0 - exp(-tg / t1);
    double rate = (isinf(t2) ? 0.0 : 1.0 / t2) - (isinf(t1) ? 0.0 : 0.5 / t1);
    if (rate < 0.0) rate = 0.0;
    const double dd = 0.5 * (1.0 - exp(-tg * rate));
    const double px = p / 4.0, py = p / 4.0;
    const double pz = (1.0 - dd) * p / 4.0 + dd * (1.0 - 3.0 * p / 4.0);
    d->thr[3 * i + 0] = orc_u32(px);
    d->thr[3 * i + 1] = orc_u32(px + py);
    d->thr[3 * i + 2] = orc_u32(px + py + pz);
    const double q1 = gamma / 2.0, q0 = 1.0 - q1;
    d->jmp[i] = orc_u32(q1);
    d->kr[3 * i + 0] = 1.0 / sqrt(q0);
    d->kr[3 * i + 1] = sqrt(1.0 - gamma) / sqrt(q0);
    d->kr[3 * i + 2] = q1 > 0.0 ? sqrt(gamma / q1) : 0.0;
  }
  orc_rng_init(&d->rng, 0.0, seed);
  d->rng.noisy = 1;
  d->rng.dev_thr = d->thr;
  d->rng.dev_jump = d->jmp;
  d->rng.dev_kraus = d->kr;
  return 0;
}

int orc_autocorr_device(const orc_problem* pr, const orc_device_noise* dv, uint64_t seed,
                        int64_t traj_offset, int32_t n_traj, double* fwd, double* echo,
                        double* zsite, int32_t n_threads) {
  orc_device_rng d;
  if (device_rng_init(&d, dv, pr->L, seed)) return -3;
  const int rc = autocorr_run(pr, &d.rng, dv->anc_factor, 1.0 - dv->readout_p01 - dv->readout_p10,
                              dv->readout_p10 - dv->readout_p01, traj_offset, n_traj, fwd, echo,
                              zsite, n_threads);
  device_rng_free(&d);
  return rc;
}

/* orc_apply_periods under device-like noise (the energy path's trajectories:
 * the state's norm carries the Kraus importance weight). */
int orc_apply_periods_device(const orc_problem* pr, const orc_device_noise* dv, uint64_t seed,
                             int32_t inst, int64_t traj, uint32_t stream, int32_t first_period,
                             int32_t n_periods, int32_t inverse, double* state,
                             double* zsite_out) {
  orc_device_rng d;
  if (device_rng_init(&d, dv, pr->L, seed)) return -3;
  cpx* psi = (cpx*)state;
  for (int k = 1; k <= n_periods; ++k) {
    if (inverse)
      period_inverse(pr, &d.rng, inst, psi, first_period - k + 1, k, (uint64_t)traj, stream);
    else
      period_forward(pr, &d.rng, inst, psi, first_period + k - 1, (uint64_t)traj, stream);
  }
  if (zsite_out) measure_z(psi, pr->L, zsite_out);
  device_rng_free(&d);
  return 0;
}

/* Basis state after the noisy neel preparation of trajectory traj (dv NULL:
 * depolarizing p). */
int64_t orc_init_mask(const orc_problem* pr, double p, const orc_device_noise* dv,
                      uint64_t seed, int64_t traj) {
  if (dv) {
    orc_device_rng d;
    if (device_rng_init(&d, dv, pr->L, seed)) return -3;
    const uint64_t m = init_mask(pr, &d.rng, (uint64_t)traj);
    device_rng_free(&d);
    return (int64_t)m;
  }
  orc_rng rng;
  orc_rng_init(&rng, p, seed);
  return (int64_t)init_mask(pr, &rng, (uint64_t)traj);
}


/* ---- period-fused CPU restatement (bench.py's cpu_baseline) -------------
 * The same trajectories, schedule and Philox draws as orc_autocorr, with each
 * period fused per state instead of gate by gate:
 *   - per site, the noisy kick of the period is one 2x2 matrix
 *     M_i = P_n G_n ... P_1 G_1 (forward) or P_n G_1^+ ... P_1 G_n^+ (inverse);
 *   - the state is kept as split real / imaginary arrays (4-wide FMA spans);
 *   - sites 0..11 are applied inside 4096-amplitude blocks, sites >= 12 on
 *     panels of 16 adjacent columns (2^(L-12) rows, copied to a contiguous
 *     buffer), i.e. two sweeps of the state per period;
 *   - the RZZ/RZ layer is D(x) = Dlo[x & 4095] * Dhi[x >> 11] (sites 0..11 and
 *     their bonds | sites >= 12 and the bonds from 11 up), applied in the
 *     high-site sweep, where <Z_j> is also accumulated.
 * Results equal orc_autocorr per trajectory to rounding (tests/test_oracle.py). */
#define FUS_LO 12
#define FUS_COLS 16

static void mat2_mul(cpx c[4], const cpx a[4], const cpx b[4]) {
  cpx r[4];
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j)
      r[2 * i + j] = cadd(cmul(a[2 * i], b[j]), cmul(a[2 * i + 1], b[2 + j]));
  memcpy(c, r, sizeof(r));
}

static void pauli_mat(int pz, cpx m[4]) {
  static const cpx P[4][4] = {{{1, 0}, {0, 0}, {0, 0}, {1, 0}},
                              {{0, 0}, {1, 0}, {1, 0}, {0, 0}},
                              {{0, 0}, {0, -1}, {0, 1}, {0, 0}},
                              {{1, 0}, {0, 0}, {0, 0}, {-1, 0}}};
  memcpy(m, P[pz], sizeof(P[pz]));
}

/* noisy kick matrix of one site: forward period `period` (row period-1) or
 * the inverse of period `period` drawn at echo step `step` */
static void fused_site_kick(const orc_problem* pr, const orc_rng* rng, int site, int period,
                            int inverse, int step, uint64_t traj, uint32_t stream, cpx m[4]) {
  pauli_mat(0, m);
  for (int q = 0; q < pr->n_sub; ++q) {
    cpx g[4], pm[4];
    kick_gate(pr, period - 1, site, inverse ? pr->n_sub - 1 - q : q, inverse, g);
    mat2_mul(m, g, m);
    const int pz = orc_pauli(rng, traj, stream, (uint32_t)(inverse ? step : period),
                             (uint32_t)site, (uint32_t)q);
    if (pz) {
      pauli_mat(pz, pm);
      mat2_mul(m, pm, m);
    }
  }
}

typedef struct { double* re; double* im; } split;

/* (a[k], b[k]) <- M (a[k], b[k]) for k < n */
static void bfly_span(double* restrict are, double* restrict aim, double* restrict bre,
                      double* restrict bim, size_t n, const cpx m[4]) {
  const double ar = m[0].re, ai = m[0].im, br = m[1].re, bi = m[1].im;
  const double cr = m[2].re, ci = m[2].im, dr = m[3].re, di = m[3].im;
  for (size_t k = 0; k < n; ++k) {
    const double ur = are[k], ui = aim[k], vr = bre[k], vi = bim[k];
    are[k] = ar * ur - ai * ui + br * vr - bi * vi;
    aim[k] = ar * ui + ai * ur + br * vi + bi * vr;
    bre[k] = cr * ur - ci * ui + dr * vr - di * vi;
    bim[k] = cr * ui + ci * ur + dr * vi + di * vr;
  }
}

/* the kick of index bit i over a contiguous span of 2^nb amplitudes */
static void kick_span(double* re, double* im, int nb, int i, const cpx m[4]) {
  const size_t bit = (size_t)1 << i, n = (size_t)1 << nb;
  if (i == 0) {
    const double ar = m[0].re, ai = m[0].im, br = m[1].re, bi = m[1].im;
    const double cr = m[2].re, ci = m[2].im, dr = m[3].re, di = m[3].im;
    for (size_t x = 0; x < n; x += 2) {
      const double ur = re[x], ui = im[x], vr = re[x + 1], vi = im[x + 1];
      re[x] = ar * ur - ai * ui + br * vr - bi * vi;
      im[x] = ar * ui + ai * ur + br * vi + bi * vr;
      re[x + 1] = cr * ur - ci * ui + dr * vr - di * vi;
      im[x + 1] = cr * ui + ci * ur + dr * vi + di * vr;
    }
    return;
  }
  for (size_t x0 = 0; x0 < n; x0 += 2 * bit)
    bfly_span(re + x0, im + x0, re + x0 + bit, im + x0 + bit, bit, m);
}

static void diag_span(double* restrict re, double* restrict im, const double* restrict dre,
                      const double* restrict dim, double sc, size_t n) {
  for (size_t k = 0; k < n; ++k) {
    const double ur = re[k], ui = im[k], cr = dre[k], ci = sc * dim[k];
    re[k] = ur * cr - ui * ci;
    im[k] = ur * ci + ui * cr;
  }
}

typedef struct {
  int L, lo;
  double *dlo_re, *dlo_im;   /* [2^lo]                       */
  double *dhi_re, *dhi_im;   /* [2^(L-lo+1)] (bits 11..L-1)   */
  double *pre, *pim;         /* panel [rows][FUS_COLS]        */
  double *rowd_re, *rowd_im; /* diagonal of one panel row     */
} fused_ws;

static double zsign(size_t x, int j) { return ((x >> j) & 1) ? -1.0 : 1.0; }

static void fused_tables(const orc_problem* pr, int inst, fused_ws* w) {
  const int L = pr->L, lo = w->lo;
  const double* h = pr->h + (size_t)inst * L;
  const double* phi = pr->phi + (size_t)inst * (L > 1 ? L - 1 : 0);
  for (size_t x = 0; x < ((size_t)1 << lo); ++x) {
    double a = 0.0;
    for (int i = 0; i < lo; ++i) a += h[i] * zsign(x, i);
    for (int i = 0; i + 1 < lo; ++i) a += phi[i] * zsign(x, i) * zsign(x, i + 1);
    w->dlo_re[x] = cos(-0.5 * a);
    w->dlo_im[x] = sin(-0.5 * a);
  }
  if (L > lo) {
    for (size_t y = 0; y < ((size_t)1 << (L - lo + 1)); ++y) {
      const size_t x = y << (lo - 1); /* bits lo-1 .. L-1 */
      double a = 0.0;
      for (int i = lo; i < L; ++i) a += h[i] * zsign(x, i);
      for (int i = lo - 1; i + 1 < L; ++i) a += phi[i] * zsign(x, i) * zsign(x, i + 1);
      w->dhi_re[y] = cos(-0.5 * a);
      w->dhi_im[y] = sin(-0.5 * a);
    }
  }
}

static void probe_span(const double* re, const double* im, size_t x0, size_t n, int j,
                       double* nn, double* zz) {
  double a = 0.0, b = 0.0;
  for (size_t k = 0; k < n; ++k) {
    const double p = re[k] * re[k] + im[k] * im[k];
    a += p;
    b += zsign(x0 + k, j) * p;
  }
  *nn += a;
  *zz += b;
}

/* kicks on sites < lo inside each 2^lo block (+ the whole diagonal and the
 * probe when L <= lo); sum |a|^2 and z_j |a|^2 of the result when zj */
static void fused_low(split psi, const fused_ws* w, const cpx (*M)[4], int diag, int conj,
                      int diag_first, int j, double* norm, double* zj) {
  const size_t blk = (size_t)1 << w->lo, n = (size_t)1 << w->L;
  const double sc = conj ? -1.0 : 1.0;
  double nn = 0.0, zz = 0.0;
  for (size_t b0 = 0; b0 < n; b0 += blk) {
    double *re = psi.re + b0, *im = psi.im + b0;
    if (diag && diag_first) diag_span(re, im, w->dlo_re, w->dlo_im, sc, blk);
    for (int i = 0; i < w->lo && i < w->L; ++i) kick_span(re, im, w->lo, i, M[i]);
    if (diag && !diag_first) diag_span(re, im, w->dlo_re, w->dlo_im, sc, blk);
    if (zj) probe_span(re, im, b0, blk, j, &nn, &zz);
  }
  if (zj) { *norm = nn; *zj = zz; }
}

/* kicks on sites >= lo and the diagonal D or D^* (before the kicks when
 * diag_first) on panels of FUS_COLS columns; optional probe after both */
static void fused_high(split psi, const fused_ws* w, const cpx (*M)[4], int conj, int diag_first,
                       int j, double* norm, double* zj) {
  const int L = w->L, lo = w->lo, hb = L - lo;
  const size_t blk = (size_t)1 << lo, rows = (size_t)1 << hb;
  const double sc = conj ? -1.0 : 1.0;
  double nn = 0.0, zz = 0.0;
  double *PR = w->pre, *PI = w->pim;
  for (size_t c0 = 0; c0 < blk; c0 += FUS_COLS) {
    for (size_t r = 0; r < rows; ++r) {
      memcpy(PR + r * FUS_COLS, psi.re + r * blk + c0, sizeof(double) * FUS_COLS);
      memcpy(PI + r * FUS_COLS, psi.im + r * blk + c0, sizeof(double) * FUS_COLS);
    }
    for (int pass = 0; pass < 2; ++pass) {
      if (pass == (diag_first ? 0 : 1)) {
        const size_t b11 = (c0 >> (lo - 1)) & 1;
        for (size_t r = 0; r < rows; ++r) {
          const double hr = w->dhi_re[(r << 1) | b11], hi = w->dhi_im[(r << 1) | b11];
          for (int c = 0; c < FUS_COLS; ++c) {
            w->rowd_re[c] = hr * w->dlo_re[c0 + c] - hi * w->dlo_im[c0 + c];
            w->rowd_im[c] = hr * w->dlo_im[c0 + c] + hi * w->dlo_re[c0 + c];
          }
          diag_span(PR + r * FUS_COLS, PI + r * FUS_COLS, w->rowd_re, w->rowd_im, sc, FUS_COLS);
        }
      } else {
        for (int i = 0; i < hb; ++i) {
          const size_t bit = (size_t)1 << i;
          for (size_t r0 = 0; r0 < rows; r0 += 2 * bit)
            bfly_span(PR + r0 * FUS_COLS, PI + r0 * FUS_COLS, PR + (r0 + bit) * FUS_COLS,
                      PI + (r0 + bit) * FUS_COLS, bit * FUS_COLS, M[lo + i]);
        }
      }
    }
    for (size_t r = 0; r < rows; ++r) {
      memcpy(psi.re + r * blk + c0, PR + r * FUS_COLS, sizeof(double) * FUS_COLS);
      memcpy(psi.im + r * blk + c0, PI + r * FUS_COLS, sizeof(double) * FUS_COLS);
      if (zj) probe_span(PR + r * FUS_COLS, PI + r * FUS_COLS, r * blk + c0, FUS_COLS, j, &nn, &zz);
    }
  }
  if (zj) { *norm = nn; *zj = zz; }
}

int orc_autocorr_fused(const orc_problem* pr, const orc_noise* nz, uint64_t seed,
                       int64_t traj_offset, int32_t n_traj, double* fwd, double* echo,
                       int32_t n_threads) {
  orc_rng rng0;
  orc_rng_init(&rng0, nz->p, seed);
  const orc_rng rng = rng0;
  const double fac = pow(1.0 - nz->p, (double)nz->n_anc);
  const int L = pr->L, T = pr->T, P = T - 1 + pr->t_offset, j = pr->probe_site;
  const int lo = L < FUS_LO ? L : FUS_LO;
  const size_t n = (size_t)1 << L;
  const int64_t S = (int64_t)pr->n_inst * n_traj;
  int err = 0;
  if (L > 40) return -1;
#ifdef _OPENMP
  if (n_threads > 0) omp_set_num_threads(n_threads);
#pragma omp parallel
#endif
  {
    fused_ws w;
    w.L = L;
    w.lo = lo;
    const size_t nlo = (size_t)1 << lo, nhi = (size_t)1 << (L - lo + 1);
    const size_t npan = (size_t)FUS_COLS << (L - lo);
    double* pool = (double*)malloc(sizeof(double) * (2 * nlo + 2 * nhi + 2 * npan + 2 * FUS_COLS +
                                                     (pr->want_echo ? 4 : 2) * n));
    cpx(*M)[4] = (cpx(*)[4])malloc(sizeof(cpx) * 4 * (size_t)L);
    int inst_tab = -1;
    if (!pool || !M) {
#ifdef _OPENMP
#pragma omp atomic write
#endif
      err = 1;
    } else {
      double* q = pool;
      w.dlo_re = q; q += nlo; w.dlo_im = q; q += nlo;
      w.dhi_re = q; q += nhi; w.dhi_im = q; q += nhi;
      w.pre = q; q += npan; w.pim = q; q += npan;
      w.rowd_re = q; q += FUS_COLS; w.rowd_im = q; q += FUS_COLS;
      split F = {q, q + n};
      q += 2 * n;
      split E = {q, q + n};
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
      for (int64_t g = 0; g < S; ++g) {
        const int inst = (int)(g / n_traj);
        const uint64_t traj = (uint64_t)(traj_offset + g % n_traj);
        if (inst != inst_tab) {
          fused_tables(pr, inst, &w);
          inst_tab = inst;
        }
        memset(F.re, 0, 2 * n * sizeof(double));
        const uint64_t m0 = init_mask(pr, &rng, traj);
        const double zinit = ((m0 >> j) & 1ull) ? -1.0 : 1.0;
        F.re[m0] = 1.0;
        for (int p = 0; p <= P; ++p) {
          const int t = p - pr->t_offset;
          double nrm = 1.0, zj = zinit;
          if (p > 0) {
            for (int i = 0; i < L; ++i) fused_site_kick(pr, &rng, i, p, 0, 0, traj, 0u, M[i]);
            if (L > lo) {
              fused_low(F, &w, (const cpx(*)[4])M, 0, 0, 0, j, NULL, NULL);
              fused_high(F, &w, (const cpx(*)[4])M, 0, 0, j, &nrm, &zj);
            } else {
              fused_low(F, &w, (const cpx(*)[4])M, 1, 0, 0, j, &nrm, &zj);
            }
          }
          (void)nrm;
          if (t < 0 || t < pr->t_first) continue;
          if (pr->want_fwd) fwd[(size_t)g * T + t] = fac * zinit * zj;
          if (pr->want_echo) {
            memcpy(E.re, F.re, 2 * n * sizeof(double));
            double ez = zinit, en = 1.0;
            for (int k = 1; k <= p; ++k) {
              const int pp = p - k + 1;
              for (int i = 0; i < L; ++i)
                fused_site_kick(pr, &rng, i, pp, 1, k, traj, (uint32_t)(1 + t), M[i]);
              const int last = k == p;
              if (L > lo) {
                fused_high(E, &w, (const cpx(*)[4])M, 1, 1, j, NULL, NULL);
                fused_low(E, &w, (const cpx(*)[4])M, 0, 0, 0, j, last ? &en : NULL,
                          last ? &ez : NULL);
              } else {
                fused_low(E, &w, (const cpx(*)[4])M, 1, 1, 1, j, last ? &en : NULL,
                          last ? &ez : NULL);
              }
            }
            (void)en;
            echo[(size_t)g * T + t] = fac * zinit * ez;
          }
        }
      }
    }
    free(pool);
    free(M);
  }
  return err ? -3 : 0;
}

/* Exposed for the RNG contract test. */
int orc_sample_pauli(double p, uint64_t seed, uint64_t traj, uint32_t stream, uint32_t period,
                     uint32_t site, uint32_t sub) {
  orc_rng rng;
  orc_rng_init(&rng, p, seed);
  return orc_pauli(&rng, traj, stream, period, site, sub);
}
