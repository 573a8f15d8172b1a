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
} orc_rng;

static void orc_rng_init(orc_rng* r, double p, uint64_t seed) {
  for (int k = 1; k <= 3; ++k) {
    double v = floor(k * p / 4.0 * 4294967296.0 + 0.5);
    if (v > 4294967295.0) v = 4294967295.0;
    r->thr[k - 1] = (uint32_t)v;
  }
  r->noisy = p > 0.0;
  r->seed = seed;
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

/* ---- gates on a 2^L statevector (bit i = site i) ------------------------ */
static void gate_1q(cpx* psi, int L, int site, const cpx m[4]) {
  const size_t n = (size_t)1 << L, bit = (size_t)1 << site;
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
  for (size_t x = 0; x < n; ++x) psi[x] = cmul(psi[x], ((x >> i) & 1) ? dn : up);
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
      gate_pauli(psi, L, i, orc_pauli(rng, traj, stream, (uint32_t)period, (uint32_t)i, (uint32_t)q));
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
      gate_pauli(psi, L, i, orc_pauli(rng, traj, stream, (uint32_t)step, (uint32_t)i, (uint32_t)q));
    }
}

static void measure_z(const cpx* psi, int L, double* out /* [1+L] */) {
  const size_t n = (size_t)1 << L;
  for (int i = 0; i <= L; ++i) out[i] = 0.0;
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
    int pz = orc_pauli(rng, traj, 0xFFFFFFFFu, 0u, (uint32_t)i, 0u);
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
int orc_autocorr(const orc_problem* pr, const orc_noise* nz, uint64_t seed, int64_t traj_offset,
                 int32_t n_traj, double* fwd, double* echo, double* zsite, int32_t n_threads) {
  const int L = pr->L, T = pr->T;
  const int P = T - 1 + pr->t_offset;
  const size_t n = (size_t)1 << L;
  const double fac = pow(1.0 - nz->p, (double)nz->n_anc);
  const int64_t S = (int64_t)pr->n_inst * n_traj;
  orc_rng rng;
  orc_rng_init(&rng, nz->p, seed);
  int err = 0;
#ifdef _OPENMP
  if (n_threads > 0) omp_set_num_threads(n_threads);
#pragma omp parallel for schedule(dynamic, 1)
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
        if (pr->want_fwd) fwd[(size_t)g * T + t] = fac * zinit * z[1 + pr->probe_site];
        if (zsite)
          for (int i = 0; i < L; ++i) zsite[((size_t)g * T + t) * L + i] = z[1 + i];
      }
      if (pr->want_echo) {
        memcpy(E, F, n * sizeof(cpx));
        for (int k = 1; k <= p; ++k)
          period_inverse(pr, &rng, inst, E, p - k + 1, k, traj, (uint32_t)(1 + t));
        measure_z(E, L, z);
        echo[(size_t)g * T + t] = fac * zinit * z[1 + pr->probe_site];
      }
    }
    free(F); free(E); free(z);
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
