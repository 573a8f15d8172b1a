// dtc_kernels.hip — gfx950 (CDNA4) kernels for the DTC Floquet period.
//
// One Floquet period of the reference (create_UF_subcircuit, fast.py:111-121):
//   RX(pi g) on every site  ->  RZZ(phi_i) on even then odd bonds  ->
//   RZ(h_i) on every site,
// with a Pauli draw after every kick gate (depolarizing noise on u3,
// fast.py:84-86).  The inverse period (fast.py:140-143) is RZ(-h), RZZ(-phi),
// RX(-pi g) with noise after each kick.
//
// Kicks on different sites commute and RZZ/RZ form one diagonal D(x), so a
// sweep is the layer sequence K_1 D K_2 D K_3 ...  The sites are split in two
// groups A (low index bits) and B (high bits) whose kicks fit a 4096-amplitude
// tile each.  A pass over group G applies K_{p,G} . D . K_{p+1,G}: it finishes
// period p on G (the other group already has K_p), closes the period with the
// diagonal, and starts period p+1 on G.  Passes alternate A, B, A, ... so every
// pass advances one full period: 32 B of HBM traffic per amplitude per period.
//
// Inside a pass a workgroup loads its tile (16 amplitudes per lane, coalesced
// 16-B loads), applies each site's 2x2 kick as register butterflies in 4-site
// rounds, re-layouts the tile through 64 KiB of XOR-swizzled (bank-conflict
// free) LDS between rounds, applies the diagonal from per-instance LDS factor
// tables, optionally reduces |a|^2 Z_i for the autocorrelator, and stores the
// tile back.  Memory-bound by design; no MFMA (complex128 butterflies are not
// GEMM-shaped).  Kicks of the RX family (every Pauli x RX(theta) has one real
// and one imaginary entry per row) run as 4-flop-per-amplitude butterflies;
// other kicks (RY products, circular polarization) use the general form.
#include <cstdlib>
#include <type_traits>

#include "dtc_device.h"
#include "dtc_kernels.h"
#include "dtc_rng.h"

// Nontemporal tile loads / stores (bit 0 load, bit 1 store), per pass family:
// A = passes over a full 12-site group (NIBS 7), B = the others.  The tile is
// touched once per pass, so streaming hints keep it from displacing lines in
// the caches: same-box A/B on C2 (profiles/r1r_nt_ab.json) 154.1k -> 159.6k
// periods*inst/s, group-B pass 1.62 -> 1.53 ms, group A unchanged.  -D
// overrides are for development A/B builds only.
#ifndef DTC_NT_A
#define DTC_NT_A 3
#endif
#ifndef DTC_NT_B
#define DTC_NT_B 3
#endif

namespace dtc {

// m <- P m for Pauli code (1 X, 2 Y, 3 Z)
__device__ __forceinline__ void pauli_left(double2* m, int pauli) {
  if (pauli == 1) {
    double2 t0 = m[0], t1 = m[1];
    m[0] = m[2]; m[1] = m[3]; m[2] = t0; m[3] = t1;
  } else if (pauli == 2) {
    // Y = [[0, -i], [i, 0]]: row0 <- -i row1, row1 <- i row0
    double2 r00 = m[0], r01 = m[1];
    m[0] = make_double2(m[2].y, -m[2].x);
    m[1] = make_double2(m[3].y, -m[3].x);
    m[2] = make_double2(-r00.y, r00.x);
    m[3] = make_double2(-r01.y, r01.x);
  } else if (pauli == 3) {
    m[2] = make_double2(-m[2].x, -m[2].y);
    m[3] = make_double2(-m[3].x, -m[3].y);
  }
}

// c <- a b (2x2 complex)
__device__ __forceinline__ void mat_mul(double2* c, const double2* a, const double2* b) {
  double2 r[4];
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j) {
      double2 x = cmul(a[2 * i + 0], b[0 + j]);
      double2 y = cmul(a[2 * i + 1], b[2 + j]);
      r[2 * i + j] = make_double2(x.x + y.x, x.y + y.y);
    }
  for (int k = 0; k < 4; ++k) c[k] = r[k];
}

__device__ __forceinline__ void dagger(double2* m) {
  double2 m01 = m[1];
  m[0].y = -m[0].y;
  m[3].y = -m[3].y;
  m[1] = make_double2(m[2].x, -m[2].y);
  m[2] = make_double2(m01.x, -m01.y);
}

// Noisy kick of one site for one layer (see KickMode).
__device__ void build_site_kick(const PrepArgs& P, const KickDesc& K, int site, uint64_t traj,
                                double2* m) {
  m[0] = make_double2(1.0, 0.0);
  m[1] = make_double2(0.0, 0.0);
  m[2] = make_double2(0.0, 0.0);
  m[3] = make_double2(1.0, 0.0);
  const bool inv = (K.mode == kKickInverse);
  if (K.mode == kKickBasisX) {
    const double r = 0.70710678118654752440;
    m[0] = make_double2(r, 0.0); m[1] = make_double2(r, 0.0);
    m[2] = make_double2(r, 0.0); m[3] = make_double2(-r, 0.0);
    return;
  }
  for (int q = 0; q < P.n_sub; ++q) {
    const int qq = inv ? (P.n_sub - 1 - q) : q;
    const double2* gp = P.kick + (((int64_t)K.row * P.L_kick + site) * P.n_sub + qq) * 4;
    double2 gm[4] = {gp[0], gp[1], gp[2], gp[3]};
    if (inv) dagger(gm);
    mat_mul(m, gm, m);
    if (P.dev_thr) {
      // device-like noise: amplitude-damping Kraus operator drawn with fixed
      // probabilities (q1 = gamma/2) and weighted by 1/sqrt(q) -- the
      // trajectory stays linear and its mean is the exact channel -- then the
      // composite dephasing + depolarizing Pauli
      int jump = 0;
      const int p = sample_device(P.seed, traj, K.stream, K.rng_period, (uint32_t)site,
                                  (uint32_t)q, P.dev_thr + 3 * site, P.dev_thr_jump[site], &jump);
      const double* kr = P.dev_kraus + 3 * site;
      if (jump) {  // K1 = [[0, b], [0, 0]]: row 0 <- b row 1, row 1 <- 0
        m[0] = make_double2(kr[2] * m[2].x, kr[2] * m[2].y);
        m[1] = make_double2(kr[2] * m[3].x, kr[2] * m[3].y);
        m[2] = make_double2(0.0, 0.0);
        m[3] = make_double2(0.0, 0.0);
      } else {     // K0 = diag(a0, a1)
        m[0] = make_double2(kr[0] * m[0].x, kr[0] * m[0].y);
        m[1] = make_double2(kr[0] * m[1].x, kr[0] * m[1].y);
        m[2] = make_double2(kr[1] * m[2].x, kr[1] * m[2].y);
        m[3] = make_double2(kr[1] * m[3].x, kr[1] * m[3].y);
      }
      pauli_left(m, p);
    } else if (P.noisy) {
      int p = sample_pauli(P.seed, traj, K.stream, K.rng_period, (uint32_t)site, (uint32_t)q,
                           P.thr1, P.thr2, P.thr3);
      pauli_left(m, p);
    }
  }
  if (K.mode == kKickUndo || K.mode == kKickUndoBasisX) dagger(m);
  if (K.mode == kKickUndoBasisX) {
    const double r = 0.70710678118654752440;
    double2 h[4] = {make_double2(r, 0.0), make_double2(r, 0.0), make_double2(r, 0.0),
                    make_double2(-r, 0.0)};
    mat_mul(m, h, m);
  }
}

// Per-site kick of a pass, canonicalised for the pass's matrix family.
// RX family: every unitary i^k [[a, ib], [ic, d]] (a, b, c, d real; Pauli x
// RX(theta) products, their daggers) has d = sigma a, c = sigma b, sigma = +-1,
// so  M = i^k * w * diag(1, sigma) * S  with
//   form A (|a| >= |b|): w = a, S = [[1, i beta], [i beta, 1]],  beta  = b / a
//   form B (|a| <  |b|): w = b, S = [[alpha, i], [i, alpha]],    alpha = a / b
// (|coef| <= 1).  S costs 4 FMAs per amplitude pair (2 per amplitude, half of
// the unfactored butterfly), sigma is a source-negate variant of the same
// FMAs, and the real scales w of all sites multiply the pass's global phase.
// RY family: real orthogonal i^k [[a, b], [c, d]] (rotation or reflection):
// d = sigma a, c = -sigma b,  M = i^k * w * diag(1, sigma) * R,
//   form A: R = [[1, beta], [-beta, 1]],  form B: R = [[alpha, 1], [-1, alpha]].
// General kicks (xy, circular, X-basis) keep the full complex 2x2.
// Device-like noise (kKindRXU / kKindRYU, one sub-gate per kick): the kick
// is a real diagonal Kraus factor times a unitary of the family (a Pauli
// after the Kraus factor moves to its right: X diag(k0, k1) = diag(k1, k0) X;
// the jump operator is diag(1, 0) X up to its weight), so
//   M = i^k * w * diag(rho0, rho1) * S,   S as in form A / B below,
// rho0 = 1 with w, S from the first row (d = rho1 a, c = rho1 b for RX,
// c = -rho1 b for RY; rho1 = sigma = +-1 when unitary), or rho0 = 0, rho1 = 1
// with w, S from the second row when the first is zero (a jump followed by an
// X or Y).  The kernel runs S (var 0 / 2) and defers every site's
// diag(rho0, rho1): they commute with the other sites' butterflies and with D,
// so a layer's factors multiply each amplitude once, prod_i rho_{i, x_i} (at
// the diagonal for the pre-kick, before the store for the post-kick): 2 FMAs
// per amplitude and site instead of the 4 of the unfactored butterfly.
struct SiteMat {
  double2 m[4];  // general form
  double coef;   // RX/RY: beta (form A) or alpha (form B)
  double scale;  // RX/RY: w
  double rho0, rho1;  // RXU/RYU: the deferred diag(rho0, rho1)
  int var;       // RX/RY: (form B ? 2 : 0) | (sigma < 0 ? 1 : 0); RXU/RYU: form B ? 2 : 0
  int k;         // power of i
};

__device__ __forceinline__ void canonicalise(int kind, const double2* m, SiteMat& sm) {
  sm.k = 0;
  sm.coef = 0.0;
  sm.scale = 1.0;
  sm.rho0 = 1.0;
  sm.rho1 = 1.0;
  sm.var = 0;
  double a, b, c, d;
  if (kind == kKindRX || kind == kKindRXU) {
    const bool a_form = (m[0].y == 0.0 && m[1].x == 0.0 && m[2].x == 0.0 && m[3].y == 0.0);
    // B form [[i a, b], [c, i d]] = i [[a, -i b], [-i c, d]]
    a = a_form ? m[0].x : m[0].y;
    b = a_form ? m[1].y : -m[1].x;
    c = a_form ? m[2].y : -m[2].x;
    d = a_form ? m[3].x : m[3].y;
    sm.k = a_form ? 0 : 1;
  } else if (kind == kKindRY || kind == kKindRYU) {
    const bool real = (m[0].y == 0.0 && m[1].y == 0.0 && m[2].y == 0.0 && m[3].y == 0.0);
    // imaginary form i [[a, b], [c, d]]
    a = real ? m[0].x : m[0].y;
    b = real ? m[1].x : m[1].y;
    c = real ? m[2].x : m[2].y;
    d = real ? m[3].x : m[3].y;
    sm.k = real ? 0 : 1;
  } else {
    for (int e = 0; e < 4; ++e) sm.m[e] = m[e];
    return;
  }
  if (kind == kKindRXU || kind == kKindRYU) {  // factored with a deferred diag(rho0, rho1)
    const bool rx = kind == kKindRXU;
    if (a != 0.0 || b != 0.0) {  // from the first row: rho0 = 1
      const bool form_b = fabs(a) < fabs(b);
      sm.scale = form_b ? b : a;
      sm.coef = form_b ? a / b : b / a;
      sm.var = form_b ? 2 : 0;
      sm.rho1 = form_b ? (rx ? c / b : -c / b) : d / a;
    } else if (c != 0.0 || d != 0.0) {  // from the second row: diag(0, 1)
      // RX: (i c, d) = w (i beta, 1) | w (i, alpha); RY: (c, d) = w (-beta, 1) | w (-1, alpha)
      const bool form_b = fabs(d) < fabs(c);
      sm.scale = form_b ? (rx ? c : -c) : d;
      sm.coef = form_b ? d / sm.scale : (rx ? c / d : -c / d);
      sm.var = form_b ? 2 : 0;
      sm.rho0 = 0.0;
    } else {  // the zero matrix: a zero-weight trajectory
      sm.scale = 0.0;
      sm.rho0 = sm.rho1 = 0.0;
    }
    return;
  }
  // sigma from a d + b c = sigma (a^2 + b^2) (RX) or a d - b c (RY)
  const double sg = kind == kKindRX ? a * d + b * c : a * d - b * c;
  const bool neg = sg < 0.0;
  const bool form_b = fabs(a) < fabs(b);
  sm.scale = form_b ? b : a;
  sm.coef = form_b ? a / b : b / a;
  sm.var = (form_b ? 2 : 0) | (neg ? 1 : 0);
}

// Pauli-frame records of a 13-site pass (dtc_tile13.hip).  The pass runs one
// butterfly for every kick, the form-B one G(f) (RX: f I + i X; RY: f I + i Y),
// so its kicks carry no variant branches (the 128-VGPR budget of the 13-bit
// tile spilled at the four-way branches, r6d).  The other forms become Paulis:
// form A is A(beta) = -i X G(-beta) (RX) or X Z G(-beta) (RY), sigma = -1 is
// a Z after the kick.  The true state is i^ph X^x Z^z (the computed state);
// a kick M = i^k' Z^n X^a G(g) on site q is run as G(+-g) (G past the frame:
// RX flips g and the sign on Z_q; RY on X_q xor Z_q), and the frame takes
// Z^n X^a.  X bits are flushed by the re-layouts (the LDS write slot of tile
// index y becomes slot(y ^ m): the tile comes out X^m-permuted), Z bits by the
// diagonal (a sign per amplitude, folded into its tables): masks chosen so the
// frame is the identity at the diagonal and at the store, the X of a kick that
// has no re-layout after it taken before it (pre-flushed; RX commutes it, RY
// flips g).  Kick order of the kernel: pre 4..8 | x1 | 0..3 | x2 | 9..12 | D
// | post 9..12 | x3 | 0..3 | x4 | 8, 4..7.  Writes f (d[0]) and variant 2 into
// the kick records, the masks into tot (kT13Mask*); returns the extra power of
// i.  The algebra is restated in numpy and checked against the direct 2x2
// products by tests/test_frame13_model.py.
__device__ int frame13_records(const PassKick& pk, KickRec* out, const int* fvar, KickRec& tot) {
  constexpr int NB = kMaxTileBits;
  const bool rx = pk.kind == kKindRX;
  int x = 0, z = 0, ph = 0;
  auto form_a = [&](int i) { return (fvar[i] >> 1) ^ 1; };
  auto zbit = [&](int i) { return rx ? (fvar[i] & 1) : ((fvar[i] & 1) ^ form_a(i)); };
  auto kick = [&](int h, int q) {
    const int i = h * NB + q;
    const int fa = form_a(i), n2 = zbit(i);
    const double g = fa ? -out[i].d[0] : out[i].d[0];
    const int flip = ((rx ? z : (x ^ z)) >> q) & 1;
    out[i].d[0] = flip ? -g : g;
    out[i].i[1] = 2;
    ph += (rx ? 3 * fa : 2 * fa) + 2 * flip;
    x ^= fa << q;
    ph += 2 * (n2 & (x >> q) & 1);
    z ^= n2 << q;
  };
  auto flush_x = [&](int m) {
    ph += 2 * (__popc(z & m) & 1);
    x ^= m;
    return m;
  };
  const bool pre = pk.pre.enabled, post = pk.post.enabled;
  auto xbits = [&](int h, int q0, int q1) {
    int m = 0;
    for (int q = q0; q <= q1; ++q) m |= form_a(h * NB + q) << q;
    return m;
  };
  int m1 = 0, m2 = 0, m3 = 0, m4 = 0;
  if (pre) {
    for (int q = 4; q <= 8; ++q) kick(0, q);
    m1 = flush_x(x);
    for (int q = 0; q <= 3; ++q) kick(0, q);
    m2 = flush_x(x ^ xbits(0, 9, 12));
    for (int q = 9; q <= 12; ++q) kick(0, q);
  }
  int npost = 0;
  if (post)
    for (int q = 0; q < NB; ++q) npost |= zbit(NB + q) << q;
  const int md = z ^ npost;
  z ^= md;
  if (post) {
    for (int q = 9; q <= 12; ++q) kick(1, q);
    m3 = flush_x(x);
    for (int q = 0; q <= 3; ++q) kick(1, q);
    m4 = flush_x(x ^ xbits(1, 4, 8));
    kick(1, 8);
    for (int q = 4; q <= 7; ++q) kick(1, q);
  }
  // cumulative: the X flushed by re-layouts 1 .. e (the kernel's xch)
  tot.i[kT13MaskX1] = m1;
  tot.i[kT13MaskX2] = m1 ^ m2;
  tot.i[kT13MaskX3] = m1 ^ m2 ^ m3;
  tot.i[kT13MaskX4] = m1 ^ m2 ^ m3 ^ m4;
  tot.i[kT13MaskZ] = md;
  return ph;
}

// The same Pauli-frame records for the 12-bit K-D-K passes of the unitary
// families (pass_body FR: nibble sets 6 and 7, the standard geometry).  Their
// program (RoundPlan): pre-kick nibbles IO -> 0 -> O with a re-layout before
// each but the first, the diagonal, post-kick nibbles O -> 0 -> IO, re-layouts
// skipped where a layout does not change.  A kick's X is flushed by the first
// re-layout after it within its half, else (the half's last nibble) by the
// last one before it; the diagonal flushes Z as in frame13_records (for a
// pass without one, the global factor's multiply; for a dual pass's echo
// branch, copied before the diagonal, its own sign flush).  The coefficients
// go to d[kFrameCoef], the masks and the extra power of i to tot (kT12*).
__device__ void frame12_records(const PassKick& pk, KickRec* out, const int* fvar, KickRec& tot) {
  constexpr int NT = kTileBits;
  const bool rx = pk.kind == kKindRX;
  int nibs = 0;
  for (int n = 0; n < 3; ++n)
    if (pk.act & (0xF << (4 * n))) nibs |= 1 << n;
  const bool pre = pk.pre.enabled, post = pk.post.enabled;
  const int IO = io_layout(nibs), O = 3 - IO;
  const bool n0 = nibs & 1, nIO = (nibs >> IO) & 1, nO = (nibs >> O) & 1;
  const int d_lay = pre ? (nO ? O : (n0 ? 0 : IO)) : IO;
  const int pO = nO ? O : d_lay, p0 = n0 ? 0 : pO, pIO = nIO ? IO : p0;
  // the program: nibble kicks (h * 4 + nibble), re-layouts (-1), the diagonal (-2)
  int ev[12], ne = 0;
  if (pre) {
    if (nIO) ev[ne++] = IO;
    if (n0) { ev[ne++] = -1; ev[ne++] = 0; }
    if (nO) { ev[ne++] = -1; ev[ne++] = O; }
  }
  ev[ne++] = -2;
  if (post) {
    if (nO) { if (d_lay != O) ev[ne++] = -1; ev[ne++] = 4 + O; }
    if (n0) { if (pO != 0) ev[ne++] = -1; ev[ne++] = 4 + 0; }
    if (nIO) { if (p0 != IO) ev[ne++] = -1; ev[ne++] = 4 + IO; }
    if (pIO != IO) ev[ne++] = -1;
  } else if (d_lay != IO) {
    ev[ne++] = -1;
  }
  auto form_a = [&](int i) { return (fvar[i] >> 1) ^ 1; };
  auto zbit = [&](int i) { return rx ? (fvar[i] & 1) : ((fvar[i] & 1) ^ form_a(i)); };
  // each kicked nibble's flush: the re-layout it is assigned to, on the read
  // side when the re-layout follows the kick (the sites are register bits of
  // its source layout, thread bits of its target: mr), on the write side when
  // it precedes it (register bits of the target, thread bits of the source:
  // mw) -- either way the mask stays off the side's register offsets
  int mw[4] = {0, 0, 0, 0}, mr[4] = {0, 0, 0, 0};
  {
    int xi = 0;  // re-layouts seen so far
    for (int e = 0; e < ne; ++e) {
      if (ev[e] == -1) ++xi;
      if (ev[e] < 0) continue;
      const int h = ev[e] >> 2, nib = ev[e] & 3;
      // the first re-layout after it within its half, else the last before it
      int after = -1, k = xi;
      for (int f = e + 1; f < ne && ev[f] != -2; ++f)
        if (ev[f] == -1) { after = k; break; }
      int m = 0;
      for (int q = 0; q < 4; ++q) m |= form_a(h * NT + 4 * nib + q) << (4 * nib + q);
      if (after >= 0 && after < 4) mr[after] |= m;
      else if (after < 0 && xi >= 1 && xi <= 4) mw[xi - 1] |= m;
    }
  }
  int npost = 0;
  if (post)
    for (int k = 0; k < NT; ++k)
      if ((nibs >> (k >> 2)) & 1) npost |= zbit(NT + k) << k;
  int x = 0, z = 0, ph = 0, xi = 0, md = 0;
  for (int e = 0; e < ne; ++e) {
    if (ev[e] == -1) {
      const int m = xi < 4 ? mw[xi] ^ mr[xi] : 0;
      ph += 2 * (__popc(z & m) & 1);
      x ^= m;
      ++xi;
    } else if (ev[e] == -2) {
      md = z ^ npost;
      z ^= md;
    } else {
      const int h = ev[e] >> 2, nib = ev[e] & 3;
      for (int q = 0; q < 4; ++q) {
        const int k = 4 * nib + q, i = h * NT + k;
        const int fa = form_a(i), n2 = zbit(i);
        const double g = fa ? -out[i].d[0] : out[i].d[0];
        const int flip = ((rx ? z : (x ^ z)) >> k) & 1;
        out[i].d[kFrameCoef] = flip ? -g : g;
        ph += (rx ? 3 * fa : 2 * fa) + 2 * flip;
        x ^= fa << k;
        ph += 2 * (n2 & (x >> k) & 1);
        z ^= n2 << k;
      }
    }
  }
  for (int e = 0; e < 4; ++e) tot.i[kT12MaskX0 + e] = mw[e] | (mr[e] << 16);
  tot.i[kT12MaskZ] = md | ((ph & 3) << kT12PhShift);
}

// Kick records (dtc_kernels.h: KickRec) of n_pass passes x batch states: one
// thread per (pass, state) builds the 24 noisy site kicks of the pass, writes
// their factored forms and the product of their global factors.
__global__ __launch_bounds__(256) void prep_kernel(PrepArgs P) {
  const int64_t id = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (id >= (int64_t)P.n_pass * P.batch) return;
  const int pass = (int)(id / P.batch);
  const int b = (int)(id % P.batch);
  const PassKick pk = P.passes ? P.passes[pass] : P.one;
  const int64_t gstate = P.batch_start + b;
  const uint64_t traj = (uint64_t)(P.traj_offset + (gstate % P.n_traj));
  KickRec* out = P.out + id * kRecPerState;
  if (pk.lc_layers > 0 && pk.lc_wide == 2) {
    // 12-site light-cone pass (dtc_kernels.h, kLcw3*): the Pauli frame over
    // all twelve tile bits, seven layers, mask bit 12 l + k in lc_mask /
    // lc_mask2; the X masks in global bit positions
    double* od = (double*)out;
    long long* oi = (long long*)out;
    int fz = 0, fx = 0;  // per tile bit
    double g2 = 1.0;
    for (int l = 0; l < kLcw3Layers; ++l) {
      for (int k = 0; k < kTileBits; ++k) {
        const int bit = 12 * l + k;
        const bool on = bit < 64 ? ((pk.lc_mask >> bit) & 1ull) : ((pk.lc_mask2 >> (bit - 64)) & 1ull);
        double fh = 0.0;
        if (l < pk.lc_layers && on) {
          const int lsite = pk.lc_gb[k];
          double2 m[4] = {make_double2(1.0, 0.0), make_double2(0.0, 0.0),
                          make_double2(0.0, 0.0), make_double2(1.0, 0.0)};
          if (lsite < P.L_real)
            build_site_kick(P, pk.lc[l], P.site_of ? P.site_of[lsite] : lsite, traj, m);
          SiteMat sm;
          canonicalise(pk.kind, m, sm);
          const int form_b = sm.var >> 1, neg = sm.var & 1;
          const double ft = form_b ? -sm.coef : sm.coef;
          const int flip = ((pk.kind == kKindRX ? fz : (fz ^ fx)) >> k) & 1;
          fh = flip ? -ft : ft;
          fz ^= (pk.kind == kKindRX ? neg : (neg ^ form_b)) << k;
          fx ^= form_b << k;
          g2 *= sm.scale * sm.scale;
        }
        od[12 * l + k] = fh;
      }
      long long mg = 0;
      for (int k = 0; k < kTileBits; ++k)
        if ((fx >> k) & 1) mg |= 1ll << pk.lc_gb[k];
      oi[kLcw3Mask + l] = mg;
    }
    od[kLcw3G2] = g2;
    return;
  }
  if (pk.lc_layers > 0 && pk.lc_wide) {
    // 10-site light-cone pass: the same Pauli frame over tile bits 2 .. 11
    // (dtc_kernels.h, kLcw*); the X masks in global bit positions
    double* od = (double*)out;
    long long* oi = (long long*)out;
    int fz = 0, fx = 0;  // per tile bit
    double g2 = 1.0;
    for (int l = 0; l < kLcwLayers; ++l) {
      for (int k = 0; k < kTileBits; ++k) {
        double fh = 0.0;
        if (k >= 2 && l < pk.lc_layers && ((pk.lc_mask >> (10 * l + k - 2)) & 1ull)) {
          const int lsite = pk.lc_gb[k];
          double2 m[4] = {make_double2(1.0, 0.0), make_double2(0.0, 0.0),
                          make_double2(0.0, 0.0), make_double2(1.0, 0.0)};
          if (lsite < P.L_real)
            build_site_kick(P, pk.lc[l], P.site_of ? P.site_of[lsite] : lsite, traj, m);
          SiteMat sm;
          canonicalise(pk.kind, m, sm);
          const int form_b = sm.var >> 1, neg = sm.var & 1;
          const double ft = form_b ? -sm.coef : sm.coef;
          const int flip = ((pk.kind == kKindRX ? fz : (fz ^ fx)) >> k) & 1;
          fh = flip ? -ft : ft;
          fz ^= (pk.kind == kKindRX ? neg : (neg ^ form_b)) << k;
          fx ^= form_b << k;
          g2 *= sm.scale * sm.scale;
        }
        od[12 * l + k] = fh;
      }
      long long mg = 0;
      for (int k = 2; k < kTileBits; ++k)
        if ((fx >> k) & 1) mg |= 1ll << pk.lc_gb[k];
      oi[kLcwMask + l] = mg;
    }
    od[kLcwG2] = g2;
    return;
  }
  if (pk.lc_layers > 0) {
    // light-cone pass: Pauli-frame records (dtc_kernels.h, kLcCoefs ..)
    double* od = (double*)out;
    long long* oi = (long long*)out;
    int fz = 0, fx = 0;  // the frame's Z / X exponents per window site
    double g2 = 1.0;
    long long packed = 0;
    for (int l = 0; l < pk.lc_layers; ++l) {
      for (int b = 0; b < kLcSites; ++b) {
        double fh = 0.0;
        if ((pk.lc_mask >> (kLcSites * l + b)) & 1ull) {
          const int lsite = pk.s + b;  // tile bit 4 + b >= c = 4
          double2 m[4] = {make_double2(1.0, 0.0), make_double2(0.0, 0.0),
                          make_double2(0.0, 0.0), make_double2(1.0, 0.0)};
          if (lsite < P.L_real)
            build_site_kick(P, pk.lc[l], P.site_of ? P.site_of[lsite] : lsite, traj, m);
          SiteMat sm;
          canonicalise(pk.kind, m, sm);
          // form A: i^k w Z^s A(beta); form B: S_B(alpha) = i X A(-alpha) (RX),
          // R_B(alpha) = Z X R_A(-alpha) (RY)
          const int form_b = sm.var >> 1, neg = sm.var & 1;
          const double ft = form_b ? -sm.coef : sm.coef;
          // the frame so far, moved past A(ft): Z flips f (RX); Z or X, not both (RY)
          const int flip = ((pk.kind == kKindRX ? fz : (fz ^ fx)) >> b) & 1;
          fh = flip ? -ft : ft;
          fz ^= (pk.kind == kKindRX ? neg : (neg ^ form_b)) << b;
          fx ^= form_b << b;
          g2 *= sm.scale * sm.scale;
        }
        od[kLcSites * l + b] = fh;
      }
      if (l < 4) packed |= (long long)(fx & 0xFF) << (8 * l);
    }
    packed |= (long long)(fx & 0xFF) << 32;
    od[kLcG2] = g2;
    oi[kLcPacked] = packed;
    return;
  }
  int ksum = 0;
  double w[2] = {1.0, 1.0};
  const int tb = pk.tb == kMaxTileBits ? kMaxTileBits : kTileBits;
  const bool frame13 = tb == kMaxTileBits && (pk.kind == kKindRX || pk.kind == kKindRY);
  // (the 12-bit passes' frame records, pass_body FR: nibble sets 6 and 7 of
  // the standard geometry -- not the 13 / 7 split's 7-site column group)
  const bool frame12 = tb == kTileBits && (pk.kind == kKindRX || pk.kind == kKindRY) &&
                       (pk.act & 0xF0) && (pk.act & 0xF00) && !(pk.c == kB7Cols && pk.act == 0xFE0);
  int fvar[2 * kMaxTileBits];
  for (int half = 0; half < 2; ++half) {
    const KickDesc& K = half == 0 ? pk.pre : pk.post;
    for (int k = 0; k < tb; ++k) {
      const int lsite = k < pk.c ? k : pk.s + k - pk.c;
      double2 m[4] = {make_double2(1.0, 0.0), make_double2(0.0, 0.0), make_double2(0.0, 0.0),
                      make_double2(1.0, 0.0)};
      if (K.enabled && (pk.act & ~(int)K.skip & (1 << k)) && lsite < P.L_real) {
        const int site = P.site_of ? P.site_of[lsite] : lsite;
        build_site_kick(P, K, site, traj, m);
      }

      SiteMat sm;
      canonicalise(pk.kind, m, sm);
      KickRec r;
      if (pk.kind == kKindGen) {
        for (int e = 0; e < 4; ++e) {
          r.d[2 * e] = sm.m[e].x;
          r.d[2 * e + 1] = sm.m[e].y;
        }
      } else if (pk.kind == kKindRXU || pk.kind == kKindRYU) {
        r.d[0] = sm.coef;
        r.i[1] = sm.var;
        r.d[2] = sm.scale * sm.scale;
        r.d[3] = sm.rho0;
        r.d[4] = sm.rho1;
        for (int e = 5; e < 8; ++e) r.d[e] = 0.0;
      } else {
        r.d[0] = sm.coef;
        r.i[1] = sm.var;
        r.d[2] = sm.scale * sm.scale;
        for (int e = 3; e < 8; ++e) r.d[e] = 0.0;
      }
      out[half * tb + k] = r;
      if (frame13 || frame12) fvar[half * tb + k] = sm.var;
      ksum += sm.k;
      w[half] *= sm.scale;
    }
  }
  KickRec tot;
  for (int e = 0; e < 8; ++e) tot.d[e] = 0.0;
  if (frame13) ksum += frame13_records(pk, out, fvar, tot);
  if (frame12) frame12_records(pk, out, fvar, tot);
  const int kph = ksum & 3;
  const double wg = w[0] * w[1];
  tot.d[0] = kph == 0 ? wg : (kph == 2 ? -wg : 0.0);
  tot.d[1] = kph == 1 ? wg : (kph == 3 ? -wg : 0.0);
  tot.d[2] = 1.0 / (w[1] * w[1]);
  out[2 * tb] = tot;
}

hipError_t launch_prep(const PrepArgs& a, hipStream_t stream) {
  if (!a.passes && a.n_pass != 1) return hipErrorInvalidValue;
  const int64_t n = (int64_t)a.n_pass * a.batch;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(prep_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, a);
  return hipGetLastError();
}

// Compile-time round plan.  NIBS = register nibbles holding active sites
// (bit n = nibble n).  IO = the load/store layout (io_layout), O = 3 - IO the
// other high nibble.
// Pre-kick rounds IO -> 0 -> O, diagonal + measurement where the pre-kick
// ends, post-kick rounds O -> 0 -> IO, store from layout IO.
template <int NIBS, int SHAPE>
struct RoundPlan {
  static constexpr int IO = io_layout(NIBS);
  static constexpr int O = 3 - IO;
  static constexpr bool n0 = NIBS & 1, nIO = (NIBS >> IO) & 1, nO = (NIBS >> O) & 1;
  static constexpr bool pre = SHAPE == kShapeK || SHAPE == kShapeKD || SHAPE == kShapeKDK;
  static constexpr bool diag =
      SHAPE == kShapeKD || SHAPE == kShapeDK || SHAPE == kShapeKDK || SHAPE == kShapeD;
  static constexpr bool post = SHAPE == kShapeDK || SHAPE == kShapeKDK;
  static constexpr int d_lay = pre ? (nO ? O : (n0 ? 0 : IO)) : IO;
  // layouts reached by the post rounds
  static constexpr int pO = nO ? O : d_lay;
  static constexpr int p0 = n0 ? 0 : pO;
  static constexpr int pIO = nIO ? IO : p0;
  // Pauli-frame passes: the real re-layouts in program order (their X-flush
  // masks; frame12_records walks the same sequence): pre IO -> 0 (xA), pre ->
  // O (xB); post d_lay -> O (x1), -> 0 (x2), -> IO (x3), -> IO (x4); without
  // a post-kick d_lay -> IO (x5)
  static constexpr int xA = 0;
  static constexpr int xB = (pre && n0) ? 1 : 0;
  static constexpr int npre = (pre && n0 ? 1 : 0) + (pre && nO ? 1 : 0);
  static constexpr bool r1 = post && nO && d_lay != O;
  static constexpr bool r2 = post && n0 && pO != 0;
  static constexpr bool r3 = post && nIO && p0 != IO;
  static constexpr int x1 = npre, x2 = x1 + (r1 ? 1 : 0), x3 = x2 + (r2 ? 1 : 0),
                       x4 = x3 + (r3 ? 1 : 0), x5 = npre;
};

// Development-only phase timing (build with -DDTC_PHASE_TIMING): wave 0 of
// every workgroup records s_memtime at phase boundaries into A.dbg_ts.
#ifdef DTC_PHASE_TIMING
#define DTC_TS(i) (ts[i] = __builtin_amdgcn_s_memtime())
#else
#define DTC_TS(i) ((void)0)
#endif

// MC, the measurements compiled in (separate instantiations, so a pass
// carries only the code it can run): 0 = none, 1 = the probe, 2 = any mode
// (per-site / energy Z), 3 = energy with the in-flight <X> points.
// SPLIT: re-layouts through a 32 KiB half-tile buffer (exchange_split), so a
// third workgroup fits a CU (dtc_kdk_pass3; development A/B, PassArgs::kdk_split)
// DUAL (a forward K-D-K that also starts an echo branch, dtc_kdk_dual): after
// the pre-kick the tile is copied; the copy takes the echo chain's first kick
// layer (A.recs2's post-kick, its global factor A.recs2's total) and is stored
// to A.dst2, then the pass goes on (diagonal, probe, post-kick, store to dst).
// GEO: tile geometry.  kGeoStd: the plan's groups (column bits at a nibble
// boundary, the diagonal's register nibble inside or outside them).  kGeoB7
// (round 6, the 13 / 7 split of L = 20, dtc_tile13.hip): the 7-site column
// group, tile bits 0..4 = global 0..4 (512-B runs), 5..11 = sites 13..19 --
// register nibble 1 holds column bit 4 (no kick: QM 14) and sites 13..15, so
// its diagonal is two window tables (start bits 4 and 13), see diag_in.
template <int SHAPE, int NIBS, int KIND, int MC = 0, bool NS = false, bool SPLIT = false,
          bool DUAL = false, int GEO = kGeoStd>
__device__ __forceinline__ void pass_body(const PassArgs& A) {
  using RP = RoundPlan<NIBS, SHAPE>;
  static_assert(GEO == kGeoStd || (NIBS == 6 && (KIND == kKindRX || KIND == kKindRY) && MC <= 1),
                "the 7-site column geometry: factored unitary kicks, the probe at most");
  // register bits of nibble N that hold sites
  constexpr auto qm = [](int N) { return (GEO == kGeoB7 && N == 1) ? 14 : 15; };
  constexpr bool kSplitDiag = GEO == kGeoB7 && RP::d_lay == 1;
  static_assert(!DUAL || (MC <= 1 && !NS &&
                          ((SHAPE == kShapeKDK &&
                            (KIND == kKindRX || KIND == kKindRY || KIND == kKindGen ||
                             KIND == kKindRXU || KIND == kKindRYU)) ||
                           (SHAPE == kShapeKD &&
                            (KIND == kKindRXU || KIND == kKindRYU || KIND == kKindGen)))),
                "dual passes: K-D-K or device-noise K-D, at most the probe");
  constexpr int kNt = NIBS == 7 ? DTC_NT_A : DTC_NT_B;
#ifdef DTC_PHASE_TIMING
  uint64_t ts[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const uint64_t rt_start = __builtin_amdgcn_s_memrealtime();
#endif
  DTC_TS(0);
  __shared__ double2 s_tile[SPLIT ? 1 : kTile];
  __shared__ double s_half[SPLIT ? kHalfSlots : 1];
  // the co-traversed dual pass's second half-tile buffer (the echo's tile)
  __shared__ double s_half2[(DUAL && SHAPE == kShapeKDK) ? kHalfSlots : 1];
  __shared__ double2 s_chunk[RP::diag ? kMaxChunks * 64 : 1];
  __shared__ double2 s_win[RP::diag ? 64 : 1];
  __shared__ double2 s_win2[kSplitDiag ? 64 : 1];  // kGeoB7: the window of start bit s
  __shared__ double s_red[kThreads / 64][kRedSlots];
  // three-per-CU energy passes: per wave, X point (post, pre), nibble, the
  // eight lane partials of the nibble's four sites (x_now)
  __shared__ double s_xpart[(SPLIT && MC == 3) ? kThreads / 64 : 1][2][3][32];
  // device-like noise: the deferred Kraus diagonals' nibble tables (record set
  // R / R2, pre / post layer, nibble, its 16 bit patterns): prod over the
  // nibble's four sites of rho_{k, x_k}, staged once per workgroup (rho_apply)
  constexpr bool kRho = KIND == kKindRXU || KIND == kKindRYU;
  constexpr int kRhoSets = DUAL ? 2 : 1;
  __shared__ double s_rho[kRho ? kRhoSets * 96 : 1];

  const int t = threadIdx.x;
  const int c = A.c, s = A.s;
  const int tile_bits = A.L_eff - kTileBits;
  const int64_t n_tiles = (int64_t)1 << tile_bits;
  // block -> (state, tile): octet layout: the eight states of an octet on
  // consecutive blocks (dtc_kernels.h state_base); the padding states of a
  // last partial octet leave at once (the whole workgroup)
  const int og = A.octet_bits;
  const int64_t b = og ? (((int64_t)blockIdx.y << 3) | (blockIdx.x & 7)) : (int64_t)blockIdx.y;
  // contiguous states (large L, C4 / C5): blocks go round-robin over the 8
  // XCDs, so XCD x takes the x-th eighth of the tiles, consecutive ones on one
  // XCD (r5q: the top 8-site group's pass at L=28, rows 16 MiB apart)
  const int64_t tile = og ? (int64_t)(blockIdx.x >> 3)
                          : ((gridDim.x & 7) ? (int64_t)blockIdx.x
                                             : (int64_t)(blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3));
  if (og && b >= A.batch) return;
  const int inst = (int)((A.batch_start + b) / A.n_traj);
  // this state's kick records (prep kernel): lane-distributed in VGPRs
  // (RecRegs), loaded with the setup; the energy passes (MC 3) read them
  // through the scalar data cache instead (RecScalar: the 24 X pair sums
  // leave no VGPRs for them at three workgroups per CU -- r5f: their spill
  // gone, pass3<7,0,3> 7.04 -> 6.90 ms; in the other passes the scalar loads
  // sit on the tile's chain, kdk3<7,0,0> 5.34 -> 6.11 ms)
  constexpr bool kScalarRec = MC == 3;
  auto load_recs = [&](const KickRec* rec) {
    if constexpr (kScalarRec) {
      return RecScalar(rec);
    } else {
      RecRegs r;
      const int lane = t & 63;
      const double2* rp = (const double2*)rec + 2 * lane;
      double2 r0 = make_double2(0.0, 0.0), r1 = make_double2(0.0, 0.0);
      if (4 * lane < 8 * kRecPerState) {
        r0 = rp[0];
        r1 = rp[1];
      }
      r.rv[0] = r0.x; r.rv[1] = r0.y; r.rv[2] = r1.x; r.rv[3] = r1.y;
      return r;
    }
  };
  const auto R = load_recs(A.recs + b * kRecPerState);
  // DUAL: the echo branch's records (its post-kick and total)
  const auto R2 = load_recs(DUAL ? A.recs2 + b * kRecPerState : A.recs + b * kRecPerState);

  const int64_t mid_mask = ((int64_t)1 << A.tile_bits_mid) - 1;
  TileMap M;
  M.c = c;
  M.s = s;
  M.cmask = (1 << c) - 1;
  M.tbase = ((tile & mid_mask) << c) | ((tile >> A.tile_bits_mid) << (s + kTileBits - c));

  // ---- diagonal tables of the state's instance: loads issued before the
  // tile's (vector memory returns in order), staged to LDS below ----
  constexpr int kChunkPerThread = (kMaxChunks * 64 + kThreads - 1) / kThreads;
  double2 dchunk[kChunkPerThread];
  double2 dwin = make_double2(1.0, 0.0), dwin2 = make_double2(1.0, 0.0);
  int g0 = -1;
  if (RP::diag) {
    const int tb = 4 * RP::d_lay;
    // (kGeoB7, nibble 1: the window of start bit 4 = the column bit c - 1, and
    // of start bit s below)
    g0 = kSplitDiag ? c - 1 : (tb >= c ? s + tb - c : (tb + 4 <= c ? tb : -1));
    const double2* dt = A.diag + (int64_t)inst * A.diag_stride;
#pragma unroll
    for (int j = 0; j < kChunkPerThread; ++j) {
      const int i = t + j * kThreads;
      if (i < A.n_chunks * 64) dchunk[j] = dt[i];
    }
    if (g0 >= 0 && t < 64) dwin = dt[(A.n_chunks + g0) * 64 + t];
    if (kSplitDiag && t < 64) dwin2 = dt[(A.n_chunks + s) * 64 + t];
  }

  // ---- the tile (coalesced 16-B loads: uniform 64-bit base + one per-lane
  // byte offset shared by all 16 accesses).  The offset is 32-bit whenever it
  // fits: always for layout 2 (thread bits = tile bits 0..7, L_eff <= 32),
  // for layout 1 (thread bits include tile bits 8..11) while tile bit 11's
  // global bit is <= 27 (the low group at any L; higher groups to L_eff 28) ----
  const int64_t vofs64 = octet_spread(M.rel(ybase<RP::IO>(t)), og) << 4;
  const uint32_t vofs = (uint32_t)vofs64;
  // the lane offset fits 32 bits while the highest lane bit's address bit is
  // <= 27 (amplitudes): tile bit 7 (layout 2) or 11 (layout 1)
  constexpr int kTopLaneBit = RP::IO == 2 ? 7 : 11;
  const int top_g = kTopLaneBit < c ? kTopLaneBit : s + kTopLaneBit - c;
  const bool ofs32 = top_g + ((og && top_g >= og) ? 3 : 0) <= 27;
  auto tile_ofs = [&](int r) -> int64_t {
    return octet_spread(M.tbase | M.rel(r << (4 * RP::IO)), og) << 4;
  };
  const int64_t sbase = state_base(b, A.state_len, og);
  double2 v[kRegs];
  bool synth = false;
  if constexpr (SHAPE == kShapeK) synth = A.basis != nullptr;
  if (synth) {
    // the first pass of a sweep: the source is the basis state |basis[b]>,
    // formed in registers (no zero-fill of the batch, no read of it)
    const int64_t m = A.basis[b];
    const int64_t x0 = M.tbase | M.rel(ybase<RP::IO>(t));
#pragma unroll
    for (int r = 0; r < kRegs; ++r)
      v[r] = make_double2((x0 | M.rel(r << (4 * RP::IO))) == m ? 1.0 : 0.0, 0.0);
  } else {
    const char* src = (const char*)(A.src + sbase);
    if (ofs32) {
#pragma unroll
      for (int r = 0; r < kRegs; ++r) {
        const char* a = src + tile_ofs(r) + vofs;
        if constexpr (kNt & 1) {
          const d2v w = __builtin_nontemporal_load((const d2v*)a);
          v[r] = make_double2(w.x, w.y);
        } else {
          v[r] = *(const double2*)a;
        }
      }
    } else {
#pragma unroll
      for (int r = 0; r < kRegs; ++r) {
        const char* a = src + tile_ofs(r) + vofs64;
        if constexpr (kNt & 1) {
          const d2v w = __builtin_nontemporal_load((const d2v*)a);
          v[r] = make_double2(w.x, w.y);
        } else {
          v[r] = *(const double2*)a;
        }
      }
    }
  }
  DTC_TS(1);
  // vmcnt(16) (gfx9 encoding: vmcnt[3:0] | vmcnt[5:4] << 14, expcnt/lgkmcnt
  // unmasked): the record and table loads have landed, the tile's 16 are in
  // flight.  Explicit, so no use of them waits for the tile.
  static_assert(kRegs == 16, "vmcnt immediate assumes 16 tile loads");
  __builtin_amdgcn_s_waitcnt(0x4F70);
  if constexpr (kRho) {
    // entry e = ((set * 2 + layer) * 3 + nibble) * 16 + pattern, one per thread
    // (a nibble without kicks: 1); made visible by the first exchange's barrier
    // or by the diagonal's (below), before the first rho_apply
    if (t < kRhoSets * 96) {
      const int set = t / 96, layer = (t / 48) & 1, nib = (t >> 4) % 3, pat = t & 15;
      double pr = 1.0;
      if ((NIBS >> nib) & 1) {
        const double* rd =
            (const double*)((set ? A.recs2 : A.recs) + b * kRecPerState) + 8 * (layer * kTileBits + 4 * nib);
#pragma unroll
        for (int q = 0; q < 4; ++q) pr *= rd[8 * q + (((pat >> q) & 1) ? 4 : 3)];
      }
      s_rho[t] = pr;
    }
    if constexpr (!RP::diag && !(RP::pre && (RP::n0 || RP::nO))) __syncthreads();
  }
  // Pauli-frame kicks (frame12_records): the unitary families' passes over
  // nibble sets 6 and 7 that measure no X in flight run one butterfly per
  // kick; the frame's X bits leave through the re-layouts' write slots
  // (fxm: mask of re-layout e in program order, RoundPlan::x*), its Z bits
  // through the diagonal (fzm: a sign per amplitude, in the window table and
  // the thread's phase) and its extra power of i through the global factor
#ifdef DTC_ADD_SLOTS
  constexpr bool FR = false;  // (the additive slots are not linear over XOR)
#else
  // (the 8-site column group's plain passes keep the variant branches: with
  // frames their full-tile re-layouts take the flush barriers and ran 1-2 %
  // slower, r6v / r6w; its dual passes, the 12-site group's and every final
  // pass gain -- dual<7> 9.60 -> 8.62 ms, kdk_final<7> 6.0 -> 5.3, C2 +1.5 %)
#ifdef DTC_FR_ALL_NIBS  // development A/B: frames for the 8-site group's plain passes too
  constexpr bool FR = (KIND == kKindRX || KIND == kKindRY) && MC != 3 && (NIBS == 6 || NIBS == 7) &&
                      GEO == kGeoStd;
#else
  constexpr bool FR = (KIND == kKindRX || KIND == kKindRY) && MC != 3 &&
                      (NIBS == 7 || (NIBS == 6 && DUAL)) && GEO == kGeoStd;
#endif
#endif
  const int fzw = FR ? R.i(kRecTotal, kT12MaskZ) : 0;
  const int fzm = fzw & (kTile - 1);
  // re-layout e's write-side and read-side masks, and the cumulative ones of
  // re-layouts 0 .. e (the XOR-slot re-layouts, dtc_device.h exchange_split)
  auto fxw = [&](int e) { return (FR && e >= 0) ? (int)(R.i(kRecTotal, kT12MaskX0 + e) & 0xFFFF) : 0; };
  auto fxr = [&](int e) {
    return (FR && e >= 0) ? (int)((R.i(kRecTotal, kT12MaskX0 + e) >> 16) & 0xFFFF) : 0;
  };
  auto fxm = [&](int e) {
    int c = 0;
    for (int k = 0; k <= e; ++k) c ^= fxw(k) ^ fxr(k);
    return c;
  };
  // re-layout e of the forward tile (RoundPlan::x*)
  auto xch_f = [&](auto from_tag, auto to_tag, int e) {
    constexpr int F = decltype(from_tag)::value, T = decltype(to_tag)::value;
    // (the pass's first re-layout has no earlier reads to wait for)
    xch_tile<SPLIT, F, T>(v, s_tile, s_half, t, fxw(e), fxr(e), fxm(e - 1), fxm(e),
                          e > 0 && (fxw(e) | fxr(e - 1)) != 0);
  };
  // i^k g
  auto rot_i = [](double2 g, int k) {
    return k == 0 ? g : (k == 1 ? make_double2(-g.y, g.x) : (k == 2 ? make_double2(-g.x, -g.y)
                                                                     : make_double2(g.y, -g.x)));
  };
  // a Z flush without a diagonal to carry it: amplitude y of layout LAY
  // negated when popcount(y & zm) is odd (sign-bit XORs, no branch)
  auto zflush = [&](auto lay_tag, double2 (&x)[kRegs], int zm) {
    constexpr int LAY = decltype(lay_tag)::value;
    const uint32_t mt = (__popc(ybase<LAY>(t) & zm) & 1) ? 0x80000000u : 0u;
    const int zr = (zm >> (4 * LAY)) & 15;
#pragma unroll
    for (int r = 0; r < kRegs; ++r) {
      const uint64_t m = (uint64_t)(mt ^ ((__popc(r & zr) & 1) ? 0x80000000u : 0u)) << 32;
      x[r].x = __longlong_as_double(__double_as_longlong(x[r].x) ^ m);
      x[r].y = __longlong_as_double(__double_as_longlong(x[r].y) ^ m);
    }
  };
  if (RP::diag) {
    const double cs = A.diag_conj ? -1.0 : 1.0;
#pragma unroll
    for (int j = 0; j < kChunkPerThread; ++j) {
      const int i = t + j * kThreads;
      if (i < A.n_chunks * 64) s_chunk[i] = make_double2(dchunk[j].x, cs * dchunk[j].y);
    }
    // (FR: the window entry of register bits (t >> 1) & 15 of layout d_lay
    // takes their share of the frame's Z flush)
    const double zs = (FR && (__popc((t >> 1) & (fzm >> (4 * RP::d_lay)) & 15) & 1)) ? -1.0 : 1.0;
    if (g0 >= 0 && t < 64) s_win[t] = make_double2(zs * dwin.x, zs * cs * dwin.y);
    if (kSplitDiag && t < 64) s_win2[t] = make_double2(dwin2.x, cs * dwin2.y);
    // made visible by the first exchange's barrier, or by this one
    if constexpr (!(RP::pre && (RP::n0 || RP::nO))) __syncthreads();
  }
  DTC_TS(2);
  // global factor of the factored kicks, i^k * w_pre * w_post, applied with
  // the diagonal (the state's arithmetic does not depend on whether it is
  // measured; a measurement between the diagonal and the post-kick divides
  // its sums by w_post^2)
  const double2 gph = rot_i(make_double2(R.d(kRecTotal, 0), R.d(kRecTotal, 1)),
                            (fzw >> kT12PhShift) & 3);
  const double inv_w2_mid = R.d(kRecTotal, 2);

  auto diag_in = [&](auto lay_tag, bool with_g) {
    constexpr int LAY = decltype(lay_tag)::value;
    const int64_t x0 = M.at(ybase<LAY>(t));
    if constexpr (kSplitDiag && LAY == 1) {
      // kGeoB7: register bit 0 = global bit c - 1 = 4, bits 1..3 = s .. s + 2:
      // no term of D couples them, so D(x) = D(x0) Wa(x) / Wa(x0) Wb(x) / Wb(x0)
      // with Wa, Wb the windows of start bits 4 and s (bits [3, 9), [s - 1,
      // s + 5)); the thread's two values of D(x0) / Wa(x0) / Wb(x0) Wa(x) are
      // formed once, then one lookup and two complex products per amplitude
      const int ia = (int)(((x0 << 1) >> (c - 1)) & 63), ib = (int)(((x0 << 1) >> s) & 63);
      const double2 wa = s_win[ia], wb = s_win2[ib];
      const double2 pc = cmul(cmul(cmul(diag_phase(s_chunk, A.n_chunks, x0), make_double2(wa.x, -wa.y)),
                                   make_double2(wb.x, -wb.y)),
                              with_g ? gph : make_double2(1.0, 0.0));
      const double2 q[2] = {cmul(pc, wa), cmul(pc, s_win[ia | 2])};
#pragma unroll
      for (int r = 0; r < kRegs; ++r) v[r] = cmul(v[r], cmul(q[r & 1], s_win2[ib | ((r >> 1) << 1)]));
      return;
    }
    // D(x) = P_C * W[x], P_C = D(x0) / W[x0] (x the global phase) thread
    // constant, W indexed by bits [g0-1, g0+5) of x: one LDS lookup and two
    // complex products per amplitude (the engine's site groups keep the
    // nibble of layout LAY inside or outside the column bits: g0 >= 0)
    const int w0i = (int)(((x0 << 1) >> g0) & 63);
    const double2 w0 = s_win[w0i];
    const double2 pc0 = cmul(cmul(diag_phase(s_chunk, A.n_chunks, x0), make_double2(w0.x, -w0.y)),
                             with_g ? gph : make_double2(1.0, 0.0));
    // (FR: the thread bits' share of the frame's Z flush)
    const double2 pc = (FR && (__popc(ybase<LAY>(t) & fzm) & 1)) ? make_double2(-pc0.x, -pc0.y) : pc0;
#pragma unroll
    for (int r = 0; r < kRegs; ++r) v[r] = cmul(v[r], cmul(pc, s_win[w0i | (r << 1)]));
  };
  // Observables of the tile: (sum |a|^2, sum z_i |a|^2 for the probe or every
  // site, and in energy mode the bond correlators sum z_i z_i+1 |a|^2).  An
  // index bit of the tile is a register bit of the layout, a thread bit or
  // (outside the tile) one sign over the tile (tbase).  Each thread forms
  // parity vectors over its registers — the total, z of each register bit,
  // z z of adjacent register bits — and a 6-stage Walsh-Hadamard transform
  // over the wave leaves, in lane m, the vector's sum signed by the lane-bit
  // parity m: every observable is one such entry (lane pattern of its thread
  // bits), summed over the 4 waves with the wave-bit signs.
  // MC == 1 (probe passes): measure_in only forms each thread's two sums;
  // the wave reductions, the barrier and the partial write run after the
  // tile's stores are issued (probe_finish), off the pass's critical path
  double pm_tot = 0.0, pm_z = 0.0, pm_inv = 1.0;
  bool pm_on = false;
  int zc_lay = -1;  // MC >= 2: layout of a measurement whose combine is pending
  double zc_inv = 1.0;
  auto measure_in = [&](auto lay_tag, double inv_w2) {
    constexpr int LAY = decltype(lay_tag)::value;
    const int64_t x0 = M.at(ybase<LAY>(t));
    const int wave = t >> 6, lane = t & 63;
    // w[m] = sum_r (-1)^popcount(r & m) |a_r|^2: the total (m = 0), z of each
    // register bit (m = 1 << j) and z z of adjacent register bits (m = 3 << j)
    // by one in-register 16-point Walsh-Hadamard transform (64 adds)
    double w[kRegs];
#pragma unroll
    for (int r = 0; r < kRegs; ++r) w[r] = fma(v[r].x, v[r].x, v[r].y * v[r].y);
#pragma unroll
    for (int b = 0; b < 4; ++b) {
#pragma unroll
      for (int r = 0; r < kRegs; ++r) {
        if (r & (1 << b)) continue;
        const double lo = w[r], hi = w[r | (1 << b)];
        w[r] = lo + hi;
        w[r | (1 << b)] = lo - hi;
      }
    }
    const double ptot = w[0];
    const double zr[4] = {w[1], w[2], w[4], w[8]};
    const bool probe_only = MC <= 1 || A.meas == kMeasProbe;
    const bool energy = MC >= 2 && A.meas == kMeasEnergy;
    auto tile_bit = [&](int site) {
      return site < c ? site : ((site >= s && site < s + kTileBits - c) ? c + site - s : -1);
    };
    if (probe_only) {
      const int site = A.probe;
      const int tb = tile_bit(site);
      double z = 0.0;
      if (tb >= 0) {
        const int j = tb - 4 * LAY;
        if (j >= 0 && j < 4)
          z = j == 0 ? zr[0] : (j == 1 ? zr[1] : (j == 2 ? zr[2] : zr[3]));
        else
          z = ((x0 >> site) & 1) ? -ptot : ptot;
      }
      if constexpr (MC == 1) {
        pm_tot = ptot;
        pm_z = z;
        pm_inv = inv_w2;
        pm_on = true;
        return;
      }
      const double tot = wave_sum(ptot);
      if (lane == 0) s_red[wave][0] = tot;
      if (tb >= 0) {
        z = wave_sum(z);
        if (lane == 0) s_red[wave][1] = z;
      }
    } else if constexpr (MC >= 2) {
      // the total: a full 6-stage transform (every lane pattern a site or a
      // bond on lane bits needs); the register-bit vectors (z of each
      // register bit, z z of adjacent register bits, and the one bond between
      // a register bit and a lane bit, host-chosen: A.zx_reg / A.zx_lane)
      // need only their wave sums: one multi-vector reduction
      double h = ptot;
      h = wht_stage<1>(h);
      h = wht_stage<2>(h);
      h = wht_stage<4>(h);
      h = wht_stage<8>(h);
      h = wht_stage<16>(h);
      h = wht_stage<32>(h);
      const int e = lane_pattern(lane);
      if (e >= 0) s_red[wave][e] = h;
      if (energy) {
        double vec[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) vec[j] = zr[j];
        vec[4] = w[3];
        vec[5] = w[6];
        vec[6] = w[12];
        double zx = 0.0;
        if (A.zx_reg >= 0) {
          const double zj = A.zx_reg == 0 ? zr[0] : (A.zx_reg == 1 ? zr[1] : (A.zx_reg == 2 ? zr[2] : zr[3]));
          zx = ((lane >> A.zx_lane) & 1) ? -zj : zj;
        }
        vec[7] = zx;
        const double r = wave_sum_multi<8>(vec);
        if ((lane & 7) == 0) s_red[wave][kRedLanes + (lane >> 3)] = r;
      } else {
        const double r = wave_sum_multi<4>(zr);
        if ((lane & 15) == 0) s_red[wave][kRedLanes + (lane >> 4)] = r;
      }
    }
    if (probe_only) {
      __syncthreads();
      if (t < 2) {
        double acc = 0.0;
        const int site = A.probe;
        const int ws = (t == 0 || tile_bit(site) >= 0) ? t : 0;
        for (int w = 0; w < kThreads / 64; ++w) acc += s_red[w][ws];
        if (ws != t && ((M.tbase >> site) & 1)) acc = -acc;
        A.partial[(b * n_tiles + tile) * A.n_obs + t] = acc * inv_w2;
      }
    } else {
      // combined after the tile's stores are issued (meas_finish)
      zc_lay = LAY;
      zc_inv = inv_w2;
    }
  };
  // Per-site / energy Z, ZZ partials of the tile from the wave sums in s_red
  // (layout lay of the measurement): one observable per thread t < n_mid.
  auto site_combine = [&](int lay, double inv_w2, int t) {
    const bool energy = MC >= 2 && A.meas == kMeasEnergy;
    const int n_mid = energy ? 2 * A.L_real : 1 + A.L_real;
    if (t >= n_mid) return;
    auto tile_bit = [&](int site) {
      return site < c ? site : ((site >= s && site < s + kTileBits - c) ? c + site - s : -1);
    };
    constexpr int NW = kThreads / 64;
    double acc = 0.0;
    // observable t: 0 norm, 1..L Z_{t-1}, L+1.. Z_i Z_i+1 (i = t-1-L)
    const int i0 = t <= A.L_real ? t - 1 : t - 1 - A.L_real;
    const int ns = t == 0 ? 0 : (t <= A.L_real ? 1 : 2);
    int regs = 0, lanes = 0, waves = 0, neg = 0;
    for (int k = 0; k < ns; ++k) {
      const int site = i0 + k;
      const int tb = tile_bit(site);
      if (tb < 0) {
        neg ^= (int)((M.tbase >> site) & 1);
      } else if (tb >= 4 * lay && tb < 4 * lay + 4) {
        regs |= 1 << (tb - 4 * lay);
      } else {
        const int q = lay == 2 ? tb : (lay == 1 ? (tb < 4 ? tb : tb - 4) : tb - 4);
        if (q < 6) lanes |= 1 << q;
        else waves |= 1 << (q - 6);
      }
    }
    // registers: none -> the total's lane pattern; one bit j -> z_j (and
    // with one lane bit: the host-chosen bond vector); adjacent bits j,
    // j+1 -> zz_j
    const int slot = regs == 0 ? max(0, lane_pattern(lanes))
                     : (__popc(regs) == 1 ? (lanes ? kRedLanes + 7 : kRedLanes + __ffs(regs) - 1)
                                          : kRedLanes + 4 + __ffs(regs) - 1);
    for (int w = 0; w < NW; ++w) acc += (__popc(w & waves) & 1) ? -s_red[w][slot] : s_red[w][slot];
    if (neg) acc = -acc;
    A.partial[(b * n_tiles + tile) * A.n_obs + t] = acc * inv_w2;
  };
  auto probe_finish = [&]() {
    const int wave = t >> 6, lane = t & 63;
    const int site = A.probe;
    const bool zin = site < c || (site >= s && site < s + kTileBits - c);
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
      for (int w = 0; w < kThreads / 64; ++w) acc += s_red[w][ws];
      if (ws != t && ((M.tbase >> site) & 1)) acc = -acc;
      acc *= pm_inv;
      A.partial[(b * n_tiles + tile) * A.n_obs + t] = acc;
    }
  };
  // <X> partials of the 4 sites in register nibble LAY (energy mode): each
  // thread's 2 Re sum conj(a_0) a_1 over its register pairs of bit q; the wave
  // reduction (wave_sum_multi<4>: lanes 0, 16, 32, 48 end with the sums of
  // register bits 0..3) runs after the stores.
  auto pair_sums = [&](auto lay_tag, double (&a)[4], double scale) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      double x = 0.0;
#pragma unroll
      for (int r = 0; r < kRegs; ++r) {
        if (r & (1 << q)) continue;
        const double2 u = v[r], w = v[r | (1 << q)];
        x = fma(u.x, w.x, fma(u.y, w.y, x));
      }
      a[q] = 2.0 * scale * x;
    }
  };
  // X before a pre- or post-kick nibble: each thread's pair sums only; their
  // wave reductions run after the tile's stores are issued (the pre-kick sums
  // stay live across the diagonal: 245 VGPRs, still 2 waves per SIMD)
  // (SPLIT, three workgroups per CU at 168 VGPRs: the 24 deferred sums do not
  // fit, so each X point is reduced into s_red at once; the slots are distinct
  // per point and read after the stores' barrier as in the deferred form)
  double xpost[SPLIT ? 1 : 3][4];
  double xpre[SPLIT ? 1 : 3][4];
  // (three per CU: each X point's four per-thread sums are reduced over lane
  // bits 5, 4 (permlane swaps) and 3 (one DPP row rotation) only, and the
  // eight partials per site left in lanes 0..7 of each 16 go to LDS (s_xpart);
  // x_combine adds them after the stores, off the tile's chain)
  auto x_now = [&](auto lay_tag, double scale, int slot0) {
    constexpr int LAY = decltype(lay_tag)::value;
    // s_xpart has a slot per wave only in the three-per-CU energy pass: any
    // other instantiation reaching here would write past it
    static_assert(SPLIT && MC == 3, "x_now: s_xpart sized for SPLIT && MC == 3 only");
    double a[4];
    pair_sums(lay_tag, a, scale);
    double u0 = a[0], w0 = a[2], u1 = a[1], w1 = a[3];
    swap_rows<32>(u0, w0);
    swap_rows<32>(u1, w1);
    double b0 = u0 + w0, b1 = u1 + w1;
    swap_rows<16>(b0, b1);
    double cc = b0 + b1;
    cc += xor_lane<8>(cc);
    const int lane = t & 63;
    const int pt = slot0 == kSlotXPre ? 1 : 0;
    if (!(lane & 8)) s_xpart[t >> 6][pt][LAY][((lane >> 4) << 3) | (lane & 7)] = cc;
  };
  auto measure_x_post = [&](auto lay_tag, double scale) {
    constexpr int LAY = decltype(lay_tag)::value;
    if constexpr (MC != 3) return;
    else if constexpr (SPLIT) x_now(lay_tag, scale, kSlotXPost);
    else pair_sums(lay_tag, xpost[LAY], scale);
  };
  auto measure_x_pre = [&](auto lay_tag, double scale) {
    constexpr int LAY = decltype(lay_tag)::value;
    if constexpr (MC != 3) return;
    else if constexpr (SPLIT) x_now(lay_tag, scale, kSlotXPre);
    else pair_sums(lay_tag, xpre[LAY], scale);
  };
  // squared share of the global factor carried by the factored kicks of
  // nibble N (records rec0 + 4N .. +3): measuring after them multiplies sums by
  // the inverse, see the scale bookkeeping at the X points below
  auto nib_w2 = [&](int N, int rec0) {
    if (KIND != kKindRX && KIND != kKindRY) return 1.0;
    double w2 = 1.0;
#pragma unroll
    for (int q = 0; q < 4; ++q) w2 *= R.d(rec0 + 4 * N + q, 2);
    return w2;
  };
  const bool x_pre = MC == 3 && (A.meas_parts & kPartXPre);
  const bool x_post = MC == 3 && (A.meas_parts & kPartXPost);
  // device-like noise: a kick layer's deferred Kraus factors (SiteMat),
  // prod over the tile bits k of rho_{k, x_k}, in layout LAY: the lane
  // nibbles' factors from the staged nibble tables (one LDS read each), times
  // the register nibble's 16 (uniform reads); record set 0 = R, 1 = R2
  auto rho_apply = [&](auto lay_tag, int rec0, double2 (&x)[kRegs], int set) {
    constexpr int LAY = decltype(lay_tag)::value;
    const int y = ybase<LAY>(t);
    const double* T = s_rho + (set * 2 + (rec0 ? 1 : 0)) * 48;
    double rt = 1.0;
#pragma unroll
    for (int n = 0; n < 3; ++n)
      if (n != LAY && ((NIBS >> n) & 1)) rt *= T[16 * n + ((y >> (4 * n)) & 15)];
#pragma unroll
    for (int r = 0; r < kRegs; ++r) {
      const double f = ((NIBS >> LAY) & 1) ? rt * T[16 * LAY + r] : rt;
      x[r].x *= f;
      x[r].y *= f;
    }
  };

  // ---- pre-kick rounds: 2 -> 0 -> 1 ----
  // (X before a nibble's pre-kick: the state is exact times the factored
  // kicks already applied, whose squared scale is 1 / prod w^2)
  using L0 = std::integral_constant<int, 0>;
  using LIO = std::integral_constant<int, RP::IO>;
  using LO = std::integral_constant<int, RP::O>;
  if constexpr (RP::pre) {
    double sc = 1.0;
    if constexpr (RP::nIO) {
      if (x_pre) measure_x_pre(LIO{}, sc);
      apply_nibble<RP::IO, KIND, qm(RP::IO), FR>(v, R, 0);
      if (x_pre) sc *= nib_w2(RP::IO, 0);
    }
    if constexpr (RP::n0) {
      xch_f(LIO{}, L0{}, RP::xA);
      if (x_pre) measure_x_pre(L0{}, sc);
      apply_nibble<0, KIND, qm(0), FR>(v, R, 0);
      if (x_pre) sc *= nib_w2(0, 0);
    }
    if constexpr (RP::nO) {
      xch_f(std::integral_constant<int, RP::n0 ? 0 : RP::IO>{}, LO{}, RP::xB);
      if (x_pre) measure_x_pre(LO{}, sc);
      apply_nibble<RP::O, KIND, qm(RP::O), FR>(v, R, 0);
    }
  }
  DTC_TS(3);
  // DUAL, unitary K-D-K: the echo branch's tile w runs its kick layer K'_1
  // beside the forward's post-kick, nibble by nibble in the same order (O ->
  // 0 -> IO), the two tiles re-laid out together through two half-tile
  // buffers (three barriers per re-layout for both) and stored after the
  // forward's tile: the pass makes the post-kick's re-layouts once, not twice.
  // Device-like noise (the forward running one layer ahead, r5: the echo's
  // start is taken before that layer, so it is never undone): both tiles take
  // the pre-kick's deferred Kraus diagonal here, each its own post-kick's
  // before the stores.
  constexpr bool kCo = DUAL && RP::post;
  double2 w[DUAL ? kRegs : 1];
  // the echo branch's frame (its records R2): Z flushed here, where the branch
  // leaves the forward before the diagonal; X masks at the shared re-layouts
  const int fzw2 = (FR && kCo) ? R2.i(kRecTotal, kT12MaskZ) : 0;
  auto fxm2 = [&](int e) {  // cumulative, as fxm
    int c = 0;
    if (FR && kCo)
      for (int k = 0; k <= e; ++k) {
        const int m = (int)R2.i(kRecTotal, kT12MaskX0 + k);
        c ^= (m & 0xFFFF) ^ ((m >> 16) & 0xFFFF);
      }
    return c;
  };
  if constexpr (kCo) {
#pragma unroll
    for (int r = 0; r < kRegs; ++r) w[r] = v[r];
    if constexpr (kRho) rho_apply(std::integral_constant<int, RP::d_lay>{}, 0, w, 0);
    if constexpr (FR) zflush(std::integral_constant<int, RP::d_lay>{}, w, fzw2 & (kTile - 1));
  } else if constexpr (DUAL) {
    // the echo branch: E = K'_1 K_p (input) -- the forward pass's D, its
    // post-kick K_{p+1} and the echo's D^* and undo of K_{p+1} cancel exactly
#pragma unroll
    for (int r = 0; r < kRegs; ++r) w[r] = v[r];
    // (device-like noise, a forward K-D: E = K'_1 D^* D K_p (input) -- the
    // pre-kick's deferred Kraus diagonal first, K'_1's before the store)
    if constexpr (kRho) rho_apply(std::integral_constant<int, RP::d_lay>{}, 0, w, 0);
    if constexpr (RP::nO) {
      xch_tile<SPLIT, RP::d_lay, RP::O>(w, s_tile, s_half, t);
      apply_nibble<RP::O, KIND, qm(RP::O)>(w, R2, kTileBits);
    }
    if constexpr (RP::n0) {
      xch_tile<SPLIT, RP::pO, 0>(w, s_tile, s_half, t);
      apply_nibble<0, KIND, qm(0)>(w, R2, kTileBits);
    }
    if constexpr (RP::nIO) {
      xch_tile<SPLIT, RP::p0, RP::IO>(w, s_tile, s_half, t);
      apply_nibble<RP::IO, KIND, qm(RP::IO)>(w, R2, kTileBits);
    }
    xch_tile<SPLIT, RP::pIO, RP::IO>(w, s_tile, s_half, t);
    if constexpr (kRho) rho_apply(LIO{}, kTileBits, w, 1);
    // the branch's global factor: i^k w of K_p and of K'_1
    const double2 gE = make_double2(R2.d(kRecTotal, 0), R2.d(kRecTotal, 1));
    char* d2 = (char*)(A.dst2 + sbase);
#pragma unroll
    for (int r = 0; r < kRegs; ++r) {
      const double2 u = cmul(w[r], gE);
      d2v x = {u.x, u.y};
      __builtin_nontemporal_store(x, (d2v*)(d2 + tile_ofs(r) + (ofs32 ? (int64_t)vofs : vofs64)));
    }
    // the forward's next re-layout writes slots other threads may still be
    // reading in the branch's last one
    __syncthreads();
  }
  if constexpr (kRho && RP::pre) rho_apply(std::integral_constant<int, RP::d_lay>{}, 0, v, 0);
  if constexpr (!RP::diag) {
    // no diagonal to carry the kicks' global factor (kick-only pass: no
    // post-kick, so applying it here, before any measurement, is exact)
#pragma unroll
    for (int r = 0; r < kRegs; ++r) v[r] = cmul(v[r], gph);
    if constexpr (FR) zflush(std::integral_constant<int, RP::d_lay>{}, v, fzm);
  }
  // ---- diagonal and measurement at d_lay ----
  using DL = std::integral_constant<int, RP::d_lay>;
  if constexpr (RP::diag) diag_in(DL{}, true);
  if constexpr (MC > 0) {
    if (A.meas != kMeasNone && !A.meas_at_end &&
        (A.meas != kMeasEnergy || (A.meas_parts & kPartZ)))
      measure_in(DL{}, inv_w2_mid);  // before the post-kick
  }
  DTC_TS(4);
  // ---- post-kick rounds: 1 -> 0 -> 2 ----
  // (X before a nibble's post-kick: scale 1 / w_post^2 times prod w^2 of the
  // post nibbles already applied)
  if constexpr (kCo) {
    static_assert(SPLIT, "co-traversed dual pass: half-tile re-layouts");
    if constexpr (RP::nO) {
      exchange_split2<RP::d_lay, RP::O>(v, w, s_half, s_half2, t, fxm(RP::x1 - 1), fxm(RP::x1),
                                     fxm2(RP::x1 - 1), fxm2(RP::x1));
      apply_nibble<RP::O, KIND, qm(RP::O), FR>(v, R, kTileBits);
      apply_nibble<RP::O, KIND, qm(RP::O), FR>(w, R2, kTileBits);
    }
    if constexpr (RP::n0) {
      exchange_split2<RP::pO, 0>(v, w, s_half, s_half2, t, fxm(RP::x2 - 1), fxm(RP::x2),
                                     fxm2(RP::x2 - 1), fxm2(RP::x2));
      apply_nibble<0, KIND, qm(0), FR>(v, R, kTileBits);
      apply_nibble<0, KIND, qm(0), FR>(w, R2, kTileBits);
    }
    if constexpr (RP::nIO) {
      exchange_split2<RP::p0, RP::IO>(v, w, s_half, s_half2, t, fxm(RP::x3 - 1), fxm(RP::x3),
                                     fxm2(RP::x3 - 1), fxm2(RP::x3));
      apply_nibble<RP::IO, KIND, qm(RP::IO), FR>(v, R, kTileBits);
      apply_nibble<RP::IO, KIND, qm(RP::IO), FR>(w, R2, kTileBits);
    }
    exchange_split2<RP::pIO, RP::IO>(v, w, s_half, s_half2, t, fxm(RP::x4 - 1), fxm(RP::x4),
                                     fxm2(RP::x4 - 1), fxm2(RP::x4));
    if constexpr (kRho) {
      rho_apply(LIO{}, kTileBits, v, 0);
      rho_apply(LIO{}, kTileBits, w, 1);
    }
  } else if constexpr (RP::post) {
    double sc = inv_w2_mid;
    if constexpr (RP::nO) {
      xch_f(std::integral_constant<int, RP::d_lay>{}, std::integral_constant<int, RP::O>{}, RP::x1);
      if (x_post) measure_x_post(LO{}, sc);
      apply_nibble<RP::O, KIND, qm(RP::O), FR>(v, R, kTileBits);
      if (x_post) sc *= nib_w2(RP::O, kTileBits);
    }
    if constexpr (RP::n0) {
      xch_f(std::integral_constant<int, RP::pO>{}, std::integral_constant<int, 0>{}, RP::x2);
      if (x_post) measure_x_post(L0{}, sc);
      apply_nibble<0, KIND, qm(0), FR>(v, R, kTileBits);
      if (x_post) sc *= nib_w2(0, kTileBits);
    }
    if constexpr (RP::nIO) {
      xch_f(std::integral_constant<int, RP::p0>{}, std::integral_constant<int, RP::IO>{}, RP::x3);
      if (x_post) measure_x_post(LIO{}, sc);
      apply_nibble<RP::IO, KIND, qm(RP::IO), FR>(v, R, kTileBits);
    }
    xch_f(std::integral_constant<int, RP::pIO>{}, std::integral_constant<int, RP::IO>{}, RP::x4);
    if constexpr (kRho) rho_apply(LIO{}, kTileBits, v, 0);
  } else {
    xch_f(std::integral_constant<int, RP::d_lay>{}, std::integral_constant<int, RP::IO>{}, RP::x5);
  }
  if constexpr (MC > 0) {
    if (A.meas != kMeasNone && A.meas_at_end) measure_in(LIO{}, 1.0);
  }
  DTC_TS(5);

  char* dst = (char*)(A.dst + sbase);
  // the stores' lane offset: recomputed from an opaque copy of t in the
  // instantiations that spilled it (three per CU, 168 VGPRs: the device-noise,
  // per-site and 8-site passes kept the load offset alive through the pass,
  // an 8-byte scratch spill per thread, r6f); the others keep the load's
  constexpr bool kRematOfs = SPLIT && (kRho || MC == 2 || NIBS != 7);
  int64_t sofs64 = vofs64;
  if constexpr (kRematOfs) {
    int tt = t;
    asm volatile("" : "+v"(tt));
    sofs64 = octet_spread(M.rel(ybase<RP::IO>(tt)), og) << 4;
  }
  const uint32_t sofs = (uint32_t)sofs64;
  if constexpr (NS) {
    // measurement-only pass (the last of an echo chain): nothing to write
  } else if (ofs32) {
#pragma unroll
    for (int r = 0; r < kRegs; ++r) {
      char* a = dst + tile_ofs(r) + sofs;
      if constexpr (kNt & 2) {
        d2v w = {v[r].x, v[r].y};
        __builtin_nontemporal_store(w, (d2v*)a);
      } else {
        *(double2*)a = v[r];
      }
    }
  } else {
#pragma unroll
    for (int r = 0; r < kRegs; ++r) {
      char* a = dst + tile_ofs(r) + sofs64;
      if constexpr (kNt & 2) {
        d2v w = {v[r].x, v[r].y};
        __builtin_nontemporal_store(w, (d2v*)a);
      } else {
        *(double2*)a = v[r];
      }
    }
  }
  if constexpr (kCo) {
    // the echo branch's tile, after the forward's: its global factor i^k w
    // of K_p and of K'_1
    const double2 gE = rot_i(make_double2(R2.d(kRecTotal, 0), R2.d(kRecTotal, 1)),
                             (fzw2 >> kT12PhShift) & 3);
    char* d2 = (char*)(A.dst2 + sbase);
#pragma unroll
    for (int r = 0; r < kRegs; ++r) {
      const double2 u = cmul(w[r], gE);
      d2v x = {u.x, u.y};
      __builtin_nontemporal_store(x, (d2v*)(d2 + tile_ofs(r) + (ofs32 ? (int64_t)sofs : sofs64)));
    }
  }
  if constexpr (MC == 1) {
    if (pm_on) probe_finish();  // workgroup-uniform (A.meas)
  }
  if constexpr (MC >= 2) {
    // measurement combines after the tile's stores are issued (one barrier)
    if constexpr (MC == 3 && !SPLIT) {
      const int wave = t >> 6, lane = t & 63;
      auto finish = [&](auto lay_tag, double (&xs)[3][4], int slot0) {
        constexpr int LAY = decltype(lay_tag)::value;
        const double k = wave_sum_multi<4>(xs[LAY]);
        if ((lane & 15) == 0) s_red[wave][slot0 + 4 * LAY + (lane >> 4)] = k;
      };
      if constexpr (RP::pre) {
        if (x_pre) {
          if constexpr (RP::nIO) finish(LIO{}, xpre, kSlotXPre);
          if constexpr (RP::n0) finish(L0{}, xpre, kSlotXPre);
          if constexpr (RP::nO) finish(LO{}, xpre, kSlotXPre);
        }
      }
      if constexpr (RP::post) {
        if (x_post) {
          if constexpr (RP::nO) finish(LO{}, xpost, kSlotXPost);
          if constexpr (RP::n0) finish(L0{}, xpost, kSlotXPost);
          if constexpr (RP::nIO) finish(LIO{}, xpost, kSlotXPost);
        }
      }
    }
    // obs [2L, 3L): X before the post-kick, [3L, 4L): X before the pre-kick
    // (0 for sites this pass does not kick), observable 2L + xo
    auto x_combine = [&](int xo) {
      const int L = A.L_real;
      if (xo < 0 || xo >= 2 * L) return;
      const bool pre = xo >= L;
      const int site = pre ? xo - L : xo;
      const int tb = site < c ? site : ((site >= s && site < s + kTileBits - c) ? c + site - s : -1);
      double acc = 0.0;
      if (tb >= 0 && ((A.act >> tb) & 1) && (pre ? x_pre : x_post)) {
        if constexpr (SPLIT && MC == 3) {
          const double* px = &s_xpart[0][pre ? 1 : 0][tb >> 2][(tb & 3) << 3];
          constexpr int kW = 2 * 3 * 32;  // doubles per wave
          for (int w = 0; w < kThreads / 64; ++w)
#pragma unroll
            for (int i = 0; i < 8; ++i) acc += px[w * kW + i];
        } else {
          const int slot = (pre ? kSlotXPre : kSlotXPost) + tb;
          for (int w = 0; w < kThreads / 64; ++w) acc += s_red[w][slot];
        }
      }
      A.partial[(b * n_tiles + tile) * A.n_obs + 2 * L + xo] = acc;
    };
    if (zc_lay >= 0 || x_pre || x_post) {
      __syncthreads();
      if (zc_lay >= 0) site_combine(zc_lay, zc_inv, t);
      // X on wave 2 (2L <= 64), beside wave 0's Z / ZZ combine
      if (x_pre || x_post) x_combine(t - 2 * kWaveSize);
    }
  }
#ifdef DTC_PHASE_TIMING
  DTC_TS(6);
  if (A.dbg_ts && t < 8 && SHAPE == DTC_PHASE_TIMING) {
    // t 0..6: phase stamps (s_memtime, per-XCD clock); 7: s_memrealtime
    // (100 MHz, chip-wide) start in bits 0..31, duration in bits 32..59
    const uint64_t rt_end = __builtin_amdgcn_s_memrealtime();
    const uint64_t val = t < 7 ? ts[t & 7]
                               : ((rt_start & 0xffffffffull) | ((rt_end - rt_start) << 32));
    A.dbg_ts[(b * n_tiles + tile) * 8 + t] = val | ((uint64_t)NIBS << 60);
  }
#endif
}

// Kernel symbols per pass shape so rocprofv3 traces separate them.
#define DTC_DEFINE_PASS(NAME, SHAPE_EXPR)                                          \
  template <int NIBS, int KIND, int MC, int GEO = kGeoStd>                         \
  __global__ __launch_bounds__(kThreads, 2) void NAME(PassArgs A) {                \
    pass_body<SHAPE_EXPR, NIBS, KIND, MC, false, false, false, GEO>(A);           \
  }
DTC_DEFINE_PASS(dtc_kdk_pass, kShapeKDK)
// the K-D-K at three workgroups per CU (half-LDS re-layouts, 168 VGPRs) for
// the nibble sets in PassArgs::kdk_split: bit NIBS for passes without or with
// the probe measurement, bit 8 + NIBS for per-site / energy ones.  Default: the
// 12-site probe passes (r3i: <7> 5.36 ms vs 6.10; the 8-site ones are 2 %
// slower at three) and every per-site / energy pass (r3r: energy K-D-K 1.81 ->
// 1.69 ms at B=256, C4 +1 %)
template <int NIBS, int KIND, int MC, int GEO = kGeoStd>
__global__ __launch_bounds__(kThreads, 3) void dtc_kdk_pass3(PassArgs A) {
  pass_body<kShapeKDK, NIBS, KIND, MC, false, true, false, GEO>(A);
}
// a forward K-D-K that also starts an echo branch (pass_body DUAL): two
// tiles in registers, so two workgroups per CU; half-tile re-layouts (their
// opaque per-thread bases keep the addresses out of the register budget: with
// full-tile ones the <7> form takes 256 VGPRs and spills 27, r4u: 9.9 -> 11.5 ms)
template <int NIBS, int KIND, int MC, int GEO = kGeoStd>
__global__ __launch_bounds__(kThreads, 2) void dtc_kdk_dual(PassArgs A) {
  pass_body<kShapeKDK, NIBS, KIND, MC, false, true, true, GEO>(A);
}
// its device-noise form: the forward K-D closing a period (device-like noise
// runs no forward layer ahead) that also starts the echo branch
template <int NIBS, int KIND, int MC, int GEO = kGeoStd>
__global__ __launch_bounds__(kThreads, 2) void dtc_kd_dual(PassArgs A) {
  pass_body<kShapeKD, NIBS, KIND, MC, false, true, true, GEO>(A);
}
DTC_DEFINE_PASS(dtc_kd_pass, kShapeKD)
DTC_DEFINE_PASS(dtc_dk_pass, kShapeDK)
DTC_DEFINE_PASS(dtc_kick_pass, kShapeK)
#undef DTC_DEFINE_PASS
// The last pass of an echo chain: same work, probe measurement, no stores
// (the echo state is never read again): 16 B of HBM traffic per amplitude.
#define DTC_DEFINE_FINAL(NAME, SHAPE_EXPR)                                         \
  template <int NIBS, int KIND, int GEO = kGeoStd>                                 \
  __global__ __launch_bounds__(kThreads, 2) void NAME(PassArgs A) {                \
    pass_body<SHAPE_EXPR, NIBS, KIND, 1, true, false, false, GEO>(A);             \
  }
DTC_DEFINE_FINAL(dtc_kdk_final, kShapeKDK)
DTC_DEFINE_FINAL(dtc_kd_final, kShapeKD)
DTC_DEFINE_FINAL(dtc_dk_final, kShapeDK)
// the kick-only end (device-like noise chains end in one) at three workgroups
// per CU with the half-tile re-layouts: a read-only pass has no stores to
// overlap its loads with, so the third workgroup's loads do (r4zc: C3's
// <7> 3.80 -> 3.03 ms, <6> 3.24 -> 2.85 ms)
template <int NIBS, int KIND, int GEO = kGeoStd>
__global__ __launch_bounds__(kThreads, 3) void dtc_kick_final(PassArgs A) {
  pass_body<kShapeK, NIBS, KIND, 1, true, true, false, GEO>(A);
}
#undef DTC_DEFINE_FINAL
// The energy sweep's last pass (one kick layer past the last period, for the
// X of its group at the last time point): measures, stores nothing.
template <int NIBS, int KIND>
__global__ __launch_bounds__(kThreads, 2) void dtc_kick_xfinal(PassArgs A) {
  pass_body<kShapeK, NIBS, KIND, 3, true>(A);
}
template <int NIBS, int MC, int GEO = kGeoStd>
__global__ __launch_bounds__(kThreads, 2) void dtc_diag_pass(PassArgs A) {
  pass_body<kShapeD, NIBS, kKindRX, MC, false, false, false, GEO>(A);
}

template <int NIBS, int KIND, int MC, int GEO = kGeoStd>
hipError_t launch_shape(const PassArgs& a, dim3 grid, int shape, hipStream_t stream) {
  dim3 block(kThreads);
  if (a.no_store) {
    if constexpr (MC == 3) {
      if (shape != kShapeK) return hipErrorInvalidValue;
      hipLaunchKernelGGL((dtc_kick_xfinal<NIBS, KIND>), grid, block, 0, stream, a);
      return hipGetLastError();
    } else if constexpr (MC != 1) {
      return hipErrorInvalidValue;  // probe passes end an echo chain, energy sweeps a kick pass
    } else {
      switch (shape) {
        case kShapeKDK: hipLaunchKernelGGL((dtc_kdk_final<NIBS, KIND, GEO>), grid, block, 0, stream, a); break;
        case kShapeKD: hipLaunchKernelGGL((dtc_kd_final<NIBS, KIND, GEO>), grid, block, 0, stream, a); break;
        case kShapeDK: hipLaunchKernelGGL((dtc_dk_final<NIBS, KIND, GEO>), grid, block, 0, stream, a); break;
        case kShapeK: hipLaunchKernelGGL((dtc_kick_final<NIBS, KIND, GEO>), grid, block, 0, stream, a); break;
        default: return hipErrorInvalidValue;
      }
      return hipGetLastError();
    }
  }
  if (a.dst2) {
    // K-D-K: unitary kicks; K-D: device-like noise (factored or general kicks)
    if constexpr (MC <= 1) {
      if (shape == kShapeKDK) {
        hipLaunchKernelGGL((dtc_kdk_dual<NIBS, KIND, MC, GEO>), grid, block, 0, stream, a);
        return hipGetLastError();
      }
    }
    if constexpr (MC <= 1 && GEO == kGeoStd && (KIND == kKindRXU || KIND == kKindRYU || KIND == kKindGen)) {
      if (shape == kShapeKD) {
        hipLaunchKernelGGL((dtc_kd_dual<NIBS, KIND, MC>), grid, block, 0, stream, a);
        return hipGetLastError();
      }
    }
    return hipErrorInvalidValue;
  }
  switch (shape) {
    case kShapeKDK:
      if constexpr (true) {
        if ((a.kdk_split >> (NIBS + (MC >= 2 ? 8 : 0))) & 1) {
          hipLaunchKernelGGL((dtc_kdk_pass3<NIBS, KIND, MC, GEO>), grid, block, 0, stream, a);
          break;
        }
      }
      hipLaunchKernelGGL((dtc_kdk_pass<NIBS, KIND, MC, GEO>), grid, block, 0, stream, a);
      break;
    case kShapeKD: hipLaunchKernelGGL((dtc_kd_pass<NIBS, KIND, MC, GEO>), grid, block, 0, stream, a); break;
    case kShapeDK: hipLaunchKernelGGL((dtc_dk_pass<NIBS, KIND, MC, GEO>), grid, block, 0, stream, a); break;
    case kShapeK: hipLaunchKernelGGL((dtc_kick_pass<NIBS, KIND, MC, GEO>), grid, block, 0, stream, a); break;
    case kShapeD:
      if constexpr (MC == 3) {
        return hipErrorInvalidValue;  // no kicks: no X point
      } else {
        hipLaunchKernelGGL((dtc_diag_pass<NIBS, MC, GEO>), grid, block, 0, stream, a);
      }
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <int NIBS, int MC>
hipError_t launch_kind_mc(const PassArgs& a, dim3 grid, int shape, int kind,
                          hipStream_t stream) {
  if constexpr (NIBS == 6 && MC <= 1) {
    // the 7-site column group of the 13 / 7 split (kGeoB7)
    if (a.c == kB7Cols) {
      if (a.s != 13 || a.act != 0xFE0) return hipErrorInvalidValue;
      switch (kind) {
        case kKindRX: return launch_shape<NIBS, kKindRX, MC, kGeoB7>(a, grid, shape, stream);
        case kKindRY: return launch_shape<NIBS, kKindRY, MC, kGeoB7>(a, grid, shape, stream);
        default: return hipErrorInvalidValue;
      }
    }
  }
  switch (kind) {
    case kKindRX: return launch_shape<NIBS, kKindRX, MC>(a, grid, shape, stream);
    case kKindRY: return launch_shape<NIBS, kKindRY, MC>(a, grid, shape, stream);
    case kKindGen: return launch_shape<NIBS, kKindGen, MC>(a, grid, shape, stream);
    case kKindRXU:
    case kKindRYU:
      // device-like noise: no in-flight X (dtc_energy_device measures X by
      // basis-change passes)
      if constexpr (MC == 3) {
        return hipErrorInvalidValue;
      } else {
        return kind == kKindRXU ? launch_shape<NIBS, kKindRXU, MC>(a, grid, shape, stream)
                                : launch_shape<NIBS, kKindRYU, MC>(a, grid, shape, stream);
      }
    default: return hipErrorInvalidValue;
  }
}

template <int NIBS>
hipError_t launch_kind(const PassArgs& a, dim3 grid, int shape, int kind, int mc,
                       hipStream_t stream) {
  switch (mc) {
    case 0: return launch_kind_mc<NIBS, 0>(a, grid, shape, kind, stream);
    case 1: return launch_kind_mc<NIBS, 1>(a, grid, shape, kind, stream);
    case 2: return launch_kind_mc<NIBS, 2>(a, grid, shape, kind, stream);
    default: return launch_kind_mc<NIBS, 3>(a, grid, shape, kind, stream);
  }
}

#ifdef DTC_DEV_KNOBS
__global__ void dbg_spacer_kernel(int us) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
  while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)us * 100) __builtin_amdgcn_s_sleep(10);
}
#endif

hipError_t launch_pass(const PassArgs& a, int batch, int shape, int kind, hipStream_t stream,
                       int* lc_variant) {
#ifdef DTC_DEV_KNOBS
  // development builds, timing probe: DTC_DBG_SPACER=<us> runs a one-wave
  // sleep kernel of that length before every 13-site pass
  if (a.tile_bits == kMaxTileBits && shape != kShapeLC)
    if (const char* e = std::getenv("DTC_DBG_SPACER"))
      hipLaunchKernelGGL(dbg_spacer_kernel, dim3(1), dim3(64), 0, stream, std::atoi(e));
#endif
  if (a.tile_bits == kMaxTileBits && shape != kShapeLC) return launch_pass13(a, batch, shape, kind, stream);
  if (a.L_eff > 32 || a.L_eff < kTileBits || a.batch != batch || batch > 65535 ||
      a.n_chunks > kMaxChunks)
    return hipErrorInvalidValue;
  const int n_tiles = 1 << (a.L_eff - kTileBits);
  if (a.octet_bits && (a.octet_bits < 4 || a.octet_bits > a.L_eff || (int64_t)n_tiles * 8 > 0x7FFFFFFF))
    return hipErrorInvalidValue;
  // octet layout: the eight states of an octet on consecutive blocks
  dim3 grid = a.octet_bits ? dim3(n_tiles * 8, (batch + 7) / 8) : dim3(n_tiles, batch);
  if (shape == kShapeLC) return launch_lightcone(a, grid, kind, stream, lc_variant);
  int nibs = 0;
  for (int n = 0; n < 3; ++n)
    if (a.act & (0xF << (4 * n))) nibs |= 1 << n;
  const bool xm = a.meas == kMeasEnergy && (a.meas_parts & (kPartXPre | kPartXPost));
  const int mc = a.meas == kMeasNone ? 0 : (a.meas == kMeasProbe ? 1 : (xm ? 3 : 2));
  switch (nibs) {
    case 4: return launch_kind<4>(a, grid, shape, kind, mc, stream);
    case 6: return launch_kind<6>(a, grid, shape, kind, mc, stream);
    case 7: return launch_kind<7>(a, grid, shape, kind, mc, stream);
    default: return hipErrorInvalidValue;  // group layouts never produce other sets
  }
}

// out[b][o] = sum over tiles of partial[b][tile][o]: one workgroup per
// (state, 8 observables), fixed summation order (strided per thread, then an
// LDS tree), so results do not depend on the batch a state ran in.
// Per-state sums over tiles: a workgroup per (state, block of up to 256
// columns); thread t sums column t % cols over every (256 / cols)-th tile,
// coalesced across the columns, then the column's groups are added in LDS
// (fixed order: results do not depend on the batch).
__global__ __launch_bounds__(256) void reduce_kernel(const double* __restrict__ partial,
                                                     int n_tiles, int n_obs, int o_first,
                                                     int n_out, int cols, int accumulate,
                                                     double* __restrict__ out,
                                                     int64_t out_stride, int splits) {
  __shared__ double s_acc[256];
  const int b = blockIdx.y, t = threadIdx.x, z = blockIdx.z;
  const int o = blockIdx.x * cols + t % cols, grp = t / cols, ngrp = 256 / cols;
  // split z of `splits` sums tiles [k0, k1) (stage 1 of a two-stage sum)
  const int per = n_tiles / splits, k0 = z * per, k1 = k0 + per;
  double acc = 0.0;
  if (o < n_out) {
    const double* p = partial + (int64_t)b * n_tiles * n_obs + o_first + o;
    double a2[4] = {0.0, 0.0, 0.0, 0.0};
    int k = k0 + grp;
    for (; k + 3 * ngrp < k1; k += 4 * ngrp) {
#pragma unroll
      for (int u = 0; u < 4; ++u) a2[u] += p[(int64_t)(k + u * ngrp) * n_obs];
    }
    for (; k < k1; k += ngrp) a2[0] += p[(int64_t)k * n_obs];
    acc = (a2[0] + a2[1]) + (a2[2] + a2[3]);
  }
  s_acc[t] = acc;
  __syncthreads();
  if (grp == 0 && o < n_out) {
    double sum = s_acc[t];
    for (int g = 1; g < ngrp; ++g) sum += s_acc[g * cols + t];
    if (splits > 1) {
      out[((int64_t)b * splits + z) * n_out + o] = sum;  // scratch: [batch][splits][n_out]
    } else {
      double* dst = out + (int64_t)b * out_stride + o;
      *dst = accumulate ? *dst + sum : sum;
    }
  }
}

hipError_t launch_reduce(const double* partial, int n_tiles, int n_obs, int batch,
                         double* out, int64_t out_stride, hipStream_t stream, int o_first,
                         int n_out, int accumulate, double* scratch) {
  if (n_out < 0) n_out = n_obs - o_first;
  if (o_first < 0 || n_out < 1 || o_first + n_out > n_obs) return hipErrorInvalidValue;
  auto cols_of = [](int n) {
    return n <= 16 ? 16 : (n <= 32 ? 32 : (n <= 64 ? 64 : (n <= 128 ? 128 : 256)));
  };
  const int cols = cols_of(n_out);
  const int splits = reduce_splits(n_tiles);
  if (splits > 1) {
    // two stages: every (state, split) a workgroup, then the splits in order
    if (!scratch || n_tiles % splits) return hipErrorInvalidValue;
    hipLaunchKernelGGL(reduce_kernel, dim3((n_out + cols - 1) / cols, batch, splits), dim3(256), 0,
                       stream, partial, n_tiles, n_obs, o_first, n_out, cols, 0, scratch,
                       (int64_t)0, splits);
    hipLaunchKernelGGL(reduce_kernel, dim3((n_out + cols - 1) / cols, batch, 1), dim3(256), 0,
                       stream, (const double*)scratch, splits, n_out, 0, n_out, cols, accumulate,
                       out, out_stride, 1);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(reduce_kernel, dim3((n_out + cols - 1) / cols, batch, 1), dim3(256), 0, stream,
                     partial, n_tiles, n_obs, o_first, n_out, cols, accumulate, out, out_stride, 1);
  return hipGetLastError();
}

// Per-instance sums over the trajectories of a batch (dtc_energy_sums):
// out[i][c] = sum over the states b of instance inst0 + i in this batch of
// vals[b][c], c < cols; states b hold instance (batch_start + b) / n_traj.
// One thread per column, states in a fixed order (four interleaved partial
// sums, combined in order).
__global__ __launch_bounds__(256) void traj_sum_kernel(const double* __restrict__ vals, int nb,
                                                       int cols, int64_t batch_start, int n_traj,
                                                       double* __restrict__ out) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= cols) return;
  const int64_t inst0 = batch_start / n_traj;
  const int64_t inst = inst0 + blockIdx.y;
  const int64_t lo0 = inst * n_traj - batch_start, hi0 = (inst + 1) * n_traj - batch_start;
  const int64_t lo = lo0 > 0 ? lo0 : 0, hi = hi0 < nb ? hi0 : nb;
  double a[4] = {0.0, 0.0, 0.0, 0.0};
  int64_t b = lo;
  for (; b + 3 < hi; b += 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u) a[u] += vals[(b + u) * cols + c];
  }
  for (; b < hi; ++b) a[0] += vals[b * cols + c];
  out[(int64_t)blockIdx.y * cols + c] = (a[0] + a[1]) + (a[2] + a[3]);
}

hipError_t launch_traj_sum(const double* vals, int nb, int cols, int64_t batch_start, int n_traj,
                           double* out, hipStream_t stream) {
  if (nb < 1 || cols < 1 || n_traj < 1 || batch_start < 0) return hipErrorInvalidValue;
  const int64_t n_inst = (batch_start + nb - 1) / n_traj - batch_start / n_traj + 1;
  hipLaunchKernelGGL(traj_sum_kernel, dim3((cols + 255) / 256, (unsigned)n_inst), dim3(256), 0,
                     stream, vals, nb, cols, batch_start, n_traj, out);
  return hipGetLastError();
}

__global__ void set_basis_kernel(double2* state, int64_t state_len, const int64_t* idx,
                                 int batch, int og) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= batch) return;
  state[state_base(b, state_len, og) + octet_spread(idx[b], og)] = make_double2(1.0, 0.0);
}

hipError_t launch_set_basis(double2* state, int64_t state_len, const int64_t* idx, int batch,
                            hipStream_t stream, int octet_bits) {
  hipLaunchKernelGGL(set_basis_kernel, dim3((batch + 63) / 64), dim3(64), 0, stream, state,
                     state_len, idx, batch, octet_bits);
  return hipGetLastError();
}

// In-place all-to-all of one slice over W = 2^k virtual shards held in one
// buffer (the one-GPU stand-in for C5's xGMI exchange, sharded.py): piece
// (r, c) = slice `slice` of chunk c of shard r trades places with piece
// (c, r), r < c.  blockIdx.y = pair; each thread moves kSwapPerThread
// amplitudes of both pieces, 16-B accesses 256 threads apart (1 KiB per wave
// instruction, coalesced), streaming hints (every byte is touched once).
// The last pre-exchange kick pass of one slice fused with the virtual ranks'
// in-place all-to-all of that slice (dtc_shard_kick_exchange_slice; C5 on one
// GPU, sharded.py inplace): the slice of piece (shard r, chunk c) is a
// 2^L_eff-amplitude state, pieces state_len apart, b = r W + c.  A workgroup
// takes tile i of the pair (r, c), (c, r) -- both tiles loaded before either
// is stored -- kicks each and stores it at its partner's place (the diagonal
// pieces in place): the exchange costs no pass of its own (it was 32 B per
// amplitude of the off-diagonal pieces, 76 of 473 ms per L=34 period, r3zk).
// grid = (tiles, W (W + 1) / 2 pair slots); contiguous states (octet_bits 0).
template <int NIBS, int KIND>
__global__ __launch_bounds__(kThreads, 2) void dtc_kick_swap_pass(PassArgs A, int k_bits) {
  static_assert(KIND == kKindRX || KIND == kKindRY || KIND == kKindGen, "unitary kick kinds");
  using RP = RoundPlan<NIBS, kShapeK>;
  __shared__ double2 s_tile[kTile];
  const int t = threadIdx.x;
  const int W = 1 << k_bits;
  int q = blockIdx.y, r = 0;
  while (q >= W - r) {  // pair slot -> (r, c), r <= c
    q -= W - r;
    ++r;
  }
  const int c_ch = r + q;
  const int64_t b1 = (int64_t)r * W + c_ch, b2 = (int64_t)c_ch * W + r;
  const int64_t tile = blockIdx.x;
  RecRegs R;  // every piece is the same trajectory: piece b1's records
  {
    const int lane = t & 63;
    const double2* rp = (const double2*)(A.recs + b1 * kRecPerState) + 2 * lane;
    double2 r0 = make_double2(0.0, 0.0), r1 = make_double2(0.0, 0.0);
    if (4 * lane < 8 * kRecPerState) {
      r0 = rp[0];
      r1 = rp[1];
    }
    R.rv[0] = r0.x; R.rv[1] = r0.y; R.rv[2] = r1.x; R.rv[3] = r1.y;
  }
  const int c = A.c, s = A.s;
  const int64_t mid_mask = ((int64_t)1 << A.tile_bits_mid) - 1;
  TileMap M;
  M.c = c;
  M.s = s;
  M.cmask = (1 << c) - 1;
  M.tbase = ((tile & mid_mask) << c) | ((tile >> A.tile_bits_mid) << (s + kTileBits - c));
  const int64_t vofs = M.rel(ybase<RP::IO>(t)) << 4;
  auto tile_ofs = [&](int rr) -> int64_t { return (M.tbase | M.rel(rr << (4 * RP::IO))) << 4; };
  const char* p1 = (const char*)(A.src + b1 * A.state_len);
  const char* p2 = (const char*)(A.src + b2 * A.state_len);
  double2 v[kRegs], w[kRegs];
#pragma unroll
  for (int rr = 0; rr < kRegs; ++rr) {
    const d2v x = __builtin_nontemporal_load((const d2v*)(p1 + tile_ofs(rr) + vofs));
    v[rr] = make_double2(x.x, x.y);
  }
  // the partner tile, loaded after v's kicks (behind v's stores): with its
  // loads issued up front both tiles were live through v's kicks and the
  // 256-VGPR budget spilled 20-100 B per thread (r6h: 11.62 -> 11.28 ms)
  auto load_w = [&]() {
    if (b2 != b1) {
#pragma unroll
      for (int rr = 0; rr < kRegs; ++rr) {
        const d2v x = __builtin_nontemporal_load((const d2v*)(p2 + tile_ofs(rr) + vofs));
        w[rr] = make_double2(x.x, x.y);
      }
    }
  };
  const double2 gph = make_double2(R.d(kRecTotal, 0), R.d(kRecTotal, 1));
  // the kick-only pass of pass_body: rounds IO -> 0 -> O, the global factor,
  // back to the IO layout
  auto kick = [&](double2 (&u)[kRegs]) {
    if constexpr (RP::nIO) apply_nibble<RP::IO, KIND>(u, R, 0);
    if constexpr (RP::n0) {
      exchange<RP::IO, 0>(u, s_tile, t);
      apply_nibble<0, KIND>(u, R, 0);
    }
    if constexpr (RP::nO) {
      exchange<RP::n0 ? 0 : RP::IO, RP::O>(u, s_tile, t);
      apply_nibble<RP::O, KIND>(u, R, 0);
    }
#pragma unroll
    for (int rr = 0; rr < kRegs; ++rr) u[rr] = cmul(u[rr], gph);
    exchange<RP::d_lay, RP::IO>(u, s_tile, t);
  };
  auto store = [&](const double2 (&u)[kRegs], const char* base) {
    char* p = (char*)base;
#pragma unroll
    for (int rr = 0; rr < kRegs; ++rr) {
      d2v x = {u[rr].x, u[rr].y};
      __builtin_nontemporal_store(x, (d2v*)(p + tile_ofs(rr) + vofs));
    }
  };
  kick(v);
  load_w();
  store(v, p2);  // (r, c) -> (c, r); the diagonal piece in place
  if (b2 != b1) {  // uniform across the workgroup
    // w's first re-layout writes slots other threads may still be reading in
    // v's last one (as in dtc_kdk_dual)
    __syncthreads();
    kick(w);
    store(w, p1);
  }
}

hipError_t launch_kick_swap(const PassArgs& a, int k_bits, int kind, hipStream_t stream) {
  const int W = 1 << k_bits;
  if (k_bits < 1 || k_bits > 6 || a.batch != W * W || a.octet_bits != 0 || a.src != a.dst ||
      a.L_eff < kTileBits || a.L_eff > 32 || a.n_chunks > kMaxChunks)
    return hipErrorInvalidValue;
  int nibs = 0;
  for (int n = 0; n < 3; ++n)
    if (a.act & (0xF << (4 * n))) nibs |= 1 << n;
  const dim3 grid(1u << (a.L_eff - kTileBits), (unsigned)(W * (W + 1) / 2)), block(kThreads);
  auto go = [&](auto nibs_tag) -> hipError_t {
    constexpr int N = decltype(nibs_tag)::value;
    switch (kind) {
      case kKindRX: hipLaunchKernelGGL((dtc_kick_swap_pass<N, kKindRX>), grid, block, 0, stream, a, k_bits); break;
      case kKindRY: hipLaunchKernelGGL((dtc_kick_swap_pass<N, kKindRY>), grid, block, 0, stream, a, k_bits); break;
      case kKindGen: hipLaunchKernelGGL((dtc_kick_swap_pass<N, kKindGen>), grid, block, 0, stream, a, k_bits); break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  };
  switch (nibs) {
    case 4: return go(std::integral_constant<int, 4>{});
    case 6: return go(std::integral_constant<int, 6>{});
    case 7: return go(std::integral_constant<int, 7>{});
    default: return hipErrorInvalidValue;
  }
}

static constexpr int kSwapPerThread = 4;

__global__ __launch_bounds__(256) void exchange_swap_kernel(double2* __restrict__ state, int nl,
                                                            int k, int nsub, int slice) {
  int p = blockIdx.y, r = 0;
  const int W = 1 << k;
  while (p >= W - 1 - r) {
    p -= W - 1 - r;
    ++r;
  }
  const int c = r + 1 + p;
  const int64_t off = ((int64_t)slice << nsub) + (int64_t)blockIdx.x * (256 * kSwapPerThread) +
                      threadIdx.x;
  d2v* a = (d2v*)(state + ((int64_t)r << nl) + ((int64_t)c << (nl - k)) + off);
  d2v* b = (d2v*)(state + ((int64_t)c << nl) + ((int64_t)r << (nl - k)) + off);
  d2v va[kSwapPerThread], vb[kSwapPerThread];
#pragma unroll
  for (int j = 0; j < kSwapPerThread; ++j) {
    va[j] = __builtin_nontemporal_load(a + 256 * j);
    vb[j] = __builtin_nontemporal_load(b + 256 * j);
  }
#pragma unroll
  for (int j = 0; j < kSwapPerThread; ++j) {
    __builtin_nontemporal_store(vb[j], a + 256 * j);
    __builtin_nontemporal_store(va[j], b + 256 * j);
  }
}

hipError_t launch_exchange_swap(double2* state, int nl, int k, int nsub, int slice,
                                hipStream_t stream) {
  // the grid covers each piece exactly: 2^nsub amplitudes, 1024 per workgroup
  if (k < 1 || nsub < 10 || nsub + k > nl || nl > 40) return hipErrorInvalidValue;
  const int pairs = ((1 << k) * ((1 << k) - 1)) / 2;
  const int64_t blocks = ((int64_t)1 << nsub) / (256 * kSwapPerThread);
  if (blocks > 0x7FFFFFFF || pairs > 65535) return hipErrorInvalidValue;
  hipLaunchKernelGGL(exchange_swap_kernel, dim3((unsigned)blocks, pairs), dim3(256), 0, stream,
                     state, nl, k, nsub, slice);
  return hipGetLastError();
}

}  // namespace dtc
