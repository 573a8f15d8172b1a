// dtc_rng.h — counter-based noise sampling shared by the HIP kernels and the
// host engine (compiled for both sides).
//
// The reference samples one Pauli per noisy gate per shot inside Aer
// (depolarizing_error(p, 1) on u1/u2/u3, fast.py:84-86):
//   I with prob 1 - 3p/4, X, Y, Z with prob p/4 each (Aer's Pauli form of
//   rho -> (1-p) rho + p I/2).
// Here the draw is a pure function of (seed, trajectory, stream, period,
// site, sub-gate) via Philox4x32-10, so trajectories are reproducible
// independently of batching and of the number of GPUs.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define DTC_HD __host__ __device__ __forceinline__
#else
#define DTC_HD static inline
#endif

namespace dtc {

// RNG stream ids
static constexpr uint32_t kStreamForward = 0u;       // forward trajectory
// echo branch at time index t uses stream 1 + t
static constexpr uint32_t kStreamPrep = 0xFFFFFFFFu; // neel X-gate prep noise

DTC_HD void mulhilo32(uint32_t a, uint32_t b, uint32_t* hi, uint32_t* lo) {
  uint64_t p = (uint64_t)a * (uint64_t)b;
  *hi = (uint32_t)(p >> 32);
  *lo = (uint32_t)p;
}

// Philox4x32 with 10 rounds (Salmon et al., SC'11): words 0 and 1 of the
// output block for counter (c0..c3) and key (k0, k1).
DTC_HD void philox_w01(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                       uint32_t k1, uint32_t* w0, uint32_t* w1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0, lo0, hi1, lo1;
    mulhilo32(0xD2511F53u, c0, &hi0, &lo0);
    mulhilo32(0xCD9E8D57u, c2, &hi1, &lo1);
    uint32_t n0 = hi1 ^ c1 ^ k0;
    uint32_t n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  *w0 = c0;
  *w1 = c1;
}

// Word 0 only.
DTC_HD uint32_t philox_w0(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                          uint32_t k0, uint32_t k1) {
  uint32_t w0, w1;
  philox_w01(c0, c1, c2, c3, k0, k1, &w0, &w1);
  return w0;
}

// Device-like noise draw of one kick sub-gate (include/dtc.h dtc_device_noise):
// word 0 -> Pauli against the site's thresholds (dephasing composed with
// depolarizing), word 1 -> amplitude-damping jump iff w1 < thr_jump.
DTC_HD int sample_device(uint64_t seed, uint64_t traj, uint32_t stream, uint32_t period,
                         uint32_t site, uint32_t sub, const uint32_t* thr, uint32_t thr_jump,
                         int* jump) {
  uint32_t x, y;
  philox_w01(site | (sub << 16), period, stream, (uint32_t)traj, (uint32_t)seed,
             (uint32_t)(seed >> 32) ^ (uint32_t)(traj >> 32), &x, &y);
  *jump = y < thr_jump ? 1 : 0;
  if (x < thr[0]) return 1;
  if (x < thr[1]) return 2;
  if (x < thr[2]) return 3;
  return 0;
}

// Pauli code: 0 = I, 1 = X, 2 = Y, 3 = Z.
// thr[k] = round(k * p/4 * 2^32) for k = 1, 2, 3 (computed on the host).
DTC_HD int sample_pauli(uint64_t seed, uint64_t traj, uint32_t stream,
                        uint32_t period, uint32_t site, uint32_t sub,
                        uint32_t thr1, uint32_t thr2, uint32_t thr3) {
  uint32_t x = philox_w0(site | (sub << 16), period, stream, (uint32_t)traj,
                         (uint32_t)seed, (uint32_t)(seed >> 32) ^ (uint32_t)(traj >> 32));
  if (x < thr1) return 1;
  if (x < thr2) return 2;
  if (x < thr3) return 3;
  return 0;
}

}  // namespace dtc
