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
static constexpr int kRegs = 16;          // amplitudes per thread (4 register bits)
static constexpr int kChunkBits = 5;      // diagonal factor tables: 5 sites + next bit
static constexpr int kMaxChunks = 8;      // L_eff <= 40
static constexpr int kMaxObs = 1 + 40;    // norm + per-site <Z_i>

enum DiagMode { kDiagNone = 0, kDiagAfter = 1, kDiagBeforeConj = 2 };
enum MeasMode { kMeasNone = 0, kMeasProbe = 1, kMeasSites = 2 };

// One pass over a batch of states: a tile covers the index bits
// [0, c) ∪ [s, s + a) with c + a = kTileBits; the kick gates of sites
// s .. s+a-1 are applied (sites >= L_real are padding: identity).
struct PassArgs {
  const double2* src;      // batch base, state b at src + b * state_len
  double2* dst;            // may alias src (in-place)
  int64_t state_len;       // 2^L_eff
  int L_eff;               // padded number of index bits (>= kTileBits)
  int L_real;              // physical sites
  int c, s, a;             // tile geometry
  int tile_bits_mid;       // s - c  (tile-id bits deposited at [c, s))
  // batch -> (instance, trajectory)
  int64_t batch_start;
  int n_traj;
  int64_t traj_offset;
  // kicks
  const double2* kick;     // [n_periods][L_real][n_sub][4]
  int n_sub;
  int kick_row;            // row of the kick table for this period
  int inverse;             // apply (G_q)^dagger in reverse sub order
  // noise
  uint32_t thr1, thr2, thr3;
  uint64_t seed;
  uint32_t stream;
  uint32_t rng_period;
  int noisy;
  // diagonal factor tables [n_inst][n_chunks][64]
  const double2* diag;
  int n_chunks;
  // measurement
  int probe;
  int n_obs;               // kMeasProbe: 2 (norm, Z_probe); kMeasSites: 1 + L_real
  double* partial;         // [B][n_tiles][n_obs]
};

hipError_t launch_pass(const PassArgs& a, int batch, int diag_mode, int meas_mode,
                       hipStream_t stream);

// out[b * out_stride + o] = sum over tiles of partial[b][tile][o] (fixed order)
hipError_t launch_reduce(const double* partial, int n_tiles, int n_obs, int batch,
                         double* out, int64_t out_stride, hipStream_t stream);

// state[b * state_len + idx[b]] = 1 (after the caller zeroed the batch)
hipError_t launch_set_basis(double2* state, int64_t state_len, const int64_t* idx,
                            int batch, hipStream_t stream);

}  // namespace dtc
