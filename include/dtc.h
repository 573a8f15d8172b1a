/*
 * dtc.h — C ABI of the MI355X DTC autocorrelator engine (libdtc_hip.so).
 *
 * This ABI replaces the one call the reference makes into its execution
 * engine for the DTC sweep:
 *
 *   backend = AerSimulator(noise_model=noise_model, device="GPU",
 *                          cuStateVec_enable=True)          fast.py:156
 *   backend.run(circ_tnoise, shots=1024).result()
 *          .get_counts(circ_tnoise)                          fast.py:211-212
 *   compute_z_expectation(counts, 1)[0]                      fast.py:92-109,213
 *
 * (fast.py = autocorr-delta-a-single-qiskit-fast.py; the same call appears at
 *  ...-polarization.py:219, ...-circular-polarization.py:241,
 *  ...-controlled-g.py:305, ...-g-optimization.py:309, ...-shots.py:214.)
 *
 * Aer runs one (L+1)-qubit circuit per time point t.  The engine instead runs
 * the folded L-qubit model: every time point of the
 * forward sweep comes from one trajectory, and every echo point t branches
 * off the forward state at t.  Results per trajectory are the ancilla
 * expectation value  a_r(t) = (1-p)^n_anc * z_j(init_r) * <Z_j>_r(t),
 * whose mean over trajectories is the expectation of
 * (n0 - n1)/shots in the reference.
 *
 * Conventions
 *  - Site i of the spin chain is bit i of the amplitude index (qiskit
 *    little-endian, circuit qubit i+1; the ancilla is folded away).
 *  - complex128 amplitudes, interleaved (re, im).
 *  - Kick matrices are complex 2x2, row-major, interleaved:
 *    {m00.re, m00.im, m01.re, m01.im, m10.re, m10.im, m11.re, m11.im}.
 *  - All host arrays are C-contiguous and owned by the caller.
 *  - Return value 0 = success; negative = error, message via
 *    dtc_last_error() (thread-local).  No C++ exception crosses the ABI.
 *  - Calls are synchronous (return after a stream sync).  One dtc_ctx per
 *    device per host thread; a ctx is not re-entrant.
 */
#ifndef DTC_H
#define DTC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DTC_ABI_VERSION 12

/* error codes */
#define DTC_OK 0
#define DTC_EINVAL (-1)   /* bad argument                          */
#define DTC_EHIP (-2)     /* HIP runtime error                     */
#define DTC_ENOMEM (-3)   /* device allocation failed              */
#define DTC_ENODEV (-4)   /* no usable gfx950 device               */

typedef struct dtc_ctx dtc_ctx;

/* One disorder sweep (fast.py:41-74 argparse + disorder load, and the circuit
 * family of fast.py:111-147 / ...-polarization.py:110-142 /
 * ...-controlled-g.py:196-241). */
typedef struct dtc_problem {
  int32_t L;           /* sites (fast.py --L)                              */
  int32_t T;           /* time points t = 0..T-1 (fast.py:48-51, --tf)      */
  int32_t n_inst;      /* disorder instances (fast.py --inst)              */
  int32_t probe_site;  /* j = int(L/2) (fast.py:221)                        */
  int32_t t_offset;    /* periods applied at t = t + t_offset: 0 for fast.py,
                          1 for controlled-g.py:416,467                    */
  int32_t n_sub;       /* noisy kick sub-gates per site per period:
                          1 (x, y), 2 (xy, yx, circular)                   */
  uint64_t init_mask;  /* Z-basis product state: bit i set = X on site i
                          (neel: fast.py:127-130)                          */
  const double* h;     /* [n_inst][L]   on-site RZ(h_i) angles              */
  const double* phi;   /* [n_inst][L-1] bond RZZ(phi_i) angles              */
  const double* kick;  /* [n_periods][L][n_sub][8] complex 2x2 kick gates,
                          row p = the (p+1)-th forward period,
                          n_periods = T - 1 + t_offset                     */
  int32_t want_fwd;    /* compute the forward autocorrelator              */
  int32_t want_echo;   /* compute the echo autocorrelator                 */
  int32_t batch;       /* states per device batch, 0 = automatic          */
  int32_t t_first;     /* outputs for t < t_first are skipped (left as 0):
                          a single-circuit call (one t) sets t_first = T-1 */
} dtc_problem;

/* Noise model (fast.py:76-86): depolarizing_error(p, 1) after every noisy
 * single-qubit gate (u2/u3 = kick gates, neel X prep, and n_anc ancilla
 * u2 gates).  p = 0 or use_noise = 0 means ideal. */
typedef struct dtc_noise {
  double p;
  int32_t n_anc;       /* noisy ancilla gates folded as (1-p)^n_anc: 6   */
  int32_t reserved;
} dtc_noise;

/* Device-like noise (the reference's
 * use_fakebackend=1 path, NoiseModel.from_backend(FakeBrisbane()) at
 * fast.py:77-79, whose calibration data is not available offline: the caller
 * supplies per-site calibration).  After every kick sub-gate on site i:
 *   thermal relaxation  amplitude damping gamma_i = 1 - exp(-gate_ns / T1_i)
 *                       and pure dephasing to the total coherence decay
 *                       exp(-gate_ns / T2_i)  (T2 clamped to 2 T1),
 *   then depolarizing_error(p_gate_i, 1).
 * Trajectories stay linear: the amplitude-damping Kraus operator is drawn with
 * fixed probabilities (jump w.p. gamma/2) and weighted by 1/sqrt(prob), so the
 * trajectory mean of the (unnormalized) <Z_j> is the exact channel's.  The
 * neel-prep X gates get the Pauli part only.  The ancilla enters as
 *   a = anc_factor * z_j(init) * <Z_j>,  reported as the read-out value
 *   (1 - p01 - p10) a + (p10 - p01)   (P(read 1|0) = p01, P(read 0|1) = p10). */
typedef struct dtc_device_noise {
  const double* p_gate;  /* [L] depolarizing parameter per kick sub-gate   */
  const double* t1_us;   /* [L] T1 (microseconds; <= 0 or inf: none)      */
  const double* t2_us;   /* [L] T2 (microseconds; <= 0 or inf: none)      */
  double gate_ns;        /* duration of one kick sub-gate                  */
  double anc_factor;     /* ancilla coherence factor ((1-p)^6 in fast.py)  */
  double readout_p01;    /* ancilla read-out P(1 | 0)                      */
  double readout_p10;    /* ancilla read-out P(0 | 1)                      */
} dtc_device_noise;

/* Context management. device = HIP device ordinal. */
int dtc_open(int32_t device, dtc_ctx** out);
int dtc_close(dtc_ctx* ctx);
/* Free the ctx's batch work buffers (state batches, partial sums, kick
 * records; the next call re-allocates what it needs) after waiting for its
 * stream -- e.g. before the caller allocates one 256 GiB sharded state on the
 * same device.  The forward prefix (dtc_prefix_*) is kept: call
 * dtc_prefix_release as well to free it (the Python wrapper does both). */
int dtc_release_buffers(dtc_ctx* ctx);
const char* dtc_last_error(void);
int32_t dtc_abi_version(void);

/* Full sweep for trajectories [traj_offset, traj_offset + n_traj) of every
 * instance.  Per-trajectory outputs (caller averages; see header comment):
 *   fwd   [n_inst][n_traj][T]     (nullable if !want_fwd)
 *   echo  [n_inst][n_traj][T]     (nullable if !want_echo)
 *   zsite [n_inst][n_traj][T][L]  forward per-site <Z_i>(t), nullable
 * Replaces the get_instances/get_single_out loops (fast.py:217-239) over
 * backend.run (fast.py:211).  The noise RNG is Philox4x32-10 keyed by seed
 * and counted by (global trajectory, stream, period, site, sub-gate), so
 * results do not depend on batching or on how trajectories are sharded. */
int dtc_autocorr(dtc_ctx* ctx, const dtc_problem* prob, const dtc_noise* noise,
                 uint64_t seed, int64_t traj_offset, int32_t n_traj,
                 double* fwd, double* echo, double* zsite);

/* dtc_autocorr under device-like noise (dtc_device_noise above); noise->p
 * and noise->n_anc are ignored.  Outputs as dtc_autocorr (zsite: unnormalized
 * per-site <Z_i>, nullable). */
int dtc_autocorr_device(dtc_ctx* ctx, const dtc_problem* prob, const dtc_device_noise* dev,
                        uint64_t seed, int64_t traj_offset, int32_t n_traj, double* fwd,
                        double* echo, double* zsite);

/* Unit-test hook: apply n_periods Floquet periods to one host state vector
 * of 2^L complex128 amplitudes (in/out).  Forward: periods first_period,
 * first_period+1, ... (1-based rows of prob->kick), RNG stream `stream`,
 * RNG period counter = period.  Inverse (fast.py:140-143): periods
 * first_period, first_period-1, ..., each U_F^-1, RNG period counter =
 * step k = 1..n_periods.  zsite_out (nullable) receives [norm, <Z_0>..<Z_{L-1}>]
 * of the final state. */
int dtc_apply_periods(dtc_ctx* ctx, const dtc_problem* prob, const dtc_noise* noise,
                      uint64_t seed, int32_t inst, int64_t traj, uint32_t stream,
                      int32_t first_period, int32_t n_periods, int32_t inverse,
                      double* state, double* zsite_out);

/* ---- One state sharded over ranks (L=34 over 8 GPUs).
 * The 2^L amplitudes are split over 2^n_global ranks; a shard holds 2^n_local
 * amplitudes (n_local = L - n_global, 12 <= n_local <= 32).  Physical index bit
 * q < n_local of a shard holds logical site site_of[q]; bit k of the rank id
 * holds site site_of[n_local + k].  A call may hold n_shards consecutive ranks
 * (first_rank ..) whose shards lie 2^n_local amplitudes apart in one device
 * buffer ("virtual ranks": one GPU emulating several; 1 per process on a
 * multi-GPU node).  Every logical bond whose two sites are both local must join
 * physically adjacent bits.  The kick on a global site is applied after the
 * caller's all-to-all exchange has made it local (the sweep driver alternates
 * two bit maps, see sharded.py); the RZZ/RZ diagonal never needs one: bonds and
 * fields on rank bits become per-rank effective fields and a per-rank phase.
 * Replaces the reference's whole-state Aer run of a circuit too large for one
 * device; there is no reference call site for it (fast.py caps L at 20). */
typedef struct dtc_shard {
  int32_t n_local;
  int32_t n_global;
  int32_t n_shards;
  int32_t first_rank;
  int32_t site_of[64];
} dtc_shard;

/* state (device pointer, n_shards * 2^n_local complex128): the Z-basis product
 * state prob->init_mask of trajectory traj (noisy X preparation, fast.py:127-130,
 * drawn as in dtc_autocorr), distributed per site_of. */
int dtc_shard_set_basis(dtc_ctx* ctx, const dtc_problem* prob, const dtc_noise* noise,
                        const dtc_shard* shard, uint64_t seed, int64_t traj, double* state);

/* One step on every shard held (device pointers; src may equal dst):
 *   dst = K_{period+1}[post_mask] . D^diag . K_period[pre_mask] . src
 * where K_p[mask] = the period-p kick (fast.py:113, forward RNG stream 0, RNG
 * period counter p, trajectory traj) on the logical sites at the physical
 * local bits in mask, and D = the RZZ+RZ layer (fast.py:115-120) of instance
 * inst.  obs (host, nullable): [n_shards][1 + n_local] = (sum |a|^2,
 * sum z_q |a|^2 per physical bit q) of each shard after D (at the end when
 * diag = 0).  Synchronous. */
int dtc_shard_step(dtc_ctx* ctx, const dtc_problem* prob, const dtc_noise* noise,
                   const dtc_shard* shard, uint64_t seed, int64_t traj, int32_t inst,
                   int32_t period, uint64_t pre_mask, int32_t diag, uint64_t post_mask,
                   const double* src, double* dst, double* obs);

/* dtc_shard_step without waiting: everything is enqueued on the ctx's stream
 * (dtc_get_stream) and obs_dev (device pointer, nullable) receives
 * [n_shards][1 + n_local] from a device reduction.  The tables of a bit map are
 * built and uploaded on its first use and cached (a sweep alternates two), so
 * the host never blocks on the stream.  The sharded sweep driver orders its
 * exchanges against these steps with events (sharded.py), and reads obs_dev
 * after its own synchronisation. */
int dtc_shard_step_async(dtc_ctx* ctx, const dtc_problem* prob, const dtc_noise* noise,
                         const dtc_shard* shard, uint64_t seed, int64_t traj, int32_t inst,
                         int32_t period, uint64_t pre_mask, int32_t diag, uint64_t post_mask,
                         const double* src, double* dst, double* obs_dev);

/* The period-`period` kick on the local bits pre_mask, restricted to slice
 * `slice` of every chunk of every shard held: a shard's top chunk_bits local
 * bits number its chunks, the next slice_bits its slices, so the call covers the
 * amplitudes whose slice bits equal `slice` (in place; asynchronous, ctx stream;
 * one launch).  pre_mask must lie below the slice bits.  With chunk_bits =
 * n_global, chunk c is what rank c receives in the period's all-to-all; the
 * sweep driver kicks slice s+1 while slice s of every chunk travels to every
 * peer at once (sharded.py). */
int dtc_shard_kick_slice(dtc_ctx* ctx, const dtc_problem* prob, const dtc_noise* noise,
                         const dtc_shard* shard, uint64_t seed, int64_t traj, int32_t period,
                         uint64_t pre_mask, int32_t chunk_bits, int32_t slice_bits,
                         int32_t slice, double* state);

/* The last pre-exchange kicks of slice `slice` (as dtc_shard_kick_slice with
 * chunk_bits = n_global) fused with its in-place exchange (as
 * dtc_shard_exchange_slice): the pass of the last site group in pre_mask
 * stores piece (r, c) at (c, r), so the exchange moves no bytes of its own
 * (one GPU holding every shard; unitary kick kinds, else the two calls). */
int dtc_shard_kick_exchange_slice(dtc_ctx* ctx, const dtc_problem* prob, const dtc_noise* noise,
                                  const dtc_shard* shard, uint64_t seed, int64_t traj,
                                  int32_t period, uint64_t pre_mask, int32_t slice_bits,
                                  int32_t slice, double* state);

/* Virtual ranks only (one process holds every shard: n_shards = 2^n_global,
 * first_rank = 0): the period's all-to-all for slice `slice`, in place.  With
 * chunk bits = the top n_global local bits and slice bits = the next
 * slice_bits, piece (shard r, chunk c, slice) trades places with piece
 * (shard c, chunk r, slice) for every r != c -- what the 2^n_global ranks'
 * exchange of that slice does over xGMI, without a second state buffer (an
 * L=34 state, 256 GiB, then fits one MI355X).  Asynchronous, ctx stream, one
 * launch; 2^(n_local - n_global - slice_bits) >= 4096.  No reference call
 * site (the reference caps L at 20, fast.py:177-178). */
int dtc_shard_exchange_slice(dtc_ctx* ctx, const dtc_shard* shard, int32_t slice_bits,
                             int32_t slice, double* state);

/* The ctx's HIP stream (hipStream_t), for ordering host-side collectives
 * against the asynchronous entry points; and a wait for everything on it. */
int dtc_get_stream(dtc_ctx* ctx, void** stream);
int dtc_synchronize(dtc_ctx* ctx);

/* Host-only: the site groups the engine's sharded steps use for an n_bits-bit
 * shard (high groups in increasing size: the top bits lie in a large group)
 * (bit masks, one per group; returns the count or a negative error). */
int32_t dtc_plan_groups(int32_t n_bits, uint64_t* masks, int32_t max_groups);

/* Forward prefix cache (the optimisation controller, SURVEY.md §8(f) row 2:
 * -g-optimization.py:359-427 re-runs the t+1-period circuit for every
 * candidate g of the last period; the t-period forward part is the same for
 * all candidates).
 * dtc_prefix_build: take the n_inst * n_traj trajectories (traj_offset ..)
 * of prob through periods 1..n_periods (noise keyed by seed, neel prep
 * included) and keep their states on the device, replacing any previous
 * prefix.  noise or dv (device-like noise, then noise is ignored).
 * dtc_autocorr_prefixed: dtc_autocorr (dv: dtc_autocorr_device, no zsite)
 * starting from those states: periods > n_periods and every echo draw their
 * noise from seed, the prefix periods keep theirs.  prob must match the
 * prefix's (instances, angles, kick rows 1..n_periods: checked by hash; the
 * same trajectories) and measure only after it (t_first + t_offset >
 * n_periods).  dtc_prefix_release frees the states. */
int dtc_prefix_build(dtc_ctx* ctx, const dtc_problem* prob, const dtc_noise* noise,
                     const dtc_device_noise* dv, uint64_t seed, int64_t traj_offset,
                     int32_t n_traj, int32_t n_periods);
int dtc_autocorr_prefixed(dtc_ctx* ctx, const dtc_problem* prob, const dtc_noise* noise,
                          const dtc_device_noise* dv, uint64_t seed, int64_t traj_offset,
                          int32_t n_traj, double* fwd, double* echo);
int dtc_prefix_release(dtc_ctx* ctx);

/* Energy observables of the forward sweep (the
 * BackendEstimatorV2 runs of autocorr-delta-a-single-qiskit-fast-energy*.py:
 * L-qubit circuit of fast.py's periods with no ancilla, energy.py:136-173).
 * Per trajectory and t (same schedule, noise and RNG contract as dtc_autocorr):
 *   z  [n_inst][n_traj][T][L]    <Z_i>
 *   zz [n_inst][n_traj][T][L-1]  <Z_i Z_{i+1}>      (nullable when L = 1)
 *   x  [n_inst][n_traj][T][L]    <X_i> (noiseless X-basis measurement)
 * in little-endian site order; the caller forms any Hamiltonian from them
 * (energy.py:83-102 builds its labels big-endian, see energy.py here). */
int dtc_energy(dtc_ctx* ctx, const dtc_problem* prob, const dtc_noise* noise, uint64_t seed,
               int64_t traj_offset, int32_t n_traj, double* z, double* zz, double* x);

/* dtc_energy under device-like noise (the FakeBrisbane estimator runs of
 * autocorr-delta-a-single-qiskit-fast-energy-fakebrisbane.py:131-192, with a
 * user-supplied calibration, see dtc_device_noise).  Same outputs, as the
 * Kraus-weighted (unnormalised) expectations of each trajectory: their mean is
 * the channel's expectation.  Read-out error is NOT applied here (anc_factor
 * and readout_p01/p10 are ignored); the caller maps the means (energy.py). */
int dtc_energy_device(dtc_ctx* ctx, const dtc_problem* prob, const dtc_device_noise* dv,
                      uint64_t seed, int64_t traj_offset, int32_t n_traj, double* z, double* zz,
                      double* x);

/* The energy estimator's trajectory means without the per-trajectory rows
 * (ABI 11): the same sweep as dtc_energy (dv == NULL) or dtc_energy_device
 * (dv != NULL; noise unused then), reduced over the n_traj trajectories of
 * each instance on the device:
 *   z_sum  [n_inst][T][L], zz_sum [n_inst][T][L-1] (nullable when L = 1),
 *   x_sum  [n_inst][T][L]
 * = the sums over trajectories of dtc_energy's z, zz, x (fixed summation
 * order within a batch, batches added on the host: equal to the host sums of
 * those rows, and invariant under a change of batch size, only up to
 * rounding -- unlike the per-trajectory rows, which are bit-identical for any
 * batching).  The energy
 * scripts need only these means (energy.py:136-173: <H> from the estimator's
 * expectation values); only a few KB per batch cross PCIe. */
int dtc_energy_sums(dtc_ctx* ctx, const dtc_problem* prob, const dtc_noise* noise,
                    const dtc_device_noise* dv, uint64_t seed, int64_t traj_offset,
                    int32_t n_traj, double* z_sum, double* zz_sum, double* x_sum);

/* Profiling: when enabled, every kernel launch is bracketed by HIP events on
 * the ctx stream and accumulated per kernel kind. */
#define DTC_KERNEL_LO_PASS 0   /* fused RZZ+RZ diagonal + low-site kick pass */
#define DTC_KERNEL_HI_PASS 1   /* high-site kick pass                        */
#define DTC_KERNEL_REDUCE 2    /* per-state observable reduction             */
#define DTC_KERNEL_INIT 3      /* basis-state preparation                    */
#define DTC_KERNEL_FINAL_PASS 4 /* last pass of an echo chain: measure, no store */
#define DTC_KERNEL_EXCHANGE 5  /* virtual ranks' in-place slice exchange        */
#define DTC_KERNEL_KINDS 6
/* total_bytes = algorithmic HBM bytes of the launches: 32 B per amplitude for a
 * pass that reads and stores its state, 16 B for one that only reads
 * (measure-only) or only stores (the first pass of a sweep, which forms the
 * basis states in registers), 32 B per amplitude an exchange moves. */
int dtc_set_profiling(dtc_ctx* ctx, int32_t on);
int dtc_kernel_stats(dtc_ctx* ctx, int32_t kind, int64_t* launches,
                     double* total_ms, double* total_bytes);
int dtc_reset_stats(dtc_ctx* ctx);
/* Light-cone ends launched since dtc_open, by kernel: counts[0] the 8-site
 * window (dtc_lc_final*), [1] the 10-site window's generic kernel
 * (dtc_lcw_final), [2] its three-re-layout C2 form (dtc_lcw2_final), [3] the
 * 12-site window (dtc_lcw3_final, six passes merged; ABI 10).
 * Independent of profiling; lets tests assert which kernel a sweep ran. */
int dtc_lightcone_counts(dtc_ctx* ctx, int64_t* counts /* [4] */);
/* Batch schedules built since dtc_open (ABI 12; test hook, no reference
 * counterpart): counts[0] echo chains whose first pass folded into the
 * forward's dual pass, [1] device-noise batches whose forward ran one kick
 * layer ahead (one pass per period), [2] device-noise batches run with K-D
 * forward passes (a chain did not fold, or DTC_NO_RUNAHEAD=1, the test switch
 * that forces this schedule; two passes per period), [3] batches run with the
 * 13 / 7 site split of L = 20 (a 13-site group in 8192-amplitude tiles, a
 * 7-site column group; opt-in with DTC_SPLIT13=1, the default keeps the
 * 12 / 8 split). */
int dtc_schedule_counts(dtc_ctx* ctx, int64_t* counts /* [4] */);

/* Device properties for reports. */
int dtc_device_info(dtc_ctx* ctx, char* name, int32_t name_len, int32_t* n_cu,
                    double* hbm_bytes);

#ifdef __cplusplus
}
#endif
#endif /* DTC_H */
