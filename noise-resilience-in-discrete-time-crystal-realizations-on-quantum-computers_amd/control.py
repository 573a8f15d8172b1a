"""Adaptive-g controllers:
autocorr-delta-a-single-qiskit-fast-controlled-g.py ("ctrlg") and
autocorr-delta-a-single-qiskit-fast-g-optimization.py ("gopt").

Both scripts run, per disorder instance, a serial loop over t = 0..T-1
(ctrlg.py:423-532, gopt.py:497-623): the circuit at time t applies t+1
periods whose kicks use the g history g_0..g_t (controlled-g.py:196-241; the
echo walks the same g values in reverse), one 1024-shot forward and one echo
estimate are taken, and the next g comes from the echo value:

* feedback (ctrlg, gopt --use_optimization 0): linear
  ``g + gain (target - echo)`` or the exponential rule of
  ``calculate_exponential_g_adjustment`` (ctrlg.py:369-420), clipped to
  [g_min, g_max];
* optimisation (gopt --use_optimization 1, gopt.py:359-427): the next g
  minimises ``(echo(g_0..g_{t-1}, g) - target)^2`` with
  ``scipy.optimize.minimize_scalar(bounds=(g_min, g_max), method="bounded")``
  over a fresh echo estimate per evaluation (grid search over 10 points as
  the fallback when the optimiser reports failure).

Each estimate here is one engine call (dtc_autocorr with a per-period kick
table, t_offset = 1 and t_first = t: only point t is measured) over ``shots``
trajectories with the reference's shot estimator emulated (one trajectory +
one ancilla draw per shot), with an independent seed per call, as the
reference's circuits are independent runs.  The controller updates are
checked bit-for-bit against the reference's own g histories
(tests/test_control_cpu.py: autocorr_data_L4 realtime runs).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import numpy as np

from .engine import SweepSpec


@dataclass
class ControllerConfig:
    """ctrlg.py / gopt.py argparse (controlled-g.py:100-110, gopt.py:104-111)."""

    target_echo: float = 1.0
    feedback_gain: float = 0.01
    exponential_feedback: int = 1
    decay_compensation: float = 0.1
    g_min: float = 0.84
    g_max: float = 1.0
    use_optimization: int = 0
    optimization_iterations: int = 5  # accepted for fidelity; unused by the reference too
    # optimisation: build the t-period forward states once per t and run only
    # the candidate's last period + echo per evaluation (dtc_prefix_*); the
    # candidates then share the prefix's noise draws (common random numbers)
    prefix_cache: int = 1

    @property
    def method_suffix(self) -> str:
        if self.use_optimization:
            return f"_optimization_iter{self.optimization_iterations}"
        return f"_exp{self.decay_compensation}" if self.exponential_feedback else "_linear"

    @property
    def method_short(self) -> str:
        if self.use_optimization:
            return "optimization"
        return "exponential" if self.exponential_feedback else "linear"


# ---- feedback rules ---------------------------------------------------------------

def feedback_update(echo_val: float, current_g: float, t: int, cfg: ControllerConfig) -> float:
    """Next g from the echo estimate at time t (ctrlg.py:369-420)."""
    err = cfg.target_echo - echo_val
    if cfg.exponential_feedback:
        # time-growing gain plus a log-ratio term, both scaled by (1 + c t)
        grow = cfg.feedback_gain * err * np.exp(cfg.decay_compensation * t)
        if echo_val > 0.01:
            ratio = np.log(cfg.target_echo / echo_val) if echo_val < cfg.target_echo else 0
            log_term = cfg.feedback_gain * ratio * 0.1
        else:
            log_term = cfg.feedback_gain * 2.0
        step = (grow + log_term) * (1 + cfg.decay_compensation * t)
        new_g = current_g + step
    else:
        new_g = current_g + cfg.feedback_gain * err
    return float(np.clip(new_g, cfg.g_min, cfg.g_max))


def adjust_g_based_on_echo(echo_values, g_values, cfg: ControllerConfig):
    """Batch (non-realtime) rule of get_instances_adaptive (ctrlg.py:355-367):
    g_t += gain (target - echo_{t-1}) for t >= 1."""
    out = list(g_values)
    for t in range(1, len(echo_values)):
        out[t] = float(np.clip(g_values[t] + cfg.feedback_gain * (cfg.target_echo
                                                                  - echo_values[t - 1]),
                               cfg.g_min, cfg.g_max))
    return out


# ---- one estimate at time t ----------------------------------------------------------

@dataclass
class PointEstimator:
    """Estimates the forward / echo ancilla values at time t for a g history
    (t+1 periods, controlled-g.py:196-241) with the engine."""

    L: int
    hs: np.ndarray       # [L]
    phis: np.ndarray     # [L-1]
    noise_prob: float = 0.05
    use_noise: int = 1
    initial_state: str = "vacuum"
    shots: int = 1024
    seed: int = 0x5EED0001
    engine: object = None
    device: object = None  # DeviceNoise (use_fakebackend=1), or None
    calls: int = field(default=0)
    prefix_periods: int = field(default=0)  # > 0: a prefix of that many periods is built

    def _eng(self):
        if self.engine is None:
            from . import sweep

            self.engine = sweep._default_engine()
        return self.engine

    def _spec(self, g_list):
        return SweepSpec(L=self.L, T=len(g_list), hs=self.hs[None, :], phis=self.phis[None, :],
                         g=[float(x) for x in g_list], noise_prob=self.noise_prob,
                         use_noise=self.use_noise, initial_state=self.initial_state, t_offset=1,
                         device=self.device)

    def _n_traj(self, spec):
        return self.shots if (spec.p > 0 or self.device is not None) else 1

    def build_prefix(self, g_prefix):
        """Forward states after the len(g_prefix) periods every candidate of
        optimize_g shares (own seed, as one more independent run)."""
        spec = self._spec(g_prefix)
        ss = np.random.SeedSequence([self.seed & 0xFFFFFFFF, self.seed >> 32, self.calls])
        self.calls += 1
        s64 = int(ss.generate_state(1, dtype=np.uint64)[0])
        self._eng().prefix_build(spec, self._n_traj(spec), len(g_prefix), seed=s64)
        self.prefix_periods = len(g_prefix)

    def release_prefix(self):
        if self.prefix_periods:
            self._eng().prefix_release()
        self.prefix_periods = 0

    def __call__(self, g_list, want_fwd=True, want_echo=True):
        from .sweep import _shot_estimate

        t = len(g_list) - 1
        spec = self._spec(g_list)
        ss = np.random.SeedSequence([self.seed & 0xFFFFFFFF, self.seed >> 32, self.calls])
        self.calls += 1
        s64 = int(ss.generate_state(1, dtype=np.uint64)[0])
        n_traj = self._n_traj(spec)
        if self.prefix_periods and self.prefix_periods == t:
            # the prefix holds periods 1..t: only period t+1 and the echo run
            out = self._eng().autocorr_prefixed(spec, n_traj, seed=s64, want_fwd=want_fwd,
                                                want_echo=want_echo, t_first=t)
        else:
            out = self._eng().autocorr(spec, n_traj, seed=s64, want_fwd=want_fwd,
                                       want_echo=want_echo, t_first=t)
        rng = np.random.default_rng(ss.spawn(1)[0])
        res = []
        for key, want in (("fwd", want_fwd), ("echo", want_echo)):
            if not want:
                res.append(None)
                continue
            a = out[key][:, :, t:t + 1]
            if not self.shots:
                res.append(float(a.mean()))
            elif self.device is not None:
                # importance-weighted trajectories are not per-shot probabilities:
                # the shots are drawn from the trajectory mean (as sweep.run_sweep)
                m = min(1.0, max(0.0, (1.0 + float(a.mean())) / 2.0))
                res.append((2.0 * rng.binomial(self.shots, m) - self.shots) / self.shots)
            else:
                res.append(float(_shot_estimate(a, self.shots, rng)[0, 0]))
        return tuple(res)


def optimize_g(est: PointEstimator, g_prefix, cfg: ControllerConfig) -> float:
    """gopt.py:359-427: bounded Brent on the squared echo distance, grid
    search fallback.  With ``cfg.prefix_cache`` every evaluation continues
    from the shared forward states of g_prefix (one period + the echo each)."""
    from scipy.optimize import minimize_scalar

    use_prefix = bool(cfg.prefix_cache) and len(g_prefix) > 0 and hasattr(est._eng(),
                                                                          "prefix_build")
    if use_prefix:
        est.build_prefix(g_prefix)
    try:
        def objective(gc):
            return (est(list(g_prefix) + [gc], want_fwd=False)[1] - cfg.target_echo) ** 2

        r = minimize_scalar(objective, bounds=(cfg.g_min, cfg.g_max), method="bounded")
        if r.success:
            return float(r.x)
        best, best_d = cfg.g_min, float("inf")
        for gc in np.linspace(cfg.g_min, cfg.g_max, 10):
            d = abs(est(list(g_prefix) + [gc], want_fwd=False)[1] - cfg.target_echo)
            if d < best_d:
                best, best_d = float(gc), d
        return best
    finally:
        if use_prefix:
            est.release_prefix()


# ---- the realtime loop --------------------------------------------------------------

@dataclass
class AdaptiveResult:
    forward: np.ndarray   # [inst][T]
    echo: np.ndarray      # [inst][T]
    g: np.ndarray         # [inst][T]


def realtime_adaptive(L, T, hs, phis, g_initial, cfg: ControllerConfig, noise_prob=0.05,
                      use_noise=1, initial_state="vacuum", shots=1024, seed=0x5EED0001,
                      engine=None, log=None, device=None) -> AdaptiveResult:
    """get_instances_adaptive_realtime (ctrlg.py:423-532, gopt.py:497-623).
    ``device``: DeviceNoise for ``--use_fakebackend 1`` (ctrlg.py:246-250)."""
    hs = np.atleast_2d(hs)
    phis = np.atleast_2d(phis)
    n_inst = hs.shape[0]
    fw = np.zeros((n_inst, T))
    ec = np.zeros((n_inst, T))
    gs = np.zeros((n_inst, T))
    for i in range(n_inst):
        est = PointEstimator(L, hs[i, :L], phis[i, :L - 1], noise_prob, use_noise, initial_state,
                             shots, seed + 7919 * i, engine, device)
        hist = []
        g = float(g_initial)
        for t in range(T):
            hist.append(g)
            f, e = est(hist)
            fw[i, t], ec[i, t], gs[i, t] = f, e, g
            if log:
                log(f"inst {i + 1} t {t:2d}: g={g:.4f} fwd={f:.4f} echo={e:.4f}")
            if t < T - 1:
                g = optimize_g(est, hist[:-1], cfg) if cfg.use_optimization else \
                    feedback_update(e, g, t, cfg)
    return AdaptiveResult(fw, ec, gs)


def fixed_g_sweep(L, T, hs, phis, g, noise_prob=0.05, use_noise=1, initial_state="vacuum",
                  shots=1024, seed=0x5EED0001, engine=None, device=None):
    """get_instances with a fixed g (ctrlg.py:583-601): all t in one engine
    sweep, t+1 periods at time t.  Returns (forward, echo), each [inst][T]."""
    from . import sweep as sw

    spec = SweepSpec(L=L, T=T, hs=np.atleast_2d(hs), phis=np.atleast_2d(phis), g=float(g),
                     noise_prob=noise_prob, use_noise=use_noise, initial_state=initial_state,
                     t_offset=1, device=device)
    noisy = spec.p > 0 or device is not None
    r = sw.run_sweep(spec, shots=shots if noisy else None, engine=engine, seed=seed)
    return r.fwd, r.echo


# ---- output files (ctrlg.py:640-737, gopt.py:740-836) ----------------------------------

def controlled_folder(L):
    return f"controlled-autocorr_data_L{L}"


def write_controlled_outputs(out_dir, state, L, inst, g_initial, cfg: ControllerConfig,
                             adaptive: AdaptiveResult, std84, std97, name_args,
                             optimization_script=False):
    """The two CSVs of the scripts.  ``std84``/``std97`` = (forward, echo) of the
    fixed-g comparisons; ``name_args`` = (randomphi, delta, amplitude, noise, use_noise)."""
    import pandas as pd

    from .envelopes import EnvelopeUnavailable, find_envelope

    T = adaptive.g.shape[1]
    ts = np.arange(T)
    av = {
        "adaptive_f": adaptive.forward.mean(axis=0), "adaptive_e": adaptive.echo.mean(axis=0),
        "g84_f": std84[0].mean(axis=0), "g84_e": std84[1].mean(axis=0),
        "g97_f": std97[0].mean(axis=0), "g97_e": std97[1].mean(axis=0),
    }
    av_g = adaptive.g.mean(axis=0)
    data = {
        "time": ts,
        "av_autocorr_adaptive": av["adaptive_f"],
        "av_autocorr_echo_adaptive": av["adaptive_e"],
        "av_g_values": av_g,
        "av_autocorr_standard_g84": av["g84_f"],
        "av_autocorr_echo_standard_g84": av["g84_e"],
        "av_autocorr_standard_g97": av["g97_f"],
        "av_autocorr_echo_standard_g97": av["g97_e"],
        "sqrt_av_autocorr_echo_adaptive": np.sqrt(np.abs(av["adaptive_e"])),
        "sqrt_av_autocorr_echo_standard_g84": np.sqrt(np.abs(av["g84_e"])),
        "sqrt_av_autocorr_echo_standard_g97": np.sqrt(np.abs(av["g97_e"])),
    }
    try:
        env = {}
        for tag in ("adaptive", "g84", "g97"):
            for kind, key in (("forward", "f"), ("echo", "e")):
                env[(tag, kind)] = find_envelope(av[f"{tag}_{key}"], 3, "controlled")
        for kind in ("forward", "echo"):
            for tag in ("adaptive", "g84", "g97"):
                up, lo = env[(tag, kind)]
                data[f"upper_env_{tag}_{kind}"] = up
                data[f"lower_env_{tag}_{kind}"] = lo
    except EnvelopeUnavailable:
        pass
    for i in range(inst):
        data[f"g_history_inst{i + 1}"] = adaptive.g[i]
        data[f"echo_adaptive_inst{i + 1}"] = adaptive.echo[i]
        data[f"forward_adaptive_inst{i + 1}"] = adaptive.forward[i]
        data[f"echo_standard_g84_inst{i + 1}"] = std84[1][i]
        data[f"forward_standard_g84_inst{i + 1}"] = std84[0][i]
        data[f"echo_standard_g97_inst{i + 1}"] = std97[1][i]
        data[f"forward_standard_g97_inst{i + 1}"] = std97[0][i]
    randomphi, delta, amplitude, noise, use_noise = name_args
    folder = os.path.join(out_dir, controlled_folder(L))
    os.makedirs(folder, exist_ok=True)
    name = (f"autocorr_data_{state}_realtime_adaptive{cfg.method_suffix}_g{g_initial}_L{L}"
            f"_inst{inst}_randomphi{randomphi}_delta{delta}_amplitude{amplitude}_noise{noise}"
            f"_usenoise{use_noise}_target{cfg.target_echo}_gain{cfg.feedback_gain}.csv")
    main_path = os.path.join(folder, name)
    pd.DataFrame(data).to_csv(main_path, index=False)

    comp = {
        "time": ts, "av_g_values": av_g,
        "av_echo_adaptive": av["adaptive_e"], "av_echo_g84": av["g84_e"],
        "av_echo_g97": av["g97_e"], "av_forward_adaptive": av["adaptive_f"],
        "av_forward_g84": av["g84_f"], "av_forward_g97": av["g97_f"],
    }
    for i in range(inst):
        comp[f"inst{i + 1}_g_values"] = adaptive.g[i]
        comp[f"inst{i + 1}_echo_adaptive"] = adaptive.echo[i]
        comp[f"inst{i + 1}_echo_g84"] = std84[1][i]
        comp[f"inst{i + 1}_echo_g97"] = std97[1][i]
    method = f"_{cfg.method_short}" if optimization_script else ""
    comp_name = (f"comparison_{state}_adaptive{method}_vs_fixed_g{g_initial}_L{L}_inst{inst}"
                 f"_target{cfg.target_echo}_gain{cfg.feedback_gain}.csv")
    comp_path = os.path.join(folder, comp_name)
    pd.DataFrame(comp).to_csv(comp_path, index=False)
    return main_path, comp_path
