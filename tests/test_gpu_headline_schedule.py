"""The headline bench line's exact schedule, per trajectory, against the oracle.

bench.py's C2 step (BASELINE.json configs[1]: L=20, g=0.97, tf=30, p=0.05,
vacuum, x kicks, hs/phis_L20 row 0, seed 0x5EED0001) runs 1024 trajectories per
launch with traj_offset = step * 1024.  At that size the engine runs every
schedule feature the line's throughput depends on at once: 29-period forward
chains, echo chains of 1..29 periods, the dual forward + echo-start pass
(dtc_kdk_dual) at every branch it fits, the 12-site light-cone end
(dtc_lcw3_final) on chains of 7..29 periods, the octet state layout filled at
B=1024, and RNG period counters up to 29 on trajectory ids past the first
batch.  The other parity tests stop at T <= 12 or resolve only ~1e-2 (the Aer
CSVs); here sampled trajectories -- ids at octet edges (7, 8), batch edges
(1023, 1024) and the second batch's last (2047) -- must equal the oracle to
1e-10 in fwd and echo at every t (reference: autocorr-delta-a-single-qiskit-
fast.py:217-239, the t loop; :140-147, the echo).

The oracle is orc_autocorr_fused, equal to the gate-by-gate oracle per
trajectory to 1e-12 (tests/test_oracle.py) and about 4 s per L=20, T=30
trajectory per host thread.
"""
import json
import os

import numpy as np
import pytest

from oracle import c_oracle

pytestmark = pytest.mark.gpu
TOL = 1e-10
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SEED = 0x5EED0001
B = 1024
# contiguous oracle ranges (OpenMP over trajectories) holding the sampled ids
RANGES = [(0, 9), (1020, 1028), (2040, 2048)]
SAMPLED = [0, 7, 8, 1023, 1024, 2047]


def _spec(pkg):
    with open(os.path.join(ROOT, "tests", "golden", "disorder.json")) as f:
        d = json.load(f)["L20"]
    hs, phis = np.array(d["hs"][:1]), np.array(d["phis"][:1])
    return pkg.SweepSpec(L=20, T=30, hs=hs, phis=phis, g=0.97, noise_prob=0.05, use_noise=1,
                         initial_state="vacuum")


def _free_device_memory(engine):
    """Earlier GPU tests leave large buffers behind (the shared engine's batch
    buffers, torch's cached blocks of the L=34 state): B=1024 L=20 states need
    32 GiB for F and E."""
    import torch

    engine.release_buffers()
    torch.cuda.empty_cache()


@pytest.fixture(scope="module")
def headline(pkg, engine):
    _free_device_memory(engine)
    spec = _spec(pkg)
    oracle = {}
    for lo, hi in RANGES:
        out = c_oracle.autocorr_fused(spec, hi - lo, seed=SEED, traj_offset=lo)
        for i in range(hi - lo):
            oracle[lo + i] = (out["fwd"][0, i], out["echo"][0, i])
    return spec, oracle


def _check(got, oracle, off, keys=("fwd", "echo"), t_first=0):
    for g in SAMPLED:
        if not off <= g < off + B:
            continue
        for k, ref in zip(("fwd", "echo"), oracle[g]):
            if k not in keys:
                continue
            err = float(np.abs(got[k][0, g - off, t_first:] - ref[t_first:]).max())
            assert err < TOL, (k, g, err)


def test_headline_schedule_matches_oracle(pkg, engine, headline):
    """Both batches of the bench's first two steps, as bench.py runs them: the
    sampled ids equal the oracle at 1e-10 (fwd and echo, t = 0..29); the
    12-site light-cone end and the dual pass both ran."""
    spec, oracle = headline
    with pkg.DtcEngine(0) as eng:
        eng.set_profiling(True)
        for off in (0, B):
            got = eng.autocorr(spec, B, seed=SEED, traj_offset=off, batch=B)
            _check(got, oracle, off)
            if off == 0:
                first = got
        counts = eng.lightcone_counts()
        lo = eng.kernel_stats()[pkg._capi.KERNEL_LO_PASS]
        eng.release_buffers()
    assert counts["lcw3"] > 0, counts
    # every echo chain of t >= 7 ends in the 12-site form (t = 7 .. 29 per batch)
    assert counts["lcw3"] >= 2 * 23, counts
    # the dual pass: fewer K-D-K launches than the unfused schedule
    os.environ["DTC_NO_DUAL"] = "1"
    try:
        with pkg.DtcEngine(0) as eng:
            eng.set_profiling(True)
            ref = eng.autocorr(spec, B, seed=SEED, traj_offset=0, batch=B)
            lo_ref = eng.kernel_stats()[pkg._capi.KERNEL_LO_PASS]
            eng.release_buffers()
    finally:
        del os.environ["DTC_NO_DUAL"]
    n_dual = lo_ref["launches"] - lo["launches"] // 2
    assert n_dual > 0, (lo, lo_ref)
    # a dual launch moves 48 B per amplitude, 16 fewer than its two passes
    assert lo["bytes"] / 2 == pytest.approx(lo_ref["bytes"] - n_dual * 16.0 * B * (1 << 20))
    assert np.abs(first["echo"] - ref["echo"]).max() < 1e-12
    assert np.abs(first["fwd"] - ref["fwd"]).max() < 1e-13


def test_headline_schedule_echo_only_and_t_first(pkg, engine, headline):
    """The same batch with the forward output off (echo only) and with
    t_first = 20 (the time points 20..29 only): the sampled ids still equal the
    oracle at 1e-10 on what each run computes."""
    spec, oracle = headline
    echo_only = engine.autocorr(spec, B, seed=SEED, traj_offset=B, batch=B, want_fwd=False)
    assert "fwd" not in echo_only or not np.any(echo_only["fwd"])
    _check(echo_only, oracle, B, keys=("echo",))
    late = engine.autocorr(spec, B, seed=SEED, traj_offset=0, batch=B, t_first=20)
    _check(late, oracle, 0, t_first=20)
    assert not np.any(late["echo"][..., :20])
    engine.release_buffers()


def test_c3_schedule_long_chains_match_oracle(pkg, engine):
    """bench.py --config c3 (BASELINE configs[2]'s device-like noise on the C2
    sweep: the stand-in calibration data/device_standin_L20.json, 1024
    trajectories per launch, traj_offset = step * 1024), both first batches:
    ids 7, 1023 and 1024 equal the gate-by-gate device oracle at 1e-10 on the
    longest echo chains (t = 26..29, the oracle run with t_first = 26 to bound
    its cost; the engine's values at t >= t_first do not depend on t_first),
    fwd and echo.  Exercises the run-ahead forward with the device K-D-K dual
    pass (dtc_kdk_dual; the K-D form dtc_kd_dual is the fallback schedule,
    test_gpu_device.py::test_device_kd_dual_forced) and the kick-only ends at
    the line's own batch: the run-ahead schedule must be the one that ran."""
    _free_device_memory(engine)
    spec = _spec(pkg)
    cal = pkg.DeviceCalibration.from_json(os.path.join(ROOT, "data", "device_standin_L20.json"))
    spec.device = cal.device_noise(20)
    from concurrent.futures import ThreadPoolExecutor

    ids = [7, 1023, 1024]

    def one(g):  # one oracle trajectory per host thread (ctypes drops the GIL)
        o = c_oracle.autocorr(spec, 1, seed=SEED, traj_offset=g, t_first=26)
        return o["fwd"][0, 0], o["echo"][0, 0]

    with ThreadPoolExecutor(len(ids)) as ex:
        ref = dict(zip(ids, ex.map(one, ids)))
    before = engine.schedule_counts()
    for off in (0, B):
        got = engine.autocorr(spec, B, seed=SEED, traj_offset=off, batch=B)
        for g in ids:
            if not off <= g < off + B:
                continue
            for k, r in zip(("fwd", "echo"), ref[g]):
                err = float(np.abs(got[k][0, g - off, 26:] - r[26:]).max())
                assert err < TOL, (k, g, err)
    after = engine.schedule_counts()
    assert after["device_runahead"] - before["device_runahead"] == 2, (before, after)
    assert after["device_kd"] == before["device_kd"], (before, after)
    engine.release_buffers()
