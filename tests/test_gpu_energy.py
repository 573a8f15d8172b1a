"""dtc_energy (HIP) vs the per-trajectory oracle (oracle/energy_oracle.py: the C
oracle's periods + numpy observables): <Z_i>, <Z_i Z_i+1>, <X_i> per
trajectory to 1e-10; the trajectory mean vs the exact density matrix."""
import numpy as np
import pytest

from oracle import dm_oracle, energy_oracle
from tests.helpers import harsh_device, random_disorder

pytestmark = pytest.mark.gpu
TOL = 1e-10


@pytest.mark.parametrize("L,T,p,state,pol", [
    (4, 8, 0.05, "vacuum", "x"),
    (5, 8, 0.05, "neel", "x"),
    (7, 6, 0.1, "neel", "circular_left"),
    (7, 6, 0.1, "vacuum", "circular_left"),
    (13, 5, 0.05, "neel", "xy"),
    (14, 5, 0.05, "vacuum", "x"),
    (17, 4, 0.02, "neel", "y"),
])
def test_energy_matches_oracle(pkg, engine, L, T, p, state, pol):
    """neel = the energy scripts' preparation (sites 2, 4, .., L-1; odd L)."""
    rng = np.random.default_rng(L + 100)
    hs, phis = random_disorder(rng, L, 2)
    spec = pkg.energy.energy_spec(L, T, hs, phis, 0.94, state, noise_prob=p, polarization=pol)
    got = engine.energy(spec, 3, seed=21)
    for inst in range(2):
        for tr in range(3):
            z, zz, x = energy_oracle.trajectory_energy(spec, inst, tr, seed=21)
            assert np.abs(got["z"][inst, tr] - z).max() < TOL
            assert np.abs(got["zz"][inst, tr] - zz).max() < TOL
            assert np.abs(got["x"][inst, tr] - x).max() < TOL


@pytest.mark.parametrize("L,state,pol", [(21, "neel", "x"), (20, "vacuum", "x"),
                                         (24, "vacuum", "y")])
def test_energy_large_matches_oracle(pkg, engine, L, state, pol):
    """Two site groups (L=20/21: sites 0-11 | 12-..) and three (L=24): every
    group's <X_i> comes from a different pass (mid-pass or next-pass entry)."""
    rng = np.random.default_rng(L + 7)
    hs, phis = random_disorder(rng, L)
    spec = pkg.energy.energy_spec(L, 3, hs, phis, 0.93, state, noise_prob=0.05, polarization=pol)
    got = engine.energy(spec, 2, seed=5)
    for tr in range(2):
        z, zz, x = energy_oracle.trajectory_energy(spec, 0, tr, seed=5)
        assert np.abs(got["z"][0, tr] - z).max() < TOL
        assert np.abs(got["zz"][0, tr] - zz).max() < TOL
        assert np.abs(got["x"][0, tr] - x).max() < TOL


def test_energy_t_offset_and_batches(pkg, engine):
    """t_offset=1 (first row after one period) and a batch split: the same
    per-trajectory values as one batch from t_offset 0 shifted by one."""
    rng = np.random.default_rng(3)
    L = 13
    hs, phis = random_disorder(rng, L)
    base = pkg.SweepSpec(L=L, T=5, hs=hs, phis=phis, g=0.95, noise_prob=0.05)
    off = pkg.SweepSpec(L=L, T=4, hs=hs, phis=phis, g=0.95, noise_prob=0.05, t_offset=1)
    a = engine.energy(base, 5, seed=9)
    b = engine.energy(off, 5, seed=9, batch=2)
    for k in ("z", "zz", "x"):
        assert np.abs(a[k][:, :, 1:] - b[k]).max() < TOL, k


def test_energy_mean_vs_density_matrix(pkg, engine):
    rng = np.random.default_rng(8)
    L, T, p, n = 4, 10, 0.1, 4096
    hs, phis = random_disorder(rng, L)
    spec = pkg.SweepSpec(L=L, T=T, hs=hs, phis=phis, g=0.97, noise_prob=p)
    got = engine.energy(spec, n, seed=3)
    exact = dm_oracle.energy_sweep(L, T, hs[0], phis[0], spec.kick, p)
    for k, key in enumerate(("z", "zz", "x")):
        v = got[key][0]
        mean, sd = v.mean(axis=0), v.std(axis=0) / np.sqrt(n) + 1e-12
        assert np.all(np.abs(mean - exact[k]) < 5 * sd), key
    e = pkg.energy.get_instances_energy(spec, 256, engine=engine)["full"]
    assert e.shape == (1, T)


@pytest.mark.parametrize("mode,cols", [
    ("full", ["time", "energy_p_0", "energy_p_0.001", "energy_p_0.01", "energy_p_0.1"]),
    ("ham-comparison", ["time", "energy_z_only_p_0.05", "energy_zz_only_p_0.05",
                        "energy_x_only_p_0.05", "energy_sum_p_0.05", "energy_full_p_0.05"]),
    ("vs-echo", ["time", "energy_with_x_p_0.1", "energy_without_x_p_0.1"]),
])
def test_energy_cli_files(pkg, golden, tmp_path, mode, cols):
    import os

    import pandas as pd

    d = golden["disorder"]["L4"]
    dis = tmp_path / "dis"
    dis.mkdir()
    pd.DataFrame(d["hs"]).to_csv(dis / "hs_L4.csv", index=False)
    pd.DataFrame(d["phis"]).to_csv(dis / "phis_L4.csv", index=False)
    out = tmp_path / "out"
    rc = pkg.energy_cli.main(["--mode", mode, "--L", "4", "--tf", "6", "--trajectories", "128",
                              "--disorder_folder", str(dis), "--out_dir", str(out)])
    assert rc == 0
    files = [os.path.join(r, f) for r, _, fs in os.walk(out) for f in fs]
    main = [f for f in files if not os.path.basename(f).startswith("comprehensive")]
    assert len(main) == 1
    df = pd.read_csv(main[0])
    assert list(df.columns) == cols and len(df) == 6
    if mode == "vs-echo":
        # vs-echo.py:436-448 without an autocorr CSV next to it (and its default
        # --use_fakebackend 1: device-like noise from the stand-in calibration)
        comp = [f for f in files if os.path.basename(f).startswith("comprehensive_data_energy_only")]
        assert len(comp) == 1
        c = pd.read_csv(comp[0])
        assert list(c.columns) == ["time", "energy_with_x", "energy_without_x"]
        assert np.allclose(c["energy_with_x"], df["energy_with_x_p_0.1"])
    else:
        assert len(files) == 1
    if mode == "full":
        # t = 0: <H>/L of the vacuum = (sum h_i + sum phi_i) / L  (X terms vanish)
        hs, phis = pkg.load_disorder(4, 1, str(dis))
        assert abs(df["energy_p_0"][0] - (hs[0].sum() + phis[0].sum()) / 4) < 1e-12


@pytest.mark.parametrize("L", [5, 7])
def test_energy_neel_mean_vs_density_matrix(pkg, engine, L):
    """The energy scripts' neel state at odd L: engine trajectory means vs the
    exact density matrix of the L-qubit energy circuit."""
    rng = np.random.default_rng(40 + L)
    T, p, n = 6, 0.08, 4096
    hs, phis = random_disorder(rng, L)
    spec = pkg.energy.energy_spec(L, T, hs, phis, 0.96, "neel", noise_prob=p)
    got = engine.energy(spec, n, seed=17)
    exact = dm_oracle.energy_sweep(L, T, hs[0], phis[0], spec.kick, p, "neel")
    for k, key in enumerate(("z", "zz", "x")):
        v = got[key][0]
        mean, sd = v.mean(axis=0), v.std(axis=0) / np.sqrt(n) + 1e-12
        assert np.all(np.abs(mean - exact[k]) < 5 * sd), key


@pytest.mark.parametrize("L,T,n_inst,n_traj,batch,state,toff,device", [
    (5, 6, 2, 7, 0, "neel", 0, False),      # instances in one batch
    (14, 5, 3, 5, 4, "vacuum", 0, False),    # batches that split instances
    (20, 4, 1, 24, 16, "vacuum", 1, False),  # octet layout, t_offset = 1
    (7, 5, 2, 6, 5, "neel", 0, True),        # device-like noise
])
def test_energy_sums_match_trajectory_rows(pkg, engine, L, T, n_inst, n_traj, batch, state, toff,
                                           device):
    """dtc_energy_sums (the per-instance trajectory sums on the device) equals
    the host sums of dtc_energy's per-trajectory rows up to rounding, for any
    batching, and get_instances_energy (which now uses it) equals the means of
    those rows."""
    rng = np.random.default_rng(L * 3 + n_traj)
    hs, phis = random_disorder(rng, L, n_inst)
    kw = {"device": harsh_device(pkg, L)} if device else {"noise_prob": 0.05}
    spec = pkg.energy.energy_spec(L, T, hs, phis, 0.93, state, t_offset=toff, **kw)
    rows = engine.energy(spec, n_traj, seed=44, traj_offset=3)
    sums = engine.energy_sums(spec, n_traj, seed=44, traj_offset=3, batch=batch)
    for key in ("z", "zz", "x"):
        ref = rows[key].sum(axis=1)
        assert sums[key].shape == ref.shape
        assert np.abs(sums[key] - ref).max() < 1e-12 * n_traj, key
    e = pkg.energy.get_instances_energy(spec, n_traj, seed=44, engine=engine, traj_offset=3)["full"]
    means = {k: v.mean(axis=1) for k, v in rows.items()}
    ref_e = np.stack([pkg.energy.energy_from_observables({k: v[i] for k, v in means.items()}, L,
                                                         0.93, hs[i], phis[i], "full")
                      for i in range(n_inst)])
    assert np.abs(e - ref_e).max() < 1e-11
    # the previous estimator, pinned independently of the affinity the sums
    # rely on: <H> (and the read-out map) per trajectory row, then the mean
    # over trajectories
    readout = None
    if device:
        readout = (np.linspace(0.01, 0.04, L), np.linspace(0.03, 0.005, L))
    per_traj = []
    for i in range(n_inst):
        row = []
        for r in range(n_traj):
            o = {k: v[i, r] for k, v in rows.items()}
            if readout is not None:
                o = pkg.energy.readout_observables(o, *readout)
            row.append(pkg.energy.energy_from_observables(o, L, 0.93, hs[i], phis[i], "full"))
        per_traj.append(np.mean(row, axis=0))
    e_ro = pkg.energy.get_instances_energy(spec, n_traj, seed=44, engine=engine, traj_offset=3,
                                           readout=readout)["full"]
    assert np.abs(e_ro - np.stack(per_traj)).max() < 1e-11
