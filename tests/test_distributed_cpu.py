"""N>1 path on CPU: world_size-2 gloo, trajectories sharded by global id and
gathered once; the gathered per-trajectory values (computed here by the C
oracle standing in for the engine, which needs a GPU) are bit-identical to a
single-process run, as are the per-t means."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _spec(pkg):
    rng = np.random.default_rng(9)
    L = 6
    hs = rng.uniform(-np.pi, np.pi, (2, L))
    ph = rng.uniform(-1.5 * np.pi, -0.5 * np.pi, (2, L - 1))
    return pkg.SweepSpec(L=L, T=5, hs=hs, phis=ph, g=0.95, noise_prob=0.1,
                         initial_state="neel")


def _worker(rank, world, port, n_traj, q):
    import sys

    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    from __graft_entry__ import load_package
    from oracle import c_oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pkg = load_package()
    spec = _spec(pkg)

    def compute(lo, hi):
        return c_oracle.autocorr(spec, hi - lo, seed=77, traj_offset=lo, n_threads=1)

    full = pkg.distributed.sharded_values(compute, n_traj, world, rank)
    if rank == 0:
        q.put({k: v for k, v in full.items()})
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n_traj", [(2, 9), (3, 8)])
def test_sharded_gather_bit_identical(pkg, world, n_traj):
    from oracle import c_oracle

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_traj, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    ref = c_oracle.autocorr(_spec(pkg), n_traj, seed=77, traj_offset=0, n_threads=1)
    for k in ("fwd", "echo"):
        assert got[k].shape == ref[k].shape
        assert np.array_equal(got[k], ref[k])
        assert np.array_equal(got[k].mean(axis=1), ref[k].mean(axis=1))


class _OracleEngine:
    """The C oracle behind DtcEngine.autocorr's signature (the engine needs a GPU)."""

    def autocorr(self, spec, n_traj, seed=0x5EED0001, traj_offset=0, want_fwd=True,
                 want_echo=True, want_zsite=False, batch=0, t_first=0):
        from oracle import c_oracle

        return c_oracle.autocorr(spec, n_traj, seed=seed, traj_offset=traj_offset,
                                 want_fwd=want_fwd, want_echo=want_echo, want_zsite=want_zsite,
                                 n_threads=1, t_first=t_first)


def test_independent_t_points_are_their_own_trajectories(pkg):
    """--independent_t (the reference's fresh circuit per t, fast.py:219-221):
    point t is the standard sweep's point t under its own key point_seed(77, t)
    (forward noise of periods 1..t and echo stream 1+t are those trajectories'),
    so the points share no noise draw across t; noiseless, it is the standard
    sweep exactly."""
    from oracle import c_oracle

    spec = _spec(pkg)
    n = 3
    eng = _OracleEngine()
    got = pkg.sweep.autocorr_independent_t(eng, spec, n, seed=77)
    keys = {pkg.sweep.point_seed(77, t) for t in range(spec.T)}
    assert len(keys) == spec.T and 77 not in keys
    for t in range(spec.T):
        ref = c_oracle.autocorr(spec, n, seed=pkg.sweep.point_seed(77, t), n_threads=1)
        for k in ("fwd", "echo"):
            assert np.abs(got[k][:, :, t] - ref[k][:, :, t]).max() < 1e-12, (k, t)
    # chunks split by trajectory offset compose to the single call (ADVICE r3:
    # the old t * n_total + lo ids made chunk 2's point 0 reuse chunk 1's point 1)
    a = pkg.sweep.autocorr_independent_t(eng, spec, 2, seed=77)
    b = pkg.sweep.autocorr_independent_t(eng, spec, 1, seed=77, lo=2)
    for k in ("fwd", "echo"):
        assert np.array_equal(np.concatenate([a[k], b[k]], axis=1), got[k])
    with pytest.raises(ValueError):
        pkg.sweep.run_sweep(spec, n_traj=1, engine=eng, independent_t=True, want_zsite=True)
    ideal = pkg.SweepSpec(L=spec.L, T=spec.T, hs=spec.hs, phis=spec.phis, g=0.95, use_noise=0,
                          initial_state="neel")
    a = pkg.sweep.run_sweep(ideal, n_traj=1, engine=eng, independent_t=True)
    b = pkg.sweep.run_sweep(ideal, n_traj=1, engine=eng)
    assert np.abs(a.fwd - b.fwd).max() < 1e-12 and np.abs(a.echo - b.echo).max() < 1e-12


def _indep_worker(rank, world, port, n_traj, q):
    import sys

    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    from __graft_entry__ import load_package

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pkg = load_package()
    res = pkg.distributed.sharded_sweep(_spec(pkg), n_traj, shots=None, seed=77,
                                        engine=_OracleEngine(), independent_t=True)
    if rank == 0:
        q.put({"fwd": res.fwd_traj, "echo": res.echo_traj})
    dist.barrier()
    dist.destroy_process_group()


def test_independent_t_sharded_bit_identical(pkg):
    """The independent-per-t mode sharded over 2 gloo ranks by trajectory
    blocks gives the single-process per-trajectory values bit for bit."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    n_traj = 5
    procs = [ctx.Process(target=_indep_worker, args=(r, 2, port, n_traj, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    ref = pkg.sweep.autocorr_independent_t(_OracleEngine(), _spec(pkg), n_traj, seed=77)
    for k in ("fwd", "echo"):
        assert np.array_equal(got[k], ref[k])
