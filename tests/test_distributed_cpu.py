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
