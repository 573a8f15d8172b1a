"""The sharded single-state path (sharded.py, config C5) on CPU: the sweep
driver with the numpy step (oracle/shard_oracle.py) in place of the engine,
virtual ranks in one process and real ranks over gloo (all_to_all_single),
against the whole-state C oracle per trajectory.  The engine's own step is
checked against dtc_autocorr on the GPU (tests/test_gpu_sharded.py)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from oracle import c_oracle
from oracle.shard_oracle import NumpyShardStepper
from tests.helpers import random_disorder

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _spec(pkg, L, T, p=0.1, state="neel", pol="circular_left", toff=0, seed=4):
    rng = np.random.default_rng(seed)
    hs, phis = random_disorder(rng, L, 2)
    return pkg.SweepSpec(L=L, T=T, hs=hs, phis=phis, g=0.91, noise_prob=p, polarization=pol,
                         initial_state=state, t_offset=toff)


def _halves(n):
    """Two site groups (as the engine has for 13 <= n <= 21): the post-kick of a
    period then covers only the top group and the next period's first step
    kicks the rest."""
    lo = (1 << (n // 2)) - 1
    return [lo, ((1 << n) - 1) ^ lo]


def test_plan_groups_partition(pkg):
    for n in (12, 13, 20, 21, 22, 28, 31, 32):
        gs = pkg._capi.plan_groups(n)
        acc = 0
        for g in gs:
            assert acc & g == 0
            acc |= g
        assert acc == (1 << n) - 1
    assert len(pkg._capi.plan_groups(20)) == 2
    assert len(pkg._capi.plan_groups(31)) == 4


def test_layout_exchange_roundtrip(pkg):
    sh = pkg.sharded
    lay = sh.initial_layout(10, 2)
    y = lay.exchanged()
    assert y.site_of[6:8] == (8, 9) and y.site_of[8:10] == (6, 7)
    assert y.exchanged() == lay
    with pytest.raises(ValueError):
        sh.initial_layout(5, 2)


@pytest.mark.parametrize("L,k,T,p,state,pol,toff", [
    (6, 1, 6, 0.0, "vacuum", "x", 0),
    (7, 2, 6, 0.1, "neel", "circular_left", 0),
    (9, 3, 5, 0.05, "neel", "xy", 1),
])
@pytest.mark.parametrize("groups", [None, _halves])
def test_virtual_ranks_match_oracle(pkg, L, k, T, p, state, pol, toff, groups):
    spec = _spec(pkg, L, T, p, state, pol, toff)
    for traj in (0, 3):
        got = pkg.sharded.sharded_forward(NumpyShardStepper(groups), spec, k, inst=1,
                                          traj=traj, seed=99)
        # the whole-state oracle for instance 1, trajectory traj
        import dataclasses
        one = dataclasses.replace(spec, hs=spec.hs[1:2], phis=spec.phis[1:2])
        ref = c_oracle.autocorr(one, 1, seed=99, traj_offset=traj, want_zsite=True,
                                want_echo=False)
        assert np.abs(got["zsite"] - ref["zsite"][0, 0]).max() < 1e-12
        assert np.abs(got["fwd"] - ref["fwd"][0, 0]).max() < 1e-12
        assert np.abs(got["norm"] - 1.0).max() < 1e-12


@pytest.mark.parametrize("L,k,T,p,state,pol,toff", [
    (6, 1, 6, 0.0, "vacuum", "x", 0),
    (7, 2, 6, 0.1, "neel", "circular_left", 0),
    (9, 3, 5, 0.05, "neel", "xy", 1),
    (10, 2, 4, 0.1, "vacuum", "x", 0),    # 4 slices per chunk
    (11, 1, 4, 0.05, "neel", "y", 0),     # 8 slices per chunk
])
@pytest.mark.parametrize("groups", [None, _halves])
def test_pipelined_virtual_ranks_match_oracle(pkg, L, k, T, p, state, pol, toff, groups):
    """The chunk-pipelined driver (kicks per destination chunk, transfers per
    chunk, device observables) gives the same per-site <Z_i(t)> as the
    whole-state oracle."""
    spec = _spec(pkg, L, T, p, state, pol, toff)
    import dataclasses
    for traj in (0, 3):
        got = pkg.sharded.sharded_forward_pipelined(NumpyShardStepper(groups), spec, k, inst=1,
                                                    traj=traj, seed=99)
        one = dataclasses.replace(spec, hs=spec.hs[1:2], phis=spec.phis[1:2])
        ref = c_oracle.autocorr(one, 1, seed=99, traj_offset=traj, want_zsite=True,
                                want_echo=False)
        assert np.abs(got["zsite"] - ref["zsite"][0, 0]).max() < 1e-12
        assert np.abs(got["fwd"] - ref["fwd"][0, 0]).max() < 1e-12


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, k, q, pipelined=False, L=8):
    import sys

    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    from __graft_entry__ import load_package

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pkg = load_package()
    spec = _spec(pkg, L, 5)
    fwd = pkg.sharded.sharded_forward_pipelined if pipelined else pkg.sharded.sharded_forward
    out = fwd(NumpyShardStepper(_halves), spec, k, inst=0, traj=2, seed=5, rank=rank,
              world=world)
    if rank == 0:
        q.put(out["zsite"])
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("k,pipelined,L", [(1, False, 8), (2, False, 8), (1, True, 8),
                                           (2, True, 8), (3, True, 10)])
def test_gloo_ranks_match_oracle(pkg, k, pipelined, L):
    """Real ranks over gloo: the all_to_all_single exchange, and the pipelined
    driver's per-chunk point-to-point transfers (rank r sends chunk r+i to rank
    r+i at step i).  World 8 is the C5 rank count: 7 peers at once per slice."""
    world = 1 << k
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, k, q, pipelined, L))
             for r in range(world)]
    for pr in procs:
        pr.start()
    got = q.get(timeout=180)
    for pr in procs:
        pr.join(timeout=180)
        assert pr.exitcode == 0
    import dataclasses
    spec = _spec(pkg, L, 5)
    one = dataclasses.replace(spec, hs=spec.hs[:1], phis=spec.phis[:1])
    ref = c_oracle.autocorr(one, 1, seed=5, traj_offset=2, want_zsite=True, want_echo=False)
    assert np.abs(got - ref["zsite"][0, 0]).max() < 1e-12


@pytest.mark.parametrize("L,k,T,p,state,pol,toff", [
    (7, 2, 6, 0.1, "neel", "circular_left", 0),
    (9, 3, 5, 0.05, "neel", "xy", 1),
    (10, 2, 4, 0.1, "vacuum", "x", 0),    # 4 slices per chunk
    (11, 1, 4, 0.05, "neel", "y", 0),     # 8 slices per chunk
])
@pytest.mark.parametrize("groups", [None, _halves])
def test_pipelined_inplace_virtual_ranks_match_oracle(pkg, L, k, T, p, state, pol, toff, groups):
    """The one-buffer variant (inplace=True: each slice's exchange swaps the
    pieces (r, c) <-> (c, r) in place, dtc_shard_exchange_slice's semantics)
    gives the whole-state oracle's per-site <Z_i(t)> -- the path that runs
    C5's L=34 layout on one GPU."""
    import dataclasses
    spec = _spec(pkg, L, T, p, state, pol, toff)
    for traj in (0, 3):
        got = pkg.sharded.sharded_forward_pipelined(NumpyShardStepper(groups), spec, k, inst=1,
                                                    traj=traj, seed=99, inplace=True)
        one = dataclasses.replace(spec, hs=spec.hs[1:2], phis=spec.phis[1:2])
        ref = c_oracle.autocorr(one, 1, seed=99, traj_offset=traj, want_zsite=True,
                                want_echo=False)
        assert np.abs(got["zsite"] - ref["zsite"][0, 0]).max() < 1e-12
        assert np.abs(got["norm"] - 1.0).max() < 1e-12


def test_inplace_exchange_is_the_all_to_all(pkg):
    """Swapping every slice in place equals the two-buffer virtual exchange
    (dst[r][c] = src[c][r]), and a second exchange restores the state."""
    import torch

    lay = pkg.sharded.initial_layout(9, 2, 0, 4)
    x = torch.randn(4 << 7, dtype=torch.complex128)
    ref = torch.empty_like(x)
    pkg.sharded.virtual_exchange(x, ref, 4)
    y = x.clone()
    st = NumpyShardStepper()
    for s in range(4):
        st.exchange_slice(lay, 2, s, y)
    assert torch.equal(y, ref)
    for s in range(4):
        st.exchange_slice(lay, 2, s, y)
    assert torch.equal(y, x)
    with pytest.raises(ValueError):
        pkg.sharded.sharded_forward_pipelined(st, _spec(pkg, 9, 3), 2, world=4, inplace=True)


@pytest.mark.parametrize("W", [2, 4, 8])
def test_slice_p2p_plan_pairs_every_send_with_a_receive(pkg, W):
    """The real-rank op list (sharded.slice_p2p_plan): at every step each
    rank sends to one peer and receives from one, every peer exactly once per
    slice, and rank r's send at step i is the receive its peer posts at step
    i (so the batched point-to-point ops of the 8-GPU exchange match up)."""
    plans = {r: pkg.sharded.slice_p2p_plan(r, W) for r in range(W)}
    for r, ops in plans.items():
        assert len(ops) == 2 * (W - 1)
        sends = [(peer, chunk) for kind, peer, chunk in ops if kind == "isend"]
        recvs = [(peer, chunk) for kind, peer, chunk in ops if kind == "irecv"]
        assert sorted(p for p, _ in sends) == sorted(set(range(W)) - {r})
        assert sorted(p for p, _ in recvs) == sorted(set(range(W)) - {r})
        assert all(p == c for p, c in sends)      # chunk d goes to rank d
        assert all(p == c for p, c in recvs)      # rank q's piece lands in slot q
        for i, ((_, d, _), (_, q, _)) in enumerate(zip(ops[0::2], ops[1::2])):
            partner = plans[d][2 * i + 1]          # d's receive at the same step
            assert partner[:2] == ("irecv", r)
            assert plans[q][2 * i][:2] == ("isend", r)


def _exchange_worker(rank, world, port, S, q):
    import sys

    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    from __graft_entry__ import load_package

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pkg = load_package()
    n = 16  # amplitudes per (chunk, slice) piece
    # piece (chunk c, slice s) of rank r holds the value r + 100 c + 10000 s + j / 64
    j = torch.arange(n, dtype=torch.float64) / 64
    src = torch.zeros(world * S * n, dtype=torch.complex128)
    sv = src.view(world, S, n)
    for c in range(world):
        for s in range(S):
            sv[c, s] = (rank + 100 * c + 10000 * s + j).to(torch.complex128)
    dst = torch.full_like(src, -1.0)
    xch = pkg.sharded._SliceExchange(NumpyShardStepper(), world, S, rank, world, None)
    for s in range(S):
        xch.send(s, src, dst)
    xch.finish()
    dv = dst.view(world, S, n)
    ok = True
    for qq in range(world):
        for s in range(S):
            want = (qq + 100 * rank + 10000 * s + j).to(torch.complex128)
            ok &= bool(torch.equal(dv[qq, s], want))
    flag = torch.tensor([1.0 if ok else 0.0])
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if rank == 0:
        q.put(float(flag.item()))
    dist.destroy_process_group()


def test_gloo_world8_slice_exchange_delivers_every_piece(pkg):
    """World 8 (the C5 rank count) over gloo: the batched point-to-point ops
    built from slice_p2p_plan deliver slice s of chunk r of every rank q into
    slot q of rank r, for every slice -- the all-to-all, piece by piece."""
    world, S = 8, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exchange_worker, args=(r, world, port, S, q))
             for r in range(world)]
    for pr in procs:
        pr.start()
    got = q.get(timeout=180)
    for pr in procs:
        pr.join(timeout=180)
        assert pr.exitcode == 0
    assert got == 1.0
