"""The sharded single-state engine path (dtc_shard_*, sharded.py; config C5)
on one GPU with virtual ranks (all 2^k shards in one process, exchange = a
strided device copy) against the single-device engine (dtc_autocorr) on the
same trajectory: per-site <Z_i(t)> to 1e-10 — the engine's effective-field
diagonal tables, the bit-map-aware kicks and noise (RNG keyed by logical site)
and the Z bookkeeping of rank bits.  The L=34 / 8-rank run itself is the same
code with collective_exchange over RCCL (bench.py --config c5)."""
import dataclasses

import numpy as np
import pytest

from tests.helpers import random_disorder

pytestmark = pytest.mark.gpu
TOL = 1e-10


@pytest.fixture(scope="module")
def stepper(pkg, engine):
    return pkg.sharded.EngineStepper(engine)


@pytest.mark.parametrize("L,k,T,p,state,pol,toff", [
    (14, 1, 6, 0.0, "vacuum", "x", 0),
    (14, 2, 6, 0.1, "neel", "circular_left", 0),
    (15, 3, 5, 0.05, "neel", "xy", 1),
    (18, 2, 6, 0.05, "vacuum", "y", 0),
    (22, 3, 5, 0.05, "neel", "x", 0),
    (26, 3, 4, 0.0, "vacuum", "x", 0),
])
def test_virtual_shards_match_engine(pkg, engine, stepper, L, k, T, p, state, pol, toff):
    rng = np.random.default_rng(L * 7 + k)
    hs, phis = random_disorder(rng, L, 2)
    spec = pkg.SweepSpec(L=L, T=T, hs=hs, phis=phis, g=0.93, noise_prob=p, polarization=pol,
                         initial_state=state, t_offset=toff)
    one = dataclasses.replace(spec, hs=hs[1:2], phis=phis[1:2])
    for traj in (0, 5):
        got = pkg.sharded.sharded_forward(stepper, spec, k, inst=1, traj=traj, seed=77)
        ref = engine.autocorr(one, 1, seed=77, traj_offset=traj, want_echo=False,
                              want_zsite=True)
        assert np.abs(got["zsite"] - ref["zsite"][0, 0]).max() < TOL
        assert np.abs(got["fwd"] - ref["fwd"][0, 0]).max() < TOL
        assert np.abs(got["norm"] - 1.0).max() < 1e-10


def test_l30_eight_virtual_ranks(pkg, engine, stepper):
    """C5's layout (3 rank bits) at the largest size that also fits whole."""
    import os

    L = 30
    hs, phis = pkg.load_disorder(34, 1, os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "data"))
    spec = pkg.SweepSpec(L=L, T=4, hs=hs, phis=phis, g=0.97, use_noise=0)
    got = pkg.sharded.sharded_forward(stepper, spec, 3)
    ref = engine.autocorr(spec, 1, want_echo=False, want_zsite=True)
    assert np.abs(got["zsite"] - ref["zsite"][0, 0]).max() < TOL
    assert np.abs(got["zsite"][1] - np.cos(np.pi * 0.97)).max() < 1e-12


@pytest.mark.parametrize("L,k,T,p,state,pol,toff", [
    (14, 1, 6, 0.0, "vacuum", "x", 0),
    (15, 3, 5, 0.05, "neel", "xy", 1),
    (22, 3, 5, 0.05, "neel", "x", 0),
    (26, 2, 4, 0.1, "vacuum", "circular_left", 0),
])
def test_pipelined_virtual_shards_match_engine(pkg, engine, stepper, L, k, T, p, state, pol,
                                               toff):
    """The production C5 driver: per-slice kicks (dtc_shard_kick_slice), slice
    transfers on a side stream ordered by events, asynchronous fused steps with
    device observables (dtc_shard_step_async) -- same values as dtc_autocorr."""
    rng = np.random.default_rng(L * 11 + k)
    hs, phis = random_disorder(rng, L, 2)
    spec = pkg.SweepSpec(L=L, T=T, hs=hs, phis=phis, g=0.93, noise_prob=p, polarization=pol,
                         initial_state=state, t_offset=toff)
    one = dataclasses.replace(spec, hs=hs[1:2], phis=phis[1:2])
    for traj in (0, 5):
        got = pkg.sharded.sharded_forward_pipelined(stepper, spec, k, inst=1, traj=traj, seed=77)
        ref = engine.autocorr(one, 1, seed=77, traj_offset=traj, want_echo=False,
                              want_zsite=True)
        assert np.abs(got["zsite"] - ref["zsite"][0, 0]).max() < TOL
        assert np.abs(got["fwd"] - ref["fwd"][0, 0]).max() < TOL
        assert np.abs(got["norm"] - 1.0).max() < 1e-10


def test_l32_eight_virtual_ranks_pipelined(pkg, engine, stepper):
    """C5's layout at L=32 (8 shards of 2^29, 64 GiB in all) against the
    whole-state engine at L=32 (64 GiB): the high site groups' 64-bit lane
    offsets on both sides (dtc_kernels.hip pass_body, ofs32 false) and the
    chunked pipeline at its largest single-GPU size."""
    import os

    import torch

    L = 32
    hs, phis = pkg.load_disorder(34, 1, os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "data"))
    spec = pkg.SweepSpec(L=L, T=3, hs=hs, phis=phis, g=0.97, use_noise=0)
    lay = pkg.sharded.initial_layout(L, 3, 0, 8)
    bufs = stepper.alloc(lay)
    got = pkg.sharded.sharded_forward_pipelined(stepper, spec, 3, buffers=bufs)
    del bufs
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    ref = engine.autocorr(spec, 1, want_echo=False, want_zsite=True)
    assert np.abs(got["zsite"] - ref["zsite"][0, 0]).max() < TOL
    assert np.abs(got["zsite"][1] - np.cos(np.pi * 0.97)).max() < 1e-12
    assert np.abs(got["norm"] - 1.0).max() < 1e-10


@pytest.mark.parametrize("L,k,T,p,state,pol,toff", [
    (22, 3, 5, 0.05, "neel", "x", 0),
    (26, 2, 4, 0.1, "vacuum", "circular_left", 0),
    (25, 3, 4, 0.05, "neel", "xy", 1),
])
def test_pipelined_inplace_virtual_shards_match_engine(pkg, engine, stepper, L, k, T, p, state,
                                                       pol, toff):
    """One state buffer: every slice's exchange is the in-place piece swap
    (dtc_shard_exchange_slice, exchange_swap_kernel) on the engine stream and
    the fused pass runs in place -- the L=34 path at sizes the whole-state
    engine also runs, per trajectory to 1e-10."""
    rng = np.random.default_rng(L * 13 + k)
    hs, phis = random_disorder(rng, L, 2)
    spec = pkg.SweepSpec(L=L, T=T, hs=hs, phis=phis, g=0.93, noise_prob=p, polarization=pol,
                         initial_state=state, t_offset=toff)
    one = dataclasses.replace(spec, hs=hs[1:2], phis=phis[1:2])
    for traj in (0, 5):
        got = pkg.sharded.sharded_forward_pipelined(stepper, spec, k, inst=1, traj=traj, seed=77,
                                                    inplace=True)
        ref = engine.autocorr(one, 1, seed=77, traj_offset=traj, want_echo=False,
                              want_zsite=True)
        assert np.abs(got["zsite"] - ref["zsite"][0, 0]).max() < TOL
        assert np.abs(got["norm"] - 1.0).max() < 1e-10
        # the fused kick+exchange pass (dtc_shard_kick_exchange_slice, the
        # default) against the kick pass followed by the swap kernel: the same
        # kicks in another kernel (bit for bit for the factored kinds; the
        # general 2x2 contracts its FMAs its own way: last-bit differences)
        sep = pkg.sharded.sharded_forward_pipelined(stepper, spec, k, inst=1, traj=traj, seed=77,
                                                    inplace=True, fuse_kick_exchange=False)
        assert np.abs(got["zsite"] - sep["zsite"]).max() < 1e-13


def test_exchange_slice_is_the_all_to_all(pkg, engine, stepper):
    """The in-place swap of every slice equals the two-buffer virtual exchange
    (dst[r][c] = src[c][r]) bit for bit, and twice is the identity."""
    import torch

    lay = pkg.sharded.initial_layout(24, 3, 0, 8)
    x = torch.randn(1 << 24, dtype=torch.complex128, device="cuda")
    ref = torch.empty_like(x)
    pkg.sharded.virtual_exchange(x, ref, 8)
    y = x.clone()
    torch.cuda.synchronize()  # the swaps run on the engine's stream
    for s in range(4):
        stepper.exchange_slice(lay, 2, s, y)
    engine.synchronize()
    assert torch.equal(y, ref)
    for s in range(4):
        stepper.exchange_slice(lay, 2, s, y)
    engine.synchronize()
    assert torch.equal(y, x)


@pytest.mark.parametrize("L,k,T,p,state,pol,toff", [
    (22, 3, 5, 0.05, "neel", "x", 0),
    (26, 2, 4, 0.1, "vacuum", "circular_left", 1),
    (30, 3, 4, 0.05, "vacuum", "x", 0),
])
def test_loopback_real_rank_exchange(pkg, engine, L, k, T, p, state, pol, toff):
    """The C5 pipeline's real-rank branch on one GPU: 2^k ranks, each its own
    engine context (stream) and two shard buffers, ``_SliceExchange`` with
    world = 2^k -- side stream waiting on the engine stream, batch_isend_irecv
    issued under the side stream, Work.wait() on it, the engine stream waiting
    for it -- over LoopbackHub (RCCL's stream semantics; RCCL itself refuses
    two ranks on one GPU).  Per-site <Z_i(t)> equal dtc_autocorr's to 1e-10 and
    every rank posts exactly slice_p2p_plan's ops, slice after slice."""
    import torch

    rng = np.random.default_rng(L * 17 + k)
    hs, phis = random_disorder(rng, L, 2)
    spec = pkg.SweepSpec(L=L, T=T, hs=hs, phis=phis, g=0.93, noise_prob=p, polarization=pol,
                         initial_state=state, t_offset=toff)
    one = dataclasses.replace(spec, hs=hs[1:2], phis=phis[1:2])
    W = 1 << k
    engines = [pkg.DtcEngine(0) for _ in range(W)]
    try:
        steppers = [pkg.sharded.EngineStepper(e) for e in engines]
        got, log = pkg.sharded.loopback_forward_pipelined(steppers, spec, k, inst=1, traj=3,
                                                          seed=77)
        del steppers
    finally:
        for e in engines:
            e.close()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    ref = engine.autocorr(one, 1, seed=77, traj_offset=3, want_echo=False, want_zsite=True)
    assert np.abs(got["zsite"] - ref["zsite"][0, 0]).max() < TOL
    assert np.abs(got["fwd"] - ref["fwd"][0, 0]).max() < TOL
    assert np.abs(got["norm"] - 1.0).max() < 1e-10
    for r in range(W):
        plan = [(kind, peer) for kind, peer, _ in pkg.sharded.slice_p2p_plan(r, W)]
        ops = [(kind, peer) for rr, kind, peer in log if rr == r]
        assert ops and len(ops) % len(plan) == 0
        assert ops == plan * (len(ops) // len(plan)), r
