"""C5 at its real size on one MI355X (one L=34 state,
2^34 complex128 = 256 GiB, as 8 virtual shards of n_local = 31).

The exchange runs in place (dtc_shard_exchange_slice: slice s of piece
(shard r, chunk c) trades places with (c, r)), so the state needs one 256 GiB
buffer instead of two and the per-rank kernels of the 8-GPU run -- n_local = 31
slice kicks, 64-bit lane offsets, 34-site diagonal tables, the largest site
group on top -- run at their production sizes.  No oracle runs an L=34 sweep,
so parity goes through size-independent properties:

* zero-bond factorisation: with two bonds switched off the chain splits into
  blocks of 11, 12 and 11 sites (the last one holds the three rank-bit sites
  and the sites the exchange swaps with them), and every per-site <Z_i(t)>
  must equal the C oracle's run of that block alone, to 1e-10;
* known answers: <Z_i(0)> = 1 and <Z_i(1)> = cos(pi g) for every i (vacuum);
* the norm stays 1.

The reference has no L=34 run (it caps L at 20, fast.py:177-178).
"""
import os

import numpy as np
import pytest

from oracle import c_oracle

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L, K = 34, 3
STATE_BYTES = 16 << L


@pytest.fixture(scope="module")
def state34(pkg, engine):
    """One 256 GiB state buffer, after the engine's batch buffers are freed.
    Skips (printing the measured free bytes) if it does not fit."""
    import torch

    engine.release_buffers()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    free, total = torch.cuda.mem_get_info()
    print(f"\nL=34: hipMemGetInfo free {free} B, total {total} B, state {STATE_BYTES} B")
    if free < STATE_BYTES + (4 << 30):
        pytest.skip(f"an L=34 state ({STATE_BYTES} B) + 4 GiB does not fit: {free} B free "
                    f"of {total}")
    buf = torch.empty(1 << L, dtype=torch.complex128, device="cuda")
    yield buf
    del buf
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def _run(pkg, engine, spec, buf):
    st = pkg.sharded.EngineStepper(engine)
    return pkg.sharded.sharded_forward_pipelined(st, spec, K, buffers=(buf,), inplace=True)


def _disorder(pkg):
    return pkg.load_disorder(L, 1, os.path.join(ROOT, "data"))


def test_l34_known_answers_and_norm(pkg, engine, state34):
    hs, phis = _disorder(pkg)
    g = 0.97
    spec = pkg.SweepSpec(L=L, T=4, hs=hs, phis=phis, g=g, use_noise=0)
    got = _run(pkg, engine, spec, state34)
    z = got["zsite"]
    assert np.abs(z[0] - 1.0).max() < 1e-12
    assert np.abs(z[1] - np.cos(np.pi * g)).max() < 1e-12
    assert np.abs(got["norm"] - 1.0).max() < 1e-10
    assert np.all(np.abs(z) <= 1.0 + 1e-12)


@pytest.mark.parametrize("pol,state", [("x", "vacuum"), ("circular_left", "neel")])
def test_l34_blocks_match_oracle(pkg, engine, state34, pol, state):
    hs, phis = _disorder(pkg)
    phis = phis.copy()
    cuts = (10, 22)                      # bonds (10,11) and (22,23) switched off
    phis[:, list(cuts)] = 0.0
    T, g = 5, 0.93
    spec = pkg.SweepSpec(L=L, T=T, hs=hs, phis=phis, g=g, polarization=pol,
                         initial_state=state, use_noise=0)
    got = _run(pkg, engine, spec, state34)
    assert np.abs(got["norm"] - 1.0).max() < 1e-10
    mask = spec.init_mask
    lo = 0
    for hi in (cuts[0] + 1, cuts[1] + 1, L):
        Lb = hi - lo
        bspec = pkg.SweepSpec(L=Lb, T=T, hs=hs[:, lo:hi], phis=phis[:, lo:hi - 1], g=g,
                              use_noise=0, kick=spec.kick[:, lo:hi],
                              init_mask_value=(mask >> lo) & ((1 << Lb) - 1))
        ref = c_oracle.autocorr(bspec, 1, want_echo=False, want_zsite=True)
        err = np.abs(got["zsite"][:, lo:hi] - ref["zsite"][0, 0]).max()
        assert err < 1e-10, (lo, hi, err)
        lo = hi
