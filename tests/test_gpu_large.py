"""C4-scale checks (L=28, noiseless forward + per-site <Z_i(t)>,
disorder data/hs_L28.csv / phis_L28.csv from tools/make_large_disorder.py).

No oracle finishes an L=28 sweep in seconds, so parity at full size goes
through properties that do not depend on size:

* factorisation: with the couplings of two bonds set to zero the chain splits
  into independent blocks, and every per-site <Z_i(t)> of the L=28 engine run
  must equal the C oracle's run of the block holding site i (L = 11, 7, 10) —
  to 1e-10, for every t < 30, with the block boundaries straddling the
  engine's 12-site tile and both 8-site column groups;
* known answers: <Z_i(0)> = 1 and <Z_i(1)> = cos(pi g) for the vacuum state;
* batching and instance sharding do not change a single bit.
"""
import dataclasses
import os

import numpy as np
import pytest

from oracle import c_oracle

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOL = 1e-10
L = 28


def _disorder(pkg, n):
    return pkg.load_disorder(L, n, os.path.join(ROOT, "data"))


@pytest.mark.parametrize("pol,state", [("x", "vacuum"), ("circular_left", "neel")])
def test_l28_blocks_match_oracle(pkg, engine, pol, state):
    hs, phis = _disorder(pkg, 2)
    phis = phis.copy()
    cuts = (10, 17)                      # bonds (10,11) and (17,18) switched off
    phis[:, list(cuts)] = 0.0
    T, g = 30, 0.93
    spec = pkg.SweepSpec(L=L, T=T, hs=hs, phis=phis, g=g, polarization=pol,
                         initial_state=state, use_noise=0)
    got = engine.autocorr(spec, 1, want_echo=False, want_zsite=True)
    mask = spec.init_mask
    lo = 0
    for hi in (cuts[0] + 1, cuts[1] + 1, L):
        Lb = hi - lo
        bspec = pkg.SweepSpec(L=Lb, T=T, hs=hs[:, lo:hi], phis=phis[:, lo:hi - 1], g=g,
                              use_noise=0, kick=spec.kick[:, lo:hi],
                              init_mask_value=(mask >> lo) & ((1 << Lb) - 1))
        ref = c_oracle.autocorr(bspec, 1, want_echo=False, want_zsite=True)
        err = np.abs(got["zsite"][..., lo:hi] - ref["zsite"]).max()
        assert err < TOL, (lo, hi, err)
        j = spec.probe_site
        if lo <= j < hi:
            zj = 1.0 - 2.0 * ((mask >> j) & 1)
            assert np.abs(got["fwd"] - zj * ref["zsite"][..., j - lo]).max() < TOL
        lo = hi


def test_l28_known_answers(pkg, engine):
    hs, phis = _disorder(pkg, 3)
    g = 0.97
    spec = pkg.SweepSpec(L=L, T=3, hs=hs, phis=phis, g=g, use_noise=0)
    z = engine.autocorr(spec, 1, want_echo=False, want_zsite=True)["zsite"]
    assert np.abs(z[:, :, 0] - 1.0).max() < 1e-12
    assert np.abs(z[:, :, 1] - np.cos(np.pi * g)).max() < 1e-12
    assert np.all(np.abs(z[:, :, 2]) <= 1.0 + 1e-12)


def test_l28_batching_and_instance_shards_bit_identical(pkg, engine):
    hs, phis = _disorder(pkg, 4)
    spec = pkg.SweepSpec(L=L, T=5, hs=hs, phis=phis, g=0.97, use_noise=0)
    full = engine.autocorr(spec, 1, want_echo=False, want_zsite=True, batch=3)
    parts = [engine.autocorr(dataclasses.replace(spec, hs=hs[i:i + 2], phis=phis[i:i + 2]), 1,
                             want_echo=False, want_zsite=True, batch=2)["zsite"]
             for i in (0, 2)]
    assert np.array_equal(full["zsite"], np.concatenate(parts, axis=0))
