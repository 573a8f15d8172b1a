"""C4 / C5 dynamics at L=28 fully coupled against the C oracle.

test_gpu_large.py pins L=28 through properties (zero-bond factorisation,
known answers); here the oracle runs the coupled chain itself: a gate-by-gate
statevector sweep of 2^28 amplitudes (oracle/dtc_oracle.c sweeps states of
2^22 amplitudes and more with all host threads; ~30-60 s for T=4 on the GPU
box's 16 cores).  The same oracle run pins two engine paths:

* C4's: dtc_autocorr with per-site <Z_i(t)> (12 + 8 + 8 site groups, two
  passes per period, the per-site measurement passes);
* C5's: the sharded pipeline (sharded.py) with 8 virtual shards (n_local = 25,
  rank bits = sites 25..27), in place with the fused kick+exchange pass --
  the code path of the L=34 one-GPU run and, but for the transport, of the
  8-GPU run.

Per-site <Z_i(t)> to 1e-10 for t < T, g = 0.97 and a disorder row of the C4
data (data/hs_L28.csv)."""
import os

import numpy as np
import pytest

from oracle import c_oracle

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOL = 1e-10
L, T, G = 28, 4, 0.97


@pytest.fixture(scope="module")
def coupled(pkg):
    hs, phis = pkg.load_disorder(L, 2, os.path.join(ROOT, "data"))
    spec = pkg.SweepSpec(L=L, T=T, hs=hs[1:2], phis=phis[1:2], g=G, polarization="circular_left",
                         initial_state="neel", use_noise=0)
    ref = c_oracle.autocorr(spec, 1, want_echo=False, want_zsite=True)
    return spec, ref


def test_l28_coupled_engine_matches_oracle(pkg, engine, coupled):
    spec, ref = coupled
    got = engine.autocorr(spec, 1, want_echo=False, want_zsite=True)
    err = np.abs(got["zsite"] - ref["zsite"]).max()
    assert err < TOL, err
    assert np.abs(got["fwd"] - ref["fwd"]).max() < TOL
    # the coupled dynamics move away from the product-state answers
    assert np.abs(ref["zsite"][0, 0, T - 1] - ref["zsite"][0, 0, 1]).max() > 1e-3


def test_l28_coupled_sharded_matches_oracle(pkg, engine, coupled):
    import torch

    spec, ref = coupled
    stepper = pkg.sharded.EngineStepper(engine)
    got = pkg.sharded.sharded_forward_pipelined(stepper, spec, 3, inplace=True)
    del stepper
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    err = np.abs(got["zsite"] - ref["zsite"][0, 0]).max()
    assert err < TOL, err
    assert np.abs(got["norm"] - 1.0).max() < 1e-10


def test_l30_coupled_c5_path_matches_oracle(pkg, engine):
    """The C5 pipeline closer to its L=34 shape: L=30 as 8 virtual shards of
    2^27 amplitudes (in place, fused kick+exchange) and the whole-state engine,
    both against one coupled oracle sweep (T=3: the oracle's 2^30-amplitude
    sweep takes about a minute on the GPU box's 16 cores)."""
    import torch

    hs, phis = pkg.load_disorder(34, 1, os.path.join(ROOT, "data"))
    spec = pkg.SweepSpec(L=30, T=3, hs=hs, phis=phis, g=G, polarization="x",
                         initial_state="neel", use_noise=0)
    ref = c_oracle.autocorr(spec, 1, want_echo=False, want_zsite=True)
    got = engine.autocorr(spec, 1, want_echo=False, want_zsite=True)
    assert np.abs(got["zsite"] - ref["zsite"]).max() < TOL
    engine.release_buffers()
    stepper = pkg.sharded.EngineStepper(engine)
    sh = pkg.sharded.sharded_forward_pipelined(stepper, spec, 3, inplace=True)
    del stepper
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    assert np.abs(sh["zsite"] - ref["zsite"][0, 0]).max() < TOL
    assert np.abs(sh["norm"] - 1.0).max() < 1e-10
