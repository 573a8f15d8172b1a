"""Bit-identity across the multi-GPU splits, at the bench lines' own sizes.

SURVEY.md §4 promises bit-identical results on 1, 2, 4 and 8 GPUs: the units
(trajectories of the C2 sweep, disorder instances of C4) are independent and
every random draw is keyed by the global trajectory id, so a rank's share must
come out of the engine exactly as it does inside the one-GPU batch.  The CPU
gloo tests cover the ranks' bookkeeping with the oracle as the compute; here
the HIP engine itself runs the splits (reference: the instance / trajectory
loops of autocorr-delta-a-single-qiskit-fast.py:217-239):

* C2 (BASELINE configs[1]: L=20, T=30, p=0.05, hs/phis_L20 row 0, seed
  0x5EED0001): one B=1024 call at offset 0 against 8 calls of B=128 at
  offsets 0..896 (the 8-GPU strong-scaling split of bench.py's step) and 2 of
  B=512 (2 GPUs) -- with the dual pass and the 12-site light-cone end active
  (asserted), fwd and echo np.array_equal;
* C4 (configs[3]: L=28, 32 instances per GPU as bench.py --config c4 runs them,
  in the contiguous layout with the XCD-aware tile order): T=3, 32 instances at
  batch 32 against 8 x 4 instances at batch 4, zsite np.array_equal.
"""
import dataclasses
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SEED = 0x5EED0001


def _free(engine):
    import torch

    engine.release_buffers()
    torch.cuda.empty_cache()


def test_c2_strong_scaling_split_bit_identical(pkg, engine):
    _free(engine)
    with open(os.path.join(ROOT, "tests", "golden", "disorder.json")) as f:
        d = json.load(f)["L20"]
    spec = pkg.SweepSpec(L=20, T=30, hs=np.array(d["hs"][:1]), phis=np.array(d["phis"][:1]),
                         g=0.97, noise_prob=0.05, use_noise=1, initial_state="vacuum")
    with pkg.DtcEngine(0) as eng:
        full = eng.autocorr(spec, 1024, seed=SEED, traj_offset=0, batch=1024)
        counts = eng.lightcone_counts()
        for n_ranks in (8, 2):
            b = 1024 // n_ranks
            parts = [eng.autocorr(spec, b, seed=SEED, traj_offset=r * b, batch=b)
                     for r in range(n_ranks)]
            for k in ("fwd", "echo"):
                got = np.concatenate([p[k] for p in parts], axis=1)
                assert got.shape == full[k].shape
                assert np.array_equal(got, full[k]), (n_ranks, k,
                                                      float(np.abs(got - full[k]).max()))
        eng.release_buffers()
    # the schedule features the line depends on ran in the full batch
    assert counts["lcw3"] >= 23, counts


def test_c4_instance_split_bit_identical(pkg, engine):
    _free(engine)
    L, n = 28, 32
    hs, phis = pkg.load_disorder(L, n, os.path.join(ROOT, "data"))
    spec = pkg.SweepSpec(L=L, T=3, hs=hs, phis=phis, g=0.97, use_noise=0)
    with pkg.DtcEngine(0) as eng:
        full = eng.autocorr(spec, 1, want_echo=False, want_zsite=True, batch=n)["zsite"]
        parts = [eng.autocorr(dataclasses.replace(spec, hs=hs[i:i + 4], phis=phis[i:i + 4]), 1,
                              want_echo=False, want_zsite=True, batch=4)["zsite"]
                 for i in range(0, n, 4)]
        eng.release_buffers()
    got = np.concatenate(parts, axis=0)
    assert got.shape == full.shape == (n, 1, 3, L)
    assert np.array_equal(got, full), float(np.abs(got - full).max())
    # known answers at full size: <Z_i(0)> = 1, <Z_i(1)> = cos(pi g)
    assert np.abs(full[:, :, 0] - 1.0).max() < 1e-12
    assert np.abs(full[:, :, 1] - np.cos(np.pi * 0.97)).max() < 1e-12
