"""One state vector split over ranks: the L=34 configuration (SURVEY.md §8(d)/(e),
C5: 2^34 complex128 = 256 GiB over 8 GPUs, 32 GiB per rank).

Layout.  With W = 2^k ranks a shard holds 2^(L-k) amplitudes.  Physical bit
q < n_local of a shard holds logical site ``site_of[q]``; bit j of the rank id
holds ``site_of[n_local + j]``.  Two bit maps alternate:

    X: local bits = sites 0 .. L-k-1, rank bits = sites L-k .. L-1
    Y: the top k local bits and the rank bits trade places

and one all-to-all (chunk c of every shard, c = value of its top k local bits,
goes to rank c) turns X into Y and back.  Every logical bond between two local
sites stays between adjacent physical bits in both maps, so the engine's
diagonal tables work unchanged: bonds and fields touching rank bits become
per-rank effective fields and a per-rank constant phase (dtc_engine.cpp:
shard_chain).  The RZZ/RZ layer never needs communication.

Schedule of period p (forward, fast.py:111-121 per period):

    step(pre = every local bit not yet kicked with K_p)        # one pass per group
    exchange                                                   # all-to-all, X <-> Y
    step(pre = top k bits, D_p, measure, post = K_{p+1} on the group holding the
         top bits (and the top bits))                          # one fused pass

so a period costs the single-device passes plus one exchange of (W-1)/W of the
shard.  The exchange is ``torch.distributed.all_to_all_single`` (RCCL over
xGMI on the GPU node, gloo in CPU tests) between processes, or a strided
device copy when one process holds all shards ("virtual ranks", used to test
the layout logic on one GPU).  Per-site <Z_i(t)> come from per-shard
(norm, z_q) partial sums: rank-bit sites take the shard's sign times its norm;
one all_reduce of L+1 doubles per period joins the ranks.

Results are the single-device engine's (same RNG contract: noise keyed by
logical site), checked in tests/test_sharded_cpu.py (numpy stepper, gloo) and
tests/test_gpu_sharded.py (engine, virtual ranks, vs dtc_autocorr).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import _capi
from .engine import N_ANCILLA_NOISY_GATES, SweepSpec


@dataclass(frozen=True)
class ShardLayout:
    n_local: int
    n_global: int
    site_of: tuple
    first_rank: int = 0
    n_shards: int = 1

    @property
    def L(self) -> int:
        return self.n_local + self.n_global

    @property
    def world(self) -> int:
        return 1 << self.n_global

    @property
    def top_mask(self) -> int:
        """Physical local bits that trade places with the rank bits."""
        k, nl = self.n_global, self.n_local
        return ((1 << k) - 1) << (nl - k)

    @property
    def local_mask(self) -> int:
        return (1 << self.n_local) - 1

    def exchanged(self) -> "ShardLayout":
        """The bit map after the all-to-all: top k local bits <-> rank bits."""
        s = list(self.site_of)
        k, nl = self.n_global, self.n_local
        top = s[nl - k:nl]
        s[nl - k:nl] = s[nl:nl + k]
        s[nl:nl + k] = top
        return ShardLayout(nl, k, tuple(s), self.first_rank, self.n_shards)

    def to_c(self) -> _capi.DtcShard:
        sh = _capi.DtcShard()
        sh.n_local = self.n_local
        sh.n_global = self.n_global
        sh.n_shards = self.n_shards
        sh.first_rank = self.first_rank
        for q, v in enumerate(self.site_of):
            sh.site_of[q] = v
        return sh


def initial_layout(L: int, n_global: int, first_rank: int = 0, n_shards: int = 1) -> ShardLayout:
    if n_global < 0 or L - n_global < 2 * n_global:
        raise ValueError("need n_local >= 2 n_global")
    return ShardLayout(L - n_global, n_global, tuple(range(L)), first_rank, n_shards)


def z_from_obs(layout: ShardLayout, obs: np.ndarray) -> np.ndarray:
    """Per-shard (norm, z_q) partials -> [norm, Z_0 .. Z_{L-1}] summed over held shards."""
    L, nl = layout.L, layout.n_local
    out = np.zeros(1 + L)
    for b in range(layout.n_shards):
        r = layout.first_rank + b
        out[0] += obs[b, 0]
        for q in range(nl):
            out[1 + layout.site_of[q]] += obs[b, 1 + q]
        for j in range(layout.n_global):
            sgn = -1.0 if (r >> j) & 1 else 1.0
            out[1 + layout.site_of[nl + j]] += sgn * obs[b, 0]
    return out


# ---- exchanges ------------------------------------------------------------------

def virtual_exchange(src, dst, world: int):
    """All shards in one buffer: dst[r][c] = src[c][r] (chunks of 2^(n_local-k))."""
    dst.view(world, world, -1).copy_(src.view(world, world, -1).transpose(0, 1))


def collective_exchange(src, dst, group=None):
    """One shard per process: all_to_all_single over the process group (RCCL
    over xGMI for "nccl", gloo on CPU)."""
    import torch
    import torch.distributed as dist

    dist.all_to_all_single(torch.view_as_real(dst), torch.view_as_real(src), group=group)


def _allreduce(vec: np.ndarray, group=None) -> np.ndarray:
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return vec
    dev = torch.device("cuda", torch.cuda.current_device()) \
        if dist.get_backend(group) == "nccl" else torch.device("cpu")
    t = torch.from_numpy(np.ascontiguousarray(vec)).to(dev)
    dist.all_reduce(t, group=group)
    return t.cpu().numpy()


# ---- steppers ---------------------------------------------------------------------

class EngineStepper:
    """The HIP engine (dtc_shard_* C ABI) on torch-allocated device buffers."""

    def __init__(self, engine):
        self.engine = engine

    def plan_groups(self, n_bits):
        return _capi.plan_groups(n_bits)

    def alloc(self, layout: ShardLayout):
        import torch

        n = layout.n_shards << layout.n_local
        dev = torch.device("cuda", torch.cuda.current_device())
        return (torch.empty(n, dtype=torch.complex128, device=dev),
                torch.empty(n, dtype=torch.complex128, device=dev))

    def set_basis(self, spec, layout, seed, traj, buf):
        import torch

        torch.cuda.synchronize()
        self.engine.shard_set_basis(spec, layout.to_c(), buf.data_ptr(), seed, traj)

    def step(self, spec, layout, seed, traj, inst, period, pre, diag, post, src, dst, want_obs):
        import torch

        torch.cuda.synchronize()  # exchanges run on torch / RCCL streams
        return self.engine.shard_step(spec, layout.to_c(), period, pre, diag, post,
                                      src.data_ptr(), dst.data_ptr(), want_obs, seed, traj, inst)


# ---- the sweep ----------------------------------------------------------------------

def sharded_forward(stepper, spec: SweepSpec, n_global: int, *, inst: int = 0, traj: int = 0,
                    seed: int = 0x5EED0001, rank: int = 0, world: int = 1, group=None,
                    exchange=None, buffers=None, on_period=None):
    """Forward sweep of one trajectory of instance ``inst`` on a sharded state.

    ``world`` processes hold 2^n_global / world shards each (1 process: virtual
    ranks; 2^n_global processes: one shard each).  Returns ``zsite`` [T][L]
    (per-site <Z_i(t)>, same meaning as dtc_autocorr's) and ``norm`` [T]."""
    L, T = spec.L, spec.T
    W = 1 << n_global
    if world not in (1, W):
        raise ValueError("world must be 1 (virtual ranks) or 2^n_global")
    n_sh = W // world
    lay = initial_layout(L, n_global, rank * n_sh, n_sh)
    if exchange is None:
        exchange = (lambda s, d: virtual_exchange(s, d, W)) if world == 1 else \
            (lambda s, d: collective_exchange(s, d, group))
    A, Bf = buffers if buffers is not None else stepper.alloc(lay)
    nl, top, allb = lay.n_local, lay.top_mask, lay.local_mask
    groups = stepper.plan_groups(nl)
    main = next(g for g in groups if (g >> (nl - 1)) & 1)
    post_bits = main | top
    P = T - 1 + spec.t_offset
    zs = np.zeros((T, L))
    norm = np.zeros(T)

    def record(t, obs, layout):
        v = _allreduce(z_from_obs(layout, obs), group)
        norm[t] = v[0]
        zs[t] = v[1:]

    stepper.set_basis(spec, lay, seed, traj, A)
    # the prepared product state (noisy X prep included): z_j(init) of the
    # ancilla fold and, for t_offset = 0, the t = 0 point
    init = _allreduce(z_from_obs(lay, stepper.step(spec, lay, seed, traj, inst, 1, 0, False, 0,
                                                   A, A, True)), group)
    zinit = 1.0 if init[1 + spec.probe_site] >= 0 else -1.0
    if spec.t_offset == 0:
        norm[0], zs[0] = init[0], init[1:]
    kicked = 0
    for p in range(1, P + 1):
        pre = allb & ~kicked
        if pre:
            stepper.step(spec, lay, seed, traj, inst, p, pre, False, 0, A, A, False)
        exchange(A, Bf)
        lay = lay.exchanged()
        post = post_bits if p < P else 0
        t = p - spec.t_offset
        obs = stepper.step(spec, lay, seed, traj, inst, p, top, True, post, Bf, A, t >= 0)
        kicked = post
        if t >= 0:
            record(t, obs, lay)
        if on_period is not None:
            on_period(p)
    fac = (1.0 - spec.p) ** N_ANCILLA_NOISY_GATES
    return {"zsite": zs, "norm": norm, "fwd": fac * zinit * zs[:, spec.probe_site]}
