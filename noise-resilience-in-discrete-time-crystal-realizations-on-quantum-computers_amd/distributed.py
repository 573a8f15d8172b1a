"""Multi-GPU sharding of the sweep: one process per GPU (torchrun), units =
(instance, trajectory) pairs — contiguous trajectory blocks per rank (noisy
sweeps, C2/C3) or contiguous instance blocks (noiseless disorder sweeps, C4:
256 instances x 1 statevector) — with no data-path collective.

Every rank computes the per-trajectory values of its block (counter-based
RNG keyed by the GLOBAL trajectory id, so values do not depend on the number
of ranks), then one all_gather of the per-trajectory arrays — the final
autocorr(t) gather, a few KB to MB over RCCL/xGMI (backend "nccl" on ROCm) or
gloo on CPU tests — after which rank 0 reduces in a fixed order.  The result
is bit-identical for any world size.
"""
from __future__ import annotations

import dataclasses

import numpy as np

from .engine import SweepSpec


def shard_range(n_traj: int, world: int, rank: int):
    """Contiguous block of trajectories [lo, hi) for ``rank``."""
    base, rem = divmod(n_traj, world)
    lo = rank * base + min(rank, rem)
    hi = lo + base + (1 if rank < rem else 0)
    return lo, hi


def gather_blocks(local: np.ndarray, n_traj: int, world: int, group=None,
                  axis: int = 1) -> np.ndarray:
    """all_gather per-rank blocks along ``axis`` (1: [n_inst][n_r][...] ->
    [n_inst][n_traj][...]; 0: instance blocks) in rank order.  Uses the default
    torch.distributed group."""
    import torch
    import torch.distributed as dist

    backend = dist.get_backend(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else \
        torch.device("cpu")
    sizes = [shard_range(n_traj, world, r) for r in range(world)]
    maxn = max(h - l for l, h in sizes)
    loc = np.moveaxis(local, axis, 0)
    pad = np.zeros((maxn,) + loc.shape[1:], dtype=np.float64)
    pad[: loc.shape[0]] = loc
    t = torch.from_numpy(np.ascontiguousarray(pad)).to(dev)
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t, group=group)
    parts = [o.cpu().numpy()[: h - l] for o, (l, h) in zip(outs, sizes)]
    return np.moveaxis(np.concatenate(parts, axis=0), 0, axis)


def sharded_values(compute, n_units: int, world: int, rank: int, group=None, axis: int = 1):
    """Run ``compute(lo, hi) -> dict of arrays whose ``axis`` spans units
    [lo, hi)`` on this rank's block and gather every array to all units."""
    lo, hi = shard_range(n_units, world, rank)
    local = compute(lo, hi)
    return {k: gather_blocks(v, n_units, world, group, axis) for k, v in local.items()}


def sub_spec(spec: SweepSpec, lo: int, hi: int) -> SweepSpec:
    """The instances [lo, hi) of a sweep (same kicks, noise, prep)."""
    return dataclasses.replace(spec, hs=spec.hs[lo:hi], phis=spec.phis[lo:hi])


def sharded_sweep(spec: SweepSpec, n_traj: int, shots=None, seed=0x5EED0001, batch=0,
                  want_fwd=True, want_echo=True, want_zsite=False, shard="auto", engine=None,
                  independent_t=False):
    """Sweep sharded over the torch.distributed world: by trajectory blocks, or
    (``shard="instances"``, default when n_traj < world) by instance blocks.
    Either way the per-trajectory values are those of a single-process run
    (``independent_t``: sweep.autocorr_independent_t per block)."""
    import torch.distributed as dist

    from . import sweep as sw

    if independent_t and want_zsite:
        raise ValueError("independent_t: per-site Z is a forward-sweep output")  # as run_sweep
    world, rank = dist.get_world_size(), dist.get_rank()
    eng = engine or sw._default_engine()
    if shard == "auto":
        shard = "trajectories" if n_traj >= world else "instances"

    def empty(n_i, n_t):
        shape = (n_i, n_t, spec.T)
        out = {}
        if want_fwd:
            out["fwd"] = np.zeros(shape)
        if want_echo:
            out["echo"] = np.zeros(shape)
        if want_zsite:
            out["zsite"] = np.zeros(shape + (spec.L,))
        return out

    if shard == "instances":
        def compute(lo, hi):
            if hi <= lo:
                return empty(0, n_traj)
            if independent_t:
                return sw.autocorr_independent_t(eng, sub_spec(spec, lo, hi), n_traj, seed=seed,
                                                 want_fwd=want_fwd, want_echo=want_echo,
                                                 batch=batch)
            return eng.autocorr(sub_spec(spec, lo, hi), n_traj, seed=seed, want_fwd=want_fwd,
                                want_echo=want_echo, want_zsite=want_zsite, batch=batch)

        full = sharded_values(compute, spec.n_inst, world, rank, axis=0)
    else:
        def compute(lo, hi):
            if hi <= lo:
                return empty(spec.n_inst, 0)
            if independent_t:
                return sw.autocorr_independent_t(eng, spec, hi - lo, seed=seed, lo=lo,
                                                 want_fwd=want_fwd, want_echo=want_echo,
                                                 batch=batch)
            return eng.autocorr(spec, hi - lo, seed=seed, traj_offset=lo, want_fwd=want_fwd,
                                want_echo=want_echo, want_zsite=want_zsite, batch=batch)

        full = sharded_values(compute, n_traj, world, rank)
    rng = np.random.default_rng(seed)
    res = {}
    for key in ("fwd", "echo"):
        if key not in full:
            res[key] = None
            continue
        a = full[key]
        res[key] = a.mean(axis=1) if shots is None else sw._shot_estimate(a, shots, rng)
    return sw.SweepResult(res["fwd"], res["echo"], full.get("fwd"), full.get("echo"),
                          full.get("zsite"))
