"""Numpy stand-in for the engine's sharded-state step (TEST INFRASTRUCTURE ONLY:
imported by tests/, never by the product).

Implements the semantics of ``dtc_shard_set_basis`` / ``dtc_shard_step``
(include/dtc.h) directly from the logical circuit, without the engine's
effective-field construction: each amplitude's logical bits are assembled
from the physical local bits and the shard's rank bits, the RZZ/RZ phase is
evaluated on the logical chain (fast.py:115-120), and each kick is the
period's sub-gate product with the same Philox Pauli draws as the C oracle
(oracle/dtc_oracle.c: orc_pauli, keyed by logical site).  With it the
sharded sweep driver (sharded.py) — bit maps, exchanges over gloo, the Z
bookkeeping — is checked on CPU against the whole-state C oracle.
"""
from __future__ import annotations

import numpy as np

from . import c_oracle

PAULI = [np.eye(2, dtype=complex), np.array([[0, 1], [1, 0]], dtype=complex),
         np.array([[0, -1j], [1j, 0]], dtype=complex), np.diag([1.0 + 0j, -1.0])]
STREAM_PREP = 0xFFFFFFFF


def _row_matrix(row):
    m = np.asarray(row, dtype=np.float64).reshape(4, 2)
    return (m[:, 0] + 1j * m[:, 1]).reshape(2, 2)


class NumpyShardStepper:
    # slices of a single amplitude are fine here (the engine needs >= 12 index
    # bits per slice: one 4096-amplitude tile), so small test states exercise
    # the sliced exchange of sharded_forward_pipelined
    min_slice_index_bits = 1

    def __init__(self, groups=None):
        self._groups = groups

    def plan_groups(self, n_bits):
        if self._groups is not None:
            return self._groups(n_bits)
        return [(1 << n_bits) - 1]

    def alloc(self, layout, n_buffers=2):
        import torch

        n = layout.n_shards << layout.n_local
        return tuple(torch.zeros(n, dtype=torch.complex128) for _ in range(n_buffers))

    # -- helpers --------------------------------------------------------
    @staticmethod
    def _kick(spec, p, site, seed, traj):
        M = np.eye(2, dtype=complex)
        for q in range(spec.n_sub):
            M = _row_matrix(spec.kick[p - 1, site, q]) @ M
            if spec.p > 0:
                M = PAULI[c_oracle.sample_pauli(spec.p, seed, traj, 0, p, site, q)] @ M
        return M

    @staticmethod
    def _apply(psi, nl, q, M):
        v = psi.reshape(psi.shape[0], 1 << (nl - q - 1), 2, 1 << q)
        a0, a1 = v[:, :, 0, :].copy(), v[:, :, 1, :].copy()
        v[:, :, 0, :] = M[0, 0] * a0 + M[0, 1] * a1
        v[:, :, 1, :] = M[1, 0] * a0 + M[1, 1] * a1

    @staticmethod
    def _logical_z(layout, rank):
        """z_i (+-1) of every logical site for every local index of a shard."""
        nl, L = layout.n_local, layout.L
        x = np.arange(1 << nl)
        z = np.empty((L, 1 << nl))
        for q in range(L):
            bit = (x >> q) & 1 if q < nl else np.full(x.shape, (rank >> (q - nl)) & 1)
            z[layout.site_of[q]] = 1.0 - 2.0 * bit
        return z

    # -- the two entry points ----------------------------------------------
    def set_basis(self, spec, layout, seed, traj, buf):
        mask = spec.init_mask
        if spec.p > 0:
            for i in range(spec.L):
                if (spec.init_mask >> i) & 1:
                    pz = c_oracle.sample_pauli(spec.p, seed, traj, STREAM_PREP, 0, i, 0)
                    if pz in (1, 2):
                        mask &= ~(1 << i)
        psi = buf.numpy().reshape(layout.n_shards, -1)
        psi[:] = 0
        local = rank = 0
        for q in range(layout.L):
            bit = (mask >> layout.site_of[q]) & 1
            if q < layout.n_local:
                local |= bit << q
            else:
                rank |= bit << (q - layout.n_local)
        b = rank - layout.first_rank
        if 0 <= b < layout.n_shards:
            psi[b, local] = 1.0

    def step(self, spec, layout, seed, traj, inst, period, pre, diag, post, src, dst, want_obs):
        nl = layout.n_local
        psi = src.numpy().reshape(layout.n_shards, -1).copy()
        for q in range(nl):
            if (pre >> q) & 1:
                self._apply(psi, nl, q, self._kick(spec, period, layout.site_of[q], seed, traj))
        obs = np.zeros((layout.n_shards, 1 + nl)) if want_obs else None
        h, ph = spec.hs[inst], spec.phis[inst]
        for b in range(layout.n_shards):
            z = self._logical_z(layout, layout.first_rank + b)
            if diag:
                ang = (h[:, None] * z).sum(axis=0)
                if spec.L > 1:
                    ang += (ph[:, None] * z[:-1] * z[1:]).sum(axis=0)
                psi[b] *= np.exp(-0.5j * ang)
            if want_obs:
                pr = np.abs(psi[b]) ** 2
                obs[b, 0] = pr.sum()
                x = np.arange(1 << nl)
                for q in range(nl):
                    obs[b, 1 + q] = ((1.0 - 2.0 * ((x >> q) & 1)) * pr).sum()
        for q in range(nl):
            if (post >> q) & 1:
                self._apply(psi, nl, q, self._kick(spec, period + 1, layout.site_of[q], seed, traj))
        dst.numpy().reshape(layout.n_shards, -1)[:] = psi
        return obs

    # -- the asynchronous interface of sharded_forward_pipelined (synchronous here) --
    def kick_slice(self, spec, layout, seed, traj, period, pre, chunk_bits, slice_bits, slice_,
                   buf):
        """K_period on the local bits ``pre`` of slice ``slice_`` of every chunk
        (top chunk_bits local bits; the next slice_bits number the slices) of
        every shard held, in place (dtc_shard_kick_slice)."""
        nl = layout.n_local
        nsub = nl - chunk_bits - slice_bits
        if pre >> nsub:
            raise ValueError("slice kick mask reaches the chunk/slice bits")
        psi = buf.numpy().reshape(layout.n_shards << chunk_bits, 1 << slice_bits, 1 << nsub)
        sub = psi[:, slice_, :].copy()
        for q in range(nsub):
            if (pre >> q) & 1:
                self._apply(sub, nsub, q, self._kick(spec, period, layout.site_of[q], seed, traj))
        psi[:, slice_, :] = sub

    def exchange_slice(self, layout, slice_bits, slice_, buf):
        """dtc_shard_exchange_slice: every shard in ``buf``; piece (shard r,
        chunk c, slice) <-> (shard c, chunk r, slice), in place."""
        W = 1 << layout.n_global
        if layout.n_shards != W or layout.first_rank != 0:
            raise ValueError("the in-place exchange needs every shard in this buffer")
        v = buf.numpy().reshape(W, W, 1 << slice_bits, -1)
        for r in range(W):
            for c in range(r + 1, W):
                tmp = v[r, c, slice_].copy()
                v[r, c, slice_] = v[c, r, slice_]
                v[c, r, slice_] = tmp

    def step_async(self, spec, layout, seed, traj, inst, period, pre, diag, post, src, dst,
                   obs_out):
        obs = self.step(spec, layout, seed, traj, inst, period, pre, diag, post, src, dst,
                        obs_out is not None)
        if obs_out is not None:
            obs_out.numpy()[...] = obs

    def obs_buffer(self, n_steps, n_shards, n_obs):
        import torch

        return torch.zeros((n_steps, n_shards, n_obs), dtype=torch.float64)

    def synchronize(self):
        pass
