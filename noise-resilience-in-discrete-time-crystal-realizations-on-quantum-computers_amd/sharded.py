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
        self._stream = None

    # -- asynchronous interface (sharded_forward_pipelined) --------------------
    def stream(self):
        """The engine's HIP stream as a torch stream (events order the exchange
        stream against it; nothing blocks the host)."""
        import torch

        if self._stream is None:
            self._stream = torch.cuda.ExternalStream(self.engine.stream_handle())
        return self._stream

    def kick_slice(self, spec, layout, seed, traj, period, pre, chunk_bits, slice_bits, slice_,
                   buf):
        self.engine.shard_kick_slice(spec, layout.to_c(), period, pre, chunk_bits, slice_bits,
                                     slice_, buf.data_ptr(), seed, traj)

    def step_async(self, spec, layout, seed, traj, inst, period, pre, diag, post, src, dst,
                   obs_out):
        self.engine.shard_step_async(spec, layout.to_c(), period, pre, diag, post,
                                     src.data_ptr(), dst.data_ptr(),
                                     obs_out.data_ptr() if obs_out is not None else None,
                                     seed, traj, inst)

    def obs_buffer(self, n_steps, n_shards, n_obs):
        import torch

        return torch.zeros((n_steps, n_shards, n_obs), dtype=torch.float64,
                           device=torch.device("cuda", torch.cuda.current_device()))

    def synchronize(self):
        self.engine.synchronize()

    def plan_groups(self, n_bits):
        return _capi.plan_groups(n_bits)

    def alloc(self, layout: ShardLayout, n_buffers: int = 2):
        import torch

        n = layout.n_shards << layout.n_local
        dev = torch.device("cuda", torch.cuda.current_device())
        return tuple(torch.empty(n, dtype=torch.complex128, device=dev)
                     for _ in range(n_buffers))

    def exchange_slice(self, layout: ShardLayout, slice_bits, slice_, buf):
        self.engine.shard_exchange_slice(layout.to_c(), slice_bits, slice_, buf.data_ptr())

    def kick_exchange_slice(self, spec, layout, seed, traj, period, pre, slice_bits, slice_, buf):
        self.engine.shard_kick_exchange_slice(spec, layout.to_c(), period, pre, slice_bits, slice_,
                                              buf.data_ptr(), seed, traj)

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


# ---- the pipelined sweep (C5 on the GPU node) -----------------------------------------

def slice_p2p_plan(rank: int, W: int):
    """The point-to-point transfers of one slice at rank ``rank`` of ``W``
    (the real-rank exchange of sharded_forward_pipelined), in posting order:
    ``[("isend" | "irecv", peer, chunk), ...]`` -- at step i = 1 .. W-1 send
    chunk d = rank+i to rank d and receive chunk q = rank-i's piece from rank q
    into chunk slot q.  Every peer appears once as a destination and once as a
    source, so all W-1 xGMI links of a rank carry one transfer per slice; the
    local chunk (c = rank) is a device copy, not listed.  Rank r's send to d
    pairs with rank d's receive from r (same step i on both sides)."""
    ops = []
    for i in range(1, W):
        d, q = (rank + i) % W, (rank - i) % W
        ops.append(("isend", d, d))
        ops.append(("irecv", q, q))
    return ops


class LoopbackHub:
    """In-process point-to-point transport between virtual ranks with RCCL's
    stream semantics, so the real-rank branch of ``_SliceExchange`` (side
    stream, ``batch_isend_irecv``, ``Work.wait``) runs on one GPU, where RCCL
    itself refuses two ranks (profiles/r3w_rccl_same_gpu_probe.txt).

    Each rank has its own transport stream (RCCL's internal stream).  At issue
    an isend / irecv records an event on the stream that is current then (the
    caller's side stream), as RCCL makes its stream wait on the current one.
    A send from r to d is matched with d's receive from r in posting order;
    the pair becomes one device copy on the sender's transport stream after
    both events, and both Works complete with it: ``Work.wait()`` makes the
    current stream wait for that copy (RCCL's ``Work.wait``).  Waiting on an
    unmatched op raises (with RCCL it would spin until the peer posts).
    ``log`` records (rank, kind, peer) per op for the op-list check."""

    def __init__(self, world: int):
        import torch

        self.world = world
        self.streams = [torch.cuda.Stream() for _ in range(world)]
        self.pending = {}  # (src, dst) -> list of ("send" | "recv", tensor, event, work)
        self.log = []

    def group(self, rank: int) -> "LoopbackGroup":
        return LoopbackGroup(self, rank)

    def _post(self, kind, rank, peer, tensor):
        import torch

        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream())
        work = _LoopbackWork()
        key = (rank, peer) if kind == "isend" else (peer, rank)
        q = self.pending.setdefault(key, [])
        self.log.append((rank, kind, peer))
        side = "send" if kind == "isend" else "recv"
        other = next((i for i, e in enumerate(q) if e[0] != side), None)
        if other is None:
            q.append((side, tensor, ev, work))
            return work
        o_side, o_tensor, o_ev, o_work = q.pop(other)
        snd, rcv = (tensor, o_tensor) if side == "send" else (o_tensor, tensor)
        src_rank = key[0]
        st = self.streams[src_rank]
        st.wait_event(ev)
        st.wait_event(o_ev)
        if snd.shape != rcv.shape:
            raise RuntimeError(f"loopback: send {tuple(snd.shape)} != recv {tuple(rcv.shape)}")
        with torch.cuda.stream(st):
            rcv.copy_(snd)
            done = torch.cuda.Event()
            done.record(st)
        work.done = o_work.done = done
        return work


class _LoopbackWork:
    done = None

    def wait(self):
        import torch

        if self.done is None:
            raise RuntimeError("loopback: wait() on an op its peer has not posted")
        torch.cuda.current_stream().wait_event(self.done)


class LoopbackGroup:
    """One virtual rank's view of a LoopbackHub, with the torch.distributed
    point-to-point surface ``_SliceExchange`` uses (``P2POp``, ``isend``,
    ``irecv``, ``batch_isend_irecv``)."""

    def __init__(self, hub: LoopbackHub, rank: int):
        self.hub, self.rank = hub, rank

    # module-like surface (the group passed as the ops' group is this object)
    def isend(self):  # marker, as torch.distributed.isend in P2POp
        raise NotImplementedError

    def irecv(self):
        raise NotImplementedError

    class P2POp:
        def __init__(self, op, tensor, peer, group):
            self.op, self.tensor, self.peer, self.group = op, tensor, peer, group

    def batch_isend_irecv(self, ops):
        works = []
        for o in ops:
            kind = "isend" if o.op == o.group.isend else "irecv"
            works.append(self.hub._post(kind, self.rank, o.peer, o.tensor))
        return works


class _SliceExchange:
    """All-to-all of one period as S slice transfers, each started as soon as
    its slice has been kicked.

    A shard's top n_global local bits number its chunks (chunk c goes to rank
    c), the next slice_bits number the slices of every chunk.  Step s sends
    slice s of every chunk to its rank and receives slice s of this rank's
    chunk from every rank -- all peers at once, so every xGMI link carries a
    transfer (one ``batch_isend_irecv`` of 7 sends and 7 receives at 8 ranks,
    ``slice_p2p_plan``; the local slice is a device copy).  The transfers run
    on a side stream that waits for the slice's kick (an event on the engine
    stream); the engine stream waits for all of them before the fused pass.
    Virtual ranks (one process): slice s of every chunk of every shard is
    copied to its shard on the side stream, or -- ``inplace`` -- swapped with
    its partner piece in the same buffer on the engine stream
    (``dtc_shard_exchange_slice``: no second state buffer, so an L=34 state
    fits one GPU).  CPU tensors (gloo tests): the same transfers,
    synchronously."""

    def __init__(self, stepper, W, S, rank, world, group, inplace=False, slice_bits=0):
        import torch

        self.W, self.S, self.rank, self.world, self.group = W, S, rank, world, group
        self.inplace, self.slice_bits = inplace, slice_bits
        self.fused = False  # set by kick_and_swap (fused in-place kick+exchange)
        self.stepper = stepper
        self.cuda = hasattr(stepper, "stream")
        self.eng = stepper.stream() if self.cuda else None
        self.side = torch.cuda.Stream() if (self.cuda and not inplace) else None
        # the point-to-point layer: torch.distributed (RCCL / gloo), or a
        # virtual rank's LoopbackGroup (same surface, one process)
        if isinstance(group, LoopbackGroup):
            self.comm = group
        else:
            import torch.distributed as dist

            self.comm = dist
        self.works = []
        self.t_events = []  # (start, end) per period, side stream (engine stream in place)

    def _mark_start(self, s, stream):
        import torch

        if s == 0:
            start = torch.cuda.Event(enable_timing=True)
            start.record(stream)
            self.t_events.append([start, None])

    def send(self, s, src, dst, layout=None):
        import torch

        W, S = self.W, self.S
        if self.inplace:
            # one process holds every shard: swap piece (r, c) <-> (c, r) of
            # slice s in place, ordered on the engine stream after its kick
            if self.cuda:
                self._mark_start(s, self.eng)
            self.stepper.exchange_slice(layout, self.slice_bits, s, src)
            return
        if self.cuda:
            ev = torch.cuda.Event()
            ev.record(self.eng)
            self.side.wait_event(ev)
            self._mark_start(s, self.side)
            ctx = torch.cuda.stream(self.side)
        else:
            import contextlib

            ctx = contextlib.nullcontext()
        with ctx:
            if self.world == 1:
                dst.view(W, W, S, -1)[:, :, s].copy_(src.view(W, W, S, -1)[:, :, s].transpose(0, 1))
                return
            sv, dv = src.view(W, S, -1), dst.view(W, S, -1)
            r = self.rank
            dv[r, s].copy_(sv[r, s])
            comm = self.comm
            ops = []
            for kind, peer, chunk in slice_p2p_plan(r, W):
                if kind == "isend":
                    ops.append(comm.P2POp(comm.isend, torch.view_as_real(sv[chunk, s]), peer,
                                          self.group))
                else:
                    ops.append(comm.P2POp(comm.irecv, torch.view_as_real(dv[chunk, s]), peer,
                                          self.group))
            reqs = comm.batch_isend_irecv(ops)
            if self.cuda:
                self.works.extend(reqs)
            else:
                for q in reqs:
                    q.wait()

    def kick_and_swap(self, s, fn):
        """In place: ``fn`` kicks slice s and exchanges it in one step (the
        fused kick+exchange pass, ordered on the engine stream).  Its window
        then holds the slice's kicks too: ``stats`` reports it under
        ``kick_exchange_ms``, not ``exchange_ms``."""
        self.fused = True
        if self.cuda:
            self._mark_start(s, self.eng)
        fn()

    def finish(self):
        import torch

        if not self.cuda:
            return
        if self.inplace:
            end = torch.cuda.Event(enable_timing=True)
            end.record(self.eng)
            self.t_events[-1][1] = end
            return
        with torch.cuda.stream(self.side):
            for w in self.works:
                w.wait()  # the side stream waits for the transfers
            end = torch.cuda.Event(enable_timing=True)
            end.record(self.side)
            self.t_events[-1][1] = end
        self.works = []
        ev = torch.cuda.Event()
        ev.record(self.side)
        self.eng.wait_event(ev)

    def exchange_ms(self):
        return [a.elapsed_time(b) for a, b in self.t_events if b is not None]


def sharded_forward_pipelined(stepper, spec: SweepSpec, n_global: int, *, inst: int = 0,
                              traj: int = 0, seed: int = 0x5EED0001, rank: int = 0,
                              world: int = 1, group=None, buffers=None, stats=None,
                              inplace: bool = False, fuse_kick_exchange: bool = True):
    """``sharded_forward`` with the exchange overlapped and no host round trip
    per period (the C5 schedule on the GPU node).

    Per period: the pre-exchange kicks (every local site group except the one
    holding the top bits, which the previous fused pass already kicked) run
    slice by slice -- chunk c (top n_global local bits = c) is what rank c
    receives, and slice s of every chunk is kicked in one launch -- and slice
    s travels to every peer at once while slice s+1 is kicked; then the fused
    pass (kick of the newly local sites, RZZ/RZ, measurement, next kick of the
    top group) runs on the received shard.  The first period also kicks the top group itself
    (one whole-shard pass) before its chunks.  Observables go to a device
    array; the host reads them once at the end and joins the ranks with one
    all-reduce.  Same results as ``sharded_forward``.

    ``inplace`` (virtual ranks only): one state buffer; each slice's exchange
    swaps the pieces (r, c) and (c, r) in place (``stepper.exchange_slice``,
    dtc_shard_exchange_slice) on the engine stream and the fused pass runs in
    place -- the layout and kernels of the 8-GPU run at a quarter of the memory
    of two buffers (an L=34 state is 256 GiB).  ``buffers`` is then ``(A,)``
    or ``(A, None)``.

    ``stats`` (dict, optional) receives the per-period exchange windows (ms,
    side-stream events; engine-stream events in place) as ``exchange_ms`` and
    the per-period wall of the engine stream (``period_ms``) on the GPU; with
    the fused in-place kick+exchange the windows include the slice kicks and go
    to ``kick_exchange_ms`` instead (``exchange_ms`` is then empty)."""
    return _run_rank(_pipelined_rank(stepper, spec, n_global, inst=inst, traj=traj, seed=seed,
                                     rank=rank, world=world, group=group, buffers=buffers,
                                     stats=stats, inplace=inplace,
                                     fuse_kick_exchange=fuse_kick_exchange), group)


def _run_rank(gen, group):
    """Drive one rank's generator in its own process: exchange marks are
    no-ops, the join is the process group's all-reduce."""
    reply = None
    while True:
        try:
            kind, val = gen.send(reply)
        except StopIteration as e:
            return e.value
        reply = _allreduce(val, group) if kind == "allreduce" else None


def loopback_forward_pipelined(steppers, spec: SweepSpec, n_global: int, *, inst: int = 0,
                               traj: int = 0, seed: int = 0x5EED0001):
    """The real-rank C5 pipeline of 2^n_global ranks in one process on one
    GPU: rank r = ``steppers[r]`` (its own engine context and stream, its own
    two shard buffers), ``_SliceExchange`` in its world-W branch over a
    LoopbackHub (RCCL's stream semantics, device copies).  The ranks advance
    in lock step between the yields of ``_pipelined_rank``; the join sums their
    vectors.  Returns (rank 0's result, the hub's op log)."""
    W = 1 << n_global
    if len(steppers) != W:
        raise ValueError("one stepper per rank")
    hub = LoopbackHub(W)
    gens = [_pipelined_rank(steppers[r], spec, n_global, inst=inst, traj=traj, seed=seed, rank=r,
                            world=W, group=hub.group(r)) for r in range(W)]
    replies = [None] * W
    results = [None] * W
    while True:
        msgs = {}
        for r in range(W):
            try:
                msgs[r] = gens[r].send(replies[r])
            except StopIteration as e:
                results[r] = e.value
        if not msgs:
            break
        kinds = {m[0] for m in msgs.values()}
        if len(msgs) != W or len(kinds) != 1:
            raise RuntimeError(f"loopback ranks out of step: {sorted(msgs)} {kinds}")
        if kinds == {"allreduce"}:
            total = sum(m[1] for m in msgs.values())
            replies = [np.array(total) for _ in range(W)]
        else:
            replies = [None] * W
    return results[0], hub.log


def _pipelined_rank(stepper, spec: SweepSpec, n_global: int, *, inst: int = 0, traj: int = 0,
                    seed: int = 0x5EED0001, rank: int = 0, world: int = 1, group=None,
                    buffers=None, stats=None, inplace: bool = False,
                    fuse_kick_exchange: bool = True):
    """One rank's ``sharded_forward_pipelined`` as a generator: it yields
    ("exchange", None) once a period's slice transfers are all posted (before
    waiting for them) and ("allreduce", vec) for the final join, receiving the
    sum.  ``_run_rank`` drives one process's rank (the yields are no-ops, the
    join is RCCL / gloo); ``loopback_forward_pipelined`` drives all the virtual
    ranks of one GPU in lock step over a LoopbackHub."""
    import torch

    L, T = spec.L, spec.T
    W = 1 << n_global
    if world not in (1, W):
        raise ValueError("world must be 1 (virtual ranks) or 2^n_global")
    n_sh = W // world
    lay = initial_layout(L, n_global, rank * n_sh, n_sh)
    if inplace and world != 1:
        raise ValueError("the in-place exchange needs every shard in one process (world 1)")
    if buffers is not None:
        A, Bf = (tuple(buffers) + (None,))[:2]
    elif inplace:
        A, Bf = stepper.alloc(lay, n_buffers=1)[0], None
    else:
        A, Bf = stepper.alloc(lay)
    if inplace:
        Bf = A
    nl, top, allb = lay.n_local, lay.top_mask, lay.local_mask
    groups = stepper.plan_groups(nl)
    main = next(g for g in groups if (g >> (nl - 1)) & 1)
    if any(g & top for g in groups if g != main):
        raise ValueError("the top local bits must all lie in one site group")
    post_bits = main | top
    # slices: the free bits of the top group just below the rank-swapped bits
    # (above every bit the pre-exchange kicks touch), at most 8 slices, each at
    # least one 4096-amplitude tile per chunk
    tile = getattr(stepper, "min_slice_index_bits", 12)
    pre_top = max((g.bit_length() - 1 for g in groups if g != main), default=-1)
    slice_bits = max(0, min(3, nl - n_global - 1 - pre_top, nl - n_global - tile))
    chunked = nl - n_global - slice_bits >= tile
    S = 1 << slice_bits if chunked else 1
    if inplace and not chunked:
        raise ValueError("the in-place exchange needs chunks of at least one tile")
    P = T - 1 + spec.t_offset
    fuse_kick = fuse_kick_exchange and hasattr(stepper, "kick_exchange_slice")
    obs = stepper.obs_buffer(P + 1, n_sh, 1 + nl)
    layouts = [lay]
    xch = _SliceExchange(stepper, W, S, rank, world, group, inplace=inplace,
                         slice_bits=slice_bits if chunked else 0)
    marks = [] if xch.cuda else None  # engine-stream events, one per period boundary

    def mark():
        if marks is not None:
            e = torch.cuda.Event(enable_timing=True)
            e.record(xch.eng)
            marks.append(e)

    stepper.set_basis(spec, lay, seed, traj, A)
    stepper.step_async(spec, lay, seed, traj, inst, 1, 0, False, 0, A, A, obs[0])
    kicked = 0
    mark()
    for p in range(1, P + 1):
        pre = allb & ~kicked
        if pre & post_bits or not chunked:
            # the first period's top group (its kicks mix the chunks), or every
            # pre-kick when a chunk is smaller than a tile
            whole = pre if not chunked else pre & post_bits
            stepper.step_async(spec, lay, seed, traj, inst, p, whole, False, 0, A, A, None)
            pre &= ~whole
        for sl in range(S):
            if inplace and pre and fuse_kick:
                # one GPU: the slice's last kick pass stores each piece at its
                # partner's place (the exchange costs no pass of its own)
                xch.kick_and_swap(sl, lambda: stepper.kick_exchange_slice(
                    spec, lay, seed, traj, p, pre, slice_bits, sl, A))
                continue
            if pre:
                stepper.kick_slice(spec, lay, seed, traj, p, pre, n_global, slice_bits if chunked
                                   else 0, sl, A)
            xch.send(sl, A, Bf, lay)
        yield ("exchange", None)  # every rank's transfers of the period are posted
        xch.finish()
        lay = lay.exchanged()
        post = post_bits if p < P else 0
        stepper.step_async(spec, lay, seed, traj, inst, p, top, True, post, Bf, A, obs[p])
        layouts.append(lay)
        kicked = post
        mark()
    stepper.synchronize()
    o = obs.cpu().numpy() if hasattr(obs, "cpu") else np.asarray(obs)
    z = np.stack([z_from_obs(layouts[p], o[p]) for p in range(P + 1)])
    z = yield ("allreduce", z)
    zinit = 1.0 if z[0, 1 + spec.probe_site] >= 0 else -1.0
    zs = np.zeros((T, L))
    norm = np.zeros(T)
    for p in range(P + 1):
        t = p - spec.t_offset
        if t >= 0:
            norm[t], zs[t] = z[p, 0], z[p, 1:]
    if stats is not None:
        windows = xch.exchange_ms() if xch.cuda else []
        # fused in place: the windows span the slice kicks as well as the swaps
        stats["exchange_ms"] = [] if xch.fused else windows
        stats["kick_exchange_ms"] = windows if xch.fused else []
        stats["period_ms"] = ([a.elapsed_time(b) for a, b in zip(marks[:-1], marks[1:])]
                              if marks else [])
    fac = (1.0 - spec.p) ** N_ANCILLA_NOISY_GATES
    return {"zsite": zs, "norm": norm, "fwd": fac * zinit * zs[:, spec.probe_site]}
