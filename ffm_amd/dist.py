"""Env sharding across ranks (one process per GPU), SURVEY.md §8(e).

Envs are independent (model/ffm_core.py:16-21 holds all per-env state), so a
node-wide run is a partition of the global env range into contiguous blocks,
one per rank, with every random draw keyed by the *global* env id (the
engine's ``env_base``).  The data path has no collective; the only exchange is
the end-of-run reduction of counters (sum) and elapsed time (max).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


def shard_range(n_global: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous block of the global env range owned by ``rank``: (env_base, count).

    Blocks differ in size by at most one env (the first ``n_global % world``
    ranks take one extra), so any ``n_global >= world`` is valid.
    """
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    if n_global < world:
        raise ValueError(f"{n_global} envs cannot be split over {world} ranks")
    q, r = divmod(n_global, world)
    count = q + (1 if rank < r else 0)
    base = rank * q + min(rank, r)
    return base, count


def weak_shard(envs_per_rank: int, rank: int) -> int:
    """env_base of ``rank`` when every rank steps ``envs_per_rank`` envs (weak scaling)."""
    return rank * envs_per_rank


_KEYS = ("agent_steps", "exits", "resets", "steps")


def reduce_counters(counters: dict, device=None, group=None) -> dict:
    """Sum the engine counters over ranks (``steps`` is per-launch, so max)."""
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return dict(counters)
    t = torch.tensor([int(counters[k]) for k in _KEYS[:3]], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    s = torch.tensor([int(counters["steps"])], dtype=torch.int64, device=device)
    dist.all_reduce(s, op=dist.ReduceOp.MAX, group=group)
    out = {k: int(v) for k, v in zip(_KEYS[:3], t.tolist())}
    out["steps"] = int(s.item())
    return out


def reduce_max(x: float, device=None, group=None) -> float:
    """Max of a float over ranks (the bench's elapsed time)."""
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


# ---------------------------------------------------------------------------
# Learning variants: the tables are shared by every env of every rank
# ---------------------------------------------------------------------------
_OWN_CHUNK = 64     # tiles per ownership chunk (learn_kernels.h kOwnChunk)


def owner_tiles(nt: int, world: int, q: int, chunk: int = _OWN_CHUNK) -> int:
    """Tiles rank q owns (learn_kernels.h owner_tiles: chunks of 64 dealt round-robin)."""
    if world <= 1:
        return nt
    nch, rem = divmod(nt, chunk)
    n = ((nch - 1 - q) // world + 1) * chunk if nch > q else 0
    return n + (rem if rem and nch % world == q else 0)


def _tiles_of(shard) -> int:
    h, w = np.asarray(shard.map).shape
    return (h * w + 3) // 4


def _row_width(shard, which: str) -> int:
    """Accumulator words per table entry: V 2 (sum of td, visits), H one per action (5 with
    the Neumann neighbourhood, 9 with Moore's)."""
    return 2 if which == "V" else int(getattr(shard, "n_actions", 5))


class OwnerCaps:
    """Fixed sizes of the owner-sharded exchange (records per destination block, V values and H
    increments per rank and step), so a step's collectives are queued without waiting for the
    GPU.  They start from bounds of the shapes (generous, and exact for V and H: a rank's tiles
    hold tiles * 1,024 slots), then follow the counts observed: every rank copies the gathered
    counts (identical everywhere) to pinned memory behind the exchange, and every `adapt_every`
    exchanges the capacities become `headroom` x the largest count observed so far, from the
    window `lag` exchanges back (the host waits only for copies that old).  They never fall
    below what any observed step needed; a count past its capacity is an error reported at the
    next sync point (never a silent drop).  `fixed` = (records, v, h) disables the adaptation."""

    exact_floor = 1 << 16    # records: 1 MB per destination block

    def __init__(self, world: int, e_max: int, agents: int, n_tiles: int, fixed=None, headroom=(1.25, 1.5, 1.5),
                 adapt_every: int = 8, lag: int = 4, granule: int = 4096, actions: int = 5):
        # records per destination move slowly (agents are conserved, the rows dealt round-robin);
        # the V / H output counts follow the crowding of the rooms: more headroom
        self.world, self.granule = int(world), int(granule)
        self.headroom = tuple(float(h) for h in headroom) if isinstance(headroom, (tuple, list)) else (float(headroom),) * 3
        self.adapt_every, self.lag = int(adapt_every), int(lag)
        self.e_max = int(e_max)
        ntk = max(owner_tiles(int(n_tiles), self.world, q) for q in range(self.world))
        self.vmax = max(1, ntk * 1024)                       # slots one rank owns
        self.actions = int(actions)                          # H row values: 5 Neumann, 9 Moore
        self.hmax = self.actions * self.vmax
        self.adaptive = fixed is None
        if fixed is not None:
            self.rmax = max(1, self.e_max * int(agents))
            self.rfloor = 0
            self.caps = tuple(int(x) for x in fixed)
        else:
            self.reconfigure(agents)

    def reconfigure(self, agents: int):
        """A new configuration (agent count or placement region) starts: restart the adaptation
        from the shape bounds of `agents` agents per env.  The counts observed under the old
        configuration say nothing about the new one (a radius-3 crowd lands on one owner's rows,
        a full room spreads over all), so they are dropped rather than scaled.  The record
        capacity never falls below `exact_floor` records: up to that size it is the exact bound
        (every record of this rank to one destination), so small configurations cannot
        overflow however their crowd is dealt.  Every rank calls it at the same step."""
        self.rmax = max(1, self.e_max * int(agents))         # one rank's records, all to one destination
        self.rfloor = min(self.rmax, self.exact_floor)
        if self.adaptive:
            r0 = min(self.rmax, max(self.rfloor, self._round(2.0 * self.rmax / self.world)))
            v0 = min(self.vmax, self.world * r0)
            self.caps = (r0, v0, min(self.hmax, self.actions * v0))
        self.max_seen = [0, 0, 0]
        self.seen = []
        self.n = 0

    def _round(self, x: float) -> int:
        g = self.granule
        return max(g, -(-int(x) // g) * g)

    def apply(self, shards):
        for s in shards:
            s.set_owner_capacity(*self.caps)

    def observe(self, rc, vc, hc) -> bool:
        """Queue pinned copies of one exchange's gathered counts; True when the capacities
        changed (the caller applies them before its next step)."""
        if not self.adaptive:
            return False
        cp = []
        for t in (rc, vc, hc):
            if t is None:
                cp.append(None)
                continue
            h = torch.empty(t.shape, dtype=t.dtype, pin_memory=t.is_cuda)
            h.copy_(t, non_blocking=True)
            cp.append(h)
        ev = None
        if rc.is_cuda:
            ev = torch.cuda.Event()
            ev.record()
        self.seen.append((ev, cp))
        self.n += 1
        if self.n % self.adapt_every or len(self.seen) <= self.lag:
            return False
        window = self.seen[: len(self.seen) - self.lag]
        del self.seen[: len(self.seen) - self.lag]
        for e, cs in window:
            if e is not None:
                e.synchronize()              # an exchange `lag` steps back: long done
            for i, h in enumerate(cs):
                if h is not None:
                    self.max_seen[i] = max(self.max_seen[i], int(h.max()))
        hr, hv, hh = self.headroom
        new = (min(self.rmax, max(self.rfloor, self._round(hr * self.max_seen[0]))),
               min(self.vmax, self._round(hv * self.max_seen[1])),
               min(self.hmax, self._round(hh * max(self.max_seen[2], 1))))
        changed = new != self.caps
        self.caps = new
        return changed

    def rescale(self, factor: float):
        """The workload grows by `factor` (more agents per env): scale the capacities and the
        observed maxima up front (the observations lag the change)."""
        if not self.adaptive or factor <= 1.0:
            return
        self.max_seen = [int(m * factor) for m in self.max_seen]
        r, v, h = self.caps
        self.caps = (min(self.rmax, self._round(r * factor)), min(self.vmax, self._round(v * factor)),
                     min(self.hmax, self._round(h * factor)))

class TableSync:
    """The batched learning step of one rank's shard, with the V / H table deltas
    exchanged so every rank ends each sync step with the tables a single device
    holding all envs would have.

    ``shard`` is an ``ffm_amd.engine.Learner`` (buffers on its device, RCCL) or
    anything with the same phase interface (tests drive the CPU restatement through
    gloo).  Increments are integers (2^-32 fixed point), so the merged sum does not
    depend on rank or arrival order: sharded == single device, bit for bit, in table
    values (hashed tables' insertion order -- the dict order of get_v_table /
    get_h_table -- differs between ranks).

    No host synchronisation inside the step loop: the record counts stay on the
    device (fixed-capacity record buffers; a step that touches more entries than the
    capacity is reported as an error at the next sync point, never silently).

    * record capacity: ``capacity`` records per rank and table; ``capacity=None``
      sizes it from the touched counts actually measured: every rank copies the
      all-gathered counts (identical on every rank) to pinned host memory behind the
      exchange, and every ``adapt_every`` exchanges the capacity becomes
      ``headroom`` x the largest count observed so far (4 K-record granularity, in
      [1,024, ``max_capacity``]; it never shrinks below what any step needed).  The
      window lags ``lag`` exchanges behind the host, whose copies it waits for (a
      bounded queue depth, not a sync), so every rank decides on the same numbers at
      the same exchange.

    * ``dense`` (default: the shard's tables are dense, i.e. ffm_unified): the whole
      fixed-point accumulator array is all-reduced (SUM; RCCL runs it as
      reduce-scatter + all-gather) and the presence bitmaps are OR-ed, instead of
      exporting touched records;
    * ``tiled`` (default: the shard is a tiled learner -- ffm_unified at block size 1 on a
      large map -- with equal env counts on every rank, at K = 1): every rank all-gathers
      the others' per-agent records (16 B each) and tile offsets (2 B per env and tile of
      4 cells) and sums them per tile of
      cells into its replicated tables: the exchange is proportional to the
      agents stepped, not to the table (C5: 84 MB per rank per step instead of 940 MB of
      accumulators);
    * ``sync_period`` K: the tables are applied (and exchanged) every K-th step only,
      the increments of K steps accumulating in between
      (``Learner.set_sync_period``); K = 1 is the reference's per-step update.
    """

    def __init__(self, shard, group=None, device=None, capacity: int | None = 1 << 16, sync_period: int = 1,
                 dense: bool | None = None, max_capacity: int = 1 << 20, headroom: float = 1.5,
                 adapt_every: int = 16, lag: int = 8, tiled_exchange: str = "owner", owner_caps=None):
        self.shard = shard
        self.group = group
        self.device = device
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.adaptive = capacity is None
        self.max_capacity = int(max_capacity)
        self.headroom = float(headroom)
        self.adapt_every, self.lag = int(adapt_every), int(lag)
        # adaptive: start generous (the first window measures), then follow the counts
        self.caps = {w: (min(1 << 17, self.max_capacity) if capacity is None else int(capacity)) for w in ("V", "H")}
        self.capacity = max(self.caps.values())
        self.seen = {"V": [], "H": []}      # (event, pinned gathered counts) per exchange
        self.n_ex = {"V": 0, "H": 0}
        self.max_count = {"V": 0, "H": 0}   # largest touched count observed (reported)
        self.sync_period = int(sync_period)
        shard.set_sync_period(self.sync_period)
        if hasattr(shard, "set_external_sync"):
            shard.set_external_sync(True)   # exports read-only; pending increments flushed collectively
        self.dense = bool(getattr(shard, "dense_tables", False)) if dense is None else bool(dense)
        # Tiled mode needs every rank tiled (a per-process property: FFM_TILED, sizes) with
        # equal env counts (records are indexed [rank * E + env]).  Every rank takes part in
        # the same collective, whatever its own flag, so a disagreement falls back instead
        # of leaving some ranks inside a collective the others never enter.
        local_tiled = bool(getattr(shard, "tiled", False)) and self.sync_period == 1 and dense is None
        local_owner = local_tiled and bool(getattr(shard, "tile_major", False))
        n_envs = int(getattr(shard, "n_envs", getattr(shard, "E", 0)))
        v = torch.tensor([int(local_tiled), int(local_owner), n_envs, -n_envs], dtype=torch.int64, device=device)
        dist.all_reduce(v, op=dist.ReduceOp.MIN, group=group)
        # owner: the tiles are dealt to the ranks, each sums its own tiles' records from all
        # ranks; replicated: every rank sums every rank's records (9.7)
        self.owner = bool(v[1].item()) and tiled_exchange == "owner"
        self.tiled = self.owner or (bool(v[0].item()) and int(v[2].item()) == -int(v[3].item()))
        if self.owner:
            shard.set_tile_owners(self.world, self.rank)
            # the exchange sizes are fixed per step (no host sync inside a step): initial
            # capacities from the shapes, then the counts observed (identical on every rank)
            self.ocaps = OwnerCaps(self.world, -int(v[3].item()), int(getattr(shard, "A", 0)),
                                   int(getattr(shard, "NT", 0)) or _tiles_of(shard), fixed=owner_caps,
                                   actions=_row_width(shard, "H"))
            self.ocaps.apply([shard])
        self.backend = dist.get_backend(group)
        self.received_bytes = 0        # per rank, summed over exchanges (owner mode)
        self.bufs = {}
        self.bytes_sent = 0          # per rank, summed over exchanges (what this rank contributes)
        self.exchanges = 0

    def _record_buffers(self, which: str):
        b = self.bufs.get(which)
        if b is None or b[0].shape[0] != self.caps[which]:
            width, cap, w, dev = _row_width(self.shard, which), self.caps[which], self.world, self.device
            b = (torch.zeros(cap, dtype=torch.int64, device=dev),
                 torch.zeros((cap, width), dtype=torch.int64, device=dev),
                 torch.zeros(1, dtype=torch.int64, device=dev),
                 torch.zeros((w, cap), dtype=torch.int64, device=dev),
                 torch.zeros((w, cap, width), dtype=torch.int64, device=dev),
                 torch.zeros(w, dtype=torch.int64, device=dev))
            self.bufs[which] = b
        return b

    def _exchange_records(self, which: str):
        keys, acc, cnt, gk, ga, gc = self._record_buffers(which)
        cap = keys.shape[0]
        self.shard.delta_export_async(which, keys.data_ptr(), acc.data_ptr(), cap, cnt.data_ptr())
        dist.all_gather([gc[r:r + 1] for r in range(self.world)], cnt, group=self.group)
        dist.all_gather([gk[r] for r in range(self.world)], keys, group=self.group)
        dist.all_gather([ga[r] for r in range(self.world)], acc, group=self.group)
        for r in range(self.world):
            if r != self.rank:
                self.shard.delta_merge_async(which, gk[r].data_ptr(), ga[r].data_ptr(), gc[r:r + 1].data_ptr(), cap)
        self.bytes_sent += 8 + keys.numel() * 8 + acc.numel() * 8
        self.received_bytes += (self.world - 1) * (8 + keys.numel() * 8 + acc.numel() * 8)
        if self.adaptive:
            self._observe(which, gc)

    def _observe(self, which: str, gc):
        """Queue a copy of the gathered counts; every adapt_every exchanges resize the
        record buffers from the counts of the window that ended `lag` exchanges ago."""
        host = torch.empty(gc.shape, dtype=gc.dtype, pin_memory=gc.is_cuda)
        host.copy_(gc, non_blocking=True)
        ev = None
        if gc.is_cuda:
            ev = torch.cuda.Event()
            ev.record()
        seen = self.seen[which]
        seen.append((ev, host))
        self.n_ex[which] += 1
        i = self.n_ex[which]
        if i % self.adapt_every or len(seen) <= self.lag:
            return
        window = seen[: len(seen) - self.lag]
        del seen[: len(seen) - self.lag]
        m = 0
        for e, h in window:
            if e is not None:
                e.synchronize()             # an exchange `lag` steps back: already done
            m = max(m, int(h.max()))
        # the capacity follows the largest count ever observed, never a window's: counts
        # fall near episode ends and jump back after lockstep resets, faster than the
        # window-old estimate could grow again
        self.max_count[which] = max(self.max_count[which], m)
        need = int(self.headroom * self.max_count[which])
        cap = min(max(1024, -(-need // 4096) * 4096), self.max_capacity)   # 4 K-record granularity
        self.caps[which] = cap
        self.capacity = max(self.caps.values())

    def rescale(self, factor: float):
        """The workload is about to grow by `factor` (e.g. a per-N driver raising N): scale the
        adaptive record capacities up front, since the observed counts lag the change by the
        adaptation window (a touched count jumping past the capacity is an error).  Every rank
        calls it with the same factor at the same step; it never shrinks a capacity."""
        if self.owner and factor > 1.0 and self.ocaps.adaptive:
            self.ocaps.rescale(factor)
            self.ocaps.apply([self.shard])
            return
        if not self.adaptive or self.dense or self.tiled or factor <= 1.0:
            return
        for w in self.caps:
            self.caps[w] = min(self.max_capacity, -(-int(self.caps[w] * factor) // 4096) * 4096)
            self.max_count[w] = max(self.max_count[w], int(self.caps[w] / self.headroom))
        self.capacity = max(self.caps.values())

    def reconfigure(self, agents: int, prev_agents: int | None = None):
        """A driver starts a new configuration of `agents` agents per env (a curriculum's next
        (radius, N), a per-N driver's next N).  Owner mode restarts its capacities from the
        new shape bounds (OwnerCaps.reconfigure); the hashed record exchange scales its
        capacity up front when N grows (`rescale`).  Collective in effect: every rank calls it
        with the same arguments at the same step (no communication of its own)."""
        if self.owner:
            if self.ocaps.adaptive:
                self.ocaps.reconfigure(agents)
                self.ocaps.apply([self.shard])
            return
        if prev_agents:
            self.rescale(agents / prev_agents)

    def _exchange_dense(self, which: str):
        acc, present = self.shard.dense_buffers(which)
        dist.all_reduce(acc, op=dist.ReduceOp.SUM, group=self.group)
        g = self.bufs.get(("present", which))
        if g is None:
            g = torch.empty((self.world, present.numel()), dtype=present.dtype, device=present.device)
            self.bufs[("present", which)] = g
        dist.all_gather([g[r] for r in range(self.world)], present, group=self.group)
        uni = g[0].clone()
        for r in range(1, self.world):
            uni.bitwise_or_(g[r])
        self.shard.dense_adopt(which, uni.data_ptr())
        self._keep = uni                 # until the adopt kernel (same stream) has read it
        self.bytes_sent += acc.numel() * 8 + present.numel() * 4
        # a ring all-reduce receives 2 (W - 1) / W of the array; the all-gather W - 1 bitmaps
        self.received_bytes += (2 * (self.world - 1) * acc.numel() * 8) // self.world + \
            (self.world - 1) * present.numel() * 4

    def _exchange(self, which: str):
        self.exchanges += 1
        (self._exchange_dense if self.dense else self._exchange_records)(which)

    # -- the owner-sharded tiled step ----------------------------------
    def _buf(self, key, shape, device, dtype=None):
        shape = tuple(shape) if isinstance(shape, (tuple, list)) else (int(shape),)
        dtype = dtype or torch.uint8
        n = int(np.prod(shape))
        b = self.bufs.get(key)
        if b is None or b.numel() < n or b.dtype != dtype:
            b = torch.empty(n, dtype=dtype, device=device)
            self.bufs[key] = b
        return b[:n].view(shape)

    def _gather(self, x, key):
        """all-gather of a fixed-size device buffer: [world, *x.shape]."""
        out = self._buf(key, (self.world,) + tuple(x.shape), x.device, x.dtype)
        dist.all_gather([out[r] for r in range(self.world)], x.contiguous(), group=self.group)
        nb = x.numel() * x.element_size()
        self.received_bytes += (self.world - 1) * nb
        self.bytes_sent += nb
        return out

    def _a2a(self, out, inp):
        """all-to-all with equal splits (gloo: staged through host memory)."""
        if self.backend == "gloo" and inp.is_cuda:
            ho = torch.empty(out.numel(), dtype=out.dtype)
            dist.all_to_all_single(ho, inp.cpu(), group=self.group)
            out.copy_(ho)
        else:
            dist.all_to_all_single(out, inp, group=self.group)
        nb = inp.numel() * inp.element_size() * (self.world - 1) // self.world
        self.received_bytes += nb
        self.bytes_sent += nb

    def _step_owner(self):
        """One owner-sharded step, queued without a host synchronisation: every collective has a
        fixed size (OwnerCaps), the counts travel on the device beside the data."""
        s, W = self.shard, self.world
        s.step_owner_local()
        b = s.owner_buffers()
        dev = b["counts"].device
        # 1. the record blocks (equal splits) and header rows, the per-destination counts
        rrecs = self._buf("rrecs", b["send_recs"].numel(), dev)
        self._a2a(rrecs, b["send_recs"])
        rhdr = self._buf("rhdr", b["send_hdr"].numel(), dev)
        self._a2a(rhdr, b["send_hdr"].reshape(-1))
        rc = self._gather(b["counts"], "rcnt")            # [W][W]: observed, never read here
        s.step_owner_v(rrecs.data_ptr(), rhdr.data_ptr())
        # 2. the V values every owner updated
        gvs, gvv = self._gather(b["v_slot"], "gvs"), self._gather(b["v_val"], "gvv")
        gvc = self._gather(b["out_counts"][:1], "gvc")
        s.step_owner_h(gvs.data_ptr(), gvv.data_ptr(), gvc.data_ptr(), b["v_capacity"])
        ghc = None
        if s.actor:
            # 3. the H increments and tile summaries every owner produced
            gk, gq = self._gather(b["h_key"], "ghk"), self._gather(b["h_q"], "ghq")
            ghc = self._gather(b["out_counts"][1:], "ghc")
            gt = self._gather(b["tsum"], "gts")
            s.step_owner_end(gk.data_ptr(), gq.data_ptr(), ghc.data_ptr(), b["h_capacity"], gt.data_ptr(),
                             b["hdr_stride"])
        else:
            s.step_owner_end(0, 0, 0, 0, 0, 0)
        self.exchanges += 1
        if self.ocaps.observe(rc, gvc, ghc):             # a decision window ended: every rank alike
            self.ocaps.apply([s])

    def sync_presence(self):
        """The owner exchange keeps H's key set exact every step, V's lazily: merge the V
        presence bitmaps of all ranks (the slots other ranks inserted join this rank's keys).
        Collective; TableSync.flush() calls it, so exports and table sizes agree everywhere."""
        s = self.shard
        _, present = s.dense_buffers("V")
        g = self._buf("presV", (self.world, present.numel()), present.device, present.dtype)
        dist.all_gather([g[r] for r in range(self.world)], present, group=self.group)
        uni = g[0].clone()
        for r in range(1, self.world):
            uni.bitwise_or_(g[r])
        s.dense_adopt("V", uni.data_ptr())
        torch.cuda.synchronize(present.device) if present.is_cuda else None

    def _step_tiled(self):
        s = self.shard
        s.step_tiled_local()
        recs, tst = s.tiled_buffers()
        g = self.bufs.get("tiled")
        if g is None:
            g = (torch.empty((self.world, recs.numel()), dtype=recs.dtype, device=recs.device),
                 torch.empty((self.world, tst.numel()), dtype=tst.dtype, device=tst.device))
            self.bufs["tiled"] = g
        dist.all_gather([g[0][r] for r in range(self.world)], recs, group=self.group)
        dist.all_gather([g[1][r] for r in range(self.world)], tst, group=self.group)
        s.step_tiled_apply(g[0].data_ptr(), g[1].data_ptr(), self.world * s.n_envs)
        self.exchanges += 1
        self.bytes_sent += recs.numel() * recs.element_size() + tst.numel() * tst.element_size()
        self.received_bytes += (self.world - 1) * (recs.numel() * recs.element_size() +
                                                   tst.numel() * tst.element_size())

    def flush(self):
        """Apply the increments pending since the last apply (sync period K > 1) on every
        rank, exchanged as at an apply step.  Collective: every rank calls it at the same
        step.  Call it before reading the tables mid-period (an export of a shared learner
        is read-only: it returns the tables as of the last apply)."""
        s = self.shard
        if self.owner:
            self.sync_presence()
            return
        if self.tiled or not s.flush_begin():    # the periods advance in lockstep: all ranks agree
            return
        self._exchange("V")
        if s.actor:
            self._exchange("H")
        s.flush_end()

    def step(self, n_steps: int = 1):
        s = self.shard
        if self.tiled:
            for _ in range(int(n_steps)):
                self._step_owner() if self.owner else self._step_tiled()
            return
        for _ in range(int(n_steps)):
            due = s.apply_due()      # host-side state, no device sync
            s.step_local()
            if due:
                self._exchange("V")
                if s.actor and not s.post_update:
                    self._exchange("H")
            s.step_apply("V")
            if s.actor:
                if s.post_update and due:
                    self._exchange("H")
                s.step_apply("H")
            s.step_end()


def _owner_step_coupled(shards, caps: OwnerCaps, bufs: dict):
    """One owner-sharded step of shards coupled in-process: TableSync._step_owner's fixed-size
    exchanges done as device copies between the shards' buffers (one device), queued with no
    host synchronisation."""
    W = len(shards)
    for s in shards:
        s.step_owner_local()
    bs = [s.owner_buffers() for s in shards]
    R, Vc, Hc, hs = bs[0]["rec_capacity"], bs[0]["v_capacity"], bs[0]["h_capacity"], bs[0]["hdr_stride"]
    dev = bs[0]["counts"].device

    # the shards pack into one shared buffer ([source][destination] blocks, set up by
    # _owner_send_buffers), so destination q reads source r's block in place at stride W * R
    big = bufs["send"]
    # header rows [source][destination] -> [destination][source]: two launches, not W * W copies
    hdr = torch.stack([b["send_hdr"] for b in bs]).transpose(0, 1).contiguous()
    bufs["hdr"] = hdr                    # alive until the V / H passes that read it have run
    rc = torch.stack([b["counts"] for b in bs])
    for q, s in enumerate(shards):
        s.step_owner_v(big.data_ptr() + q * 16 * R, hdr[q].data_ptr(), W * R)
    # the V / H outputs were written in place into the gathered buffers (_owner_send_buffers)
    gvs, gvv, gvc = bufs["gvs"], bufs["gvv"], bufs["gvc"]
    for s in shards:
        s.step_owner_h(gvs.data_ptr(), gvv.data_ptr(), gvc.data_ptr(), Vc)
    ghc = None
    if not shards[0].actor:
        for s in shards:
            s.step_owner_end(0, 0, 0, 0, 0, 0)
    else:
        gk, gq, ghc = bufs["ghk"], bufs["ghq"], bufs["ghc"]
        gt = torch.stack([b["tsum"] for b in bs])
        bufs["gts"] = gt
        for s in shards:
            s.step_owner_end(gk.data_ptr(), gq.data_ptr(), ghc.data_ptr(), Hc, gt.data_ptr(), hs)
    if caps.observe(rc, gvc, ghc):
        caps.apply(shards)
        _owner_send_buffers(shards, caps, bufs)


def _owner_send_buffers(shards, caps: OwnerCaps, bufs: dict):
    """One send buffer for all coupled shards: shard r packs its W blocks at [r][0..W)."""
    W, (R, Vc, Hc) = len(shards), caps.caps
    for s in shards:
        s.set_owner_send_buffer(None)
        s.set_owner_output_buffers(None, None)
    for k in ("send", "gvs", "gvv", "gvc", "ghk", "ghq", "ghc"):
        bufs.pop(k, None)
    torch.cuda.synchronize()
    dev = shards[0].owner_buffers()["counts"].device
    big = torch.empty(W * W * R * 16, dtype=torch.uint8, device=dev)
    bufs["send"] = big
    g = {"gvs": torch.empty((W, 4 * Vc), dtype=torch.uint8, device=dev),
         "gvv": torch.empty((W, 8 * Vc), dtype=torch.uint8, device=dev),
         "gvc": torch.zeros(W, dtype=torch.int64, device=dev),
         "ghk": torch.empty((W, 4 * Hc), dtype=torch.uint8, device=dev),
         "ghq": torch.empty((W, 8 * Hc), dtype=torch.uint8, device=dev),
         "ghc": torch.zeros(W, dtype=torch.int64, device=dev)}
    bufs.update(g)
    for r, s in enumerate(shards):
        s.set_owner_send_buffer(big.data_ptr() + r * W * R * 16)
        s.set_owner_output_buffers((g["gvs"][r].data_ptr(), g["gvv"][r].data_ptr(), g["gvc"][r:].data_ptr()),
                                   (g["ghk"][r].data_ptr(), g["ghq"][r].data_ptr(), g["ghc"][r:].data_ptr()))


def sync_presence_coupled(shards):
    """TableSync.sync_presence for coupled shards: the union of the V presence bitmaps."""
    ps = [s.dense_buffers("V")[1] for s in shards]
    uni = ps[0].clone()
    for p in ps[1:]:
        uni.bitwise_or_(p)
    for s in shards:
        s.dense_adopt("V", uni.data_ptr())
    torch.cuda.synchronize()


def step_coupled(shards, n_steps: int = 1, device=None, capacity: int = 1 << 16, sync_period: int = 1,
                 dense: bool = False, async_records: bool = False, tiled: bool = False, owner: bool = False,
                 owner_caps=None):
    """TableSync's protocol for several shards driven by one process (e.g. one
    Learner per device, or shards of one device): the same phases, with the
    collectives replaced by handing every shard the others' records (or, dense,
    the summed accumulators and the presence union).

    ``async_records``: the records travel exactly as TableSync moves them, with no
    host synchronisation: fixed-capacity device buffers filled by
    ``delta_export_async`` (the record count stays in device memory) and read by
    ``delta_merge_async`` (min(count, capacity) records); an export that needs more
    than ``capacity`` is reported at the shard's next sync point."""
    for s in shards:
        s.set_sync_period(sync_period)
    if owner:      # TableSync's owner-sharded exchange: shard q sums the tiles it owns
        W = len(shards)
        st = getattr(shards[0], "_coupled", None)
        if st is None or st[0] != W:
            for q, s in enumerate(shards):
                s.set_tile_owners(W, q)
            caps = OwnerCaps(W, max(s.n_envs for s in shards), shards[0].A, _tiles_of(shards[0]), fixed=owner_caps,
                             actions=_row_width(shards[0], "H"))
            caps.apply(shards)
            st = (W, caps, {})
            _owner_send_buffers(shards, caps, st[2])
            for s in shards:
                s._coupled = st
        for _ in range(int(n_steps)):
            _owner_step_coupled(shards, st[1], st[2])
        if W > 1:
            sync_presence_coupled(shards)  # V's key set, as TableSync.flush() merges it
        return
    if tiled:      # TableSync's tiled exchange: every shard sums all shards' records (equal E)
        for _ in range(int(n_steps)):
            for s in shards:
                s.step_tiled_local()
            bufs = [s.tiled_buffers() for s in shards]
            recs = torch.cat([b[0] for b in bufs])
            tst = torch.cat([b[1] for b in bufs])
            for s in shards:
                s.step_tiled_apply(recs.data_ptr(), tst.data_ptr(), len(shards) * shards[0].n_envs)
            torch.cuda.synchronize()
        return

    def export_async(s, which):
        width = _row_width(s, which)
        k = torch.zeros(capacity, dtype=torch.int64, device=device)
        a = torch.zeros((capacity, width), dtype=torch.int64, device=device)
        c = torch.zeros(1, dtype=torch.int64, device=device)
        s.delta_export_async(which, k.data_ptr(), a.data_ptr(), capacity, c.data_ptr())
        return k, a, c

    def export(s, which):
        width = _row_width(s, which)   # accumulator words (V: sum of td, visits)
        cap = capacity
        while True:
            k = torch.empty(cap, dtype=torch.int64, device=device)
            a = torch.empty((cap, width), dtype=torch.int64, device=device)
            n = s.delta_export(which, k.data_ptr(), a.data_ptr(), cap)
            if n <= cap:
                return k, a, n
            cap = n

    def exchange(which):
        if dense:
            bufs = [s.dense_buffers(which) for s in shards]
            tot = torch.stack([b[0] for b in bufs]).sum(0)
            uni = bufs[0][1].clone()
            for b in bufs[1:]:
                uni.bitwise_or_(b[1])
            for s, b in zip(shards, bufs):
                b[0].copy_(tot)
                s.dense_adopt(which, uni.data_ptr())
            torch.cuda.synchronize()
            return
        if async_records:
            recs = [export_async(s, which) for s in shards]
            for i, s in enumerate(shards):
                for j, (k, a, c) in enumerate(recs):
                    if j != i:
                        s.delta_merge_async(which, k.data_ptr(), a.data_ptr(), c.data_ptr(), capacity)
            torch.cuda.synchronize()      # the record buffers outlive the merges that read them
            return
        recs = [export(s, which) for s in shards]
        for i, s in enumerate(shards):
            for j, (k, a, n) in enumerate(recs):
                if j != i and n:
                    s.delta_merge(which, k.data_ptr(), a.data_ptr(), n)
            if device is not None and str(device).startswith("cuda"):
                torch.cuda.synchronize()

    for _ in range(int(n_steps)):
        due = shards[0].apply_due()
        for s in shards:
            s.step_local()
        actor, post = shards[0].actor, shards[0].post_update
        if due:
            exchange("V")
            if actor and not post:
                exchange("H")
        for s in shards:
            s.step_apply("V")
        if actor:
            if post and due:
                exchange("H")
            for s in shards:
                s.step_apply("H")
        for s in shards:
            s.step_end()
