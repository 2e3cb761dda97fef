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
                 adapt_every: int = 16, lag: int = 8, tiled_exchange: str = "owner"):
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
        self.backend = dist.get_backend(group)
        self.received_bytes = 0        # per rank, summed over exchanges (owner mode)
        self.bufs = {}
        self.bytes_sent = 0          # per rank, summed over exchanges (what this rank contributes)
        self.exchanges = 0

    def _record_buffers(self, which: str):
        b = self.bufs.get(which)
        if b is None or b[0].shape[0] != self.caps[which]:
            width, cap, w, dev = (2 if which == "V" else 5), self.caps[which], self.world, self.device
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
        if not self.adaptive or self.dense or self.tiled or factor <= 1.0:
            return
        for w in self.caps:
            self.caps[w] = min(self.max_capacity, -(-int(self.caps[w] * factor) // 4096) * 4096)
            self.max_count[w] = max(self.max_count[w], int(self.caps[w] / self.headroom))
        self.capacity = max(self.caps.values())

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

    def _exchange(self, which: str):
        self.exchanges += 1
        (self._exchange_dense if self.dense else self._exchange_records)(which)

    # -- the owner-sharded tiled step ----------------------------------
    def _host(self, t):
        """A small device tensor on the host (the step's size decisions: a host sync)."""
        return t.cpu().numpy()

    def _gather_rows(self, x, n_bytes: int, key):
        """all-gather the first n_bytes of every rank's byte buffer x: [world, n_bytes]
        (a rank whose buffer is shorter sends a zero-padded copy)."""
        n = max(int(n_bytes), 1)
        src = x[:n] if x.numel() >= n else torch.nn.functional.pad(x, (0, n - x.numel()))
        out = self._buf(key, (self.world, n), x.device)
        dist.all_gather([out[r] for r in range(self.world)], src.contiguous(), group=self.group)
        self.received_bytes += (self.world - 1) * n
        self.bytes_sent += n
        return out

    def _buf(self, key, shape, device):
        shape = tuple(shape) if isinstance(shape, (tuple, list)) else (int(shape),)
        b = self.bufs.get(key)
        if b is None or b.numel() < int(np.prod(shape)):
            b = torch.empty(int(np.prod(shape)), dtype=torch.uint8, device=device)
            self.bufs[key] = b
        return b[: int(np.prod(shape))].view(shape)

    def _a2av(self, out, inp, out_splits, in_splits):
        """all-to-all with uneven byte splits (gloo: staged through host memory)."""
        if self.backend == "gloo" and inp.is_cuda:
            ho = torch.empty(out.numel(), dtype=torch.uint8)
            dist.all_to_all_single(ho, inp.cpu(), out_splits, in_splits, group=self.group)
            out.copy_(ho)
        else:
            dist.all_to_all_single(out, inp, out_splits, in_splits, group=self.group)

    def _step_owner(self):
        s, W, r = self.shard, self.world, self.rank
        s.step_owner_local()
        b = s.owner_buffers()
        dev = b["counts"].device
        hs = b["hdr_stride"]
        # 1. the record counts (per destination) and new-slot counts of every rank
        g = self._buf("counts", (W, 8 * (W + 2)), dev)
        dist.all_gather([g[q] for q in range(W)], b["counts"].view(torch.uint8), group=self.group)
        allc = self._host(g).view(np.int64).reshape(W, W + 2)
        send, recv = allc[r, :W], allc[:, r]
        rrecs = self._buf("rrecs", 16 * max(1, int(recv.sum())), dev)
        self._a2av(rrecs[: 16 * int(recv.sum())], b["send_recs"][: 16 * int(send.sum())],
                   [16 * int(x) for x in recv], [16 * int(x) for x in send])
        rhdr = self._buf("rhdr", (W, 4 * hs), dev)
        self._a2av(rhdr.view(-1), b["send_hdr"].reshape(-1), [4 * hs] * W, [4 * hs] * W)
        nmax = max(1, int(allc[:, W:].max()))
        gv = self._gather_rows(b["new_v"], 4 * nmax, "gnewv")
        gh = self._gather_rows(b["new_h"], 4 * nmax, "gnewh")
        s.step_owner_v(rrecs.data_ptr(), rhdr.data_ptr(), recv, gv.data_ptr(), gh.data_ptr(), allc[:, W:], nmax)
        self.received_bytes += 16 * int(recv.sum() - recv[r]) + 4 * hs * (W - 1)
        self.bytes_sent += 16 * int(send.sum() - send[r]) + 4 * hs * (W - 1)
        # 2. the V values every owner updated
        b = s.owner_buffers()
        vc = self._gather_rows(b["out_counts"].view(torch.uint8)[:8], 8, "vcnt")
        vcount = self._host(vc).view(np.int64).reshape(W)
        vmax = max(1, int(vcount.max()))
        gs = self._gather_rows(b["v_slot"], 4 * vmax, "gvs")
        gval = self._gather_rows(b["v_val"], 8 * vmax, "gvv")
        s.step_owner_h(gs.data_ptr(), gval.data_ptr(), vcount, vmax)
        if not s.actor:
            s.step_owner_end(0, 0, None, 0, 0, 0)
            self.exchanges += 1
            return
        # 3. the H increments and tile summaries every owner produced
        hc = self._gather_rows(b["out_counts"].view(torch.uint8)[8:16], 8, "hcnt")
        hcount = self._host(hc).view(np.int64).reshape(W)
        hmax = max(1, int(hcount.max()))
        gk = self._gather_rows(b["h_key"], 4 * hmax, "ghk")
        gq = self._gather_rows(b["h_q"], 8 * hmax, "ghq")
        gt = self._gather_rows(b["tsum"], 40 * hs, "gts")
        s.step_owner_end(gk.data_ptr(), gq.data_ptr(), hcount, hmax, gt.data_ptr(), hs)
        self.exchanges += 1

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

    def flush(self):
        """Apply the increments pending since the last apply (sync period K > 1) on every
        rank, exchanged as at an apply step.  Collective: every rank calls it at the same
        step.  Call it before reading the tables mid-period (an export of a shared learner
        is read-only: it returns the tables as of the last apply)."""
        s = self.shard
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


def _owner_step_coupled(shards):
    """One owner-sharded step of shards coupled in-process: TableSync._step_owner's
    exchanges done by slicing the shards' buffers (one device)."""
    W = len(shards)
    for s in shards:
        s.step_owner_local()
    bs = [s.owner_buffers() for s in shards]
    hs = bs[0]["hdr_stride"]
    allc = torch.stack([b["counts"] for b in bs]).cpu().numpy()
    offs = np.concatenate([np.zeros((W, 1), np.int64), np.cumsum(allc[:, :W], axis=1)], axis=1)
    nmax = max(1, int(allc[:, W:].max()))

    def rows(key, nbytes):
        out = []
        for b in bs:
            x = b[key]
            out.append(x[:nbytes] if x.numel() >= nbytes else torch.nn.functional.pad(x, (0, nbytes - x.numel())))
        return torch.stack(out).contiguous()

    gv, gh = rows("new_v", 4 * nmax), rows("new_h", 4 * nmax)
    keep = [gv, gh]
    for q, s in enumerate(shards):
        recv = allc[:, q]
        recs = torch.cat([bs[r]["send_recs"][16 * int(offs[r, q]): 16 * int(offs[r, q + 1])] for r in range(W)]
                         + [torch.empty(16, dtype=torch.uint8, device=gv.device)])
        hdr = torch.stack([bs[r]["send_hdr"][q] for r in range(W)]).contiguous()
        keep += [recs, hdr]
        s.step_owner_v(recs.data_ptr(), hdr.data_ptr(), recv, gv.data_ptr(), gh.data_ptr(), allc[:, W:], nmax)
    bs = [s.owner_buffers() for s in shards]
    vcount = torch.stack([b["out_counts"][0] for b in bs]).cpu().numpy()
    vmax = max(1, int(vcount.max()))
    gs, gval = rows("v_slot", 4 * vmax), rows("v_val", 8 * vmax)
    for s in shards:
        s.step_owner_h(gs.data_ptr(), gval.data_ptr(), vcount, vmax)
    if not shards[0].actor:
        for s in shards:
            s.step_owner_end(0, 0, None, 0, 0, 0)
    else:
        hcount = torch.stack([b["out_counts"][1] for b in bs]).cpu().numpy()
        hmax = max(1, int(hcount.max()))
        gk, gq, gt = rows("h_key", 4 * hmax), rows("h_q", 8 * hmax), rows("tsum", 40 * hs)
        for s in shards:
            s.step_owner_end(gk.data_ptr(), gq.data_ptr(), hcount, hmax, gt.data_ptr(), hs)
    torch.cuda.synchronize()      # the gathered buffers outlive the kernels that read them
    del keep


def step_coupled(shards, n_steps: int = 1, device=None, capacity: int = 1 << 16, sync_period: int = 1,
                 dense: bool = False, async_records: bool = False, tiled: bool = False, owner: bool = False):
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
        for q, s in enumerate(shards):
            if getattr(s, "_owners", None) != (len(shards), q):
                s.set_tile_owners(len(shards), q)
                s._owners = (len(shards), q)
        for _ in range(int(n_steps)):
            _owner_step_coupled(shards)
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
        width = 2 if which == "V" else 5
        k = torch.zeros(capacity, dtype=torch.int64, device=device)
        a = torch.zeros((capacity, width), dtype=torch.int64, device=device)
        c = torch.zeros(1, dtype=torch.int64, device=device)
        s.delta_export_async(which, k.data_ptr(), a.data_ptr(), capacity, c.data_ptr())
        return k, a, c

    def export(s, which):
        width = 2 if which == "V" else 5   # accumulator words (V: sum of td, visits)
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
