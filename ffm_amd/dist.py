"""Env sharding across ranks (one process per GPU), SURVEY.md §8(e).

Envs are independent (model/ffm_core.py:16-21 holds all per-env state), so a
node-wide run is a partition of the global env range into contiguous blocks,
one per rank, with every random draw keyed by the *global* env id (the
engine's ``env_base``).  The data path has no collective; the only exchange is
the end-of-run reduction of counters (sum) and elapsed time (max).
"""
from __future__ import annotations

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
def all_gather_varlen(keys: torch.Tensor, acc: torch.Tensor, n: int, group=None):
    """All-gather each rank's first ``n`` records (keys [cap], acc [cap, width]).

    Counts first, then the records padded to the longest list (one collective
    per array; RCCL on device tensors, gloo on host tensors).  Returns
    (counts, keys [world, m], acc [world, m, width]) with m = max(counts)."""
    world = dist.get_world_size(group)
    cnt = torch.tensor([int(n)], dtype=torch.int64, device=keys.device)
    counts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(counts, cnt, group=group)
    counts = [int(c.item()) for c in counts]
    m = max(counts)
    if m == 0:
        return counts, None, None
    if m > keys.shape[0]:
        raise ValueError(f"record buffers hold {keys.shape[0]} < {m}")
    ks = [torch.empty_like(keys[:m]) for _ in range(world)]
    acs = [torch.empty_like(acc[:m]) for _ in range(world)]
    dist.all_gather(ks, keys[:m].contiguous(), group=group)
    dist.all_gather(acs, acc[:m].contiguous(), group=group)
    return counts, torch.stack(ks), torch.stack(acs)


class TableSync:
    """The batched learning step of one rank's shard, with the V / H table deltas
    exchanged so every rank ends each step with the tables a single device
    holding all envs would have.

    ``shard`` is an ``ffm_amd.engine.Learner`` (records on its device, RCCL) or
    anything with the same phase interface (tests drive the CPU restatement
    through gloo).  Increments are integers (2^-32 fixed point), so the merged sum
    does not depend on rank or arrival order: sharded == single device, bit for bit.
    """

    def __init__(self, shard, group=None, device=None, capacity: int = 1 << 16):
        self.shard = shard
        self.group = group
        self.device = device
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.bufs = {}
        self.capacity = int(capacity)
        self.records_sent = 0

    def _buffers(self, which: str, cap: int):
        width = 1 if which == "V" else 5
        b = self.bufs.get(which)
        if b is None or b[0].shape[0] < cap:
            b = (torch.empty(cap, dtype=torch.int64, device=self.device),
                 torch.empty((cap, width), dtype=torch.int64, device=self.device))
            self.bufs[which] = b
        return b

    def _exchange(self, which: str):
        keys, acc = self._buffers(which, self.capacity)
        n = self.shard.delta_export(which, keys.data_ptr(), acc.data_ptr(), keys.shape[0])
        m = torch.tensor([n], dtype=torch.int64, device=self.device)
        dist.all_reduce(m, op=dist.ReduceOp.MAX, group=self.group)      # every rank holds the longest list
        m = int(m.item())
        if m > keys.shape[0]:
            self.capacity = max(m, 2 * self.capacity)
            keys, acc = self._buffers(which, self.capacity)
            n = self.shard.delta_export(which, keys.data_ptr(), acc.data_ptr(), keys.shape[0])
        counts, gk, ga = all_gather_varlen(keys, acc, n, self.group)
        self.records_sent += n
        for r in range(self.world):
            if r == self.rank or counts[r] == 0:
                continue
            kr, ar = gk[r].contiguous(), ga[r].contiguous()
            self.shard.delta_merge(which, kr.data_ptr(), ar.data_ptr(), counts[r])
            self._keep = (kr, ar)      # alive until the merge has consumed them

    def step(self, n_steps: int = 1):
        s = self.shard
        for _ in range(int(n_steps)):
            s.step_local()
            self._exchange("V")
            if s.actor and not s.post_update:
                self._exchange("H")
            s.step_apply("V")
            if s.actor:
                if s.post_update:
                    self._exchange("H")
                s.step_apply("H")
            s.step_end()


def step_coupled(shards, n_steps: int = 1, device=None, capacity: int = 1 << 16):
    """TableSync's protocol for several shards driven by one process (e.g. one
    Learner per device, or shards of one device): the same phases, with the
    all-gather replaced by handing every shard the others' records."""
    bufs = {}

    def export(i, s, which):
        width = 1 if which == "V" else 5
        cap = capacity
        while True:
            k = torch.empty(cap, dtype=torch.int64, device=device)
            a = torch.empty((cap, width), dtype=torch.int64, device=device)
            n = s.delta_export(which, k.data_ptr(), a.data_ptr(), cap)
            if n <= cap:
                bufs[(i, which)] = (k, a)
                return n
            cap = n

    def exchange(which):
        ns = [export(i, s, which) for i, s in enumerate(shards)]
        for i, s in enumerate(shards):
            for j in range(len(shards)):
                if j != i and ns[j]:
                    k, a = bufs[(j, which)]
                    s.delta_merge(which, k.data_ptr(), a.data_ptr(), ns[j])
            if device is not None and str(device).startswith("cuda"):
                torch.cuda.synchronize()

    for _ in range(int(n_steps)):
        for s in shards:
            s.step_local()
        actor, post = shards[0].actor, shards[0].post_update
        exchange("V")
        if actor and not post:
            exchange("H")
        for s in shards:
            s.step_apply("V")
        if actor:
            if post:
                exchange("H")
            for s in shards:
                s.step_apply("H")
        for s in shards:
            s.step_end()
