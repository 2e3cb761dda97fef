"""Per-rank bodies of the world-size-2 ``gloo`` tests (tests/test_dist.py).

Each rank steps its shard of the global env range (ffm_amd.dist.shard_range),
keyed by global env id, then the shards are gathered on rank 0 and compared
with a single-process run of the whole range.  ``backend`` is the CPU oracle
(tests here) or the HIP engine on cuda:0 (the -m gpu variant).
"""
from __future__ import annotations

import os

import numpy as np
import torch.distributed as dist

PARAMS = {"k_S": 3, "k_D": 1, "diffuse": 0.2, "decay": 0.2, "neighborhood": "neumann"}
SEED, A, STEPS = 42, 32, 40


def room():
    from ffm_amd.data import make_room, l1_sff
    m = make_room(12, 12)
    return m, l1_sff(m)


def run_oracle(env_base, n):
    """Philox-mode run of envs [env_base, env_base+n) on the CPU oracle."""
    from oracle import oracle as O
    m, s = room()
    core = O.Core(m, s, PARAMS)
    pos = np.zeros((n, A), np.uint16)
    for e in range(n):
        pos[e] = core.reset_philox(A, SEED, 0, env_base + e)
    cnt = np.full(n, A, np.int32)
    dff = np.zeros((n, 12, 12), np.float32)
    eps = np.zeros(n, np.int32)
    tot = 0
    for t in range(1, STEPS + 1):
        tot += core.step_philox_batch(pos, cnt, dff, eps, SEED, t, True, A, env_base, 1)
    return pos, cnt, dff.reshape(n, -1), eps, {"agent_steps": tot, "exits": 0, "resets": int(eps.sum()),
                                                "steps": STEPS}


def run_engine(env_base, n):
    """The same on the MI355X through the C ABI (all ranks share cuda:0)."""
    from ffm_amd.engine import Engine
    m, s = room()
    eng = Engine(m, s, n_envs=n, n_agents=A, params=PARAMS, rng="philox", seed=SEED,
                 auto_reset=True, env_base=env_base, device=0)
    eng.reset()
    eng.step(STEPS)
    pos, cnt, dff = eng.get_state()
    eps = eng.get_episodes() if hasattr(eng, "get_episodes") else np.zeros(n, np.int32)
    c = eng.counters()
    eng.close()
    return pos, cnt, dff.reshape(n, -1), eps, c


def worker(rank, world, port, n_global, backend, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ffm_amd.dist import shard_range, reduce_counters
        base, n = shard_range(n_global, rank, world)
        run = run_oracle if backend == "oracle" else run_engine
        pos, cnt, dff, eps, c = run(base, n)
        # live agents only: slots past count are unspecified
        mask = np.arange(A)[None, :] < cnt[:, None]
        pos = np.where(mask, pos, 0xFFFF).astype(np.int32)
        # shards differ in size by one env: gather as objects (small test sizes)
        gathered = []
        for p in (pos, cnt, dff.view(np.int32)):
            parts = [None] * world
            dist.all_gather_object(parts, p)
            gathered.append(np.concatenate(parts))
        red = reduce_counters(c)
        if rank == 0:
            np.savez(out_path, pos=gathered[0], cnt=gathered[1], dff=gathered[2],
                     agent_steps=red["agent_steps"], steps=red["steps"])
    finally:
        dist.destroy_process_group()


# ---------------------------------------------------------------------------
# Learning variants: shards share the V / H tables through TableSync
# ---------------------------------------------------------------------------
LEARN_STEPS, LEARN_N, LEARN_MAX = 50, 16, 30


def learn_params(variant):
    return {"epsilon": 0.1, "block_size": 1} if variant != "ac" else {}


def learn_summary(shards_or_state):
    pos, cnt, dff, eps, est, tabs = shards_or_state
    mask = np.arange(pos.shape[1])[None, :] < cnt[:, None]
    return dict(pos=np.where(mask, pos, 0xFFFF).astype(np.int32), cnt=cnt, dff=dff.reshape(len(cnt), -1).view(np.int32),
                eps=eps, est=est, **tabs)


def sorted_tables(learn):
    out = {}
    for which, T in (("V", learn.V), ("H", learn.Ht)):
        k, v = T.export()
        o = np.argsort(k)
        out[f"{which}_keys"] = k[o]
        out[f"{which}_vals"] = np.asarray(v)[o].view(np.uint64)
    return out


def run_learn_oracle(variant, mode, env_base, n, coupled_shards=1, sync_period=1, steps=LEARN_STEPS,
                     flush_at=None):
    """Single shard (or `coupled_shards` shards coupled in-process) of the batched
    learning step on the CPU restatement, tables applied every `sync_period` steps
    (flush_at: the pending increments applied after that many steps, as
    TableSync.flush does; the tables right after it are returned as well)."""
    from oracle import learn as LO
    from ffm_amd.dist import shard_range, step_coupled
    m, s = room()
    learns, shards = [], []
    for r in range(coupled_shards):
        b, c = shard_range(n, r, coupled_shards)
        L = LO.Learn(m, s, variant, mode, learn_params(variant), log2_cap=20)
        learns.append(L)
        shards.append(LO.Shard(L, c, LEARN_N, LEARN_N, SEED, env_base + b, LEARN_MAX))
    mid = None
    if flush_at is not None:
        assert coupled_shards == 1
        step_coupled(shards, flush_at, device="cpu", sync_period=sync_period)
        if shards[0].flush_begin():
            shards[0].flush_end()
        mid = sorted_tables(learns[0])
        steps -= flush_at
    step_coupled(shards, steps, device="cpu", sync_period=sync_period)
    cat = lambda f: np.concatenate([f(x) for x in shards])
    out = ((cat(lambda x: x.pos), cat(lambda x: x.counts), cat(lambda x: x.dff), cat(lambda x: x.episodes),
            cat(lambda x: x.ep_steps), sorted_tables(learns[0])), [sorted_tables(L) for L in learns])
    return out if flush_at is None else out + (mid,)


def learn_worker(rank, world, port, n_global, variant, mode, out_path, sync_period=1, steps=LEARN_STEPS,
                 adaptive=False, flush_at=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import learn as LO
        from ffm_amd.dist import TableSync, shard_range
        m, s = room()
        base, n = shard_range(n_global, rank, world)
        L = LO.Learn(m, s, variant, mode, learn_params(variant), log2_cap=20)
        shard = LO.Shard(L, n, LEARN_N, LEARN_N, SEED, base, LEARN_MAX)
        if adaptive:   # record capacity sized from the measured touched counts
            sync = TableSync(shard, device="cpu", capacity=None, sync_period=sync_period, adapt_every=4, lag=2)
        else:
            sync = TableSync(shard, device="cpu", capacity=8192, sync_period=sync_period)
        mid = None
        if flush_at is not None:      # a collective flush in the middle of a sync period
            sync.step(flush_at)
            assert not shard.apply_due() or sync_period == 1
            sync.flush()
            assert shard.since_apply == 0
            mids = [None] * world
            dist.all_gather_object(mids, sorted_tables(L))
            mid = mids
            sync.step(steps - flush_at)
        else:
            sync.step(steps)
        assert sync.exchanges > 0
        parts = {}
        for name, a in (("pos", shard.pos), ("cnt", shard.counts), ("dff", shard.dff), ("eps", shard.episodes),
                        ("est", shard.ep_steps)):
            g = [None] * world
            dist.all_gather_object(g, a)
            parts[name] = np.concatenate(g)
        tabs = [None] * world
        dist.all_gather_object(tabs, sorted_tables(L))
        if rank == 0:
            summ = learn_summary((parts["pos"], parts["cnt"], parts["dff"], parts["eps"], parts["est"], tabs[0]))
            for r in range(1, world):      # every rank ends with the same tables
                for k, v in tabs[r].items():
                    summ[f"r{r}_{k}"] = v
            if mid is not None:
                for r in range(world):
                    for k, v in mid[r].items():
                        summ[f"mid{r}_{k}"] = v
            summ["caps"] = np.array([sync.caps["V"], sync.caps["H"]])
            summ["max_count"] = np.array([sync.max_count["V"], sync.max_count["H"]])
            np.savez(out_path, **summ)
    finally:
        dist.destroy_process_group()


def rccl_learn_worker(rank, world, port, variant, mode, n, steps, sync_period, dense, out_path):
    """RCCL (backend "nccl") TableSync over a GPU Learner on cuda:0 (world 1 on the
    one-GPU box: the collectives run through RCCL on device buffers), against one
    Learner stepping the same envs without the exchange, same sync period."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    try:
        from ffm_amd.data import make_room, l1_sff
        from ffm_amd.dist import TableSync
        from ffm_amd.engine import Learner
        m = make_room(12, 12)
        s = l1_sff(m)
        kw = dict(mode=mode, params={"epsilon": 0.1, "block_size": 1}, rng="philox", seed=21, auto_reset=True,
                  max_steps=40, n_envs=n, n_agents=32)
        one = Learner(m, s, variant, **kw)
        one.set_sync_period(sync_period)
        one.reset()
        one.step(steps)
        sh = Learner(m, s, variant, **kw)
        sh.reset()
        sync = TableSync(sh, device="cuda", capacity=1 << 16, sync_period=sync_period, dense=dense)
        sync.step(steps)
        torch.cuda.synchronize()
        res = {"exchanges": np.array(sync.exchanges)}
        for which in ["V"] + (["H"] if one.actor else []):
            for tag, L in (("one", one), ("sync", sh)):
                k, v = L.export_table(which)
                o = np.argsort(k)
                res[f"{tag}_{which}_k"] = np.asarray(k)[o]
                res[f"{tag}_{which}_v"] = np.asarray(v)[o].view(np.uint64)
        for tag, L in (("one", one), ("sync", sh)):
            p, c, d = L.get_state()
            res[f"{tag}_cnt"] = c
            res[f"{tag}_dff"] = d.view(np.uint32)
        one.close()
        sh.close()
        np.savez(out_path, **res)
    finally:
        dist.destroy_process_group()
