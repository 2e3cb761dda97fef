"""Multi-rank sharding: world-size-2 ``gloo`` runs.

The union of the ranks' shards, each keyed by global env id, must equal a
single-process run of the whole env range bit for bit, and the counter
reduction must equal the single run's totals.
"""
from __future__ import annotations

import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import dist_worker as W
from ffm_amd.dist import shard_range, weak_shard


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("n,world", [(7, 2), (8, 3), (65536, 8), (5, 5)])
def test_shard_range_partitions(n, world):
    spans = [shard_range(n, r, world) for r in range(world)]
    assert spans[0][0] == 0
    for (b0, c0), (b1, _) in zip(spans, spans[1:]):
        assert b0 + c0 == b1
    assert sum(c for _, c in spans) == n
    assert max(c for _, c in spans) - min(c for _, c in spans) <= 1


def test_shard_range_rejects_bad_input():
    with pytest.raises(ValueError):
        shard_range(1, 0, 2)
    with pytest.raises(ValueError):
        shard_range(8, 2, 2)
    assert weak_shard(65536, 3) == 3 * 65536


def _run_world(backend, n_global, tmp_path, world=2):
    out = str(tmp_path / f"{backend}.npz")
    mp.spawn(W.worker, args=(world, _port(), n_global, backend, out), nprocs=world, join=True)
    return np.load(out)


def _single(run, n_global):
    pos, cnt, dff, eps, c = run(0, n_global)
    mask = np.arange(W.A)[None, :] < cnt[:, None]
    return np.where(mask, pos, 0xFFFF).astype(np.int32), cnt, dff.view(np.int32), c


def test_gloo_world2_sharded_oracle_equals_single_run(tmp_path):
    n = 37   # odd: ranks hold 19 and 18 envs
    got = _run_world("oracle", n, tmp_path)
    pos, cnt, dff, c = _single(W.run_oracle, n)
    assert np.array_equal(got["cnt"], cnt)
    assert np.array_equal(got["pos"], pos)
    assert np.array_equal(got["dff"], dff)
    assert int(got["agent_steps"]) == c["agent_steps"]
    assert int(got["steps"]) == W.STEPS


@pytest.mark.gpu
def test_gloo_world2_sharded_engine_equals_oracle(tmp_path):
    n = 301
    got = _run_world("engine", n, tmp_path)
    pos, cnt, dff, c = _single(W.run_oracle, n)
    assert np.array_equal(got["cnt"], cnt)
    assert np.array_equal(got["pos"], pos)
    assert np.array_equal(got["dff"], dff)
    assert int(got["agent_steps"]) == c["agent_steps"]


LEARN_VARIANTS = [("ac", None), ("unified", "critic_only"), ("unified", "actor_only"), ("unified", "both"),
                  ("actor_only", None)]


@pytest.mark.parametrize("variant,mode", LEARN_VARIANTS)
def test_coupled_learning_shards_equal_single_run(variant, mode):
    """ffm_amd.dist.step_coupled: 3 shards exchanging table deltas == one batch of
    all envs, bit for bit (states and V / H tables); every shard ends with the
    same tables."""
    n = 41
    single, _ = W.run_learn_oracle(variant, mode, 0, n, coupled_shards=1)
    coupled, per = W.run_learn_oracle(variant, mode, 0, n, coupled_shards=3)
    a, b = W.learn_summary(single), W.learn_summary(coupled)
    for k in a:
        assert np.array_equal(a[k], b[k]), k
    for t in per[1:]:
        for k in t:
            assert np.array_equal(t[k], per[0][k]), k
    assert a["eps"].sum() > 0 and len(a["V_keys"]) > 50


@pytest.mark.parametrize("variant,mode", [("unified", "actor_only"), ("unified", "both"), ("actor_only", None)])
def test_sync_period_coupled_equals_single_and_changes_dynamics(variant, mode):
    """A table sync period K = 4 (increments of 4 steps applied together): 3 coupled
    shards == one batch of all envs at the same K, and K = 4 differs from K = 1."""
    n = 41
    one4, _ = W.run_learn_oracle(variant, mode, 0, n, sync_period=4, steps=52)
    three4, _ = W.run_learn_oracle(variant, mode, 0, n, coupled_shards=3, sync_period=4, steps=52)
    one1, _ = W.run_learn_oracle(variant, mode, 0, n, steps=52)
    a, b, c = W.learn_summary(one4), W.learn_summary(three4), W.learn_summary(one1)
    for k in a:
        assert np.array_equal(a[k], b[k]), k
    assert not np.array_equal(a["V_vals"], c["V_vals"]) or len(a["V_keys"]) != len(c["V_keys"])


@pytest.mark.parametrize("sync_period", [1, 4])
@pytest.mark.parametrize("variant,mode", [("unified", "actor_only"), ("actor_only", None), ("ac", None)])
def test_gloo_world2_table_sync_equals_single_run(variant, mode, sync_period, tmp_path):
    """TableSync over a real world-2 gloo group (fixed-capacity delta records, counts
    on the device side, no host sync in the loop) == a single-process batch of all
    envs with the same table sync period."""
    n = 37
    out = str(tmp_path / "learn.npz")
    steps = 52          # a whole number of sync windows: every rank holds every key
    mp.spawn(W.learn_worker, args=(2, _port(), n, variant, mode, out, sync_period, steps), nprocs=2, join=True)
    got = dict(np.load(out))
    single, _ = W.run_learn_oracle(variant, mode, 0, n, sync_period=sync_period, steps=steps)
    want = W.learn_summary(single)
    for k in want:
        assert np.array_equal(got[k], want[k]), k
        if k.startswith(("V_", "H_")):
            assert np.array_equal(got[f"r1_{k}"], want[k]), f"rank 1 {k}"


@pytest.mark.parametrize("variant,mode", [("actor_only", None), ("ac", None)])
def test_gloo_world2_adaptive_record_capacity(variant, mode, tmp_path):
    """TableSync(capacity=None): the record buffers follow the measured touched counts
    (identical on every rank: they come from the all-gathered counts), shrink from the
    generous start to headroom x the observed maximum, and the result is still the
    single-process batch bit for bit."""
    n, steps = 37, 52
    out = str(tmp_path / "learn.npz")
    mp.spawn(W.learn_worker, args=(2, _port(), n, variant, mode, out, 1, steps, True), nprocs=2, join=True)
    got = dict(np.load(out))
    single, _ = W.run_learn_oracle(variant, mode, 0, n, steps=steps)
    want = W.learn_summary(single)
    for k in want:
        assert np.array_equal(got[k], want[k]), k
    caps, mx = got["caps"], got["max_count"]
    assert (mx > 0).all() or variant == "ac"
    assert caps[0] < (1 << 17) and caps[0] >= 1.5 * mx[0]


@pytest.mark.parametrize("variant,mode", [("unified", "actor_only"), ("actor_only", None)])
def test_gloo_world2_flush_mid_period_keeps_ranks_in_step(variant, mode, tmp_path):
    """a sharded K = 4 run that reads its tables in the middle of a period.
    TableSync.flush() exchanges the pending deltas and applies them on every rank at the
    same step, so after it both ranks hold the same tables (== one batch of all envs
    flushed at that step), their periods restart together, and the rest of the run still
    equals the single-process run bit for bit."""
    n, steps, flush_at = 37, 50, 22      # 22 = 5 periods of 4 + 2 pending steps; 28 more: 7 periods
    out = str(tmp_path / "learn.npz")
    mp.spawn(W.learn_worker, args=(2, _port(), n, variant, mode, out, 4, steps, False, flush_at), nprocs=2,
             join=True)
    got = dict(np.load(out))
    single, _, mid = W.run_learn_oracle(variant, mode, 0, n, sync_period=4, steps=steps, flush_at=flush_at)
    want = W.learn_summary(single)
    for k in want:
        assert np.array_equal(got[k], want[k]), k
        if k.startswith(("V_", "H_")):
            assert np.array_equal(got[f"r1_{k}"], want[k]), f"rank 1 {k}"
    for k, v in mid.items():
        for r in (0, 1):
            assert np.array_equal(got[f"mid{r}_{k}"], v), f"rank {r} {k} after the flush"


def test_owner_caps_reconfigure_restarts_from_shape_bounds():
    """OwnerCaps (the owner-sharded exchange's fixed sizes): a new configuration drops the old
    configuration's observations and restarts from the new shape bounds; a record capacity
    below the exact floor is the exact bound (every record to one destination), so a small
    radius curriculum whose crowd lands on one owner cannot overflow."""
    import torch
    from ffm_amd.dist import OwnerCaps
    E, world, nt = 64, 8, 16384
    oc = OwnerCaps(world, E, 10, nt, adapt_every=2, lag=1)
    assert oc.caps[0] == E * 10                        # N = 10: the exact bound (640 records)
    for _ in range(4):                                 # observed: every record to one owner
        rc = torch.full((world, world), 0, dtype=torch.int64)
        rc[0, 0] = E * 10
        oc.observe(rc, torch.tensor([5000]), torch.tensor([9000]))
    assert oc.caps[0] == E * 10                        # never below the exact floor
    oc.reconfigure(90)                                 # the curriculum's next N: 9x the agents
    assert oc.caps[0] == E * 90 and oc.max_seen == [0, 0, 0] and oc.seen == []
    big = OwnerCaps(world, 512, 8192, nt)              # C5: the floor is 65,536 records
    assert big.rfloor == OwnerCaps.exact_floor and big.caps[0] == 2 * 512 * 8192 // world
