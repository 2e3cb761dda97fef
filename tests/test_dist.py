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
