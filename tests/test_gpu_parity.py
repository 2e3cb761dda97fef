"""GPU parity: the HIP step (through the C ABI) against the reference's golden
vectors (MT replay) and against the CPU restatement (Philox mode) at scale.

Bars: integer agent positions/counts bit-exact; DFF float32 bit-exact (the
north star allows 1e-5, the kernel meets 0 ULP); RNG streams left in the same
state as the reference's.
"""
import random

import numpy as np
import pytest

from golden_util import case_names, dff_hash, load_case

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.init()


def _engine(**kw):
    from ffm_amd.engine import Engine
    return Engine(**kw)


# ---------------------------------------------------------------------------
# NumPy float32 exp on the device, every float32 in [-104, -0]
# ---------------------------------------------------------------------------
def test_np_expf_device_exhaustive():
    from ffm_amd.engine import np_expf_device
    from oracle import oracle as O
    lo = int(np.float32(-0.0).view(np.uint32))
    hi = int(np.float32(-104.0).view(np.uint32))
    chunk = 1 << 26
    y = torch.empty(chunk, dtype=torch.float32, device="cuda")
    for start in range(lo, hi + 1, chunk):
        n = min(chunk, hi + 1 - start)
        bits = np.arange(start, start + n, dtype=np.uint32)
        x_host = bits.view(np.float32)
        x = torch.from_numpy(bits.view(np.int32)).to("cuda").view(torch.float32)
        np_expf_device(x.data_ptr(), y.data_ptr(), n)
        torch.cuda.synchronize()
        got = y[:n].cpu().numpy().view(np.uint32)
        want = O.np_expf(x_host, nthreads=16).view(np.uint32)
        bad = np.flatnonzero(got != want)
        assert bad.size == 0, f"{bad.size} mismatches, first x={x_host[bad[0]]!r}"


# ---------------------------------------------------------------------------
# MT replay: every golden episode, all seeds of a case batched as envs
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("kernel", ["auto", "block"])
@pytest.mark.parametrize("name", case_names())
def test_engine_replays_reference_goldens(name, kernel):
    """kernel="auto": wave-per-env kernel where A <= 64 (block kernel otherwise);
    kernel="block": the block-per-env kernel forced for every case."""
    case = load_case(name)
    H, W = case.map.shape
    E = len(case.episodes)
    A = case.N
    eng = _engine(map_array=case.map, sff=case.sff, n_envs=E, n_agents=0, agent_capacity=A,
                  params=case.params, rng="mt", auto_reset=False,
                  envs_per_block=1 if kernel == "block" else 0)
    free = np.flatnonzero(case.map.reshape(-1) == 0)
    pos0 = np.full((E, A), 0xFFFF, np.uint16)
    for e, ep in enumerate(case.episodes):
        rs = np.random.RandomState(ep.seed)
        r = random.Random(ep.seed)
        init = free[rs.choice(len(free), case.N, replace=False)]
        assert np.array_equal(init, ep.init)
        pos0[e, :case.N] = init
        eng.load_rng_from(e, rs, r)
    eng.set_state(0, positions=pos0, counts=np.full(E, case.N, np.int32),
                  dff=np.zeros((E, H, W), np.float32))
    T = max(len(ep.counts) for ep in case.episodes)
    for t in range(T):
        eng.step(1)
        pos, cnt, dff = eng.get_state()
        for e, ep in enumerate(case.episodes):
            if t >= len(ep.counts):
                continue
            assert cnt[e] == ep.counts[t], f"seed {ep.seed} step {t}: count"
            assert np.array_equal(pos[e, :cnt[e]], ep.cells[t]), f"seed {ep.seed} step {t}: positions"
            assert dff_hash(dff[e]) == int(ep.hashes[t]), f"seed {ep.seed} step {t}: DFF bits"
            if ep.full:
                assert np.array_equal(dff[e].view(np.uint32), ep.full[t].view(np.uint32))
            if t == len(ep.counts) - 1:
                rs, r = np.random.RandomState(), random.Random()
                eng.store_rng_to(e, rs, r)
                assert list(rs._bit_generator.random_raw(4)) == list(ep.np_tail), "np stream"
                assert [r.getrandbits(32) for _ in range(4)] == list(ep.py_tail), "py stream"
    eng.close()


def test_dropin_model_runs_main_py_config():
    """ffm_amd.model.ffm_core.FloorFieldModel driven like main.py:17-57."""
    import os
    import tempfile
    from ffm_amd.model.ffm_core import FloorFieldModel
    case = load_case("main_50x50_N100")
    ep = case.episodes[0]
    with tempfile.TemporaryDirectory() as td:
        sff_path = os.path.join(td, "sff.npy")
        np.save(sff_path, case.sff)
        np.random.seed(ep.seed)
        random.seed(ep.seed)
        model = FloorFieldModel(case.map.astype(np.int32), sff_path, case.N, dict(case.params))
        W = case.map.shape[1]
        assert np.array_equal(model.positions[:, 0] * W + model.positions[:, 1], ep.init)
        step = 0
        while model.positions.shape[0] > 0:
            model.step()
            p = model.positions
            assert np.array_equal(p[:, 0] * W + p[:, 1], ep.cells[step]), f"step {step}"
            assert dff_hash(model.dff) == int(ep.hashes[step]), f"step {step}: DFF"
            step += 1
        assert step == len(ep.counts)
        assert list(np.random.mtrand._rand._bit_generator.random_raw(4)) == list(ep.np_tail)
        assert [random.getrandbits(32) for _ in range(4)] == list(ep.py_tail)


# ---------------------------------------------------------------------------
# Philox mode: GPU == CPU restatement at scale
# ---------------------------------------------------------------------------
def obstacle_room(H, W):
    """A room with an inner wall (a gap of two cells), a pillar and two exits (top and left
    walls): blocked cells inside the room and two exits' SFF basins."""
    from ffm_amd.data import make_room
    m = make_room(H, W)
    m[H // 2, 1:W - 3] = 2                  # inner wall, open at its right end
    m[H // 4:H // 4 + 2, W // 3:W // 3 + 2] = 2
    m[H - H // 3, 0] = 3                    # second exit in the left wall
    return m


def _philox_compare(H, W, N, E, T, params, seed=42, env_base=0, envs_per_block=0, nthreads=16, fused=1,
                    exit_pos=None, room=None):
    from ffm_amd.data import make_room, l1_sff
    from oracle import oracle as O
    m = room(H, W) if room is not None else make_room(H, W, exit_pos)
    s = l1_sff(m)
    eng = _engine(map_array=m, sff=s, n_envs=E, n_agents=N, params=params, rng="philox",
                  seed=seed, auto_reset=True, env_base=env_base, envs_per_block=envs_per_block)
    core = O.Core(m, s, params)
    pos = np.full((E, N), 0xFFFF, np.uint16)
    cnt = np.zeros(E, np.int32)
    dff = np.zeros((E, H, W), np.float32)
    eps = np.zeros(E, np.int32)
    cpu_steps = 0
    eng.reset()
    # engine.reset() used t=0 for placement; mirror it on the CPU
    for e in range(E):
        pos[e] = core.reset_philox(N, seed, 0, env_base + e)
    cnt[:] = N
    for t in range(1, T + 1):
        cpu_steps += core.step_philox_batch(pos, cnt, dff, eps, seed, t, True, N, env_base, nthreads)
    if fused > 1:
        eng.set_fused_steps(fused)
    eng.step(T)
    gpos, gcnt, gdff = eng.get_state()
    assert np.array_equal(gcnt, cnt), "counts"
    for e in range(E):
        assert np.array_equal(gpos[e, :cnt[e]], pos[e, :cnt[e]]), f"env {e} positions"
    assert np.array_equal(gdff.view(np.uint32), dff.view(np.uint32)), "DFF bits"
    c = eng.counters()
    assert c["agent_steps"] == cpu_steps
    assert c["resets"] == int(eps.sum())
    assert c["steps"] == T
    eng.close()
    return cnt, eps


@pytest.mark.parametrize("epb", [0, -2, -1])
def test_philox_config2_full_size_matches_cpu(epb):
    """12x12, 32 agents, 65,536 envs (BASELINE config 2) for 150 steps (epb=0: auto,
    the group kernel; -2: the lane kernel; -1: the wave kernel)."""
    cnt, eps = _philox_compare(12, 12, 32, 65536, 150,
                               {"k_S": 3, "k_D": 1, "diffuse": 0.2, "decay": 0.2, "neighborhood": "neumann"},
                               envs_per_block=epb)
    assert eps.sum() > 0  # auto-reset exercised


@pytest.mark.parametrize("H,N,E,epb,nbh", [(12, 32, 65536, 0, "neumann"), (12, 32, 4096, -2, "neumann"),
                                          (64, 512, 48, 0, "neumann"), (110, 60, 6, 0, "neumann"),
                                          (12, 32, 4096, 0, "moore"), (64, 512, 48, 0, "moore")])
def test_engine_reset_envs_matches_cpu(H, N, E, epb, nbh):
    """reset(env_mask) through the ABI (ffm_engine_reset_envs): mid-run, a random
    third of the envs is re-placed (C2's 65,536 envs on the group kernel, the lane kernel, and
    C3's 64x64 room); the oracle re-places the same envs with reset_philox at the same step
    index.  Positions, counts, DFF bits and episode counters equal the oracle's, before and
    after the reset, and the unmasked envs are untouched.  The 110x110 room's free list exceeds
    the wave reset's LDS, so it re-places through core_block_reset_kernel's masked form."""
    import torch
    from ffm_amd.data import make_room, l1_sff
    from oracle import oracle as O
    params = {"k_S": 3, "k_D": 1, "diffuse": 0.2, "decay": 0.2, "neighborhood": nbh}
    m = make_room(H, H)
    s = l1_sff(m)
    seed, T1, T2 = 11, 25, 25
    eng = _engine(map_array=m, sff=s, n_envs=E, n_agents=N, params=params, rng="philox", seed=seed,
                  auto_reset=True, envs_per_block=epb)
    core = O.Core(m, s, params)
    pos = np.stack([core.reset_philox(N, seed, 0, e) for e in range(E)])
    cnt = np.full(E, N, np.int32)
    dff = np.zeros((E, H, H), np.float32)
    eps = np.zeros(E, np.int32)
    eng.reset()
    for t in range(1, T1 + 1):
        core.step_philox_batch(pos, cnt, dff, eps, seed, t, True, N, 0, 16)
    eng.step(T1)
    mask = np.random.default_rng(5).random(E) < 0.33
    before = eng.get_state()
    eng.reset_envs(torch.as_tensor(mask.astype(np.uint8)).cuda())   # device mask, read in place
    tr = T1 + 1                                                      # the placement's step index
    gpos, gcnt, gdff = eng.get_state()
    for e in np.flatnonzero(mask):
        pos[e] = core.reset_philox(N, seed, tr, e)
        cnt[e] = N
        dff[e] = 0.0
    keep = ~mask
    assert np.array_equal(gcnt[keep], before[1][keep]) and np.array_equal(gdff[keep], before[2][keep])
    assert np.array_equal(gcnt, cnt), "counts after reset_envs"
    for e in range(E):
        assert np.array_equal(gpos[e, :cnt[e]], pos[e, :cnt[e]]), f"env {e} positions after reset_envs"
    assert np.array_equal(gdff.view(np.uint32), dff.view(np.uint32)), "DFF after reset_envs"
    for t in range(tr + 1, tr + 1 + T2):
        core.step_philox_batch(pos, cnt, dff, eps, seed, t, True, N, 0, 16)
    eng.step(T2)
    gpos, gcnt, gdff = eng.get_state()
    assert np.array_equal(gcnt, cnt), "counts"
    for e in range(E):
        assert np.array_equal(gpos[e, :cnt[e]], pos[e, :cnt[e]]), f"env {e} positions"
    assert np.array_equal(gdff.view(np.uint32), dff.view(np.uint32)), "DFF bits"
    assert eng.counters()["resets"] == int(eps.sum())
    eng.close()


def test_engine_reset_envs_errors():
    """reset_envs is Philox-only (MT engines draw placements on the host) and checks its mask."""
    import torch
    from ffm_amd.data import make_room, l1_sff
    m = make_room(12, 12)
    s = l1_sff(m)
    mt = _engine(map_array=m, sff=s, n_envs=4, n_agents=8, rng="mt", seed=1)
    with pytest.raises(NotImplementedError, match="MT mode"):
        mt.reset_envs(torch.ones(4, dtype=torch.uint8, device="cuda"))
    mt.close()
    ph = _engine(map_array=m, sff=s, n_envs=4, n_agents=8, rng="philox", seed=1)
    with pytest.raises(ValueError, match="n_envs"):
        ph.reset_envs(np.ones(5, np.uint8))
    ph.reset()
    before = ph.get_state()
    ph.reset_envs(np.zeros(4, np.uint8))          # an empty mask re-places nothing
    after = ph.get_state()
    assert all(np.array_equal(x, y) for x, y in zip(before, after))
    ph.close()


@pytest.mark.parametrize("epb", [-3, -2, -1, 3])
@pytest.mark.parametrize("N", [32, 60])
@pytest.mark.parametrize("params", [
    {"k_S": 3, "k_D": 1, "diffuse": 0.2, "decay": 0.2, "neighborhood": "moore"},
    {"k_S": 1.5, "k_D": 2.5, "diffuse": 0.3, "decay": 0.1, "neighborhood": "neumann"},
])
def test_philox_12x12_param_points(params, N, epb):
    """All kernels (epb=-3 / -2: group / lane kernel where A <= 32, else the block
    kernel; -1: wave kernel, 2 or 1 env per wave; 3: block kernel, odd K)."""
    _philox_compare(12, 12, N, 2047, 120, params, seed=7, envs_per_block=epb)


def test_philox_odd_shapes():
    """Non-square room, runtime-dimension wave kernel, few agents (4 envs/wave lanes idle)."""
    _philox_compare(9, 17, 5, 777, 80, {"k_S": 2, "k_D": 1, "diffuse": 0.25, "decay": 0.3,
                                        "neighborhood": "neumann"}, seed=123)
    _philox_compare(20, 11, 40, 301, 80, {"neighborhood": "moore"}, seed=5, env_base=1 << 20)


@pytest.mark.parametrize("epb", [-3, -2, -1, 3])
@pytest.mark.parametrize("nbh", ["neumann", "moore"])
def test_philox_interior_exit_all_kernels(nbh, epb):
    """An exit inside the room (every neighbour of it a free cell: four or eight exit-forced
    requesters of one cell, so exits are contested and decided by friction draws,
    model/ffm_core.py:66-72, 90-98) on every step kernel -- group, lane, wave and block --
    and through K fused steps; positions, counts and DFF equal the CPU restatement."""
    p = {"k_S": 3, "k_D": 1, "diffuse": 0.2, "decay": 0.2, "neighborhood": nbh}
    cnt, eps = _philox_compare(12, 12, 32, 2047, 120, p, seed=17, envs_per_block=epb, exit_pos=(6, 5))
    assert eps.sum() > 0
    if epb == -3:
        _philox_compare(12, 12, 32, 1001, 60, p, seed=18, fused=10, exit_pos=(4, 7))
        _philox_compare(40, 40, 300, 33, 60, p, seed=19, exit_pos=(20, 20))


@pytest.mark.parametrize("epb", [-3, -2, -1, 3])
@pytest.mark.parametrize("nbh", ["neumann", "moore"])
def test_philox_obstacles_and_two_exits_all_kernels(nbh, epb):
    """Blocked cells inside the room (an inner wall with a gap, a pillar) and two exits on
    every step kernel; a 40x40 room of the same layout on the block kernel."""
    p = {"k_S": 3, "k_D": 1, "diffuse": 0.2, "decay": 0.2, "neighborhood": nbh}
    _, eps = _philox_compare(12, 12, 30, 2047, 120, p, seed=27, envs_per_block=epb, room=obstacle_room)
    assert eps.sum() > 0
    if epb == -3:
        _philox_compare(12, 12, 30, 1001, 60, p, seed=28, fused=10, room=obstacle_room)
        _philox_compare(40, 40, 300, 33, 60, p, seed=29, room=obstacle_room)


@pytest.mark.parametrize("epb", [-3, -2])
@pytest.mark.parametrize("E", [1, 5, 333, 5121])
def test_philox_lane_small_and_ragged_env_counts(E, epb):
    """Group / lane kernel with fewer envs than waves, env counts that leave the last
    group or pair part empty."""
    _philox_compare(12, 12, 32, E, 90, {"neighborhood": "neumann"}, seed=11, envs_per_block=epb)


@pytest.mark.parametrize("N", [1, 7, 19])
def test_philox_group_few_agents(N):
    """Group kernel with few agents per env (many envs per chunk, odd position
    strides), Moore and Neumann."""
    _philox_compare(12, 12, N, 3001, 70, {"neighborhood": "neumann"}, seed=21, envs_per_block=-3)
    _philox_compare(12, 12, N, 1003, 70, {"neighborhood": "moore", "k_D": 2}, seed=22, envs_per_block=-3)


def test_philox_lane_shapes():
    """Lane kernel at runtime dimensions: 14x16 Moore (H*W = 224: two DFF slots per
    lane), and an 8x8 room with 3 agents (most lanes idle, slot-less lanes)."""
    _philox_compare(14, 16, 20, 999, 90, {"neighborhood": "moore", "k_D": 2}, seed=3, envs_per_block=-2)
    _philox_compare(8, 8, 3, 1000, 60, {"neighborhood": "neumann"}, seed=4, env_base=12345,
                    envs_per_block=-2)


@pytest.mark.parametrize("fused", [10, 7])
def test_philox_multi_step_config2_full_size(fused):
    """K steps per launch (core_multi_kernel, state on chip) at BASELINE config 2:
    150 steps in launches of 10 (or 7: a short last launch) equal 150 single steps."""
    cnt, eps = _philox_compare(12, 12, 32, 65536, 150,
                               {"k_S": 3, "k_D": 1, "diffuse": 0.2, "decay": 0.2, "neighborhood": "neumann"},
                               fused=fused)
    assert eps.sum() > 0  # inline auto-reset exercised


@pytest.mark.parametrize("args", [
    (12, 12, 32, 2047, 120, {"k_S": 3, "k_D": 1, "diffuse": 0.2, "decay": 0.2, "neighborhood": "moore"}, 9),
    (12, 12, 32, 5, 90, {"neighborhood": "neumann"}, 4),
    (12, 12, 32, 1, 90, {"neighborhood": "neumann"}, 90),
    (14, 16, 20, 999, 90, {"neighborhood": "moore", "k_D": 2}, 8),
    (8, 8, 3, 1000, 60, {"neighborhood": "neumann"}, 16),
    (64, 64, 512, 64, 30, {"neighborhood": "neumann"}, 10),   # not a multi-step shape: one launch per step
])
def test_philox_multi_step_shapes(args):
    H, W, N, E, T, params, k = args
    _philox_compare(H, W, N, E, T, params, seed=31, fused=k)


def test_philox_config3_64x64_matches_cpu():
    """64x64, 512 agents (BASELINE config 3), 512 envs, 60 steps."""
    _philox_compare(64, 64, 512, 512, 60,
                    {"k_S": 3, "k_D": 1, "diffuse": 0.2, "decay": 0.2, "neighborhood": "neumann"})


@pytest.mark.timeout(600)
def test_philox_config3_full_size_matches_cpu():
    """BASELINE config 3 at its full size: 64x64, 512 agents, 8,192 envs (the bench's C3
    grid and block geometry) for 40 steps, every env bit-exact vs the oracle (round 5 covered
    this shape only through the bench's CPU leg)."""
    _philox_compare(64, 64, 512, 8192, 40,
                    {"k_S": 3, "k_D": 1, "diffuse": 0.2, "decay": 0.2, "neighborhood": "neumann"})


def test_philox_big_maps_global_scratch():
    """Maps whose env state exceeds the LDS (the block kernel with its grid, DFF tile and
    u32 padded cells in a global scratch region; placement by workgroups): the BASELINE
    config-5 room 256x256 with 8,192 agents (65,536 cells: padded indices past u16), a
    150x150 room, and a 110x110 room with few agents, so envs empty and auto-reset."""
    p = {"k_S": 3, "k_D": 1, "diffuse": 0.2, "decay": 0.2, "neighborhood": "neumann"}
    _philox_compare(256, 256, 8192, 6, 40, p, seed=5)
    _philox_compare(150, 150, 2000, 16, 60, dict(p, neighborhood="moore"), seed=6, env_base=77)
    _philox_compare(110, 110, 12, 64, 400, p, seed=7)
    # inner walls and two exits beyond the LDS (the global-scratch grid's blocked cells)
    _philox_compare(150, 150, 2000, 8, 40, dict(p, neighborhood="moore"), seed=8, room=obstacle_room)
    _philox_compare(256, 256, 4000, 4, 30, p, seed=9, room=obstacle_room)


@pytest.mark.parametrize("nbh", ["neumann", "moore"])
@pytest.mark.parametrize("H,N,room", [(12, 30, "obstacles"), (12, 30, "interior"), (40, 200, "obstacles")])
def test_mt_rooms_match_oracle_stream(H, N, room, nbh):
    """MT (reference-stream) mode on rooms with inner walls and two exits, and with an exit
    inside the room (contested exits), against the oracle's MT step: positions, DFF bits and
    both generators' positions."""
    import random as pyrandom
    from ffm_amd.data import make_room, l1_sff
    from oracle import oracle as O
    W = H
    m = obstacle_room(H, W) if room == "obstacles" else make_room(H, W, (H // 2, W // 2 - 1))
    s = l1_sff(m).astype(np.float64)
    p = {"k_S": 3, "k_D": 1, "diffuse": 0.2, "decay": 0.2, "neighborhood": nbh}
    E, T = 3, 60
    eng = _engine(map_array=m, sff=s, n_envs=E, n_agents=0, agent_capacity=N, params=p, rng="mt",
                  auto_reset=False)
    core = O.Core(m, s, p)
    pos0 = np.full((E, N), 0xFFFF, np.uint16)
    cpu = []
    for e in range(E):
        rs, r = np.random.RandomState(200 + e), pyrandom.Random(200 + e)
        npr, pyr = O.MT.from_numpy(rs), O.MT.from_python(r)
        init = core.init_agents_mt(N, npr)
        pos0[e] = init
        npr.to_numpy(rs)
        eng.load_rng_from(e, rs, r)
        cpu.append([init, np.zeros((H, W), np.float32), npr, pyr])
    eng.set_state(0, positions=pos0, counts=np.full(E, N, np.int32), dff=np.zeros((E, H, W), np.float32))
    for _ in range(T):
        for c in cpu:
            c[0] = core.step_mt(c[0], c[1], c[2], c[3])
    eng.step(T)
    gp, gc, gd = eng.get_state()
    for e, c in enumerate(cpu):
        assert gc[e] == len(c[0])
        assert np.array_equal(gp[e, :gc[e]], c[0]), f"env {e} positions"
        assert np.array_equal(gd[e].view(np.uint32), c[1].view(np.uint32)), f"env {e} DFF"
        rs, r = np.random.RandomState(), pyrandom.Random()
        eng.store_rng_to(e, rs, r)
        want_np, want_py = np.random.RandomState(), pyrandom.Random()
        c[2].to_numpy(want_np)
        c[3].to_python(want_py)
        assert list(rs._bit_generator.random_raw(4)) == list(want_np._bit_generator.random_raw(4))
        assert [r.getrandbits(32) for _ in range(4)] == [want_py.getrandbits(32) for _ in range(4)]
    eng.close()


def test_mt_big_map_matches_oracle_stream():
    """MT (reference-stream) mode on a map beyond the LDS: 160x160, 600 agents, f64 SFF
    (main.py's data path), against the oracle's MT step (pinned to the reference by the
    golden replays) -- positions, DFF bits and both generators' positions."""
    import random as pyrandom
    from ffm_amd.data import make_room, l1_sff
    from oracle import oracle as O
    H = W = 160
    m = make_room(H, W)
    s = l1_sff(m).astype(np.float64)
    p = {"k_S": 3, "k_D": 1, "diffuse": 0.2, "decay": 0.2, "neighborhood": "neumann"}
    E, N, T = 2, 600, 40
    eng = _engine(map_array=m, sff=s, n_envs=E, n_agents=0, agent_capacity=N, params=p, rng="mt",
                  auto_reset=False)
    core = O.Core(m, s, p)
    pos0 = np.full((E, N), 0xFFFF, np.uint16)
    cpu = []
    for e in range(E):
        rs, r = np.random.RandomState(100 + e), pyrandom.Random(100 + e)
        npr, pyr = O.MT.from_numpy(rs), O.MT.from_python(r)
        init = core.init_agents_mt(N, npr)
        pos0[e] = init
        npr.to_numpy(rs)
        eng.load_rng_from(e, rs, r)
        cpu.append([init, np.zeros((H, W), np.float32), npr, pyr])
    eng.set_state(0, positions=pos0, counts=np.full(E, N, np.int32), dff=np.zeros((E, H, W), np.float32))
    for _ in range(T):
        for c in cpu:
            c[0] = core.step_mt(c[0], c[1], c[2], c[3])
    eng.step(T)
    gp, gc, gd = eng.get_state()
    for e, c in enumerate(cpu):
        assert gc[e] == len(c[0])
        assert np.array_equal(gp[e, :gc[e]], c[0]), f"env {e} positions"
        assert np.array_equal(gd[e].view(np.uint32), c[1].view(np.uint32)), f"env {e} DFF"
        rs, r = np.random.RandomState(), pyrandom.Random()
        eng.store_rng_to(e, rs, r)
        want_np, want_py = np.random.RandomState(), pyrandom.Random()
        c[2].to_numpy(want_np)
        c[3].to_python(want_py)
        assert list(rs._bit_generator.random_raw(4)) == list(want_np._bit_generator.random_raw(4))
        assert [r.getrandbits(32) for _ in range(4)] == [want_py.getrandbits(32) for _ in range(4)]
    eng.close()


def test_sharding_invariance():
    """Envs keyed by global id: two shards == one engine (the multi-GPU contract)."""
    from ffm_amd.data import make_room, l1_sff
    m = make_room(12, 12)
    s = l1_sff(m)
    p = {"neighborhood": "neumann"}
    full = _engine(map_array=m, sff=s, n_envs=4096, n_agents=32, params=p, seed=3)
    a = _engine(map_array=m, sff=s, n_envs=1000, n_agents=32, params=p, seed=3, env_base=0)
    b = _engine(map_array=m, sff=s, n_envs=3096, n_agents=32, params=p, seed=3, env_base=1000)
    for eng in (full, a, b):
        eng.reset()
        eng.step(90)
    fp, fc, fd = full.get_state()
    ap, ac, ad = a.get_state()
    bp, bc, bd = b.get_state()
    assert np.array_equal(fc, np.concatenate([ac, bc]))
    assert np.array_equal(fd, np.concatenate([ad, bd]))
    for e in range(4096):
        q = ap[e] if e < 1000 else bp[e - 1000]
        assert np.array_equal(fp[e, :fc[e]], q[:fc[e]])


def test_full_size_invariants_and_determinism():
    """Size-independent properties at BASELINE config 2 size."""
    from ffm_amd.data import make_room, l1_sff
    m = make_room(12, 12)
    s = l1_sff(m)
    p = {"neighborhood": "neumann"}
    outs = []
    for _ in range(2):
        eng = _engine(map_array=m, sff=s, n_envs=65536, n_agents=32, params=p, seed=11)
        eng.reset()
        eng.step(300)
        outs.append(eng.get_state())
        c = eng.counters()
        eng.close()
    (p1, c1, d1), (p2, c2, d2) = outs
    assert np.array_equal(c1, c2) and np.array_equal(d1.view(np.uint32), d2.view(np.uint32))
    assert np.array_equal(p1, p2)
    assert (c1 >= 0).all() and (c1 <= 32).all()
    assert (d1 >= 0).all() and np.isfinite(d1).all()
    flat = m.reshape(-1)
    for e in range(0, 65536, 97):
        cells = p1[e, :c1[e]]
        assert len(set(cells.tolist())) == len(cells)
        assert (flat[cells] == 0).all()
    assert c["steps"] == 300 and c["agent_steps"] > 0


def test_update_dff_entry_point():
    """ffm_engine_update_dff == the reference's update_dff expression."""
    from ffm_amd.data import make_room, l1_sff
    from oracle import oracle as O
    m = make_room(9, 13)
    s = l1_sff(m)
    rs = np.random.RandomState(5)
    for nbname in ("neumann", "moore"):
        p = {"diffuse": 0.3, "decay": 0.15, "neighborhood": nbname}
        eng = _engine(map_array=m, sff=s, n_envs=3, n_agents=0, agent_capacity=4, params=p, auto_reset=False)
        d = (rs.exponential(1.0, (3, 9, 13)) * (rs.uniform(size=(3, 9, 13)) < 0.6)).astype(np.float32)
        eng.set_state(0, dff=d)
        eng.update_dff()
        _, _, got = eng.get_state()
        core = O.Core(m, s, p)
        for e in range(3):
            want = d[e].copy()
            core.update_dff(want)
            assert np.array_equal(got[e].view(np.uint32), want.view(np.uint32))
        eng.close()


def test_invalid_inputs_raise():
    from ffm_amd.data import make_room, l1_sff
    m = make_room(12, 12)
    s = l1_sff(m)
    with pytest.raises(ValueError):
        _engine(map_array=m, sff=s, n_envs=1, n_agents=101)  # more agents than free cells
    bad = m.copy()
    bad[0, 3] = 0
    with pytest.raises(ValueError):
        _engine(map_array=bad, sff=s, n_envs=1, n_agents=4)  # open border
    eng = _engine(map_array=m, sff=s, n_envs=2, n_agents=4, auto_reset=False)
    with pytest.raises(ValueError):
        eng.set_state(0, positions=np.zeros((1, 4), np.uint16), counts=np.array([2], np.int32))  # wall cell
    eng.close()


def test_philox_block_kernel_capped_placement_keys():
    """Block kernel with more free cells than the LDS key capacity (40x40 room, 16 agents:
    F = 1444 > 2A + 16 + 8 sqrt(2A + 16) + 64): auto-resets draw their placement from the
    thresholded candidates kept in LDS, identical to the oracle's full sort."""
    cnt, eps = _philox_compare(40, 40, 16, 300, 200, {"neighborhood": "neumann"}, seed=13, envs_per_block=1)
    assert eps.sum() > 0


@pytest.mark.parametrize("H,W,N,epb,fused", [(12, 12, 20, 0, 1), (12, 12, 32, 0, 10), (12, 12, 20, -2, 1),
                                             (20, 24, 60, 2, 1)])
def test_engine_trajectory_capture_matches_cpu(H, W, N, epb, fused):
    """Batched positions log (model/ffm_core.py:119-133 run(), main.py:44-54 positions_log):
    the rows captured after every step of every selected episode equal the CPU
    restatement's positions after that step, and each episode ends with the empty row of
    the step that emptied the room (before the auto-reset re-placed it).  Capture turns
    fused steps off (one launch per step); the group, lane and block kernels."""
    from ffm_amd.data import make_room, l1_sff
    from oracle import oracle as O
    m = make_room(H, W)
    s = l1_sff(m)
    p = {"k_S": 3, "k_D": 1, "diffuse": 0.2, "decay": 0.2, "neighborhood": "neumann"}
    E, T, seed = 300, 160, 13
    sel = np.array([0, 7, 100, 298, 299], np.int32)
    ph = np.array([0, 1, 0, 1, 1], np.int32)
    eng = _engine(map_array=m, sff=s, n_envs=E, n_agents=N, params=p, rng="philox", seed=seed, auto_reset=True,
                  envs_per_block=epb)
    if fused > 1:
        eng.set_fused_steps(fused)
    eng.set_trajectory_capture(sel, period=2, phases=ph, capacity_rows=len(sel) * 64)
    eng.reset()
    got = {}
    for _ in range(T // 40):
        eng.step(40)
        for key, (st, ps) in eng.drain_trajectories().items():
            g = got.setdefault(key, ([], []))
            g[0].extend(st)
            g[1].extend(ps)
    core = O.Core(m, s, p)
    pos = np.stack([core.reset_philox(N, seed, 0, e) for e in range(E)])
    cnt = np.full(E, N, np.int32)
    dff = np.zeros((E, H, W), np.float32)
    eps = np.zeros(E, np.int32)
    steps = np.zeros(E, np.int32)
    want = {}
    for t in range(1, T + 1):
        k0 = eps.copy()
        core.step_philox_batch(pos, cnt, dff, eps, seed, t, True, N, 0, 8)
        for e, q in zip(sel.tolist(), ph.tolist()):
            k = int(k0[e])
            steps[e] += 1
            ended = eps[e] != k0[e]
            if (k + q) % 2 == 0:
                c = 0 if ended else int(cnt[e])
                cells = pos[e, :c].astype(np.int32)
                w = want.setdefault((e, k), ([], []))
                w[0].append(int(steps[e]))
                w[1].append(np.stack([cells // W, cells % W], axis=1))
            if ended:
                steps[e] = 0
    assert sorted(got) == sorted(want)
    for key, (st, ps) in want.items():
        assert got[key][0] == st, f"{key}: steps"
        for a, b in zip(got[key][1], ps):
            assert np.array_equal(a, b), f"{key}: positions"
    ended = [v for v in want.values() if len(v[1][-1]) == 0]
    if N <= 20:     # short episodes: every selected env completes some within T steps
        assert len(ended) >= len(sel), "whole episodes, each ending with its empty row"
    gp, gc, _ = eng.get_state()
    assert np.array_equal(gc, cnt)
    eng.set_trajectory_capture([])
    eng.step(1)
    assert eng.drain_trajectories() == {}
    eng.close()


def test_engine_trajectory_capture_stops_when_empty_without_auto_reset():
    """auto_reset off: an emptied env logs its final empty row once, then nothing (the
    reference's run() stops there)."""
    from ffm_amd.data import make_room, l1_sff
    m = make_room(12, 12)
    eng = _engine(map_array=m, sff=l1_sff(m), n_envs=8, n_agents=3, rng="philox", seed=2, auto_reset=False)
    eng.set_trajectory_capture([0, 5], period=1)
    eng.reset()
    eng.step(200)
    tr = eng.drain_trajectories()
    _, gc, _ = eng.get_state()
    assert (gc[[0, 5]] == 0).all()
    for (env, k), (st, ps) in tr.items():
        assert k == 0 and st == list(range(1, len(st) + 1))
        assert len(ps[-1]) == 0 and all(len(q) > 0 for q in ps[:-1])
    eng.close()
