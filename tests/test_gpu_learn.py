"""GPU parity of the learning variants (ffm_ac_core, ffm_unified critic_only /
actor_only / both, ffm_actor_only) through the C ABI (ffm_learner_*).

* MT mode against the golden vectors recorded from the reference itself
  (tests/golden/learn_*.npz): positions, DFF bits, both RNG streams and the final
  V / H tables (keys, dict order, value bits) must all be equal.
* Philox (batched) mode against the CPU restatement of the same batched
  semantics (oracle/ffm_learn_oracle.c) at sizes it finishes in seconds:
  positions, counts, episode ends, DFF bits and the V / H tables bit for bit.
* Size-independent properties at BASELINE config-4 / config-5 scale.
"""
import glob
import json
import os

import numpy as np
import pytest

from golden_util import GOLDEN_DIR, dff_hash
from test_learn_oracle import pretrained

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

CASES = sorted(os.path.basename(p)[6:-4] for p in glob.glob(os.path.join(GOLDEN_DIR, "learn_*.npz")))
VARIANTS = [("ac", None), ("unified", "critic_only"), ("unified", "actor_only"), ("unified", "both"),
            ("actor_only", None)]


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.init()


def _learner(*a, **kw):
    from ffm_amd.engine import Learner
    return Learner(*a, **kw)


def _mt_words(m):
    return np.ctypeslib.as_array(m.mt).copy(), int(m.pos)


# ---------------------------------------------------------------------------
# MT mode: every golden episode of every seed
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("name", CASES)
def test_learner_replays_reference_goldens(name):
    from oracle import oracle as O
    z = np.load(os.path.join(GOLDEN_DIR, f"learn_{name}.npz"), allow_pickle=False)
    z = {k: z[k] for k in z.files}
    params = json.loads(str(z["params"]))
    variant, mode = str(z["variant"]), str(z["mode"]) or None
    H, W = z["map"].shape
    N, n_ep = int(z["N"]), int(z["n_ep"])
    core = O.Core(z["map"], z["sff"], {"neighborhood": "neumann"})
    ep_i = step_i = cell_i = 0
    v_off = h_off = 0
    for si, seed in enumerate(z["seeds"]):
        L = _learner(z["map"], z["sff"], variant, n_envs=1, n_agents=0, agent_capacity=max(N, 1), mode=mode,
                     params=params, rng="mt", auto_reset=False)
        inert_k, inert_v = pretrained(z, variant, lambda k, v, w="V": L.set_h_extra(v) if w == "Hx"
                                      else L.import_table(w, k, v))
        np_rng, py_rng = O.seeded_np(int(seed)), O.seeded_py(int(seed))
        for ep in range(n_ep):
            if ep > 0 and int(z["reload_v"]):
                L.set_v_default(-1.0)           # model/ffm_ac_core.py:343
            L.set_epsilon(float(z["eps"][ep_i]))
            pos = core.init_agents_mt(N, np_rng)
            ni = int(z["init_n"][ep_i])
            init = z["init"][sum(z["init_n"][:ep_i]):sum(z["init_n"][:ep_i]) + ni]
            assert np.array_equal(pos, init), f"seed {seed} ep {ep}: initial placement"
            cells = np.full((1, max(N, 1)), 0xFFFF, np.uint16)
            cells[0, :len(pos)] = pos
            L.set_state(0, positions=cells, counts=np.array([len(pos)], np.int32),
                        dff=np.zeros((1, H, W), np.float32))
            nk, npos = _mt_words(np_rng)
            pk, ppos = _mt_words(py_rng)
            L.set_mt_state(0, nk, npos, pk, ppos)
            for t in range(int(z["nsteps"][ep_i])):
                L.step(1)
                gp, gc, gd = L.get_state()
                c = int(z["counts"][step_i])
                assert int(gc[0]) == c, f"seed {seed} ep {ep} step {t}: count {gc[0]} != {c}"
                assert np.array_equal(gp[0, :c], z["cells"][cell_i:cell_i + c]), f"seed {seed} ep {ep} step {t}"
                assert dff_hash(gd[0]) == int(z["dff_hash"][step_i]), f"seed {seed} ep {ep} step {t}: DFF"
                cell_i += c
                step_i += 1
            nk, npos, pk, ppos = L.get_mt_state(0)
            np.ctypeslib.as_array(np_rng.mt)[:] = nk
            np_rng.pos = npos
            np.ctypeslib.as_array(py_rng.mt)[:] = pk
            py_rng.pos = ppos
            ep_i += 1
        vk, vv = L.export_table("V")
        vk, vv = np.concatenate([inert_k, vk]), np.concatenate([inert_v, vv])
        nv = int(z["v_n"][si])
        assert len(vk) == nv, f"seed {seed}: |V| {len(vk)} != {nv}"
        assert np.array_equal(vk, z["v_keys"][v_off:v_off + nv]), f"seed {seed}: V keys / order"
        assert np.array_equal(vv.view(np.uint64), z["v_vals"][v_off:v_off + nv].view(np.uint64)), \
            f"seed {seed}: V values"
        v_off += nv
        nh = int(z["h_n"][si])
        if nh:
            hk, hv = L.export_table("H")
            assert len(hk) == nh, f"seed {seed}: |H| {len(hk)} != {nh}"
            assert np.array_equal(hk, z["h_keys"][h_off:h_off + nh]), f"seed {seed}: H keys / order"
            assert np.array_equal(hv.view(np.uint64), z["h_vals"][h_off:h_off + nh].view(np.uint64)), \
                f"seed {seed}: H values"
            h_off += nh
        tails = [O.lib().ffo_mt_next(np_rng) for _ in range(4)]
        assert tails == [int(x) for x in z["np_tail"][si]], "NumPy stream position"
        tails = [O.lib().ffo_mt_next(py_rng) for _ in range(4)]
        assert tails == [int(x) for x in z["py_tail"][si]], "CPython stream position"
        L.close()


@pytest.mark.parametrize("variant,mode", VARIANTS)
@pytest.mark.parametrize("nbh", ["neumann", "moore"])
@pytest.mark.parametrize("room", ["obstacles", "interior"])
def test_learner_mt_rooms_match_oracle_stream(variant, mode, nbh, room):
    """MT (reference-stream) learning on rooms the goldens do not hold -- inner walls and two
    exits, an exit inside the room (contested exits) -- against the oracle's MT learning step
    (pinned to the reference by the golden replays): positions and DFF after every step,
    then the V / H tables in insertion (dict) order and both generators' positions."""
    from oracle import oracle as O
    from oracle import learn as LO
    from ffm_amd.data import make_room, l1_sff
    from test_gpu_parity import obstacle_room
    H = W = 12
    m = obstacle_room(H, W) if room == "obstacles" else make_room(H, W, (6, 5))
    s = l1_sff(m).astype(np.float64)
    p = {"epsilon": 0.1, "block_size": 1} if variant != "ac" else {}
    p["neighborhood"] = nbh
    N, T, seed = 20, 60, 41
    core = O.Core(m, s, {"neighborhood": "neumann"})
    L = _learner(m, s, variant, n_envs=1, n_agents=0, agent_capacity=N, mode=mode, params=p, rng="mt",
                 auto_reset=False)
    cpu = LO.Learn(m, s, variant, mode, p, log2_cap=20)
    np_rng, py_rng = O.seeded_np(seed), O.seeded_py(seed)
    pos = core.init_agents_mt(N, np_rng)
    cells = np.full((1, N), 0xFFFF, np.uint16)
    cells[0, :len(pos)] = pos
    L.set_state(0, positions=cells, counts=np.array([len(pos)], np.int32), dff=np.zeros((1, H, W), np.float32))
    nk, npos = _mt_words(np_rng)
    pk, ppos = _mt_words(py_rng)
    L.set_mt_state(0, nk, npos, pk, ppos)
    dff = np.zeros((H, W), np.float32)
    for t in range(T):
        pos = cpu.step_mt(pos, dff, np_rng, py_rng)
        L.step(1)
        gp, gc, gd = L.get_state()
        assert int(gc[0]) == len(pos), f"step {t}: count"
        assert np.array_equal(gp[0, :len(pos)], pos), f"step {t}: positions"
        assert np.array_equal(gd[0].view(np.uint32), dff.view(np.uint32)), f"step {t}: DFF"
        if len(pos) == 0:
            break
    for which, tab in (("V", cpu.V), ("H", cpu.Ht)):
        ck, cv = tab.export()
        if which == "H" and len(ck) == 0:     # no actor table (ac, critic_only)
            continue
        gk, gv = L.export_table(which)
        assert np.array_equal(np.asarray(ck, np.uint64), np.asarray(gk, np.uint64)), f"{which} keys / order"
        assert np.array_equal(np.asarray(cv).view(np.uint64), np.asarray(gv).view(np.uint64)), f"{which} values"
    nk, npos, pk, ppos = L.get_mt_state(0)
    assert np.array_equal(nk, np.ctypeslib.as_array(np_rng.mt)) and npos == int(np_rng.pos)
    assert np.array_equal(pk, np.ctypeslib.as_array(py_rng.mt)) and ppos == int(py_rng.pos)
    L.close()


# ---------------------------------------------------------------------------
# Philox (batched) mode: GPU == CPU restatement
# ---------------------------------------------------------------------------
def _random_rank_table(H, W, bs, seed=0, frac=0.6, width=5):
    """A trained-actor-like H over the rank keys of an H x W map (ffm_trained_core input;
    width 9 for the Moore neighbourhood)."""
    from ffm_amd import learn_keys as K
    rs = np.random.RandomState(seed)
    keys = [K.pack(((c >> 0) & 3, (c >> 2) & 3, (c >> 4) & 3, (c >> 6) & 3), bx, by)
            for bx in range((H - 1) // bs + 1) for by in range((W - 1) // bs + 1) for c in range(256)
            if rs.uniform() < frac]
    return np.array(keys, np.uint64), rs.standard_normal((len(keys), width)) * 3.0


def _philox_compare(variant, mode, params, H, W, N, E, T, A=None, max_steps=60, seed=42, env_base=0,
                    nthreads=16, sff_dtype=np.float32, log2_cap=22, chunks=1, reset_at=None, expect_tiled=None,
                    exit_pos=None, room=None):
    """reset_at = (T1, fraction): after T1 steps a random fraction of the envs is re-placed
    through Learner.reset_envs (the CPU side: reset_philox at step index T1 + 1), then the
    remaining T - T1 steps run.  expect_tiled: assert the learner's step path (tiled or not)."""
    from ffm_amd.data import make_room, l1_sff
    from oracle import learn as LO
    from oracle import oracle as O
    m = room(H, W) if room is not None else make_room(H, W, exit_pos)
    s = l1_sff(m).astype(sff_dtype)
    A = A or N
    L = _learner(m, s, variant, n_envs=E, n_agents=N, agent_capacity=A, mode=mode, params=params,
                 rng="philox", seed=seed, auto_reset=True, max_steps=max_steps, env_base=env_base)
    if expect_tiled is not None:
        assert L.tiled == expect_tiled
    cpu = LO.Learn(m, s, variant, mode, params, log2_cap=log2_cap)
    if variant == "trained":
        hk, hv = _random_rank_table(H, W, int(params.get("block_size", 5)), seed=seed,
                                    width=9 if params.get("neighborhood") == "moore" else 5)
        L.import_table("H", hk, hv)
        cpu.Ht.load(hk, hv)
    core = O.Core(m, s, {"neighborhood": "neumann"})
    pos = np.full((E, A), 0xFFFF, np.uint16)
    for e in range(E):
        pos[e, :N] = core.reset_philox(N, seed, 0, env_base + e)
    counts = np.full(E, N, np.int32)
    dff = np.zeros((E, H, W), np.float32)
    eps = np.zeros(E, np.int32)
    ep_steps = np.zeros(E, np.int32)
    L.reset()
    gp, gc, _ = L.get_state()
    assert np.array_equal(gc, counts)
    assert np.array_equal(gp[:, :N], pos[:, :N]), "reset placement"
    tot = 0
    T1 = T if reset_at is None else int(reset_at[0])
    for t in range(1, T1 + 1):
        tot += cpu.step_philox_batch(pos, counts, dff, eps, ep_steps, seed, t, True, N, max_steps, env_base,
                                     nthreads)
        if chunks > 1 and t % (T // chunks) == 0:
            print(f"  cpu step {t}/{T}", flush=True)   # progress of a long comparison
    L.step(T1)
    if reset_at is not None:
        import torch
        mask = np.random.default_rng(T1).random(E) < float(reset_at[1])
        L.reset_envs(torch.as_tensor(mask.astype(np.uint8)).cuda())
        for e in np.flatnonzero(mask):
            pos[e] = 0xFFFF
            pos[e, :N] = core.reset_philox(N, seed, T1 + 1, env_base + e)
            counts[e], ep_steps[e] = N, 0
            dff[e] = 0.0
        for t in range(T1 + 2, T + 2):
            tot += cpu.step_philox_batch(pos, counts, dff, eps, ep_steps, seed, t, True, N, max_steps, env_base,
                                         nthreads)
        L.step(T - T1)
    gp, gc, gd = L.get_state()
    geps, gst = L.episodes()
    assert np.array_equal(gc, counts), "counts"
    assert np.array_equal(geps, eps), "episodes"
    assert np.array_equal(gst, ep_steps), "steps into the episode"
    for e in range(E):
        assert np.array_equal(gp[e, :counts[e]], pos[e, :counts[e]]), f"env {e} positions"
    assert np.array_equal(gd.view(np.uint32), dff.view(np.uint32)), "DFF bits"
    for which, tab in (("V", cpu.V), ("H", cpu.Ht)):
        if which == "H" and variant not in ("actor_only", "trained") and mode in (None, "critic_only"):
            continue
        ck, cv = tab.export()
        gk, gv = L.export_table(which)
        assert len(gk) == len(ck), f"|{which}|"
        oc, og = np.argsort(ck), np.argsort(gk)
        assert np.array_equal(ck[oc], gk[og]), f"{which} keys"
        assert np.array_equal(np.asarray(cv)[oc].view(np.uint64), np.asarray(gv)[og].view(np.uint64)), \
            f"{which} values"
    c = L.counters()
    assert c["agent_steps"] == tot
    assert c["resets"] == int(eps.sum())
    assert c["steps"] == T
    L.close()
    return counts, eps


@pytest.mark.parametrize("variant,mode,params,H,N,E", [
    ("actor_only", None, {"epsilon": 0.2}, 12, 32, 4096),
    ("unified", "actor_only", {"block_size": 1}, 12, 32, 2048),
    ("unified", "actor_only", {"block_size": 1}, 64, 512, 16),
    ("unified", "both", {"block_size": 1, "neighborhood": "moore"}, 64, 512, 16),
])
def test_learner_reset_envs_matches_cpu(variant, mode, params, H, N, E):
    """reset(env_mask) of the batched learner (ffm_learner_reset_envs): a random half of the
    envs re-placed mid-run; positions, counts, DFF, episode counters and the V / H tables equal
    the CPU restatement re-placing the same envs (model/ffm_unified.py:800-812 per env)."""
    _philox_compare(variant, mode, params, H, H, N, E, 60, max_steps=40, reset_at=(23, 0.5))


def test_learner_philox_trained_matches_cpu():
    """ffm_trained_core batched: a read-only trained H, float32 policy, always-a-winner
    conflicts; 12x12 block 1 and an odd room with block 3."""
    _philox_compare("trained", None, {"block_size": 1}, 12, 12, 32, 2048, 120)
    _philox_compare("trained", None, {"block_size": 3, "k_A": 4}, 11, 17, 20, 333, 90, A=24, seed=9,
                    env_base=1 << 20)


@pytest.mark.parametrize("variant,mode", VARIANTS)
def test_learner_philox_12x12_matches_cpu(variant, mode):
    """12x12, 32 agents (configs 2/4 geometry), epsilon > 0 (exercises randint), 2,048 envs."""
    p = {"epsilon": 0.1, "block_size": 1} if variant != "ac" else {}
    _, eps = _philox_compare(variant, mode, p, 12, 12, 32, 2048, 120)
    assert eps.sum() > 0


@pytest.mark.parametrize("variant,mode", VARIANTS)
def test_learner_philox_odd_shapes_and_f64_sff(variant, mode):
    """Non-square room, block size 2, f64 SFF (main.py's data path), spare agent capacity,
    env ids offset (a later shard)."""
    p = {"epsilon": 0.05, "block_size": 2, "k_S": 4} if variant != "ac" else {"block_size": 2}
    _philox_compare(variant, mode, p, 11, 17, 20, 333, 90, A=24, max_steps=40, seed=9, env_base=1 << 20,
                    sff_dtype=np.float64)


@pytest.mark.parametrize("variant,mode", [("unified", "actor_only"), ("actor_only", None), ("ac", None)])
def test_learner_philox_large_rooms(variant, mode):
    """Workgroup-per-env kernel at 256 and 1,024 agent lanes (40x40 / 200 agents; 64x64 / 600)."""
    p = {"block_size": 5}
    _philox_compare(variant, mode, p, 40, 40, 200, 64, 40, max_steps=30, seed=3)
    _philox_compare(variant, mode, p, 64, 64, 600, 16, 25, max_steps=20, seed=4)


@pytest.mark.parametrize("variant,mode", VARIANTS + [("trained", None)])
def test_learner_philox_moore_matches_cpu(variant, mode):
    """The Moore neighbourhood in the batched learner (model/ffm_unified.py:173-185,
    model/ffm_actor_only.py:87-93): nine moves, nine-value H rows, requesters on a
    target's eight neighbours, eight decisions per ffm_actor_only agent, the
    eight-neighbour stencil.  12x12 / 32 agents at 2,048 envs; then the 256-lane,
    1,024-lane and four-agents-per-lane workgroup shapes (odd room, env ids offset)."""
    p = {"neighborhood": "moore", "epsilon": 0.1, "block_size": 1} if variant != "ac" else {"neighborhood": "moore"}
    _, eps = _philox_compare(variant, mode, p, 12, 12, 32, 2048, 120)
    assert eps.sum() > 0
    p = dict(p, block_size=5)
    _philox_compare(variant, mode, p, 40, 40, 200, 64, 40, max_steps=30, seed=3)
    _philox_compare(variant, mode, p, 64, 64, 600, 16, 25, max_steps=20, seed=4)
    _philox_compare(variant, mode, dict(p, k_D=2), 50, 77, 1300, 6, 16, A=2000, max_steps=10, seed=6,
                    env_base=77)


def test_learner_philox_large_placement_matches_cpu():
    """On-device placement of more agents than the sampled threshold holds (16,383 -- the
    batched learner's agent capacity -- of the 21,904 free cells of a 150x150 room: the exact
    histogram threshold of reset_env), then three tiled steps at sixteen agents per lane:
    positions, DFF and tables equal the CPU restatement.  (A 256x256 env of this many
    agents exceeds the batch kernel's LDS; its placement limit is the kernel's.)"""
    _philox_compare("unified", "actor_only", {"epsilon": 0.1, "block_size": 1}, 150, 150, 16383, 2, 3,
                    max_steps=20, seed=11, log2_cap=24)


@pytest.mark.parametrize("mode", ["critic_only", "actor_only", "both"])
def test_learner_philox_tiled_step_matches_cpu(mode):
    """The tiled step (ffm_unified at block size 1 on the raster batch kernel, DESIGN.md
    9.7): per-agent records summed per tile of cells in LDS instead of the fixed-point
    accumulators, H statistics kept per tile (incremental, rescans when an extreme moves
    inward).  Positions, DFF, V and H equal the CPU restatement bit for bit."""
    p = {"epsilon": 0.1, "block_size": 1}
    _philox_compare("unified", mode, p, 64, 64, 600, 16, 30, max_steps=20, seed=4)
    _philox_compare("unified", mode, dict(p, k_A=3.0, step_penalty=-1.0), 48, 40, 300, 24, 45, A=320,
                    max_steps=25, seed=6, env_base=77)


@pytest.mark.parametrize("mode", ["critic_only", "actor_only", "both"])
def test_learner_philox_tiled_moore_step_matches_cpu(mode):
    """The tiled step with the Moore neighbourhood (model/ffm_unified.py:173-185): records
    carry nine moves and up to eight requesters of a target, the tile passes sum and apply
    nine-value H rows (and rescan them for the statistics).  Positions, DFF, V and H equal
    the CPU restatement bit for bit; a square room, then an odd one with spare capacity."""
    p = {"epsilon": 0.1, "block_size": 1, "neighborhood": "moore"}
    _philox_compare("unified", mode, p, 64, 64, 600, 16, 30, max_steps=20, seed=4, expect_tiled=True)
    _philox_compare("unified", mode, dict(p, k_A=3.0, step_penalty=-1.0), 48, 40, 300, 24, 45, A=320,
                    max_steps=25, seed=6, env_base=77, expect_tiled=True)


@pytest.mark.parametrize("nbh,mode", [("neumann", "critic_only"), ("neumann", "actor_only"),
                                      ("moore", "critic_only"), ("moore", "both")])
def test_learner_philox_contested_exits_match_cpu(nbh, mode):
    """Exit-forced agents that lose their exit (model/ffm_unified.py:326-336: every agent next
    to an exit requests it; one requester enters, the others stay): the reference reads their
    V(s) at the next step although it never looked their V(s') up (a terminal transition), so
    the batch kernel inserts every V(s) for such maps instead of trusting the chain of last
    step's s' (LearnArgs::v_chain).  An exit inside the room (four or eight requesters) and
    the wall exit under Moore (three), on the tiled and the per-env shapes."""
    p = {"epsilon": 0.1, "block_size": 1, "neighborhood": nbh}
    _philox_compare("unified", mode, p, 40, 40, 300, 16, 40, max_steps=30, seed=5, exit_pos=(20, 20),
                    expect_tiled=True)
    _philox_compare("unified", mode, p, 24, 24, 60, 64, 40, max_steps=30, seed=6, exit_pos=(11, 13),
                    expect_tiled=False)
    if nbh == "moore":
        _philox_compare("unified", mode, p, 24, 24, 200, 32, 40, max_steps=30, seed=7)


@pytest.mark.parametrize("variant,mode", VARIANTS + [("trained", None)])
@pytest.mark.parametrize("nbh", ["neumann", "moore"])
def test_learner_philox_interior_exit_all_variants(variant, mode, nbh):
    """Every learning variant with an exit inside the room (contested exits, terminal
    transitions of the losers' neighbours), 12x12 at 1,024 envs and a 40x40 room on the
    256-lane shape; states and tables equal the CPU restatement bit for bit."""
    p = {"epsilon": 0.1, "block_size": 1} if variant != "ac" else {}
    p["neighborhood"] = nbh
    _philox_compare(variant, mode, p, 12, 12, 32, 1024, 80, max_steps=40, seed=23, exit_pos=(6, 5))
    _philox_compare(variant, mode, dict(p, block_size=5) if variant != "ac" else p, 40, 40, 200, 16, 40,
                    max_steps=30, seed=24, exit_pos=(20, 21))


@pytest.mark.parametrize("variant,mode", VARIANTS + [("trained", None)])
@pytest.mark.parametrize("nbh", ["neumann", "moore"])
def test_learner_philox_obstacles_and_two_exits_all_variants(variant, mode, nbh):
    """Every learning variant on a room with blocked cells inside (an inner wall with a gap,
    a pillar: the state keys' blocked classes away from the border) and two exits, 12x12 at
    1,024 envs and 40x40 on the 256-lane shape, then the tiled ffm_unified step on a 64x64
    room of the same layout."""
    from test_gpu_parity import obstacle_room
    p = {"epsilon": 0.1, "block_size": 1} if variant != "ac" else {}
    p["neighborhood"] = nbh
    _philox_compare(variant, mode, p, 12, 12, 30, 1024, 80, max_steps=40, seed=33, room=obstacle_room)
    _philox_compare(variant, mode, dict(p, block_size=5) if variant != "ac" else p, 40, 40, 200, 16, 40,
                    max_steps=30, seed=34, room=obstacle_room)
    if variant == "unified":
        _philox_compare(variant, mode, p, 64, 64, 600, 8, 30, max_steps=20, seed=35, room=obstacle_room,
                        expect_tiled=True)


@pytest.mark.parametrize("mode", ["actor_only", "both"])
def test_learner_philox_phase_split_step_matches_cpu(monkeypatch, mode):
    """The phase-split batch step (prep / decide / resolve / learn launches,
    taken by ffm_unified's actor modes above 1,024 agents per env with tiled records):
    positions, DFF, V and H equal the CPU restatement bit for bit -- a square room, then an
    odd width (state-map words across rows), spare agent capacity, env ids offset, episodes
    through max_steps.  Then the fused kernel's compile-time ffm_unified form (the default
    for these shapes) on the same cases."""
    p = {"epsilon": 0.1, "block_size": 1}
    monkeypatch.setenv("FFM_BATCH_PHASES", "1")
    _philox_compare("unified", mode, p, 64, 64, 1500, 12, 30, max_steps=20, seed=4)
    _philox_compare("unified", mode, dict(p, k_A=3.0, step_penalty=-1.0), 50, 77, 1300, 10, 26, A=2000,
                    max_steps=12, seed=6, env_base=77)
    monkeypatch.delenv("FFM_BATCH_PHASES")
    _philox_compare("unified", mode, p, 64, 64, 1500, 12, 30, max_steps=20, seed=4)
    _philox_compare("unified", mode, dict(p, k_A=3.0, step_penalty=-1.0), 50, 77, 1300, 10, 26, A=2000,
                    max_steps=12, seed=6, env_base=77)


@pytest.mark.parametrize("H,W", [(70, 256), (40, 512)])
def test_learner_philox_column_stencil_shapes(H, W):
    """The separate DFF stencil in row-segment strips (learn_stencil_col_kernel, W % 256 ==
    0): a last strip of 6 rows (70 = 2 x 32 + 6) and two 256-cell segments per row (the
    neighbours across a segment edge); the DFF equals the CPU restatement bit for bit."""
    p = {"epsilon": 0.1, "block_size": 1}
    _philox_compare("unified", "actor_only", p, H, W, 300, 6, 20, max_steps=15, seed=5)


@pytest.mark.parametrize("n,N,T,nbh", [(520, 600, 8, "neumann"), (300, 3000, 6, "neumann"), (520, 600, 8, "moore"),
                                       (300, 3000, 6, "moore")])
def test_learner_tiled_general_tile_pass_equals_accumulators(monkeypatch, n, N, T, nbh):
    """The tile passes' general form (records beyond one window: more than 512 envs, or a
    crowded tile with more than 1,024 records; the fast form holds one window in
    registers) against the accumulator path (FFM_TILED=0) on the same inputs: states,
    V and H bit for bit (Neumann's five-value and Moore's nine-value rows)."""
    from ffm_amd.data import make_room, l1_sff
    m = make_room(64, 64)
    s = l1_sff(m)
    kw = dict(mode="actor_only", params={"epsilon": 0.1, "block_size": 1, "neighborhood": nbh}, rng="philox",
              seed=12, auto_reset=True, max_steps=15)
    tiled = _learner(m, s, "unified", n_envs=n, n_agents=N, **kw)
    monkeypatch.setenv("FFM_TILED", "0")
    acc = _learner(m, s, "unified", n_envs=n, n_agents=N, **kw)
    assert tiled.tiled and not acc.tiled
    for L in (tiled, acc):
        L.reset()
        L.step(T)
    (p0, c0, d0), (p1, c1, d1) = tiled.get_state(), acc.get_state()
    assert np.array_equal(c0, c1) and np.array_equal(p0, p1)
    assert np.array_equal(d0.view(np.uint32), d1.view(np.uint32))
    for which in ("V", "H"):
        (k0, v0), (k1, v1) = tiled.export_table(which), acc.export_table(which)
        o0, o1 = np.argsort(k0), np.argsort(k1)
        assert np.array_equal(k0[o0], k1[o1]), which
        assert np.array_equal(np.asarray(v0)[o0].view(np.uint64), np.asarray(v1)[o1].view(np.uint64)), which
    for L in (tiled, acc):
        L.close()


def test_learner_tiled_buffers_are_collective_dtypes():
    """The tiled exchange's buffers are byte tensors: gloo and RCCL carry uint8, neither
    carries 16-bit integers (the uint16 tile offsets once went out as int16 and the
    all-gather raised "Invalid scalar type").  Sizes: 16 B per agent slot, 2 B per env
    and tile boundary."""
    import torch
    from ffm_amd.data import make_room, l1_sff
    m = make_room(64, 64)
    L = _learner(m, l1_sff(m), "unified", n_envs=4, n_agents=600, mode="actor_only",
                 params={"epsilon": 0.1, "block_size": 1}, rng="philox", seed=3, auto_reset=True, max_steps=20)
    assert L.tiled
    L.reset()
    L.step_tiled_local()
    recs, tst = L.tiled_buffers()
    assert recs.dtype == torch.uint8 and tst.dtype == torch.uint8
    assert recs.numel() == 4 * 600 * 16
    assert tst.numel() == 4 * (64 * 64 // 4 + 1) * 2
    L.step_tiled_apply(recs.data_ptr(), tst.data_ptr(), 4)     # ends the step (own records only)
    L.get_state()
    L.close()


@pytest.mark.parametrize("mode", ["actor_only", "both"])
def test_learner_tiled_shards_equal_one_learner(mode):
    """The tiled step across ranks (TableSync's exchange for tiled learners, coupled in one
    process): two shards all-gather each other's per-agent records and tile offsets and
    sum them per tile into their replicated tables; the tables (values, and the key sets
    including the slots only the other shard created) and the env states equal one
    learner stepping all envs, bit for bit."""
    from ffm_amd.data import make_room, l1_sff
    from ffm_amd.dist import step_coupled
    m = make_room(64, 64)
    s = l1_sff(m)
    p = {"epsilon": 0.1, "block_size": 1}
    n, N, T = 16, 600, 30
    kw = dict(mode=mode, params=p, rng="philox", seed=8, auto_reset=True, max_steps=20)
    one = _learner(m, s, "unified", n_envs=n, n_agents=N, **kw)
    assert one.tiled
    one.reset()
    one.step(T)
    shards = [_learner(m, s, "unified", n_envs=n // 2, n_agents=N, env_base=r * (n // 2), **kw) for r in range(2)]
    for L in shards:
        L.reset()
    step_coupled(shards, T, device="cuda", tiled=True)
    op, oc, od = one.get_state()
    sp = [L.get_state() for L in shards]
    assert np.array_equal(oc, np.concatenate([x[1] for x in sp]))
    assert np.array_equal(od.view(np.uint32), np.concatenate([x[2] for x in sp]).view(np.uint32))
    for which in ("V", "H"):
        k0, v0 = one.export_table(which)
        o0 = np.argsort(k0)
        for L in shards:
            k, v = L.export_table(which)
            o = np.argsort(k)
            assert np.array_equal(k[o], k0[o0]), which
            assert np.array_equal(np.asarray(v)[o].view(np.uint64), np.asarray(v0)[o0].view(np.uint64)), which
    for L in shards + [one]:
        L.close()


@pytest.mark.parametrize("mode,world,N,nbh", [("actor_only", 3, 600, "neumann"), ("both", 2, 600, "neumann"),
                                              ("critic_only", 3, 600, "neumann"), ("actor_only", 1, 600, "neumann"),
                                              ("both", 3, 1500, "neumann"), ("actor_only", 3, 600, "moore"),
                                              ("both", 2, 1500, "moore")])
def test_learner_owner_shards_equal_one_learner(mode, world, N, nbh):
    """The owner-sharded tiled step (TableSync's exchange for tiled learners,
    coupled in one process): the 1,024 tiles of a 64x64 room are dealt to the shards in
    chunks of 64, each shard sums only its own tiles' records from every shard (all-to-all),
    adopts the others' new slots, and takes the others' updated V values, H increments and
    tile summaries.  Shards of unequal size (envs 7 / 5 / 4) end with the tables (values and
    key sets) and env states of one learner stepping all envs, bit for bit (Neumann, and
    Moore's nine-value rows: H increments keyed with actions up to 8)."""
    from ffm_amd.data import make_room, l1_sff
    from ffm_amd.dist import step_coupled
    m = make_room(64, 64)
    s = l1_sff(m)
    p = {"epsilon": 0.1, "block_size": 1, "neighborhood": nbh}
    sizes = {1: [16], 2: [9, 7], 3: [7, 5, 4]}[world]
    n, T = sum(sizes), 30
    kw = dict(mode=mode, params=p, rng="philox", seed=8, auto_reset=True, max_steps=20)
    one = _learner(m, s, "unified", n_envs=n, n_agents=N, **kw)
    assert one.tiled and one.tile_major
    one.reset()
    one.step(T)
    bases = np.concatenate([[0], np.cumsum(sizes)])
    shards = [_learner(m, s, "unified", n_envs=c, n_agents=N, env_base=int(b), **kw) for b, c in zip(bases, sizes)]
    for L in shards:
        L.reset()
    step_coupled(shards, T, device="cuda", owner=True)
    op, oc, od = one.get_state()
    sp = [L.get_state() for L in shards]
    assert np.array_equal(oc, np.concatenate([x[1] for x in sp]))
    assert np.array_equal(od.view(np.uint32), np.concatenate([x[2] for x in sp]).view(np.uint32))
    for which in ("V", "H") if mode != "critic_only" else ("V",):
        k0, v0 = one.export_table(which)
        o0 = np.argsort(k0)
        assert len(k0) > 1000
        for L in shards:
            k, v = L.export_table(which)
            o = np.argsort(k)
            assert np.array_equal(k[o], k0[o0]), which
            assert np.array_equal(np.asarray(v)[o].view(np.uint64), np.asarray(v0)[o0].view(np.uint64)), which
    for L in shards + [one]:
        L.close()


def test_learner_tile_major_equals_env_major(monkeypatch):
    """The tile-major record layout (pack: column scan, tile offsets, scatter) and the
    env-major tile passes (FFM_TILE_MAJOR=0) give the same tables and states at a size whose
    tiles need the general (multi-window) form in both: 700 envs > the env-major window."""
    from ffm_amd.data import make_room, l1_sff
    m = make_room(64, 64)
    s = l1_sff(m)
    kw = dict(mode="actor_only", params={"epsilon": 0.1, "block_size": 1}, rng="philox", seed=3, auto_reset=True,
              max_steps=25)
    out = []
    for tm in ("1", "0"):
        monkeypatch.setenv("FFM_TILE_MAJOR", tm)   # 1: tile-major on one device too; 0: env-major only
        L = _learner(m, s, "unified", n_envs=700, n_agents=300, **kw)
        assert L.tile_major == (tm == "1")
        L.reset()
        L.step(12)
        st = L.get_state()
        tabs = {w: L.export_table(w) for w in ("V", "H")}
        L.close()
        out.append((st, tabs))
    (s0, t0), (s1, t1) = out
    assert np.array_equal(s0[1], s1[1]) and np.array_equal(s0[2].view(np.uint32), s1[2].view(np.uint32))
    for w in ("V", "H"):
        (k0, v0), (k1, v1) = t0[w], t1[w]
        o0, o1 = np.argsort(k0), np.argsort(k1)
        assert np.array_equal(k0[o0], k1[o1])
        assert np.array_equal(np.asarray(v0)[o0].view(np.uint64), np.asarray(v1)[o1].view(np.uint64))


def test_learner_philox_config5_geometry():
    """256x256 room, 8,192 agents (BASELINE config 5, ffm_unified actor_only): thresholded
    on-device placement (> 16,384 free cells) and the 8-agents-per-lane kernel."""
    _philox_compare("unified", "actor_only", {"block_size": 5}, 256, 256, 8192, 4, 6, max_steps=300, seed=5)


@pytest.mark.timeout(900)
def test_learner_philox_config5_through_truncation():
    """The bench's config-5 workload itself (run_unified_actor_training.py parameters,
    block 1, epsilon 0.2, max_steps 300) on 8 envs for 310 steps: every env is
    truncated at step 300 and auto-reset, the H statistics are populated for 300
    steps, and positions, DFF bits, V and H must equal the CPU restatement."""
    import bench
    cfg = bench.LEARN_CONFIGS[5]
    counts, eps = _philox_compare(cfg["variant"], cfg["mode"], cfg["params"], 256, 256, 8192, 8, 310,
                                  max_steps=cfg["max_steps"], seed=42, log2_cap=24, chunks=10)
    assert (eps == 1).all(), "every env truncates once at max_steps = 300"


@pytest.mark.timeout(900)
def test_learner_philox_config4_bench_workload_matches_cpu():
    """The bench's config-4 workload itself (bench.LEARN_CONFIGS[4]: run_actor_only_training.py's
    MODEL_PARAMS -- gamma 0.95, alpha_v 0.1, step_penalty 0, epsilon 0.2 -- max_steps 1000,
    12x12, 32 agents) on 4,096 envs for 300 steps: positions, counts, episode ends, DFF bits
    and the V / H tables equal the CPU restatement bit for bit."""
    import bench
    cfg = bench.LEARN_CONFIGS[4]
    counts, eps = _philox_compare(cfg["variant"], cfg["mode"], cfg["params"], 12, 12, 32, 4096, 300,
                                  max_steps=cfg["max_steps"], seed=42, log2_cap=22, chunks=10)
    assert eps.sum() > 3500, "most envs have emptied and restarted"


def test_learner_table_import_export_roundtrip():
    from ffm_amd.data import make_room, l1_sff
    from ffm_amd import learn_keys as K
    m = make_room(12, 12)
    L = _learner(m, l1_sff(m), "unified", n_envs=4, n_agents=8, mode="both", params={"block_size": 1})
    rs = np.random.RandomState(0)
    keys = np.array(sorted({K.pack(rs.randint(0, 4, 4), rs.randint(0, 12), rs.randint(0, 12))
                            for _ in range(500)}), np.uint64)
    rs.shuffle(keys)
    vv = rs.standard_normal(len(keys))
    hv = rs.standard_normal((len(keys), 5))
    L.import_table("V", keys, vv)
    L.import_table("H", keys[::-1], hv[::-1])
    k1, v1 = L.export_table("V")
    k2, v2 = L.export_table("H")
    assert np.array_equal(k1, keys) and np.array_equal(v1.view(np.uint64), vv.view(np.uint64))
    assert np.array_equal(k2, keys[::-1]) and np.array_equal(v2.view(np.uint64), hv[::-1].view(np.uint64))
    assert L.table_size("V") == len(keys)
    L.close()


@pytest.mark.parametrize("variant,mode", [("actor_only", None), ("unified", "actor_only")])
def test_learner_full_size_invariants(variant, mode):
    """BASELINE config-4 geometry (12x12, 32 agents, 65,536 envs per GPU): determinism over
    two runs, valid occupancy, finite tables, episodes truncated at max_steps."""
    from ffm_amd.data import make_room, l1_sff
    m = make_room(12, 12)
    s = l1_sff(m)
    p = {"epsilon": 0.2, "block_size": 1}
    outs = []
    for _ in range(2):
        L = _learner(m, s, variant, n_envs=65536, n_agents=32, mode=mode, params=p, seed=8, max_steps=100)
        L.reset()
        L.step(120)
        outs.append((*L.get_state(), *L.episodes(), *L.export_table("V"), *L.export_table("H")))
        c = L.counters()
        L.close()
    a, b = outs
    for x, y in zip(a[:5], b[:5]):
        assert np.array_equal(np.asarray(x), np.asarray(y))
    for i in (5, 7):       # tables: same entries (insertion order may differ), same bits
        oa, ob = np.argsort(a[i]), np.argsort(b[i])
        assert np.array_equal(a[i][oa], b[i][ob])
        assert np.array_equal(a[i + 1][oa].view(np.uint64), b[i + 1][ob].view(np.uint64))
        assert np.isfinite(a[i + 1]).all()
    pos, cnt, dff, eps, st = a[:5]
    assert (cnt >= 0).all() and (cnt <= 32).all() and (st < 100).all()
    assert eps.sum() >= 65536        # every env ended at least one episode in 120 steps
    flat = m.reshape(-1)
    for e in range(0, 65536, 101):
        cells = pos[e, :cnt[e]]
        assert len(set(cells.tolist())) == len(cells) and (flat[cells] == 0).all()
    assert (dff >= 0).all() and np.isfinite(dff).all()
    assert c["steps"] == 120 and c["agent_steps"] > 0


def test_learner_full_hashed_table_reports_instead_of_hanging():
    """A hashed table past 7/8 load refuses new keys; the host raises MemoryError."""
    from ffm_amd.data import make_room, l1_sff
    m = make_room(12, 12)
    L = _learner(m, l1_sff(m), "ac", n_envs=256, n_agents=32, log2_v_capacity=8)
    L.reset()
    L.step(10)
    with pytest.raises(MemoryError):
        L.counters()
    L.close()


def test_learner_unified_dense_table_rejects_foreign_keys():
    from ffm_amd.data import make_room, l1_sff
    from ffm_amd import learn_keys as K
    m = make_room(12, 12)
    L = _learner(m, l1_sff(m), "unified", n_envs=1, n_agents=4, mode="both", params={"block_size": 5})
    L.import_table("V", [K.pack((1, 2, 3, 0), 2, 2)], [1.5])      # blocks 0..2 exist at bs 5
    with pytest.raises(ValueError):
        L.import_table("V", [K.pack((1, 2, 3, 0), 3, 0)], [1.5])
    with pytest.raises(ValueError):
        L.import_table("H", [K.pack((1,) * 13, 0, 0)], np.zeros((1, 5)))
    L.close()


@pytest.mark.parametrize("variant,mode,sync,dense,nbh", [v + (1, False, "neumann") for v in VARIANTS] + [
    ("unified", "actor_only", 1, True, "neumann"), ("unified", "both", 4, True, "neumann"),
    ("unified", "critic_only", 4, True, "neumann"), ("actor_only", None, 4, False, "neumann"),
    ("unified", "actor_only", 1, False, "moore"), ("actor_only", None, 4, False, "moore"),
    ("unified", "both", 1, True, "moore")])
def test_learner_coupled_shards_equal_one_learner(variant, mode, sync, dense, nbh):
    """Multi-GPU contract on one device: three Learner shards (env_base offsets) stepped
    through ffm_amd.dist.step_coupled (delta export -> merge of the others' records ->
    apply; dense: summed fixed-point accumulators + presence union) end every sync step
    with the tables of ONE learner holding all envs at the same table sync period, bit
    for bit, and the same env states.  Moore: the H records carry nine increments."""
    from ffm_amd.data import make_room, l1_sff
    from ffm_amd.dist import shard_range, step_coupled
    m = make_room(12, 12)
    s = l1_sff(m)
    p = {"epsilon": 0.1, "block_size": 1} if variant != "ac" else {}
    p["neighborhood"] = nbh
    n, N, T = 3001, 32, 60
    kw = dict(mode=mode, params=p, rng="philox", seed=21, auto_reset=True, max_steps=40)
    one = _learner(m, s, variant, n_envs=n, n_agents=N, **kw)
    one.set_sync_period(sync)
    one.reset()
    one.step(T)
    shards = []
    for r in range(3):
        b, c = shard_range(n, r, 3)
        L = _learner(m, s, variant, n_envs=c, n_agents=N, env_base=b, **kw)
        L.reset()
        shards.append(L)
    step_coupled(shards, T, device="cuda", capacity=1024, sync_period=sync, dense=dense)
    op, oc, od = one.get_state()
    sp = [L.get_state() for L in shards]
    assert np.array_equal(oc, np.concatenate([x[1] for x in sp]))
    assert np.array_equal(od.view(np.uint32), np.concatenate([x[2] for x in sp]).view(np.uint32))
    pos = np.concatenate([x[0] for x in sp])
    for e in range(0, n, 7):
        assert np.array_equal(op[e, :oc[e]], pos[e, :oc[e]])
    assert np.array_equal(one.episodes()[0], np.concatenate([L.episodes()[0] for L in shards]))
    tabs = ["V"] + (["H"] if one.actor else [])
    for which in tabs:
        k0, v0 = one.export_table(which)
        o0 = np.argsort(k0)
        for L in shards:
            k, v = L.export_table(which)
            o = np.argsort(k)
            assert np.array_equal(k[o], k0[o0]), which
            assert np.array_equal(np.asarray(v)[o].view(np.uint64), np.asarray(v0)[o0].view(np.uint64)), which
    for L in shards + [one]:
        L.close()


@pytest.mark.parametrize("variant,mode,sync", [("actor_only", None, 1), ("actor_only", None, 4), ("ac", None, 1),
                                               ("unified", "actor_only", 3)])
def test_learner_async_records_equal_one_learner(variant, mode, sync):
    """TableSync's record path without host syncs, on the GPU kernels: two Learner shards
    exchange their deltas through delta_export_async (record count left in device
    memory, fixed-capacity buffers, 4 accumulator copies summed by the export) and
    delta_merge_async (count read on the device), sync period K; the tables end bit-equal
    to one Learner holding all envs, and the env states equal."""
    from ffm_amd.data import make_room, l1_sff
    from ffm_amd.dist import shard_range, step_coupled
    m = make_room(12, 12)
    s = l1_sff(m)
    p = {"epsilon": 0.1, "block_size": 1} if variant != "ac" else {}
    n, N, T = 1500, 32, 48     # a whole number of sync periods: every shard holds every key
    kw = dict(mode=mode, params=p, rng="philox", seed=33, auto_reset=True, max_steps=30)
    one = _learner(m, s, variant, n_envs=n, n_agents=N, **kw)
    one.set_sync_period(sync)
    one.reset()
    one.step(T)
    shards = []
    for r in range(2):
        b, c = shard_range(n, r, 2)
        L = _learner(m, s, variant, n_envs=c, n_agents=N, env_base=b, **kw)
        L.reset()
        shards.append(L)
    step_coupled(shards, T, device="cuda", capacity=1 << 17, sync_period=sync, async_records=True)
    assert one.counters()["agent_steps"] == sum(L.counters()["agent_steps"] for L in shards)
    op, oc, od = one.get_state()
    sp = [L.get_state() for L in shards]
    assert np.array_equal(oc, np.concatenate([x[1] for x in sp]))
    assert np.array_equal(od.view(np.uint32), np.concatenate([x[2] for x in sp]).view(np.uint32))
    for which in ["V"] + (["H"] if one.actor else []):
        k0, v0 = one.export_table(which)
        o0 = np.argsort(k0)
        for L in shards:
            k, v = L.export_table(which)
            o = np.argsort(k)
            assert np.array_equal(k[o], k0[o0]), which
            assert np.array_equal(np.asarray(v)[o].view(np.uint64), np.asarray(v0)[o0].view(np.uint64)), which
    for L in shards + [one]:
        L.close()


def test_learner_async_records_too_small_capacity_is_reported():
    """An asynchronous delta export with more touched entries than its buffer holds drops
    the surplus records on the device and is reported loudly (ValueError, FFM_E_INVALID)
    at the shard's next sync point, and by the next step once the flag copy has landed."""
    from ffm_amd.data import make_room, l1_sff
    from ffm_amd.dist import step_coupled
    m = make_room(12, 12)
    s = l1_sff(m)
    kw = dict(params={"epsilon": 0.1}, rng="philox", seed=3, auto_reset=True, max_steps=30)
    shards = [_learner(m, s, "actor_only", n_envs=256, n_agents=32, env_base=256 * r, **kw) for r in range(2)]
    for L in shards:
        L.reset()
    with pytest.raises(ValueError, match="record buffer too small"):
        # the next step_local raises once the flag copy queued by step_end has landed;
        # counters() (a sync point) raises in any case
        step_coupled(shards, 3, device="cuda", capacity=16, async_records=True)
        shards[0].counters()
    with pytest.raises(ValueError, match="record buffer too small"):
        shards[1].counters()
    with pytest.raises(ValueError, match="record buffer too small"):
        shards[1].step_local()
    for L in shards:
        L.close()


@pytest.mark.parametrize("variant,mode,dense", [("unified", "actor_only", True), ("actor_only", None, False)])
def test_rccl_table_sync_equals_one_learner(variant, mode, dense, tmp_path):
    """The RCCL branch of ffm_amd.dist.TableSync (backend "nccl" = RCCL on ROCm) on the
    one-GPU box, world 1: the dense accumulator all-reduce + presence all-gather / the
    fixed-capacity record all-gathers run through RCCL on device buffers, and the
    tables end bit-equal to one Learner stepping the same envs (sync period 4)."""
    import socket
    import torch.multiprocessing as mp
    import dist_worker as W
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    out = str(tmp_path / "rccl.npz")
    mp.spawn(W.rccl_learn_worker, args=(1, port, variant, mode, 512, 24, 4, dense, out), nprocs=1, join=True)
    r = dict(np.load(out))
    assert int(r["exchanges"]) > 0
    for k in [k for k in r if k.startswith("one_")]:
        assert np.array_equal(r[k], r["sync_" + k[4:]]), k


@pytest.mark.parametrize("variant,mode,stride", [("unified", "actor_only", 1), ("actor_only", None, 3),
                                                 ("unified", "critic_only", 1)])
def test_learner_curriculum_schedule_and_episode_log(variant, mode, stride):
    """The batched training drivers' knobs against the CPU restatement: radius-limited
    placement (model/ffm_unified.py:150-171: min(N, cells within the radius)), the
    per-env epsilon schedule (run_unified_actor_training.py:253-259; stride 3: env g at
    episode (g % 7) * 3 of a run-wide schedule, run_actor_only_training.py:190-196), and the
    episode log (one record per ended episode: env, index, steps, emptied)."""
    from ffm_amd.data import make_room, l1_sff
    from oracle import learn as LO
    from oracle import oracle as O
    m = make_room(12, 12)
    s = l1_sff(m)
    p = {"block_size": 1, "step_penalty": -1.0, "gamma": 0.99, "alpha_v": 0.01}
    E, N, T, seed, maxs = 600, 30, 160, 7, 40
    L = _learner(m, s, variant, n_envs=E, n_agents=N, mode=mode, params=p, seed=seed, max_steps=maxs)
    ncell = L.set_radius_placement((0, 6), 4, N)
    n = min(N, ncell)
    L.set_epsilon_schedule(0.2, 0.01, 1, 10)
    L.set_epsilon_phase(7, stride)              # env g starts the schedule at episode (g % 7) * stride
    L.reset()
    cpu = LO.Learn(m, s, variant, mode, p, log2_cap=22)
    cpu.set_epsilon_schedule(0.2, 0.01, 1, 10)
    cpu.set_epsilon_phase(7, stride)
    sh = LO.Shard(cpu, E, N, n, seed, 0, maxs, nthreads=16)
    free = np.argwhere(m == 0)
    r = np.abs(free[:, 0]) + np.abs(free[:, 1] - 6) <= 4
    cells = (free[r, 0] * 12 + free[r, 1]).astype(np.uint16)
    assert len(cells) == ncell
    sh.set_placement(cells, n)
    sh.pos[:] = 0xFFFF
    for e in range(E):
        sh.pos[e, :n] = O.reset_philox_list(cells, n, seed, 0, e)
    sh.counts[:] = n
    for _ in range(T):
        sh.step_local()
        sh.step_apply("V")
        if sh.actor:
            sh.step_apply("H")
        sh.step_end()
    L.step(T)
    gp, gc, gd = L.get_state()
    assert np.array_equal(gc, sh.counts)
    assert np.array_equal(gd.view(np.uint32), sh.dff.view(np.uint32))
    for e in range(E):
        assert np.array_equal(gp[e, :gc[e]], sh.pos[e, :gc[e]])
    eps_, _ = L.episodes()
    assert np.array_equal(eps_, sh.episodes)
    log = L.drain_episodes()
    want = np.array(sorted(sh.log), np.int32).reshape(-1, 4)
    assert np.array_equal(log, want)
    assert len(log) > E and set(np.unique(log[:, 3])) <= {0, 1}
    assert (log[log[:, 3] == 0, 2] == maxs).all()       # truncated episodes ran max_steps
    assert L.drain_episodes().shape == (0, 4)             # drained
    k0, v0 = L.export_table("V")
    k1, v1 = cpu.V.export()
    assert np.array_equal(np.sort(k0), np.sort(k1))
    assert np.array_equal(v0[np.argsort(k0)].view(np.uint64), v1[np.argsort(k1)].view(np.uint64))
    L.close()


@pytest.mark.parametrize("variant,mode,nbh", [("actor_only", None, "neumann"), ("unified", "actor_only", "neumann"),
                                              ("unified", "critic_only", "neumann"), ("unified", "critic_only", "moore"),
                                              ("actor_only", None, "moore")])
def test_learner_trajectory_capture_matches_cpu(variant, mode, nbh):
    """Batched trajectory capture (run(return_trajectory=True) rows, model/ffm_unified.py:902-931;
    the drivers keep every 100th episode's, run_actor_only_training.py:199-218) against the CPU
    restatement stepped in phases: the positions after every step of every captured episode,
    including the final rows of emptied and of truncated (max_steps) episodes."""
    from ffm_amd.data import make_room, l1_sff
    from oracle import learn as LO
    m = make_room(12, 12)
    s = l1_sff(m)
    p = {"epsilon": 0.1, "block_size": 1, "neighborhood": nbh}
    E, N, T, seed, maxs = 96, 12, 120, 11, 30
    sel = np.array([0, 5, 17, 42, 95], np.int32)
    ph = np.array([0, 1, 2, 1, 0], np.int32)
    period = 2
    L = _learner(m, s, variant, n_envs=E, n_agents=N, mode=mode, params=p, seed=seed, max_steps=maxs)
    L.set_trajectory_capture(sel, period=period, phases=ph, capacity_rows=len(sel) * 40)
    L.reset()
    got = {}
    for _ in range(T // 30):
        L.step(30)
        for key, (st, ps) in L.drain_trajectories().items():
            g = got.setdefault(key, ([], []))
            g[0].extend(st)
            g[1].extend(ps)
    cpu = LO.Learn(m, s, variant, mode, p, log2_cap=20)
    sh = LO.Shard(cpu, E, N, N, seed, 0, maxs, nthreads=8)
    want = {}
    for _ in range(T):
        sh.step_local()
        sh.step_apply("V")
        if sh.actor:
            sh.step_apply("H")
        for e, q in zip(sel.tolist(), ph.tolist()):
            k = int(sh.episodes[e])
            if (k + q) % period == 0:
                c = int(sh.counts[e])
                cells = sh.pos[e, :c].astype(np.int32)
                w = want.setdefault((e, k), ([], []))
                w[0].append(int(sh.ep_steps[e]) + 1)
                w[1].append(np.stack([cells // 12, cells % 12], axis=1))
        sh.step_end()
    assert sorted(got) == sorted(want)
    for key, (st, ps) in want.items():
        assert got[key][0] == st, f"{key}: steps"
        assert len(got[key][1]) == len(ps)
        for a, b in zip(got[key][1], ps):
            assert np.array_equal(a, b), f"{key}: positions"
    assert len(want) >= 2 * len(sel)
    if mode == "critic_only":      # SFF-led agents: emptied episodes end with an empty row
        assert any(len(v[1][-1]) == 0 for v in want.values())
    else:                          # near-random walkers: truncated at max_steps
        assert any(len(v[0]) == maxs for v in want.values())
    L.set_trajectory_capture([])
    L.step(1)
    assert L.drain_trajectories() == {}
    L.close()


def test_train_writes_reference_trajectory_files(tmp_path):
    """ffm_amd.train.run_curriculum keeps every n-th episode's trajectory in the file format of
    run_actor_only_training.py:206-218 (positions as an object array of per-step [n_t, 2]
    arrays, episode, N, total_episode, steps), consistent with steps_per_episode.csv."""
    import csv
    from ffm_amd.data import make_room, l1_sff
    from ffm_amd.train import run_curriculum
    m = make_room(12, 12)
    p = {"k_D": 1, "k_A": 10, "alpha_v": 0.1, "alpha_h": 0.1, "gamma": 0.95, "exit_reward": 100.0,
         "step_penalty": 0.0, "collision_penalty": -1.0, "neighborhood": "neumann"}
    L = _learner(m, l1_sff(m), "actor_only", n_envs=16, n_agents=8, params=p, seed=3, max_steps=60)
    res = run_curriculum(L, (0, 6), [3, 5], [1, 8], 40, 0.2, 0.01, str(tmp_path), verbose=False,
                         trajectory_every=10)
    L.close()
    with open(tmp_path / "steps_per_episode.csv") as f:
        rows = list(csv.DictReader(f))
    files = sorted((tmp_path / "trajectories").glob("trajectory_N*_ep*_total*.npz"))
    assert res["trajectories"] == len(files) == 4 * len(res["configs"])   # 48 episodes per config: 10..40
    by_total = {int(r["episode_num"]): r for r in rows}
    for fp in files:
        z = np.load(fp, allow_pickle=True)    # written by this test, an object array as the reference's
        steps, ep, total, N = int(z["steps"]), int(z["episode"]), int(z["total_episode"]), int(z["N"])
        assert ep % 10 == 0 and len(z["positions"]) == steps
        r = by_total[total]
        assert int(r["steps"]) == steps and int(r["N"]) == N
        assert all(q.shape[1] == 2 and len(q) <= N for q in z["positions"])
        assert len(z["positions"][-1]) == 0 or steps == 60


# model/ffm_unified.py critic_only on the 12x12 room with run_unified_critic_training.py's
# MODEL_PARAMS: mean steps per episode per (radius, N), 1000 reference episodes each
# (output/logs/unified_critic_training/run_20260117_101523/summary.txt:38-82 of the reference).
REF_CRITIC_MEAN_STEPS = {(5, 10): 19.71, (15, 1): 7.95, (15, 10): 21.46, (15, 20): 40.46, (15, 50): 99.56}


def test_batched_critic_curriculum_matches_reference_logged_means(tmp_path):
    """Distributional pin of the batched semantics against the reference's own run
    log: critic_only's policy does not read V, so the episode-length distribution per
    (radius, N) is fixed by the dynamics alone.  ffm_amd.train.run_curriculum runs
    the same curriculum batched; each mean must lie within 4 standard errors of the
    logged one (the reference's standard error estimated from our spread, n = 1000)."""
    import csv
    from ffm_amd.data import make_room, l1_sff
    from ffm_amd.engine import Learner
    from ffm_amd.train import run_curriculum
    m = make_room(12, 12)
    p = {"k_S": 10, "k_D": 1, "k_A": 10, "alpha_v": 0.01, "alpha_h": 0.1, "gamma": 0.99, "exit_reward": 100.0,
         "step_penalty": -1.0, "collision_penalty": -1.0, "neighborhood": "neumann", "block_size": 1}
    L = Learner(m, l1_sff(m), "unified", n_envs=2048, n_agents=50, mode="critic_only", params=p, seed=3,
                max_steps=300)
    res = run_curriculum(L, (0, 6), [5, 15], [1, 10, 20, 50], 4096, out_dir=str(tmp_path), verbose=False)
    got = {(c["radius"], c["N"]): c for c in res["configs"]}
    assert (5, 20) in got and (5, 50) not in got           # N above the cells in radius 5 is skipped
    for key, ref in REF_CRITIC_MEAN_STEPS.items():
        c = got[key]
        se = np.sqrt(c["std_steps"] ** 2 / c["episodes"] + c["std_steps"] ** 2 / 1000)
        assert abs(c["mean_steps"] - ref) <= max(4 * se, 0.05), (key, c["mean_steps"], ref, se)
        assert c["emptied"] == c["episodes"]                # no truncation at 300 steps
    with open(tmp_path / "steps_per_episode.csv") as f:
        rows = list(csv.reader(f))
    assert rows[0] == ["episode_num", "config_idx", "radius", "N", "steps", "v_table_size", "h_table_size",
                       "epsilon"]
    assert len(rows) == 1 + 4096 * len(res["configs"])      # 2 episodes of every one of the 2048 envs
    assert (tmp_path / "summary.txt").exists() and (tmp_path / "V_table.pkl").exists()
    L.close()


# The reference's unified actor_only run on its block_size-1 critic
# (output/logs/unified_actor_training/run_20260119_070834/steps_per_episode.csv of the
# reference, 100 episodes per configuration): mean steps and standard errors.
REF_ACTOR_MEAN_STEPS = {(9, 40): (80.30, 0.14), (11, 70): (139.87, 0.13), (15, 90): (179.75, 0.13)}


def test_batched_actor_curriculum_on_batched_critic_matches_reference_log(tmp_path):
    """Batched actor-learning dynamics against the reference's logged actor run.  A
    critic is trained by the batched critic_only curriculum (its V must stay in the
    range the rewards allow: a state visited k times in a step moves by
    (1 - (1 - alpha)^k) * mean(td), never by k * alpha * td), then the unified
    actor_only curriculum runs on it with 10 envs (the reference's per-configuration
    epsilon decay over 10 episodes per env), the whole curriculum as the logged run
    did (H carries over from one configuration to the next).  Agents must learn to leave: the mean
    episode length of the crowded configurations lies within 3 % of the logged one
    (the logged standard errors are 0.1 %; our 100-episode means carry the batched
    semantics and a different critic)."""
    from ffm_amd.data import make_room, l1_sff
    from ffm_amd.engine import Learner
    from ffm_amd.train import run_curriculum
    m = make_room(12, 12)
    p = {"k_S": 10, "k_D": 1, "k_A": 10, "alpha_v": 0.01, "alpha_h": 0.1, "gamma": 0.99, "exit_reward": 100.0,
         "step_penalty": -1.0, "collision_penalty": -1.0, "neighborhood": "neumann", "block_size": 1}
    C = Learner(m, l1_sff(m), "unified", n_envs=4096, n_agents=90, mode="critic_only", params=p, seed=5,
                max_steps=300)
    run_curriculum(C, (0, 6), [3, 5, 7, 9, 11, 13, 15], [1, 10, 20, 30, 40, 50, 60, 70, 80, 90], 1000,
                   verbose=False)
    vk, vv = C.export_table("V")
    C.close()
    assert np.isfinite(vv).all() and vv.min() > -150.0 and vv.max() < 150.0, (vv.min(), vv.max())
    A = Learner(m, l1_sff(m), "unified", n_envs=10, n_agents=90, mode="actor_only", params=p, seed=6,
                max_steps=300)
    A.import_table("V", vk, vv)
    res = run_curriculum(A, (0, 6), [3, 5, 7, 9, 11, 13, 15], [1, 10, 20, 30, 40, 50, 60, 70, 80, 90], 100,
                         0.2, 0.01, verbose=False)   # H learns along the whole curriculum, as in the log
    got = {(c["radius"], c["N"]): c for c in res["configs"]}
    for key, (ref, _se) in REF_ACTOR_MEAN_STEPS.items():
        c = got[key]
        assert abs(c["mean_steps"] - ref) <= 0.03 * ref, (key, c["mean_steps"], ref)
        assert c["emptied"] == c["episodes"]                # every episode ends with the room empty
    assert A.table_size("H") > 1000
    A.close()


MID_DENSITY = [(9, 30), (11, 30), (11, 40), (13, 30), (15, 30), (15, 40)]


def test_batched_actor_curriculum_mid_density_at_bench_envs():
    """Batched actor dynamics at the C5 bench's env count (E = 512, one episode per env per
    configuration, envs spread over the per-configuration epsilon schedule) against the
    reference's logged actor run (tests/golden/ref_unified_actor_run_20260119_070834.json,
    100 episodes per configuration).  Mid-density configurations, where the learned policy
    and not only exit throughput sets the episode length: at least 5 of 6 within 3
    combined standard errors, all within 1.5 %.  (the sparse, N = 10
    configurations deviate by 4-8 SE at E >= 512 -- every episode of a configuration
    then learns from the same H at once, E times the reference's updates per episode --
    and the crowded ones agree within 1 %.)"""
    from ffm_amd.data import make_room, l1_sff
    from ffm_amd.engine import Learner
    from ffm_amd.train import run_curriculum
    ref = {(c["radius"], c["N"]): c for c in
           json.load(open(os.path.join(GOLDEN_DIR, "ref_unified_actor_run_20260119_070834.json")))["configs"]}
    m = make_room(12, 12)
    p = {"k_S": 10, "k_D": 1, "k_A": 10, "alpha_v": 0.01, "alpha_h": 0.1, "gamma": 0.99, "exit_reward": 100.0,
         "step_penalty": -1.0, "collision_penalty": -1.0, "neighborhood": "neumann", "block_size": 1}
    radii, ns = [3, 5, 7, 9, 11, 13, 15], [1, 10, 20, 30, 40, 50, 60, 70, 80, 90]
    C = Learner(m, l1_sff(m), "unified", n_envs=4096, n_agents=90, mode="critic_only", params=p, seed=42,
                max_steps=300)
    run_curriculum(C, (0, 6), radii, ns, 1000, verbose=False)
    vk, vv = C.export_table("V")
    C.close()
    A = Learner(m, l1_sff(m), "unified", n_envs=512, n_agents=90, mode="actor_only", params=p, seed=42,
                max_steps=300)
    A.import_table("V", vk, vv)
    res = run_curriculum(A, (0, 6), radii, ns, 100, 0.2, 0.01, verbose=False)
    A.close()
    got = {(c["radius"], c["N"]): c for c in res["configs"]}
    rows, ok = [], 0
    for key in MID_DENSITY:
        r, c = ref[key], got[key]
        se = c["std_steps"] / np.sqrt(c["episodes"])
        dev = (c["mean_steps"] - r["mean_steps"]) / np.hypot(r["se"], se)
        rel = abs(c["mean_steps"] - r["mean_steps"]) / r["mean_steps"]
        rows.append((key, round(c["mean_steps"], 2), r["mean_steps"], round(float(dev), 2), round(rel, 4)))
        ok += abs(dev) <= 3.0
        assert rel <= 0.015, rows
    assert ok >= 5, rows


def _per_n_run(tmp, world=1, rank=0, envs=16, sync=None):
    """A small run of the config-4 driver (ffm_amd.train.run_per_n, run_actor_only_training.py's
    loop) on a 12x12 room: two N patterns, 40 episodes each, trajectories every 10th."""
    from ffm_amd import train as T
    from ffm_amd.data import make_room, l1_sff
    m = make_room(12, 12)
    s = l1_sff(m)
    d = T.driver_settings("actor_only")
    E = envs // world
    L = _learner(m, s, "actor_only", n_envs=E, n_agents=8, params=d["params"], seed=11, max_steps=30,
                 env_base=rank * E)
    g = T._Group(sync(L) if sync else None)
    res = T.run_per_n(L, [4, 8], 40, d["eps"], tmp, trajectory_every=10, group=g, verbose=False, params=d["params"],
                      global_envs=envs)
    L.close()
    return res


def test_per_n_driver_writes_reference_outputs(tmp_path):
    """run_actor_only_training.py's outputs from the batched driver: per-N H snapshots, the
    final V / H pickles, training_results.pkl with every episode numbered 1..total in
    order, the one linear epsilon over all episodes (:190-196), trajectories of every 10th
    pattern episode."""
    import pickle
    out = str(tmp_path / "run")
    res = _per_n_run(out)
    total = 80
    for f in ("H_actor_N4_total40ep.pkl", "H_actor_N8_total40ep.pkl", f"V_updated_total{total}ep.pkl",
              f"H_actor_total{total}ep.pkl", "training_results.pkl", "summary.txt"):
        assert os.path.exists(os.path.join(out, f)), f
    with open(os.path.join(out, "training_results.pkl"), "rb") as f:
        r = pickle.load(f)      # written by the test's own run
    eps = [e["episode_num"] for e in r["all_episodes"]]
    assert eps == list(range(1, total + 1))
    for e in r["all_episodes"]:
        want = float(np.clip(0.2 + (0.01 - 0.2) * ((e["episode_num"] - 1) / (total - 1)), 0.0, 1.0))
        assert e["epsilon"] == want
        assert 1 <= e["steps"] <= 30
    assert [p["N"] for p in r["results_by_n"]] == [4, 8]
    with open(os.path.join(out, f"H_actor_total{total}ep.pkl"), "rb") as f:
        H = pickle.load(f)
    assert len(H) == r["final_h_states"] > 0 and all(len(v) == 5 for v in H.values())
    traj = sorted(os.listdir(os.path.join(out, "trajectories")))
    assert len(traj) == 8 and traj[0].startswith("trajectory_N4_ep00010_total00010")
    assert res["model_params"]["gamma"] == 0.95


def _per_n_worker(rank, world, port, out, res_path):
    import pickle
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ffm_amd.dist import TableSync
        res = _per_n_run(out, world, rank, sync=lambda L: TableSync(L, device="cuda", capacity=None))
        if rank == 0:
            with open(res_path, "wb") as f:
                pickle.dump(res, f)
    finally:
        dist.destroy_process_group()


def test_per_n_driver_sharded_gloo_world2_equals_single(tmp_path):
    """The config-4 driver sharded over two ranks on one GPU (gloo; TableSync exchanges the
    hashed tables' records; global env ids): the per-episode results and the H / V pickles
    equal a single process stepping the same 16 global envs, bit for bit."""
    import pickle
    import socket
    import torch.multiprocessing as mp
    one = _per_n_run(str(tmp_path / "one"))
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    res_path = str(tmp_path / "two.pkl")
    mp.spawn(_per_n_worker, args=(2, port, str(tmp_path / "two"), res_path), nprocs=2, join=True)
    with open(res_path, "rb") as f:
        two = pickle.load(f)
    strip = lambda rows: [(e["episode_num"], e["N"], e["steps"], e["emptied"], e["epsilon"]) for e in rows]
    assert strip(one["all_episodes"]) == strip(two["all_episodes"])
    for name in ("H_actor_N4_total40ep.pkl", "H_actor_N8_total40ep.pkl", "V_updated_total80ep.pkl",
                 "H_actor_total80ep.pkl"):
        with open(tmp_path / "one" / name, "rb") as f:
            a = pickle.load(f)
        with open(tmp_path / "two" / name, "rb") as f:
            b = pickle.load(f)
        assert a.keys() == b.keys(), name
        for k in a:
            assert np.array_equal(np.asarray(a[k], np.float64).view(np.uint64),
                                  np.asarray(b[k], np.float64).view(np.uint64)), name


def _owner_sync_worker(rank, world, port, sizes, mode, T, out_path):
    import pickle
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ffm_amd.data import make_room, l1_sff
        from ffm_amd.dist import TableSync
        m = make_room(64, 64)
        s = l1_sff(m)
        base = int(sum(sizes[:rank]))
        L = _learner(m, s, "unified", n_envs=sizes[rank], n_agents=600, mode=mode,
                     params={"epsilon": 0.1, "block_size": 1}, rng="philox", seed=8, auto_reset=True, max_steps=20,
                     env_base=base)
        L.reset()
        sync = TableSync(L, device="cuda")
        assert sync.tiled and sync.owner
        sync.step(T)
        sync.flush()                 # V's key set: the presence union (collective)
        torch.cuda.synchronize()
        st = L.get_state()
        tabs = {w: L.export_table(w) for w in (("V", "H") if L.actor else ("V",))}
        parts = [None] * world
        dist.all_gather_object(parts, (st[1], st[2], tabs, sync.received_bytes, sync.exchanges))
        if rank == 0:
            with open(out_path, "wb") as f:
                pickle.dump(parts, f)
        L.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["actor_only", "critic_only"])
def test_gloo_world2_owner_table_sync_equals_one_learner(mode, tmp_path):
    """TableSync's owner-sharded exchange over a real process group (two ranks on one GPU,
    gloo; all-to-all of the packed records, all-gathers of new slots, V values, H increments
    and tile summaries; shards of 9 and 7 envs): both ranks end with the tables of one
    learner stepping all 16 envs, and the env states agree, bit for bit."""
    import pickle
    import socket
    import torch.multiprocessing as mp
    from ffm_amd.data import make_room, l1_sff
    sizes, T = [9, 7], 25
    m = make_room(64, 64)
    s = l1_sff(m)
    one = _learner(m, s, "unified", n_envs=16, n_agents=600, mode=mode, params={"epsilon": 0.1, "block_size": 1},
                   rng="philox", seed=8, auto_reset=True, max_steps=20)
    one.reset()
    one.step(T)
    _, oc, od = one.get_state()
    otabs = {w: one.export_table(w) for w in (("V", "H") if one.actor else ("V",))}
    one.close()
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    out = str(tmp_path / "owner.pkl")
    mp.spawn(_owner_sync_worker, args=(2, port, sizes, mode, T, out), nprocs=2, join=True)
    with open(out, "rb") as f:
        parts = pickle.load(f)
    assert np.array_equal(oc, np.concatenate([p[0] for p in parts]))
    assert np.array_equal(od.view(np.uint32), np.concatenate([p[1] for p in parts]).view(np.uint32))
    for p in parts:
        assert p[3] > 0 and p[4] == T
        for w, (k0, v0) in otabs.items():
            k, v = p[2][w]
            o0, o = np.argsort(k0), np.argsort(k)
            assert np.array_equal(k[o], k0[o0]), w
            assert np.array_equal(np.asarray(v)[o].view(np.uint64), np.asarray(v0)[o0].view(np.uint64)), w


def test_learner_episode_caps_stop_envs_after_their_quota():
    """ffm_learner_set_episode_caps: env e ends exactly caps[e] episodes after the reset and
    then stays empty (a zero quota: empty from the reset).  critic_only's policy does not read
    the tables, so every env's first caps[e] episodes are those of an uncapped run, step for
    step (placement and decision streams are keyed by step, env and agent)."""
    from ffm_amd.data import make_room, l1_sff
    m = make_room(12, 12)
    s = l1_sff(m)
    E, N, maxs = 64, 20, 40
    caps = (np.arange(E) % 4).astype(np.int32)
    logs = []
    for capped in (False, True):
        L = _learner(m, s, "unified", n_envs=E, n_agents=N, mode="critic_only", params={"block_size": 1}, seed=5,
                     max_steps=maxs)
        if capped:
            L.set_episode_caps(caps)
        L.reset()
        done = []
        for _ in range(20):
            L.step(16)
            done.append(L.drain_episodes())
        log = np.concatenate(done)
        eps, _ = L.episodes()
        _, cnt, _ = L.get_state()
        if capped:
            assert np.array_equal(eps, caps)
            assert (cnt == 0).all()
            assert np.array_equal(np.bincount(log[:, 0], minlength=E), caps)
            L.set_episode_caps(None)
            L.reset()
            _, cnt, _ = L.get_state()
            assert (cnt == N).all()                        # quotas removed: every env placed again
        L.close()
        logs.append(log)
    full, capped_log = logs
    keep = full[full[:, 1] < caps[full[:, 0]]]
    assert np.array_equal(keep[np.lexsort((keep[:, 1], keep[:, 0]))],
                          capped_log[np.lexsort((capped_log[:, 1], capped_log[:, 0]))])


def _c5_curriculum_run(tmp, world=1, rank=0, sync=None, envs=4):
    """The C5 workload through ffm_amd.train.run_curriculum's full-room mode: 256x256 room,
    8,192 agents, ffm_unified actor_only with run_unified_actor_training.py's MODEL_PARAMS,
    max_steps 300, epsilon 0.2 -> 0.01, one episode per env, a trajectory every 2nd."""
    from ffm_amd import train as T
    from ffm_amd.data import make_room, l1_sff
    m = make_room(256, 256)
    d = T.driver_settings("unified")
    E = envs // world
    L = _learner(m, l1_sff(m), "unified", n_envs=E, n_agents=8192, mode="actor_only", params=d["params"], seed=13,
                 max_steps=d["max_steps"], env_base=rank * E)
    g = T._Group(sync(L) if sync else None)
    res = T.run_curriculum(L, (0, 128), [None], [8192], envs, *d["eps"], tmp, verbose=False, trajectory_every=2,
                           group=g, global_envs=envs)
    L.close()
    return res


def _c5_curriculum_worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ffm_amd.dist import TableSync

        def sync(L):
            ts = TableSync(L, device="cuda", capacity=None)
            assert ts.owner                     # C5 shards through the owner-sharded tile exchange
            return ts

        _c5_curriculum_run(out, world, rank, sync=sync)
    finally:
        dist.destroy_process_group()


def _growing_curriculum_run(tmp, world=1, rank=0, sync=None, envs=128):
    """A radius / N curriculum whose crowd grows: radius 4 with N = 10 (a crowd on one
    owner's rows), then radius 25 with N = 10 and N = 300, on the tiled 64x64 learner (agent
    capacity above 256: the raster batch kernel, so the owner exchange)."""
    from ffm_amd import train as T
    from ffm_amd.data import make_room, l1_sff
    m = make_room(64, 64)
    d = T.driver_settings("unified")
    E = envs // world
    L = _learner(m, l1_sff(m), "unified", n_envs=E, n_agents=300, mode="actor_only", params=d["params"], seed=21,
                 max_steps=60, env_base=rank * E)
    g = T._Group(sync(L) if sync else None)
    res = T.run_curriculum(L, (0, 32), [4, 25], [10, 300], envs, *d["eps"], tmp, verbose=False, group=g,
                           global_envs=envs)
    L.close()
    return res


def _growing_curriculum_worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ffm_amd.dist import TableSync

        def sync(L):
            ts = TableSync(L, device="cuda", capacity=None)
            assert ts.owner
            return ts

        _growing_curriculum_run(out, world, rank, sync=sync)
    finally:
        dist.destroy_process_group()


def test_growing_curriculum_sharded_gloo_world2_equals_single(tmp_path):
    """the owner exchange's capacities adapt to the counts observed, so a
    curriculum whose next configuration crowds more records onto one owner (radius 4, N = 10
    -> radius 25, N = 300) overflowed them.  TableSync.reconfigure restarts them from the new
    configuration's shape bounds: the two-rank run completes and writes the files of one
    process stepping the same 128 global envs."""
    import csv
    import socket
    import torch.multiprocessing as mp
    one = tmp_path / "one"
    res = _growing_curriculum_run(str(one))
    assert [(c["radius"], c["N"]) for c in res["configs"]] == [(4, 10), (25, 10), (25, 300)]
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    two = tmp_path / "two"
    mp.spawn(_growing_curriculum_worker, args=(2, port, str(two)), nprocs=2, join=True)
    with open(one / "steps_per_episode.csv") as f:
        a = list(csv.reader(f))
    with open(two / "steps_per_episode.csv") as f:
        b = list(csv.reader(f))
    assert a == b and len(a) == 1 + 3 * 128


def test_c5_curriculum_sharded_gloo_world2_equals_single(tmp_path):
    """Row R3: the C5 learning loop (full-room ffm_unified actor_only, 256x256, 8,192 agents)
    sharded over two ranks on one GPU (gloo; TableSync's owner-sharded tile exchange; global
    env ids) writes the files of one process stepping the same 4 global envs:
    steps_per_episode.csv and the trajectories identical, the V / H pickles equal as dicts
    (keys and value bits; dict order is insertion order, which the ranks' exchange changes)."""
    import csv
    import pickle
    import socket
    import torch.multiprocessing as mp
    one = tmp_path / "one"
    res = _c5_curriculum_run(str(one))
    assert res["configs"][0]["episodes"] == 4 and res["trajectories"] == 2
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    two = tmp_path / "two"
    mp.spawn(_c5_curriculum_worker, args=(2, port, str(two)), nprocs=2, join=True)
    with open(one / "steps_per_episode.csv") as f:
        a = list(csv.reader(f))
    with open(two / "steps_per_episode.csv") as f:
        b = list(csv.reader(f))
    assert a == b and len(a) == 5 and all(r[2] == "full" and r[3] == "8192" for r in a[1:])
    for name in ("V_table.pkl", "H_table.pkl"):
        with open(one / name, "rb") as f:
            x = pickle.load(f)      # written by this test's runs
        with open(two / name, "rb") as f:
            y = pickle.load(f)
        assert x.keys() == y.keys() and len(x) > 10000, name
        for k in x:
            assert np.array_equal(np.asarray(x[k], np.float64).view(np.uint64),
                                  np.asarray(y[k], np.float64).view(np.uint64)), name
    ta = sorted(p.name for p in (one / "trajectories").iterdir())
    tb = sorted(p.name for p in (two / "trajectories").iterdir())
    assert ta == tb and len(ta) == 2
    for n in ta:
        za, zb = np.load(one / "trajectories" / n, allow_pickle=True), np.load(two / "trajectories" / n,
                                                                              allow_pickle=True)
        assert int(za["steps"]) == int(zb["steps"]) and len(za["positions"]) == len(zb["positions"])
        assert all(np.array_equal(p, q) for p, q in zip(za["positions"], zb["positions"]))
    sa = (one / "summary.txt").read_text().splitlines()
    sb = (two / "summary.txt").read_text().splitlines()
    assert [l for l in sa if not l.startswith("seconds")] == [l for l in sb if not l.startswith("seconds")]


@pytest.mark.timeout(900)
def test_learner_owner_8_shards_c5_full_size_equal_one_learner():
    """The owner-sharded exchange at the C5 N = 8 shape itself: 8 coupled shards of 512 envs
    (256x256 room, 8,192 agents, bench.LEARN_CONFIGS[5], global env ids r * 512 + e) against
    one learner stepping all 4,096 envs, for 305 steps: through the lockstep truncation and
    reset at step 300, with tiles holding thousands of records from eight sources (the
    multi-window general forms).  Positions, counts, DFF bits and the V / H tables (keys and
    value bits) of every shard equal the single learner's."""
    import bench
    from ffm_amd.data import make_room, l1_sff
    from ffm_amd.dist import step_coupled
    cfg = bench.LEARN_CONFIGS[5]
    m = make_room(256, 256)
    s = l1_sff(m)
    W, E, T = 8, 512, 305
    kw = dict(mode=cfg["mode"], params=cfg["params"], rng="philox", seed=42, auto_reset=True,
              max_steps=cfg["max_steps"], log2_v_capacity=24, log2_h_capacity=24)
    one = _learner(m, s, cfg["variant"], n_envs=W * E, n_agents=8192, **kw)
    one.reset()
    one.step(T)
    op, oc, od = one.get_state()
    eps1, _ = one.episodes()
    assert (eps1 == 1).all()                     # every env truncated at 300 and re-placed
    tabs1 = {w: one.export_table(w) for w in ("V", "H")}
    one.close()
    shards = [_learner(m, s, cfg["variant"], n_envs=E, n_agents=8192, env_base=r * E, **kw) for r in range(W)]
    for L in shards:
        L.reset()
    step_coupled(shards, T, device="cuda", owner=True)
    for r, L in enumerate(shards):
        p, c, d = L.get_state()
        sl = slice(r * E, (r + 1) * E)
        assert np.array_equal(c, oc[sl]), r
        assert np.array_equal(d.view(np.uint32), od[sl].view(np.uint32)), r
        for e in range(E):
            assert np.array_equal(p[e, :c[e]], op[r * E + e, :c[e]]), (r, e)
        del p, d
    for w in ("V", "H"):
        k0, v0 = tabs1[w]
        o0 = np.argsort(k0)
        assert len(k0) > 100000, w
        for L in shards:
            k, v = L.export_table(w)
            o = np.argsort(k)
            assert np.array_equal(k[o], k0[o0]), w
            assert np.array_equal(np.asarray(v)[o].view(np.uint64), np.asarray(v0)[o0].view(np.uint64)), w
    for L in shards:
        L.close()
