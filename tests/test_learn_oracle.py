"""The learning-variant restatement (oracle/ffm_learn_oracle.c) against golden
vectors recorded from the reference itself (tests/golden/gen_golden_learn.py):
ffm_ac_core, ffm_unified (critic_only / actor_only / both) and ffm_actor_only,
several episodes per seed with the tables carried over, epsilon schedules and
the set_v_table default quirk.  Positions, DFF bits, both RNG streams and the
final V / H tables (keys, values and dict order) must all be equal."""
from __future__ import annotations

import glob
import json
import os

import numpy as np
import pytest

from golden_util import GOLDEN_DIR, dff_hash
from oracle import learn as LO
from oracle import oracle as O

CASES = sorted(os.path.basename(p)[6:-4] for p in glob.glob(os.path.join(GOLDEN_DIR, "learn_*.npz")))


def load(name):
    z = np.load(os.path.join(GOLDEN_DIR, f"learn_{name}.npz"), allow_pickle=False)
    return {k: z[k] for k in z.files}


def pretrained(z, variant, load):
    """A fixture's pretrained critic (model/ffm_unified.py:84-110, model/ffm_actor_only.py:55-70).
    ffm_unified loads it into V; ffm_actor_only keys it by tuples that its bytes keys
    never match, so it stays inert and only leads get_v_table()'s order.
    Returns that inert prefix (keys, values)."""
    none = (np.zeros(0, np.uint64), np.zeros(0, np.float64))
    if "pre_h_keys" in z:                # ffm_trained_core: the trained H (model/ffm_trained_core.py:51-68)
        load(z["pre_h_keys"], z["pre_h_vals"], "H")
        if "pre_h_odd_vals" in z:        # rows of another length: only their values' min / max (:228-267)
            load(None, z["pre_h_odd_vals"], "Hx")
        return none
    if "pre_keys" not in z:
        return none
    if variant == "unified":
        load(z["pre_keys"], z["pre_vals"])
        return none
    return z["pre_keys"], z["pre_vals"]


def replay(z, make_step):
    """Drive one fixture through `make_step(learn, seed)`; returns per-seed learn objects."""
    params = json.loads(str(z["params"]))
    variant, mode = str(z["variant"]), str(z["mode"]) or None
    H, W = z["map"].shape
    N, n_ep = int(z["N"]), int(z["n_ep"])
    core = O.Core(z["map"], z["sff"], {"neighborhood": "neumann"})
    ep_i = step_i = cell_i = 0
    v_off = h_off = 0
    for si, seed in enumerate(z["seeds"]):
        L = LO.Learn(z["map"], z["sff"], variant, mode, params)
        inert_k, inert_v = pretrained(z, variant, lambda k, v, w="V": L.Ht.set_extra(v) if w == "Hx"
                                      else (L.V if w == "V" else L.Ht).load(k, v))
        np_rng, py_rng = O.seeded_np(int(seed)), O.seeded_py(int(seed))
        for ep in range(n_ep):
            if ep > 0 and int(z["reload_v"]):
                L.set_v_default(-1.0)           # model/ffm_ac_core.py:343
            L.set_epsilon(float(z["eps"][ep_i]))
            pos = core.init_agents_mt(N, np_rng)
            ni = int(z["init_n"][ep_i])
            init = z["init"][sum(z["init_n"][:ep_i]):sum(z["init_n"][:ep_i]) + ni]
            assert np.array_equal(pos, init), f"seed {seed} ep {ep}: initial placement"
            dff = np.zeros((H, W), np.float32)
            for t in range(int(z["nsteps"][ep_i])):
                pos = make_step(L, pos, dff, np_rng, py_rng)
                c = int(z["counts"][step_i])
                assert len(pos) == c, f"seed {seed} ep {ep} step {t}: count {len(pos)} != {c}"
                assert np.array_equal(pos, z["cells"][cell_i:cell_i + c]), f"seed {seed} ep {ep} step {t}: cells"
                assert dff_hash(dff) == int(z["dff_hash"][step_i]), f"seed {seed} ep {ep} step {t}: DFF"
                cell_i += c
                step_i += 1
            ep_i += 1
        vk, vv = L.V.export()
        vk, vv = np.concatenate([inert_k, vk]), np.concatenate([inert_v, vv])
        nv = int(z["v_n"][si])
        assert len(vk) == nv, f"seed {seed}: |V| {len(vk)} != {nv}"
        assert np.array_equal(vk, z["v_keys"][v_off:v_off + nv]), f"seed {seed}: V keys / order"
        assert np.array_equal(vv.view(np.uint64), z["v_vals"][v_off:v_off + nv].view(np.uint64)), \
            f"seed {seed}: V values"
        v_off += nv
        nh = int(z["h_n"][si])
        if nh:
            hk, hv = L.Ht.export()
            assert len(hk) == nh, f"seed {seed}: |H| {len(hk)} != {nh}"
            assert np.array_equal(hk, z["h_keys"][h_off:h_off + nh]), f"seed {seed}: H keys / order"
            assert np.array_equal(hv.view(np.uint64), z["h_vals"][h_off:h_off + nh].view(np.uint64)), \
                f"seed {seed}: H values"
            h_off += nh
        tails = [O.lib().ffo_mt_next(np_rng) for _ in range(4)]
        assert tails == [int(x) for x in z["np_tail"][si]], "NumPy stream position"
        tails = [O.lib().ffo_mt_next(py_rng) for _ in range(4)]
        assert tails == [int(x) for x in z["py_tail"][si]], "CPython stream position"


@pytest.mark.parametrize("name", CASES)
def test_learn_oracle_matches_reference_goldens(name):
    z = load(name)
    replay(z, lambda L, pos, dff, a, b: L.step_mt(pos, dff, a, b))


def test_encoders_match_reference_examples():
    """Hand-built state maps against the reference's encoding rules
    (model/ffm_unified.py:205-256, model/ffm_ac_core.py:75-105, model/ffm_actor_only.py:115-141)."""
    from ffm_amd import learn_keys as K
    sm = np.full((7, 7), 0, np.uint8)
    sm[0, :] = sm[-1, :] = sm[:, 0] = sm[:, -1] = 2
    sm[0, 3] = 3
    sm[1, 3] = 1          # the agent
    sm[1, 2] = 1          # neighbour to the left
    sm[2, 4] = 1          # diagonal-forward of D
    # agent at (1,3): U -> exit cell (3), diagonals (0,2),(0,4) walls, two ahead OOB -> rank 2
    #                 D -> (2,3) free, diagonals (2,2) free, (2,4) person -> rank 1
    #                 L -> (1,2) person -> rank 0
    #                 R -> (1,4) free, diag (0,4) wall, (2,4) person -> rank 1
    k = LO.encode_rank(sm, 1, 3, 1)
    assert K.to_rank_tuple(k) == ((2, 1, 0, 1), (1, 3))
    k = LO.encode_rank(sm, 1, 3, 2)
    assert K.to_rank_tuple(k) == ((2, 1, 0, 1), (0, 1))
    k13 = LO.encode_cells13(sm, 1, 3, 3, 2)
    cells, blk = K.unpack(k13, 13)
    assert cells == (2, 3, 2, 1, 1, 0, 0, 0, 1, 2, 0, 0, 0) and blk == (0, 1)
    k13 = LO.encode_cells13(sm, 1, 3, 5, 0)
    cells, blk = K.unpack(k13, 13)
    assert cells == (2, 3, 2, 1, 1, 0, 0, 0, 1, 0, 0, 0, 0) and blk == (0, 0)


def test_det_exp_is_close_to_libm():
    xs = np.concatenate([-np.logspace(-12, np.log10(740), 4000), np.linspace(-5, 0, 1001)])
    got = np.array([LO.det_exp(x) for x in xs])
    ref = np.exp(xs)
    rel = np.abs(got - ref) / np.maximum(ref, 1e-300)
    assert rel.max() < 4e-16
    assert LO.det_exp(0.0) == 1.0 and LO.det_exp(-np.inf) == 0.0


def test_learn_keys_roundtrip():
    from ffm_amd import learn_keys as K
    import pickle
    k = ((3, 0, 2, 1), (11, 7))
    assert K.to_rank_tuple(K.from_rank_tuple(k)) == k
    cells = tuple(np.int64(v) for v in (2, 2, 2, 0, 1, 0, 0, 3, 0, 2, 0, 1, 0))
    b = pickle.dumps((cells, (np.int64(0), np.int64(2))))
    assert K.to_cells_bytes(K.from_cells_bytes(b)) == b


def _batched(variant, mode, params, E, T, nthreads, N=16, max_steps=60):
    z = np.load(os.path.join(GOLDEN_DIR, "room_12x12_reference.npz"))
    L = LO.Learn(z["map"], z["sff"], variant, mode, params)
    core = O.Core(z["map"], z["sff"], {"neighborhood": "neumann"})
    A = 32
    pos = np.zeros((E, A), np.uint16)
    for e in range(E):
        pos[e, :N] = core.reset_philox(N, 42, 0, e)
    counts = np.full(E, N, np.int32)
    dff = np.zeros((E, 12, 12), np.float32)
    eps = np.zeros(E, np.int32)
    eps_steps = np.zeros(E, np.int32)
    tot = 0
    for t in range(1, T + 1):
        tot += L.step_philox_batch(pos, counts, dff, eps, eps_steps, 42, t, True, N, max_steps, 0, nthreads)
    vk, vv = L.V.export()
    hk, hv = L.Ht.export()
    ov, oh = np.argsort(vk), np.argsort(hk)
    return pos, counts, dff, eps, tot, vk[ov], vv[ov], hk[oh], hv[oh]


@pytest.mark.parametrize("variant,mode", [("ac", None), ("unified", "actor_only"), ("actor_only", None)])
def test_batched_moore_semantics_independent_of_threads(variant, mode):
    """The batched step with the Moore neighbourhood (nine moves, nine-value H rows, eight
    ffm_actor_only decisions per agent): the same fixed-point sums whatever the threads."""
    p = {"epsilon": 0.1, "block_size": 1, "neighborhood": "moore"} if variant != "ac" else {"neighborhood": "moore"}
    a = _batched(variant, mode, p, 64, 70, 1)
    b = _batched(variant, mode, p, 64, 70, 5)
    for x, y in zip(a, b):
        assert np.array_equal(np.asarray(x), np.asarray(y))
    assert a[3].sum() > 0
    if variant != "ac":
        assert np.asarray(a[8]).shape[1] == 9     # nine-value H rows


@pytest.mark.parametrize("variant,mode", [("ac", None), ("unified", "critic_only"), ("unified", "actor_only"),
                                          ("unified", "both"), ("actor_only", None)])
def test_batched_semantics_independent_of_threads(variant, mode):
    """The batched (Philox) step sums the increments of all envs in fixed point:
    the result cannot depend on how the envs are scheduled."""
    p = {"epsilon": 0.1, "block_size": 1} if variant != "ac" else {}
    a = _batched(variant, mode, p, 96, 70, 1)
    b = _batched(variant, mode, p, 96, 70, 6)
    for x, y in zip(a, b):
        assert np.array_equal(np.asarray(x), np.asarray(y))
    assert a[3].sum() > 0            # episodes ended (exits or truncation) and were re-placed
    assert len(a[5]) > 100
