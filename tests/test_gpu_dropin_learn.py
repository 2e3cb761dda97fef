"""The drop-in learning classes (ffm_amd.model.ffm_ac_core / ffm_unified /
ffm_actor_only) driven exactly like the reference's training drivers drive the
reference's classes (seed, construct, reset / set_epsilon / set_v_table between
episodes, step until empty or max_steps; tests/golden/gen_golden_learn.py), on
the GPU, against the golden vectors recorded from the reference itself:
positions, DFF bits, the returned V / H dicts (keys, insertion order, value
bits) and both global RNG streams afterwards.
"""
import glob
import json
import os
import pickle
import random

import numpy as np
import pytest

from golden_util import GOLDEN_DIR, dff_hash

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

CASES = sorted(os.path.basename(p)[6:-4] for p in glob.glob(os.path.join(GOLDEN_DIR, "learn_*.npz")))


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.init()


def _pack(variant, k):
    from ffm_amd import learn_keys as K
    if variant == "unified":
        return K.from_rank_tuple(k)
    if isinstance(k, (bytes, bytearray)):
        return K.from_cells_bytes(bytes(k))
    return K.from_cells_tuple(k)


@pytest.mark.parametrize("name", CASES)
def test_dropin_class_reproduces_reference_driver_loop(name, tmp_path):
    from ffm_amd import learn_keys as K
    from ffm_amd.model.ffm_ac_core import FloorFieldModel as AC
    from ffm_amd.model.ffm_actor_only import FloorFieldModelActorOnly as AO
    from ffm_amd.model.ffm_unified import FloorFieldModelUnified as UNI
    from ffm_amd.model.ffm_trained_core import FloorFieldModel as TR
    z = np.load(os.path.join(GOLDEN_DIR, f"learn_{name}.npz"), allow_pickle=False)
    z = {k: z[k] for k in z.files}
    params = json.loads(str(z["params"]))
    variant, mode = str(z["variant"]), str(z["mode"]) or None
    W = z["map"].shape[1]
    N, n_ep, max_steps = int(z["N"]), int(z["n_ep"]), int(z["max_steps"])
    sff_path = str(tmp_path / "sff.npy")
    np.save(sff_path, z["sff"])
    kw = {}
    if "pre_h_keys" in z:            # a trained actor, pickled as run_trained_ffm.py loads it
        kw["h_table_path"] = str(tmp_path / "h.pkl")
        rows = {pickle.dumps(K.to_rank_tuple(k)): [float(x) for x in v]
                for k, v in zip(z["pre_h_keys"], z["pre_h_vals"])}
        if "pre_h_odd_keys" in z:    # rows of other lengths (model/ffm_trained_core.py:228-267)
            ends = np.cumsum(z["pre_h_odd_lens"])
            for k, e, n in zip(z["pre_h_odd_keys"], ends, z["pre_h_odd_lens"]):
                rows[pickle.dumps(K.to_rank_tuple(k))] = [float(x) for x in z["pre_h_odd_vals"][e - n:e]]
        with open(kw["h_table_path"], "wb") as f:
            pickle.dump(rows, f)
    if "pre_keys" in z:
        kw["pretrained_v_path"] = str(tmp_path / "v.pkl")
        if variant == "unified":
            d = {pickle.dumps(K.to_rank_tuple(k)): float(v) for k, v in zip(z["pre_keys"], z["pre_vals"])}
        else:
            d = {K.to_cells_bytes(k): float(v) for k, v in zip(z["pre_keys"], z["pre_vals"])}
        with open(kw["pretrained_v_path"], "wb") as f:
            pickle.dump(d, f)
    ep_i = step_i = cell_i = v_off = h_off = 0
    for si, seed in enumerate(z["seeds"]):
        np.random.seed(int(seed))
        random.seed(int(seed))
        if variant == "unified":
            model = UNI(z["map"], sff_path, N, learning_mode=mode, params=dict(params), **kw)
        elif variant == "ac":
            model = AC(z["map"], sff_path, N, params=dict(params))
        elif variant == "trained":
            model = TR(z["map"], sff_path, N, kw["h_table_path"], params=dict(params))
        else:
            model = AO(z["map"], sff_path, N, params=dict(params), **kw)
        for ep in range(n_ep):
            if ep > 0 and variant == "trained":      # run_trained_ffm.py:227-237
                model.positions = model.initialize_agents()
                model.dff = np.zeros_like(model.map_array, dtype=np.float32)
            elif ep > 0:
                if int(z["reload_v"]):
                    model.set_v_table(model.get_v_table())
                model.reset()
            if variant != "ac" and (z["eps"] != 0).any():
                model.set_epsilon(float(z["eps"][ep_i]))
            p0 = model.positions
            ni = int(z["init_n"][ep_i])
            off = int(z["init_n"][:ep_i].sum())
            assert np.array_equal(p0[:, 0] * W + p0[:, 1], z["init"][off:off + ni]), f"seed {seed} ep {ep}: init"
            steps = 0
            while model.positions.shape[0] > 0 and steps < max_steps:
                model.step()
                steps += 1
                p = model.positions
                c = int(z["counts"][step_i])
                assert p.shape[0] == c, f"seed {seed} ep {ep} step {steps}: count"
                assert np.array_equal(p[:, 0] * W + p[:, 1], z["cells"][cell_i:cell_i + c]), \
                    f"seed {seed} ep {ep} step {steps}: positions"
                assert dff_hash(model.dff) == int(z["dff_hash"][step_i]), f"seed {seed} ep {ep} step {steps}: DFF"
                cell_i += c
                step_i += 1
            assert steps == int(z["nsteps"][ep_i])
            ep_i += 1
        if variant == "trained":
            assert list(np.random.mtrand._rand._bit_generator.random_raw(4)) == list(z["np_tail"][si])
            assert [random.getrandbits(32) for _ in range(4)] == list(z["py_tail"][si])
            assert len(model.H) == len(z["pre_h_keys"]) + len(z.get("pre_h_odd_keys", ()))
            model.close()
            continue
        V = model.get_v_table()
        nv = int(z["v_n"][si])
        assert len(V) == nv
        assert np.array_equal(np.array([_pack(variant, k) for k in V], np.uint64), z["v_keys"][v_off:v_off + nv])
        assert np.array_equal(np.array(list(V.values()), np.float64).view(np.uint64),
                              z["v_vals"][v_off:v_off + nv].view(np.uint64))
        v_off += nv
        sz = model.get_v_table_size()
        assert (sz[1] if isinstance(sz, tuple) else sz) == nv
        nh = int(z["h_n"][si])
        Ht = model.get_h_table() if hasattr(model, "get_h_table") else None
        if nh:
            assert len(Ht) == nh
            assert np.array_equal(np.array([_pack(variant, k) for k in Ht], np.uint64),
                                  z["h_keys"][h_off:h_off + nh])
            assert all(isinstance(r, list) and len(r) == z["h_vals"].shape[1] for r in Ht.values())
            assert np.array_equal(np.array(list(Ht.values()), np.float64).view(np.uint64),
                                  z["h_vals"][h_off:h_off + nh].view(np.uint64))
            assert model.get_h_table_size() == (nh, z["h_vals"].shape[1] * nh)
            h_off += nh
        else:
            assert not Ht
        assert list(np.random.mtrand._rand._bit_generator.random_raw(4)) == list(z["np_tail"][si])
        assert [random.getrandbits(32) for _ in range(4)] == list(z["py_tail"][si])
        model.close()


def test_dropin_unified_radius_reset_and_trajectory(tmp_path):
    """reset(exit_pos, radius) (model/ffm_unified.py:131-171, 800-812) and
    run(return_trajectory=True) (:882-932)."""
    from ffm_amd.data import make_room, l1_sff
    from ffm_amd.model.ffm_unified import FloorFieldModelUnified as UNI
    m = make_room(12, 12)
    sff_path = str(tmp_path / "sff.npy")
    np.save(sff_path, l1_sff(m))
    np.random.seed(1)
    random.seed(1)
    model = UNI(m, sff_path, 30, learning_mode="both", params={"block_size": 1, "epsilon": 0.1})
    model.reset(exit_pos=(0, 6), radius=3)
    p = model.positions
    assert 0 < p.shape[0] <= 30 and (np.abs(p[:, 0]) + np.abs(p[:, 1] - 6) <= 3).all()
    steps, traj = model.run(max_steps=200, return_trajectory=True)
    assert steps == len(traj) and traj.dtype == object
    model.reset(exit_pos=(0, 6), radius=0)          # no free cell within radius 0: empty placement
    assert model.positions.shape == (0, 2)
    assert model.run(max_steps=5) == 0
    model.close()
