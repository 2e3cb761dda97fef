"""CPU-side checks of the C ABI library and the drop-in host logic (no GPU)."""
import ctypes
import inspect
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib():
    from ffm_amd import build as B
    B.build()
    from ffm_amd.engine import load_library
    return load_library()


def header_functions():
    txt = open(os.path.join(ROOT, "include", "ffm_amd.h")).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\**\s+\**(ffm_\w+)\s*\(", txt, re.M)))


def test_library_exports_every_header_symbol(lib):
    names = header_functions()
    assert len(names) >= 15
    so = ctypes.CDLL(os.path.join(ROOT, "ffm_amd", "_lib", "libffm_amd.so"))
    for n in names:
        assert hasattr(so, n), n
    from ffm_amd.engine import EXPORTED
    assert sorted(EXPORTED) == names


def test_abi_version(lib):
    from ffm_amd.engine import ABI_VERSION
    assert lib.ffm_abi_version() == ABI_VERSION == 2


def test_engine_fails_loudly_without_gpu(lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from ffm_amd.data import make_room, l1_sff
    from ffm_amd.engine import Engine
    m = make_room(12, 12)
    with pytest.raises((RuntimeError, MemoryError)):
        Engine(m, l1_sff(m), n_envs=4, n_agents=8)


def test_engine_validation_before_device(lib):
    from ffm_amd.data import make_room, l1_sff
    from ffm_amd.engine import Engine
    m = make_room(12, 12)
    with pytest.raises(ValueError):
        Engine(m, l1_sff(m), n_envs=1, n_agents=101)
    bad = m.copy()
    bad[5, 0] = 0
    with pytest.raises(ValueError):
        Engine(bad, l1_sff(m), n_envs=1, n_agents=1)
    with pytest.raises(ValueError):
        Engine(m, l1_sff(m)[:5], n_envs=1, n_agents=1)


def test_learner_fails_loudly_without_gpu(lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from ffm_amd.data import make_room, l1_sff
    from ffm_amd.engine import Learner
    m = make_room(12, 12)
    for variant, mode in (("ac", None), ("unified", "both"), ("actor_only", None)):
        with pytest.raises((RuntimeError, MemoryError)):
            Learner(m, l1_sff(m), variant, n_envs=4, n_agents=8, mode=mode)


def test_learner_validation_before_device(lib):
    """The reference's ValueErrors (model/ffm_unified.py:59-63; np.random.choice at
    model/ffm_unified.py:146) come before any device work."""
    from ffm_amd.data import make_room, l1_sff
    from ffm_amd.engine import Learner
    m = make_room(12, 12)
    s = l1_sff(m)
    with pytest.raises(ValueError):
        Learner(m, s, "unified", n_envs=1, n_agents=4, mode="greedy")
    with pytest.raises(ValueError):
        Learner(m, s, "nope", n_envs=1, n_agents=4)
    with pytest.raises(ValueError):
        Learner(m, s, "ac", n_envs=1, n_agents=101)
    with pytest.raises(ValueError):
        Learner(m, s, "ac", n_envs=1, n_agents=4, params={"neighborhood": "hex"})
    odd = m.copy()
    odd[5, 5] = 4            # a map value outside the learning variants' state keys
    with pytest.raises(NotImplementedError):
        Learner(odd, s, "ac", n_envs=1, n_agents=4)
    bad = m.copy()
    bad[5, 0] = 0
    with pytest.raises(ValueError):
        Learner(bad, s, "unified", n_envs=1, n_agents=4)


def test_missing_library_raises(monkeypatch, tmp_path):
    import ffm_amd.engine as E
    monkeypatch.setattr(E, "_lib", None)
    monkeypatch.setattr(E, "LIB_PATH", str(tmp_path / "nope.so"))
    with pytest.raises(ImportError):
        E.load_library()


def test_dropin_signature_matches_reference():
    from ffm_amd.model.ffm_core import FloorFieldModel
    sig = inspect.signature(FloorFieldModel.__init__)
    assert list(sig.parameters) == ["self", "map_array", "sff_path", "N", "params"]
    assert sig.parameters["params"].default is None
    for meth in ("initialize_agents", "get_neighbors", "step", "update_dff", "run"):
        assert callable(getattr(FloorFieldModel, meth))
    assert list(inspect.signature(FloorFieldModel.run).parameters) == ["self", "save_prefix", "save_interval"]


def test_dropin_initialization_consumes_rng_like_reference(tmp_path):
    """initialize_agents (model/ffm_core.py:23-26) against the golden initial placements."""
    import random
    from golden_util import load_case
    from ffm_amd.model.ffm_core import FloorFieldModel
    case = load_case("neumann_12x12_N8")
    sff_path = str(tmp_path / "sff.npy")
    np.save(sff_path, case.sff)
    W = case.map.shape[1]
    for ep in case.episodes[:6]:
        np.random.seed(ep.seed)
        random.seed(ep.seed)
        m = FloorFieldModel(case.map, sff_path, case.N, dict(case.params))
        assert np.array_equal(m.positions[:, 0] * W + m.positions[:, 1], ep.init)
        assert m.positions.dtype == np.int64
        assert m.dff.dtype == np.float32 and not m.dff.any()
        assert m.neighbors == [(-1, 0), (1, 0), (0, -1), (0, 1)]
    with pytest.raises(ValueError):
        FloorFieldModel(case.map, sff_path, 101, dict(case.params))


def test_room_generator_matches_reference_recipe():
    from golden_util import GOLDEN_DIR
    from ffm_amd.data import make_room, l1_sff
    z = np.load(os.path.join(GOLDEN_DIR, "room_12x12_reference.npz"))
    assert np.array_equal(make_room(12, 12), z["map"])
    s = l1_sff(make_room(12, 12))
    assert s.dtype == z["sff"].dtype == np.float32
    assert np.array_equal(s, z["sff"])


def test_learning_dropin_signatures_match_reference():
    """Constructor and method signatures of the reference classes:
    model/ffm_ac_core.py:9, model/ffm_unified.py:27-35, model/ffm_actor_only.py:21-23."""
    from ffm_amd.model.ffm_ac_core import FloorFieldModel as AC
    from ffm_amd.model.ffm_actor_only import FloorFieldModelActorOnly as AO
    from ffm_amd.model.ffm_unified import FloorFieldModelUnified as UNI
    sig = lambda f: list(inspect.signature(f).parameters)
    assert sig(AC.__init__) == ["self", "map_array", "sff_path", "N", "params"]
    assert sig(UNI.__init__) == ["self", "map_array", "sff_path", "N", "learning_mode", "pretrained_v_path", "params"]
    assert inspect.signature(UNI.__init__).parameters["learning_mode"].default == "critic_only"
    assert sig(AO.__init__) == ["self", "map_array", "sff_path", "N", "pretrained_v_path", "params"]
    assert sig(AC.run) == ["self", "save_prefix", "save_interval", "max_steps"]
    for c in (UNI, AO):
        assert sig(c.run) == ["self", "save_prefix", "save_interval", "max_steps", "return_trajectory"]
    assert sig(UNI.reset) == ["self", "exit_pos", "radius"] and sig(UNI.initialize_agents) == sig(UNI.reset)
    for c, meths in ((AC, ["get_v_table", "set_v_table", "get_v_table_size", "reset", "step", "update_dff"]),
                     (UNI, ["get_v_table", "set_v_table", "get_v_table_size", "get_h_table", "get_h_table_size",
                            "set_epsilon", "step", "update_dff"]),
                     (AO, ["get_v_table", "get_v_table_size", "get_h_table", "get_h_table_size", "set_epsilon",
                           "reset", "step", "update_dff"])):
        for m in meths:
            assert callable(getattr(c, m)), (c, m)


def test_trained_dropin_signature_matches_reference():
    """model/ffm_trained_core.py:20 FloorFieldModel(map_array, sff_path, N, h_table_path, params=None)."""
    from ffm_amd.model.ffm_trained_core import FloorFieldModel as TR
    assert list(inspect.signature(TR.__init__).parameters) == ["self", "map_array", "sff_path", "N", "h_table_path",
                                                              "params"]
    assert list(inspect.signature(TR.run).parameters) == ["self", "save_prefix", "save_interval", "max_steps"]
    for m in ("initialize_agents", "get_neighbors", "step", "update_dff"):
        assert callable(getattr(TR, m))


def test_unified_dropin_rejects_bad_mode_before_device(tmp_path):
    """ValueError of model/ffm_unified.py:59-63, raised before any device work."""
    from ffm_amd.data import make_room, l1_sff
    from ffm_amd.model.ffm_unified import FloorFieldModelUnified as UNI
    m = make_room(12, 12)
    p = str(tmp_path / "s.npy")
    np.save(p, l1_sff(m))
    with pytest.raises(ValueError, match="learning_mode must be one of"):
        UNI(m, p, 4, learning_mode="greedy")
