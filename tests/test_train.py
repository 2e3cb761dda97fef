"""The training drivers' settings (ffm_amd/train.py) against the reference drivers'
module constants: ``--variant actor_only`` runs run_actor_only_training.py's
MODEL_PARAMS, N list, episodes, MAX_STEPS and epsilon, ``--variant ac``
run_critic_training.py's, ``--variant unified`` run_unified_*_training.py's -- and
each is what main() hands the Learner."""
from __future__ import annotations

import ast
import os

import numpy as np
import pytest

from ffm_amd import train as T

REF = "/root/reference"


def _ref_constants(script):
    """Module-level constants of a reference driver, read as text (never imported)."""
    path = os.path.join(REF, script)
    if not os.path.exists(path):
        pytest.skip("reference checkout absent")
    tree = ast.parse(open(path, encoding="utf-8").read())
    out = {}
    for node in tree.body:
        if isinstance(node, ast.Assign) and len(node.targets) == 1 and isinstance(node.targets[0], ast.Name):
            try:
                out[node.targets[0].id] = ast.literal_eval(node.value)
            except ValueError:
                if isinstance(node.value, ast.Dict):      # MODEL_PARAMS references EPSILON_START
                    d = {}
                    for k, v in zip(node.value.keys, node.value.values):
                        d[ast.literal_eval(k)] = (out[v.id] if isinstance(v, ast.Name) else ast.literal_eval(v))
                    out[node.targets[0].id] = d
    return out


@pytest.mark.parametrize("variant,script", [("actor_only", "run_actor_only_training.py"),
                                            ("ac", "run_critic_training.py")])
def test_driver_settings_match_reference_constants(variant, script):
    c = _ref_constants(script)
    d = T.driver_settings(variant)
    assert d["params"] == c["MODEL_PARAMS"]
    assert d["n_list"] == c["N_FIXED"] + list(range(c["N_START"], c["N_END"] + 1, c["N_STEP"]))
    assert d["episodes"] == c["EPISODES_PER_N"]
    assert d["max_steps"] == c["MAX_STEPS"]
    if "EPSILON_START" in c:
        assert d["eps"] == (c["EPSILON_START"], c["EPSILON_END"])


def test_unified_driver_settings_match_reference_constants():
    c = _ref_constants("run_unified_actor_training.py")
    d = T.driver_settings("unified")
    for k, v in c["MODEL_PARAMS"].items():
        if k in d["params"]:
            assert d["params"][k] == v, k
    assert d["max_steps"] == c["MAX_STEPS"]


class _Stop(Exception):
    pass


@pytest.mark.parametrize("variant", ["actor_only", "ac", "unified"])
def test_main_passes_the_variants_own_params(variant, monkeypatch):
    """main() builds the Learner with the chosen driver's MODEL_PARAMS and MAX_STEPS (the
    round-3 bug: every variant got ffm_unified's)."""
    seen = {}

    def fake_learner(m, s, v, **kw):
        seen.update(kw, variant=v)
        raise _Stop

    monkeypatch.setattr(T, "Learner", fake_learner)
    with pytest.raises(_Stop):
        T.main(["--variant", variant, "--envs", "8"])
    d = T.DRIVERS[variant]
    assert seen["variant"] == variant
    assert seen["params"] == d["params"]
    assert seen["max_steps"] == d["max_steps"]
    assert seen["n_agents"] == max(d["n_list"])


def test_main_overrides_from_command_line(monkeypatch):
    seen = {}

    def fake_learner(m, s, v, **kw):
        seen.update(kw)
        raise _Stop

    monkeypatch.setattr(T, "Learner", fake_learner)
    with pytest.raises(_Stop):
        T.main(["--variant", "actor_only", "--n", "32", "--max-steps", "200", "--envs", "8"])
    assert seen["n_agents"] == 32 and seen["max_steps"] == 200
    assert seen["params"]["gamma"] == 0.95 and seen["params"]["step_penalty"] == 0.0
    assert np.isclose(seen["params"]["alpha_v"], 0.1)
