"""Drop-in ``FloorFieldModelActorOnly`` of ``model/ffm_actor_only.py``
(SoraKurihara/FFM), the config-4 model, stepped on the MI355X (see
``_learn_model``), quirks included: one decision per neighbour
(model/ffm_actor_only.py:214-355) and a uniform policy over the valid moves
whenever any move is invalid (:294-304).

Keys: the step encodes states as ``pickle.dumps((cells13, (bx, by)))`` bytes
(:102-147), while a pretrained critic is re-keyed by tuples of ints (:59-64).
Bytes never equal tuples, so in the reference the pretrained entries are never
read or updated by the step; they only count in ``len(V)``.  This class keeps
them the same way: host-side, inert, first in ``get_v_table()``'s order.
"""
from __future__ import annotations

import pickle

import numpy as np

from ._learn_model import LearnModel, cells_bytes_key


class FloorFieldModelActorOnly(LearnModel):
    """model/ffm_actor_only.py:13-664."""

    _variant = "actor_only"

    def __init__(self, map_array, sff_path, N, pretrained_v_path=None, params=None):
        default_params = {                                    # :24-40
            "k_D": 1,
            "k_A": 10,
            "diffuse": 0.2,
            "decay": 0.2,
            "neighborhood": "neumann",
            "alpha_v": 0.1,
            "gamma": 0.95,
            "exit_reward": 100.0,
            "step_penalty": 0.0,
            "collision_penalty": -1.0,
            "alpha_h": 0.1,
            "epsilon": 0.0,
        }
        self._init_model(map_array, sff_path, N, params, default_params)
        self.sff = np.where(np.isinf(self._sff_raw), 0.0, self._sff_raw).astype(np.float32)   # :44-48
        self.positions = self.initialize_agents()
        self.neighbors = self.get_neighbors()
        self._v_pretrained = {}
        if pretrained_v_path:                                 # :55-70
            with open(pretrained_v_path, "rb") as f:
                pretrained = pickle.load(f)
            for k, v in pretrained.items():
                real_key = pickle.loads(k)
                clean_key = tuple(tuple(int(x) for x in sub) for sub in real_key)
                self._v_pretrained[clean_key] = v
            self.initial_v_size = len(self._v_pretrained)
            print(f"✓ 事前学習済みCriticを読み込みました: {self.initial_v_size}状態")
        else:
            self.initial_v_size = 0
            print("⚠ 事前学習済みCriticなしで開始します")
        self.alpha_v = self.params["alpha_v"]
        self.gamma = self.params["gamma"]
        self.alpha_h = self.params["alpha_h"]
        self.epsilon = self.params.get("epsilon", 0.0)
        self._learner.set_epsilon(self.epsilon)

    def initialize_agents(self):
        """:80-85"""
        return self._draw_all_free()

    def reset(self):
        """:557-563"""
        self.positions = self.initialize_agents()
        self.dff = np.zeros_like(self.map_array, dtype=np.float32)

    def get_v_table(self):
        """:565-572"""
        return {**self._v_pretrained, **self._export("V", cells_bytes_key)}

    def get_v_table_size(self):
        """:574-583"""
        current = len(self._v_pretrained) + self._learner.table_size("V")
        return (self.initial_v_size, current, current - self.initial_v_size)

    def get_h_table(self):
        """:585-592"""
        return self._export("H", cells_bytes_key)

    def get_h_table_size(self):
        """:603-611"""
        n = self._learner.table_size("H")
        return (n, self._learner.n_actions * n)

    @property
    def V(self):
        return self.get_v_table()

    @property
    def H(self):
        return self.get_h_table()

    def run(self, save_prefix=None, save_interval=100, max_steps=None, return_trajectory=False):
        """:613-664"""
        return self._run(save_prefix, save_interval, max_steps, return_trajectory)
