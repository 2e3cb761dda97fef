"""Drop-in ``FloorFieldModelUnified`` of ``model/ffm_unified.py``
(SoraKurihara/FFM): critic_only / actor_only / both learning over rank-encoded
states, stepped on the MI355X (see ``_learn_model``).

Table keys are the reference's tuples ``((r_U, r_D, r_L, r_R), (bx, by))`` of
plain ints (model/ffm_unified.py:188-269); H rows are lists of five floats.
"""
from __future__ import annotations

import pickle

import numpy as np

from .. import learn_keys as K
from ._learn_model import LearnModel, rank_key


class FloorFieldModelUnified(LearnModel):
    """model/ffm_unified.py:13-931."""

    _variant = "unified"

    def __init__(self, map_array, sff_path, N, learning_mode="critic_only", pretrained_v_path=None, params=None):
        default_params = {                                    # :36-53
            "k_S": 10,
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
            "block_size": 5,
            "alpha_h": 0.1,
            "epsilon": 0.0,
        }
        valid_modes = ["critic_only", "actor_only", "both"]   # :59-63
        if learning_mode not in valid_modes:
            raise ValueError(f"learning_mode must be one of {valid_modes}, got {learning_mode}")
        self.learning_mode = learning_mode
        self._init_model(map_array, sff_path, N, params, default_params, mode=learning_mode)
        if learning_mode == "critic_only":                    # :68-77
            self.sff = self._sff_raw
        else:
            self.sff = np.where(np.isinf(self._sff_raw), 0.0, self._sff_raw).astype(np.float32)
        self.positions = self.initialize_agents()
        self.neighbors = self.get_neighbors()
        if pretrained_v_path and learning_mode in ["actor_only", "both"]:     # :84-110
            with open(pretrained_v_path, "rb") as f:
                pretrained = pickle.load(f)
            table = {}
            for k_bytes, v in pretrained.items():
                try:
                    original = pickle.loads(k_bytes)
                except TypeError:
                    original = k_bytes
                ranks = tuple(int(r) for r in original[0])
                block = (int(original[1][0]), int(original[1][1]))
                table[(ranks, block)] = v
            self._import_v(table, K.from_rank_tuple, 0.0)
            self.initial_v_size = len(table)
            print(f"✓ 事前学習済みCriticを読み込みました: {self.initial_v_size}状態")
        else:
            self.initial_v_size = 0
            if learning_mode == "actor_only":
                print("⚠ 警告: actor_onlyモードですが事前学習済みCriticが指定されていません")
        self.alpha_v = self.params["alpha_v"]                 # :117-129
        self.gamma = self.params["gamma"]
        self.block_size = self.params["block_size"]
        if learning_mode in ["actor_only", "both"]:
            self.alpha_h = self.params["alpha_h"]
            self.epsilon = self.params.get("epsilon", 0.0)
            self._learner.set_epsilon(self.epsilon)
        else:
            self.alpha_h = None
            self.epsilon = None

    def initialize_agents(self, exit_pos=None, radius=None):
        """:131-171: all free cells, or the free cells within L1 distance `radius` of `exit_pos`."""
        if exit_pos is None or radius is None:
            return self._draw_all_free()
        exit_x, exit_y = exit_pos
        free_cells = np.argwhere(self.map_array == 0)
        radius_mask = np.abs(free_cells[:, 0] - exit_x) + np.abs(free_cells[:, 1] - exit_y) <= radius
        radius_cells = free_cells[radius_mask]
        available_count = len(radius_cells)
        actual_N = min(self.N, available_count)
        if actual_N == 0:
            return np.empty((0, 2), dtype=np.int32)
        return radius_cells[np.random.choice(available_count, actual_N, replace=False)]

    def reset(self, exit_pos=None, radius=None):
        """:800-812: new placement and DFF; V / H are kept."""
        self.positions = self.initialize_agents(exit_pos=exit_pos, radius=radius)
        self.dff = np.zeros_like(self.map_array, dtype=np.float32)

    def get_v_table(self):
        return self._export("V", rank_key)

    def set_v_table(self, v_table):
        """:823-830: the table becomes v_table; states read later default to 0.0."""
        self._import_v(v_table, K.from_rank_tuple, 0.0)

    def get_v_table_size(self):
        """:832-845"""
        current = self._learner.table_size("V")
        if self.learning_mode == "actor_only":
            return (self.initial_v_size, current, current - self.initial_v_size)
        return current

    def get_h_table(self):
        """:847-856"""
        if self.learning_mode in ["actor_only", "both"]:
            return self._export("H", rank_key)
        return None

    def set_epsilon(self, epsilon):
        """:859-867"""
        if self.learning_mode in ["actor_only", "both"]:
            super().set_epsilon(epsilon)

    def get_h_table_size(self):
        """:869-880"""
        if self.learning_mode in ["actor_only", "both"]:
            n = self._learner.table_size("H")
            return (n, self._learner.n_actions * n)
        return None

    @property
    def V(self):
        return self.get_v_table()

    @property
    def H(self):
        return self.get_h_table()

    def run(self, save_prefix=None, save_interval=100, max_steps=None, return_trajectory=False):
        """:882-932"""
        return self._run(save_prefix, save_interval, max_steps, return_trajectory)
