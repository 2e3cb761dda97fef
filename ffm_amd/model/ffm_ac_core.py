"""Drop-in ``FloorFieldModel`` of ``model/ffm_ac_core.py`` (SoraKurihara/FFM):
ffm_core stepping with always-a-winner conflicts and a TD(0) critic V over
13-cell state keys, stepped on the MI355X (see ``_learn_model``).

V keys are the reference's: ``pickle.dumps((cells13, (bx, by)))`` of numpy.int64
scalars (model/ffm_ac_core.py:62-109).
"""
from __future__ import annotations

import numpy as np

from .. import learn_keys as K
from ._learn_model import LearnModel, cells_bytes_key


class FloorFieldModel(LearnModel):
    """model/ffm_ac_core.py:8-390."""

    _variant = "ac"

    def __init__(self, map_array, sff_path, N, params=None):
        default_params = {                                    # :10-23
            "k_S": 10,
            "k_D": 1,
            "diffuse": 0.2,
            "decay": 0.2,
            "neighborhood": "neumann",
            "alpha_v": 0.1,
            "gamma": 0.95,
            "exit_reward": 100.0,
            "step_penalty": 0.0,
            "collision_penalty": -1.0,
            "block_size": 3,
        }
        self._init_model(map_array, sff_path, N, params, default_params)
        self.sff = self._sff_raw                              # :28
        self.positions = self.initialize_agents()             # :31
        self.neighbors = self.get_neighbors()
        self.alpha_v = self.params["alpha_v"]                 # :36-38
        self.gamma = self.params["gamma"]
        self.block_size = self.params["block_size"]

    def initialize_agents(self):
        """:40-45"""
        return self._draw_all_free()

    def reset(self):
        """:319-325: new placement and DFF; V is kept."""
        self.positions = self.initialize_agents()
        self.dff = np.zeros_like(self.map_array, dtype=np.float32)

    def get_v_table(self):
        """:327-334"""
        return self._export("V", cells_bytes_key)

    def set_v_table(self, v_table):
        """:336-343: the table becomes v_table; states read later default to -1.0."""
        self._import_v(v_table, K.from_cells_bytes, -1.0)

    def get_v_table_size(self):
        """:345-352"""
        return self._learner.table_size("V")

    @property
    def V(self):
        return self.get_v_table()

    def run(self, save_prefix=None, save_interval=100, max_steps=None):
        """:354-390"""
        return self._run(save_prefix, save_interval, max_steps, False)
