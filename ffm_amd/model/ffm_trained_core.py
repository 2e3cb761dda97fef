"""Drop-in ``FloorFieldModel`` of ``model/ffm_trained_core.py`` (SoraKurihara/FFM):
evacuation driven by a trained actor (the H table of an ffm_unified run), stepped
on the MI355X (see ``_learn_model``).  Nothing is learned; the table is read only.

The trained table is a pickle whose keys are ``pickle.dumps(((r_U, r_D, r_L, r_R),
(bx, by)))`` bytes and whose values are lists of action preferences, one per move
(five, or nine with the Moore neighbourhood: model/ffm_trained_core.py:51-68, 76-85,
228-236); ``H`` exposes it re-keyed by tuples of ints, as the reference does.
"""
from __future__ import annotations

import pickle

import numpy as np

from .. import learn_keys as K
from ._learn_model import LearnModel


class FloorFieldModel(LearnModel):
    """model/ffm_trained_core.py:13-390."""

    _variant = "trained"

    def __init__(self, map_array, sff_path, N, h_table_path, params=None):
        default_params = {                                    # :29-36
            "k_D": 1,
            "k_A": 10,
            "diffuse": 0.2,
            "decay": 0.2,
            "neighborhood": "neumann",
            "block_size": 5,
        }
        self._init_model(map_array, sff_path, N, params, default_params)
        self.sff = np.where(np.isinf(self._sff_raw), 0.0, self._sff_raw).astype(np.float32)   # :41-43
        self.positions = self.initialize_agents()
        self.neighbors = self.get_neighbors()
        self.block_size = self.params["block_size"]
        with open(h_table_path, "rb") as f:                   # :51-68
            h_table_pickled = pickle.load(f)
        self.H = {}
        for k_bytes, v in h_table_pickled.items():
            original = pickle.loads(k_bytes)
            ranks = tuple(int(r) for r in original[0])
            block = (int(original[1][0]), int(original[1][1]))
            self.H[(ranks, block)] = v
        # one preference per move: the neighbours then stay, 5 (neumann) or 9 (moore, :76-85).
        # A row of another length scores as a missing state (zeros, :228-239) but its values
        # still join the table's min / max (:242-267): they go to the learner's extra
        # statistics instead of the table.
        width = len(self.neighbors) + 1
        if any(not isinstance(v, list) for v in self.H.values()):
            raise NotImplementedError("trained H rows must be lists of preferences (model/ffm_trained_core.py:242-249)")
        rows = [(K.from_rank_tuple(k), v) for k, v in self.H.items() if len(v) == width]
        if rows:
            self._learner.import_table("H", np.array([k for k, _ in rows], np.uint64),
                                       np.array([[float(x) for x in v] for _, v in rows], np.float64))
        odd = [float(x) for v in self.H.values() if len(v) != width for x in v]
        if odd:
            self._learner.set_h_extra(np.array(odd, np.float64))
        print(f"✓ 学習済みHテーブルを読み込みました: {len(self.H)}状態")

    def initialize_agents(self):
        """:70-74"""
        return self._draw_all_free()

    def run(self, save_prefix=None, save_interval=100, max_steps=None):
        """:361-390"""
        return self._run(save_prefix, save_interval, max_steps, False)
