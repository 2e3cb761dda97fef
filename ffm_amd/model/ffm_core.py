"""Drop-in ``FloorFieldModel`` (reference: SoraKurihara/FFM ``model/ffm_core.py``).

Same constructor, methods, attributes and RNG consumption as the reference
class, so ``main.py``-style drivers run unchanged with
``from ffm_amd.model.ffm_core import FloorFieldModel``.  ``step()`` and
``update_dff()`` run on the MI355X through the C ABI (one env, MT mode): the
process-global NumPy and CPython generators are handed to the device before
each step and taken back after it, so a seeded run reproduces the reference
bit for bit (tests/test_gpu_parity.py) and interleaves correctly with any other
``np.random`` / ``random`` use by the caller.

Value semantics as in the reference: ``step()`` rebinds ``positions`` and
``dff`` (model/ffm_core.py:102,115); both attributes are assignable
(``run_trained_ffm.py:235-236``).
"""
from __future__ import annotations

import numpy as np

from ..engine import Engine


class FloorFieldModel:
    """model/ffm_core.py:6-133."""

    def __init__(self, map_array, sff_path, N, params=None):
        default_params = {                                   # :8-14
            "k_S": 3,
            "k_D": 1,
            "diffuse": 0.2,
            "decay": 0.2,
            "neighborhood": "moore",
        }
        self.params = default_params if params is None else {**default_params, **params}   # :15
        self.map_array = map_array.astype(np.uint8)          # :16
        self.sff = np.load(sff_path, mmap_mode="r")          # :17
        self._H, self._W = self.map_array.shape
        self._dff_host = np.zeros_like(self.map_array, dtype=np.float32)   # :18
        self._dff_exposed = True
        self.N = N                                           # :19
        self._engine = None
        self._capacity = 0
        self._pos_host = None
        self._pos_exposed = True
        self.positions = self.initialize_agents()            # :20
        self.neighbors = self.get_neighbors()                # :21

    # -- reference methods ------------------------------------------------------
    def initialize_agents(self):
        """model/ffm_core.py:23-26 (host: draws the placement from np.random)."""
        free_cells = np.argwhere(self.map_array == 0)
        selected = free_cells[np.random.choice(len(free_cells), self.N, replace=False)]
        return selected

    def get_neighbors(self):
        """model/ffm_core.py:28-34."""
        if self.params["neighborhood"] == "neumann":
            return [(-1, 0), (1, 0), (0, -1), (0, 1)]
        return [(-1, -1), (-1, 0), (-1, 1),
                (0, -1), (0, 1),
                (1, -1), (1, 0), (1, 1)]

    def step(self):
        """model/ffm_core.py:36-104 on the GPU (fused decide/resolve/exit/DFF kernel)."""
        eng = self._sync_to_device()
        eng.load_rng_from(0)
        eng.step(1)
        eng.store_rng_to(0)
        self._pull()

    def update_dff(self):
        """model/ffm_core.py:106-117 on the GPU."""
        eng = self._sync_to_device()
        eng.update_dff()
        self._pull()

    def run(self, save_prefix=None, save_interval=100):
        """model/ffm_core.py:119-133."""
        buffer = []
        step = 0
        while self.positions.shape[0] > 0:
            self.step()
            buffer.append(np.copy(self.positions))
            step += 1
            if save_prefix and (step % save_interval == 0):
                np.savez_compressed(f"{save_prefix}_{step}.npz", positions=np.array(buffer, dtype=np.int32))
                buffer = []
        if save_prefix and buffer:
            np.savez_compressed(f"{save_prefix}_final.npz", positions=np.array(buffer, dtype=np.int32))

    # -- attributes with the reference's value semantics ---------------------------
    @property
    def positions(self):
        self._pos_exposed = True
        return self._pos_host

    @positions.setter
    def positions(self, value):
        v = np.asarray(value)
        if v.size == 0:
            v = np.zeros((0, 2), dtype=np.int64)
        if v.ndim != 2 or v.shape[1] != 2:
            raise ValueError("positions must be an [n, 2] array of (x, y) cells")
        self._pos_host = v
        self._pos_exposed = True

    @property
    def dff(self):
        self._dff_exposed = True
        return self._dff_host

    @dff.setter
    def dff(self, value):
        v = np.asarray(value)
        if v.shape != self.map_array.shape:
            raise ValueError("dff must have the map's shape")
        self._dff_host = v
        self._dff_exposed = True

    # -- device plumbing -------------------------------------------------------------
    def _ensure_engine(self, n: int) -> Engine:
        if self._engine is None or n > self._capacity:
            cap = max(1, int(n), int(self.N) if self.N else 1)
            self._engine = Engine(self.map_array, np.asarray(self.sff), n_envs=1, n_agents=0,
                                  agent_capacity=cap, params=self.params, rng="mt", auto_reset=False)
            self._capacity = cap
            self._pos_exposed = self._dff_exposed = True
        return self._engine

    def _sync_to_device(self) -> Engine:
        pos = self._pos_host
        n = int(pos.shape[0])
        eng = self._ensure_engine(n)
        cells = None
        if self._pos_exposed:
            p = np.asarray(pos, dtype=np.int64)
            cells = np.full((1, self._capacity), 0xFFFF, dtype=np.uint16)
            cells[0, :n] = p[:, 0] * self._W + p[:, 1]
        dff = np.asarray(self._dff_host, dtype=np.float32)[None] if self._dff_exposed else None
        eng.set_state(0, positions=cells, counts=np.array([n], np.int32) if cells is not None else None, dff=dff)
        self._pos_exposed = self._dff_exposed = False
        return eng

    def _pull(self):
        pos, cnt, dff = self._engine.get_state(0, 1)
        c = pos[0, : int(cnt[0])].astype(np.int64)
        self._pos_host = np.stack([c // self._W, c % self._W], axis=1)
        self._dff_host = dff[0]
        self._pos_exposed = self._dff_exposed = False
