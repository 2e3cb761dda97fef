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
from ._device_state import DeviceEnvState


class FloorFieldModel(DeviceEnvState):
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
        self._init_state(self.map_array.shape)               # dff zeros f32, :18
        self.N = N                                           # :19
        self._engine = None
        self._capacity = 0
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
        self._pull(eng)

    def update_dff(self):
        """model/ffm_core.py:106-117 on the GPU."""
        eng = self._sync_to_device()
        eng.update_dff()
        self._pull(eng)

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
        eng = self._ensure_engine(int(self._pos_host.shape[0]))
        self._push(eng, self._capacity)
        return eng
