"""Shared plumbing of the drop-in learning classes (ffm_ac_core, ffm_unified,
ffm_actor_only): one env of a device ``Learner`` in reference-exact (MT) mode.

``step()`` hands the process-global NumPy and CPython generators to the device,
runs the reference's step there (learn_exact_kernel: agents, targets and table
updates in the reference's order) and takes the generators back, so a seeded
driver reproduces the reference bit for bit and interleaves correctly with its
own ``np.random`` / ``random`` use (tests/test_gpu_dropin_learn.py).  The V / H
tables live on the device for the model's whole life; ``get_v_table`` /
``get_h_table`` return them as the reference's dicts (same keys, values and
insertion order), and ``V`` / ``H`` are read-only snapshots of those dicts.
"""
from __future__ import annotations

import numpy as np

from .. import learn_keys as K
from ..engine import Engine, Learner
from ._device_state import DeviceEnvState


class LearnModel(DeviceEnvState):
    _variant = None                 # "ac" / "unified" / "actor_only"

    def _init_model(self, map_array, sff_path, N, params, default_params, mode=None):
        self.params = default_params if params is None else {**default_params, **params}
        self.map_array = map_array.astype(np.uint8)
        self._sff_raw = np.load(sff_path, mmap_mode="r")
        self._init_state(self.map_array.shape)
        self.N = N
        self._mode = mode
        self._dff_engine = None
        free = int(np.count_nonzero(self.map_array == 0))
        self._capacity = max(1, free)
        # agent capacity = every free cell: N may change between episodes (drivers
        # assign model.N before reset(), run_unified_actor_training.py:244)
        self._learner = Learner(self.map_array, np.asarray(self._sff_raw), self._variant, n_envs=1, n_agents=0,
                                agent_capacity=self._capacity, mode=mode, params=self.params, rng="mt",
                                auto_reset=False)

    # -- reference methods --------------------------------------------------------
    def get_neighbors(self):
        if self.params["neighborhood"] == "neumann":
            return [(-1, 0), (1, 0), (0, -1), (0, 1)]
        return [(-1, -1), (-1, 0), (-1, 1), (0, -1), (0, 1), (1, -1), (1, 0), (1, 1)]

    def _draw_all_free(self):
        free_cells = np.argwhere(self.map_array == 0)
        return free_cells[np.random.choice(len(free_cells), self.N, replace=False)]

    def step(self):
        L = self._learner
        self._push(L, self._capacity)
        L.load_rng_from(0)
        L.step(1)
        L.store_rng_to(0)
        self._pull(L)

    def update_dff(self):
        """model/ffm_unified.py:779-798 (= ffm_core.update_dff) on the GPU."""
        if self._dff_engine is None:
            self._dff_engine = Engine(self.map_array, np.asarray(self._sff_raw), n_envs=1, n_agents=0,
                                      agent_capacity=1, params=self.params, rng="mt", auto_reset=False)
        eng = self._dff_engine
        eng.set_state(0, dff=np.asarray(self._dff_host, dtype=np.float32)[None])
        eng.update_dff()
        _, _, d = eng.get_state(0, 1)
        self._dff_host = d[0]
        self._dff_exposed = True

    def _run(self, save_prefix, save_interval, max_steps, return_trajectory):
        buffer = []
        trajectory = [] if return_trajectory else None
        step = 0
        while self.positions.shape[0] > 0:
            if max_steps is not None and step >= max_steps:
                break
            self.step()
            positions_copy = np.copy(self.positions)
            buffer.append(positions_copy)
            if return_trajectory:
                trajectory.append(positions_copy)
            step += 1
            if save_prefix and (step % save_interval == 0):
                np.savez_compressed(f"{save_prefix}_{step}.npz", positions=np.array(buffer, dtype=np.int32))
                buffer = []
        if save_prefix and buffer:
            np.savez_compressed(f"{save_prefix}_final.npz", positions=np.array(buffer, dtype=np.int32))
        if return_trajectory:
            return step, np.array(trajectory, dtype=object)
        return step

    # -- tables ------------------------------------------------------------------------
    def _export(self, which, to_key):
        keys, vals = self._learner.export_table(which)
        if which == "V":
            return {to_key(k): float(v) for k, v in zip(keys.tolist(), vals.tolist())}
        return {to_key(k): [float(x) for x in row] for k, row in zip(keys.tolist(), vals.tolist())}

    def _import_v(self, table, from_key, default):
        keys = np.array([from_key(k) for k in table.keys()], dtype=np.uint64)
        vals = np.array([float(v) for v in table.values()], dtype=np.float64)
        self._learner.set_v_default(default)
        self._learner.import_table("V", keys, vals)

    def set_epsilon(self, epsilon):
        self.epsilon = float(np.clip(epsilon, 0.0, 1.0))
        self._learner.set_epsilon(self.epsilon)

    def close(self):
        for d in (getattr(self, "_learner", None), getattr(self, "_dff_engine", None)):
            if d is not None:
                d.close()


def rank_key(k):
    return K.to_rank_tuple(k)


def cells_bytes_key(k):
    return K.to_cells_bytes(k)
