"""Host mirror of one device env with the reference classes' value semantics.

The reference model classes own ``positions`` (int64 [n, 2]) and ``dff``
(float32 [H, W]) and rebind both every step (e.g. model/ffm_core.py:102,115);
callers read, copy and sometimes assign them (main.py:44-46,
run_trained_ffm.py:235-236).  The drop-in classes keep those host arrays and
move them to / from env 0 of a device engine (``Engine`` or ``Learner``, both
expose ``set_state`` / ``get_state``) only when they changed.
"""
from __future__ import annotations

import numpy as np


class DeviceEnvState:
    """Mixin: ``positions`` / ``dff`` properties backed by env 0 of ``self._device()``."""

    def _init_state(self, shape):
        self._H, self._W = shape
        self._dff_host = np.zeros(shape, dtype=np.float32)
        self._dff_exposed = True
        self._pos_host = np.zeros((0, 2), dtype=np.int64)
        self._pos_exposed = True

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
        if v.shape != (self._H, self._W):
            raise ValueError("dff must have the map's shape")
        self._dff_host = v
        self._dff_exposed = True

    def _push(self, dev, capacity: int):
        """Upload what the caller may have changed since the last pull."""
        pos = self._pos_host
        n = int(pos.shape[0])
        if n > capacity:
            raise ValueError(f"{n} agents exceed the engine capacity {capacity}")
        cells = None
        if self._pos_exposed:
            p = np.asarray(pos, dtype=np.int64)
            cells = np.full((1, capacity), 0xFFFF, dtype=np.uint16)
            cells[0, :n] = p[:, 0] * self._W + p[:, 1]
        dff = np.asarray(self._dff_host, dtype=np.float32)[None] if self._dff_exposed else None
        dev.set_state(0, positions=cells, counts=np.array([n], np.int32) if cells is not None else None, dff=dff)
        self._pos_exposed = self._dff_exposed = False

    def _pull(self, dev):
        pos, cnt, dff = dev.get_state(0, 1)
        c = pos[0, : int(cnt[0])].astype(np.int64)
        self._pos_host = np.stack([c // self._W, c % self._W], axis=1)
        self._dff_host = dff[0]
        self._pos_exposed = self._dff_exposed = False
