"""Packed 64-bit state keys of the learning variants, and their conversions
to and from the reference's dict keys.

The reference keys its V and H tables by Python objects:

* ``ffm_unified``: ``((r_U, r_D, r_L, r_R), (bx, by))`` of plain ints
  (``model/ffm_unified.py:188-269``);
* ``ffm_ac_core`` / ``ffm_actor_only``: ``pickle.dumps((cells13, (bx, by)))``
  where every number is a ``numpy.int64`` scalar (``model/ffm_ac_core.py:62-109``,
  ``model/ffm_actor_only.py:102-147``); the actor-only class re-keys a loaded
  critic by the equivalent tuple of plain ints (``:59-64``).

On the device a key is one u64: 2 bits per cell value (13 cells, or the 4
ranks) in bits [0, 26), bx in bits [26, 45), by in bits [45, 64).  The agent's
own cell (cell 4 of the 13) always holds 1, so the all-ones word never occurs
and marks an empty hash slot.
"""
from __future__ import annotations

import importlib.util
import pickle
import sys

import numpy as np


def ensure_numpy_core_alias() -> None:
    """Let table pickles written under NumPy 2 load under NumPy 1.x.

    NumPy 2 pickles its scalars as ``numpy._core.multiarray.scalar``; NumPy 1.x
    has no ``numpy._core`` package.  The reference aliases the module at import
    (model/ffm_unified.py:8-10, model/ffm_actor_only.py:8-10); every loader of
    this package goes through here, so one guarded alias serves them all.
    Under NumPy 2 the real package exists and nothing changes."""
    if "numpy._core" in sys.modules or importlib.util.find_spec("numpy._core") is not None:
        return
    sys.modules["numpy._core"] = np.core
    sys.modules["numpy._core.multiarray"] = np.core.multiarray


ensure_numpy_core_alias()

EMPTY_KEY = (1 << 64) - 1
_BX_SHIFT, _BY_SHIFT = 26, 45
_BLOCK_MASK = (1 << 19) - 1


def pack(cells, bx: int, by: int) -> int:
    k = 0
    for i, c in enumerate(cells):
        c = int(c)
        if not 0 <= c <= 3:
            raise ValueError(f"state cell value {c} outside 0..3")
        k |= c << (2 * i)
    if not (0 <= int(bx) <= _BLOCK_MASK and 0 <= int(by) <= _BLOCK_MASK):
        raise ValueError("block index out of range")
    return k | (int(bx) << _BX_SHIFT) | (int(by) << _BY_SHIFT)


def unpack(key: int, ncells: int):
    key = int(key)
    cells = tuple((key >> (2 * i)) & 3 for i in range(ncells))
    return cells, ((key >> _BX_SHIFT) & _BLOCK_MASK, (key >> _BY_SHIFT) & _BLOCK_MASK)


# ---- reference key objects -------------------------------------------------
def from_rank_tuple(k) -> int:
    """((r0, r1, r2, r3), (bx, by)) -> packed key (model/ffm_unified.py:269)."""
    ranks, (bx, by) = k
    return pack(ranks, bx, by)


def to_rank_tuple(key: int):
    ranks, blk = unpack(key, 4)
    return (tuple(int(r) for r in ranks), (int(blk[0]), int(blk[1])))


class KeyUnpickler(pickle.Unpickler):
    """Decodes key bytes (and table pickles) with every global refused except NumPy's scalar
    reconstruction: a key is a pickled tuple of NumPy integer scalars (model/ffm_ac_core.py:109),
    and nothing in it may run code."""

    _NUMPY = {("numpy.core.multiarray", "scalar"), ("numpy._core.multiarray", "scalar"), ("numpy", "dtype")}

    def __init__(self, f, numpy_scalars: bool = True):
        super().__init__(f)
        self.numpy_scalars = numpy_scalars

    def find_class(self, module, name):
        if self.numpy_scalars and (module, name) in self._NUMPY:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"pickle refers to {module}.{name}: refused")


def loads_key(b: bytes):
    import io
    return KeyUnpickler(io.BytesIO(b)).load()


def from_cells_bytes(b: bytes) -> int:
    """pickle.dumps((cells13, (bx, by))) -> packed key (model/ffm_ac_core.py:109), decoded
    with KeyUnpickler (NumPy scalars only)."""
    cells, (bx, by) = loads_key(b)
    return pack(cells, bx, by)


def to_cells_bytes(key: int) -> bytes:
    """Packed key -> the reference's bytes key (numpy.int64 scalars, protocol default)."""
    cells, (bx, by) = unpack(key, 13)
    return pickle.dumps((tuple(np.int64(c) for c in cells), (np.int64(bx), np.int64(by))))


def from_cells_tuple(k) -> int:
    cells, (bx, by) = k
    return pack(cells, bx, by)


def to_cells_tuple(key: int):
    cells, blk = unpack(key, 13)
    return (tuple(int(c) for c in cells), (int(blk[0]), int(blk[1])))
