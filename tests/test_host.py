"""Host-side logic that needs no GPU: key packing, the numpy._core alias used by
the table loaders, bench helpers."""
import importlib
import pickle
import sys

import numpy as np

from ffm_amd import learn_keys as K


def test_numpy_core_alias_loads_numpy2_key_pickles(monkeypatch):
    """A table pickle written under NumPy 2 names numpy._core.multiarray.scalar
    (model/ffm_unified.py:8-10 aliases it for NumPy 1.x).  Simulate an
    interpreter without numpy._core: the alias must make such bytes load."""
    b = K.to_cells_bytes(K.pack([1, 0, 2, 3, 1, 0, 0, 0, 2, 3, 0, 1, 2], 4, 7))
    assert b"numpy._core" in b or b"numpy.core" in b
    saved = {k: v for k, v in sys.modules.items() if k == "numpy._core" or k.startswith("numpy._core.")}
    for k in saved:
        monkeypatch.delitem(sys.modules, k)
    monkeypatch.setattr(importlib.util, "find_spec", lambda name, *a: None)
    K.ensure_numpy_core_alias()
    assert sys.modules["numpy._core"] is np.core
    key = K.from_cells_bytes(b)
    assert K.unpack(key, 13) == ((1, 0, 2, 3, 1, 0, 0, 0, 2, 3, 0, 1, 2), (4, 7))


def test_numpy_core_alias_noop_under_numpy2():
    before = sys.modules.get("numpy._core")
    K.ensure_numpy_core_alias()
    assert sys.modules.get("numpy._core") is before


def test_rank_key_roundtrip():
    k = ((3, 0, 2, 1), (255, 17))
    assert K.to_rank_tuple(K.from_rank_tuple(k)) == k
    b = pickle.dumps(k)
    assert K.to_rank_tuple(K.from_rank_tuple(pickle.loads(b))) == k
