"""ctypes front-end of the CPU restatement in ``oracle/ffm_oracle.c``.

TEST INFRASTRUCTURE ONLY: imported by ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg, never by the product (``ffm_amd/``).

Restates the reference's ``model/ffm_core.py`` (SoraKurihara/FFM) step,
update_dff and initialize_agents; parity is pinned against golden vectors made
by the reference itself (``tests/golden/gen_golden.py``).
"""
from __future__ import annotations

import ctypes as C
import os
import random
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libffm_oracle.so")
_lib = None


class MT(C.Structure):
    _fields_ = [("mt", C.c_uint32 * 624), ("pos", C.c_int32)]

    # -- conversions to/from the interpreter's own generators --------------
    @classmethod
    def from_numpy(cls, rs: np.random.RandomState | None = None) -> "MT":
        st = (rs if rs is not None else np.random.mtrand._rand).get_state(legacy=True)
        m = cls()
        np.ctypeslib.as_array(m.mt)[:] = np.asarray(st[1], dtype=np.uint32)
        m.pos = int(st[2])
        return m

    def to_numpy(self, rs: np.random.RandomState | None = None) -> None:
        rs = rs if rs is not None else np.random.mtrand._rand
        st = rs.get_state(legacy=True)
        rs.set_state(("MT19937", np.ctypeslib.as_array(self.mt).copy(), int(self.pos), st[3], st[4]))

    @classmethod
    def from_python(cls, r: random.Random | None = None) -> "MT":
        st = (r if r is not None else random._inst).getstate()
        m = cls()
        np.ctypeslib.as_array(m.mt)[:] = np.asarray(st[1][:624], dtype=np.uint32)
        m.pos = int(st[1][624])
        return m

    def to_python(self, r: random.Random | None = None) -> None:
        r = r if r is not None else random._inst
        st = r.getstate()
        words = tuple(int(w) for w in np.ctypeslib.as_array(self.mt)) + (int(self.pos),)
        r.setstate((st[0], words, st[2]))


class CoreCfg(C.Structure):
    _fields_ = [
        ("H", C.c_int32), ("W", C.c_int32),
        ("map", C.c_void_p), ("sff32", C.c_void_p), ("sff64", C.c_void_p),
        ("nb", C.c_int32),
        ("k_S", C.c_double), ("k_D", C.c_double),
        ("diffuse", C.c_double), ("decay", C.c_double),
    ]


def build() -> str:
    """Compile the restatement (make in oracle/)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        P = C.c_void_p
        L.ffo_mt_seed_np.argtypes = [C.POINTER(MT), C.c_uint32]
        L.ffo_mt_seed_py.argtypes = [C.POINTER(MT), P, C.c_int]
        L.ffo_mt_next.argtypes = [C.POINTER(MT)]
        L.ffo_mt_next.restype = C.c_uint32
        L.ffo_mt_u53.argtypes = [C.POINTER(MT)]
        L.ffo_mt_u53.restype = C.c_double
        L.ffo_np_permutation.argtypes = [C.POINTER(MT), C.c_int64, P]
        L.ffo_py_randbelow.argtypes = [C.POINTER(MT), C.c_uint32]
        L.ffo_py_randbelow.restype = C.c_uint32
        L.ffo_np_expf.argtypes = [C.c_float]
        L.ffo_np_expf.restype = C.c_float
        L.ffo_np_expf_array.argtypes = [P, P, C.c_int64, C.c_int]
        L.ffo_np_sumf.argtypes = [P, C.c_int]
        L.ffo_np_sumf.restype = C.c_float
        L.ffo_np_sumd.argtypes = [P, C.c_int]
        L.ffo_np_sumd.restype = C.c_double
        L.ffo_philox.argtypes = [P, P, P]
        L.ffo_core_step_mt.argtypes = [C.POINTER(CoreCfg), P, P, P, C.POINTER(MT), C.POINTER(MT)]
        L.ffo_core_step_mt.restype = C.c_int
        L.ffo_update_dff.argtypes = [C.POINTER(CoreCfg), P]
        L.ffo_init_agents_mt.argtypes = [C.POINTER(CoreCfg), C.c_int32, C.POINTER(MT), P]
        L.ffo_init_agents_mt.restype = C.c_int
        L.ffo_core_step_philox_batch.argtypes = [
            C.POINTER(CoreCfg), C.c_int64, C.c_int32, P, P, P, P, C.c_uint64, C.c_uint32,
            C.c_int32, C.c_int32, C.c_int64, C.POINTER(C.c_uint64), C.c_int]
        L.ffo_reset_philox.argtypes = [C.POINTER(CoreCfg), C.c_int32, C.c_uint64, C.c_uint32,
                                       C.c_int64, P]
        L.ffo_reset_philox_list.argtypes = [P, C.c_int32, C.c_int32, C.c_uint64, C.c_uint32, C.c_int64, P]
        _lib = L
    return _lib


def _ptr(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def seeded_np(seed: int) -> MT:
    m = MT()
    lib().ffo_mt_seed_np(C.byref(m), seed & 0xFFFFFFFF)
    return m


def seeded_py(seed: int) -> MT:
    n = abs(int(seed))
    key = []
    while True:
        key.append(n & 0xFFFFFFFF)
        n >>= 32
        if n == 0:
            break
    k = np.asarray(key, dtype=np.uint32)
    m = MT()
    lib().ffo_mt_seed_py(C.byref(m), _ptr(k), len(key))
    return m


class Core:
    """One ffm_core configuration (map + SFF + params) for the restatement."""

    def __init__(self, map_array, sff, params: dict, neighborhood: str | None = None):
        defaults = {"k_S": 3, "k_D": 1, "diffuse": 0.2, "decay": 0.2, "neighborhood": "moore"}
        p = {**defaults, **(params or {})}
        if neighborhood is not None:
            p["neighborhood"] = neighborhood
        self.params = p
        self.map = np.ascontiguousarray(map_array, dtype=np.uint8)
        sff = np.asarray(sff)
        self.sff32 = np.ascontiguousarray(sff, dtype=np.float32) if sff.dtype == np.float32 else None
        self.sff64 = None if self.sff32 is not None else np.ascontiguousarray(sff, dtype=np.float64)
        self.H, self.W = self.map.shape
        self.nb = 4 if p["neighborhood"] == "neumann" else 8
        self.cfg = CoreCfg(self.H, self.W, self.map.ctypes.data,
                           self.sff32.ctypes.data if self.sff32 is not None else None,
                           self.sff64.ctypes.data if self.sff64 is not None else None,
                           self.nb, float(p["k_S"]), float(p["k_D"]),
                           float(p["diffuse"]), float(p["decay"]))

    # -- MT (reference-stream) mode ----------------------------------------
    def init_agents_mt(self, N: int, np_rng: MT) -> np.ndarray:
        out = np.zeros(max(N, 1), dtype=np.int32)
        rc = lib().ffo_init_agents_mt(C.byref(self.cfg), N, C.byref(np_rng), _ptr(out))
        if rc != 0:
            raise ValueError("Cannot take a larger sample than population when 'replace=False'")
        return out[:N]

    def step_mt(self, pos: np.ndarray, dff: np.ndarray, np_rng: MT, py_rng: MT) -> np.ndarray:
        """pos: int32 cell indices; dff float32 [H,W] updated in place. Returns new pos."""
        p = np.ascontiguousarray(pos, dtype=np.int32).copy()
        n = np.array([p.shape[0]], dtype=np.int32)
        if p.size == 0:
            p = np.zeros(1, dtype=np.int32)
        assert dff.dtype == np.float32 and dff.flags.c_contiguous
        lib().ffo_core_step_mt(C.byref(self.cfg), _ptr(p), _ptr(n), _ptr(dff),
                               C.byref(np_rng), C.byref(py_rng))
        return p[: int(n[0])]

    def update_dff(self, dff: np.ndarray) -> None:
        lib().ffo_update_dff(C.byref(self.cfg), _ptr(dff))

    # -- Philox (production) mode ------------------------------------------
    def step_philox_batch(self, pos, counts, dff, episodes, seed, t, auto_reset, N_reset,
                          env_base=0, nthreads=1) -> int:
        E, A_cap = pos.shape
        for a, dt in ((pos, np.uint16), (counts, np.int32), (dff, np.float32)):
            assert a.dtype == dt and a.flags.c_contiguous
        tot = C.c_uint64(0)
        lib().ffo_core_step_philox_batch(
            C.byref(self.cfg), E, A_cap, _ptr(pos), _ptr(counts), _ptr(dff), _ptr(episodes),
            seed, t, int(auto_reset), N_reset, env_base, C.byref(tot), nthreads)
        return int(tot.value)

    def reset_philox(self, N, seed, t, genv) -> np.ndarray:
        out = np.zeros(max(N, 1), dtype=np.uint16)
        lib().ffo_reset_philox(C.byref(self.cfg), N, seed, t, genv, _ptr(out))
        return out[:N]


def reset_philox_list(cells, N, seed, t, genv) -> np.ndarray:
    """Philox placement over an explicit candidate list (radius curriculum)."""
    c = np.ascontiguousarray(cells, dtype=np.uint16)
    out = np.zeros(max(N, 1), dtype=np.uint16)
    lib().ffo_reset_philox_list(_ptr(c), len(c), N, seed, t, genv, _ptr(out))
    return out[:N]


def np_expf(x: np.ndarray, nthreads: int = 8) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32)
    y = np.empty_like(x)
    lib().ffo_np_expf_array(_ptr(x), _ptr(y), x.size, nthreads)
    return y


def np_sumf(a: np.ndarray) -> np.float32:
    a = np.ascontiguousarray(a, dtype=np.float32)
    return np.float32(lib().ffo_np_sumf(_ptr(a), a.size))


def philox(ctr, key) -> np.ndarray:
    c = np.asarray(ctr, dtype=np.uint32)
    k = np.asarray(key, dtype=np.uint32)
    o = np.zeros(4, dtype=np.uint32)
    lib().ffo_philox(_ptr(c), _ptr(k), _ptr(o))
    return o
