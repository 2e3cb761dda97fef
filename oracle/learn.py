"""ctypes front-end of the learning-variant restatement (``oracle/ffm_learn_oracle.c``).

TEST INFRASTRUCTURE ONLY: imported by ``tests/`` and ``bench.py``'s
``cpu_baseline`` leg, never by the product (``ffm_amd/``).

Restates ``model/ffm_ac_core.py``, ``model/ffm_unified.py`` and
``model/ffm_actor_only.py`` of the reference (SoraKurihara/FFM); pinned by
``tests/golden/learn_*.npz`` (recorded from the reference itself).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import oracle as O

VARIANTS = {"ac": 1, "unified": 2, "actor_only": 3, "trained": 4}
MODES = {"critic_only": 0, "actor_only": 1, "both": 2}

# Class defaults of the reference (merged under the caller's params like the reference does).
DEFAULTS = {
    # model/ffm_ac_core.py:10-23
    "ac": {"k_S": 10, "k_D": 1, "diffuse": 0.2, "decay": 0.2, "neighborhood": "neumann", "alpha_v": 0.1,
           "gamma": 0.95, "exit_reward": 100.0, "step_penalty": 0.0, "collision_penalty": -1.0,
           "block_size": 3},
    # model/ffm_unified.py:36-53
    "unified": {"k_S": 10, "k_D": 1, "k_A": 10, "diffuse": 0.2, "decay": 0.2, "neighborhood": "neumann",
                "alpha_v": 0.1, "gamma": 0.95, "exit_reward": 100.0, "step_penalty": 0.0,
                "collision_penalty": -1.0, "block_size": 5, "alpha_h": 0.1, "epsilon": 0.0},
    # model/ffm_actor_only.py:24-40 (block size 5 is hard-coded at :143)
    "actor_only": {"k_D": 1, "k_A": 10, "diffuse": 0.2, "decay": 0.2, "neighborhood": "neumann",
                   "alpha_v": 0.1, "gamma": 0.95, "exit_reward": 100.0, "step_penalty": 0.0,
                   "collision_penalty": -1.0, "alpha_h": 0.1, "epsilon": 0.0},
    # model/ffm_trained_core.py:29-36 (inference only: no learning parameters)
    "trained": {"k_D": 1, "k_A": 10, "diffuse": 0.2, "decay": 0.2, "neighborhood": "neumann", "block_size": 5},
}


class LearnCfg(C.Structure):
    _fields_ = [
        ("H", C.c_int32), ("W", C.c_int32), ("map", C.c_void_p), ("sff32", C.c_void_p),
        ("sff64", C.c_void_p), ("variant", C.c_int32), ("mode", C.c_int32),
        ("k_S", C.c_double), ("k_D", C.c_double), ("k_A", C.c_double), ("diffuse", C.c_double),
        ("decay", C.c_double), ("alpha_v", C.c_double), ("alpha_h", C.c_double), ("gamma", C.c_double),
        ("exit_reward", C.c_double), ("step_penalty", C.c_double), ("collision_penalty", C.c_double),
        ("epsilon", C.c_double), ("v_default", C.c_double), ("block_size", C.c_int32),
        ("eps_start", C.c_double), ("eps_end", C.c_double), ("eps_offset", C.c_double), ("eps_span", C.c_double),
        ("nb", C.c_int32), ("eps_phase", C.c_int32), ("eps_stride", C.c_int64),
    ]


_done = False


def _lib():
    global _done
    L = O.lib()
    if not _done:
        P = C.c_void_p
        L.ffo_tab_new.argtypes = [C.c_int32, C.c_int32]
        L.ffo_tab_new.restype = P
        L.ffo_tab_free.argtypes = [P]
        L.ffo_tab_size.argtypes = [P]
        L.ffo_tab_size.restype = C.c_int64
        L.ffo_tab_export.argtypes = [P, P, P]
        L.ffo_tab_import.argtypes = [P, P, P, C.c_int64]
        L.ffo_tab_import.restype = C.c_int
        L.ffo_learn_step_mt.argtypes = [C.POINTER(LearnCfg), P, P, P, P, P, C.POINTER(O.MT), C.POINTER(O.MT)]
        L.ffo_learn_step_mt.restype = C.c_int
        L.ffo_learn_step_philox_batch.argtypes = [
            C.POINTER(LearnCfg), P, P, C.c_int64, C.c_int32, P, P, P, P, P, C.c_uint64, C.c_uint32,
            C.c_int32, C.c_int32, C.c_int32, C.c_int64, C.POINTER(C.c_uint64), C.c_int]
        L.ffo_learn_step_philox_batch.restype = C.c_int
        L.ffo_lbatch_new.argtypes = [C.POINTER(LearnCfg), P, P, C.c_int64, C.c_int32]
        L.ffo_lbatch_new.restype = P
        L.ffo_lbatch_free.argtypes = [P]
        L.ffo_lbatch_local.argtypes = [P, P, P, P, P, C.c_uint64, C.c_uint32, C.c_int64, C.POINTER(C.c_uint64),
                                       C.c_int]
        L.ffo_lbatch_set_placement.argtypes = [P, P, C.c_int32]
        L.ffo_lbatch_local.restype = C.c_int
        L.ffo_lbatch_apply.argtypes = [P, C.c_int]
        L.ffo_lbatch_post.argtypes = [P]
        L.ffo_lbatch_flush.argtypes = [P]
        L.ffo_lbatch_end.argtypes = [P, P, P, P, P, P, C.c_uint64, C.c_uint32, C.c_int32, C.c_int32, C.c_int32,
                                     C.c_int64, P]
        L.ffo_lbatch_end.restype = C.c_int64
        L.ffo_tab_delta_export.argtypes = [P, P, P]
        L.ffo_tab_delta_export.restype = C.c_int64
        L.ffo_tab_delta_merge.argtypes = [P, P, P, C.c_int64, P]
        L.ffo_tab_delta_merge.restype = C.c_int
        L.ffo_det_exp.argtypes = [C.c_double]
        L.ffo_det_exp.restype = C.c_double
        L.ffo_encode_rank.argtypes = [P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]
        L.ffo_encode_rank.restype = C.c_uint64
        L.ffo_encode_cells13.argtypes = [P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]
        L.ffo_encode_cells13.restype = C.c_uint64
        L.ffo_tab_set_extra.argtypes = [P, P, C.c_int64]
        _done = True
    return L


class Table:
    def __init__(self, width: int, log2_cap: int = 20):
        self.width = width
        self.accw = 2 if width == 1 else width   # accumulator words (V: sum of td, visits)
        self.h = _lib().ffo_tab_new(width, log2_cap)

    def __del__(self):
        if getattr(self, "h", None):
            _lib().ffo_tab_free(self.h)
            self.h = None

    def __len__(self):
        return int(_lib().ffo_tab_size(self.h))

    def export(self):
        n = len(self)
        k = np.zeros(max(n, 1), np.uint64)
        v = np.zeros((max(n, 1), self.width), np.float64)
        _lib().ffo_tab_export(self.h, O._ptr(k), O._ptr(v))
        return k[:n], (v[:n, 0] if self.width == 1 else v[:n])

    def load(self, keys, vals):
        k = np.ascontiguousarray(keys, np.uint64)
        v = np.ascontiguousarray(vals, np.float64).reshape(len(k), self.width)
        if _lib().ffo_tab_import(self.h, O._ptr(k), O._ptr(v), len(k)):
            raise RuntimeError("table full")

    def set_extra(self, vals):
        """ffm_trained_core: values of rows of another length (they join the min / max only)."""
        v = np.ascontiguousarray(vals, np.float64).ravel()
        _lib().ffo_tab_set_extra(self.h, O._ptr(v) if len(v) else None, len(v))


class Learn:
    """One learning-variant configuration with its V and H tables."""

    def __init__(self, map_array, sff, variant: str, mode: str | None = None, params: dict | None = None,
                 log2_cap: int = 20):
        p = {**DEFAULTS[variant], **(params or {})}
        self.params, self.variant = p, variant
        self.mode = mode or ("actor_only" if variant == "actor_only" else "critic_only")
        self.map = np.ascontiguousarray(map_array, dtype=np.uint8)
        sff = np.asarray(sff)
        self.sff32 = np.ascontiguousarray(sff, np.float32) if sff.dtype == np.float32 else None
        self.sff64 = None if self.sff32 is not None else np.ascontiguousarray(sff, np.float64)
        self.H, self.W = self.map.shape
        self.V = Table(1, log2_cap)
        # H rows: one value per move (neighbours + stay): 5, or 9 with the Moore neighbourhood
        moore = p.get("neighborhood", "neumann") == "moore"
        self.n_actions = 9 if moore and variant in ("unified", "actor_only", "trained") else 5
        self.Ht = Table(self.n_actions, log2_cap)
        self.cfg = LearnCfg(
            self.H, self.W, self.map.ctypes.data,
            self.sff32.ctypes.data if self.sff32 is not None else None,
            self.sff64.ctypes.data if self.sff64 is not None else None,
            VARIANTS[variant], MODES[self.mode] if variant == "unified" else (0 if variant == "ac" else 1),
            float(p.get("k_S", 0.0)), float(p["k_D"]), float(p.get("k_A", 0.0)), float(p["diffuse"]),
            float(p["decay"]), float(p.get("alpha_v", 0.0)), float(p.get("alpha_h", 0.0)), float(p.get("gamma", 0.0)),
            float(p.get("exit_reward", 0.0)), float(p.get("step_penalty", 0.0)), float(p.get("collision_penalty", 0.0)),
            float(p.get("epsilon", 0.0)), 0.0, int(p.get("block_size", 5)))
        self.cfg.nb = 8 if p.get("neighborhood", "neumann") == "moore" else 4

    def set_epsilon(self, e: float):
        self.cfg.epsilon = float(min(max(e, 0.0), 1.0))

    def set_v_default(self, v: float):
        self.cfg.v_default = float(v)

    def set_epsilon_schedule(self, start: float, end: float, offset: float, span: float):
        self.cfg.eps_start, self.cfg.eps_end = float(start), float(end)
        self.cfg.eps_offset, self.cfg.eps_span = float(offset), float(span)

    def set_epsilon_phase(self, period: int, stride: int = 1):
        """Global env g adds (g % period) * stride to its ended-episode count in the schedule."""
        self.cfg.eps_phase = int(period)
        self.cfg.eps_stride = int(stride)

    def step_mt(self, pos, dff, np_rng, py_rng):
        p = np.ascontiguousarray(pos, dtype=np.int32).copy()
        n = np.array([p.shape[0]], dtype=np.int32)
        if p.size == 0:
            p = np.zeros(1, np.int32)
        assert dff.dtype == np.float32 and dff.flags.c_contiguous
        rc = _lib().ffo_learn_step_mt(C.byref(self.cfg), self.V.h, self.Ht.h, O._ptr(p), O._ptr(n),
                                      O._ptr(dff), C.byref(np_rng), C.byref(py_rng))
        if rc:
            raise RuntimeError("oracle table full")
        return p[: int(n[0])]

    def step_philox_batch(self, pos, counts, dff, episodes, ep_steps, seed, t, auto_reset, N_reset,
                          max_steps=0, env_base=0, nthreads=1) -> int:
        E, A_cap = pos.shape
        for a, dt in ((pos, np.uint16), (counts, np.int32), (dff, np.float32), (ep_steps, np.int32)):
            assert a.dtype == dt and a.flags.c_contiguous
        tot = C.c_uint64(0)
        rc = _lib().ffo_learn_step_philox_batch(
            C.byref(self.cfg), self.V.h, self.Ht.h, E, A_cap, O._ptr(pos), O._ptr(counts), O._ptr(dff),
            O._ptr(episodes), O._ptr(ep_steps), seed, t, int(auto_reset), N_reset, max_steps, env_base,
            C.byref(tot), nthreads)
        if rc:
            raise RuntimeError("oracle table full")
        return int(tot.value)


class Shard:
    """The batched step of envs [env_base, env_base + E) in phases, with the
    Learner's phase interface (ffm_amd.dist.TableSync): the CPU side of the
    multi-rank tests.  Record buffers are host pointers."""

    def __init__(self, learn: Learn, E: int, A: int, N: int, seed: int, env_base: int, max_steps: int,
                 nthreads: int = 1):
        from . import oracle as O
        self.L, self.E, self.A, self.N = learn, E, A, N
        self.seed, self.env_base, self.max_steps, self.nthreads = seed, env_base, max_steps, nthreads
        self.variant, self.mode = learn.variant, learn.mode
        core = O.Core(learn.map, learn.sff32 if learn.sff32 is not None else learn.sff64, {"neighborhood": "neumann"})
        self.pos = np.full((E, A), 0xFFFF, np.uint16)
        for e in range(E):
            self.pos[e, :N] = core.reset_philox(N, seed, 0, env_base + e)
        self.counts = np.full(E, N, np.int32)
        self.dff = np.zeros((E,) + learn.map.shape, np.float32)
        self.episodes = np.zeros(E, np.int32)
        self.ep_steps = np.zeros(E, np.int32)
        self.t = 1
        self.agent_steps = 0
        self.log = []
        self.sync_period, self.since_apply = 1, 0
        self.dense_tables = False
        self.b = _lib().ffo_lbatch_new(C.byref(learn.cfg), learn.V.h, learn.Ht.h, E, A)

    def __del__(self):
        if getattr(self, "b", None):
            _lib().ffo_lbatch_free(self.b)
            self.b = None

    @property
    def actor(self):
        return self.variant == "actor_only" or (self.variant == "unified" and self.mode != "critic_only")

    @property
    def post_update(self):
        return self.variant == "unified" and self.mode == "actor_only"

    def _tab(self, which):
        return self.L.V if which == "V" else self.L.Ht

    def step_local(self):
        tot = C.c_uint64(0)
        if _lib().ffo_lbatch_local(self.b, O._ptr(self.pos), O._ptr(self.counts), O._ptr(self.dff),
                                   O._ptr(self.episodes), self.seed, self.t, self.env_base, C.byref(tot),
                                   self.nthreads):
            raise RuntimeError("oracle table full")
        self.agent_steps += int(tot.value)

    def set_sync_period(self, k: int):
        """The engine's table sync period (ffm_learner_set_sync_period)."""
        self.sync_period, self.since_apply = int(k), 0

    def apply_due(self) -> bool:
        return self.since_apply + 1 >= self.sync_period

    def set_external_sync(self, on: bool = True):
        """The engine's shared-learner flag: the CPU tables are read-only on export anyway."""
        self.external_sync = bool(on)

    def flush_begin(self) -> bool:
        return self.since_apply != 0

    def flush_end(self):
        """Apply the pending (exchanged) increments of V and H without the post-update pass
        (ffm_learner_flush_end) and restart the period."""
        _lib().ffo_lbatch_flush(self.b)
        self.since_apply = 0

    def step_apply(self, which):
        if self.apply_due():
            _lib().ffo_lbatch_apply(self.b, 0 if which == "V" else 1)
        elif which == "V":
            _lib().ffo_lbatch_post(self.b)

    def set_placement(self, cells, n_agents: int):
        c = np.ascontiguousarray(cells, np.uint16)
        _lib().ffo_lbatch_set_placement(self.b, O._ptr(c), len(c))
        self.N = int(n_agents)

    def step_end(self):
        log = np.zeros((self.E, 4), np.int32)
        n = _lib().ffo_lbatch_end(self.b, O._ptr(self.pos), O._ptr(self.counts), O._ptr(self.dff),
                                  O._ptr(self.episodes), O._ptr(self.ep_steps), self.seed, self.t, 1, self.N,
                                  self.max_steps, self.env_base, O._ptr(log))
        self.log.extend(map(tuple, log[:n].tolist()))
        self.t += 1
        self.since_apply = 0 if self.apply_due() else self.since_apply + 1

    def delta_export(self, which, keys_ptr, acc_ptr, cap):
        T = self._tab(which)
        n = len(T)          # upper bound on the records
        if n > cap:
            return n
        return int(_lib().ffo_tab_delta_export(T.h, keys_ptr, acc_ptr))

    def delta_export_async(self, which, keys_ptr, acc_ptr, cap, count_ptr):
        """The engine's asynchronous export: the count goes to memory (here host memory)."""
        T = self._tab(which)
        tmp_k = np.empty(max(len(T), 1), np.uint64)
        tmp_a = np.empty((max(len(T), 1), T.accw), np.int64)
        n = int(_lib().ffo_tab_delta_export(T.h, O._ptr(tmp_k), O._ptr(tmp_a)))
        m = min(n, int(cap))
        C.memmove(keys_ptr, tmp_k.ctypes.data, m * 8)
        C.memmove(acc_ptr, tmp_a.ctypes.data, m * 8 * T.accw)
        C.c_int64.from_address(count_ptr).value = n
        if n > cap:
            raise RuntimeError("asynchronous delta export: record buffer too small")

    def delta_merge_async(self, which, keys_ptr, acc_ptr, count_ptr, cap):
        self.delta_merge(which, keys_ptr, acc_ptr, min(C.c_int64.from_address(count_ptr).value, int(cap)))

    def delta_merge(self, which, keys_ptr, acc_ptr, n):
        T = self._tab(which)
        init = np.full(T.width, self.L.cfg.v_default if which == "V" else 0.0, np.float64)
        if _lib().ffo_tab_delta_merge(T.h, keys_ptr, acc_ptr, int(n), O._ptr(init)):
            raise RuntimeError("oracle table full")


def det_exp(x: float) -> float:
    return float(_lib().ffo_det_exp(float(x)))


def encode_rank(sm, x, y, bs):
    sm = np.ascontiguousarray(sm, np.uint8)
    return int(_lib().ffo_encode_rank(O._ptr(sm), sm.shape[0], sm.shape[1], x, y, bs))


def encode_cells13(sm, x, y, bs, oob):
    sm = np.ascontiguousarray(sm, np.uint8)
    return int(_lib().ffo_encode_cells13(O._ptr(sm), sm.shape[0], sm.shape[1], x, y, bs, oob))
