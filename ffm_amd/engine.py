"""Python binding of the C ABI in ``include/ffm_amd.h`` (ctypes).

``Engine`` owns E independent environments of the reference's
``FloorFieldModel`` (SoraKurihara/FFM ``model/ffm_core.py``) on one MI355X and
steps all of them with one fused HIP kernel launch per step.  There is no CPU
fallback: if the HIP library is missing, importing the engine raises.
"""
from __future__ import annotations

import ctypes as C
import os
import random as _pyrandom

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FFM_LIB_PATH") or os.path.join(_HERE, "_lib", "libffm_amd.so")

ABI_VERSION = 2
OK, E_INVALID, E_HIP, E_NOMEM, E_UNSUPPORTED = 0, -1, -2, -3, -4
VARIANT_CORE = 0
RNG_PHILOX, RNG_MT = 0, 1
SFF_F32, SFF_F64 = 0, 1

EXPORTED = [
    "ffm_last_error", "ffm_abi_version", "ffm_engine_create", "ffm_engine_destroy",
    "ffm_engine_reset", "ffm_engine_reset_envs", "ffm_engine_step", "ffm_engine_update_dff", "ffm_engine_set_state",
    "ffm_engine_get_state", "ffm_engine_set_mt_state", "ffm_engine_get_mt_state",
    "ffm_engine_get_counters", "ffm_engine_device_buffers", "ffm_engine_get_step_index",
    "ffm_engine_set_step_index", "ffm_engine_set_fused_steps", "ffm_np_expf_device",
    "ffm_engine_set_trajectory_capture", "ffm_engine_drain_trajectory",
    "ffm_learner_create", "ffm_learner_destroy", "ffm_learner_reset", "ffm_learner_reset_envs", "ffm_learner_step",
    "ffm_learner_set_state", "ffm_learner_get_state", "ffm_learner_get_episodes",
    "ffm_learner_set_mt_state", "ffm_learner_get_mt_state", "ffm_learner_get_counters",
    "ffm_learner_set_epsilon", "ffm_learner_set_v_default", "ffm_learner_table_size",
    "ffm_learner_export_table", "ffm_learner_import_table", "ffm_learner_get_step_index",
    "ffm_learner_set_step_index", "ffm_learner_step_local", "ffm_learner_step_apply", "ffm_learner_step_end",
    "ffm_learner_delta_export", "ffm_learner_delta_merge", "ffm_learner_set_placement",
    "ffm_learner_set_epsilon_schedule", "ffm_learner_set_epsilon_phase", "ffm_learner_drain_episodes",
    "ffm_learner_set_trajectory_capture", "ffm_learner_drain_trajectory",
    "ffm_learner_delta_export_async", "ffm_learner_delta_merge_async", "ffm_learner_set_sync_period",
    "ffm_learner_apply_due", "ffm_learner_dense_buffers", "ffm_learner_dense_adopt",
    "ffm_learner_tiled_buffers", "ffm_learner_step_tiled_local", "ffm_learner_step_tiled_apply",
    "ffm_learner_set_external_sync", "ffm_learner_flush_begin", "ffm_learner_flush_end",
    "ffm_learner_set_tile_owners", "ffm_learner_owner_buffers", "ffm_learner_step_owner_local",
    "ffm_learner_step_owner_v", "ffm_learner_step_owner_h", "ffm_learner_step_owner_end",
    "ffm_learner_set_epsilon_stride", "ffm_learner_set_episode_caps", "ffm_learner_set_owner_capacity",
    "ffm_learner_set_owner_send_buffer", "ffm_learner_set_owner_output_buffers", "ffm_learner_set_h_extra",
]

VARIANT_AC, VARIANT_UNIFIED, VARIANT_ACTOR_ONLY, VARIANT_TRAINED = 1, 2, 3, 4
LEARN_MODES = {"critic_only": 0, "actor_only": 1, "both": 2}
TABLE_V, TABLE_H = 0, 1


class EngineDesc(C.Structure):
    _fields_ = [
        ("abi_version", C.c_int32), ("variant", C.c_int32),
        ("H", C.c_int32), ("W", C.c_int32),
        ("map", C.c_void_p), ("sff", C.c_void_p), ("sff_dtype", C.c_int32),
        ("neighborhood", C.c_int32),
        ("k_S", C.c_double), ("k_D", C.c_double), ("diffuse", C.c_double), ("decay", C.c_double),
        ("n_envs", C.c_int64), ("agent_capacity", C.c_int32), ("n_agents", C.c_int32),
        ("rng_mode", C.c_int32), ("auto_reset", C.c_int32), ("seed", C.c_uint64),
        ("env_base", C.c_int64), ("device", C.c_int32), ("envs_per_block", C.c_int32),
    ]


class LearnDesc(C.Structure):
    _fields_ = [
        ("mode", C.c_int32), ("k_A", C.c_double),
        ("alpha_v", C.c_double), ("alpha_h", C.c_double), ("gamma", C.c_double),
        ("exit_reward", C.c_double), ("step_penalty", C.c_double), ("collision_penalty", C.c_double),
        ("epsilon", C.c_double), ("v_default", C.c_double),
        ("block_size", C.c_int32), ("max_steps", C.c_int32),
        ("log2_v_capacity", C.c_int32), ("log2_h_capacity", C.c_int32),
        ("eps_start", C.c_double), ("eps_end", C.c_double), ("eps_offset", C.c_double), ("eps_span", C.c_double),
    ]


class OwnerBuffers(C.Structure):
    """ffm_owner_buffers (include/ffm_amd.h): the owner-sharded exchange's device buffers."""
    _fields_ = [
        ("world", C.c_int32), ("rank", C.c_int32),
        ("send_recs", C.c_void_p), ("send_rec_capacity", C.c_int64),
        ("send_hdr", C.c_void_p), ("hdr_stride", C.c_int64),
        ("counts", C.c_void_p),
        ("v_slot", C.c_void_p), ("v_val", C.c_void_p), ("h_key", C.c_void_p), ("h_q", C.c_void_p),
        ("out_counts", C.c_void_p), ("v_capacity", C.c_int64), ("h_capacity", C.c_int64),
        ("tsum", C.c_void_p), ("tsum_count", C.c_int64),
    ]


class DeviceBuffers(C.Structure):
    _fields_ = [
        ("positions", C.c_void_p), ("counts", C.c_void_p), ("dff", C.c_void_p),
        ("episodes", C.c_void_p), ("counters", C.c_void_p),
        ("mt_np", C.c_void_p), ("mt_py", C.c_void_p), ("counter_slots", C.c_int64),
    ]


_lib = None


def load_library():
    """Load libffm_amd.so.  Raises (never falls back) when it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"ffm_amd HIP library not found at {LIB_PATH}; build it with "
            "`python -m ffm_amd.build` (hipcc --offload-arch=gfx950)")
    L = C.CDLL(LIB_PATH)
    P, i32, i64 = C.c_void_p, C.c_int32, C.c_int64
    L.ffm_last_error.restype = C.c_char_p
    L.ffm_abi_version.restype = C.c_int
    L.ffm_engine_create.argtypes = [C.POINTER(EngineDesc), C.POINTER(P)]
    L.ffm_engine_destroy.argtypes = [P]
    L.ffm_engine_reset.argtypes = [P, P]
    L.ffm_engine_reset_envs.argtypes = [P, P, P]
    L.ffm_engine_step.argtypes = [P, i32, P]
    L.ffm_engine_update_dff.argtypes = [P, P]
    L.ffm_engine_set_state.argtypes = [P, i64, i64, P, P, P, P]
    L.ffm_engine_get_state.argtypes = [P, i64, i64, P, P, P, P]
    L.ffm_engine_set_mt_state.argtypes = [P, i64, P, i32, P, i32, P]
    L.ffm_engine_get_mt_state.argtypes = [P, i64, P, C.POINTER(i32), P, C.POINTER(i32), P]
    L.ffm_engine_get_counters.argtypes = [P, P, P]
    L.ffm_engine_device_buffers.argtypes = [P, C.POINTER(DeviceBuffers)]
    L.ffm_engine_get_step_index.argtypes = [P, C.POINTER(C.c_uint32)]
    L.ffm_engine_set_step_index.argtypes = [P, C.c_uint32]
    L.ffm_engine_set_fused_steps.argtypes = [P, i32]
    L.ffm_engine_set_trajectory_capture.argtypes = [P, P, P, i32, i32, i64, P]
    L.ffm_engine_drain_trajectory.argtypes = [P, P, P, i64, C.POINTER(i64), C.POINTER(i64), P]
    L.ffm_np_expf_device.argtypes = [P, P, i64, P]
    L.ffm_learner_create.argtypes = [C.POINTER(EngineDesc), C.POINTER(LearnDesc), C.POINTER(P)]
    L.ffm_learner_destroy.argtypes = [P]
    L.ffm_learner_reset.argtypes = [P, P]
    L.ffm_learner_reset_envs.argtypes = [P, P, P]
    L.ffm_learner_step.argtypes = [P, i32, P]
    L.ffm_learner_set_state.argtypes = [P, i64, i64, P, P, P, P]
    L.ffm_learner_get_state.argtypes = [P, i64, i64, P, P, P, P]
    L.ffm_learner_get_episodes.argtypes = [P, i64, i64, P, P, P]
    L.ffm_learner_set_mt_state.argtypes = [P, i64, P, i32, P, i32, P]
    L.ffm_learner_get_mt_state.argtypes = [P, i64, P, C.POINTER(i32), P, C.POINTER(i32), P]
    L.ffm_learner_get_counters.argtypes = [P, P, P]
    L.ffm_learner_set_epsilon.argtypes = [P, C.c_double]
    L.ffm_learner_set_v_default.argtypes = [P, C.c_double, P]
    L.ffm_learner_set_h_extra.argtypes = [P, C.c_int64, C.c_double, C.c_double, C.c_int32]
    L.ffm_learner_table_size.argtypes = [P, i32, C.POINTER(i64), P]
    L.ffm_learner_export_table.argtypes = [P, i32, P, P, i64, C.POINTER(i64), P]
    L.ffm_learner_import_table.argtypes = [P, i32, P, P, i64, P]
    L.ffm_learner_get_step_index.argtypes = [P, C.POINTER(C.c_uint32)]
    L.ffm_learner_set_step_index.argtypes = [P, C.c_uint32]
    L.ffm_learner_step_local.argtypes = [P, P]
    L.ffm_learner_step_apply.argtypes = [P, i32, P]
    L.ffm_learner_step_end.argtypes = [P, P]
    L.ffm_learner_delta_export.argtypes = [P, i32, P, P, i64, C.POINTER(i64), P]
    L.ffm_learner_delta_merge.argtypes = [P, i32, P, P, i64, P]
    L.ffm_learner_set_placement.argtypes = [P, P, i32, i32]
    L.ffm_learner_set_epsilon_schedule.argtypes = [P, C.c_double, C.c_double, C.c_double, C.c_double]
    L.ffm_learner_set_epsilon_phase.argtypes = [P, i32]
    L.ffm_learner_set_epsilon_stride.argtypes = [P, i64]
    L.ffm_learner_set_episode_caps.argtypes = [P, P, i64]
    L.ffm_learner_drain_episodes.argtypes = [P, P, i64, C.POINTER(i64), C.POINTER(i64), P]
    L.ffm_learner_set_trajectory_capture.argtypes = [P, P, P, i32, i32, i64, P]
    L.ffm_learner_delta_export_async.argtypes = [P, i32, P, P, i64, P, P]
    L.ffm_learner_delta_merge_async.argtypes = [P, i32, P, P, P, i64, P]
    L.ffm_learner_set_sync_period.argtypes = [P, i32]
    L.ffm_learner_apply_due.argtypes = [P, C.POINTER(i32)]
    L.ffm_learner_dense_buffers.argtypes = [P, i32, C.POINTER(P), C.POINTER(i64), C.POINTER(P), C.POINTER(i64)]
    L.ffm_learner_dense_adopt.argtypes = [P, i32, P, P]
    L.ffm_learner_tiled_buffers.argtypes = [P, C.POINTER(P), C.POINTER(i64), C.POINTER(P), C.POINTER(i64)]
    L.ffm_learner_step_tiled_local.argtypes = [P, P]
    L.ffm_learner_step_tiled_apply.argtypes = [P, P, P, i64, P]
    L.ffm_learner_drain_trajectory.argtypes = [P, P, P, i64, C.POINTER(i64), C.POINTER(i64), P]
    L.ffm_learner_set_tile_owners.argtypes = [P, i32, i32]
    L.ffm_learner_owner_buffers.argtypes = [P, C.POINTER(OwnerBuffers)]
    L.ffm_learner_step_owner_local.argtypes = [P, P]
    L.ffm_learner_set_owner_capacity.argtypes = [P, i64, i64, i64]
    L.ffm_learner_step_owner_v.argtypes = [P, P, P, i64, P]
    L.ffm_learner_set_owner_send_buffer.argtypes = [P, P]
    L.ffm_learner_set_owner_output_buffers.argtypes = [P, P, P, P, P, P, P]
    L.ffm_learner_step_owner_h.argtypes = [P, P, P, P, i64, P]
    L.ffm_learner_step_owner_end.argtypes = [P, P, P, P, i64, P, i64, P]
    L.ffm_learner_set_external_sync.argtypes = [P, i32]
    L.ffm_learner_flush_begin.argtypes = [P, C.POINTER(i32)]
    L.ffm_learner_flush_end.argtypes = [P, P]
    for name in EXPORTED:
        if name != "ffm_last_error":
            getattr(L, name).restype = C.c_int
    if L.ffm_abi_version() != ABI_VERSION:
        raise ImportError("libffm_amd.so ABI version mismatch; rebuild")
    _lib = L
    return L


def _check(rc: int):
    if rc == OK:
        return
    msg = _lib.ffm_last_error().decode(errors="replace")
    if rc == E_INVALID:
        raise ValueError(msg)
    if rc == E_UNSUPPORTED:
        raise NotImplementedError(msg)
    if rc == E_NOMEM:
        raise MemoryError(msg)
    raise RuntimeError(msg)


def _stream_handle(stream):
    if stream is None:
        return None
    if isinstance(stream, int):
        return stream
    return int(getattr(stream, "cuda_stream"))


def _device_mask(mask, n: int, device: int):
    """reset_envs' mask as n bytes on the device (a torch CUDA tensor is used in place)."""
    import torch
    dev = torch.device("cuda", device)
    m = mask if isinstance(mask, torch.Tensor) else torch.as_tensor(np.asarray(mask))
    if m.numel() != n:
        raise ValueError(f"mask must have n_envs = {n} entries, got {m.numel()}")
    m = m.reshape(-1).to(device=dev)
    return (m != 0).to(torch.uint8).contiguous() if m.dtype != torch.uint8 else m.contiguous()


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class _DevArray:
    """A device buffer of the library, exposed to torch.as_tensor (zero copy)."""

    def __init__(self, ptr: int, n: int, typestr: str):
        self.__cuda_array_interface__ = {"shape": (int(n),), "typestr": typestr, "data": (int(ptr), False),
                                         "version": 3, "strides": None}


DEFAULT_PARAMS = {"k_S": 3, "k_D": 1, "diffuse": 0.2, "decay": 0.2, "neighborhood": "moore"}


class Engine:
    """E environments of ``FloorFieldModel`` on one GPU.

    rng="philox": production mode, every draw keyed by (seed, step, env, agent).
    rng="mt": each env carries its own NumPy-legacy and CPython MT19937 state and
    consumes it exactly like the reference (bit-exact replay).
    """

    def __init__(self, map_array, sff, n_envs: int, n_agents: int, agent_capacity: int | None = None,
                 params: dict | None = None, rng: str = "philox", seed: int = 42,
                 auto_reset: bool = True, env_base: int = 0, device: int = 0,
                 envs_per_block: int = 0):
        L = load_library()
        p = {**DEFAULT_PARAMS, **(params or {})}
        self.params = p
        self.map = np.ascontiguousarray(map_array, dtype=np.uint8)
        if self.map.ndim != 2:
            raise ValueError("map must be 2-D")
        self.H, self.W = self.map.shape
        sff = np.asarray(sff)
        if sff.shape != self.map.shape:
            raise ValueError("sff shape must equal map shape")
        if sff.dtype == np.float32:
            self.sff = np.ascontiguousarray(sff)
            sdt = SFF_F32
        else:
            self.sff = np.ascontiguousarray(sff, dtype=np.float64)
            sdt = SFF_F64
        nbn = p.get("neighborhood", "moore")
        self.nb = 4 if nbn == "neumann" else 8
        self.n_envs = int(n_envs)
        self.n_agents = int(n_agents)
        self.A = int(agent_capacity if agent_capacity is not None else max(1, n_agents))
        self.rng = rng
        d = EngineDesc()
        d.abi_version = ABI_VERSION
        d.variant = VARIANT_CORE
        d.H, d.W = self.H, self.W
        d.map = self.map.ctypes.data
        d.sff = self.sff.ctypes.data
        d.sff_dtype = sdt
        d.neighborhood = self.nb
        d.k_S, d.k_D = float(p["k_S"]), float(p["k_D"])
        d.diffuse, d.decay = float(p["diffuse"]), float(p["decay"])
        d.n_envs = self.n_envs
        d.agent_capacity = self.A
        d.n_agents = self.n_agents
        d.rng_mode = {"philox": RNG_PHILOX, "mt": RNG_MT}[rng]
        d.auto_reset = int(bool(auto_reset))
        d.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        d.env_base = int(env_base)
        d.device = int(device)
        d.envs_per_block = int(envs_per_block)
        self.device = int(device)
        h = C.c_void_p()
        _check(L.ffm_engine_create(C.byref(d), C.byref(h)))
        self._h = h
        self._L = L

    # -- lifecycle ---------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None):
            self._L.ffm_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # -- the hot path ------------------------------------------------------
    def reset(self, stream=None):
        _check(self._L.ffm_engine_reset(self._h, _stream_handle(stream)))

    def reset_envs(self, mask, stream=None):
        """reset(env_mask): re-place only the envs with a nonzero mask entry (n_envs entries:
        a torch CUDA tensor on the engine's device is read in place, anything else is
        uploaded).  See ffm_engine_reset_envs."""
        m = _device_mask(mask, self.n_envs, self.device)
        _check(self._L.ffm_engine_reset_envs(self._h, C.c_void_p(m.data_ptr()), _stream_handle(stream)))
        self._mask_keep = m      # alive until the next call: the launch reads it asynchronously

    def step(self, n_steps: int = 1, stream=None):
        _check(self._L.ffm_engine_step(self._h, int(n_steps), _stream_handle(stream)))

    def set_fused_steps(self, k: int):
        """Steps per launch in step(n) (1 = one launch per step); see ffm_engine_set_fused_steps."""
        _check(self._L.ffm_engine_set_fused_steps(self._h, int(k)))

    def update_dff(self, stream=None):
        _check(self._L.ffm_engine_update_dff(self._h, _stream_handle(stream)))

    # -- episode I/O ---------------------------------------------------------
    def set_trajectory_capture(self, envs, period: int = 1, phases=None, capacity_rows: int | None = None,
                               stream=None):
        """Capture `positions` after every step of episode k of env envs[i] (local index)
        whenever (k + phases[i]) % period == 0 (k counted from the last reset, 0-based):
        the per-step log of model/ffm_core.py:119-133 / main.py:44-54, batched.
        drain_trajectories() returns it.  envs=[] turns capture off.  Default capacity:
        1,024 steps of every selected env between drains."""
        envs = np.ascontiguousarray(envs, np.int32).reshape(-1)
        ph = None if phases is None else np.ascontiguousarray(phases, np.int32).reshape(-1)
        if ph is not None and len(ph) != len(envs):
            raise ValueError("phases must have one entry per selected env")
        cap = int(capacity_rows) if capacity_rows else max(1, 1024 * len(envs))
        self._traj_cap = cap if len(envs) else 0
        _check(self._L.ffm_engine_set_trajectory_capture(
            self._h, _ptr(envs) if len(envs) else None, _ptr(ph) if ph is not None and len(ph) else None,
            len(envs), int(period), cap, _stream_handle(stream)))

    def drain_trajectories(self, stream=None) -> dict:
        """Rows captured since the last drain, grouped: {(global env, episode k): (steps [T],
        positions list of T int32 [n_t, 2] arrays)} in step order -- the positions_log of
        main.py:44-54 (its last entry the empty array of the step that emptied the room)."""
        cap = getattr(self, "_traj_cap", 0)
        if not cap:
            return {}
        meta = np.empty((cap, 4), np.int32)
        cells = np.empty((cap, self.A), np.uint16)
        n, dropped = C.c_int64(), C.c_int64()
        _check(self._L.ffm_engine_drain_trajectory(self._h, _ptr(meta), _ptr(cells), cap, C.byref(n),
                                                   C.byref(dropped), _stream_handle(stream)))
        if dropped.value:
            raise RuntimeError(f"trajectory buffer overflowed: {dropped.value} rows lost (drain more often)")
        meta, cells = meta[: n.value], cells[: n.value]
        order = np.lexsort((meta[:, 2], meta[:, 1], meta[:, 0]))
        out = {}
        for r in order.tolist():
            env, k, st, c = meta[r].tolist()
            cc = cells[r, :c].astype(np.int32)
            steps, pos = out.setdefault((env, k), ([], []))
            steps.append(st)
            pos.append(np.stack([cc // self.W, cc % self.W], axis=1))
        return out

    # -- state transfer -----------------------------------------------------
    def get_state(self, env0: int = 0, n: int | None = None, stream=None):
        n = self.n_envs - env0 if n is None else n
        pos = np.empty((n, self.A), np.uint16)
        cnt = np.empty(n, np.int32)
        dff = np.empty((n, self.H, self.W), np.float32)
        _check(self._L.ffm_engine_get_state(self._h, env0, n, _ptr(pos), _ptr(cnt), _ptr(dff),
                                            _stream_handle(stream)))
        return pos, cnt, dff

    def set_state(self, env0: int = 0, positions=None, counts=None, dff=None, stream=None):
        n = None
        arrs = []
        for a, dt in ((positions, np.uint16), (counts, np.int32), (dff, np.float32)):
            if a is None:
                arrs.append(None)
                continue
            a = np.ascontiguousarray(a, dtype=dt)
            n = a.shape[0] if n is None else n
            if a.shape[0] != n:
                raise ValueError("inconsistent env counts")
            arrs.append(a)
        if n is None:
            return
        if arrs[0] is not None and arrs[0].shape[1:] != (self.A,):
            raise ValueError(f"positions must be [n, {self.A}]")
        if arrs[2] is not None and arrs[2].reshape(n, -1).shape[1] != self.H * self.W:
            raise ValueError("dff must be [n, H, W]")
        _check(self._L.ffm_engine_set_state(self._h, env0, n, _ptr(arrs[0]), _ptr(arrs[1]),
                                            _ptr(arrs[2]), _stream_handle(stream)))

    def set_mt_state(self, env: int, np_key, np_pos: int, py_key, py_pos: int, stream=None):
        nk = np.ascontiguousarray(np_key, dtype=np.uint32)
        pk = np.ascontiguousarray(py_key, dtype=np.uint32)
        if nk.size != 624 or pk.size != 624:
            raise ValueError("MT19937 keys must have 624 words")
        _check(self._L.ffm_engine_set_mt_state(self._h, env, _ptr(nk), int(np_pos), _ptr(pk),
                                               int(py_pos), _stream_handle(stream)))

    def get_mt_state(self, env: int, stream=None):
        nk = np.empty(624, np.uint32)
        pk = np.empty(624, np.uint32)
        npos, ppos = C.c_int32(), C.c_int32()
        _check(self._L.ffm_engine_get_mt_state(self._h, env, _ptr(nk), C.byref(npos), _ptr(pk),
                                               C.byref(ppos), _stream_handle(stream)))
        return nk, int(npos.value), pk, int(ppos.value)

    # MT helpers bridging the interpreter's generators ------------------------
    def load_rng_from(self, env: int, np_rs: np.random.RandomState | None = None,
                      py_r: _pyrandom.Random | None = None):
        st = (np_rs if np_rs is not None else np.random.mtrand._rand).get_state(legacy=True)
        ps = (py_r if py_r is not None else _pyrandom._inst).getstate()
        self.set_mt_state(env, st[1], st[2], np.asarray(ps[1][:624], np.uint32), ps[1][624])

    def store_rng_to(self, env: int, np_rs: np.random.RandomState | None = None,
                     py_r: _pyrandom.Random | None = None):
        nk, npos, pk, ppos = self.get_mt_state(env)
        rs = np_rs if np_rs is not None else np.random.mtrand._rand
        st = rs.get_state(legacy=True)
        rs.set_state(("MT19937", nk, npos, st[3], st[4]))
        r = py_r if py_r is not None else _pyrandom._inst
        ps = r.getstate()
        r.setstate((ps[0], tuple(int(w) for w in pk) + (ppos,), ps[2]))

    # -- telemetry -------------------------------------------------------------
    def counters(self, stream=None) -> dict:
        c = np.zeros(4, np.uint64)
        _check(self._L.ffm_engine_get_counters(self._h, _ptr(c), _stream_handle(stream)))
        return {"agent_steps": int(c[0]), "exits": int(c[1]), "resets": int(c[2]), "steps": int(c[3])}

    def device_buffers(self) -> dict:
        b = DeviceBuffers()
        _check(self._L.ffm_engine_device_buffers(self._h, C.byref(b)))
        return {k: b.__getattribute__(k) for k, _ in DeviceBuffers._fields_}

    @property
    def step_index(self) -> int:
        t = C.c_uint32()
        _check(self._L.ffm_engine_get_step_index(self._h, C.byref(t)))
        return int(t.value)

    @step_index.setter
    def step_index(self, t: int):
        _check(self._L.ffm_engine_set_step_index(self._h, int(t) & 0xFFFFFFFF))


def np_expf_device(x_dev_ptr: int, y_dev_ptr: int, n: int, stream=None):
    L = load_library()
    _check(L.ffm_np_expf_device(x_dev_ptr, y_dev_ptr, n, _stream_handle(stream)))


# ---------------------------------------------------------------------------
# Learning variants: ffm_ac_core, ffm_unified, ffm_actor_only
# ---------------------------------------------------------------------------
# Class defaults of the reference, merged under the caller's params the way
# the reference merges them ({**defaults, **params}).
LEARN_DEFAULTS = {
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
    # model/ffm_trained_core.py:29-36 (inference: no learning parameters)
    "trained": {"k_D": 1, "k_A": 10, "diffuse": 0.2, "decay": 0.2, "neighborhood": "neumann", "block_size": 5},
}
_LEARN_VARIANTS = {"ac": VARIANT_AC, "unified": VARIANT_UNIFIED, "actor_only": VARIANT_ACTOR_ONLY,
                   "trained": VARIANT_TRAINED}


class Learner:
    """E environments of one learning model class plus its shared V / H tables.

    variant: "ac" (model/ffm_ac_core.py), "unified" (model/ffm_unified.py, with
    ``mode`` critic_only / actor_only / both), "actor_only"
    (model/ffm_actor_only.py) or "trained" (model/ffm_trained_core.py: import
    the trained H with ``import_table("H", ...)``; nothing is learned).  rng="mt" reproduces the reference bit for bit
    (per-env MT19937 streams, agents and table updates in the reference's
    order); rng="philox" is the batched production step.
    Table keys are packed u64 (ffm_amd/learn_keys.py).
    """

    def __init__(self, map_array, sff, variant: str, n_envs: int, n_agents: int,
                 agent_capacity: int | None = None, mode: str | None = None, params: dict | None = None,
                 rng: str = "philox", seed: int = 42, auto_reset: bool = True, max_steps: int = 0,
                 env_base: int = 0, device: int = 0, log2_v_capacity: int = 0, log2_h_capacity: int = 0):
        L = load_library()
        if variant not in _LEARN_VARIANTS:
            raise ValueError(f"variant must be one of {sorted(_LEARN_VARIANTS)}")
        p = {**LEARN_DEFAULTS[variant], **(params or {})}
        self.params, self.variant = p, variant
        self.mode = mode or ("actor_only" if variant == "actor_only" else "critic_only")
        if variant == "unified" and self.mode not in LEARN_MODES:
            raise ValueError(f"learning_mode must be one of {list(LEARN_MODES)}")
        self.map = np.ascontiguousarray(map_array, dtype=np.uint8)
        if self.map.ndim != 2:
            raise ValueError("map must be 2-D")
        self.H, self.W = self.map.shape
        sff = np.asarray(sff)
        if sff.shape != self.map.shape:
            raise ValueError("sff shape must equal map shape")
        if sff.dtype == np.float32:
            self.sff, sdt = np.ascontiguousarray(sff), SFF_F32
        else:
            self.sff, sdt = np.ascontiguousarray(sff, dtype=np.float64), SFF_F64
        self.n_envs, self.n_agents = int(n_envs), int(n_agents)
        self.A = int(agent_capacity if agent_capacity is not None else max(1, n_agents))
        self.rng = rng
        self.env_base, self.max_steps = int(env_base), int(max_steps)
        d = EngineDesc()
        d.abi_version = ABI_VERSION
        d.variant = _LEARN_VARIANTS[variant]
        d.H, d.W = self.H, self.W
        d.map, d.sff, d.sff_dtype = self.map.ctypes.data, self.sff.ctypes.data, sdt
        nbn = p.get("neighborhood", "neumann")
        if nbn not in ("neumann", "moore"):
            raise ValueError(f"neighborhood must be 'neumann' or 'moore', got {nbn!r}")
        d.neighborhood = 4 if nbn == "neumann" else 8
        # H rows: one value per move (the neighbours, then stay)
        self.n_actions = d.neighborhood + 1
        d.k_S, d.k_D = float(p.get("k_S", 0.0)), float(p["k_D"])
        d.diffuse, d.decay = float(p["diffuse"]), float(p["decay"])
        d.n_envs, d.agent_capacity, d.n_agents = self.n_envs, self.A, self.n_agents
        d.rng_mode = {"philox": RNG_PHILOX, "mt": RNG_MT}[rng]
        d.auto_reset = int(bool(auto_reset))
        d.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        d.env_base, d.device = int(env_base), int(device)
        self.device = int(device)
        ld = LearnDesc()
        ld.mode = LEARN_MODES.get(self.mode, 1) if variant == "unified" else (1 if variant == "actor_only" else 0)
        ld.k_A = float(p.get("k_A", 0.0))
        ld.alpha_v, ld.alpha_h = float(p.get("alpha_v", 0.0)), float(p.get("alpha_h", 0.0))
        ld.gamma = float(p.get("gamma", 0.0))
        ld.exit_reward, ld.step_penalty = float(p.get("exit_reward", 0.0)), float(p.get("step_penalty", 0.0))
        ld.collision_penalty = float(p.get("collision_penalty", 0.0))
        ld.epsilon = float(min(max(float(p.get("epsilon", 0.0)), 0.0), 1.0))
        ld.v_default = 0.0
        ld.block_size = int(p.get("block_size", 5))
        ld.max_steps = int(max_steps)
        ld.log2_v_capacity, ld.log2_h_capacity = int(log2_v_capacity), int(log2_h_capacity)
        h = C.c_void_p()
        _check(L.ffm_learner_create(C.byref(d), C.byref(ld), C.byref(h)))
        self._h, self._L = h, L

    def close(self):
        if getattr(self, "_h", None):
            self._L.ffm_learner_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # -- stepping ------------------------------------------------------------------
    def reset(self, stream=None):
        _check(self._L.ffm_learner_reset(self._h, _stream_handle(stream)))

    def reset_envs(self, mask, stream=None):
        """reset(env_mask) of the batched learner: the masked envs only (ffm_learner_reset_envs)."""
        m = _device_mask(mask, self.n_envs, self.device)
        _check(self._L.ffm_learner_reset_envs(self._h, C.c_void_p(m.data_ptr()), _stream_handle(stream)))
        self._mask_keep = m

    def step(self, n_steps: int = 1, stream=None):
        _check(self._L.ffm_learner_step(self._h, int(n_steps), _stream_handle(stream)))

    def set_epsilon(self, eps: float):
        _check(self._L.ffm_learner_set_epsilon(self._h, float(eps)))

    def set_h_extra(self, values):
        """ffm_trained_core: the values of trained H rows whose length is not the move count
        (model/ffm_trained_core.py:228-267: such a state scores as a missing row, but its
        values join the whole-table min / max of the normalisation)."""
        v = np.asarray(values, dtype=np.float64).ravel()
        if len(v) == 0:
            _check(self._L.ffm_learner_set_h_extra(self._h, 0, 0.0, 0.0, 0))
            return
        fin = np.isfinite(v)
        nf = int(not fin.all())
        mn, mx = (float(v[fin].min()), float(v[fin].max())) if fin.any() else (0.0, 0.0)
        _check(self._L.ffm_learner_set_h_extra(self._h, len(v), mn, mx, nf))

    def set_placement(self, cells=None, n_agents: int | None = None):
        """Placement candidates of later resets (cell indices x*W+y; None = every free
        cell) and the agents placed, min(N, len(cells)) like model/ffm_unified.py:150-171."""
        c = np.zeros(0, np.uint16) if cells is None else np.ascontiguousarray(cells, dtype=np.uint16)
        n = int(n_agents if n_agents is not None else self.n_agents)
        _check(self._L.ffm_learner_set_placement(self._h, _ptr(c) if len(c) else None, len(c), n))
        self.n_agents = n

    def set_radius_placement(self, exit_pos, radius: int, N: int):
        """The radius curriculum of run_unified_*_training.py: free cells within L1
        distance `radius` of `exit_pos` (row-major), min(N, their count) agents."""
        free = np.argwhere(self.map == 0)
        m = np.abs(free[:, 0] - exit_pos[0]) + np.abs(free[:, 1] - exit_pos[1]) <= radius
        cells = (free[m, 0] * self.W + free[m, 1]).astype(np.uint16)
        self.set_placement(cells if len(cells) else None, min(int(N), len(cells)))
        return len(cells)

    def set_epsilon_schedule(self, start: float, end: float, offset: float, span: float):
        """Per-env epsilon clip(start + (end - start) * (k + offset) / span) after k ended episodes."""
        _check(self._L.ffm_learner_set_epsilon_schedule(self._h, float(start), float(end), float(offset),
                                                          float(span)))

    def set_epsilon_phase(self, period: int, stride: int = 1):
        """Env g starts the epsilon schedule at its ((g % period) * stride)-th episode (0 = off)."""
        _check(self._L.ffm_learner_set_epsilon_phase(self._h, int(period)))
        _check(self._L.ffm_learner_set_epsilon_stride(self._h, int(stride)))

    def set_episode_caps(self, caps=None):
        """Env e ends at most caps[e] episodes after a reset, then stays empty (its quota of
        the driver's episode count); None removes the quotas."""
        if caps is None:
            _check(self._L.ffm_learner_set_episode_caps(self._h, None, 0))
            return
        c = np.ascontiguousarray(caps, np.int32).reshape(-1)
        if len(c) != self.n_envs:
            raise ValueError("episode caps: one entry per env")
        _check(self._L.ffm_learner_set_episode_caps(self._h, _ptr(c), len(c)))

    def drain_episodes(self, stream=None) -> np.ndarray:
        """Ended episodes since the last drain: int32 [n, 4] rows {global env, episode index,
        steps, emptied}, sorted by (env, episode)."""
        cap = max(16 * self.n_envs, 4096)
        buf = np.empty((cap, 4), np.int32)
        n, dropped = C.c_int64(), C.c_int64()
        _check(self._L.ffm_learner_drain_episodes(self._h, _ptr(buf), cap, C.byref(n), C.byref(dropped),
                                                  _stream_handle(stream)))
        if dropped.value:
            raise RuntimeError(f"episode log overflowed: {dropped.value} records lost (drain more often)")
        out = buf[: n.value]
        return out[np.lexsort((out[:, 1], out[:, 0]))]

    def set_trajectory_capture(self, envs, period: int = 100, phases=None, capacity_rows: int | None = None,
                               stream=None):
        """Capture the positions after every step of episode k of env envs[i] (local index)
        whenever (k + phases[i]) % period == 0 (k counted from the last reset, 0-based);
        drain_trajectories() returns them.  envs=[] turns capture off.  Default capacity:
        1,024 steps of every selected env between drains."""
        envs = np.ascontiguousarray(envs, np.int32).reshape(-1)
        ph = None if phases is None else np.ascontiguousarray(phases, np.int32).reshape(-1)
        if ph is not None and len(ph) != len(envs):
            raise ValueError("phases must have one entry per selected env")
        cap = int(capacity_rows) if capacity_rows else max(1, 1024 * len(envs))
        self._traj_cap = cap if len(envs) else 0
        _check(self._L.ffm_learner_set_trajectory_capture(
            self._h, _ptr(envs) if len(envs) else None, _ptr(ph) if ph is not None and len(ph) else None,
            len(envs), int(period), cap, _stream_handle(stream)))

    def drain_trajectories(self, stream=None) -> dict:
        """Rows captured since the last drain, grouped: {(global env, episode k): (steps [T],
        positions list of T int32 [n_t, 2] arrays)} in step order -- the reference's
        run(return_trajectory=True) list of `positions` copies (model/ffm_unified.py:902-931)."""
        cap = getattr(self, "_traj_cap", 0)
        if not cap:
            return {}
        meta = np.empty((cap, 4), np.int32)
        cells = np.empty((cap, self.A), np.uint16)
        n, dropped = C.c_int64(), C.c_int64()
        _check(self._L.ffm_learner_drain_trajectory(self._h, _ptr(meta), _ptr(cells), cap, C.byref(n),
                                                    C.byref(dropped), _stream_handle(stream)))
        if dropped.value:
            raise RuntimeError(f"trajectory buffer overflowed: {dropped.value} rows lost (drain more often)")
        meta, cells = meta[: n.value], cells[: n.value]
        order = np.lexsort((meta[:, 2], meta[:, 1], meta[:, 0]))
        out = {}
        for r in order.tolist():
            env, k, st, c = meta[r].tolist()
            cc = cells[r, :c].astype(np.int32)
            steps, pos = out.setdefault((env, k), ([], []))
            steps.append(st)
            pos.append(np.stack([cc // self.W, cc % self.W], axis=1))
        return out

    def set_v_default(self, v: float, stream=None):
        _check(self._L.ffm_learner_set_v_default(self._h, float(v), _stream_handle(stream)))

    # -- state -----------------------------------------------------------------------
    def get_state(self, env0: int = 0, n: int | None = None, stream=None):
        n = self.n_envs - env0 if n is None else n
        pos = np.empty((n, self.A), np.uint16)
        cnt = np.empty(n, np.int32)
        dff = np.empty((n, self.H, self.W), np.float32)
        _check(self._L.ffm_learner_get_state(self._h, env0, n, _ptr(pos), _ptr(cnt), _ptr(dff),
                                             _stream_handle(stream)))
        return pos, cnt, dff

    def set_state(self, env0: int = 0, positions=None, counts=None, dff=None, stream=None):
        n = None
        arrs = []
        for a, dt in ((positions, np.uint16), (counts, np.int32), (dff, np.float32)):
            if a is None:
                arrs.append(None)
                continue
            a = np.ascontiguousarray(a, dtype=dt)
            n = a.shape[0] if n is None else n
            if a.shape[0] != n:
                raise ValueError("inconsistent env counts")
            arrs.append(a)
        if n is None:
            return
        if arrs[0] is not None and arrs[0].shape[1:] != (self.A,):
            raise ValueError(f"positions must be [n, {self.A}]")
        if arrs[2] is not None and arrs[2].reshape(n, -1).shape[1] != self.H * self.W:
            raise ValueError("dff must be [n, H, W]")
        _check(self._L.ffm_learner_set_state(self._h, env0, n, _ptr(arrs[0]), _ptr(arrs[1]), _ptr(arrs[2]),
                                             _stream_handle(stream)))

    def episodes(self, env0: int = 0, n: int | None = None, stream=None):
        n = self.n_envs - env0 if n is None else n
        eps = np.empty(n, np.int32)
        st = np.empty(n, np.int32)
        _check(self._L.ffm_learner_get_episodes(self._h, env0, n, _ptr(eps), _ptr(st), _stream_handle(stream)))
        return eps, st

    def set_mt_state(self, env: int, np_key, np_pos: int, py_key, py_pos: int, stream=None):
        nk = np.ascontiguousarray(np_key, dtype=np.uint32)
        pk = np.ascontiguousarray(py_key, dtype=np.uint32)
        if nk.size != 624 or pk.size != 624:
            raise ValueError("MT19937 keys must have 624 words")
        _check(self._L.ffm_learner_set_mt_state(self._h, env, _ptr(nk), int(np_pos), _ptr(pk), int(py_pos),
                                                _stream_handle(stream)))

    def get_mt_state(self, env: int, stream=None):
        nk = np.empty(624, np.uint32)
        pk = np.empty(624, np.uint32)
        npos, ppos = C.c_int32(), C.c_int32()
        _check(self._L.ffm_learner_get_mt_state(self._h, env, _ptr(nk), C.byref(npos), _ptr(pk), C.byref(ppos),
                                                _stream_handle(stream)))
        return nk, int(npos.value), pk, int(ppos.value)

    def load_rng_from(self, env: int, np_rs: np.random.RandomState | None = None,
                      py_r: _pyrandom.Random | None = None):
        st = (np_rs if np_rs is not None else np.random.mtrand._rand).get_state(legacy=True)
        ps = (py_r if py_r is not None else _pyrandom._inst).getstate()
        self.set_mt_state(env, st[1], st[2], np.asarray(ps[1][:624], np.uint32), ps[1][624])

    def store_rng_to(self, env: int, np_rs: np.random.RandomState | None = None,
                     py_r: _pyrandom.Random | None = None):
        nk, npos, pk, ppos = self.get_mt_state(env)
        rs = np_rs if np_rs is not None else np.random.mtrand._rand
        st = rs.get_state(legacy=True)
        rs.set_state(("MT19937", nk, npos, st[3], st[4]))
        r = py_r if py_r is not None else _pyrandom._inst
        ps = r.getstate()
        r.setstate((ps[0], tuple(int(w) for w in pk) + (ppos,), ps[2]))

    # -- tables ------------------------------------------------------------------------
    def table_size(self, which: str = "V", stream=None) -> int:
        n = C.c_int64()
        _check(self._L.ffm_learner_table_size(self._h, TABLE_V if which == "V" else TABLE_H, C.byref(n),
                                              _stream_handle(stream)))
        return int(n.value)

    def export_table(self, which: str = "V", stream=None):
        """(keys u64 [n], values f64 [n] or [n, n_actions]) in insertion order."""
        w = TABLE_V if which == "V" else TABLE_H
        width = 1 if w == TABLE_V else self.n_actions
        cap = self.table_size(which, stream)
        keys = np.empty(max(cap, 1), np.uint64)
        vals = np.empty((max(cap, 1), width), np.float64)
        n = C.c_int64()
        _check(self._L.ffm_learner_export_table(self._h, w, _ptr(keys), _ptr(vals), cap, C.byref(n),
                                                _stream_handle(stream)))
        n = int(n.value)
        return keys[:n], (vals[:n, 0] if width == 1 else vals[:n])

    def import_table(self, which: str, keys, vals, stream=None):
        w = TABLE_V if which == "V" else TABLE_H
        width = 1 if w == TABLE_V else self.n_actions
        k = np.ascontiguousarray(keys, dtype=np.uint64)
        v = np.ascontiguousarray(vals, dtype=np.float64).reshape(len(k), width)
        _check(self._L.ffm_learner_import_table(self._h, w, _ptr(k), _ptr(v), len(k), _stream_handle(stream)))

    # -- the batched step in phases (multi-rank table exchange, ffm_amd/dist.py) -----------
    @property
    def actor(self) -> bool:
        return self.variant == "actor_only" or (self.variant == "unified" and self.mode != "critic_only")

    @property
    def post_update(self) -> bool:
        """ffm_unified actor_only: the actor's increments use the V of after the V apply."""
        return self.variant == "unified" and self.mode == "actor_only"

    def step_local(self, stream=None):
        _check(self._L.ffm_learner_step_local(self._h, _stream_handle(stream)))

    def step_apply(self, which: str, stream=None):
        _check(self._L.ffm_learner_step_apply(self._h, TABLE_V if which == "V" else TABLE_H, _stream_handle(stream)))

    def step_end(self, stream=None):
        _check(self._L.ffm_learner_step_end(self._h, _stream_handle(stream)))

    def delta_export(self, which: str, keys_ptr: int, acc_ptr: int, cap: int, stream=None) -> int:
        """Write this step's touched entries of table `which` to device buffers (u64 keys,
        i64 [width] increments) and return the record count.  A count above `cap`
        means the buffers were too small: nothing usable was written, call again
        with buffers of that size (the export does not change the table)."""
        n = C.c_int64()
        rc = self._L.ffm_learner_delta_export(self._h, TABLE_V if which == "V" else TABLE_H, keys_ptr, acc_ptr,
                                              int(cap), C.byref(n), _stream_handle(stream))
        if rc == E_INVALID and n.value > cap:
            return int(n.value)
        _check(rc)
        return int(n.value)

    def delta_merge(self, which: str, keys_ptr: int, acc_ptr: int, n: int, stream=None):
        _check(self._L.ffm_learner_delta_merge(self._h, TABLE_V if which == "V" else TABLE_H, keys_ptr, acc_ptr,
                                               int(n), _stream_handle(stream)))

    def delta_export_async(self, which: str, keys_ptr: int, acc_ptr: int, cap: int, count_ptr: int, stream=None):
        """delta_export without a host sync: the record count goes to the device int64 at
        count_ptr; a count above cap is reported at the next sync point."""
        _check(self._L.ffm_learner_delta_export_async(self._h, TABLE_V if which == "V" else TABLE_H, keys_ptr,
                                                      acc_ptr, int(cap), count_ptr, _stream_handle(stream)))

    def delta_merge_async(self, which: str, keys_ptr: int, acc_ptr: int, count_ptr: int, cap: int, stream=None):
        _check(self._L.ffm_learner_delta_merge_async(self._h, TABLE_V if which == "V" else TABLE_H, keys_ptr,
                                                     acc_ptr, count_ptr, int(cap), _stream_handle(stream)))

    def set_sync_period(self, k: int):
        """Apply the tables every k-th step (increments of k steps accumulate; default 1)."""
        _check(self._L.ffm_learner_set_sync_period(self._h, int(k)))

    def set_external_sync(self, on: bool = True):
        """Tables shared with other ranks (TableSync): exports are read-only and the pending
        increments are applied only collectively (flush_begin / flush_end)."""
        _check(self._L.ffm_learner_set_external_sync(self._h, int(bool(on))))

    def flush_begin(self) -> bool:
        """True: increments are pending and a flush phase is open (exchange, then flush_end)."""
        p = C.c_int32()
        _check(self._L.ffm_learner_flush_begin(self._h, C.byref(p)))
        return bool(p.value)

    def flush_end(self, stream=None):
        _check(self._L.ffm_learner_flush_end(self._h, _stream_handle(stream)))

    def apply_due(self) -> bool:
        d = C.c_int32()
        _check(self._L.ffm_learner_apply_due(self._h, C.byref(d)))
        return bool(d.value)

    @property
    def dense_tables(self) -> bool:
        """ffm_unified / ffm_trained_core rank-key tables are dense (slot = key)."""
        if not hasattr(self, "_dense"):
            a, p, na, npw = C.c_void_p(), C.c_void_p(), C.c_int64(), C.c_int64()
            self._dense = self._L.ffm_learner_dense_buffers(self._h, TABLE_V, C.byref(a), C.byref(na), C.byref(p),
                                                            C.byref(npw)) == OK
        return self._dense

    def dense_buffers(self, which: str):
        """(acc int64 [cap * width], presence int32 [cap / 32]) torch views of the device
        buffers of a dense table (zero copy)."""
        import torch
        a, p, na, npw = C.c_void_p(), C.c_void_p(), C.c_int64(), C.c_int64()
        _check(self._L.ffm_learner_dense_buffers(self._h, TABLE_V if which == "V" else TABLE_H, C.byref(a),
                                                 C.byref(na), C.byref(p), C.byref(npw)))
        dev = torch.device("cuda", self.device)
        return (torch.as_tensor(_DevArray(a.value, na.value, "<i8"), device=dev),
                torch.as_tensor(_DevArray(p.value, npw.value, "<i4"), device=dev))

    def dense_adopt(self, which: str, union_ptr: int, stream=None):
        _check(self._L.ffm_learner_dense_adopt(self._h, TABLE_V if which == "V" else TABLE_H, union_ptr,
                                               _stream_handle(stream)))

    # -- the tiled step across ranks -----------------------------------------
    @property
    def tiled(self) -> bool:
        """ffm_unified at block size 1 on a large map: the step sums per-agent records per
        tile of cells (ffm_learner_step_tiled_*)."""
        if not hasattr(self, "_tiled"):
            r, t, nr, nt = C.c_void_p(), C.c_void_p(), C.c_int64(), C.c_int64()
            self._tiled = self._L.ffm_learner_tiled_buffers(self._h, C.byref(r), C.byref(nr), C.byref(t),
                                                            C.byref(nt)) == OK
        return self._tiled

    def tiled_buffers(self):
        """(records uint8 [E * A * 16], tile offsets uint8 [E * (NT + 1) * 2]: the bytes of
        the uint16 offsets -- uint8 is carried by every collective backend, 16-bit integers
        by neither gloo nor RCCL) torch views of this learner's device buffers (zero copy),
        filled by step_tiled_local."""
        import torch
        r, t, nr, nt = C.c_void_p(), C.c_void_p(), C.c_int64(), C.c_int64()
        _check(self._L.ffm_learner_tiled_buffers(self._h, C.byref(r), C.byref(nr), C.byref(t), C.byref(nt)))
        dev = torch.device("cuda", self.device)
        return (torch.as_tensor(_DevArray(r.value, nr.value, "|u1"), device=dev),
                torch.as_tensor(_DevArray(t.value, 2 * nt.value, "|u1"), device=dev))

    def step_tiled_local(self, stream=None):
        _check(self._L.ffm_learner_step_tiled_local(self._h, _stream_handle(stream)))

    def step_tiled_apply(self, recs_ptr: int, tstart_ptr: int, n_envs_all: int, stream=None):
        _check(self._L.ffm_learner_step_tiled_apply(self._h, recs_ptr, tstart_ptr, int(n_envs_all),
                                                    _stream_handle(stream)))

    # -- the owner-sharded tiled step -----------------------------------------
    @property
    def tile_major(self) -> bool:
        """Tiled learners can reorder their records tile-major (the owner-sharded exchange)
        unless FFM_TILE_MAJOR=0; one device steps tile-major only with FFM_TILE_MAJOR=1."""
        return self.tiled and os.environ.get("FFM_TILE_MAJOR", "") != "0"

    def set_tile_owners(self, world: int, rank: int):
        """Deal the tiles of cells over `world` ranks; this learner owns rank `rank`'s."""
        _check(self._L.ffm_learner_set_tile_owners(self._h, int(world), int(rank)))

    def set_owner_capacity(self, records: int, v_out: int, h_out: int):
        """Fixed exchange sizes of the owner-sharded step: records per destination block, V
        values and H increments this rank's tiles may emit per step (a count past its capacity
        is an error at the next sync point)."""
        _check(self._L.ffm_learner_set_owner_capacity(self._h, int(records), int(v_out), int(h_out)))

    def owner_buffers(self) -> dict:
        """Torch views (zero copy) of the exchange buffers: byte views where a collective
        carries them (records, headers, outputs), int64 views for the device counts."""
        import torch
        b = OwnerBuffers()
        _check(self._L.ffm_learner_owner_buffers(self._h, C.byref(b)))
        dev = torch.device("cuda", self.device)

        def view(ptr, n, typestr):
            if not ptr or n <= 0:
                return torch.empty(0, dtype=torch.uint8, device=dev)
            return torch.as_tensor(_DevArray(ptr, n, typestr), device=dev)

        w, hs, rc = int(b.world), int(b.hdr_stride), int(b.send_rec_capacity)
        vc, hc = int(b.v_capacity), int(b.h_capacity)
        return {
            "world": w, "rank": int(b.rank), "hdr_stride": hs, "rec_capacity": rc, "v_capacity": vc,
            "h_capacity": hc, "tsum_count": int(b.tsum_count),
            "send_recs": view(b.send_recs, 16 * w * rc, "|u1"),
            "send_hdr": view(b.send_hdr, 4 * w * hs, "|u1").view(w, 4 * hs),
            "counts": view(b.counts, w, "<i8"),
            "v_slot": view(b.v_slot, 4 * vc, "|u1"), "v_val": view(b.v_val, 8 * vc, "|u1"),
            "h_key": view(b.h_key, 4 * hc, "|u1"), "h_q": view(b.h_q, 8 * hc, "|u1"),
            "out_counts": view(b.out_counts, 2, "<i8"),
            "tsum": view(b.tsum, 40 * hs, "|u1"),
        }

    def step_owner_local(self, stream=None):
        _check(self._L.ffm_learner_step_owner_local(self._h, _stream_handle(stream)))

    def set_owner_send_buffer(self, ptr: int | None):
        """Pack the owner exchange's send blocks into this device buffer (world * rec_capacity
        records) instead of the learner's own; None restores it."""
        _check(self._L.ffm_learner_set_owner_send_buffer(self._h, ptr))

    def set_owner_output_buffers(self, v=None, h=None):
        """v / h: (slot or key, value or increment, count) device pointers the owner passes
        write instead of the learner's own buffers; None restores them."""
        v = v or (None, None, None)
        h = h or (None, None, None)
        _check(self._L.ffm_learner_set_owner_output_buffers(self._h, *v, *h))

    def step_owner_v(self, recs_ptr: int, hdrs_ptr: int, src_stride: int = 0, stream=None):
        """recs: the received record blocks (source r's block at r * src_stride records; 0 =
        rec_capacity), hdrs: the received header rows ([world][hdr_stride] u32), device pointers."""
        _check(self._L.ffm_learner_step_owner_v(self._h, recs_ptr, hdrs_ptr, int(src_stride), _stream_handle(stream)))

    def step_owner_h(self, v_slot_ptr: int, v_val_ptr: int, v_counts_ptr: int, v_stride: int, stream=None):
        """The gathered V outputs ([world][v_stride]) and their counts (device int64 [world])."""
        _check(self._L.ffm_learner_step_owner_h(self._h, v_slot_ptr, v_val_ptr, v_counts_ptr, int(v_stride),
                                                _stream_handle(stream)))

    def step_owner_end(self, h_key_ptr: int, h_q_ptr: int, h_counts_ptr: int, h_stride: int, tsum_ptr: int,
                       tsum_stride: int, stream=None):
        _check(self._L.ffm_learner_step_owner_end(self._h, h_key_ptr, h_q_ptr, h_counts_ptr, int(h_stride), tsum_ptr,
                                                  int(tsum_stride), _stream_handle(stream)))

    # -- telemetry -----------------------------------------------------------------------
    def counters(self, stream=None) -> dict:
        c = np.zeros(4, np.uint64)
        _check(self._L.ffm_learner_get_counters(self._h, _ptr(c), _stream_handle(stream)))
        return {"agent_steps": int(c[0]), "exits": int(c[1]), "resets": int(c[2]), "steps": int(c[3])}

    @property
    def step_index(self) -> int:
        t = C.c_uint32()
        _check(self._L.ffm_learner_get_step_index(self._h, C.byref(t)))
        return int(t.value)

    @step_index.setter
    def step_index(self, t: int):
        _check(self._L.ffm_learner_set_step_index(self._h, int(t) & 0xFFFFFFFF))
