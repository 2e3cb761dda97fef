"""Batched curriculum training on the GPU learner, the batched counterpart of the
reference's drivers (run_unified_critic_training.py, run_unified_actor_training.py,
run_actor_only_training.py of SoraKurihara/FFM).

The reference runs one episode at a time: for every (radius, N) configuration
(radius-limited placement around the exit, model/ffm_unified.py:150-171; N above
the cells within the radius is skipped, run_unified_critic_training.py:190-197)
it runs EPISODES_PER_CONFIG episodes of at most MAX_STEPS steps, with a linear
epsilon schedule in the actor drivers, and writes ``steps_per_episode.csv``,
``summary.txt`` and the V / H tables.  Here E envs run those episodes in
parallel on one device (the batched semantics of DESIGN.md section 9); an env
that ends an episode starts the next one at once, and the configuration is done
once every env has ended ceil(episodes_per_config / E) episodes; exactly those
episodes (the first ones of every env) are reported, so the sample is not biased
towards short episodes, which end first.  The per-env epsilon follows
the reference's local schedule ``start + (end - start) * episode / episodes``
with the episode index counted per env (``Learner.set_epsilon_schedule``).

    python -m ffm_amd.train --variant unified --mode critic_only --out runs/critic
    python -m ffm_amd.train --variant actor_only --n 32 --envs 65536 --out runs/actor   # config 4
    python -m torch.distributed.run --nproc-per-node 8 -m ffm_amd.train --variant actor_only --n 32 --envs 65536

The per-N drivers (``--variant actor_only``: run_actor_only_training.py; ``--variant ac``:
run_critic_training.py) shard over ranks under torch.distributed.run: every rank steps
its own global env ids and ffm_amd.dist.TableSync exchanges the table increments.
"""
from __future__ import annotations

import argparse
import csv
import math
import os
import pickle
import time

import numpy as np

from . import learn_keys as K
from .data import l1_sff, make_room
from .engine import Learner


def available_cells(map_array, exit_pos, radius) -> int:
    """run_unified_critic_training.py count_available_cells: free cells within L1 `radius`."""
    free = np.argwhere(np.asarray(map_array) == 0)
    return int((np.abs(free[:, 0] - exit_pos[0]) + np.abs(free[:, 1] - exit_pos[1]) <= radius).sum())


def _load_table(path: str) -> dict:
    """A table pickle write_outputs / run_per_n wrote: a dict of bytes / tuple keys and float
    values, read with every global refused (the file runs no code)."""
    with open(path, "rb") as f:
        table = K.KeyUnpickler(f, numpy_scalars=False).load()
    if not isinstance(table, dict):
        raise ValueError(f"{path}: not a table (dict)")
    return table


def load_critic(L: Learner, path: str):
    """Import a V table pickled by write_outputs (a dict keyed like the reference's V)."""
    table = _load_table(path)
    conv = K.from_rank_tuple if L.variant in ("unified", "trained") else K.from_cells_bytes
    keys = np.array([conv(k) for k in table], np.uint64)
    vals = np.array(list(table.values()), np.float64)
    L.import_table("V", keys, vals)


def _key_obj(variant, k):
    return K.to_rank_tuple(k) if variant in ("unified", "trained") else K.to_cells_bytes(k)


def trajectory_selection(E: int, per_env: int, every: int, env_base: int = 0):
    """Envs and capture phases for the trajectories of every `every`-th episode.

    Within a configuration the reported episodes are numbered env-major over the global
    envs, episode n = g * per_env + k + 1 for global env g's k-th episode (k < per_env); the
    reference keeps the trajectory of every episode with n % every == 0
    (run_actor_only_training.py:199-218), i.e. (k + phase_g) % every == 0 with
    phase_g = (g * per_env + 1) % every.  Returns local env indices (g = env_base + e)."""
    envs, phases = [], []
    for e in range(E):
        ph = ((env_base + e) * per_env + 1) % every
        if (-ph) % every < per_env:
            envs.append(e)
            phases.append(ph)
    return np.asarray(envs, np.int32), np.asarray(phases, np.int32)


def save_trajectory(out_dir: str, N: int, episode: int, total: int, positions: list, steps: int):
    """One trajectory file as run_actor_only_training.py:206-218 writes it."""
    os.makedirs(out_dir, exist_ok=True)
    traj = np.empty(len(positions), dtype=object)      # np.array(trajectory, dtype=object)
    for i, p in enumerate(positions):
        traj[i] = p
    np.savez_compressed(os.path.join(out_dir, f"trajectory_N{N}_ep{episode:05d}_total{total:05d}.npz"),
                        positions=traj, episode=episode, N=N, total_episode=total, steps=steps)


def run_curriculum(learner: Learner, exit_pos, radius_list, n_list, episodes_per_config: int,
                   eps_start: float | None = None, eps_end: float | None = None, out_dir: str | None = None,
                   log_every: int = 16, verbose: bool = True, trajectory_every: int = 0,
                   eps_phase: bool = True, group: "_Group | None" = None, global_envs: int | None = None) -> dict:
    """Run every (radius, N) configuration; return per-configuration statistics and
    (when `out_dir` is given) write the reference's output files there, with the
    trajectory of every `trajectory_every`-th episode under out_dir/trajectories.

    A radius of None places over every free cell (the full room: the C5 workload,
    256x256 with 8,192 agents).  Sharded (`group` holds a TableSync): every rank steps its
    own global envs [env_base, env_base + E) of G = `global_envs`, the tables are shared,
    the episode rows of all ranks are merged and rank 0 writes the outputs -- the files a
    single process stepping all G envs writes.

    Epsilon (actor modes) decays linearly over the P = episodes_per_config episodes of a
    configuration (run_unified_actor_training.py:253-259: episode j of P explores with
    start + (end - start) * j / P).  With fewer envs than P, env g runs ceil(P / G) episodes
    and decays over its own; with G >= P (one episode per env) and eps_phase, env g plays
    episode 1 + g % P of the schedule, so the G episodes cover it.  Every env runs exactly
    ceil(P / G) episodes per configuration (ffm_learner_set_episode_caps): no episode trains
    the tables without being reported."""
    L = learner
    g = group or _Group()
    E = L.n_envs
    G = int(global_envs or E * g.world)
    env_base = L.env_base
    per_env = max(1, math.ceil(episodes_per_config / G))
    phased = bool(eps_phase) and per_env == 1 and G >= episodes_per_config > 1
    chunk = max(1, min(int(log_every), 16))      # the episode log holds 16 steps of episode ends
    rows, configs = [], []
    episode_num = 0
    n_traj = 0
    prev_n = None
    t_start = time.time()
    tsel, tph = (trajectory_selection(E, per_env, trajectory_every, env_base) if trajectory_every > 0
                 else (np.zeros(0, np.int32), None))
    if len(tsel):
        L.set_trajectory_capture(tsel, period=trajectory_every, phases=tph, capacity_rows=len(tsel) * chunk * 2)
    L.set_episode_caps(np.full(E, per_env, np.int32))
    if out_dir and g.rank == 0:
        os.makedirs(out_dir, exist_ok=True)
    for radius in radius_list:
        avail = available_cells(L.map, exit_pos, radius) if radius is not None else int((L.map == 0).sum())
        for N in n_list:
            if N > avail:                                # run_unified_critic_training.py:190-197
                continue
            if g.sync is not None:                       # the exchange sizes follow the configuration
                g.sync.reconfigure(N, prev_n)
            prev_n = N
            if radius is None:
                L.set_placement(None, n_agents=N)        # every free cell: the full-room reset
            else:
                L.set_radius_placement(exit_pos, radius, N)
            if eps_start is not None and L.actor:
                # local linear decay per configuration (run_unified_actor_training.py:253-259)
                if phased:
                    L.set_epsilon_schedule(eps_start, eps_end, 1, episodes_per_config)
                    L.set_epsilon_phase(episodes_per_config)
                else:
                    L.set_epsilon_schedule(eps_start, eps_end, 1, per_env)
            v0 = g.table_size(L, "V")
            L.reset()
            done, trajs = [], {}
            while True:
                g.step(L, chunk)
                d = L.drain_episodes()
                if len(d):
                    done.append(d)
                if len(tsel):
                    for key, val in L.drain_trajectories().items():
                        st, ps = trajs.setdefault(key, ([], []))
                        st.extend(val[0])
                        ps.extend(val[1])
                if g.min_int(int(L.episodes()[0].min())) >= per_env:
                    break
            ended = np.concatenate(done) if done else np.zeros((0, 4), np.int32)
            ended = ended[ended[:, 1] < per_env]
            v1 = g.table_size(L, "V")
            h1 = g.table_size(L, "H") if L.actor else 0
            base = episode_num
            for env, k, steps, emptied in ended.tolist():
                idx = env * per_env + k                  # env-major position among all G * per_env episodes
                tr = trajs.get((env, k))
                if tr is not None and out_dir and (idx + 1) % trajectory_every == 0:
                    assert len(tr[0]) == steps and tr[0] == list(range(1, steps + 1)), "trajectory rows"
                    save_trajectory(os.path.join(out_dir, "trajectories"), N, idx + 1, base + idx + 1, tr[1],
                                    steps)
                    n_traj += 1
            ended = np.concatenate(g.gather(ended))
            ended = ended[np.lexsort((ended[:, 1], ended[:, 0]))]   # env-major: episode g * per_env + k + 1
            for env, k, steps, emptied in ended.tolist():
                episode_num += 1
                j, span = ((k + 1 + env % episodes_per_config, episodes_per_config) if phased   # env: global id
                           else (k + 1, per_env))
                eps = (min(max(eps_start + (eps_end - eps_start) * (j / span), 0.0), 1.0)
                       if eps_start is not None and L.actor else 0.0)
                rows.append([episode_num, len(configs) + 1, "full" if radius is None else radius, N, steps, v1, h1,
                             f"{eps:.6f}"])
            mean = float(ended[:, 2].mean())
            configs.append({"radius": radius, "N": N, "episodes": len(ended), "mean_steps": mean,
                            "std_steps": float(ended[:, 2].std()), "emptied": int(ended[:, 3].sum()),
                            "v_before": v0, "v_after": v1})
            if verbose and g.rank == 0:
                print(f"radius={'full' if radius is None else radius}, N={N:3d}: mean steps={mean:7.2f} over "
                      f"{len(ended)} episodes, V {v0} -> {v1}", flush=True)
    if len(tsel):
        L.set_trajectory_capture([])
    L.set_episode_caps(None)
    n_traj = int(sum(g.gather(n_traj)))
    result = {"configs": configs, "rows": rows, "seconds": time.time() - t_start, "trajectories": n_traj,
              "global_envs": G}
    if out_dir:
        g.flush()
        if g.rank == 0:
            tables = {w: _pickle_table(L, w) for w in (("V", "H") if L.actor else ("V",))}
            write_outputs(L, result, out_dir, exit_pos, radius_list, n_list, episodes_per_config, tables)
    return result


def write_outputs(L: Learner, result: dict, out_dir: str, exit_pos, radius_list, n_list, episodes_per_config,
                  tables: dict | None = None):
    """steps_per_episode.csv (run_unified_actor_training.py:407-431), summary.txt, V / H
    tables pickled as the reference's get_v_table / get_h_table dicts (`tables`: those dicts,
    exported beforehand; default: exported here)."""
    tables = tables or {w: _pickle_table(L, w) for w in (("V", "H") if L.actor else ("V",))}
    os.makedirs(out_dir, exist_ok=True)
    with open(os.path.join(out_dir, "steps_per_episode.csv"), "w", newline="", encoding="utf-8") as f:
        w = csv.writer(f)
        w.writerow(["episode_num", "config_idx", "radius", "N", "steps", "v_table_size", "h_table_size",
                    "epsilon"])
        w.writerows(result["rows"])
    with open(os.path.join(out_dir, "V_table.pkl"), "wb") as f:
        pickle.dump(tables["V"], f)
    if L.actor:
        with open(os.path.join(out_dir, "H_table.pkl"), "wb") as f:
            pickle.dump(tables["H"], f)
    with open(os.path.join(out_dir, "summary.txt"), "w", encoding="utf-8") as f:
        f.write("=" * 80 + "\n")
        f.write(f"batched curriculum ({L.variant}{'/' + L.mode if L.variant == 'unified' else ''}), "
                f"{result.get('global_envs', L.n_envs)} envs, seed-keyed Philox streams\n")
        f.write("=" * 80 + "\n")
        f.write(f"exit: {tuple(exit_pos)}\nradius list: {list(radius_list)}\nN list: {list(n_list)}\n")
        f.write(f"episodes per configuration: {episodes_per_config}\nparams: {L.params}\n")
        f.write(f"final V states: {len(tables['V'])}\n")
        f.write(f"seconds: {result['seconds']:.1f}\n\nper configuration:\n" + "-" * 80 + "\n")
        for c in result["configs"]:
            rad = "full" if c["radius"] is None else f"{c['radius']:2d}"
            f.write(f"radius={rad}, N={c['N']:3d}: mean steps={c['mean_steps']:7.2f}, "
                    f"V states {c['v_before']:6d} -> {c['v_after']:6d} (+{c['v_after'] - c['v_before']:5d})\n")


# ---------------------------------------------------------------------------
# The per-N drivers: run_actor_only_training.py (ffm_actor_only, config 4) and
# run_critic_training.py (ffm_ac_core)
# ---------------------------------------------------------------------------
# Each reference driver's module constants (MODEL_PARAMS, N list, episodes, MAX_STEPS, epsilon).
DRIVERS = {
    "actor_only": {     # run_actor_only_training.py:27-58
        "script": "run_actor_only_training.py",
        "params": {"k_D": 1, "k_A": 10, "alpha_v": 0.1, "alpha_h": 0.1, "gamma": 0.95, "exit_reward": 100.0,
                   "step_penalty": 0.0, "collision_penalty": -1.0, "neighborhood": "neumann", "epsilon": 0.2},
        "n_list": [1, 1],                   # N_FIXED + range(N_START, N_END + 1, N_STEP) = [1] + [1]
        "episodes": 10000, "max_steps": 1000, "eps": (0.2, 0.01), "trajectory_every": 100,
    },
    "ac": {             # run_critic_training.py:19-43
        "script": "run_critic_training.py",
        "params": {"k_S": 10, "k_D": 1, "alpha_v": 0.01, "gamma": 0.99, "exit_reward": 100.0, "step_penalty": -1.0,
                   "collision_penalty": -1.0, "neighborhood": "neumann", "block_size": 5},
        "n_list": [1] + list(range(10, 101, 10)),
        "episodes": 1000, "max_steps": 500, "eps": None, "trajectory_every": 0,
    },
    "unified": {        # run_unified_{critic,actor}_training.py MODEL_PARAMS
        "script": "run_unified_actor_training.py",
        "params": {"k_S": 10, "k_D": 1, "k_A": 10, "alpha_v": 0.01, "alpha_h": 0.1, "gamma": 0.99,
                   "exit_reward": 100.0, "step_penalty": -1.0, "collision_penalty": -1.0, "neighborhood": "neumann",
                   "block_size": 1},
        "n_list": [1] + list(range(10, 91, 10)),
        "episodes": 1000, "max_steps": 300, "eps": (0.2, 0.01), "trajectory_every": 100,
    },
}


class _Group:
    """The ranks of a sharded run (torch.distributed), or one process."""

    def __init__(self, sync=None):
        self.sync = sync
        if sync is not None:
            import torch.distributed as dist
            self.dist, self.rank, self.world = dist, dist.get_rank(), dist.get_world_size()
        else:
            self.dist, self.rank, self.world = None, 0, 1

    def step(self, L, n):
        if self.sync is not None:
            self.sync.step(n)
        else:
            L.step(n)

    def min_int(self, x: int) -> int:
        if self.dist is None:
            return int(x)
        import torch
        t = torch.tensor([int(x)], dtype=torch.int64, device=self.sync.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN)
        return int(t.item())

    def gather(self, obj) -> list:
        if self.dist is None:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def flush(self):
        if self.sync is not None:
            self.sync.flush()

    def table_size(self, L, which: str) -> int:
        """The table's size on every rank.  The owner exchange keeps H's key set exact every
        step and V's lazily, so only V's presence is merged first (collective: every rank
        calls it together).  The other exchanges insert every rank's keys at each sync step;
        with a sync period K > 1 the size between sync steps is that of the last one -- a
        flush here would apply the pending increments early and change the apply schedule
        (and so the learned values) against a single device with the same K."""
        if self.sync is not None and which == "V" and getattr(self.sync, "owner", False):
            self.sync.sync_presence()
        return L.table_size(which)


def _pickle_table(L: Learner, which: str) -> dict:
    """get_v_table() / get_h_table() of the reference's model (key objects, insertion order)."""
    keys, vals = L.export_table(which)
    if which == "V":
        return {_key_obj(L.variant, k): float(v) for k, v in zip(keys.tolist(), vals.tolist())}
    return {_key_obj(L.variant, k): [float(x) for x in r] for k, r in zip(keys.tolist(), vals.tolist())}


def run_per_n(learner: Learner, n_list, episodes_per_n: int, eps=None, out_dir: str | None = None,
              trajectory_every: int = 0, group: _Group | None = None, log_every: int = 16, verbose: bool = True,
              params: dict | None = None, global_envs: int | None = None, inert_v: dict | None = None) -> dict:
    """The reference's per-N drivers (run_actor_only_training.py:165-300, run_critic_training.py:
    136-209), batched: for every N of n_list the E envs (of every rank) run
    `episodes_per_n` full-room episodes in parallel (placement over every free cell,
    model/ffm_actor_only.py:557-563), the tables shared by all of them.

    Episodes are numbered env-major over the global envs: env g's k-th episode of pattern
    i is pattern episode g * per_env + k + 1 (per_env = ceil(P / G) for G global envs) and
    run episode i * P + that.  Env g runs exactly the min(per_env, P - g * per_env) episodes
    numbered <= P (ffm_learner_set_episode_caps; the envs past their quota stay empty until
    the pattern ends), so the tables learn from exactly the P episodes of a pattern the
    reference's driver runs, every one of them reported.  With `eps`, the
    explore rate follows the drivers' one linear schedule over all episodes of the run
    (run_actor_only_training.py:190-196: start + (end - start) * (j - 1) / (total - 1) for
    run episode j).  Trajectories of pattern episodes that are multiples of
    `trajectory_every` (:199-218).  Writes the driver's files (per-N H snapshots, the final
    tables, training_results.pkl, summary.txt) on rank 0."""
    L = learner
    g = group or _Group()
    E = L.n_envs
    G = int(global_envs or E * g.world)
    env_base = L.env_base
    P = int(episodes_per_n)
    per_env = max(1, math.ceil(P / G))
    total = len(n_list) * P
    chunk = max(1, min(int(log_every), 16))
    actor = L.actor
    t_start = time.time()
    all_results, episode_results = [], []
    inert_v = dict(inert_v or {})      # ffm_actor_only's pretrained critic: counted, never read (its module doc)
    v_initial = len(inert_v)
    n_traj = 0
    if out_dir and g.rank == 0:
        os.makedirs(out_dir, exist_ok=True)
    # trajectories: pattern episode n = g * per_env + k + 1 with n % every == 0, n <= P
    tsel, tph = np.zeros(0, np.int32), None
    if trajectory_every > 0:
        envs, phases = [], []
        for e in range(E):
            ph = ((env_base + e) * per_env + 1) % trajectory_every
            if (-ph) % trajectory_every < per_env:
                envs.append(e)
                phases.append(ph)
        tsel, tph = np.asarray(envs, np.int32), np.asarray(phases, np.int32)
        if len(tsel):
            L.set_trajectory_capture(tsel, period=trajectory_every, phases=tph, capacity_rows=len(tsel) * chunk * 2)
    gids = env_base + np.arange(E, dtype=np.int64)
    caps = np.clip(P - gids * per_env, 0, per_env).astype(np.int32)   # this rank's envs' episode quotas
    L.set_episode_caps(caps)
    prev_n = None
    for pi, N in enumerate(n_list):
        if g.sync is not None:
            g.sync.reconfigure(N, prev_n)                  # the touched records grow with N
        prev_n = N
        L.set_placement(None, n_agents=N)                  # every free cell: the full-room reset
        base = pi * P                                      # run episodes before this pattern
        if eps is not None and actor:
            es, ee = eps
            if total > 1:
                L.set_epsilon_schedule(es, ee, base, total - 1)
                L.set_epsilon_phase(G, per_env)            # + g * per_env: env-major numbering
            else:
                L.set_epsilon_schedule(es, ee, 0, 0)
                L.set_epsilon(es)
        L.reset()
        done, trajs, sizes = [], {}, []
        while True:
            g.step(L, chunk)
            d = L.drain_episodes()
            vs = g.table_size(L, "V") + v_initial
            hs = g.table_size(L, "H") if actor else 0
            if len(d):
                done.append(np.concatenate([d, np.full((len(d), 1), len(sizes), np.int64)], axis=1))
            sizes.append((vs, hs))
            if len(tsel):
                for key, val in L.drain_trajectories().items():
                    st, ps = trajs.setdefault(key, ([], []))
                    st.extend(val[0])
                    ps.extend(val[1])
            if g.min_int(int((L.episodes()[0] - caps).min())) >= 0:
                break
        ended = np.concatenate(done) if done else np.zeros((0, 5), np.int64)
        ended = ended[ended[:, 1] < per_env]
        n_pat = ended[:, 0] * per_env + ended[:, 1] + 1       # pattern episode (global env g = column 0)
        keep = n_pat <= P
        ended, n_pat = ended[keep], n_pat[keep]
        rows = []
        for (genv, k, steps, emptied, ci), n in zip(ended.tolist(), n_pat.tolist()):
            j = base + n
            vs, hs = sizes[ci]
            e_j = 0.0
            if eps is not None and actor:
                prog = (j - 1) / (total - 1) if total > 1 else 0.0
                e_j = float(np.clip(eps[0] + (eps[1] - eps[0]) * prog, 0.0, 1.0))
            rows.append({"episode_num": j, "N": N, "steps": int(steps), "emptied": int(emptied),
                         "v_initial_size": v_initial, "v_current_size": vs, "v_new_states": vs - v_initial,
                         "h_states": hs, "h_total_actions": hs * L.n_actions, "epsilon": e_j, "v_table_size": vs})
            tr = trajs.get((genv, k))
            if tr is not None and out_dir and n % trajectory_every == 0:
                assert len(tr[0]) == steps and tr[0] == list(range(1, steps + 1)), "trajectory rows"
                save_trajectory(os.path.join(out_dir, "trajectories"), N, n, j, tr[1], steps)
                n_traj += 1
        rows = sorted(sum(g.gather(rows), []), key=lambda r: r["episode_num"])
        pattern = {"N": N, "episodes": [r["episode_num"] - base for r in rows],
                   "v_initial_size": [r["v_initial_size"] for r in rows],
                   "v_current_size": [r["v_current_size"] for r in rows],
                   "v_new_states": [r["v_new_states"] for r in rows],
                   "h_table_sizes": [(r["h_states"], r["h_total_actions"]) for r in rows],
                   "v_table_sizes": [r["v_table_size"] for r in rows],
                   "avg_steps": [r["steps"] for r in rows], "epsilons": [r["epsilon"] for r in rows]}
        all_results.append(pattern)
        episode_results.extend(rows)
        g.flush()
        if actor:
            h_n = _pickle_table(L, "H")
            if out_dir and g.rank == 0:                     # run_actor_only_training.py:293-300
                with open(os.path.join(out_dir, f"H_actor_N{N}_total{P}ep.pkl"), "wb") as f:
                    pickle.dump(h_n, f)
        vsz, hsz = g.table_size(L, "V"), (g.table_size(L, "H") if actor else 0)    # collective: every rank
        if verbose and g.rank == 0:
            print(f"N={N:3d}: mean steps={np.mean(pattern['avg_steps']):7.2f} over {len(rows)} episodes, "
                  f"V {vsz}, H {hsz}", flush=True)
    g.flush()
    L.set_episode_caps(None)
    result = {"n_list": list(n_list), "episodes_per_n": P, "model_params": dict(params or {}),
              "results_by_n": all_results, "all_episodes": episode_results, "total_time": time.time() - t_start,
              "trajectories": n_traj}
    if len(tsel):
        L.set_trajectory_capture([])
    v_table = {**inert_v, **_pickle_table(L, "V")}
    h_table = _pickle_table(L, "H") if actor else {}
    result["final_v_table_size"] = result["final_v_current_size"] = len(v_table)
    if actor:
        result.update(final_v_initial_size=v_initial, final_v_new_states=len(v_table) - v_initial,
                      final_h_states=len(h_table), final_h_total_actions=len(h_table) * L.n_actions,
                      epsilon_start=eps[0] if eps else None, epsilon_end=eps[1] if eps else None)
    if out_dir and g.rank == 0:
        _write_per_n_outputs(out_dir, L, result, v_table, h_table, total)
    return result


def _write_per_n_outputs(out_dir, L, result, v_table, h_table, total):
    """The final tables, training_results.pkl and summary.txt of the driver
    (run_actor_only_training.py:317-443, run_critic_training.py:216-309)."""
    actor = L.actor
    vname = f"V_updated_total{total}ep.pkl" if actor else f"V_integrated_total{total}ep.pkl"
    with open(os.path.join(out_dir, vname), "wb") as f:
        pickle.dump(v_table, f)
    if actor:
        with open(os.path.join(out_dir, f"H_actor_total{total}ep.pkl"), "wb") as f:
            pickle.dump(h_table, f)
    with open(os.path.join(out_dir, "training_results.pkl"), "wb") as f:
        pickle.dump(result, f)
    vals = list(v_table.values())
    with open(os.path.join(out_dir, "summary.txt"), "w", encoding="utf-8") as f:
        f.write("=" * 80 + "\n")
        f.write(f"batched {L.variant} training, {L.n_envs} envs per rank, seed-keyed Philox streams\n")
        f.write("=" * 80 + "\n")
        f.write(f"total time: {result['total_time']:.1f} s\n")
        f.write(f"final V states: {len(v_table)}\n")
        if vals:
            f.write(f"  V range: [{min(vals):.2f}, {max(vals):.2f}]\n  V mean: {np.mean(vals):.2f}\n")
        if actor:
            f.write(f"  actor H states: {len(h_table)} (actions: {len(h_table) * L.n_actions})\n")
            hv = [x for r in h_table.values() for x in r]
            if hv:
                f.write(f"  H logit range: [{min(hv):.2f}, {max(hv):.2f}]\n  H mean logit: {np.mean(hv):.2f}\n")
            if result.get("epsilon_start") is not None:
                f.write(f"  epsilon schedule: start={result['epsilon_start']:.3f}, end={result['epsilon_end']:.3f}\n")
        f.write(f"\nN list: {result['n_list']}\ntotal episodes: {total}\n"
                f"episodes per N: {result['episodes_per_n']}\nmax steps: {L.max_steps}\n")
        f.write("\nmodel parameters:\n")
        for k, v in result["model_params"].items():
            f.write(f"  {k}: {v}\n")
        f.write("\nper N:\n" + "-" * 80 + "\n")
        for r in result["results_by_n"]:
            v0, v1 = r["v_current_size"][0], r["v_current_size"][-1]
            line = (f"N={r['N']:3d}: mean steps={np.mean(r['avg_steps']):6.2f}, V states {v0:5d}->{v1:5d} "
                    f"(+{v1 - v0:4d})")
            if actor:
                line += f", H states {r['h_table_sizes'][-1][0]:5d} (actions: {r['h_table_sizes'][-1][1]})"
            f.write(line + "\n")


def driver_settings(variant: str, a=None) -> dict:
    """The settings a run of `variant` uses: the reference driver's constants, overridden by
    the command line where given (a: parsed arguments)."""
    d = {k: (list(v) if isinstance(v, list) else v) for k, v in DRIVERS[variant].items()}
    d["params"] = dict(d["params"])
    if a is not None:
        if a.max_steps is not None:
            d["max_steps"] = a.max_steps
        if a.episodes is not None:
            d["episodes"] = a.episodes
        if a.n is not None:
            d["n_list"] = [int(x) for x in a.n.split(",")]
        if a.eps is not None:
            d["eps"] = tuple(float(x) for x in a.eps.split(","))
        if a.trajectory_every is not None:
            d["trajectory_every"] = a.trajectory_every
    return d


def _init_dist():
    """torch.distributed.run sets WORLD_SIZE / RANK / LOCAL_RANK: one rank per GPU."""
    if int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        return None
    import torch
    import torch.distributed as dist
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("FFM_DIST_BACKEND", "nccl")
    dev = local if backend == "nccl" else int(os.environ.get("FFM_DEVICE", str(local)))
    torch.cuda.set_device(dev)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    else:
        dist.init_process_group(backend)
    return dev


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--variant", default="unified", choices=["unified", "actor_only", "ac"],
                    help="unified: the radius curriculum (run_unified_*_training.py); actor_only: "
                         "run_actor_only_training.py; ac: run_critic_training.py")
    ap.add_argument("--mode", default="critic_only", choices=["critic_only", "actor_only", "both"])
    ap.add_argument("--size", type=int, default=12)
    ap.add_argument("--map", default=None, help="map .npy (default: the synthetic --size room)")
    ap.add_argument("--sff", default=None, help="SFF .npy (default: the L1 distance field of the map)")
    ap.add_argument("--envs", type=int, default=4096, help="envs per rank")
    ap.add_argument("--radius", default="3,5,7,9,11,13,15",
                    help="radius list of the curriculum, or 'full' for full-room placement over every free cell "
                         "(the C5 workload: --size 256 --n 8192 --mode actor_only)")
    ap.add_argument("--n", default=None, help="N list (default: the driver's)")
    ap.add_argument("--episodes", type=int, default=None, help="episodes per configuration / per N")
    ap.add_argument("--max-steps", type=int, default=None)
    ap.add_argument("--eps", default=None, help="epsilon start,end (actor modes)")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--out", default=None)
    ap.add_argument("--critic", default=None,
                    help="pretrained V table (a V_table.pkl this tool wrote; the reference's actor drivers "
                         "load their critic run's pickle, run_unified_actor_training.py PRETRAINED_CRITIC)")
    ap.add_argument("--trajectory-every", type=int, default=None,
                    help="save every n-th episode's trajectory (default: the driver's, 100 for actor modes)")
    ap.add_argument("--no-eps-phase", action="store_true",
                    help="with envs >= episodes: every env at the schedule's first episode (no spread)")
    a = ap.parse_args(argv)
    d = driver_settings(a.variant, a)
    if a.map:
        m = np.load(a.map, allow_pickle=False).astype(np.uint8)
    else:
        m = make_room(a.size, a.size)
    s = np.load(a.sff, allow_pickle=False) if a.sff else l1_sff(m)
    dev = _init_dist()
    rank = 0
    if dev is not None:
        import torch.distributed as dist
        rank = dist.get_rank()
    n_list = d["n_list"]
    L = Learner(m, s, a.variant, n_envs=a.envs, n_agents=max(n_list), mode=a.mode if a.variant == "unified" else None,
                params=d["params"], seed=a.seed, max_steps=d["max_steps"], env_base=rank * a.envs,
                device=dev or 0)
    inert = None
    if a.critic and a.variant == "actor_only":
        # model/ffm_actor_only.py:55-66 re-keys the pretrained critic by tuples of ints, which never
        # equal the step's pickled-bytes keys: the entries only count (the drop-in class does the same)
        table = _load_table(a.critic)
        inert = {tuple(tuple(int(x) for x in sub) for sub in K.loads_key(k)): v for k, v in table.items()}
    elif a.critic:
        load_critic(L, a.critic)
    group = _Group()
    if dev is not None:
        from .dist import TableSync
        # ffm_unified's tables: the owner-sharded tiled exchange on large maps at block size 1
        # (C5), the dense all-reduce otherwise; the 13-cell tables: record all-gathers
        group = _Group(TableSync(L, device="cuda", capacity=None))
    if a.variant == "unified":
        es, ee = d["eps"]
        radius = [None] if a.radius == "full" else [int(x) for x in a.radius.split(",")]
        run_curriculum(L, (0, m.shape[1] // 2), radius, n_list, d["episodes"], es, ee, a.out,
                       trajectory_every=d["trajectory_every"] if L.actor else 0, eps_phase=not a.no_eps_phase,
                       group=group, global_envs=a.envs * group.world)
        if dev is not None:
            import torch.distributed as dist
            dist.destroy_process_group()
        return
    run_per_n(L, n_list, d["episodes"], d["eps"], a.out, d["trajectory_every"] if L.actor else 0, group,
              params=d["params"], inert_v=inert)
    if dev is not None:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
