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


def load_critic(L: Learner, path: str):
    """Import a V table pickled by write_outputs (a dict keyed like the reference's V)."""
    with open(path, "rb") as f:
        table = pickle.load(f)   # written by this tool (write_outputs), never a reference file
    conv = K.from_rank_tuple if L.variant in ("unified", "trained") else K.from_cells_bytes
    keys = np.array([conv(k) for k in table], np.uint64)
    vals = np.array(list(table.values()), np.float64)
    L.import_table("V", keys, vals)


def _key_obj(variant, k):
    return K.to_rank_tuple(k) if variant in ("unified", "trained") else K.to_cells_bytes(k)


def trajectory_selection(E: int, per_env: int, every: int):
    """Envs and capture phases for the trajectories of every `every`-th episode.

    Within a configuration the reported episodes are numbered env-major, episode
    n = e * per_env + k + 1 for env e's k-th episode (k < per_env); the reference keeps
    the trajectory of every episode with n % every == 0 (run_actor_only_training.py:199-218),
    i.e. (k + phase_e) % every == 0 with phase_e = (e * per_env + 1) % every."""
    envs, phases = [], []
    for e in range(E):
        ph = (e * per_env + 1) % every
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
                   eps_phase: bool = True) -> dict:
    """Run every (radius, N) configuration; return per-configuration statistics and
    (when `out_dir` is given) write the reference's output files there, with the
    trajectory of every `trajectory_every`-th episode under out_dir/trajectories.

    Epsilon (actor modes) decays linearly over the P = episodes_per_config episodes of a
    configuration (run_unified_actor_training.py:253-259: episode j of P explores with
    start + (end - start) * j / P).  With fewer envs than P, env e runs ceil(P / E)
    episodes and decays over its own; with E >= P (one episode per env) and eps_phase,
    env g plays episode 1 + g % P of the schedule, so the E episodes cover it."""
    L = learner
    E = L.n_envs
    per_env = max(1, math.ceil(episodes_per_config / E))
    phased = bool(eps_phase) and per_env == 1 and E >= episodes_per_config > 1
    chunk = max(1, min(int(log_every), 16))      # the episode log holds 16 steps of episode ends
    rows, configs = [], []
    episode_num = 0
    n_traj = 0
    t_start = time.time()
    tsel, tph = (trajectory_selection(E, per_env, trajectory_every) if trajectory_every > 0
                 else (np.zeros(0, np.int32), None))
    if len(tsel):
        L.set_trajectory_capture(tsel, period=trajectory_every, phases=tph, capacity_rows=len(tsel) * chunk * 2)
    for radius in radius_list:
        avail = available_cells(L.map, exit_pos, radius)
        for N in n_list:
            if N > avail:                                # run_unified_critic_training.py:190-197
                continue
            L.set_radius_placement(exit_pos, radius, N)
            if eps_start is not None and L.actor:
                # local linear decay per configuration (run_unified_actor_training.py:253-259)
                if phased:
                    L.set_epsilon_schedule(eps_start, eps_end, 1, episodes_per_config)
                    L.set_epsilon_phase(episodes_per_config)
                else:
                    L.set_epsilon_schedule(eps_start, eps_end, 1, per_env)
            v0 = L.table_size("V")
            L.reset()
            done, trajs = [], {}
            while True:
                L.step(chunk)
                d = L.drain_episodes()
                if len(d):
                    done.append(d)
                if len(tsel):
                    for key, val in L.drain_trajectories().items():
                        st, ps = trajs.setdefault(key, ([], []))
                        st.extend(val[0])
                        ps.extend(val[1])
                if L.episodes()[0].min() >= per_env:
                    break
            ended = np.concatenate(done)
            ended = ended[ended[:, 1] < per_env]
            ended = ended[np.lexsort((ended[:, 1], ended[:, 0]))]   # env-major: episode e * per_env + k + 1
            v1 = L.table_size("V")
            h1 = L.table_size("H") if L.actor else 0
            base = episode_num
            for idx, (env, k, steps, emptied) in enumerate(ended.tolist()):
                episode_num += 1
                j, span = ((k + 1 + env % episodes_per_config, episodes_per_config) if phased   # env: global id
                           else (k + 1, per_env))
                eps = (min(max(eps_start + (eps_end - eps_start) * (j / span), 0.0), 1.0)
                       if eps_start is not None and L.actor else 0.0)
                rows.append([episode_num, len(configs) + 1, radius, N, steps, v1, h1, f"{eps:.6f}"])
                tr = trajs.get((env, k))
                if tr is not None and out_dir and (idx + 1) % trajectory_every == 0:
                    assert len(tr[0]) == steps and tr[0] == list(range(1, steps + 1)), "trajectory rows"
                    save_trajectory(os.path.join(out_dir, "trajectories"), N, idx + 1, base + idx + 1, tr[1],
                                    steps)
                    n_traj += 1
            mean = float(ended[:, 2].mean())
            configs.append({"radius": radius, "N": N, "episodes": len(ended), "mean_steps": mean,
                            "std_steps": float(ended[:, 2].std()), "emptied": int(ended[:, 3].sum()),
                            "v_before": v0, "v_after": v1})
            if verbose:
                print(f"radius={radius:2d}, N={N:3d}: mean steps={mean:7.2f} over {len(ended)} episodes, "
                      f"V {v0} -> {v1}", flush=True)
    if len(tsel):
        L.set_trajectory_capture([])
    result = {"configs": configs, "rows": rows, "seconds": time.time() - t_start, "trajectories": n_traj}
    if out_dir:
        write_outputs(L, result, out_dir, exit_pos, radius_list, n_list, episodes_per_config)
    return result


def write_outputs(L: Learner, result: dict, out_dir: str, exit_pos, radius_list, n_list, episodes_per_config):
    """steps_per_episode.csv (run_unified_actor_training.py:407-431), summary.txt, V / H
    tables pickled as the reference's get_v_table / get_h_table dicts."""
    os.makedirs(out_dir, exist_ok=True)
    with open(os.path.join(out_dir, "steps_per_episode.csv"), "w", newline="", encoding="utf-8") as f:
        w = csv.writer(f)
        w.writerow(["episode_num", "config_idx", "radius", "N", "steps", "v_table_size", "h_table_size",
                    "epsilon"])
        w.writerows(result["rows"])
    vk, vv = L.export_table("V")
    with open(os.path.join(out_dir, "V_table.pkl"), "wb") as f:
        pickle.dump({_key_obj(L.variant, k): float(v) for k, v in zip(vk.tolist(), vv.tolist())}, f)
    if L.actor:
        hk, hv = L.export_table("H")
        with open(os.path.join(out_dir, "H_table.pkl"), "wb") as f:
            pickle.dump({_key_obj(L.variant, k): [float(x) for x in r] for k, r in zip(hk.tolist(), hv.tolist())},
                        f)
    with open(os.path.join(out_dir, "summary.txt"), "w", encoding="utf-8") as f:
        f.write("=" * 80 + "\n")
        f.write(f"batched curriculum ({L.variant}{'/' + L.mode if L.variant == 'unified' else ''}), "
                f"{L.n_envs} envs, seed-keyed Philox streams\n")
        f.write("=" * 80 + "\n")
        f.write(f"exit: {tuple(exit_pos)}\nradius list: {list(radius_list)}\nN list: {list(n_list)}\n")
        f.write(f"episodes per configuration: {episodes_per_config}\nparams: {L.params}\n")
        f.write(f"final V states: {L.table_size('V')}\n")
        f.write(f"seconds: {result['seconds']:.1f}\n\nper configuration:\n" + "-" * 80 + "\n")
        for c in result["configs"]:
            f.write(f"radius={c['radius']:2d}, N={c['N']:3d}: mean steps={c['mean_steps']:7.2f}, "
                    f"V states {c['v_before']:6d} -> {c['v_after']:6d} (+{c['v_after'] - c['v_before']:5d})\n")


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--variant", default="unified", choices=["unified", "actor_only", "ac"])
    ap.add_argument("--mode", default="critic_only", choices=["critic_only", "actor_only", "both"])
    ap.add_argument("--size", type=int, default=12)
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--radius", default="3,5,7,9,11,13,15")
    ap.add_argument("--n", default="1,10,20,30,40,50,60,70,80,90")
    ap.add_argument("--episodes", type=int, default=1000, help="episodes per configuration")
    ap.add_argument("--max-steps", type=int, default=300)
    ap.add_argument("--eps", default="0.2,0.01", help="epsilon start,end (actor modes)")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--out", default=None)
    ap.add_argument("--critic", default=None,
                    help="pretrained V table (a V_table.pkl this tool wrote; the reference's actor drivers "
                         "load their critic run's pickle, run_unified_actor_training.py PRETRAINED_CRITIC)")
    ap.add_argument("--trajectory-every", type=int, default=None,
                    help="save every n-th episode's trajectory (default 100 for actor modes, as "
                         "run_actor_only_training.py; 0 = none)")
    ap.add_argument("--no-eps-phase", action="store_true",
                    help="with envs >= episodes: every env at the schedule's first episode (no spread)")
    a = ap.parse_args()
    m = make_room(a.size, a.size)
    # run_unified_*_training.py MODEL_PARAMS
    params = {"k_S": 10, "k_D": 1, "k_A": 10, "alpha_v": 0.01, "alpha_h": 0.1, "gamma": 0.99,
              "exit_reward": 100.0, "step_penalty": -1.0, "collision_penalty": -1.0, "neighborhood": "neumann",
              "block_size": 1}
    n_list = [int(x) for x in a.n.split(",")]
    L = Learner(m, l1_sff(m), a.variant, n_envs=a.envs, n_agents=max(n_list), mode=a.mode, params=params,
                seed=a.seed, max_steps=a.max_steps)
    if a.critic:
        load_critic(L, a.critic)
    es, ee = (float(x) for x in a.eps.split(","))
    every = a.trajectory_every if a.trajectory_every is not None else (100 if L.actor else 0)
    run_curriculum(L, (0, a.size // 2), [int(x) for x in a.radius.split(",")], n_list, a.episodes, es, ee, a.out,
                   trajectory_every=every, eps_phase=not a.no_eps_phase)


if __name__ == "__main__":
    main()
