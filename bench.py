#!/usr/bin/env python3
"""Headline benchmark: agent-steps/s of the batched ffm_core step on MI355X.

Workload (BASELINE.json configs[1]): 12x12 room (create_12x12_map_and_sff.py
recipe), 32 agents per env, 65,536 envs per GPU, default_config.yaml params
(k_S 3, k_D 1, diffuse 0.2, decay 0.2, neumann), Philox RNG seeded 42,
on-device auto-reset.  One bench "step" = one FloorFieldModel.step() of every
env = one launch of the fused HIP kernel over inputs resident in HBM.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4|5]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

--config picks a BASELINE.json workload: 2 (default, the headline line),
3 (64x64 room, 512 agents, 8,192 envs), 4 (ffm_actor_only learning step,
12x12, 32 agents, 65,536 envs per GPU, run_actor_only_training.py params) or
5 (ffm_unified actor_only learning step, 256x256, 8,192 agents, 512 envs per
GPU, run_unified_actor_training.py params).  Configs 4 and 5 step the
learner (ffm_learner_*): its V / H tables are shared by all envs of a GPU.

Multi-GPU: envs are sharded by global id (weak scaling, 65,536 per GPU); the
only collective is the final reduction of counters and times (RCCL).

Rank 0 prints ONE JSON line.  `roofline.achieved` = algorithmic bytes per
launch (2*(2A + 4*H*W + 4) per env) / mean per-launch kernel
time measured with HIP events on the launch stream; `traffic` comes from the
committed rocprofv3 PMC summary (profiles/) when present; `cpu_baseline` times
the CPU restatement (oracle/, Philox mode, OpenMP) on a bounded sample and
checks the sample's first envs bit-exactly against a fresh GPU run.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0     # MI355X HBM3E spec (MI355X_MICROARCH.md)
METRIC = "agent-steps/sec (whole node), 12×12 grid × 64k envs, 1/2/4/8 GPU"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--config", type=int, default=2, choices=(2, 3, 4, 5))
    ap.add_argument("--steps", type=int, default=None,
                    help="default 500 (config 2), 1500 (config 3: one episode), 300 (config 4), "
                         "300 (config 5: one whole max_steps episode per window)")
    ap.add_argument("--warmup", type=int, default=None, help="default 50 (config 2), 20 (config 3), 30 (config 4), 5 (config 5)")
    ap.add_argument("--burn-in", type=int, default=None,
                    help="untimed steps after reset before the warmup, so the timed envs are desynchronised "
                         "(steady state) instead of all starting their first episode together; default 1000 "
                         "(config 2), 300 (config 5: one whole episode, so the timed episodes start on "
                         "populated tables), else 0")
    ap.add_argument("--envs", type=int, default=None, help="envs per GPU")
    ap.add_argument("--global-envs", type=int, default=None,
                    help="configs 2/3: envs of the WHOLE job, split over the ranks (strong scaling: the "
                         "metric's '64k envs' read as a global count; 'scaling' becomes 'strong'); "
                         "default: --envs per GPU (weak scaling)")
    ap.add_argument("--size", type=int, default=None)
    ap.add_argument("--agents", type=int, default=None)
    ap.add_argument("--neighborhood", default="neumann")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--envs-per-block", type=int, default=0)
    ap.add_argument("--cpu-envs", type=int, default=4096)
    ap.add_argument("--cpu-steps", type=int, default=0, help="0 = size the sample to ~15 s")
    ap.add_argument("--cpu-budget", type=float, default=60.0,
                    help="configs 2/3: seconds the CPU baseline may take to replay ALL envs of the timed engine "
                         "through every step it ran (and check them bit-exactly); beyond it a bounded sample")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0 = this process's CPU share (OMP_NUM_THREADS, else its affinity set)")
    ap.add_argument("--repeats", type=int, default=5,
                    help="timed regions of K steps each, back to back; value = their median (BASELINE.md 3)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--multi-step", type=int, default=50,
                    help="config 2: also time step(K) with this many steps fused per launch "
                         "(ffm_engine_set_fused_steps; a secondary field, 0 = skip)")
    ap.add_argument("--log2-table", type=int, default=0, help="learner V/H hash capacity (0 = engine default)")
    ap.add_argument("--sync-period", type=int, default=1,
                    help="learner configs: apply / exchange the tables every K steps (1 = the reference's per-step)")
    ap.add_argument("--traffic-json", default=None,
                    help="PMC traffic summary (default: profiles/traffic_<H>x<W>_A<A>_E<E>.json)")
    a = ap.parse_args()
    # config 3: an episode takes 1,491 +- 31 steps (oracle, 64 envs), so its envs stay in
    # phase; every timed window spans one episode and averages a whole evacuation
    size, agents, envs, steps, warmup = {2: (12, 32, 65536, 500, 50), 3: (64, 512, 8192, 1500, 20),
                                         4: (12, 32, 65536, 300, 30), 5: (256, 8192, 512, 300, 5)}[a.config]
    a.size = a.size or size
    a.agents = a.agents or agents
    a.envs = a.envs or envs
    a.steps = a.steps if a.steps is not None else steps
    a.warmup = a.warmup if a.warmup is not None else warmup
    a.burn_in = a.burn_in if a.burn_in is not None else {2: 1000, 5: 300}.get(a.config, 0)
    return a


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # FFM_BENCH_REHEARSE=1 (diagnostic): every rank on cuda:0 over gloo, to rehearse
        # the multi-rank path on a one-GPU box; the real runs use RCCL, one GPU per rank.
        if os.environ.get("FFM_BENCH_REHEARSE") == "1":
            torch.cuda.set_device(0)
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)

    if args.config in (4, 5):
        return bench_learner(args, world, rank, torch, dist)

    from ffm_amd.data import make_room, l1_sff
    from ffm_amd.engine import Engine

    H = W = args.size
    A = args.agents
    E = args.envs
    strong = args.global_envs is not None
    if strong:   # strong scaling: the job's envs split over the ranks (global ids stay contiguous)
        if args.global_envs % world:
            raise SystemExit("--global-envs must divide by the number of ranks")
        E = args.global_envs // world
    m = make_room(H, W)
    s = l1_sff(m)
    params = {"k_S": 3, "k_D": 1, "diffuse": 0.2, "decay": 0.2, "neighborhood": args.neighborhood}
    eng = Engine(m, s, n_envs=E, n_agents=A, params=params, rng="philox", seed=args.seed,
                 auto_reset=True, env_base=rank * E, device=torch.cuda.current_device(),
                 envs_per_block=args.envs_per_block)
    stream = torch.cuda.current_stream()
    eng.reset(stream)
    # burn-in: every env starts its first episode at the same step; after ~10 episodes
    # the episode phases are spread out and each step sees the steady-state population
    eng.step(args.burn_in + args.warmup, stream)
    torch.cuda.synchronize()

    # Timed regions: K back-to-back step launches on the stream, nothing in between.
    reps = timed_repeats(args, world, dist, torch, lambda: eng.step(args.steps, stream),
                         lambda: eng.counters(stream))
    elapsed, agent_steps = reps["elapsed"], reps["agent_steps"]

    # Kernel time for the roofline: HIP events on the launch stream bracketing
    # nk back-to-back launches (a separate pass, so events do not perturb
    # `value`); per-launch event pairs would add their own gaps to each launch.
    # nk = the window length, so the pass averages the same phases as a timed window
    # (config 3: one episode, its in-phase reset burst included).
    nk = min(args.steps, 2000)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    eng.step(nk, stream)
    ev1.record(stream)
    torch.cuda.synchronize()
    kern_ms = [ev0.elapsed_time(ev1) / nk]
    # the engine's state after every single-step launch it ran (the CPU baseline replays
    # all envs through the same steps and compares them bit for bit)
    single_steps = args.burn_in + args.warmup + reps["summary"]["n"] * args.steps + nk
    snap = eng.get_state() if rank == 0 and world == 1 and not args.no_cpu else None

    # Achievable HBM bandwidth on this box: a device-to-device copy of the same
    # number of bytes one launch moves (read + write), for context beside `peak`.
    copy_gbs = copy_bandwidth(torch, stream, E * (2 * A + 4 * H * W + 4))

    # Secondary line: the same steps with K fused per launch (state on chip between
    # the K steps of an env pair; bit-identical results, tests/test_gpu_parity.py).
    multi = None
    if args.multi_step > 1 and args.config == 2:
        eng.set_fused_steps(args.multi_step)
        eng.step(args.multi_step, stream)
        torch.cuda.synchronize()
        mr = timed_repeats(args, world, dist, torch, lambda: eng.step(args.steps, stream),
                           lambda: eng.counters(stream))
        eng.set_fused_steps(1)
        multi = {"fused_steps": args.multi_step, "value": mr["agent_steps"] / mr["elapsed"],
                 "unit": "agent-steps/s", "ms_per_step": mr["elapsed"] / args.steps * 1e3,
                 "env_steps_per_s": E * world * args.steps / mr["elapsed"],
                 "repeats": mr["summary"],
                 "note": "ffm_engine_step(K) with K steps per launch (core_multi_kernel where the shape "
                         "allows it, else one launch per step); the headline value is one launch per step"}

    if rank == 0:
        bytes_per_env_step = 2 * (2 * A + 4 * H * W + 4)
        mean_kernel_s = float(np.mean(kern_ms)) / 1e3
        achieved = E * bytes_per_env_step / mean_kernel_s / 1e9
        traffic = traffic_src = None
        tpath = args.traffic_json or os.path.join(ROOT, "profiles", f"traffic_{H}x{W}_A{A}_E{E}.json")
        neumann = args.neighborhood == "neumann"      # the committed profiles are the Neumann configs'
        if os.path.exists(tpath) and (neumann or args.traffic_json):
            with open(tpath) as f:
                tj = json.load(f)
            if tj.get("config") == f"{H}x{W}_A{A}_E{E}":
                traffic = tj.get("hbm_bytes_per_launch")
                traffic_src = profile_source(tpath, tj)
        # the step kernel's VALU issue fraction (its real bound at 12x12) from a committed
        # PMC summary (tools/pmc.sh + tools/valu_json.py)
        valu = None
        vpath = os.path.join(ROOT, "profiles", f"valu_{H}x{W}_A{A}_E{E}.json")
        if os.path.exists(vpath) and neumann:
            with open(vpath) as f:
                vj = json.load(f)
            if vj.get("config") == f"{H}x{W}_A{A}_E{E}":
                valu = vj
        out = {
            "metric": METRIC,
            "value": agent_steps / elapsed,
            "unit": "agent-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {
                "workload": (f"ffm_core step, {H}x{W} room, {A} agents/env, {E} envs/GPU"
                             + (f" ({E * world} envs for the whole job, split over {world} GPUs)" if strong else "")
                             + ", "
                             f"{args.neighborhood}, Philox seed {args.seed}, on-device auto-reset, "
                             + (f"steady state (envs desynchronised by a {args.burn_in}-step untimed burn-in "
                                f"after reset)" if args.burn_in else
                                "all envs start their first episode in phase (no burn-in)"
                                + (f"; {args.steps}-step timed windows, about one episode (1,491 +- 31 steps) "
                                   f"each, so every window averages a whole evacuation"
                                   if H == 64 and args.steps >= 1400 else ""))),
                "burn_in_steps": args.burn_in,
                "map": f"{H}x{W}", "agents_per_env": A, "envs_per_gpu": E,
                "global_envs": E * world, "parallelism": f"env-sharded x{world}",
            },
            "env_steps_per_s": E * world * args.steps / elapsed,
            "mean_live_agents_per_env_step": agent_steps / (E * world * args.steps),
            "repeats": reps["summary"],
            "kernel_ms_mean": float(np.mean(kern_ms)),
            "kernel_ms_median": float(np.median(kern_ms)),
            "roofline": {
                "bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": achieved / PEAK_HBM_GBS, "traffic": traffic,
                "traffic_source": traffic_src,
                "bytes_per_launch_algorithmic": E * bytes_per_env_step,
                # BASELINE.md 3's form: env-steps/s of the timed windows (launch gaps included) x B
                "frac_env_rate": E * world * args.steps / elapsed * bytes_per_env_step / 1e9 / world / PEAK_HBM_GBS,
                "achievable_copy_GBs": copy_gbs,
                "frac_of_copy": achieved / copy_gbs if copy_gbs else None,
                **({"valu_issue_frac": valu["valu_issue_frac"], "valu_per_wave": valu["valu_per_wave"],
                    "valu_source": profile_source(os.path.join(ROOT, "profiles", f"valu_{H}x{W}_A{A}_E{E}.json"),
                                                  valu) + f"; {valu['formula']}",
                    "valu_calibration": VALU_CALIBRATION} if valu else {}),
            },
            "cpu_baseline": None,
            "multi_step": multi,
        }
        if not args.no_cpu and world == 1:     # the CPU baseline is an N = 1 measurement
            out["cpu_baseline"] = cpu_baseline(args, m, s, params, snap, single_steps)
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


# run_actor_only_training.py:47-58 (epsilon = EPSILON_START, :40) and
# run_unified_actor_training.py:58-70 (epsilon = EPSILON_START, :51).
LEARN_CONFIGS = {
    4: dict(variant="actor_only", mode=None, max_steps=1000,      # run_actor_only_training.py:37
            params={"k_D": 1, "k_A": 10, "alpha_v": 0.1, "alpha_h": 0.1, "gamma": 0.95, "exit_reward": 100.0,
                    "step_penalty": 0.0, "collision_penalty": -1.0, "neighborhood": "neumann", "epsilon": 0.2}),
    5: dict(variant="unified", mode="actor_only", max_steps=300,  # run_unified_actor_training.py:47
            params={"k_S": 10, "k_D": 1, "k_A": 10, "alpha_v": 0.01, "alpha_h": 0.1, "gamma": 0.99,
                    "exit_reward": 100.0, "step_penalty": -1.0, "collision_penalty": -1.0,
                    "neighborhood": "neumann", "block_size": 1, "epsilon": 0.2}),
}


VALU_CALIBRATION = ("profiles/r06/alu/valu_calibration.json: saturated microkernels of known VALU count read "
                     "0.995 (v_mul_hi/lo_u32), 1.014 (v_mad_u64_u32) and 0.985 (v_exp_f32) by this formula, but "
                     "1.83 for plain xor/add: simple 32-bit ops issue faster than one per 4 clocks, so 1.0 is the "
                     "ceiling of multiply/transcendental-bound code only")


def profile_source(path, d):
    """Where a derived bench field comes from: a committed PMC profile, not this run."""
    rel = os.path.relpath(path, ROOT)
    when = d.get("measured", "an earlier round")
    return f"committed profile {rel} (measured {when}; not measured in this run)"


def timed_repeats(args, world, dist, torch, run_k, counters):
    """args.repeats timed regions of exactly K steps, each bracketed by a barrier and
    a device sync on both sides; per region the time is the max over ranks and the
    agent-steps the sum.  Returns the median region (by rate) and a summary."""
    rows = []
    for _ in range(max(1, args.repeats)):
        c0 = counters()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run_k()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        c1 = counters()
        n = c1["agent_steps"] - c0["agent_steps"]
        if world > 1:
            from ffm_amd.dist import reduce_counters, reduce_max
            el = reduce_max(el, device="cuda")
            n = reduce_counters({k: c1[k] - c0[k] for k in ("agent_steps", "exits", "resets", "steps")},
                                device="cuda")["agent_steps"]
        rows.append((n / el, el, n))
    med = sorted(rows)[(len(rows) - 1) // 2]
    return {"elapsed": med[1], "agent_steps": med[2],
            "summary": {"n": len(rows), "pick": "median rate",
                        "values": [r[0] for r in rows], "elapsed_s": [round(r[1], 6) for r in rows]}}


def cpu_share():
    """Threads for the CPU baseline and the host facts reported beside it.

    The GPU box gives each GPU a share of the host (OMP_NUM_THREADS is set to it
    there); os.cpu_count() reports the whole machine, whose other cores belong to
    other jobs, so the baseline runs on the share and reports nproc next to it."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS", "")
    threads = int(omp) if omp.isdigit() and int(omp) > 0 else aff
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return min(threads, aff), {"nproc": os.cpu_count(), "affinity_cpus": aff,
                               "omp_num_threads": omp or None, "cpu_model": model}


def learner_bytes_per_env_step(H, W, A, D, actions=5):
    """Algorithmic HBM bytes of one learning step of one env at full occupancy
    (DESIGN.md section 9.4): the ffm_core state round trip, 2*(2A + 4HW + 4),
    plus per agent two V reads (key + value, 16 B each) and one fixed-point
    increment (8 B read + 8 B write), and for actor variants the H row (8 B key +
    8 B per action: 40 B Neumann, 72 B Moore) and its increment (16 B)."""
    per_agent = 2 * 16 + 16 + (8 + 8 * actions + 16)
    return 2 * (2 * A + 4 * H * W + 4) + A * per_agent


def bench_learner(args, world, rank, torch, dist):
    from ffm_amd.data import make_room, l1_sff
    from ffm_amd.engine import Learner
    cfg = dict(LEARN_CONFIGS[args.config])
    if args.neighborhood != "neumann":     # a variant of the workload (the BASELINE configs are Neumann)
        cfg["params"] = dict(cfg["params"], neighborhood=args.neighborhood)
    H = W = args.size
    A, E = args.agents, args.envs
    m = make_room(H, W)
    s = l1_sff(m)
    L = Learner(m, s, cfg["variant"], n_envs=E, n_agents=A, mode=cfg["mode"], params=cfg["params"],
                rng="philox", seed=args.seed, auto_reset=True, max_steps=cfg["max_steps"], env_base=rank * E,
                device=torch.cuda.current_device(), log2_v_capacity=args.log2_table,
                log2_h_capacity=args.log2_table)
    stream = torch.cuda.current_stream()
    L.reset(stream)
    if world > 1:
        # the ranks share V / H: every step exchanges the table deltas over RCCL
        from ffm_amd.dist import TableSync
        # hashed tables: record buffers sized from the measured touched counts
        sync = TableSync(L, device="cuda", capacity=None, sync_period=args.sync_period)
        run = sync.step
    else:
        L.set_sync_period(args.sync_period)
        run = lambda k: L.step(k, stream)  # noqa: E731
    run(args.burn_in + args.warmup)
    torch.cuda.synchronize()
    print(f"[bench] config {args.config}: burn-in + warmup done", file=sys.stderr, flush=True)
    sent0 = sync.bytes_sent if world > 1 else 0
    recv0 = getattr(sync, "received_bytes", 0) if world > 1 else 0
    reps = timed_repeats(args, world, dist, torch, lambda: run(args.steps), lambda: L.counters(stream))
    sent_timed = (sync.bytes_sent - sent0) if world > 1 else 0
    recv_timed = (getattr(sync, "received_bytes", 0) - recv0) if world > 1 else 0
    elapsed, agent_steps = reps["elapsed"], reps["agent_steps"]
    print(f"[bench] timed regions {reps['summary']['elapsed_s']} s", file=sys.stderr, flush=True)
    # the event pass spans a whole timed window (config 5: one episode, its lockstep
    # truncation and reset included), so the roofline averages what `value` averages
    nk = min(args.steps, 300)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    run(nk)
    ev1.record(stream)
    torch.cuda.synchronize()
    step_ms = ev0.elapsed_time(ev1) / nk
    if world > 1:
        sync.flush()       # the ranks' key sets merged (the owner exchange keeps V's lazily)
    v_size, h_size = L.table_size("V"), L.table_size("H")
    if rank == 0:
        D = 4 if cfg["variant"] == "actor_only" else 1
        bpe = learner_bytes_per_env_step(H, W, A, D, 9 if args.neighborhood == "moore" else 5)
        achieved = E * bpe / (step_ms / 1e3) / 1e9
        # PMC HBM bytes of the batch kernel (tools/traffic.sh <out> --config 4|5)
        traffic = traffic_src = None
        tpath = os.path.join(ROOT, "profiles", f"traffic_{H}x{W}_A{A}_E{E}_learn{args.config}.json")
        if os.path.exists(tpath) and args.neighborhood == "neumann":     # (profiled on the Neumann configs)
            with open(tpath) as f:
                tj = json.load(f)
            if tj.get("config") == f"{H}x{W}_A{A}_E{E}_learn{args.config}":
                traffic = tj.get("hbm_bytes_per_launch")
                traffic_src = profile_source(tpath, tj)
        out = {
            "metric": METRIC, "value": agent_steps / elapsed, "unit": "agent-steps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32+f64",
            "data": "synthetic",
            "config": {
                "workload": (f"config {args.config}: {cfg['variant']}"
                             f"{'/' + cfg['mode'] if cfg['mode'] else ''} learning step, {H}x{W} room, "
                             f"{A} agents/env, {E} envs/GPU, epsilon {cfg['params']['epsilon']}, "
                             + (f"{args.neighborhood} neighbourhood, " if args.neighborhood != "neumann" else "")
                             + f"max_steps {cfg['max_steps']}, Philox seed {args.seed}, on-device auto-reset"
                             + (f", {args.burn_in}-step untimed burn-in" if args.burn_in else "")
                             + (f"; every {args.steps}-step timed window is one whole episode of every env (the "
                                f"envs run in lockstep: each episode truncates at max_steps), its start on the "
                                f"tables the previous episodes built and its lockstep reset included"
                                if args.config == 5 and args.steps == cfg["max_steps"] else "")
                             + (f", tables applied every {args.sync_period} steps" if args.sync_period > 1 else "")),
                "burn_in_steps": args.burn_in,
                "map": f"{H}x{W}", "agents_per_env": A, "envs_per_gpu": E, "global_envs": E * world,
                "parallelism": f"env-sharded x{world}",
            },
            "env_steps_per_s": E * world * args.steps / elapsed,
            "mean_live_agents_per_env_step": agent_steps / (E * world * args.steps),
            "repeats": reps["summary"],
            "step_ms_events": step_ms,
            "tables": {"V": v_size, "H": h_size},
            "table_sync": (dict({"period": args.sync_period,
                                 "mode": ("owner-sharded tiles: records all-to-all, updates all-gathered"
                                          if getattr(sync, "owner", False) else
                                          "tiled records all-gather" if sync.tiled else
                                          "dense all-reduce" if sync.dense else "records (adaptive capacity)"),
                                 "bytes_per_rank_per_step": sent_timed / (reps["summary"]["n"] * args.steps),
                                 "received_bytes_per_rank_per_step": recv_timed / (reps["summary"]["n"] * args.steps),
                                 "note": "bytes this rank contributes to / receives from the collectives per "
                                         "step, over the timed regions (fixed-capacity buffers: the bytes on the "
                                         "wire, not the touched counts)"},
                                **({} if sync.dense or sync.tiled else {"record_capacity": dict(sync.caps),
                                                          "max_touched_records": dict(sync.max_count)}))
                           if world > 1 else {"period": args.sync_period}),
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": achieved / PEAK_HBM_GBS, "traffic": traffic,
                         "traffic_kernel": "learn_batch_kernel (PMC FETCH_SIZE x2 + WRITE_SIZE)",
                         "traffic_source": traffic_src,
                         "bytes_per_launch_algorithmic": E * bpe,
                         # BASELINE.md 3's form: env-steps/s of the timed windows x the bytes per env-step
                         "frac_env_rate": E * args.steps / elapsed * bpe / 1e9 / PEAK_HBM_GBS,
                         "note": "whole learning step (all kernels) timed with HIP events"},
            "cpu_baseline": None,
        }
        if not args.no_cpu and world == 1:
            out["cpu_baseline"] = cpu_baseline_learner(args, cfg, m, s)
        print(json.dumps(out), flush=True)
    L.close()
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline_learner(args, cfg, m, s):
    """The batched learning restatement (oracle/ffm_learn_oracle.c) on a bounded
    sample; its state after the sample is checked bit-exactly against a fresh
    GPU learner stepped the same number of steps."""
    from oracle import learn as LO
    from oracle import oracle as O
    from ffm_amd.engine import Learner
    H, W = m.shape
    A = args.agents
    share, host = cpu_share()
    threads = args.cpu_threads or share
    # the OpenMP loop runs over envs: C5 steps as many envs as threads (8,192 agents each),
    # so every reported core has an env of its own
    E = min(args.cpu_envs, 1024) if args.config == 4 else max(2, threads)
    cpu = LO.Learn(m, s, cfg["variant"], cfg["mode"], cfg["params"], log2_cap=22 if args.config == 4 else 24)
    core = O.Core(m, s, {"neighborhood": "neumann"})
    pos = np.full((E, A), 0xFFFF, np.uint16)
    for e in range(E):
        pos[e] = core.reset_philox(A, args.seed, 0, e)
    cnt = np.full(E, A, np.int32)
    dff = np.zeros((E, H, W), np.float32)
    eps = np.zeros(E, np.int32)
    est = np.zeros(E, np.int32)
    t, total = 1, 0
    tb = time.perf_counter()
    while time.perf_counter() - tb < 12.0 or t <= 3:
        total += cpu.step_philox_batch(pos, cnt, dff, eps, est, args.seed, t, True, A, cfg["max_steps"], 0,
                                       threads)
        t += 1
    elapsed = time.perf_counter() - tb
    g = Learner(m, s, cfg["variant"], n_envs=E, n_agents=A, mode=cfg["mode"], params=cfg["params"],
                rng="philox", seed=args.seed, auto_reset=True, max_steps=cfg["max_steps"])
    g.reset()
    g.step(t - 1)
    gp, gc, gd = g.get_state()
    tables = {"V": (g.export_table("V"), cpu.V.export())}
    if cfg["variant"] == "actor_only" or cfg["mode"] in ("actor_only", "both"):
        tables["H"] = (g.export_table("H"), cpu.Ht.export())
    g.close()

    def same_table(gkv, ckv):
        (gk, gv), (ck, cv) = gkv, ckv
        return (np.array_equal(np.sort(gk), np.sort(ck))
                and np.array_equal(gv[np.argsort(gk)].view(np.uint64), cv[np.argsort(ck)].view(np.uint64)))

    state_ok = bool(np.array_equal(gc, cnt) and np.array_equal(gd.view(np.uint32), dff.view(np.uint32))
                    and all(np.array_equal(gp[e, :gc[e]], pos[e, :gc[e]]) for e in range(E)))
    tab_ok = {k: bool(same_table(*v)) for k, v in tables.items()}
    ok = state_ok and all(tab_ok.values())
    return {
        "value": total / elapsed, "unit": "agent-steps/s", "cores": min(threads, E), "kind": "port",
        "sample": (f"oracle/ffm_learn_oracle.c batched Philox mode, {E} envs x {t - 1} steps of the same "
                   f"workload (OpenMP {threads} threads, {host['cpu_model']}); positions, counts, DFF and "
                   f"tables {'/'.join(tables)} bit-exact vs GPU: {ok}"),
        "seconds": elapsed, "bit_exact_vs_gpu": ok, "bit_exact_tables": tab_ok, "host": host,
        "threads_note": "the GPU's host-CPU share on the box (OMP_NUM_THREADS); nproc is the whole machine",
    }


def copy_bandwidth(torch, stream, nbytes, reps=50):
    """GB/s (read + write bytes) of a device-to-device copy of `nbytes`."""
    n = max(1, nbytes // 4)
    src = torch.ones(n, dtype=torch.float32, device="cuda")
    dst = torch.empty_like(src)
    with torch.cuda.stream(stream):
        for _ in range(5):
            dst.copy_(src)
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(reps):
            dst.copy_(src)
        b.record(stream)
    torch.cuda.synchronize()
    sec = a.elapsed_time(b) / 1e3 / reps
    del src, dst
    return 2 * n * 4 / sec / 1e9


def cpu_baseline(args, m, s, params, snap, single_steps):
    """Time the CPU restatement (oracle/, Philox mode) on the same workload.

    Full replay (the default whenever it fits --cpu-budget): every env of the timed
    engine, from the same reset, through every single-step launch the engine ran
    (burn-in, warmup, timed regions, event pass); the oracle's state is then compared
    bit for bit with the engine's snapshot -- all envs, positions, counts and DFF.
    The timed span is the replay's steady-state tail, the last ~15 s (the first
    steps are the post-reset transient).  Otherwise a bounded sample of --cpu-envs
    envs, checked against a fresh GPU engine."""
    from oracle import oracle as O
    from ffm_amd.engine import Engine
    A = args.agents
    H, W = m.shape
    share, host = cpu_share()
    threads = args.cpu_threads or share
    core = O.Core(m, s, params)

    def fresh(E):
        pos = np.stack([core.reset_philox(A, args.seed, 0, e) for e in range(E)])
        return pos, np.full(E, A, np.int32), np.zeros((E, H, W), np.float32), np.zeros(E, np.int32)

    # calibrate on 512 envs x 8 steps, then decide between the full replay and a sample
    pc, cc, dc, ec = fresh(min(512, args.envs))
    tb = time.perf_counter()
    for t in range(1, 9):
        core.step_philox_batch(pc, cc, dc, ec, args.seed, t, True, A, 0, threads)
    env_step_s = (time.perf_counter() - tb) / (8 * len(cc))
    full = (snap is not None and not args.cpu_steps
            and env_step_s * args.envs * single_steps < args.cpu_budget)
    E = args.envs if full else args.cpu_envs
    pos, cnt, dff, eps = fresh(E)
    total = 0
    t = 1
    tb = time.perf_counter()
    if full:
        # time the replay's last ~15 s: steps from t_timed on
        t_timed = max(1, single_steps - int(15.0 / max(env_step_s * E, 1e-9)))
        t_start = None
        while t <= single_steps:
            if t == t_timed:
                t_start, total = time.perf_counter(), 0
            total += core.step_philox_batch(pos, cnt, dff, eps, args.seed, t, True, A, 0, threads)
            t += 1
        elapsed = time.perf_counter() - t_start
        steps = single_steps - t_timed + 1
    else:
        steps = 0
        while (args.cpu_steps and steps < args.cpu_steps) or (not args.cpu_steps and time.perf_counter() - tb < 15.0):
            total += core.step_philox_batch(pos, cnt, dff, eps, args.seed, t, True, A, 0, threads)
            t += 1
            steps += 1
        elapsed = time.perf_counter() - tb
    # single-thread rate on a smaller slice of the same state (~3 s)
    n1 = min(E, 512)
    p1, c1_, d1, e1 = pos[:n1].copy(), cnt[:n1].copy(), dff[:n1].copy(), eps[:n1].copy()
    t1, tot1, st1 = t, 0, time.perf_counter()
    while time.perf_counter() - st1 < 3.0:
        tot1 += core.step_philox_batch(p1, c1_, d1, e1, args.seed, t1, True, A, 0, 1)
        t1 += 1
    one_thread = tot1 / (time.perf_counter() - st1)
    if full:
        gp, gc, gd = snap
        what = f"all {E} envs of the timed engine after its {single_steps} single-step launches"
    else:
        g = Engine(m, s, n_envs=E, n_agents=A, params=params, rng="philox", seed=args.seed,
                   auto_reset=True, env_base=0)
        g.reset()
        g.step(t - 1)
        gp, gc, gd = g.get_state()
        g.close()
        what = f"all {E} envs of a fresh GPU engine after {t - 1} steps"
    ok = bool(np.array_equal(gc, cnt) and np.array_equal(gd.view(np.uint32), dff.view(np.uint32))
              and all(np.array_equal(gp[e, :gc[e]], pos[e, :gc[e]]) for e in range(E)))
    return {
        "value": total / elapsed, "unit": "agent-steps/s", "cores": min(threads, E), "kind": "port",
        "sample": (f"oracle/ffm_oracle.c Philox mode, {E} envs x {steps} steps of the same workload "
                   + (f"(the last {steps} of a {single_steps}-step replay) " if full else "")
                   + f"(OpenMP {threads} threads, {host['cpu_model']}); {what} bit-exact vs the oracle: {ok}"),
        "seconds": elapsed, "bit_exact_vs_gpu": ok, "checked_envs": E, "checked_steps": single_steps if full else t - 1,
        "value_1thread": one_thread,
        "value_per_core_x_nproc": one_thread * (host["nproc"] or 1), "host": host,
        "threads_note": ("the GPU's host-CPU share on the box (OMP_NUM_THREADS); nproc is the whole machine, "
                         "value_per_core_x_nproc extrapolates the 1-thread rate to every core"),
    }


if __name__ == "__main__":
    main()
