#!/usr/bin/env python3
"""Headline benchmark: agent-steps/s of the batched ffm_core step on MI355X.

Workload (BASELINE.json configs[1]): 12x12 room (create_12x12_map_and_sff.py
recipe), 32 agents per env, 65,536 envs per GPU, default_config.yaml params
(k_S 3, k_D 1, diffuse 0.2, decay 0.2, neumann), Philox RNG seeded 42,
on-device auto-reset.  One bench "step" = one FloorFieldModel.step() of every
env = one launch of the fused HIP kernel over inputs resident in HBM.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

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
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--size", type=int, default=12)
    ap.add_argument("--agents", type=int, default=32)
    ap.add_argument("--neighborhood", default="neumann")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--envs-per-block", type=int, default=0)
    ap.add_argument("--cpu-envs", type=int, default=4096)
    ap.add_argument("--cpu-steps", type=int, default=0, help="0 = size the sample to ~15 s")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = min(16, cpu count)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_config2.json"))
    return ap.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)

    from ffm_amd.data import make_room, l1_sff
    from ffm_amd.engine import Engine

    H = W = args.size
    A = args.agents
    E = args.envs
    m = make_room(H, W)
    s = l1_sff(m)
    params = {"k_S": 3, "k_D": 1, "diffuse": 0.2, "decay": 0.2, "neighborhood": args.neighborhood}
    eng = Engine(m, s, n_envs=E, n_agents=A, params=params, rng="philox", seed=args.seed,
                 auto_reset=True, env_base=rank * E, device=torch.cuda.current_device(),
                 envs_per_block=args.envs_per_block)
    stream = torch.cuda.current_stream()
    eng.reset(stream)
    eng.step(args.warmup, stream)
    torch.cuda.synchronize()
    c0 = eng.counters(stream)

    # Timed region: K back-to-back step launches on the stream, nothing in between.
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.step(args.steps, stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    c1 = eng.counters(stream)
    elapsed = t1 - t0
    agent_steps = c1["agent_steps"] - c0["agent_steps"]

    # Kernel time for the roofline: HIP events on the launch stream bracketing
    # nk back-to-back launches (a separate pass, so events do not perturb
    # `value`); per-launch event pairs would add their own gaps to each launch.
    nk = min(args.steps, 200)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    eng.step(nk, stream)
    ev1.record(stream)
    torch.cuda.synchronize()
    kern_ms = [ev0.elapsed_time(ev1) / nk]

    # Achievable HBM bandwidth on this box: a device-to-device copy of the same
    # number of bytes one launch moves (read + write), for context beside `peak`.
    copy_gbs = copy_bandwidth(torch, stream, E * (2 * A + 4 * H * W + 4))

    if world > 1:
        from ffm_amd.dist import reduce_counters, reduce_max
        elapsed = reduce_max(elapsed, device="cuda")
        d = {k: c1[k] - c0[k] for k in ("agent_steps", "exits", "resets", "steps")}
        agent_steps = reduce_counters(d, device="cuda")["agent_steps"]

    if rank == 0:
        bytes_per_env_step = 2 * (2 * A + 4 * H * W + 4)
        mean_kernel_s = float(np.mean(kern_ms)) / 1e3
        achieved = E * bytes_per_env_step / mean_kernel_s / 1e9
        traffic = None
        if os.path.exists(args.traffic_json):
            with open(args.traffic_json) as f:
                tj = json.load(f)
            if tj.get("config") == f"{H}x{W}_A{A}_E{E}":
                traffic = tj.get("hbm_bytes_per_launch")
        out = {
            "metric": METRIC,
            "value": agent_steps / elapsed,
            "unit": "agent-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {
                "workload": (f"ffm_core step, {H}x{W} room, {A} agents/env, {E} envs/GPU, "
                             f"{args.neighborhood}, Philox seed {args.seed}, on-device auto-reset"),
                "map": f"{H}x{W}", "agents_per_env": A, "envs_per_gpu": E,
                "global_envs": E * world, "parallelism": f"env-sharded x{world}",
            },
            "env_steps_per_s": E * world * args.steps / elapsed,
            "kernel_ms_mean": float(np.mean(kern_ms)),
            "kernel_ms_median": float(np.median(kern_ms)),
            "roofline": {
                "bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": achieved / PEAK_HBM_GBS, "traffic": traffic,
                "bytes_per_launch_algorithmic": E * bytes_per_env_step,
                "achievable_copy_GBs": copy_gbs,
                "frac_of_copy": achieved / copy_gbs if copy_gbs else None,
            },
            "cpu_baseline": None,
        }
        if not args.no_cpu:
            out["cpu_baseline"] = cpu_baseline(args, m, s, params, torch)
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


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


def cpu_baseline(args, m, s, params, torch):
    """Time the CPU restatement (oracle/, Philox mode) on a bounded sample of the
    same workload; check its first envs bit-exactly against a fresh GPU run."""
    from oracle import oracle as O
    from ffm_amd.engine import Engine
    A, E = args.agents, args.cpu_envs
    H, W = m.shape
    threads = args.cpu_threads or min(16, os.cpu_count() or 1)
    core = O.Core(m, s, params)
    pos = np.stack([core.reset_philox(A, args.seed, 0, e) for e in range(E)])
    cnt = np.full(E, A, np.int32)
    dff = np.zeros((E, H, W), np.float32)
    eps = np.zeros(E, np.int32)
    # calibrate: a few steps, then size the sample to ~15 s of CPU work
    t = 1
    ta = time.perf_counter()
    calib = 0
    for _ in range(5):
        calib += core.step_philox_batch(pos, cnt, dff, eps, args.seed, t, True, A, 0, threads)
        t += 1
    dt = time.perf_counter() - ta
    steps = args.cpu_steps or max(10, int(15.0 / max(dt / 5, 1e-6)))
    tb = time.perf_counter()
    total = 0
    for _ in range(steps):
        total += core.step_philox_batch(pos, cnt, dff, eps, args.seed, t, True, A, 0, threads)
        t += 1
    elapsed = time.perf_counter() - tb
    # single-thread rate on a smaller slice of the same state (~3 s)
    n1 = min(E, 512)
    p1, c1_, d1, e1 = pos[:n1].copy(), cnt[:n1].copy(), dff[:n1].copy(), eps[:n1].copy()
    t1, tot1, st1 = t, 0, time.perf_counter()
    while time.perf_counter() - st1 < 3.0:
        tot1 += core.step_philox_batch(p1, c1_, d1, e1, args.seed, t1, True, A, 0, 1)
        t1 += 1
    one_thread = tot1 / (time.perf_counter() - st1)
    # bit-exact check of the first envs against a fresh GPU engine
    nchk = min(1024, E)
    g = Engine(m, s, n_envs=nchk, n_agents=A, params=params, rng="philox", seed=args.seed,
               auto_reset=True, env_base=0)
    g.reset()
    g.step(t - 1)
    gp, gc, gd = g.get_state()
    g.close()
    ok = bool(np.array_equal(gc, cnt[:nchk]) and np.array_equal(gd.view(np.uint32), dff[:nchk].view(np.uint32))
              and all(np.array_equal(gp[e, :gc[e]], pos[e, :gc[e]]) for e in range(nchk)))
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {
        "value": total / elapsed, "unit": "agent-steps/s", "cores": threads, "kind": "port",
        "sample": (f"oracle/ffm_oracle.c Philox mode, {E} envs x {steps} steps of the same workload "
                   f"(OpenMP {threads} threads, {model}); first {nchk} envs bit-exact vs GPU: {ok}"),
        "seconds": elapsed, "bit_exact_vs_gpu": ok, "value_1thread": one_thread,
    }


if __name__ == "__main__":
    main()
