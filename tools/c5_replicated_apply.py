"""C5 at N ranks on one GPU: the per-rank table-update cost of a tiled exchange.

Couples `--shards` learners of 512 envs each (the C5 bench's per-GPU env count, global
env ids r * 512 + e) through ffm_amd.dist.step_coupled on cuda:0, so every shard's
apply sums the records of all shards' envs, as each rank does at N = shards.  Run
under `rocprofv3 --kernel-trace --stats` to get the per-launch tile-pass times.

    python tools/c5_replicated_apply.py [--shards 8] [--steps 20] [--warmup 10] [--owner]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from ffm_amd.data import make_room, l1_sff  # noqa: E402
from ffm_amd.dist import step_coupled  # noqa: E402
from ffm_amd.engine import Learner  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shards", type=int, default=8)
    ap.add_argument("--envs", type=int, default=512)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--owner", action="store_true", help="owner-sharded exchange (DESIGN 9.8)")
    a = ap.parse_args()
    cfg = bench.LEARN_CONFIGS[5]
    m = make_room(256, 256)
    s = l1_sff(m)
    shards = [Learner(m, s, cfg["variant"], n_envs=a.envs, n_agents=8192, mode=cfg["mode"], params=cfg["params"],
                      rng="philox", seed=42, auto_reset=True, max_steps=cfg["max_steps"], env_base=r * a.envs,
                      log2_v_capacity=24, log2_h_capacity=24) for r in range(a.shards)]
    for L in shards:
        L.reset()
    kw = {"owner": True} if a.owner else {"tiled": True}
    step_coupled(shards, a.warmup, **kw)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    step_coupled(shards, a.steps, **kw)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    out = {"shards": a.shards, "envs_per_shard": a.envs, "steps": a.steps, "owner": a.owner,
           "ms_per_coupled_step": 1e3 * el / a.steps,
           "V": shards[0].table_size("V"), "H": shards[0].table_size("H")}
    if a.owner:     # the last step's exchange volumes per shard (records in, V values out, H increments out)
        b = [L.owner_buffers() for L in shards]
        out["records_out"] = [int(x["counts"][: a.shards].sum()) for x in b]
        g = shards[0]._coupled[2]        # coupled shards write their outputs into the gathered buffers
        out["v_values_out"] = g["gvc"].tolist()
        out["h_increments_out"] = g["ghc"].tolist()
        out["capacities"] = {"records_per_destination": b[0]["rec_capacity"], "v": b[0]["v_capacity"],
                             "h": b[0]["h_capacity"]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
