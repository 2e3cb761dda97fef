"""C5 diagnostic: how much of the dense V / H accumulator arrays one learning step
touches (nonzero words), per slot and per 64-slot block, for E envs (512 = one rank
of the 8-GPU config, 4096 = the union over 8 ranks).  Sizes a sparse table exchange.

    python tools/c5_touched.py [E ...]
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from ffm_amd.data import make_room, l1_sff  # noqa: E402
from ffm_amd.engine import Learner  # noqa: E402


def frac(acc, width):
    a = acc.view(-1, width)
    slot = (a != 0).any(dim=1)
    blk = slot.view(-1, 64).any(dim=1)
    return int(slot.sum()), int(blk.sum()), a.shape[0], blk.numel()


def main():
    cfg = bench.LEARN_CONFIGS[5]
    m = make_room(256, 256)
    s = l1_sff(m)
    out = {}
    for E in [int(x) for x in sys.argv[1:]] or [512, 4096]:
        L = Learner(m, s, cfg["variant"], n_envs=E, n_agents=8192, mode=cfg["mode"], params=cfg["params"],
                    rng="philox", seed=42, auto_reset=True, max_steps=cfg["max_steps"])
        L.reset()
        rows = []
        for t in range(60):
            L.step_local()
            if t % 10 == 9:
                accv, _ = L.dense_buffers("V")
                torch.cuda.synchronize()
                v = frac(accv, 2)
            L.step_apply("V")
            if t % 10 == 9:
                acch, _ = L.dense_buffers("H")
                torch.cuda.synchronize()
                h = frac(acch, 5)
                live = int(L.get_state()[1].sum())
                rows.append({"step": t + 1, "live_agents": live, "V_slots": v[0], "V_blocks": v[1],
                             "H_slots": h[0], "H_blocks": h[1], "slots": v[2], "blocks": v[3],
                             "V_present": L.table_size("V"), "H_present": L.table_size("H")})
                print(E, rows[-1], flush=True)
            L.step_apply("H")
            L.step_end()
        L.close()
        out[E] = rows
    print(json.dumps(out))


if __name__ == "__main__":
    main()
