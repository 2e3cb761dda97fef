"""Diagnostic: Philox GPU vs oracle on one config for the library in FFM_LIB_PATH.
    python tools/quick_parity.py [E] [T] [epb]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from ffm_amd.data import make_room, l1_sff  # noqa: E402
from ffm_amd.engine import Engine  # noqa: E402
from oracle import oracle as O  # noqa: E402

E = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
T = int(sys.argv[2]) if len(sys.argv) > 2 else 150
epb = int(sys.argv[3]) if len(sys.argv) > 3 else 0
p = {"k_S": 3, "k_D": 1, "diffuse": 0.2, "decay": 0.2, "neighborhood": "neumann"}
m = make_room(12, 12)
s = l1_sff(m)
eng = Engine(m, s, n_envs=E, n_agents=32, params=p, rng="philox", seed=42, auto_reset=True, envs_per_block=epb)
core = O.Core(m, s, p)
pos = np.stack([core.reset_philox(32, 42, 0, e) for e in range(E)])
cnt = np.full(E, 32, np.int32)
dff = np.zeros((E, 12, 12), np.float32)
eps = np.zeros(E, np.int32)
eng.reset()
first_bad = None
for t in range(1, T + 1):
    core.step_philox_batch(pos, cnt, dff, eps, 42, t, True, 32, 0, 16)
    eng.step(1)
    gp, gc, gd = eng.get_state()
    bad = np.nonzero(gc != cnt)[0]
    dbad = np.nonzero((gd.view(np.uint32) != dff.view(np.uint32)).reshape(E, -1).any(1))[0]
    pbad = [e for e in range(E) if not np.array_equal(gp[e, :cnt[e]], pos[e, :cnt[e]])]
    if len(bad) or len(dbad) or pbad:
        print(f"t={t}: count mismatches {len(bad)} {bad[:8]}, dff {len(dbad)} {dbad[:8]}, pos {len(pbad)} {pbad[:8]}")
        e = (list(bad) + list(dbad) + pbad)[0]
        print(" env", e, "gpu cnt", gc[e], "cpu cnt", cnt[e], "eps cpu", eps[e])
        print(" gpu pos", gp[e, :max(gc[e], cnt[e])])
        print(" cpu pos", pos[e, :max(gc[e], cnt[e])])
        first_bad = t
        break
print("first bad step:", first_bad)
