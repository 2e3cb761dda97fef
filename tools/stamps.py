"""Diagnostic: per-phase cycle shares of the wave kernel (FFM_STAMPS build)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from ffm_amd.data import make_room, l1_sff  # noqa: E402
from ffm_amd.engine import Engine, load_library  # noqa: E402

L = load_library()
L.ffm_debug_read.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
m = make_room(12, 12)
epb = int(sys.argv[1]) if len(sys.argv) > 1 else 0   # 0: auto (lane kernel), -1: wave kernel
eng = Engine(m, l1_sff(m), n_envs=65536, n_agents=32, params={"neighborhood": "neumann"}, seed=42,
             envs_per_block=epb)
eng.reset()
eng.step(20)
torch.cuda.synchronize()
base = np.zeros(16, np.uint64)
L.ffm_debug_read(eng._h, base.ctypes.data, 16)
eng.step(100)
torch.cuda.synchronize()
after = np.zeros(16, np.uint64)
L.ffm_debug_read(eng._h, after.ctypes.data, 16)
d = (after - base).astype(np.float64)
names = (["head/pp", "marks", "decide", "req-write", "resolve", "exits", "stencil", "stage+store"] if epb == -1 else
         ["head+mark", "decide", "resolve", "exits", "pos+reset", "dma-issue", "stencil", "dff-store"])
tot = d[:8].sum()
waves = d[8]
print(f"waves*launches={waves:.0f}  cycles/wave/launch={tot / waves:.0f}")
for k in range(8):
    print(f"{names[k]:12s} {d[k] / tot * 100:6.1f}%  {d[k] / waves:10.0f} cyc/wave/launch")
