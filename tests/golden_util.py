"""Helpers to read the golden fixtures written by tests/golden/gen_golden.py."""
from __future__ import annotations

import glob
import hashlib
import json
import os
from dataclasses import dataclass

import numpy as np

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def dff_hash(d: np.ndarray) -> int:
    b = hashlib.blake2b(np.ascontiguousarray(d, dtype=np.float32).tobytes(), digest_size=8).digest()
    return int(np.frombuffer(b, dtype=np.uint64)[0])


@dataclass
class Episode:
    seed: int
    init: np.ndarray          # [N] int cells
    counts: np.ndarray        # [T]
    cells: list               # T arrays of int cells
    hashes: np.ndarray        # [T] uint64
    full: list                # T arrays [H,W] f32, or []
    np_tail: np.ndarray
    py_tail: np.ndarray


@dataclass
class Case:
    name: str
    map: np.ndarray
    sff: np.ndarray
    params: dict
    N: int
    episodes: list
    max_steps: int


def case_names():
    return sorted(os.path.basename(p)[5:-4] for p in glob.glob(os.path.join(GOLDEN_DIR, "core_*.npz")))


def load_case(name: str) -> Case:
    z = np.load(os.path.join(GOLDEN_DIR, f"core_{name}.npz"), allow_pickle=False)
    seeds = z["seeds"]
    nsteps = z["nsteps"]
    counts = z["counts"].astype(np.int64)
    cells = z["cells"].astype(np.int64)
    hashes = z["dff_hash"]
    full = z["dff_full"]
    eps = []
    so, co = 0, 0
    for i, s in enumerate(seeds):
        T = int(nsteps[i])
        cnt = counts[so:so + T]
        per = []
        for c in cnt:
            per.append(cells[co:co + c])
            co += c
        eps.append(Episode(int(s), z["init"][i].astype(np.int64), cnt, per, hashes[so:so + T],
                           [], z["np_tail"][i], z["py_tail"][i]))
        so += T
    # full DFFs belong to the first seeds in order
    fo = 0
    for ep in eps:
        T = len(ep.counts)
        if fo + T <= full.shape[0]:
            ep.full = [full[fo + t] for t in range(T)]
            fo += T
        else:
            break
    return Case(name, z["map"], z["sff"], json.loads(str(z["params"])), int(z["N"]), eps,
                int(z["max_steps"]))
