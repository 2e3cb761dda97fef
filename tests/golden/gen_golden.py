#!/usr/bin/env python3
"""Generate golden vectors by running the reference itself (container only).

Run here, where the read-only reference is mounted:

    python tests/golden/gen_golden.py [--ref /root/reference]

It imports ``model.ffm_core.FloorFieldModel`` from the reference
(SoraKurihara/FFM), seeds NumPy's and CPython's global generators exactly as
``main.py:23-26`` does, and records whole episodes.  The reference's source
never leaves this container: only the recorded arrays (inputs and outputs)
are written, as small ``.npz`` fixtures next to this script.

Fixture layout (one file per case):
  map [H,W] u8, sff [H,W] (f32 or f64), params json, N, seeds [S]
  init      [S, N] int16      initial agent cells (x*W+y)
  nsteps    [S]    int32      steps recorded per seed
  counts    [sum(nsteps)] int16     agents alive after each step
  cells     [sum(counts)] int16     agent cells after each step, in order
  dff_hash  [sum(nsteps)] uint64    blake2b-64 of the DFF float32 bytes
  dff_full  [F, H, W] float32 DFF after each step of the first seed(s)
  np_tail / py_tail [S, 4] uint32  next raw 32-bit words of both RNG streams
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import random
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def dff_hash(d: np.ndarray) -> np.uint64:
    return np.frombuffer(hashlib.blake2b(np.ascontiguousarray(d, dtype=np.float32).tobytes(),
                                         digest_size=8).digest(), dtype=np.uint64)[0]


def reference_12x12(ref: str, out_dir: str):
    """Run the reference's own create_12x12_map_and_sff.py in a scratch cwd."""
    with tempfile.TemporaryDirectory() as td:
        subprocess.run([sys.executable, os.path.join(ref, "create_12x12_map_and_sff.py")],
                       cwd=td, check=True, stdout=subprocess.DEVNULL)
        m = np.load(os.path.join(td, "data/maps/simple_room_12x12.npy"))
        s = np.load(os.path.join(td, "data/sff/distance_L1_12x12.npy"))
    np.savez_compressed(os.path.join(out_dir, "room_12x12_reference.npz"), map=m, sff=s)
    return m, s


def run_case(name, FloorFieldModel, map_array, sff, params, N, seeds, max_steps, full_seeds):
    H, W = map_array.shape
    with tempfile.TemporaryDirectory() as td:
        sff_path = os.path.join(td, "sff.npy")
        np.save(sff_path, sff)
        init, nsteps, counts, cells, hashes, full = [], [], [], [], [], []
        np_tail, py_tail = [], []
        for si, seed in enumerate(seeds):
            np.random.seed(seed)
            random.seed(seed)
            model = FloorFieldModel(map_array, sff_path, N, dict(params))
            init.append((model.positions[:, 0] * W + model.positions[:, 1]).astype(np.int16))
            steps = 0
            while model.positions.shape[0] > 0 and steps < max_steps:
                model.step()
                steps += 1
                p = model.positions
                counts.append(p.shape[0])
                cells.extend((p[:, 0] * W + p[:, 1]).astype(np.int16).tolist())
                hashes.append(dff_hash(model.dff))
                if si < full_seeds:
                    full.append(np.array(model.dff, dtype=np.float32))
            nsteps.append(steps)
            bg = np.random.mtrand._rand._bit_generator
            np_tail.append(np.asarray(bg.random_raw(4), dtype=np.uint32))
            py_tail.append(np.asarray([random.getrandbits(32) for _ in range(4)], dtype=np.uint32))
    out = dict(
        map=map_array.astype(np.uint8), sff=sff, params=json.dumps(params), N=np.int32(N),
        seeds=np.asarray(seeds, dtype=np.int64), init=np.stack(init).astype(np.int16),
        nsteps=np.asarray(nsteps, dtype=np.int32), counts=np.asarray(counts, dtype=np.int16),
        cells=np.asarray(cells, dtype=np.int16), dff_hash=np.asarray(hashes, dtype=np.uint64),
        dff_full=np.asarray(full, dtype=np.float32).reshape(-1, H, W),
        np_tail=np.stack(np_tail), py_tail=np.stack(py_tail), max_steps=np.int32(max_steps),
    )
    path = os.path.join(HERE, f"core_{name}.npz")
    np.savez_compressed(path, **out)
    print(f"{name}: seeds={len(seeds)} steps={sum(nsteps)} -> {os.path.getsize(path)} B")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--only", default="", help="comma-separated case names to (re)generate")
    args = ap.parse_args()
    only = set(filter(None, args.only.split(",")))
    sys.path.insert(0, args.ref)
    from model.ffm_core import FloorFieldModel  # the reference itself

    global run_case
    _run = run_case

    def run_case(name, *a, **kw):        # noqa: F811 -- filter by --only
        if not only or name in only:
            _run(name, *a, **kw)

    yaml_params = {"k_S": 3, "k_D": 1, "diffuse": 0.2, "decay": 0.2, "neighborhood": "neumann"}
    m12, s12 = reference_12x12(args.ref, HERE)
    # config 1: 12x12, 8 agents (default_config.yaml params)
    run_case("neumann_12x12_N8", FloorFieldModel, m12, s12, yaml_params, 8, list(range(24)), 10_000, 2)
    # config-2 semantics: 12x12, 32 agents
    run_case("neumann_12x12_N32", FloorFieldModel, m12, s12, yaml_params, 32, list(range(12)), 10_000, 1)
    # class-default Moore neighbourhood (exercises the 8-lane float32 sum at >= 8 candidates)
    moore = dict(yaml_params, neighborhood="moore")
    run_case("moore_12x12_N32", FloorFieldModel, m12, s12, moore, 32, list(range(12)), 10_000, 1)
    run_case("moore_12x12_N12", FloorFieldModel, m12, s12, moore, 12, list(range(12, 24)), 10_000, 0)
    # friction-heavy and other parameter points
    hot = {"k_S": 1.5, "k_D": 2.5, "diffuse": 0.3, "decay": 0.1, "neighborhood": "neumann"}
    run_case("neumann_12x12_N60_hot", FloorFieldModel, m12, s12, hot, 60, list(range(100, 106)), 10_000, 0)
    # config 3 semantics (64x64, 512 agents), truncated episodes
    sys.path.insert(0, os.path.dirname(HERE))
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from ffm_amd.data import make_room, l1_sff
    m64 = make_room(64, 64)
    run_case("neumann_64x64_N512", FloorFieldModel, m64, l1_sff(m64), yaml_params, 512, [7], 40, 0)
    # BASELINE config-3 geometry at depth: 4 seeds x 200 steps (episodes last ~300 steps)
    run_case("neumann_64x64_N512_s4", FloorFieldModel, m64, l1_sff(m64), yaml_params, 512, [31, 32, 33, 34],
             200, 1)
    # main.py configuration: 50x50 room, float64 L1 SFF, N=100, seed 42, until empty
    m50 = np.load(os.path.join(args.ref, "data/maps/simple_room.npy"))
    s50 = np.load(os.path.join(args.ref, "data/sff/distance_L1.npy"))
    run_case("main_50x50_N100", FloorFieldModel, m50, s50, yaml_params, 100, [42], 100_000, 0)


if __name__ == "__main__":
    main()
