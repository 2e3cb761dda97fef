#!/usr/bin/env python3
"""Golden vectors of the reference's learning variants (container only).

    python tests/golden/gen_golden_learn.py [--ref /root/reference]

Imports the reference's own classes (SoraKurihara/FFM):
  * model/ffm_ac_core.py      FloorFieldModel            (critic, 13-cell keys)
  * model/ffm_unified.py      FloorFieldModelUnified     (critic_only / actor_only / both)
  * model/ffm_actor_only.py   FloorFieldModelActorOnly   (config-4 actor, 13-cell keys)
seeds NumPy's and CPython's global generators, and records several episodes
per seed with the tables carried across episodes (``reset()`` between them,
like the training drivers, e.g. run_unified_actor_training.py:270-300).
Only recorded arrays leave this container, as ``learn_*.npz`` fixtures.

Per case: map, sff, params (json), variant, mode, N, seeds, episodes per
seed, epsilon per episode; per step: counts / cells (as in gen_golden.py) and
a DFF hash; per seed: the V table and H table at the end, in dict insertion
order, keys packed by ffm_amd/learn_keys.py, and the RNG tails.  One case also
calls ``set_v_table(get_v_table())`` between episodes (model/ffm_ac_core.py:335-343:
missing states then default to -1.0).
"""
from __future__ import annotations

import argparse
import contextlib
import io
import json
import os
import pickle
import random
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))
from golden_util import dff_hash  # noqa: E402
from ffm_amd import learn_keys as K  # noqa: E402


def pack_key(variant, k):
    if variant == "unified":
        return K.from_rank_tuple(k)
    if isinstance(k, (bytes, bytearray)):
        return K.from_cells_bytes(bytes(k))
    return K.from_cells_tuple(k)


def run_case(name, variant, cls, map_array, sff, params, N, seeds, n_ep, max_steps, mode=None,
             eps_sched=None, reload_v=False, pretrained=None):
    """pretrained: (keys, values) of a critic pickled as the drivers' pretrained_v_path
    (bytes keys, run_actor_only_training.py:24, run_unified_actor_training.py:30)."""
    H, W = map_array.shape
    init, nsteps, counts, cells, hashes = [], [], [], [], []
    vk, vv, vn, hk, hv, hn, np_tail, py_tail, eps_list = [], [], [], [], [], [], [], [], []
    with tempfile.TemporaryDirectory() as td:
        sff_path = os.path.join(td, "sff.npy")
        np.save(sff_path, sff)
        kw = {}
        if pretrained is not None:
            kw["pretrained_v_path"] = os.path.join(td, "v.pkl")
            with open(kw["pretrained_v_path"], "wb") as f:
                pickle.dump(dict(zip(pretrained[0], pretrained[1])), f)
        for seed in seeds:
            np.random.seed(seed)
            random.seed(seed)
            with contextlib.redirect_stdout(io.StringIO()):
                if variant == "unified":
                    model = cls(map_array, sff_path, N, learning_mode=mode, params=dict(params), **kw)
                else:
                    model = cls(map_array, sff_path, N, params=dict(params), **kw)
            for ep in range(n_ep):
                if ep > 0:
                    if reload_v:
                        model.set_v_table(model.get_v_table())
                    model.reset()
                e = 0.0 if eps_sched is None else float(eps_sched[ep])
                if eps_sched is not None:
                    model.set_epsilon(e)
                eps_list.append(e)
                p0 = model.positions
                init.append((p0[:, 0] * W + p0[:, 1]).astype(np.int64))
                steps = 0
                while model.positions.shape[0] > 0 and steps < max_steps:
                    model.step()
                    steps += 1
                    p = model.positions
                    counts.append(p.shape[0])
                    cells.extend((p[:, 0] * W + p[:, 1]).astype(np.int64).tolist())
                    hashes.append(dff_hash(model.dff))
                nsteps.append(steps)
            V = model.get_v_table()
            vk.extend(pack_key(variant, k) for k in V.keys())
            vv.extend(float(v) for v in V.values())
            vn.append(len(V))
            Ht = model.get_h_table() if hasattr(model, "get_h_table") else None
            if Ht:
                hk.extend(pack_key(variant, k) for k in Ht.keys())
                hv.extend(list(map(float, r)) for r in Ht.values())
                hn.append(len(Ht))
            else:
                hn.append(0)
            bg = np.random.mtrand._rand._bit_generator
            np_tail.append(np.asarray(bg.random_raw(4), dtype=np.uint32))
            py_tail.append(np.asarray([random.getrandbits(32) for _ in range(4)], dtype=np.uint32))
    cdt = np.int16 if H * W <= 32767 and N <= 32767 else np.int32   # cells of a 256x256 map need 17 bits
    out = dict(
        map=map_array.astype(np.uint8), sff=sff, params=json.dumps(params), variant=variant,
        mode=mode or "", N=np.int32(N), seeds=np.asarray(seeds, np.int64), n_ep=np.int32(n_ep),
        max_steps=np.int32(max_steps), reload_v=np.int32(reload_v), eps=np.asarray(eps_list),
        init=np.concatenate(init).astype(cdt), init_n=np.asarray([len(i) for i in init], np.int32),
        nsteps=np.asarray(nsteps, np.int32), counts=np.asarray(counts, cdt),
        cells=np.asarray(cells, cdt), dff_hash=np.asarray(hashes, np.uint64),
        v_keys=np.asarray(vk, np.uint64), v_vals=np.asarray(vv, np.float64), v_n=np.asarray(vn, np.int64),
        h_keys=np.asarray(hk, np.uint64),
        h_vals=np.asarray(hv, np.float64).reshape(-1, 9 if params.get("neighborhood") == "moore" else 5),
        h_n=np.asarray(hn, np.int64), np_tail=np.stack(np_tail), py_tail=np.stack(py_tail),
    )
    if pretrained is not None:
        out["pre_keys"] = np.asarray([pack_key(variant if variant == "unified" else "ac", pickle.loads(k))
                                      if variant == "unified" else K.from_cells_bytes(k)
                                      for k in pretrained[0]], np.uint64)
        out["pre_vals"] = np.asarray(pretrained[1], np.float64)
    path = os.path.join(HERE, f"learn_{name}.npz")
    np.savez_compressed(path, **out)
    print(f"{name}: seeds={len(seeds)} episodes={len(nsteps)} steps={sum(nsteps)} |V|={vn} |H|={hn} "
          f"-> {os.path.getsize(path)} B")


def run_trained_case(name, cls, map_array, sff, params, N, seeds, n_ep, max_steps, h_table):
    """model/ffm_trained_core.py driven like run_trained_ffm.py:213-295: per episode
    model.N, model.positions = model.initialize_agents(), model.dff = zeros, run."""
    H, W = map_array.shape
    width = 9 if params.get("neighborhood") == "moore" else 5
    init, nsteps, counts, cells, hashes, np_tail, py_tail = [], [], [], [], [], [], []
    with tempfile.TemporaryDirectory() as td:
        sff_path = os.path.join(td, "sff.npy")
        np.save(sff_path, sff)
        h_path = os.path.join(td, "h.pkl")
        with open(h_path, "wb") as f:      # bytes keys: the loader calls pickle.loads on them (:55-68)
            pickle.dump({pickle.dumps(k): list(v) for k, v in h_table.items()}, f)
        for seed in seeds:
            np.random.seed(seed)
            random.seed(seed)
            with contextlib.redirect_stdout(io.StringIO()):
                model = cls(map_array, sff_path, N, h_path, params=dict(params))
            for ep in range(n_ep):
                if ep > 0:
                    model.positions = model.initialize_agents()
                    model.dff = np.zeros_like(model.map_array, dtype=np.float32)
                p0 = model.positions
                init.append((p0[:, 0] * W + p0[:, 1]).astype(np.int16))
                steps = 0
                while model.positions.shape[0] > 0 and steps < max_steps:
                    model.step()
                    steps += 1
                    p = model.positions
                    counts.append(p.shape[0])
                    cells.extend((p[:, 0] * W + p[:, 1]).astype(np.int16).tolist())
                    hashes.append(dff_hash(model.dff))
                nsteps.append(steps)
            bg = np.random.mtrand._rand._bit_generator
            np_tail.append(np.asarray(bg.random_raw(4), dtype=np.uint32))
            py_tail.append(np.asarray([random.getrandbits(32) for _ in range(4)], dtype=np.uint32))
    out = dict(
        map=map_array.astype(np.uint8), sff=sff, params=json.dumps(params), variant="trained", mode="",
        N=np.int32(N), seeds=np.asarray(seeds, np.int64), n_ep=np.int32(n_ep), max_steps=np.int32(max_steps),
        reload_v=np.int32(0), eps=np.zeros(len(nsteps)),
        init=np.concatenate(init).astype(np.int16), init_n=np.asarray([len(i) for i in init], np.int32),
        nsteps=np.asarray(nsteps, np.int32), counts=np.asarray(counts, np.int16),
        cells=np.asarray(cells, np.int16), dff_hash=np.asarray(hashes, np.uint64),
        v_keys=np.zeros(0, np.uint64), v_vals=np.zeros(0, np.float64), v_n=np.zeros(len(seeds), np.int64),
        h_keys=np.zeros(0, np.uint64), h_vals=np.zeros((0, width), np.float64), h_n=np.zeros(len(seeds), np.int64),
        np_tail=np.stack(np_tail), py_tail=np.stack(py_tail),
        pre_h_keys=np.asarray([K.from_rank_tuple(k) for k, v in h_table.items() if len(v) == width], np.uint64),
        pre_h_vals=np.asarray([list(map(float, v)) for v in h_table.values() if len(v) == width],
                              np.float64).reshape(-1, width),
    )
    odd = [(k, v) for k, v in h_table.items() if len(v) != width]
    if odd:   # rows of another length: scored as missing, counted in the min / max (:228-267)
        out["pre_h_odd_keys"] = np.asarray([K.from_rank_tuple(k) for k, _ in odd], np.uint64)
        out["pre_h_odd_lens"] = np.asarray([len(v) for _, v in odd], np.int32)
        out["pre_h_odd_vals"] = np.asarray([float(x) for _, v in odd for x in v], np.float64)
    path = os.path.join(HERE, f"learn_{name}.npz")
    np.savez_compressed(path, **out)
    print(f"{name}: seeds={len(seeds)} episodes={len(nsteps)} steps={sum(nsteps)} |H|={len(h_table)} "
          f"-> {os.path.getsize(path)} B")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--only", default="", help="comma-separated case names to (re)generate")
    args = ap.parse_args()
    only = set(filter(None, args.only.split(",")))
    sys.path.insert(0, args.ref)
    from model.ffm_ac_core import FloorFieldModel as AC
    from model.ffm_unified import FloorFieldModelUnified as UNI
    from model.ffm_actor_only import FloorFieldModelActorOnly as AO
    from model.ffm_trained_core import FloorFieldModel as TR

    global run_case
    _run = run_case

    def run_case(name, *a, **kw):        # noqa: F811 -- filter by --only
        if not only or name in only:
            _run(name, *a, **kw)

    z = np.load(os.path.join(HERE, "room_12x12_reference.npz"))
    m12, s12 = z["map"], z["sff"]
    # ffm_ac_core with its class defaults (k_S 10, block 3), then the set_v_table quirk.
    run_case("ac_12x12_N8", "ac", AC, m12, s12, {}, 8, [0, 1, 2], 3, 400)
    run_case("ac_12x12_N32_reload", "ac", AC, m12, s12, {"k_S": 3, "block_size": 5}, 32, [3, 4], 3, 400,
             reload_v=True)
    # ffm_ac_core with the Moore neighbourhood (model/ffm_ac_core.py:47-60; update_dff's 8 terms)
    run_case("ac_moore_12x12_N16", "ac", AC, m12, s12, {"k_S": 3, "neighborhood": "moore"}, 16, [7, 8], 3, 400)
    # ffm_unified, run_unified_*_training.py parameters (block 1) and class defaults (block 5)
    uni_p = {"k_S": 10, "k_D": 1, "k_A": 10, "alpha_v": 0.01, "alpha_h": 0.1, "gamma": 0.99,
             "exit_reward": 100.0, "step_penalty": -1.0, "collision_penalty": -1.0,
             "neighborhood": "neumann", "block_size": 1}
    run_case("unified_critic_12x12_N16", "unified", UNI, m12, s12, uni_p, 16, [5, 6], 3, 300,
             mode="critic_only")
    run_case("unified_critic_12x12_N40_bs5", "unified", UNI, m12, s12, {}, 40, [7], 2, 300,
             mode="critic_only")
    eps = np.linspace(0.2, 0.01, 4)
    run_case("unified_actor_12x12_N16", "unified", UNI, m12, s12, uni_p, 16, [8, 9], 4, 300,
             mode="actor_only", eps_sched=eps)
    run_case("unified_both_12x12_N24", "unified", UNI, m12, s12, dict(uni_p, block_size=5), 24, [10], 4, 300,
             mode="both", eps_sched=eps)
    run_case("unified_actor_12x12_N30_eps0", "unified", UNI, m12, s12, uni_p, 30, [11], 3, 300,
             mode="actor_only")
    # ffm_actor_only, run_actor_only_training.py parameters (no pretrained critic)
    ao_p = {"k_D": 1, "k_A": 10, "alpha_v": 0.1, "alpha_h": 0.1, "gamma": 0.95, "exit_reward": 100.0,
            "step_penalty": 0.0, "collision_penalty": -1.0, "neighborhood": "neumann"}
    run_case("actoronly_12x12_N16", "actor_only", AO, m12, s12, ao_p, 16, [12, 13], 4, 300,
             eps_sched=eps)
    run_case("actoronly_12x12_N32_eps0", "actor_only", AO, m12, s12, ao_p, 32, [14], 2, 300)
    # the Moore neighbourhood (model/ffm_unified.py:173-185, model/ffm_actor_only.py:87-93):
    # nine moves, 9-value H rows, 8-term update_dff; ffm_actor_only's inner loop then
    # makes up to eight decisions per agent
    mo = {"neighborhood": "moore"}
    run_case("unified_moore_critic_12x12_N16", "unified", UNI, m12, s12, dict(uni_p, **mo), 16, [23, 24], 3, 300,
             mode="critic_only")
    run_case("unified_moore_actor_12x12_N16", "unified", UNI, m12, s12, dict(uni_p, **mo), 16, [25, 26], 4, 300,
             mode="actor_only", eps_sched=eps)
    run_case("unified_moore_both_12x12_N20", "unified", UNI, m12, s12, dict(uni_p, block_size=5, **mo), 20, [27], 4,
             300, mode="both", eps_sched=eps)
    run_case("actoronly_moore_12x12_N16", "actor_only", AO, m12, s12, dict(ao_p, **mo), 16, [28, 29], 4, 300,
             eps_sched=eps)

    # BASELINE config-5 geometry (256x256 room, 8,192 agents, block 1, the
    # run_unified_actor_training.py parameters), truncated: every reference step
    # rebuilds an O(N) occupied set per agent (model/ffm_unified.py:297-299) and
    # the actor scans the whole H table per agent (:413-422).
    from ffm_amd.data import make_room, l1_sff
    m256 = make_room(256, 256)
    s256 = l1_sff(m256)
    run_case("unified_critic_256x256_N8192", "unified", UNI, m256, s256, uni_p, 8192, [21], 1, 20,
             mode="critic_only")
    run_case("unified_actor_256x256_N8192", "unified", UNI, m256, s256, uni_p, 8192, [22], 1, 3,
             mode="actor_only", eps_sched=[0.2])

    # pretrained critics (the drivers' pretrained_v_path): a critic recorded by the
    # reference itself, pickled with bytes keys like the critic-training scripts
    # write them; ffm_unified re-keys them to tuples and uses them, ffm_actor_only's
    # tuple keys never meet its bytes keys (model/ffm_actor_only.py:59-64).
    np.random.seed(99)
    random.seed(99)
    with tempfile.TemporaryDirectory() as td, contextlib.redirect_stdout(io.StringIO()):
        sp = os.path.join(td, "s.npy")
        np.save(sp, s12)
        cu = UNI(m12, sp, 16, learning_mode="critic_only", params=dict(uni_p))
        for _ in range(3):
            cu.reset()
            cu.run(max_steps=300)
        Vu = cu.get_v_table()
        ca = AC(m12, sp, 16, params={"k_S": 3, "block_size": 5})
        for _ in range(3):
            ca.reset()
            ca.run(max_steps=300)
        Va = ca.get_v_table()
    pre_u = ([pickle.dumps(k) for k in Vu.keys()], [float(v) for v in Vu.values()])
    pre_a = (list(Va.keys()), [float(v) for v in Va.values()])
    run_case("unified_actor_pretrained_12x12_N16", "unified", UNI, m12, s12, uni_p, 16, [15], 3, 300,
             mode="actor_only", eps_sched=eps, pretrained=pre_u)
    run_case("actoronly_pretrained_12x12_N16", "actor_only", AO, m12, s12, ao_p, 16, [16], 3, 300,
             eps_sched=eps, pretrained=pre_a)

    # ffm_trained_core with an H trained by the reference's unified actor
    # (run_trained_ffm.py loads such a table, :141-203)
    if not only or {"trained_12x12_N24", "trained_12x12_N40_bs5", "trained_oddrows_12x12_N24"} & only:
        np.random.seed(17)
        random.seed(17)
        with tempfile.TemporaryDirectory() as td, contextlib.redirect_stdout(io.StringIO()):
            sp = os.path.join(td, "s.npy")
            np.save(sp, s12)
            tables = {}
            for bs in (1, 5):
                ua = UNI(m12, sp, 24, learning_mode="both", params=dict(uni_p, block_size=bs))
                for ep in range(6):
                    ua.set_epsilon(0.2)
                    ua.reset()
                    ua.run(max_steps=200)
                tables[bs] = ua.get_h_table()
        tr_p = {"k_D": 1, "k_A": 10, "neighborhood": "neumann", "block_size": 1}
        if not only or "trained_12x12_N24" in only:
            run_trained_case("trained_12x12_N24", TR, m12, s12, tr_p, 24, [18, 19], 3, 300, tables[1])
        if not only or "trained_12x12_N40_bs5" in only:
            run_trained_case("trained_12x12_N40_bs5", TR, m12, s12, {}, 40, [20], 3, 300, tables[5])
        if not only or "trained_oddrows_12x12_N24" in only:
            # rows of other lengths (model/ffm_trained_core.py:228-249): every fourth state's
            # row shortened or lengthened, with the table's extremes among them; a few states
            # the actor never stored; one empty row
            rs = np.random.RandomState(31)
            t1 = dict(tables[1])
            vals = np.concatenate([np.asarray(v, np.float64) for v in t1.values()])
            lo, hi = float(vals.min()), float(vals.max())
            for i, k in enumerate(list(t1)):
                if i % 4 == 1:
                    n = int(rs.choice([1, 3, 4, 6, 9]))
                    t1[k] = [float(x) for x in rs.uniform(lo, hi, n)]
            ks = list(t1)
            t1[ks[2]] = [hi + 7.5, 0.25, lo]
            t1[ks[6]] = [lo - 3.25]
            t1[ks[10]] = []
            for c in range(6):
                t1[((3, 3, c % 4, (c + 1) % 4), (100 + c, 200 - c))] = [float(x) for x in rs.uniform(lo, hi, 2)]
            run_trained_case("trained_oddrows_12x12_N24", TR, m12, s12, tr_p, 24, [24, 25], 3, 300, t1)

    # ffm_trained_core with the Moore neighbourhood (:76-85, nine-value rows :228-236), driven
    # by the nine-value H of a Moore unified actor
    if not only or "trained_moore_12x12_N20" in only:
        np.random.seed(23)
        random.seed(23)
        with tempfile.TemporaryDirectory() as td, contextlib.redirect_stdout(io.StringIO()):
            sp = os.path.join(td, "s.npy")
            np.save(sp, s12)
            ua = UNI(m12, sp, 20, learning_mode="both", params=dict(uni_p, block_size=1, neighborhood="moore"))
            for ep in range(6):
                ua.set_epsilon(0.2)
                ua.reset()
                ua.run(max_steps=200)
            table_m = ua.get_h_table()
        assert all(len(v) == 9 for v in table_m.values())
        run_trained_case("trained_moore_12x12_N20", TR, m12, s12,
                         {"k_D": 1, "k_A": 10, "neighborhood": "moore", "block_size": 1}, 20, [21, 22], 3, 300,
                         table_m)


if __name__ == "__main__":
    main()
