"""Compare batched unified actor curricula (tools/actor_pin.sh output) with the
reference's logged run, per (radius, N): mean steps, and the deviation in units of
the combined standard error sqrt(se_ref^2 + se_ours^2).

    python tools/actor_pin_compare.py <actor_pin dir> [E-tags ...] > comparison.txt
"""
import csv
import json
import math
import os
import sys
from collections import defaultdict

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.path.join(HERE, "..", "tests", "golden", "ref_unified_actor_run_20260119_070834.json")


def ours(path):
    by = defaultdict(list)
    with open(os.path.join(path, "steps_per_episode.csv")) as f:
        for r in csv.DictReader(f):
            by[(int(r["radius"]), int(r["N"]))].append(int(r["steps"]))
    out = {}
    for k, xs in by.items():
        m = sum(xs) / len(xs)
        sd = math.sqrt(sum((x - m) ** 2 for x in xs) / max(1, len(xs) - 1))
        out[k] = (m, sd / math.sqrt(len(xs)), len(xs))
    return out


def main():
    d = sys.argv[1]
    tags = sys.argv[2:] or ["e10", "e512", "e4096", "e4096_nophase"]
    ref = {(c["radius"], c["N"]): c for c in json.load(open(REF))["configs"]}
    runs = {t: ours(os.path.join(d, "actor_" + t)) for t in tags if os.path.exists(os.path.join(d, "actor_" + t))}
    print("unified actor_only curriculum, mean steps per episode; dev = (ours - ref) / sqrt(se_ref^2 + se_ours^2)")
    print("reference: output/logs/unified_actor_training/run_20260119_070834 (100 episodes per configuration)")
    hdr = f"{'radius':>6} {'N':>3} {'ref':>8} {'se':>5}" + "".join(f" | {t:>13} {'n':>5} {'dev':>6}" for t in runs)
    print(hdr)
    summ = {t: [] for t in runs}
    for key in sorted(ref):
        c = ref[key]
        line = f"{key[0]:6d} {key[1]:3d} {c['mean_steps']:8.2f} {c['se']:5.2f}"
        for t, r in runs.items():
            if key not in r:
                line += f" | {'-':>13} {'-':>5} {'-':>6}"
                continue
            m, se, n = r[key]
            dev = (m - c["mean_steps"]) / math.sqrt(c["se"] ** 2 + se ** 2) if (c["se"] or se) else 0.0
            summ[t].append((key, dev, (m - c["mean_steps"]) / c["mean_steps"]))
            line += f" | {m:8.2f}±{se:4.2f} {n:5d} {dev:+6.1f}"
        print(line)
    print()
    for t, rows in summ.items():
        devs = [abs(x[1]) for x in rows]
        rel = [abs(x[2]) for x in rows]
        within = sum(1 for x in devs if x <= 3.0)
        print(f"{t}: {within}/{len(rows)} configurations within 3 SE; median |dev| {sorted(devs)[len(devs) // 2]:.1f} SE; "
              f"median |rel| {100 * sorted(rel)[len(rel) // 2]:.1f} %; max |rel| {100 * max(rel):.1f} %")


if __name__ == "__main__":
    main()
