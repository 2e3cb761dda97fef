#!/usr/bin/env python3
"""Per-configuration episode-length statistics of the reference's logged unified
actor_only run (container only; the reference does not travel):

    python tests/golden/gen_actor_log_stats.py [--ref /root/reference]

Reads output/logs/unified_actor_training/run_20260119_070834/steps_per_episode.csv
(100 episodes per (radius, N), the curriculum of run_unified_actor_training.py) and
writes ref_unified_actor_run_20260119_070834.json: for every configuration the
episode count, mean steps, standard deviation and standard error of the mean.
"""
import argparse
import csv
import json
import math
import os
from collections import defaultdict

HERE = os.path.dirname(os.path.abspath(__file__))
RUN = "output/logs/unified_actor_training/run_20260119_070834/steps_per_episode.csv"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    a = ap.parse_args()
    by = defaultdict(list)
    with open(os.path.join(a.ref, RUN)) as f:
        for r in csv.DictReader(f):
            by[(int(r["radius"]), int(r["N"]))].append(int(r["steps"]))
    out = []
    for (radius, n), xs in sorted(by.items()):
        m = sum(xs) / len(xs)
        sd = math.sqrt(sum((x - m) ** 2 for x in xs) / (len(xs) - 1))
        out.append({"radius": radius, "N": n, "episodes": len(xs), "mean_steps": m, "std_steps": sd,
                    "se": sd / math.sqrt(len(xs))})
    path = os.path.join(HERE, "ref_unified_actor_run_20260119_070834.json")
    with open(path, "w") as f:
        json.dump({"source": RUN, "configs": out}, f, indent=1)
    print(f"{len(out)} configurations -> {path}")


if __name__ == "__main__":
    main()
