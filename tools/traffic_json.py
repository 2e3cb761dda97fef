"""Per-launch HBM bytes of the step kernel (configs 2, 3) or of the learner's batch
kernel (configs 4, 5) from the two PMC passes of tools/traffic.sh.

FETCH_SIZE / WRITE_SIZE are in KiB.  gfx950 correction (MI355X_MICROARCH.md,
HBM/rocprofv3 section): FETCH_SIZE counts 128-B streaming requests at 64 B, so
it is doubled; WRITE_SIZE is exact for 16-B-per-lane stores.
"""
import csv
import json
import time
import os
import sys

out = sys.argv[1]
args = sys.argv[2:]


def arg(name, default):
    return args[args.index(name) + 1] if name in args else default


cfg = int(arg("--config", 2))
KERNELS = ("learn_batch_kernel",) if cfg in (4, 5) else ("core_group_kernel", "core_lane_kernel", "core_wave_kernel", "core_block_kernel")


def per_dispatch(path, counter):
    vals = []
    for root, _, files in os.walk(path):
        for f in files:
            if f.endswith("counter_collection.csv"):
                with open(os.path.join(root, f)) as fh:
                    for r in csv.DictReader(fh):
                        if any(k in r["Kernel_Name"] for k in KERNELS):
                            if r["Counter_Name"] == counter:
                                vals.append(float(r["Counter_Value"]))
    return vals


f = per_dispatch(os.path.join(out, "fetch"), "FETCH_SIZE")
w = per_dispatch(os.path.join(out, "write"), "WRITE_SIZE")
f = f[10:] or f   # drop the warmup launches
w = w[10:] or w
fk = sum(f) / len(f)
wk = sum(w) / len(w)

dS, dA, dE = {2: (12, 32, 65536), 3: (64, 512, 8192), 4: (12, 32, 65536), 5: (256, 8192, 512)}[cfg]
E = int(arg("--envs", dE)); S = int(arg("--size", dS)); A = int(arg("--agents", dA))
alg = E * 2 * (2 * A + 4 * S * S + 4)
if cfg in (4, 5):      # bench.py learner_bytes_per_env_step
    alg += E * A * (2 * 16 + 16 + (8 + 40 + 16))
res = {
    "config": f"{S}x{S}_A{A}_E{E}" + (f"_learn{cfg}" if cfg in (4, 5) else ""),
    "hbm_bytes_per_launch": 2 * fk * 1024 + wk * 1024,
    "fetch_size_kib_raw": fk, "write_size_kib_raw": wk,
    "read_bytes_corrected": 2 * fk * 1024, "write_bytes": wk * 1024,
    "algorithmic_bytes_per_launch": alg,
    "launches": [len(f), len(w)],
    "correction": "FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM/rocprofv3 section); WRITE_SIZE as is",
}
res["traffic_over_algorithmic"] = res["hbm_bytes_per_launch"] / alg
if cfg in (4, 5):
    # the whole learning step: every step kernel's mean bytes per launch (batch, tile / apply /
    # post passes, stencil, reset), summed -- FETCH x2 + WRITE as above
    def by_kernel(path, counter):
        acc = {}
        for root, _, files in os.walk(path):
            for fn in files:
                if fn.endswith("counter_collection.csv"):
                    with open(os.path.join(root, fn)) as fh:
                        for r in csv.DictReader(fh):
                            if r["Counter_Name"] == counter and "learn_" in r["Kernel_Name"]:
                                name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
                                acc.setdefault(name, []).append(float(r["Counter_Value"]))
        return {k: sum(v[10:] or v) / len(v[10:] or v) for k, v in acc.items()}
    fb, wb = by_kernel(os.path.join(out, "fetch"), "FETCH_SIZE"), by_kernel(os.path.join(out, "write"), "WRITE_SIZE")
    per = {k: 2 * fb.get(k, 0.0) * 1024 + wb.get(k, 0.0) * 1024 for k in set(fb) | set(wb)}
    res["per_kernel_bytes_per_launch"] = per
    res["note"] = ("per-kernel means include kernels that do not run every step (resets); "
                   "hbm_bytes_per_launch is learn_batch_kernel's")
    # FETCH_SIZE counts random 64-B lines once and streams / 128-B lines half
    # (profiles/r05/fetch_calibration.json): the batch kernel mixes both
    lo = fk * 1024 + wk * 1024
    res["hbm_bytes_per_launch_if_all_reads_random_64B"] = lo
    res["traffic_over_algorithmic_range"] = [lo / alg, res["traffic_over_algorithmic"]]
    res["calibration"] = ("profiles/r05/fetch_calibration.json (tools/fetchbench.hip, 2 GiB table, every line "
                          "once): FETCH_SIZE = 0.5 x the bytes of 16-B/lane streaming reads and of random 128-B "
                          "lines, 1.0 x the bytes of random 64-B lines, 64 B per random 8-B or 16-B read. This "
                          "kernel mixes streamed bytes (x2) with random 64-B table lines (x1), so its traffic lies "
                          "in traffic_over_algorithmic_range; hbm_bytes_per_launch keeps the x2 upper bound.")
res["measured"] = os.environ.get("FFM_MEASURED", time.strftime("%Y-%m-%d"))   # e.g. "round 6, <commit>"
print(json.dumps(res, indent=1))
with open(os.path.join(out, "traffic.json"), "w") as fh:
    json.dump(res, fh, indent=1)
