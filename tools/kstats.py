"""Mean duration per kernel from a rocprofv3 kernel trace, skipping each kernel's
first `skip` dispatches (warmup).  python tools/kstats.py run_kernel_trace.csv [skip]"""
import csv
import sys
from collections import defaultdict

skip = int(sys.argv[2]) if len(sys.argv) > 2 else 0
d = defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"].replace("ffm::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    d[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    w = v[skip:] if len(v) > skip else v
    print(f"{k:60s} n={len(w):4d} mean={sum(w) / len(w):9.1f} us min={min(w):8.1f} max={max(w):8.1f}")
