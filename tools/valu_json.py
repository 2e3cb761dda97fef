"""VALU issue fraction of the step kernel from the counter passes of tools/pmc.sh
(median per dispatch), written as profiles/valu_<H>x<W>_A<A>_E<E>.json for bench.py's
roofline.valu_issue_frac.

    valu_issue_frac = SQ_ACTIVE_INST_VALU / (8 * SQ_BUSY_CYCLES)

Calibration (round 6, tools/alu_pmc.sh, profiles/r06/alu/valu_calibration.json): saturated
microkernels of a known VALU count read 0.995 (v_mul_hi_u32 / v_mul_lo_u32), 1.014
(v_mad_u64_u32) and 0.985 (v_exp_f32), but 1.83 for plain 32-bit xor / add, which issue faster
than one wave-instruction per 4 clocks on gfx950.  So 1.0 is the ceiling only for
multiply / transcendental-bound code, and a mixed kernel can read slightly above 1 while
saturated (C3's 1.02).

SQ_ACTIVE_INST_VALU sums, over every wave, the quad-cycles (4 clocks, one wave64 VALU
instruction on a 16-lane SIMD) it spent issuing VALU; SQ_BUSY_CYCLES sums the busy
clocks of the 32 shader engines of 32 SIMDs each.  Their ratio scaled by 4 * 32 / 1024
= 1/8 is the fraction of an average SIMD's clocks its vector pipe was issuing.  (The
r03 group kernel reads 0.76 this way, its VALU count x 4 clocks against the kernel time
gives the same.)  GRBM_GUI_ACTIVE is kept in the counters; it sums over XCDs and is not
used.

    python tools/valu_json.py <pmc out dir> <H> <W> <A> <E> [kernel substring]
"""
import collections
import csv
import glob
import json
import time
import os
import statistics
import sys

out, H, W, A, E = sys.argv[1], *map(int, sys.argv[2:6])
kern = sys.argv[6] if len(sys.argv) > 6 else "core_group_kernel"
agg = collections.defaultdict(list)
for f in glob.glob(f"{out}/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
med = {k: statistics.median(v[5:] or v) for k, v in agg.items()}
frac = med["SQ_ACTIVE_INST_VALU"] / (8 * med["SQ_BUSY_CYCLES"])
res = {"config": f"{H}x{W}_A{A}_E{E}", "kernel": kern, "valu_issue_frac": frac,
       "valu_per_wave": med["SQ_INSTS_VALU"] / med["SQ_WAVES"], "salu_per_wave": med["SQ_INSTS_SALU"] / med["SQ_WAVES"],
       "lds_per_wave": med["SQ_INSTS_LDS"] / med["SQ_WAVES"],
       "wait_frac": med.get("SQ_WAIT_ANY", 0) / med["SQ_WAVE_CYCLES"] if "SQ_WAVE_CYCLES" in med else None,
       "lds_bank_conflict_frac": (med["SQ_LDS_BANK_CONFLICT"] / med["SQ_LDS_IDX_ACTIVE"]
                                  if "SQ_LDS_IDX_ACTIVE" in med else None),
       "counters": med,
       "formula": "SQ_ACTIVE_INST_VALU / (8 * SQ_BUSY_CYCLES), median per dispatch"}
if frac > 0.97:
    res["note"] = ("saturated: the SIMDs' vector pipes issue on (nearly) every cycle; SQ_INSTS_VALU x 4 "
                   "clocks / 1024 SIMDs = %.0f clocks per SIMD against SQ_BUSY_CYCLES / 32 = %.0f, so a "
                   "value at or just above 1 is counter skew, and the kernel is VALU-issue-bound"
                   % (med["SQ_INSTS_VALU"] * 4 / 1024, med["SQ_BUSY_CYCLES"] / 32))
res["measured"] = os.environ.get("FFM_MEASURED", time.strftime("%Y-%m-%d"))   # e.g. "round 6, <commit>"
path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                    f"valu_{H}x{W}_A{A}_E{E}.json")
with open(path, "w") as f:
    json.dump(res, f, indent=1)
print(json.dumps({k: v for k, v in res.items() if k != "counters"}))
