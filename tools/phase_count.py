"""Static instruction mix per phase of the C2 wave kernel (diagnostic).

Compiles core_step.hip with -DFFM_MARKS (asm markers at the STAMP points) and
counts VALU / SALU / LDS / VMEM instructions between consecutive markers.
Rarely-taken branches inside a phase are counted too (static, not dynamic).
"""
import re
import subprocess
import sys

args = sys.argv[1:]
src = args[0] if args else "ffm_amd/csrc/core_step.hip"
extra = args[1:]
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                "-fno-gpu-flush-denormals-to-zero", "-fhip-fp32-correctly-rounded-divide-sqrt", "--cuda-device-only",
                "-S", "-DFFM_MARKS", *extra, src, "-o", "/tmp/phase.s"], check=True, capture_output=True)
s = open("/tmp/phase.s").read()
name = "_ZN3ffm16core_wave_kernelILi4ELb0ELi2ELi12ELi12EEEvNS_12CoreStepArgsE"
i = s.index(name + ":")
body = s[i:s.index(".Lfunc_end", i)].splitlines()
names = {0: "load/pp", 1: "marks", 2: "decide", 3: "rq write", 4: "resolve", 5: "compaction",
         6: "stencil", 7: "stage/store/reset"}
cur = "pre-loop"
counts = {}
for l in body:
    t = l.strip()
    m = re.search(r"@PHASE (\d+)", t)
    if m:
        cur = names[int(m.group(1))] + f" (<{m.group(1)})"
        continue
    if not t or t.startswith((";", ".")) or t.endswith(":"):
        continue
    op = t.split()[0]
    k = ("valu" if op.startswith("v_") else "salu" if op.startswith("s_") else "lds" if op.startswith("ds_")
         else "vmem" if op.startswith(("global_", "buffer_", "flat_")) else "other")
    c = counts.setdefault(cur, {})
    c[k] = c.get(k, 0) + 1
for k, v in counts.items():
    print(f"{k:28s} " + " ".join(f"{a}={v.get(a, 0):4d}" for a in ("valu", "salu", "lds", "vmem")))
