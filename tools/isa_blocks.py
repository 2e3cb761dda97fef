"""Per-basic-block instruction counts of one kernel in a hipcc -S listing (static ISA
view: VALU / SALU / LDS / VMEM per block, branch targets), for reading where a kernel's
issue slots go.  python tools/isa_blocks.py file.s <kernel-symbol-substring>"""
import re
import sys

lines = open(sys.argv[1]).read().split("\n")
key = sys.argv[2]
start = [i for i, l in enumerate(lines) if key in l and l.split(":")[0].strip().startswith("_Z") and ":" in l
         and not l.startswith("\t")][0]
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
blocks, cur = [], ("entry", [])
for l in lines[start + 1:end]:
    m = re.match(r"^(\.LBB\d+_\d+):", l)
    if m:
        blocks.append(cur)
        cur = (m.group(1), [])
        continue
    t = l.strip()
    if not t or t.startswith(";") or t.startswith("."):
        continue
    cur[1].append(t)
blocks.append(cur)
T = [0, 0, 0, 0]
for name, ins in blocks:
    v = sum(1 for x in ins if x.startswith("v_"))
    s_ = sum(1 for x in ins if x.startswith("s_") and not x.startswith(("s_waitcnt", "s_nop")))
    d = sum(1 for x in ins if x.startswith("ds_"))
    g = sum(1 for x in ins if x.startswith(("buffer_", "global_", "flat_")))
    T = [T[0] + v, T[1] + s_, T[2] + d, T[3] + g]
    br = [x.split()[0] + " " + x.split()[-1] for x in ins if x.startswith(("s_cbranch", "s_branch"))]
    print(f"{name:14s} v={v:4d} s={s_:4d} ds={d:3d} vm={g:3d} {' | '.join(br)}")
print("total", T)
