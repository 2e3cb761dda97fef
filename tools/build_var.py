"""Diagnostic / A-B variants of one kernel source: python tools/build_var.py [--src core_group.hip]
name:DEF=1,DEF2=3 ...  -> lad/libffm_amd_<name>.so (only that source recompiled with the defines,
the product objects for the rest; lad/ travels to the GPU box).  Prints each variant's VGPR /
SGPR / spill / occupancy lines of the product kernels from a -S listing."""
import os
import re
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ffm_amd import build as B  # noqa: E402

args = sys.argv[1:]
src = "core_group.hip"
if args and args[0] == "--src":
    src, args = args[1], args[2:]
specs = []
for a in args:
    name, _, defs = a.partition(":")
    specs.append((name, [d for d in defs.split(",") if d]))
root = os.path.join(os.path.dirname(B.HERE), "lad")
B.build()


def one(spec):
    name, defs = spec
    B.build(out=os.path.join(root, f"libffm_amd_{name}.so"), defines=defs, only=[src])
    lst = os.path.join("/tmp", f"var_{name}.s")
    flags = [f for f in B.FLAGS if f not in ("-shared", "-fPIC")]
    subprocess.run([os.environ.get("HIPCC", "/opt/rocm/bin/hipcc"), *flags, *[f"-D{d}" for d in defs],
                    "--cuda-device-only", "-S", "-o", lst, os.path.join(B.CSRC, src)], check=True,
                   stderr=subprocess.DEVNULL)
    txt = open(lst).read()
    out = []
    for m in re.finditer(r"^(_Z\S*kernel\S*):.*?; NumVgprs: (\d+).*?; ScratchSize: (\d+).*?; Occupancy: (\d+)", txt,
                         re.S | re.M):
        out.append(f"  {m.group(1)[:70]} vgpr={m.group(2)} scratch={m.group(3)} occ={m.group(4)}")
    return name, out


with ThreadPoolExecutor(4) as ex:
    for name, out in ex.map(one, specs):
        print(name)
        print("\n".join(out[:4]))
