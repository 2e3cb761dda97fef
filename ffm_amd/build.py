"""Build the HIP extension (libffm_amd.so) in-tree for gfx950.

hipcc drives both the device (gfx950) and host code; the library exports
the C ABI declared in include/ffm_amd.h.  Kernels are compiled with
-ffp-contract=off (NumPy rounds every product and sum separately) and with
IEEE float32 division and denormals, which the bit-exact parity relies on.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB_DIR = os.path.join(HERE, "_lib")
LIB_PATH = os.path.join(LIB_DIR, "libffm_amd.so")
SOURCES = ["core_step.hip", "core_lane.hip", "core_group.hip", "core_multi.hip", "learn_step.hip", "engine.cpp", "learn_engine.cpp"]
HEADERS = ["device_common.h", "core_common.h", "lane_common.h", "wave_reset.h", "kernels.h", "learn_kernels.h", os.path.join("..", "..", "include", "ffm_amd.h")]
ARCH = os.environ.get("FFM_OFFLOAD_ARCH", "gfx950")
FLAGS = [
    f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
    "-ffp-contract=off", "-fno-gpu-flush-denormals-to-zero",
    "-fhip-fp32-correctly-rounded-divide-sqrt", "-Wall",
]


def _stale() -> bool:
    if not os.path.exists(LIB_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)] + [os.path.join(CSRC, h) for h in HEADERS]
    deps.append(os.path.abspath(__file__))
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force: bool = False, verbose: bool = False, out: str | None = None, defines=(), only=None) -> str:
    """Compile the library; `out`/`defines` make diagnostic variants (tools/ablate.sh).
    `only` (with `out`): compile just those sources with the defines and link them with the
    product build's objects of the others (diagnostic builds of one kernel file).

    Each source compiles to its own object in parallel (the kernels' translation
    units are independent), then hipcc links the shared library."""
    from concurrent.futures import ThreadPoolExecutor
    target = out or LIB_PATH
    if out is None and not force and not _stale():
        return LIB_PATH
    os.makedirs(os.path.dirname(target), exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    objdir = target + ".obj"
    os.makedirs(objdir, exist_ok=True)
    cflags = [f for f in FLAGS if f != "-shared"] + [f"-D{d}" for d in defines]

    def compile_one(src):
        obj = os.path.join(objdir, src + ".o")
        cmd = [hipcc, *cflags, "-c", "-o", obj, os.path.join(CSRC, src)]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True, cwd=CSRC)
        return obj

    todo = [src for src in SOURCES if only is None or src in only]
    with ThreadPoolExecutor(max_workers=min(len(SOURCES), os.cpu_count() or 1)) as ex:
        done = dict(zip(todo, ex.map(compile_one, todo)))
    objs = [done.get(src) or os.path.join(LIB_PATH + ".obj", src + ".o") for src in SOURCES]
    tmp = target + ".tmp"
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(tmp, target)
    return target


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
