"""Diagnostic builds of the C2 group kernel's skeleton ladder (core_group.hip FFM_GROUP_LADDER
0-3; 4 is the product).  Only core_group.hip is recompiled; the other objects come from the
product build.  Output: lad/libffm_amd_lad<n>.so (timing only: results are invalid)."""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ffm_amd import build as B  # noqa: E402

levels = [int(x) for x in sys.argv[1:]] or [0, 1, 2, 3]
extra = os.environ.get("FFM_LADDER_DEFINES", "").split()
root = os.path.join(os.path.dirname(B.HERE), "lad")   # shipped to the GPU box (build_abl is not)
B.build()
with ThreadPoolExecutor(4) as ex:
    list(ex.map(lambda n: B.build(out=os.path.join(root, f"libffm_amd_lad{n}.so"),
                                  defines=[f"FFM_GROUP_LADDER={n}", *extra], only=["core_group.hip"]), levels))
print("built ladder", levels)
