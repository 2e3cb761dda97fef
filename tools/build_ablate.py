"""Build diagnostic variants of the library with FFM_ABLATE bits (see core_step.hip)."""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ffm_amd import build as B  # noqa: E402

pad = int(os.environ.get("FFM_LDS_PAD", "0"))
# each argument: MASK or MASK:WAVES_PER_EU
specs = sys.argv[1:] or ["0", "1", "2", "4", "64", "128", "256", "384", "3", "71"]
masks = [(int(x.split(":")[0]), int(x.split(":")[1]) if ":" in x else 0) for x in specs]
root = os.path.join(os.path.dirname(B.HERE), "build_abl")
for f in os.listdir(root) if os.path.isdir(root) else []:
    if f.startswith("libffm_amd_abl"):
        os.remove(os.path.join(root, f))
with ThreadPoolExecutor(4) as ex:
    list(ex.map(lambda mw: B.build(out=os.path.join(root, f"libffm_amd_abl{mw[0]}" + (f"_w{mw[1]}" if mw[1] else "") + ".so"),
                                   defines=[f"FFM_ABLATE={mw[0]}", f"FFM_LDS_PAD={pad}", f"FFM_WAVES_PER_EU={mw[1]}"]), masks))
print("built", masks, "pad", pad)
