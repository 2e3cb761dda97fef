"""Build diagnostic variants of the library with FFM_ABLATE bits (see core_step.hip)."""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ffm_amd import build as B  # noqa: E402

pad = int(os.environ.get("FFM_LDS_PAD", "0"))
masks = [int(x) for x in sys.argv[1:]] or [0, 1, 2, 4, 64, 128, 256, 128 | 256, 1 | 2, 1 | 2 | 4 | 64]
root = os.path.join(os.path.dirname(B.HERE), "build_abl")
for f in os.listdir(root) if os.path.isdir(root) else []:
    if f.startswith("libffm_amd_abl"):
        os.remove(os.path.join(root, f))
with ThreadPoolExecutor(4) as ex:
    list(ex.map(lambda m: B.build(out=os.path.join(root, f"libffm_amd_abl{m}.so"),
                                  defines=[f"FFM_ABLATE={m}", f"FFM_LDS_PAD={pad}"]), masks))
print("built", masks, "pad", pad)
