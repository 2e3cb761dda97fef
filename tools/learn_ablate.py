"""Build diagnostic variants of the library with FFM_LABLATE bits (learn_step.hip)."""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ffm_amd import build as B  # noqa: E402

masks = [int(x) for x in sys.argv[1:]] or [0, 1, 2, 4, 6, 8]
root = os.path.join(os.path.dirname(B.HERE), "build_abl")
os.makedirs(root, exist_ok=True)
with ThreadPoolExecutor(3) as ex:
    list(ex.map(lambda m: B.build(out=os.path.join(root, f"libffm_amd_labl{m}.so"), defines=[f"FFM_LABLATE={m}"] + os.environ.get("FFM_EXTRA_DEFINES", "").split()),
                masks))
print("built", masks)
