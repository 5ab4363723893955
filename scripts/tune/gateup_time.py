"""bench.py's roofline measurement alone (decode gate/up GEMV, 50 launches rotating 18 layers)."""
import json
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "paligemma-multimodal-system_amd")]
import torch  # noqa: E402
import bench  # noqa: E402
from pghip import configs, synthetic, weights  # noqa: E402
cfg = configs.PT_224
w = weights.PackedWeights(cfg, synthetic.SyntheticStateDict(cfg).__getitem__, parts=("text",))


class E:
    pass


e = E()
e.w = w
ts = sorted(bench.time_dominant_kernel(e)[0] for _ in range(5))
print(json.dumps({"lib": os.path.basename(os.environ.get("PGHIP_LIB", "libpghip.so")), "gateup_us": round(ts[2] * 1e6, 2)}))
