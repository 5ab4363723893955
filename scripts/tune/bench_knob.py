"""Run bench.py with engine class attributes overridden: python scripts/tune/bench_knob.py ATTR=VALUE [...] -- <bench args>"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "paligemma-multimodal-system_amd")]
from pghip import engine  # noqa: E402

i = sys.argv.index("--")
for kv in sys.argv[1:i]:
    k, v = kv.split("=")
    setattr(engine.PaliGemmaEngine, k, type(getattr(engine.PaliGemmaEngine, k))(v))
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[i + 1:]
runpy.run_path(sys.argv[0], run_name="__main__")
