"""Time the graph-replayed decode step of the engine (pt-224, B=1) for one library build.

    PGHIP_LIB=scripts/tune/var_x.so python scripts/tune/decode_step.py [--split-o 2 --split-down 4 --split-keys 32]

Prints one JSON line: ms/token over --steps replays (median of 5 rounds) and the first greedy ids.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "paligemma-multimodal-system_amd")]
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="pt-224")
ap.add_argument("--steps", type=int, default=100)
ap.add_argument("--split-o", type=int, default=None)
ap.add_argument("--split-down", type=int, default=None)
ap.add_argument("--split-keys", type=int, default=None)
ap.add_argument("--batch", type=int, default=1)
ap.add_argument("--split-target", type=int, default=None)
ap.add_argument("--fp8", action="store_true")
a = ap.parse_args()

from pghip import configs, engine, synthetic, weights  # noqa: E402
import bench  # noqa: E402

cfg = configs.CONFIGS[a.config]
sd = synthetic.SyntheticStateDict(cfg)
eng = engine.PaliGemmaEngine(cfg, weights.PackedWeights(cfg, sd.__getitem__, fp8=a.fp8))
if a.split_o:
    eng.split_o = a.split_o
if a.split_down:
    eng.split_down = a.split_down
if a.split_keys:
    eng.DECODE_SPLIT_KEYS = a.split_keys
if a.split_target:
    eng.DECODE_SPLIT_TARGET = a.split_target
B = a.batch
ids, px = bench.synthetic_inputs(cfg, B, [2, 651, 4906, 603, 476, 2121, 576, 108])
ids, px = ids.cuda(), px.cuda()
T = a.steps + 1
cache, feats, logits, nxt = eng.prefill_request(ids, px, torch.ones_like(ids), T + 8)
sampler = dict(do_sample=False)
st = eng.decode_state(B, cache, nxt, T + 8, sampler=sampler)      # chained unless PG_CHAIN_EMBED=0
eng.sample(logits, st, sampler, advance=False, feats=feats)
replay = eng._graph_step(st, cache, feats, sampler)
snap = {k: st[k].clone() for k in ("ids", "pos", "kv_len", "step")}
times = []
for rnd in range(5):
    for k, v in snap.items():
        st[k].copy_(v)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(a.steps):
        replay()
    e1.record()
    torch.cuda.synchronize()
    times.append(e0.elapsed_time(e1) / a.steps)
ids_out = st["hist"][: a.steps + 1, 0].tolist()
print(json.dumps({"lib": os.path.basename(os.environ.get("PGHIP_LIB", "libpghip.so")), "split_o": eng.split_o,
                  "split_down": eng.split_down, "split_keys": eng.DECODE_SPLIT_KEYS, "B": B,
                  "ms_per_token": round(sorted(times)[2], 4), "all": [round(t, 4) for t in times],
                  "ids16": ids_out[:16]}), flush=True)
