"""Two-stream decode diagnostics (pt-224, B=1): graph-replayed and eager ms/token with PG_DECODE_BANK on / off, and
the gate/up bank kernel's in-kernel stamps (start, wait satisfied, pairs done, end per workgroup) of one replayed
step, per layer relative to the step's first stamp."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "paligemma-multimodal-system_amd")]
import torch  # noqa: E402

from pghip import _lib, configs, engine, synthetic, weights  # noqa: E402
import bench  # noqa: E402

cfg = configs.CONFIGS["pt-224"]
eng = engine.PaliGemmaEngine(cfg, weights.PackedWeights(cfg, synthetic.SyntheticStateDict(cfg).__getitem__))
ids, px = bench.synthetic_inputs(cfg, 1, [2, 651, 4906, 603, 476, 2121, 576, 108])
ids, px = ids.cuda(), px.cuda()


def run(bank: bool, graph: bool, steps: int = 60, stamps=None):
    eng.DECODE_BANK = bank
    eng.DECODE_SPLIT_KEYS_SMALL = eng.BANK_SPLIT_KEYS
    eng.graphs.clear()
    T = steps + 1
    cache, feats, logits, nxt = eng.prefill_request(ids, px, torch.ones_like(ids), T + 8)
    sampler = dict(do_sample=False)
    st = eng.decode_state(1, cache, nxt, T + 8, sampler=sampler)
    eng.sample(logits, st, sampler, advance=False, feats=feats)
    if stamps is not None:
        _lib.load().pg_gateup_bank_stamps(stamps.data_ptr())
    fn = eng._graph_step(st, cache, feats, sampler) if graph else (lambda: eng.decode_step(st, cache, feats, sampler))
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps - 1):
        fn()
    e1.record()
    torch.cuda.synchronize()
    if stamps is not None:
        _lib.load().pg_gateup_bank_stamps(None)
    eng.check()
    return e0.elapsed_time(e1) / (steps - 1), st["hist"][:12, 0].tolist()


out = {}
for graph in (True, False):
    for bank in (False, True, False, True):
        ms, ids16 = run(bank, graph)
        out.setdefault(f"{'graph' if graph else 'eager'}_bank{int(bank)}", []).append(round(ms, 4))
        print(json.dumps({"graph": graph, "bank": bank, "ms_per_token": round(ms, 4), "ids": ids16}), flush=True)
stamps = torch.zeros(64 * 256 * 4, dtype=torch.int64, device="cuda")
run(True, True, steps=4, stamps=stamps)
s = stamps.view(64, 256, 4).cpu()
# the capture used slots 18..35 (the warm-up step 0..17); every replay rewrote them: the last replay's values
lay = s[18:36].double()
t0 = lay[0, :, 0].min()
print("layer  start_min start_med  wait_med  wait_max  pairs_med  end_med  end_max   (us from layer 0's first start)")
for l in range(18):
    v = (lay[l] - t0) / 100.0
    med = v.median(0).values
    print(f"{l:5d} {v[:, 0].min():9.2f} {med[0]:9.2f} {med[1]:9.2f} {v[:, 1].max():9.2f} {med[2]:9.2f} {med[3]:9.2f} "
          f"{v[:, 3].max():8.2f}")
print(json.dumps(out))
