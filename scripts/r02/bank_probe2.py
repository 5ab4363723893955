"""Two-stream decode timeline (pt-224, B=1, graph-replayed): ms/token for the variant the environment selects
(PG_DECODE_BANK, PG_BANK_INFL, PG_BANK_QKV_WAIT), then per layer the workgroup start / end stamps of the q|k|v,
o_proj and down GEMVs (pg_gemv_stamps) and of the gate/up bank kernel (start, wait satisfied, end), in us from
layer 0's first q|k|v start."""
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
eng.DECODE_SPLIT_KEYS_SMALL = eng.BANK_SPLIT_KEYS
ids, px = bench.synthetic_inputs(cfg, 1, [2, 651, 4906, 603, 476, 2121, 576, 108])
ids, px = ids.cuda(), px.cuda()
bank = eng._bank_on(1)


def run(steps, stamps=False):
    eng.graphs.clear()
    T = steps + 1
    cache, feats, logits, nxt = eng.prefill_request(ids, px, torch.ones_like(ids), T + 8)
    sampler = dict(do_sample=False)
    st = eng.decode_state(1, cache, nxt, T + 8, sampler=sampler)
    eng.sample(logits, st, sampler, advance=False, feats=feats)
    if stamps:
        gs = torch.zeros(128 * 2048 * 2, dtype=torch.int64, device="cuda")
        bs = torch.zeros(64 * 256 * 4, dtype=torch.int64, device="cuda")
        _lib.load().pg_gemv_stamps(gs.data_ptr())
        _lib.load().pg_gateup_bank_stamps(bs.data_ptr())
    fn = eng._graph_step(st, cache, feats, sampler)
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps - 1):
        fn()
    e1.record()
    torch.cuda.synchronize()
    eng.check()
    if stamps:
        _lib.load().pg_gemv_stamps(None)
        _lib.load().pg_gateup_bank_stamps(None)
        return gs.view(128, 2048, 2).cpu(), bs.view(64, 256, 4).cpu()
    return e0.elapsed_time(e1) / (steps - 1)


ms = [round(run(60), 4) for _ in range(3)]
print(json.dumps({"bank": bank, "infl": os.environ.get("PG_BANK_INFL", "8"), "qkv_wait": eng.BANK_QKV_WAIT,
                  "ms_per_token": ms}), flush=True)
gs, bs = run(3, stamps=True)
per = 3 if bank else 4                          # gemv launches per layer (one-stream: q|k|v, o, gate/up, down)


def span(slot, nwg):
    v = gs[slot % 128, :nwg].double()
    ok = v[:, 0] > 0
    return v[ok, 0].min(), v[ok, 1].max()


base = 55 if bank else 73
t0 = span(base, 160)[0]
print("layer   qkv_s   qkv_e    o_s     o_e   | G_s    G_wait  G_e  |  down_s  down_e   (us)")
for l in range(18):
    qs, qe = span(base + per * l, 160)
    os_, oe = span(base + per * l + 1, 128)
    ds, de = span(base + per * l + per - 1, 1024)
    row = f"{l:5d} {(qs - t0) / 100:7.2f} {(qe - t0) / 100:7.2f} {(os_ - t0) / 100:7.2f} {(oe - t0) / 100:7.2f} |"
    if bank:
        b = bs[18 + l].double()
        row += f" {(b[:, 0].min() - t0) / 100:7.2f} {(b[:, 1].median() - t0) / 100:7.2f} {(b[:, 3].max() - t0) / 100:7.2f} |"
    else:
        gus, gue = span(base + per * l + 2, 1024)
        row += f" {(gus - t0) / 100:7.2f}       - {(gue - t0) / 100:7.2f} |"
    row += f" {(ds - t0) / 100:7.2f} {(de - t0) / 100:7.2f}"
    print(row)
