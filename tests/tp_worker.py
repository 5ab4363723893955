"""Rank body of tests/test_tp_gpu.py (launched by torch.distributed.run, 2 ranks on one HIP device,
gloo transport, or pg_allreduce_xgmi with TP_COMM=xgmi): the tensor-parallel engine against the reference's golden
vectors and the single-rank engine.  TP_CFG=tiny (default) uses the tiny fixtures; TP_CFG=pt-224 runs the full-size
PaliGemma-3B-224 (BASELINE configs[3]'s mix-224 architecture) against tests/golden/pt224.npz.  Writes one JSON
verdict per rank to $TP_OUT/rank<r>.json."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "paligemma-multimodal-system_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def err(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def topp_draw_ok(logits, got, T, P, u):
    """The kernel's top-p draw `got` equals the oracle's explicit-uniform inverse-CDF draw (oracle.sample_top_p) from
    logits [V], up to fp32 summation order: the kept set may differ by a token whose mass ranked before it lies
    within 1e-5 of top_p (the reference's torch.cumsum vs the kernel's select), and the draw may fall on either side
    of a CDF step within 1e-6 of the uniform's position."""
    from oracle import paligemma_oracle as O
    if got == int(O.sample_top_p(logits[None], T, P, np.array([u], np.float32))[0, 0]):
        return True
    x = logits.astype(np.float64) / T
    p = np.exp(x - x.max())
    p /= p.sum()
    order = np.argsort(-p, kind="stable")
    before = np.empty_like(p)
    before[order] = np.cumsum(p[order]) - p[order]
    kept = before <= P
    variants = [kept] + [np.where(np.arange(p.size) == t, ~kept, kept) for t in np.nonzero(np.abs(before - P) < 1e-5)[0]]
    for k in variants:
        q = np.where(k, p, 0.0)
        c = np.cumsum(q)
        t = u * c[-1]
        lo = c[got] - q[got]
        if q[got] > 0 and lo - 1e-6 * c[-1] <= t <= c[got] + 1e-6 * c[-1]:
            return True
    return False


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    from pghip import configs, engine, synthetic, weights
    from pghip.tp import TPComm, XgmiComm
    if os.environ.get("TP_CFG", "tiny") != "tiny":
        return full_size(rank, world, os.environ["TP_CFG"])
    cfg = configs.TINY
    sd = synthetic.SyntheticStateDict(cfg)
    comm = XgmiComm(cap=1 << 20) if os.environ.get("TP_COMM") == "xgmi" else TPComm()
    tp = engine.PaliGemmaEngine(cfg, weights.PackedWeights(cfg, sd.__getitem__, tp_rank=rank, tp_world=world),
                                comm=comm)
    solo = engine.PaliGemmaEngine(cfg, weights.PackedWeights(cfg, sd.__getitem__))
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "tiny.npz")))
    out = {"rank": rank, "world": world, "comm": type(comm).__name__, "graph": comm.capturable}
    for B in (1, 2):
        p = f"b{B}_"
        ids = torch.from_numpy(g[p + "input_ids"]).cuda()
        px = torch.from_numpy(g[p + "pixel_values"]).cuda()
        Bv, L = ids.shape
        cache = tp.new_cache(Bv, L + 8)
        resid = torch.empty(Bv * L, tp.w.hidden, device="cuda")
        tp.embed_merge(ids, tp.vision(px), resid)
        pos = torch.arange(1, L + 1, dtype=torch.int32).repeat(Bv, 1)
        logits, _ = tp.gemma_prefill(resid, pos, cache, Bv, L)
        out[f"prefill_err_b{B}"] = err(logits.cpu().numpy(), g[p + "logits"].reshape(Bv * L, -1))
    ids = torch.from_numpy(g["b1_input_ids"]).cuda()
    px = torch.from_numpy(g["b1_pixel_values"]).cuda()
    am = torch.ones_like(ids)
    out["greedy"] = tp.generate(ids, px, am, len(g["greedy_ids"]))[0].tolist()
    out["greedy_ref"] = g["greedy_ids"].tolist()
    # long teacher-forced decode: TP logits (gathered full vocabulary) vs the single-rank engine
    steps = 20
    caches, nxts, feats = [], [], []
    for e in (tp, solo):
        c, f, lg, n = e.prefill_request(ids, px, am, steps)
        caches.append(c), nxts.append(n), feats.append(f)
    st = [e.decode_state(1, c, n, steps) for e, c, n in zip((tp, solo), caches, nxts)]
    worst, agree = 0.0, True
    for t in range(steps - 1):
        tok = 7 + 13 * t
        lgs = []
        for e, s, c, f in zip((tp, solo), st, caches, feats):
            s["ids"].fill_(tok)
            lgs.append(e.decode_step(s, c, f, dict(do_sample=False)).clone())
        if int(st[0]["ids"][0]) != int(st[1]["ids"][0]):
            agree = False
        # the greedy TP path returns the local vocabulary slice; compare it with the same slice
        lo = tp.w.vocab_offset
        worst = max(worst, err(lgs[0].cpu().numpy(), lgs[1][:, lo:lo + tp.w.vocab_local].cpu().numpy()))
    out["decode_slice_err"] = worst
    out["decode_argmax_agree"] = agree
    # top-p sampling with the same uniforms through the gathered logits
    u = torch.rand(9, 1, generator=torch.Generator().manual_seed(3))
    out["sampled_tp"] = tp.generate(ids, px, am, 8, do_sample=True, temperature=0.8, top_p=0.9, uniforms=u,
                                    stop_token=None)[0].tolist()
    out["sampled_solo"] = solo.generate(ids, px, am, 8, do_sample=True, temperature=0.8, top_p=0.9, uniforms=u,
                                        stop_token=None)[0].tolist()
    torch.cuda.synchronize()
    out["xgmi_err"] = int(comm.err.item()) if isinstance(comm, XgmiComm) else 0
    if isinstance(comm, XgmiComm):
        comm.close()
    with open(os.path.join(os.environ["TP_OUT"], f"rank{rank}.json"), "w") as f:
        json.dump(out, f)
    dist.barrier()
    dist.destroy_process_group()


def full_size(rank, world, name):
    """Full-size TP=2 (BASELINE configs[3]: mix-224 = the pt-224 architecture) on one device, on the better-conditioned
    synthetic recipe of tests/golden/pt224wc.npz (whose reference greedy ids have margins >= 0.127): prefill /
    teacher-forced decode logits against the single-rank engine, 32 free-running greedy ids against the reference's,
    and top-p sampling with fixed uniforms (every teacher-forced draw, and the first free-running one, must be the
    explicit-uniform inverse-CDF draw of the gathered logits)."""
    from PIL import Image
    from oracle import paligemma_oracle as O
    from pghip import configs, engine, synthetic, weights
    from pghip.tp import TPComm, XgmiComm
    from processing_paligemma import process_images
    cfg = configs.CONFIGS[name]
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "pt224wc.npz")))
    sd = synthetic.SyntheticStateDict(cfg, linear_gain=float(g["linear_gain"]))
    comm = XgmiComm() if os.environ.get("TP_COMM") == "xgmi" else TPComm()
    tp = engine.PaliGemmaEngine(cfg, weights.PackedWeights(cfg, sd.__getitem__, tp_rank=rank, tp_world=world),
                                comm=comm)
    solo = engine.PaliGemmaEngine(cfg, weights.PackedWeights(cfg, sd.__getitem__))
    img = np.random.default_rng(int(g["seeds"][0])).integers(0, 256, (1, 224, 224, 3), dtype=np.uint8)
    pv = np.stack(process_images([Image.fromarray(img[0])], 224, 1 / 255.0, Image.Resampling.BICUBIC))
    assert np.array_equal(pv.astype(np.float32).reshape(-1)[::9973], g["i0_pixel_sample"])
    ids = torch.from_numpy(g["i0_input_ids"]).cuda()
    px = torch.from_numpy(pv.astype(np.float32)).cuda()
    am = torch.ones_like(ids)
    ref_ids = g["i0_greedy_ids"].tolist()
    out = {"rank": rank, "world": world, "comm": type(comm).__name__, "graph": comm.capturable, "config": name}
    steps = 16
    res = []
    for e in (tp, solo):
        c, f, lg, n = e.prefill_request(ids, px, am, steps + 2)
        res.append((c, f, lg.clone(), n))
    out["prefill_err_vs_solo"] = err(res[0][2].cpu().numpy(), res[1][2].cpu().numpy())
    out["prefill_top1"] = int(res[0][2][0].argmax())
    out["ref_top1"] = ref_ids[0]
    # teacher-forced decode with the reference's ids: the full gathered logits (top-p sampler path) vs single rank
    st = [e.decode_state(1, c, n, steps + 2) for e, (c, f, lg, n) in zip((tp, solo), res)]
    worst, disagree = 0.0, []
    samp = dict(do_sample=True, temperature=0.8, top_p=0.9)
    for t in range(1, steps):
        lgs = []
        for e, s_, (c, f, lg, n) in zip((tp, solo), st, res):
            s_["ids"].fill_(ref_ids[t - 1])
            s_["step"].zero_()
            samp["uniforms"] = torch.full((4, 1), 0.5, device="cuda")
            lgs.append(e.decode_step(s_, c, f, samp).clone())
        a, b = lgs[0][0].cpu().numpy(), lgs[1][0].cpu().numpy()
        worst = max(worst, err(a, b))
        sb = np.sort(b)[::-1]
        if sb[0] - sb[1] > 0.05 and int(a.argmax()) != int(b.argmax()):
            disagree.append(t)
        # the sampled id is the oracle's explicit-uniform draw from the same (TP-gathered) logits
        got = int(st[0]["ids"][0])
        if not topp_draw_ok(a, got, 0.8, 0.9, 0.5):
            disagree.append(("topp", t, got, int(O.sample_top_p(a[None], 0.8, 0.9, np.array([0.5], np.float32))[0, 0])))
    out["decode_err_vs_solo"] = worst
    out["decode_disagree"] = disagree
    # free-running greedy through the decode graph (when the communicator allows) vs the reference's 32 ids, and
    # top-p with fixed uniforms: the first draw against the oracle's on the TP prefill logits
    out["greedy_tp"] = tp.generate(ids, px, am, len(ref_ids), stop_token=None)[0].tolist()
    out["greedy_ref"] = ref_ids
    u = torch.rand(9, 1, generator=torch.Generator().manual_seed(4321))
    out["sampled_tp"] = tp.generate(ids, px, am, 8, do_sample=True, temperature=0.8, top_p=0.9, uniforms=u,
                                    stop_token=None)[0].tolist()
    # (free-running draws are not compared with the single-rank engine: the TP logits differ from it by ~1e-2 in
    # another fp32 summation order, and on this flat synthetic distribution that moves a uniform across a CDF
    # boundary within a few steps -- measured at step 1.  Each draw's parity is the teacher-forced check above.)
    out["sampled_first_ok"] = topp_draw_ok(res[0][2][0].float().cpu().numpy(), out["sampled_tp"][0], 0.8, 0.9,
                                           float(u[0, 0]))
    torch.cuda.synchronize()
    out["xgmi_err"] = int(comm.err.item()) if isinstance(comm, XgmiComm) else 0
    if isinstance(comm, XgmiComm):
        comm.close()
    with open(os.path.join(os.environ["TP_OUT"], f"rank{rank}.json"), "w") as f:
        json.dump(out, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
