"""End-to-end parity of the HIP engine against the oracle and the reference's golden vectors.

Tolerances: the reference computes in fp32; the HIP path keeps the residual stream and
all accumulations in fp32 but feeds bf16 operands to the MFMAs, so a logit differs from
the fp32 oracle by bf16 rounding noise.  Stated bound: scaled max error
max|hip - oracle| / max|oracle| < 3e-2 on logits / features; greedy ids must be
identical wherever the oracle's top1-top2 margin exceeds 0.1 (in logit units).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

TOL = 3e-2


def err(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


@pytest.fixture(scope="module")
def tiny():
    if not torch.cuda.is_available():
        pytest.skip("needs the HIP device")
    from oracle import configs as ocfg, synth, paligemma_oracle as O
    from pghip import configs, engine, synthetic, weights
    cfg = configs.TINY
    eng = engine.PaliGemmaEngine(cfg, weights.PackedWeights(cfg, synthetic.SyntheticStateDict(cfg).__getitem__))
    orc = O.PaliGemmaOracle(ocfg.TINY, synth.generate_state_dict(ocfg.TINY), recompute_vision=False)
    return eng, orc


@pytest.mark.parametrize("B", [1, 2])
def test_tiny_vision_and_prefill_vs_golden(tiny, golden, B):
    eng, orc = tiny
    g = golden("tiny")
    p = f"b{B}_"
    px = torch.from_numpy(g[p + "pixel_values"]).cuda()
    feats, hid = eng.vision(px, want_hidden=True)
    assert err(hid.cpu().numpy(), g[p + "vision_out"].reshape(-1, hid.shape[1])) < TOL
    assert err(feats.cpu().numpy(), g[p + "proj_out"].reshape(-1, feats.shape[1])) < TOL
    ids = torch.from_numpy(g[p + "input_ids"]).cuda()
    Bv, L = ids.shape
    cache = eng.new_cache(Bv, L + 8)
    resid = torch.empty(Bv * L, eng.w.hidden, device="cuda")
    eng.embed_merge(ids, feats, resid)
    pos = torch.arange(1, L + 1, dtype=torch.int32).repeat(Bv, 1)
    logits, _ = eng.gemma_prefill(resid, pos, cache, Bv, L)
    assert err(logits.cpu().numpy(), g[p + "logits"].reshape(Bv * L, -1)) < TOL
    k0 = cache.k[0, :, :L].float().cpu().numpy()
    assert err(k0, g[p + "k_cache0"][:, 0]) < TOL


def test_tiny_greedy_matches_reference_loop(tiny, golden):
    eng, _ = tiny
    g = golden("tiny")
    ids = torch.from_numpy(g["b1_input_ids"]).cuda()
    px = torch.from_numpy(g["b1_pixel_values"]).cuda()
    for use_graph in (False, True):
        out = eng.generate(ids, px, torch.ones_like(ids), len(g["greedy_ids"]), use_graph=use_graph)
        assert out[0].tolist() == g["greedy_ids"].tolist()


@pytest.mark.parametrize("B", [1, 3])
def test_chained_embed_generation_matches_unchained(tiny, golden, B):
    """Chained greedy decode (pg_argmax_embed writes the next step's input rows, no embed launch per step)
    == the unchained loop (embed_merge at the start of every step): identical tokens, graph and eager."""
    eng, _ = tiny
    g = golden("tiny")
    ids = torch.from_numpy(g["b1_input_ids"]).cuda().repeat(B, 1)
    px = torch.from_numpy(g["b2_pixel_values"]).cuda()
    px = torch.cat([px, px])[:B]
    outs = []
    try:
        for chain in (True, False):
            eng.CHAIN_EMBED = chain
            for use_graph in (True, False):
                outs.append(eng.generate(ids, px, torch.ones_like(ids), 14, stop_token=None,
                                         use_graph=use_graph).tolist())
    finally:
        eng.CHAIN_EMBED = type(eng).CHAIN_EMBED
    assert all(o == outs[0] for o in outs[1:])


@pytest.mark.parametrize("fuse_max_b,use_fin", [(2, True), (2, False), (0, True)])
def test_tiny_teacher_forced_decode_vs_oracle(tiny, golden, fuse_max_b, use_fin):
    """Long decode (no EOS stop) with the oracle's greedy continuation: per-step logits.  Layer forms:
    in-kernel split-K finalisation with the split-KV merge in the o_proj prologue (default, single rank),
    split-K partials reduced by the next GEMV's RMSNorm prologue (the TP form), and the unfused layer
    (fuse_max_b=0, the B > 2 path)."""
    from oracle import paligemma_oracle as O
    eng, orc = tiny
    eng.FUSE_MAX_B, eng.USE_FIN = fuse_max_b, use_fin
    g = golden("tiny")
    ids_np = g["b1_input_ids"]
    steps = 24
    ref_ids, ref_logits = O.generate(orc, ids_np, g["b1_pixel_values"], np.ones_like(ids_np), steps,
                                     stop_token=None, record_logits=True)
    ids = torch.from_numpy(ids_np).cuda()
    cache, feats, logits, nxt = eng.prefill_request(ids, torch.from_numpy(g["b1_pixel_values"]).cuda(),
                                                    torch.ones_like(ids), steps)
    assert err(logits.cpu().numpy(), ref_logits[0]) < TOL
    st = eng.decode_state(1, cache, nxt, steps)
    for t in range(1, steps):
        st["ids"].fill_(ref_ids[t - 1])                                 # teacher forcing
        lg = eng.decode_step(st, cache, feats, dict(do_sample=False))
        assert err(lg.cpu().numpy(), ref_logits[t]) < TOL, t
        top = np.sort(ref_logits[t][0])[::-1]
        if top[0] - top[1] > 0.1:
            assert int(st["ids"][0]) == ref_ids[t], t
    eng.FUSE_MAX_B, eng.USE_FIN = type(eng).FUSE_MAX_B, type(eng).USE_FIN


@pytest.mark.slow
def test_pt224_full_size_parity(golden):
    """Full-size synthetic PaliGemma-3B-224 against the reference's own run and the oracle.

    The synthetic init (Linear std 2/sqrt(fan_in), chosen so greedy decoding does not
    degenerate) amplifies rounding through 45 layers: the ORACLE itself, computed with bf16 operands
    where the HIP path has them, lands ~10% (scaled max) away from its own fp32 logits.  So:
      (1) every one of the 27 SigLIP + 18 Gemma layers, fed the HIP path's own layer input, must
          match the fp32 oracle layer to < 2e-2 (no error accumulation: this is the kernel check);
      (2) end-to-end prefill logits must be within 1.5x the intrinsic bf16 error of the model;
      (3) the top-1 token of the prefill must match the reference.
    """
    from oracle import paligemma_oracle as O
    from pghip import configs, engine, synthetic, weights
    g = golden("pt224")
    cfg = configs.PT_224
    sd = synthetic.SyntheticStateDict(cfg)
    eng = engine.PaliGemmaEngine(cfg, weights.PackedWeights(cfg, sd.__getitem__))
    W = {k: sd[k].float().cpu().numpy() for k in sd.keys()}
    ids = g["input_ids"]
    px = g["pixel_values"]
    vtaps = []
    feats = eng.vision(torch.from_numpy(px).cuda(), taps=vtaps)
    vc = cfg["vision_config"]
    for i in range(vc["num_hidden_layers"]):
        x = vtaps[i].cpu().numpy()[None]
        lp = f"vision_tower.model.encoder.layers.{i}."
        y = x + O.siglip_attention(W, lp + "self_attn.", vc, O.layer_norm(x, W[lp + "layer_norm1.weight"],
                                                                          W[lp + "layer_norm1.bias"], 1e-6))
        y = y + O.siglip_mlp(W, lp + "mlp.", O.layer_norm(y, W[lp + "layer_norm2.weight"],
                                                          W[lp + "layer_norm2.bias"], 1e-6))
        assert err(vtaps[i + 1].cpu().numpy()[None] - x, y - x) < 2e-2, f"vision layer {i}"
    L = ids.shape[1]
    resid = torch.empty(L, eng.w.hidden, device="cuda")
    eng.embed_merge(torch.from_numpy(ids).cuda(), feats, resid)
    ttaps = []
    cache = eng.new_cache(1, L + 4)
    logits, _ = eng.gemma_prefill(resid, torch.arange(1, L + 1, dtype=torch.int32)[None], cache, 1, L,
                                  logits_rows=torch.tensor([L - 1], dtype=torch.int32, device="cuda"), taps=ttaps)
    tc = cfg["text_config"]
    pos = np.arange(1, L + 1)[None]
    mask = np.zeros((1, 1, L, L), np.float32)
    for i in range(tc["num_hidden_layers"]):
        x = ttaps[i].cpu().numpy()[None]
        lp = f"language_model.model.layers.{i}."
        y = x + O.gemma_attention(W, lp + "self_attn.", tc, i, O.rms_norm(x, W[lp + "input_layernorm.weight"]),
                                  pos, mask, None)
        y = y + O.gemma_mlp(W, lp + "mlp.", O.rms_norm(y, W[lp + "post_attention_layernorm.weight"]))
        assert err(ttaps[i + 1].cpu().numpy()[None] - x, y - x) < 2e-2, f"gemma layer {i}"
    lg = logits[0].cpu().numpy()
    with O.bf16_operands():
        lg16 = O.PaliGemmaOracle(cfg, W, recompute_vision=False).forward(
            ids, px, np.ones_like(ids), O.KVCache(), logits_rows=slice(-1, None))["logits"][0, -1]
    intrinsic = err(lg16, g["prefill_last_logits"])
    assert err(lg, g["prefill_last_logits"]) < 1.5 * intrinsic, (err(lg, g["prefill_last_logits"]), intrinsic)
    assert int(np.argmax(lg)) == int(g["greedy_ids"][0])


@pytest.mark.slow
def test_pt224_full_size_teacher_forced_decode(golden):
    """Full-size PaliGemma-3B-224 decode against the reference's own 16 greedy steps (tests/golden/pt224.npz):
    the graph-free decode step is fed the reference's tokens (teacher forcing) and its logits are compared
    with the reference's top-64 logits of every step.  Bound: max error on those 64 logits < 15% of their
    scale (the synthetic model's intrinsic bf16 sensitivity is ~10%, see test_pt224_full_size_parity), and
    the top-1 id must equal the reference's at every step whose reference top1-top2 margin exceeds 0.5 logits:
    twice this recipe's per-logit bf16 error (0.21-0.44 measured per step, scripts/tune/tf_errors.py; bf16 cannot
    order closer pairs reliably).  The checked steps are fixed by the golden (4 of 16), not by the run's own error,
    so a rounding-order change in a kernel cannot move a step out of the check.  The bit-exact greedy check is
    test_pt224_free_running_greedy_ids_equal_reference (better-conditioned recipe)."""
    from pghip import configs, engine, synthetic, weights
    g = golden("pt224")
    cfg = configs.PT_224
    sd = synthetic.SyntheticStateDict(cfg)
    eng = engine.PaliGemmaEngine(cfg, weights.PackedWeights(cfg, sd.__getitem__))
    ids = torch.from_numpy(g["input_ids"]).cuda()
    px = torch.from_numpy(g["pixel_values"]).cuda()
    steps = len(g["greedy_ids"])
    cache, feats, logits, nxt = eng.prefill_request(ids, px, torch.ones_like(ids), steps)
    st = eng.decode_state(1, cache, nxt, steps)
    checked = 0
    for t in range(steps):
        if t == 0:
            lg = logits[0].cpu().numpy()
        else:
            st["ids"].fill_(int(g["greedy_ids"][t - 1]))
            lg = eng.decode_step(st, cache, feats, dict(do_sample=False))[0].cpu().numpy()
        top_ids, top_v = g["step_top64_ids"][t], g["step_top64_values"][t]
        e = float(np.abs(lg[top_ids] - top_v).max())
        assert e < 0.15 * float(np.abs(top_v).max()), (t, e)
        if g["margin"][t] > 0.5:
            assert e < 0.5 * float(g["margin"][t]) + 0.05, (t, e, float(g["margin"][t]))
            assert int(np.argmax(lg)) == int(g["greedy_ids"][t]), (t, e, float(g["margin"][t]))
            checked += 1
    assert checked == int((g["margin"] > 0.5).sum()) == 4, checked


@pytest.mark.slow
def test_pt224_decode_bit_reproducible_run_to_run(golden):
    """The same full-size PaliGemma-3B-224 request decoded three times in one process -- eager steps, hipGraph
    replays, eager again -- gives bitwise-equal logits at every step and the same ids (greedy ids
    must not depend on the run).  Batch-1 decode adds the o_proj / down_proj split-K partials into the residual with
    atomics whose arrival order varies; the default fixed-point accumulator (PG_EPI_FX_ADD, engine.DECODE_ADD "fx")
    makes that sum exact, so nothing downstream can differ.  The prefill logits are compared too."""
    from pghip import configs, engine, synthetic, weights
    g = golden("pt224")
    cfg = configs.PT_224
    eng = engine.PaliGemmaEngine(cfg, weights.PackedWeights(cfg, synthetic.SyntheticStateDict(cfg).__getitem__))
    assert eng.DECODE_ADD == "fx"
    ids = torch.from_numpy(g["input_ids"]).cuda()
    px = torch.from_numpy(g["pixel_values"]).cuda()
    steps, V = 24, eng.w.vocab

    def run(graph):
        cache, feats, logits, nxt = eng.prefill_request(ids, px, torch.ones_like(ids), steps + 1)
        sampler = dict(do_sample=False)
        st = eng.decode_state(1, cache, nxt, steps + 1, sampler=sampler)
        eng.sample(logits, st, sampler, advance=False, feats=feats)
        out = [logits[:, :V].clone()]
        replay = eng._graph_step(st, cache, feats, sampler) if graph else None
        for _ in range(steps):
            if graph:
                replay()
                lg = eng._buf("d_logits", (1, eng.w.vocab_local_pad), torch.float32)[:, :V]
            else:
                lg = eng.decode_step(st, cache, feats, sampler)
            out.append(lg.clone())
        torch.cuda.synchronize()
        return torch.cat(out), st["hist"][:steps + 1, 0].cpu()

    runs = [run(False), run(True), run(False)]
    for lg, hist in runs[1:]:
        assert torch.equal(hist, runs[0][1]), (hist.tolist(), runs[0][1].tolist())
        diff = (lg != runs[0][0]).any(-1).nonzero().flatten().tolist()
        assert not diff, f"logits differ at steps {diff}"


def test_decode_step_starts_from_a_clean_fx_accumulator(tiny, golden):
    """The batch-1 decode residual's fixed-point accumulator carries no state between steps: a step that
    begins with garbage left in it -- as after an interrupted step -- gives the same logits, bit for bit, as a step from
    a zero accumulator, because layer 0's q|k|v GEMV clears it (PgFusedArgs.amax_zero on the bf16 GEMV, ABI 12) before
    any FX_ADD producer adds into it.  And a status word set by an overflowing FX_ADD makes generate() raise."""
    eng, _ = tiny
    assert eng.DECODE_ADD == "fx"
    g = golden("tiny")
    ids = torch.from_numpy(g["b1_input_ids"]).cuda()
    px = torch.from_numpy(g["b1_pixel_values"]).cuda()
    cache, feats, logits, nxt = eng.prefill_request(ids, px, torch.ones_like(ids), 8)
    sampler = dict(do_sample=False)
    st = eng.decode_state(1, cache, nxt, 8, sampler=sampler)
    eng.sample(logits, st, sampler, advance=False, feats=feats)
    eng.decode_step(st, cache, feats, sampler)                 # one step so every workspace exists
    torch.cuda.synchronize()
    snap = {k: st[k].clone() for k in ("ids", "pos", "kv_len", "step", "hist")}
    res0 = eng._ws["d_res_a"].clone() if st.get("chain") else None

    def step(dirty):
        for k, v in snap.items():
            st[k].copy_(v)
        if res0 is not None:
            eng._ws["d_res_a"].copy_(res0)
        fx = eng._ws["d_fx"]
        if dirty:
            fx.copy_(torch.randint(-2 ** 40, 2 ** 40, fx.shape, dtype=torch.int64))
        out = eng.decode_step(st, cache, feats, sampler).clone()
        torch.cuda.synchronize()
        assert int(fx.abs().sum()) == 0                        # the step's last layer leaves it zero again
        return out

    clean = step(False)
    assert torch.equal(step(True), clean)
    eng.fx_status().fill_(1)                                   # as an FX_ADD launch given an Inf would
    with pytest.raises(FloatingPointError):
        eng.generate(ids, px, torch.ones_like(ids), 4)
    assert int(eng.fx_status().item()) == 0


def test_batched_generation_per_row_eos(tiny, golden):
    """B = 2 rows of the same request (+ one different image): each row equals its own B = 1 run, cut at
    its own EOS (tokens after a row's EOS come back as pad)."""
    eng, _ = tiny
    g = golden("tiny")
    ids1 = torch.from_numpy(g["b1_input_ids"]).cuda()
    px1 = torch.from_numpy(g["b1_pixel_values"]).cuda()
    px2 = torch.from_numpy(g["b2_pixel_values"][1:2]).cuda()
    single = [eng.generate(ids1, p, torch.ones_like(ids1), 12)[0].tolist() for p in (px1, px2)]
    ids = ids1.repeat(2, 1)
    rows = eng.generate(ids, torch.cat([px1, px2]), torch.ones_like(ids), 12, return_list=True)
    assert rows == single
    out = eng.generate(ids, torch.cat([px1, px2]), torch.ones_like(ids), 12, pad_token=0)
    for b in range(2):
        assert out[b, : len(single[b])].tolist() == single[b]
        assert (out[b, len(single[b]):] == 0).all()


# ---------------------------------------------------------------- fp8 Gemma linears (BASELINE configs[4])
TOL_FP8 = 0.12  # e4m3 operands (3 mantissa bits), per-row / per-channel scales: looser than bf16 (measured 0.086)


@pytest.fixture(scope="module")
def tiny_fp8():
    if not torch.cuda.is_available():
        pytest.skip("needs the HIP device")
    from pghip import configs, engine, synthetic, weights
    cfg = configs.TINY
    return engine.PaliGemmaEngine(cfg, weights.PackedWeights(cfg, synthetic.SyntheticStateDict(cfg).__getitem__,
                                                             fp8=True))


def test_tiny_fp8_prefill_and_batched_decode_vs_oracle(tiny_fp8, golden):
    """fp8 engine (Gemma q|k|v, o, gate/up, down as PG_FP8 GEMMs for > 16 rows): prefill logits of the golden
    prompt replicated to a batch of 20 (every GEMM on the fp8 path), then teacher-forced decode steps at
    B = 20 (fp8 tile GEMMs) against the fp32 oracle; greedy ids must agree where the oracle's top-1/top-2
    margin exceeds 0.5 logits."""
    from oracle import configs as ocfg, synth, paligemma_oracle as O
    eng = tiny_fp8
    orc = O.PaliGemmaOracle(ocfg.TINY, synth.generate_state_dict(ocfg.TINY), recompute_vision=False)
    g = golden("tiny")
    ids_np = g["b1_input_ids"]
    steps, B = 8, 20
    ref_ids, ref_logits = O.generate(orc, ids_np, g["b1_pixel_values"], np.ones_like(ids_np), steps,
                                     stop_token=None, record_logits=True)
    ids = torch.from_numpy(ids_np).cuda().repeat(B, 1)
    px = torch.from_numpy(g["b1_pixel_values"]).cuda().repeat(B, 1, 1, 1)
    cache, feats, logits, nxt = eng.prefill_request(ids, px, torch.ones_like(ids), steps)
    worst = err(logits[:1].cpu().numpy(), ref_logits[0])
    assert worst < TOL_FP8, worst
    assert torch.equal(logits[0], logits[B - 1])                         # rows are independent
    st = eng.decode_state(B, cache, nxt, steps)
    for t in range(1, steps):
        st["ids"].fill_(ref_ids[t - 1])
        lg = eng.decode_step(st, cache, feats, dict(do_sample=False))
        e = err(lg[:1].cpu().numpy(), ref_logits[t])
        worst = max(worst, e)
        assert e < TOL_FP8, (t, e)
        top = np.sort(ref_logits[t][0])[::-1]
        if top[0] - top[1] > 0.5:
            assert int(st["ids"][0]) == ref_ids[t], t
    print(f"fp8 tiny worst scaled logit error {worst:.4f}")


@pytest.mark.parametrize("B", [8, 16])
def test_tiny_batched_decode_fin_path_vs_oracle(tiny, golden, B):
    """Batched decode (5..16 rows) with in-kernel split-K finalisation: merge kernel + o_proj / down_proj
    F32_FIN (residual, x' and per-tile-pair sums of squares) feeding PRO_X_RSTD GEMVs with two 16-row tiles
    per workgroup.  Per-step logits of every row against the oracle, and against the unfused layer."""
    from oracle import paligemma_oracle as O
    eng, orc = tiny
    g = golden("tiny")
    ids_np = g["b1_input_ids"]
    steps = 10
    ref_ids, ref_logits = O.generate(orc, ids_np, g["b1_pixel_values"], np.ones_like(ids_np), steps,
                                     stop_token=None, record_logits=True)
    ids = torch.from_numpy(ids_np).cuda().repeat(B, 1)
    px = torch.from_numpy(g["b1_pixel_values"]).cuda().repeat(B, 1, 1, 1)
    outs = {}
    for use_fin in (True, False):
        eng.USE_FIN = use_fin
        try:
            cache, feats, logits, nxt = eng.prefill_request(ids, px, torch.ones_like(ids), steps)
            st = eng.decode_state(B, cache, nxt, steps)
            lgs = []
            for t in range(1, steps):
                st["ids"].fill_(ref_ids[t - 1])
                lg = eng.decode_step(st, cache, feats, dict(do_sample=False)).clone()
                for row in (0, B - 1):
                    assert err(lg[row:row + 1].cpu().numpy(), ref_logits[t]) < TOL, (use_fin, t, row)
                lgs.append(lg)
            outs[use_fin] = torch.stack(lgs)
        finally:
            eng.USE_FIN = type(eng).USE_FIN
    assert err(outs[True].cpu().numpy(), outs[False].cpu().numpy()) < 5e-3


@pytest.mark.slow
def test_pt224_free_running_greedy_ids_equal_reference(golden):
    """Bit-exact greedy ids at full size: PaliGemma-3B-224 on the better-conditioned synthetic recipe (Linear std
    1.6/sqrt(fan_in); tests/golden/make_golden.py make_pt224wc), three images, 32 free-running greedy tokens each
    through the bench's exact decode path (chained argmax+embed, hipGraph-replayed steps, default splits) must equal
    the reference's own test_inference ids -- one differing token fails.  The reference's smallest top1-top2 margin
    over the 96 steps is stated in the fixture (>= 0.1 logits, against ~0.02 of bf16 rounding on that difference
    measured with the oracle's bf16-operand mode).  The same three requests as ONE batch (B = 3: the unfused batched
    layer, per-row state) must give the same ids."""
    from pghip import configs, engine, synthetic, weights
    g = golden("pt224wc")
    cfg = configs.PT_224
    sd = synthetic.SyntheticStateDict(cfg, linear_gain=float(g["linear_gain"]))
    eng = engine.PaliGemmaEngine(cfg, weights.PackedWeights(cfg, sd.__getitem__))
    from test_large_gpu import _pixels
    pvs, ids_all, want = [], [], []
    for j in range(len(g["seeds"])):
        pvs.append(_pixels(g, j, 224))
        ids_all.append(g[f"i{j}_input_ids"])
        want.append(g[f"i{j}_greedy_ids"].tolist())
        ids = torch.from_numpy(ids_all[-1]).cuda()
        px = torch.from_numpy(pvs[-1]).cuda()
        got = eng.generate(ids, px, torch.ones_like(ids), len(want[-1]), stop_token=None, use_graph=True)
        assert got[0].tolist() == want[-1], (j, got[0].tolist(), want[-1], float(g[f"i{j}_margin"].min()))
    ids = torch.from_numpy(np.concatenate(ids_all)).cuda()
    px = torch.from_numpy(np.concatenate(pvs)).cuda()
    got = eng.generate(ids, px, torch.ones_like(ids), len(want[0]), stop_token=None, use_graph=True)
    assert got.tolist() == want


@pytest.mark.gpu
def test_bench_prints_one_contract_json_line():
    """bench.py (the driver's contract): one JSON line on stdout with the required keys, BASELINE.json's metric and
    configs[1] workload, a roofline object with achieved / peak / frac consistent with each other, and a
    cpu_baseline object from the oracle port on a bounded sample (here 2 steps after 1 warmup)."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "2", "--warmup", "1"],
                       capture_output=True, text=True, timeout=280, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    o = json.loads(lines[0])
    base = json.load(open(os.path.join(root, "BASELINE.json")))
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in o, k
    assert o["metric"] == base["metric"] and o["n_gpus"] == 1 and o["steps"] == 2 and o["warmup"] == 1
    assert o["value"] > 0 and o["higher_is_better"] is True and o["scaling"] == "weak" and o["dtype"] == "bf16"
    assert "configs[1]" in o["config"]["workload"]
    rf = o["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
    assert 0 < rf["frac"] <= 1 and abs(rf["achieved"] / rf["peak"] - rf["frac"]) < 1e-3
    cb = o["cpu_baseline"]
    assert cb["kind"] in ("port", "reference") and cb["value"] and cb["value"] > 0 and cb["cores"] >= 1
