"""BASELINE configs[2] (pt-448, 1024 image tokens, batch 16) and configs[4] (pt-896, 4096 image tokens, batch 32,
fp8 Gemma linears) through the HIP path at their own sizes, against the reference's own runs
(tests/golden/pt448.npz, pt896.npz; tests/golden/make_golden.py make_large) and the fp32 oracle.

Tolerances, as test_engine_gpu.py's full-size pt-224 tests (the synthetic 2/sqrt(fan_in) init amplifies bf16
rounding to ~10% of the logit scale end to end, so the end-to-end bound is relative to that, and the kernels are
checked layer by layer without accumulation):
  * every SigLIP / Gemma layer, fed the HIP path's own input, matches the fp32 oracle layer to < 2e-2 (scaled);
  * the reference's top-64 logits of every teacher-forced step lie within 15% of their scale (bf16); with fp8
    e4m3 operands within 1.5x the distance of the fp32 oracle run on the same operand rounding (a fixture of
    tests/golden/make_emu.py: derived per image and step, not a flat percentage);
  * free-running greedy ids equal the reference's exactly at pt-448 x 16 (two images) and pt-896 (bf16), on the
    better-conditioned synthetic recipe whose margins exceed the bf16 error (tests/golden/pt448wc.npz, pt896wc.npz);
  * the top-1 id equals the reference's wherever the reference's top1-top2 margin exceeds twice that step's
    measured error;
  * the rows of a batch that hold the same request agree to 2e-2 (scaled): rows in a ragged last row block run
    with another split-K summation order (row-blocked GEMMs), and the synthetic init amplifies that fp32 ordering
    noise like bf16 rounding (measured 5.6e-3 at pt-448 x16); cross-row contamination would show as O(1).
"""
import numpy as np
import pytest
import torch

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

PROMPT = [2, 651, 4906, 603, 476, 2121, 576, 108]


def err(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def _pixels(g, j, size):
    """The golden request's pixel values, regenerated from its image seed through the host pre-processing (bit-exact
    with the reference's process_images, test_host.py) and checked against the stored checksums."""
    from PIL import Image
    from processing_paligemma import process_images
    img = np.random.default_rng(int(g["seeds"][j])).integers(0, 256, (1, size, size, 3), dtype=np.uint8)
    pv = np.stack(process_images([Image.fromarray(img[0])], size, 1 / 255.0, Image.Resampling.BICUBIC)).astype(np.float32)
    assert np.array_equal(pv.reshape(-1)[::9973], g[f"i{j}_pixel_sample"])
    assert abs(float(pv.astype(np.float64).sum()) - float(g[f"i{j}_pixel_sum"])) < 1e-6 * pv.size
    return pv


def _engine(name, fp8=False, linear_gain=2.0):
    from pghip import configs, engine, synthetic, weights
    cfg = configs.CONFIGS[name]
    sd = synthetic.SyntheticStateDict(cfg, linear_gain=linear_gain)
    return cfg, sd, engine.PaliGemmaEngine(cfg, weights.PackedWeights(cfg, sd.__getitem__, fp8=fp8))


def _layer_checks(eng, cfg, sd, ids, pv, vis_layers, txt_layers, tol=2e-2):
    """The HIP path's SigLIP and Gemma layers, each fed the HIP path's own input, against the fp32 oracle layer.
    Returns the prefill's last-position logits."""
    from oracle import paligemma_oracle as O
    W = {}

    def w(k):
        if k not in W:
            W[k] = sd[k].float().cpu().numpy()
        return W[k]
    vtaps = []
    feats = eng.vision(torch.from_numpy(pv).cuda(), taps=vtaps)
    vc = cfg["vision_config"]
    for i in vis_layers:
        x = vtaps[i].cpu().numpy()[None]
        lp = f"vision_tower.model.encoder.layers.{i}."
        Wl = {k: w(k) for k in sd.keys() if k.startswith(lp)}
        y = x + O.siglip_attention(Wl, lp + "self_attn.", vc, O.layer_norm(x, Wl[lp + "layer_norm1.weight"],
                                                                           Wl[lp + "layer_norm1.bias"], 1e-6))
        y = y + O.siglip_mlp(Wl, lp + "mlp.", O.layer_norm(y, Wl[lp + "layer_norm2.weight"],
                                                           Wl[lp + "layer_norm2.bias"], 1e-6))
        assert err(vtaps[i + 1].cpu().numpy()[None] - x, y - x) < tol, f"vision layer {i}"
    del vtaps
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
    for i in txt_layers:
        x = ttaps[i].cpu().numpy()[None]
        lp = f"language_model.model.layers.{i}."
        Wl = {k: w(k) for k in sd.keys() if k.startswith(lp)}
        y = x + O.gemma_attention(Wl, lp + "self_attn.", tc, i, O.rms_norm(x, Wl[lp + "input_layernorm.weight"]),
                                  pos, mask, None)
        y = y + O.gemma_mlp(Wl, lp + "mlp.", O.rms_norm(y, Wl[lp + "post_attention_layernorm.weight"]))
        assert err(ttaps[i + 1].cpu().numpy()[None] - x, y - x) < tol, f"gemma layer {i}"
    return logits[0].cpu().numpy()


def _check_step(lg, g, p, t, tol, checked):
    top_ids, top_v = g[p + "step_top_ids"][t], g[p + "step_top_values"][t]
    e = float(np.abs(lg[top_ids] - top_v).max())
    assert e < tol * float(np.abs(top_v).max()), (p, t, e)
    if g[p + "margin"][t] > 2 * e:
        assert int(np.argmax(lg)) == int(g[p + "greedy_ids"][t]), (p, t, e, float(g[p + "margin"][t]))
        checked.append((p, t))
    return e


def test_pt448_layers_vs_oracle_and_reference(golden):
    """pt-448 (N = 1024, L = 1032), batch 1: all 27 SigLIP and 18 Gemma layers against the oracle, the prefill's
    top-64 logits against the reference's."""
    g = golden("pt448")
    cfg, sd, eng = _engine("pt-448")
    pv = _pixels(g, 0, 448)
    lg = _layer_checks(eng, cfg, sd, g["i0_input_ids"], pv, range(27), range(18))
    _check_step(lg, g, "i0_", 0, 0.15, [])


def test_pt448_batch16_prefill_and_decode_vs_reference(golden):
    """BASELINE configs[2]: batch 16 (8 rows of each of the reference's two pt-448 requests) through the batched
    prefill (16512 rows: row-blocked 256x256 GEMMs, 12-wave flash attention) and 8 teacher-forced batched decode
    steps (split-KV attention over 1.03 k keys, the merge kernel and the F32_FIN GEMVs of 5..16 rows): every row
    against its request's reference logits; rows of one request agree with each other."""
    g = golden("pt448")
    cfg, sd, eng = _engine("pt-448")
    pvs = [_pixels(g, j, 448) for j in range(2)]
    ids = torch.from_numpy(np.concatenate([g["i0_input_ids"]] * 8 + [g["i1_input_ids"]] * 8)).cuda()
    px = torch.from_numpy(np.concatenate([pvs[0]] * 8 + [pvs[1]] * 8)).cuda()
    steps = len(g["i0_greedy_ids"])
    cache, feats, logits, nxt = eng.prefill_request(ids, px, torch.ones_like(ids), steps + 2)
    st = eng.decode_state(16, cache, nxt, steps + 2)
    checked, worst = [], 0.0
    for t in range(steps):
        if t > 0:
            for j in range(2):
                st["ids"][8 * j:8 * j + 8].fill_(int(g[f"i{j}_greedy_ids"][t - 1]))
            logits = eng.decode_step(st, cache, feats, dict(do_sample=False))
        lg = logits.cpu().numpy()
        for j in range(2):
            rows = lg[8 * j:8 * j + 8]
            for r in (0, 7):
                worst = max(worst, _check_step(rows[r], g, f"i{j}_", t, 0.15, checked))
            assert err(rows, np.broadcast_to(rows[0], rows.shape)) < 2e-2, (j, t)
    assert len(checked) >= 4, checked
    print(f"pt448 x16: worst top-64 error {worst:.4f}, top-1 checked at {len(checked)} (image, step) pairs")


def test_pt896_layers_vs_oracle_and_reference(golden):
    """pt-896 (N = 4096, L = 4104), batch 1, bf16: SigLIP layers 0 / 13 / 26 and Gemma layers 0 / 9 / 17 against
    the oracle (the flash attention over 4096 / 4104 keys; a subset keeps the numpy oracle to about a minute), the
    prefill's top-64 logits against the reference's."""
    g = golden("pt896")
    cfg, sd, eng = _engine("pt-896")
    pv = _pixels(g, 0, 896)
    lg = _layer_checks(eng, cfg, sd, g["i0_input_ids"], pv, (0, 13, 26), (0, 9, 17))
    _check_step(lg, g, "i0_", 0, 0.15, [])


def _fp8_batch32(golden, name, images):
    """BASELINE configs[4] on one device: pt-896 at batch 32 with the Gemma linears and (at 17..32 rows) the lm_head
    on e4m3 operands (per-row / per-channel scales): the fp8 tile GEMMs of the 131 k-row prefill and the fp8 GEMVs of
    the teacher-forced decode steps over 4.1 k keys.  32 rows dealt in equal blocks to the golden's images.  Bound,
    per image and step: the reference's top-64 logits within 1.5x the distance of the fp32 oracle run on the same
    e4m3 / bf16 operand rounding (tests/golden/make_emu.py, <name>_fp8emu.npz) -- derived, not a flat percentage; the
    top-1 id equal to the reference's wherever its margin exceeds twice the step's measured error (a minimum count of
    such checks is asserted); rows of one image equal to each other (< 2e-2)."""
    g, em = golden(name), golden(name + "_fp8emu")
    gain = float(g["linear_gain"]) if "linear_gain" in g else 2.0
    cfg, sd, eng = _engine("pt-896", fp8=True, linear_gain=gain)
    B = 32
    per = B // len(images)
    pvs = [_pixels(g, j, 896) for j in images]
    ids = torch.from_numpy(np.concatenate([g[f"i{j}_input_ids"] for j in images for _ in range(per)])).cuda()
    px = torch.from_numpy(np.concatenate([pv for pv in pvs for _ in range(per)])).cuda()
    steps = len(g[f"i{images[0]}_greedy_ids"])
    cache, feats, logits, nxt = eng.prefill_request(ids, px, torch.ones_like(ids), steps + 2)
    st = eng.decode_state(B, cache, nxt, steps + 2)
    checked, worst = [], 0.0
    for t in range(steps):
        if t > 0:
            for k, j in enumerate(images):
                st["ids"][k * per:(k + 1) * per].fill_(int(g[f"i{j}_greedy_ids"][t - 1]))
            logits = eng.decode_step(st, cache, feats, dict(do_sample=False))
        lg = logits.cpu().numpy()
        for k, j in enumerate(images):
            p = f"i{j}_"
            rows = lg[k * per:(k + 1) * per]
            top_v = g[p + "step_top_values"][t]
            emu = float(np.abs(em[p + "emu_top_values"][t] - top_v).max())
            tol = 1.5 * emu / float(np.abs(top_v).max())
            for r in (0, per - 1):
                worst = max(worst, _check_step(rows[r], g, p, t, tol, checked) / emu)
            assert err(rows, np.broadcast_to(rows[0], rows.shape)) < 2e-2, (j, t)
    print(f"{name} x32 fp8: worst top-64 error {worst:.3f}x the emulated e4m3 distance, top-1 checked at "
          f"{len(checked)} (row, step) pairs")
    return checked


def test_pt896_batch32_fp8_vs_reference(golden):
    """The default recipe's pt-896 request (tests/golden/pt896.npz, 3 steps) on all 32 rows.  Its top1-top2 margins
    (0.03-0.20) lie below the e4m3 operands' error (the emulation itself flips step 1's argmax), so the top-1 ids are
    checked on the better-conditioned recipe below; here the bound on the top-64 logits carries the check."""
    _fp8_batch32(golden, "pt896", [0])


def test_pt896_batch32_fp8_two_images_vs_reference(golden):
    """The better-conditioned recipe's two pt-896 requests (tests/golden/pt896wc.npz, 16 steps), 16 rows each."""
    checked = _fp8_batch32(golden, "pt896wc", [0, 1])
    assert len(checked) >= 40, checked          # 2 images x 2 rows x 16 steps; step 0's small margins may skip


def test_pt448_batch16_free_running_greedy_ids_equal_reference(golden):
    """BASELINE configs[2] (pt-448, batch 16) free-running: two images (tests/golden/pt448wc.npz seeds 1236 / 1237,
    the two whose first-token margins exceed 0.1 on the better-conditioned recipe), 8 rows each, 24 greedy tokens
    through the bench's decode path (chained argmax + embed, hipGraph replay): every row's ids equal the reference's
    own loop exactly -- one differing id fails."""
    g = golden("pt448wc")
    cfg, sd, eng = _engine("pt-448", linear_gain=float(g["linear_gain"]))
    images = [2, 3]
    pvs = [_pixels(g, j, 448) for j in images]
    ids = torch.from_numpy(np.concatenate([g[f"i{j}_input_ids"] for j in images for _ in range(8)])).cuda()
    px = torch.from_numpy(np.concatenate([pv for pv in pvs for _ in range(8)])).cuda()
    steps = len(g["i2_greedy_ids"])
    out = eng.generate(ids, px, torch.ones_like(ids), steps, stop_token=None)
    for k, j in enumerate(images):
        want = g[f"i{j}_greedy_ids"].tolist()
        for r in range(8):
            assert out[k * 8 + r].tolist() == want, (j, r, out[k * 8 + r].tolist(), want)


def test_pt896_free_running_greedy_ids_equal_reference(golden):
    """pt-896 (4096 image tokens, bf16) free-running: the two requests of tests/golden/pt896wc.npz as one batch of 2,
    16 greedy tokens each through the bench's decode path: ids equal to the reference's loop exactly."""
    g = golden("pt896wc")
    cfg, sd, eng = _engine("pt-896", linear_gain=float(g["linear_gain"]))
    pvs = [_pixels(g, j, 896) for j in (0, 1)]
    ids = torch.from_numpy(np.concatenate([g["i0_input_ids"], g["i1_input_ids"]])).cuda()
    px = torch.from_numpy(np.concatenate(pvs)).cuda()
    out = eng.generate(ids, px, torch.ones_like(ids), len(g["i0_greedy_ids"]), stop_token=None)
    for j in (0, 1):
        assert out[j].tolist() == g[f"i{j}_greedy_ids"].tolist(), (j, out[j].tolist())
