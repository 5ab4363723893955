"""CPU-side checks: drop-in API surface, state-dict key parity, configs/recipes, the C-ABI library's
exported symbols, host pre-processing vs the reference's own outputs, and no CPU fallback."""
import os
import re

import numpy as np
import pytest
import torch

from conftest import ROOT

from oracle import configs as ocfg, synth


def _tiny_model():
    from modeling_paligemma import PaliGemmaConfig, PaliGemmaForConditionalGeneration
    return PaliGemmaForConditionalGeneration(PaliGemmaConfig(**ocfg.TINY))


def test_state_dict_keys_equal_reference_layout():
    m = _tiny_model()
    keys = set(m.state_dict().keys())
    want = set(synth.state_dict_shapes(ocfg.TINY)) | {"language_model.lm_head.weight"}
    assert keys == want
    sd = m.state_dict()
    for k, shp in synth.state_dict_shapes(ocfg.TINY).items():
        assert tuple(sd[k].shape) == tuple(shp), k


def test_reference_checkpoint_loads_strict_false_and_ties():
    m = _tiny_model()
    sd = {k: torch.from_numpy(v) for k, v in synth.generate_state_dict(ocfg.TINY).items()}
    res = m.load_state_dict(sd, strict=False)
    assert set(res.missing_keys) == {"language_model.lm_head.weight"} and not res.unexpected_keys
    m.tie_weights()
    assert m.language_model.lm_head.weight is m.language_model.model.embed_tokens.weight


def test_configs_and_recipes_match_oracle():
    from pghip import configs, synthetic
    assert configs.CONFIGS == ocfg.CONFIGS
    for name in ("pt-224", "tiny"):
        shapes = synth.state_dict_shapes(ocfg.CONFIGS[name])
        assert synthetic.state_dict_shapes(configs.CONFIGS[name]) == shapes
        for k, s in shapes.items():
            assert synthetic.recipe(k, s) == synth.recipe(k, s), k
            assert synthetic.seed_of(k) == synth.seed_of(k), k


def test_library_exports_every_header_symbol():
    from pghip import _lib
    hdr = open(os.path.join(ROOT, "include", "pghip.h")).read()
    declared = set(re.findall(r"^int (pg_\w+)\(", hdr, re.M))
    assert declared == set(_lib.SIGNATURES), declared ^ set(_lib.SIGNATURES)
    lib = _lib.load()
    for name in declared:
        assert hasattr(lib, name), name
    assert lib.pg_abi_version() == _lib.ABI_VERSION == 13


def test_library_matches_source_tree():
    """The library carries the hash of the sources it was built from (pghip/build.py), and it equals the hash of
    this tree: a stale prebuilt libpghip.so cannot be the one the GPU suite loads (_lib.load refuses it)."""
    from pghip import _lib, build
    assert build.library_hash() == build.source_hash() == _lib.source_hash()
    assert len(build.source_hash()) == 64


def test_no_cpu_fallback():
    m = _tiny_model()
    ids = torch.tensor([[299] * 16 + [2, 5, 108]])
    with pytest.raises(RuntimeError, match="HIP"):
        m(input_ids=ids, pixel_values=torch.zeros(1, 3, 56, 56), attention_mask=torch.ones_like(ids))
    from modeling_gemma import GemmaMLP, GemmaConfig
    mlp = GemmaMLP(GemmaConfig(hidden_size=128, intermediate_size=320))
    with pytest.raises(RuntimeError, match="HIP"):
        mlp(torch.zeros(1, 2, 128))


@pytest.mark.parametrize("name", ["tiny", "pt224"])
def test_process_images_matches_reference(golden, name):
    """Host pre-processing against pixel values the reference's process_images made."""
    from PIL import Image
    from processing_paligemma import process_images
    g = golden(name)
    imgs = g["images_u8"] if "images_u8" in g else g["b1_images_u8"]
    want = g["pixel_values"] if "pixel_values" in g else g["b1_pixel_values"]
    got = np.stack(process_images([Image.fromarray(im) for im in imgs], imgs.shape[1], 1 / 255.0,
                                  Image.Resampling.BICUBIC))
    assert np.array_equal(got.astype(np.float32), want)


def test_gemma_string_list_repr_quirk():
    from processing_paligemma import create_gemma_string
    assert create_gemma_string(["caption en"], 2, "<image>", "<bos>") == "<image><image><bos>['caption en']\n"


def test_hf_key_remap():
    from utils import remap_hf_key
    assert remap_hf_key("vision_tower.vision_model.encoder.layers.3.self_attn.q_proj.weight") == \
        "vision_tower.model.encoder.layers.3.self_attn.query_proj.weight"
    assert remap_hf_key("vision_tower.vision_model.embeddings.position_embedding.weight") == \
        "vision_tower.model.embeddings.positional_embeddings.weight"
    assert remap_hf_key("language_model.model.layers.0.self_attn.q_proj.weight") == \
        "language_model.model.layers.0.self_attn.q_proj.weight"


def test_kvcache_reference_api_on_static_store():
    from modeling_gemma import KVCache
    kv = KVCache()
    assert kv.num_items() == 0
    k = torch.randn(2, 1, 5, 32)
    v = torch.randn(2, 1, 5, 32)
    K, V = kv.update(k, v, 0)
    kv.update(k, v, 1)
    assert kv.num_items() == 5 and K.shape == (2, 1, 5, 32)
    K2, V2 = kv.update(k[:, :, :1], v[:, :, :1], 0)
    assert K2.shape == (2, 1, 6, 32)
    assert torch.allclose(K2[:, :, :5].float(), k.to(torch.bfloat16).float())
    assert torch.allclose(V2[:, :, 5].float(), v[:, :, 0].to(torch.bfloat16).float())
    assert len(kv.k_cache) == 2 and kv.v_cache[1].shape == (2, 1, 5, 32)


@pytest.mark.parametrize("H,W,S", [(480, 640, 224), (37, 51, 224), (224, 500, 224), (1000, 224, 448), (224, 224, 224)])
def test_pil_bicubic_restatement_is_bit_exact(H, W, S):
    """oracle/pil_resample.py + pghip.image.resample_coeffs == PIL Image.resize(BICUBIC) (Pillow 12.2.0), and the
    normalise table == the reference's rescale/normalise (processing_paligemma.py:22-35)."""
    from PIL import Image
    from oracle.pil_resample import resize_u8
    from pghip.image import normalise_lut, resample_coeffs
    img = np.random.default_rng(H * W + S).integers(0, 256, (H, W, 3), dtype=np.uint8)
    ref = np.array(Image.fromarray(img).resize((S, S), resample=Image.Resampling.BICUBIC))
    assert np.array_equal(resize_u8(img, S, resample_coeffs), ref)
    x = (np.arange(256, dtype=np.uint8) * (1 / 255.0)).astype(np.float32)
    assert np.array_equal(normalise_lut(), (x - np.float32(0.5)) / np.float32(0.5))


def test_frag_pack_layout_and_roundtrip():
    """weights.frag_pack puts W[16t+r][64c+16g+8s+e] at ((((t*K/64+c)*2+s)*64+16g+r)*8+e) (include/pghip.h
    PG_W_FRAG) and frag_unpack inverts it."""
    from pghip.weights import frag_pack, frag_unpack
    N, K = 48, 192
    w = torch.arange(N * K, dtype=torch.int64).reshape(N, K)
    p = frag_pack(w).reshape(-1)
    for (n, k) in [(0, 0), (17, 65), (47, 191), (31, 100), (5, 24)]:
        t, r, c, kk = n // 16, n % 16, k // 64, k % 64
        g, s, e = kk // 16, (kk % 16) // 8, kk % 8
        assert int(p[(((t * (K // 64) + c) * 2 + s) * 64 + 16 * g + r) * 8 + e]) == n * K + k
    assert torch.equal(frag_unpack(frag_pack(w)), w)
    with pytest.raises(ValueError):
        frag_pack(torch.zeros(40, 128))


def test_packed_weights_frag_flags():
    """Gemma matrices fragment-packed when every shape allows it (full size, tiny), row-major for toy TP shards."""
    from pghip.weights import PackedWeights, frag_unpack, rope_row_perm
    cfg = ocfg.TINY
    W = synth.generate_state_dict(cfg)
    P = PackedWeights(cfg, lambda k: torch.from_numpy(W[k]), device="cpu", parts=("text",))
    assert P.frag and P.wflag == 0x100 and P.vocab_local_pad % 16 == 0
    down = frag_unpack(P.tl[0]["down_w"]).float().numpy()
    want = W["language_model.model.layers.0.mlp.down_proj.weight"]
    assert np.array_equal(down[:, :want.shape[1]], want.astype(np.float32))
    lm = frag_unpack(P.lm_w).float().numpy()[:cfg["text_config"]["vocab_size"]]
    assert np.array_equal(lm, W["language_model.model.embed_tokens.weight"].astype(np.float32))
    P4 = PackedWeights(cfg, lambda k: torch.from_numpy(W[k]), device="cpu", parts=("text",), tp_rank=1, tp_world=4)
    assert not P4.frag and P4.wflag == 0


def test_packed_weights_refuse_attention_bias():
    """GemmaAttention with attention_bias=True adds q/k/v/o biases (modeling_gemma.py:295-298); the HIP q|k|v and
    o epilogues carry none, so packing must fail loudly instead of silently dropping them."""
    import copy
    from pghip.weights import PackedWeights
    cfg = copy.deepcopy(ocfg.TINY)
    W = synth.generate_state_dict(cfg)
    cfg["text_config"]["attention_bias"] = True
    with pytest.raises(NotImplementedError):
        PackedWeights(cfg, lambda k: torch.from_numpy(W[k]), device="cpu", parts=("text",))
    cfg["text_config"]["attention_bias"] = False
    Wb = dict(W, **{"language_model.model.layers.0.self_attn.q_proj.bias": np.zeros(1, np.float32)})
    with pytest.raises(NotImplementedError):
        PackedWeights(cfg, lambda k: torch.from_numpy(Wb[k]), device="cpu", parts=("text",))


def test_processor_call_matches_reference_fixture(golden):
    """PaliGemmaProcessor.__call__ (processing_paligemma.py:129-145,197-209) against the reference's own outputs on
    an offline tokenizer (tests/golden/tokenizer, make_golden.py make_processor): the added <image> / <seg> / <loc>
    token ids, the list-repr prompt string's token ids and attention mask (prompts with <loc>/<seg> tokens among
    them), and the pixel values, token for token."""
    from transformers import AutoTokenizer
    from processing_paligemma import PaliGemmaProcessor
    from PIL import Image
    g = golden("processor")
    img = Image.fromarray(np.random.default_rng(99).integers(0, 256, (1, 300, 300, 3), dtype=np.uint8)[0])
    for j, prompt in enumerate(g["prompts"].tolist()):
        tok = AutoTokenizer.from_pretrained(os.path.join(ROOT, "tests", "golden", "tokenizer"))
        p = PaliGemmaProcessor(tok, num_image_tokens=16, image_size=56)
        res = p(images=[img], text=[prompt])
        assert np.array_equal(res["input_ids"].numpy(), g[f"p{j}_input_ids"]), prompt
        assert np.array_equal(res["attention_mask"].numpy(), g[f"p{j}_attention_mask"]), prompt
        assert np.array_equal(res["pixel_values"].numpy(), g[f"p{j}_pixel_values"]), prompt
        if j == 0:
            assert tok.image_token_id == int(g["image_token_id"]) and len(tok) == int(g["vocab_len"])
            assert tok.convert_tokens_to_ids(["<seg000>", "<seg127>", "<loc0000>", "<loc1023>"]) == \
                g["added_ids"].tolist()


def test_load_hf_model_remaps_reports_and_drops(tmp_path):
    """utils.load_hf_model on an HF-layout checkpoint (newer transformers names: model.vision_tower.vision_model.*,
    model.language_model.*, model.multi_modal_projector.*, q_proj / position_embedding) with a projector bias and
    no lm_head bias: remap_hf_keys=True loads every SigLIP / Gemma / projector tensor (values equal), the projector
    bias is dropped with a warning (the reference projector has bias=False) or refused, the missing lm_head bias is
    reported (or zeroed on request), and strict=True raises on what strict=False only reports."""
    import json as _json
    import shutil
    from safetensors.torch import save_file
    from utils import load_hf_model
    cfg = ocfg.TINY
    W = synth.generate_state_dict(cfg)
    inv = {"vision_tower.model.": "model.vision_tower.vision_model.", "positional_embeddings": "position_embedding",
           "query_proj": "q_proj", "key_proj": "k_proj", "value_proj": "v_proj",
           "language_model.model.": "model.language_model.", "multi_modal_projector.": "model.multi_modal_projector."}
    hf = {}
    for k, v in W.items():
        if k == "language_model.lm_head.bias":
            continue                                   # HF PaliGemma has no lm_head bias
        h = k
        for a, b in inv.items():
            h = h.replace(a, b)
        hf[h] = torch.from_numpy(v.copy())
    hf["model.multi_modal_projector.linear.bias"] = torch.zeros(cfg["projection_dim"])
    d = tmp_path / "ckpt"
    d.mkdir()
    save_file(hf, str(d / "model.safetensors"))
    (d / "config.json").write_text(_json.dumps(cfg))
    for f in os.listdir(os.path.join(ROOT, "tests", "golden", "tokenizer")):
        shutil.copy(os.path.join(ROOT, "tests", "golden", "tokenizer", f), d / f)
    with pytest.warns(UserWarning, match="multi_modal_projector.linear.bias"):
        model, tok, rep = load_hf_model(str(d), "cpu", remap_hf_keys=True, return_report=True)
    sd = model.state_dict()
    for k, v in W.items():
        if k != "language_model.lm_head.bias":
            assert np.array_equal(sd[k].float().numpy(), v), k
    assert rep.missing == ["language_model.lm_head.bias"] and rep.unexpected == [] and rep.remapped > 0
    assert model.language_model.lm_head.weight is model.language_model.model.embed_tokens.weight
    with pytest.raises(ValueError, match="bias"):
        load_hf_model(str(d), "cpu", remap_hf_keys=True, projector_bias="refuse")
    with pytest.warns(UserWarning):
        model, tok, rep = load_hf_model(str(d), "cpu", remap_hf_keys=True, zero_missing_lm_head_bias=True,
                                        return_report=True)
    assert rep.missing == [] and float(model.language_model.lm_head.bias.detach().abs().sum()) == 0.0
    with pytest.warns(UserWarning, match="missing"):
        _, _, rep = load_hf_model(str(d), "cpu", return_report=True)     # the reference's behaviour: no remap
    assert any(k.startswith("vision_tower.model.") for k in rep.missing) and len(rep.unexpected) > 0
    with pytest.raises(KeyError):
        load_hf_model(str(d), "cpu", strict=True)


@pytest.mark.parametrize("nkv", [1, 2])
def test_kvcache_grow_and_partial_repack_keep_decode_order_copies(nkv):
    """modeling_gemma.KVCache on CPU tensors: appends of 40 then 1-token steps past the first capacity (64 -> grown),
    with nkv kv heads.  The canonical K / V^T views equal the appended states, and the decode-order copies kd / vd that
    update() repacks block by block (only the 32-key blocks it touched) and that KVStore.copy_prefix_from carries over
    equal ops.decode_cache_pack of the whole canonical cache, head by head."""
    from modeling_gemma import KVCache
    from pghip import ops
    torch.manual_seed(0)
    B, hd, layers = 2, 32, 2
    kv = KVCache()
    ks, vs = [[] for _ in range(layers)], [[] for _ in range(layers)]
    for L in [40] + [1] * 50:
        for i in range(layers):
            k = torch.randn(B, nkv, L, hd).bfloat16()
            v = torch.randn(B, nkv, L, hd).bfloat16()
            ks[i].append(k), vs[i].append(v)
            kv.update(k, v, i)
    st = kv._store
    n = kv.num_items()
    assert n == 90 and st.Smax >= 128
    for i in range(layers):
        K, V = kv.k_cache[i], kv.v_cache[i]
        assert torch.equal(K, torch.cat(ks[i], 2)) and torch.equal(V, torch.cat(vs[i], 2))
        kd, vd = ops.decode_cache_pack(st.k[i], st.vt[i], nkv)
        nb = -(-n // 32) * 32
        got_k = st.kd[i].view(B, nkv, st.Smax, hd)[:, :, :nb]
        got_v = st.vd[i].view(B, nkv, st.Smax, hd)[:, :, :nb]
        assert torch.equal(got_k, kd[:, :, :nb]) and torch.equal(got_v, vd[:, :, :nb])


def test_engine_refuses_split_knobs_the_kernels_reject(monkeypatch):
    """A split-K knob outside what the in-kernel finalisation takes (PG_SPLIT_DOWN=16 at batch 16 once made
    pg_gemm_fused(F32_FIN) fail at launch) is refused when the engine is built, before any launch."""
    from pghip import configs, engine, weights
    cfg = configs.TINY
    W = synth.generate_state_dict(cfg)
    P = weights.PackedWeights(cfg, lambda k: torch.from_numpy(W[k]), device="cpu")
    engine.PaliGemmaEngine(cfg, P, device="cpu")
    monkeypatch.setenv("PG_SPLIT_DOWN", "16")
    with pytest.raises(ValueError, match="split-K 16"):
        engine.PaliGemmaEngine(cfg, P, device="cpu")


def test_bench_refuses_world_size_other_than_gpus():
    """bench.py under a launcher whose WORLD_SIZE differs from --gpus fails loudly before touching the device (the
    driver's N-GPU line must come from N ranks)."""
    import subprocess
    import sys
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr and "--gpus 4" in r.stderr, r.stderr[-2000:]
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "0"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "--gpus must be >= 1" in r.stderr, r.stderr[-2000:]


_SNIPPET = """
0000000000001000 <k>:
\tv_mfma_f32_16x16x32_bf16 a[0:3], v[6:9], v[10:13], 0     // 000000001000: D3B58000 02028906
\ts_cmpk_lt_i32 s23, 0x80                                    // 000000001008: B3170080
\ts_cbranch_scc1 3                                           // 00000000100C: BF850003 <k+0x1c>
\ts_nop 7                                                    // 000000001010: BF800007
\ts_nop 7                                                    // 000000001014: BF800007
\ts_nop 7                                                    // 000000001018: BF800007
\tv_accvgpr_read_b32 v9, a3                                  // 00000000101C: D3D84009 18000103
\ts_endpgm                                                   // 000000001024: BF810000
"""


def test_mfma_hazard_scan_catches_a_branch_skipping_read():
    """tests/mfma_hazard.py on the round-5 pattern: the fall-through path waits out the MFMA's latency (s_nops), the
    taken branch reaches a read of its accumulator 2 wait states after it -- reported; with the branch removed, not."""
    import mfma_hazard as H
    bad, n = H.find_hazards(_SNIPPET)
    assert n == 1 and len(bad) == 1 and bad[0][2].startswith("v_accvgpr_read_b32 v9, a3") and bad[0][3] == 2, bad
    bad, _ = H.find_hazards(_SNIPPET.replace("s_cbranch_scc1 3", "s_nop 0"))
    assert bad == [], bad


def test_library_has_no_mfma_result_read_hazards():
    """Every kernel of the built libpghip.so (gfx950 code objects, disassembled): no instruction on any path after a
    v_mfma* reads its result before the MFMA's wait states have elapsed (tests/mfma_hazard.py).  Found, and fenced, in
    round 6: attn_decode_wg_kernel's one-round branch stored the accumulators one instruction after the last MFMA."""
    import mfma_hazard as H
    from pghip import _lib
    if not all(os.path.exists(os.path.join(H.LLVM, t)) for t in ("llvm-objdump", "llvm-objcopy",
                                                                   "clang-offload-bundler")):
        pytest.skip("ROCm LLVM tools not present")
    cos = H.code_objects(_lib.LIB_PATH)
    assert len(cos) >= 4
    total = 0
    for co in cos:
        bad, n = H.find_hazards(H.disassemble(co))
        total += n
        assert bad == [], bad[:5]
    assert total > 10000, total                      # the GEMM / GEMV / attention kernels were all scanned


def test_c_abi_header_compiles_as_c_and_cpp():
    """include/pghip.h is the drop-in boundary a C / C++ binding includes: it must compile on its own as both (round 6
    found a missing enum comma that only a compiler would catch)."""
    import shutil
    import subprocess
    import tempfile
    inc = os.path.join(ROOT, "include")
    src = '#include "pghip.h"\nint main(void) { return (int)PG_EPI_F32_RES + (int)sizeof(PgFusedArgs) * 0; }\n'
    with tempfile.TemporaryDirectory() as d:
        for cc, ext in (("gcc", "c"), ("g++", "cpp")):
            if shutil.which(cc) is None:
                pytest.skip(f"{cc} not installed")
            f = os.path.join(d, "t." + ext)
            open(f, "w").write(src)
            r = subprocess.run([cc, "-fsyntax-only", "-Wall", "-D__HIP_PLATFORM_AMD__", "-I", inc, "-I",
                                "/opt/rocm/include", f], capture_output=True, text=True)
            assert r.returncode == 0, (cc, r.stderr[-2000:])
