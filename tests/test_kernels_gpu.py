"""Per-kernel numerics on the HIP device: each libpghip entry point against a plain
PyTorch fp32 reference of the same op on the same (bf16-representable) inputs."""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("needs the HIP device")
    from pghip import _lib
    _lib.load()


def err(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def rnd(*shape, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(torch.bfloat16).cuda()


def test_synth_fill_bit_identical_to_numpy():
    from oracle import synth
    from pghip import synthetic
    for name, shape in [("language_model.model.layers.3.mlp.gate_proj.weight", (64, 2048)),
                        ("vision_tower.model.encoder.layers.0.layer_norm1.weight", (1152,)),
                        ("language_model.lm_head.bias", (4096,))]:
        ref = synth.generate(name, shape)
        g32 = synthetic.generate(name, shape, dtype=torch.float32).cpu().numpy()
        g16 = synthetic.generate(name, shape, dtype=torch.bfloat16).float().cpu().numpy()
        assert np.array_equal(ref.view(np.uint32), g32.view(np.uint32)), name
        assert np.array_equal(ref, g16), name


@pytest.mark.parametrize("M", [1, 3, 16, 17, 200, 300])
@pytest.mark.parametrize("N,K", [(256, 128), (2560, 2048), (300, 192)])
def test_gemm_plain_and_bias(M, N, K):
    from pghip import ops
    A, W = rnd(M, K, seed=1), rnd(N, K, scale=1 / math.sqrt(K), seed=2)
    bias = torch.randn(N).cuda()
    ref = A.float() @ W.float().t() + bias
    out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    ops.gemm(A, W, out, bias=bias)
    assert err(out, ref) < 1e-2
    outf = torch.empty(M, N, dtype=torch.float32, device="cuda")
    ops.gemm(A, W, outf, epi=ops.EPI_F32, bias=bias)
    assert err(outf, ref) < 1e-5


@pytest.mark.parametrize("M", [1, 8, 64, 264])
def test_gemm_split_k_partials(M):
    from pghip import ops
    K, N = 4096, 512
    A, W = rnd(M, K, seed=3), rnd(N, K, scale=1 / 64, seed=4)
    bias = torch.randn(N).cuda()
    for s in (1, 2, 4):
        part = torch.empty(s, M, N, dtype=torch.float32, device="cuda")
        ops.gemm(A, W, part, epi=ops.EPI_F32, bias=bias, ksplit=s)
        assert err(part.sum(0), A.float() @ W.float().t() + bias) < 1e-5


@pytest.mark.parametrize("tile", ["g256", "t64", "n64"])
def test_gemm_split_k_past_the_end_of_k(tile):
    """A split whose ceil-sized k-slices run past K (32 k-tiles in 12 slices of 3: slice 11 is empty) stores a zero
    slab and reads nothing past K, on the 256x256 kernel (264 x 32768: 256 tiles), the 64-row and the 64x64 tiles."""
    from pghip import ops
    M, N, K, s = (264, 32768, 2048, 12) if tile == "g256" else (100, 512, 2048, 12)
    A, W = rnd(M, K, seed=51), rnd(N, K, scale=1 / 45, seed=52)
    part = torch.full((s, M, N), float("nan"), dtype=torch.float32, device="cuda")
    ops.gemm(A, W, part, epi=ops.EPI_F32 | (ops.TILE_N64 if tile == "n64" else 0), ksplit=s)
    torch.cuda.synchronize()
    assert (part[11] == 0).all()
    assert err(part.sum(0), A.float() @ W.float().t()) < 1e-5


@pytest.mark.parametrize("M,N,K,s", [(300, 256, 512, 2), (16512, 2048, 2048, 1), (16512, 2048, 4096, 3)])
def test_gemm_slab_rows_row_blocks(M, N, K, s):
    """PgFusedArgs.slab_rows: a split-K fp32 GEMM issued as a head of whole 256-row tiles plus a ragged tail,
    both writing into one [s][M][N] slab tensor (engine._row_head), equals the one-launch result."""
    from pghip import ops
    A, W = rnd(M, K, seed=31), rnd(N, K, scale=1 / math.sqrt(K), seed=32)
    Mh = M // 256 * 256
    one = torch.empty(s, M, N, dtype=torch.float32, device="cuda")
    ops.gemm(A, W, one, epi=ops.EPI_F32, ksplit=s)
    two = torch.full((s, M, N), float("nan"), dtype=torch.float32, device="cuda")
    fr = ops.fused_args(slab_rows=M)
    ops.gemm_fused(A[:Mh], W, two, fr, epi=ops.EPI_F32, M=Mh, ksplit=s, ldc=N)
    ops.gemm_fused(A[Mh:], W, two.view(-1)[Mh * N:], fr, epi=ops.EPI_F32, M=M - Mh, ksplit=s, ldc=N)
    assert not torch.isnan(two).any()
    ref = A.float() @ W.float().t()
    assert err(two.sum(0), ref) < 1e-5 and err(one.sum(0), ref) < 1e-5
    assert torch.equal(two[:, :Mh], one[:, :Mh])        # the head's tiles are the same launches' tiles


def test_slab_sum_into_strided_rows():
    from pghip import ops
    part = torch.randn(5, 40, 64).cuda()
    out = torch.full((3, 100, 64), 7.0, device="cuda")
    ops.slab_sum(part, out[0, 60:])
    assert torch.allclose(out[0, 60:], part.sum(0), atol=1e-6, rtol=0)
    assert (out[0, :60] == 7.0).all() and (out[1:] == 7.0).all()


@pytest.mark.parametrize("M,N,K,epi,s", [(300, 300, 128, "gelu", 1), (300, 300, 128, "f32", 2),
                                         (16384, 1152, 1152, "f32", 1), (16384, 4304, 1152, "gelu", 1)])
def test_gemm_column_blocks(M, N, K, epi, s):
    """engine._gemm_cols: whole 256-column tiles + the ragged remaining columns as two GEMMs on column views
    of one output (bias sliced, slabs keep their stride) equal the one-launch GEMM."""
    from pghip import ops
    A, W = rnd(M, K, seed=33), rnd(N, K, scale=1 / math.sqrt(K), seed=34)
    bias = torch.randn(N).cuda() * 0.1
    e = ops.EPI_BF16_GELU if epi == "gelu" else ops.EPI_F32
    shape = (M, N) if epi == "gelu" else (s, M, N)
    dt = torch.bfloat16 if epi == "gelu" else torch.float32
    one = torch.empty(shape, dtype=dt, device="cuda")
    two = torch.full(shape, float("nan"), dtype=dt, device="cuda")
    ops.gemm(A, W, one, epi=e, bias=bias, ksplit=s)
    Nh = N // 256 * 256
    ops.gemm(A, W[:Nh], two[..., :Nh], epi=e, bias=bias[:Nh], ksplit=s)
    ops.gemm(A, W[Nh:], two[..., Nh:], epi=e, bias=bias[Nh:], ksplit=s)
    assert not torch.isnan(two.float()).any()
    got = two.float() if epi == "gelu" else two.sum(0)
    want = A.float() @ W.float().t() + bias
    want = torch.nn.functional.gelu(want, approximate="tanh") if epi == "gelu" else want
    assert err(got, want) < (1e-2 if epi == "gelu" else 1e-5)


@pytest.mark.parametrize("M", [1, 16, 150])
def test_gemm_gelu_and_gelu_mul(M):
    from pghip import ops
    K, I = 256, 320
    A = rnd(M, K, seed=5)
    g, u = rnd(I, K, scale=0.1, seed=6), rnd(I, K, scale=0.1, seed=7)
    gu = torch.stack([g.view(I // 16, 16, K), u.view(I // 16, 16, K)], 1).reshape(2 * I, K).contiguous()
    out = torch.empty(M, I, dtype=torch.bfloat16, device="cuda")
    ops.gemm(A, gu, out, epi=ops.EPI_BF16_GELU_MUL)
    ref = torch.nn.functional.gelu(A.float() @ g.float().t(), approximate="tanh") * (A.float() @ u.float().t())
    assert err(out, ref) < 1e-2
    bias = torch.randn(I).cuda() * 0.1
    out2 = torch.empty(M, I, dtype=torch.bfloat16, device="cuda")
    ops.gemm(A, g, out2, epi=ops.EPI_BF16_GELU, bias=bias)
    assert err(out2, torch.nn.functional.gelu(A.float() @ g.float().t() + bias, approximate="tanh")) < 1e-2


@pytest.mark.parametrize("M", [256, 264, 288])
def test_gemm_tile_m1_batch1_prefill(M):
    """PG_TILE_M1 (all 256..288 rows in one row tile; the batch-1 prefill Gemma gate/up, down and o) against a
    torch fp32 matmul: the gelu*up epilogue, and fp32 split-K slabs at the engine's splits (8, 16) with a
    ragged last k-slice; rows past M are never written."""
    from pghip import ops
    K, I = 2048, 640
    A = rnd(M, K, seed=41)
    g, u = rnd(I, K, scale=1 / math.sqrt(K), seed=42), rnd(I, K, scale=1 / math.sqrt(K), seed=43)
    gu = torch.stack([g.view(I // 16, 16, K), u.view(I // 16, 16, K)], 1).reshape(2 * I, K).contiguous()
    out = torch.full((M + 8, I), 7.0, dtype=torch.bfloat16, device="cuda")
    ops.gemm(A, gu, out[:M], epi=ops.EPI_BF16_GELU_MUL | ops.TILE_M1)
    ref = torch.nn.functional.gelu(A.float() @ g.float().t(), approximate="tanh") * (A.float() @ u.float().t())
    assert err(out[:M], ref) < 1e-2 and (out[M:] == 7.0).all()
    for K2, s in ((2048, 8), (3072 + 64, 16)):
        A2, W2 = rnd(M, K2, seed=44), rnd(512, K2, scale=1 / math.sqrt(K2), seed=45)
        bias = torch.randn(512).cuda() * 0.1
        part = torch.empty(s, M, 512, dtype=torch.float32, device="cuda")
        ops.gemm(A2, W2, part, epi=ops.EPI_F32 | ops.TILE_M1, ksplit=s, bias=bias)
        assert err(part.sum(0), A2.float() @ W2.float().t() + bias) < 1e-4
    with pytest.raises(RuntimeError):                   # outside 256..288 rows the flag is refused
        ops.gemm(A[:200], gu, out[:200], epi=ops.EPI_BF16_GELU_MUL | ops.TILE_M1)


@pytest.mark.parametrize("M", [17, 64, 256, 264, 300])
def test_gemm_tile_n64_bit_identical(M):
    """PG_TILE_N64 (64 x 64 output tiles) computes every output from the same 16 x 16 x 32 MFMA sequence as the
    64 x 128 / 128 x 128 / 256 x 256 tilings: bit-identical bf16, gelu*up, fp32 split-K slabs (fragment-packed W
    too) and fp8 outputs, and within bf16 rounding of a torch fp32 matmul."""
    from pghip import ops
    from pghip.weights import frag_pack
    K, N = 1024, 704
    A, W = rnd(M, K, seed=61), rnd(N, K, scale=1 / math.sqrt(K), seed=62)
    bias = torch.randn(N).cuda() * 0.1
    for epi in (ops.EPI_BF16, ops.EPI_BF16_GELU_MUL):
        a = torch.empty(M, N // (2 if epi == ops.EPI_BF16_GELU_MUL else 1), dtype=torch.bfloat16, device="cuda")
        b = torch.full_like(a, float("nan"))
        kw = {} if epi == ops.EPI_BF16_GELU_MUL else {"bias": bias}
        ops.gemm(A, W, a, epi=epi, **kw)
        ops.gemm(A, W, b, epi=epi | ops.TILE_N64, **kw)
        assert torch.equal(a, b)
        if epi == ops.EPI_BF16:
            assert err(b, A.float() @ W.float().t() + bias) < 1e-2
    Wf = frag_pack(W)
    for s in (1, 3):
        a = torch.empty(s, M, N, dtype=torch.float32, device="cuda")
        b = torch.full_like(a, float("nan"))
        ops.gemm(A, W, a, epi=ops.EPI_F32, ksplit=s, bias=bias)
        ops.gemm(A, Wf, b, epi=ops.EPI_F32 | ops.W_FRAG | ops.TILE_N64, ksplit=s, bias=bias)
        assert torch.equal(a, b)
        assert err(b.sum(0), A.float() @ W.float().t() + bias) < 1e-4


@pytest.mark.parametrize("M", [1, 2, 5, 16, 17, 264])
@pytest.mark.parametrize("N,K", [(256, 128), (2048, 2048), (320, 1024)])
def test_gemm_frag_packed_weights_bit_identical(M, N, K):
    """W_FRAG (fragment-packed W, the Gemma HBM layout) feeds the GEMV and the tile GEMM exactly the
    values the row-major layout does: outputs are bit-identical, for every Gemma epilogue."""
    from pghip import ops
    from pghip.weights import frag_pack
    A, W = rnd(M, K, seed=21), rnd(N, K, scale=1 / math.sqrt(K), seed=22)
    Wp = frag_pack(W)
    bias = torch.randn(N).cuda()
    for epi, dt, ks in ((ops.EPI_BF16, torch.bfloat16, 1), (ops.EPI_F32, torch.float32, 1),
                        (ops.EPI_F32, torch.float32, 4), (ops.EPI_BF16_GELU_MUL, torch.bfloat16, 1)):
        n_out = N // 2 if epi == ops.EPI_BF16_GELU_MUL else N
        shape = (ks, M, n_out) if epi == ops.EPI_F32 else (M, n_out)
        a, b = torch.empty(shape, dtype=dt, device="cuda"), torch.empty(shape, dtype=dt, device="cuda")
        bb = None if epi == ops.EPI_BF16_GELU_MUL else bias
        ops.gemm(A, W, a, epi=epi, bias=bb, ksplit=ks)
        ops.gemm(A, Wp, b, epi=epi | ops.W_FRAG, bias=bb, ksplit=ks)
        assert torch.equal(a, b), (epi, ks)


def test_gemm_vt_and_pos_epilogues():
    from pghip import ops
    M, K, hv = 40, 192, 64
    A, W = rnd(M, K, seed=8), rnd(3 * hv, K, scale=0.1, seed=9)
    bias = torch.randn(3 * hv).cuda()
    out = torch.zeros(M, 3 * hv, dtype=torch.bfloat16, device="cuda")
    vt = torch.zeros(hv, M, dtype=torch.bfloat16, device="cuda")
    ops.gemm(A, W, out, epi=ops.EPI_BF16_VT, bias=bias, aux_out=vt, aux_ld=M, aux_n=2 * hv)
    ref = A.float() @ W.float().t() + bias
    assert err(out[:, :2 * hv], ref[:, :2 * hv]) < 1e-2
    assert err(vt, ref[:, 2 * hv:].t()) < 1e-2
    pos = torch.randn(8, 3 * hv).cuda()
    o2 = torch.empty(M, 3 * hv, dtype=torch.float32, device="cuda")
    ops.gemm(A, W, o2, epi=ops.EPI_F32_POS, bias=bias, aux=pos, aux_rows=8)
    assert err(o2, ref + pos[torch.arange(M) % 8]) < 1e-5


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("H", [128, 1152, 2048])
def test_norm_residual(mode, H):
    from pghip import ops
    M, S = 37, 3
    resid = torch.randn(M, H).cuda()
    part = torch.randn(S, M, H).cuda()
    w, b = torch.randn(H).cuda() * 0.1 + (1 if mode == 0 else 0), torch.randn(H).cuda() * 0.1
    x = resid + part.sum(0)
    if mode == 0:
        ref = torch.nn.functional.layer_norm(x, (H,), w, b, 1e-6)
    else:
        ref = x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + 1e-6) * (1 + w)
    out = torch.empty(M, H, dtype=torch.bfloat16, device="cuda")
    of = torch.empty(M, H, dtype=torch.float32, device="cuda")
    ops.norm_residual(resid, w, b=b if mode == 0 else None, mode=mode, partials=part, nsplit=S, out=out, out_f32=of)
    assert err(resid, x) < 1e-6
    assert err(of, ref) < 1e-5
    assert err(out, ref) < 1e-2


def _attn_ref(q, k, v, scale, mask=None):
    s = (q.float() @ k.float().transpose(-1, -2)) * scale
    if mask is not None:
        s = s + mask
    return torch.softmax(s, -1) @ v.float()


@pytest.mark.parametrize("B,N,nh,hd", [(1, 256, 16, 72), (2, 16, 8, 24), (1, 100, 4, 64),
                                       (4, 256, 16, 72), (10, 104, 16, 72),     # LDS-staged kernel
                                       (1, 1024, 16, 72), (16, 1024, 16, 72),  # pt-448 (B = 1, BASELINE configs[2])
                                       (2, 4096, 16, 72)])                     # pt-896 (BASELINE configs[4])
def test_attention_vision_layout(B, N, nh, hd):
    """SigLIP: q/k from the fused QKV buffer, V^T from the transposed side buffer.  Large batches take
    the LDS-staged kernel (>= 1024 sixteen-row groups), including a ragged last key block (N=104)."""
    from pghip import ops
    hv = nh * hd
    M = B * N
    qkv = rnd(M, 3 * hv, seed=10)
    vt = torch.zeros(hv, M + 32, dtype=torch.bfloat16, device="cuda")
    vt[:, :M] = qkv[:, 2 * hv:].t()
    o = torch.empty(M, hv, dtype=torch.bfloat16, device="cuda")
    ops.attention(qkv, 3 * hv, o, hv, qkv[:, hv:], N * 3 * hv, hd, 3 * hv, vt, N, hd * (M + 32), M + 32,
                  B=B, Lq=N, Lkv=N, Hq=nh, Hkv=nh, D=hd, scale=hd ** -0.5)
    x = qkv.view(B, N, 3, nh, hd).permute(2, 0, 3, 1, 4)
    ref = _attn_ref(x[0], x[1], x[2], hd ** -0.5).permute(0, 2, 1, 3).reshape(M, hv)
    assert err(o, ref) < 2e-2


@pytest.mark.parametrize("B,L,nh,nkv,hd,masked", [(1, 264, 8, 1, 256, False), (2, 24, 4, 1, 32, True),
                                                  (1, 70, 8, 2, 64, False),
                                                  (8, 300, 8, 1, 256, False), (16, 130, 8, 1, 256, True),
                                                  (14, 300, 8, 1, 256, False),    # 12-wave flash kernel
                                                  (1, 1032, 8, 1, 256, False), (16, 1032, 8, 1, 256, False),  # pt-448
                                                  (2, 4104, 8, 1, 256, False),                               # pt-896
                                                  (32, 1000, 8, 1, 256, False)])      # 8 waves x 32 rows, 32-key blocks
def test_attention_cache_layout_prefill_and_decode(B, L, nh, nkv, hd, masked):
    """Gemma: MQA/GQA from the static cache (K rows, V^T), prefill and split-KV decode, up to the pt-896 prefix
    (4104 keys: the multi-block, multi-round decode splits of BASELINE configs[4] over 4.2 k keys)."""
    from pghip import ops
    Smax = max(320, (L + 8 + 63) // 64 * 64)
    kvd = nkv * hd
    q = rnd(B * L, nh * hd, seed=11)
    kc = torch.zeros(B, Smax, kvd, dtype=torch.bfloat16, device="cuda")
    vtc = torch.zeros(B, kvd, Smax, dtype=torch.bfloat16, device="cuda")
    kk, vv = rnd(B, L, kvd, seed=12), rnd(B, L, kvd, seed=13)
    kc[:, :L] = kk
    vtc[:, :, :L] = vv.transpose(1, 2)
    mask = None
    if masked:
        mask = torch.triu(torch.full((L, L), -1e9), 1).expand(B, L, L).contiguous().cuda()
    o = torch.empty(B * L, nh * hd, dtype=torch.bfloat16, device="cuda")
    ops.attention(q, nh * hd, o, nh * hd, kc, Smax * kvd, hd, kvd, vtc, kvd * Smax, hd * Smax, Smax,
                  B=B, Lq=L, Lkv=L, Hq=nh, Hkv=nkv, D=hd, scale=hd ** -0.5, mask=mask,
                  mask_bs=(L * L if masked else 0), mask_rs=(L if masked else 0))
    qh = q.view(B, L, nh, hd).transpose(1, 2)
    g = nh // nkv
    kh = kk.view(B, L, nkv, hd).transpose(1, 2).repeat_interleave(g, 1)
    vh = vv.view(B, L, nkv, hd).transpose(1, 2).repeat_interleave(g, 1)
    ref = _attn_ref(qh, kh, vh, hd ** -0.5, None if mask is None else mask[:, None])
    assert err(o, ref.transpose(1, 2).reshape(B * L, nh * hd)) < 2e-2
    # decode: the last row's query against all L keys, split-KV + combine, Lkv from device memory
    if masked:
        return
    qd = q.view(B, L, nh * hd)[:, -1].contiguous()
    lkv = torch.tensor([L - 1], dtype=torch.int32, device="cuda")
    SK = 64
    nsplit = ((Smax + SK - 1) // SK + 3) // 4 * 4
    dt = (hd + 15) // 16 * 16
    po = torch.empty(B * nkv * nsplit * 16 * dt, device="cuda")
    pml = torch.empty(B * nkv * nsplit * 16 * 2, device="cuda")
    od = torch.empty(B, nh * hd, dtype=torch.bfloat16, device="cuda")
    ops.attention(qd, nh * hd, od, nh * hd, kc, Smax * kvd, hd, kvd, vtc, kvd * Smax, hd * Smax, Smax,
                  B=B, Lq=1, Lkv=1, lkv_dev=lkv, Hq=nh, Hkv=nkv, D=hd, scale=hd ** -0.5, split_keys=SK,
                  nsplit=nsplit, part_o=po, part_ml=pml)
    ops.attn_combine(po, pml, od, nh * hd, B=B, Hq=nh, Hkv=nkv, D=hd, nsplit=nsplit)
    assert err(od, ref[:, :, -1].reshape(B, nh * hd)) < 2e-2
    # kcap = Smax: every split's first block is loaded before the kv length is read (rows past it masked after
    # the loads land).  One-block splits (32 keys): bit-identical to the kcap = 0 kernel.  2- and 4k-block splits
    # at head_dim 256 run one wave per block, k rounds per wave, merged in LDS (attn_decode_wg_kernel): same bound.
    for sk in (32, 64, 128, 256, 384, 512):
        ns = ((Smax + sk - 1) // sk + 3) // 4 * 4
        po1 = torch.empty(B * nkv * ns * 16 * dt, device="cuda")
        pml1 = torch.empty(B * nkv * ns * 16 * 2, device="cuda")
        outs = []
        kd, vd = ops.decode_cache_pack(kc, vtc, nkv)      # kcap > 0 reads the decode-order copies
        for kcap in (0, Smax):
            od2 = torch.empty_like(od)
            ops.attention(qd, nh * hd, od2, nh * hd, kc, Smax * kvd, hd, kvd, vtc, kvd * Smax, hd * Smax, Smax,
                          B=B, Lq=1, Lkv=1, lkv_dev=lkv, Hq=nh, Hkv=nkv, D=hd, scale=hd ** -0.5, split_keys=sk,
                          nsplit=ns, part_o=po1, part_ml=pml1, kcap=kcap, kd=kd, vd=vd)
            ops.attn_combine(po1, pml1, od2, nh * hd, B=B, Hq=nh, Hkv=nkv, D=hd, nsplit=ns)
            assert err(od2, ref[:, :, -1].reshape(B, nh * hd)) < 2e-2, (sk, kcap)
            outs.append(od2)
        if sk == 32:
            assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("B,L,nh,nkv,hd,kcap", [(3, 200, 8, 1, 256, 256), (4, 40, 4, 1, 32, 64),
                                                 (5, 300, 8, 2, 256, 448),                # GQA: 2 kv heads
                                                 (16, 1033, 8, 1, 256, 1216),             # pt-448 x16 decode
                                                 (32, 4169, 8, 1, 256, 4224),             # pt-896 x32 decode
                                                 (8, 97, 8, 1, 256, 128)])
def test_attn_decode_fused(B, L, nh, nkv, hd, kcap):
    """pg_attn_decode (split-KV attention + in-launch merge, B > 2) against fp32 softmax attention over the first L
    cached keys; rows past L hold finite stale values (the static cache after a longer request), every split plan
    (2 / 4 waves, 1..16 splits, several rounds) agrees, repeated calls are bit-identical and leave the tickets zero.
    Where the plan allows it (one kv head, 4 waves) the second call also writes the fp8 row copy, which must equal
    pg_quant_fp8 of the bf16 output byte for byte (ABI 7).  The staggered form (PG_ATTN_PIPE: next block's loads
    between the phases, contiguous per-split block ranges) is bit-identical to the plain one."""
    from pghip import ops
    kvd = nkv * hd
    q = rnd(B, nh * hd, seed=31)
    kc = rnd(B, kcap, kvd, seed=32)                  # stale finite rows past L
    vtc = rnd(B, kvd, kcap, seed=33)
    lkv = torch.tensor([L - 1], dtype=torch.int32, device="cuda")
    g = nh // nkv
    kf = kc[:, :L].float().view(B, L, nkv, hd).transpose(1, 2).repeat_interleave(g, 1)       # [B][nh][L][hd]
    vf = vtc[:, :, :L].float().view(B, nkv, hd, L).transpose(2, 3).repeat_interleave(g, 1)
    ref = _attn_ref(q.view(B, nh, 1, hd), kf, vf, hd ** -0.5).reshape(B, nh * hd)
    cnt = torch.zeros(B * nkv, dtype=torch.int32, device="cuda")
    kd, vd = ops.decode_cache_pack(kc, vtc, nkv)
    nblk = kcap // 32
    plans = {ops.decode_plan(B, nkv, kcap)}
    for nw in (2, 4):
        for ns in (1, 3, 16):
            if nw * ns <= nblk:
                plans.add((ns, nw, -(-nblk // (nw * ns))))
    outs = {}
    for plan in sorted(plans):
        ns = plan[0]
        po = torch.empty(B * nkv * ns * 16 * hd, device="cuda")
        pml = torch.empty(B * nkv * ns * 16 * 2, device="cuda")
        o = torch.empty(B, nh * hd, dtype=torch.bfloat16, device="cuda")
        q8ok = ops.attn_decode_q8_ok(nh, nkv, hd, plan[1])
        q8 = torch.full((B, nh * hd), 0x55, dtype=torch.uint8, device="cuda")
        q8s = torch.zeros(B, device="cuda")
        saved = ops.ATTN_PIPE
        try:
            for rep in range(3):
                ops.ATTN_PIPE = rep != 2
                ops.attn_decode(q, nh * hd, o, nh * hd, kd, vd,
                                B=B, Lkv=1, lkv_dev=lkv, Hq=nh, Hkv=nkv, D=hd, scale=hd ** -0.5, kcap=kcap, part_o=po,
                                part_ml=pml, counters=cnt, plan=plan, q8=q8 if rep == 1 and q8ok else None,
                                q8_scale=q8s if rep == 1 and q8ok else None)
                torch.cuda.synchronize()
                assert int(cnt.abs().sum()) == 0, plan
                if rep == 0:
                    first = o.clone()
                assert torch.equal(first, o), (plan, rep)
        finally:
            ops.ATTN_PIPE = saved
        if q8ok:
            r8, rs = ops.quant_fp8(o)
            assert torch.equal(q8, r8) and torch.equal(q8s, rs), plan
        assert err(o, ref) < 2e-2, plan
        outs[plan] = o
    base = next(iter(outs.values()))
    for plan, o in outs.items():
        assert err(o, base.float()) < 1e-2, plan


@pytest.mark.parametrize("B,L,nh,nkv,hd,nks", [(1, 264, 8, 1, 256, 5), (1, 256, 16, 16, 72, 4),
                                                (1, 100, 8, 1, 256, 5), (2, 130, 4, 2, 64, 8),
                                                (1, 264, 8, 1, 256, 0), (1, 256, 16, 16, 72, 0)])
def test_attention_prefill_key_split(B, L, nh, nkv, hd, nks):
    """Key-split prefill attention (batch-1 grids: each split walks its share of the 64-key blocks, writes (O, m, l),
    and pg_attention merges them): against a torch fp32 reference and the unsplit kernel, including splits left
    without keys (L = 100 in 5 splits of one block).  nks 0 = the engine's policy (ops.prefill_key_splits: 5 for the
    pt-224 Gemma prefill, 4 for SigLIP)."""
    from pghip import ops
    if nks == 0:
        nks = ops.prefill_key_splits(B, L, L, nh, nkv)
        assert nks == (5 if hd == 256 else 4)
    Smax = (L + 8 + 63) // 64 * 64
    kvd = nkv * hd
    q = rnd(B * L, nh * hd, seed=71)
    kc = torch.zeros(B, Smax, kvd, dtype=torch.bfloat16, device="cuda")
    vtc = torch.zeros(B, kvd, Smax, dtype=torch.bfloat16, device="cuda")
    kk, vv = rnd(B, L, kvd, seed=72), rnd(B, L, kvd, seed=73)
    kc[:, :L] = kk
    vtc[:, :, :L] = vv.transpose(1, 2)
    args = (q, nh * hd, None, nh * hd, kc, Smax * kvd, hd, kvd, vtc, kvd * Smax, hd * Smax, Smax)
    kw = dict(B=B, Lq=L, Lkv=L, Hq=nh, Hkv=nkv, D=hd, scale=hd ** -0.5)
    one = torch.empty(B * L, nh * hd, dtype=torch.bfloat16, device="cuda")
    ops.attention(*args[:2], one, *args[3:], **kw)
    no, nml = ops.prefill_split_workspace(B, L, nh, nkv, hd, nks)
    po = torch.full((no,), float("nan"), device="cuda")
    pml = torch.full((nml,), float("nan"), device="cuda")
    split = torch.full_like(one, float("nan"))
    ops.attention(*args[:2], split, *args[3:], nsplit=nks, part_o=po, part_ml=pml, **kw)
    g = nh // nkv
    qh = q.view(B, L, nh, hd).transpose(1, 2)
    kh = kk.view(B, L, nkv, hd).transpose(1, 2).repeat_interleave(g, 1)
    vh = vv.view(B, L, nkv, hd).transpose(1, 2).repeat_interleave(g, 1)
    ref = _attn_ref(qh, kh, vh, hd ** -0.5).transpose(1, 2).reshape(B * L, nh * hd)
    assert not torch.isnan(split.float()).any()
    assert err(split, ref) < 2e-2 and err(split, one) < 1e-2
    with pytest.raises(RuntimeError):                   # more splits than the merge takes
        ops.attention(*args[:2], split, *args[3:], nsplit=9, part_o=po, part_ml=pml, **kw)


def test_rope_kv_write_matches_reference_formula():
    from oracle import paligemma_oracle as O
    from pghip import engine, ops
    B, L, nh, nkv, hd, Smax = 2, 5, 4, 1, 32, 64
    qkv = rnd(B * L, (nh + 2 * nkv) * hd, seed=14)
    q0 = qkv.clone()
    pos = (torch.arange(L) + 1).repeat(B).to(torch.int32).cuda()
    cos_t, sin_t = engine.rope_tables(hd, 128, 10000.0, "cuda")
    kc = torch.zeros(B, Smax, nkv * hd, dtype=torch.bfloat16, device="cuda")
    vtc = torch.zeros(B, nkv * hd, Smax, dtype=torch.bfloat16, device="cuda")
    ops.rope_kv_write(qkv, pos, cos_t, sin_t, kc, vtc, T=B * L, L=L, Hq=nh, Hkv=nkv, D=hd, Smax=Smax, slot_base=3)
    x = q0.float().cpu().numpy().reshape(B, L, nh + 2, hd)
    cos, sin = O.rope_cos_sin(hd, pos.cpu().numpy().reshape(B, L))
    qr, kr = O.apply_rotary_pos_emb(x[:, :, :nh].transpose(0, 2, 1, 3), x[:, :, nh:nh + 1].transpose(0, 2, 1, 3),
                                    cos, sin)
    assert err(qkv[:, :nh * hd].float(), torch.from_numpy(qr.transpose(0, 2, 1, 3).reshape(B * L, -1))) < 1e-2
    assert err(kc[:, 3:3 + L].float(), torch.from_numpy(kr.transpose(0, 2, 1, 3).reshape(B, L, -1))) < 1e-2
    assert torch.equal(vtc[:, :, 3:3 + L].transpose(1, 2), q0.view(B, L, -1)[:, :, (nh + 1) * hd:])


def test_im2col_merge_rank():
    from pghip import ops
    B, C, H, p = 2, 3, 28, 14
    px = torch.randn(B, C, H, H).cuda()
    out = torch.empty(B * 4, 640, dtype=torch.bfloat16, device="cuda")
    ops.patch_im2col(px, p, out)
    ref = px.view(B, C, 2, p, 2, p).permute(0, 2, 4, 1, 3, 5).reshape(B * 4, C * p * p)
    assert torch.equal(out[:, :588], ref.to(torch.bfloat16)) and out[:, 588:].abs().max().item() == 0
    ids = torch.tensor([[9, 9, 2, 5, 0, 9], [9, 0, 9, 7, 9, 3]], dtype=torch.int64).cuda()
    rank = torch.empty(12, dtype=torch.int32, device="cuda")
    ops.image_rank(ids.view(-1), 9, rank)
    flat = ids.view(-1).cpu()
    assert rank.cpu().tolist() == [int((flat[:i] == 9).sum()) for i in range(12)]
    emb = rnd(16, 64, seed=15)
    feat = torch.randn(6, 64).cuda()
    res = torch.empty(12, 64, device="cuda")
    ops.embed_merge(ids.view(-1), rank, emb, feat, 6, res, image_id=9, pad_id=0, img_scale=0.125, normalizer=8.0)
    for i, t in enumerate(flat.tolist()):
        if t == 0:
            want = torch.zeros(64)
        elif t == 9:
            want = feat[int((flat[:i] == 9).sum())].cpu() * 0.125 * 8.0
        else:
            want = emb[t].float().cpu() * 8.0
        assert torch.allclose(res[i].cpu(), want), i


def test_argmax_first_index_and_state_advance():
    from pghip import ops
    V = 257216
    x = torch.randn(3, V).cuda()
    x[1, 1000] = 50.0
    x[1, 77] = 50.0
    ids = torch.empty(3, dtype=torch.int64, device="cuda")
    ws = torch.empty(3 * 64 * 2, device="cuda")
    hist = torch.zeros(4, 3, dtype=torch.int64, device="cuda")
    step = torch.tensor([2], dtype=torch.int32, device="cuda")
    pos = torch.tensor([5, 6, 7], dtype=torch.int32, device="cuda")
    kv = torch.tensor([9], dtype=torch.int32, device="cuda")
    ops.argmax(x, ids, ws, hist=hist, step=step, pos=pos, kv_len=kv)
    want = torch.argmax(x.cpu(), -1)
    assert ids.cpu().tolist() == want.tolist() and ids[1].item() == 77
    assert hist[2].cpu().tolist() == want.tolist()
    assert step.item() == 3 and kv.item() == 10 and pos.cpu().tolist() == [6, 7, 8]
    # a step past the history's rows is not recorded (the state still advances)
    guard = torch.full((6, 3), -7, dtype=torch.int64, device="cuda")
    step.fill_(4)
    ops.argmax(x, ids, ws, hist=guard[:4], step=step, pos=pos, kv_len=kv)
    assert (guard[4:] == -7).all() and step.item() == 5 and ids.cpu().tolist() == want.tolist()
    # more rows than the final pass has waves (16): rows strided over the waves, ties across chunk edges
    B = 20
    x = torch.randn(B, V).cuda()
    x[:, 4019] = 40.0
    x[:, 4020] = 40.0
    x[7, 257215] = 60.0
    ids = torch.empty(B, dtype=torch.int64, device="cuda")
    ws = torch.empty(B * 64 * 2, device="cuda")
    hist = torch.zeros(3, B, dtype=torch.int64, device="cuda")
    step = torch.tensor([1], dtype=torch.int32, device="cuda")
    pos = torch.arange(B, dtype=torch.int32, device="cuda")
    kv.fill_(3)
    ops.argmax(x, ids, ws, hist=hist, step=step, pos=pos, kv_len=kv)
    want = torch.argmax(x.cpu(), -1)
    assert ids.cpu().tolist() == want.tolist() and ids[7].item() == 257215 and ids[0].item() == 4019
    assert hist[1].cpu().tolist() == want.tolist() and (hist[0] == 0).all() and (hist[2] == 0).all()
    assert step.item() == 2 and kv.item() == 4 and pos.cpu().tolist() == list(range(1, B + 1))


@pytest.mark.parametrize("B", [1, 5, 20])
def test_argmax_embed_equals_argmax_then_embed_merge(B):
    """pg_argmax_embed == pg_argmax followed by pg_embed_merge(rank=None) of the winners, bit-exact: ids,
    history, state advance and the next step's rows, including pad-token and image-token winners (the image
    rank counts earlier rows with the image token; ranks past n_feat give zero rows)."""
    from pghip import ops
    V, Ve, H, n_feat = 257216, 257216, 2048, 2
    image_id, pad_id = 257152, 0
    gen = torch.Generator().manual_seed(B)
    x = torch.randn(B, V, generator=gen).cuda()
    forced = {0: image_id, 1: pad_id, 2: image_id, 3: image_id, 4: 257215}
    for b, t in forced.items():
        if b < B:
            x[b, t] = 99.0
    embed = (torch.randn(Ve, H, generator=gen) * 0.05).to(torch.bfloat16).cuda()
    feat = torch.randn(n_feat, H, generator=gen).cuda()
    kw = dict(image_id=image_id, pad_id=pad_id, img_scale=2048 ** -0.5, normalizer=2048 ** 0.5)
    outs = []
    for fused in (True, False):
        ids = torch.empty(B, dtype=torch.int64, device="cuda")
        ws = torch.empty(B * 64 * 2, device="cuda")
        hist = torch.zeros(3, B, dtype=torch.int64, device="cuda")
        step = torch.tensor([1], dtype=torch.int32, device="cuda")
        pos = torch.arange(B, dtype=torch.int32, device="cuda")
        kv = torch.tensor([9], dtype=torch.int32, device="cuda")
        res = torch.full((B, H), float("nan"), device="cuda")
        st = dict(hist=hist, step=step, pos=pos, kv_len=kv)
        if fused:
            ops.argmax_embed(x, ids, ws, embed, feat, n_feat, res, **kw, **st)
        else:
            ops.argmax(x, ids, ws, **st)
            ops.embed_merge(ids, None, embed, feat, n_feat, res, **kw)
        outs.append([t.cpu() for t in (ids, hist, step, pos, kv, res)])
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    ids, res = outs[0][0], outs[0][5]
    assert ids.tolist()[: min(B, 5)] == [forced[b] for b in range(min(B, 5))]
    if B >= 4:                                       # third image winner: rank 2 >= n_feat -> zeros
        assert (res[3] == 0).all() and (res[1] == 0).all() and (res[0] != 0).any() and (res[2] != 0).any()


def test_topp_matches_reference_filter(golden):
    from oracle import paligemma_oracle as O
    from pghip import ops
    g = golden("topp")
    for ci in range(4):
        logits = torch.from_numpy(g[f"c{ci}_logits"]).cuda()
        T, P = float(g[f"c{ci}_T"]), float(g[f"c{ci}_p"])
        V = logits.shape[1]
        u = torch.tensor([[0.0], [0.37], [0.999]], dtype=torch.float32).cuda()
        probs = torch.empty(1, V, device="cuda")
        ids = torch.empty(1, dtype=torch.int64, device="cuda")
        step = torch.zeros(1, dtype=torch.int32, device="cuda")
        for k in range(3):
            ops.topp_sample(logits, ids, u, temperature=T, top_p=P, step=step, probs_out=probs)
            want = O.sample_top_p(logits.cpu().numpy(), T, P, u[k].cpu().numpy())[0, 0]
            got = ids.item()
            pr = probs.cpu().numpy()[0]
            kept = set(np.nonzero(pr)[0].tolist())
            ref_ids = g[f"c{ci}_kept_ids"]
            ref_kept = set(ref_ids.tolist())
            if kept != ref_kept:
                # only a token whose mass ranked before it lands on top_p within fp32 summation-order rounding may
                # differ (the reference's torch.cumsum vs the kernel's radix select)
                p64 = np.exp((g[f"c{ci}_logits"][0].astype(np.float64) / T) - (g[f"c{ci}_logits"][0].max() / T))
                p64 /= p64.sum()
                order = np.argsort(-p64, kind="stable")
                before = dict(zip(order.tolist(), (np.cumsum(p64[order]) - p64[order]).tolist()))
                diff = kept ^ ref_kept
                assert len(diff) == 1 and abs(before[next(iter(diff))] - P) < 1e-5, (ci, len(kept), len(ref_kept))
            assert got in kept
            if kept == ref_kept:
                assert got == want, (ci, k, got, want)
            # the renormalised distribution: probs_out against the reference's probs_sort (c*_kept_probs, the
            # tensor it hands to torch.multinomial, inference.py:104), over the common kept set
            common = np.array(sorted(kept & ref_kept))
            ref_p = dict(zip(ref_ids.tolist(), g[f"c{ci}_kept_probs"].tolist()))
            a = pr[common] / pr[common].sum()
            b = np.array([ref_p[i] for i in common.tolist()])
            b = b / b.sum()
            assert np.abs(a - b).max() <= 1e-4 * b.max() + 1e-7, (ci, float(np.abs(a - b).max()))


@pytest.mark.parametrize("M", [1, 5, 16])
def test_gemm_fused_rmsnorm_prologue(M):
    """x = RMSNorm(resid + sum partials)*(1+w) built in-kernel; resid_out written once."""
    from pghip import ops
    K, N, S = 2048, 512, 4
    resid = torch.randn(M, K).cuda()
    part = torch.randn(S, M, K).cuda() * 0.5
    w = torch.randn(K).cuda() * 0.1
    W = rnd(N, K, scale=1 / 45, seed=20)
    out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    rout = torch.zeros(M, K).cuda()
    fa = ops.fused_args(pro_mode=ops.PRO_RMSNORM, resid_in=resid, resid_out=rout, partials=part, nsplit=S,
                        norm_w=w, eps=1e-6)
    ops.gemm_fused(None, W, out, fa, epi=ops.EPI_BF16, M=M)
    x = resid + part.sum(0)
    xn = (x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + 1e-6) * (1 + w)).to(torch.bfloat16).float()
    assert err(rout, x) < 1e-6
    assert err(out, xn @ W.float().t()) < 1e-2


@pytest.mark.parametrize("B", [1, 3])
def test_gemm_fused_attention_merge_prologue(B):
    """o_proj GEMV whose prologue merges split-KV attention partials == attention+combine+GEMV."""
    from pghip import ops
    nh, nkv, hd, L, Smax = 8, 1, 256, 200, 256
    kvd = nkv * hd
    q = rnd(B, nh * hd, seed=21)
    kc, vtc = rnd(B, Smax, kvd, seed=22), rnd(B, kvd, Smax, seed=23)
    lkv = torch.tensor([L], dtype=torch.int32, device="cuda")
    SK, nsplit, dt = 32, 8, 256
    po = torch.empty(B * nkv * nsplit * 16 * dt, device="cuda")
    pml = torch.empty(B * nkv * nsplit * 16 * 2, device="cuda")
    ops.attention(q, nh * hd, None, nh * hd, kc, Smax * kvd, hd, kvd, vtc, kvd * Smax, hd * Smax, Smax,
                  B=B, Lq=1, Lkv=0, lkv_dev=lkv, Hq=nh, Hkv=nkv, D=hd, scale=hd ** -0.5, split_keys=SK,
                  nsplit=nsplit, part_o=po, part_ml=pml)
    ref_o = torch.empty(B, nh * hd, dtype=torch.bfloat16, device="cuda")
    ops.attn_combine(po, pml, ref_o, nh * hd, B=B, Hq=nh, Hkv=nkv, D=hd, nsplit=nsplit)
    Wo = rnd(2048, nh * hd, scale=1 / 45, seed=24)
    for z in (1, 2):
        part = torch.empty(z, B, 2048, device="cuda")
        fa = ops.fused_args(pro_mode=ops.PRO_ATTN_COMBINE, part_o=po, part_ml=pml, asplit=nsplit, head_dim=hd,
                            dtw=dt, q_per_kv=nh // nkv, kv_heads=nkv)
        ops.gemm_fused(None, Wo, part, fa, epi=ops.EPI_F32, M=B, ksplit=z)
        assert err(part.sum(0), ref_o.float() @ Wo.float().t()) < 1e-2
    # and the attention itself against a float reference
    kf = kc[:, :L].float()
    vf = vtc[:, :, :L].float().transpose(1, 2)
    s = torch.einsum("bhd,bkd->bhk", q.view(B, nh, hd).float(), kf) * hd ** -0.5
    ref = torch.einsum("bhk,bkd->bhd", torch.softmax(s, -1), vf).reshape(B, -1)
    assert err(ref_o, ref) < 2e-2


@pytest.mark.parametrize("M,z,frag", [(1, 1, True), (1, 8, True), (2, 2, True), (5, 4, False), (16, 3, True)])
def test_gemm_f32_add_epilogue_residual_accumulates(M, z, frag):
    """PG_EPI_F32_ADD: the GEMV adds its split-K partials (+ bias, once) into the residual with float atomics:
    resid += x . W^T, equal to the fp32 reference up to the fp32 order of the split sums; rows past M untouched;
    with the attention-merge prologue (o_proj) as well."""
    from pghip import ops
    from pghip.weights import frag_pack
    K, N = 2048, 1024
    x = rnd(M, K, seed=31)
    W = rnd(N, K, scale=1 / 45, seed=32)
    bias = torch.randn(N).cuda() * 0.1
    resid = torch.randn(M + 1, N).cuda()
    r0 = resid.clone()
    Wk = frag_pack(W) if frag else W
    ops.gemm_fused(x, Wk, resid, ops.fused_args(), epi=ops.EPI_F32_ADD | (ops.W_FRAG if frag else 0), M=M, ksplit=z,
                   bias=bias)
    ref = r0[:M] + x.float() @ W.float().t() + bias
    assert err(resid[:M], ref) < 1e-5
    assert torch.equal(resid[M:], r0[M:])


@pytest.mark.parametrize("M,L,H", [(1, 1, 512), (3, 1, 512), (40, 20, 512), (264, 264, 512), (264, 264, 2048)])
def test_gemm_fused_qkv_rope_epilogue(M, L, H):
    """q|k|v GEMM with RoPE + KV append in the epilogue == plain GEMM + pg_rope_kv_write (H = 2048 at M = 264:
    split K + pg_gemm_finalize)."""
    from pghip import engine, ops
    from pghip.weights import rope_row_perm
    nh, nkv, hd, Smax = 8, 1, 256, 320
    nblk = nh + 2 * nkv
    W = rnd(nblk * hd, H, scale=1 / 22, seed=25)
    Wp = W.view(nblk, hd, H)[:, rope_row_perm(hd).cuda(), :].reshape(nblk * hd, H).contiguous()
    x = rnd(M, H, seed=26)
    B = M // L
    pos = (torch.arange(M) % L + 7).to(torch.int32).cuda()
    cos_t, sin_t = engine.rope_tables(hd, 1024, 10000.0, "cuda")
    slot = torch.tensor([5], dtype=torch.int32, device="cuda")
    # reference path
    qkv = torch.empty(M, nblk * hd, dtype=torch.bfloat16, device="cuda")
    ops.gemm(x, W, qkv)
    kc_r = torch.zeros(B, Smax, nkv * hd, dtype=torch.bfloat16, device="cuda")
    vt_r = torch.zeros(B, nkv * hd, Smax, dtype=torch.bfloat16, device="cuda")
    ops.rope_kv_write(qkv, pos, cos_t, sin_t, kc_r, vt_r, T=M, L=L, Hq=nh, Hkv=nkv, D=hd, Smax=Smax, slot_base=3,
                      slot_dev=slot)
    # fused
    q = torch.empty(M, nh * hd, dtype=torch.bfloat16, device="cuda")
    kc = torch.zeros_like(kc_r)
    vt = torch.zeros_like(vt_r)
    kd = torch.zeros(B * Smax * nkv * hd, dtype=torch.bfloat16, device="cuda")
    vd = torch.zeros_like(kd)
    fa = ops.fused_args(head_dim=hd, cos_t=cos_t, sin_t=sin_t, pos=pos, rows_per_batch=L, slot_dev=slot, slot_base=3,
                        kc=kc, vtc=vt, smax=Smax, q_heads=nh, kv_heads=nkv, kd=kd, vd=vd)
    ops.gemm_fused(x, Wp, q, fa, epi=ops.EPI_QKV_ROPE, M=M)
    assert err(q, qkv[:, :nh * hd]) < 1e-2
    assert err(kc, kc_r) < 1e-2
    assert err(vt, vt_r) < 1e-2
    # the decode-order copies (ABI 6) hold exactly the canonical cache's bytes, permuted (csrc dec_koff / dec_voff)
    kd_r, vd_r = ops.decode_cache_pack(kc, vt, nkv)
    assert torch.equal(kd.view_as(kd_r), kd_r) and torch.equal(vd.view_as(vd_r), vd_r)


@pytest.mark.parametrize("H,W,S", [(480, 640, 224), (37, 51, 224), (224, 500, 224), (1000, 224, 448),
                                   (224, 224, 224), (300, 448, 448)])
def test_image_preprocess_bit_exact_with_reference_host_path(H, W, S):
    """pg_image_preprocess == the reference's process_images (PIL BICUBIC + rescale + normalise + CHW)."""
    from PIL import Image
    from processing_paligemma import process_images
    from pghip import image
    img = Image.fromarray(np.random.default_rng(H + W).integers(0, 256, (H, W, 3), dtype=np.uint8))
    ref = process_images([img], S, scale_factor=1 / 255.0, resampling=Image.Resampling.BICUBIC)[0]
    out = image.preprocess([img], S)
    assert out.shape == (1, 3, S, S) and out.dtype == torch.float32
    assert np.array_equal(out[0].cpu().numpy(), ref)


@pytest.mark.parametrize("M,N,K", [(4200, 4096, 640), (16384, 1152, 1152), (2100, 8192, 256), (4113, 4096, 192)])
def test_gemm256_large_m(M, N, K):
    """The 256x256 large-M GEMM (chosen when its grid fills every CU), ragged M/N edges, odd K-tile counts,
    row-major and fragment-packed W, against a torch fp32 matmul of the same bf16 operands."""
    from pghip import ops
    from pghip.weights import frag_pack
    A, W = rnd(M, K, seed=31), rnd(N, K, scale=1 / math.sqrt(K), seed=32)
    bias = torch.randn(N).cuda()
    ref = A.float() @ W.float().t() + bias
    out = torch.empty(M, N, dtype=torch.float32, device="cuda")
    ops.gemm(A, W, out, epi=ops.EPI_F32, bias=bias)
    assert err(out, ref) < 1e-5
    for ks in (2, 3):   # split-K fp32 slabs (bias on slab 0), ragged last slice
        part = torch.empty(ks, M, N, dtype=torch.float32, device="cuda")
        ops.gemm(A, W, part, epi=ops.EPI_F32, bias=bias, ksplit=ks)
        assert err(part.sum(0), ref) < 1e-5, ks
    outb = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    if N % 16 == 0 and K % 64 == 0:
        ops.gemm(A, frag_pack(W), outb, epi=ops.EPI_BF16 | ops.W_FRAG, bias=bias)
    else:
        ops.gemm(A, W, outb, bias=bias)
    assert err(outb, ref) < 1e-2
    if N % 32 == 0:
        h = torch.empty(M, N // 2, dtype=torch.bfloat16, device="cuda")
        ops.gemm(A, W, h, epi=ops.EPI_BF16_GELU_MUL)
        g = (A.float() @ W.float().t()).view(M, N // 32, 2, 16)
        want = (torch.nn.functional.gelu(g[:, :, 0], approximate="tanh") * g[:, :, 1]).reshape(M, N // 2)
        assert err(h, want) < 1e-2


@pytest.mark.parametrize("M,N,K", [(264, 2560, 2048), (256, 1536, 1152), (256, 640, 1152)])
def test_split_k_finalize_epilogues(M, N, K):
    """Small-M bf16-epilogue GEMMs split K into fp32 slabs + pg_gemm_finalize: same outputs as the one-launch
    fused epilogue (bf16, gelu, gelu*up, V^T side output), up to fp32 summation order."""
    from pghip import ops
    assert ops.finalize_split(M, N, K) > 1
    A, W = rnd(M, K, seed=41), rnd(N, K, scale=1 / math.sqrt(K), seed=42)
    bias = torch.randn(N).cuda() * 0.1
    cases = [(ops.EPI_BF16, bias), (ops.EPI_BF16_GELU, bias), (ops.EPI_BF16_GELU_MUL, None)]
    if N % 12 == 0:                                   # q | k | v with a V^T side output (SigLIP layout)
        cases.append((ops.EPI_BF16_VT, bias))
    for epi, bb in cases:
        outs = []
        for split in (True, False):
            ops.FINALIZE_SPLIT = split
            try:
                n_out = N // 2 if epi == ops.EPI_BF16_GELU_MUL else N
                o = torch.zeros(M, n_out, dtype=torch.bfloat16, device="cuda")
                vt = torch.zeros(N // 3, M, dtype=torch.bfloat16, device="cuda")
                kw = dict(aux_out=vt, aux_ld=M, aux_n=N - N // 3) if epi == ops.EPI_BF16_VT else {}
                ops.gemm(A, W, o, epi=epi, bias=bb, **kw)
                outs.append((o, vt))
            finally:
                ops.FINALIZE_SPLIT = True
        assert err(outs[0][0], outs[1][0]) < 1e-2, epi
        assert err(outs[0][1].float(), outs[1][1].float()) < 1e-2 or epi != ops.EPI_BF16_VT, epi


# ---------------------------------------------------------------- fp8 e4m3 path (BASELINE configs[4])
def _deq(q, s):
    return q.view(torch.float8_e4m3fn).float() * s[:, None]


@pytest.mark.parametrize("M,K", [(1, 8), (7, 2048), (300, 16384), (64, 1152), (32, 16384), (3, 24576), (2, 40960),
                                 (4103, 2048), (1030, 1152), (2049, 4096), (1024, 24)])   # the wave-per-row form
def test_quant_fp8_rows_bit_identical_to_host_rule(M, K):
    """pg_quant_fp8 (row absmax / 448 scale, RNE e4m3) gives the same bytes and scales as the host rule the
    weights use (weights.quant_rows_fp8), including an all-zero row (scale 1); from 1024 rows (K <= 4096) the
    one-wave-per-row kernel, a ragged last workgroup included."""
    from pghip import ops
    from pghip.weights import quant_rows_fp8
    x = rnd(M, K, scale=3.0, seed=51)
    x[0] = 0
    if M > 2:
        x[1, :] *= 1e-3
    q, s = ops.quant_fp8(x)
    q_ref, s_ref = quant_rows_fp8(x)
    assert torch.equal(s, s_ref)
    assert torch.equal(q, q_ref)
    assert err(_deq(q, s), x.float()) < 0.07          # e4m3: 3 mantissa bits


@pytest.mark.parametrize("M,N,K", [(300, 384, 512), (4200, 4096, 640), (33, 1152, 1152)])
def test_gemm_f32_res_adds_into_the_residual_bit_exactly(M, N, K):
    """PG_EPI_F32_RES (ABI 13): the producing tile GEMM adds acc + bias into the fp32 residual in its epilogue; equal
    bit for bit to the PG_EPI_F32 slab plus the one fp32 add the norm kernel makes (resid + slab), on the bf16 tile
    and 256 x 256 kernels (row-major and fragment-packed W), the fp8 kernels (row scales) and the fp8 MX-rows-in
    tile; the columns past N and the rows of another GEMM untouched."""
    from pghip import ops
    from pghip.weights import frag_pack, quant_rows_fp8
    A, W = rnd(M, K, seed=61), rnd(N, K, scale=1 / math.sqrt(K), seed=62)
    bias = torch.randn(N).cuda()
    resid0 = torch.randn(M, N + 8, device="cuda")                 # ldc > N: the pad columns must stay
    cases = [("bf16", lambda out, e: ops.gemm(A, W, out, epi=e, bias=bias))]
    if K % 64 == 0 and N % 16 == 0:
        Wf = frag_pack(W)
        cases.append(("bf16 frag", lambda out, e: ops.gemm(A, Wf, out, epi=e | ops.W_FRAG, bias=bias)))
    if K % 128 == 0 and M > 16:
        a8, sa = ops.quant_fp8(A)
        w8, sw = quant_rows_fp8(W)
        cases.append(("fp8", lambda out, e: ops.gemm8(a8, sa, w8, sw, out, epi=e, bias=bias)))
    for name, run in cases:
        slab = torch.empty(M, N + 8, device="cuda")
        run(slab, ops.EPI_F32)
        out = resid0.clone()
        run(out, ops.EPI_F32_RES)
        assert torch.equal(out[:, :N], resid0[:, :N] + slab[:, :N]), name
        assert torch.equal(out[:, N:], resid0[:, N:]), name
    if M > 32 and K % 128 == 0:                                  # MX rows in (the prefill down projection's form)
        q = torch.randint(0, 126, (M, K), dtype=torch.uint8, device="cuda")     # finite e4m3 bytes
        sc = torch.randint(120, 134, (M, K // 32), dtype=torch.uint8, device="cuda")
        w8, sw = quant_rows_fp8(W)
        slab = torch.empty(M, N + 8, device="cuda")
        ops.gemm8(q, None, w8, sw, slab, epi=ops.EPI_F32, mx_in=sc)
        out = resid0.clone()
        ops.gemm8(q, None, w8, sw, out, epi=ops.EPI_F32_RES, mx_in=sc)
        assert torch.equal(out[:, :N], resid0[:, :N] + slab[:, :N])
    with pytest.raises(ValueError):                                # one split only
        ops.gemm(A, W, resid0.clone(), epi=ops.EPI_F32_RES, ksplit=2)


@pytest.mark.parametrize("M,N,K", [(300, 384, 512), (1024, 2048, 2048), (4096, 4096, 256), (4200, 4096, 640)])
def test_gemm_fp8_matches_fp32_matmul_of_dequantised_operands(M, N, K):
    """PG_FP8 GEMM (16x16x128 block-scaled MFMA, unit block scales, row scales in the epilogue) on the tile
    and the 256x256 kernels: equal to a torch fp32 matmul of the dequantised e4m3 operands up to fp32
    summation order; split-K slabs, bf16 and gelu*up epilogues."""
    from pghip import ops
    from pghip.weights import quant_rows_fp8
    A, W = rnd(M, K, seed=52), rnd(N, K, scale=1 / math.sqrt(K), seed=53)
    bias = torch.randn(N).cuda()
    a8, sa = ops.quant_fp8(A)
    w8, sw = quant_rows_fp8(W)
    ref = _deq(a8, sa) @ _deq(w8, sw).t()
    out = torch.empty(M, N, dtype=torch.float32, device="cuda")
    ops.gemm8(a8, sa, w8, sw, out, epi=ops.EPI_F32, bias=bias)
    # (the reference rounds every dequantised operand to fp32; the kernel scales the exact e4m3 products once)
    assert err(out, ref + bias) < 5e-5
    part = torch.empty(3, M, N, dtype=torch.float32, device="cuda")
    ops.gemm8(a8, sa, w8, sw, part, epi=ops.EPI_F32, bias=bias, ksplit=3)
    assert err(part.sum(0), ref + bias) < 5e-5
    outb = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    ops.gemm8(a8, sa, w8, sw, outb, epi=ops.EPI_BF16, bias=bias)
    assert err(outb, ref + bias) < 1e-2
    h = torch.empty(M, N // 2, dtype=torch.bfloat16, device="cuda")
    ops.gemm8(a8, sa, w8, sw, h, epi=ops.EPI_BF16_GELU_MUL)
    g = ref.view(M, N // 32, 2, 16)
    want = (torch.nn.functional.gelu(g[:, :, 0], approximate="tanh") * g[:, :, 1]).reshape(M, N // 2)
    assert err(h, want) < 1e-2
    # and the quantisation error against the bf16 product stays at the e4m3 level
    assert err(out - bias, A.float() @ W.float().t()) < 0.1


@pytest.mark.parametrize("M,H,nsplit", [(5, 2048, 0), (300, 2048, 3), (17, 1152, 1)])
def test_norm_residual_fp8_equals_quantised_bf16_output(M, H, nsplit):
    """pg_norm_residual_fp8 == pg_quant_fp8(pg_norm_residual bf16 output), bytes and scales; the residual
    update is the same."""
    from pghip import ops
    g = torch.Generator().manual_seed(61)
    resid = torch.randn(M, H, generator=g).cuda()
    part = torch.randn(max(nsplit, 1), M, H, generator=g).cuda() * 0.1
    w = torch.randn(H, generator=g).cuda() * 0.1
    r1, r2 = resid.clone(), resid.clone()
    xn = torch.empty(M, H, dtype=torch.bfloat16, device="cuda")
    ops.norm_residual(r1, w, mode=ops.NORM_RMS, partials=part, nsplit=nsplit, out=xn)
    q_ref, s_ref = ops.quant_fp8(xn)
    q = torch.empty(M, H, dtype=torch.uint8, device="cuda")
    s = torch.empty(M, dtype=torch.float32, device="cuda")
    ops.norm_residual_fp8(r2, w, q, s, mode=ops.NORM_RMS, partials=part, nsplit=nsplit)
    assert torch.equal(r1, r2)
    assert torch.equal(s, s_ref)
    assert torch.equal(q, q_ref)


@pytest.mark.parametrize("M,N,K,ks", [(32, 2560, 2048, 1), (17, 2048, 16384, 8), (24, 4096, 2048, 2),
                                      (9, 512, 256, 1), (32, 32160, 2048, 1), (32, 16384, 2048, 1),
                                      # ragged K splits (the runtime-trip-count forms, CPW = 0): K-split and wide
                                      # kernels; and more splits than 128-k chunks (the last splits own none)
                                      (20, 1024, 1152, 2), (32, 4096, 2048, 3), (20, 16384, 1152, 2),
                                      (24, 512, 256, 4), (24, 16384, 256, 4),
                                      # an lm_head-sized grid (8192 tiles)
                                      (20, 131072, 1024, 1)])
def test_gemv8_fragment_packed_matches_the_fp8_tile_gemm(M, N, K, ks):
    """The fp8 weight-streaming GEMV (fragment-packed e4m3 weights, weights.frag_pack8; 17..32-row batched decode and
    the fp8 lm_head): equal to a torch fp32 matmul of the dequantised operands up to fp32 summation order, for the
    fp32 slab (split-K), bf16 and gelu*up epilogues; the pack / unpack pair is a bijection.  Splits past the last
    128-k chunk write zero slabs."""
    from pghip import ops
    from pghip.weights import frag_pack8, frag_unpack8, quant_rows_fp8
    A, W = rnd(M, K, seed=71), rnd(N, K, scale=1 / math.sqrt(K), seed=72)
    bias = torch.randn(N).cuda()
    a8, sa = ops.quant_fp8(A)
    w8, sw = quant_rows_fp8(W)
    w8f = frag_pack8(w8)
    assert torch.equal(frag_unpack8(w8f), w8)
    ref = _deq(a8, sa) @ _deq(w8, sw).t()
    part = torch.empty(ks, M, N, dtype=torch.float32, device="cuda")
    ops.gemm8(a8, sa, w8f, sw, part, epi=ops.EPI_F32, bias=bias, ksplit=ks, frag=True)
    assert err(part.sum(0), ref + bias) < 5e-5
    resid = torch.randn(M, N).cuda()                  # the float-atomic residual add (batched fp8 decode)
    r0 = resid.clone()
    ops.gemm8(a8, sa, w8f, sw, resid, epi=ops.EPI_F32_ADD, bias=bias, ksplit=ks, frag=True)
    assert err(resid - r0, ref + bias) < 5e-5
    if ks == 1:
        outb = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        ops.gemm8(a8, sa, w8f, sw, outb, epi=ops.EPI_BF16, bias=bias, frag=True)
        assert err(outb, ref + bias) < 1e-2
        h = torch.empty(M, N // 2, dtype=torch.bfloat16, device="cuda")
        ops.gemm8(a8, sa, w8f, sw, h, epi=ops.EPI_BF16_GELU_MUL, frag=True)
        g = ref.view(M, N // 32, 2, 16)
        want = (torch.nn.functional.gelu(g[:, :, 0], approximate="tanh") * g[:, :, 1]).reshape(M, N // 2)
        assert err(h, want) < 1e-2


@pytest.mark.parametrize("M,I,H,ks", [(32, 16384, 2048, 8), (17, 4096, 1024, 2), (24, 2048, 512, 1), (9, 4096, 512, 2)])
def test_gemm8_hx_equals_the_quantiser_route(M, I, H, ks):
    """The batched fp8 decode MLP without pg_quant_fp8 (ABI 9): the gate/up GEMV max-es each row's |h| into
    amax_out, the down GEMV (pro_mode 5, ops.gemm8_hx) quantises bf16 h while staging it.  h, the row maxima
    (448 x quant_fp8's scales) and the down slabs are bit-identical to gate/up -> quant_fp8 -> gemm8; another fp8
    GEMV launch's amax_zero clears stale maxima first (the engine's QKV GEMV)."""
    from pghip import ops
    from pghip.weights import frag_pack8, quant_rows_fp8
    x = rnd(M, H, seed=81)
    Wgu, Wd = rnd(2 * I, H, scale=1 / math.sqrt(H), seed=82), rnd(H, I, scale=1 / math.sqrt(I), seed=83)
    x8, xs = ops.quant_fp8(x)
    gu8, gus = quant_rows_fp8(Wgu)
    d8, ds = quant_rows_fp8(Wd)
    gu8f, d8f = frag_pack8(gu8), frag_pack8(d8)
    ld = 32
    amax = torch.full((M * ld,), 0x7F000000, dtype=torch.int32, device="cuda")     # stale maxima
    w0, s0 = quant_rows_fp8(rnd(16, H, seed=84))
    tmp = torch.empty(M, 16, dtype=torch.bfloat16, device="cuda")
    ops.gemm8(x8, xs, frag_pack8(w0), s0, tmp, epi=ops.EPI_BF16, frag=True,
              fa=ops.fused_args(amax_zero=amax, amax_zero_n=M * ld))
    torch.cuda.synchronize()
    assert int(amax.abs().sum()) == 0
    h1 = torch.empty(M, I, dtype=torch.bfloat16, device="cuda")
    ops.gemm8(x8, xs, gu8f, gus, h1, epi=ops.EPI_BF16_GELU_MUL, frag=True,
              fa=ops.fused_args(amax_out=amax, amax_ld=ld))
    h0 = torch.empty_like(h1)
    ops.gemm8(x8, xs, gu8f, gus, h0, epi=ops.EPI_BF16_GELU_MUL, frag=True)
    assert torch.equal(h0, h1)
    h8, hs = ops.quant_fp8(h0)
    got = amax.view(M, ld)[:, 0].view(torch.float32)
    assert torch.equal(got, h0.float().abs().amax(1))   # (the scale amax / 448 is divided in-kernel: torch's
    assert torch.allclose(got / 448, hs, rtol=1e-6, atol=0)  # tensor / scalar multiplies by the reciprocal)
    p0 = torch.empty(ks, M, H, dtype=torch.float32, device="cuda")
    p1 = torch.empty_like(p0)
    ops.gemm8(h8, hs, d8f, ds, p0, epi=ops.EPI_F32, ksplit=ks, frag=True)
    ops.gemm8_hx(h0, amax, ld, d8f, ds, p1, M=M, ksplit=ks)
    torch.cuda.synchronize()
    if (H // 16 + 3) // 4 * ks >= 256:       # the quantiser route also ran the wide form: the same sums
        assert torch.equal(p0, p1)
    else:                                    # it ran the K-split form: fp32 summation order differs
        assert torch.allclose(p0, p1, rtol=1e-5, atol=1e-5)


def _mx_quant(h):
    """Torch restatement of the MX rule (PgFusedArgs.mx_out, csrc/common.h mx_exp): per 32 columns e = the smallest
    exponent with max |h| <= 448 * 2^e, bytes e4m3(h / 2^e), scales e + 127 stored [M][4][K/128] (block 4c + g at
    [m][g][c])."""
    M, K = h.shape
    b = h.view(M, K // 32, 32)
    amax = b.abs().amax(2)
    f, k = torch.frexp(amax)
    ex = (k - 9 + (f * 512 > 448).int()).clamp(-127, 127)
    ex = torch.where(amax > 0, ex, torch.zeros_like(ex))
    q = (b / torch.exp2(ex.float())[..., None]).to(torch.float8_e4m3fn).view(torch.uint8).reshape(M, K)
    sc = (ex + 127).to(torch.uint8).view(M, K // 128, 4).permute(0, 2, 1).contiguous()
    return q, sc.view(-1)


def _mx_deq(q8, sc, M, K):
    s = sc.view(M, 4, K // 128).permute(0, 2, 1).reshape(M, K // 32).float()
    return (q8.view(torch.float8_e4m3fn).float().view(M, K // 32, 32) * torch.exp2(s - 127)[..., None]).view(M, K)


@pytest.mark.parametrize("M,I,H,ks", [(32, 16384, 2048, 8), (32, 2048, 2048, 1), (17, 4096, 1024, 2),
                                      (24, 2048, 512, 1), (9, 256, 512, 1), (32, 16384, 2048, 16)])
def test_mx_h_gate_up_and_down(M, I, H, ks):
    """The batched fp8 decode MLP on MX rows (ABI 11, engine.MX_H): the gate/up GEMV writes h as e4m3 bytes with one
    E8M0 scale per 32 columns (mx_out) -- bit-identical to the torch MX rule applied to the bf16 gelu*up launch's h --
    and the down GEMV reading those block scales into its MFMAs (mx_in; the wide and the K-split forms) equals a torch
    fp32 matmul of the dequantised operands up to summation order; also on scales spread over 2^-10 .. 2^10."""
    from pghip import ops
    from pghip.weights import frag_pack8, quant_rows_fp8
    x = rnd(M, H, seed=85)
    Wgu, Wd = rnd(2 * I, H, scale=1 / math.sqrt(H), seed=86), rnd(H, I, scale=1 / math.sqrt(I), seed=87)
    x8, xs = ops.quant_fp8(x)
    gu8, gus = quant_rows_fp8(Wgu)
    d8, ds = quant_rows_fp8(Wd)
    gu8f, d8f = frag_pack8(gu8), frag_pack8(d8)
    h0 = torch.empty(M, I, dtype=torch.bfloat16, device="cuda")
    ops.gemm8(x8, xs, gu8f, gus, h0, epi=ops.EPI_BF16_GELU_MUL, frag=True)
    h8 = torch.full((M, I), 0x55, dtype=torch.uint8, device="cuda")
    hs = torch.full((M * I // 32,), 0x55, dtype=torch.uint8, device="cuda")
    ops.gemm8(x8, xs, gu8f, gus, h8, epi=ops.EPI_BF16_GELU_MUL, frag=True, mx_out=hs)
    q_ref, s_ref = _mx_quant(h0.float())
    assert torch.equal(hs, s_ref)
    assert torch.equal(h8, q_ref)
    assert err(_mx_deq(h8, hs, M, I), h0.float()) < 0.07          # e4m3: 3 mantissa bits per block
    # float64 reference: the MX rows' block magnitudes spread (gelu*up h, and random scales over 2^20) makes the fp32
    # summation order show at ~6e-5 of the row max at K = 2048 for the K-split form
    for scales, tol in ((hs, 1e-4), (torch.randint(117, 138, (M * I // 32,), dtype=torch.uint8, device="cuda"), 3e-4)):
        ref = (_mx_deq(h8, scales, M, I).double() @ _deq(d8, ds).double().t()).float()
        part = torch.empty(ks, M, H, dtype=torch.float32, device="cuda")
        ops.gemm8(h8, None, d8f, ds, part, epi=ops.EPI_F32, ksplit=ks, frag=True, mx_in=scales)
        assert err(part.sum(0), ref) < tol, (float(err(part.sum(0), ref)), tol)


@pytest.mark.parametrize("M,I,H,ks", [(300, 1024, 512, 1), (33, 2048, 2048, 2), (1100, 16384, 2048, 3),
                                      (4200, 4096, 1024, 1)])
def test_mx_h_prefill_tiles(M, I, H, ks):
    """The fp8 prefill MLP on MX rows (ABI 12, engine.MX_PREFILL): the 128 x 128 fp8 gate/up tile writes h as e4m3
    with one E8M0 scale per 32 columns, natural layout [M][I/32] -- bit-identical to the torch MX rule on the bf16
    gelu*up tile's h (one e4m3 step allowed where the two launches' bf16 h differ by an ulp) -- and the 256 x 256 fp8
    fp32-slab GEMM reading those block scales beside the rows (mx_in) equals a float64 matmul of the dequantised
    operands up to fp32 summation order; also on scales spread over 2^-10 .. 2^10 and with split-K slabs."""
    from pghip import ops
    from pghip.weights import quant_rows_fp8
    x = rnd(M, H, seed=91)
    Wgu, Wd = rnd(2 * I, H, scale=1 / math.sqrt(H), seed=92), rnd(H, I, scale=1 / math.sqrt(I), seed=93)
    x8, xs = ops.quant_fp8(x)
    gu8, gus = quant_rows_fp8(Wgu)
    d8, ds = quant_rows_fp8(Wd)
    h0 = torch.empty(M, I, dtype=torch.bfloat16, device="cuda")
    ops.gemm8(x8, xs, gu8, gus, h0, epi=ops.EPI_BF16_GELU_MUL)
    h8 = torch.full((M, I), 0x55, dtype=torch.uint8, device="cuda")
    hs = torch.full((M, I // 32), 0x55, dtype=torch.uint8, device="cuda")
    ops.gemm8(x8, xs, gu8, gus, h8, epi=ops.EPI_BF16_GELU_MUL, mx_out=hs)
    q_ref, s_ref = _mx_quant(h0.float())
    s_ref = s_ref.view(M, 4, I // 128).permute(0, 2, 1).reshape(M, I // 32)      # natural [M][I/32] order
    same_s = (hs == s_ref).float().mean().item()
    same_q = (h8 == q_ref).float().mean().item()
    assert same_s > 0.999 and same_q > 0.999, (same_s, same_q)
    deq = (h8.view(torch.float8_e4m3fn).float().view(M, I // 32, 32) * torch.exp2(hs.float() - 127)[..., None])
    assert err(deq.view(M, I), h0.float()) < 0.07                      # e4m3: 3 mantissa bits per block
    unit = torch.full((M, I // 32), 127, dtype=torch.uint8, device="cuda")
    for scales, tol in ((unit, 1e-4), (hs, 1e-4),
                        (torch.randint(117, 138, (M, I // 32), dtype=torch.uint8, device="cuda"), 3e-4)):
        dq = (h8.view(torch.float8_e4m3fn).double().view(M, I // 32, 32) *
              torch.exp2(scales.double() - 127)[..., None]).view(M, I)
        ref = (dq @ _deq(d8, ds).double().t()).float()
        part = torch.empty(ks, M, H, dtype=torch.float32, device="cuda")
        ops.gemm8(h8, None, d8, ds, part, epi=ops.EPI_F32, ksplit=ks, mx_in=scales)
        assert err(part.sum(0), ref) < tol, (float(err(part.sum(0), ref)), tol, int((scales == 127).all()))


@pytest.mark.parametrize("M,H,nsplit,I", [(32, 2048, 8, 16384), (17, 2048, 2, 4096), (24, 3072, 0, 1024),
                                          (32, 2048, 11, 2048), (20, 1024, 1, 2048)])
def test_mx_norm_rows_and_rstd_consumers(M, H, nsplit, I):
    """pg_norm_residual_mx (ABI 11, engine.MX_NORM): the residual update equals resid + the slabs in slab order
    (bitwise), the e4m3 rows and E8M0 block scales equal the torch MX rule on x*(1+w) (bitwise), the per-256-column
    sums of squares (per 1024 columns) match; an fp8 GEMV fed those rows (mx_in + ss_in) equals rstd * the fp32 matmul of the dequantised
    rows -- the RMSNorm split at rstd -- for the fp32 slab and the gelu*up (with MX h out) epilogues."""
    from pghip import ops
    from pghip.weights import frag_pack8, quant_rows_fp8
    g = torch.Generator().manual_seed(95)
    resid = (torch.randn(M, H, generator=g) * 3).cuda()
    part = (torch.randn(max(nsplit, 1), M, H, generator=g) * 0.5).cuda()
    w = (torch.randn(H, generator=g) * 0.2).cuda()
    want = resid.clone()
    for s in range(nsplit):
        want += part[s]
    r = resid.clone()
    q = torch.empty(M, H, dtype=torch.uint8, device="cuda")
    qs = torch.empty(M * H // 32, dtype=torch.uint8, device="cuda")
    ss = torch.empty(M, H // 1024, device="cuda")
    ops.norm_residual_mx(r, w, q, qs, ss, partials=part, nsplit=nsplit)
    assert torch.equal(r, want)
    q_ref, s_ref = _mx_quant(want * (1 + w))
    assert torch.equal(qs, s_ref)
    assert torch.equal(q, q_ref)
    assert torch.allclose(ss, want.view(M, H // 1024, 1024).pow(2).sum(-1), rtol=1e-5, atol=0)
    r2 = resid.clone()
    ops.norm_residual_mx(r2, w, q, qs, ss, partials=part, nsplit=nsplit, write_resid=False)
    assert torch.equal(r2, resid)
    rstd = torch.rsqrt(want.double().pow(2).mean(-1, keepdim=True) + 1e-6)
    xd = _mx_deq(q, qs, M, H).double()
    Wd = rnd(H, H, scale=1 / math.sqrt(H), seed=96)
    d8, ds = quant_rows_fp8(Wd)
    out = torch.empty(2, M, H, device="cuda")
    ops.gemm8(q, None, frag_pack8(d8), ds, out, epi=ops.EPI_F32, M=M, ksplit=2, frag=True, mx_in=qs, ss_in=ss)
    ref = (rstd * (xd @ _deq(d8, ds).double().t())).float()
    assert err(out.sum(0), ref) < 1e-4, float(err(out.sum(0), ref))
    Wgu = rnd(2 * I, H, scale=1 / math.sqrt(H), seed=97)
    gu8, gus = quant_rows_fp8(Wgu)
    h8 = torch.empty(M, I, dtype=torch.uint8, device="cuda")
    hs = torch.empty(M * I // 32, dtype=torch.uint8, device="cuda")
    if H // 128 not in (8, 16):     # MX rows in + MX h out need the wide form's compile-time 8 or 16 chunks
        from pghip import _lib
        with pytest.raises(_lib.PgHipError):
            ops.gemm8(q, None, frag_pack8(gu8), gus, h8, epi=ops.EPI_BF16_GELU_MUL, M=M, frag=True, mx_in=qs,
                      ss_in=ss, mx_out=hs)
        return
    ops.gemm8(q, None, frag_pack8(gu8), gus, h8, epi=ops.EPI_BF16_GELU_MUL, M=M, frag=True, mx_in=qs, ss_in=ss,
              mx_out=hs)
    gg = (rstd * (xd @ _deq(gu8, gus).double().t())).float().view(M, I // 16, 2, 16)
    hw = (torch.nn.functional.gelu(gg[:, :, 0], approximate="tanh") * gg[:, :, 1]).reshape(M, I)
    assert err(_mx_deq(h8, hs, M, I), hw) < 0.07                # e4m3 h per 32-column block


@pytest.mark.parametrize("M,N,K,ks", [(16, 2048, 16384, 8), (16, 2048, 2048, 2), (8, 1024, 4096, 4), (16, 512, 1024, 1)])
def test_gemv_fin_residual_xprime_and_pair_sums(M, N, K, ks):
    """PG_EPI_F32_FIN on the bf16 GEMV (5..16-row decode): the residual += x.W^T (+ bias) finalised in-kernel, x' =
    bf16(resid * (1 + w)) and one sum of squares per 32-column tile pair -- at the shapes that run 4 tiles per
    workgroup (N 2048 x 8 splits: the pt-448 x16 down projection) and the 2-tile ones; the tickets are left zero."""
    from pghip import ops
    from pghip.weights import frag_pack
    tiles = N // 16
    x, W = rnd(M, K, seed=91), rnd(N, K, scale=1 / math.sqrt(K), seed=92)
    bias = torch.randn(N).cuda() * 0.1
    resid0 = torch.randn(M, N).cuda()
    norm_w = torch.randn(N).cuda() * 0.1
    res = resid0.clone()
    cnt = torch.zeros(tiles, dtype=torch.int32, device="cuda")
    ss = torch.full((M, tiles), -1.0, device="cuda")
    xq = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    part = torch.empty(ks, M, N, dtype=torch.float32, device="cuda")
    fa = ops.fused_args(fin_cnt=cnt, fin_resid=res, ss_out=ss, ss_ld=tiles, fin_x=xq, norm_w=norm_w)
    ops.gemm_fused(x, frag_pack(W), part, fa, epi=ops.EPI_F32_FIN | ops.W_FRAG, M=M, ksplit=ks, bias=bias)
    torch.cuda.synchronize()
    ref = resid0 + x.float() @ W.float().t() + bias
    assert err(res, ref) < 1e-4
    assert err(xq, ref * (1 + norm_w)) < 1e-2
    pairs = (ref * ref).view(M, tiles // 2, 32).sum(-1)
    assert torch.allclose(ss[:, :tiles // 2], pairs, rtol=1e-4, atol=1e-3)
    assert int(cnt.abs().sum()) == 0


@pytest.mark.parametrize("M,z,pro", [(1, 1, 0), (1, 8, 0), (2, 2, 0), (1, 2, 2), (2, 4, 2), (16, 3, 0)])
def test_gemv_fx_add_fixed_point_residual(M, z, pro):
    """PG_EPI_FX_ADD (ABI 10): the GEMV adds round(partial * 2^32) into an int64 accumulator with integer atomics.
    The accumulated value equals x.W^T (+ bias once) to the fp32 reference's tolerance, rows past M stay zero, and --
    the point of the fixed-point form -- the same launches give the same bits every time (integer addition is
    associative, so the split arrival order does not matter); with the attention-merge prologue (o_proj) too."""
    from pghip import ops
    from pghip.weights import frag_pack
    N = 1024
    bias = torch.randn(N).cuda() * 0.1
    if pro == 2:                    # o_proj: x is the merge of split-KV attention partials
        nh, hd, nsplit, dt = 8, 256, 8, 256
        K = nh * hd
        gq = torch.Generator().manual_seed(35)
        po = torch.randn(M * nsplit * 16 * dt, generator=gq).cuda()
        pml = torch.stack([torch.randn(M * nsplit * 16, generator=gq),
                           torch.rand(M * nsplit * 16, generator=gq) + 0.5], -1).reshape(-1).contiguous().cuda()
        fa = lambda: ops.fused_args(pro_mode=ops.PRO_ATTN_COMBINE, part_o=po, part_ml=pml, asplit=nsplit,  # noqa
                                    head_dim=hd, dtw=dt, q_per_kv=nh, kv_heads=1)
        x = torch.empty(M, K, dtype=torch.bfloat16, device="cuda")
        ops.attn_combine(po, pml, x, K, B=M, Hq=nh, Hkv=1, D=hd, nsplit=nsplit)
        A = None
    else:
        K = 2048
        x = rnd(M, K, seed=33)
        fa, A = ops.fused_args, x
    W = rnd(N, K, scale=1 / 45, seed=34)
    Wk = frag_pack(W)
    runs = []
    for _ in range(3):
        acc = torch.zeros(M + 1, N, dtype=torch.int64, device="cuda")
        ops.gemm_fused(A, Wk, acc, fa(), epi=ops.EPI_FX_ADD | ops.W_FRAG, M=M, ksplit=z, bias=bias)
        runs.append(acc)
    torch.cuda.synchronize()
    ref = x.float() @ W.float().t() + bias
    got = runs[0][:M].double() / ops.FX_SCALE
    # (pro 2: the prologue's merge and pg_attn_combine may round a merged element to bf16 one ulp apart)
    assert err(got.float(), ref) < (5e-4 if pro == 2 else 1e-5)
    assert int(runs[0][M:].abs().sum()) == 0
    assert all(torch.equal(runs[0], r) for r in runs[1:])


def test_fx_add_range_check_sets_status():
    """PG_EPI_FX_ADD's range check (ABI 12, PgFusedArgs.status): a partial the int64 accumulator cannot hold -- an Inf
    or NaN from upstream, or |v| >= 2^31 -- is saturated (value +-2^30, NaN as 0) instead of wrapping through the
    undefined float->int conversion, and the status word is set; in-range launches leave it zero and their rows
    exact.  Row 0 is normal, row 1 gets an Inf in x (its dot products are +-Inf or NaN), row 2 a huge finite value."""
    from pghip import ops
    from pghip.weights import frag_pack
    M, N, K = 3, 256, 2048
    x = rnd(M, K, seed=40)
    W = rnd(N, K, scale=1 / 45, seed=41)
    Wk = frag_pack(W)
    st = torch.zeros(1, dtype=torch.int32, device="cuda")
    acc = torch.zeros(M, N, dtype=torch.int64, device="cuda")
    ops.gemm_fused(x[:1], Wk, acc, ops.fused_args(status=st), epi=ops.EPI_FX_ADD | ops.W_FRAG, M=1, ksplit=2)
    torch.cuda.synchronize()
    assert int(st.item()) == 0
    assert err((acc[0].double() / ops.FX_SCALE).float(), x[0].float() @ W.float().t()) < 1e-5
    xb = x.clone()
    xb[1, 5] = float("inf")
    xb[2, :] = 3e4                                     # x.W ~ 3e4 * 2048 * |w| ~ 1e8 .. beyond 2^31 for some n
    xb[2, :64] = 3e38
    acc.zero_()
    ops.gemm_fused(xb, Wk, acc, ops.fused_args(status=st), epi=ops.EPI_FX_ADD | ops.W_FRAG, M=M, ksplit=2)
    torch.cuda.synchronize()
    assert int(st.item()) == 1
    v = acc.double() / ops.FX_SCALE
    assert err(v[0].float(), x[0].float() @ W.float().t()) < 1e-5      # the in-range row is untouched
    lim = 2.0 ** 31                                    # 2 splits x +-2^30 at most: a finite, flagged value
    assert bool((v[1:].abs() <= lim).all()) and bool((v[1:].abs() >= 2 ** 29).any())


@pytest.mark.parametrize("M", [1, 2])
def test_fx_accumulator_consumers_rmsnorm_and_fin_clear(M):
    """The fixed-point accumulator's life in a decode step: an FX_ADD launch with resid_in folds the fp32 residual rows
    into it (split 0) beside its own partials; a pro_mode 1 GEMV normalises the accumulator alone (resid_in null) or
    resid_in + fx; a PG_EPI_F32_FIN GEMV finalises fx + its split-K slabs into fin_resid (not reading fin_resid's old
    rows) and leaves fx zero (the step's last down_proj)."""
    from pghip import ops
    from pghip.weights import frag_pack
    H, N2, K2, ks = 2048, 2048, 4096, 4
    resid = torch.randn(M, H).cuda()
    xo, Wo = rnd(M, 1024, seed=38), rnd(H, 1024, scale=1 / 32, seed=39)
    fx = torch.zeros(M, H, dtype=torch.int64, device="cuda")
    ops.gemm_fused(xo, frag_pack(Wo), fx, ops.fused_args(resid_in=resid), epi=ops.EPI_FX_ADD | ops.W_FRAG, M=M, ksplit=2)
    torch.cuda.synchronize()
    dval = (fx.double() / ops.FX_SCALE).float()
    assert err(dval, resid + xo.float() @ Wo.float().t()) < 1e-5
    w = torch.randn(H).cuda() * 0.1
    W = rnd(512, H, scale=1 / 45, seed=35)
    xn = (dval * torch.rsqrt(dval.pow(2).mean(-1, keepdim=True) + 1e-6) * (1 + w)).to(torch.bfloat16).float()
    for rin in (None, torch.zeros_like(resid)):        # the accumulator alone, or + zero fp32 rows
        out = torch.empty(M, 512, dtype=torch.bfloat16, device="cuda")
        fa = ops.fused_args(pro_mode=ops.PRO_RMSNORM, resid_in=rin, fx=fx, nsplit=0, norm_w=w, eps=1e-6)
        ops.gemm_fused(None, frag_pack(W), out, fa, epi=ops.EPI_BF16 | ops.W_FRAG, M=M)
        assert err(out, xn @ W.float().t()) < 1e-2
    # FIN: fx + x.W^T into res (whose old rows are garbage), fx cleared
    tiles = N2 // 16
    x2, W2 = rnd(M, K2, seed=36), rnd(N2, K2, scale=1 / 64, seed=37)
    res = torch.full((M, H), 1e3, device="cuda")
    cnt = torch.zeros(tiles, dtype=torch.int32, device="cuda")
    ss = torch.zeros(M, tiles, device="cuda")
    xq = torch.empty(M, N2, dtype=torch.bfloat16, device="cuda")
    part = torch.empty(ks, M, N2, device="cuda")
    fa = ops.fused_args(fin_cnt=cnt, fin_resid=res, ss_out=ss, ss_ld=tiles, fin_x=xq, norm_w=w, fx=fx)
    ops.gemm_fused(x2, frag_pack(W2), part, fa, epi=ops.EPI_F32_FIN | ops.W_FRAG, M=M, ksplit=ks)
    torch.cuda.synchronize()
    ref = dval + x2.float() @ W2.float().t()
    assert err(res, ref) < 1e-4
    assert int(fx.abs().sum()) == 0 and int(cnt.abs().sum()) == 0
