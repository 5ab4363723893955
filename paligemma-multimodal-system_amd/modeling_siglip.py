"""SigLIP vision tower — drop-in for the reference's ``modeling_siglip`` module, computed by libpghip.

Same names, constructor arguments, module tree and state-dict keys as the reference
(modeling_siglip.py:10-334).  ``SiglipVisionModel.forward`` runs the whole tower as one
kernel sequence (im2col -> patch GEMM with bias+position epilogue -> per layer LayerNorm,
fused QKV GEMM (V written transposed), flash attention, out GEMM, LayerNorm, fc1 GEMM+GELU,
fc2 GEMM -> post-LayerNorm); the sub-modules' forwards run their own part through the same
kernels.  The residual stream is fp32, MFMA operands bf16.  HIP tensors only.
``SiglipAttention.forward`` returns ``(out, weights)``: the flash kernel never forms the score matrix, so weights is
None unless asked for (``module.return_attn_weights = True`` or PG_ATTN_WEIGHTS=1); then pg_attn_probs forms what
the reference returns there (:157), the scaled scores from before the softmax.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from pghip import ops
from pghip.engine import PaliGemmaEngine
from pghip.weights import PackedWeights


def _require_hip(t: torch.Tensor, what: str):
    if not t.is_cuda:
        raise RuntimeError(f"{what}: the pghip path runs on the HIP device only (got {t.device})")


def _rup(x, m):
    return (x + m - 1) // m * m


def _bf(t):
    return t.detach().to(torch.bfloat16).contiguous()


def _f32(t):
    return t.detach().to(torch.float32).contiguous()


class _Pack:
    def __init__(self):
        self.key, self.val = None, None

    def get(self, params, build):
        key = tuple((p.data_ptr(), p._version, p.device) for p in params)
        if key != self.key:
            self.val, self.key = build(), key
        return self.val


class SiglipVisionConfig:
    """Vision hyper-parameters (modeling_siglip.py:10-38); unknown keys accepted."""

    def __init__(self, image_size: int = 224, patch_size: int = 16, num_channels: int = 3, hidden_size: int = 768,
                 intermediate_size: int = 3072, num_hidden_layers: int = 12, num_attention_heads: int = 12,
                 attention_dropout: float = 0.0, layer_norm_eps: float = 1e-6, num_image_tokens: int = None,
                 **kwargs):
        self.image_size, self.patch_size, self.num_channels = image_size, patch_size, num_channels
        self.hidden_size, self.intermediate_size = hidden_size, intermediate_size
        self.num_hidden_layers, self.num_attention_heads = num_hidden_layers, num_attention_heads
        self.attention_dropout, self.layer_norm_eps = attention_dropout, layer_norm_eps
        self.num_image_tokens = num_image_tokens
        for k, v in kwargs.items():
            setattr(self, k, v)

    def as_dict(self) -> dict:
        return {k: v for k, v in vars(self).items() if not k.startswith("_")}


class LayerNorm(nn.LayerNorm):
    """nn.LayerNorm (same parameters / keys) whose forward is the pghip norm kernel (fp32 out)."""

    def forward(self, x):
        _require_hip(x, "LayerNorm")
        r = x.reshape(-1, x.shape[-1]).to(torch.float32).contiguous()
        out = torch.empty_like(r)
        ops.norm_residual(r, _f32(self.weight), b=_f32(self.bias), mode=ops.NORM_LAYER, eps=self.eps, out_f32=out,
                          write_resid=False)
        return out.view(x.shape)


class SiglipAttention(nn.Module):
    """Bidirectional multi-head attention (modeling_siglip.py:41-157) on the flash kernel."""

    def __init__(self, config: SiglipVisionConfig):
        super().__init__()
        self.embed_dim, self.num_heads = config.hidden_size, config.num_attention_heads
        self.head_dim = self.embed_dim // self.num_heads
        self.scale = 1 / (self.head_dim ** 0.5)
        self.dropout = config.attention_dropout
        self.key_proj = nn.Linear(self.embed_dim, self.embed_dim)
        self.value_proj = nn.Linear(self.embed_dim, self.embed_dim)
        self.query_proj = nn.Linear(self.embed_dim, self.embed_dim)
        self.out_proj = nn.Linear(self.embed_dim, self.embed_dim)
        self._pk = _Pack()
        self.return_attn_weights = ops.ATTN_WEIGHTS

    def packed(self):
        ps = [self.query_proj.weight, self.key_proj.weight, self.value_proj.weight, self.out_proj.weight,
              self.query_proj.bias, self.key_proj.bias, self.value_proj.bias, self.out_proj.bias]
        return self._pk.get(ps, lambda: (
            torch.cat([_bf(self.query_proj.weight), _bf(self.key_proj.weight), _bf(self.value_proj.weight)]),
            torch.cat([_f32(self.query_proj.bias), _f32(self.key_proj.bias), _f32(self.value_proj.bias)]),
            _bf(self.out_proj.weight), _f32(self.out_proj.bias)))

    def forward(self, x):
        _require_hip(x, "SiglipAttention")
        B, N, E = x.shape
        if E % 64:
            raise ValueError(f"hidden size {E} must be a multiple of 64 for the MFMA path")
        wqkv, bqkv, wo, bo = self.packed()
        M = B * N
        xb = x.reshape(M, E).to(torch.bfloat16).contiguous()
        qkv = torch.empty(M, 3 * E, dtype=torch.bfloat16, device=x.device)
        vt = torch.zeros(E, M + 32, dtype=torch.bfloat16, device=x.device)
        ops.gemm(xb, wqkv, qkv, epi=ops.EPI_BF16_VT, bias=bqkv, aux_out=vt, aux_ld=M + 32, aux_n=2 * E)
        o = torch.empty(M, E, dtype=torch.bfloat16, device=x.device)
        hd = self.head_dim
        ops.attention(qkv, 3 * E, o, E, qkv[:, E:], N * 3 * E, hd, 3 * E, vt, N, hd * (M + 32), M + 32,
                      B=B, Lq=N, Lkv=N, Hq=self.num_heads, Hkv=self.num_heads, D=hd, scale=self.scale)
        out = torch.empty(M, E, dtype=torch.float32, device=x.device)
        ops.gemm(o, wo, out, epi=ops.EPI_F32, bias=bo)
        weights = None
        if self.return_attn_weights:        # what the reference returns (:157): its scaled scores from before the softmax
            weights = ops.attn_probs(qkv, 3 * E, qkv[:, E:], N * 3 * E, hd, 3 * E, B=B, Lq=N, Lkv=N,
                                     Hq=self.num_heads, Hkv=self.num_heads, D=hd, scale=self.scale, probs=False)
        return out.view(B, N, E), weights


class SiglipMLP(nn.Module):
    """fc2(gelu_tanh(fc1(x))) (modeling_siglip.py:160-186); GELU fused into the fc1 GEMM epilogue."""

    def __init__(self, config: SiglipVisionConfig):
        super().__init__()
        self.intermediate_size, self.embed_dim = config.intermediate_size, config.hidden_size
        self.fc1 = nn.Linear(self.embed_dim, self.intermediate_size)
        self.fc2 = nn.Linear(self.intermediate_size, self.embed_dim)
        self._pk = _Pack()

    def packed(self):
        def build():
            I, E = self.intermediate_size, self.embed_dim
            Ip = _rup(I, 64)
            w1 = torch.zeros(Ip, E, dtype=torch.bfloat16, device=self.fc1.weight.device)
            w1[:I] = _bf(self.fc1.weight)
            b1 = torch.zeros(Ip, dtype=torch.float32, device=self.fc1.weight.device)
            b1[:I] = _f32(self.fc1.bias)
            w2 = torch.zeros(E, Ip, dtype=torch.bfloat16, device=self.fc2.weight.device)
            w2[:, :I] = _bf(self.fc2.weight)
            return w1, b1, w2, _f32(self.fc2.bias)
        return self._pk.get([self.fc1.weight, self.fc1.bias, self.fc2.weight, self.fc2.bias], build)

    def forward(self, x):
        _require_hip(x, "SiglipMLP")
        w1, b1, w2, b2 = self.packed()
        xb = x.reshape(-1, x.shape[-1]).to(torch.bfloat16).contiguous()
        h = torch.empty(xb.shape[0], w1.shape[0], dtype=torch.bfloat16, device=x.device)
        ops.gemm(xb, w1, h, epi=ops.EPI_BF16_GELU, bias=b1)
        out = torch.empty(xb.shape[0], self.embed_dim, dtype=torch.float32, device=x.device)
        ops.gemm(h, w2, out, epi=ops.EPI_F32, bias=b2)
        return out.view(*x.shape[:-1], self.embed_dim)


class SiglipEncoderLayer(nn.Module):
    """Pre-LN block: x + attn(LN1(x)), then x + mlp(LN2(x)) (modeling_siglip.py:189-221)."""

    def __init__(self, config: SiglipVisionConfig):
        super().__init__()
        self.layer_norm_eps, self.embed_dim = config.layer_norm_eps, config.hidden_size
        self.layer_norm1 = LayerNorm(normalized_shape=self.embed_dim, eps=self.layer_norm_eps)
        self.self_attn = SiglipAttention(config)
        self.mlp = SiglipMLP(config)
        self.layer_norm2 = LayerNorm(normalized_shape=self.embed_dim, eps=self.layer_norm_eps)

    def forward(self, x):
        x = x.to(torch.float32)
        a, _ = self.self_attn(self.layer_norm1(x))
        x = x + a
        return x + self.mlp(self.layer_norm2(x))


class SiglipEncoder(nn.Module):
    """Stack of encoder layers (modeling_siglip.py:224-239)."""

    def __init__(self, config: SiglipVisionConfig):
        super().__init__()
        self.num_hidden_layers, self.hidden_size = config.num_hidden_layers, config.hidden_size
        self.layers = nn.ModuleList([SiglipEncoderLayer(config) for _ in range(self.num_hidden_layers)])

    def forward(self, x):
        for layer in self.layers:
            x = layer(x)
        return x


class SiglipVisionEmbeddings(nn.Module):
    """Conv patch embedding + learned positions (modeling_siglip.py:241-299) as im2col + one GEMM whose
    epilogue adds the conv bias and the position embedding."""

    def __init__(self, config: SiglipVisionConfig):
        super().__init__()
        self.patch_size, self.image_size = config.patch_size, config.image_size
        self.num_patches = (self.image_size // self.patch_size) ** 2
        self.num_channels, self.embed_dim = config.num_channels, config.hidden_size
        self.patch_embedding = nn.Conv2d(in_channels=self.num_channels, out_channels=self.embed_dim,
                                         stride=self.patch_size, kernel_size=self.patch_size, padding="valid")
        self.positional_embeddings = nn.Embedding(self.num_patches, self.embed_dim)
        self.position_ids = torch.arange(self.num_patches).expand((1, -1))
        self.register_buffer(name="postion_ids", tensor=self.position_ids, persistent=False)
        self._pk = _Pack()

    def packed(self):
        def build():
            E, C, p = self.embed_dim, self.num_channels, self.patch_size
            kraw = C * p * p
            w = torch.zeros(E, _rup(kraw, 64), dtype=torch.bfloat16, device=self.patch_embedding.weight.device)
            w[:, :kraw] = _bf(self.patch_embedding.weight).reshape(E, kraw)
            return w, _f32(self.patch_embedding.bias), _f32(self.positional_embeddings.weight)
        ps = [self.patch_embedding.weight, self.patch_embedding.bias, self.positional_embeddings.weight]
        return self._pk.get(ps, build)

    def forward(self, x: torch.FloatTensor):
        _require_hip(x, "SiglipVisionEmbeddings")
        w, b, pos = self.packed()
        B = x.shape[0]
        n = (x.shape[2] // self.patch_size) * (x.shape[3] // self.patch_size)
        patches = torch.empty(B * n, w.shape[1], dtype=torch.bfloat16, device=x.device)
        ops.patch_im2col(x.to(torch.float32), self.patch_size, patches)
        out = torch.empty(B * n, self.embed_dim, dtype=torch.float32, device=x.device)
        ops.gemm(patches, w, out, epi=ops.EPI_F32_POS, bias=b, aux=pos, aux_rows=n)
        return out.view(B, n, self.embed_dim)


class SiglipTransformer(nn.Module):
    """embeddings -> encoder -> post-LayerNorm (modeling_siglip.py:303-320)."""

    def __init__(self, config: SiglipVisionConfig):
        super().__init__()
        self.config = config
        self.embeddings = SiglipVisionEmbeddings(config)
        self.encoder = SiglipEncoder(config)
        self.post_layernorm = LayerNorm(config.hidden_size, eps=config.layer_norm_eps)

    def forward(self, x):
        return self.post_layernorm(self.encoder(self.embeddings(x)))


class SiglipVisionModel(nn.Module):
    """(B, C, H, W) pixels -> (B, num_patches, hidden) fp32 (modeling_siglip.py:324-334).

    Runs the fused whole-tower kernel sequence of pghip.engine (packed once, re-packed
    when parameters change)."""

    def __init__(self, config: SiglipVisionConfig):
        super().__init__()
        self.config = config
        self.model = SiglipTransformer(self.config)
        self._pk = _Pack()

    def _engine(self, device):
        def build():
            sd = {"vision_tower." + k: v for k, v in self.state_dict().items()}
            cfg = {"vision_config": self.config.as_dict()}
            return PaliGemmaEngine(cfg, PackedWeights(cfg, sd.__getitem__, device=device, parts=("vision",)),
                                   device=device)
        return self._pk.get(list(self.parameters()), build)

    def forward(self, x):
        _require_hip(x, "SiglipVisionModel")
        _, hid = self._engine(x.device).vision(x, want_hidden=True)
        n = hid.shape[0] // x.shape[0]
        return hid.view(x.shape[0], n, -1)
