"""Tensor-parallel sharding on the CPU (gloo, world size 2 and 4): the per-rank weight slices
PackedWeights(tp_rank, tp_world) produces, run through the oracle's own layer functions and summed
with a torch.distributed SUM all-reduce — exactly the data flow of the HIP engine under TP — must
reproduce the unsharded oracle layer (modeling_gemma.py:264-358 attention, :210-218 MLP, :530-534
lm_head).  Runs with no GPU: it checks the sharding plan and the collective, not the kernels
(tests/test_tp_gpu.py runs the kernels with two ranks on one device)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import configs as ocfg, synth
from oracle import paligemma_oracle as O


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _unpack_layer(P, i):
    """Packed (kernel-layout) slices of layer i back to reference-layout weights of this shard."""
    from pghip.weights import frag_unpack, rope_row_perm
    L = {k: (frag_unpack(v) if P.frag and v.dim() == 2 else v) for k, v in P.tl[i].items()}
    hd, H, nb = P.head_dim, P.hidden, P.heads + 2 * P.kv_heads
    inv = torch.argsort(rope_row_perm(hd))
    qkv = L["qkv_w"].float().view(nb, hd, H)[:, inv, :]
    q = qkv[:P.heads].reshape(-1, H)
    k = qkv[P.heads:P.heads + P.kv_heads].reshape(-1, H)
    v = qkv[P.heads + P.kv_heads:].reshape(-1, H)
    gu = L["gu_w"].float().view(P.inter // 16, 2, 16, H)
    lp = f"language_model.model.layers.{i}."
    f = lambda t: t.numpy().astype(np.float32)  # noqa: E731
    return {lp + "self_attn.q_proj.weight": f(q), lp + "self_attn.k_proj.weight": f(k),
            lp + "self_attn.v_proj.weight": f(v), lp + "self_attn.o_proj.weight": f(L["o_w"].float()),
            lp + "mlp.gate_proj.weight": f(gu[:, 0].reshape(-1, H)), lp + "mlp.up_proj.weight": f(gu[:, 1].reshape(-1, H)),
            lp + "mlp.down_proj.weight": f(L["down_w"].float())}


def _worker(rank, world, port, cfg_name):
    from pghip.weights import PackedWeights
    dist.init_process_group("gloo", rank=rank, world_size=world, init_method=f"tcp://127.0.0.1:{port}")
    try:
        cfg = ocfg.CONFIGS[cfg_name]
        tc = cfg["text_config"]
        W = synth.generate_state_dict(cfg)
        P = PackedWeights(cfg, lambda k: torch.from_numpy(W[k]), device="cpu", parts=("text",), tp_rank=rank,
                          tp_world=world)
        assert P.heads * world == tc["num_attention_heads"] and P.inter_real * world == tc["intermediate_size"]
        rng = np.random.default_rng(7)
        B, L, H = 2, 9, tc["hidden_size"]
        x = (rng.standard_normal((B, L, H)) * 0.5).astype(np.float32)
        pos = np.tile(np.arange(1, L + 1), (B, 1))
        mask = np.triu(np.full((L, L), -1e9, np.float32), 1)[None, None].repeat(B, 0)
        tc_local = dict(tc, num_attention_heads=P.heads, intermediate_size=P.inter)
        for i in range(tc["num_hidden_layers"]):
            lp = f"language_model.model.layers.{i}."
            Wl = _unpack_layer(P, i)
            part = O.gemma_attention(Wl, lp + "self_attn.", tc_local, i, x, pos, mask, None)
            t = torch.from_numpy(np.ascontiguousarray(part))
            dist.all_reduce(t)
            full = O.gemma_attention(W, lp + "self_attn.", tc, i, x, pos, mask, None)
            np.testing.assert_allclose(t.numpy(), full, rtol=0, atol=2e-5 * np.abs(full).max())
            part = O.gemma_mlp(Wl, lp + "mlp.", x)
            t = torch.from_numpy(np.ascontiguousarray(part))
            dist.all_reduce(t)
            full = O.gemma_mlp(W, lp + "mlp.", x)
            np.testing.assert_allclose(t.numpy(), full, rtol=0, atol=2e-5 * np.abs(full).max())
        # vocabulary-parallel lm_head: each rank fills its slot of a zeroed buffer, SUM all-reduce gathers
        xr = x.reshape(-1, H)
        g = torch.zeros(xr.shape[0], world, P.vocab_local_pad)
        from pghip.weights import frag_unpack
        lm_w = frag_unpack(P.lm_w) if P.frag else P.lm_w
        g[:, rank] = torch.from_numpy(xr) @ lm_w.float().T + P.lm_bias
        dist.all_reduce(g)
        full = xr @ W["language_model.model.embed_tokens.weight"].T + W["language_model.lm_head.bias"]
        np.testing.assert_allclose(g[:, :, :P.vocab_local].reshape(xr.shape[0], -1).numpy(), full, rtol=0, atol=2e-5 * np.abs(full).max())
        # greedy merge of per-rank (max, first index) pairs == global argmax (lowest index on ties)
        loc = g[:, rank, :P.vocab_local]
        pairs = torch.zeros(world, xr.shape[0], 2)
        mx, ix = loc.max(-1)
        pairs[rank, :, 0], pairs[rank, :, 1] = mx, (ix + P.vocab_offset).float()
        dist.all_reduce(pairs)
        best = pairs[:, :, 0].argmax(0)                                   # first rank holding the max
        merged = pairs[best, torch.arange(xr.shape[0]), 1].long()
        assert merged.tolist() == full.argmax(-1).tolist()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_tp_sharding_matches_unsharded_oracle(world):
    mp.spawn(_worker, args=(world, _free_port(), "tiny"), nprocs=world, join=True)


def test_tp_rejects_bad_split():
    from pghip.weights import PackedWeights
    cfg = ocfg.TINY
    W = synth.generate_state_dict(cfg)
    with pytest.raises(ValueError):
        PackedWeights(cfg, lambda k: torch.from_numpy(W[k]), device="cpu", parts=("text",), tp_rank=0, tp_world=3)
