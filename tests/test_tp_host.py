"""Tensor-parallel sharding on the CPU (gloo, world size 2, 4 and 8): the per-rank weight slices
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
    from pghip.weights import PackedWeights, frag_unpack
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
            # the MLP's row-parallel partial sum, all-reduced in row chunks issued asynchronously before any is
            # waited on (engine._row_parallel at T >= 2 * AR_CHUNK_ROWS): the same sums as one all-reduce
            part = O.gemma_mlp(Wl, lp + "mlp.", x).reshape(B * L, H)
            t = torch.from_numpy(np.ascontiguousarray(part))
            bounds = [B * L * c // 3 for c in range(4)]
            works = [dist.all_reduce(t[r0:r1], async_op=True) for r0, r1 in zip(bounds[:-1], bounds[1:])]
            for wk in works:
                wk.wait()
            full = O.gemma_mlp(W, lp + "mlp.", x).reshape(B * L, H)
            np.testing.assert_allclose(t.numpy(), full, rtol=0, atol=2e-5 * np.abs(full).max())
        # vocabulary-parallel lm_head (engine.lm_head): every rank's slice [rows][vocab_local_pad], all-gathered in
        # rank order, the padding dropped, slices concatenated
        xr = x.reshape(-1, H)
        rows = xr.shape[0]
        lm_w = frag_unpack(P.lm_w) if P.frag else P.lm_w
        loc = (torch.from_numpy(xr) @ lm_w.float().T + P.lm_bias).contiguous()
        g = torch.empty(world, rows, P.vocab_local_pad)
        dist.all_gather_into_tensor(g.view(-1), loc.view(-1))
        got = g[:, :, :P.vocab_local].permute(1, 0, 2).reshape(rows, -1)
        full = xr @ W["language_model.model.embed_tokens.weight"].T + W["language_model.lm_head.bias"]
        np.testing.assert_allclose(got.numpy(), full, rtol=0, atol=2e-5 * np.abs(full).max())
        # greedy (engine.decode_step, pg_argmax_pairs + pg_argmax_merge): each rank's (max, first global index)
        # pair per row, all-gathered [W][rows][2]; the merge keeps the largest value, the lowest index on ties.
        # Ties across ranks are forced on row 0 (the same value planted in every rank's slice) -> rank 0's index.
        loc = loc[:, :P.vocab_local].clone()
        loc[0, 5] = 1e4
        mx, ix = loc.max(-1)
        mine = torch.stack([mx, (ix + P.vocab_offset).float()], -1).contiguous()
        pairs = torch.empty(world, rows, 2)
        dist.all_gather_into_tensor(pairs.view(-1), mine.view(-1))
        best = pairs[:, :, 0].argmax(0)                                   # first rank holding the max
        merged = pairs[best, torch.arange(rows), 1].long()
        ref = full.copy()
        for r in range(world):
            ref[0, r * P.vocab_local + 5] = 1e4
        assert merged.tolist() == ref.argmax(-1).tolist()
        assert merged[0].item() == 5
        # data-parallel SigLIP (engine.vision with B >= W, B % W == 0): rank r encodes images [r*B/W, (r+1)*B/W)
        # and the projected features are all-gathered in rank order = image order
        vcfg = cfg["vision_config"]
        n_img = (vcfg["image_size"] // vcfg["patch_size"]) ** 2
        Bi = world
        px = rng.standard_normal((Bi, 3, vcfg["image_size"], vcfg["image_size"])).astype(np.float32)
        Bl = Bi // world
        mine = O.multi_modal_projector(W, O.siglip_vision_model(W, vcfg, px[rank * Bl:(rank + 1) * Bl]))
        feats = torch.empty(Bi * n_img * mine.shape[-1])
        dist.all_gather_into_tensor(feats, torch.from_numpy(np.ascontiguousarray(mine)).view(-1))
        full = O.multi_modal_projector(W, O.siglip_vision_model(W, vcfg, px))
        np.testing.assert_allclose(feats.view(full.shape).numpy(), full, rtol=0, atol=1e-5 * np.abs(full).max())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("cfg_name,world", [("tiny", 2), ("tiny", 4), ("tiny8", 2), ("tiny8", 4), ("tiny8", 8)])
def test_tp_sharding_matches_unsharded_oracle(cfg_name, world):
    """world 8 on tiny8 = one q head, 80 intermediate columns and 38 vocabulary rows per rank: the TP=8 split of
    BASELINE configs[4] (modeling_gemma.py:205-218 MLP, :255-259 q/k/v/o, :484/:523 lm_head)."""
    mp.spawn(_worker, args=(world, _free_port(), cfg_name), nprocs=world, join=True)


def test_tp_rejects_bad_split():
    from pghip.weights import PackedWeights
    cfg = ocfg.TINY
    W = synth.generate_state_dict(cfg)
    with pytest.raises(ValueError):
        PackedWeights(cfg, lambda k: torch.from_numpy(W[k]), device="cpu", parts=("text",), tp_rank=0, tp_world=3)
