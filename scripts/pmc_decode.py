"""Eager batch-1 decode steps of the bench workload (pt-224), for rocprofv3 --pmc passes over every decode kernel
(graph replays are not attributed per dispatch, so the steps run eagerly; the kernels are the same):

    rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmcd_f -o run --output-format csv -- python scripts/pmc_decode.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "paligemma-multimodal-system_amd")]
import torch  # noqa: E402
from pghip import configs, engine, synthetic, weights  # noqa: E402
import bench  # noqa: E402

cfg = configs.PT_224
sd = synthetic.SyntheticStateDict(cfg)
eng = engine.PaliGemmaEngine(cfg, weights.PackedWeights(cfg, sd.__getitem__))
ids, px = bench.synthetic_inputs(cfg, 1, [2, 651, 4906, 603, 476, 2121, 576, 108])
ids, px = ids.cuda(), px.cuda()
sampler = dict(do_sample=False)
cache, feats, logits, nxt = eng.prefill_request(ids, px, torch.ones_like(ids), 64)
st = eng.decode_state(1, cache, nxt, 64, sampler=sampler)
eng.sample(logits, st, sampler, advance=False, feats=feats)
for _ in range(6):
    eng.decode_step(st, cache, feats, sampler)
torch.cuda.synchronize()
print("decode steps done")
