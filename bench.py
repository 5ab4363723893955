"""Headline bench: PaliGemma-3B image->text tokens/s + prefill ms on MI355X.

A "step" = one full request of BASELINE.json configs[1] (PaliGemma-3B-pt-224, bf16, batch 1,
greedy): synthetic 224x224 image + 8-token prompt resident in HBM -> SigLIP -> projector ->
merge -> Gemma prefill -> 128 greedy tokens (graph-replayed decode steps; EOS ignored so the
token count is fixed).  value = generated tokens / step wall time over all ranks.

Multi-GPU (torch.distributed.run, one rank per GPU): --parallel dp (default) runs one request per
rank (independent replicas, weak scaling; no data-path collective); value = all ranks' tokens /
max-over-ranks time.  --parallel tp shards the Gemma decoder over all ranks (q heads, gate/up
columns, vocabulary; a SUM all-reduce after o_proj and down_proj over xGMI peer stores: one-shot for
decode-size slabs, reduce-scatter + all-gather for prefill chunks; --comm rccl uses the process
group's collective instead) and runs ONE request across them (strong scaling: per-token latency); value = that
request's tokens / time.  `--gpus N` without WORLD_SIZE launches the N ranks itself (a torch.distributed.run child).

Extra fields: prefill_ms, decode_tok_s, decode HBM fraction; "roofline" for the dominant
kernel (the decode gate/up GEMV, HIP events on the stream it runs on); "cpu_baseline" = the
oracle (numpy port of the reference path, fp32, vision re-run per token as the reference does)
on a bounded sample, rank 0, N=1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "paligemma-multimodal-system_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

try:
    with open(os.path.join(ROOT, "BASELINE.json")) as _f:
        BASELINE_METRIC = json.load(_f)["metric"]
except Exception:  # pragma: no cover
    BASELINE_METRIC = "image->text tokens/sec + prefill ms, PaliGemma-3B-224 at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
BF16_PEAK_TFS = 2500.0     # dense bf16 MFMA
FP8_PEAK_TFS = 5000.0      # dense fp8 e4m3 MFMA


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def synthetic_inputs(cfg, B, prompt_ids):
    from pghip.configs import num_image_tokens
    n = num_image_tokens(cfg)
    size = cfg["vision_config"].get("image_size", 224)
    rng = np.random.default_rng(1234)
    img = rng.integers(0, 256, (B, size, size, 3), dtype=np.uint8)
    px = ((img.astype(np.float32) * np.float32(1 / 255.0)) - np.float32(0.5)) / np.float32(0.5)
    px = torch.from_numpy(np.ascontiguousarray(px.transpose(0, 3, 1, 2)))
    ids = torch.tensor([[cfg["image_token_index"]] * n + prompt_ids] * B, dtype=torch.int64)
    return ids, px


def prefill_flops(cfg, B, L):
    """sum 2*M*N*K over linears + attention + last-token lm_head."""
    v, t = cfg["vision_config"], cfg["text_config"]
    n = (v.get("image_size", 224) // v["patch_size"]) ** 2
    hv, iv, lv = v["hidden_size"], v["intermediate_size"], v["num_hidden_layers"]
    vis = 2 * n * (3 * 14 * 14) * hv + lv * (2 * n * hv * hv * 4 + 2 * n * hv * iv * 2 + 4 * n * n * hv)
    vis += 2 * n * hv * cfg.get("projection_dim", 2048)
    H, I, nh, nkv, hd = t["hidden_size"], t["intermediate_size"], t["num_attention_heads"], t["num_key_value_heads"], 256
    per = 2 * L * H * (nh * hd + 2 * nkv * hd) + 2 * L * nh * hd * H + 2 * L * H * I * 3 + 4 * L * L * nh * hd
    txt = t["num_hidden_layers"] * per + 2 * H * t["vocab_size"]
    return B * (vis + txt)


def gemma_linear_flops(cfg, B, L):
    """The Gemma decoder linears' share of prefill_flops (the part the --fp8 path runs on e4m3 MFMA)."""
    t = cfg["text_config"]
    H, I, nh, nkv, hd = t["hidden_size"], t["intermediate_size"], t["num_attention_heads"], t["num_key_value_heads"], 256
    per = 2 * L * H * (nh * hd + 2 * nkv * hd) + 2 * L * nh * hd * H + 2 * L * H * I * 3
    return B * t["num_hidden_layers"] * per


def time_dominant_kernel(eng, reps=50):
    """Average duration of the decode gate/up GEMV (the largest byte stream of a decode step) with HIP
    events on the current stream, which is the stream it is launched on."""
    from pghip import ops
    w = eng.w
    L0 = w.tl[0]
    x = torch.randn(1, w.hidden, device="cuda").to(torch.bfloat16)
    h = torch.empty(1, w.inter, dtype=torch.bfloat16, device="cuda")
    for _ in range(5):
        ops.gemm(x, L0["gu_w"], h, epi=ops.EPI_BF16_GELU_MUL | w.wflag)
    # rotate over the 18 layers' weights so every launch streams from HBM (no L2/MALL reuse).  The launches are
    # replayed from a captured graph: issued eagerly, a slow host (~40 us per Python launch on some boxes) cannot
    # keep ahead of 21 us kernels, and the events would time the host instead of the kernel
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        ops.gemm(x, L0["gu_w"], h, epi=ops.EPI_BF16_GELU_MUL | w.wflag)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        for i in range(reps):
            ops.gemm(x, w.tl[i % len(w.tl)]["gu_w"], h, epi=ops.EPI_BF16_GELU_MUL | w.wflag)
    g.replay()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    for _ in range(4):          # keep the stream busy while the host enqueues the timed replay
        ops.gemm(x, L0["gu_w"], h, epi=ops.EPI_BF16_GELU_MUL | w.wflag)
    ev0.record()
    g.replay()
    ev1.record()
    torch.cuda.synchronize()
    avg_s = ev0.elapsed_time(ev1) / 1e3 / reps
    nbytes = L0["gu_w"].numel() * 2 + w.hidden * 2 + w.inter * 2
    return avg_s, nbytes


def pmc_traffic():
    """HBM bytes per launch of the roofline kernel from the committed rocprofv3 --pmc passes
    (scripts/gpu_pmc_gateup.sh -> profiles/*pmc_gateup.json: FETCH_SIZE x2 (gfx950) + WRITE_SIZE), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_gateup.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        rec = json.load(f)
    return rec.get("traffic_bytes_per_launch"), os.path.relpath(files[-1], ROOT)


def cpu_baseline(cfg, ids, px, budget_tokens=24):
    """The oracle (numpy fp32 port of the reference path) on the host: one request of the same workload,
    bounded to `budget_tokens` generated tokens (prefill + decode steps, vision re-run per call as the
    reference's modeling_paligemma.py:281 does).  Weights: the same synthetic tensors, copied from HBM."""
    from oracle import paligemma_oracle as O
    from pghip import synthetic
    try:
        from threadpoolctl import threadpool_info
        threads = max([p.get("num_threads", 1) for p in threadpool_info() if p.get("user_api") == "blas"] or [1])
    except Exception:
        threads = os.cpu_count()
    sd = synthetic.SyntheticStateDict(cfg)
    W = {k: sd[k].float().cpu().numpy() for k in sd.keys()}
    torch.cuda.empty_cache()
    orc = O.PaliGemmaOracle(cfg, W, recompute_vision=True)
    t0 = time.perf_counter()
    out = O.generate(orc, ids.numpy(), px.numpy(), np.ones_like(ids.numpy()), budget_tokens, stop_token=None)
    dt = time.perf_counter() - t0
    del W, orc
    return {"value": round(len(out) * ids.shape[0] / dt, 4), "unit": "tokens/s", "cores": int(threads),
            "kind": "port",
            "sample": f"{len(out)} generated tokens of the same request (1 prefill L={ids.shape[1]} + "
                      f"{len(out) - 1} decode steps re-running SigLIP like the reference), fp32 numpy, {dt:.1f} s"}


class Runner:
    """One request of the bench workload on an engine: prefill (vision + merge + Gemma prefill, first token
    sampled) into a static cache, then T-1 decode steps replayed from one captured hipGraph (eager steps when
    the collectives cannot be captured)."""

    def __init__(self, eng, ids, px, T, sampler, graph_prefill=False, rank=0):
        B, L = ids.shape
        self.state = state = {}
        mask = torch.ones_like(ids)
        cache, feats, logits, nxt = eng.prefill_request(ids, px, mask, T)
        st = eng.decode_state(B, cache, nxt, T, sampler=sampler)
        eng.sample(logits, st, sampler, advance=False, feats=feats)
        state.update(cache=cache, feats=feats, st=st)
        try:
            if not eng.comm.capturable:
                raise RuntimeError(f"{eng.comm.backend} collectives are not graph-capturable")
            self.replay = eng._graph_step(st, cache, feats, sampler)
            self.graph_mode = "hipgraph"
        except Exception as e:  # collectives that cannot be captured: eager decode steps
            log(f"[bench] rank {rank}: decode-step capture failed ({e}); running eager steps")
            torch.cuda.synchronize()
            self.replay = lambda: eng.decode_step(state["st"], state["cache"], state["feats"], sampler)  # noqa
            self.graph_mode = "eager"
        rows = eng._buf("p_rows", (B,), torch.int32)
        rows.copy_(torch.arange(B, dtype=torch.int32) * L + (L - 1))
        pos_pf = torch.arange(1, L + 1, device="cuda", dtype=torch.int32).repeat(B, 1)

        def prefill():
            # vision + merge + Gemma prefill into the decode graph's static cache / state, first token sampled
            f = eng.vision(px)
            resid = eng._buf("p_resid", (B * L, eng.w.hidden), torch.float32)
            eng.embed_merge(ids, f, resid)
            lg, _ = eng.gemma_prefill(resid, pos_pf, cache, B, L, logits_rows=rows)
            state["st"]["pos"].fill_(L + 1)
            state["st"]["kv_len"].fill_(L)
            state["st"]["step"].zero_()
            state["feats"].copy_(f)
            eng.sample(lg, state["st"], sampler, advance=False, feats=state["feats"])

        # optionally the prefill's ~400 launches as one hipGraph (fixed request shape, as a serving replica would
        # hold one per shape bucket); measured slower than eager launches on MI355X (pt-224 6.0 vs 5.76 ms,
        # pt-448 x16 91.6 vs 89.0 ms), so eager is the default
        self.prefill_run, self.prefill_mode = prefill, "eager"
        if self.graph_mode == "hipgraph" and graph_prefill:
            try:
                prefill()                                  # every workspace allocated outside capture
                torch.cuda.synchronize()
                g_pf = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g_pf):
                    prefill()
                torch.cuda.synchronize()
                self.prefill_run, self.prefill_mode = g_pf.replay, "hipgraph"
            except Exception as e:
                log(f"[bench] rank {rank}: prefill capture failed ({e}); eager prefill")
                torch.cuda.synchronize()
        self.T, self.L = T, L

    def request(self):
        self.prefill_run()
        for _ in range(self.T - 1):
            self.replay()


def tp_leg(spec, rank, world, dist, steps=2):
    """One tensor-parallel run over the ranks [0, spec["tp"]) (q heads, gate/up columns and the
    vocabulary split; SigLIP data-parallel over the images when the batch covers the ranks; decode-size
    collectives as pg_allreduce_xgmi / pg_allgather_xgmi one-shot peer stores over xGMI, prefill chunks on the
    reduce-scatter + all-gather pg_allreduce_xgmi_rs, anything beyond their buffers on the process group),
    timing `steps` requests of spec's workload.  Every rank of the world takes part in the phase agreements;
    ranks outside the TP group idle.  Phases: communicator setup, engine build (local only: packing, no
    collective), a first request (prefill + decode-graph capture), timed requests.  After each phase all ranks
    agree on its outcome (MIN of an ok flag), so a failure on one rank stops every rank at the same point and no
    rank waits in a collective its peers skipped.  Any failure is reported in the record, never
    raised."""
    from pghip import configs, engine, synthetic, weights
    from pghip.tp import XgmiComm
    tp = spec["tp"]
    cfg = configs.CONFIGS[spec["config"]]
    B, T, fp8, sample = spec["batch"], spec["tokens"], spec.get("fp8", False), spec.get("sample", False)
    out = {"tp": tp, "config": spec["config"], "batch": B, "tokens": T, "fp8": fp8,
           "sampler": "top-p T=0.8 p=0.9 (uniforms seed 4321)" if sample else "greedy", "baseline": spec["baseline"],
           "comm": "xGMI peer-store kernels: pg_allreduce_xgmi / pg_allgather_xgmi (decode-size), pg_allreduce_xgmi_rs (prefill chunks)",
           "scaling": "strong"}
    member = rank < tp
    group = dist.new_group(list(range(tp))) if tp < world else None     # every rank calls new_group
    state = {}

    def phase(name, fn):
        err = None
        try:
            if member:
                fn()
        except Exception as e:  # noqa: BLE001 (reported in the JSON line)
            err = f"{name}: {type(e).__name__}: {e}"
        torch.cuda.synchronize()
        ok = torch.tensor([0 if err else 1], device="cuda")
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if err:
            out["error"] = err[:300]
        elif not int(ok.item()):
            out["error"] = f"{name}: failed on another rank"
        return int(ok.item()) == 1

    def make_comm():
        state["comm"] = XgmiComm(group=group)
        t = torch.full((4096,), float(rank + 1), device="cuda")     # rank-dependent values, summed exactly
        state["comm"].all_reduce(t)
        torch.cuda.synchronize()
        if not (int(state["comm"].err.item()) == 0 and bool((t == tp * (tp + 1) / 2).all())):
            raise RuntimeError("xGMI sanity all-reduce gave a wrong sum or timed out")

    def build():
        sd = synthetic.SyntheticStateDict(cfg)
        state["eng"] = engine.PaliGemmaEngine(
            cfg, weights.PackedWeights(cfg, sd.__getitem__, tp_rank=rank, tp_world=tp, fp8=fp8), comm=state["comm"])
        ids, px = synthetic_inputs(cfg, B, PROMPT)
        state["ids"], state["px"] = ids.cuda(), px.cuda()

    def first():
        if sample:
            g = torch.Generator().manual_seed(4321)
            sampler = dict(do_sample=True, temperature=0.8, top_p=0.9, uniforms=torch.rand(T + 1, B, generator=g).cuda())
        else:
            sampler = dict(do_sample=False)
        state["run"] = Runner(state["eng"], state["ids"], state["px"], T, sampler, False, rank)
        state["run"].request()
        torch.cuda.synchronize()
        state["comm"].check()

    def timed():
        run = state["run"]
        g = state["comm"]._dist
        torch.cuda.synchronize()
        g.barrier(group=group)
        t0 = time.perf_counter()
        for _ in range(steps):
            run.request()
        torch.cuda.synchronize()
        g.barrier(group=group)
        el = torch.tensor([time.perf_counter() - t0], device="cuda")
        g.all_reduce(el, op=g.ReduceOp.MAX, group=group)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        run.prefill_run()
        ev[1].record()
        torch.cuda.synchronize()
        pf_ms = ev[0].elapsed_time(ev[1])
        ev[0].record()
        for _ in range(T - 1):
            run.replay()
        ev[1].record()
        torch.cuda.synchronize()
        dec = ev[0].elapsed_time(ev[1]) / (T - 1)
        state["comm"].check()
        L = state["ids"].shape[1]
        out.update(tokens_per_s=round(B * T * steps / el.item(), 2), ms_per_request=round(el.item() / steps * 1e3, 3),
                   prefill_ms=round(pf_ms, 3), decode_ms_per_token=round(dec, 4), decode=run.graph_mode,
                   prefill_tflops=round(prefill_flops(cfg, B, L) / (pf_ms / 1e3) / 1e12, 2))

    for name, fn in (("xgmi setup", make_comm), ("tp engine build", build), ("first request", first),
                     ("timed requests", timed)):
        if not phase(name, fn):
            break
    comm = state.pop("comm", None)
    state.clear()
    if comm is not None:
        try:
            comm.close()
        except Exception:
            pass
    torch.cuda.empty_cache()
    return out


def tp_specs(world):
    """The tensor-parallel legs of a multi-GPU bench run: the headline workload over all N GPUs (the TP curve),
    BASELINE configs[3] (mix-224 = the pt-224 architecture, top-p, TP=2) and configs[4] (pt-896, batch 32, fp8
    Gemma linears, TP=N: TP=8 on the 8-GPU node)."""
    return {
        "tp": dict(tp=world, config="pt-224", batch=1, tokens=128, baseline="BASELINE.json configs[1] workload over "
                   f"{world} GPUs (strong scaling of the per-token latency)"),
        "configs[3]": dict(tp=2, config="mix-224", batch=1, tokens=128, sample=True,
                           baseline="BASELINE.json configs[3]: PaliGemma-3B-mix-224 top-p sampling, Gemma TP=2"),
        "configs[4]": dict(tp=world, config="pt-896", batch=32, tokens=128, fp8=True,
                           baseline=f"BASELINE.json configs[4]: PaliGemma-3B-pt-896 batch 32, fp8 MFMA, TP={world}"
                                    + ("" if world == 8 else " (the config names TP=8)")),
    }


PROMPT = [2, 651, 4906, 603, 476, 2121, 576, 108]


def _launch_ranks(n: int) -> int:
    """`bench.py --gpus N` (N > 1) run without a launcher: the same command as N ranks under
    `python -m torch.distributed.run --nproc-per-node N` on 127.0.0.1, as a CHILD process (the parent has made no HIP
    call and never execs).  Rank 0's JSON line is relayed to stdout; everything else the job prints goes to stderr.
    Returns the job's exit code."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    log(f"[bench] --gpus {n}: launching {n} ranks: {' '.join(cmd)}")
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True)
    relayed = 0
    for line in proc.stdout:
        if line.startswith("{") and '"metric"' in line and not relayed:
            print(line.rstrip("\n"), flush=True)
            relayed += 1
        else:
            sys.stderr.write(line)
    rc = proc.wait()
    if rc == 0 and not relayed:
        log("[bench] the rank job printed no JSON line")
        return 1
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="pt-224")
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--gen-tokens", type=int, default=128)
    ap.add_argument("--parallel", default="dp", choices=["dp", "tp"])
    ap.add_argument("--comm", default="xgmi", choices=["xgmi", "rccl"],
                    help="TP all-reduce: the xGMI peer-store kernels (one-shot for decode-size slabs, reduce-scatter + "
                    "all-gather for prefill chunks; RCCL/gloo beyond their buffers), or the process group's collective only")
    ap.add_argument("--fp8", action="store_true",
                    help="Gemma linears as fp8 e4m3 (per-channel / per-row scales) for GEMMs over 16 rows, as BASELINE "
                    "configs[4]")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--graph-prefill", action="store_true",
                    help="replay the prefill as one hipGraph (measured 0.96-0.97x of eager launches: off by default)")
    ap.add_argument("--no-tp-curve", action="store_true",
                    help="with --gpus N > 1 and --parallel dp: skip the extra tensor-parallel legs (the headline request "
                    "over all N GPUs, BASELINE configs[3] at TP=2 and configs[4] at TP=N), reported beside the "
                    "data-parallel value")
    ap.add_argument("--sample", action="store_true", help="top-p sampling (T=0.8, p=0.9, uniforms seed 4321) "
                    "instead of greedy, as BASELINE configs[3]")
    args = ap.parse_args()

    if args.gpus < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1 (got {args.gpus})")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher around us: start the N ranks as a child torch.distributed.run job (nothing here has touched the
        # GPU yet, and the parent never does), relay rank 0's JSON line and exit with the job's return code
        sys.exit(_launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} from the launcher but --gpus {args.gpus}: they must agree "
                         "(one rank per GPU)")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # PG_BENCH_BACKEND=gloo rehearses the multi-rank code paths with several ranks on one GPU
    backend = os.environ.get("PG_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        from datetime import timedelta
        # a bounded collective timeout: a rank stuck in a collective its peers never issue ends the job with an
        # error after 10 minutes instead of holding the node
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=timedelta(minutes=10))
        else:
            dist.init_process_group(backend, timeout=timedelta(minutes=10))

    from pghip import configs, engine, synthetic, weights
    cfg = configs.CONFIGS[args.config]
    B, T = args.batch, args.gen_tokens
    t0 = time.perf_counter()
    sd = synthetic.SyntheticStateDict(cfg)
    tp = world if args.parallel == "tp" else 1
    if tp > 1:
        from pghip.tp import TPComm, XgmiComm
        comm = XgmiComm() if args.comm == "xgmi" else TPComm()
        eng = engine.PaliGemmaEngine(cfg, weights.PackedWeights(cfg, sd.__getitem__, tp_rank=rank, tp_world=tp,
                                                                fp8=args.fp8), comm=comm)
    else:
        eng = engine.PaliGemmaEngine(cfg, weights.PackedWeights(cfg, sd.__getitem__, fp8=args.fp8))
    torch.cuda.synchronize()
    log(f"[bench] rank {rank}: weights generated+packed in {time.perf_counter() - t0:.1f}s "
        f"({eng.w.nbytes() / 1e9:.2f} GB)")
    ids_cpu, px_cpu = synthetic_inputs(cfg, B, PROMPT)
    ids, px = ids_cpu.cuda(), px_cpu.cuda()
    mask = torch.ones_like(ids)
    L = ids.shape[1]

    # one request = prefill + T-1 graph-replayed decode steps (first token comes from the prefill)
    if args.sample:
        g = torch.Generator().manual_seed(4321)
        sampler = dict(do_sample=True, temperature=0.8, top_p=0.9,
                       uniforms=torch.rand(T + 1, B, generator=g).cuda())
    else:
        sampler = dict(do_sample=False)
    run = Runner(eng, ids, px, T, sampler, args.graph_prefill, rank)
    request, prefill_run, replay, state = run.request, run.prefill_run, run.replay, run.state
    graph_mode, prefill_mode = run.graph_mode, run.prefill_mode

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        request()
    barrier()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        request()
    barrier()
    elapsed = time.perf_counter() - t_start
    if dist is not None:
        tt = torch.tensor([elapsed], device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = tt.item()
    ms_per_step = elapsed / args.steps * 1e3
    tokens = B * T * args.steps * (world // tp)
    value = tokens / elapsed

    # prefill-only and decode-only timings (same stream, events)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    ev[0].record()
    for _ in range(3):
        prefill_run()
    ev[1].record()
    state["st"]["kv_len"].fill_(L)
    state["st"]["pos"].fill_(L + 1)
    state["st"]["step"].zero_()
    ev[2].record()
    for _ in range(T - 1):
        replay()
    ev[3].record()
    torch.cuda.synchronize()
    prefill_ms = ev[0].elapsed_time(ev[1]) / 3
    decode_ms_tok = ev[2].elapsed_time(ev[3]) / (T - 1)
    step_bytes = eng.w.decode_weight_bytes_fp8() if args.fp8 and B > 16 else eng.w.decode_weight_bytes()
    kv_bytes = B * (L + T // 2) * eng.w.t_layers * 2 * eng.w.kv_heads * eng.w.head_dim * 2
    decode_hbm = (step_bytes + kv_bytes) / (decode_ms_tok / 1e3) / 1e9
    pf_flops = prefill_flops(cfg, B, L)
    # roofline time of the prefill: fp8 flops (Gemma linears under --fp8) at the dense fp8 peak, the rest at bf16
    f8 = gemma_linear_flops(cfg, B, L) if args.fp8 and B * L > 16 else 0
    pf_ideal_s = (pf_flops - f8) / (BF16_PEAK_TFS * 1e12) + f8 / (FP8_PEAK_TFS * 1e12)

    kern_s, kern_bytes = time_dominant_kernel(eng)
    achieved = kern_bytes / kern_s / 1e9
    traffic, traffic_src = pmc_traffic()
    kern_desc = f"gemv_kernel<GELU_MUL,2> (decode gate/up, 2x{eng.w.inter}x{eng.w.hidden} bf16)"

    comm_used = eng.comm
    tp_recs = None
    if world > 1 and tp == 1 and not args.no_tp_curve:
        # the data-parallel engine is freed first (the TP legs build their own)
        del state, eng, run, request, prefill_run, replay, sd
        torch.cuda.empty_cache()
        comm_used = None
        tp_recs = {name: tp_leg(spec, rank, world, dist) for name, spec in tp_specs(world).items()}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        del state, eng, run, request, prefill_run, replay
        torch.cuda.empty_cache()
        try:
            cpu = cpu_baseline(cfg, ids_cpu, px_cpu)
        except Exception as e:  # report, do not fail the bench
            cpu = {"value": None, "unit": "tokens/s", "cores": os.cpu_count(), "kind": "port", "sample": f"failed: {e}"}

    baseline_ref = {("pt-224", 1): "BASELINE.json configs[1]", ("pt-448", 16): "BASELINE.json configs[2]"}.get(
        (args.config, B), "not a BASELINE.json config")
    if args.config == "pt-896" and B == 32 and args.fp8:
        baseline_ref = f"BASELINE.json configs[4] shapes (fp8) at {'TP=%d' % tp if tp > 1 else 'one GPU'}"
    if tp == 2 and args.sample and args.config in ("pt-224", "mix-224"):
        baseline_ref = "BASELINE.json configs[3] (mix-224 = the pt-224 architecture)"
    if rank == 0:
        rec = {
            "metric": BASELINE_METRIC,
            "value": round(value, 2), "unit": "tokens/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
            "scaling": "weak" if tp == 1 else "strong", "vs_baseline": None,
            "dtype": "fp8-e4m3 Gemma linears (>16 rows), bf16 elsewhere" if args.fp8 else "bf16", "data": "synthetic (random-init weights of the "
            "PaliGemma-3B architecture, name-seeded; random 224x224 image; 8-token prompt)",
            "config": {"workload": f"PaliGemma-3B-{args.config} image->text, batch {B}, prefill L={L}, "
                                   f"{T} {'top-p' if args.sample else 'greedy'} tokens ({baseline_ref})",
                       "global_batch": B * (world // tp), "seq_len": L + T,
                       "parallelism": f"dp{world}" if tp == 1 else f"tp{tp}-{args.comm}", "decode": graph_mode, "prefill": prefill_mode},
            "prefill_ms": round(prefill_ms, 3),
            "prefill_tflops": round(pf_flops / (prefill_ms / 1e3) / 1e12, 2),
            "prefill_mfma_frac": round(pf_ideal_s / (prefill_ms / 1e3), 4),
            "decode_ms_per_token": round(decode_ms_tok, 4),
            "decode_tok_s": round(B / (decode_ms_tok / 1e3), 1),
            "decode_hbm_gbs": round(decode_hbm, 1),
            "decode_hbm_frac": round(decode_hbm / HBM_PEAK_GBS, 4),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "traffic_source": traffic_src,
                         "kernel": kern_desc,
                         "kernel_avg_us": round(kern_s * 1e6, 2), "bytes_per_launch": kern_bytes},
            "cpu_baseline": cpu,
        }
        if tp_recs is not None:
            rec.update(tp_recs)
        print(json.dumps(rec), flush=True)
    if comm_used is not None and hasattr(comm_used, "check"):
        comm_used.check()                      # a timed-out exchange invalidates the run
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
