"""Tensor-parallel engine on the HIP device: 2, 4 or 8 ranks share one MI355X over the gloo transport or the xGMI
exchange (RCCL refuses two ranks on one GPU; the 8-GPU RCCL run is the driver's scaling bench).  Checks the
sharded kernels, the partial-sum all-reduces and the vocabulary-parallel greedy / top-p paths
against the reference's golden vectors and the single-rank engine.  Tolerance as
tests/test_engine_gpu.py (scaled max error < 3e-2 vs the fp32 reference); TP vs single-rank
differs only by the fp32 summation order of partials (< 5e-3)."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _launch(worker, tmp_path, nproc=2, timeout=600, **env):
    # ranks sharing ONE device: at most 2 hardware queues per rank (TP_HW_QUEUES), so the 8 ranks' queues -- and this
    # pytest process's own, which holds a context from the earlier tests -- all stay mapped at once.  An oversubscribed
    # queue set is time-sliced, and a rank whose queue is not mapped cannot reach an exchange its peers spin in (an
    # occasional 20 s xGMI timeout at 8 ranks x 4 queues in round 5; DESIGN §6 has the analysis).  A real node has a
    # device per rank, at most 4 queues each.
    env = dict(os.environ, TP_OUT=str(tmp_path), GPU_MAX_HW_QUEUES=os.environ.get("TP_HW_QUEUES", "2"), **env)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "tests", worker)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return [json.load(open(tmp_path / f"rank{i}.json")) for i in range(nproc)]


@pytest.mark.parametrize("world", [2, 4, 8])
def test_xgmi_allreduce_ranks_on_one_device(tmp_path, world):
    """pg_allreduce_xgmi / pg_allgather_xgmi / pg_allreduce_xgmi_rs between `world` processes sharing the device
    through IPC-mapped exchange buffers (the 8-rank case is the TP=8 exchange of BASELINE configs[4]): bit-exact
    against the rank-order fp32 sum / concatenation for ragged sizes (one and many workgroups, both buffer sets, the
    one-shot and the reduce-scatter + all-gather form), back to back with different sizes and forms and no host sync,
    split-K slabs summed on the way in, all-gathers interleaved with all-reduces, identical on every rank, inside a
    captured hipGraph, and without a timeout.  Prints both forms' time for a 4 MB message on this shared device."""
    if not torch.cuda.is_available():
        pytest.skip("needs the HIP device")
    res = _launch("xgmi_worker.py", tmp_path, nproc=world)
    print(json.dumps({"world": world, "timing": res[0]["timing"], "rs_wg": res[0]["rs_wg"]}))
    for o in res:
        assert o["err"] == 0, o
        assert o["ranks_per_device"] == world and o["rs_wg"] == max(8, 256 // world), o
        assert o["rs_calls"] > 0, o
        assert o["bad"] == [], o
        assert o["graph_bad"] == [], o
        assert o["seq_bad"] == [], o
        assert o["gather_bad"] == [], o
    assert len({o["digest"] for o in res}) == 1


# (config, ranks, transport, prefill chunk rows, fp8): TP 2 on tiny (4 q heads); TP 4 / 8 on tiny8 (8 q heads: one per
# rank at TP 8, the split of BASELINE configs[4]); chunk rows 8 make every prefill o_proj / down_proj run as row chunks
# whose all-reduces are issued asynchronously (xGMI side stream / async gloo) while the next chunk's GEMM runs.
TP_CASES = [("tiny", 2, "gloo", None, False), ("tiny", 2, "xgmi", None, False),
            ("tiny8", 4, "xgmi", 8, False), ("tiny8", 8, "xgmi", None, False), ("tiny8", 8, "gloo", 8, False),
            ("tiny8", 8, "xgmi", 8, True)]


@pytest.mark.parametrize("cfg,world,comm,chunk,fp8", TP_CASES, ids=lambda v: str(v))
def test_tp_engine_on_one_device(tmp_path, cfg, world, comm, chunk, fp8):
    """The tensor-parallel engine with `world` ranks sharing the device, against the reference's goldens (prefill
    logits of every golden batch: B = 8 at TP 8 runs the SigLIP tower data-parallel, one image per rank; the 12
    greedy ids of the reference's own loop) and the single-rank engine (prefill, 19 teacher-forced decode steps,
    top-p draws with the same uniforms).  fp8: every linear of more than 16 rows on the fp8 MFMA, TP and single rank
    each within the fp8 bound of the fp32 references (they quantise different weight slices), plus a 24-row
    teacher-forced decode (the fp8 decode path) against the oracle."""
    if not torch.cuda.is_available():
        pytest.skip("needs the HIP device")
    env = dict(TP_COMM=comm, TP_CFG=cfg)
    if chunk:
        env["TP_CHUNK"] = str(chunk)
    if fp8:
        env["TP_FP8"] = "1"
    res = _launch("tp_worker.py", tmp_path, nproc=world, **env)
    print(json.dumps(res[0]))
    for o in res:
        assert o["xgmi_err"] == 0, o
        assert o["graph"] == (comm == "xgmi"), o
        assert o["world"] == world and (chunk is None or o["chunk_rows"] == chunk), o
        # vs the fp32 reference: within 1.5x the model's intrinsic sensitivity to the path's operand rounding (the
        # oracle run with bf16 operands, and e4m3 Gemma linears for fp8), as the full-size tests bound it
        pre = [int(k[len("prefill_err_b"):]) for k in o if k.startswith("prefill_err_b")]
        assert pre and all(o[f"prefill_err_b{B}"] < 1.5 * o[f"intrinsic_b{B}"] for B in pre), o
        # vs the single-rank engine: other fp32 summation orders of the rank partials (bf16); fp8 ranks quantise
        # other weight slices (o / down rows over a K slice get their own scales), so the fp8 bound applies
        for B in pre:
            assert o[f"prefill_err_vs_solo_b{B}"] < (1.5 * o[f"intrinsic_b{B}"] if fp8 else 5e-3), (B, o)
        # the data-parallel SigLIP slice takes the whole batch's split choices: bit-identical features once a rank's
        # slice is a tile GEMM (> 16 rows; a slice of <= 16 rows runs the decode GEMV, another summation order)
        assert all(o[f"vision_dp_bitexact_b{B}"] for B in o["vision_dp"] if B // world * 16 > 16), o
        if cfg == "tiny8" and world == 8:
            assert 16 in o["vision_dp"], o            # two images per rank through the data-parallel SigLIP
        tol = 1.5 * max(o[f"intrinsic_b{B}"] for B in pre)
        if fp8:
            assert o["decode_slice_err"] < tol, o
            assert o["fp8_decode24_err"] < 1.5 * o["fp8_decode24_intrinsic"], o
        else:
            assert o["greedy"] == o["greedy_ref"], o
            assert o["decode_slice_err"] < 0.5 * o["intrinsic_b1"], o      # fp32 order, bf16-amplified
            assert o["decode_argmax_agree"], o
            assert o["sampled_tp"] == o["sampled_solo"], o
    assert all(o["greedy"] == res[0]["greedy"] and o["sampled_tp"] == res[0]["sampled_tp"] for o in res)


def _check_896(res, min_checked):
    """Verdicts of tp_worker.full_size_896 (BASELINE configs[4]): bounded by the fp32 oracle run on the same e4m3 /
    bf16 operand rounding (tests/golden/make_emu.py), not a flat percentage.  The sharded run is bounded by the
    emulation of the SHARDED form (<golden>_fp8emu_tp8.npz: the row-parallel o_proj / down_proj quantised per rank on
    their K slices and summed in rank order, make_emu.py --tp 8); the single-rank engine by the single-rank emulation
    (<golden>_fp8emu.npz).  Both at 1.5x, on every row of every block."""
    for o in res:
        assert o["xgmi_err"] == 0 and o["vision_dp"], o
        assert o["emu_tp_fixture"] and o["rows_checked"] == o["B"], o
        assert o["fallbacks"] == 0, o                  # every collective went through the xGMI kernels
        assert o["rs_calls"] > 0 and o["chunk_allreduce_ok"], o   # prefill chunks on the reduce-scatter + all-gather
        assert o["emu_ratio"] < 1.5, o                 # reference top-64 within 1.5x the emulated TP e4m3 distance
        assert o["top64_rel"] < 0.3, o                 # and within 30% of the top-64 scale (non-vacuous at any margin)
        assert o["top1_bad"] == [] and o["top1_checked"] >= min_checked, o
        assert o["row_spread"] < 2e-2, o               # rows of one request agree
    r0 = res[0]
    assert r0["solo_emu_ratio"] < 1.5 and r0["solo_top1_bad"] == [], r0
    assert r0["vs_solo_emu_ratio"] < 3.0 and r0["vs_solo_top1_agree"], r0
    assert all(o["top1"] == r0["top1"] for o in res)


@pytest.mark.slow
def test_tp8_pt896_fp8_batch32(tmp_path):
    """BASELINE configs[4] at its own shape: PaliGemma-3B-pt-896, batch 32, fp8 Gemma linears, TP=8 (one q head, 2048
    gate/up columns, a 2048-row down slice and 32,152 vocabulary rows per rank; modeling_gemma.py:205-218, 255-259,
    356, 523), eight ranks on one device over the xGMI kernels (cap 2^23: every 4096-row prefill chunk runs as the
    reduce-scatter + all-gather, every decode message as the one-shot exchange; nothing travels over the process
    group).  The better-conditioned recipe's two images, 16 rows each (4 images per rank through the data-parallel
    SigLIP), prefill plus 15 teacher-forced decode steps on the sharded 17..32-row fp8 GEMVs and the fp8
    vocabulary-slice lm_head: every row within 1.5x the emulated TP e4m3 distance of the reference's top-64 logits, the
    reference's top-1 wherever its margin exceeds twice the step's distance, and against the single-rank fp8 engine."""
    if not torch.cuda.is_available():
        pytest.skip("needs the HIP device")
    res = _launch("tp_worker.py", tmp_path, nproc=8, timeout=1100, TP_COMM="xgmi", TP_CFG="pt-896", TP_B="32",
                  TP_GOLDEN="pt896wc")
    print(json.dumps({k: v for k, v in res[0].items() if k != "top1"}))
    assert all(o["B"] == 32 and o["cap"] == 1 << 23 for o in res)
    _check_896(res, min_checked=40)


@pytest.mark.slow
def test_tp8_pt896_fp8_batch8(tmp_path):
    """The default recipe's pt-896 request (tests/golden/pt896.npz, 3 steps) at TP=8, batch 8 (one image per rank):
    the same emulation-derived bounds as the batch-32 test.  Its top1-top2 margins (0.03-0.20) lie below the e4m3
    error, so few steps reach the top-1 check; the 30% top-64 bound keeps the test from passing on bounds alone."""
    if not torch.cuda.is_available():
        pytest.skip("needs the HIP device")
    res = _launch("tp_worker.py", tmp_path, nproc=8, timeout=1100, TP_COMM="xgmi", TP_CFG="pt-896", TP_B="8",
                  TP_GOLDEN="pt896")
    print(json.dumps({k: v for k, v in res[0].items() if k != "top1"}))
    _check_896(res, min_checked=0)


@pytest.mark.slow
def test_bench_gpus2_launches_two_ranks():
    """`python bench.py --gpus 2` with no launcher around it (the driver's N > 1 command line) starts two ranks as a
    torch.distributed.run child and relays rank 0's line: n_gpus 2, the data-parallel value, and the tensor-parallel
    legs (the headline request at TP=2, configs[3] top-p at TP=2, configs[4] pt-896 x32 fp8 at TP=2), none failed.
    The two ranks share this one device over gloo (PG_BENCH_BACKEND=gloo); on the 8-GPU node the backend is RCCL."""
    if not torch.cuda.is_available():
        pytest.skip("needs the HIP device")
    env = dict(os.environ, PG_BENCH_BACKEND="gloo", GPU_MAX_HW_QUEUES="2")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0"],
                       env=env, capture_output=True, text=True, timeout=1100)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout[-2000:]
    rec = json.loads(lines[0])
    print(json.dumps(rec))
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2" and rec["config"]["global_batch"] == 2, rec
    assert rec["value"] > 0 and rec["scaling"] == "weak", rec
    for leg, tp in (("tp", 2), ("configs[3]", 2), ("configs[4]", 2)):
        assert leg in rec and "error" not in rec[leg], rec.get(leg)
        assert rec[leg]["tp"] == tp and rec[leg]["tokens_per_s"] > 0, rec[leg]
    assert rec["configs[4]"]["fp8"] and rec["configs[4]"]["batch"] == 32
    assert rec["configs[3]"]["sampler"].startswith("top-p")


@pytest.mark.slow
@pytest.mark.parametrize("comm", ["gloo", "xgmi"])
def test_tp2_full_size_pt224(tmp_path, comm):
    """Full-size PaliGemma-3B-224 at TP=2 (BASELINE configs[3]: mix-224 top-p, which has the pt-224 architecture),
    two ranks on one device, on the pt224wc recipe.  Against the single-rank engine: prefill and every teacher-forced
    decode step's gathered logits < 2e-2 scaled (the rank-partitioned partial sums are added in another fp32 order,
    which the synthetic init amplifies through 18 layers: measured 1.1e-2 on the default recipe), the same top-1
    wherever the single-rank margin exceeds 0.05, every top-p draw equal to the oracle's explicit-uniform inverse
    CDF of the TP logits (and the first free-running draw with fixed uniforms; later free-running draws are not
    compared with the single-rank engine, see tp_worker.full_size).  Against the reference: the 32 free-running
    greedy ids of tests/golden/pt224wc.npz image 0, exactly."""
    if not torch.cuda.is_available():
        pytest.skip("needs the HIP device")
    res = _launch("tp_worker.py", tmp_path, timeout=900, TP_COMM=comm, TP_CFG="pt-224")
    for o in res:
        assert o["xgmi_err"] == 0, o
        assert o["prefill_err_vs_solo"] < 2e-2, o
        assert o["prefill_top1"] == o["ref_top1"], o
        assert o["decode_err_vs_solo"] < 2e-2, o
        assert o["decode_disagree"] == [], o
        assert o["greedy_tp"] == o["greedy_ref"], o
        assert o["sampled_first_ok"], o
    assert res[0]["greedy_tp"] == res[1]["greedy_tp"] and res[0]["sampled_tp"] == res[1]["sampled_tp"]
