"""Tensor-parallel engine on the HIP device: two ranks share one MI355X over the gloo transport
(RCCL refuses two ranks on one GPU; the 8-GPU RCCL run is the driver's scaling bench).  Checks the
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
    env = dict(os.environ, TP_OUT=str(tmp_path), **env)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "tests", worker)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return [json.load(open(tmp_path / f"rank{i}.json")) for i in range(nproc)]


@pytest.mark.parametrize("world", [2, 4, 8])
def test_xgmi_allreduce_ranks_on_one_device(tmp_path, world):
    """pg_allreduce_xgmi / pg_allgather_xgmi between `world` processes sharing the device through IPC-mapped
    exchange buffers (the 8-rank case is the TP=8 exchange of BASELINE configs[4]): bit-exact against the
    rank-order fp32 sum / concatenation for ragged sizes (one and many workgroups, both buffer sets), back to
    back with different sizes and no host sync, all-gathers interleaved with all-reduces, identical on every
    rank, inside a captured hipGraph, and without a timeout."""
    if not torch.cuda.is_available():
        pytest.skip("needs the HIP device")
    res = _launch("xgmi_worker.py", tmp_path, nproc=world)
    for o in res:
        assert o["err"] == 0, o
        assert o["bad"] == [], o
        assert o["graph_bad"] == [], o
        assert o["seq_bad"] == [], o
        assert o["gather_bad"] == [], o
    assert len({o["digest"] for o in res}) == 1


@pytest.mark.parametrize("comm", ["gloo", "xgmi"])
def test_tp2_engine_on_one_device(tmp_path, comm):
    if not torch.cuda.is_available():
        pytest.skip("needs the HIP device")
    res = _launch("tp_worker.py", tmp_path, TP_COMM=comm)
    for o in res:
        assert o["xgmi_err"] == 0, o
        assert o["graph"] == (comm == "xgmi"), o
        assert o["prefill_err_b1"] < 3e-2 and o["prefill_err_b2"] < 3e-2, o
        assert o["greedy"] == o["greedy_ref"], o
        assert o["decode_slice_err"] < 5e-3, o
        assert o["decode_argmax_agree"], o
        assert o["sampled_tp"] == o["sampled_solo"], o
    assert res[0]["greedy"] == res[1]["greedy"] and res[0]["sampled_tp"] == res[1]["sampled_tp"]


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
