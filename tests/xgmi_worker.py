"""Rank body of tests/test_tp_gpu.py::test_xgmi_allreduce_ranks_on_one_device (torch.distributed.run, 2 / 4 / 8
ranks on one HIP device; gloo only carries the IPC handles).  Every rank can regenerate every rank's seeded input, so
each checks pg_allreduce_xgmi (one-shot, up to 2^15 elements here) and pg_allreduce_xgmi_rs (reduce-scatter +
all-gather, above) bit-exactly against the fp32 sum in rank order, and times both forms on a 4 MB message."""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "paligemma-multimodal-system_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def rank_data(n, r, it):
    return torch.randn(n, generator=torch.Generator().manual_seed(1000 * it + 17 * r + n))


def expected(n, world, it):
    s = rank_data(n, 0, it)
    for r in range(1, world):
        s = s + rank_data(n, r, it)
    return s


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    from pghip.tp import XgmiComm
    # one-shot up to 2^15 elements, reduce-scatter + all-gather above (the product default switches at 2^18)
    comm = XgmiComm(cap=1 << 20, rs_cap=1 << 21, rs_min=1 << 15)
    bad, dig = [], hashlib.sha256()
    # ragged sizes: one workgroup, partial last chunk, many workgroups, the caps themselves; each twice (both sets)
    sizes = ([4, 1000, 8192, 8196, 2048 * 16, 32772, 257216, 3 * 8192 * 64 + 4, 1 << 20, 1 << 21] if world <= 2 else
             [4, 8196, 2048 * 16, 32772, 65540 + 8 * 1024 * 3, 1 << 20])
    for it, n in enumerate(sizes * 2):
        t = rank_data(n, rank, it).cuda()
        comm.all_reduce(t)
        got = t.cpu()
        if not torch.equal(got, expected(n, world, it)):
            bad.append([n, it, float((got - expected(n, world, it)).abs().max())])
        dig.update(got.numpy().tobytes())
    # back to back without a host sync: one-chunk, multi-chunk-per-workgroup and cap-sized exchanges
    # interleaved, so a workgroup that reused a buffer set early would corrupt a peer's unread slots
    seq = [2048, 600000, 4, 1 << 20, 2048, 524292, 8196, 1 << 20, 1 << 21, 40000, 4, 1 << 21]
    ins = [rank_data(n, rank, 200 + i).cuda() for i, n in enumerate(seq)]
    torch.cuda.synchronize()
    dist.barrier()
    for t in ins:
        comm.all_reduce(t)
    torch.cuda.synchronize()
    seq_bad = [[n, i] for i, (n, t) in enumerate(zip(seq, ins)) if not torch.equal(t.cpu(), expected(n, world, 200 + i))]
    # split-K slabs summed on the way in (slab order, then rank order), both forms
    for it, n in enumerate([8192, 300004]):
        ns = 3
        part = torch.stack([rank_data(n, rank, 500 + 10 * it + s_) for s_ in range(ns)]).cuda()
        comm.all_reduce_slabs(part, ns)
        want = None
        for r in range(world):
            c = rank_data(n, r, 500 + 10 * it)
            for s_ in range(1, ns):
                c = c + rank_data(n, r, 500 + 10 * it + s_)
            want = c if want is None else want + c
        if not torch.equal(part[0].cpu(), want):
            seq_bad.append(["slabs", n])
    # all-gather in rank order (pg_allgather_xgmi), interleaved with all-reduces on the same buffer / epochs
    gather_bad = []
    for it, n in enumerate([4, 2048, 32160, 8196, 1 << 20 if world <= 2 else 1 << 18]):
        t = rank_data(n, rank, 300 + it).cuda()
        out = torch.empty(world * n, device="cuda")
        comm.all_gather(out, t)
        r = rank_data(8, rank, 400 + it).cuda()
        comm.all_reduce(r)
        want = torch.cat([rank_data(n, q, 300 + it) for q in range(world)])
        if not torch.equal(out.cpu(), want) or not torch.equal(r.cpu(), expected(8, world, 400 + it)):
            gather_bad.append(n)
    # captured: three exchanges of different sizes in one graph, replayed with fresh inputs
    sizes = [2048, 2048 * 16, 4 * 8192, 131076]
    static = [torch.zeros(n, device="cuda") for n in sizes]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for t in static:
                comm.all_reduce(t)
    graph_bad = []
    for rep in range(4):
        it = 100 + rep
        for t, n in zip(static, sizes):
            t.copy_(rank_data(n, rank, it))
        torch.cuda.synchronize()
        dist.barrier()
        g.replay()
        torch.cuda.synchronize()
        for t, n in zip(static, sizes):
            if not torch.equal(t.cpu(), expected(n, world, it)):
                graph_bad.append([n, rep])
    # timing of a 4 MB message (a 512-row prefill chunk) in both forms, ranks sharing this one device (no xGMI link is
    # crossed here: the numbers bound the kernels' own cost, not the link rate)
    timing = {}
    t = torch.ones(1 << 20, device="cuda")
    for form, rs_min in (("rs", comm.rs_min), ("oneshot", 1 << 30)):
        saved, comm.rs_min = comm.rs_min, rs_min
        ts = []
        for _ in range(6):
            torch.cuda.synchronize()
            dist.barrier()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            comm.all_reduce(t)
            ev[1].record()
            torch.cuda.synchronize()
            ts.append(ev[0].elapsed_time(ev[1]) * 1e3)
        comm.rs_min = saved
        timing[f"{form}_4MB_us"] = sorted(ts[1:])[len(ts[1:]) // 2]
    out = {"rank": rank, "err": int(comm.err.item()), "diag": comm.diagnostics(), "bad": bad, "graph_bad": graph_bad,
           "seq_bad": seq_bad, "gather_bad": gather_bad, "rs_calls": comm.rs_calls, "rs_wg": comm.rs_wg,
           "ranks_per_device": comm.ranks_per_device, "timing": timing,
           "digest": dig.hexdigest()}
    del g
    comm.close()
    with open(os.path.join(os.environ["TP_OUT"], f"rank{rank}.json"), "w") as f:
        json.dump(out, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
