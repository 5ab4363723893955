"""Grid-barrier cost (scripts/tune/grid_barrier.hip): us per barrier round for 256 / 512 co-resident workgroups,
with 0 / 1 / 4 KiB stored per workgroup before each barrier and read by the neighbour after it; against the cost
of a kernel boundary (a graph of dependent empty launches).

    hipcc --offload-arch=gfx950 -O3 -fPIC -shared scripts/tune/grid_barrier.hip -o scripts/tune/lib/grid_barrier.so
    python scripts/tune/grid_barrier.py
"""
import ctypes as C
import os

import torch

lib = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "grid_barrier.so"))
lib.gb_run.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
err = torch.zeros(1, dtype=torch.int32, device="cuda")
buf = torch.zeros(512 * 1024, device="cuda")
for nwg in (256, 512):
    for words in (0, 256, 1024):
        cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
        s = torch.cuda.current_stream().cuda_stream
        lib.gb_run(cnt.data_ptr(), nwg, 10, buf.data_ptr(), words, err.data_ptr(), s)
        torch.cuda.synchronize()
        res = []
        for iters in (10, 210):
            cnt.zero_()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            lib.gb_run(cnt.data_ptr(), nwg, iters, buf.data_ptr(), words, err.data_ptr(), s)
            e1.record()
            torch.cuda.synchronize()
            res.append(e0.elapsed_time(e1) * 1e3)
        per = (res[1] - res[0]) / 200
        print(f"nwg {nwg:4d} words {words:5d}: {per:6.2f} us per barrier round (launch of 10 rounds {res[0]:.1f} us)"
              f"  err={int(err.item())}", flush=True)
        if int(err.item()):
            raise SystemExit("a barrier timed out")
