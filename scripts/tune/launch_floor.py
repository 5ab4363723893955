import ctypes as C, os, torch
lib = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "launch_floor.so"))
lib.launch_tiny.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p]
p = torch.zeros(16, device="cuda")
N = 200
for grid in (1, 256, 2048):
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(20): lib.launch_tiny(p.data_ptr(), grid, 256, s)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(N): lib.launch_tiny(p.data_ptr(), grid, 256, s)
    e1.record(); torch.cuda.synchronize()
    eager = e0.elapsed_time(e1) / N * 1e3
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(N): lib.launch_tiny(p.data_ptr(), grid, 256, torch.cuda.current_stream().cuda_stream)
    g.replay(); torch.cuda.synchronize()
    e0.record()
    for _ in range(5): g.replay()
    e1.record(); torch.cuda.synchronize()
    graph = e0.elapsed_time(e1) / (5 * N) * 1e3
    print(f"grid {grid:5d}: eager {eager:6.2f} us/launch   graph {graph:6.2f} us/launch")
