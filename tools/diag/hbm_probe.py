"""Streaming read bandwidth of an 8.6 GB buffer (the filter's G halves at batch 128)."""
import ctypes, os, sys, time
import torch
here = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(here, "..", "..", "build_diag", "libhbm_probe.so"))
dev = "cuda:0"
n = 128 * 4096 * 4096 * 4  # bytes: Gh + Gl for 128 matrices
buf = torch.empty(n, dtype=torch.uint8, device=dev)
buf.random_(0, 255)
out = torch.zeros(4, dtype=torch.int32, device=dev)
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
for grid in (1024, 2048, 4096, 8192, 16384):
    lib.hbm_probe(ctypes.c_void_p(buf.data_ptr()), ctypes.c_int64(n), ctypes.c_void_p(out.data_ptr()), grid, s)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        lib.hbm_probe(ctypes.c_void_p(buf.data_ptr()), ctypes.c_int64(n), ctypes.c_void_p(out.data_ptr()), grid, s)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 5
    print(f"grid {grid:6d}: {n / dt / 1e12:.2f} TB/s ({dt * 1e3:.2f} ms for {n / 1e9:.1f} GB)")
