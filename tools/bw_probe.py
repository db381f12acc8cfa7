"""Streaming-copy bandwidth on zero vs random data, in and beyond the 256 MiB
Infinity Cache (torch copy_ kernels, HIP events).  Diagnostic for the
data-dependent Jacobi timing."""
import json

import torch

dev = torch.device("cuda:0")


def bw(n_bytes, fill, reps=50):
    n = n_bytes // 4
    src = torch.empty(n, dtype=torch.float32, device=dev)
    if fill == "zero":
        src.zero_()
    elif fill == "random":
        src.uniform_(-1.0, 1.0)
    elif fill == "sparse":        # 3 % nonzero
        src.uniform_(-1.0, 1.0)
        src[torch.rand(n, device=dev) > 0.03] = 0.0
    dst = torch.empty_like(src)
    for _ in range(5):
        dst.copy_(src)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        dst.copy_(src)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    return 2 * n * 4 / (ms * 1e-3) / 1e9


for size_mb in (64, 1024, 4096):
    for fill in ("zero", "random", "sparse"):
        print(json.dumps({"bytes_per_buffer_MiB": size_mb, "fill": fill,
                          "copy_GBps": round(bw(size_mb << 20, fill), 1)}), flush=True)
# random, then zero again (order effects)
print(json.dumps({"bytes_per_buffer_MiB": 1024, "fill": "zero(again)",
                  "copy_GBps": round(bw(1 << 30, "zero"), 1)}), flush=True)
