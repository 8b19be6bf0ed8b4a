"""Sustained dense f16 / bf16 GEMM rate of the vendor library (torch.matmul -> hipBLASLt) on this
MI355X, as an independent check of the power-limited MFMA ceiling that DESIGN.md §4 measures with
scripts/microbench/mfma_shape_side.hip.  Each shape runs back to back for >= SECONDS of wall time
(long enough for the clock to settle under the power limit); random N(0,1) operands.

    python scripts/microbench/gemm_f16_ceiling.py        # prints one line per (dtype, shape)
"""
import os
import time

import torch

SECONDS = float(os.environ.get("SECONDS_PER_SHAPE", "3"))
PEAK = {torch.float16: 2516.8, torch.bfloat16: 2516.8}   # MI355X dense f16/bf16 MFMA TFLOP/s


def run(dtype, m, n, k):
    g = torch.Generator(device="cuda").manual_seed(0)
    a = torch.randn(m, k, device="cuda", dtype=dtype, generator=g)
    b = torch.randn(k, n, device="cuda", dtype=dtype, generator=g)
    c = torch.empty(m, n, device="cuda", dtype=dtype)
    for _ in range(3):
        torch.matmul(a, b, out=c)
    torch.cuda.synchronize()
    iters, t0 = 0, time.perf_counter()
    while True:
        for _ in range(10):
            torch.matmul(a, b, out=c)
        iters += 10
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if dt >= SECONDS:
            break
    tf = 2.0 * m * n * k * iters / dt / 1e12
    print(f"{str(dtype).split('.')[-1]:9s} {m}x{n}x{k}: {tf:7.1f} TFLOP/s sustained over {dt:.1f} s "
          f"= {tf / PEAK[dtype]:.3f} of the dense peak", flush=True)


if __name__ == "__main__":
    print(torch.cuda.get_device_name(0), flush=True)
    for dtype in (torch.float16, torch.bfloat16):
        for shape in ((8192, 8192, 8192), (16384, 16384, 8192), (4096, 4096, 16384)):
            run(dtype, *shape)
