"""Standalone weight-gradient launch for profiling (rocprofv3 PMC / kernel stats): nerf_wgrad on
the training step's hidden-layer shape (262,144 samples x 256 x 256, rows of the gradient and
activation buffers as in the training workspace), ITERS launches."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nerfmi import _lib as L  # noqa: E402

M = 262144
N = int(os.environ.get("N", "256"))   # 1: density head, 3: rgb head, 128: dir layer
K = int(os.environ.get("K", "256"))   # 63: layer 0 / the skip layer's PE columns
ITERS = int(os.environ.get("ITERS", "20"))
lib, dev = L.load(), L.device()
g = torch.Generator(device=dev).manual_seed(0)
LDA = int(os.environ.get("LDA", L.GRAD_ROW))   # row strides (floats): the training workspace's by default
LDX = int(os.environ.get("LDX", L.SAVE_ROW))
a = torch.randn(M, LDA, device=dev, generator=g)
x = torch.randn(M, LDX, device=dev, generator=g)
ow, ob = torch.empty(N, K, device=dev), torch.empty(N, device=dev)
ws = torch.empty(lib.nerf_wgrad_workspace_bytes(M, N, K), dtype=torch.uint8, device=dev)
for i in range(ITERS + 2):
    if i == 2:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
    L.check(lib.nerf_wgrad(L.ptr(a), LDA, N, L.ptr(x), LDX, K, 1, M, L.ptr(ow), L.ptr(ob), 0, L.ptr(ws),
                           ws.numel(), L.stream()), "wgrad")
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / ITERS
print(f"wgrad {M}x{N}x{K}: {dt * 1e3:.3f} ms/launch, {2 * M * N * (K + 1) / dt / 1e12:.1f} TFLOP/s")
