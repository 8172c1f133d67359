#!/usr/bin/env python3
"""Reference point only (not a product path): the vendor library's f16 GEMM rate (torch.matmul
-> hipBLASLt) on the encoder's large-v3 shapes, to size the headroom of the hand-written MFMA
GEMMs (tools/gemm_bench.cpp measures those on the same shapes)."""
import torch

torch.backends.cuda.matmul.allow_fp16_reduced_precision_reduction = False
for M in (6000, 12000):
    for name, N, K in (("qkv", 3840, 1280), ("o", 1280, 1280), ("fc1", 5120, 1280), ("fc2", 1280, 5120),
                       ("xkv", 81920, 1280)):
        a = torch.randn(M, K, device="cuda", dtype=torch.float16)
        w = torch.randn(N, K, device="cuda", dtype=torch.float16)
        for _ in range(3):
            torch.matmul(a, w.t())
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        it = 20
        e0.record()
        for _ in range(it):
            torch.matmul(a, w.t())
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / it
        print("%-4s M=%5d N=%5d K=%4d  %8.1f us  %7.1f TFLOP/s" % (name, M, N, K, us, 2.0 * M * N * K / us / 1e6),
              flush=True)
