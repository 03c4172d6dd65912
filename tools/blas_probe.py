#!/usr/bin/env python3
"""Library-GEMM probe: torch.mm (hipBLASLt / rocBLAS on ROCm) bf16 at the 1x1-conv shapes of IRV1 and
ResNet-50 (M = B * H * W pixels, N = Cout, K = Cin), HIP-event timed, beside our implicit GEMM's per-launch
times from the layer profiles -- decides whether plain 1x1 convs should go to the library."""
import json
import torch

SHAPES = [  # (name, M, N, K)
    ("irv1 block17 down 896->256", 16384, 256, 896), ("irv1 block17 up 256->896", 16384, 896, 256),
    ("irv1 block35 down 256->96", 73984, 96, 256), ("irv1 block35 up 96->256", 73984, 256, 96),
    ("irv1 block8 down 1792->384", 2304, 384, 1792), ("irv1 block8 up 384->1792", 2304, 1792, 384),
    ("r50 l1 1x1 64->64", 802816, 64, 64), ("r50 l1 1x1 64->256", 802816, 256, 64),
    ("r50 l2 1x1 512->128", 200704, 128, 512), ("r50 l3 1x1 1024->256", 50176, 256, 1024),
    ("r50 l4 1x1 2048->512", 12544, 512, 2048),
]
for name, M, N, K in SHAPES:
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        y = a @ w
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        y = a @ w
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "us": round(us, 2),
                      "tflops": round(2.0 * M * N * K / us / 1e6, 1)}), flush=True)
