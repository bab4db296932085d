"""hipBLASLt (torch.matmul, bf16) TFLOP/s at the engine's GEMM shapes: the library bar the hand-written
GEMM is compared against (measurement only; the product path never calls it)."""
import json

import torch

SHAPES = [("gate_up 240s", 3000, 12288, 2048), ("down 240s", 3000, 2048, 6144), ("qkv 240s", 3000, 4096, 2048),
          ("o/cross 240s", 3000, 2048, 2048), ("gate_up bs8", 24000, 12288, 2048), ("square 4096", 4096, 4096, 4096),
          ("square 8192", 8192, 8192, 8192)]
for name, M, N, K in SHAPES:
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        c = a @ w.t()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    it = 20
    e0.record()
    for _ in range(it):
        c = a @ w.t()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / it
    print(json.dumps({"shape": name, "MNK": [M, N, K], "torch_bf16_tflops": round(2.0 * M * N * K / ms / 1e9, 1)}),
          flush=True)
