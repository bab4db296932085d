import json, os, sys
ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path.insert(0, os.path.join(ROOT, "ace-step-1.5-ggml_amd"))
from acestep_mi355x import capi
M, N, K = 3000, 4096, 2048
for v in (4, 7, 16, 2, 5):
    row = {"shape": "qkv 240s plain", "variant": v}
    for epi in (0, 1):
        ms = capi.bench_gemm(M, N, K, variant=v, epi=epi, iters=20)
        row[f"epi{epi}_us"] = round(ms * 1e3, 1)
        row[f"epi{epi}_tf"] = round(2.0 * M * N * K / (ms / 1e3) / 1e12, 1)
    print(json.dumps(row), flush=True)
