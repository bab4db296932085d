import json, os, sys
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "ace-step-1.5-ggml_amd"))
from acestep_mi355x import capi
for name, M, N, K, epi in [("gate_up 60s", 750, 12288, 2048, 4), ("qkv 60s", 750, 4096, 2048, 0),
                           ("o 60s", 750, 2048, 2048, 2), ("cross_q 60s", 750, 2048, 2048, 0),
                           ("down 60s", 750, 2048, 6144, 2)]:
    row = {"shape": name}
    for v in (1, 4, 6, 7, 8, 9):
        ms = capi.bench_gemm(M, N, K, variant=v, epi=epi, iters=50)
        row[f"v{v}"] = round(2.0 * M * N * K / (ms / 1e3) / 1e12, 1)
    print(json.dumps(row), flush=True)
