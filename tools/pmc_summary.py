"""Per-launch HBM bytes per kernel from the rocprofv3 --pmc passes of tools/gpu_pmc.sh.

Usage: python tools/pmc_summary.py gpurun_out/pmc  > summary.json
FETCH_SIZE / WRITE_SIZE are in KiB per dispatch; on gfx950 FETCH_SIZE counts half the bytes of a wide
streaming read (MI355X_MICROARCH.md, HBM section), so fetch bytes = 2 x 1024 x FETCH_SIZE.  The
"gate_up" entry is the MLP gate|up GEMM (the SwiGLU-epilogue GEMM, EPI 4); "attention" the f8c attention kernels
(attn_kh_kernel instances -- full layers -- and attn2_kernel<..., F8 = true> ones -- sliding / cross), launch-weighted.  "build" is
acestep_mi355x.source_hash() of the tree the passes ran: bench.py uses the bytes only when its own tree has the same
hash (and the same workload), so a changed kernel never reports stale traffic.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def read_counter(root, name):
    per_kernel = defaultdict(list)
    for path in glob.glob(os.path.join(root, name, "**", "*counter_collection.csv"), recursive=True):
        with open(path, newline="") as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != name:
                    continue
                per_kernel[row.get("Kernel_Name", "?")].append(float(row["Counter_Value"]))
    return per_kernel


def main(root, bench_json=None):
    fetch = read_counter(root, "FETCH_SIZE")
    write = read_counter(root, "WRITE_SIZE")
    out = {"unit": "bytes per launch", "fetch_correction": 2.0, "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [])
        w = write.get(k, [])
        fb = 2.0 * 1024.0 * sum(f) / len(f) if f else None
        wb = 1024.0 * sum(w) / len(w) if w else None
        out["kernels"][k] = {"fetch_bytes": fb, "write_bytes": wb, "launches": max(len(f), len(w)),
                             "hbm_bytes": (fb or 0.0) + (wb or 0.0)}
    pat = re.compile(r"gemm_kernel<\d+, \d+, \d+, \d+, (?:true|false), 4, \d+[,>]|gemm_q_kernel<\d+, \d+, \d+, \d+, 4, \d+[,>]")
    gu = [k for k in out["kernels"] if pat.search(k)]
    if gu:
        out["gate_up"] = {"kernel": gu[0], **out["kernels"][gu[0]]}
    att = [k for k in out["kernels"] if "attn_kh_kernel" in k
           or ("attn2_kernel" in k and k.replace(" ", "").endswith("1,true>(acemi::AttnArgs)"))]
    if att:
        n = sum(out["kernels"][k]["launches"] for k in att)
        out["attention"] = {"kernels": att, "launches": n,
                            "hbm_bytes": sum(out["kernels"][k]["hbm_bytes"] * out["kernels"][k]["launches"]
                                             for k in att) / max(n, 1)}
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ace-step-1.5-ggml_amd"))
    from acestep_mi355x import source_hash
    out["build"] = source_hash()
    if bench_json:  # the workload these passes ran (bench.py matches it before using the bytes)
        with open(bench_json, "r", encoding="utf-8") as f:
            line = [ln for ln in f if ln.startswith("{")][-1]
        c = json.loads(line)["config"]
        out["config"] = {k: c[k] for k in ("latent_frames", "enc_len", "batch_per_gpu", "weights")}
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc", sys.argv[2] if len(sys.argv) > 2 else None)
