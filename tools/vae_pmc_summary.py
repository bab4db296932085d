"""Per-stage HBM bytes of the 240 s VAE decode from the counter passes of tools/gpu_vae_pmc.sh, beside the
stage's algorithmic bytes (each tensor read or written once: input Snake fp16, weights fp16, the residual x f32
read when the conv adds to it, x f32 written, the next Snake fp16 written).  FETCH_SIZE / WRITE_SIZE are KiB per
dispatch; on gfx950 FETCH_SIZE counts half the bytes of a wide streaming read (MI355X_MICROARCH.md), so fetch
bytes = 2 x 1024 x FETCH_SIZE.  Usage: python tools/vae_pmc_summary.py gpurun_out/vae_pmc 6000"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tools"), os.path.join(ROOT, "ace-step-1.5-ggml_amd")]
from vae_profile import plan  # noqa: E402
from acestep_mi355x.synthetic import VAE_FULL_CONFIG  # noqa: E402


def counter(root, name):
    rows = []
    for path in glob.glob(os.path.join(root, name, "**", "*counter_collection.csv"), recursive=True):
        with open(path, newline="") as f:
            for r in csv.DictReader(f):
                if r.get("Counter_Name") == name and "conv_gemm_kernel" in r.get("Kernel_Name", ""):
                    rows.append((int(r.get("Dispatch_Id", r.get("Correlation_Id", 0))), float(r["Counter_Value"])))
    rows.sort()
    return [v for _, v in rows]


def main(root, frames):
    stages = [s for s in plan(VAE_FULL_CONFIG, frames) if "VALU" not in s[0]]
    fetch, write = counter(root, "FETCH_SIZE"), counter(root, "WRITE_SIZE")
    n = len(stages)
    fetch, write = fetch[-n:], write[-n:]
    out = []
    for (name, M, N, K, flops), f, w in zip(stages, fetch, write):
        out.append({"stage": name, "fetch_MB": round(2 * 1024 * f / 1e6, 1), "write_MB": round(1024 * w / 1e6, 1)})
    tot_f = sum(o["fetch_MB"] for o in out)
    tot_w = sum(o["write_MB"] for o in out)
    print(json.dumps({"frames": frames, "total_fetch_GB": round(tot_f / 1e3, 2), "total_write_GB": round(tot_w / 1e3, 2),
                      "stages": out}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
