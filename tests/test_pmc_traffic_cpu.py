"""CPU: the HBM-traffic plumbing behind bench.py's `roofline.traffic` -- tools/pmc_summary.py on synthetic rocprofv3
counter files (the gfx950 FETCH_SIZE x 2 correction, launch weighting, which kernels count as gate|up and as the f8c
attention operator, the source-hash build stamp) and bench.py's refusal of a summary from another build or workload."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ace-step-1.5-ggml_amd"))

GU = "void acemi::gemm_detail::gemm_kernel<192, 128, 2, 2, false, 4, 1, false>(acemi::gemm_detail::GemmParams)"
KH = "void acemi::(anonymous namespace)::attn_kh_kernel<false, false>(acemi::AttnArgs)"
A2 = "void acemi::(anonymous namespace)::attn2_kernel<false, true, true, true, 1, true>(acemi::AttnArgs)"
A2_F32 = "void acemi::(anonymous namespace)::attn2_kernel<false, true, true, true, 1, false>(acemi::AttnArgs)"
OTHER = "void acemi::(anonymous namespace)::rmsnorm_mod_persist_kernel<false, 4>(float const*, int, int)"


def _write(root, counter, rows):
    d = os.path.join(root, counter, "box")
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "pmc_counter_collection.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for i, (k, v) in enumerate(rows):
            w.writerow({"Dispatch_Id": i, "Kernel_Name": k, "Counter_Name": counter, "Counter_Value": v})


def test_pmc_summary_on_synthetic_counters(tmp_path):
    # KiB per dispatch; FETCH_SIZE is doubled (gfx950 reports half of a wide streaming read), WRITE_SIZE is exact
    _write(str(tmp_path), "FETCH_SIZE", [(GU, 100.0), (GU, 300.0), (KH, 10.0), (KH, 10.0), (A2, 40.0), (A2_F32, 999.0),
                                         (OTHER, 5.0)])
    _write(str(tmp_path), "WRITE_SIZE", [(GU, 50.0), (GU, 50.0), (KH, 4.0), (KH, 4.0), (A2, 8.0), (A2_F32, 1.0),
                                         (OTHER, 1.0)])
    bench_log = tmp_path / "bench.log"
    bench_log.write_text("noise\n" + json.dumps({"config": {"latent_frames": 6000, "enc_len": 512, "batch_per_gpu": 1,
                                                            "weights": "q8_0", "other": 1}}) + "\n")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), str(tmp_path), str(bench_log)],
                         capture_output=True, text=True, check=True).stdout
    d = json.loads(out)
    k = 1024.0
    assert d["gate_up"]["kernel"] == GU
    assert d["gate_up"]["hbm_bytes"] == 2 * k * 200.0 + k * 50.0
    # f8c attention: both kernels (attn_kh full layers, attn2 f8c short ranges), launch-weighted; attn2's f32 mode excluded
    att = d["attention"]
    assert sorted(att["kernels"]) == sorted([KH, A2]) and att["launches"] == 3
    assert abs(att["hbm_bytes"] - (2 * (2 * k * 10.0 + k * 4.0) + (2 * k * 40.0 + k * 8.0)) / 3) < 1e-6
    from acestep_mi355x import source_hash
    assert d["build"] == source_hash()
    assert d["config"] == {"latent_frames": 6000, "enc_len": 512, "batch_per_gpu": 1, "weights": "q8_0"}


def test_bench_uses_traffic_only_from_the_same_build_and_workload(tmp_path, monkeypatch):
    sys.path.insert(0, ROOT)
    import bench
    summary = {"config": {"latent_frames": 6000, "enc_len": 512, "batch_per_gpu": 1, "weights": "q8_0"},
               "build": "0123456789abcdef", "gate_up": {"hbm_bytes": 2.9e8}, "attention": {"hbm_bytes": 6.6e7}}
    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "pmc_traffic.json").write_text(json.dumps(summary))
    monkeypatch.setattr(bench.os.path, "abspath", lambda p: str(tmp_path / "bench.py"))
    monkeypatch.setattr(bench, "source_hash", lambda: "0123456789abcdef")
    assert bench.pmc_traffic(6000, 512, 1, "q8_0", "gate_up") == 2.9e8
    assert bench.pmc_traffic(6000, 512, 1, "q8_0", "attention") == 6.6e7
    assert bench.pmc_traffic(3000, 512, 1, "q8_0", "gate_up") is None   # another workload
    assert bench.pmc_traffic(6000, 512, 1, "bf16", "gate_up") is None
    monkeypatch.setattr(bench, "source_hash", lambda: "fedcba9876543210")
    assert bench.pmc_traffic(6000, 512, 1, "q8_0", "gate_up") is None   # another build: no stale bytes
