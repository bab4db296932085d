"""bench.py's multi-rank code path (torchrun launch, process group, conditioning broadcast, shard selection,
barriers, max-over-ranks timing, one JSON line from rank 0) on CPU: `--emulate` runs it with gloo and the
host-emulated library (tests/host/kernel_emul.cpp) on the tiny config.  CPU only; not a measurement."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,bpg", [(2, 1), (4, 2), (8, 1)])
def test_bench_multi_rank_path_emulated(world, bpg):
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from hostlib import CLANG
    if not os.path.exists(CLANG):
        pytest.skip("host clang++ not available")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--emulate", "--gpus", str(world), "--batch-per-gpu", str(bpg), "--steps", "2", "--warmup", "1",
           "--seconds", "2", "--enc-len", "16", "--qtype", "bf16", "--no-profile", "--no-bf16-line",
           "--no-cpu-baseline"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    d = json.loads(lines[0])
    assert d["metric"].startswith("EMULATED")
    assert d["n_gpus"] == world and d["config"]["global_batch"] == world * bpg
    assert d["config"]["batch_per_gpu"] == bpg and d["finite"] is True
    assert d["value"] > 0 and d["steps"] == 2
    # per-rank elapsed (max-over-ranks timing) and the conditioning broadcast of the multi-GPU path
    assert len(d["ranks"]["elapsed_s"]) == world and max(d["ranks"]["elapsed_s"]) * d["value"] > 0
    assert d["ranks"]["items_per_rank"] == [bpg] * world
    T = int(round(2 * 25))
    assert d["ranks"]["broadcast_bytes_per_rank"] == 4 * world * bpg * (T * 64 + T * 128 + 16 * 256)
