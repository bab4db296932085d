"""world_size-2 gloo tests of the batch-sharded sampler (CPU): the conditioning broadcast reaches every
rank unchanged, gather_latents restores the global item order, and the whole sharded generation
(product sampling loop through the host-emulated library) equals the single-process result."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, B, q):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "ace-step-1.5-ggml_amd"))
    from acestep_mi355x.sampler import Conditioning, broadcast_conditioning, gather_latents, shard_indices
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        T, L, audio, ctxd, H = 6, 3, 4, 8, 5
        shapes = dict(B=B, T=T, L=L, audio=audio, ctx=ctxd, H=H, mask=True, enc_mask=True)
        cond = None
        if rank == 0:
            g = torch.Generator().manual_seed(0)
            cond = Conditioning(noise=torch.randn(B, T, audio, generator=g), context=torch.randn(B, T, ctxd, generator=g),
                                enc=torch.randn(B, L, H, generator=g), enc_mask=torch.ones(B, L, dtype=torch.int32),
                                mask=torch.arange(B * T, dtype=torch.int32).reshape(B, T))
        got = broadcast_conditioning(cond, shapes, torch.device("cpu"))
        items = shard_indices(B, world, rank)
        # "sample": x0 = noise + item id, computed only for the local shard
        x_local = got.noise[items] + torch.tensor(items, dtype=torch.float32)[:, None, None]
        full = gather_latents(x_local, B)
        digest = (float(got.noise.sum()), float(got.enc.sum()), int(got.mask.sum()))
        q.put((rank, digest, None if full is None else full.clone(), got.noise.clone()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("B", [2, 3, 5])
def test_broadcast_and_gather_world2(B):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, B, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r, digest, full, noise = q.get(timeout=120)
        res[r] = (digest, full, noise)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][0] == res[1][0]
    assert res[1][1] is None
    full, noise = res[0][1], res[0][2]
    expect = noise + torch.arange(B, dtype=torch.float32)[:, None, None]
    torch.testing.assert_close(full, expect)


def _gen_worker(rank, world, port, lib, ckpt, B, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "ace-step-1.5-ggml_amd")]
    from acestep_mi355x.capi import GGMLCAPIBridge
    from acestep_mi355x.sampler import Conditioning, broadcast_conditioning, gather_latents, generate_local, shard_indices
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        T, L = 24, 5
        shapes = dict(B=B, T=T, L=L, audio=64, ctx=128, H=256, mask=False, enc_mask=False)
        cond = None
        if rank == 0:
            g = torch.Generator().manual_seed(3)
            cond = Conditioning(noise=torch.randn(B, T, 64, generator=g), context=torch.randn(B, T, 128, generator=g),
                                enc=torch.randn(B, L, 256, generator=g))
        got = broadcast_conditioning(cond, shapes, torch.device("cpu"))
        br = GGMLCAPIBridge(lib_path=lib)
        br.load_dit(ckpt)
        x = generate_local(br, got, shard_indices(B, world, rank), [1.0, 0.75, 0.5, 0.25], cache_cross=True)
        full = gather_latents(x, B)
        br.close()
        q.put((rank, None if full is None else full.clone()))
    finally:
        dist.destroy_process_group()


def test_generate_local_world2_equals_single_process(tiny_ckpt):
    """The real sampling path across 2 gloo ranks — conditioning broadcast, each rank's shard through the
    product's device generation loop (ace_mi_dit_sample_ex, here the host-emulated library), gather —
    gives the single-process result for every item."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from hostlib import CLANG, build_host_lib
    if not os.path.exists(CLANG):
        pytest.skip("host clang++ not available")
    lib = build_host_lib()
    B = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gen_worker, args=(r, 2, port, lib, tiny_ckpt, B, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from acestep_mi355x.capi import GGMLCAPIBridge
    from acestep_mi355x.sampler import Conditioning, generate_local
    g = torch.Generator().manual_seed(3)
    cond = Conditioning(noise=torch.randn(B, 24, 64, generator=g), context=torch.randn(B, 24, 128, generator=g),
                        enc=torch.randn(B, 5, 256, generator=g))
    br = GGMLCAPIBridge(lib_path=lib)
    br.load_dit(tiny_ckpt)
    ref = generate_local(br, cond, list(range(B)), [1.0, 0.75, 0.5, 0.25], cache_cross=True)
    br.close()
    assert res[1] is None
    torch.testing.assert_close(res[0], ref, rtol=1e-6, atol=1e-6)
