"""world_size-2 gloo tests of the batch-sharded sampler collectives (CPU): the conditioning
broadcast reaches every rank unchanged and gather_latents restores the global item order."""
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
