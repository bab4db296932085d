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
        # numpy, not torch tensors: a torch tensor crosses the queue as a shared fd that dies with this process
        q.put((rank, digest, None if full is None else full.numpy().copy(), got.noise.numpy().copy()))
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
        res[r] = (digest, None if full is None else torch.from_numpy(full), torch.from_numpy(noise))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][0] == res[1][0]
    assert res[1][1] is None
    full, noise = res[0][1], res[0][2]
    expect = noise + torch.arange(B, dtype=torch.float32)[:, None, None]
    torch.testing.assert_close(full, expect)


SCHED = [1.0, 0.75, 0.5, 0.25]


def _cond(B, seed=3, nc=False):
    from acestep_mi355x.sampler import Conditioning
    g = torch.Generator().manual_seed(seed + (100 if nc else 0))
    return Conditioning(noise=torch.randn(B, 24, 64, generator=g), context=torch.randn(B, 24, 128, generator=g),
                        enc=torch.randn(B, 5, 256, generator=g))


def _run_flow(br, cond, B, items, method, cover, decode, cond_nc=None):
    from acestep_mi355x.sampler import decode_local, generate_local
    x = generate_local(br, cond, items, SCHED, infer_method=method, seed=11, cache_cross=True,
                       cover_steps=-1 if cover is None else cover, cond_non_cover=cond_nc if cover is not None else None)
    return decode_local(br, x) if decode else x


def _gen_worker(rank, world, port, lib, ckpt, vae, B, method, cover, decode, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "ace-step-1.5-ggml_amd")]
    from acestep_mi355x.capi import GGMLCAPIBridge
    from acestep_mi355x.sampler import broadcast_conditioning, gather_latents, shard_indices
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        shapes = dict(B=B, T=24, L=5, audio=64, ctx=128, H=256, mask=False, enc_mask=False)
        got = broadcast_conditioning(_cond(B) if rank == 0 else None, shapes, torch.device("cpu"))
        got_nc = broadcast_conditioning(_cond(B, nc=True) if rank == 0 else None, shapes, torch.device("cpu"))
        br = GGMLCAPIBridge(lib_path=lib)
        br.load_dit(ckpt)
        if decode:
            br.load_vae(vae)
        x = _run_flow(br, got, B, shard_indices(B, world, rank), method, cover, decode, got_nc)
        full = gather_latents(x.contiguous(), B)
        br.close()
        q.put((rank, None if full is None else full.numpy().copy()))
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module")
def tiny_vae():
    import tempfile
    from acestep_mi355x.synthetic import VAE_TINY_CONFIG, write_vae_checkpoint
    d = tempfile.mkdtemp(prefix="acemi_dvae_")
    write_vae_checkpoint(d, VAE_TINY_CONFIG, seed=1)
    return d


# (world, B, method, cover_steps, decode): the ODE loop at world 2 (B=3, a ragged shard), SDE with
# whole-batch noise (ADVICE: the result must not depend on the world size), the audio-cover switch
# at step 0 and 2, the configs[4] flow (bs=4 over 4 ranks: DiT loop, VAE decode, audio gather) and
# the configs[3] latent flow (bs=8 over 8 ranks)
FLOWS = [(2, 3, "ode", None, False), (2, 3, "sde", None, False), (3, 4, "sde", 2, False), (2, 2, "ode", 0, False),
         (4, 4, "ode", None, True), (4, 3, "ode", None, True), (8, 8, "ode", None, False)]


@pytest.mark.parametrize("world,B,method,cover,decode", FLOWS)
def test_sharded_flow_equals_single_process(tiny_ckpt, tiny_vae, world, B, method, cover, decode):
    """The real sampling path across `world` gloo ranks — conditioning broadcast, each rank's shard through the
    product's device generation loop (ace_mi_dit_sample_ex, here the host-emulated library), optionally its
    VAE decode, gather — gives the single-process result for every item, in item order."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from hostlib import CLANG, build_host_lib
    if not os.path.exists(CLANG):
        pytest.skip("host clang++ not available")
    lib = build_host_lib()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gen_worker, args=(r, world, port, lib, tiny_ckpt, tiny_vae, B, method, cover, decode, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {r: (None if a is None else torch.from_numpy(a)) for r, a in (q.get(timeout=600) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from acestep_mi355x.capi import GGMLCAPIBridge
    br = GGMLCAPIBridge(lib_path=lib)
    br.load_dit(tiny_ckpt)
    if decode:
        br.load_vae(tiny_vae)
    ref = _run_flow(br, _cond(B), B, list(range(B)), method, cover, decode, _cond(B, nc=True))
    n_audio = br.vae_out_len(24) if decode else None
    br.close()
    assert all(res[r] is None for r in range(1, world))
    assert res[0].shape == ref.shape
    torch.testing.assert_close(res[0], ref, rtol=1e-6, atol=1e-6)
    if decode:
        assert ref.shape[1] == 2 and ref.shape[2] == n_audio


def test_sde_noise_is_independent_per_item():
    """Per-item SDE draws: items differ from each other, and a rank's slice (only its own items drawn) equals the
    single-process slice of the same items."""
    from acestep_mi355x.sampler import sde_noise
    a = sde_noise(3, [0, 1, 2, 3], 5, 2, 7, "cpu")
    b = sde_noise(3, [0, 1, 2, 3], 5, 2, 7, "cpu")
    torch.testing.assert_close(a, b)
    assert not torch.allclose(a[:, 0], a[:, 1])
    torch.testing.assert_close(sde_noise(3, [1, 3], 5, 2, 7, "cpu"), a[:, [1, 3]])
    assert not torch.allclose(sde_noise(3, [0, 1], 5, 2, None, "cpu"), sde_noise(3, [0, 1], 5, 2, None, "cpu"))


def test_sde_noise_seed_mapping_is_pinned():
    """The seed -> noise mapping (item b: torch CPU generator seeded with seed * 1000003 + b) is an intentional
    deviation from the reference's single (bsz, T, C) MLX draw per step (generate.py:187, not reproducible without
    MLX); the committed fixture (tests/golden/make_sde_noise_fixture.py) catches any change to the stream."""
    import json
    import os
    import torch
    from acestep_mi355x.sampler import sde_noise
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "sde_noise_seed7.json"),
              encoding="utf-8") as f:
        g = json.load(f)
    x = sde_noise(g["n_draws"], g["items"], g["T"], g["C"], g["seed"], "cpu")
    torch.testing.assert_close(x.reshape(-1), torch.tensor(g["values"], dtype=torch.float32), rtol=0, atol=0)
