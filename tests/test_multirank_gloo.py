"""N > 1 path on CPU: tile sharding, the gather to rank 0 and the
reassembly, over gloo.

Each rank "renders" its tiles with a deterministic stand-in f(j, i) packed the
way rtw_render_device packs them (the kernel's own sharding and the native
assembler are covered on the GPU by test_gpu_parity.py); what runs here is the
host logic of bench.py itself -- bench.make_step (render into the packed
buffer, dist.gather into the rows of one [N, numel] tensor, assemble on rank
0) and bench.run_steps (warm-up, barriers, timed steps, max over ranks) --
with sharding.assemble, the torch restatement of rtw_assemble_tiles, in place
of the device kernel.
"""
import os
import socket
import time

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ray_tracing_weekend_amd import sharding


def _image(h, w):
    j = np.arange(h, dtype=np.float64)[:, None, None]
    i = np.arange(w, dtype=np.float64)[None, :, None]
    c = np.arange(3, dtype=np.float64)[None, None, :]
    return j * 1000.0 + i + c / 8.0


def _owner(h, w, n):
    """independent statement of the assignment: pixel (i, j) lies in tile
    T = (j // 8) * ceil(w / 8) + i // 8, which rank T % n renders"""
    tx = (w + 7) // 8
    j, i = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    return ((j // 8) * tx + i // 8) % n


def _worker(rank, world, port, h, w, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        full = torch.from_numpy(_image(h, w))
        max_tiles = sharding.tiles_for_rank(w, h, 0, world)
        buf = torch.full((max_tiles * 64 * 3,), -1.0, dtype=torch.float64)
        gathered = torch.empty((world, buf.numel()), dtype=torch.float64) if rank == 0 else None
        image = torch.full((h, w, 3), np.nan, dtype=torch.float64) if rank == 0 else None
        seeds = []

        def render(seed, out):          # stand-in for rtw_render_device: this rank's tiles, packed
            seeds.append(seed)
            packed = sharding.pack(full, rank, world).reshape(-1)
            out[: packed.numel()] = packed
            time.sleep(0.01 * (rank + 1))

        def assemble(ranks, img):       # stand-in for rtw_assemble_tiles
            sharding.assemble(img, list(ranks.unbind(0)))

        step = bench.make_step(render, assemble, dist, rank, world, buf, gathered, image)
        elapsed = bench.run_steps(step, 3, 2, dist, lambda: None, device="cpu")
        ok = seeds == [1000, 1001, 0, 1, 2]
        # the timed region is the slowest rank's: >= 3 steps x 10 ms x world
        ok = ok and elapsed >= 0.03 * world * 0.99
        if rank == 0:
            ok = ok and bool(torch.equal(image, full))
        t = torch.tensor([sharding.tiles_for_rank(w, h, rank, world)], dtype=torch.int64)
        dist.all_reduce(t)
        ok = ok and int(t) == sharding.n_tiles(w, h)
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


def _worker_image_device(rank, world, port, h, w, q):
    """The orchestration of rtw_render_image_device (capi.cpp) on a
    multi-device context, one gloo rank per device: every rank renders its
    tiles into an equal-size buffer of rank 0's tile count -- rank 0 in place,
    into slot 0 of the gather target (ncclGather's in-place form,
    rccl.h:729-733); the tails past a rank's own tiles hold garbage (NaN here),
    which the assembly must never read -- then ONE gather to rank 0 and the
    assembly with the slot stride."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        full = torch.from_numpy(_image(h, w))
        per = max(sharding.tiles_for_rank(w, h, 0, world) * 64 * 3, 1)
        target = torch.full((world, per), np.nan, dtype=torch.float64) if rank == 0 else None
        send = target[0] if rank == 0 else torch.full((per,), np.nan, dtype=torch.float64)
        packed = sharding.pack(full, rank, world).reshape(-1)
        send[: packed.numel()] = packed
        dist.gather(send, list(target.unbind(0)) if rank == 0 else None, dst=0)
        ok = True
        if rank == 0:
            img = torch.full((h, w, 3), -7.0, dtype=torch.float64)
            sharding.assemble(img, list(target.unbind(0)))
            ok = bool(torch.equal(img, full))
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,h,w", [(2, 27, 5), (3, 41, 30), (4, 9, 17)])
def test_image_device_orchestration_gathers_in_place(world, h, w):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_image_device, args=(r, world, port, h, w, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = dict(q.get(timeout=5) for _ in procs)
    assert res == {r: True for r in range(world)}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,h,w", [(2, 27, 5), (2, 800, 12), (2, 8, 3), (3, 41, 30)])
def test_bench_step_gathers_and_reassembles(world, h, w):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, h, w, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = dict(q.get(timeout=5) for _ in procs)
    assert res == {r: True for r in range(world)}


@pytest.mark.parametrize("h,w", [(0, 5), (1, 1), (7, 9), (8, 8), (9, 17), (27, 5), (225, 400), (800, 1200)])
@pytest.mark.parametrize("n", [1, 2, 3, 8])
def test_rank_tiles_partition(h, w, n):
    own = _owner(h, w, n)
    full = torch.from_numpy(_image(h, w))
    for k in range(n):
        assert sharding.tiles_for_rank(w, h, k, n) == len(sharding.rank_tiles(w, h, k, n))
        if h and w:
            # rank k's packed buffer holds exactly the pixels it owns
            packed = sharding.pack(full, k, n)
            vals = set(map(tuple, packed[(packed != 0).any(-1)].tolist()))
            mine = set(map(tuple, full[torch.from_numpy(own == k)].tolist()))
            assert vals == mine - {(0.0, 0.125, 0.25)} or vals == mine
    assert sum(sharding.tiles_for_rank(w, h, k, n) for k in range(n)) == sharding.n_tiles(w, h)


@pytest.mark.parametrize("h,w", [(1, 1), (27, 5), (225, 400), (800, 1200), (2160, 3840)])
@pytest.mark.parametrize("n", [1, 2, 3, 8])
def test_tiles_for_rank_match_c_abi(h, w, n):
    from ray_tracing_weekend_amd import tile_size, tiles_for_rank
    assert tile_size() == sharding.TILE
    for k in range(n):
        assert tiles_for_rank(w, h, k, n) == sharding.tiles_for_rank(w, h, k, n)


def test_pack_assemble_round_trip_single_process():
    h, w, n = 41, 30, 3
    full = torch.from_numpy(_image(h, w))
    bufs = []
    for k in range(n):
        p = sharding.pack(full, k, n).reshape(-1)
        b = torch.zeros(sharding.tiles_for_rank(w, h, 0, n) * 64 * 3, dtype=torch.float64)
        b[: p.numel()] = p
        bufs.append(b)
    img = torch.empty_like(full)
    assert torch.equal(sharding.assemble(img, bufs), full)


def test_c4_shares_balance():
    """C4 (3840x2160) over 8 ranks: 16 200 tiles each, every rank's tiles spread
    over the whole image height (the cost profile of the image is sampled)."""
    w, h, n = 3840, 2160, 8
    tx = w // 8
    for k in range(n):
        t = np.array(sharding.rank_tiles(w, h, k, n))
        assert len(t) == 16200
        rows = np.bincount(t // tx, minlength=h // 8)
        assert rows.min() == rows.max() == tx // n


def test_bad_rank_rejected():
    with pytest.raises(ValueError):
        sharding.tiles_for_rank(10, 10, 2, 2)
