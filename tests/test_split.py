"""The cost-dealt rank split (ABI 10) on CPU: rtw_split_deal
(the C-ABI's host function, no GPU call) against its numpy restatement
sharding.deal, the invariants every split keeps (each rank's round-robin tile
count, so packed buffers and the gather keep their size), and the
one-process-per-GPU orchestration of bench.py (each rank's counted costs
all-reduced over gloo, the same deal on every rank, render into the packed
buffer, gather, assemble by the split)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import ray_tracing_weekend_amd as rtw
from ray_tracing_weekend_amd import sharding


def _costs(w, h, seed, heavy=0.1):
    """a cost field shaped like a render's: mostly cheap tiles, a clustered
    fraction of expensive ones (glass), ties included"""
    rng = np.random.default_rng(seed)
    n = sharding.n_tiles(w, h)
    c = rng.integers(10, 100, n)
    hot = rng.random(n) < heavy
    c[hot] += rng.integers(1000, 50000, hot.sum())
    c[::5] = 7                                   # many equal costs: the tie rules decide
    return c.astype(np.uint32)


@pytest.mark.parametrize("w,h,n", [(1200, 800, 8), (1200, 800, 2), (37, 23, 3), (120, 72, 8), (5, 5, 2),
                                   (8, 8, 3), (64, 40, 1), (200, 120, 7),
                                   (1200, 800, 256), (2048, 8, 256)])
def test_deal_matches_restatement_and_keeps_counts(w, h, n):
    c = _costs(w, h, w * 31 + h + n)
    a = rtw.split_deal(c, w, h, n)
    assert np.array_equal(a, sharding.deal(c, w, h, n))
    assert np.array_equal(a, rtw.split_deal(c, w, h, n))          # deterministic
    cnt = np.bincount(a, minlength=n)
    assert cnt.tolist() == [rtw.tiles_for_rank(w, h, r, n) for r in range(n)]


def test_deal_balances_the_dealt_cost():
    """C2's tile grid over 8 ranks: the dealt costs within 0.1 % of each other
    (the round robin of the same field: several %)"""
    w, h, n = 1200, 800, 8
    c = _costs(w, h, 5, heavy=0.05).astype(np.float64)
    a = rtw.split_deal(c.astype(np.uint32), w, h, n)
    load = np.bincount(a, weights=c, minlength=n)
    rr = np.bincount(np.arange(c.size) % n, weights=c, minlength=n)
    assert load.max() / load.mean() - 1 < 1e-3
    assert rr.max() / rr.mean() - 1 > 10 * (load.max() / load.mean() - 1)


def test_deal_rejects_bad_arguments():
    c = np.ones(sharding.n_tiles(16, 16), np.uint32)
    with pytest.raises(rtw.RenderError):
        rtw.split_deal(c, 16, 16, 0)
    with pytest.raises(rtw.RenderError):
        rtw.split_deal(c, 16, 16, 1000)                           # > RTW_MAX_RANKS
    with pytest.raises(rtw.RenderError):
        rtw.split_deal(c[:-1], 16, 16, 2)


def test_split_pack_assemble_round_trip():
    h, w, n = 41, 30, 3
    full = torch.arange(h * w * 3, dtype=torch.float64).reshape(h, w, 3) + 1
    split = rtw.split_deal(_costs(w, h, 3), w, h, n)
    per = sharding.tiles_for_rank(w, h, 0, n) * 64 * 3
    bufs = []
    for k in range(n):
        p = sharding.pack(full, k, n, split).reshape(-1)
        b = torch.full((per,), float("nan"), dtype=torch.float64)
        b[: p.numel()] = p
        bufs.append(b)
        assert sharding.rank_tiles(w, h, k, n, split) == np.nonzero(split == k)[0].tolist()
    img = torch.empty_like(full)
    assert torch.equal(sharding.assemble(img, bufs, split=split), full)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, h, w, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        full_cost = _costs(w, h, 11)
        # what rtw_tile_costs returns after this rank's counting render (the round
        # robin): its own tiles' costs, zeros elsewhere
        local = np.zeros_like(full_cost)
        mine = sharding.rank_tiles(w, h, rank, world)
        local[mine] = full_cost[mine]
        got = {}
        split, cost = bench.balance_split(local, dist, "cpu", lambda c: sharding.deal(c, w, h, world),
                                          lambda s, c: got.update(split=s, cost=c))
        ok = np.array_equal(cost, full_cost) and np.array_equal(split, sharding.deal(full_cost, w, h, world))
        ok = ok and got["split"] is split
        # every rank holds the same split
        t = torch.from_numpy(split.astype(np.int64))
        t0 = t.clone()
        dist.broadcast(t0, 0)
        ok = ok and torch.equal(t, t0)
        # the bench step with the split: pack, gather, assemble
        image_full = torch.arange(h * w * 3, dtype=torch.float64).reshape(h, w, 3)
        buf = torch.full((sharding.tiles_for_rank(w, h, 0, world) * 64 * 3,), -1.0, dtype=torch.float64)
        gathered = torch.empty((world, buf.numel()), dtype=torch.float64) if rank == 0 else None
        image = torch.full((h, w, 3), np.nan, dtype=torch.float64) if rank == 0 else None

        def render(seed, out):
            p = sharding.pack(image_full, rank, world, split).reshape(-1)
            out[: p.numel()] = p

        def assemble(ranks, img):
            sharding.assemble(img, list(ranks.unbind(0)), split=split)

        step = bench.make_step(render, assemble, dist, rank, world, buf, gathered, image)
        bench.run_steps(step, 2, 1, dist, lambda: None, device="cpu")
        if rank == 0:
            ok = ok and bool(torch.equal(image, image_full))
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,h,w", [(2, 80, 120), (3, 41, 30)])
def test_bench_balance_split_orchestration(world, h, w):
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
