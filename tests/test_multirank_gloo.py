"""N > 1 path on CPU: row-tile sharding, the gather to rank 0 and the
reassembly, with world_size 2 over gloo.

Each rank "renders" its rows with a deterministic stand-in f(j, i) (the
kernel's own sharding is covered on the GPU by
test_gpu_parity.py::test_rank_sharding_reassembles_the_image); what is tested
here is the host logic bench.py runs: which rows a rank owns, the packed
buffer sized by rtw_rows_for_rank, dist.gather, sharding.assemble.
"""
import os
import socket

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


def _tile_owner_rows(h, rank, n, tile=8):
    # independent statement of the assignment: tile row t -> rank t % n
    return [j for j in range(h) if (j // tile) % n == rank]


def _worker(rank, world, port, h, w, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        full = torch.from_numpy(_image(h, w))
        mine = sharding.rank_rows(h, rank, world)
        max_rows = max(len(sharding.rank_rows(h, k, world)) for k in range(world))
        buf = torch.full((max_rows, w, 3), -1.0, dtype=torch.float64)
        buf[: len(mine)] = full[mine]
        gathered = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
        dist.gather(buf, gathered, dst=0)
        ok = True
        if rank == 0:
            image = torch.full((h, w, 3), np.nan, dtype=torch.float64)
            sharding.assemble(image, gathered, h)
            ok = bool(torch.equal(image, full))
        t = torch.tensor([len(mine)], dtype=torch.int64)
        dist.all_reduce(t)
        ok = ok and int(t) == h
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("h,w", [(27, 5), (800, 4), (8, 3)])
def test_gather_reassembles_image_world2(h, w):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, h, w, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = dict(q.get(timeout=5) for _ in procs)
    assert res == {0: True, 1: True}


@pytest.mark.parametrize("h", [0, 1, 7, 8, 9, 27, 225, 800])
@pytest.mark.parametrize("n", [1, 2, 3, 8])
def test_rank_rows_partition(h, n):
    rows = [sharding.rank_rows(h, k, n) for k in range(n)]
    for k in range(n):
        assert rows[k] == _tile_owner_rows(h, k, n)
    assert sorted(sum(rows, [])) == list(range(h))


@pytest.mark.parametrize("h", [1, 27, 225, 800])
@pytest.mark.parametrize("n", [1, 2, 3, 8])
def test_rank_rows_match_c_abi(h, n):
    from ray_tracing_weekend_amd import rows_for_rank, tile_rows
    assert tile_rows() == sharding.TILE_ROWS
    for k in range(n):
        assert rows_for_rank(h, k, n) == len(sharding.rank_rows(h, k, n))


def test_assemble_three_ranks_single_process():
    h, w, n = 41, 6, 3
    full = torch.from_numpy(_image(h, w))
    bufs = []
    for k in range(n):
        r = sharding.rank_rows(h, k, n)
        b = torch.zeros((24, w, 3), dtype=torch.float64)
        b[: len(r)] = full[r]
        bufs.append(b)
    img = torch.empty_like(full)
    assert torch.equal(sharding.assemble(img, bufs, h), full)


def test_bad_rank_rejected():
    with pytest.raises(ValueError):
        sharding.rank_rows(10, 2, 2)
