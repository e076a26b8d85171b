"""Tile sharding of one image over ranks.

The image is cut into 8x8 tiles T = ty * tiles_x + tx (row j = 0 at the
bottom).  By default tile T belongs to rank T % nranks (the round robin): the
interleave is fine-grained, so every rank samples the image's whole cost
profile.  A dealt split (``split``: tile -> rank, rtw_set_split / ``deal``)
gives the tiles to the ranks by their counted costs instead, keeping each
rank's round-robin tile count.  Each rank's ``rtw_render_device`` output
holds its tiles packed in increasing T (the k-th tile at
``[k * 64 + ly * 8 + lx]``); rank 0 gathers the equal-size packed buffers (one
RCCL gather) and un-interleaves them on the device with ``rtw_assemble_tiles``.

This module is the numpy / torch restatement of that layout: the deal, the
index maps, and an ``assemble`` that the CPU tests (gloo) and the GPU test of
the native assembler use as the reference.  The reference renders on one host
(``camera.rs:315-388``: one rayon task per pixel, balanced by work stealing,
``:340-353``), so this exchange step has no counterpart there.
"""
from __future__ import annotations

import functools

import numpy as np
import torch

TILE = 8      # == rtw_tile_size() == kTile in csrc/rtw_kernels.h


def n_tiles(width: int, height: int, tile: int = TILE) -> int:
    return ((width + tile - 1) // tile) * ((height + tile - 1) // tile)


def tiles_for_rank(width: int, height: int, rank: int, nranks: int) -> int:
    """Number of tiles ``rank`` renders (== rtw_tiles_for_rank)."""
    if nranks < 1 or not 0 <= rank < nranks:
        raise ValueError(f"bad rank {rank} of {nranks}")
    n = n_tiles(width, height)
    return (n - rank + nranks - 1) // nranks if rank < n else 0


def deal(tile_cost, width: int, height: int, nranks: int) -> np.ndarray:
    """Restatement of rtw_split_deal: tiles costliest first (ties: lower
    index), each to the rank of least dealt cost (ties: lower rank) that is
    still below its round-robin tile count.  uint32 [n_tiles] tile -> rank."""
    n = n_tiles(width, height)
    cost = np.asarray(tile_cost, np.int64).reshape(-1)
    if cost.size != n:
        raise ValueError(f"{cost.size} costs for {n} tiles")
    room = [tiles_for_rank(width, height, r, nranks) for r in range(nranks)]
    load = [0] * nranks
    out = np.zeros(n, np.uint32)
    for t in np.argsort(-cost, kind="stable"):
        best = min((r for r in range(nranks) if room[r]), key=lambda r: (load[r], r))
        out[t] = best
        load[best] += int(cost[t])
        room[best] -= 1
    return out


def rank_tiles(width: int, height: int, rank: int, nranks: int, split=None) -> list[int]:
    """Global tile ids of ``rank`` in the order they are packed (``split``:
    a dealt tile -> rank array; None: the round robin)."""
    if split is not None:
        return np.nonzero(np.asarray(split).reshape(-1) == rank)[0].tolist()
    return list(range(rank, n_tiles(width, height), nranks)) if tiles_for_rank(width, height, rank, nranks) else []


def _key(split):
    return None if split is None else np.asarray(split, np.uint32).tobytes()


@functools.lru_cache(maxsize=64)
def _maps(width: int, height: int, rank: int, nranks: int, device: str, split_key=None):
    """(slots, pixels): for every in-image pixel of the rank's packed tiles,
    its slot in the packed buffer and its index in the flattened image."""
    tiles_x = (width + TILE - 1) // TILE
    split = None if split_key is None else np.frombuffer(split_key, np.uint32)
    t = torch.tensor(rank_tiles(width, height, rank, nranks, split), dtype=torch.long)
    lane = torch.arange(64, dtype=torch.long)
    i = (t % tiles_x)[:, None] * TILE + (lane % TILE)[None, :]
    j = (t // tiles_x)[:, None] * TILE + (lane // TILE)[None, :]
    slot = torch.arange(t.numel() * 64, dtype=torch.long).view(-1, 64)
    ok = (i < width) & (j < height)
    return slot[ok].to(device), (j * width + i)[ok].to(device)


def pack(image: torch.Tensor, rank: int, nranks: int, split=None) -> torch.Tensor:
    """The rank's packed tile buffer ``[tiles * 64, 3]`` cut out of a full
    image ``[H, W, 3]`` (pixels outside the image: 0) -- what
    rtw_render_device writes for that rank."""
    height, width = image.shape[:2]
    slots, pix = _maps(width, height, rank, nranks, str(image.device), _key(split))
    out = torch.zeros((tiles_for_rank(width, height, rank, nranks) * 64, 3), dtype=image.dtype,
                      device=image.device)
    out[slots] = image.reshape(-1, 3)[pix]
    return out


def assemble(image: torch.Tensor, gathered, height: int | None = None, split=None) -> torch.Tensor:
    """Scatter the ranks' packed tile buffers ``gathered[k]`` (each at least
    ``tiles_for_rank(W, H, k, N) * 64 * 3`` elements) into ``image``
    (``[H, W, 3]``); the torch restatement of rtw_assemble_tiles."""
    h, width = image.shape[:2]
    height = h if height is None else height
    nranks = len(gathered)
    flat = image.view(-1, 3)
    for k, buf in enumerate(gathered):
        slots, pix = _maps(width, height, k, nranks, str(image.device), _key(split))
        flat.index_copy_(0, pix, buf.reshape(-1, 3)[slots])
    return image
