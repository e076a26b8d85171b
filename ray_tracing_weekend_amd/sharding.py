"""Row-tile sharding of one image over ranks.

The image is cut into 8-row tile rows; tile row ``t`` belongs to rank
``t % nranks`` (sky rows are cheap and sphere rows expensive, so interleaving
balances the ranks).  Each rank's ``rtw_render_device`` output holds its rows
packed in increasing order; rank 0 gathers the packed buffers (one RCCL
gather) and scatters them back into image rows with one indexed copy per rank.

This is the host side of the only exchange step of the path -- the reference
renders on one host (``camera.rs:315-388``), so it has no counterpart there.
"""
from __future__ import annotations

import functools

import torch

TILE_ROWS = 8      # == rtw_tile_rows() == kTile in csrc/rtw_kernels.h


def rank_rows(height: int, rank: int, nranks: int, tile: int = TILE_ROWS) -> list[int]:
    """Image rows (j index, 0 = bottom) that ``rank`` renders, in the order
    they are packed in its output buffer."""
    if nranks < 1 or not 0 <= rank < nranks:
        raise ValueError(f"bad rank {rank} of {nranks}")
    rows = []
    for t in range(rank, (height + tile - 1) // tile, nranks):
        rows.extend(range(t * tile, min(height, (t + 1) * tile)))
    return rows


@functools.lru_cache(maxsize=64)
def _index(height: int, rank: int, nranks: int, device: str) -> torch.Tensor:
    return torch.tensor(rank_rows(height, rank, nranks), dtype=torch.long, device=device)


def assemble(image: torch.Tensor, gathered, height: int) -> torch.Tensor:
    """Scatter the ranks' packed row buffers ``gathered[k]`` (shape
    ``[>= rows of rank k, W, 3]``) into ``image`` (``[height, W, 3]``)."""
    nranks = len(gathered)
    for k, buf in enumerate(gathered):
        idx = _index(height, k, nranks, str(image.device))
        image.index_copy_(0, idx, buf[: idx.numel()])
    return image
