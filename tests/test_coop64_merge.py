"""The list-order merge of the f64 wave-cooperative light-grid walk
(render_kernel.hpp lights_pdf_grid_coop64), restated in Python: a ray's hit
lights are found by several pieces of its walk (and the big list), each piece
keeps only its kPieceIds smallest list indices >= lo, the ray's owner keeps
its kMax smallest of what it is offered, and every index up to `bound` (the
largest kept index of any list that had to drop one) is summed before the
next pass starts at bound + 1.  The sum must visit every hit index exactly
once, in ascending order (HittableList::pdf_value's list order,
hittable_list.rs:408-419) -- which is what makes the f64 walk bit-identical
to the per-lane walk -- and every pass must make progress."""
import random

import pytest

INF = 0xFFFFFFFF


def keep_smallest(ids, k, lo):
    """A piece's slot: (count of indices >= lo, the k smallest of them sorted)."""
    cand = sorted(i for i in ids if i >= lo)
    return len(cand), cand[:k]


def owner_pass(pieces, big, lo, k_piece, k_max):
    """One pass of the owner: returns (the indices summed in order, bound)."""
    kept, dropped = [], False
    bound = INF

    def add(i):
        nonlocal dropped
        # the device's insertion into ids[kMax]: the largest gives way
        if len(kept) == k_max:
            dropped = True
            if i > kept[-1]:
                return
            kept.pop()
        kept.append(i)
        kept.sort()

    for i in big:
        if i >= lo:
            add(i)
    for ids in pieces:
        cnt, ent = keep_smallest(ids, k_piece, lo)
        for i in ent:
            add(i)
        if cnt > k_piece:
            bound = min(bound, ent[k_piece - 1])
    if dropped:
        bound = min(bound, kept[k_max - 1])
    return [i for i in kept if i <= bound], bound


def coop_sum_order(pieces, big, k_piece, k_max):
    order, lo, passes = [], 0, 0
    while True:
        summed, bound = owner_pass(pieces, big, lo, k_piece, k_max)
        passes += 1
        order += summed
        if bound == INF:
            return order, passes
        assert summed, "a pass that sums nothing cannot advance"
        lo = bound + 1


@pytest.mark.parametrize("k_piece,k_max", [(4, 8), (6, 8), (6, 12), (1, 1), (2, 3)])
def test_every_hit_once_in_list_order(k_piece, k_max):
    rng = random.Random(1234 + 17 * k_piece + k_max)
    for _ in range(3000):
        n_hits = rng.choice([0, 1, 2, 3, 5, 8, 9, 10, 12, 20, 40])
        hits = rng.sample(range(50000), n_hits)
        n_big = rng.choice([0, 0, 1, 2])
        big, rest = hits[:n_big], hits[n_big:]
        n_pieces = rng.randint(1, 12)
        pieces = [[] for _ in range(n_pieces)]
        for i in rest:                      # every hit found by exactly one piece
            pieces[rng.randrange(n_pieces)].append(i)
        order, passes = coop_sum_order(pieces, big, k_piece, k_max)
        assert order == sorted(hits)
        # at least one index per pass; one pass when nothing has to be dropped
        assert passes <= max(1, len(hits))
        if len(hits) <= min(k_piece, k_max):
            assert passes == 1


def test_c5_skimming_ray_takes_two_passes_at_the_default():
    """~10 hits spread over the pieces of a ray skimming C5's light layer:
    the default (6 per piece, 8 per owner) sums them in two passes."""
    pieces = [[101, 7], [50000, 3, 9000], [12, 13], [44], [], [20001, 5]]
    order, passes = coop_sum_order(pieces, [], 6, 8)
    assert order == sorted(i for p in pieces for i in p)
    assert passes == 2
