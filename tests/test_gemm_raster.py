"""Host restatement of the GEMM workgroup -> job map (csrc/gemm_core.h: xcd_lin, tile_of,
job_of) checked for being a bijection: every (batch entry, K piece, row tile, column tile)
job is computed by exactly one workgroup for any grid the launcher builds
(gemm_f32.hip launch: n1 whole-K tiles + tiles_m * tiles_n * batch * split split jobs), and
every tile of one K piece sits on one XCD (workgroup id mod 8) except where the XCD ranges
cut the job list."""
import itertools

import pytest


def xcd_lin(bid, n):
    q, r = divmod(n, 8)
    xcd, idx = bid % 8, bid // 8
    return (xcd * (q + 1) if xcd < r else r * (q + 1) + (xcd - r) * q) + idx


def tile_of(bid, ntiles, tiles_m, tiles_n, group_m, remap=True):
    if group_m <= 0:
        return bid // tiles_n, bid % tiles_n
    lin = xcd_lin(bid, ntiles) if remap else bid
    per_group = group_m * tiles_n
    grp = lin // per_group
    first_m = grp * group_m
    gm = min(tiles_m - first_m, group_m)
    in_grp = lin % per_group
    return first_m + in_grp % gm, in_grp // gm


def job_of(bid, tiles_m1, tiles_m, tiles_n, batch, split, group_m):
    n1 = tiles_m1 * tiles_n
    if bid < n1:
        tm, tn = tile_of(bid, n1, tiles_m1, tiles_n, group_m)
        return (0, 0, tm, tn)
    bid -= n1
    n2 = tiles_m * tiles_n
    if group_m > 0:
        bid = xcd_lin(bid, n2 * batch * split)
    zb, t2 = divmod(bid, n2)
    b, sidx = divmod(zb, split)
    tm2, tn = tile_of(t2, n2, tiles_m, tiles_n, group_m, remap=False)
    return (b, sidx, tiles_m1 + tm2, tn)


SHAPES = [  # (tiles_m1, tiles_m, tiles_n, batch, split)
    (0, 75, 24, 1, 1), (0, 2, 18, 1, 64), (0, 3, 5, 1, 7), (64, 11, 24, 1, 4),
    (0, 1, 1, 96, 1), (0, 2, 3, 40, 1), (0, 9, 2, 3, 5), (0, 13, 7, 1, 1),
]


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("group_m", [0, 8])
def test_job_map_is_a_bijection(shape, group_m):
    tiles_m1, tiles_m, tiles_n, batch, split = shape
    nblocks = tiles_m1 * tiles_n + tiles_m * tiles_n * batch * split
    jobs = [job_of(b, tiles_m1, tiles_m, tiles_n, batch, split, group_m) for b in range(nblocks)]
    expect = {(0, 0, tm, tn) for tm, tn in itertools.product(range(tiles_m1), range(tiles_n))}
    expect |= {(b, s, tiles_m1 + tm, tn) for b, s, tm, tn in
               itertools.product(range(batch), range(split), range(tiles_m), range(tiles_n))}
    assert len(set(jobs)) == nblocks and set(jobs) == expect


def test_split_pieces_stay_on_one_xcd():
    # wgrad-like: 2 x 18 tiles, 64 K pieces -> each XCD owns 8 whole pieces
    tiles_m, tiles_n, split = 2, 18, 64
    xcd_of = {}
    for bid in range(tiles_m * tiles_n * split):
        _, s, _, _ = job_of(bid, 0, tiles_m, tiles_n, 1, split, 8)
        xcd_of.setdefault(s, set()).add(bid % 8)
    assert all(len(x) == 1 for x in xcd_of.values())
