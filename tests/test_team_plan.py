"""CPU check of the team (latency) mode's ownership plan (egnn_eval.hpp team_exchange).

The exchange rebuilds a molecule's edge aggregates from the G members' parts: message rows from the member holding
the receiver's first tile (plus, without stored segment parts, the member holding its second tile), continuation rows
(Net::cross) from the member holding their tile, shift rows from the one or two members holding the receiver's tiles.
The rebuilt values equal a single workgroup's because (1) every receiver's edges lie in at most two consecutive
tiles, (2) every edge tile belongs to exactly one member (t mod G), and (3) a member that holds none of a receiver's
tiles contributes nothing for it.  This test restates the edge layout (graph.py:6-14 receiver-major, packed for
N <= 33, receiver-tiled with 64 slots per receiver beyond) and the plan's index rules in numpy and checks those
properties, and that summing the owners' parts in the plan's order reproduces a single workgroup's sums bitwise for
random fp32 edge values, for every N in 2 ... 64 and G in 2 ... 8 or G = the tiles per molecule."""
import numpy as np
import pytest


def slots_per_receiver(n):
    return n - 1 if n <= 33 else 64          # ecnf_hip.hip edge_slots_per_receiver


def tiles(n):
    sr = slots_per_receiver(n)
    return (n * sr + 31) // 32


def first_tile(i, n):
    return (i * slots_per_receiver(n)) >> 5


def last_tile(i, n):
    return (i * slots_per_receiver(n) + n - 2) >> 5


@pytest.mark.parametrize("n", list(range(2, 65)))
def test_receiver_segments_touch_at_most_two_consecutive_tiles(n):
    sr = slots_per_receiver(n)
    for i in range(n):
        t = {(i * sr + j) >> 5 for j in range(n - 1)}
        assert t == set(range(first_tile(i, n), last_tile(i, n) + 1)) and len(t) <= 2


# G in 2 ... 8 (the tile-dealt mode) and G = tiles per molecule (the column-split mode, one tile per member)
@pytest.mark.parametrize("n,G", [(n, G) for n in (2, 4, 5, 13, 19, 22, 29, 33, 34, 40, 64)
                                 for G in sorted(set(range(2, 9)) | {max(2, tiles(n))})])
def test_rebuilt_aggregates_equal_single_workgroup(n, G):
    rng = np.random.default_rng(n * 10 + G)
    sr = slots_per_receiver(n)
    nt = tiles(n)
    val = rng.standard_normal(nt * 32).astype(np.float32)
    recv = np.full(nt * 32, -1)
    for i in range(n):
        for j in range(n - 1):
            recv[i * sr + j] = i
    # a single workgroup: per (receiver, tile) part sums, then 0 + a + b in fp32 (commutative for two parts)
    parts = {}
    for t in range(nt):
        for i in set(recv[t * 32:(t + 1) * 32]) - {-1}:
            sel = recv[t * 32:(t + 1) * 32] == i
            parts[(i, t)] = np.float32(val[t * 32:(t + 1) * 32][sel].sum(dtype=np.float32))
    single = np.zeros(n, np.float32)
    for (i, t), v in sorted(parts.items()):
        single[i] = np.float32(single[i] + v)
    # team: member r holds the parts of its tiles (t mod G == r), zeros elsewhere
    slot = np.zeros((G, n), np.float32)
    for (i, t), v in parts.items():
        r = t % G
        slot[r, i] = np.float32(slot[r, i] + v)
    rebuilt = np.zeros(n, np.float32)
    for i in range(n):
        o0, o1 = first_tile(i, n) % G, last_tile(i, n) % G
        rebuilt[i] = slot[o0, i] if o1 == o0 else np.float32(slot[o0, i] + slot[o1, i])
        # a member owning neither tile contributes exactly zero
        for r in set(range(G)) - {o0, o1}:
            assert slot[r, i] == 0
    assert np.array_equal(rebuilt, single)
