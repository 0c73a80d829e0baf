"""The sharded placement's view plan on the host (no GPU): shine_plan_sharded_views, the plan that shine_open_ex maps for
SHINE_PLACE_SHARDED (csrc/views.cc, used by capi.cc map_sharded).

The reference places each record on memory node RemotePtr bits 63..48 (remote_pointer.hh:9-22) and compute nodes
split queries id % num_clients (read_data.hh:57-58).  Here memory node s lives on GPU slot s % G, and every slot maps
the whole id space into a view of its own.  Checked for G in {2, 4, 8} GPUs, for the 8 memory nodes of cfg 4 and with
slots repeating one GPU (the one-GPU emulation):
* every view covers [0, G x stride) without gaps or overlaps, one stripe per slot, in offset order;
* its own stripe and its copies of the other stripes' hot prefixes are backed by the view's own GPU ("local stripes
  are mapped from local handles"); the other stripes' cold rows are backed by their owners' GPUs (xGMI);
* every view grants access to exactly the handle's distinct GPUs (G descriptors with G distinct GPUs);
* every ordered pair of distinct GPUs is checked for a peer path, and no pair of a GPU with itself.
"""
import itertools

import pytest

import shine_amd
from shine_amd import _lib as L

MiB = 1 << 20


def _check(gpus, stride, cached):
    plan = shine_amd.plan_sharded_views(gpus, stride, cached)
    G = len(gpus)
    uniq = sorted(set(gpus))
    eff_cached = min(cached, stride) if G > 1 else 0
    by_view = {}
    for p in plan["pieces"]:
        by_view.setdefault(p["view_slot"], []).append(p)
    assert sorted(by_view) == list(range(G))
    for o, pieces in by_view.items():
        # coverage: contiguous pieces from 0 to G * stride
        pos = 0
        for p in pieces:
            assert p["offset"] == pos and p["size"] > 0
            pos += p["size"]
        assert pos == G * stride
        for p in pieces:
            q = p["stripe"]
            assert q * stride <= p["offset"] < (q + 1) * stride
            hot = p["offset"] < q * stride + eff_cached
            if q == o:
                assert p["kind"] == L.VIEW_OWN and p["backing_device"] == gpus[o]
            elif hot:
                assert p["kind"] == L.VIEW_COPY and p["backing_device"] == gpus[o]  # the local cache of q's prefix
                assert p["size"] == eff_cached
            else:
                assert p["kind"] == L.VIEW_PEER and p["backing_device"] == gpus[q]  # q's HBM, read over xGMI
        # one piece per stripe, or two when the stripe has a hot prefix and a cold rest
        per = (1 if eff_cached in (0, stride) else 2)
        assert len(pieces) == G * per
        assert plan["access"][o] == uniq
    assert sorted(plan["peer_pairs"]) == sorted((a, b) for a, b in itertools.permutations(uniq, 2))
    return plan


@pytest.mark.parametrize("G", [2, 4, 8])
@pytest.mark.parametrize("cached", [0, 2 * MiB, 64 * MiB])
def test_view_plan_distinct_gpus(G, cached):
    plan = _check(list(range(G)), 64 * MiB, cached)
    assert all(len(a) == G for a in plan["access"])  # exactly G access descriptors per view
    # the xGMI share of a view: (G - 1) of G stripes less their cached prefixes
    peer = sum(p["size"] for p in plan["pieces"] if p["view_slot"] == 0 and p["kind"] == L.VIEW_PEER)
    assert peer == (G - 1) * (64 * MiB - min(cached, 64 * MiB))


@pytest.mark.parametrize("G", [2, 4, 8])
def test_view_plan_eight_memory_nodes_over_gpus(G):
    """cfg 4: 8 memory-node dumps over G GPUs (node s on slot s % G): the plan is per slot, so G slots, each with
    a stripe of 8 / G memory nodes; a whole stripe cached (cache fraction 1) has no cold rest and no peer piece."""
    plan = _check(list(range(G)), 32 * MiB, 32 * MiB)
    assert not any(p["kind"] == L.VIEW_PEER for p in plan["pieces"])


def test_view_plan_repeated_gpu():
    """8 slots on one GPU (the one-GPU emulation of cfg 4): one access descriptor, no peer pair, every piece local."""
    plan = _check([0] * 8, 8 * MiB, 2 * MiB)
    assert plan["peer_pairs"] == []
    assert all(p["backing_device"] == 0 for p in plan["pieces"])
    assert all(a == [0] for a in plan["access"])


def test_view_plan_two_gpus_four_slots():
    plan = _check([0, 1, 0, 1], 16 * MiB, 4 * MiB)
    assert sorted(plan["peer_pairs"]) == [(0, 1), (1, 0)]


def test_view_plan_single_slot_has_no_cache():
    plan = _check([3], 8 * MiB, 4 * MiB)
    assert len(plan["pieces"]) == 1 and plan["pieces"][0]["kind"] == L.VIEW_OWN


def test_view_plan_rejects_bad_arguments():
    with pytest.raises(shine_amd.ShineError):
        shine_amd.plan_sharded_views([], 8 * MiB)
    with pytest.raises(shine_amd.ShineError):
        shine_amd.plan_sharded_views([0, 1], 0)
