"""The dynamic cache's host policy engine (csrc/cache.cc, behind shine_selftest_cache) against its independent
restatement (oracle/cache_ref.py) — CPU only.  Random call logs: admissions before and after the cache fills, coins,
always-admitted keys, repeated keys, rescues of cooling entries; the final contents and the admission / eviction /
rescue counts must agree exactly.  Capacity: the reference's formula (compute_node.cc:40-56, hnsw.hh:309-321)."""
import ctypes as C

import numpy as np
import pytest

import cache_ref as CR
from shine_amd import _lib as L


def _engine(entries, seed, calls):
    off, cand, roff, resc = [0], [], [0], []
    for cands, rescued in calls:
        for q, key, always, coin in cands:
            cand += [q, key, (1 if always else 0) | (2 if coin else 0)]
        off.append(off[-1] + len(cands))
        resc += list(rescued)
        roff.append(roff[-1] + len(rescued))
    a = lambda x: np.ascontiguousarray(np.array(x, dtype=np.uint32))
    off, cand, roff, resc = a(off), a(cand or [0]), a(roff), a(resc or [0])
    keys = np.empty(entries + 1, np.uint32)
    n = C.c_uint64()
    counts = np.zeros(3, np.uint64)
    p = lambda x: x.ctypes.data_as(C.c_void_p)
    L.check(L.lib().shine_selftest_cache(entries, seed, len(calls), p(off), p(cand), p(roff), p(resc), p(keys),
                                         keys.size, C.byref(n), p(counts)))
    return keys[:n.value], counts


@pytest.mark.parametrize("entries,seed", [(7, 11), (64, 1), (61, 5), (500, 99)])
def test_engine_equals_restatement(entries, seed):
    rng = np.random.default_rng(entries * 1000 + seed)
    ref = CR.RefCache(entries, seed)
    calls = []
    for call in range(40):
        # rescues: hits on entries cooling at the call's start (and some keys that are not)
        cooling = [k for k, c in ref.cooling.items() if c]
        rescued = list(rng.choice(cooling, size=min(len(cooling), int(rng.integers(0, 6))), replace=False)) if cooling else []
        rescued += [int(x) for x in rng.integers(0, 4 * entries + 10, 2)]
        cands = [(int(rng.integers(0, 30)), int(rng.integers(0, 4 * entries + 10)), bool(rng.random() < 0.1),
                  bool(rng.random() < 0.01)) for _ in range(int(rng.integers(0, 3 * entries + 5)))]
        calls.append((cands, [int(x) for x in rescued]))
        ref.apply_call(calls[-1][1], cands)
    keys, counts = _engine(entries, seed, calls)
    np.testing.assert_array_equal(keys, np.array(sorted(ref.keys()), np.uint32))
    assert list(counts) == [ref.admitted, ref.evicted, ref.rescued]
    assert ref.is_full() and ref.evicted > 0


def test_capacity_formula():
    # ratio % of estimate_index_size over 16 + 4d bytes per entry (compute_node.cc:40-54)
    est = CR.estimate_index_size(1_000_000, 16, 128)
    assert abs(CR.capacity(1_000_000, 16, 128, 5.0) - est * 0.05 / 528) < 1
    assert CR.capacity(6000, 12, 96, 5.0) == 453


def test_a_cache_no_larger_than_its_cooling_table_is_refused():
    """With no more entries than the cooling table holds (6 per bucket), random cooling never pushes a key out and the
    reference's evict() loops forever (cache.hh:232-311); the engine refuses such a size instead."""
    with pytest.raises(L.ShineError):
        _engine(6, 1, [([(0, k, False, False) for k in range(20)], [])])
